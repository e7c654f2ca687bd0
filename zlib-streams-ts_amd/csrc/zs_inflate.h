// zs_inflate.h -- inflate kernel interface (inflate.hip) and message table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZS_PHASE_NONE_ 0
#define ZS_PHASE_PROCESS_ 2
#define ZS_PHASE_FINISH_ 3

// z_stream messages (inflate.ts:397-1031, inffast.ts:108,197,210)
enum zs_msg_id {
  ZS_MSG_NONE = 0,
  ZS_MSG_HEADER_CHECK,
  ZS_MSG_METHOD,
  ZS_MSG_WINDOW,
  ZS_MSG_FLAGS,
  ZS_MSG_HEADER_CRC,
  ZS_MSG_BLOCK_TYPE,
  ZS_MSG_STORED_LEN,
  ZS_MSG_TOO_MANY,
  ZS_MSG_TOO_MANY_D64,
  ZS_MSG_CODE_LENGTHS,
  ZS_MSG_REPEAT,
  ZS_MSG_MISSING_EOB,
  ZS_MSG_LITLEN_SET,
  ZS_MSG_DIST_SET,
  ZS_MSG_LITLEN_CODE,
  ZS_MSG_DIST_CODE,
  ZS_MSG_TOO_FAR,
  ZS_MSG_DATA_CHECK,
  ZS_MSG_LENGTH_CHECK,
  ZS_MSG_CAPACITY,
  ZS_MSG_COUNT
};

struct zs_inflate_result {
  int32_t status;
  int32_t phase;
  int32_t msg;
  uint32_t out_len;
  uint32_t consumed;
};

__global__ void zs_k_inflate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint32_t* out_cap, int wbits, zs_inflate_result* res);
size_t zs_inflate_smem_bytes(int wbits);
