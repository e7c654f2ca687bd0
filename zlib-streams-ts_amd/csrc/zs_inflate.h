// zs_inflate.h -- inflate kernel interface (inflate.hip) and message table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZS_PHASE_NONE_ 0
#define ZS_PHASE_PROCESS_ 2
#define ZS_PHASE_FINISH_ 3
// inflate kernel flags
#define ZS_INF_REF_WRAP 1  // reproduce the reference's inflate_fast window-wrap copy (inffast.ts:133-147)

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

// Outcome of the lane-per-member fast path (inflate_lane.hip).
struct zs_lane_res {
  uint32_t bail;      // 0: decoded cleanly; 1: the exact path decides
  uint32_t out_len;
  uint32_t consumed;
  uint32_t want;      // trailer check value (zlib: adler32, gzip: crc32)
};

__global__ void zs_k_inflate(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint32_t* out_cap, int wbits, zs_inflate_result* res,
                             const zs_lane_res* only, int flags);
// A member the lane kernel leaves to the large-member paths (the segmented, split
// or wave decode) when wave_min is set: more input bytes than wave_min, or a high
// expansion (a cap past 64 KiB and at least 8 bytes of it per input byte: long
// copies, which one lane makes byte by byte -- deflate64's zeros_100k.deflate64 took a
// lane 4.3 ms; the wave decoders copy 64 bytes at a time)
static __host__ __device__ inline bool zs_inf_expands(uint32_t in_len, uint32_t out_cap) {
  return out_cap > 65536u && out_cap / 8u >= in_len;
}
static __host__ __device__ inline bool zs_inf_large(uint32_t in_len, uint32_t out_cap, uint32_t wave_min) {
  return wave_min && (in_len > wave_min || zs_inf_expands(in_len, out_cap));
}
struct zs_lane_tabs;
template <int RT, bool REFW>
__global__ void zs_k_inflate_lane(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                  const uint64_t* out_off, const uint32_t* out_cap, int wbits, uint32_t n_members,
                                  zs_lane_tabs* tabs, zs_lane_res* res, uint32_t* lens_out, int flags,
                                  uint32_t wave_min, const uint32_t* list);
template <bool REFW>
__global__ void zs_k_inflate_wave(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                  const uint64_t* out_off, const uint32_t* out_cap, int wbits, const uint32_t* list,
                                  uint32_t n_list, zs_lane_res* res, uint32_t* lens_out, const uint32_t* n_dev);
__global__ void zs_k_inflate_lane_verify(zs_lane_res* res, const uint32_t* check, uint32_t n);
size_t zs_inflate_smem_bytes(int wbits);
size_t zs_inflate_lane_lds_bytes(bool root);
size_t zs_inflate_lane_scratch_bytes();
size_t zs_inflate_wave_lds_bytes(bool d64);
