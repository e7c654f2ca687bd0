// zs_split.h -- the split decode of large members (inflate_split.hip): layout
// shared with the host (capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zs_inflate.h"

#define ZS_SPLIT_MAX 64u           // bit ranges searched per member (pieces <= this)
#define ZS_SPLIT_MIN_SPAN 16384u   // bits per range at least (2 KiB of input)
#define ZS_SPLIT_MARK_MAX 65280u   // markers: 255 + k for the byte k before the piece, k <= this
#define ZS_SPLIT_BAIL 1u
#define ZS_SPLIT_FINAL 2u

struct zs_split_piece_res {
  uint64_t end;    // bit position where the piece stopped
  uint32_t count;  // values it produced
  uint32_t flags;  // ZS_SPLIT_BAIL, ZS_SPLIT_FINAL
  uint32_t next;   // the piece whose start it stopped at (piece order), if neither flag
  uint32_t pad;
};

// a member's chain of pieces and its outcome (zs_k_split_chain .. zs_k_split_final)
struct zs_split_member {
  uint32_t nchain, total, consumed, bad;
  uint32_t piece[ZS_SPLIT_MAX];  // chain entry -> piece
  uint32_t off[ZS_SPLIT_MAX];    // chain entry -> output offset
};

static __host__ __device__ inline uint64_t zs_split_span(uint32_t n) {
  const uint64_t nbits = 8ull * n;
  const uint64_t s = (nbits + ZS_SPLIT_MAX - 1) / ZS_SPLIT_MAX;
  return s < ZS_SPLIT_MIN_SPAN ? (uint64_t)ZS_SPLIT_MIN_SPAN : s;
}

__global__ void zs_k_split_find(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                const uint32_t* list, int wbits, uint64_t* found);
__global__ void zs_k_split_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                  const uint32_t* list, int wbits, const uint64_t* found, zs_split_piece_res* pres,
                                  uint16_t* scratch, uint32_t piece_cap);
__global__ void zs_k_split_chain(const uint32_t* in_len, const uint32_t* out_cap, const uint32_t* list,
                                 uint32_t n_list, const zs_split_piece_res* pres, zs_split_member* mem);
__global__ void zs_k_split_place(const zs_split_piece_res* pres, zs_split_member* mem, const uint16_t* scratch,
                                 uint32_t piece_cap, uint32_t* val, uint64_t val_stride);
__global__ void zs_k_split_jump(const zs_split_member* mem, uint32_t* val, uint64_t val_stride);
__global__ void zs_k_split_write(const uint32_t* list, zs_split_member* mem, const uint32_t* val, uint64_t val_stride,
                                 uint8_t* out, const uint64_t* out_off);
__global__ void zs_k_split_final(const uint32_t* list, uint32_t n_list, const zs_split_member* mem, zs_lane_res* res,
                                 uint32_t* lens_out);
size_t zs_split_lds_bytes(bool d64);
