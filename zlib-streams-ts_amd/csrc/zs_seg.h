// zs_seg.h -- the segmented decode of members (inflate_seg.hip): records shared
// with the host (capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zs_inflate.h"
#include "zs_inftab.h"
#include "zs_split.h"

#define ZS_SEG_LANES 64u    // pieces per block wave (one lane each)
#define ZS_SEG_W 2048u      // bits of a lane's start window whose symbol starts it records (the sync bitmap)
#define ZS_SEG_CKB 128u     // spacing of a lane's (position, output count) checkpoints in its window
#define ZS_SEG_NCK (ZS_SEG_W / ZS_SEG_CKB)
#define ZS_SEG_NEV 4u       // sub-chunk crossing events a lane records
#define ZS_SEG_NEOB 4u      // end-of-block codes a lane logs
#define ZS_SEG_PAD 16u      // u16 values of padding behind each piece's scratch
#define ZS_SEG_TAB (ENOUGH_LENS + ENOUGH_DISTS_9)  // cached table entries per block
#define ZS_SEG_NONE 0xffffffffu

// block flags
#define ZS_SEG_B_OK 1u     // header parsed, tables cached, its pieces chain to an end of block
#define ZS_SEG_B_FINAL 2u  // BFINAL set

// One candidate block (zs_k_split_find's found[] entry, given a compact index by zs_k_seg_alloc).
struct zs_seg_blk {
  uint32_t m, r;     // member (list index), range of the finder
  uint32_t hdr;      // bit of the block header
  uint32_t sym0;     // bit of the first symbol
  uint32_t end;      // bit past the end-of-block code
  uint32_t flags;
  uint32_t lbits, dbits, dofs;  // table roots, distance table offset in the cached codes
  uint32_t nl, S;    // lanes, bits per lane
  uint32_t pad;
};

// One lane of a block wave: a piece of the block, [start, end) in bits.
struct zs_seg_lane {
  // zs_k_seg_sync
  uint32_t start, end;   // start ZS_SEG_NONE: no piece (the lane was absorbed by the one before)
  uint32_t cnt;          // output values of the piece
  uint32_t last_len;     // values of its last symbol (0: an end of block)
  uint32_t nev, ev_k0;   // sub-chunk crossing events: how many, the first sub-chunk index
  uint32_t ev_o[ZS_SEG_NEV];  // their symbols' output positions, relative to the piece start
  // zs_k_seg_plan
  uint32_t O;            // member output position of the piece start
  uint32_t off;          // its scratch offset (u16 values; a multiple of 8)
  uint32_t dend;         // bit where zs_k_seg_decode stops (past merged pieces)
  uint32_t dcnt;         // values zs_k_seg_decode writes (merged pieces included)
  uint32_t B, wn, wh, cend;  // the reference's call state at the start (zs_refcalls)
  uint32_t act;          // bit 0: decoded (a piece that is not merged), bit 1: the fast flag
};

struct zs_seg_mem {
  uint32_t bad, total, consumed, want, npieces;
  uint32_t pad[3];
};

__global__ void zs_k_seg_alloc(const uint64_t* found, uint32_t n_list, uint32_t* cidx, zs_seg_blk* blk,
                               uint32_t* counter, uint32_t cap_blocks, zs_seg_mem* mem);
template <bool D64>
__global__ void zs_k_seg_sync(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* list,
                              int wbits, const uint64_t* found, const uint32_t* counter, zs_seg_blk* blk,
                              zs_seg_lane* lanes, zcode* tcache, uint32_t smin);
__global__ void zs_k_seg_plan(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                              const uint32_t* out_cap, const uint32_t* list, uint32_t n_list, int wbits, int refw,
                              const uint32_t* cidx, zs_seg_blk* blk, zs_seg_lane* lanes, zs_seg_mem* mem,
                              const uint32_t* pbase, uint4* ptab);
template <bool D64, bool REFW>
__global__ void zs_k_seg_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* list,
                                const uint32_t* counter, const zs_seg_blk* blk, const zs_seg_lane* lanes,
                                const zcode* tcache, zs_seg_mem* mem, const uint64_t* sbase, uint16_t* scratch);
__global__ void zs_k_seg_resolve(const uint32_t* list, const zs_seg_mem* mem, const uint32_t* pbase,
                                 const uint4* ptab, const uint64_t* sbase, const uint16_t* scratch, uint8_t* out,
                                 const uint64_t* out_off, zs_lane_res* res, uint32_t* lens_out, uint32_t* n_ok);
