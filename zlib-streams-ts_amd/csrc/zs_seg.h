// zs_seg.h -- the segmented decode of members (inflate_seg.hip): records shared
// with the host (capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zs_inflate.h"
#include "zs_inftab.h"
#include "zs_split.h"

#define ZS_SEG_LANES 64u    // pieces per span (one lane each)
#define ZS_SEG_W 1024u      // bits of a lane's start window whose symbol starts it records (the sync bitmaps; 2048 in
                            // the walk instance for batches of few large members: fewer chains that do not meet)
#ifndef ZS_SEG_CKB
// spacing of a lane's (position, output count) checkpoints in its window: 256 bits keeps the
// 1,024-bit walk at 25 KB of LDS, six walks per CU instead of five (4,096 x 256 KiB decode 14.45 ->
// 13.73 ms, C5-i 8.98 -> 8.47 ms; the re-decode from a checkpoint is at most 256 bits)
#define ZS_SEG_CKB 256u
#endif
#define ZS_SEG_NEV 4u       // sub-chunk crossing events a lane records
#define ZS_SEG_NEOB 4u      // end-of-block codes a lane logs
#define ZS_SEG_PAD 16u      // u16 values of padding behind each piece's scratch
#define ZS_SEG_TAB (ENOUGH_LENS + ENOUGH_DISTS_9)  // cached table entries per block
#define ZS_SEG_NONE 0xffffffffu
#define ZS_SEG_BIG_BITS (1u << 21)  // members with more input bits: block starts from the finder as extra entries
#define ZS_SEG_SPLIT_BITS (1u << 18)  // deflate64 members with more input bits: the split decode (long copies)
#define ZS_SEG_BLOCK_BITS 16384u    // span slots per member: one per this many input bits (+ capi.cpp's margin)
#define ZS_SEG_SMAX 8192u           // bits per lane at most (a span's lanes: seg_bits, then from the block before)

// span flags
#define ZS_SEG_B_OK 1u     // header parsed (FIRST), the span's pieces chain from its start to its end
#define ZS_SEG_B_FINAL 2u  // ends the member's final block
#define ZS_SEG_B_FIRST 4u  // starts a block (its header at hdr)
#define ZS_SEG_B_EOB 8u    // ends its block (else the entry's next span continues it)
#define ZS_SEG_B_STORED 16u  // a stored block (BTYPE 0): one piece, lane 0, its bytes copied from the input
#define ZS_SEG_B_SPLIT 32u   // (split mode) the pieces' second halves are in the next slot, which the decode runs too

// One span: a stretch of one block whose symbols a wave's lanes decode from
// sym0 + j S (zs_k_seg_walk); its lanes' pieces in zs_seg_lane[span * 64 + j].
struct zs_seg_blk {
  uint32_t m, e;     // member (list index), entry
  uint32_t hdr;      // bit of the block header (FIRST), else = sym0
  uint32_t sym0;     // bit of the span's first symbol
  uint32_t end;      // bit where the span ends (past the end-of-block code, or the next span's sym0)
  uint32_t flags;
  uint32_t lbits, dbits, dofs, tab;  // table roots, distance table offset, the span slot caching the tables
  uint32_t nl, S;    // lanes, bits per lane
  uint32_t next;     // the entry's next span (ZS_SEG_NONE: its last)
  uint32_t pad[3];
};

// One lane of a span: a piece of the block, [start, end) in bits.
struct zs_seg_lane {
  // zs_k_seg_walk
  uint32_t start, end;   // start ZS_SEG_NONE: no piece (the lane was absorbed by the one before)
  uint32_t cnt;          // output values of the piece
  uint32_t last_len;     // values of its last symbol (0: an end of block)
  uint32_t nev, ev_k0;   // sub-chunk crossing events: how many, the first sub-chunk index
  uint32_t ev_o[ZS_SEG_NEV];  // their symbols' output positions, relative to the piece start
  // (split mode) where the plan may cut the piece in two: the first symbol start past
  // the lane's middle (ZS_SEG_NONE: none), the values before it, the values of the symbol before it
  uint32_t mb, mc, mll;
  // zs_k_seg_plan
  uint32_t O;            // member output position of the piece start
  uint32_t off;          // its scratch offset (u16 values; a multiple of 8)
  uint32_t dend;         // bit where zs_k_seg_decode stops (past merged pieces)
  uint32_t dcnt;         // values zs_k_seg_decode writes (merged pieces included)
  uint32_t B, wn, wh, cend;  // the reference's call state at the start (zs_refcalls)
  uint32_t act;          // bit 0: decoded (a piece that is not merged), bit 1: the fast flag
};

// One entry of a member: where a walk starts (entry 0: the member's first bit;
// a big member's entries e >= 1: the finder's block start in bit range e).
struct zs_seg_ent {
  uint32_t start, first, end, flags;  // first span; end: the block boundary it stopped at; flags 1 ok, 2 final
};

struct zs_seg_mem {
  uint32_t bad, total, consumed, want, npieces, nalloc;  // nalloc: span slots taken (zs_k_seg_walk)
  uint32_t pad[2];
};

template <bool D64, uint32_t W, bool ST>  // W: the sync window (1024, or 2048 for a batch of few large members);
                                          // ST: large members, the bookkeeping-free stretch (inflate_seg.hip)
__global__ void zs_k_seg_walk(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* list,
                              uint32_t n_list, const uint32_t* big, uint32_t n_big, int wbits, const uint64_t* found,
                              const uint32_t* spb, zs_seg_blk* blk, zs_seg_lane* lanes, zcode* tcache,
                              zs_seg_ent* ents, zs_seg_mem* mem, uint32_t* nspan, uint32_t* spans, uint32_t sbits,
                              int split);
__global__ void zs_k_seg_plan(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                              const uint32_t* out_cap, const uint32_t* list, uint32_t n_list, int wbits, int refw,
                              const zs_seg_blk* blk, zs_seg_lane* lanes, const zs_seg_ent* ents, zs_seg_mem* mem,
                              const uint32_t* pbase, uint4* ptab);
template <bool D64, bool REFW>
__global__ void zs_k_seg_decode(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint32_t* list,
                                const uint32_t* nspan, const uint32_t* spans, const zs_seg_blk* blk, const zs_seg_lane* lanes, const zcode* tcache,
                                zs_seg_mem* mem, const uint64_t* sbase, uint16_t* scratch);
template <uint32_t T, uint32_t RING>  // threads per member, its LDS ring of final bytes (dynamic LDS)
__global__ void zs_k_seg_resolve(const uint32_t* list, const zs_seg_mem* mem, const uint32_t* pbase,
                                 const uint4* ptab, const uint64_t* sbase, const uint16_t* scratch, uint8_t* out,
                                 const uint64_t* out_off, zs_lane_res* res, uint32_t* lens_out, uint32_t* n_ok,
                                 uint32_t* n_left, uint32_t* left);
