// zs_kernels.h -- kernel entry points and the batch descriptor shared by the
// HIP translation units and the C-ABI host layer (capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Per-block record written by the parse / tree kernels.
struct zs_block {
  uint32_t sym_start;   // first symbol (index into the stream's symbol array)
  uint32_t sym_count;
  uint32_t in_start;    // input byte range covered by the block
  uint32_t in_end;
  uint32_t type;        // 0 stored, 1 static, 2 dynamic (trees.ts:574-583)
  uint32_t hdr_bits;    // dynamic-tree header bits (send_all_trees)
  uint32_t data_bits;   // symbol bits incl. END_BLOCK
  uint32_t last;        // bit 0: final block; bit 1: block began before the slid window (reference would copy from a negative index)
  uint32_t pad;
  uint64_t bit_off;     // bit offset of the 3-bit block header in the stream output
  uint64_t bit_end;     // bit offset just past the block (before the final byte pad)
};

// Per-stream record.
struct zs_stream {
  uint32_t nsym;
  uint32_t nblk;
  uint64_t total_bits;  // deflate payload bits (after the wrapper header)
  uint32_t out_len;     // bytes incl. wrapper
  int32_t status;       // Z_STREAM_END / Z_BUF_ERROR
  uint32_t check;       // adler32 / crc32 of the input (wrappers)
  uint32_t pad;
};

// ORD: same-address LDS atomics of one instruction apply in lane order (zs_selftest); false: the ballot form
template <bool ORD>
__global__ void zs_k_prev(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base,
                          uint16_t* prevd, uint32_t min_len);
__global__ void zs_k_match(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base,
                           const uint16_t* prevd, uint2* mres, int chain, int nice, uint32_t min_len);
// levels 4..9 (deflate_sweep.hip), one workgroup per WINDOW: the inserted
// positions from `base` up to its own positions' end ohi (at most 65,535; a
// stream of up to 65,537 bytes is one window, base 0); the window writes the
// results of its own positions [olo, ohi) (window-relative), members at
// members + mb (u16, window-relative)
struct zs_sweep_seg {
  uint32_t s, base, olo, ohi;
  uint64_t mb;
  uint64_t pad;
};
#define ZS_SEG_WPOS 65535u   // inserted positions per window at most (u16 members; bucket counts fit 16 bits)
#define ZS_SEG_FIRST 65520u  // own positions of a long stream's first window ...
#define ZS_SEG_OWN 32752u    // ... and of its later ones, after a 32,768-position look-back (> MAX_DIST);
                             // multiples of 16: every window starts 16-byte aligned with its stream
// zs_k_bucket's workgroup: wave 0 claims, the others scatter (a multiple of 64 dividing 16384: the scan's slices)
#define ZS_BK_THREADS 512u
template <bool ORD>
__global__ void zs_k_bucket(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base,
                            const zs_sweep_seg* segs, uint16_t* members, uint2* mres);
__global__ void zs_k_sweep(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base,
                           const zs_sweep_seg* segs, const uint16_t* members, uint2* mres, int chain, int nice);
// the lazy parse (deflate_parse.hip): pass A stages 32 match-table entries per lane in LDS
#define ZS_PARSE_DECL(name)                                                                                        \
  __global__ void name(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base, \
                       const uint32_t* blk_base, const uint2* mres, uint32_t* syms, zs_block* blocks,              \
                       zs_stream* streams, uint32_t* scratch, int good, int lazy);
ZS_PARSE_DECL(zs_k_parse)
ZS_PARSE_DECL(zs_k_parse_2w)  // two waves per stream, ZS_PARSE2W_SEG-position segments
ZS_PARSE_DECL(zs_k_parse_4w)  // four waves per stream, ZS_PARSE4W_SEG-position segments
// parse scratch words per 1024-position segment (deflate_parse.hip)
#define ZS_PARSE_SEG 1024u
#define ZS_PARSE_SEG_WORDS 3596u
#define ZS_PARSE2W_SEG 512u
#define ZS_PARSE2W_SEG_WORDS 2060u
#define ZS_PARSE4W_SEG 256u
#define ZS_PARSE4W_SEG_WORDS 1292u
template <int NW, bool ORD>
__global__ void zs_k_fast(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, const uint64_t* pos_base,
                          const uint32_t* blk_base, uint32_t* syms, zs_block* blocks, zs_stream* streams, int chain,
                          int lazy, int nice);
__global__ void zs_k_fast_serial(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                                 const uint64_t* pos_base, const uint32_t* blk_base, uint32_t* syms, zs_block* blocks,
                                 zs_stream* streams, int chain, int lazy, int nice);
__global__ void zs_k_trees(const uint8_t* in, const uint64_t* in_off, const uint64_t* pos_base, const uint32_t* blk_base,
                           const uint32_t* syms, zs_block* blocks, const zs_stream* streams, uint32_t* codes,
                           uint32_t* hdr, int nstreams);
__global__ void zs_k_layout(const uint32_t* blk_base, zs_block* blocks, zs_stream* streams, const uint32_t* out_cap,
                            uint8_t* out, const uint64_t* out_off, int wrap, int nstreams);
__global__ void zs_k_emit(const uint8_t* in, const uint64_t* in_off, const uint64_t* pos_base, const uint32_t* blk_base,
                          const uint32_t* syms, const zs_block* blocks, const zs_stream* streams, const uint32_t* codes,
                          const uint32_t* hdr, uint8_t* out, const uint64_t* out_off, int wrap);
__global__ void zs_k_stored(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                            const uint64_t* out_off, const uint32_t* out_cap, const uint32_t* check, int wrap,
                            int32_t* status, uint32_t* out_len_res);
__global__ void zs_k_wrap(const zs_stream* streams, uint8_t* out, const uint64_t* out_off, const uint32_t* in_len,
                          int wrap, int level, int nstreams);
__global__ void zs_k_checksum(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t* check,
                              int kind, const uint32_t* seeds = nullptr);
__global__ void zs_k_selftest(uint32_t* bad, int rounds);
