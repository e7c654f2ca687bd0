// deflate_emit.hip -- Huffman tree construction, block layout and bit packing.
//
//   zs_k_trees  : one wave per block.  The wave histograms the block's symbols
//                 with LDS atomics; lane 0 then runs the serial heart of the
//                 reference's exact tree construction (the heap ordered by freq
//                 then depth, trees.ts:167-316; the bit lengths follow by the
//                 wave, with lane 0's overflow repair), the tree run-length coding
//                 (trees.ts:318-447) and the stored/static/dynamic choice
//                 (trees.ts:554-583); the wave does the rest in parallel
//                 (frequency set-up, canonical codes by per-length ballots,
//                 payload bit counts, the code table and header stores).
//   zs_k_layout : one lane per stream: bit offset of every block (stored
//                 blocks depend on byte alignment), output length, status, and
//                 zeroing of the words that two writers share.
//   zs_k_emit   : one 256-thread workgroup per block.  Symbol bit lengths are
//                 prefix-summed across the workgroup; codes are OR-ed into an
//                 LDS bit buffer aligned to the output's 32-bit word grid and
//                 written out with coalesced stores (atomic OR only on the two
//                 words a block shares with its neighbours).
//   zs_k_wrap   : zlib / gzip header and trailer (deflate.ts:753-806, 964-983).
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

// ------------------------------------------------------------ tree building
static constexpr int ZS_EXTRA_BLBITS[ZS_BL_CODES] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
struct zs_tw {  // LDS workspace of one wave, common/types.ts DeflateState tree fields
  // (the length arrays 16-byte aligned: zs_run_at reads eight lengths at a time)
  uint16_t llen[ZS_HEAP_SIZE] __attribute__((aligned(16)));
  uint16_t dlen[2 * ZS_D_CODES + 1] __attribute__((aligned(16)));
  uint16_t lfreq[ZS_HEAP_SIZE], ldad[ZS_HEAP_SIZE];  // (the codes go straight to HBM: zs_gen_codes_out)
  uint16_t dfreq[2 * ZS_D_CODES + 1], ddad[2 * ZS_D_CODES + 1];
  uint16_t bfreq[2 * ZS_BL_CODES + 1], blen[2 * ZS_BL_CODES + 1], bdad[2 * ZS_BL_CODES + 1], bcode[2 * ZS_BL_CODES + 1];
  int16_t heap[2 * ZS_L_CODES + 1];
  uint32_t hk[2 * ZS_L_CODES + 4] __attribute__((aligned(16)));  // working heap: freq << 17 | depth << 10 | node
                                                                   // (+2: the sift reads grandchildren 2j..2j+3)
  // the distance tree's own heap arrays: it is built beside the literal/length tree
  int16_t heapd[2 * ZS_D_CODES + 1];
  uint32_t hkd[2 * ZS_D_CODES + 4] __attribute__((aligned(16)));
  uint16_t bl_count[16];
  uint16_t tally[ZS_L_CODES + ZS_D_CODES];  // the block's true counts (the histogram itself lives in hk)
  uint32_t hdr[ZS_HDR_WORDS];
  uint32_t bc[4];  // lane 0 -> wave: type, max codes, header bits
  uint32_t b32[32];  // scan_tree's bl_tree frequencies (LDS atomics)
};

struct zs_tdesc {
  uint16_t *freq, *len, *dad, *code;
  const uint32_t* stat;  // static tree (code | len << 16) or nullptr
  const int* extra;
  int extra_base, elems, max_length, max_code;
};

struct zs_tstate {
  zs_tw* w;
  uint32_t* hk;     // the tree's heap entries (then gen_bitlen's ancestor words)
  int16_t* heap;    // the tree's heap[] (trees.ts: s.heap), heap_size entries
  int heap_size;
  int heap_len, heap_max;
  uint32_t opt_len, static_len;
  // header bit writer
  uint32_t hbits;
};

// The heap orders nodes by freq, then depth (smaller(n, m): freq[n] < freq[m] ||
// (freq[n] == freq[m] && depth[n] <= depth[m]), trees.ts:163-165).  Each heap
// entry carries its own key -- freq << 17 | depth << 10 | node, so the order is
// the order of (entry >> 10) -- and a sift step costs one LDS read of the two
// children instead of a dependent chain through the freq and depth arrays.
// Widths: a block's total frequency is at most 16,384 (ZS_SYM_END symbols +
// end-of-block), below 2^15; depths stay far below 2^7; nodes below 2^10.
static __device__ __forceinline__ uint32_t zs_hkey(uint32_t e) { return e >> 10; }

// pqdownheap (trees.ts:167-185), two levels per LDS round trip: the children
// j, j + 1 and all four grandchildren 2j .. 2j + 3 are read together (entries
// past heap_len are read but never selected: the j < heap_len / j2 <= heap_len
// tests guard them).
static __device__ void zs_pqdownheap(zs_tstate& t, int k) {
  uint32_t* hk = t.hk;
  const uint32_t v = hk[k], kv = zs_hkey(v);
  const int len = t.heap_len;
  int j = k << 1;
  while (j <= len) {
    const uint2 ch = *reinterpret_cast<const uint2*>(&hk[j]);  // j even: 8-byte aligned
    const uint4 gc = *reinterpret_cast<const uint4*>(&hk[2 * j]);  // 2j multiple of 4: 16-byte aligned
    const bool right = j < len && zs_hkey(ch.y) <= zs_hkey(ch.x);
    const uint32_t c = right ? ch.y : ch.x;
    if (kv <= zs_hkey(c)) break;
    hk[k] = c;
    k = j + (right ? 1 : 0);
    const int j2 = k << 1;
    if (j2 > len) break;
    const uint32_t a2 = right ? gc.z : gc.x, b2 = right ? gc.w : gc.y;
    const bool right2 = j2 < len && zs_hkey(b2) <= zs_hkey(a2);
    const uint32_t c2 = right2 ? b2 : a2;
    if (kv <= zs_hkey(c2)) break;
    hk[k] = c2;
    k = j2 + (right2 ? 1 : 0);
    j = k << 1;
  }
  hk[k] = v;
}

// pqdownheap of a value v the caller holds in a register (placed at k, i.e.
// hk[k] = v then the sift): no LDS read of hk[k] first, and it returns the
// entry that ends at k -- the new root for k = 1 -- so the merge loop reads
// neither hk[1] back
static __device__ uint32_t zs_pqdownheap_v(zs_tstate& t, int k, uint32_t v) {
  uint32_t* hk = t.hk;
  const uint32_t kv = zs_hkey(v);
  const int len = t.heap_len, k0 = k;
  uint32_t top = v;
  int j = k << 1;
  while (j <= len) {
    const uint2 ch = *reinterpret_cast<const uint2*>(&hk[j]);
    const uint4 gc = *reinterpret_cast<const uint4*>(&hk[2 * j]);
    const bool right = j < len && zs_hkey(ch.y) <= zs_hkey(ch.x);
    const uint32_t c = right ? ch.y : ch.x;
    if (kv <= zs_hkey(c)) break;
    hk[k] = c;
    if (k == k0) top = c;
    k = j + (right ? 1 : 0);
    const int j2 = k << 1;
    if (j2 > len) break;
    const uint32_t a2 = right ? gc.z : gc.x, b2 = right ? gc.w : gc.y;
    const bool right2 = j2 < len && zs_hkey(b2) <= zs_hkey(a2);
    const uint32_t c2 = right2 ? b2 : a2;
    if (kv <= zs_hkey(c2)) break;
    hk[k] = c2;
    k = j2 + (right2 ? 1 : 0);
    j = k << 1;
  }
  hk[k] = v;
  return top;
}

// gen_codes (trees.ts:54-76) by the wave: symbol n's code is the first code of
// its length plus the number of symbols m < n of the same length, counted
// with one ballot per length over 64 symbols at a time.  All lanes call it.
static __device__ void zs_gen_codes_wave(const uint16_t* bl_count, const uint16_t* len, uint16_t* code, int max_code,
                                         uint32_t lane) {
  uint32_t fc[16];
  uint32_t c = 0;
#pragma unroll
  for (int b = 1; b <= 15; b++) {
    c = (c + bl_count[b - 1]) << 1;
    fc[b] = c;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  for (int n0 = 0; n0 <= max_code; n0 += 64) {
    const int n = n0 + (int)lane;
    const uint32_t l = n <= max_code ? len[n] : 0u;
    uint32_t my = 0;
#pragma unroll
    for (int b = 1; b <= 15; b++) {
      const uint64_t mk = __ballot(l == (uint32_t)b);
      my = l == (uint32_t)b ? fc[b] + (uint32_t)__popcll(mk & below) : my;
      fc[b] += (uint32_t)__popcll(mk);
    }
    if (l) code[n] = (uint16_t)(__builtin_bitreverse32(my) >> (32 - l));
  }
}

// zs_gen_codes_wave for the literal/length and distance trees, written straight
// to the block's code table in HBM as code | length << 16 (0 for an unused
// symbol): all ncodes entries, so the workspace needs no code arrays
static __device__ void zs_gen_codes_out(const uint16_t* bl_count, const uint16_t* len, uint32_t* out, int max_code,
                                        int ncodes, uint32_t lane) {
  uint32_t fc[16];
  uint32_t c = 0;
#pragma unroll
  for (int b = 1; b <= 15; b++) {
    c = (c + bl_count[b - 1]) << 1;
    fc[b] = c;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  for (int n0 = 0; n0 < ncodes; n0 += 64) {
    const int n = n0 + (int)lane;
    const uint32_t l = n <= max_code ? len[n] : 0u;
    uint32_t my = 0;
#pragma unroll
    for (int b = 1; b <= 15; b++) {
      const uint64_t mk = __ballot(l == (uint32_t)b);
      my = l == (uint32_t)b ? fc[b] + (uint32_t)__popcll(mk & below) : my;
      fc[b] += (uint32_t)__popcll(mk);
    }
    if (n < ncodes) out[n] = l ? (__builtin_bitreverse32(my) >> (32 - l)) | (l << 16) : 0u;
  }
}

// the leaves in symbol order (trees.ts:276-284) by the wave: heap entry i is
// the i-th symbol with a nonzero frequency, placed by a ballot prefix; all
// lanes call it, before zs_build_tree on lane 0
static __device__ void zs_tree_leaves_wave(zs_tstate& t, zs_tdesc& d, uint32_t lane) {
  uint32_t* hk = t.hk;
  const uint64_t below = (1ull << lane) - 1ull;
  int hl = 0, max_code = -1;
  for (int n0 = 0; n0 < d.elems; n0 += 64) {
    const int n = n0 + (int)lane;
    const uint32_t f = n < d.elems ? d.freq[n] : 0u;
    const uint64_t m = __ballot(f != 0u);
    if (n < d.elems) {
      if (f) hk[hl + 1 + __popcll(m & below)] = (f << 17) | (uint32_t)n;
      else d.len[n] = 0;
    }
    if (m) max_code = n0 + 63 - (int)__clzll(m);
    hl += __popcll(m);
  }
  t.heap_len = hl;
  d.max_code = max_code;
}

// trees.ts:290-304 by the wave (after zs_tree_leaves_wave): the padding to two
// nodes (wave-uniform; lane 0 stores), then the heapify level by level from the
// deepest: the sequential n = heap_len / 2 .. 1 order sifts every deeper node
// before a shallower one, and the nodes of one level own disjoint subtrees,
// so sifting a level's nodes at once (one lane each) gives the same heap
static __device__ void zs_tree_heapify_wave(zs_tstate& t, zs_tdesc& d, uint32_t lane) {
  uint32_t* hk = t.hk;
  int max_code = d.max_code;
  while (t.heap_len < 2) {
    const int node = max_code < 2 ? ++max_code : 0;
    ++t.heap_len;
    if (lane == 0) {
      hk[t.heap_len] = (1u << 17) | (uint32_t)node;
      d.freq[node] = 1;
    }
    t.opt_len--;
    if (d.stat) t.static_len -= d.stat[node] >> 16;
  }
  d.max_code = max_code;
  __syncthreads();
  const int last = t.heap_len / 2;
  for (int lv = 31 - __clz(last); lv >= 0; lv--) {
    const int hi = min((2 << lv) - 1, last);
    for (int n = (1 << lv) + (int)lane; n <= hi; n += 64) zs_pqdownheap(t, n);
    __syncthreads();
  }
}

static __device__ void zs_build_tree(zs_tstate& t, zs_tdesc& d) {  // trees.ts:305-316, lane 0 (heap built)
  int16_t* heap = t.heap;
  uint32_t* hk = t.hk;
  int node;
  t.heap_max = t.heap_size;
  node = d.elems;
  uint32_t root = hk[1];
  do {
    const uint32_t en = root;
    const uint32_t last = hk[t.heap_len--];
    const uint32_t em = zs_pqdownheap_v(t, 1, last);
    const uint32_t nn = en & 1023u, mm = em & 1023u;
    heap[--t.heap_max] = (int16_t)nn;
    heap[--t.heap_max] = (int16_t)mm;
    const uint32_t f = (en >> 17) + (em >> 17);
    const uint32_t dn = (en >> 10) & 127u, dm = (em >> 10) & 127u;
    d.freq[node] = (uint16_t)f;
    d.dad[nn] = d.dad[mm] = (uint16_t)node;
    root = zs_pqdownheap_v(t, 1, (f << 17) | (((dn >= dm ? dn : dm) + 1) << 10) | (uint32_t)node);
    node++;
  } while (t.heap_len >= 2);
  heap[--t.heap_max] = (int16_t)(root & 1023u);
  // the bit lengths follow by the wave (zs_gen_bitlen_wave), then the codes (zs_gen_codes_wave)
}

// gen_bitlen (trees.ts:187-259) by the wave.  Without overflow a node's
// length is its depth, so the depths come from pointer jumping over dad[]
// (anc/dep in the free hk[] words, a few synchronous rounds instead of one
// dependent LDS round trip per node); lengths clamp at max_length, and
// overflow counts every non-root node deeper than max_length -- the nodes the
// serial loop clamps.  bl_count, opt_len and static_len are the same sums.
// The overflow repair (rare) stays serial on lane 0.  All lanes call it after
// zs_build_tree on lane 0 (t.heap_max, d.max_code: lane 0's).
#define ZS_GB_PER_LANE ((ZS_HEAP_SIZE + 63) / 64)
static __device__ void zs_gen_bitlen_wave(zs_tstate& t, zs_tdesc& d, uint32_t lane) {
  int16_t* heap = t.heap;
  uint16_t* bl_count = t.w->bl_count;
  uint32_t* anc = t.hk;  // free after the build: anc[node] = ancestor << 16 | depth to it
  const int hm = __builtin_amdgcn_readlane(t.heap_max, 0);
  const int max_code = __builtin_amdgcn_readlane(d.max_code, 0);
  const int root = heap[hm];
  if (lane < 16) bl_count[lane] = 0;
  int nd[ZS_GB_PER_LANE];
#pragma unroll
  for (int r = 0; r < ZS_GB_PER_LANE; r++) {
    const int h = hm + (int)lane + 64 * r;
    nd[r] = h < t.heap_size ? heap[h] : -1;
    if (nd[r] >= 0) anc[nd[r]] = nd[r] == root ? (uint32_t)root << 16 : ((uint32_t)d.dad[nd[r]] << 16) | 1u;
  }
  __syncthreads();
  for (int round = 0; round < 10; round++) {  // depth <= ZS_HEAP_SIZE < 2^10
    uint32_t nv[ZS_GB_PER_LANE];
    bool moved = false;
#pragma unroll
    for (int r = 0; r < ZS_GB_PER_LANE; r++) {
      nv[r] = 0;
      if (nd[r] < 0) continue;
      const uint32_t e = anc[nd[r]], a = e >> 16;
      if ((int)a == root) { nv[r] = e; continue; }
      const uint32_t f = anc[a];
      nv[r] = (f & 0xffff0000u) | ((e & 0xffffu) + (f & 0xffffu));
      moved = true;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ZS_GB_PER_LANE; r++)
      if (nd[r] >= 0) anc[nd[r]] = nv[r];
    __syncthreads();
    if (!__builtin_amdgcn_ballot_w64(moved)) break;
  }
  uint32_t opt = 0, stat = 0;
  int overflow = 0;
#pragma unroll
  for (int r = 0; r < ZS_GB_PER_LANE; r++) {
    const int n = nd[r];
    if (n < 0) continue;
    if (n == root) { d.len[n] = 0; continue; }
    int bits = (int)(anc[n] & 0xffffu);
    if (bits > d.max_length) { bits = d.max_length; overflow++; }
    d.len[n] = (uint16_t)bits;
    if (n > max_code) continue;
    atomicAdd(reinterpret_cast<uint32_t*>(&bl_count[bits & ~1]), 1u << (16 * (bits & 1)));
    const int xbits = n >= d.extra_base ? d.extra[n - d.extra_base] : 0;
    const uint32_t f = d.freq[n];
    opt += f * (uint32_t)(bits + xbits);
    if (d.stat) stat += f * ((d.stat[n] >> 16) + (uint32_t)xbits);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    opt += __shfl_xor(opt, o, 64);
    stat += __shfl_xor(stat, o, 64);
    overflow += __shfl_xor(overflow, o, 64);
  }
  t.opt_len += opt;
  t.static_len += stat;
  __syncthreads();
  if (overflow == 0 || lane != 0) return;
  int bits, n, m, h = t.heap_size;  // trees.ts:222-258, serial
  do {
    bits = d.max_length - 1;
    while (bl_count[bits] == 0) bits--;
    bl_count[bits]--;
    bl_count[bits + 1] += 2;
    bl_count[d.max_length]--;
    overflow -= 2;
  } while (overflow > 0);
  for (bits = d.max_length; bits != 0; bits--) {
    n = bl_count[bits];
    while (n != 0) {
      m = heap[--h];
      if (m > d.max_code) continue;
      if (d.len[m] != bits) {
        t.opt_len += (uint32_t)((bits - (int)d.len[m]) * (int)d.freq[m]);
        d.len[m] = (uint16_t)bits;
      }
      n--;
    }
  }
}

static __device__ __forceinline__ void zs_hput(zs_tstate& t, uint32_t v, int n) {
  uint32_t* h = t.w->hdr;
  const uint32_t pos = t.hbits;
  h[pos >> 5] |= v << (pos & 31);
  if ((pos & 31) + n > 32) h[(pos >> 5) + 1] |= v >> (32 - (pos & 31));
  t.hbits += n;
}

// ---- scan_tree / send_tree (trees.ts:318-414) over maximal runs, one lane per
// run.  The serial automaton's chunking of a run of r equal lengths v depends
// on (v, r) alone: entering a run the state is always (max, min) = (138, 3)
// for v = 0 and (7, 4) otherwise (the previous length differs), and inside a
// run it is (138, 3) for zeros and (6, 3) otherwise, with prevlen = v after
// the first chunk.  So each run's codes (symbol, extra value, extra bits) are
// enumerated by its own lane: frequencies by LDS atomics, the header bits at
// the run's offset from a prefix sum over the runs in index order.
template <class F>
static __device__ __forceinline__ void zs_run_codes(uint32_t v, uint32_t r, F&& f) {
  if (v == 0) {
    while (r) {
      const uint32_t c = r < 138u ? r : 138u;
      r -= c;
      if (c < 3) for (uint32_t k = 0; k < c; k++) f(0u, 0u, 0u);
      else if (c <= 10) f(17u, c - 3u, 3u);
      else f(18u, c - 11u, 7u);
    }
  } else {
    uint32_t c = r < 7u ? r : 7u;
    r -= c;
    if (c < 4) for (uint32_t k = 0; k < c; k++) f(v, 0u, 0u);
    else { f(v, 0u, 0u); f(16u, c - 4u, 2u); }
    while (r) {
      c = r < 6u ? r : 6u;
      r -= c;
      if (c < 3) for (uint32_t k = 0; k < c; k++) f(v, 0u, 0u);
      else f(16u, c - 3u, 2u);
    }
  }
}
// lane's run in the 64-index chunk at n0 of len[0..max_code] (guard len[max_code + 1] = 0xffff already
// set): returns true with (v, r) if index n0 + lane starts a run
static __device__ __forceinline__ bool zs_run_at(const uint16_t* len, int max_code, int n0, uint32_t lane,
                                                 uint32_t& v, uint32_t& r) {
  const int n = n0 + (int)lane;
  if (n > max_code) return false;
  v = len[n];
  if (n > 0 && len[n - 1] == v) return false;
  // the run's end (the guard ends every run): eight lengths per LDS read where
  // aligned -- a run of unused symbols is often a hundred long (len is 16-byte
  // aligned and holds max_code + 9 entries or more)
  int m = n + 1;
  const uint32_t vv = v | (v << 16);
  for (;;) {
    if ((m & 7) == 0) {
      const uint4 q = *reinterpret_cast<const uint4*>(&len[m]);
      if (q.x == vv && q.y == vv && q.z == vv && q.w == vv) {
        m += 8;
        continue;
      }
    }
    if (len[m] != v) break;
    m++;
  }
  r = (uint32_t)(m - n);
  return true;
}
// all lanes: scan_tree's bl_tree frequencies of one tree, added to b32[]
static __device__ void zs_scan_tree_wave(const uint16_t* len, int max_code, uint32_t* b32, uint32_t lane) {
  for (int n0 = 0; n0 <= max_code; n0 += 64) {
    uint32_t v = 0, r = 0;
    if (zs_run_at(len, max_code, n0, lane, v, r))
      zs_run_codes(v, r, [&](uint32_t sym, uint32_t, uint32_t) { atomicAdd(&b32[sym], 1u); });
  }
}
// all lanes: send_tree's header bits of one tree at bit `base` of hdr[] (zeroed); returns the end bit
static __device__ uint32_t zs_send_tree_wave(const uint16_t* len, int max_code, const uint16_t* bc, const uint16_t* bl,
                                             uint32_t* hdr, uint32_t base, uint32_t lane) {
  for (int n0 = 0; n0 <= max_code; n0 += 64) {
    uint32_t v = 0, r = 0, bits = 0;
    const bool st = zs_run_at(len, max_code, n0, lane, v, r);
    if (st) zs_run_codes(v, r, [&](uint32_t sym, uint32_t, uint32_t xb) { bits += bl[sym] + xb; });
    uint32_t incl = bits;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    uint32_t pos = base + incl - bits;
    auto put = [&](uint32_t val, uint32_t nb) {
      if (nb == 0) return;
      atomicOr(&hdr[pos >> 5], val << (pos & 31u));
      if ((pos & 31u) + nb > 32u) atomicOr(&hdr[(pos >> 5) + 1], val >> (32u - (pos & 31u)));
      pos += nb;
    };
    if (st)
      zs_run_codes(v, r, [&](uint32_t sym, uint32_t xv, uint32_t xb) {
        put(bc[sym], bl[sym]);
        put(xv, xb);
      });
    base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  }
  return base;
}

#ifndef ZS_HIST_INFLIGHT
#define ZS_HIST_INFLIGHT 32u  // histogram: symbol loads in flight per lane before their atomics
#endif
#ifndef ZS_TR_PROF
#define ZS_TR_PROF 0  // timing experiments: wall-clock per phase summed over blocks (0 in the product)
#endif
#if ZS_TR_PROF
__device__ unsigned long long zs_tr_stat[8];  // histogram, L heap, L lengths + codes, D tree, bl tree, rest, blocks
extern "C" int zs_trees_stats(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(zs_tr_stat), sizeof(zs_tr_stat));
}
#define TR_MARK(i) do { if (threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); atomicAdd(&zs_tr_stat[i], t_ - tr_t); tr_t = t_; } } while (0)
#else
#define TR_MARK(i) do { } while (0)
#endif
__global__ __launch_bounds__(64) void zs_k_trees(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                 const uint64_t* __restrict__ pos_base,
                                                 const uint32_t* __restrict__ blk_base,
                                                 const uint32_t* __restrict__ syms, zs_block* __restrict__ blocks,
                                                 const zs_stream* __restrict__ streams, uint32_t* __restrict__ codes,
                                                 uint32_t* __restrict__ hdr, int nstreams) {
  __shared__ zs_tw w;
  const int s = blockIdx.y;
  const uint32_t b = blockIdx.x;
  if (b >= streams[s].nblk) return;
  const uint32_t bi = blk_base[s] + b;
  zs_block blk = blocks[bi];
  const uint32_t lane = threadIdx.x;
  const uint32_t* sy = syms + pos_base[s] + s + blk.sym_start;
#if ZS_TR_PROF
  unsigned long long tr_t = wall_clock64();
  if (threadIdx.x == 0) atomicAdd(&zs_tr_stat[7], 1ull);
#endif
  uint32_t* const hist = w.hk + 192;  // the histogram: hk past the code maps, free until the heap
  static_assert(sizeof(w.hk) >= 4 * (192 + ZS_L_CODES + ZS_D_CODES), "histogram in hk");
  for (uint32_t i = lane; i < ZS_L_CODES + ZS_D_CODES; i += 64) hist[i] = 0;
  for (uint32_t i = lane; i < ZS_HDR_WORDS; i += 64) w.hdr[i] = 0;
  // the length and distance code maps in LDS (the histogram's lookups would
  // otherwise be a memory round trip each, behind the symbol's own load)
  uint8_t* const lcode8 = reinterpret_cast<uint8_t*>(w.hk);  // hk is free until the heap
  uint8_t* const dcode8 = lcode8 + 256;
  static_assert(sizeof(w.hk) >= 768, "code maps in hk");
  for (uint32_t i = lane; i < 256; i += 64) lcode8[i] = ZS_LENGTH_CODE[i];
  for (uint32_t i = lane; i < 512; i += 64) dcode8[i] = ZS_DIST_CODE[i];
  __syncthreads();
  // histogram (deflate/utils.ts:55-81 tallies, done in parallel); ZS_HIST_INFLIGHT
  // symbol loads in flight per lane before their atomics, so the wave waits for
  // memory once per 64 * ZS_HIST_INFLIGHT symbols rather than once per 64
  for (uint32_t i0 = 0; i0 < blk.sym_count; i0 += 64 * ZS_HIST_INFLIGHT) {
    uint32_t v[ZS_HIST_INFLIGHT];
#pragma unroll
    for (uint32_t k = 0; k < ZS_HIST_INFLIGHT; k++) {
      const uint32_t i = i0 + 64 * k + lane;
      v[k] = i < blk.sym_count ? sy[i] : 0xffffffffu;
    }
#pragma unroll
    for (uint32_t k = 0; k < ZS_HIST_INFLIGHT; k++) {
      if (v[k] == 0xffffffffu) continue;
      if (v[k] & 0x80000000u) {
        const uint32_t lc = (v[k] >> 16) & 0xff, dist = (v[k] & 0xffffu) - 1;
        atomicAdd(&hist[lcode8[lc] + 257u], 1u);
        atomicAdd(&hist[ZS_L_CODES + dcode8[dist < 256 ? dist : 256 + (dist >> 7)]], 1u);
      } else {
        atomicAdd(&hist[v[k]], 1u);
      }
    }
  }
  __syncthreads();
  // init_block (trees.ts:90-103) + tally counts
  for (uint32_t i = lane; i < ZS_L_CODES + ZS_D_CODES; i += 64) w.tally[i] = (uint16_t)hist[i];  // <= 16,383
  for (uint32_t i = lane; i < ZS_L_CODES; i += 64) w.lfreq[i] = i == ZS_END_BLOCK ? 1 : (uint16_t)hist[i];
  for (uint32_t i = lane; i < ZS_D_CODES; i += 64) w.dfreq[i] = (uint16_t)hist[ZS_L_CODES + i];
  if (lane < ZS_BL_CODES) w.bfreq[lane] = 0;
  __syncthreads();
  TR_MARK(0);
  // the serial parts run in lane 0 (its registers hold t and the max codes),
  // the code assignment in the whole wave between them
  zs_tstate t;
  t.w = &w;
  t.hk = w.hk;
  t.heap = w.heap;
  t.heap_size = ZS_HEAP_SIZE;
  t.opt_len = 0;
  t.static_len = 0;
  t.hbits = 0;
  zs_tdesc L = {w.lfreq, w.llen, w.ldad, nullptr, ZS_STATIC_LTREE, ZS_EXTRA_LBITS, 257, ZS_L_CODES, 15, 0};
  zs_tdesc D = {w.dfreq, w.dlen, w.ddad, nullptr, ZS_STATIC_DTREE, ZS_EXTRA_DBITS, 0, ZS_D_CODES, 15, 0};
  uint32_t* const cout = codes + (size_t)bi * (ZS_L_CODES + ZS_D_CODES);  // (used by emit for dynamic blocks only)
  zs_tdesc B = {w.bfreq, w.blen, w.bdad, w.bcode, nullptr, nullptr, 0, ZS_BL_CODES, 7, 0};
  B.extra = ZS_EXTRA_BLBITS;
  // the literal/length and distance trees are independent until the bl tree:
  // their heaps are built at once, lane 0 the first and lane 1 the second (one
  // instruction stream, per-lane arrays), their sums added after
  zs_tstate td = t;
  td.hk = w.hkd;
  td.heap = w.heapd;
  td.heap_size = 2 * ZS_D_CODES + 1;
  td.opt_len = 0;
  td.static_len = 0;
  zs_tree_leaves_wave(t, L, lane);
  __syncthreads();
  zs_tree_heapify_wave(t, L, lane);
  zs_tree_leaves_wave(td, D, lane);
  __syncthreads();
  zs_tree_heapify_wave(td, D, lane);
  {
    int hm = 0;
    if (lane < 2) {
      zs_tstate tt = lane ? td : t;
      zs_tdesc dd = lane ? D : L;
      zs_build_tree(tt, dd);
      hm = tt.heap_max;
    }
    t.heap_max = __builtin_amdgcn_readlane(hm, 0);
    td.heap_max = __builtin_amdgcn_readlane(hm, 1);
  }
  __syncthreads();
  TR_MARK(1);
  zs_gen_bitlen_wave(t, L, lane);
  __syncthreads();
  zs_gen_codes_out(w.bl_count, w.llen, cout, __builtin_amdgcn_readlane(L.max_code, 0), ZS_L_CODES, lane);
  __syncthreads();
  TR_MARK(2);
  zs_gen_bitlen_wave(td, D, lane);
  __syncthreads();
  zs_gen_codes_out(w.bl_count, w.dlen, cout + ZS_L_CODES, __builtin_amdgcn_readlane(D.max_code, 0), ZS_D_CODES, lane);
  __syncthreads();
  t.opt_len += td.opt_len;
  t.static_len += td.static_len;
  TR_MARK(3);
  // build_bl_tree (trees.ts:416-432): scan_tree of both trees by runs (all lanes), then the tree (lane 0)
  const int lmax = __builtin_amdgcn_readlane(L.max_code, 0), dmax = __builtin_amdgcn_readlane(D.max_code, 0);
  if (lane < 32) w.b32[lane] = 0;
  if (lane == 0) {
    w.llen[lmax + 1] = 0xffff;  // scan_tree's guards (trees.ts:328), read by send_tree too
    w.dlen[dmax + 1] = 0xffff;
  }
  __syncthreads();
  zs_scan_tree_wave(w.llen, lmax, w.b32, lane);
  zs_scan_tree_wave(w.dlen, dmax, w.b32, lane);
  __syncthreads();
  if (lane < ZS_BL_CODES) w.bfreq[lane] = (uint16_t)(w.bfreq[lane] + w.b32[lane]);
  __syncthreads();
  zs_tree_leaves_wave(t, B, lane);
  __syncthreads();
  zs_tree_heapify_wave(t, B, lane);
  if (lane == 0) zs_build_tree(t, B);
  __syncthreads();
  zs_gen_bitlen_wave(t, B, lane);
  __syncthreads();
  zs_gen_codes_wave(w.bl_count, w.blen, w.bcode, __builtin_amdgcn_readlane(B.max_code, 0), lane);
  __syncthreads();
  if (lane == 0) {
    int max_blindex;
    for (max_blindex = ZS_BL_CODES - 1; max_blindex >= 3; max_blindex--)
      if (w.blen[ZS_BL_ORDER[max_blindex]] != 0) break;
    t.opt_len += 3u * ((uint32_t)max_blindex + 1) + 5 + 5 + 4;
    uint32_t opt_lenb = (t.opt_len + 3 + 7) >> 3;
    const uint32_t static_lenb = (t.static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    const uint32_t stored_len = blk.in_end - blk.in_start;
    uint32_t type;
    if (stored_len + 4 <= opt_lenb) type = 0;
    else if (static_lenb == opt_lenb) type = 1;
    else type = 2;
    if (type == 2) {
      // send_all_trees (trees.ts:434-447): the counts and the bl_tree lengths here, the two trees by all lanes
      const int lcodes = L.max_code + 1, dcodes = D.max_code + 1, blcodes = max_blindex + 1;
      zs_hput(t, (uint32_t)(lcodes - 257), 5);
      zs_hput(t, (uint32_t)(dcodes - 1), 5);
      zs_hput(t, (uint32_t)(blcodes - 4), 4);
      for (int rank = 0; rank < blcodes; rank++) zs_hput(t, w.blen[ZS_BL_ORDER[rank]], 3);
    }
    w.bc[0] = type;
    w.bc[1] = t.hbits;
  }
  __syncthreads();
  TR_MARK(4);
  const uint32_t type = w.bc[0];
  uint32_t hbits = w.bc[1];
  if (type == 2) {
    hbits = zs_send_tree_wave(w.llen, lmax, w.bcode, w.blen, w.hdr, hbits, lane);
    hbits = zs_send_tree_wave(w.dlen, dmax, w.bcode, w.blen, w.hdr, hbits, lane);
    __syncthreads();
  }
  // exact payload bits of the chosen coding, from the true counts
  uint32_t data_bits = 0;
  if (type != 0) {
    for (uint32_t i = lane; i < ZS_L_CODES; i += 64) {
      const uint32_t f = i == ZS_END_BLOCK ? 1u : w.tally[i];
      const uint32_t len = type == 1 ? ZS_STATIC_LTREE[i] >> 16 : w.llen[i];
      if (f) data_bits += f * (len + (i >= 257 ? (uint32_t)ZS_EXTRA_LBITS[i - 257] : 0u));
    }
    if (lane < ZS_D_CODES) {
      const uint32_t f = w.tally[ZS_L_CODES + lane];
      const uint32_t len = type == 1 ? 5u : w.dlen[lane];
      if (f) data_bits += f * (len + (uint32_t)ZS_EXTRA_DBITS[lane]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) data_bits += __shfl_xor(data_bits, d, 64);
  }
  if (type == 2) {
    uint32_t* hout = hdr + (size_t)bi * ZS_HDR_WORDS;
    for (uint32_t i = lane; i < (hbits + 31) / 32; i += 64) hout[i] = w.hdr[i];
  }
  if (lane == 0) {
    blk.type = type;
    blk.hdr_bits = type == 2 ? hbits : 0;
    blk.data_bits = data_bits;
    blocks[bi] = blk;
  }
  TR_MARK(5);
}

// --------------------------------------------------------------- layout
__global__ void zs_k_layout(const uint32_t* __restrict__ blk_base, zs_block* __restrict__ blocks,
                            zs_stream* __restrict__ streams, const uint32_t* __restrict__ out_cap,
                            uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, int wrap, int nstreams) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  zs_stream st = streams[s];
  const uint32_t hl = wrap == 1 ? 2u : wrap == 2 ? 10u : 0u, tl = wrap == 1 ? 4u : wrap == 2 ? 8u : 0u;
  uint64_t off = (uint64_t)hl * 8;
  zs_block* blk = blocks + blk_base[s];
  int bad = 0;
  for (uint32_t b = 0; b < st.nblk; b++) {
    zs_block k = blk[b];
    k.bit_off = off;
    if (k.type == 0) {
      if (k.last & 2u) bad = 1;  // stored block starting before the slid window: not reproducible
      off += 3;
      off = (off + 7) & ~7ull;
      off += 32 + 8ull * (k.in_end - k.in_start);
    } else {
      off += 3 + k.hdr_bits + k.data_bits;
    }
    k.bit_end = off;
    if (k.last & 1u) off = (off + 7) & ~7ull;  // bi_windup (trees.ts:587-589)
    blk[b] = k;
  }
  st.total_bits = off;
  const uint64_t out_len = off / 8 + tl;
  st.out_len = (uint32_t)out_len;
  st.status = bad ? ZS_Z_STREAM_ERROR : (out_len <= out_cap[s] ? ZS_Z_STREAM_END : ZS_Z_BUF_ERROR);
  streams[s] = st;
  if (st.status != ZS_Z_STREAM_END) return;
  // zero the words written by more than one writer (atomic OR targets)
  uint32_t* ow = (uint32_t*)(out + out_off[s]);
  for (uint32_t i = 0; i < (hl + 3) / 4; i++) ow[i] = 0;
  for (uint32_t b = 0; b < st.nblk; b++) {
    const zs_block k = blk[b];
    ow[k.bit_off >> 5] = 0;
    ow[(k.bit_end - 1) >> 5] = 0;
  }
  const uint64_t tb = off / 8;
  for (uint64_t by = tb > 0 ? tb - 1 : 0; by < (out_len + 3) / 4 * 4; by += 4) ow[by >> 2] = 0;
}

// -------------------------------------------------------------------- emit
#define ZS_EMIT_THREADS 256
#ifndef ZS_EMIT_PER_THREAD
#define ZS_EMIT_PER_THREAD 4  // symbols per thread and chunk (A/B: 2, 8, 16)
#endif
// the stage holds the block header, the dynamic tree header and one chunk's
// bits (at most 15 + 5 + 15 + 13 = 48 per symbol) past the carried word
#define ZS_STAGE_WORDS (ZS_HDR_WORDS + 2 + ZS_EMIT_THREADS * ZS_EMIT_PER_THREAD * 48 / 32)
static_assert(ZS_EMIT_THREADS == 256, "zs_k_emit builds its 256-entry length table one entry per thread");

static __device__ __forceinline__ uint32_t zs_block_scan(uint32_t v, uint32_t* tmp, uint32_t& total) {
  // exclusive scan over the 256-thread workgroup (one barrier: the caller's
  // later barriers keep tmp from being rewritten while it is read)
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) tmp[wv] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (uint32_t i = 0; i < wv; i++) pre += tmp[i];
  total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  return pre + x - v;
}

static __device__ __forceinline__ void zs_stage_or(uint32_t* st, uint64_t rel, uint64_t v, uint32_t n) {
  if (!n) return;
  const uint32_t wi = (uint32_t)(rel >> 5), sh = (uint32_t)(rel & 31);
  atomicOr(&st[wi], (uint32_t)(v << sh));
  if (sh + n > 32) atomicOr(&st[wi + 1], (uint32_t)(v >> (32 - sh)));
  if (sh + n > 64) atomicOr(&st[wi + 2], (uint32_t)(v >> (64 - sh)));
}

__global__ __launch_bounds__(ZS_EMIT_THREADS) void zs_k_emit(
    const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off, const uint64_t* __restrict__ pos_base,
    const uint32_t* __restrict__ blk_base, const uint32_t* __restrict__ syms, const zs_block* __restrict__ blocks,
    const zs_stream* __restrict__ streams, const uint32_t* __restrict__ codes, const uint32_t* __restrict__ hdr,
    uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off, int wrap) {
  __shared__ uint32_t stage[ZS_STAGE_WORDS + 4];
  __shared__ uint32_t tbl[ZS_L_CODES + ZS_D_CODES];
  __shared__ uint32_t ltab[256];
  __shared__ uint2 dt[ZS_D_CODES];
  __shared__ uint8_t dcode[512];
  __shared__ uint32_t scan_tmp[4];
  const int s = blockIdx.y;
  const uint32_t b = blockIdx.x;
  const zs_stream st = streams[s];
  if (b >= st.nblk || st.status != ZS_Z_STREAM_END) return;
  const uint32_t bi = blk_base[s] + b;
  const zs_block blk = blocks[bi];
  uint32_t* ow = (uint32_t*)(out + out_off[s]);
  const uint64_t off0 = blk.bit_off, off1 = blk.bit_end;
  const uint64_t first_w = off0 >> 5, last_w = (off1 - 1) >> 5;
  const bool first_shared = (off0 & 31) != 0, last_shared = (off1 & 31) != 0;
  auto put_word = [&](uint64_t gw, uint32_t v) {
    if ((gw == first_w && first_shared) || (gw == last_w && last_shared)) {
      if (v) atomicOr(&ow[gw], v);
    } else {
      ow[gw] = v;
    }
  };
  const uint32_t hdr3 = (blk.type << 1) | (blk.last & 1u);  // block header (trees.ts:449-451,578,581)

  if (blk.type == 0) {  // stored block: every word computed independently (trees.ts:449-464)
    const uint8_t* src = in + in_off[s] + blk.in_start;
    const uint32_t slen = blk.in_end - blk.in_start;
    const uint64_t B0 = ((off0 + 3 + 7) & ~7ull) >> 3;  // first byte after bi_windup
    const uint64_t B1 = B0 + 4 + slen;
    for (uint64_t gw = first_w + threadIdx.x; gw <= last_w; gw += ZS_EMIT_THREADS) {
      uint32_t v = 0;
      if (gw == first_w) v |= hdr3 << (off0 & 31);
      for (uint32_t k = 0; k < 4; k++) {
        const uint64_t by = gw * 4 + k;
        if (by < B0 || by >= B1) continue;
        const uint64_t r = by - B0;
        uint32_t c;
        if (r < 2) c = (slen >> (8 * r)) & 0xff;
        else if (r < 4) c = (~slen >> (8 * (r - 2))) & 0xff;
        else c = src[r - 4];
        v |= c << (8 * k);
      }
      put_word(gw, v);
    }
    return;
  }

  // Huffman-coded block.  The thread's symbols of the first chunk are loaded
  // before the tables are set up, and each chunk's loads are issued before the
  // previous chunk is coded (PT consecutive symbols per thread).
  constexpr uint32_t PT = ZS_EMIT_PER_THREAD, chunk = ZS_EMIT_THREADS * PT;
  const uint32_t* sy = syms + pos_base[s] + s + blk.sym_start;
  const uint32_t nsym = blk.sym_count;
  uint32_t nx[PT];
  auto fetch = [&](uint32_t c0) __attribute__((always_inline)) {
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) {
      const uint32_t i = c0 + threadIdx.x * PT + k;
      nx[k] = i < nsym ? sy[i] : 0u;
    }
  };
  fetch(0);
  const uint32_t* ctab = codes + (size_t)bi * (ZS_L_CODES + ZS_D_CODES);
  for (uint32_t i = threadIdx.x; i < ZS_L_CODES + ZS_D_CODES; i += ZS_EMIT_THREADS) {
    if (blk.type == 1) tbl[i] = i < ZS_L_CODES ? ZS_STATIC_LTREE[i] : ZS_STATIC_DTREE[i - ZS_L_CODES];
    else tbl[i] = ctab[i];
  }
  for (uint32_t i = threadIdx.x; i < 512; i += ZS_EMIT_THREADS) dcode[i] = ZS_DIST_CODE[i];
  for (uint32_t i = threadIdx.x; i < ZS_STAGE_WORDS + 4; i += ZS_EMIT_THREADS) stage[i] = 0;
  __syncthreads();
  // a match's codes from LDS: ltab[lc] = the length code's bits and its extra
  // bits (<= 20) | their count << 24; dt[dc] = the distance code's bits | its
  // length << 16 | extra bits << 24, and the code's base distance
  {
    const uint32_t lc = threadIdx.x;  // ZS_EMIT_THREADS == 256 lengths
    const uint32_t code = ZS_LENGTH_CODE[lc];
    const uint32_t e1 = tbl[code + 257];
    const uint32_t xl = (uint32_t)ZS_EXTRA_LBITS[code];
    // code 285 (length 258) has no extra bits: lc - base must not leak (trees.ts:495-499)
    const uint32_t xv = (lc - (uint32_t)ZS_BASE_LENGTH[code]) & ((1u << xl) - 1u);
    ltab[lc] = ((e1 & 0xffffu) | (xv << (e1 >> 16))) | (((e1 >> 16) + xl) << 24);
    if (lc < ZS_D_CODES) {
      const uint32_t e2 = tbl[ZS_L_CODES + lc];
      dt[lc] = make_uint2((e2 & 0xffffu) | ((e2 >> 16) << 16) | ((uint32_t)ZS_EXTRA_DBITS[lc] << 24),
                          (uint32_t)ZS_BASE_DIST[lc]);
    }
  }
  uint64_t wbase = first_w;  // global word index of stage[0]
  uint64_t pos = off0;
  if (threadIdx.x == 0) zs_stage_or(stage, pos - wbase * 32, hdr3, 3);
  pos += 3;
  if (blk.type == 2) {
    const uint32_t* hsrc = hdr + (size_t)bi * ZS_HDR_WORDS;
    const uint32_t hw = (blk.hdr_bits + 31) / 32;
    for (uint32_t i = threadIdx.x; i < hw; i += ZS_EMIT_THREADS) {
      const uint32_t nb = min(32u, blk.hdr_bits - 32 * i);
      const uint32_t v = nb == 32 ? hsrc[i] : (hsrc[i] & ((1u << nb) - 1));
      zs_stage_or(stage, pos - wbase * 32 + 32 * i, v, nb);
    }
    pos += blk.hdr_bits;
  }
  __syncthreads();
  for (uint32_t c0 = 0;; c0 += chunk) {
    const bool final_chunk = c0 + chunk >= nsym;
    uint32_t x[PT];
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) x[k] = nx[k];
    if (!final_chunk) fetch(c0 + chunk);
    uint64_t v[PT];
    uint32_t n[PT];
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) {
      const uint32_t i = c0 + threadIdx.x * PT + k;
      v[k] = 0;
      n[k] = 0;
      if (i < nsym) {
        if (x[k] & 0x80000000u) {  // compress_block (trees.ts:476-520)
          const uint32_t lc = (x[k] >> 16) & 0xff, dist = (x[k] & 0xffffu) - 1;
          const uint32_t le = ltab[lc];
          const uint2 de = dt[dcode[dist < 256 ? dist : 256 + (dist >> 7)]];
          uint32_t nb = le >> 24;
          uint64_t acc = le & 0xffffffu;
          acc |= (uint64_t)(de.x & 0xffffu) << nb;
          nb += (de.x >> 16) & 0xffu;
          acc |= (uint64_t)(dist - de.y) << nb;
          nb += de.x >> 24;
          v[k] = acc;
          n[k] = nb;
        } else {
          const uint32_t e = tbl[x[k]];
          v[k] = e & 0xffffu;
          n[k] = e >> 16;
        }
      }
      tot += n[k];
    }
    uint32_t total;
    const uint32_t pre = zs_block_scan(tot, scan_tmp, total);
    uint64_t rel = pos - wbase * 32 + pre;
#pragma unroll
    for (uint32_t k = 0; k < PT; k++) {
      zs_stage_or(stage, rel, v[k], n[k]);
      rel += n[k];
    }
    pos += total;
    if (final_chunk && threadIdx.x == 0) {  // END_BLOCK
      const uint32_t e = tbl[ZS_END_BLOCK];
      zs_stage_or(stage, pos - wbase * 32, e & 0xffffu, e >> 16);
    }
    if (final_chunk) pos += tbl[ZS_END_BLOCK] >> 16;
    __syncthreads();
    // write out complete words; keep the partial one
    const uint64_t done_w = final_chunk ? ((pos + 31) >> 5) : (pos >> 5);
    const uint32_t nw = (uint32_t)(done_w - wbase);
    for (uint32_t i = threadIdx.x; i < nw; i += ZS_EMIT_THREADS) put_word(wbase + i, stage[i]);
    if (final_chunk) break;
    const uint32_t carry = stage[nw];
    __syncthreads();
    // only words 0 .. nw were written (no bit lies past pos): clear those, the
    // partial one moved to the front (the next scan's barrier orders it before
    // the next chunk's ORs)
    for (uint32_t i = threadIdx.x; i <= nw; i += ZS_EMIT_THREADS) stage[i] = i == 0 ? carry : 0u;
    wbase = done_w;
  }
}

// -------------------------------------------------------------------- wrap
__global__ void zs_k_wrap(const zs_stream* __restrict__ streams, uint8_t* __restrict__ out,
                          const uint64_t* __restrict__ out_off, const uint32_t* __restrict__ in_len, int wrap,
                          int level, int nstreams) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams || wrap == 0) return;
  const zs_stream st = streams[s];
  if (st.status != ZS_Z_STREAM_END) return;
  uint32_t* ow = (uint32_t*)(out + out_off[s]);
  auto put_byte = [&](uint64_t at, uint32_t c) { atomicOr(&ow[at >> 2], (c & 0xffu) << (8 * (at & 3))); };
  const uint64_t tb = st.total_bits / 8;
  if (wrap == 1) {  // zlib: deflate.ts:753-786, 980-983
    uint32_t header = (8u + ((15u - 8u) << 4)) << 8;
    const uint32_t lf = level < 2 ? 0u : level < 6 ? 1u : level == 6 ? 2u : 3u;
    header |= lf << 6;
    header += 31 - (header % 31);
    put_byte(0, header >> 8);
    put_byte(1, header);
    for (int i = 0; i < 4; i++) put_byte(tb + i, st.check >> (24 - 8 * i));
  } else {  // gzip: deflate.ts:787-806, 971-979
    const uint32_t xfl = level == 9 ? 2u : level < 2 ? 4u : 0u;
    const uint8_t h[10] = {31, 139, 8, 0, 0, 0, 0, 0, (uint8_t)xfl, 255};
    for (int i = 0; i < 10; i++) put_byte(i, h[i]);
    for (int i = 0; i < 4; i++) put_byte(tb + i, st.check >> (8 * i));
    for (int i = 0; i < 4; i++) put_byte(tb + 4 + i, in_len[s] >> (8 * i));
  }
}

// ------------------------------------------------------------------- level 0
// deflate_stored (deflate.ts:1140-1279) under the stream layer's call pattern
// (streams.ts:78-93: 32 KiB input sub-chunks per deflate(Z_NO_FLUSH) call, each
// with a fresh 64 KiB output buffer, then deflate(Z_FINISH)): every full
// sub-chunk leaves as one 32768-byte stored block copied straight from the
// input, and Z_FINISH emits the remainder (possibly empty) as the last block.
// The layout is a function of the length alone (pinned for 0..1 MiB against the
// reference: tests/golden/deflate_level0.json), so each thread writes four
// output words, mapping every output byte to a header byte or an input byte.
__global__ __launch_bounds__(256) void zs_k_stored(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint32_t* __restrict__ in_len, uint8_t* __restrict__ out,
                                                   const uint64_t* __restrict__ out_off,
                                                   const uint32_t* __restrict__ out_cap,
                                                   const uint32_t* __restrict__ check, int wrap, int32_t* status,
                                                   uint32_t* out_len_res) {
  const uint32_t s = blockIdx.y;
  const uint32_t n = in_len[s];
  const uint32_t hl = wrap == 0 ? 0 : wrap == 1 ? 2 : 10, tl = wrap == 0 ? 0 : wrap == 1 ? 4 : 8;
  const uint32_t nblk = n / ZS_STORED_CHUNK + 1;
  const uint64_t body = 5ull * nblk + n;
  const uint64_t total = hl + body + tl;
  const bool fits = total <= out_cap[s];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    status[s] = fits ? ZS_Z_STREAM_END : ZS_Z_BUF_ERROR;
    out_len_res[s] = fits ? (uint32_t)total : 0u;  // as zs_k_finish: failed streams produce nothing
  }
  if (!fits) return;
  const uint8_t* src = in + in_off[s];
  uint32_t* ow = (uint32_t*)(out + out_off[s]);
  const uint32_t ck = wrap ? check[s] : 0;
  const uint32_t xfl = 4u;  // level < 2 (deflate.ts:795)
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) {
    const uint64_t w = w0 + q;
    if (4 * w >= total) break;
    uint32_t word = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint64_t o = 4 * w + j;
      uint32_t b = 0;
      if (o >= total) {
        b = 0;
      } else if (o < hl) {
        if (wrap == 1) b = o == 0 ? 0x78u : 0x01u;  // level_flags 0 (deflate.ts:757-771)
        else b = o == 0 ? 31u : o == 1 ? 139u : o == 2 ? 8u : o == 8 ? xfl : o == 9 ? 255u : 0u;
      } else if (o < hl + body) {
        const uint64_t r = o - hl;
        const uint32_t k = (uint32_t)(r / (ZS_STORED_CHUNK + 5)), p = (uint32_t)(r % (ZS_STORED_CHUNK + 5));
        const uint32_t len = k + 1 == nblk ? n - k * ZS_STORED_CHUNK : ZS_STORED_CHUNK;
        if (p == 0) b = k + 1 == nblk ? 1u : 0u;  // BFINAL, BTYPE 00, then byte alignment
        else if (p < 3) b = (len >> (8 * (p - 1))) & 0xffu;
        else if (p < 5) b = (~len >> (8 * (p - 3))) & 0xffu;
        else b = src[(uint64_t)k * ZS_STORED_CHUNK + p - 5];
      } else {
        const uint32_t t = (uint32_t)(o - hl - body);
        if (wrap == 1) b = (ck >> (24 - 8 * t)) & 0xffu;                        // adler32, big-endian
        else b = t < 4 ? (ck >> (8 * t)) & 0xffu : (n >> (8 * (t - 4))) & 0xffu;  // crc32, ISIZE
      }
      word |= b << (8 * j);
    }
    ow[w] = word;
  }
}
