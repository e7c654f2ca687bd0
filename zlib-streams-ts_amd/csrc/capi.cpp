// capi.cpp -- the C-ABI host layer of libzsgpu.so (include/zs_gpu.h).
//
// Owns one device context per GPU: a HIP stream, a growable device workspace
// and the launch sequence of the batch engines.  No torch types cross this
// boundary; callers hand in plain pointers (device or host) and sizes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zs_gpu.h"
#include "zs_common.h"
#include "zs_kernels.h"
#include "zs_inflate.h"
#include "zs_split.h"
#include "zs_seg.h"


namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, const char* a = "") {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, a);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                          \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) return fail(ZS_MEM_ERROR, "%s", hipGetErrorString(e_)); \
  } while (0)

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 8, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// pinned host staging (grows on demand, reused across calls)
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

const zs_level_cfg kLevels[10] = {{0, 0, 0, 0},     {4, 4, 8, 4},     {4, 5, 16, 8},     {4, 6, 32, 32},
                                  {4, 4, 16, 16},   {8, 16, 32, 32},  {8, 16, 128, 128}, {8, 32, 128, 256},
                                  {32, 128, 258, 1024}, {32, 258, 258, 4096}};  // deflate.ts:86-103

}  // namespace

void zs_set_last_error(const std::string& msg) { g_err = msg; }

#define ZS_PARSE2W_AUTO 2048u  // batches below this many streams parse with two waves per stream (option parse_waves = 0)

struct zs_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool timing = false;
  bool check_phases = false;  // synchronise after every phase and name the one that failed
  // workspace
  Buf meta, prevd, mres, syms, blocks, streams, codes, hdr, check, istate, pscr, ltabs, lres, llen, lstat;
  bool inflate_fast = true;
  bool inflate_ref_wrap = true;  // reproduce the reference's inflate_fast window-wrap copy (inffast.ts:133-147)
  bool match_sweep = true;   // 0: the chain-walk kernels for every stream (a cross-check of the sweep)
  int lane_block = 0;        // members per workgroup of the inflate lane path (0: chosen from the batch size)
  int cur_pw = 1;            // waves per stream of the current deflate batch's parse (zs_k_parse / _2w / _4w)
  int parse_waves = 0;       // L4..9 one-wave parse: waves per stream (1, 2; 0: chosen from the batch size)
  std::vector<uint32_t> hwin0;  // the sweep's windows: each stream's first (sweep_table)
  std::vector<uint64_t> hpos;
  bool fast_group = true;    // L1..3: zs_k_fast (group-speculative) instead of zs_k_fast_serial
  // the chain builders (zs_k_bucket, zs_k_prev, zs_k_fast) let same-address LDS atomics of
  // one instruction apply in lane order (1) or rank equal hashes by ballots (0); 0 when the
  // self-test finds the order violated on this device
  bool lane_order = true;
  bool lane_order_ok = true;  // the self-test's verdict
  uint32_t inflate_wave_min = 32768;  // members with more input bytes decode one per wave (inflate_wave.hip); 0: never
  uint32_t lane_large_min = 2304;     // this many large members or more: one LANE each (zs_k_inflate_lane<.., true>); 256 KiB members: wave kernel 26.9 / 68.5 / 128 ms at 1024 / 2048 / 4096, lanes 68.6 / 78.3 / 77.7
  hipStream_t side = nullptr;         // second stream: the wave-per-member kernel runs beside the lane kernel
  hipStream_t side2 = nullptr;        // third: the split decode, beside the segmented decode
  hipEvent_t fork = nullptr, join = nullptr, join2 = nullptr;
  Buf wlist;
  std::vector<uint32_t> hwlist;
  // split decode of large members (inflate_split.hip): deflate64, or raw deflate without the window-wrap copy
  bool inflate_split = true;
  Buf slist, sfound, spres, sscr, smem, sval;
  std::vector<uint32_t> hslist;
  // segmented decode (inflate_seg.hip): a member's blocks cut into lane-sized pieces that synchronise
  bool inflate_seg = true;
  uint32_t seg_bits = 0;            // input bits per lane of an entry's first block (later ones: from the block before);
                                    // 0: 4096 for members of 64 KiB of input or more on average, else 2048
  uint32_t seg_small_batch = 16384; // batches of at most this many members ...
  uint32_t seg_small_min = 4096;    // ... send members with more input bytes than this to it too
  bool seg_wide = true;             // the 2048-bit sync window for a batch of few large members
  int seg_split = 2;                // pieces cut in two at the walk's mid points (0 off, 1 on, 2 auto: small batches)
  uint32_t seg_big_bits = ZS_SEG_BIG_BITS;  // members with more input bits also walk from the finder's block starts
  uint64_t seg_scratch_max = 16ull << 30;  // bytes of u16 piece scratch the segmented decode may take per batch
  uint32_t ncu = 256;               // compute units of the device
  Buf glist, gfound, gbig, gbigs, gspb, gspl, gflist, gent, gblk, glanes, gtab, gmem, gpbase, gplist, gsbase, gscr, gcnt;
  std::vector<uint32_t> hglist, hgpbase, hgspb, hgbig, hgbig_s;
  bool seg_used = false;            // the last inflate batch ran it
  std::vector<uint64_t> hgsbase;
  // host staging for the host-buffer entry points
  Buf d_in, d_out, d_res, d_pack, d_offs;
  HostBuf h_in, h_out, h_res, h_offs;
  hipStream_t h2d = nullptr, d2h = nullptr;  // the host entries' copies, beside the kernels (host_batch)
  std::vector<hipEvent_t> hev;               // their events, reused
  bool keep_counts = false;                  // a later chunk of one host batch: the lane / seg counts go on
  std::vector<uint8_t> hmeta;
  size_t last_n = 0;
  // timing
  struct Mark {
    std::string name;
    hipEvent_t ev;
    hipStream_t st;
  };
  std::vector<Mark> marks;  // a phase = the time between consecutive marks on the same stream
  // folded (pending) results since the last query: marks are folded in when
  // more than kMaxMarks are pending, so an unqueried timing run stays bounded
  std::vector<std::pair<std::string, double>> phase_acc;
  double total_acc = 0;
  bool acc_any = false;
  std::vector<std::pair<std::string, double>> phase_ms;  // the last query's results
  double total_ms = -1;
  // inflate lane count of the last batch: copied to pinned memory on the batch's stream, then an event
  uint32_t* lane_count_host = nullptr;
  hipEvent_t lane_ev = nullptr;
};
static constexpr size_t kMaxMarks = 1024;
static void fold_marks(zs_ctx* c);

// Phase boundary: records a timing event and, with check_phases, waits for the
// phase and reports a launch or execution error under the phase's name.
static int mark(zs_ctx* c, hipStream_t st, const char* name) {
  if (c->check_phases) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      const std::string msg = std::string(name) + ": " + hipGetErrorString(e);
      return fail(ZS_MEM_ERROR, "%s", msg.c_str());
    }
  }
  if (!c->timing) return ZS_OK;
  if (c->marks.size() >= kMaxMarks) fold_marks(c);
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return ZS_OK;
  (void)hipEventRecord(e, st);
  c->marks.push_back({name, e, st});
  return ZS_OK;
}
#define MARK(name)                              \
  do {                                          \
    const int r_ = mark(c, st, name);           \
    if (r_ != ZS_OK) return r_;                 \
  } while (0)

// Folds the pending marks into the accumulated phase times: waits for the
// last one, keeps it as the anchor of the next marks (so the time between two
// folds is not lost) and destroys the others.
static void fold_marks(zs_ctx* c) {
  if (c->marks.size() < 2) return;
  (void)hipEventSynchronize(c->marks.back().ev);
  for (size_t i = 1; i < c->marks.size(); i++) {
    size_t j = i;  // the previous mark on the same stream
    while (j-- > 0 && c->marks[j].st != c->marks[i].st) {}
    if (j == (size_t)-1) continue;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->marks[j].ev, c->marks[i].ev);
    c->phase_acc.emplace_back(c->marks[i].name, ms);
  }
  float tot = 0;
  (void)hipEventElapsedTime(&tot, c->marks.front().ev, c->marks.back().ev);
  c->total_acc += tot;
  c->acc_any = true;
  for (size_t i = 0; i + 1 < c->marks.size(); i++) (void)hipEventDestroy(c->marks[i].ev);
  c->marks.erase(c->marks.begin(), c->marks.end() - 1);
}

// Turns the marks of every batch since the last query into phase times (waits
// for the last one).  Batch calls never wait for their marks, so a timed
// sequence of batches runs back to back.
static void collect_marks(zs_ctx* c) {
  fold_marks(c);
  for (auto& m : c->marks) (void)hipEventDestroy(m.ev);
  c->marks.clear();
  if (!c->acc_any) return;  // nothing new: keep the last results
  c->phase_ms.swap(c->phase_acc);
  c->phase_acc.clear();
  c->total_ms = c->total_acc;
  c->total_acc = 0;
  c->acc_any = false;
}

extern "C" {

const char* zs_last_error(void) { return g_err.c_str(); }
const char* zs_version(void) { return "zs_gpu 0.1 (gfx950)"; }

int zs_ctx_create(int device, zs_ctx** out) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0)
    return fail(ZS_STREAM_ERROR, "no HIP device %s", std::to_string(device).c_str());
  HIPCHK(hipSetDevice(device));
  zs_ctx* c = new zs_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(ZS_MEM_ERROR, "%s", hipGetErrorString(e));
  }
  int prio_lo = 0, prio_hi = 0;  // (numerically lower = higher priority)
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithPriority(&c->side2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipEventCreateWithFlags(&c->join2, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->join, hipEventDisableTiming) != hipSuccess) {
    zs_ctx_destroy(c);
    return fail(ZS_MEM_ERROR, "%s", "cannot create the side stream");
  }
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      c->ncu = (uint32_t)ncu;
  }
  // the chain builders use lane-ordered LDS atomics where the device applies them so:
  // check before any use; a device that violates it gets the ballot-ranked form
  uint64_t bad = 0;
  const int st = zs_selftest(c, &bad);
  if (st != ZS_OK) {
    const std::string why = zs_last_error();
    zs_ctx_destroy(c);
    return fail(ZS_STREAM_ERROR, "self-test failed: %s", why.c_str());
  }
  c->lane_order = c->lane_order_ok = bad == 0;
  *out = c;
  return ZS_OK;
}

int zs_selftest(zs_ctx* c, uint64_t* violations) {
  if (!c || !violations) return fail(ZS_STREAM_ERROR, "invalid arguments");
  *violations = 0;
  HIPCHK(hipSetDevice(c->device));
  uint32_t* d_bad = nullptr;
  HIPCHK(hipMalloc(&d_bad, sizeof(uint32_t)));
  hipError_t e = hipMemsetAsync(d_bad, 0, sizeof(uint32_t), c->stream);
  if (e == hipSuccess) {
    zs_k_selftest<<<256, 64, 0, c->stream>>>(d_bad, 32);
    e = hipGetLastError();
  }
  uint32_t h = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&h, d_bad, sizeof h, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_bad);
  if (e != hipSuccess) return fail(ZS_MEM_ERROR, "%s", hipGetErrorString(e));
  *violations = h;
  return ZS_OK;
}

void zs_ctx_destroy(zs_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (Buf* b : {&c->lstat, &c->ltabs, &c->lres, &c->llen, &c->pscr, &c->meta, &c->prevd, &c->mres, &c->syms, &c->blocks, &c->streams, &c->codes, &c->hdr, &c->check,
                 &c->istate, &c->d_in, &c->d_out, &c->d_res, &c->d_pack, &c->wlist, &c->slist, &c->sfound,
                 &c->spres, &c->sscr, &c->smem, &c->sval, &c->glist, &c->gfound, &c->gbig, &c->gbigs, &c->gspb, &c->gspl, &c->gflist, &c->gent, &c->gblk,
                 &c->glanes, &c->gtab, &c->gmem, &c->gpbase, &c->gplist, &c->gsbase, &c->gscr, &c->gcnt})
    if (b->p) (void)hipFree(b->p);
  for (HostBuf* b : {&c->h_in, &c->h_out, &c->h_res, &c->h_offs})
    if (b->p) (void)hipHostFree(b->p);
  if (c->d_offs.p) (void)hipFree(c->d_offs.p);
  for (hipEvent_t e : c->hev) (void)hipEventDestroy(e);
  for (hipStream_t q : {c->h2d, c->d2h})
    if (q) {
      (void)hipStreamSynchronize(q);
      (void)hipStreamDestroy(q);
    }
  for (auto& m : c->marks) (void)hipEventDestroy(m.ev);
  if (c->lane_ev) (void)hipEventSynchronize(c->lane_ev);
  if (c->lane_count_host) (void)hipHostFree(c->lane_count_host);
  if (c->lane_ev) (void)hipEventDestroy(c->lane_ev);
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->fork) (void)hipEventDestroy(c->fork);
  if (c->join) (void)hipEventDestroy(c->join);
  if (c->side2) (void)hipStreamSynchronize(c->side2);
  if (c->join2) (void)hipEventDestroy(c->join2);
  if (c->side2) (void)hipStreamDestroy(c->side2);
  if (c->side) (void)hipStreamDestroy(c->side);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

void zs_set_timing(zs_ctx* c, int on) { c->timing = on != 0; }

int zs_set_option(zs_ctx* c, const char* name, int value) {
  if (!c || !name) return fail(ZS_STREAM_ERROR, "invalid arguments");
  if (!strcmp(name, "timing")) c->timing = value != 0;
  else if (!strcmp(name, "inflate_fast")) c->inflate_fast = value != 0;
  else if (!strcmp(name, "inflate_ref_wrap")) c->inflate_ref_wrap = value != 0;
  else if (!strcmp(name, "check_phases")) c->check_phases = value != 0;
  else if (!strcmp(name, "match_sweep")) c->match_sweep = value != 0;
  else if (!strcmp(name, "fast_group")) c->fast_group = value != 0;
  else if (!strcmp(name, "lane_order")) {
    if (value && !c->lane_order_ok)
      return fail(ZS_STREAM_ERROR, "lane_order: this device does not apply LDS atomics in lane order");
    c->lane_order = value != 0;
  }
  else if (!strcmp(name, "inflate_split")) c->inflate_split = value != 0;
  else if (!strcmp(name, "inflate_seg")) c->inflate_seg = value != 0;
  else if (!strcmp(name, "seg_wide")) c->seg_wide = value != 0;
  else if (!strcmp(name, "seg_split")) {
    if (value < 0 || value > 2) return fail(ZS_STREAM_ERROR, "seg_split must be 0, 1 or 2 (auto)");
    c->seg_split = value;
  }
  else if (!strcmp(name, "seg_big_bits")) {
    if (value < 65536) return fail(ZS_STREAM_ERROR, "seg_big_bits must be >= 65536");
    c->seg_big_bits = (uint32_t)value;
  }
  else if (!strcmp(name, "seg_scratch_mb")) {
    if (value < 0) return fail(ZS_STREAM_ERROR, "seg_scratch_mb must be >= 0");
    c->seg_scratch_max = (uint64_t)value << 20;
  }
  else if (!strcmp(name, "seg_bits")) {
    if (value != 0 && (value < (int)ZS_SEG_W || value > (int)ZS_SEG_SMAX))
      return fail(ZS_STREAM_ERROR, "seg_bits must be 0 (auto) or 1024 .. 8192");
    c->seg_bits = (uint32_t)value;
  } else if (!strcmp(name, "seg_small_batch")) {
    if (value < 0) return fail(ZS_STREAM_ERROR, "seg_small_batch must be >= 0");
    c->seg_small_batch = (uint32_t)value;
  } else if (!strcmp(name, "seg_small_min")) {
    if (value < 0) return fail(ZS_STREAM_ERROR, "seg_small_min must be >= 0");
    c->seg_small_min = (uint32_t)value;
  }
  else if (!strcmp(name, "parse_waves")) {
    if (value < 0 || value > 4 || value == 3) return fail(ZS_STREAM_ERROR, "parse_waves must be 0, 1, 2 or 4");
    c->parse_waves = value;
  }
  else if (!strcmp(name, "lane_block")) {
    if (value != 0 && (value < 1 || value > 64 || (value & (value - 1))))
      return fail(ZS_STREAM_ERROR, "lane_block must be 0 or a power of two <= 64");
    c->lane_block = value;
  } else if (!strcmp(name, "lane_large_min")) {
    if (value < 0) return fail(ZS_STREAM_ERROR, "lane_large_min must be >= 0");
    c->lane_large_min = (uint32_t)value;
  } else if (!strcmp(name, "inflate_wave_min")) {
    if (value < 0) return fail(ZS_STREAM_ERROR, "inflate_wave_min must be >= 0");
    c->inflate_wave_min = (uint32_t)value;
  } else return fail(ZS_STREAM_ERROR, "unknown option %s", name);
  return ZS_OK;
}
double zs_last_batch_ms(zs_ctx* c) {
  collect_marks(c);
  return c->total_ms;
}
uint32_t zs_last_inflate_lane_count(zs_ctx* c) {
  if (!c || !c->lane_count_host || hipEventSynchronize(c->lane_ev) != hipSuccess) return 0;
  return *(volatile uint32_t*)c->lane_count_host;
}
uint32_t zs_last_inflate_seg_count(zs_ctx* c) {
  uint32_t v = 0;
  if (!c || !c->seg_used || !c->gcnt.p || hipStreamSynchronize(c->side) != hipSuccess ||
      hipMemcpy(&v, c->gcnt.as<uint32_t>() + 1, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return v;
}
double zs_last_phase_ms(zs_ctx* c, const char* phase) {
  collect_marks(c);
  double t = -1;
  for (auto& p : c->phase_ms)
    if (p.first == phase) t = (t < 0 ? 0 : t) + p.second;
  return t;
}

uint64_t zs_deflate_bound(uint64_t n, int wbits) {  // deflate.ts:615-674, memLevel 8 / windowBits 15
  const uint64_t wraplen = wbits < 0 ? 0 : (wbits > 15 ? 18 : 6);
  const uint64_t b = n + (n >> 12) + (n >> 14) + (n >> 25) + 13 - 6 + wraplen;
  return b;  // (output capacities must still be multiples of 4: round up when allocating)
}

}  // extern "C"

// Device metadata block: in_off | in_len | out_off | out_cap | pos_base | blk_base
struct MetaLayout {
  size_t in_off, in_len, out_off, out_cap, pos_base, blk_base, segs, win0, bytes;
  explicit MetaLayout(uint32_t n, uint32_t nwin = 0) {
    size_t o = 0;
    auto take = [&](size_t b) { size_t r = o; o = (o + b + 255) & ~size_t(255); return r; };
    in_off = take(8ull * n);
    in_len = take(4ull * n);
    out_off = take(8ull * n);
    out_cap = take(4ull * n);
    pos_base = take(8ull * n);
    blk_base = take(4ull * n);
    segs = take(sizeof(zs_sweep_seg) * nwin);  // the sweep's windows (levels 4..9)
    win0 = take(nwin ? 4ull * n : 0);          // each stream's first window
    bytes = o;
  }
};

__global__ void zs_k_finish(const zs_stream* streams, int32_t* status, uint32_t* out_len, int n) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  status[s] = streams[s].status;
  out_len[s] = streams[s].status == ZS_Z_STREAM_END ? streams[s].out_len : 0u;
}

__global__ void zs_k_copy_check(const uint32_t* check, zs_stream* streams, int n) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) streams[s].check = check[s];
}

// level 0: stored blocks (zs_k_stored), trailer checksums from zs_k_checksum
static int deflate_stored_batch(zs_ctx* c, int wrap, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                                const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off,
                                const uint32_t* out_cap, int32_t* d_status, uint32_t* d_out_len, hipStream_t st) {
  MetaLayout ml(n);
  c->hmeta.resize(ml.bytes);
  c->last_n = n;
  uint8_t* hm = c->hmeta.data();
  memcpy(hm + ml.in_off, in_off, 8ull * n);
  memcpy(hm + ml.in_len, in_len, 4ull * n);
  memcpy(hm + ml.out_off, out_off, 8ull * n);
  memcpy(hm + ml.out_cap, out_cap, 4ull * n);
  uint64_t max_total = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t t = (wrap == 0 ? 0 : wrap == 1 ? 6 : 18) + 5ull * (in_len[i] / ZS_STORED_CHUNK + 1) + in_len[i];
    max_total = std::max(max_total, t);
  }
  HIPCHK(c->meta.ensure(ml.bytes));
  HIPCHK(c->check.ensure(4ull * n));
  HIPCHK(hipMemcpyAsync(c->meta.p, hm, ml.bytes, hipMemcpyHostToDevice, st));
  uint8_t* dm = c->meta.as<uint8_t>();
  const uint64_t* d_in_off = (const uint64_t*)(dm + ml.in_off);
  const uint32_t* d_in_len = (const uint32_t*)(dm + ml.in_len);
  MARK("start");
  if (wrap) {
    zs_k_checksum<<<n, 64, 0, st>>>(d_in, d_in_off, d_in_len, c->check.as<uint32_t>(), wrap == 1 ? 1 : 2);
    MARK("checksum");
  }
  const dim3 g((unsigned)((max_total + 4095) / 4096), n);  // 256 threads x 16 bytes per workgroup
  zs_k_stored<<<g, 256, 0, st>>>(d_in, d_in_off, d_in_len, d_out, (const uint64_t*)(dm + ml.out_off),
                                 (const uint32_t*)(dm + ml.out_cap), c->check.as<uint32_t>(), wrap, d_status,
                                 d_out_len);
  MARK("stored");
  HIPCHK(hipGetLastError());
  return ZS_OK;  // timing marks are collected when queried (no wait here)
}

// The L4..9 parse runs two waves per stream (zs_k_parse_2w: 512-position
// segments, two rounds' speculative passes at once) for a batch of n streams?
// The whole batch decides (chunks of one batch share the scratch layout).
static int parse_waves_for(const zs_ctx* c, uint32_t n, int level) {
  (void)level;
  if (c->parse_waves) return c->parse_waves;
  return n < ZS_PARSE2W_AUTO ? 2 : 1;
}
static uint32_t parse_seg(int w) {
  return w == 4 ? ZS_PARSE4W_SEG : w == 2 ? ZS_PARSE2W_SEG : ZS_PARSE_SEG;
}
static uint32_t parse_seg_words(int w) {
  return w == 4 ? ZS_PARSE4W_SEG_WORDS : w == 2 ? ZS_PARSE2W_SEG_WORDS : ZS_PARSE_SEG_WORDS;
}

// The sweep's window table of a batch (into `out`, batch stream indices) and each
// stream's first window (win0[n] = the total).  Members: u16 per position for a
// stream of one window (pos_base); 65,536 per window after them for longer ones.
static void sweep_table(uint32_t n, const uint32_t* in_len, const uint64_t* pos, uint64_t P, zs_sweep_seg* out,
                        std::vector<uint32_t>& win0, uint64_t& members) {
  uint64_t mb = (P + 7) & ~7ull;
  uint32_t w = 0;
  win0.resize(n + 1);
  for (uint32_t i = 0; i < n; i++) {
    win0[i] = w;
    const uint32_t len = in_len[i];
    if (len <= 65537u) {
      if (out) out[w] = {i, 0u, 0u, len, pos[i], 0};
      w++;
      continue;
    }
    for (uint64_t lo = 0; lo < len; mb += 65536, w++) {
      const uint32_t base = lo == 0 ? 0u : (uint32_t)lo - 32768u;
      if (out) out[w] = {i, base, (uint32_t)lo - base, lo == 0 ? ZS_SEG_FIRST : 32768u + ZS_SEG_OWN, mb, 0};
      lo += lo == 0 ? ZS_SEG_FIRST : ZS_SEG_OWN;
    }
  }
  win0[n] = w;
  members = mb;
}

// The match finding of streams [a, e) of a batch (levels 4..9) on stream st
// (device arrays of the whole batch).  With the sweep, every stream is cut into
// WINDOWS of at most 65,535 inserted positions (zs_sweep_seg, sweep_table): a
// stream of up to 65,537 bytes is one; a longer one has a first window owning
// positions [0, 65520) and then windows owning 32,752 positions each after a
// 32,768-position look-back (more than MAX_DIST: every candidate of an own
// position is in its window).
static int deflate_match(zs_ctx* c, hipStream_t st, const zs_level_cfg& cfg, uint32_t a, uint32_t e,
                         uint32_t max_len, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                         const uint64_t* d_pos, const zs_sweep_seg* d_segs) {
  const uint32_t n = e - a;
  if (c->match_sweep) {
    const uint32_t w0 = c->hwin0[a], nw = c->hwin0[e] - w0;
    // a window: counting sort by hash + lock-step sweep (deflate_sweep.hip)
    (c->lane_order ? zs_k_bucket<true> : zs_k_bucket<false>)<<<nw, ZS_BK_THREADS, 0, st>>>(
        d_in, d_in_off, d_in_len, d_pos, d_segs + w0, c->prevd.as<uint16_t>(), c->mres.as<uint2>());
    MARK("bucket");
    zs_k_sweep<<<nw, 1024, 0, st>>>(d_in, d_in_off, d_in_len, d_pos, d_segs + w0, c->prevd.as<uint16_t>(),
                                    c->mres.as<uint2>(), cfg.chain, cfg.nice);
    MARK("sweep");
  } else {
    // cross-check (option match_sweep = 0): the chain-walk kernels for every stream
    const dim3 g((max_len + 8191) / 8192, n);
    (c->lane_order ? zs_k_prev<true> : zs_k_prev<false>)<<<n, 64, 0, st>>>(d_in, d_in_off + a, d_in_len + a,
                                                                           d_pos + a, c->prevd.as<uint16_t>(), 0u);
    MARK("prev");
    if (max_len) zs_k_match<<<g, 1024, 0, st>>>(d_in, d_in_off + a, d_in_len + a, d_pos + a, c->prevd.as<uint16_t>(),
                                                 c->mres.as<uint2>(), cfg.chain, cfg.nice, 0u);
    MARK("match");
  }
  return ZS_OK;
}

// The rest of the deflate sequence of streams [0, n) on stream st: the parse
// (levels 4..9) or deflate_fast (1..3), trees, layout, emit, wrapper, statuses.
// Per-stream arrays are offset to the first stream; syms and pscr too (kernels
// index them by the launch-local stream index).
static int deflate_tail(zs_ctx* c, hipStream_t st, int level, int wrap, const zs_level_cfg& cfg, uint32_t n,
                        uint32_t max_blk, const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len,
                        uint8_t* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap, const uint64_t* d_pos,
                        const uint32_t* d_blk, zs_stream* d_st, uint32_t* syms, uint32_t* pscr, int32_t* d_status,
                        uint32_t* d_out_len) {
  zs_block* d_bk = c->blocks.as<zs_block>();
  const int nthreads_s = 256, nblocks_s = (int)((n + 255) / 256);
  if (level >= 4) {
    const int pw = c->cur_pw;  // waves per stream of the lazy parse (deflate_parse.hip)
    auto parse = pw == 4 ? zs_k_parse_4w : pw == 2 ? zs_k_parse_2w : zs_k_parse;
    parse<<<n, 64 * pw, 0, st>>>(d_in, d_in_off, d_in_len, d_pos, d_blk, c->mres.as<uint2>(), syms, d_bk, d_st,
                                 pscr, cfg.good, cfg.lazy);
    MARK("parse");
  } else {
    const int fast_smem = 2 * 32768 * 2 + 32768;  // head[] + prev[] (u16 x 32 K each) + the 32 KiB input ring
    // levels 1..3: the group-speculative replay (default) or the step-by-step one (fast_group = 0)
    auto fast = !c->fast_group ? zs_k_fast_serial
                : c->lane_order   ? (cfg.nice <= 8 ? zs_k_fast<2, true> : cfg.nice <= 16 ? zs_k_fast<4, true> : zs_k_fast<8, true>)
                                  : (cfg.nice <= 8 ? zs_k_fast<2, false> : cfg.nice <= 16 ? zs_k_fast<4, false> : zs_k_fast<8, false>);
    HIPCHK(hipFuncSetAttribute((const void*)fast, hipFuncAttributeMaxDynamicSharedMemorySize, fast_smem));
    fast<<<n, 64, fast_smem, st>>>(d_in, d_in_off, d_in_len, d_pos, d_blk, syms, d_bk, d_st,
                                        cfg.chain, cfg.lazy, cfg.nice);
    MARK("fast");
  }
  zs_k_trees<<<dim3(max_blk, n), 64, 0, st>>>(d_in, d_in_off, d_pos, d_blk, syms, d_bk, d_st,
                                              c->codes.as<uint32_t>(), c->hdr.as<uint32_t>(), (int)n);
  MARK("trees");
  zs_k_layout<<<nblocks_s, nthreads_s, 0, st>>>(d_blk, d_bk, d_st, d_out_cap, d_out, d_out_off, wrap, (int)n);
  MARK("layout");
  zs_k_emit<<<dim3(max_blk, n), 256, 0, st>>>(d_in, d_in_off, d_pos, d_blk, syms, d_bk, d_st,
                                              c->codes.as<uint32_t>(), c->hdr.as<uint32_t>(), d_out, d_out_off, wrap);
  MARK("emit");
  if (wrap) zs_k_wrap<<<nblocks_s, nthreads_s, 0, st>>>(d_st, d_out, d_out_off, d_in_len, wrap, level, (int)n);
  zs_k_finish<<<nblocks_s, nthreads_s, 0, st>>>(d_st, d_status, d_out_len, (int)n);
  MARK("finish");
  return ZS_OK;
}

// The deflate launch sequence of a batch (levels 1..9) on stream st.  (A
// pipeline of chunks of streams -- chunk j's parse .. emit on a side stream
// beside chunk j + 1's sweep -- measured slower twice: DESIGN 5,
// tools/variants/r05_paths.patch.)
static int deflate_launch(zs_ctx* c, hipStream_t st, int level, int wrap, const zs_level_cfg& cfg, uint32_t n,
                          const uint32_t* in_len, const zs_sweep_seg* d_segs, const uint32_t* d_win0,
                          const uint8_t* d_in, const uint64_t* d_in_off, const uint32_t* d_in_len, uint8_t* d_out,
                          const uint64_t* d_out_off, const uint32_t* d_out_cap, const uint64_t* d_pos,
                          const uint32_t* d_blk, zs_stream* d_st, uint32_t* syms, uint32_t* pscr, uint32_t* check,
                          int32_t* d_status, uint32_t* d_out_len) {
  const int nthreads_s = 256, nblocks_s = (int)((n + 255) / 256);
  MARK("start");
  if (wrap) {
    zs_k_checksum<<<n, 64, 0, st>>>(d_in, d_in_off, d_in_len, check, wrap == 1 ? 1 : 2);
    zs_k_copy_check<<<nblocks_s, nthreads_s, 0, st>>>(check, d_st, (int)n);
    MARK("checksum");
  }
  uint32_t mlen = 0, mblk = 0;
  for (uint32_t i = 0; i < n; i++) {
    mlen = std::max(mlen, in_len[i]);
    mblk = std::max(mblk, in_len[i] / ZS_SYM_END + 2);
  }
  if (level >= 4) {
    const int r = deflate_match(c, st, cfg, 0, n, mlen, d_in, d_in_off, d_in_len, d_pos, d_segs);
    if (r != ZS_OK) return r;
  }
  return deflate_tail(c, st, level, wrap, cfg, n, mblk, d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_cap, d_pos,
                      d_blk, d_st, syms, pscr, d_status, d_out_len);
}

// Per-stream check value (the reference's strm.adler after the stream,
// deflate.ts:155-159,462,778,788): adler32 (zlib) / crc32 (gzip) of the input,
// 1 for deflate-raw (adler32(0), never updated without a wrapper); 0 for a
// stream that failed.
__global__ void zs_k_deflate_check(const int32_t* status, const uint32_t* check, int wrap, uint32_t* out, int n) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  out[s] = status[s] != ZS_Z_STREAM_END ? 0u : wrap ? check[s] : 1u;
}

extern "C" int zs_deflate_batch_device(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* d_in,
                                       const uint64_t* in_off, const uint32_t* in_len, uint8_t* d_out,
                                       const uint64_t* out_off, const uint32_t* out_cap, int32_t* d_status,
                                       uint32_t* d_out_len, void* hip_stream) {
  return zs_deflate_batch_device_ex(c, level, wbits, n, d_in, in_off, in_len, d_out, out_off, out_cap, d_status,
                                    d_out_len, nullptr, hip_stream);
}

// The device compress.  out_cap[i] is the stream's capacity as the caller set
// it (Z_BUF_ERROR past it, exactly); the kernels store whole dwords, so the
// stream's region must reach out_off[i] + out_cap[i] rounded up to 4.
// `caller_regions` (the public device entries): the regions are the caller's
// buffers, so capacities must be multiples of 4; the host entries stage in
// regions of the capacities rounded up and pass the exact capacities.
static int deflate_device(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                          const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off, const uint32_t* out_cap,
                          int32_t* d_status, uint32_t* d_out_len, uint32_t* d_check, void* hip_stream,
                          bool caller_regions);

extern "C" int zs_deflate_batch_device_ex(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* d_in,
                                          const uint64_t* in_off, const uint32_t* in_len, uint8_t* d_out,
                                          const uint64_t* out_off, const uint32_t* out_cap, int32_t* d_status,
                                          uint32_t* d_out_len, uint32_t* d_check, void* hip_stream) {
  return deflate_device(c, level, wbits, n, d_in, in_off, in_len, d_out, out_off, out_cap, d_status, d_out_len,
                        d_check, hip_stream, true);
}

static int deflate_device(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                          const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off, const uint32_t* out_cap,
                          int32_t* d_status, uint32_t* d_out_len, uint32_t* d_check, void* hip_stream,
                          bool caller_regions) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  if (level == -1) level = 6;  // Z_DEFAULT_COMPRESSION, deflate.ts:268-270
  int wrap;
  if (wbits == -15) wrap = 0;
  else if (wbits == 15) wrap = 1;
  else if (wbits == 31) wrap = 2;
  else return fail(ZS_STREAM_ERROR, "unsupported windowBits (use -15, 15 or 31)");
  if (level < 0 || level > 9) return fail(ZS_STREAM_ERROR, "invalid level");  // deflate.ts:281-294
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  for (uint32_t i = 0; i < n; i++)
    if ((out_off[i] & 3) || (caller_regions && (out_cap[i] & 3)))
      return fail(ZS_STREAM_ERROR, "output offsets/capacities must be multiples of 4");
  if (level == 0) {
    const int r = deflate_stored_batch(c, wrap, n, d_in, in_off, in_len, d_out, out_off, out_cap, d_status,
                                       d_out_len, st);
    if (r == ZS_OK && d_check) {
      zs_k_deflate_check<<<(n + 255) / 256, 256, 0, st>>>(d_status, c->check.as<uint32_t>(), wrap, d_check, (int)n);
      HIPCHK(hipGetLastError());
    }
    return r;
  }
  // host-side layout: workspace bases (and the sweep's windows, levels 4..9)
  const bool sweep = level >= 4 && c->match_sweep;
  uint64_t P = 0, members = 0;
  uint32_t B = 0, max_len = 0, max_blk = 0;
  c->hpos.resize(n);
  for (uint32_t i = 0; i < n; i++) {
    c->hpos[i] = P;
    P += ((uint64_t)in_len[i] + 7) & ~7ull;  // per-position tables start 8-aligned (16-B link loads in zs_k_match)
  }
  if (sweep) sweep_table(n, in_len, c->hpos.data(), P, nullptr, c->hwin0, members);
  MetaLayout ml(n, sweep ? c->hwin0[n] : 0u);
  c->hmeta.resize(ml.bytes);
  c->last_n = n;
  uint8_t* hm = c->hmeta.data();
  memcpy(hm + ml.in_off, in_off, 8ull * n);
  memcpy(hm + ml.in_len, in_len, 4ull * n);
  memcpy(hm + ml.out_off, out_off, 8ull * n);
  memcpy(hm + ml.out_cap, out_cap, 4ull * n);
  uint64_t* pos_base = (uint64_t*)(hm + ml.pos_base);
  uint32_t* blk_base = (uint32_t*)(hm + ml.blk_base);
  memcpy(pos_base, c->hpos.data(), 8ull * n);
  if (sweep) {
    sweep_table(n, in_len, pos_base, P, (zs_sweep_seg*)(hm + ml.segs), c->hwin0, members);
    memcpy(hm + ml.win0, c->hwin0.data(), 4ull * n);
  }
  for (uint32_t i = 0; i < n; i++) {
    blk_base[i] = B;
    const uint32_t nb = in_len[i] / ZS_SYM_END + 2;
    B += nb;
    max_len = std::max(max_len, in_len[i]);
    max_blk = std::max(max_blk, nb);
  }
  HIPCHK(c->meta.ensure(ml.bytes));
  HIPCHK(c->prevd.ensure(2 * std::max(members, P) + 128));
  HIPCHK(c->mres.ensure(8 * P + 64));
  HIPCHK(c->syms.ensure(4 * (P + n) + 64));
  c->cur_pw = level >= 4 ? parse_waves_for(c, n, level) : 1;
  if (level >= 4)
    HIPCHK(c->pscr.ensure(4ull * parse_seg_words(c->cur_pw) * (P / parse_seg(c->cur_pw) + n + 1)));
  HIPCHK(c->blocks.ensure(sizeof(zs_block) * (size_t)B));
  HIPCHK(c->streams.ensure(sizeof(zs_stream) * (size_t)n));
  HIPCHK(c->codes.ensure(4ull * (ZS_L_CODES + ZS_D_CODES) * B));
  HIPCHK(c->hdr.ensure(4ull * ZS_HDR_WORDS * B));
  HIPCHK(c->check.ensure(4ull * n));
  HIPCHK(hipMemcpyAsync(c->meta.p, hm, ml.bytes, hipMemcpyHostToDevice, st));
  uint8_t* dm = c->meta.as<uint8_t>();
  (void)max_len;
  (void)max_blk;
  const int r = deflate_launch(c, st, level, wrap, kLevels[level], n, in_len, (const zs_sweep_seg*)(dm + ml.segs),
                               (const uint32_t*)(dm + ml.win0), d_in,
                               (const uint64_t*)(dm + ml.in_off), (const uint32_t*)(dm + ml.in_len), d_out,
                               (const uint64_t*)(dm + ml.out_off), (const uint32_t*)(dm + ml.out_cap),
                               (const uint64_t*)(dm + ml.pos_base), (const uint32_t*)(dm + ml.blk_base),
                               c->streams.as<zs_stream>(), c->syms.as<uint32_t>(), c->pscr.as<uint32_t>(),
                               c->check.as<uint32_t>(), d_status, d_out_len);
  if (r != ZS_OK) return r;
  if (d_check)
    zs_k_deflate_check<<<(n + 255) / 256, 256, 0, st>>>(d_status, c->check.as<uint32_t>(), wrap, d_check, (int)n);
  MARK("end");
  HIPCHK(hipGetLastError());
  return ZS_OK;  // timing marks are collected when queried (no wait here)
}

// ---------------------------------------------------------- host buffers
// The host-buffer entry points: the caller's streams are packed (in parallel)
// into a pinned staging buffer and copied to HBM; after the batch the outputs
// are compacted on the device (4-aligned, in stream order) and come back in one
// copy of exactly the produced bytes, which the host then scatters to the
// caller's offsets -- chunk by chunk, overlapped with the kernels (host_batch).
static void par_copy(uint32_t n, uint8_t* dst, const uint64_t* dst_off, const uint8_t* src, const uint64_t* src_off,
                     const uint32_t* len, uint64_t total) {
  const int T = total >= (32u << 20) ? 8 : (total >= (4u << 20) ? 4 : 1);
  auto part = [&](int t) {
    for (uint32_t i = (uint32_t)t; i < n; i += (uint32_t)T)
      if (len[i]) memcpy(dst + dst_off[i], src + src_off[i], len[i]);
  };
  if (T == 1) { part(0); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back(part, t);
  for (auto& x : th) x.join();
}

static int stage_in(zs_ctx* c, uint32_t n, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                    std::vector<uint64_t>& doff, uint64_t& total) {
  total = 0;
  doff.resize(n);
  for (uint32_t i = 0; i < n; i++) { doff[i] = total; total += in_len[i]; }
  HIPCHK(c->d_in.ensure(total + 16));
  HIPCHK(c->h_in.ensure(total + 16));
  par_copy(n, c->h_in.as<uint8_t>(), doff.data(), in, in_off, in_len, total);
  if (total) HIPCHK(hipMemcpyAsync(c->d_in.p, c->h_in.p, total, hipMemcpyHostToDevice, c->stream));
  return ZS_OK;
}

// dst[poff[s] ...] = src[soff[s] ...], len[s] bytes (all offsets multiples of 4)
__global__ void zs_k_compact(const uint8_t* __restrict__ src, const uint64_t* __restrict__ offs,
                             const uint32_t* __restrict__ len, uint8_t* __restrict__ dst, uint32_t n) {
  const uint32_t s = blockIdx.x;
  if (s >= n) return;
  const uint32_t words = (len[s] + 3) / 4;
  const uint32_t* a = (const uint32_t*)(src + offs[s]);
  uint32_t* b = (uint32_t*)(dst + offs[n + s]);
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) b[i] = a[i];
}

// The host-buffer entries, pipelined: the batch runs as a few chunks of
// streams ([1/8, 3/8, 3/8, 1/8] of them for batches of 32 MB or more), so that
// packing chunk k+1 into the pinned staging and its H2D copy (stream h2d) run
// while chunk k's kernels do (the context's stream), and chunk k-1's output
// compaction, D2H copy (stream d2h) and scatter into the caller's buffers run
// while chunk k+1's do.  `launch(a, b, doff, ooff, ocap, d_res)` enqueues the
// device batch of streams [a, b) on c->stream; d_res holds nres u32 arrays of n
// entries (array r at d_res + r n), res_host the caller's nres arrays, of which
// res_host[len_idx] is the output length.  Outputs land at out + out_off[i].
template <class Launch>
static int host_batch_run(zs_ctx* c, uint32_t n, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                          const std::vector<uint32_t>& ocap, uint32_t nres, uint32_t* const* res_host,
                          uint32_t len_idx, uint8_t* out, const uint64_t* out_off, Launch launch) {
  std::vector<uint64_t> doff(n), ooff(n);
  uint64_t tin = 0, tout = 0;
  for (uint32_t i = 0; i < n; i++) {
    doff[i] = tin;
    tin += in_len[i];
    ooff[i] = tout;
    tout += ocap[i];
  }
  HIPCHK(c->d_in.ensure(tin + 16));
  HIPCHK(c->h_in.ensure(tin + 16));
  HIPCHK(c->d_out.ensure(tout + 16));
  // the packed outputs (d_pack, h_out) hold produced bytes, not capacities: a
  // first guess, grown in after_kernels once the chunks before are scattered
  const uint64_t pack0 = std::min<uint64_t>(tout, std::max<uint64_t>(4 * tin, 64ull << 20)) + 16;
  HIPCHK(c->d_pack.ensure(pack0));
  HIPCHK(c->h_out.ensure(pack0));
  HIPCHK(c->d_res.ensure(4ull * nres * n + 16));
  HIPCHK(c->h_res.ensure(4ull * nres * n + 16));
  HIPCHK(c->d_offs.ensure(16ull * n + 16));
  HIPCHK(c->h_offs.ensure(16ull * n + 16));
  std::vector<uint32_t> bnd{0};
  if (n >= 64 && tin >= (32ull << 20))
    for (uint32_t f : {1u, 4u, 7u}) bnd.push_back((uint32_t)((uint64_t)n * f / 8));
  bnd.push_back(n);
  const uint32_t K = (uint32_t)bnd.size() - 1;
  while (c->hev.size() < 3 * K) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->hev.push_back(e);
  }
  hipEvent_t* ev_in = c->hev.data();
  hipEvent_t* ev_k = ev_in + K;
  hipEvent_t* ev_out = ev_k + K;
  uint8_t* hin = c->h_in.as<uint8_t>();
  uint32_t* dres = c->d_res.as<uint32_t>();
  uint32_t* hres = c->h_res.as<uint32_t>();
  uint64_t* hoffs = c->h_offs.as<uint64_t>();
  std::vector<uint64_t> poff(n);
  std::vector<char> scattered(K, 0);
  uint64_t packed = 0;  // bytes of the pack buffers in use (chunks not yet scattered)
  // chunk k's bytes are in pinned memory: into the caller's buffers
  auto after_copy = [&](uint32_t k) -> int {
    if (scattered[k]) return ZS_OK;
    const uint32_t a = bnd[k], b = bnd[k + 1];
    HIPCHK(hipEventSynchronize(ev_out[k]));
    uint64_t bytes = 0;
    for (uint32_t i = a; i < b; i++) bytes += res_host[len_idx][i];
    par_copy(b - a, out, out_off + a, c->h_out.as<uint8_t>(), poff.data() + a, res_host[len_idx] + a, bytes);
    scattered[k] = 1;
    return ZS_OK;
  };
  // chunk k's results are in: the caller's arrays, then its compaction and D2H (stream d2h)
  auto after_kernels = [&](uint32_t k) -> int {
    const uint32_t a = bnd[k], b = bnd[k + 1], m = b - a;
    HIPCHK(hipEventSynchronize(ev_k[k]));
    for (uint32_t r = 0; r < nres; r++)
      if (res_host[r]) memcpy(res_host[r] + a, hres + (size_t)r * n + a, 4ull * m);
    const uint32_t* len = res_host[len_idx];
    uint64_t Pk = 0;
    for (uint32_t i = a; i < b; i++) {
      if (len[i] > ocap[i])
        return fail(ZS_MEM_ERROR, "stream %s reported more output than its capacity", std::to_string(i).c_str());
      Pk += ((uint64_t)len[i] + 3) & ~3ull;
    }
    if (packed + Pk + 16 > std::min(c->d_pack.cap, c->h_out.cap)) {
      // the pack buffers are full: scatter the chunks still in them, then start over (grown)
      for (uint32_t j = 0; j < k; j++) {
        const int rc = after_copy(j);
        if (rc != ZS_OK) return rc;
      }
      packed = 0;
      HIPCHK(c->d_pack.ensure(Pk + 16));
      HIPCHK(c->h_out.ensure(Pk + 16));
    }
    uint64_t P = packed;
    for (uint32_t i = a; i < b; i++) {
      hoffs[2 * a + (i - a)] = ooff[i];
      hoffs[2 * a + m + (i - a)] = poff[i] = P;
      P += ((uint64_t)len[i] + 3) & ~3ull;
    }
    if (P > packed) {
      uint64_t* doffs = c->d_offs.as<uint64_t>() + 2 * a;
      HIPCHK(hipMemcpyAsync(doffs, hoffs + 2 * a, 16ull * m, hipMemcpyHostToDevice, c->d2h));
      zs_k_compact<<<m, 256, 0, c->d2h>>>(c->d_out.as<uint8_t>(), doffs, dres + (size_t)len_idx * n + a,
                                          c->d_pack.as<uint8_t>(), m);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(c->h_out.as<uint8_t>() + packed, c->d_pack.as<uint8_t>() + packed, P - packed,
                            hipMemcpyDeviceToHost, c->d2h));
    }
    packed = P;
    HIPCHK(hipEventRecord(ev_out[k], c->d2h));
    return ZS_OK;
  };
  for (uint32_t k = 0; k < K; k++) {
    const uint32_t a = bnd[k], b = bnd[k + 1], m = b - a;
    const uint64_t bytes = (b < n ? doff[b] : tin) - doff[a];
    par_copy(m, hin, doff.data() + a, in, in_off + a, in_len + a, bytes);
    if (bytes) HIPCHK(hipMemcpyAsync(c->d_in.as<uint8_t>() + doff[a], hin + doff[a], bytes, hipMemcpyHostToDevice, c->h2d));
    HIPCHK(hipEventRecord(ev_in[k], c->h2d));
    HIPCHK(hipStreamWaitEvent(c->stream, ev_in[k], 0));
    std::vector<uint32_t*> dr(nres);
    for (uint32_t r = 0; r < nres; r++) dr[r] = dres + (size_t)r * n + a;
    c->keep_counts = k > 0;
    int rc = launch(a, b, doff.data() + a, ooff.data() + a, ocap.data() + a, dr.data());
    c->keep_counts = false;
    if (rc != ZS_OK) return rc;
    for (uint32_t r = 0; r < nres; r++)
      HIPCHK(hipMemcpyAsync(hres + (size_t)r * n + a, dr[r], 4ull * m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipEventRecord(ev_k[k], c->stream));
    if (k >= 1 && (rc = after_kernels(k - 1)) != ZS_OK) return rc;
    if (k >= 2 && (rc = after_copy(k - 2)) != ZS_OK) return rc;
  }
  int rc = after_kernels(K - 1);
  if (rc == ZS_OK && K >= 2) rc = after_copy(K - 2);
  if (rc == ZS_OK) rc = after_copy(K - 1);
  return rc;
}

// host_batch_run, and on any error the copies and kernels it left in flight
// are waited for before returning (the next call reuses the staging buffers)
template <class Launch>
static int host_batch(zs_ctx* c, uint32_t n, const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len,
                      const std::vector<uint32_t>& ocap, uint32_t nres, uint32_t* const* res_host, uint32_t len_idx,
                      uint8_t* out, const uint64_t* out_off, Launch launch) {
  const int rc = host_batch_run(c, n, in, in_off, in_len, ocap, nres, res_host, len_idx, out, out_off, launch);
  if (rc != ZS_OK) {
    (void)hipStreamSynchronize(c->h2d);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->d2h);
  }
  return rc;
}

extern "C" int zs_deflate_batch(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                const uint32_t* in_len, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                int32_t* status, uint32_t* out_len) {
  return zs_deflate_batch_ex(c, level, wbits, n, in, in_off, in_len, out, out_off, out_cap, status, out_len, nullptr);
}

extern "C" int zs_deflate_batch_ex(zs_ctx* c, int level, int wbits, uint32_t n, const uint8_t* in,
                                   const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                   const uint64_t* out_off, const uint32_t* out_cap, int32_t* status,
                                   uint32_t* out_len, uint32_t* check) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  // device regions: the caller's capacity rounded up to whole words (the kernels store dwords);
  // the caller's exact capacities are the Z_BUF_ERROR limits
  std::vector<uint32_t> ocap(n);
  for (uint32_t i = 0; i < n; i++) ocap[i] = (uint32_t)std::min<uint64_t>(0xfffffffcull, ((uint64_t)out_cap[i] + 3) & ~3ull);
  uint32_t* res[3] = {(uint32_t*)status, out_len, check};
  return host_batch(c, n, in, in_off, in_len, ocap, 3, res, 1, out, out_off,
                    [&](uint32_t a, uint32_t b, const uint64_t* doff, const uint64_t* ooff, const uint32_t*,
                        uint32_t** dr) {
                      return deflate_device(c, level, wbits, b - a, c->d_in.as<uint8_t>(), doff, in_len + a,
                                            c->d_out.as<uint8_t>(), ooff, out_cap + a, (int32_t*)dr[0], dr[1],
                                            check ? dr[2] : nullptr, c->stream, false);
                    });  // out_len is 0 for failed streams
}

static int checksum_batch(zs_ctx* c, int kind, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                          const uint32_t* in_len, const uint32_t* seeds, uint32_t* d_check, void* hip_stream) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  MetaLayout ml(n);
  c->hmeta.resize(ml.bytes + (seeds ? 4ull * n : 0));
  memcpy(c->hmeta.data() + ml.in_off, in_off, 8ull * n);
  memcpy(c->hmeta.data() + ml.in_len, in_len, 4ull * n);
  if (seeds) memcpy(c->hmeta.data() + ml.bytes, seeds, 4ull * n);
  HIPCHK(c->meta.ensure(c->hmeta.size()));
  HIPCHK(hipMemcpyAsync(c->meta.p, c->hmeta.data(), c->hmeta.size(), hipMemcpyHostToDevice, st));
  MARK("start");
  zs_k_checksum<<<n, 64, 0, st>>>(d_in, (const uint64_t*)(c->meta.as<uint8_t>() + ml.in_off),
                                  (const uint32_t*)(c->meta.as<uint8_t>() + ml.in_len), d_check, kind,
                                  seeds ? (const uint32_t*)(c->meta.as<uint8_t>() + ml.bytes) : nullptr);
  MARK("checksum");
  HIPCHK(hipGetLastError());
  return ZS_OK;  // timing marks are collected when queried (no wait here)
}

extern "C" int zs_crc32_batch_device(zs_ctx* c, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                                     const uint32_t* in_len, const uint32_t* seeds, uint32_t* d_check,
                                     void* hip_stream) {
  return checksum_batch(c, 2, n, d_in, in_off, in_len, seeds, d_check, hip_stream);
}
extern "C" int zs_adler32_batch_device(zs_ctx* c, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                                       const uint32_t* in_len, const uint32_t* seeds, uint32_t* d_check,
                                       void* hip_stream) {
  return checksum_batch(c, 1, n, d_in, in_off, in_len, seeds, d_check, hip_stream);
}

// host buffers: staged through the context's pinned buffer, results copied back
static int checksum_host(zs_ctx* c, int kind, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                         const uint32_t* in_len, const uint32_t* seeds, uint32_t* check) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  std::vector<uint64_t> doff;
  uint64_t total = 0;
  int r = stage_in(c, n, in, in_off, in_len, doff, total);
  if (r != ZS_OK) return r;
  HIPCHK(c->d_res.ensure(4ull * n + 16));
  r = checksum_batch(c, kind, n, c->d_in.as<uint8_t>(), doff.data(), in_len, seeds, c->d_res.as<uint32_t>(), nullptr);
  if (r != ZS_OK) return r;
  HIPCHK(hipMemcpyAsync(check, c->d_res.p, 4ull * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return ZS_OK;
}
extern "C" int zs_crc32_batch(zs_ctx* c, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                              const uint32_t* in_len, const uint32_t* seeds, uint32_t* check) {
  return checksum_host(c, 2, n, in, in_off, in_len, seeds, check);
}
extern "C" int zs_adler32_batch(zs_ctx* c, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                const uint32_t* in_len, const uint32_t* seeds, uint32_t* check) {
  return checksum_host(c, 1, n, in, in_off, in_len, seeds, check);
}

// ------------------------------------------------------------------ corpus
namespace {
const char* kVocab =
    "the of and to in is that for it as was with be by on not he this are or his from at which but have an they you "
    "were her she there been one all we their has would when if so no will more can out said up what about its into "
    "them than only other new some could time these two may then do first any my now such like our over man me even "
    "most made after also did many before must through back years where much your way well down should because each "
    "just those people how too little state good very make world still own see men work long get here between both "
    "life being under never day same another know while last might us great old year off come since against go came "
    "right used take three";

struct XS {
  uint32_t s;
  explicit XS(uint32_t seed) : s(seed ? seed : 1) {}
  uint32_t operator()() {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
  }
};

void gen_text(uint32_t seed, uint8_t* out, uint32_t n, const std::vector<std::string>& V) {
  XS r(seed);
  uint32_t o = 0, w = 0;
  while (o < n) {
    const uint32_t a = r();
    const uint32_t idx = std::min(a % 144u, (a >> 12) % 144u);
    const std::string& word = V[idx];
    for (size_t i = 0; i < word.size() && o < n; i++) out[o++] = (uint8_t)word[i];
    if (o < n) out[o++] = (++w % 13 == 0) ? 10 : 32;
  }
}
}  // namespace

extern "C" void zs_corpus(int kind, uint32_t first, uint32_t n_streams, uint32_t len, uint8_t* out, int threads) {
  std::vector<std::string> V;
  {
    std::string all(kVocab), cur;
    for (char ch : all) {
      if (ch == ' ') { V.push_back(cur); cur.clear(); }
      else cur.push_back(ch);
    }
    V.push_back(cur);
  }
  auto one = [&](uint32_t i) {
    const uint32_t seed = 0x9e3779b9u ^ (first + i);
    uint8_t* o = out + (size_t)i * len;
    if (kind == 2) {
      XS r(seed);
      for (uint32_t j = 0; j < len; j++) o[j] = (uint8_t)r();
      return;
    }
    gen_text(seed, o, len, V);
    if (kind == 1) {
      XS r(seed ^ 0x85ebca6bu);
      for (uint32_t k = 0; k + 8192 <= len; k += 8192)
        for (uint32_t j = 0; j < 1024; j++) o[k + 4096 + j] = (uint8_t)r();
    }
  };
  if (threads < 1) threads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (uint32_t i = (uint32_t)t; i < n_streams; i += (uint32_t)threads) one(i);
    });
  for (auto& x : th) x.join();
}

// ------------------------------------------------------------ introspection
// Copies an intermediate array of stream `s` of the last deflate batch to host
// memory: what = 0 prevd (u16/position, 0xffff = no link), 1 match table (u32x2/position),
// 2 symbols (u32 each; count = streams[s].nsym), 3 blocks (zs_block each),
// 4 stream record (zs_stream).  Returns the number of bytes copied.
extern "C" uint64_t zs_debug_fetch(zs_ctx* c, int what, uint32_t s, void* dst, uint64_t cap) {
  if (c && what >= 16 && what <= 21) {
    // the segmented decode's records of the last inflate batch: 16 counters (-, members
    // finished), 17 spans (zs_seg_blk), 18 lanes (zs_seg_lane), 19 members (zs_seg_mem), 20 found[]
    // (big members), 21 entries (zs_seg_ent)
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    const Buf* b = what == 16 ? &c->gcnt : what == 17 ? &c->gblk : what == 18 ? &c->glanes : what == 19 ? &c->gmem
                   : what == 21 ? &c->gent : &c->gfound;
    const uint64_t bytes = std::min<uint64_t>(cap, b->cap);
    if (!b->p || !bytes || hipMemcpy(dst, b->p, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return bytes;
  }
  if (!c || !c->streams.p) return 0;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  (void)hipDeviceSynchronize();
  zs_stream st;
  if (hipMemcpy(&st, c->streams.as<zs_stream>() + s, sizeof st, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  uint64_t pos_base = 0;
  uint32_t blk_base = 0, n = 0;
  // meta layout of the last call: recompute offsets from the host copy
  const size_t nstreams = c->last_n;
  MetaLayout m2((uint32_t)nstreams);
  const uint8_t* hm = c->hmeta.data();
  pos_base = ((const uint64_t*)(hm + m2.pos_base))[s];
  blk_base = ((const uint32_t*)(hm + m2.blk_base))[s];
  n = ((const uint32_t*)(hm + m2.in_len))[s];
  const void* src = nullptr;
  uint64_t bytes = 0;
  switch (what) {
    case 0: src = c->prevd.as<uint16_t>() + pos_base; bytes = 2ull * n; break;
    case 1: src = c->mres.as<uint2>() + pos_base; bytes = 8ull * n; break;
    case 2: src = c->syms.as<uint32_t>() + pos_base + s; bytes = 4ull * st.nsym; break;
    case 3: src = c->blocks.as<zs_block>() + blk_base; bytes = sizeof(zs_block) * st.nblk; break;
    case 4: src = c->streams.as<zs_stream>() + s; bytes = sizeof(zs_stream); break;
    case 5: src = c->codes.as<uint32_t>() + (size_t)blk_base * (ZS_L_CODES + ZS_D_CODES); bytes = 4ull * (ZS_L_CODES + ZS_D_CODES) * st.nblk; break;
    case 6: src = c->hdr.as<uint32_t>() + (size_t)blk_base * ZS_HDR_WORDS; bytes = 4ull * ZS_HDR_WORDS * st.nblk; break;
    default: return 0;
  }
  bytes = std::min(bytes, cap);
  if (bytes && hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return bytes;
}

// ------------------------------------------------------------------ inflate
static const char* kInflateMsgs[ZS_MSG_COUNT] = {
    "",
    "incorrect header check",
    "unknown compression method",
    "invalid window size",
    "unknown header flags set",
    "header crc mismatch",
    "invalid block type",
    "invalid stored block lengths",
    "too many length or distance symbols",
    "too many length",
    "invalid code lengths set",
    "invalid bit length repeat",
    "invalid code -- missing end-of-block",
    "invalid literal/lengths set",
    "invalid distances set",
    "invalid literal/length code",
    "invalid distance code",
    "invalid distance too far back",
    "incorrect data check",
    "incorrect length check",
    "output capacity exceeded",
};

extern "C" const char* zs_inflate_message(int32_t i) { return (i >= 0 && i < ZS_MSG_COUNT) ? kInflateMsgs[i] : ""; }

__global__ void zs_k_inflate_finish(const zs_inflate_result* r, const zs_lane_res* lane, int32_t* status,
                                    int32_t* phase, int32_t* msg, uint32_t* out_len, uint32_t* consumed, int n,
                                    uint32_t* lane_count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  if (lane && lane[s].bail == 0) {  // clean member from the lane path
    atomicAdd(lane_count, 1u);
    status[s] = ZS_Z_STREAM_END;
    phase[s] = ZS_PHASE_NONE_;
    msg[s] = ZS_MSG_NONE;
    out_len[s] = lane[s].out_len;
    consumed[s] = lane[s].consumed;
    return;
  }
  status[s] = r[s].status;
  phase[s] = r[s].phase;
  msg[s] = r[s].msg;
  out_len[s] = r[s].out_len;
  consumed[s] = r[s].consumed;
}

// Per-stream check value (the reference's strm.adler after a successful
// stream, inflate.ts:105,1014,1080): the adler32 (zlib) / crc32 (gzip) of the
// output -- equal to the verified trailer, so read from it; 0 for raw and
// deflate64-raw (createStream's initial _adler, common/utils.ts:49, never
// updated without a wrapper) and for a failed stream.
__global__ void zs_k_inflate_check(const uint8_t* in, const uint64_t* in_off, const int32_t* status,
                                   const uint32_t* consumed, int wbits, uint32_t* out, int n) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  uint32_t v = 0;
  if (status[s] == ZS_Z_STREAM_END && wbits > 0) {
    const uint8_t* t = in + in_off[s] + consumed[s] - (wbits == 31 ? 8 : 4);
    v = wbits == 31 ? (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24
                    : (uint32_t)t[0] << 24 | (uint32_t)t[1] << 16 | (uint32_t)t[2] << 8 | (uint32_t)t[3];
  }
  out[s] = v;
}

// The segmented decode of the members in c->hglist (inflate_seg.hip) on the side
// stream, after the caller's stream reaches this point; then the wave kernel over
// the same members for any the pieces could not finish (skip_done: the others
// return at once), the exact kernel after it for whatever fails there.
// a member's pieces' bound and its u16 scratch elements in the segmented decode (seg_launch)
static uint32_t seg_pmax(uint32_t in_len) {
  const uint64_t nbits = 8ull * in_len;
  const uint64_t spans = nbits / ZS_SEG_BLOCK_BITS + 2 * nbits / (64ull * ZS_SEG_W) + 8;
  // (x 2: split mode cuts pieces in two)
  return 2u * (uint32_t)std::min<uint64_t>(spans * ZS_SEG_LANES, nbits / ZS_SEG_W + spans + 1);
}
static uint64_t seg_scratch_elems(uint32_t in_len, uint32_t out_cap) {
  return (((uint64_t)out_cap + 7) & ~7ull) + ZS_SEG_PAD * (uint64_t)seg_pmax(in_len) + 16;
}

static int seg_launch(zs_ctx* c, hipStream_t st, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* d_ioff,
                      const uint32_t* d_ilen, uint8_t* d_out, const uint64_t* d_ooff, const uint32_t* d_ocap,
                      const uint32_t* in_len, const uint32_t* out_cap, zs_lane_res* lres) {
  const uint32_t ng = (uint32_t)c->hglist.size();
  const bool d64 = wbits == -16;
  const bool refw = c->inflate_ref_wrap && !d64;
  // per member: span slots (one per ZS_SEG_BLOCK_BITS input bits for the blocks, twice the
  // spans of the narrowest lanes, 8 more), the pieces' bound and their u16
  // scratch (each piece 16-byte aligned and padded); members over seg_big_bits
  // input bits also walk from the finder's block starts
  c->hgpbase.assign(ng + 1, 0);
  c->hgsbase.assign(ng + 1, 0);
  c->hgspb.assign(ng + 1, 0);
  c->hgbig.clear();
  for (uint32_t k = 0; k < ng; k++) {
    const uint32_t i = c->hglist[k];
    const uint64_t nbits = 8ull * in_len[i];
    const uint64_t spans = 2 * (nbits / ZS_SEG_BLOCK_BITS + 2 * nbits / (64ull * ZS_SEG_W) + 8);  // (x 2: split mode)
    c->hgspb[k + 1] = c->hgspb[k] + (uint32_t)spans;
    c->hgpbase[k + 1] = c->hgpbase[k] + seg_pmax(in_len[i]);
    c->hgsbase[k + 1] = c->hgsbase[k] + seg_scratch_elems(in_len[i], out_cap[i]);
    if (nbits > c->seg_big_bits) c->hgbig.push_back(k);
  }
  const uint32_t nb = c->hgspb[ng], nbig = (uint32_t)c->hgbig.size();
  HIPCHK(c->glist.ensure(4ull * ng));
  HIPCHK(c->gspb.ensure(4ull * (ng + 1)));
  HIPCHK(c->gbig.ensure(4ull * nbig + 4));
  HIPCHK(c->gfound.ensure(8ull * ZS_SPLIT_MAX * nbig + 8));
  HIPCHK(c->gblk.ensure(sizeof(zs_seg_blk) * nb));
  HIPCHK(c->glanes.ensure(sizeof(zs_seg_lane) * ZS_SEG_LANES * nb));
  HIPCHK(c->gtab.ensure(sizeof(zcode) * ZS_SEG_TAB * nb));
  HIPCHK(c->gent.ensure(sizeof(zs_seg_ent) * ZS_SPLIT_MAX * ng));
  HIPCHK(c->gmem.ensure(sizeof(zs_seg_mem) * ng));
  HIPCHK(c->gpbase.ensure(4ull * (ng + 1)));
  HIPCHK(c->gplist.ensure(16ull * c->hgpbase[ng] + 16));
  HIPCHK(c->gsbase.ensure(8ull * (ng + 1)));
  HIPCHK(c->gscr.ensure(2ull * c->hgsbase[ng] + 64));
  HIPCHK(c->gcnt.ensure(16));
  // the big members' stream indices for the finder, then their list indices for the walk
  c->hgbig_s.resize(nbig);
  for (uint32_t k = 0; k < nbig; k++) c->hgbig_s[k] = c->hglist[c->hgbig[k]];
  HIPCHK(hipMemcpyAsync(c->glist.p, c->hglist.data(), 4ull * ng, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->gspb.p, c->hgspb.data(), 4ull * (ng + 1), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->gpbase.p, c->hgpbase.data(), 4ull * (ng + 1), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->gsbase.p, c->hgsbase.data(), 8ull * (ng + 1), hipMemcpyHostToDevice, st));
  if (nbig) {
    HIPCHK(c->gbigs.ensure(4ull * nbig));
    HIPCHK(hipMemcpyAsync(c->gbigs.p, c->hgbig_s.data(), 4ull * nbig, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->gbig.p, c->hgbig.data(), 4ull * nbig, hipMemcpyHostToDevice, st));
  }
  // fresh records: members (span counters), entries (start 0 = none), spans (member NONE)
  HIPCHK(hipMemsetAsync(c->gmem.p, 0, sizeof(zs_seg_mem) * ng, st));
  HIPCHK(hipMemsetAsync(c->gent.p, 0, sizeof(zs_seg_ent) * ZS_SPLIT_MAX * ng, st));
  HIPCHK(hipMemsetAsync(c->gblk.p, 0xff, sizeof(zs_seg_blk) * nb, st));
  // the spans taken (the decode's work list), and (unless a later chunk of one host batch) the members finished
  HIPCHK(c->gspl.ensure(4ull * nb + 4));
  HIPCHK(c->gflist.ensure(4ull * ng));
  HIPCHK(hipMemsetAsync(c->gcnt.as<uint32_t>() + 2, 0, 8, st));  // spans taken, members left over
  if (!c->keep_counts) HIPCHK(hipMemsetAsync(c->gcnt.p, 0, 8, st));
  HIPCHK(hipEventRecord(c->fork, st));
  HIPCHK(hipStreamWaitEvent(c->side, c->fork, 0));
  hipStream_t sd = c->side;
  if (int r = mark(c, sd, "start")) return r;
  const uint32_t* gl = c->glist.as<uint32_t>();
  uint64_t* gf = c->gfound.as<uint64_t>();
  uint32_t* cnt = c->gcnt.as<uint32_t>();
  zs_seg_blk* gb = c->gblk.as<zs_seg_blk>();
  zs_seg_lane* gln = c->glanes.as<zs_seg_lane>();
  zcode* gt = c->gtab.as<zcode>();
  zs_seg_ent* ge = c->gent.as<zs_seg_ent>();
  zs_seg_mem* gm = c->gmem.as<zs_seg_mem>();
  const uint32_t* gspb = c->gspb.as<uint32_t>();
  if (nbig) {
    zs_k_split_find<<<nbig * ZS_SPLIT_MAX, 256, 0, sd>>>(d_in, d_ioff, d_ilen, c->gbigs.as<uint32_t>(), wbits, gf);
    if (int r = mark(c, sd, "seg_find")) return r;
  }
  const uint32_t nwalk = ng + nbig * (ZS_SPLIT_MAX - 1u);
  // The sync window: 2048 bits when the walks all fit the chip at once (the 2048-bit
  // instance takes 49 KB of LDS: three per CU) and the members are large (blocks
  // wide enough for lanes of >= 2048 bits), so that fewer neighbours fail to meet
  // (512 x 256 KiB: 5.3 -> 4.2 ms); otherwise 1024 (occupancy: 1,024 x 256 KiB 7.6 vs 6.6 ms)
  uint64_t gbits = 0;
  for (uint32_t k = 0; k < ng; k++) gbits += 8ull * in_len[c->hglist[k]];
  const bool large = gbits >= 65536ull * 8 * ng;  // members of 64 KiB of input or more on average
  const bool w2k = c->seg_wide && nwalk <= 3u * c->ncu && large;
  // (large deflate members: the instance whose lanes decode the stretch between their sync windows
  // without the windows' bookkeeping)
  auto walk = d64 ? (w2k ? zs_k_seg_walk<true, 2048u, false> : zs_k_seg_walk<true, 1024u, false>)
                  : (w2k ? zs_k_seg_walk<false, 2048u, true>
                         : large ? zs_k_seg_walk<false, 1024u, true> : zs_k_seg_walk<false, 1024u, false>);
  // bits per lane: large members (4,096 x 256 KiB: 17.2 -> 15.9 ms, its 512-member shard 3.70 -> 3.57) walk fewer,
  // wider spans; 64 KiB members keep 2048 (the 1,024-member gunzip shard: 2.11 vs 2.45 ms, the decode's pieces
  // too few to fill the chip) -- tools/segbits_ab.sh
  const uint32_t sbits = c->seg_bits ? c->seg_bits : gbits >= (1ull << 19) * ng ? 4096u : 2048u;
  // Split mode: the plan cuts each piece in two at the first symbol start past its lane's middle (the walk
  // records it), so the decode runs twice the pieces, each half as long.  The resolve then takes twice the
  // rounds (one piece per round) and the plan twice the steps, so it pays only where the decode of few large
  // members leaves SIMDs idle: a rank's 512 x 256 KiB shard 3.13 -> 2.93 ms (decode 1.36 -> 0.78, plan
  // 0.08 -> 0.20, resolve 0.30 -> 0.50); 1,024 x 256 KiB 5.07 -> 5.52, C5-i's 1,024 x 64 KiB 1.93 -> 2.09
  // (profiles/r06/seg/split_*)
  const int split = c->seg_split == 2 ? (ng <= 2u * c->ncu && large ? 1 : 0) : c->seg_split;
  walk<<<nwalk, 64, 0, sd>>>(d_in, d_ioff, d_ilen, gl, ng, c->gbig.as<uint32_t>(), nbig, wbits, gf, gspb, gb, gln, gt,
                             ge, gm, cnt + 2, c->gspl.as<uint32_t>(), std::max<uint32_t>(sbits, w2k ? 2048u : 0u),
                             split);
  if (int r = mark(c, sd, "seg_walk")) return r;
  zs_k_seg_plan<<<ng, 64, 0, sd>>>(d_in, d_ioff, d_ilen, d_ocap, gl, ng, wbits, refw ? 1 : 0, gb, gln, ge, gm,
                                   c->gpbase.as<uint32_t>(), c->gplist.as<uint4>());
  if (int r = mark(c, sd, "seg_plan")) return r;
  const uint64_t* sb = c->gsbase.as<uint64_t>();
  uint16_t* scr = c->gscr.as<uint16_t>();
  // one wave per span taken, grid-stride over the work list
  const uint32_t gdec = std::min<uint32_t>(nb, 8192u);
  const uint32_t* spl = c->gspl.as<uint32_t>();
  if (d64)
    zs_k_seg_decode<true, false><<<gdec, 64, 0, sd>>>(d_in, d_ioff, d_ilen, gl, cnt + 2, spl, gb, gln, gt, gm, sb, scr);
  else if (refw)
    zs_k_seg_decode<false, true><<<gdec, 64, 0, sd>>>(d_in, d_ioff, d_ilen, gl, cnt + 2, spl, gb, gln, gt, gm, sb, scr);
  else
    zs_k_seg_decode<false, false><<<gdec, 64, 0, sd>>>(d_in, d_ioff, d_ilen, gl, cnt + 2, spl, gb, gln, gt, gm, sb, scr);
  if (int r = mark(c, sd, "seg_decode")) return r;
  // the resolve: four members per CU (256 threads, a 32 KiB ring) unless the batch is too small to fill them
  const bool rsmall = ng <= 2u * c->ncu;
  const int rsm = rsmall ? 65536 : 32768;
  auto resolve = rsmall ? zs_k_seg_resolve<512u, 65536u> : zs_k_seg_resolve<256u, 32768u>;
  HIPCHK(hipFuncSetAttribute((const void*)resolve, hipFuncAttributeMaxDynamicSharedMemorySize, rsm));
  resolve<<<ng, rsmall ? 512u : 256u, rsm, sd>>>(gl, gm, c->gpbase.as<uint32_t>(), c->gplist.as<uint4>(), sb, scr, d_out,
                                           d_ooff, lres, c->llen.as<uint32_t>(), cnt + 1, cnt + 3,
                                           c->gflist.as<uint32_t>());
  if (int r = mark(c, sd, "seg_resolve")) return r;
  // members the pieces could not finish: the wave kernel (skip_done), then the exact kernel
  const size_t wsm = zs_inflate_wave_lds_bytes(d64);
  const void* wk = refw ? (const void*)zs_k_inflate_wave<true> : (const void*)zs_k_inflate_wave<false>;
  HIPCHK(hipFuncSetAttribute(wk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wsm));
  // (the members the resolve listed: usually none, so a small grid walks the list)
  const uint32_t gfb = std::min<uint32_t>(ng, 256u);
  const uint32_t* fl = c->gflist.as<uint32_t>();
  if (refw)
    zs_k_inflate_wave<true><<<gfb, 64, wsm, sd>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, fl, ng, lres,
                                                  c->llen.as<uint32_t>(), cnt + 3);
  else
    zs_k_inflate_wave<false><<<gfb, 64, wsm, sd>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, fl, ng, lres,
                                                   c->llen.as<uint32_t>(), cnt + 3);
  HIPCHK(hipGetLastError());
  if (int r = mark(c, sd, "seg_fallback")) return r;
  (void)n;
  (void)d_ocap;
  return ZS_OK;
}

extern "C" int zs_inflate_batch_device(zs_ctx* c, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                                       const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off,
                                       const uint32_t* out_cap, int32_t* d_status, int32_t* d_phase, int32_t* d_msg,
                                       uint32_t* d_out_len, uint32_t* d_consumed, void* hip_stream) {
  return zs_inflate_batch_device_ex(c, wbits, n, d_in, in_off, in_len, d_out, out_off, out_cap, d_status, d_phase,
                                    d_msg, d_out_len, d_consumed, nullptr, hip_stream);
}

// The device decode.  out_cap[i] is the member's capacity as the caller set it
// (Z_BUF_ERROR past it, exactly); the decoders store whole dwords, so the
// member's region must reach out_off[i] + out_cap[i] rounded up to 4.
// `caller_regions`: the regions are the caller's own buffers (the public
// device entries), so capacities must be multiples of 4 -- no store may pass
// the last member's end.  The host entries decode into their own staging,
// whose regions are the capacities rounded up, and pass their callers' exact
// capacities with caller_regions = false.
static int inflate_device(zs_ctx* c, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                          const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off, const uint32_t* out_cap,
                          int32_t* d_status, int32_t* d_phase, int32_t* d_msg, uint32_t* d_out_len,
                          uint32_t* d_consumed, uint32_t* d_check, void* hip_stream, bool caller_regions);

extern "C" int zs_inflate_batch_device_ex(zs_ctx* c, int wbits, uint32_t n, const uint8_t* d_in,
                                          const uint64_t* in_off, const uint32_t* in_len, uint8_t* d_out,
                                          const uint64_t* out_off, const uint32_t* out_cap, int32_t* d_status,
                                          int32_t* d_phase, int32_t* d_msg, uint32_t* d_out_len,
                                          uint32_t* d_consumed, uint32_t* d_check, void* hip_stream) {
  return inflate_device(c, wbits, n, d_in, in_off, in_len, d_out, out_off, out_cap, d_status, d_phase, d_msg,
                        d_out_len, d_consumed, d_check, hip_stream, true);
}

static int inflate_device(zs_ctx* c, int wbits, uint32_t n, const uint8_t* d_in, const uint64_t* in_off,
                          const uint32_t* in_len, uint8_t* d_out, const uint64_t* out_off, const uint32_t* out_cap,
                          int32_t* d_status, int32_t* d_phase, int32_t* d_msg, uint32_t* d_out_len,
                          uint32_t* d_consumed, uint32_t* d_check, void* hip_stream, bool caller_regions) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  // inflateInit2_ / inflateReset2 validation (inflate.ts:138-192) for the stream-layer formats
  if (!(wbits == -15 || wbits == 15 || wbits == 31 || wbits == -16))
    return fail(ZS_STREAM_ERROR, "unsupported windowBits (use -15, 15, 31 or -16)");
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  if (!c->keep_counts) c->seg_used = false;
  // the decoders store whole dwords (up to 3 bytes past a member's end): offsets are
  // multiples of 4, and so are the capacities of regions the caller owns
  for (uint32_t i = 0; i < n; i++)
    if ((out_off[i] & 3) || (caller_regions && (out_cap[i] & 3)))
      return fail(ZS_STREAM_ERROR, "output offsets/capacities must be multiples of 4");
  MetaLayout ml(n);
  c->hmeta.resize(ml.bytes);
  c->last_n = n;
  uint8_t* hm = c->hmeta.data();
  memcpy(hm + ml.in_off, in_off, 8ull * n);
  memcpy(hm + ml.in_len, in_len, 4ull * n);
  memcpy(hm + ml.out_off, out_off, 8ull * n);
  memcpy(hm + ml.out_cap, out_cap, 4ull * n);
  HIPCHK(c->meta.ensure(ml.bytes));
  HIPCHK(c->istate.ensure(sizeof(zs_inflate_result) * (size_t)n));
  HIPCHK(hipMemcpyAsync(c->meta.p, hm, ml.bytes, hipMemcpyHostToDevice, st));
  uint8_t* dm = c->meta.as<uint8_t>();
  const size_t smem = zs_inflate_smem_bytes(wbits);
  HIPCHK(hipFuncSetAttribute((const void*)zs_k_inflate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
  const uint64_t* d_ioff = (const uint64_t*)(dm + ml.in_off);
  const uint32_t* d_ilen = (const uint32_t*)(dm + ml.in_len);
  const uint64_t* d_ooff = (const uint64_t*)(dm + ml.out_off);
  const uint32_t* d_ocap = (const uint32_t*)(dm + ml.out_cap);
  zs_lane_res* lres = nullptr;
  MARK("start");
  if (c->inflate_fast) {
    // lane-per-member fast path; anything but a clean end of stream goes to the exact kernel.
    // A lane's decode is a dependent chain of loads, so the chip wants many
    // waves more than full ones: up to 16,384 members, thin workgroups (one
    // wave each) until ~4096 waves; above, 1024 waves of up to 64 members.
    // Measured (MI355X): 65,536 members want 64 per workgroup (every lane resident at
    // once, 548 B of LDS each); 8,192 want two (C5-i 29.5 -> 23.7 ms at 8 -> 2: four
    // waves per SIMD hide each other's waits, with little divergence inside each).
    uint32_t B = (uint32_t)c->lane_block;
    if (!B) {
      if (n <= 16384u)
        for (B = 1; B < 64 && (n + B - 1) / B > 4608u;) B <<= 1;  // (~4096 waves; a few members over 8,192 keep two per wave)
      else
        for (B = 64; B > 8 && (n + B - 1) / B < 1024u;) B >>= 1;
    }
    HIPCHK(c->ltabs.ensure(zs_inflate_lane_scratch_bytes() * (size_t)n));
    HIPCHK(c->lres.ensure(sizeof(zs_lane_res) * (size_t)n));
    HIPCHK(c->llen.ensure(8ull * n));
    lres = c->lres.as<zs_lane_res>();
    // narrow workgroups afford per-lane root tables (inflate_lane.hip)
    const bool lroot = B <= 16;
    const size_t lsm = B * zs_inflate_lane_lds_bytes(lroot);
    // Large members (more than inflate_wave_min input bytes) decode one per wave
    // on the side stream, beside the lane kernel: one lane would take the
    // batch's whole time on such a member.  The wave kernel tracks the
    // reference's inflate() calls and reproduces their window-wrap copy
    // (inflate_wave.hip, zs_refcalls); the lane kernel skips exactly these members.
    uint32_t wave_min = 0;
    c->hwlist.clear();
    c->hslist.clear();
    c->hglist.clear();
    // "Large" members decode beside the lane kernel.  With the segmented decode on,
    // a small batch's members are large from seg_small_min bytes on: one lane each
    // would leave most of the chip idle (the per-rank shards of the 8-GPU configs).
    uint32_t big_min = c->inflate_wave_min;
    if (c->inflate_seg && n <= c->seg_small_batch && c->seg_small_min && (!big_min || c->seg_small_min < big_min))
      big_min = c->seg_small_min;
    // Large raw members whose decode carries no call-boundary behaviour
    // (deflate64; raw deflate without the window-wrap copy) are cut at their
    // block boundaries and decoded piecewise (inflate_split.hip); the rest of
    // the large members take the wave kernel.  The pieces' u16 scratch is
    // bounded: members past kSplitScratch take the wave kernel too.
    const bool splittable = c->inflate_split && (wbits == -16 || (wbits == -15 && !c->inflate_ref_wrap));
    uint32_t piece_cap = 0;
    uint64_t val_stride = 0;  // u32 values per split member
    if (big_min) {
      constexpr size_t kSplitScratch = 2ull << 30;
      constexpr uint32_t kPieceCapMax = 4u << 20;  // values per piece
      // the segmented decode's u16 scratch (2 bytes per byte of capacity) is
      // bounded too (option seg_scratch_mb): members past it take the split / wave kernels
      uint64_t seg_bytes = 0;
      for (uint32_t i = 0; i < n; i++) {
        if (!zs_inf_large(in_len[i], out_cap[i], big_min)) continue;
        // (the segmented decode keeps bit positions in 32 bits; members with long
        // blocks or long copies -- large deflate64 ones, high expansions -- decode
        // faster with a wave per block / per member, which copies 64 bytes at a time)
        const bool longcopies = zs_inf_expands(in_len[i], out_cap[i]) ||
                                (wbits == -16 && 8ull * in_len[i] > ZS_SEG_SPLIT_BITS);
        if (c->inflate_seg && in_len[i] < (1u << 29) && !longcopies &&
            seg_bytes + 2 * seg_scratch_elems(in_len[i], out_cap[i]) <= c->seg_scratch_max) {
          seg_bytes += 2 * seg_scratch_elems(in_len[i], out_cap[i]);
          c->hglist.push_back(i);
          continue;
        }
        const uint32_t pc = (std::min(out_cap[i], kPieceCapMax) + 1u) & ~1u;
        const uint32_t npc = std::max(piece_cap, pc);
        const uint64_t nvs = std::max<uint64_t>(val_stride, (out_cap[i] + 3ull) & ~3ull);
        if (splittable && (2ull * ZS_SPLIT_MAX * npc + 4ull * nvs) * (c->hslist.size() + 1) <= kSplitScratch) {
          c->hslist.push_back(i);
          piece_cap = npc;
          val_stride = nvs;
        } else {
          c->hwlist.push_back(i);
        }
      }
      if (!c->hwlist.empty() || !c->hslist.empty() || !c->hglist.empty()) wave_min = big_min;
    }
    if (!c->hslist.empty()) {  // on the third stream (high priority), beside the segmented decode
      const uint32_t ns = (uint32_t)c->hslist.size();
      HIPCHK(c->slist.ensure(4ull * ns));
      HIPCHK(c->sfound.ensure(8ull * ZS_SPLIT_MAX * ns));
      HIPCHK(c->spres.ensure(sizeof(zs_split_piece_res) * ZS_SPLIT_MAX * ns));
      HIPCHK(c->sscr.ensure(2ull * ZS_SPLIT_MAX * piece_cap * ns));
      HIPCHK(hipMemcpyAsync(c->slist.p, c->hslist.data(), 4ull * ns, hipMemcpyHostToDevice, st));
      HIPCHK(hipEventRecord(c->fork, st));
      HIPCHK(hipStreamWaitEvent(c->side2, c->fork, 0));
      if (int r = mark(c, c->side2, "start")) return r;
      const uint32_t* sl = c->slist.as<uint32_t>();
      uint64_t* sf = c->sfound.as<uint64_t>();
      zs_split_piece_res* sp = c->spres.as<zs_split_piece_res>();
      zs_k_split_find<<<ns * ZS_SPLIT_MAX, 256, 0, c->side2>>>(d_in, d_ioff, d_ilen, sl, wbits, sf);
      if (int r = mark(c, c->side2, "split_find")) return r;
      const size_t ssm = zs_split_lds_bytes(wbits == -16);
      HIPCHK(hipFuncSetAttribute((const void*)zs_k_split_decode, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ssm));
      zs_k_split_decode<<<ns * ZS_SPLIT_MAX, 64, ssm, c->side2>>>(d_in, d_ioff, d_ilen, sl, wbits, sf, sp,
                                                                  c->sscr.as<uint16_t>(), piece_cap);
      if (int r = mark(c, c->side2, "split_decode")) return r;
      HIPCHK(c->smem.ensure(sizeof(zs_split_member) * ns));
      HIPCHK(c->sval.ensure(4ull * val_stride * ns + 16));
      zs_split_member* sm = c->smem.as<zs_split_member>();
      uint32_t* sv = c->sval.as<uint32_t>();
      zs_k_split_chain<<<(ns + 63) / 64, 64, 0, c->side2>>>(d_ilen, d_ocap, sl, ns, sp, sm);
      zs_k_split_place<<<ns * ZS_SPLIT_MAX, 256, 0, c->side2>>>(sp, sm, c->sscr.as<uint16_t>(), piece_cap, sv, val_stride);
      // the jump and write grids cover the largest member (grid-stride beyond)
      const uint32_t gx = (uint32_t)std::min<uint64_t>(1024, (val_stride + 1023) / 1024);
      for (int k = 0; k < 6; k++) zs_k_split_jump<<<dim3(gx, ns), 256, 0, c->side2>>>(sm, sv, val_stride);
      zs_k_split_write<<<dim3(gx, ns), 256, 0, c->side2>>>(sl, sm, sv, val_stride, d_out, d_ooff);
      zs_k_split_final<<<(ns + 63) / 64, 64, 0, c->side2>>>(sl, ns, sm, lres, c->llen.as<uint32_t>());
      HIPCHK(hipGetLastError());
      if (int r = mark(c, c->side2, "split_resolve")) return r;
      HIPCHK(hipEventRecord(c->join2, c->side2));
    }
    // the segmented decode after the split kernels are queued: its grids would
    // otherwise fill the chip ahead of the split decode's few long pieces (C5-ii:
    // the 2.19 MB fixture's split decode took 8.0 ms beside it, 2.5 ms alone)
    c->seg_used |= !c->hglist.empty();
    if (!c->hglist.empty()) {
      const int r = seg_launch(c, st, wbits, n, d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, in_len, out_cap, lres);
      if (r != ZS_OK) return r;
      // (the join below waits for the side stream's last kernel)
      if (c->hwlist.empty()) HIPCHK(hipEventRecord(c->join, c->side));
    }
    if (!c->hwlist.empty()) {
      const uint32_t nw = (uint32_t)c->hwlist.size();
      HIPCHK(c->wlist.ensure(4ull * nw));
      HIPCHK(hipMemcpyAsync(c->wlist.p, c->hwlist.data(), 4ull * nw, hipMemcpyHostToDevice, st));
      HIPCHK(hipEventRecord(c->fork, st));
      HIPCHK(hipStreamWaitEvent(c->side, c->fork, 0));
      const size_t wsm = zs_inflate_wave_lds_bytes(wbits == -16);
      // deflate64 never runs inflate_fast in the reference: no window-wrap copy to reproduce
      const bool refw = c->inflate_ref_wrap && wbits != -16;
      const void* wk = refw ? (const void*)zs_k_inflate_wave<true> : (const void*)zs_k_inflate_wave<false>;
      HIPCHK(hipFuncSetAttribute(wk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wsm));
      if (int r = mark(c, c->side, "start")) return r;
      // Many large members: one lane each (the lane kernel's REFW instance,
      // the reference's calls tracked per lane) -- a wave per member keeps its
      // bookkeeping in scalars, and the waves of a CU share one scalar unit
      // (4,096 x 256 KiB: wave kernel 176 ms)
      bool lanes = refw && c->lane_large_min && nw >= c->lane_large_min;
      for (uint32_t i = 0; lanes && i < nw; i++) lanes = in_len[c->hwlist[i]] < (1u << 29);  // 32-bit bit positions
      if (lanes) {
        // thin workgroups to ~4096 waves (4,096 x 256 KiB: one lane per wave 95 ms, two 110, four 144)
        uint32_t B2 = 1;
        while (B2 < 64 && (nw + B2 - 1) / B2 > 4096u) B2 <<= 1;
        const bool lroot2 = B2 <= 16;
        const size_t lsm2 = B2 * zs_inflate_lane_lds_bytes(lroot2);
        const void* lk2 = lroot2 ? (const void*)zs_k_inflate_lane<2, true> : (const void*)zs_k_inflate_lane<0, true>;
        HIPCHK(hipFuncSetAttribute(lk2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lsm2));
        if (lroot2)
          zs_k_inflate_lane<2, true><<<(nw + B2 - 1) / B2, B2, lsm2, c->side>>>(
              d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, nw, (zs_lane_tabs*)c->ltabs.p, lres,
              c->llen.as<uint32_t>(), ZS_INF_REF_WRAP, 0u, c->wlist.as<uint32_t>());
        else
          zs_k_inflate_lane<0, true><<<(nw + B2 - 1) / B2, B2, lsm2, c->side>>>(
              d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, nw, (zs_lane_tabs*)c->ltabs.p, lres,
              c->llen.as<uint32_t>(), ZS_INF_REF_WRAP, 0u, c->wlist.as<uint32_t>());
      } else if (refw)
        zs_k_inflate_wave<true><<<nw, 64, wsm, c->side>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits,
                                                          c->wlist.as<uint32_t>(), nw, lres, c->llen.as<uint32_t>(),
                                                          nullptr);
      else
        zs_k_inflate_wave<false><<<nw, 64, wsm, c->side>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits,
                                                           c->wlist.as<uint32_t>(), nw, lres, c->llen.as<uint32_t>(),
                                                          nullptr);
      HIPCHK(hipGetLastError());
      if (int r = mark(c, c->side, lanes ? "inflate_large" : "inflate_wave")) return r;
      HIPCHK(hipEventRecord(c->join, c->side));
    }
    // Narrow workgroups with large members beside them (side stream): the
    // LDS-canon instance, 68 VGPRs, so the side stream's waves find slots on
    // every SIMD (C5-ii: 34 -> 26 ms); alone, the register instance (C5-i:
    // 24.4 vs 25.7 ms)
    const int rt = !lroot ? 0 : wave_min ? 2 : 1;
    const void* lk = rt == 2 ? (const void*)zs_k_inflate_lane<2, false>
                   : rt == 1 ? (const void*)zs_k_inflate_lane<1, false> : (const void*)zs_k_inflate_lane<0, false>;
    HIPCHK(hipFuncSetAttribute(lk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lsm));
    const uint32_t lgrid = (n + B - 1) / B;
    const int lflags = c->inflate_ref_wrap ? ZS_INF_REF_WRAP : 0;
    zs_lane_tabs* const lt = (zs_lane_tabs*)c->ltabs.p;
    if (rt == 2)
      zs_k_inflate_lane<2, false><<<lgrid, B, lsm, st>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, n, lt, lres,
                                                         c->llen.as<uint32_t>(), lflags, wave_min, nullptr);
    else if (rt == 1)
      zs_k_inflate_lane<1, false><<<lgrid, B, lsm, st>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, n, lt, lres,
                                                         c->llen.as<uint32_t>(), lflags, wave_min, nullptr);
    else
      zs_k_inflate_lane<0, false><<<lgrid, B, lsm, st>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits, n, lt, lres,
                                                         c->llen.as<uint32_t>(), lflags, wave_min, nullptr);
    MARK("inflate_lane");
    // Members the single-call instance bailed on whose cap allows more than one
    // inflate() call of the reference (more than 32 KiB of input, or output past
    // 64 KiB): re-run by the call-tracking instance, here, before the exact kernel
    if (c->inflate_ref_wrap && wbits != -16) {
      const size_t lsmr = 64 * zs_inflate_lane_lds_bytes(false);
      HIPCHK(hipFuncSetAttribute((const void*)zs_k_inflate_lane<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lsmr));
      zs_k_inflate_lane<0, true><<<(n + 63) / 64, 64, lsmr, st>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits,
                                                                  n, lt, lres, c->llen.as<uint32_t>(), ZS_INF_REF_WRAP,
                                                                  wave_min, nullptr);
      MARK("inflate_long");
    }
    if (wave_min) {
      if (!c->hglist.empty() || !c->hwlist.empty()) HIPCHK(hipStreamWaitEvent(st, c->join, 0));
      if (!c->hslist.empty()) HIPCHK(hipStreamWaitEvent(st, c->join2, 0));
      MARK("inflate_join");  // the caller's stream waiting for the side streams beyond the lane kernel
    }
    if (wbits > 0) {  // trailer checks over the decoded bytes: adler32 (zlib) / crc32 (gzip)
      uint32_t* chk = c->llen.as<uint32_t>() + n;
      zs_k_checksum<<<n, 64, 0, st>>>(d_out, d_ooff, c->llen.as<uint32_t>(), chk, wbits == 31 ? 2 : 1);
      zs_k_inflate_lane_verify<<<(n + 255) / 256, 256, 0, st>>>(lres, chk, n);
      MARK("inflate_check");
    }
  }
  zs_k_inflate<<<n, 64, smem, st>>>(d_in, d_ioff, d_ilen, d_out, d_ooff, d_ocap, wbits,
                                    c->istate.as<zs_inflate_result>(), lres, c->inflate_ref_wrap ? ZS_INF_REF_WRAP : 0);
  MARK("inflate");
  HIPCHK(c->lstat.ensure(16));
  if (!c->keep_counts) HIPCHK(hipMemsetAsync(c->lstat.p, 0, 4, st));
  zs_k_inflate_finish<<<(n + 255) / 256, 256, 0, st>>>(c->istate.as<zs_inflate_result>(), lres, d_status, d_phase,
                                                       d_msg, d_out_len, d_consumed, (int)n, c->lstat.as<uint32_t>());
  if (!c->lane_count_host) {
    HIPCHK(hipHostMalloc((void**)&c->lane_count_host, 64, hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&c->lane_ev, hipEventDisableTiming));
  }
  HIPCHK(hipMemcpyAsync(c->lane_count_host, c->lstat.p, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(c->lane_ev, st));
  if (d_check)
    zs_k_inflate_check<<<(n + 255) / 256, 256, 0, st>>>(d_in, d_ioff, d_status, d_consumed, wbits, d_check, (int)n);
  MARK("finish");
  HIPCHK(hipGetLastError());
  return ZS_OK;  // timing marks are collected when queried (no wait here)
}

extern "C" int zs_inflate_batch(zs_ctx* c, int wbits, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                const uint32_t* in_len, uint8_t* out, const uint64_t* out_off, const uint32_t* out_cap,
                                int32_t* status, int32_t* phase, int32_t* msg, uint32_t* out_len, uint32_t* consumed) {
  return zs_inflate_batch_ex(c, wbits, n, in, in_off, in_len, out, out_off, out_cap, status, phase, msg, out_len,
                             consumed, nullptr);
}

extern "C" int zs_inflate_batch_ex(zs_ctx* c, int wbits, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                   const uint32_t* in_len, uint8_t* out, const uint64_t* out_off,
                                   const uint32_t* out_cap, int32_t* status, int32_t* phase, int32_t* msg,
                                   uint32_t* out_len, uint32_t* consumed, uint32_t* check) {
  if (!c) return fail(ZS_STREAM_ERROR, "null context");
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return ZS_OK;
  // device regions: the caller's capacity rounded up to whole words (the decoders store dwords)
  std::vector<uint32_t> ocap(n), creq(out_cap, out_cap + n);
  for (uint32_t i = 0; i < n; i++) ocap[i] = (uint32_t)std::min<uint64_t>(0xfffffffcull, ((uint64_t)out_cap[i] + 3) & ~3ull);
  uint32_t* res[6] = {(uint32_t*)status, (uint32_t*)phase, (uint32_t*)msg, out_len, consumed, check};
  return host_batch(c, n, in, in_off, in_len, ocap, 6, res, 3, out, out_off,
                    [&](uint32_t a, uint32_t b, const uint64_t* doff, const uint64_t* ooff, const uint32_t*,
                        uint32_t** dr) {
                      // regions of ocap (rounded up) bytes; the caller's exact capacities as the limits
                      return inflate_device(c, wbits, b - a, c->d_in.as<uint8_t>(), doff, in_len + a,
                                            c->d_out.as<uint8_t>(), ooff, creq.data() + a, (int32_t*)dr[0],
                                            (int32_t*)dr[1], (int32_t*)dr[2], dr[3], dr[4], check ? dr[5] : nullptr,
                                            c->stream, false);
                    });
}
