// pool.cpp -- host-side entry points above the per-device context
// (include/zs_gpu.h): unbounded-output decode and the multi-GPU pool.
//
// * zs_inflate_batch_auto: DecompressionStream semantics for the output size.
//   The reference's stream layer loops over pooled 64 KiB output buffers until
//   Z_STREAM_END (src/mod/streams.ts:46,132-182), so a member's output is never
//   capped.  Here a first pass decodes every member into a capacity guessed
//   from its input; the members that ran out of room (ZS_MSG_CAPACITY, a
//   condition the reference cannot have) are decoded again, only they, with
//   eight times the room, until every member fits.  Decoding is deterministic
//   and the capacity only decides whether a member fits, so the bytes, status
//   and message of every member are those of an unbounded decode.
// * zs_pool_*: one context per device of a device mask; a batch is split into
//   contiguous stream ranges shard_range(n, G, k) = [k n / G, (k + 1) n / G)
//   (SURVEY.md 8(e)), one host thread per device, each writing its streams'
//   results straight into the caller's arrays at their own offsets.  No data
//   crosses devices: the host already holds every stream's size, so the only
//   collective of the multi-process path (the RCCL size all-gather,
//   zsamd/shard.py) is not needed inside one process.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zs_gpu.h"
#include "zs_inflate.h"

void zs_set_last_error(const std::string& msg);  // capi.cpp: what zs_last_error() returns on this thread

namespace {

struct Shard {
  uint32_t a, b;
};

Shard shard_range(uint32_t n, uint32_t g, uint32_t k) {
  return {(uint32_t)((uint64_t)n * k / g), (uint32_t)((uint64_t)n * (k + 1) / g)};
}

constexpr uint64_t kCapMax = 0xfffffffcull;  // largest u32 capacity that is a multiple of 4

uint32_t first_cap(uint32_t in_len) {
  const uint64_t c = std::max<uint64_t>(65536, 4ull * in_len);
  return (uint32_t)std::min<uint64_t>(kCapMax, (c + 3) & ~3ull);
}

}  // namespace

extern "C" void zs_free(void* p) { free(p); }

extern "C" int zs_inflate_batch_auto(zs_ctx* c, int wbits, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                     const uint32_t* in_len, uint8_t** out, uint64_t* out_off, int32_t* status,
                                     int32_t* phase, int32_t* msg, uint32_t* out_len, uint32_t* consumed,
                                     uint32_t* check) {
  if (!out || !out_off) return ZS_STREAM_ERROR;
  *out = nullptr;
  // pass buffers: pass 0 holds every member, later passes the retried ones
  // (buffers uninitialised: the host entry writes only the produced bytes, so
  // pages of capacity a member does not use are never touched)
  struct Pass {
    std::vector<uint32_t> idx, cap;
    std::vector<uint64_t> off;
    std::unique_ptr<uint8_t, decltype(&free)> buf{nullptr, &free};
    bool alloc(uint64_t bytes) {
      buf.reset((uint8_t*)malloc(bytes));
      return buf != nullptr;
    }
  };
  std::vector<Pass> passes(1);
  std::vector<uint32_t> where(n, 0);   // the pass a member's final output is in
  std::vector<uint32_t> slot(n, 0);    // its index in that pass
  {
    Pass& p = passes[0];
    p.idx.resize(n);
    p.cap.resize(n);
    p.off.resize(n);
    uint64_t o = 0;
    for (uint32_t i = 0; i < n; i++) {
      p.idx[i] = i;
      p.cap[i] = first_cap(in_len[i]);
      p.off[i] = o;
      o += p.cap[i];
      slot[i] = i;
    }
    if (!p.alloc(o + 4)) return ZS_MEM_ERROR;
    const int r = zs_inflate_batch_ex(c, wbits, n, in, in_off, in_len, p.buf.get(), p.off.data(), p.cap.data(),
                                      status, phase, msg, out_len, consumed, check);
    if (r != ZS_OK) return r;
  }
  for (;;) {
    const Pass& last = passes.back();
    Pass nx;
    uint64_t o = 0;
    for (size_t k = 0; k < last.idx.size(); k++) {
      const uint32_t i = last.idx[k];
      if (!(status[i] == ZS_BUF_ERROR && msg[i] == ZS_MSG_CAPACITY) || last.cap[k] >= kCapMax) continue;
      nx.idx.push_back(i);
      const uint32_t cap = (uint32_t)std::min<uint64_t>(kCapMax, 8ull * last.cap[k]);
      nx.cap.push_back(cap);
      nx.off.push_back(o);
      o += cap;
    }
    if (nx.idx.empty()) break;
    const uint32_t m = (uint32_t)nx.idx.size();
    std::vector<uint64_t> ioff(m);
    std::vector<uint32_t> ilen(m), cons(m), olen(m), chk(m);
    std::vector<int32_t> st(m), ph(m), ms(m);
    for (uint32_t k = 0; k < m; k++) {
      ioff[k] = in_off[nx.idx[k]];
      ilen[k] = in_len[nx.idx[k]];
    }
    if (!nx.alloc(o + 4)) return ZS_MEM_ERROR;
    const int r = zs_inflate_batch_ex(c, wbits, m, in, ioff.data(), ilen.data(), nx.buf.get(), nx.off.data(),
                                      nx.cap.data(), st.data(), ph.data(), ms.data(), olen.data(), cons.data(),
                                      check ? chk.data() : nullptr);
    if (r != ZS_OK) return r;
    for (uint32_t k = 0; k < m; k++) {
      const uint32_t i = nx.idx[k];
      status[i] = st[k];
      phase[i] = ph[k];
      msg[i] = ms[k];
      out_len[i] = olen[k];
      consumed[i] = cons[k];
      if (check) check[i] = chk[k];
      where[i] = (uint32_t)passes.size();
      slot[i] = k;
    }
    passes.push_back(std::move(nx));
  }
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; i++) {
    out_off[i] = total;
    total += out_len[i];
  }
  uint8_t* res = (uint8_t*)malloc(total ? total : 1);
  if (!res) return ZS_MEM_ERROR;
  for (uint32_t i = 0; i < n; i++)
    if (out_len[i]) {
      const Pass& p = passes[where[i]];
      memcpy(res + out_off[i], p.buf.get() + p.off[slot[i]], out_len[i]);
    }
  *out = res;
  return ZS_OK;
}

// ------------------------------------------------------------------ pool
struct zs_pool {
  std::vector<int> devices;
  std::vector<zs_ctx*> ctx;
  std::mutex mtx;  // one batch at a time (the contexts' workspaces are reused)
};

extern "C" int zs_pool_create(uint64_t device_mask, zs_pool** out) {
  if (!out) return ZS_STREAM_ERROR;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    zs_set_last_error("no HIP device");
    return ZS_STREAM_ERROR;
  }
  zs_pool* p = new zs_pool();
  for (int d = 0; d < std::min(ndev, 64); d++)
    if (device_mask == 0 || ((device_mask >> d) & 1u)) p->devices.push_back(d);
  const uint64_t known = ndev >= 64 ? ~0ull : (1ull << ndev) - 1;
  if (p->devices.empty() || (device_mask & ~known) != 0) {
    delete p;
    zs_set_last_error("device mask names no device, or a device that does not exist");
    return ZS_STREAM_ERROR;
  }
  for (int d : p->devices) {
    zs_ctx* c = nullptr;
    const int r = zs_ctx_create(d, &c);
    if (r != ZS_OK) {
      const std::string e = zs_last_error();
      zs_pool_destroy(p);
      zs_set_last_error(e);
      return r;
    }
    p->ctx.push_back(c);
  }
  *out = p;
  return ZS_OK;
}

extern "C" int zs_pool_create_list(const int* devices, int n, zs_pool** out) {
  if (!out || !devices || n <= 0) {
    zs_set_last_error("invalid arguments");
    return ZS_STREAM_ERROR;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    zs_set_last_error("no HIP device");
    return ZS_STREAM_ERROR;
  }
  zs_pool* p = new zs_pool();
  for (int k = 0; k < n; k++) {
    if (devices[k] < 0 || devices[k] >= ndev) {
      delete p;
      zs_set_last_error("device list names a device that does not exist");
      return ZS_STREAM_ERROR;
    }
    p->devices.push_back(devices[k]);
  }
  for (int d : p->devices) {
    zs_ctx* c = nullptr;
    const int r = zs_ctx_create(d, &c);
    if (r != ZS_OK) {
      const std::string e = zs_last_error();
      zs_pool_destroy(p);
      zs_set_last_error(e);
      return r;
    }
    p->ctx.push_back(c);
  }
  *out = p;
  return ZS_OK;
}

extern "C" void zs_pool_destroy(zs_pool* p) {
  if (!p) return;
  for (zs_ctx* c : p->ctx) zs_ctx_destroy(c);
  delete p;
}

extern "C" int zs_pool_size(const zs_pool* p) { return p ? (int)p->devices.size() : 0; }
extern "C" int zs_pool_device(const zs_pool* p, int k) {
  return p && k >= 0 && k < (int)p->devices.size() ? p->devices[k] : -1;
}

// Runs fn(k, shard) for every device k on its own thread; returns the first
// failing code (its message in zs_last_error() on the calling thread).
template <class F>
static int run_sharded(zs_pool* p, uint32_t n, F fn) {
  if (!p) {
    zs_set_last_error("null pool");
    return ZS_STREAM_ERROR;
  }
  std::lock_guard<std::mutex> lk(p->mtx);
  const uint32_t G = (uint32_t)p->ctx.size();
  std::vector<int> rc(G, ZS_OK);
  std::vector<std::string> err(G);
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < G; k++)
    th.emplace_back([&, k] {
      const Shard s = shard_range(n, G, k);
      rc[k] = fn(k, s);
      if (rc[k] != ZS_OK) err[k] = zs_last_error();
    });
  for (auto& t : th) t.join();
  for (uint32_t k = 0; k < G; k++)
    if (rc[k] != ZS_OK) {
      zs_set_last_error("device " + std::to_string(p->devices[k]) + ": " + err[k]);
      return rc[k];
    }
  return ZS_OK;
}

extern "C" int zs_pool_deflate_batch(zs_pool* p, int level, int wbits, uint32_t n, const uint8_t* in,
                                     const uint64_t* in_off, const uint32_t* in_len, uint8_t* out,
                                     const uint64_t* out_off, const uint32_t* out_cap, int32_t* status,
                                     uint32_t* out_len, uint32_t* check) {
  return run_sharded(p, n, [&](uint32_t k, Shard s) {
    if (s.a == s.b) return (int)ZS_OK;
    return zs_deflate_batch_ex(p->ctx[k], level, wbits, s.b - s.a, in, in_off + s.a, in_len + s.a, out,
                               out_off + s.a, out_cap + s.a, status + s.a, out_len + s.a,
                               check ? check + s.a : nullptr);
  });
}

extern "C" int zs_pool_inflate_batch(zs_pool* p, int wbits, uint32_t n, const uint8_t* in, const uint64_t* in_off,
                                     const uint32_t* in_len, uint8_t* out, const uint64_t* out_off,
                                     const uint32_t* out_cap, int32_t* status, int32_t* phase, int32_t* msg,
                                     uint32_t* out_len, uint32_t* consumed, uint32_t* check) {
  return run_sharded(p, n, [&](uint32_t k, Shard s) {
    if (s.a == s.b) return (int)ZS_OK;
    return zs_inflate_batch_ex(p->ctx[k], wbits, s.b - s.a, in, in_off + s.a, in_len + s.a, out, out_off + s.a,
                               out_cap + s.a, status + s.a, phase + s.a, msg + s.a, out_len + s.a,
                               consumed + s.a, check ? check + s.a : nullptr);
  });
}

extern "C" int zs_pool_inflate_batch_auto(zs_pool* p, int wbits, uint32_t n, const uint8_t* in,
                                          const uint64_t* in_off, const uint32_t* in_len, uint8_t** out,
                                          uint64_t* out_off, int32_t* status, int32_t* phase, int32_t* msg,
                                          uint32_t* out_len, uint32_t* consumed, uint32_t* check) {
  if (!out || !out_off) return ZS_STREAM_ERROR;
  *out = nullptr;
  const uint32_t G = p ? (uint32_t)p->ctx.size() : 0;
  std::vector<uint8_t*> part(G, nullptr);
  const int r = run_sharded(p, n, [&](uint32_t k, Shard s) {
    if (s.a == s.b) return (int)ZS_OK;
    return zs_inflate_batch_auto(p->ctx[k], wbits, s.b - s.a, in, in_off + s.a, in_len + s.a, &part[k],
                                 out_off + s.a, status + s.a, phase + s.a, msg + s.a, out_len + s.a,
                                 consumed + s.a, check ? check + s.a : nullptr);
  });
  if (r == ZS_OK) {  // one buffer: the shards' outputs back to back, offsets rebased
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += out_len[i];
    uint8_t* res = (uint8_t*)malloc(total ? total : 1);
    if (res) {
      uint64_t base = 0;
      for (uint32_t k = 0; k < G; k++) {
        const Shard s = shard_range(n, G, k);
        uint64_t bytes = 0;
        for (uint32_t i = s.a; i < s.b; i++) bytes += out_len[i];
        if (bytes) memcpy(res + base, part[k], bytes);
        for (uint32_t i = s.a; i < s.b; i++) out_off[i] += base;
        base += bytes;
      }
      *out = res;
    }
    for (uint8_t* q : part) free(q);
    return res ? ZS_OK : ZS_MEM_ERROR;
  }
  for (uint8_t* q : part) free(q);
  return r;
}
