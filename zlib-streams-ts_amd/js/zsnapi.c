/*
 * zsnapi.c -- the thin N-API addon between the JavaScript host side
 * (streams-api.mjs) and libzsgpu.so (include/zs_gpu.h).  Plain C against
 * node_api.h (N-API v8): it reads the callers' Uint8Array backing stores for
 * the duration of one call (napi_get_typedarray_info, SURVEY.md 8(b)
 * "Ownership"), copies them into one buffer the batch owns before the call
 * returns (the caller may then modify, transfer or detach its buffers: N-API
 * cannot pin an ArrayBuffer), hands that to zs_deflate_batch /
 * zs_inflate_batch on the worker thread, and returns the outputs as views of ONE external ArrayBuffer that the batch's
 * output buffer becomes (freed when the views are collected: no copy back
 * either).  The batch calls return Promises: the GPU work runs on a libuv
 * worker thread (napi_async_work), so the event loop keeps running.  A batch
 * runs on a device set (SURVEY.md 8(b) "device mask"): a zs_pool per distinct
 * set, created lazily on the JS thread, splits it into contiguous stream
 * ranges with one host thread per GPU (so an 8-GPU batch is not capped by
 * libuv's 4-thread pool); batches on one set are serialized by the pool.
 */
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/zs_gpu.h"

#define MAX_DEV 64
static zs_ctx *g_ctx[MAX_DEV]; /* selfTest only */

#define MAX_POOLS 64
static struct {
  uint64_t mask;
  zs_pool *pool;
} g_pools[MAX_POOLS];
static int g_npools;

#define NAPI_OK(call)                                      \
  do {                                                     \
    if ((call) != napi_ok) {                               \
      napi_throw_error(env, NULL, "N-API call failed: " #call); \
      return NULL;                                         \
    }                                                      \
  } while (0)

static napi_value throw_code(napi_env env, int code, const char *msg) {
  char c[16];
  snprintf(c, sizeof c, "%d", code);
  napi_throw_error(env, c, msg);
  return NULL;
}

static void throw_unavailable(napi_env env) {
  /* no device / self-test failure: the engine is unavailable, never a CPU fallback */
  char m[600];
  snprintf(m, sizeof m, "MI355X engine unavailable: %s", zs_last_error());
  napi_throw_error(env, "ZS_UNAVAILABLE", m);
}

static zs_ctx *ctx_for(napi_env env, int dev) {
  if (dev < 0 || dev >= MAX_DEV) {
    throw_code(env, ZS_STREAM_ERROR, "device index out of range");
    return NULL;
  }
  if (!g_ctx[dev]) {
    zs_ctx *c = NULL;
    if (zs_ctx_create(dev, &c) != ZS_OK) {
      throw_unavailable(env);
      return NULL;
    }
    g_ctx[dev] = c;
  }
  return g_ctx[dev];
}

/* device spec: a device index, an array of them, or undefined (device 0) -> bit mask;
 * 0 on an invalid spec (a JS exception is pending) */
static uint64_t device_mask(napi_env env, napi_value v) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok) return 0;
  if (t == napi_undefined || t == napi_null) return 1;
  bool arr = false;
  napi_is_array(env, v, &arr);
  uint32_t n = 1;
  if (arr) napi_get_array_length(env, v, &n);
  uint64_t m = 0;
  for (uint32_t i = 0; i < n; i++) {
    napi_value e = v;
    if (arr) napi_get_element(env, v, i, &e);
    napi_valuetype et;
    int32_t d = -1;
    if (napi_typeof(env, e, &et) == napi_ok && et == napi_number) napi_get_value_int32(env, e, &d);
    if (d < 0 || d >= MAX_DEV) {
      napi_throw_error(env, "ZS_BAD_DEVICE", "devices must be GPU indices in 0..63");
      return 0;
    }
    m |= 1ull << d;
  }
  if (!m) napi_throw_error(env, "ZS_BAD_DEVICE", "devices must name at least one GPU");
  return m;
}

static zs_pool *pool_for(napi_env env, uint64_t mask) {
  for (int i = 0; i < g_npools; i++)
    if (g_pools[i].mask == mask) return g_pools[i].pool;
  if (g_npools == MAX_POOLS) {
    napi_throw_error(env, "ZS_BAD_DEVICE", "too many distinct device sets");
    return NULL;
  }
  zs_pool *p = NULL;
  const int r = zs_pool_create(mask, &p);
  if (r != ZS_OK) {
    if (r == ZS_STREAM_ERROR && strstr(zs_last_error(), "device mask")) napi_throw_error(env, "ZS_BAD_DEVICE", zs_last_error());
    else throw_unavailable(env);
    return NULL;
  }
  g_pools[g_npools].mask = mask;
  g_pools[g_npools].pool = p;
  g_npools++;
  return p;
}

/* Borrowed view of one input. */
typedef struct {
  const uint8_t *p;
  size_t n;
} view;

static int get_views(napi_env env, napi_value arr, view **out, uint32_t *count) {
  bool is_arr = false;
  if (napi_is_array(env, arr, &is_arr) != napi_ok || !is_arr) return -1;
  uint32_t n = 0;
  if (napi_get_array_length(env, arr, &n) != napi_ok) return -1;
  view *v = (view *)calloc(n ? n : 1, sizeof(view));
  if (!v) return -1;
  for (uint32_t i = 0; i < n; i++) {
    napi_value e;
    bool is_ta = false;
    napi_typedarray_type t;
    size_t len = 0, off = 0;
    void *data = NULL;
    napi_value ab;
    if (napi_get_element(env, arr, i, &e) != napi_ok || napi_is_typedarray(env, e, &is_ta) != napi_ok || !is_ta ||
        napi_get_typedarray_info(env, e, &t, &len, &data, &ab, &off) != napi_ok || t != napi_uint8_array) {
      free(v);
      return -2;
    }
    v[i].p = (const uint8_t *)data;
    v[i].n = len;
  }
  *out = v;
  *count = n;
  return 0;
}

static napi_value make_u8(napi_env env, const uint8_t *src, size_t n) {
  void *data = NULL;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, n, &data, &ab) != napi_ok) return NULL;
  if (n) memcpy(data, src, n);
  if (napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}

static napi_value make_32(napi_env env, const void *src, size_t n, napi_typedarray_type type) {
  void *data = NULL;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, 4 * n, &data, &ab) != napi_ok) return NULL;
  if (n) memcpy(data, src, 4 * n);
  if (napi_create_typedarray(env, type, n, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}
#define make_i32(env, src, n) make_32(env, src, n, napi_int32_array)
#define make_u32(env, src, n) make_32(env, src, n, napi_uint32_array)

/* an output capacity: a number clamped to 0 .. 4 GiB - 4 (the ABI's u32 lengths) */
static uint32_t arg_cap(napi_env env, napi_value v, uint32_t dflt) {
  napi_valuetype t;
  double x = dflt;
  if (napi_typeof(env, v, &t) == napi_ok && t == napi_number) napi_get_value_double(env, v, &x);
  if (!(x > 0)) return 0;
  if (x > 4294967292.0) x = 4294967292.0;
  return (uint32_t)x;
}

static int32_t arg_i32(napi_env env, napi_value v, int32_t dflt) {
  napi_valuetype t;
  int32_t x = dflt;
  if (napi_typeof(env, v, &t) == napi_ok && t == napi_number) napi_get_value_int32(env, v, &x);
  return x;
}

/* One batch in flight: a copy of the inputs taken on the JS thread when the
 * call is made (the caller may modify, transfer or detach its buffers right
 * after: N-API cannot pin an ArrayBuffer's memory), the GPU work on a libuv
 * worker thread (napi_async_work), results built back on the JS thread. */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  int inflate;   /* 0 compress, 1 decompress */
  int unbounded; /* decompress without a caller capacity: zs_pool_inflate_batch_auto */
  int wbits, level;
  uint32_t n;
  zs_pool *pool;
  uint64_t *in_off, *out_off;
  uint32_t *in_len, *cap, *olen, *cons, *check;
  int32_t *status, *phase, *msg;
  uint8_t *base;       /* inputs: base + in_off[i] (the job's own copy) */
  uint8_t *out;
  int out_given;       /* out now belongs to the results' external ArrayBuffer */
  int rc;
  char err[512];
} job;

static void job_free(job *j) {
  if (!j) return;
  free(j->in_off); free(j->out_off); free(j->in_len); free(j->cap); free(j->olen); free(j->cons); free(j->check);
  free(j->status); free(j->phase); free(j->msg); free(j->base);
  if (!j->out_given) {
    if (j->unbounded) zs_free(j->out);
    else free(j->out);
  }
  free(j);
}

static job *job_new(uint32_t n) {
  job *j = (job *)calloc(1, sizeof(job));
  if (!j) return NULL;
  j->n = n;
  j->in_off = (uint64_t *)calloc(n + 1, 8);
  j->out_off = (uint64_t *)calloc(n + 1, 8);
  j->in_len = (uint32_t *)calloc(n + 1, 4);
  j->cap = (uint32_t *)calloc(n + 1, 4);
  j->olen = (uint32_t *)calloc(n + 1, 4);
  j->cons = (uint32_t *)calloc(n + 1, 4);
  j->check = (uint32_t *)calloc(n + 1, 4);
  j->status = (int32_t *)calloc(n + 1, 4);
  j->phase = (int32_t *)calloc(n + 1, 4);
  j->msg = (int32_t *)calloc(n + 1, 4);
  if (!j->in_off || !j->out_off || !j->in_len || !j->cap || !j->olen || !j->cons || !j->check || !j->status ||
      !j->phase || !j->msg) {
    job_free(j);
    return NULL;
  }
  return j;
}

/* worker thread: no N-API calls here */
static void job_execute(napi_env env, void *data) {
  job *j = (job *)data;
  (void)env;
  if (j->n == 0) j->rc = ZS_OK;
  else if (j->inflate && j->unbounded)
    j->rc = zs_pool_inflate_batch_auto(j->pool, j->wbits, j->n, j->base, j->in_off, j->in_len, &j->out, j->out_off,
                                       j->status, j->phase, j->msg, j->olen, j->cons, j->check);
  else if (j->inflate)
    j->rc = zs_pool_inflate_batch(j->pool, j->wbits, j->n, j->base, j->in_off, j->in_len, j->out, j->out_off, j->cap,
                                  j->status, j->phase, j->msg, j->olen, j->cons, j->check);
  else
    j->rc = zs_pool_deflate_batch(j->pool, j->level, j->wbits, j->n, j->base, j->in_off, j->in_len, j->out,
                                  j->out_off, j->cap, j->status, j->olen, j->check);
  if (j->rc != ZS_OK) snprintf(j->err, sizeof j->err, "%s", zs_last_error());  /* the error is per thread */
}

static void free_out(napi_env env, void *data, void *hint) {
  (void)env;
  if (hint) zs_free(data);
  else free(data);
}

static napi_value build_result(napi_env env, job *j) {
  napi_value outs, obj;
  if (napi_create_array_with_length(env, j->n, &outs) != napi_ok || napi_create_object(env, &obj) != napi_ok) return NULL;
  napi_value msgs = NULL;
  if (j->inflate && napi_create_array_with_length(env, j->n, &msgs) != napi_ok) return NULL;
  /* the outputs: views of the batch's output buffer, which becomes an external
   * ArrayBuffer (copies only where the runtime refuses external buffers) */
  napi_value ab = NULL;
  uint64_t span = 0;
  for (uint32_t i = 0; i < j->n; i++)
    if (j->status[i] == ZS_STREAM_END && j->out_off[i] + j->olen[i] > span) span = j->out_off[i] + j->olen[i];
  if (j->out && span &&
      napi_create_external_arraybuffer(env, j->out, (size_t)span, free_out, j->unbounded ? (void *)1 : NULL, &ab) ==
          napi_ok)
    j->out_given = 1;
  for (uint32_t i = 0; i < j->n; i++) {
    const size_t len = j->status[i] == ZS_STREAM_END ? j->olen[i] : 0;
    napi_value u = NULL;
    if (ab && len) {
      if (napi_create_typedarray(env, napi_uint8_array, len, ab, (size_t)j->out_off[i], &u) != napi_ok) u = NULL;
    } else {
      u = make_u8(env, j->out ? j->out + j->out_off[i] : NULL, len);
    }
    if (!u || napi_set_element(env, outs, i, u) != napi_ok) return NULL;
    if (j->inflate) {
      napi_value s;
      const char *m = zs_inflate_message(j->msg[i]);
      if (napi_create_string_utf8(env, m ? m : "", NAPI_AUTO_LENGTH, &s) != napi_ok ||
          napi_set_element(env, msgs, i, s) != napi_ok)
        return NULL;
    }
  }
  napi_set_named_property(env, obj, "status", make_i32(env, j->status, j->n));
  napi_set_named_property(env, obj, "check", make_u32(env, j->check, j->n));
  if (j->inflate) {
    napi_set_named_property(env, obj, "phase", make_i32(env, j->phase, j->n));
    napi_set_named_property(env, obj, "consumed", make_i32(env, (const int32_t *)j->cons, j->n));
    napi_set_named_property(env, obj, "message", msgs);
  }
  napi_set_named_property(env, obj, "outputs", outs);
  return obj;
}

/* JS thread: settle the promise */
static void job_complete(napi_env env, napi_status st, void *data) {
  job *j = (job *)data;
  napi_value v = NULL;
  if (st == napi_ok && j->rc == ZS_OK) v = build_result(env, j);
  if (v) {
    napi_resolve_deferred(env, j->deferred, v);
  } else {
    char c[16];
    napi_value code, msg, e;
    const int rc = j->rc != ZS_OK ? j->rc : ZS_MEM_ERROR;
    snprintf(c, sizeof c, "%d", rc);
    napi_create_string_utf8(env, c, NAPI_AUTO_LENGTH, &code);
    napi_create_string_utf8(env, j->rc != ZS_OK ? j->err : "could not build the batch result", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, code, msg, &e);
    napi_reject_deferred(env, j->deferred, e);
  }
  napi_delete_async_work(env, j->work);
  job_free(j);
}

/* the inputs copied, packed, into one buffer the job owns */
static int copy_inputs(job *j, const view *v) {
  uint64_t tot = 0;
  for (uint32_t i = 0; i < j->n; i++) {
    j->in_off[i] = tot;
    j->in_len[i] = (uint32_t)v[i].n;
    tot += v[i].n;
  }
  j->base = (uint8_t *)malloc(tot ? tot : 1);
  if (!j->base) return -1;
  for (uint32_t i = 0; i < j->n; i++)
    if (v[i].n) memcpy(j->base + j->in_off[i], v[i].p, v[i].n);
  return 0;
}

static napi_value queue_job(napi_env env, job *j, const char *name) {
  napi_value promise, res_name;
  if (napi_create_promise(env, &j->deferred, &promise) != napi_ok ||
      napi_create_string_utf8(env, name, NAPI_AUTO_LENGTH, &res_name) != napi_ok ||
      napi_create_async_work(env, NULL, res_name, job_execute, job_complete, j, &j->work) != napi_ok ||
      napi_queue_async_work(env, j->work) != napi_ok) {
    job_free(j);
    return throw_code(env, ZS_MEM_ERROR, "could not queue the batch");
  }
  return promise;
}

/* compressBatch(inputs: Uint8Array[], wbits, level, devices: number | number[]) ->
 *   Promise<{status: Int32Array, check: Uint32Array, outputs: Uint8Array[]}> */
static napi_value CompressBatch(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) return throw_code(env, ZS_STREAM_ERROR, "compressBatch(inputs, wbits, level[, devices])");
  view *v = NULL;
  uint32_t n = 0;
  if (get_views(env, argv[0], &v, &n) != 0) return throw_code(env, ZS_STREAM_ERROR, "inputs must be Uint8Array[]");
  napi_value undef;
  napi_get_undefined(env, &undef);
  const uint64_t mask = device_mask(env, argc > 3 ? argv[3] : undef);
  zs_pool *pool = mask ? pool_for(env, mask) : NULL;
  job *j = pool ? job_new(n) : NULL;
  if (!j) {
    free(v);
    return pool ? throw_code(env, ZS_MEM_ERROR, "out of host memory") : NULL;
  }
  j->pool = pool;
  j->wbits = arg_i32(env, argv[1], -15);
  j->level = arg_i32(env, argv[2], -1);
  uint64_t tout = 0;
  for (uint32_t i = 0; i < n; i++) {
    j->out_off[i] = tout;
    j->cap[i] = (uint32_t)((zs_deflate_bound(v[i].n, j->wbits) + 3) & ~3ull);
    tout += j->cap[i];
  }
  j->out = (uint8_t *)malloc(tout ? tout : 1);  /* (uninitialised: only the outputs are written) */
  if (!j->out || copy_inputs(j, v) != 0) {
    free(v);
    job_free(j);
    return throw_code(env, ZS_MEM_ERROR, "out of host memory");
  }
  free(v);
  return queue_job(env, j, "zs.compressBatch");
}

/* decompressBatch(inputs: Uint8Array[], wbits, outCapacity: number | number[] | undefined, devices) ->
 *   Promise<{status, phase: Int32Array, message: string[], outputs: Uint8Array[], consumed: Int32Array,
 *            check: Uint32Array}>
 * outCapacity undefined: unbounded output, as DecompressionStream (zs_pool_inflate_batch_auto). */
static napi_value DecompressBatch(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) return throw_code(env, ZS_STREAM_ERROR, "decompressBatch(inputs, wbits[, outCapacity[, devices]])");
  view *v = NULL;
  uint32_t n = 0;
  if (get_views(env, argv[0], &v, &n) != 0) return throw_code(env, ZS_STREAM_ERROR, "inputs must be Uint8Array[]");
  napi_value undef;
  napi_get_undefined(env, &undef);
  const uint64_t mask = device_mask(env, argc > 3 ? argv[3] : undef);
  zs_pool *pool = mask ? pool_for(env, mask) : NULL;
  job *j = pool ? job_new(n) : NULL;
  if (!j) {
    free(v);
    return pool ? throw_code(env, ZS_MEM_ERROR, "out of host memory") : NULL;
  }
  j->inflate = 1;
  j->pool = pool;
  j->wbits = arg_i32(env, argv[1], -15);
  napi_valuetype ct = napi_undefined;
  if (argc > 2) napi_typeof(env, argv[2], &ct);
  j->unbounded = ct == napi_undefined || ct == napi_null;
  bool caps_arr = false;
  if (!j->unbounded) napi_is_array(env, argv[2], &caps_arr);
  const uint32_t cap_all = caps_arr || j->unbounded ? 0 : arg_cap(env, argv[2], 1 << 16);
  uint64_t tout = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t c = cap_all;
    if (caps_arr) {
      napi_value e;
      napi_get_element(env, argv[2], i, &e);
      c = arg_cap(env, e, 1 << 16);
    }
    j->out_off[i] = tout;
    j->cap[i] = c;  /* exact: Z_BUF_ERROR past it (the host entry stages in word-aligned regions itself) */
    tout += j->cap[i];
  }
  j->out = j->unbounded ? NULL : (uint8_t *)malloc(tout ? tout : 1);  /* unbounded: the library allocates it */
  if ((!j->unbounded && !j->out) || copy_inputs(j, v) != 0) {
    free(v);
    job_free(j);
    return throw_code(env, ZS_MEM_ERROR, "out of host memory");
  }
  free(v);
  return queue_job(env, j, "zs.decompressBatch");
}

static napi_value DeflateBound(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], r;
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  double len = 0;
  napi_get_value_double(env, argv[0], &len);
  NAPI_OK(napi_create_double(env, (double)zs_deflate_bound((uint64_t)len, argc > 1 ? arg_i32(env, argv[1], -15) : -15), &r));
  return r;
}

static napi_value Version(napi_env env, napi_callback_info info) {
  napi_value r;
  (void)info;
  NAPI_OK(napi_create_string_utf8(env, zs_version(), NAPI_AUTO_LENGTH, &r));
  return r;
}

static napi_value SelfTest(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], r;
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  zs_ctx *ctx = ctx_for(env, argc ? arg_i32(env, argv[0], 0) : 0);
  if (!ctx) return NULL;
  uint64_t bad = 0;
  int rc = zs_selftest(ctx, &bad);
  if (rc != ZS_OK) return throw_code(env, rc, zs_last_error());
  NAPI_OK(napi_create_double(env, (double)bad, &r));
  return r;
}

static napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"compressBatch", NULL, CompressBatch, NULL, NULL, NULL, napi_default, NULL},
      {"decompressBatch", NULL, DecompressBatch, NULL, NULL, NULL, napi_default, NULL},
      {"deflateBound", NULL, DeflateBound, NULL, NULL, NULL, napi_default, NULL},
      {"version", NULL, Version, NULL, NULL, NULL, napi_default, NULL},
      {"selfTest", NULL, SelfTest, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
