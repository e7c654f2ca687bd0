/*
 * zsnapi.c -- the thin N-API addon between the JavaScript host side
 * (streams-api.mjs) and libzsgpu.so (include/zs_gpu.h).  Plain C against
 * node_api.h (N-API v8): it borrows the callers' Uint8Array backing stores for
 * the duration of one call (napi_get_typedarray_info), packs them into one
 * host batch, runs zs_deflate_batch / zs_inflate_batch on the GPU and returns
 * fresh Uint8Arrays -- nothing is retained after the call (SURVEY.md 8(b)
 * "Ownership").  Synchronous; one device context per GPU, created lazily.
 */
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/zs_gpu.h"

#define MAX_DEV 64
static zs_ctx *g_ctx[MAX_DEV];

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

static zs_ctx *ctx_for(napi_env env, int dev) {
  if (dev < 0 || dev >= MAX_DEV) {
    throw_code(env, ZS_STREAM_ERROR, "device index out of range");
    return NULL;
  }
  if (!g_ctx[dev]) {
    zs_ctx *c = NULL;
    int r = zs_ctx_create(dev, &c);
    if (r != ZS_OK) {  /* no device / self-test failure: the engine is unavailable, never a CPU fallback */
      char m[600];
      snprintf(m, sizeof m, "MI355X engine unavailable: %s", zs_last_error());
      napi_throw_error(env, "ZS_UNAVAILABLE", m);
      return NULL;
    }
    g_ctx[dev] = c;
  }
  return g_ctx[dev];
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

static napi_value make_i32(napi_env env, const int32_t *src, size_t n) {
  void *data = NULL;
  napi_value ab, ta;
  if (napi_create_arraybuffer(env, 4 * n, &data, &ab) != napi_ok) return NULL;
  if (n) memcpy(data, src, 4 * n);
  if (napi_create_typedarray(env, napi_int32_array, n, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}

static int32_t arg_i32(napi_env env, napi_value v, int32_t dflt) {
  napi_valuetype t;
  int32_t x = dflt;
  if (napi_typeof(env, v, &t) == napi_ok && t == napi_number) napi_get_value_int32(env, v, &x);
  return x;
}

/* compressBatch(inputs: Uint8Array[], wbits, level, device) ->
 *   {status: Int32Array, outputs: Uint8Array[]} */
static napi_value CompressBatch(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) return throw_code(env, ZS_STREAM_ERROR, "compressBatch(inputs, wbits, level[, device])");
  view *v = NULL;
  uint32_t n = 0;
  if (get_views(env, argv[0], &v, &n) != 0) return throw_code(env, ZS_STREAM_ERROR, "inputs must be Uint8Array[]");
  const int wbits = arg_i32(env, argv[1], -15), level = arg_i32(env, argv[2], -1);
  const int dev = argc > 3 ? arg_i32(env, argv[3], 0) : 0;
  zs_ctx *ctx = ctx_for(env, dev);
  if (!ctx) { free(v); return NULL; }
  uint64_t *in_off = (uint64_t *)calloc(n + 1, 8), *out_off = (uint64_t *)calloc(n + 1, 8);
  uint32_t *in_len = (uint32_t *)calloc(n + 1, 4), *cap = (uint32_t *)calloc(n + 1, 4), *olen = (uint32_t *)calloc(n + 1, 4);
  int32_t *status = (int32_t *)calloc(n + 1, 4);
  uint64_t tin = 0, tout = 0;
  for (uint32_t i = 0; i < n; i++) {
    in_off[i] = tin;
    in_len[i] = (uint32_t)v[i].n;
    tin += v[i].n;
    out_off[i] = tout;
    cap[i] = (uint32_t)((zs_deflate_bound(v[i].n, wbits) + 3) & ~3ull);
    tout += cap[i];
  }
  uint8_t *blob = (uint8_t *)malloc(tin ? tin : 1), *out = (uint8_t *)malloc(tout ? tout : 1);
  napi_value res = NULL;
  if (!in_off || !out_off || !in_len || !cap || !olen || !status || !blob || !out) {
    throw_code(env, ZS_MEM_ERROR, "out of host memory");
    goto done;
  }
  for (uint32_t i = 0; i < n; i++)
    if (v[i].n) memcpy(blob + in_off[i], v[i].p, v[i].n);
  int r = n ? zs_deflate_batch(ctx, level, wbits, n, blob, in_off, in_len, out, out_off, cap, status, olen) : ZS_OK;
  if (r != ZS_OK) {
    throw_code(env, r, zs_last_error());
    goto done;
  }
  napi_value outs, obj;
  if (napi_create_array_with_length(env, n, &outs) != napi_ok || napi_create_object(env, &obj) != napi_ok) goto done;
  for (uint32_t i = 0; i < n; i++) {
    napi_value u = make_u8(env, out + out_off[i], status[i] == ZS_STREAM_END ? olen[i] : 0);
    if (!u || napi_set_element(env, outs, i, u) != napi_ok) goto done;
  }
  napi_set_named_property(env, obj, "status", make_i32(env, status, n));
  napi_set_named_property(env, obj, "outputs", outs);
  res = obj;
done:
  free(v); free(in_off); free(out_off); free(in_len); free(cap); free(olen); free(status); free(blob); free(out);
  return res;
}

/* decompressBatch(inputs: Uint8Array[], wbits, outCapacity: number | number[], device) ->
 *   {status, phase: Int32Array, message: string[], outputs: Uint8Array[], consumed: Int32Array} */
static napi_value DecompressBatch(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) return throw_code(env, ZS_STREAM_ERROR, "decompressBatch(inputs, wbits, outCapacity[, device])");
  view *v = NULL;
  uint32_t n = 0;
  if (get_views(env, argv[0], &v, &n) != 0) return throw_code(env, ZS_STREAM_ERROR, "inputs must be Uint8Array[]");
  const int wbits = arg_i32(env, argv[1], -15);
  const int dev = argc > 3 ? arg_i32(env, argv[3], 0) : 0;
  zs_ctx *ctx = ctx_for(env, dev);
  if (!ctx) { free(v); return NULL; }
  bool caps_arr = false;
  napi_is_array(env, argv[2], &caps_arr);
  const int32_t cap_all = caps_arr ? 0 : arg_i32(env, argv[2], 1 << 16);
  uint64_t *in_off = (uint64_t *)calloc(n + 1, 8), *out_off = (uint64_t *)calloc(n + 1, 8);
  uint32_t *in_len = (uint32_t *)calloc(n + 1, 4), *cap = (uint32_t *)calloc(n + 1, 4);
  uint32_t *olen = (uint32_t *)calloc(n + 1, 4), *cons = (uint32_t *)calloc(n + 1, 4);
  int32_t *status = (int32_t *)calloc(n + 1, 4), *phase = (int32_t *)calloc(n + 1, 4), *msg = (int32_t *)calloc(n + 1, 4);
  uint64_t tin = 0, tout = 0;
  uint8_t *blob = NULL, *out = NULL;
  napi_value res = NULL;
  if (!in_off || !out_off || !in_len || !cap || !olen || !cons || !status || !phase || !msg) {
    throw_code(env, ZS_MEM_ERROR, "out of host memory");
    goto done;
  }
  for (uint32_t i = 0; i < n; i++) {
    int32_t c = cap_all;
    if (caps_arr) {
      napi_value e;
      napi_get_element(env, argv[2], i, &e);
      c = arg_i32(env, e, 1 << 16);
    }
    if (c < 0) c = 0;
    in_off[i] = tin;
    in_len[i] = (uint32_t)v[i].n;
    tin += v[i].n;
    out_off[i] = tout;
    cap[i] = ((uint32_t)c + 3u) & ~3u;
    tout += cap[i];
  }
  blob = (uint8_t *)malloc(tin ? tin : 1);
  out = (uint8_t *)malloc(tout ? tout : 1);
  if (!blob || !out) {
    throw_code(env, ZS_MEM_ERROR, "out of host memory");
    goto done;
  }
  for (uint32_t i = 0; i < n; i++)
    if (v[i].n) memcpy(blob + in_off[i], v[i].p, v[i].n);
  int r = n ? zs_inflate_batch(ctx, wbits, n, blob, in_off, in_len, out, out_off, cap, status, phase, msg, olen, cons)
            : ZS_OK;
  if (r != ZS_OK) {
    throw_code(env, r, zs_last_error());
    goto done;
  }
  napi_value outs, msgs, obj;
  if (napi_create_array_with_length(env, n, &outs) != napi_ok || napi_create_array_with_length(env, n, &msgs) != napi_ok ||
      napi_create_object(env, &obj) != napi_ok)
    goto done;
  for (uint32_t i = 0; i < n; i++) {
    napi_value u = make_u8(env, out + out_off[i], status[i] == ZS_STREAM_END ? olen[i] : 0), s;
    const char *m = zs_inflate_message(msg[i]);
    if (!u || napi_set_element(env, outs, i, u) != napi_ok) goto done;
    if (napi_create_string_utf8(env, m ? m : "", NAPI_AUTO_LENGTH, &s) != napi_ok || napi_set_element(env, msgs, i, s) != napi_ok)
      goto done;
  }
  napi_set_named_property(env, obj, "status", make_i32(env, status, n));
  napi_set_named_property(env, obj, "phase", make_i32(env, phase, n));
  napi_set_named_property(env, obj, "consumed", make_i32(env, (const int32_t *)cons, n));
  napi_set_named_property(env, obj, "message", msgs);
  napi_set_named_property(env, obj, "outputs", outs);
  res = obj;
done:
  free(v); free(in_off); free(out_off); free(in_len); free(cap); free(olen); free(cons); free(status); free(phase);
  free(msg); free(blob); free(out);
  return res;
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
