// temporary: inflate entry points until inflate.hip lands
#include "../../include/zs_gpu.h"
extern "C" int zs_inflate_batch_device(zs_ctx*, int, uint32_t, const uint8_t*, const uint64_t*, const uint32_t*,
                                       uint8_t*, const uint64_t*, const uint32_t*, int32_t*, int32_t*, int32_t*,
                                       uint32_t*, uint32_t*, void*) { return ZS_STREAM_ERROR; }
extern "C" int zs_inflate_batch(zs_ctx*, int, uint32_t, const uint8_t*, const uint64_t*, const uint32_t*, uint8_t*,
                                const uint64_t*, const uint32_t*, int32_t*, int32_t*, int32_t*, uint32_t*, uint32_t*) {
  return ZS_STREAM_ERROR;
}
extern "C" const char* zs_inflate_message(int32_t) { return ""; }
