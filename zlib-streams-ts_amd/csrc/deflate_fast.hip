// deflate_fast.hip -- placeholder for the greedy levels 1..3 (deflate_fast,
// deflate.ts:1281-1350); see DESIGN.md.  Marks every stream unsupported.
#include <hip/hip_runtime.h>
#include "zs_common.h"
#include "zs_kernels.h"

__global__ void zs_k_fast(const uint8_t*, const uint64_t*, const uint32_t*, const uint64_t*, const uint32_t*, uint32_t*,
                          zs_block*, zs_stream* streams, int, int, int) {
  if (threadIdx.x == 0) { streams[blockIdx.x].nsym = 0; streams[blockIdx.x].nblk = 0; }
}
