// k_md5.hip — MD5 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Md5, md5)
}  // namespace lcbgpu

#ifdef LCB_TILE_TRACE
// Diagnostic builds only: where the tile and fixed-stride kernels record
// their per-tile / per-wave timing (NULL: off).
extern "C" int lcb_debug_tile_trace(void* tiles, void* fixed) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(lcbgpu::g_tile_trace), &tiles, sizeof tiles) != hipSuccess) return 5;
    if (hipMemcpyToSymbol(HIP_SYMBOL(lcbgpu::g_fixed_trace), &fixed, sizeof fixed) != hipSuccess) return 5;
    return 0;
}
#endif
