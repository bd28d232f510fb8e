// k_sha224.hip — SHA224 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Sha256<true>, sha224)
}  // namespace lcbgpu
