// k_sha256.hip — SHA256 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Sha256<false>, sha256)
}  // namespace lcbgpu
