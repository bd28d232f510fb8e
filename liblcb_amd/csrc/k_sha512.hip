// k_sha512.hip — SHA512 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Sha512<false>, sha512)
}  // namespace lcbgpu
