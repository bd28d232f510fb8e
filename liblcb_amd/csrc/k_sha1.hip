// k_sha1.hip — SHA1 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Sha1, sha1)
}  // namespace lcbgpu
