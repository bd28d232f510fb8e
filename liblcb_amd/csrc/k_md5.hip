// k_md5.hip — MD5 batch kernels (md_kernels.hpp), one translation unit per
// algorithm so the library compiles in parallel.
#include "md_kernels.hpp"

namespace lcbgpu {
LCB_MD_FAMILY(Md5, md5)
}  // namespace lcbgpu
