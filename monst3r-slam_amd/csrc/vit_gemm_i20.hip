// Instantiation unit of the GEMM launcher (see vit_gemm_kern.h).
#include "vit_gemm_kern.h"

namespace m3s_gemm {
template int launch_pp<0, 192>(Args&, int, hipStream_t);
}  // namespace m3s_gemm
