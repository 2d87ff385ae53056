// Instantiation unit of the GEMM launcher (see vit_gemm_kern.h).
#include "vit_gemm_kern.h"

namespace m3s_gemm {
template int launch<64, 128, 64, 2, 2, 3, 2, true>(Args&, int, hipStream_t);
}  // namespace m3s_gemm
