// Instantiation unit of the GEMM launcher (see vit_gemm_kern.h).
#include "vit_gemm_kern.h"

namespace m3s_gemm {
template int launch<128, 128, 64, 4, 2, 3, 1, true>(Args&, int, hipStream_t);
}  // namespace m3s_gemm
