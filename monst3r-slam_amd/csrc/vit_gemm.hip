// Batched bf16 MFMA GEMM with fused epilogues for the ViT / DPT path (gfx950).
//
//   C[g] = epi(A[g] · B[g]^T)       A [M][K] (or implicit 3x3-conv rows of an NHWC image),
//                                   B [N][K] weights (K contiguous: torch Linear layout)
// Tile 128x128x32, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x16_bf16; LDS double buffer with rows padded to 80 B (conflict-free
// ds_read_b128 for the 32x32x16 fragment reads), global→register→LDS staging with the
// next K-tile's loads in flight during the current tile's MFMAs (one barrier per tile).
// Epilogue: bias, GELU(erf), ReLU, f32/bf16 residual, f32/bf16 store, and the
// ConvTranspose(k=s, stride=s) scatter into NHWC.  blockIdx.z = batch (per-batch
// pointer strides: decoder sides / models run as one launch).
#include "vit_common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int LDS_STRIDE = BK + 8;  // bf16 elements per LDS row (80 B)
constexpr int NT = 256;

struct Args {
  const bf16_t* A;
  int64_t lda, sA;
  const bf16_t* B;
  int64_t ldb, sB;
  void* C;
  int64_t ldc, sC;
  const float* bias;
  int64_t sBias;
  const void* R;
  int64_t ldr, sR;
  int M, N, K, flags, mode;
  int Hin, Win, Cin, Hout, Wout, stride;
  int ct_s, ct_cout, ct_gw;
};

template <int MODE>
__device__ __forceinline__ uint4 load_a_chunk(const Args& a, const bf16_t* A, int m, int k) {
  uint4 z = make_uint4(0, 0, 0, 0);
  if (m >= a.M) return z;
  if (MODE == 0) {
    return *reinterpret_cast<const uint4*>(A + (int64_t)m * a.lda + k);
  } else {
    // implicit 3x3 conv, pad 1: K ordered (ky, kx, ci)
    const int tap = k / a.Cin;
    const int ci = k - tap * a.Cin;
    const int ky = tap / 3, kx = tap - ky * 3;
    const int oy = m / a.Wout, ox = m - oy * a.Wout;
    const int iy = oy * a.stride + ky - 1, ix = ox * a.stride + kx - 1;
    if (iy < 0 || iy >= a.Hin || ix < 0 || ix >= a.Win) return z;
    return *reinterpret_cast<const uint4*>(A + ((int64_t)iy * a.Win + ix) * a.Cin + ci);
  }
}

__device__ __forceinline__ uint4 relu8(uint4 v) {
  // bf16 ReLU on 8 packed values: clear negative lanes (sign bit set) to +0
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t x = w[i];
    uint32_t lo = (x & 0x8000u) ? 0u : (x & 0xffffu);
    uint32_t hi = (x & 0x80000000u) ? 0u : (x & 0xffff0000u);
    w[i] = lo | hi;
  }
  return v;
}

template <int MODE>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(Args a) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM][LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN][LDS_STRIDE];

  const int g = blockIdx.z;
  const bf16_t* A = a.A + (int64_t)g * a.sA;
  const bf16_t* B = a.B + (int64_t)g * a.sB;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const bool relu_in = (a.flags & M3S_PRO_RELU) != 0;

  // staging assignment: 2 chunks of 16 B per thread per operand
  int st_row[2], st_kc[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int c = tid + i * NT;
    st_row[i] = c >> 2;
    st_kc[i] = (c & 3) * 8;
  }
  uint4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; i++) {
      ra[i] = load_a_chunk<MODE>(a, A, m0 + st_row[i], k0 + st_kc[i]);
      if (relu_in) ra[i] = relu8(ra[i]);
      const int n = n0 + st_row[i];
      rb[i] = n < a.N ? *reinterpret_cast<const uint4*>(B + (int64_t)n * a.ldb + k0 + st_kc[i])
                      : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; i++) {
      *reinterpret_cast<uint4*>(&As[buf][st_row[i]][st_kc[i]]) = ra[i];
      *reinterpret_cast<uint4*>(&Bs[buf][st_row[i]][st_kc[i]]) = rb[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  const int nk = a.K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  const int fr = lane & 31;
  const int fk = (lane >> 5) * 8;
  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK / 16; kk++) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; i++)
        af[i] = *reinterpret_cast<const bf16x8*>(&As[cur][wm * 64 + i * 32 + fr][kk * 16 + fk]);
#pragma unroll
      for (int j = 0; j < 2; j++)
        bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][wn * 64 + j * 32 + fr][kk * 16 + fk]);
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const float* bias = a.bias ? a.bias + (int64_t)g * a.sBias : nullptr;
  const bool f_bias = (a.flags & M3S_EPI_BIAS) && bias;
  const bool f_gelu = a.flags & M3S_EPI_GELU;
  const bool f_relu = a.flags & M3S_EPI_RELU;
  const bool f_res32 = a.flags & M3S_EPI_RES_F32;
  const bool f_res16 = a.flags & M3S_EPI_RES_BF16;
  const bool f_out32 = a.flags & M3S_EPI_OUT_F32;
  const bool f_convt = a.flags & M3S_EPI_CONVT;
  char* Cb = reinterpret_cast<char*>(a.C) + (int64_t)g * a.sC * (f_out32 ? 4 : 2);
  const char* Rb = a.R ? reinterpret_cast<const char*>(a.R) + (int64_t)g * a.sR * (f_res32 ? 4 : 2)
                       : nullptr;
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int n = n0 + wn * 64 + j * 32 + (lane & 31);
    if (n >= a.N) continue;
    float bv = 0.f;
    int co = n, ca = 0, cb = 0;
    if (f_convt) {
      const int ss = a.ct_s;
      co = n % a.ct_cout;
      const int ab = n / a.ct_cout;
      ca = ab / ss;
      cb = ab - ca * ss;
    }
    if (f_bias) bv = bias[co];
#pragma unroll
    for (int i = 0; i < 2; i++) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bv;
        if (f_gelu) v = gelu_erf(v);
        int64_t off;
        if (f_convt) {
          const int ti = m / a.ct_gw, tj = m - ti * a.ct_gw;
          const int64_t oy = (int64_t)ti * a.ct_s + ca, ox = (int64_t)tj * a.ct_s + cb;
          off = (oy * ((int64_t)a.ct_gw * a.ct_s) + ox) * a.ct_cout + co;
        } else {
          off = (int64_t)m * a.ldc + n;
        }
        if (f_res32) v += reinterpret_cast<const float*>(Rb)[(int64_t)m * a.ldr + n];
        if (f_res16) v += bf2f(reinterpret_cast<const bf16_t*>(Rb)[(int64_t)m * a.ldr + n]);
        if (f_relu) v = fmaxf(v, 0.f);
        if (f_out32) reinterpret_cast<float*>(Cb)[off] = v;
        else reinterpret_cast<bf16_t*>(Cb)[off] = f2bf(v);
      }
    }
  }
}

}  // namespace

extern "C" int m3s_vit_gemm(const m3s_gemm_desc* d, void* stream) {
  if (!d || !d->A || !d->B || !d->C) return M3S_ERR_INVALID_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch <= 0) return M3S_ERR_INVALID_ARG;
  if (d->K % BK != 0) return M3S_ERR_INVALID_ARG;
  if (d->mode == 1 && (d->Cin % BK != 0 || d->K != 9 * d->Cin)) return M3S_ERR_INVALID_ARG;
  if ((d->flags & (M3S_EPI_RES_F32 | M3S_EPI_RES_BF16)) && !d->R) return M3S_ERR_INVALID_ARG;
  if ((d->flags & M3S_EPI_CONVT) && (d->ct_s <= 0 || d->ct_cout <= 0 || d->ct_gw <= 0))
    return M3S_ERR_INVALID_ARG;
  if (((uintptr_t)d->A | (uintptr_t)d->B) % 16) return M3S_ERR_INVALID_ARG;
  if (d->mode == 0 && (d->lda % 8 || d->ldb % 8)) return M3S_ERR_INVALID_ARG;
  if (d->batch > 65535) return M3S_ERR_TOO_LARGE;
  Args a;
  a.A = reinterpret_cast<const bf16_t*>(d->A);
  a.lda = d->lda;
  a.sA = d->strideA;
  a.B = reinterpret_cast<const bf16_t*>(d->B);
  a.ldb = d->ldb;
  a.sB = d->strideB;
  a.C = d->C;
  a.ldc = d->ldc;
  a.sC = d->strideC;
  a.bias = d->bias;
  a.sBias = d->strideBias;
  a.R = d->R;
  a.ldr = d->ldr;
  a.sR = d->strideR;
  a.M = d->M;
  a.N = d->N;
  a.K = d->K;
  a.flags = d->flags;
  a.mode = d->mode;
  a.Hin = d->Hin;
  a.Win = d->Win;
  a.Cin = d->Cin;
  a.Hout = d->Hout;
  a.Wout = d->Wout;
  a.stride = d->stride;
  a.ct_s = d->ct_s;
  a.ct_cout = d->ct_cout;
  a.ct_gw = d->ct_gw;
  dim3 grid(m3s_div_up(d->N, BN), m3s_div_up(d->M, BM), (unsigned)d->batch);
  if (d->mode == 0)
    hipLaunchKernelGGL(gemm_kernel<0>, grid, dim3(NT), 0, m3s_stream(stream), a);
  else
    hipLaunchKernelGGL(gemm_kernel<1>, grid, dim3(NT), 0, m3s_stream(stream), a);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
