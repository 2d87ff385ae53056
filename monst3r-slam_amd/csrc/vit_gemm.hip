// Batched bf16 MFMA GEMM with fused epilogues for the ViT / DPT path (gfx950).
//
//   C[g] = epi(A[g] · B[g]^T)       A [M][K] (or implicit 3x3-conv rows of an NHWC image),
//                                   B [N][K] weights (K contiguous: torch Linear layout)
// Tiles (templated): BM x BN x BK with 256 threads = 4 waves laid out WM x WN; each wave
// owns (BM/WM) x (BN/WN) = a grid of 32x32 v_mfma_f32_32x32x16_bf16 accumulators.
// LDS: double buffer, rows padded by 16 B (conflict-free ds_read_b128 of the 32x32x16
// fragments: consecutive rows land 4 banks apart).  Global→register→LDS staging with the
// next K-tile's 16-B loads issued before the current tile's MFMAs (one barrier per tile).
// Implicit conv: the staged rows' output pixels are decoded once; per K-tile the tap
// (ky, kx) and channel offset are block-uniform (Cin % BK == 0), so a row's source address
// is one multiply-add and a bounds test (zero padding).
// Epilogue: bias, GELU(erf), ReLU, f32/bf16 residual, f32/bf16 store, ConvTranspose(k=s)
// scatter; blockIdx.z = batch.  XCD-aware tile order: consecutive N-tiles of one M-row
// band are mapped to the same XCD (blockIdx.x % 8 groups), sharing the A panel in L2.
#include "vit_common.h"

namespace {

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
  int tiles_m, tiles_n;
};

__device__ __forceinline__ uint4 relu8(uint4 v) {
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

template <int BM, int BN, int BK, int WM, int WN, int MODE>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(Args a) {
  constexpr int LDS = BK + 8;                 // padded row (bf16 elements)
  constexpr int CPR = BK / 8;                 // 16-B chunks per row
  constexpr int A_CH = BM * CPR / NT;         // A chunks per thread per K-tile
  constexpr int B_CH = BN * CPR / NT;
  constexpr int TM = BM / WM / 32;            // 32x32 accumulators per wave (M)
  constexpr int TN = BN / WN / 32;
  static_assert(A_CH >= 1 && B_CH >= 1, "tile too small for 256 threads");
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM][LDS];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN][LDS];

  // XCD-aware tile order: blocks b, b+8, b+16.. share an XCD; give them consecutive
  // N-tiles of one M band (bijective remap, cdna_hip_programming.md T1).
  const int nwg = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x;
  int wgid = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int tm = wgid / a.tiles_n, tn = wgid - tm * a.tiles_n;
  const int g = blockIdx.z;
  const bf16_t* A = a.A + (int64_t)g * a.sA;
  const bf16_t* B = a.B + (int64_t)g * a.sB;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const bool relu_in = (a.flags & M3S_PRO_RELU) != 0;

  // staging assignment (fixed rows per thread); conv rows decoded once
  int a_row[A_CH], a_kc[A_CH];
  int64_t a_base[A_CH];
  int a_iy[A_CH], a_ix[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; i++) {
    const int c = tid + i * NT;
    a_row[i] = c / CPR;
    a_kc[i] = (c % CPR) * 8;
    const int m = m0 + a_row[i];
    a_ok[i] = m < a.M;
    if (MODE == 0) {
      a_base[i] = (int64_t)(a_ok[i] ? m : 0) * a.lda;
    } else {
      const int mm = a_ok[i] ? m : 0;
      const int oy = mm / a.Wout, ox = mm - (mm / a.Wout) * a.Wout;
      a_iy[i] = oy * a.stride - 1;
      a_ix[i] = ox * a.stride - 1;
    }
  }
  int b_row[B_CH], b_kc[B_CH];
  bool b_ok[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; i++) {
    const int c = tid + i * NT;
    b_row[i] = c / CPR;
    b_kc[i] = (c % CPR) * 8;
    b_ok[i] = (n0 + b_row[i]) < a.N;
  }

  uint4 ra[A_CH], rb[B_CH];
  auto gload = [&](int k0) {
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < A_CH; i++)
        ra[i] = a_ok[i] ? *reinterpret_cast<const uint4*>(A + a_base[i] + k0 + a_kc[i])
                        : make_uint4(0, 0, 0, 0);
    } else {
      const int tap = k0 / a.Cin;  // block-uniform: Cin % BK == 0
      const int ci0 = k0 - tap * a.Cin;
      const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
      for (int i = 0; i < A_CH; i++) {
        const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
        const bool ok = a_ok[i] && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
        ra[i] = ok ? *reinterpret_cast<const uint4*>(A + ((int64_t)iy * a.Win + ix) * a.Cin +
                                                     ci0 + a_kc[i])
                   : make_uint4(0, 0, 0, 0);
      }
    }
    if (relu_in) {
#pragma unroll
      for (int i = 0; i < A_CH; i++) ra[i] = relu8(ra[i]);
    }
#pragma unroll
    for (int i = 0; i < B_CH; i++)
      rb[i] = b_ok[i] ? *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + b_row[i]) * a.ldb + k0 +
                                                        b_kc[i])
                      : make_uint4(0, 0, 0, 0);
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; i++) *reinterpret_cast<uint4*>(&As[buf][a_row[i]][a_kc[i]]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; i++) *reinterpret_cast<uint4*>(&Bs[buf][b_row[i]][b_kc[i]]) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
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
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; i++)
        af[i] = *reinterpret_cast<const bf16x8*>(
            &As[cur][wm * (BM / WM) + i * 32 + fr][kk * 16 + fk]);
#pragma unroll
      for (int j = 0; j < TN; j++)
        bfr[j] = *reinterpret_cast<const bf16x8*>(
            &Bs[cur][wn * (BN / WN) + j * 32 + fr][kk * 16 + fk]);
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
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
  const char* Rb =
      a.R ? reinterpret_cast<const char*>(a.R) + (int64_t)g * a.sR * (f_res32 ? 4 : 2) : nullptr;
#pragma unroll
  for (int j = 0; j < TN; j++) {
    const int n = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
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
    for (int i = 0; i < TM; i++) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int m = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
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

template <int BM, int BN, int BK, int WM, int WN>
int launch(Args& a, int batch, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  dim3 grid((unsigned)(a.tiles_m * a.tiles_n), 1, (unsigned)batch);
  if (a.mode == 0)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, 0>), grid, dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, 1>), grid, dim3(NT), 0, s, a);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

}  // namespace

extern "C" int m3s_vit_gemm(const m3s_gemm_desc* d, void* stream) {
  if (!d || !d->A || !d->B || !d->C) return M3S_ERR_INVALID_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch <= 0) return M3S_ERR_INVALID_ARG;
  if (d->K % 32 != 0) return M3S_ERR_INVALID_ARG;
  if (d->mode == 1 && (d->Cin % 32 != 0 || d->K != 9 * d->Cin)) return M3S_ERR_INVALID_ARG;
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
  hipStream_t s = m3s_stream(stream);
  const bool k64 = (d->K % 64 == 0) && (d->mode == 0 || d->Cin % 64 == 0);
  // Tile choice: the 128x128 tile unless it leaves most of the 256 CUs idle; then halve M.
  const int64_t tiles128 = (int64_t)((d->M + 127) / 128) * ((d->N + 127) / 128) * d->batch;
  if (tiles128 < 192 && d->M <= 1024) {
    if (k64) return launch<64, 128, 64, 2, 2>(a, d->batch, s);
    return launch<64, 128, 32, 2, 2>(a, d->batch, s);
  }
  if (k64) return launch<128, 128, 64, 2, 2>(a, d->batch, s);
  return launch<128, 128, 32, 2, 2>(a, d->batch, s);
}
