// Batched bf16 MFMA GEMM with fused epilogues for the ViT / DPT path (gfx950).
//
//   C[g] = epi(A[g] · B[g]^T)       A [M][K] (or implicit 3x3-conv rows of an NHWC image),
//                                   B [N][K] weights (K contiguous: torch Linear layout)
// Tiles (templated): BM x BN x BK with 256 threads = 4 waves laid out WM x WN; each wave
// owns (BM/WM) x (BN/WN) = a grid of 32x32 v_mfma_f32_32x32x16_bf16 accumulators.
// LDS: double buffer, rows padded by 16 B (conflict-free ds_read_b128 of the 32x32x16
// fragments: consecutive rows land 4 banks apart).
// Pipeline: global→register→LDS with prefetch distance 2 (two register sets): the loads
// of K-tile t+2 are issued before tile t's MFMAs and written to LDS only after tile t+1's
// MFMAs, so each load has two MFMA phases to land (the M = 768 transformer GEMMs run one
// workgroup per CU and are latency-bound otherwise).  One barrier per K-tile.
// Implicit conv: the staged rows' output pixels are decoded once; per K-tile the tap
// (ky, kx) and channel offset are block-uniform (Cin % BK == 0).
// Split-K (small tile grids): grid.z = batch x splits, f32 partials to a workspace, then a
// reduce kernel applies the epilogue (deterministic, no atomics).
// Epilogue: bias, GELU(erf), ReLU, f32/bf16 residual, f32/bf16 store, ConvTranspose(k=s)
// scatter.  XCD-aware bijective tile order (cdna_hip_programming.md T1).
#include <type_traits>
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
  int splits;
  float* ws;  // split-K partials [batch*splits][M][N]
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

// Shared epilogue for one element (m, n) of batch g.
struct Epi {
  const float* bias;
  const char* R;
  char* C;
  int flags;
  int64_t ldc, ldr;
  int ct_s, ct_cout, ct_gw;
};

__device__ __forceinline__ Epi make_epi(const Args& a, int g) {
  Epi e;
  const bool out32 = a.flags & M3S_EPI_OUT_F32;
  const bool res32 = a.flags & M3S_EPI_RES_F32;
  e.bias = (a.bias && (a.flags & M3S_EPI_BIAS)) ? a.bias + (int64_t)g * a.sBias : nullptr;
  e.R = a.R ? reinterpret_cast<const char*>(a.R) + (int64_t)g * a.sR * (res32 ? 4 : 2) : nullptr;
  e.C = reinterpret_cast<char*>(a.C) + (int64_t)g * a.sC * (out32 ? 4 : 2);
  e.flags = a.flags;
  e.ldc = a.ldc;
  e.ldr = a.ldr;
  e.ct_s = a.ct_s;
  e.ct_cout = a.ct_cout;
  e.ct_gw = a.ct_gw;
  return e;
}

__device__ __forceinline__ void epi_store(const Epi& e, float v, int m, int n) {
  int co = n, ca = 0, cb = 0;
  const bool convt = e.flags & M3S_EPI_CONVT;
  if (convt) {
    co = n % e.ct_cout;
    const int ab = n / e.ct_cout;
    ca = ab / e.ct_s;
    cb = ab - ca * e.ct_s;
  }
  if (e.bias) v += e.bias[co];
  if (e.flags & M3S_EPI_GELU) v = gelu_erf(v);
  int64_t off;
  if (convt) {
    const int ti = m / e.ct_gw, tj = m - ti * e.ct_gw;
    const int64_t oy = (int64_t)ti * e.ct_s + ca, ox = (int64_t)tj * e.ct_s + cb;
    off = (oy * ((int64_t)e.ct_gw * e.ct_s) + ox) * e.ct_cout + co;
  } else {
    off = (int64_t)m * e.ldc + n;
  }
  if (e.flags & M3S_EPI_RES_F32) v += reinterpret_cast<const float*>(e.R)[(int64_t)m * e.ldr + n];
  if (e.flags & M3S_EPI_RES_BF16)
    v += bf2f(reinterpret_cast<const bf16_t*>(e.R)[(int64_t)m * e.ldr + n]);
  if (e.flags & M3S_EPI_RELU) v = fmaxf(v, 0.f);
  if (e.flags & M3S_EPI_OUT_F32) reinterpret_cast<float*>(e.C)[off] = v;
  else reinterpret_cast<bf16_t*>(e.C)[off] = f2bf(v);
}

template <int BM, int BN, int BK, int WM, int WN, int MODE, bool SPLIT>
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

  const int nwg = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x;
  int wgid = orig;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int tm = wgid / a.tiles_n, tn = wgid - tm * a.tiles_n;
  const int zz = blockIdx.z;
  const int g = SPLIT ? zz / a.splits : zz;
  const int split = SPLIT ? zz - g * a.splits : 0;
  const bf16_t* A = a.A + (int64_t)g * a.sA;
  const bf16_t* B = a.B + (int64_t)g * a.sB;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const bool relu_in = (a.flags & M3S_PRO_RELU) != 0;

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
    a_base[i] = 0;
    a_iy[i] = 0;
    a_ix[i] = 0;
    if (MODE == 0) {
      a_base[i] = (int64_t)(a_ok[i] ? m : 0) * a.lda;
    } else {
      const int mm = a_ok[i] ? m : 0;
      const int oy = mm / a.Wout, ox = mm - oy * a.Wout;
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

  uint4 ra[2][A_CH], rb[2][B_CH];
  // register-set indices must be compile-time constants (a runtime index sends the
  // arrays to scratch): the K loop below is unrolled by two with integral_constant sets
  auto gload = [&](auto setc, int k0) {
    constexpr int set = decltype(setc)::value;
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < A_CH; i++)
        ra[set][i] = a_ok[i] ? *reinterpret_cast<const uint4*>(A + a_base[i] + k0 + a_kc[i])
                             : make_uint4(0, 0, 0, 0);
    } else {
      const int tap = k0 / a.Cin;  // block-uniform: Cin % BK == 0
      const int ci0 = k0 - tap * a.Cin;
      const int ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
      for (int i = 0; i < A_CH; i++) {
        const int iy = a_iy[i] + ky, ix = a_ix[i] + kx;
        const bool ok = a_ok[i] && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
        ra[set][i] = ok ? *reinterpret_cast<const uint4*>(A + ((int64_t)iy * a.Win + ix) * a.Cin +
                                                          ci0 + a_kc[i])
                        : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; i++)
      rb[set][i] = b_ok[i] ? *reinterpret_cast<const uint4*>(
                                 B + (int64_t)(n0 + b_row[i]) * a.ldb + k0 + b_kc[i])
                           : make_uint4(0, 0, 0, 0);
  };
  auto lstore = [&](auto setc, int buf) {
    constexpr int set = decltype(setc)::value;
#pragma unroll
    for (int i = 0; i < A_CH; i++)
      *reinterpret_cast<uint4*>(&As[buf][a_row[i]][a_kc[i]]) = relu_in ? relu8(ra[set][i])
                                                                        : ra[set][i];
#pragma unroll
    for (int i = 0; i < B_CH; i++)
      *reinterpret_cast<uint4*>(&Bs[buf][b_row[i]][b_kc[i]]) = rb[set][i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  const int fr = lane & 31;
  const int fk = (lane >> 5) * 8;
  int nk = a.K / BK;
  int kbase = 0;
  if (SPLIT) {
    const int per = (nk + a.splits - 1) / a.splits;
    kbase = split * per;
    nk = min(per, nk - kbase);
    if (nk < 0) nk = 0;
  }
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (nk > 0) {
    gload(I0{}, (kbase + 0) * BK);
    if (nk > 1) gload(I1{}, (kbase + 1) * BK);
    lstore(I0{}, 0);
    __syncthreads();
  }
  auto step = [&](int kt, auto curc) {
    constexpr int cur = decltype(curc)::value;
    using Other = std::integral_constant<int, cur ^ 1>;
    // prefetch tile kt+2 into register set `cur` (its tile kt is already in LDS)
    if (kt + 2 < nk) gload(curc, (kbase + kt + 2) * BK);
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
    if (kt + 1 < nk) lstore(Other{}, cur ^ 1);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, I0{});
    if (kt + 1 < nk) step(kt + 1, I1{});
  }

  if (SPLIT) {
    float* P = a.ws + (int64_t)zz * a.M * a.N;
#pragma unroll
    for (int j = 0; j < TN; j++) {
      const int n = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
      if (n >= a.N) continue;
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const int m = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (m < a.M) P[(int64_t)m * a.N + n] = acc[i][j][r];
        }
    }
    return;
  }
  const Epi e = make_epi(a, g);
#pragma unroll
  for (int j = 0; j < TN; j++) {
    const int n = n0 + wn * (BN / WN) + j * 32 + (lane & 31);
    if (n >= a.N) continue;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int m = m0 + wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.M) epi_store(e, acc[i][j][r], m, n);
      }
  }
}

// Sum the split-K partials (fixed order) and apply the epilogue; 4 columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(Args a) {
  const int64_t per_b = (int64_t)a.M * a.N;
  const int64_t idx4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int g = blockIdx.y;
  if (idx4 >= per_b) return;
  const Epi e = make_epi(a, g);
  const float* P = a.ws + (int64_t)g * a.splits * per_b;
  float4 s = *reinterpret_cast<const float4*>(P + idx4);
  for (int k = 1; k < a.splits; k++) {
    const float4 t = *reinterpret_cast<const float4*>(P + k * per_b + idx4);
    s.x += t.x;
    s.y += t.y;
    s.z += t.z;
    s.w += t.w;
  }
  const int m = (int)(idx4 / a.N);
  const int n = (int)(idx4 - (int64_t)m * a.N);
  epi_store(e, s.x, m, n);
  epi_store(e, s.y, m, n + 1);
  epi_store(e, s.z, m, n + 2);
  epi_store(e, s.w, m, n + 3);
}

template <int BM, int BN, int BK, int WM, int WN>
int launch(Args& a, int batch, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const bool split = a.splits > 1;
  dim3 grid((unsigned)(a.tiles_m * a.tiles_n), 1, (unsigned)(batch * (split ? a.splits : 1)));
  if (split) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, 0, true>), grid, dim3(NT), 0, s, a);
    M3S_LAUNCH_CHECK();
    const int64_t per_b = (int64_t)a.M * a.N;
    dim3 rg(m3s_div_up(per_b / 4, 256), (unsigned)batch);
    hipLaunchKernelGGL(splitk_reduce_kernel, rg, dim3(256), 0, s, a);
  } else if (a.mode == 0) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, 0, false>), grid, dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, 1, false>), grid, dim3(NT), 0, s, a);
  }
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
  a.splits = 1;
  a.ws = reinterpret_cast<float*>(d->workspace);
  hipStream_t s = m3s_stream(stream);
  const bool k64 = (d->K % 64 == 0) && (d->mode == 0 || d->Cin % 64 == 0);
  const int64_t tiles128 = (int64_t)((d->M + 127) / 128) * ((d->N + 127) / 128) * d->batch;
  const bool small_grid = tiles128 < 192 && d->M <= 1024;
  if (small_grid && k64) {
    // 64x128 tiles; split K when the grid still cannot fill the 256 CUs
    const int64_t tiles = (int64_t)((d->M + 63) / 64) * ((d->N + 127) / 128) * d->batch;
    int splits = d->split_k;
    if (splits <= 0) {
      splits = 1;
      while (tiles * splits < 384 && (d->K / 64) / (splits * 2) >= 8) splits *= 2;
    }
    const bool can_split = d->mode == 0 && !(d->flags & M3S_EPI_CONVT) && d->N % 4 == 0 &&
                           d->workspace &&
                           (int64_t)splits * d->batch * d->M * d->N * 4 <= d->workspace_bytes;
    if (splits > 1 && can_split) a.splits = splits;
    return launch<64, 128, 64, 2, 2>(a, d->batch, s);
  }
  if (small_grid) return launch<64, 128, 32, 2, 2>(a, d->batch, s);
  if (k64) return launch<128, 128, 64, 2, 2>(a, d->batch, s);
  return launch<128, 128, 32, 2, 2>(a, d->batch, s);
}
