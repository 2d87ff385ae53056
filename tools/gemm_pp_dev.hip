// Prototype of the 256x256 8-wave ping-pong bf16 GEMM main loop (tools/gemm_pp_dev.py),
// C = A · B^T with A [M][K], B [N][K] bf16, C bf16 — the main loop in isolation, before it
// moves into csrc/vit_gemm_kern.h with the product epilogues.
//
// Schedule (one K-tile = 4 phases; two wave groups, one barrier apart):
//   LDS: 2 buffers x 4 half-tile slots {A rows 0-127, A rows 128-255, B cols 0-127,
//   B cols 128-255}, 16 KB each (128 KB).  Phase p of K-tile t computes block quadrant
//   (QM, QN) = (0,0), (0,1), (1,1), (1,0) over K = 64: every wave its 64x32 share of that
//   128x128 quadrant, 16 v_mfma_f32_16x16x32_bf16.  Fragments are read where the quadrant
//   changes them (A0+B0, B1, A1, B0: 28 ds_read_b128 per K-tile per wave) and held in one
//   register set across phases.
//   Phase p also issues half-tile p of K-tile t+1 (order A0, B0, B1, A1) into the other
//   buffer, and waits vmcnt(4): the half-tile issued two phases earlier is retired.
//   Group 1 (waves 4-7) runs one barrier behind group 0, so on every SIMD one wave is in
//   its MFMA segment while its partner issues reads / DMA (MI355X_MICROARCH.md "Two waves
//   per SIMD").  The RAW / WAR distances of this order are checked in DESIGN.md §4.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace pp {
constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int HB = 128 * BK * 2;       // half-tile bytes
constexpr int BUFB = 4 * HB;           // one K-tile buffer
constexpr int RING = 2 * BUFB;         // 128 KB
constexpr int CST = BN + 4;            // epilogue f32 row stride
constexpr int EPIB = 128 * CST * 4;    // one 128-row pass
constexpr int LDSB = EPIB > RING ? EPIB : RING;
constexpr uint32_t OOB = 0x80000000u;
constexpr int32_t NUM_RECORDS = 0x7ffffff0;

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)(lds), 16, voff, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int PRIO>
__global__ __launch_bounds__(NT, 1) void gemm_pp(const bf16_t* __restrict__ A,
                                                 const bf16_t* __restrict__ B, bf16_t* C, int M,
                                                 int N, int K, int lda, int ldb, int ldc,
                                                 long sA, long sB, long sC, int group_m) {
  __shared__ __attribute__((aligned(16))) char lds[LDSB];
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int total = gridDim.x;
  const int orig = blockIdx.x;
  int wid_lin = orig;
  if (total >= 16) {
    const int q = total / 8, r = total % 8, xcd = orig % 8;
    wid_lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  const int z = wid_lin / nwg;
  const int wg = wid_lin - z * nwg;
  int tm, tn;
  if (group_m > 0) {
    const int per = group_m * tiles_n;
    const int grp = wg / per, first = grp * group_m;
    const int gsz = min(tiles_m - first, group_m);
    const int in = wg - grp * per;
    tm = first + in % gsz;
    tn = in / gsz;
  } else {
    tm = wg / tiles_n;
    tn = wg - tm * tiles_n;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(A + z * sA), (short)0, NUM_RECORDS, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(B + z * sB), (short)0, NUM_RECORDS, 0x00020000);

  // DMA: a half-tile is 128 rows x 8 chunks of 16 B; thread chunk q = i*512 + tid lands at
  // row q >> 3, slot q & 7 and carries logical chunk slot ^ ((row >> 1) & 7)
  uint32_t off[4][2];
  int kc[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int q = i * NT + tid;
    const int r = q >> 3, p = q & 7;
    kc[i] = (p ^ ((r >> 1) & 7)) * 8;
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const int row = (h & 1) * 128 + r;
      if (h < 2) {
        const int m = m0 + row;
        off[h][i] = m < M ? (uint32_t)(((int64_t)m * lda + kc[i]) * 2) : OOB;
      } else {
        const int n = n0 + row;
        off[h][i] = n < N ? (uint32_t)(((int64_t)n * ldb + kc[i]) * 2) : OOB;
      }
    }
  }
  // slot index: A0 0, A1 1, B0 2, B1 3
  const int nk = (K + BK - 1) / BK;
  auto issue = [&](int t, int h) {  // half-tile h of K-tile t
    char* dst = lds + (t & 1) * BUFB + h * HB + wid * 64 * 16;
    const int k0 = t * BK;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t vo = (k0 + kc[i] < K) ? off[h][i] + (uint32_t)k0 * 2 : OOB;
      glds16(h < 2 ? rA : rB, dst + i * NT * 16, vo);
    }
  };

  // fragment addresses: lane reads row (lane & 15) of a 16-row tile, chunk 4s + (lane >> 4)
  // swizzled by ((row >> 1) & 7) = (lane & 15) >> 1 (tile bases are multiples of 16 rows)
  const int fr = lane & 15, fc = lane >> 4, sw = fr >> 1;
  const int lo0 = fr * 128 + ((fc ^ sw) << 4);
  const int lo1 = fr * 128 + (((fc ^ sw) ^ 4) << 4);

  bf16x8 af[4][2], bfr[2][2];
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a0 = 0; a0 < 2; a0++)
#pragma unroll
    for (int a1 = 0; a1 < 2; a1++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[a0][a1][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_a = [&](const char* slot) {
    const char* base = slot + wr * 64 * 128;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      af[i][0] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + lo0);
      af[i][1] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + lo1);
    }
  };
  auto read_b = [&](const char* slot) {
    const char* base = slot + wc * 32 * 128;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      bfr[j][0] = *reinterpret_cast<const bf16x8*>(base + j * 16 * 128 + lo0);
      bfr[j][1] = *reinterpret_cast<const bf16x8*>(base + j * 16 * 128 + lo1);
    }
  };
  auto mfmas = [&](f32x4 (&c)[4][2]) {
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bfr[j][s], c[i][j], 0, 0, 0);
  };

  // prologue: K-tile 0 into buffer 0; A0 and B0 retired before the loop's first reads
  issue(0, 0);
  issue(0, 2);
  issue(0, 3);
  issue(0, 1);
  vm_wait<4>();
  bar();
  if (wr == 1) bar();   // the stagger
  if (PRIO == 2 && wr == 1) __builtin_amdgcn_s_setprio(1);

#define M3S_PP_SEG(READS, ISSUE_H, QM, QN)        \
  READS;                                          \
  issue(t + 1, ISSUE_H);                          \
  vm_wait<4>();                                   \
  bar();                                          \
  if (PRIO == 1) __builtin_amdgcn_s_setprio(1);   \
  mfmas(acc[QM][QN]);                             \
  if (PRIO == 1) __builtin_amdgcn_s_setprio(0);   \
  bar();

  int t = 0;
  for (; t < nk - 1; t++) {
    const char* cur = lds + (t & 1) * BUFB;
    M3S_PP_SEG((read_a(cur), read_b(cur + 2 * HB)), 0, 0, 0)
    M3S_PP_SEG(read_b(cur + 3 * HB), 2, 0, 1)
    M3S_PP_SEG(read_a(cur + HB), 3, 1, 1)
    M3S_PP_SEG(read_b(cur + 2 * HB), 1, 1, 0)
  }
#undef M3S_PP_SEG
  // last K-tile: nothing left to issue (phase 0 retires B1, phase 1 A1)
#define M3S_PP_TAIL(READS, W, QM, QN)             \
  READS;                                          \
  vm_wait<W>();                                   \
  bar();                                          \
  if (PRIO == 1) __builtin_amdgcn_s_setprio(1);   \
  mfmas(acc[QM][QN]);                             \
  if (PRIO == 1) __builtin_amdgcn_s_setprio(0);   \
  bar();
  {
    const char* cur = lds + (t & 1) * BUFB;
    M3S_PP_TAIL((read_a(cur), read_b(cur + 2 * HB)), 2, 0, 0)
    M3S_PP_TAIL(read_b(cur + 3 * HB), 0, 0, 1)
    M3S_PP_TAIL(read_a(cur + HB), 0, 1, 1)
    M3S_PP_TAIL(read_b(cur + 2 * HB), 0, 1, 0)
  }
#undef M3S_PP_TAIL
  if (wr == 0) bar();   // re-align the groups
  vm_wait<0>();
  bar();

  // epilogue: two 128-row passes through an f32 LDS tile, 16-B bf16 stores
  float* cs = reinterpret_cast<float*>(lds);
  bf16_t* Cz = C + z * sC;
#pragma unroll
  for (int pass = 0; pass < 2; pass++) {
    if (pass) bar();
#pragma unroll
    for (int qn = 0; qn < 2; qn++)
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int row = wr * 64 + i * 16 + fc * 4 + r;
            const int col = qn * 128 + wc * 32 + j * 16 + fr;
            cs[row * CST + col] = pass == 0 ? acc[0][qn][i][j][r] : acc[1][qn][i][j][r];
          }
    bar();
#pragma unroll
    for (int v = 0; v < 8; v++) {
      const int idx = v * NT + tid;
      const int row = idx >> 5, c = (idx & 31) * 8;
      const int m = m0 + pass * 128 + row, n = n0 + c;
      if (m < M && n < N) {
        const float4 x0 = *reinterpret_cast<const float4*>(cs + row * CST + c);
        const float4 x1 = *reinterpret_cast<const float4*>(cs + row * CST + c + 4);
        bf16x8 o;
        o[0] = (bf16_t)x0.x; o[1] = (bf16_t)x0.y; o[2] = (bf16_t)x0.z; o[3] = (bf16_t)x0.w;
        o[4] = (bf16_t)x1.x; o[5] = (bf16_t)x1.y; o[6] = (bf16_t)x1.z; o[7] = (bf16_t)x1.w;
        *reinterpret_cast<bf16x8*>(Cz + (int64_t)m * ldc + n) = o;
      }
    }
  }
}
}  // namespace pp

extern "C" int pp_gemm(const void* A, const void* B, void* C, int M, int N, int K, int batch,
                       int lda, int ldb, int ldc, long sA, long sB, long sC, int group_m,
                       int prio, void* stream) {
  if (K % 8 || N % 8 || ldc % 8) return -1;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256) * batch;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define M3S_PP_L(P)                                                                      \
  hipLaunchKernelGGL(pp::gemm_pp<P>, dim3(tiles), dim3(512), 0, s, (const bf16_t*)A,          \
                     (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb, ldc, sA, sB, sC, group_m)
  if (prio == 1) M3S_PP_L(1);
  else if (prio == 2) M3S_PP_L(2);
  else M3S_PP_L(0);
#undef M3S_PP_L
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
