// GEMM kernel templates and launchers (vit_gemm.hip's kernel side), shared by the
// dispatcher (vit_gemm.hip) and the per-configuration instantiation units
// (vit_gemm_i*.hip), compiled in parallel.  A -DM3S_GEMM_STAMPS build compiles the
// dispatcher alone, instantiating everything in one unit.
#pragma once
// Batched bf16 MFMA GEMM with fused epilogues for the ViT / DPT path (gfx950).
//
//   C[g] = epi(A[g] · B[g]^T)       A [M][K] (or implicit 3x3-conv rows of an NHWC image),
//                                   B [N][K] weights (K contiguous: torch Linear layout)
//
// Main loop (cdna_hip_programming.md §5 "Pipelining across barriers"):
//  * operands go HBM → LDS with 16-B LDS-DMA buffer loads (buffer_load_dwordx4 … lds), a
//    ring of STAGES K-tiles in one __shared__ array; tile t+STAGES-1 is issued right after
//    the barrier that retires tile t, so STAGES-1 tiles are in flight during each MFMA
//    phase; counted `s_waitcnt vmcnt(N)` + raw s_barrier (never __syncthreads, whose fence
//    would drain the DMA queue).
//  * out-of-range rows, K tails and conv zero padding are buffer out-of-bounds reads
//    (voffset ≥ num_records → the hardware writes zeros): no branches around loads.
//  * LDS image is lane-linear per wave instruction (what the DMA writes); bank conflicts of
//    the ds_read_b128 fragment reads are removed by XOR-swizzling the 16-B chunk index with
//    the row (applied to the per-lane GLOBAL address at load time and to the read address).
//  * 4 waves, each a grid of 32x32 v_mfma_f32_32x32x16_bf16 accumulators.
// Epilogue: accumulators → LDS f32 tile → row-contiguous 8-column vectors per thread:
//   bias, GELU(erf), 2D RoPE (croco RoPE2D, via a per-token cos/sin table), f32/bf16
//   residual, ReLU, f32/bf16 store, ConvTranspose(k=s) scatter — 16-B loads/stores.
// Split-K (tile grids that cannot fill 256 CUs): batch x splits groups of workgroups; each
//   writes its f32 partial tile to a workspace and bumps the tile's counter (agent-scope
//   release); the LAST split of a tile (acquire) sums the partials in split order — fixed,
//   so deterministic whichever workgroup finishes last — and runs the normal epilogue (any
//   flag set, LayerNorm fold included).  One launch; counters return to zero.
// Implicit conv (MODE 1, MODE 2 = ReLU on A): per K-tile the tap (ky, kx) and channel
//   offset are block-uniform (Cin % BK == 0); ReLU is applied to the A fragments in
//   registers (v_pk_max_i16 on the bf16 bits).
// XCD-aware bijective tile order (cdna_hip_programming.md T1).
#include <stdlib.h>
#include <algorithm>
#include <type_traits>
#include "vit_common.h"

namespace m3s_gemm {

constexpr int NT = 256;
constexpr uint32_t OOB = 0x80000000u;      // any voffset ≥ num_records reads as zero
constexpr int32_t NUM_RECORDS = 0x7ffffff0;

typedef short s16x2 __attribute__((ext_vector_type(2)));

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
  int nmajor;              // tile order within a group (see gemm_kernel)
  int group_m;             // > 0: grouped order, group_m M-bands per group (see gemm_kernel)
  int splits;
  int vec;                 // 8-wide vector epilogue allowed (alignment / N % 8 checked on host)
  float* ws;               // split-K partials [batch*splits][M][N]
  int* cnt;                // split-K tile counters [batch][tiles] (zero between launches)
  int fused;               // split-K: 1 = the last split reduces + epilogue, 0 = reduce kernel
  const float* rope_tab;   // [tokens][2 (y,x)][2 (cos,sin)][16]
  int rope_cols, rope_tokens;
  int wmod;                // > 0: weights / bias of batch g % wmod
  const float* dpt_w4;     // DPT_OUT tail (see m3s_gemm_desc)
  const float* dpt_b4;
  float* dpt_pts;
  float* dpt_conf;
  float dpt_conf_min;
  const float* cscale;     // IN_FP8: per-column dequant scale, batch stride sCscale
  int64_t sCscale;
  bf16_t* C2;              // LN_STATS: bf16 copy of C
  float* stats;            // LN_STATS out / LN_FOLD in: [batch][M][groups] x (mean, M2)
  int a_xor;               // LN_FOLD: A and stats of batch g ^ a_xor
  const float* ln_c1;      // LN_FOLD: row sums of the gamma-folded weight (stride sBias)
  float ln_eps;
  int ln_groups;           // LN_FOLD: 128-column groups per stats row (LayerNorm dim / 128)
  const float* ln_c3;      // LN_FOLD + IN_FP8: Σ_k shift[k] B[n][k], added after the dequant
  const float* ln_shift;   // LN_STATS: non-null → C2 = e4m3((C − shift[n]) · ln_qscale[g])
  const float* ln_qscale;  //   (one scale per weight batch, device memory: re-calibration
                           //   in place reaches captured graphs)
  unsigned long long* tl;  // step-timeline slot or null (common.h)
};

// Row statistics of a LN_FOLD consumer from the producer's per-128-column (mean_t, M2_t)
// groups (all of equal size, so no pairwise weights): mean = Σ mean_t / G,
// M2 = Σ M2_t + 128 Σ (mean_t − mean)², biased variance M2 / (128 G) as nn.LayerNorm.
// Fixed order → deterministic.  mu / rstd of row m of batch gs; groups ≤ 8.
__device__ __forceinline__ void ln_row_stats(const Args& a, int64_t gs, int m, int groups,
                                             float& mu, float& rs) {
  const float2* st = reinterpret_cast<const float2*>(a.stats) + (gs * a.M + m) * groups;
  float2 s[8];
#pragma unroll
  for (int t = 0; t < 8; t++) s[t] = t < groups ? st[t] : make_float2(0.f, 0.f);
  float sm = 0.f, m2 = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) sm += s[t].x;
  const float mean = sm / (float)groups;
#pragma unroll
  for (int t = 0; t < 8; t++) {
    const float d = t < groups ? s[t].x - mean : 0.f;
    m2 += fmaf(128.f * d, d, s[t].y);
  }
  mu = mean;
  rs = 1.0f / sqrtf(m2 / (128.f * (float)groups) + a.ln_eps);
}

// Sum over the 16 lanes of a DPP row (xor 1, xor 2 in the quad, then half-row and row
// mirrors pair every lane with the other half): 4 VALU ops with DPP operands.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

// LN_STATS producer: (mean, M2) of the 128 columns [n, n + 128) of row m held by 16
// consecutive lanes (8 values each; n = 8·(lane % 16) + group base), written by the
// group's first lane.  All 16 lanes of a group are active together (rows are uniform).
__device__ __forceinline__ void ln_group_stats(const Args& a, int64_t g, int m, int n,
                                               const float* x) {
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) s += x[t];
  s = sum16(s);
  const float mean = s * (1.0f / 128.0f);
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < 8; t++) {
    const float d = x[t] - mean;
    q = fmaf(d, d, q);
  }
  q = sum16(q);
  if ((threadIdx.x & 15) == 0) {
    const int groups = a.N >> 7;
    reinterpret_cast<float2*>(a.stats)[(g * a.M + m) * groups + (n >> 7)] = make_float2(mean, q);
  }
}

__device__ __forceinline__ void store_bf16x8(bf16_t* p, const float* x) {
  bf16x8 o;
#pragma unroll
  for (int t = 0; t < 8; t++) o[t] = f2bf(x[t]);
  *reinterpret_cast<bf16x8*>(p) = o;
}

// LN_STATS: the copy of the 8 stored values [n, n+8) of row m that the LN_FOLD consumer
// reads as A — bf16, or (ln_shift set: the fp8 consumer) e4m3 of (x − shift[n]) · qscale,
// the per-channel calibrated shift centring each channel before the 3-bit mantissa.
// ln_c2_operands loads a thread's 8 shifts + the scale once, ahead of the epilogue's
// stores: a load issued between them would wait for every store before it (vmcnt counts
// both), one memory round trip per row vector.  (Measured cost of the whole LN_STATS
// epilogue on the 1,024-token residual GEMMs: 0.6-2.4 us per launch, tools/ls_cost_probe.py)
__device__ __forceinline__ void ln_c2_operands(const Args& a, int64_t g, int n, float* sh,
                                               float& q) {
  const int64_t gw = a.wmod > 0 ? g % a.wmod : g;
  const float* p = a.ln_shift + gw * a.sBias + n;
  *reinterpret_cast<float4*>(sh) = *reinterpret_cast<const float4*>(p);
  *reinterpret_cast<float4*>(sh + 4) = *reinterpret_cast<const float4*>(p + 4);
  q = a.ln_qscale[gw];
}

__device__ __forceinline__ void ln_store_c2(const Args& a, int64_t g, int64_t off,
                                            const float* x, const float* sh, float q) {
  if (a.ln_shift) {
    uint8_t* p = reinterpret_cast<uint8_t*>(a.C2) + g * a.sC + off;
    *reinterpret_cast<uint2*>(p) =
        make_uint2(pack4_fp8((x[0] - sh[0]) * q, (x[1] - sh[1]) * q, (x[2] - sh[2]) * q,
                             (x[3] - sh[3]) * q),
                   pack4_fp8((x[4] - sh[4]) * q, (x[5] - sh[5]) * q, (x[6] - sh[6]) * q,
                             (x[7] - sh[7]) * q));
  } else {
    store_bf16x8(a.C2 + g * a.sC + off, x);
  }
}

// ---------------------------------------------------------------------------------------
// epilogue
// ---------------------------------------------------------------------------------------
struct Epi {
  const float* bias;
  const char* R;
  char* C;
  int flags;
  int64_t ldc, ldr;
  int ct_s, ct_cout, ct_gw;
  const float* rope_tab;
  int rope_cols, rope_tokens;
};

__device__ __forceinline__ Epi make_epi(const Args& a, int g) {
  Epi e;
  const bool out32 = a.flags & M3S_EPI_OUT_F32;
  const bool res32 = a.flags & M3S_EPI_RES_F32;
  const int64_t gw = a.wmod > 0 ? g % a.wmod : g;
  e.bias = (a.bias && (a.flags & M3S_EPI_BIAS)) ? a.bias + gw * a.sBias : nullptr;
  e.R = a.R ? reinterpret_cast<const char*>(a.R) + (int64_t)g * a.sR * (res32 ? 4 : 2) : nullptr;
  const int osz = out32 ? 4 : ((a.flags & M3S_EPI_OUT_FP8) ? 1 : 2);
  e.C = reinterpret_cast<char*>(a.C) + (int64_t)g * a.sC * osz;
  e.flags = a.flags;
  e.ldc = a.ldc;
  e.ldr = a.ldr;
  e.ct_s = a.ct_s;
  e.ct_cout = a.ct_cout;
  e.ct_gw = a.ct_gw;
  e.rope_tab = a.rope_tab;
  e.rope_cols = a.rope_cols;
  e.rope_tokens = a.rope_tokens;
  return e;
}

// output element offset of (m, n) (ConvTranspose scatter: n = (a*s + b)*Cout + co)
__device__ __forceinline__ int64_t out_offset(const Epi& e, int m, int n, int& co) {
  if (e.flags & M3S_EPI_CONVT) {
    co = n % e.ct_cout;
    const int ab = n / e.ct_cout;
    const int ca = ab / e.ct_s, cb = ab - ca * e.ct_s;
    const int ti = m / e.ct_gw, tj = m - ti * e.ct_gw;
    const int64_t oy = (int64_t)ti * e.ct_s + ca, ox = (int64_t)tj * e.ct_s + cb;
    return (oy * ((int64_t)e.ct_gw * e.ct_s) + ox) * e.ct_cout + co;
  }
  co = n;
  return (int64_t)m * e.ldc + n;
}

// RoPE2D on an 8-column group [n, n+8) of one head (head dim 64 = [y | x] halves; in a
// half, pairs (i, i+16)): v are the group's values, p the partner group's (n ^ 16).
__device__ __forceinline__ void rope8(const Epi& e, float* v, const float* p, int m, int n) {
  const int s = m % e.rope_tokens;
  const int half = (n >> 5) & 1;
  const int i0 = n & 15;
  const float* t = e.rope_tab + ((int64_t)s * 2 + half) * 32;
  const float4 c0 = *reinterpret_cast<const float4*>(t + i0);
  const float4 c1 = *reinterpret_cast<const float4*>(t + i0 + 4);
  const float4 s0 = *reinterpret_cast<const float4*>(t + 16 + i0);
  const float4 s1 = *reinterpret_cast<const float4*>(t + 16 + i0 + 4);
  const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sg = (n & 16) ? 1.f : -1.f;  // lower: u c - v s; upper: v c + u s
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = v[i] * cs[i] + sg * p[i] * sn[i];
}

// 8 consecutive columns [n, n+8) of row m; p = partner columns (n ^ 16) for RoPE or null.
__device__ __forceinline__ void epi_vec8(const Epi& e, float* v, float* p, int m, int n) {
  int co;
  const int64_t off = out_offset(e, m, n, co);
  if (e.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(e.bias + co);
    const float4 b1 = *reinterpret_cast<const float4*>(e.bias + co + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if (e.flags & M3S_EPI_GELU) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gelu_erf(v[i]);
  }
  if ((e.flags & M3S_EPI_ROPE) && n < e.rope_cols) {
    const int pn = n ^ 16;
    if (e.bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(e.bias + pn);
      const float4 b1 = *reinterpret_cast<const float4*>(e.bias + pn + 4);
      p[0] += b0.x; p[1] += b0.y; p[2] += b0.z; p[3] += b0.w;
      p[4] += b1.x; p[5] += b1.y; p[6] += b1.z; p[7] += b1.w;
    }
    rope8(e, v, p, m, n);
  }
  if (e.flags & M3S_EPI_RES_F32) {
    const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)m * e.ldr + n;
    const float4 r0 = *reinterpret_cast<const float4*>(r);
    const float4 r1 = *reinterpret_cast<const float4*>(r + 4);
    v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
    v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
  }
  if (e.flags & M3S_EPI_RES_BF16) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(
        reinterpret_cast<const bf16_t*>(e.R) + (int64_t)m * e.ldr + n);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] += bf2f(r[i]);
  }
  if (e.flags & M3S_EPI_RELU) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = fmaxf(v[i], 0.f);
  }
  if (e.flags & M3S_EPI_OUT_F32) {
    float* c = reinterpret_cast<float*>(e.C) + off;
    *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else if (e.flags & M3S_EPI_OUT_FP8) {
    *reinterpret_cast<uint2*>(e.C + off) = make_uint2(pack4_fp8(v[0], v[1], v[2], v[3]),
                                                      pack4_fp8(v[4], v[5], v[6], v[7]));
  } else {
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; i++) o[i] = f2bf(v[i]);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16_t*>(e.C) + off) = o;
  }
}

// one element (tails / unaligned shapes); p = partner value (RoPE) incl. its bias
__device__ __forceinline__ void epi_one(const Epi& e, float v, float p, int m, int n) {
  int co;
  const int64_t off = out_offset(e, m, n, co);
  if (e.bias) v += e.bias[co];
  if (e.flags & M3S_EPI_GELU) v = gelu_erf(v);
  if ((e.flags & M3S_EPI_ROPE) && n < e.rope_cols) {
    if (e.bias) p += e.bias[n ^ 16];
    const int s = m % e.rope_tokens, half = (n >> 5) & 1, i = n & 15;
    const float* t = e.rope_tab + ((int64_t)s * 2 + half) * 32;
    v = v * t[i] + ((n & 16) ? 1.f : -1.f) * p * t[16 + i];
  }
  if (e.flags & M3S_EPI_RES_F32) v += reinterpret_cast<const float*>(e.R)[(int64_t)m * e.ldr + n];
  if (e.flags & M3S_EPI_RES_BF16)
    v += bf2f(reinterpret_cast<const bf16_t*>(e.R)[(int64_t)m * e.ldr + n]);
  if (e.flags & M3S_EPI_RELU) v = fmaxf(v, 0.f);
  if (e.flags & M3S_EPI_OUT_F32) reinterpret_cast<float*>(e.C)[off] = v;
  else if (e.flags & M3S_EPI_OUT_FP8) e.C[off] = (char)(pack4_fp8(v, 0.f, 0.f, 0.f) & 0xff);
  else reinterpret_cast<bf16_t*>(e.C)[off] = f2bf(v);
}

// ---------------------------------------------------------------------------------------
// main kernel
// ---------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int STAGES, int NTH = 256>
struct Cfg {
  // the f32 epilogue tile of a 256x256 block (266 KB) exceeds the 160 KB LDS: it is
  // written and stored in two passes of 128 rows
  static constexpr int PASSES = (BM * (BN + 4) * 4 > 160 * 1024) ? 2 : 1;
  static constexpr int EROWS = BM / PASSES;
  static constexpr int CPR = BK / 8;                 // 16-B chunks per row
  static constexpr int RPB = 256 / (BK * 2);         // rows per 256-B LDS bank row
  static constexpr int A_CH = BM * CPR / NTH;        // DMA chunks per thread per K-tile
  static constexpr int B_CH = BN * CPR / NTH;
  static constexpr int L = A_CH + B_CH;              // vmcnt units per K-tile
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int ST_BYTES = (BM + BN) * BK * 2;
  static constexpr int CST = BN + 4;                 // epilogue f32 row stride
  static constexpr int EPI_BYTES = EROWS * CST * 4;
  static constexpr int LDS_BYTES = STAGES * ST_BYTES > EPI_BYTES ? STAGES * ST_BYTES : EPI_BYTES;
};

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)(lds), 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  // the builtin (not inline asm) so the compiler's own wait-count tracking sees the DMA
  // retired — otherwise it later waits vmcnt(0) before every ds_read of the epilogue,
  // i.e. behind each preceding global store.  gfx9 encoding: vmcnt[3:0] | vmcnt[5:4]<<14,
  // expcnt[6:4] = 7, lgkmcnt[11:8] = 15 (no wait on those).
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ bf16x8 relu_frag(bf16x8 x) {
  // bf16 ReLU on the bit patterns: negative values are negative int16s (−0 → +0)
  s16x2* w = reinterpret_cast<s16x2*>(&x);
  const s16x2 z = {0, 0};
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = __builtin_elementwise_max(w[i], z);
  return x;
}

// Optional in-kernel timeline (build with -DM3S_GEMM_STAMPS, tools/gemm_stamps.py): wave 0
// of each workgroup accumulates s_memtime deltas per phase into g_m3s_stamps[block][8].
#ifdef M3S_GEMM_STAMPS
__device__ long long* g_m3s_stamps;
#define M3S_T(v) long long v = (long long)__builtin_amdgcn_s_memtime()
// [0] prologue [1] vmcnt wait [2] barrier [3] MFMA phases (per-K-tile sums) [4] epilogue
// [5] K-tiles [6] block total [7] start (shader cycles) [8] epilogue ([9..11] unused)
// [12] / [13] s_memrealtime (100 MHz) at start / end [14] 1 = early exit (non-last split)
// [15] first K-tile wait (prologue issue → first fragments read) [16] tail K-tiles
#define M3S_STAMP_OUT_(early)                                                     \
  if (tid == 0) {                                                                 \
    M3S_T(t_end);                                                                 \
    long long* o = g_m3s_stamps + (int64_t)blockIdx.x * 20;                       \
    o[8] = t_end - t_loop;                                                        \
    o[9] = o[10] = o[11] = 0;                                                     \
    o[0] = t_pro - t_start;                                                       \
    o[1] = s_wait;                                                                \
    o[2] = s_bar;                                                                 \
    o[3] = s_comp;                                                                \
    o[4] = t_end - t_loop;                                                        \
    o[5] = nk;                                                                    \
    o[6] = t_end - t_start;                                                       \
    o[7] = t_start;                                                               \
    o[12] = rt_start;                                                             \
    o[13] = (long long)__builtin_amdgcn_s_memrealtime();                          \
    o[14] = early;                                                                \
    o[15] = t_first - t_pro;                                                      \
    o[16] = t_loop - t_steady;                                                    \
  }
#define M3S_STAMP_OUT() M3S_STAMP_OUT_(0)
#define M3S_STAMP_EARLY() M3S_STAMP_OUT_(1)
#else
#define M3S_T(v)
#define M3S_STAMP_OUT()
#define M3S_STAMP_EARLY()
#endif

// ---------------------------------------------------------------------------------------
// epilogue (shared by gemm_kernel and the 256x256 ping-pong gemm_pp_kernel)
// ---------------------------------------------------------------------------------------
// The block's f32 accumulator tile goes through LDS in PASSES passes of BM / PASSES rows:
// store_acc(pass, cs) writes the accumulators of that pass's rows into cs[row][CST]
// (CST = BN + 4), then row-contiguous 8-column vectors per thread run the fused epilogue
// (bias, LayerNorm fold, GELU, RoPE, residual, ReLU, f32 / bf16 / e4m3 stores, LayerNorm
// statistics, ConvTranspose scatter, the DPT tail) — or, split-K, the slice's partial
// tile is published and the tile's last slice reduces.  Returns false for a split-K slice
// that is not its tile's last (it stored nothing).
template <int BM, int BN, int NT, int PASSES, int LDS_BYTES, bool SPLIT, int EPI, class StoreAcc>
__device__ __forceinline__ bool gemm_epilogue(const Args& a, char* lds, int g, int zz, int nwg,
                                              int wgid, int split, int m0, int n0,
                                              M3sTlEnd& tl_end, StoreAcc&& store_acc) {
  constexpr int CST = BN + 4;
  constexpr int EROWS = BM / PASSES;
  constexpr bool DPT = EPI >= 0 && (EPI & M3S_EPI_DPT_OUT) != 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  constexpr int VPR = BN / 8;                 // 8-column vectors per row
  static_assert(PASSES == 1 || !SPLIT, "two-pass epilogue: unsplit");
  constexpr int NV = EROWS * VPR / NT;        // vectors per thread (per pass)
  constexpr int RSTEP = NT / VPR;             // rows between one thread's vectors
  static_assert(NT % VPR == 0, "epilogue layout");
  // Vector path: a thread owns columns [n, n+8) of rows r0 + v*RSTEP.  Its bias and, per
  // group of EG vectors, the residual (or RoPE cos/sin) operands are loaded ahead of use —
  // the first group before the LDS round trip — so their latency is overlapped.
  // EG must divide NV (96-row tiles have NV = 6: groups of 4 would run past the tile into
  // the next tile's rows)
  constexpr int EG = NV % 4 == 0 ? 4 : NV % 3 == 0 ? 3 : NV % 2 == 0 ? 2 : 1;
  const int ec = (tid % VPR) * 8, er0 = tid / VPR;
  const int en = n0 + ec;
  const int fl = EPI >= 0 ? EPI : a.flags;
  const bool vec = EPI >= 0 ? true : (a.vec != 0);
  const bool vec_path = vec && en < a.N;
  float e_b[8], e_pb[8], e_x[EG][16];
  float e_c1[8], e_pc1[8], e_mu[EG], e_rs[EG];  // LN_FOLD: c1 columns, row mean / rstd
  float e_sh[8], e_q = 0.f;                     // LN_STATS e4m3 copy: shifts, scale
  // LN_FOLD: the 16 lanes of a row group own rows er0 + v·RSTEP (v < NV ≤ 16); lane v
  // combines the statistics of row v once, the others read it by lane shuffle
  float ln_mu = 0.f, ln_rs = 0.f;
  static_assert(NV <= 16, "one row per lane of the group");
  int rb = 0;                                 // first tile row of the epilogue pass
  auto ln_setup = [&]() {
    if ((fl & M3S_EPI_LN_FOLD) && (lane & 15) < NV)
      ln_row_stats(a, g ^ a.a_xor, min(m0 + rb + er0 + (lane & 15) * RSTEP, a.M - 1),
                   a.ln_groups, ln_mu, ln_rs);
  };
  Epi e = make_epi(a, g);
  e.flags = fl;
  const bool e_rope = (fl & M3S_EPI_ROPE) && en < a.rope_cols;
  auto e_prefetch = [&](int v0) {
#pragma unroll
    for (int u = 0; u < EG; u++) {
      const int m = min(m0 + rb + er0 + (v0 + u) * RSTEP, a.M - 1);  // rows ≥ M are not stored
      if (fl & M3S_EPI_LN_FOLD) {  // row v0 + u's statistics, held by lane v0 + u of the row group
        const int src = (lane & ~15) | (v0 + u);
        e_mu[u] = __shfl(ln_mu, src, 64);
        e_rs[u] = __shfl(ln_rs, src, 64);
      }
#pragma unroll
      for (int t = 0; t < 16; t++) e_x[u][t] = 0.f;
      if (fl & M3S_EPI_RES_F32) {
        const float* r = reinterpret_cast<const float*>(e.R) + (int64_t)m * e.ldr + en;
        *reinterpret_cast<float4*>(&e_x[u][0]) = *reinterpret_cast<const float4*>(r);
        *reinterpret_cast<float4*>(&e_x[u][4]) = *reinterpret_cast<const float4*>(r + 4);
      } else if (fl & M3S_EPI_RES_BF16) {
        const bf16x8 r = *reinterpret_cast<const bf16x8*>(
            reinterpret_cast<const bf16_t*>(e.R) + (int64_t)m * e.ldr + en);
#pragma unroll
        for (int t = 0; t < 8; t++) e_x[u][t] = bf2f(r[t]);
      } else if (e_rope) {  // RoPE GEMMs carry no residual: cos → [0, 8), sin → [8, 16)
        const float* tb = e.rope_tab +
                          ((int64_t)(m % e.rope_tokens) * 2 + ((en >> 5) & 1)) * 32 + (en & 15);
        *reinterpret_cast<float4*>(&e_x[u][0]) = *reinterpret_cast<const float4*>(tb);
        *reinterpret_cast<float4*>(&e_x[u][4]) = *reinterpret_cast<const float4*>(tb + 4);
        *reinterpret_cast<float4*>(&e_x[u][8]) = *reinterpret_cast<const float4*>(tb + 16);
        *reinterpret_cast<float4*>(&e_x[u][12]) = *reinterpret_cast<const float4*>(tb + 20);
      }
    }
  };
  auto epi_setup = [&](bool prefetch_rows) {
    if (!vec_path) return;
    int co;
    (void)out_offset(e, m0, en, co);
#pragma unroll
    for (int t = 0; t < 8; t++) e_b[t] = e_pb[t] = 0.f;
    if (e.bias) {
      *reinterpret_cast<float4*>(&e_b[0]) = *reinterpret_cast<const float4*>(e.bias + co);
      *reinterpret_cast<float4*>(&e_b[4]) = *reinterpret_cast<const float4*>(e.bias + co + 4);
      if (e_rope) {
        *reinterpret_cast<float4*>(&e_pb[0]) = *reinterpret_cast<const float4*>(e.bias + (en ^ 16));
        *reinterpret_cast<float4*>(&e_pb[4]) =
            *reinterpret_cast<const float4*>(e.bias + (en ^ 16) + 4);
      }
    }
    if (fl & M3S_EPI_LN_FOLD) {
      const float* c1 = a.ln_c1 + (int64_t)(a.wmod > 0 ? g % a.wmod : g) * a.sBias;
      *reinterpret_cast<float4*>(&e_c1[0]) = *reinterpret_cast<const float4*>(c1 + en);
      *reinterpret_cast<float4*>(&e_c1[4]) = *reinterpret_cast<const float4*>(c1 + en + 4);
      if (e_rope) {
        *reinterpret_cast<float4*>(&e_pc1[0]) = *reinterpret_cast<const float4*>(c1 + (en ^ 16));
        *reinterpret_cast<float4*>(&e_pc1[4]) =
            *reinterpret_cast<const float4*>(c1 + (en ^ 16) + 4);
      }
    }
    if ((fl & M3S_EPI_LN_STATS) && a.ln_shift) ln_c2_operands(a, g, en, e_sh, e_q);
    if (prefetch_rows) e_prefetch(0);
  };
  if (!SPLIT) epi_setup(false);   // split-K: only the tile's last split needs the operands
  float* cs = reinterpret_cast<float*>(lds);
  // DPT tail operands: w4 [4][128] then the conv bias [128] (zeros without BIAS), requested
  // now and written beside the tile after the K-loop's last LDS reads
  float4 dpt_stage = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (DPT) {
    const int gw = a.wmod > 0 ? g % a.wmod : g;
    if (tid < 128)
      dpt_stage = reinterpret_cast<const float4*>(a.dpt_w4 + (int64_t)gw * 512)[tid];
    else if (tid < 160 && (EPI & M3S_EPI_BIAS))
      dpt_stage = reinterpret_cast<const float4*>(a.bias + (int64_t)gw * a.sBias)[tid - 128];
  }
#pragma unroll
  for (int pass = 0; pass < PASSES; pass++) {
  rb = pass * EROWS;
  if (!SPLIT) {
    ln_setup();
    if (vec_path) e_prefetch(0);
  }
  block_sync_lds();
  store_acc(pass, cs);
  if constexpr (DPT) {
    if (tid < 160)
      reinterpret_cast<float4*>(lds + LDS_BYTES + 16)[tid] = dpt_stage;
  }
  block_sync_lds();
  tl_end.mark(3);

  if constexpr (DPT) {
    // fused DPT tail, all BN = 128 channels of a pixel (row) in the LDS tile: TPR threads
    // per row (every thread of the block busy: 2-4 per row) each take 32 / TPR of the
    // row's 4-channel groups — group q = (k % G) + G·h + 16·(k / G), G = 16 / TPR, so the
    // 16 lanes of one ds_read_b128 hit 16 different bank quads — against the 1x1 weights
    // and bias staged in LDS (broadcast reads), then the TPR partial sums meet by lane
    // shuffle.  (One row per thread with the weights read from global memory took 8.8 us
    // of a 27 us head.2 block in the C3 step: the block log, round 5.)
    static_assert(BN == 128 && !SPLIT && PASSES == 1,
                  "DPT_OUT needs the full 128-channel row in one tile");
    constexpr int TPR = NT >= BM ? NT / BM : 1;
    static_assert(TPR == 1 || TPR == 2 || TPR == 4 || TPR == 8, "threads per row");
    constexpr int G = 16 / (TPR > 16 ? 16 : TPR);
    const int gw = a.wmod > 0 ? g % a.wmod : g;
    const float* b4 = a.dpt_b4 + (int64_t)gw * 4;
    const float b40 = b4[0], b41 = b4[1], b42 = b4[2], b43 = b4[3];
    const float* wl = reinterpret_cast<const float*>(lds + LDS_BYTES + 16);
    const float* bl = wl + 512;
    const int h = tid % TPR;
    for (int row = tid / TPR; row < BM; row += NT / TPR) {
      const int m = m0 + row;
      float o4[4] = {0.f, 0.f, 0.f, 0.f};
      const float* src = cs + row * CST;
#pragma unroll 8
      for (int k = 0; k < 32 / TPR; k++) {
        const int c = 4 * ((k % G) + G * h + 16 * (k / G));
        float4 x = *reinterpret_cast<const float4*>(src + c);
        if constexpr ((EPI & M3S_EPI_BIAS) != 0) {
          const float4 bb = *reinterpret_cast<const float4*>(bl + c);
          x.x += bb.x;
          x.y += bb.y;
          x.z += bb.z;
          x.w += bb.w;
        }
        x.x = fmaxf(x.x, 0.f);
        x.y = fmaxf(x.y, 0.f);
        x.z = fmaxf(x.z, 0.f);
        x.w = fmaxf(x.w, 0.f);
#pragma unroll
        for (int oo = 0; oo < 4; oo++) {
          const float4 w = *reinterpret_cast<const float4*>(wl + oo * 128 + c);
          o4[oo] += w.x * x.x + w.y * x.y + w.z * x.z + w.w * x.w;
        }
      }
#pragma unroll
      for (int off = 1; off < TPR; off <<= 1)
#pragma unroll
        for (int oo = 0; oo < 4; oo++) o4[oo] += __shfl_xor(o4[oo], off, 64);
      if (h == 0 && m < a.M) {
        o4[0] += b40;
        o4[1] += b41;
        o4[2] += b42;
        o4[3] += b43;
        // reg_dense_depth('exp') + conf ('exp', conf_min): as dpt_out_kernel (vit_misc.hip)
        const float d = sqrtf(o4[0] * o4[0] + o4[1] * o4[1] + o4[2] * o4[2]);
        const float sc = expm1f(d) / fmaxf(d, 1e-8f);
        float* P = a.dpt_pts + ((int64_t)g * a.M + m) * 3;
        P[0] = o4[0] * sc;
        P[1] = o4[1] * sc;
        P[2] = o4[2] * sc;
        a.dpt_conf[(int64_t)g * a.M + m] = a.dpt_conf_min + expf(o4[3]);
      }
    }
    return true;
  }

  if constexpr (SPLIT) {
    // publish this split's partial tile; the tile's last split sums them all
    int& s_last = *reinterpret_cast<int*>(lds + LDS_BYTES);
    const int64_t per_b = (int64_t)a.M * a.N;
    float* P = a.ws + (int64_t)zz * per_b;
#pragma unroll 4
    for (int v = 0; v < NV; v++) {
      const int idx = v * NT + tid;
      const int row = idx / VPR, c = (idx % VPR) * 8;
      const int m = m0 + row, n = n0 + c;
      if (m >= a.M || n >= a.N) continue;
      const float* src = cs + row * CST + c;
      float* dst = P + (int64_t)m * a.N + n;
      if (vec) {
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
        *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(src + 4);
      } else {
        for (int t = 0; t < 8 && n + t < a.N; t++) dst[t] = src[t];
      }
    }
    if (!a.fused) return false;  // splitk_reduce_kernel follows
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      // the fence's own wait can be dropped by the compiler: wait here, before the ticket
      // (cdna_hip_programming.md Guideline 16, Pitfall 12)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int* ctr = a.cnt + (int64_t)g * nwg + wgid;
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == a.splits - 1;
      if (s_last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ln_setup();
    epi_setup(true);
    const float* P0 = a.ws + (int64_t)g * a.splits * per_b;
    // slab by slab, all of this thread's vectors of a slab in flight at once (one L2
    // round trip per slab instead of one per vector); the sum stays in split order
    float xs[NV][8];
#pragma unroll
    for (int v = 0; v < NV; v++)
#pragma unroll
      for (int t = 0; t < 8; t++) xs[v][t] = 0.f;
    for (int k = 0; k < a.splits; k++) {
      float ys[NV][8];
#pragma unroll
      for (int v = 0; v < NV; v++) {
        const int idx = v * NT + tid;
        const int row = idx / VPR, c = (idx % VPR) * 8;
        const int m = m0 + row, n = n0 + c;
        const float* src = cs + row * CST + c;
        if (k == split) {  // this workgroup's own partial is still in LDS
          *reinterpret_cast<float4*>(&ys[v][0]) = *reinterpret_cast<const float4*>(src);
          *reinterpret_cast<float4*>(&ys[v][4]) = *reinterpret_cast<const float4*>(src + 4);
        } else if (m < a.M && vec && n < a.N) {
          const float* q = P0 + k * per_b + (int64_t)m * a.N + n;
          *reinterpret_cast<float4*>(&ys[v][0]) = *reinterpret_cast<const float4*>(q);
          *reinterpret_cast<float4*>(&ys[v][4]) = *reinterpret_cast<const float4*>(q + 4);
        } else {
          const float* q = P0 + k * per_b + (int64_t)m * a.N + n;
#pragma unroll
          for (int t = 0; t < 8; t++) ys[v][t] = (m < a.M && n + t < a.N) ? q[t] : 0.f;
        }
      }
#pragma unroll
      for (int v = 0; v < NV; v++)
#pragma unroll
        for (int t = 0; t < 8; t++) xs[v][t] += ys[v][t];
    }
    block_sync_lds();  // every own-slab LDS read above is done before the overwrite
#pragma unroll
    for (int v = 0; v < NV; v++) {
      const int idx = v * NT + tid;
      const int row = idx / VPR, c = (idx % VPR) * 8;
      float* dst = cs + row * CST + c;
      *reinterpret_cast<float4*>(dst) = make_float4(xs[v][0], xs[v][1], xs[v][2], xs[v][3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(xs[v][4], xs[v][5], xs[v][6], xs[v][7]);
    }
    block_sync_lds();
  }
  if (vec_path) {
    const float sg = (en & 16) ? 1.f : -1.f;
    const bool has_res = fl & (M3S_EPI_RES_F32 | M3S_EPI_RES_BF16);
    const bool rope_now = e_rope && !has_res;
    // per group: all LDS reads first, then the math and the global stores (a ds_read issued
    // after a global store waits for that store: the compiler cannot prove it does not
    // alias the LDS-DMA ring — one such wait per group instead of one per vector)
#pragma unroll
    for (int v0 = 0; v0 < NV; v0 += EG) {
      if (v0 > 0) e_prefetch(v0);
      float xv[EG][8], pv[EG][8];
#pragma unroll
      for (int u = 0; u < EG; u++) {
        const int row = er0 + (v0 + u) * RSTEP;
        const float* src = cs + row * CST + ec;
        *reinterpret_cast<float4*>(&xv[u][0]) = *reinterpret_cast<const float4*>(src);
        *reinterpret_cast<float4*>(&xv[u][4]) = *reinterpret_cast<const float4*>(src + 4);
        if (rope_now) {
          const float* psrc = cs + row * CST + (ec ^ 16);
          *reinterpret_cast<float4*>(&pv[u][0]) = *reinterpret_cast<const float4*>(psrc);
          *reinterpret_cast<float4*>(&pv[u][4]) = *reinterpret_cast<const float4*>(psrc + 4);
        }
      }
#pragma unroll
      for (int u = 0; u < EG; u++) {
        const int m = m0 + rb + er0 + (v0 + u) * RSTEP;
        if (m >= a.M) continue;
        float* x = xv[u];
        if (fl & M3S_EPI_LN_FOLD) {  // LN(x) W^T + b = rstd (acc - mean c1) + c2
#pragma unroll
          for (int t = 0; t < 8; t++) x[t] = fmaf(e_rs[u], fmaf(-e_mu[u], e_c1[t], x[t]), e_b[t]);
          if (rope_now) {  // the partner columns' final values
#pragma unroll
            for (int t = 0; t < 8; t++)
              pv[u][t] = fmaf(e_rs[u], fmaf(-e_mu[u], e_pc1[t], pv[u][t]), e_pb[t]);
          }
        } else {
#pragma unroll
          for (int t = 0; t < 8; t++) x[t] += e_b[t];
          if (rope_now) {
#pragma unroll
            for (int t = 0; t < 8; t++) pv[u][t] += e_pb[t];
          }
        }
        if (fl & M3S_EPI_GELU) {
#pragma unroll
          for (int t = 0; t < 8; t++) x[t] = gelu_erf(x[t]);
        }
        if (rope_now) {
#pragma unroll
          for (int t = 0; t < 8; t++)
            x[t] = x[t] * e_x[u][t] + sg * pv[u][t] * e_x[u][8 + t];
        }
        if (has_res) {
#pragma unroll
          for (int t = 0; t < 8; t++) x[t] += e_x[u][t];
        }
        if (fl & M3S_EPI_RELU) {
#pragma unroll
          for (int t = 0; t < 8; t++) x[t] = fmaxf(x[t], 0.f);
        }
        int co;
        const int64_t off = out_offset(e, m, en, co);
        if (fl & M3S_EPI_OUT_F32) {
          float* cp = reinterpret_cast<float*>(e.C) + off;
          *reinterpret_cast<float4*>(cp) = make_float4(x[0], x[1], x[2], x[3]);
          *reinterpret_cast<float4*>(cp + 4) = make_float4(x[4], x[5], x[6], x[7]);
          if (fl & M3S_EPI_LN_STATS) {  // the next LayerNorm's input: A copy + row stats
            ln_store_c2(a, g, off, x, e_sh, e_q);
            ln_group_stats(a, g, m, en, x);
          }
        } else if (fl & M3S_EPI_OUT_FP8) {
          *reinterpret_cast<uint2*>(e.C + off) = make_uint2(pack4_fp8(x[0], x[1], x[2], x[3]),
                                                            pack4_fp8(x[4], x[5], x[6], x[7]));
        } else {
          bf16x8 o;
#pragma unroll
          for (int t = 0; t < 8; t++) o[t] = f2bf(x[t]);
          *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16_t*>(e.C) + off) = o;
        }
      }
    }
  } else if (!vec) {
    const bool rope = fl & M3S_EPI_ROPE;
    for (int v = 0; v < NV; v++) {
      const int idx = v * NT + tid;
      const int row = idx / VPR, c = (idx % VPR) * 8;
      const int m = m0 + rb + row, n = n0 + c;
      if (m >= a.M || n >= a.N) continue;
      const float* src = cs + row * CST + c;
      const float* psrc = cs + row * CST + (c ^ 16);
      for (int t = 0; t < 8 && n + t < a.N; t++) epi_one(e, src[t], rope ? psrc[t] : 0.f, m, n + t);
    }
  }
  }  // pass (the next pass's first barrier orders these LDS reads before its writes)
  return true;
}


// 1-D grid over (batch x split) groups x tiles.  Workgroups are dispatched to the 8 XCDs
// round-robin by linear id; the bijective remap gives each XCD a contiguous range of
// remapped ids (cdna_hip_programming.md T1), so neighbouring tiles share its L2.  Within a
// group the tile order is M-major (an XCD sweeps N for one A band: A reused) or N-major (an
// XCD sweeps the M bands of a few weight columns: B reused), whichever the host estimated
// to fetch fewer bytes, or grouped (runs of group_m M-bands swept column by column, so an
// XCD's contiguous chunk of tiles is a compact group_m x (chunk / group_m) block: fewer
// distinct A bands + B columns fetched into its L2 than one row or column of tiles).
// Split-K keeps split-major ids: an XCD's contiguous chunk then holds ONE K-slice of a run
// of tiles, whose A / B slices fit its 4 MB L2 (measured: putting a tile's slices on one
// XCD instead — same-XCD slab reads for the reducer — fetched more from beyond L2 than it
// saved, tools/gemm_split_probe.py).
__device__ __forceinline__ void block_tile(const Args& a, int& zz, int& wgid, int& tm, int& tn) {
  const int nwg = a.tiles_m * a.tiles_n;
  const int total = gridDim.x;
  const int orig = blockIdx.x;
  int wid_lin = orig;
  if (total >= 16) {
    const int q = total / 8, r = total % 8, xcd = orig % 8;
    wid_lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  zz = wid_lin / nwg;
  wgid = wid_lin - zz * nwg;
  if (a.group_m > 0) {
    const int per_group = a.group_m * a.tiles_n;
    const int grp = wgid / per_group;
    const int first_m = grp * a.group_m;
    const int gsz = min(a.tiles_m - first_m, a.group_m);
    const int in = wgid - grp * per_group;
    tm = first_m + in % gsz;
    tn = in / gsz;
  } else if (a.nmajor) {
    tn = wgid / a.tiles_m;
    tm = wgid - tn * a.tiles_m;
  } else {
    tm = wgid / a.tiles_n;
    tn = wgid - tm * a.tiles_n;
  }
}

// EPI >= 0: the epilogue flag set, fixed at compile time (straight-line epilogue code, and
// the 8-wide vector path assumed); EPI < 0: flags read at run time.
// F8: A and B hold OCP fp8 e4m3 bytes.  K / lda / ldb / strides then arrive in 2-byte units
// (host halves them), so the LDS-DMA ring, swizzle and row bytes are those of the bf16
// kernel; only the fragments differ: a 32x32x64 scaled MFMA consumes 64 bytes of a row per
// phase, lane half h holding bytes [32h, 32h + 32) (two swizzled 16-B chunks).
template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, int MODE, bool SPLIT,
          int EPI, bool F8 = false>
__global__ __launch_bounds__(WM * WN * 64, OCC) void gemm_kernel(Args a) {
  constexpr int NT = WM * WN * 64;            // 4 waves (8: two per SIMD, see T128W8)
  M3S_T(t_start);
  m3s_tl_begin(a.tl);
  M3sTlEnd tl_end{a.tl};
#ifdef M3S_GEMM_STAMPS
  const long long rt_start = (long long)__builtin_amdgcn_s_memrealtime();
#endif
  using C = Cfg<BM, BN, BK, STAGES, NT>;
  constexpr int TM = BM / WM / 32;            // 32x32 accumulators per wave (M)
  constexpr int TN = BN / WN / 32;
  static_assert(C::A_CH >= 1 && C::B_CH >= 1, "tile too small for 256 threads");
  static_assert((C::A_CH * NT) % C::CPR == 0 && 32 % (C::RPB * C::CPR) == 0, "swizzle");
  static_assert(C::L * (STAGES - 2) <= 63, "vmcnt range");
  // ALL LDS in one array (the split-K last-arriver flag included, at its end): a second
  // __shared__ object made hipcc wait vmcnt(0) before the LDS reads of every MFMA phase in
  // the SPLIT instantiations — the DMA ring drained 4x per K-tile (cdna_hip_programming.md
  // §5 'Projection GEMM at M = 256' item 4(a)); measured as split-K K-tiles 2.4x slower
  // (+ the DPT tail's 1x1 weights and conv bias, staged once per block: DPT_OUT below)
  constexpr bool DPT = EPI >= 0 && (EPI & M3S_EPI_DPT_OUT) != 0;
  __shared__ __attribute__((aligned(16))) char lds[C::LDS_BYTES + 16 + (DPT ? 640 * 4 : 0)];

  // tile of this workgroup (block_tile: XCD-aware order)
  const int nwg = a.tiles_m * a.tiles_n;
  int zz, wgid, tm, tn;
  block_tile(a, zz, wgid, tm, tn);
  const int g = SPLIT ? zz / a.splits : zz;
  const int split = SPLIT ? zz - g * a.splits : 0;
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.A + (int64_t)(g ^ a.a_xor) * a.sA), (short)0, NUM_RECORDS, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.B + (int64_t)(a.wmod > 0 ? g % a.wmod : g) * a.sB), (short)0,
      NUM_RECORDS, 0x00020000);

  // per-thread DMA chunks: chunk q = i*NT + tid lands at LDS row q / CPR, slot q % CPR and
  // carries logical K-chunk slot ^ swz(row)
  uint32_t a_off[C::A_CH];
  int a_kc[C::A_CH], a_iy[C::A_CH], a_ix[C::A_CH];
#pragma unroll
  for (int i = 0; i < C::A_CH; i++) {
    const int q = i * NT + tid;
    const int r = q / C::CPR, p = q % C::CPR;
    const int kc = (p ^ ((r / C::RPB) % C::CPR)) * 8;
    const int m = m0 + r;
    a_kc[i] = kc;
    if (MODE == 0) {
      a_off[i] = m < a.M ? (uint32_t)(((int64_t)m * a.lda + kc) * 2) : OOB;
      a_iy[i] = a_ix[i] = 0;
    } else {
      const int oy = m / a.Wout, ox = m - oy * a.Wout;
      a_iy[i] = m < a.M ? oy * a.stride - 1 : -(1 << 20);  // OOB rows never pass the bounds test
      a_ix[i] = ox * a.stride - 1;
      a_off[i] = 0;
    }
  }
  uint32_t b_off[C::B_CH];
  int b_kc[C::B_CH];
#pragma unroll
  for (int i = 0; i < C::B_CH; i++) {
    const int q = i * NT + tid;
    const int r = q / C::CPR, p = q % C::CPR;
    const int kc = (p ^ ((r / C::RPB) % C::CPR)) * 8;
    const int n = n0 + r;
    b_kc[i] = kc;
    b_off[i] = n < a.N ? (uint32_t)(((int64_t)n * a.ldb + kc) * 2) : OOB;
  }

  // One DMA chunk j (< A_CH: A, else B) of K-tile k0 into stage buffer sb.  The conv tap
  // (ky, kx) / channel offset ci0 are block-uniform per K-tile.
  auto issue_chunk = [&](int j, int k0, char* sb, int ky, int kx, int ci0) {
    if (j < C::A_CH) {
      uint32_t vo;
      if (MODE == 0) {
        vo = (k0 + a_kc[j] < a.K) ? a_off[j] + (uint32_t)k0 * 2 : OOB;
      } else {
        const int iy = a_iy[j] + ky, ix = a_ix[j] + kx;
        const bool ok = (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        vo = ok ? (uint32_t)((((int64_t)iy * a.Win + ix) * a.Cin + ci0 + a_kc[j]) * 2) : OOB;
      }
      glds16(rA, sb + (j * NT + wid * 64) * 16, vo);
    } else {
      const int i = j - C::A_CH;
      const uint32_t vo = (k0 + b_kc[i] < a.K) ? b_off[i] + (uint32_t)k0 * 2 : OOB;
      glds16(rB, sb + C::A_BYTES + (i * NT + wid * 64) * 16, vo);
    }
  };
  auto tap_of = [&](int k0, int& ky, int& kx, int& ci0) {
    ky = kx = ci0 = 0;
    if (MODE != 0) {
      const int tap = k0 / a.Cin;  // Cin % BK == 0
      ci0 = k0 - tap * a.Cin;
      ky = tap / 3;
      kx = tap - ky * 3;
    }
  };
  auto issue = [&](int ktile, int stage) {
    const int k0 = ktile * BK;
    int ky, kx, ci0;
    tap_of(k0, ky, kx, ci0);
#pragma unroll
    for (int j = 0; j < C::L; j++) issue_chunk(j, k0, lds + stage * C::ST_BYTES, ky, kx, ci0);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  const int fr = lane & 31;
  const int fh = lane >> 5;
  const int fsw = (fr / C::RPB) % C::CPR;     // row swizzle of this lane's fragment rows
  int nk = (a.K + BK - 1) / BK;
  int kbase = 0;
  if (SPLIT) {
    const int per = (nk + a.splits - 1) / a.splits;
    kbase = split * per;
    nk = min(per, nk - kbase);
    if (nk < 0) nk = 0;
  }

#pragma unroll
  for (int s = 0; s < STAGES - 1; s++)
    if (s < nk) issue(kbase + s, s);
  M3S_T(t_pro);
  tl_end.mark(0);
#ifdef M3S_GEMM_STAMPS
  long long s_wait = 0, s_bar = 0, s_comp = 0;
#endif

  // K loop.  Fragments are double-buffered in registers: a phase (16 of the K-tile's BK)
  // issues the LDS reads of the NEXT phase, its share of the DMA of tile kt+STAGES-1, then
  // its MFMAs; the last phase issues its MFMAs first, then retires tile kt+1 (counted
  // vmcnt + barrier: the MFMAs keep the matrix pipe busy meanwhile) and reads tile kt+1's
  // first fragments.  The steady-state loop (every tile prefetches) is branch-free, so the
  // scheduler sees whole phases; sched_group_barrier pins the read / DMA / MFMA order.
  constexpr int KK = F8 ? BK / 32 : BK / 16;  // MFMA phases per K-tile
  constexpr int NR = (TM + TN) * (F8 ? 2 : 1); // ds_read_b128 per phase
  constexpr int NM = TM * TN;                 // MFMAs per phase
  using frag_t = std::conditional_t<F8, i32x8, bf16x8>;
  frag_t fa[2][TM], fb[2][TN];
  auto read_frags = [&](int buf, const char* sA, int kk) {
    const char* sB = sA + C::A_BYTES;
    if constexpr (F8) {
      const int s0 = ((kk * 4 + 2 * fh) ^ fsw) * 16, s1 = ((kk * 4 + 2 * fh + 1) ^ fsw) * 16;
#pragma unroll
      for (int i = 0; i < TM; i++) {
        const char* row = sA + (wm * (BM / WM) + i * 32 + fr) * (BK * 2);
        const int4 lo = *reinterpret_cast<const int4*>(row + s0);
        const int4 hi = *reinterpret_cast<const int4*>(row + s1);
        fa[buf][i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
#pragma unroll
      for (int j = 0; j < TN; j++) {
        const char* row = sB + (wn * (BN / WN) + j * 32 + fr) * (BK * 2);
        const int4 lo = *reinterpret_cast<const int4*>(row + s0);
        const int4 hi = *reinterpret_cast<const int4*>(row + s1);
        fb[buf][j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      }
    } else {
      const int slot = ((kk * 2 + fh) ^ fsw) * 16;
#pragma unroll
      for (int i = 0; i < TM; i++) {
        fa[buf][i] = *reinterpret_cast<const bf16x8*>(
            sA + (wm * (BM / WM) + i * 32 + fr) * (BK * 2) + slot);
        if (MODE == 2) fa[buf][i] = relu_frag(fa[buf][i]);
      }
#pragma unroll
      for (int j = 0; j < TN; j++)
        fb[buf][j] = *reinterpret_cast<const bf16x8*>(
            sB + (wn * (BN / WN) + j * 32 + fr) * (BK * 2) + slot);
    }
  };
  auto mfmas = [&](int cur) {
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
      for (int j = 0; j < TN; j++) {
        if constexpr (F8)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
              fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0, 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][i], fb[cur][j], acc[i][j],
                                                              0, 0, 0);
      }
  };
  auto stage_of = [&](int t) { return lds + (t % STAGES) * C::ST_BYTES; };
  // retire the oldest DMA tile, leaving `ahead` (≤ STAGES - 2) younger tiles in flight
  auto wait_ahead = [&](int ahead) {
    if (STAGES >= 6 && ahead >= 4) vm_wait<C::L * (STAGES >= 6 ? 4 : 0)>();
    else if (STAGES >= 5 && ahead >= 3) vm_wait<C::L * (STAGES >= 5 ? 3 : 0)>();
    else if (STAGES >= 4 && ahead >= 2) vm_wait<C::L * 2>();
    else if (ahead >= 1) vm_wait<C::L>();
    else vm_wait<0>();
  };
  if (nk > 0) {
    wait_ahead(min(nk - 1, STAGES - 2));
    block_sync_lds();
    read_frags(0, lds, 0);
  }
  M3S_T(t_first);
  tl_end.mark(1);

  const int nsteady = nk - (STAGES - 1);      // kt < nsteady: tile kt+STAGES-1 exists
  int kt = 0;
  for (; kt < nsteady; kt++) {
    M3S_T(t0);
    M3S_T(t1);
    M3S_T(t2);
    const int pk0 = (kbase + kt + STAGES - 1) * BK;
    char* psb = lds + ((kt + STAGES - 1) % STAGES) * C::ST_BYTES;
    int pky, pkx, pci0;
    tap_of(pk0, pky, pkx, pci0);
    const char* sA = stage_of(kt);
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
      const int cur = kk & 1;
      if (kk + 1 < KK) {
        read_frags(cur ^ 1, sA, kk + 1);
#pragma unroll
        for (int j = 0; j < C::L; j++)
          if (j * KK / C::L == kk) issue_chunk(j, pk0, psb, pky, pkx, pci0);
        mfmas(cur);
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
      } else {
#pragma unroll
        for (int j = 0; j < C::L; j++)
          if (j * KK / C::L == kk) issue_chunk(j, pk0, psb, pky, pkx, pci0);
        mfmas(cur);
        __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        // retire tile kt+1: tiles kt+2 .. kt+STAGES-1 (STAGES-2 of them) stay in flight
        vm_wait<C::L * (STAGES - 2)>();
        block_sync_lds();
        read_frags(cur ^ 1, stage_of(kt + 1), 0);
      }
    }
#ifdef M3S_GEMM_STAMPS
    M3S_T(t3);
    s_wait += t1 - t0;
    s_bar += t2 - t1;
    s_comp += t3 - t2;
#endif
  }
  M3S_T(t_steady);
  // tail: the last STAGES-1 tiles (nothing left to prefetch)
  for (; kt < nk; kt++) {
    const char* sA = stage_of(kt);
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
      const int cur = kk & 1;
      if (kk + 1 < KK) {
        read_frags(cur ^ 1, sA, kk + 1);
        mfmas(cur);
      } else {
        mfmas(cur);
        if (kt + 1 < nk) {
          wait_ahead(min(nk - 2 - kt, STAGES - 2));
          block_sync_lds();
          read_frags(cur ^ 1, stage_of(kt + 1), 0);
        }
      }
    }
  }
  M3S_T(t_loop);
  tl_end.mark(2);
  if constexpr (F8) {  // dequant: acc(i, j) *= col_scale[n] (n = this lane's column)
    const int64_t gw = a.wmod > 0 ? g % a.wmod : g;
    const float* cs_g = a.cscale + gw * a.sCscale;
    // LN_FOLD consumer of a shifted e4m3 copy: + c3[n] = Σ_k shift[k] B[n][k] restores
    // Σ_k x[k] B[n][k] before the epilogue's rstd (acc − mean c1) + c2
    // (split-K: the first split's partial carries it, so the sum adds it once)
    const float* c3_g = (a.ln_c3 && split == 0) ? a.ln_c3 + gw * a.sBias : nullptr;
#pragma unroll
    for (int j = 0; j < TN; j++) {
      const int n = n0 + wn * (BN / WN) + j * 32 + fr;
      const float sc = n < a.N ? cs_g[n] : 0.f;
      if (c3_g) {
        const float c3 = n < a.N ? c3_g[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
          for (int r = 0; r < 16; r++) acc[i][j][r] = fmaf(acc[i][j][r], sc, c3);
      } else {
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
          for (int r = 0; r < 16; r++) acc[i][j][r] *= sc;
      }
    }
  }

  // ---- epilogue through LDS: f32 tile [EROWS][CST] per pass (gemm_epilogue) ----
  const bool stored = gemm_epilogue<BM, BN, NT, C::PASSES, C::LDS_BYTES, SPLIT, EPI>(
      a, lds, g, zz, nwg, wgid, split, m0, n0, tl_end, [&](int pass, float* cs) {
        const int rb = pass * C::EROWS;
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
          for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
              const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh - rb;
              if (C::PASSES == 1 || wm == pass)
                cs[row * C::CST + wn * (BN / WN) + j * 32 + fr] = acc[i][j][r];
            }
      });
  if (stored) {
    M3S_STAMP_OUT();
  } else {
    M3S_STAMP_EARLY();
  }
}

// Unfused split-K: sum the partials (fixed order) and apply the epilogue; 8 columns per
// thread, the whole chip reducing (the fused path reduces a tile on one CU).
template <int Unused>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(Args a) {
  const M3sTlEnd tl_end{a.tl};   // the GEMM's slot: the reduce extends its end
  const int vpr = (a.N + 7) / 8;
  const int64_t vid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y;
  if (vid >= (int64_t)a.M * vpr) return;
  const int m = (int)(vid / vpr);
  const int n = (int)(vid - (int64_t)m * vpr) * 8;
  const int64_t per_b = (int64_t)a.M * a.N;
  const Epi e = make_epi(a, g);
  const float* P = a.ws + (int64_t)g * a.splits * per_b + (int64_t)m * a.N;
  const bool rope = (a.flags & M3S_EPI_ROPE) && n < a.rope_cols;
  float x[8], p[8];
  if (a.vec) {
#pragma unroll
    for (int t = 0; t < 8; t++) x[t] = p[t] = 0.f;
    for (int k = 0; k < a.splits; k++) {
      const float* q = P + k * per_b;
      const float4 u0 = *reinterpret_cast<const float4*>(q + n);
      const float4 u1 = *reinterpret_cast<const float4*>(q + n + 4);
      x[0] += u0.x; x[1] += u0.y; x[2] += u0.z; x[3] += u0.w;
      x[4] += u1.x; x[5] += u1.y; x[6] += u1.z; x[7] += u1.w;
      if (rope) {
        const float4 w0 = *reinterpret_cast<const float4*>(q + (n ^ 16));
        const float4 w1 = *reinterpret_cast<const float4*>(q + (n ^ 16) + 4);
        p[0] += w0.x; p[1] += w0.y; p[2] += w0.z; p[3] += w0.w;
        p[4] += w1.x; p[5] += w1.y; p[6] += w1.z; p[7] += w1.w;
      }
    }
    epi_vec8(e, x, p, m, n);  // x now holds the stored values
    if (a.flags & M3S_EPI_LN_STATS) {
      float sh[8], q = 0.f;
      if (a.ln_shift) ln_c2_operands(a, g, n, sh, q);
      ln_store_c2(a, g, (int64_t)m * a.ldc + n, x, sh, q);
      ln_group_stats(a, g, m, n, x);
    }
  } else {
    for (int t = 0; t < 8 && n + t < a.N; t++) {
      float s = 0.f, ps = 0.f;
      for (int k = 0; k < a.splits; k++) {
        s += P[k * per_b + n + t];
        if (rope) ps += P[k * per_b + ((n + t) ^ 16)];
      }
      epi_one(e, s, ps, m, n + t);
    }
  }
}

// Tile order of a launch (block_tile): the operand bytes an XCD's L2 must fetch for its
// contiguous chunk of T tiles — M-major touches ceil(T / tiles_n) A bands and min(T,
// tiles_n) B columns, N-major ceil(T / tiles_m) B columns and min(T, tiles_m) A bands, a
// grouped order G bands x ceil(T / G) columns; the cheapest line order, or the grouped one
// if ≥ 10 % below it.  Implicit convs keep M-major.
inline void set_order(Args& a, int BM, int BN, int64_t groups) {
  a.nmajor = 0;
  a.group_m = 0;
  if (a.mode != 0) return;
  const int64_t T = ((int64_t)a.tiles_m * a.tiles_n * groups + 7) / 8;
  const double band = (double)BM * a.K * 2, col = (double)BN * a.K * 2;
  const double costM = band * std::min<int64_t>(a.tiles_m, (T + a.tiles_n - 1) / a.tiles_n + 1) +
                       col * std::min<int64_t>(T, a.tiles_n);
  const double costN = col * std::min<int64_t>(a.tiles_n, (T + a.tiles_m - 1) / a.tiles_m + 1) +
                       band * std::min<int64_t>(T, a.tiles_m);
  a.nmajor = costN < costM;
  double best = std::min(costM, costN);
  for (int G = 2; G < a.tiles_m && G <= 16; G++) {
    if (T > (int64_t)G * a.tiles_n) break;
    const double c = band * G + col * (double)((T + G - 1) / G);
    if (c < 0.9 * best) {
      best = c;
      a.group_m = G;
    }
  }
  if (const char* e = getenv("M3S_GEMM_ORDER")) {  // tuning override: 0 / 1 / -G
    const int v = atoi(e);
    a.nmajor = v == 1;
    a.group_m = v < 0 ? -v : 0;
  }
}

// ---------------------------------------------------------------------------------------
// T256PP: 256x256 tiles, 8 waves in two ping-pong groups (round 6)
// ---------------------------------------------------------------------------------------
// cdna_hip_programming.md §5's 256² 8-phase structure, derived for this library's operand
// layout (tools/gemm_pp_dev.hip is the isolated main loop; 4096³: 1.51 PF/s vs 1.36 for
// hipBLASLt on the same box, profiles/r06_gemm_pp_dev.txt):
//  * LDS: 2 K-tile buffers x 4 half-tile slots {A rows 0-127, A rows 128-255, B cols 0-127,
//    B cols 128-255} of 128 x 64 bf16 (16 KB), filled by LDS-DMA with the chunk swizzle of
//    gemm_kernel (chunk ^ ((row >> 1) & 7)).
//  * A K-tile is 4 phases; phase p computes block quadrant (QM, QN) = (0,0), (0,1), (1,1),
//    (1,0) over K = 64: each wave its 64 x 32 share (16 v_mfma_f32_16x16x32_bf16 — the
//    16x16 shape holds a higher clock than 32x32x16 under load, MI355X_MICROARCH.md 'DVFS
//    give-back' 7).  Fragments are read only where the quadrant changes them (A0+B0, B1,
//    A1, B0: 28 ds_read_b128 per wave per K-tile) into one register set.
//  * Phase p also issues half-tile p of K-tile t+1 (A0, B0, B1, A1) into the other buffer
//    and waits vmcnt(4) (the half-tile issued two phases earlier is retired).  Phases are
//    [reads, DMA, wait] barrier [16 MFMAs] barrier; waves 4-7 run one barrier behind waves
//    0-3, so on each SIMD one wave's MFMA segment runs beside its partner's read / DMA
//    segment, and the younger group holds s_setprio 1 (§5.5 T5 static form).
//  * Ordering (phase index P = 4t + p; group 0 reads phase P before global barrier 2P, group
//    1 before 2P + 1): a half-tile issued at phase I may be read at phase Q ≥ I + 3 (both
//    groups' covering waits precede a barrier the reader has passed) and a slot read last
//    at phase Q may be refilled at I ≥ Q + 2 (every read of phase Q has completed before
//    barrier 2Q + 2).  The order above meets both with one slack phase: (t+1, A0) issued
//    at 4t reads 4t+4, last read of (t-1, A0) 4t-4; B0 4t+1 / 4t+4, 4t-1; B1 4t+2 / 4t+5,
//    4t-3; A1 4t+3 / 4t+6, 4t-2.
//  * The last K-tile issues nothing (its phases wait vmcnt(2), then 0).
// Implicit conv (MODE 1 / 2) as gemm_kernel: the tap and channel offset are block-uniform
// per K-tile (Cin % 64 == 0), ReLU (MODE 2) on the A fragments.  Unsplit; the epilogue is
// gemm_epilogue's, in two 128-row passes (QM = 0, then 1).
// BM = 192 (T192PP, round 6): the same schedule on 192 x 256 tiles — A half-tiles of 96
// rows (each wave group's share 48 rows = 3 MFMA row tiles); a half-tile still takes two
// 16-B DMA chunks per thread (the vmcnt counts assume it): the 256 chunks past row 96 go
// to a 4-KB junk area with out-of-range offsets (zeros, no memory read).  For grids that a
// 256-row tile leaves on a partial wave (M = 768: 4 row tiles instead of 3).
template <int MODE, int EPI, int BM = 256>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(Args a) {
  static_assert(BM == 256 || BM == 192, "T256PP / T192PP");
  constexpr int BN = 256, BK = 64, NT = 512;
  constexpr int HA = BM / 2;             // A half-tile rows
  constexpr int FA = HA / 32;            // 16-row MFMA tiles per wave group per half
  constexpr int HBA = HA * BK * 2;       // A half-tile bytes
  constexpr int HB = 128 * BK * 2;       // B half-tile bytes
  constexpr int SOFF[4] = {0, HBA, 2 * HBA, 2 * HBA + HB};   // slots A0 A1 B0 B1
  constexpr int BUFB = 2 * HBA + 2 * HB; // one K-tile
  constexpr int RING = 2 * BUFB;
  constexpr int JUNK = HA == 128 ? 0 : 4 * 1024;
  constexpr int EPIB = HA * (BN + 4) * 4;
  constexpr int LDS_BYTES = EPIB > RING + JUNK ? EPIB : RING + JUNK;
  static_assert(EPI < 0 || (EPI & (M3S_EPI_DPT_OUT | M3S_EPI_OUT_FP8)) == 0, "not on T256PP");
  m3s_tl_begin(a.tl);
  M3sTlEnd tl_end{a.tl};
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES + 16];
  const int nwg = a.tiles_m * a.tiles_n;
  int zz, wgid, tm, tn;
  block_tile(a, zz, wgid, tm, tn);
  const int g = zz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;   // ping-pong group, column of the quadrant

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.A + (int64_t)(g ^ a.a_xor) * a.sA), (short)0, NUM_RECORDS, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.B + (int64_t)(a.wmod > 0 ? g % a.wmod : g) * a.sB), (short)0,
      NUM_RECORDS, 0x00020000);

  // DMA: a half-tile is 128 rows x 8 chunks of 16 B; thread chunk q = i*512 + tid lands at
  // row q >> 3, slot q & 7 and carries logical chunk slot ^ ((row >> 1) & 7).  off[h][i]:
  // byte offset of row (h & 1)·128 + (q >> 3) of slot h (A0 A1 B0 B1) at k = 0 (GEMM rows;
  // conv rows keep their input pixel instead)
  uint32_t off[4][2];
  int kc[2], a_iy[2][2], a_ix[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int q = i * NT + tid;
    const int r = q >> 3, p = q & 7;
    kc[i] = (p ^ ((r >> 1) & 7)) * 8;
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const int row = (h & 1) * (h < 2 ? HA : 128) + r;
      if (h < 2) {
        const int m = r < HA ? m0 + row : a.M;   // chunks past the A half-tile: junk
        if (MODE == 0) {
          off[h][i] = m < a.M ? (uint32_t)(((int64_t)m * a.lda + kc[i]) * 2) : OOB;
        } else {
          const int oy = m / a.Wout, ox = m - oy * a.Wout;
          a_iy[h][i] = m < a.M ? oy * a.stride - 1 : -(1 << 20);
          a_ix[h][i] = ox * a.stride - 1;
          off[h][i] = 0;
        }
      } else {
        const int n = n0 + row;
        off[h][i] = n < a.N ? (uint32_t)(((int64_t)n * a.ldb + kc[i]) * 2) : OOB;
      }
    }
  }
  const int nk = (a.K + BK - 1) / BK;
  // half-tile h of K-tile t into its slot of buffer t & 1
  auto issue = [&](int t, int h) {
    char* dst = lds + (t & 1) * BUFB + SOFF[h] + wid * 64 * 16;
    const int k0 = t * BK;
    int ky = 0, kx = 0, ci0 = 0;
    if (MODE != 0 && h < 2) {
      const int tap = k0 / a.Cin;
      ci0 = k0 - tap * a.Cin;
      ky = tap / 3;
      kx = tap - ky * 3;
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
      uint32_t vo;
      if (MODE != 0 && h < 2) {
        const int iy = a_iy[h][i] + ky, ix = a_ix[h][i] + kx;
        const bool ok = (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
        vo = ok ? (uint32_t)((((int64_t)iy * a.Win + ix) * a.Cin + ci0 + kc[i]) * 2) : OOB;
      } else {
        vo = (k0 + kc[i] < a.K) ? off[h][i] + (uint32_t)k0 * 2 : OOB;
      }
      // (T192PP: waves 4-7's second A chunk lands in the junk area, out of range)
      char* d = (JUNK && h < 2 && i == 1 && wid >= 4) ? lds + RING + (wid - 4) * 64 * 16
                                                      : dst + i * NT * 16;
      if (JUNK && h < 2 && i == 1 && wid >= 4) vo = OOB;
      glds16(h < 2 ? rA : rB, d, vo);
    }
  };

  // fragments: lane reads row (lane & 15) of a 16-row tile, chunk 4s + (lane >> 4),
  // swizzled by ((row >> 1) & 7) = (lane & 15) >> 1 (tile bases are multiples of 16 rows)
  const int fr = lane & 15, fc = lane >> 4, sw = fr >> 1;
  const int lo0 = fr * 128 + ((fc ^ sw) << 4);
  const int lo1 = fr * 128 + (((fc ^ sw) ^ 4) << 4);
  bf16x8 af[FA][2], bfr[2][2];
  f32x4 acc[2][2][FA][2];
#pragma unroll
  for (int x = 0; x < 2; x++)
#pragma unroll
    for (int y = 0; y < 2; y++)
#pragma unroll
      for (int i = 0; i < FA; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto read_a = [&](const char* slot) {
    const char* base = slot + wr * (HA / 2) * 128;
#pragma unroll
    for (int i = 0; i < FA; i++) {
      af[i][0] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + lo0);
      af[i][1] = *reinterpret_cast<const bf16x8*>(base + i * 16 * 128 + lo1);
      if (MODE == 2) {
        af[i][0] = relu_frag(af[i][0]);
        af[i][1] = relu_frag(af[i][1]);
      }
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
  auto mfmas = [&](f32x4 (&c)[FA][2]) {
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int i = 0; i < FA; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bfr[j][s], c[i][j], 0, 0, 0);
  };
  auto bar = []() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: K-tile 0 into buffer 0; A0 and B0 retired before the first reads
  if (nk > 0) {
    issue(0, 0);
    issue(0, 2);
    issue(0, 3);
    issue(0, 1);
  }
  tl_end.mark(0);
  vm_wait<4>();
  bar();
  if (wr == 1) {
    bar();                          // the stagger
    __builtin_amdgcn_s_setprio(1);  // the younger group wins VALU / LDS arbitration
  }
  tl_end.mark(1);
#define M3S_PP_PHASE(READS, ISSUE, WAIT, QM, QN) \
  READS;                                         \
  ISSUE;                                         \
  vm_wait<WAIT>();                               \
  bar();                                         \
  mfmas(acc[QM][QN]);                            \
  bar();
  int t = 0;
  for (; t < nk - 1; t++) {
    const char* cur = lds + (t & 1) * BUFB;
    M3S_PP_PHASE((read_a(cur), read_b(cur + SOFF[2])), issue(t + 1, 0), 4, 0, 0)
    M3S_PP_PHASE(read_b(cur + SOFF[3]), issue(t + 1, 2), 4, 0, 1)
    M3S_PP_PHASE(read_a(cur + SOFF[1]), issue(t + 1, 3), 4, 1, 1)
    M3S_PP_PHASE(read_b(cur + SOFF[2]), issue(t + 1, 1), 4, 1, 0)
  }
  if (nk > 0) {   // the last K-tile: nothing to issue (phase 0 retires B1, phase 1 A1)
    const char* cur = lds + (t & 1) * BUFB;
    M3S_PP_PHASE((read_a(cur), read_b(cur + SOFF[2])), (void)0, 2, 0, 0)
    M3S_PP_PHASE(read_b(cur + SOFF[3]), (void)0, 0, 0, 1)
    M3S_PP_PHASE(read_a(cur + SOFF[1]), (void)0, 0, 1, 1)
    M3S_PP_PHASE(read_b(cur + SOFF[2]), (void)0, 0, 1, 0)
  }
#undef M3S_PP_PHASE
  if (wr == 1) __builtin_amdgcn_s_setprio(0);
  else bar();                       // re-align the groups
  vm_wait<0>();
  tl_end.mark(2);
  (void)gemm_epilogue<BM, BN, NT, 2, LDS_BYTES, false, EPI>(
      a, lds, g, zz, nwg, wgid, 0, m0, n0, tl_end, [&](int pass, float* cs) {
#pragma unroll
        for (int qn = 0; qn < 2; qn++)
#pragma unroll
          for (int i = 0; i < FA; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
#pragma unroll
              for (int r = 0; r < 4; r++) {
                const int row = wr * (HA / 2) + i * 16 + fc * 4 + r;
                const int col = qn * 128 + wc * 32 + j * 16 + fr;
                cs[row * (BN + 4) + col] = pass == 0 ? acc[0][qn][i][j][r] : acc[1][qn][i][j][r];
              }
      });
}

template <int MODE, int E, int BM>
bool try_epi_pp(Args& a, dim3 grid, hipStream_t s, int key, bool biased_only = false) {
  if (key == E && !biased_only) {
    hipLaunchKernelGGL((gemm_pp_kernel<MODE, E, BM>), grid, dim3(512), 0, s, a);
    return true;
  }
  if (key == (E | M3S_EPI_BIAS)) {
    hipLaunchKernelGGL((gemm_pp_kernel<MODE, E | M3S_EPI_BIAS, BM>), grid, dim3(512), 0, s, a);
    return true;
  }
  return false;
}

// T256PP launcher (unsplit): the epilogue sets of launch_main as straight-line variants,
// the run-time-flag epilogue otherwise
template <int MODE, int BM = 256>
int launch_pp(Args& a, int batch, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + 255) / 256;
  if ((int64_t)a.tiles_m * a.tiles_n * batch >= (1ll << 31)) return M3S_ERR_TOO_LARGE;
  const dim3 grid((unsigned)(a.tiles_m * a.tiles_n * batch));
  a.splits = 1;
  set_order(a, BM, 256, batch);
  // large grids (both tile dimensions >= 8, GEMM mode): the 32 tiles an XCD runs at once as
  // 4 A bands x 8 B columns instead of one band x 32 columns — set_order's whole-panel
  // model stops grouping once an XCD's share exceeds a group, but at one 256^2 block per CU
  // what the L2 holds is the concurrent tiles' current K-slices (8192^3: 1271 -> 1486
  // TF/s, profiles/r06_pp_bench_order.txt)
  if (a.mode == 0 && a.group_m == 0 && a.tiles_m >= 8 && a.tiles_n >= 8 &&
      !getenv("M3S_GEMM_ORDER"))
    a.group_m = 4;
  const int key = (a.flags & ~(M3S_PRO_RELU | (a.bias ? 0 : M3S_EPI_BIAS)));
  bool done = false;
  if (a.vec) {
    if constexpr (MODE == 0) {
      constexpr int LF = M3S_EPI_LN_FOLD, LS = M3S_EPI_LN_STATS;
      done = try_epi_pp<0, 0, BM>(a, grid, s, key) ||
             try_epi_pp<0, M3S_EPI_ROPE, BM>(a, grid, s, key) ||
             try_epi_pp<0, M3S_EPI_GELU, BM>(a, grid, s, key) ||
             try_epi_pp<0, M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, BM>(a, grid, s, key) ||
             try_epi_pp<0, M3S_EPI_OUT_F32, BM>(a, grid, s, key) ||
             try_epi_pp<0, LF | M3S_EPI_ROPE, BM>(a, grid, s, key, true) ||
             try_epi_pp<0, LF | M3S_EPI_GELU, BM>(a, grid, s, key, true) ||
             try_epi_pp<0, LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, BM>(a, grid, s, key, true) ||
             try_epi_pp<0, LS | M3S_EPI_OUT_F32, BM>(a, grid, s, key, true);
    } else {
      done = try_epi_pp<MODE, 0, BM>(a, grid, s, key) ||
             try_epi_pp<MODE, M3S_EPI_RES_BF16, BM>(a, grid, s, key) ||
             try_epi_pp<MODE, M3S_EPI_RELU, BM>(a, grid, s, key);
    }
  }
  if (!done) hipLaunchKernelGGL((gemm_pp_kernel<MODE, -1, BM>), grid, dim3(512), 0, s, a);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

// ---------------------------------------------------------------------------------------
// tile configurations
// ---------------------------------------------------------------------------------------
// (4- and 5-stage 128x128 / 6-stage 64x128 rings were measured on the M = 768 shapes at
// ±3 % of these — tools/gemm_depth.py — and dropped: the first-tile latency, not the ring
// depth, bounds those blocks)
// T64D / T128D: deep DMA rings (6 / 4 stages, one block per CU) for grids that leave most
// CUs with a single block: a lone block's bytes in flight (stages ahead x stage bytes) over
// the fetch latency bound its operand rate (Little's law), and so the skinny M = 768 shapes
// T128W8: 128x128 with 8 waves (two per SIMD, each 32x64): one wave's LDS-DMA issue
// (≈60-185 cycles per 1-KB piece, MI355X_MICROARCH.md) overlaps the other's MFMAs, where
// the 4-wave block leaves the matrix pipe idle during its own issue
// T256W8: 256x128 with 8 waves (4 x 2, each 64x64): per CU the LDS-DMA path moves
// (BM + BN)·BK·2 bytes per K-tile at ≈64 B/clk against 2·BM·BN·BK MFMA FLOPs at ≈4k
// FLOP/clk, i.e. fetch / MFMA cycles ≈ 64·(BM + BN) / (BM·BN): 1.5 for 64x128, 1.0 for
// 128², 0.75 here — the first tile whose K-loop the matrix pipe can pace.  For the M = 768
// batched decoder GEMMs it trades 2x fewer blocks for that; T256 is the 4-wave form.
// T256SQ: 256x256 with 8 waves (2 x 4, each 128x64), a 2-stage ring of 64 KB K-tiles and
// the epilogue in two 128-row passes (the f32 tile would need 266 KB of LDS): fetch / MFMA
// cycles ≈ 0.5, the shape of cdna_hip_programming.md §5's 256² template — the most MFMA
// work per staged byte, for launches that can spend fewer CUs (large-M convs, the local-
// feature MLP, GEMMs sharing the chip with other chains)
// T256PP: 256x256, the 8-wave ping-pong kernel above (round 6); T192PP: its 192x256 form
enum TileCfg { T128 = 1, T64 = 2, T128K32 = 3, T256 = 6, T128O2 = 7, T96 = 8, T96O2 = 9,
               T64D = 10, T128D = 11, T128W8 = 12, T256W8 = 13, T256SQ = 14, T256PP = 15,
               T192PP = 16 };

// Epilogue flag sets compiled as straight-line variants (8-wide vector path), per mode:
//   GEMM: bf16 out, +RoPE, +GELU, f32 residual → f32, f32 out;  conv: bf16 out, +bf16
//   residual, +ReLU.  Any other combination (or an unaligned shape) runs the generic
//   run-time-flag epilogue.  Each set exists with and without bias.
template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, int MODE, int E,
          bool F8 = false, bool SP = false>
bool try_epi(Args& a, dim3 grid, hipStream_t s, int key) {
  if (key == E) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, MODE, SP, E, F8>), grid,
                       dim3(WM * WN * 64), 0, s, a);
    return true;
  }
  if (key == (E | M3S_EPI_BIAS)) {
    hipLaunchKernelGGL(
        (gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, MODE, SP, E | M3S_EPI_BIAS, F8>), grid,
        dim3(WM * WN * 64), 0, s, a);
    return true;
  }
  return false;
}

// the same, biased set only (the LayerNorm-fold sets always carry a bias)
template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, int MODE, int E,
          bool SP = false>
bool try_epi_b(Args& a, dim3 grid, hipStream_t s, int key) {
  if (key != (E | M3S_EPI_BIAS)) return false;
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, MODE, SP, E | M3S_EPI_BIAS>),
                     grid, dim3(WM * WN * 64), 0, s, a);
  return true;
}

// fp8 operands.  GEMM mode: the epilogue sets the ViT uses — qkv / q / kv (+RoPE), fc1
// (+GELU, fp8 out for the next fp8 GEMM), proj / fc2 (f32 residual), plain bf16 / f32.
// Implicit conv (MODE 1, C5's full-resolution DPT head convs, round 5): bf16 out (head.0)
// and ReLU + the fused DPT tail (head.2).  The A operand is e4m3 NHWC and Cin arrives in
// 2-byte units like K, so the tap / channel addressing is the bf16 kernel's unchanged.
// SP: split-K (round 6: the residual GEMMs of the fp8 frame — N = 768 / 1024 at 1,024
// tokens fill a quarter to half of the chip; partials are dequantised before the sum)
template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, int MODE, bool SP = false>
void launch_main_f8(Args& a, dim3 grid, hipStream_t s) {
  const int key = a.flags & ~(M3S_IN_FP8 | (a.bias ? 0 : M3S_EPI_BIAS));
  if constexpr (SP) {
    static_assert(MODE == 0, "fp8 split-K: GEMM mode");
    constexpr int LS = M3S_EPI_LN_STATS | M3S_EPI_BIAS;
    if (a.vec && try_epi<BM, BN, BK, WM, WN, STAGES, OCC, 0, M3S_EPI_RES_F32 | M3S_EPI_OUT_F32,
                         true, true>(a, grid, s, key))
      return;
    if (a.vec && key == (LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32)) {
      hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, 0, true,
                                      LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, true>),
                         grid, dim3(WM * WN * 64), 0, s, a);
      return;
    }
    hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, 0, true, -1, true>), grid,
                       dim3(WM * WN * 64), 0, s, a);
    return;
  }
  if (a.vec) {
    if constexpr (MODE == 0) {
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, 0, M3S_EPI_ROPE, true>(a, grid, s, key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, 0, M3S_EPI_GELU | M3S_EPI_OUT_FP8, true>(
              a, grid, s, key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, 0, M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, true>(
              a, grid, s, key))
        return;
      // the LayerNorm fold on e4m3 operands (round 6): consumers qkv / q (+RoPE) and fc1
      // (+GELU, e4m3 out), producers the residual GEMMs (f32 x + shifted e4m3 copy + stats)
      constexpr int LF = M3S_EPI_LN_FOLD | M3S_EPI_BIAS, LS = M3S_EPI_LN_STATS | M3S_EPI_BIAS;
      if (key == (LF | M3S_EPI_ROPE)) {
        hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, 0, false,
                                        LF | M3S_EPI_ROPE, true>),
                           grid, dim3(WM * WN * 64), 0, s, a);
        return;
      }
      if (key == (LF | M3S_EPI_GELU | M3S_EPI_OUT_FP8)) {
        hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, 0, false,
                                        LF | M3S_EPI_GELU | M3S_EPI_OUT_FP8, true>),
                           grid, dim3(WM * WN * 64), 0, s, a);
        return;
      }
      if (key == (LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32)) {
        hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, 0, false,
                                        LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, true>),
                           grid, dim3(WM * WN * 64), 0, s, a);
        return;
      }
    } else if constexpr (BN == 128) {
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_RELU | M3S_EPI_DPT_OUT, true>(
              a, grid, s, key))
        return;
    }
    if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, 0, true>(a, grid, s, key)) return;
  }
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, MODE, false, -1, true>), grid,
                     dim3(WM * WN * 64), 0, s, a);
}

template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, int MODE, bool SP = false>
void launch_main(Args& a, dim3 grid, hipStream_t s) {
  const int key = (a.flags & ~(M3S_PRO_RELU | (a.bias ? 0 : M3S_EPI_BIAS)));
  if (a.vec) {
    if (MODE == 0) {
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, 0, false, SP>(a, grid, s, key)) return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_ROPE, false, SP>(a, grid, s, key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_GELU, false, SP>(a, grid, s, key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, false,
                  SP>(a, grid, s, key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_OUT_F32, false, SP>(a, grid, s,
                                                                                    key))
        return;
      // LayerNorm fold (the ViT blocks' norm → projection pairs): consumers qkv / q / kv
      // (+RoPE) and fc1 (+GELU), producers the residual GEMMs and the embeddings
      if constexpr (BK == 64 && OCC <= 2 && (BM != 96 || OCC == 1) &&
                    ((BN == 128 && (BM == 64 || BM == 96 || BM == 128 || BM == 256) &&
                      (BM != 256 || OCC == 1)) ||
                     (BN == 256 && BM == 256 && OCC == 1))) {
        constexpr int LF = M3S_EPI_LN_FOLD, LS = M3S_EPI_LN_STATS;
        if (try_epi_b<BM, BN, BK, WM, WN, STAGES, OCC, MODE, LF | M3S_EPI_ROPE, SP>(a, grid, s,
                                                                                     key))
          return;
        if (try_epi_b<BM, BN, BK, WM, WN, STAGES, OCC, MODE, LF | M3S_EPI_GELU, SP>(a, grid, s,
                                                                                     key))
          return;
        if (try_epi_b<BM, BN, BK, WM, WN, STAGES, OCC, MODE,
                      LS | M3S_EPI_RES_F32 | M3S_EPI_OUT_F32, SP>(a, grid, s, key))
          return;
        if (try_epi_b<BM, BN, BK, WM, WN, STAGES, OCC, MODE, LS | M3S_EPI_OUT_F32, SP>(a, grid, s,
                                                                                        key))
          return;
      }
    } else {
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, 0, false, SP>(a, grid, s, key)) return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_RES_BF16, false, SP>(a, grid, s,
                                                                                     key))
        return;
      if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_RELU, false, SP>(a, grid, s, key))
        return;
      if constexpr (BN == 128 && !SP)
        if (try_epi<BM, BN, BK, WM, WN, STAGES, OCC, MODE, M3S_EPI_RELU | M3S_EPI_DPT_OUT>(
                a, grid, s, key))
          return;
    }
  }
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, WM, WN, STAGES, OCC, MODE, SP, -1>), grid,
                     dim3(WM * WN * 64), 0, s, a);
}

template <int BM, int BN, int BK, int WM, int WN, int STAGES, int OCC, bool F8 = false>
int launch(Args& a, int batch, hipStream_t s) {
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const bool split = a.splits > 1;
  const int64_t groups = (int64_t)batch * (split ? a.splits : 1);
  if ((int64_t)a.tiles_m * a.tiles_n * groups >= (1ll << 31)) return M3S_ERR_TOO_LARGE;
  dim3 grid((unsigned)(a.tiles_m * a.tiles_n * groups));
  set_order(a, BM, BN, groups);
  if (split) {
    // split-K (fused last-split epilogue): 128^2 GEMM tiles, 64x128 GEMM / conv tiles
    constexpr bool CAN = (BM == 128 && BN == 128 && BK == 64) ||
                         (BM == 64 && BN == 128 && BK == 64) ||
                         (BM == 256 && BN == 128 && BK == 64);
    if constexpr (CAN && F8) {
      if (a.mode != 0) return M3S_ERR_INVALID_ARG;
      launch_main_f8<BM, BN, BK, WM, WN, STAGES, OCC, 0, true>(a, grid, s);
    } else if constexpr (CAN) {
      if (a.mode == 0)
        launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 0, true>(a, grid, s);
      else if (a.flags & M3S_PRO_RELU)
        launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 2, true>(a, grid, s);
      else
        launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 1, true>(a, grid, s);
    } else {
      return M3S_ERR_INVALID_ARG;
    }
    if (!a.fused) {
      M3S_LAUNCH_CHECK();
      const int64_t nv = (int64_t)a.M * ((a.N + 7) / 8);
      hipLaunchKernelGGL(splitk_reduce_kernel<0>, dim3(m3s_div_up(nv, 256), (unsigned)batch),
                         dim3(256), 0, s, a);
    }
  } else if constexpr (F8) {
    if (a.mode == 0)
      launch_main_f8<BM, BN, BK, WM, WN, STAGES, OCC, 0>(a, grid, s);
    else
      launch_main_f8<BM, BN, BK, WM, WN, STAGES, OCC, 1>(a, grid, s);
  } else if (a.mode == 0) {
    launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 0>(a, grid, s);
  } else if (a.flags & M3S_PRO_RELU) {
    launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 2>(a, grid, s);
  } else {
    launch_main<BM, BN, BK, WM, WN, STAGES, OCC, 1>(a, grid, s);
  }
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

}  // namespace m3s_gemm
