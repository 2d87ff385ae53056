// Attention and 2-D RoPE for the CroCo ViT (gfx950).
//
// rope2d_kernel: in-place RoPE100 on a bf16 q or k view (croco curope kernels.cu:17-82,
//   pos_embed.py:106-158): head dim 64 = [y half | x half]; within a half, pairs
//   (i, i+16), angle = pos * base^(-i/16); f32 math, one bf16 rounding.
// attn_kernel: flash-style softmax(q k^T / 8) v, one wave per 32 query rows.
//   S^T = K Q^T with v_mfma_f32_32x32x16_bf16 (keys on the accumulator rows, queries on
//   the lanes), so the online-softmax max / sum per query are lane-local (+ one xor-32
//   exchange).  P^T stays in registers as the B operand of O^T = V^T P^T; V^T fragments
//   come from an LDS image of the V tile via ds_read_b64_tr_b16 (hardware transpose).
//   Keys beyond sk are masked (any token count, e.g. 14x14 at 224^2).
#include "vit_common.h"

namespace {

constexpr int HD = 64;
constexpr int QT = 32;   // query rows per wave
constexpr int KT = 32;   // keys per tile
constexpr int VS = 72;   // LDS row stride (bf16) of the V tile: 144 B, 16-B aligned rows

typedef short s16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void rope2d_kernel(bf16_t* __restrict__ t, int64_t ld,
                                                     int64_t stride, const int64_t* __restrict__ pos,
                                                     int64_t stride_pos, int S, int heads,
                                                     float base, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  // idx -> (b, s, head, half)
  const int half = (int)(idx & 1);
  int64_t r = idx >> 1;
  const int hd = (int)(r % heads);
  r /= heads;
  const int s = (int)(r % S);
  const int64_t b = r / S;
  const float p = (float)pos[b * stride_pos + (int64_t)s * 2 + half];  // (y, x)
  bf16_t* row = t + b * stride + (int64_t)s * ld + hd * HD + half * 32;
  uint4 raw[4];
#pragma unroll
  for (int c = 0; c < 4; c++) raw[c] = reinterpret_cast<const uint4*>(row)[c];
  const bf16_t* vals = reinterpret_cast<const bf16_t*>(raw);
  float u[16], v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    u[i] = bf2f(vals[i]);
    v[i] = bf2f(vals[i + 16]);
  }
  bf16_t outv[32];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const float inv_freq = 1.0f / powf(base, (float)i / 16.0f);
    const float f = p * inv_freq;
    const float c = cosf(f), sn = sinf(f);
    outv[i] = f2bf(u[i] * c - v[i] * sn);
    outv[i + 16] = f2bf(v[i] * c + u[i] * sn);
  }
#pragma unroll
  for (int c = 0; c < 4; c++)
    reinterpret_cast<uint4*>(row)[c] = reinterpret_cast<const uint4*>(outv)[c];
}

__device__ __forceinline__ bf16x8 load8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__global__ __launch_bounds__(64) void attn_kernel(
    const bf16_t* __restrict__ q, int64_t ldq, int64_t sq_b, const bf16_t* __restrict__ k,
    const bf16_t* __restrict__ v, int64_t ldkv, int64_t skv_b, bf16_t* __restrict__ o,
    int64_t ldo, int64_t so_b, int Sq, int Sk, float c_log2) {
  __shared__ __attribute__((aligned(16))) bf16_t Vs[KT][VS];
  const int lane = threadIdx.x;
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = blockIdx.x * QT;
  const int h = blockIdx.y;
  const int64_t b = blockIdx.z;
  const bf16_t* Q = q + b * sq_b + h * HD;
  const bf16_t* K = k + b * skv_b + h * HD;
  const bf16_t* V = v + b * skv_b + h * HD;

  const int qrow = q0 + r;
  bf16x8 qf[4];
  const bf16x8 zero8 = {};
#pragma unroll
  for (int ks = 0; ks < 4; ks++)
    qf[ks] = qrow < Sq ? load8(Q + (int64_t)qrow * ldq + ks * 16 + 8 * hh) : zero8;

  f32x16 oacc[2];
#pragma unroll
  for (int d = 0; d < 2; d++)
#pragma unroll
    for (int i = 0; i < 16; i++) oacc[d][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  const int nkt = (Sk + KT - 1) / KT;
  // V staging: lane -> key row (lane >> 1), 32-wide d half (lane & 1)
  const int vr = lane >> 1, vh = (lane & 1) * 32;
  // tr-read addressing inside a 16-lane group
  const int gi = lane & 15, gq = gi >> 2, gp = gi & 3, gsel = (lane >> 4) & 1;

  for (int kt = 0; kt < nkt; kt++) {
    const int key = kt * KT + r;
    const bool kvalid = key < Sk;
    bf16x8 kf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ks++)
      kf[ks] = kvalid ? load8(K + (int64_t)key * ldkv + ks * 16 + 8 * hh) : zero8;
    // stage V tile (previous tile's reads are complete after the barrier below)
    const int vkey = kt * KT + vr;
    uint4 vv[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
      vv[c] = vkey < Sk ? *reinterpret_cast<const uint4*>(V + (int64_t)vkey * ldkv + vh + 8 * c)
                        : make_uint4(0, 0, 0, 0);
    f32x16 s;
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ks++) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[ks], qf[ks], s, 0, 0, 0);
    // online softmax over this tile's keys (rows of s)
    float tmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int kr = kt * KT + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (kr >= Sk) s[i] = -INFINITY;
      tmax = fmaxf(tmax, s[i]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m, tmax);
    const float alpha = (m == -INFINITY) ? 0.f : exp2f((m - m_new) * c_log2);
    float rs = 0.f;
    float p[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      p[i] = (s[i] == -INFINITY) ? 0.f : exp2f((s[i] - m_new) * c_log2);
      rs += p[i];
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
#pragma unroll
    for (int d = 0; d < 2; d++)
#pragma unroll
      for (int i = 0; i < 16; i++) oacc[d][i] *= alpha;
    bf16x8 pf[2];
#pragma unroll
    for (int ss = 0; ss < 2; ss++)
#pragma unroll
      for (int j = 0; j < 8; j++) pf[ss][j] = f2bf(p[8 * ss + j]);

    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++) *reinterpret_cast<uint4*>(&Vs[vr][vh + 8 * c]) = vv[c];
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 2; d++) {
      const int d0 = d * 32 + 16 * gsel + 4 * gp;
#pragma unroll
      for (int ss = 0; ss < 2; ss++) {
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)&Vs[16 * ss + 4 * hh + gq][d0]);
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)&Vs[16 * ss + 8 + 4 * hh + gq][d0]);
        bf16x8 vf;
        const bf16x4 lob = __builtin_bit_cast(bf16x4, lo);
        const bf16x4 hib = __builtin_bit_cast(bf16x4, hi);
        vf[0] = lob[0];
        vf[1] = lob[1];
        vf[2] = lob[2];
        vf[3] = lob[3];
        vf[4] = hib[0];
        vf[5] = hib[1];
        vf[6] = hib[2];
        vf[7] = hib[3];
        oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[ss], oacc[d], 0, 0, 0);
      }
    }
  }
  if (qrow >= Sq) return;
  const float inv_l = 1.0f / l;
  bf16_t* O = o + b * so_b + (int64_t)qrow * ldo + h * HD;
#pragma unroll
  for (int d = 0; d < 2; d++)
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int dd = d * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      O[dd] = f2bf(oacc[d][i] * inv_l);
    }
}

}  // namespace

extern "C" int m3s_vit_rope(void* d_t, int64_t ld, int64_t stride, const int64_t* d_pos,
                            int64_t stride_pos, int64_t batch, int64_t S, int64_t heads,
                            float base, void* stream) {
  if (!d_t || !d_pos || batch <= 0 || S <= 0 || heads <= 0) return M3S_ERR_INVALID_ARG;
  if (((uintptr_t)d_t) % 16 || ld % 8 || stride % 8) return M3S_ERR_INVALID_ARG;
  const int64_t total = batch * S * heads * 2;
  hipLaunchKernelGGL(rope2d_kernel, dim3(m3s_div_up(total, 256)), dim3(256), 0,
                     m3s_stream(stream), reinterpret_cast<bf16_t*>(d_t), ld, stride, d_pos,
                     stride_pos, (int)S, (int)heads, base, total);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_vit_attention(const void* d_q, int64_t ld_q, int64_t stride_q, const void* d_k,
                                 const void* d_v, int64_t ld_kv, int64_t stride_kv,
                                 const int64_t* d_qpos, const int64_t* d_kpos, int64_t stride_pos,
                                 void* d_o, int64_t ld_o, int64_t stride_o, int64_t batch,
                                 int64_t heads, int64_t sq, int64_t sk, float rope_base,
                                 void* stream) {
  if (!d_q || !d_k || !d_v || !d_o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0)
    return M3S_ERR_INVALID_ARG;
  if ((((uintptr_t)d_q) | ((uintptr_t)d_k) | ((uintptr_t)d_v)) % 16) return M3S_ERR_INVALID_ARG;
  if (ld_q % 8 || ld_kv % 8 || stride_q % 8 || stride_kv % 8) return M3S_ERR_INVALID_ARG;
  if (batch > 65535 || heads > 65535) return M3S_ERR_TOO_LARGE;
  // RoPE is applied by m3s_vit_rope on q and k beforehand (rope_base kept for the ABI;
  // positions are consumed there).
  (void)d_qpos;
  (void)d_kpos;
  (void)stride_pos;
  (void)rope_base;
  const float c_log2 = 0.125f * 1.4426950408889634f;  // head_dim^-0.5 * log2(e)
  dim3 grid(m3s_div_up(sq, QT), (unsigned)heads, (unsigned)batch);
  hipLaunchKernelGGL(attn_kernel, grid, dim3(64), 0, m3s_stream(stream),
                     reinterpret_cast<const bf16_t*>(d_q), ld_q, stride_q,
                     reinterpret_cast<const bf16_t*>(d_k), reinterpret_cast<const bf16_t*>(d_v),
                     ld_kv, stride_kv, reinterpret_cast<bf16_t*>(d_o), ld_o, stride_o, (int)sq,
                     (int)sk, c_log2);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
