// Frontend tracking glue around the pose solve (FrameTracker2.track, tracker2.py:127-257,
// use_calib False, dynamic mask off) as three gfx950 kernels instead of ~25 elementwise /
// gather / reduce launches of the torch restatement (frontend.Tracker.track_outputs):
//
//   glue_pre   per keyframe pixel i (tracker2.py:127-196; frame.py:60-124 get_points_poses):
//                Qk = sqrt(Qff[idx] * Qkf), Xf = Xf_canon[idx], Ck = C / N,
//                valid_opt = valid_match & (Cf[idx] > C_conf) & (Ck > C_conf) & (Qk > Q_conf),
//                valid_kf  = valid_match & (Qk > Q_conf);
//              per-workgroup counts of valid_opt / valid_kf (no atomics: fixed partials),
//              and the unique-match scratch row cleared.
//   (pose GN: m3s_track_rays on Xf, X_canon, Qk, valid_opt)
//   glue_post  lost = match_frac < min_match_frac | Cholesky failure (tracker2.py:196-236);
//              keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf) 'weighted_pointmap'
//              (tracker2.py:238-243, frame.py:105-109) masked off when lost; C += Ckf,
//              N += 1 unless lost; the unique-match scratch: sel[idx[i]] = 1 for valid
//              matches (idempotent stores).
//   glue_final one workgroup: unique_frac = |{sel > 0}| / n, match_frac_k, and the new-
//              keyframe test min(match_frac_k, unique_frac) < thresh & !lost (:246-257).
// Everything stays on the device; the flags are written as u8 for lazy host reads.
#include "common.h"

namespace {

constexpr int kT = 256;

__device__ __forceinline__ int block_sum_int(int v, int* sh) {
  v = m3s_wave_sum_int(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int t = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kT / 64; i++) t += sh[i];
  return t;  // valid in thread 0
}

__global__ __launch_bounds__(kT) void glue_pre_kernel(
    const float* __restrict__ X, const float* __restrict__ C, const float* __restrict__ Q,
    const int64_t* __restrict__ idx, const uint8_t* __restrict__ valid_match,
    const float* __restrict__ kf_C, const float* __restrict__ kf_N, int64_t n, float Q_conf,
    float C_conf, float* __restrict__ Xf, float* __restrict__ Qk, uint8_t* __restrict__ valid_opt,
    int2* __restrict__ counts, uint8_t* __restrict__ sel) {
  __shared__ int sh[kT / 64];
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  int c_opt = 0, c_kf = 0;
  if (i < n) {
    const int64_t j = idx[i];
    const float qk = sqrtf(Q[j] * Q[n + i]);          // Qff[idx] * Qkf (X/C/Q: [2][n])
    Qk[i] = qk;
    Xf[3 * i] = X[3 * j];
    Xf[3 * i + 1] = X[3 * j + 1];
    Xf[3 * i + 2] = X[3 * j + 2];
    const float ck = kf_C[i] / kf_N[0];
    const bool vm = valid_match[i] != 0;
    const bool vq = qk > Q_conf;
    const bool vo = vm && (C[j] > C_conf) && (ck > C_conf) && vq;
    valid_opt[i] = vo;
    c_opt = vo;
    c_kf = vm && vq;
    sel[i] = 0;
  }
  const int a = block_sum_int(c_opt, sh);
  const int b = block_sum_int(c_kf, sh);
  if (threadIdx.x == 0) counts[blockIdx.x] = make_int2(a, b);
}

// sum of the pre-kernel partials (every workgroup reads them: ≤ a few KB from L2)
__device__ __forceinline__ int2 sum_counts(const int2* __restrict__ counts, int nb, int* sh) {
  int a = 0, b = 0;
  for (int k = threadIdx.x; k < nb; k += kT) {
    const int2 c = counts[k];
    a += c.x;
    b += c.y;
  }
  a = block_sum_int(a, sh);
  b = block_sum_int(b, sh);
  __syncthreads();
  if (threadIdx.x == 0) sh[0] = a, sh[1] = b;
  __syncthreads();
  return make_int2(sh[0], sh[1]);
}

__global__ __launch_bounds__(kT) void glue_post_kernel(
    const float* __restrict__ X, const float* __restrict__ C, const int64_t* __restrict__ idx,
    const uint8_t* __restrict__ valid_match, const int2* __restrict__ counts, int nb,
    const int* __restrict__ info, const float* __restrict__ T, int64_t n, float min_match_frac,
    float* __restrict__ kf_X, float* __restrict__ kf_C, float* __restrict__ kf_N,
    uint8_t* __restrict__ sel) {
  __shared__ int sh[kT / 64];
  const int2 cnt = sum_counts(counts, nb, sh);
  const float match_frac = (float)cnt.x / (float)n;
  const bool lost = (match_frac < min_match_frac) || (info[1] != 0);
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i < n) {
    if (valid_match[i]) sel[idx[i]] = 1;
    const float ckf = C[n + i];
    if (!lost) {
      // Xkk = T_CkCf.act(Xkf): s (X + qw uv + q x uv) + t, uv = 2 q x X (frontend.sim3_act)
      const float tx = T[0], ty = T[1], tz = T[2], qx = T[3], qy = T[4], qz = T[5], qw = T[6],
                  s = T[7];
      const float px = X[3 * (n + i)], py = X[3 * (n + i) + 1], pz = X[3 * (n + i) + 2];
      const float ux = 2.0f * (qy * pz - qz * py), uy = 2.0f * (qz * px - qx * pz),
                  uz = 2.0f * (qx * py - qy * px);
      const float cx = qy * uz - qz * uy, cy = qz * ux - qx * uz, cz = qx * uy - qy * ux;
      const float xk[3] = {s * (px + qw * ux + cx) + tx, s * (py + qw * uy + cy) + ty,
                           s * (pz + qw * uz + cz) + tz};
      const float c0 = kf_C[i];
      const float den = c0 + ckf;
#pragma unroll
      for (int d = 0; d < 3; d++) kf_X[3 * i + d] = (c0 * kf_X[3 * i + d] + ckf * xk[d]) / den;
      kf_C[i] = c0 + ckf;
    }
  }
  if (i == 0 && !lost) kf_N[0] += 1.0f;
}

__global__ __launch_bounds__(1024) void glue_final_kernel(
    const uint8_t* __restrict__ sel, const int2* __restrict__ counts, int nb,
    const int* __restrict__ info, int64_t n, float min_match_frac, float match_frac_thresh,
    uint8_t* __restrict__ flags, float* __restrict__ fracs) {
  __shared__ int sh[16];
  int a = 0, b = 0, u = 0;
  for (int k = threadIdx.x; k < nb; k += 1024) {
    const int2 c = counts[k];
    a += c.x;
    b += c.y;
  }
  const int64_t n16 = n / 16;
  for (int64_t k = threadIdx.x; k < n16; k += 1024) {
    const uint4 v = reinterpret_cast<const uint4*>(sel)[k];
    u += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) +
         __builtin_popcount(v.w);  // sel bytes are 0 or 1
  }
  for (int64_t k = n16 * 16 + threadIdx.x; k < n; k += 1024) u += sel[k];
  int vals[3] = {a, b, u};
  int tot[3];
  for (int q = 0; q < 3; q++) {
    int v = m3s_wave_sum_int(vals[q]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < 16; w++) t += sh[w];
    tot[q] = t;
  }
  if (threadIdx.x == 0) {
    const float match_frac = (float)tot[0] / (float)n;
    const float match_frac_k = (float)tot[1] / (float)n;
    const float unique_frac = (float)tot[2] / (float)n;
    const bool lost = (match_frac < min_match_frac) || (info[1] != 0);
    const bool new_kf = (fminf(match_frac_k, unique_frac) < match_frac_thresh) && !lost;
    flags[0] = new_kf;
    flags[1] = lost;
    fracs[0] = match_frac;
    fracs[1] = match_frac_k;
    fracs[2] = unique_frac;
  }
}

}  // namespace

extern "C" size_t m3s_glue_workspace_bytes(int64_t n) {
  const int64_t nb = m3s_div_up(n, kT);
  return (size_t)(nb * 8 + ((n + 15) / 16) * 16 + 256);
}

extern "C" int m3s_track_glue_pre(const float* d_X, const float* d_C, const float* d_Q,
                                  const int64_t* d_idx, const uint8_t* d_valid_match,
                                  const float* d_kf_C, const float* d_kf_N, int64_t n,
                                  float Q_conf, float C_conf, float* d_Xf, float* d_Qk,
                                  uint8_t* d_valid_opt, void* d_workspace, void* stream) {
  if (!d_X || !d_C || !d_Q || !d_idx || !d_valid_match || !d_kf_C || !d_kf_N || !d_Xf ||
      !d_Qk || !d_valid_opt || !d_workspace || n <= 0)
    return M3S_ERR_INVALID_ARG;
  if ((uintptr_t)d_workspace % 16) return M3S_ERR_INVALID_ARG;
  const int64_t nb = m3s_div_up(n, kT);
  if (nb >= (1ll << 31)) return M3S_ERR_TOO_LARGE;
  int2* counts = reinterpret_cast<int2*>(d_workspace);
  uint8_t* sel = reinterpret_cast<uint8_t*>(d_workspace) + ((nb * 8 + 15) / 16) * 16;
  hipLaunchKernelGGL(glue_pre_kernel, dim3((unsigned)nb), dim3(kT), 0, m3s_stream(stream), d_X,
                     d_C, d_Q, d_idx, d_valid_match, d_kf_C, d_kf_N, n, Q_conf, C_conf, d_Xf,
                     d_Qk, d_valid_opt, counts, sel);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_track_glue_post(const float* d_X, const float* d_C, const int64_t* d_idx,
                                   const uint8_t* d_valid_match, const int* d_info,
                                   const float* d_T_CkCf, int64_t n, float min_match_frac,
                                   float match_frac_thresh, float* d_kf_X, float* d_kf_C,
                                   float* d_kf_N, uint8_t* d_flags, float* d_fracs,
                                   void* d_workspace, void* stream) {
  if (!d_X || !d_C || !d_idx || !d_valid_match || !d_info || !d_T_CkCf || !d_kf_X || !d_kf_C ||
      !d_kf_N || !d_flags || !d_fracs || !d_workspace || n <= 0)
    return M3S_ERR_INVALID_ARG;
  if ((uintptr_t)d_workspace % 16) return M3S_ERR_INVALID_ARG;
  const int64_t nb = m3s_div_up(n, kT);
  if (nb >= (1ll << 31)) return M3S_ERR_TOO_LARGE;
  const int2* counts = reinterpret_cast<const int2*>(d_workspace);
  uint8_t* sel = reinterpret_cast<uint8_t*>(d_workspace) + ((nb * 8 + 15) / 16) * 16;
  hipStream_t s = m3s_stream(stream);
  hipLaunchKernelGGL(glue_post_kernel, dim3((unsigned)nb), dim3(kT), 0, s, d_X, d_C, d_idx,
                     d_valid_match, counts, (int)nb, d_info, d_T_CkCf, n, min_match_frac, d_kf_X,
                     d_kf_C, d_kf_N, sel);
  M3S_LAUNCH_CHECK();
  hipLaunchKernelGGL(glue_final_kernel, dim3(1), dim3(1024), 0, s, sel, counts, (int)nb, d_info, n,
                     min_match_frac, match_frac_thresh, d_flags, d_fracs);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
