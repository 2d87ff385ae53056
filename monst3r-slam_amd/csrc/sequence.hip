// Streaming C3 sequence plumbing (BASELINE configs[2]: 200-frame 384x512 tracking loop),
// replayable from one captured HIP graph per parity: every per-frame index lives on the
// device, so the same launches process frame t, t+1, ... without host work.
//
//   seq_gather        image of frame (*frame + offset) from the sequence staged in HBM into
//                     the encoder's input buffer (clamped to the last frame)
//   seq_pair_outputs  stand-in for the trained networks' pair outputs (random weights carry
//                     no geometry): after the pair inference has written X / C / D16 / Q,
//                     they are overwritten in stream order with the staged scene geometry of
//                     frame t = *frame against the current keyframe j = *kf_frame:
//                       X[0] = Xcam[t]                 (frame's own pointmap, camera t)
//                       X[1] = T_t^-1 T_j Xcam[j]      (keyframe pixels in camera t)
//                       C / Q = the frame's staged confidences, D16[0] = D[t], D16[1] = D[j]
//   seq_advance       the main loop's bookkeeping after FrameTracker2.track
//                     (main_monster_slam.py:292-321, tracker2.py:238-257): log (iterations,
//                     new_kf, lost, keyframe, T_WCf) of frame t; the next frame starts from
//                     T_WCf unless lost; on new_kf the frame becomes the keyframe
//                     (keyframes.append(frame): X_canon = Xff, C = Cff, N = 1 — the frame's
//                     first update_pointmap, frame.py:60-124 — T_WC = T_WCf, cached encoder
//                     features) and idx_f2k resets to the identity (reset_idx_f2k); *frame += 1.
#include <hip/hip_fp16.h>

#include "common.h"

namespace {

constexpr int kThreads = 256;

__global__ void seq_gather_kernel(const uint4* __restrict__ src, int64_t frame_vec,
                                  const int* __restrict__ frame, int offset, int nframes,
                                  uint4* __restrict__ dst) {
  int f = *frame + offset;
  f = f < 0 ? 0 : (f > nframes - 1 ? nframes - 1 : f);
  const uint4* s = src + (int64_t)f * frame_vec;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < frame_vec;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = s[i];
}

// 3x4 [sR | t] of the Sim3 T = [t, q xyzw, s]
__device__ __forceinline__ void sim3_matrix(const float* T, float* M) {
  const float x = T[3], y = T[4], z = T[5], w = T[6], s = T[7];
  M[0] = s * (1.f - 2.f * (y * y + z * z));
  M[1] = s * (2.f * (x * y - z * w));
  M[2] = s * (2.f * (x * z + y * w));
  M[4] = s * (2.f * (x * y + z * w));
  M[5] = s * (1.f - 2.f * (x * x + z * z));
  M[6] = s * (2.f * (y * z - x * w));
  M[8] = s * (2.f * (x * z - y * w));
  M[9] = s * (2.f * (y * z + x * w));
  M[10] = s * (1.f - 2.f * (x * x + y * y));
  M[3] = T[0];
  M[7] = T[1];
  M[11] = T[2];
}

__global__ __launch_bounds__(kThreads) void seq_pair_outputs_kernel(
    const float* __restrict__ Xcam, const float* __restrict__ C_own,
    const float* __restrict__ C_other, const float* __restrict__ Q_own,
    const float* __restrict__ Q_other, const uint4* __restrict__ D16, const float* __restrict__ T_gt,
    const int* __restrict__ frame, const int* __restrict__ kf_frame, int nframes, int64_t n,
    float* __restrict__ X, float* __restrict__ C, uint4* __restrict__ Dout,
    float* __restrict__ Q) {
  int t = *frame, j = *kf_frame;
  t = t > nframes - 1 ? nframes - 1 : t;
  __shared__ float M[12];
  if (threadIdx.x == 0) {
    // T_t^-1 T_j (f64 composition, one rounding to f32 per entry)
    double A[12], B[12];
    float Ma[12], Mb[12];
    sim3_matrix(T_gt + 8 * t, Ma);
    sim3_matrix(T_gt + 8 * j, Mb);
    for (int i = 0; i < 12; i++) {
      A[i] = Ma[i];
      B[i] = Mb[i];
    }
    // inverse of [sR | t]: (sR)^-1 = R^T / s = (sR)^T / s^2
    const double s2 = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
    double Ri[9], ti[3];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) Ri[3 * r + c] = A[4 * c + r] / s2;
    for (int r = 0; r < 3; r++)
      ti[r] = -(Ri[3 * r] * A[3] + Ri[3 * r + 1] * A[7] + Ri[3 * r + 2] * A[11]);
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++)
        M[4 * r + c] = (float)(Ri[3 * r] * B[c] + Ri[3 * r + 1] * B[4 + c] + Ri[3 * r + 2] * B[8 + c]);
      M[4 * r + 3] =
          (float)(Ri[3 * r] * B[3] + Ri[3 * r + 1] * B[7] + Ri[3 * r + 2] * B[11] + ti[r]);
    }
  }
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (k >= n) return;
  const float* xt = Xcam + ((int64_t)t * n + k) * 3;
  const float* xj = Xcam + ((int64_t)j * n + k) * 3;
  const float a0 = xj[0], a1 = xj[1], a2 = xj[2];
  X[3 * k] = xt[0];
  X[3 * k + 1] = xt[1];
  X[3 * k + 2] = xt[2];
  float* X1 = X + 3 * n;
  X1[3 * k] = M[0] * a0 + M[1] * a1 + M[2] * a2 + M[3];
  X1[3 * k + 1] = M[4] * a0 + M[5] * a1 + M[6] * a2 + M[7];
  X1[3 * k + 2] = M[8] * a0 + M[9] * a1 + M[10] * a2 + M[11];
  C[k] = C_own[(int64_t)t * n + k];
  C[n + k] = C_other[(int64_t)t * n + k];
  Q[k] = Q_own[(int64_t)t * n + k];
  Q[n + k] = Q_other[(int64_t)t * n + k];
  // 24 halfs = 48 B = 3 x 16 B per pixel
  const uint4* dt = D16 + ((int64_t)t * n + k) * 3;
  const uint4* dj = D16 + ((int64_t)j * n + k) * 3;
  uint4* o0 = Dout + k * 3;
  uint4* o1 = Dout + (n + k) * 3;
#pragma unroll
  for (int v = 0; v < 3; v++) {
    o0[v] = dt[v];
    o1[v] = dj[v];
  }
}

// log row: iterations, new_kf, lost, keyframe frame (after this frame), 4 x pad → then T_WCf
constexpr int kLogInts = 8;

__global__ __launch_bounds__(kThreads) void seq_advance_kernel(
    const uint8_t* __restrict__ flags, const int* __restrict__ info,
    const float* __restrict__ T_WCf, const float* __restrict__ Xff, const float* __restrict__ Cff,
    const uint4* __restrict__ feat_i, int64_t feat_vec, int64_t n, float* __restrict__ kf_X,
    float* __restrict__ kf_C, float* __restrict__ kf_N, float* __restrict__ kf_T,
    uint4* __restrict__ kf_feat, int64_t* __restrict__ idx_f2k, float* __restrict__ T_prev,
    int* __restrict__ frame, int* __restrict__ kf_frame, int* __restrict__ log_i,
    float* __restrict__ log_T, int nlog) {
  const bool new_kf = flags[0] != 0, lost = flags[1] != 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int t = *frame;
    if (new_kf) *kf_frame = t;
    if (t < nlog) {
      int* L = log_i + (int64_t)t * kLogInts;
      L[0] = info[0];
      L[1] = new_kf;
      L[2] = lost;
      L[3] = *kf_frame;
      L[4] = info[1];
      L[5] = info[3];
      float* LT = log_T + (int64_t)t * 8;
      for (int i = 0; i < 8; i++) LT[i] = T_WCf[i];
    }
    if (!lost)
      for (int i = 0; i < 8; i++) T_prev[i] = T_WCf[i];
    if (new_kf) {
      for (int i = 0; i < 8; i++) kf_T[i] = T_WCf[i];
      kf_N[0] = 1.f;
    }
    *frame = t + 1;
  }
  if (!new_kf) return;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x; k < n; k += stride) {
    kf_X[3 * k] = Xff[3 * k];
    kf_X[3 * k + 1] = Xff[3 * k + 1];
    kf_X[3 * k + 2] = Xff[3 * k + 2];
    kf_C[k] = Cff[k];
    idx_f2k[k] = k;
  }
  for (int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x; k < feat_vec; k += stride)
    kf_feat[k] = feat_i[k];
}

}  // namespace

extern "C" int m3s_seq_gather(const void* d_src, int64_t frame_bytes, const int* d_frame,
                              int offset, int nframes, void* d_dst, void* stream) {
  if (!d_src || !d_frame || !d_dst || nframes < 1 || frame_bytes <= 0 || frame_bytes % 16)
    return M3S_ERR_INVALID_ARG;
  if (((uintptr_t)d_src | (uintptr_t)d_dst) & 15) return M3S_ERR_INVALID_ARG;
  const int64_t vec = frame_bytes / 16;
  unsigned blocks = m3s_div_up(vec, kThreads);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(seq_gather_kernel, dim3(blocks), dim3(kThreads), 0, m3s_stream(stream),
                     reinterpret_cast<const uint4*>(d_src), vec, d_frame, offset, nframes,
                     reinterpret_cast<uint4*>(d_dst));
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_seq_pair_outputs(const float* d_Xcam, const float* d_C_own,
                                    const float* d_C_other, const float* d_Q_own,
                                    const float* d_Q_other, const void* d_D16, const float* d_T_gt,
                                    const int* d_frame, const int* d_kf_frame, int nframes,
                                    int64_t n, float* d_X, float* d_C, void* d_D16_out,
                                    float* d_Q, void* stream) {
  if (!d_Xcam || !d_C_own || !d_C_other || !d_Q_own || !d_Q_other || !d_D16 || !d_T_gt ||
      !d_frame || !d_kf_frame || !d_X || !d_C || !d_D16_out || !d_Q || n < 1 || nframes < 1)
    return M3S_ERR_INVALID_ARG;
  if (((uintptr_t)d_D16 | (uintptr_t)d_D16_out) & 15) return M3S_ERR_INVALID_ARG;
  hipLaunchKernelGGL(seq_pair_outputs_kernel, dim3(m3s_div_up(n, kThreads)), dim3(kThreads), 0,
                     m3s_stream(stream), d_Xcam, d_C_own, d_C_other, d_Q_own, d_Q_other,
                     reinterpret_cast<const uint4*>(d_D16), d_T_gt, d_frame, d_kf_frame, nframes,
                     n, d_X, d_C, reinterpret_cast<uint4*>(d_D16_out), d_Q);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_seq_advance(const uint8_t* d_flags, const int* d_info, const float* d_T_WCf,
                               const float* d_Xff, const float* d_Cff, const void* d_feat_i,
                               int64_t feat_bytes, int64_t n, float* d_kf_X, float* d_kf_C,
                               float* d_kf_N, float* d_kf_T, void* d_kf_feat, int64_t* d_idx_f2k,
                               float* d_T_prev, int* d_frame, int* d_kf_frame, int* d_log_i,
                               float* d_log_T, int nlog, void* stream) {
  if (!d_flags || !d_info || !d_T_WCf || !d_Xff || !d_Cff || !d_kf_X || !d_kf_C || !d_kf_N ||
      !d_kf_T || !d_idx_f2k || !d_T_prev || !d_frame || !d_kf_frame || n < 1 ||
      (nlog > 0 && (!d_log_i || !d_log_T)) || feat_bytes < 0 || feat_bytes % 16 ||
      (feat_bytes > 0 && (!d_feat_i || !d_kf_feat)))
    return M3S_ERR_INVALID_ARG;
  if (((uintptr_t)d_feat_i | (uintptr_t)d_kf_feat) & 15) return M3S_ERR_INVALID_ARG;
  unsigned blocks = m3s_div_up(n, kThreads);
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(seq_advance_kernel, dim3(blocks), dim3(kThreads), 0, m3s_stream(stream),
                     d_flags, d_info, d_T_WCf, d_Xff, d_Cff,
                     reinterpret_cast<const uint4*>(d_feat_i), feat_bytes / 16, n, d_kf_X, d_kf_C,
                     d_kf_N, d_kf_T, reinterpret_cast<uint4*>(d_kf_feat), d_idx_f2k, d_T_prev,
                     d_frame, d_kf_frame, d_log_i, d_log_T, nlog);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
