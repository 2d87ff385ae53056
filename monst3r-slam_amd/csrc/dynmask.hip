// Dynamic-mask arithmetic of MonST3R-SLAM (gfx950), HBM-bound elementwise passes:
//   m3s_flow_error_mask   get_dynamic_mask's error map → min-max normalisation → threshold
//                         (mast3r_slam/monst3r_utils.py:625-637)
//   m3s_apply_dynamic_mask apply_dynamic_mask_to_pointmaps (monst3r_utils.py:300-341)
//   m3s_ego_flow          ego-motion flow of get_dynamic_mask (:566-614) from the mono depth
#include "common.h"

namespace {

// err >= 0, so its IEEE bits order like unsigned integers: min / max by integer atomics.
__global__ __launch_bounds__(64) void flow_err_init_kernel(unsigned* mm) {
  if (threadIdx.x == 0) {
    mm[0] = 0x7f800000u;  // +inf
    mm[1] = 0u;
  }
}

__global__ __launch_bounds__(256) void flow_err_kernel(const float* __restrict__ flow,
                                                       const float* __restrict__ ego, int64_t n,
                                                       float* __restrict__ err,
                                                       unsigned* __restrict__ mm) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float e = 0.f;
  bool ok = i < n;
  if (ok) {
    const float dx = flow[i] - ego[i];
    const float dy = flow[n + i] - ego[n + i];
    e = sqrtf(dx * dx + dy * dy);  // torch.norm(flow_diff, dim=0)
    err[i] = e;
  }
  float lo = ok ? e : INFINITY, hi = ok ? e : 0.f;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, off, 64));
    hi = fmaxf(hi, __shfl_xor(hi, off, 64));
  }
  __shared__ float slo[4], shi[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    slo[w] = lo;
    shi[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    lo = fminf(fminf(slo[0], slo[1]), fminf(slo[2], slo[3]));
    hi = fmaxf(fmaxf(shi[0], shi[1]), fmaxf(shi[2], shi[3]));
    atomicMin(&mm[0], __float_as_uint(lo));
    atomicMax(&mm[1], __float_as_uint(hi));
  }
}

__global__ __launch_bounds__(256) void flow_mask_kernel(const float* __restrict__ err,
                                                        const unsigned* __restrict__ mm,
                                                        int64_t n, float thr,
                                                        uint8_t* __restrict__ mask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float lo = __uint_as_float(mm[0]), hi = __uint_as_float(mm[1]);
  // (err - min) / (max - min) if max > min else 0  (two IEEE ops, as torch evaluates them)
  const float v = hi > lo ? (err[i] - lo) / (hi - lo) : 0.f;
  mask[i] = v > thr ? 1 : 0;
}

template <typename DT>
__global__ __launch_bounds__(256) void apply_mask_kernel(const uint8_t* __restrict__ mask,
                                                         float* __restrict__ C,
                                                         float* __restrict__ Q,
                                                         DT* __restrict__ D, int64_t hw,
                                                         int64_t total, int fdim, float value) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  if (!mask[i % hw]) return;
  C[i] = value;
  if (Q) Q[i] = value;
  if (D) {
    DT* d = D + i * fdim;
    for (int k = 0; k < fdim; k++) d[k] = (DT)0.f;
  }
}

// Ego-motion flow: pixel (x, y) of frame i with depth z = pts[p].z (mono res_i pts3d)
// lands at K_j (R_ji d K_i^-1 [x y 1]^T + t_ji) in frame j; flow = projection - (x, y).
// prm: R_ji (9, row-major), t_ji (3), K_j (9), K_i^-1 (9) = 30 floats in device memory
// (so a captured graph reads the current pose).  Out: [3][n] (flow x, flow y, valid).
__global__ __launch_bounds__(256) void ego_flow_kernel(const float* __restrict__ pts,
                                                       const float* __restrict__ prm, int w,
                                                       int64_t n, float* __restrict__ ego) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = (float)(i % w), y = (float)(i / w);
  const float z = pts[3 * i + 2];
  // inv_depth = 1 / (depth + 1e-6) (:586), then depth = 1 / inv_depth inside the warp
  const float inv_depth = 1.0f / (z + 1e-6f);
  const float d = 1.0f / inv_depth;
  const float* R = prm;
  const float* t = prm + 9;
  const float* Kj = prm + 12;
  const float* Ki = prm + 21;
  const float cx = d * (Ki[0] * x + Ki[1] * y + Ki[2]);
  const float cy = d * (Ki[3] * x + Ki[4] * y + Ki[5]);
  const float cz = d * (Ki[6] * x + Ki[7] * y + Ki[8]);
  const float qx = R[0] * cx + R[1] * cy + R[2] * cz + t[0];
  const float qy = R[3] * cx + R[4] * cy + R[5] * cz + t[1];
  const float qz = R[6] * cx + R[7] * cy + R[8] * cz + t[2];
  const float px = Kj[0] * qx + Kj[1] * qy + Kj[2] * qz;
  const float py = Kj[3] * qx + Kj[4] * qy + Kj[5] * qz;
  const float pz = Kj[6] * qx + Kj[7] * qy + Kj[8] * qz;
  const bool ok = pz > 1e-6f;
  ego[i] = ok ? px / pz - x : 0.f;
  ego[n + i] = ok ? py / pz - y : 0.f;
  ego[2 * n + i] = ok ? 1.f : 0.f;
}

}  // namespace

extern "C" int m3s_ego_flow(const float* d_pts, const float* d_params, int64_t h, int64_t w,
                            float* d_ego, void* stream) {
  if (!d_pts || !d_params || !d_ego || h <= 0 || w <= 0) return M3S_ERR_INVALID_ARG;
  const int64_t n = h * w;
  hipLaunchKernelGGL(ego_flow_kernel, dim3(m3s_div_up(n, 256)), dim3(256), 0,
                     m3s_stream(stream), d_pts, d_params, (int)w, n, d_ego);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_flow_error_mask(const float* d_flow, const float* d_ego_flow, int64_t n,
                                   float threshold, uint8_t* d_mask, float* d_workspace,
                                   void* stream) {
  if (!d_flow || !d_ego_flow || !d_mask || !d_workspace || n <= 0) return M3S_ERR_INVALID_ARG;
  hipStream_t s = m3s_stream(stream);
  unsigned* mm = reinterpret_cast<unsigned*>(d_workspace);
  float* err = d_workspace + 64;
  hipLaunchKernelGGL(flow_err_init_kernel, dim3(1), dim3(64), 0, s, mm);
  hipLaunchKernelGGL(flow_err_kernel, dim3(m3s_div_up(n, 256)), dim3(256), 0, s, d_flow,
                     d_ego_flow, n, err, mm);
  hipLaunchKernelGGL(flow_mask_kernel, dim3(m3s_div_up(n, 256)), dim3(256), 0, s, err, mm, n,
                     threshold, d_mask);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_apply_dynamic_mask(const uint8_t* d_mask, float* d_C, float* d_Q, void* d_D,
                                      int D_is_f16, int64_t batch, int64_t hw, int64_t fdim,
                                      float value, int zero_descriptors, void* stream) {
  if (!d_mask || !d_C || batch <= 0 || hw <= 0 || fdim < 0) return M3S_ERR_INVALID_ARG;
  if (d_D && fdim == 0) return M3S_ERR_INVALID_ARG;
  (void)zero_descriptors;  // the reference zeroes D whenever it is given (:333-335)
  const int64_t total = batch * hw;
  dim3 grid(m3s_div_up(total, 256));
  hipStream_t s = m3s_stream(stream);
  if (D_is_f16)
    hipLaunchKernelGGL((apply_mask_kernel<_Float16>), grid, dim3(256), 0, s, d_mask, d_C, d_Q,
                       reinterpret_cast<_Float16*>(d_D), hw, total, (int)fdim, value);
  else
    hipLaunchKernelGGL((apply_mask_kernel<float>), grid, dim3(256), 0, s, d_mask, d_C, d_Q,
                       reinterpret_cast<float*>(d_D), hw, total, (int)fdim, value);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
