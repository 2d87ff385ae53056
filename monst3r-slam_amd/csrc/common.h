// Shared helpers for the MI355X (gfx950) HIP kernels of the MonST3R-SLAM hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/monst3r_slam_amd.h"

#define M3S_WAVE 64

#define M3S_LAUNCH_CHECK()                                  \
  do {                                                      \
    hipError_t e__ = hipGetLastError();                     \
    if (e__ != hipSuccess) return M3S_ERR_HIP;              \
  } while (0)

#define M3S_HIP_CHECK(x)                                    \
  do {                                                      \
    hipError_t e__ = (x);                                   \
    if (e__ != hipSuccess) return M3S_ERR_HIP;              \
  } while (0)

static inline hipStream_t m3s_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline unsigned m3s_div_up(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

// Full-wave (64-lane) butterfly sum; every lane ends with the total.
__device__ __forceinline__ float m3s_wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int m3s_wave_sum_int(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double m3s_wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
