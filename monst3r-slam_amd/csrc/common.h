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

// ---- step timeline (diagnostic, include/monst3r_slam_amd.h m3s_timeline_set) ----
// While a timeline buffer is set, each instrumented launch (GEMM, attention) takes the next
// slot: M3S_TL_SUB pairs of u64 s_memrealtime stamps (100 MHz), [0] = earliest block start
// (atomic min by one lane per block), [1] = latest wave end (atomic max by one lane per
// wave), block b updating pair b % M3S_TL_SUB — one address per launch took every block's
// atomics in series and stretched the step 1.4x.  The slot pointer travels in the kernel
// arguments, so a captured graph keeps its launches' slots; with no buffer set the pointer
// is null and the kernels only test it.
// A slot is M3S_TL_SLOT u64: the M3S_TL_SUB pairs, then a header the host fills before a
// replay — [0] a block-log buffer or 0, [1] its u32 record counter, [2] its capacity in
// records — through which the first wave of every block appends one 64-B record {start,
// end, slot address, HW_ID | XCC_ID << 32, phase marks 0-3} (bench.step_timeline: which
// CUs are busy when; the GEMM marks prologue issued / first K-tile ready / K-loop done /
// epilogue tile in LDS, s_memrealtime, 0 where a kernel sets none).
enum { M3S_TL_GEMM = 1, M3S_TL_ATTN = 2, M3S_TL_CONV = 3 };  // CONV: implicit 3x3 GEMM
#define M3S_TL_SUB 64
#define M3S_TL_SLOT (2 * M3S_TL_SUB + 4)
unsigned long long* m3s_timeline_take(int kind, double flops, int64_t d0, int64_t d1, int64_t d2,
                                        int64_t d3);  // capi.cpp; null when off

__device__ __forceinline__ unsigned long long* m3s_tl_pair(unsigned long long* tl) {
  return tl + 2 * ((blockIdx.x + blockIdx.y * 7) % M3S_TL_SUB);
}
__device__ __forceinline__ void m3s_tl_begin(unsigned long long* tl) {
  if (tl && threadIdx.x == 0)
    atomicMin(m3s_tl_pair(tl), (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
struct M3sTlEnd {  // stamps the wave's end on every return path
  unsigned long long* p;
  unsigned long long t0;
  unsigned long long ph[4] = {0ull, 0ull, 0ull, 0ull};
  __device__ __forceinline__ M3sTlEnd(unsigned long long* slot)
      : p(slot), t0(slot ? (unsigned long long)__builtin_amdgcn_s_memrealtime() : 0ull) {}
  // phase mark i (block log only; wave-uniform branch, nothing when the timeline is off)
  __device__ __forceinline__ void mark(int i) {
    if (p) ph[i] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ ~M3sTlEnd() {
    if (p && (threadIdx.x & 63) == 0) {
      const unsigned long long now = (unsigned long long)__builtin_amdgcn_s_memrealtime();
      atomicMax(m3s_tl_pair(p) + 1, now);
      unsigned long long* log =
          threadIdx.x == 0 ? reinterpret_cast<unsigned long long*>(p[2 * M3S_TL_SUB]) : nullptr;
      if (log) {
        unsigned* cnt = reinterpret_cast<unsigned*>(p[2 * M3S_TL_SUB + 1]);
        const unsigned i = atomicAdd(cnt, 1u);
        if (i < (unsigned)p[2 * M3S_TL_SUB + 2]) {
          unsigned hw, xcc;
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
          asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
          ulonglong2* r = reinterpret_cast<ulonglong2*>(log + 8 * (size_t)i);
          r[0] = make_ulonglong2(t0, now);
          r[1] = make_ulonglong2(reinterpret_cast<unsigned long long>(p),
                                 (unsigned long long)hw | ((unsigned long long)xcc << 32));
          r[2] = make_ulonglong2(ph[0], ph[1]);
          r[3] = make_ulonglong2(ph[2], ph[3]);
        }
      }
    }
  }
};
