// Library-level entry points of the C ABI (include/monst3r_slam_amd.h).
#include <mutex>
#include <vector>
#include <hip/hip_runtime.h>
#include "../../include/monst3r_slam_amd.h"

extern "C" const char* m3s_status_string(int status) {
  switch (status) {
    case M3S_OK: return "ok";
    case M3S_ERR_INVALID_ARG: return "invalid argument";
    case M3S_ERR_HIP: return "HIP runtime error";
    case M3S_ERR_TOO_LARGE: return "size exceeds kernel capacity";
    case M3S_ERR_NOT_PD: return "Cholesky failed (system not positive definite)";
    case M3S_ERR_NO_DEVICE: return "no HIP device";
    default: return "unknown status";
  }
}

extern "C" int m3s_version(void) { return (0 << 16) | (5 << 8) | 0; }

// ---- step timeline (common.h) ----
#define M3S_TL_SUB_HOST 64   // = M3S_TL_SUB: stamp pairs per slot
// The slot globals are shared by every host thread that launches (a mutex: two threads
// capturing at once must not hand out one slot twice or tear the metadata vectors).
namespace {
std::mutex g_tl_mu;
unsigned long long* g_tl = nullptr;
int g_tl_cap = 0, g_tl_n = 0;
std::vector<int> g_tl_kind;
std::vector<double> g_tl_flops;
std::vector<int64_t> g_tl_dims;
}  // namespace

unsigned long long* m3s_timeline_take(int kind, double flops, int64_t d0, int64_t d1, int64_t d2,
                                      int64_t d3) {
  std::lock_guard<std::mutex> lk(g_tl_mu);
  if (!g_tl || g_tl_n >= g_tl_cap) return nullptr;
  g_tl_kind.push_back(kind);
  g_tl_flops.push_back(flops);
  g_tl_dims.insert(g_tl_dims.end(), {d0, d1, d2, d3});
  return g_tl + (2 * M3S_TL_SUB_HOST + 4) * (int64_t)g_tl_n++;   // M3S_TL_SLOT u64 per slot
}

extern "C" int m3s_timeline_set(void* d_buf, int capacity) {
  if (d_buf && capacity <= 0) return M3S_ERR_INVALID_ARG;
  if (d_buf) {
    // every slot's 4-u64 header (block-log pointer, counter, capacity) starts zeroed: a
    // caller that fills only the stamp pairs (or allocates the slots uninitialised) gets no
    // block log instead of a garbage pointer dereferenced inside a captured step
    if (hipMemset2D(reinterpret_cast<char*>(d_buf) + 128 * 8, 132 * 8, 0,
                    4 * 8, (size_t)capacity) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      return M3S_ERR_INVALID_ARG;
  }
  std::lock_guard<std::mutex> lk(g_tl_mu);
  g_tl = reinterpret_cast<unsigned long long*>(d_buf);
  g_tl_cap = d_buf ? capacity : 0;
  if (d_buf) {
    g_tl_n = 0;
    g_tl_kind.clear();
    g_tl_flops.clear();
    g_tl_dims.clear();
  }
  return M3S_OK;
}

extern "C" int m3s_timeline_count(void) {
  std::lock_guard<std::mutex> lk(g_tl_mu);
  return g_tl_n;
}

extern "C" int m3s_timeline_meta(int* kinds, double* flops, int64_t* dims, int capacity) {
  if (!kinds || !flops || !dims || capacity < 0) return M3S_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_tl_mu);
  for (int i = 0; i < g_tl_n && i < capacity; i++) {
    kinds[i] = g_tl_kind[i];
    flops[i] = g_tl_flops[i];
    for (int j = 0; j < 4; j++) dims[4 * i + j] = g_tl_dims[4 * i + j];
  }
  return M3S_OK;
}

extern "C" int m3s_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
