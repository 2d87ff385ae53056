// Library-level entry points of the C ABI (include/monst3r_slam_amd.h).
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

extern "C" int m3s_version(void) { return (0 << 16) | (1 << 8) | 0; }

extern "C" int m3s_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
