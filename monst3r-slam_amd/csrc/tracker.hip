// Frontend pose tracker (FrameTracker2.opt_pose_ray_dist_sim3 / opt_pose_calib_sim3,
// tracker2.py:299-409), ONE gfx950 kernel per Gauss-Newton iteration:
//   every workgroup: per point residual (4 rows ray+dist, or 3 rows u,v,log z), Jacobian
//     J = -d(rd)/dP * [I, -[P]x, P], Huber-robust whitening, and the 28+7+1 sums of A^T A,
//     -A^T b and 0.5 b^T b; wave64 butterfly + LDS → one partial row per workgroup;
//   the LAST workgroup to finish (agent-scope release / ticket / acquire,
//     cdna_hip_programming.md §6 G16): f64 reduction of the partials in fixed block order
//     (deterministic), 7x7 Cholesky, tau = H^-1 g, T <- Exp(tau) * T (lietorch retr),
//     check_convergence (nonlinear_optimizer.py:5-25, NaN-aware on iteration 0), done flag.
// Default: all iterations in one persistent launch (track_persistent_kernel, grid
// barrier per iteration, every workgroup takes the same step); M3S_TRACK_PERSISTENT=0
// enqueues one launch per iteration instead (the remaining ones return at entry once
// the done flag is set).  If the persistent launch loses co-residency (a barrier wait
// times out because not all of its workgroups got a CU next to the concurrently running
// kernels) it stops with a consistent state (pose after the last completed iteration) and
// the finish launch runs the remaining iterations in one 1024-thread workgroup; info[3]
// reports it.  A timeout is never a Cholesky failure.
#include <algorithm>
#include "common.h"
#include "sim3.h"

namespace {

constexpr int kThreads = 256;
constexpr int kBlocks = 512;
constexpr int kPersistentBlocks = 256;  // one per CU: co-resident next to other kernels
constexpr int kAcc = 36;  // 28 H upper, 7 g, 1 cost
static_assert(kAcc % 4 == 0, "partial rows are read as float4");

enum : int { TRACK_RAYS = 0, TRACK_CALIB = 1 };

struct TrackState {
  float T[8];        // current T_CkCf
  double old_cost;
  int done, fail, iters, conv;
  unsigned ticket;   // workgroups of the current iteration that have published partials
  int abort;         // persistent launch: a barrier wait timed out (co-residency lost)
  int recovered;     // iterations the finish launch ran after an aborted persistent launch
};

struct TrackParams {
  float si0, si1;  // 1/sigma for the two residual groups
  float huber_k;
  float fx, fy, cx, cy;  // calib only (read from K on device in init)
  float border, depth_eps;
  int h, w;
};

__device__ __forceinline__ float huber_w(float r, float k) {
  // nonlinear_optimizer.huber: 1 if |r| < k else k / |r|
  const float a = fabsf(r);
  return a < k ? 1.0f : k / a;
}

__device__ __forceinline__ void acc_row(float* acc, float ws, const float* J, float r) {
  // A_row = ws * J_row, b = ws * r
  float a[7];
#pragma unroll
  for (int n = 0; n < 7; n++) a[n] = ws * J[n];
  const float bb = ws * r;
  int l = 0;
#pragma unroll
  for (int n = 0; n < 7; n++) {
#pragma unroll
    for (int m = 0; m <= n; m++) {
      acc[l] += a[n] * a[m];
      l++;
    }
  }
#pragma unroll
  for (int n = 0; n < 7; n++) acc[28 + n] -= a[n] * bb;
  acc[35] += 0.5f * bb * bb;
}

// J row = -(d row) * [I, -[P]x, P], with d = d(residual row)/dP (1x3)
__device__ __forceinline__ void jac_row(const float* d, const float* P, float* J) {
  J[0] = -d[0];
  J[1] = -d[1];
  J[2] = -d[2];
  // d * (-[P]x): -[P]x = [[0, z, -y], [-z, 0, x], [y, -x, 0]]
  J[3] = -(d[1] * -P[2] + d[2] * P[1]);
  J[4] = -(d[0] * P[2] + d[2] * -P[0]);
  J[5] = -(d[0] * -P[1] + d[1] * P[0]);
  J[6] = -(d[0] * P[0] + d[1] * P[1] + d[2] * P[2]);
}

__global__ __launch_bounds__(256) void track_init_kernel(const float* __restrict__ Twc_k,
                                                         const float* __restrict__ Twc_f,
                                                         TrackState* st, uint4* gran,
                                                         int gran_vec) {
  // the persistent launch's hand-off granules start zeroed (was a memset node)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < gran_vec; i += gridDim.x * 256)
    gran[i] = make_uint4(0u, 0u, 0u, 0u);
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  // T_CkCf = T_WCk^-1 * T_WCf
  m3s_rel_sim3<float>(Twc_k, Twc_k + 3, Twc_k[7], Twc_f, Twc_f + 3, Twc_f[7], st->T, st->T + 3,
                      st->T + 7);
  st->old_cost = __builtin_inf();
  st->done = 0;
  st->fail = 0;
  st->iters = 0;
  st->conv = 0;
  st->ticket = 0;
  st->abort = 0;
  st->recovered = 0;
}

__device__ void track_solve(TrackState* st, const float* partial, int nblocks, float rel_error,
                            float delta_norm);

// per-point residuals / Jacobians of the points k = first, first + stride, ... into acc
template <int MODE>
__device__ __forceinline__ void track_points(const float* T, const TrackParams& prm,
                                             const float* __restrict__ Xf,
                                             const float* __restrict__ Xk,
                                             const float* __restrict__ Qk,
                                             const uint8_t* __restrict__ valid,
                                             const float* __restrict__ meas_k,
                                             const uint8_t* __restrict__ valid_meas, int64_t n,
                                             float* acc, int64_t first, int64_t stride) {
  for (int64_t k = first; k < n; k += stride) {
    const float X[3] = {Xf[3 * k], Xf[3 * k + 1], Xf[3 * k + 2]};
    float P[3];
    m3s_act_sim3<float>(T, T + 3, T[7], X, P);
    const float vq = (valid[k] ? 1.f : 0.f) * sqrtf(Qk[k]);
    if (MODE == TRACK_RAYS) {
      // rd_k (precomputed in the reference, tracker2.py:327)
      const float K3[3] = {Xk[3 * k], Xk[3 * k + 1], Xk[3 * k + 2]};
      const float dk = sqrtf(K3[0] * K3[0] + K3[1] * K3[1] + K3[2] * K3[2]);
      const float dk_inv = 1.0f / dk;
      const float d = sqrtf(P[0] * P[0] + P[1] * P[1] + P[2] * P[2]);
      const float d_inv = 1.0f / d;
      const float r[3] = {d_inv * P[0], d_inv * P[1], d_inv * P[2]};
      const float res[4] = {dk_inv * K3[0] - r[0], dk_inv * K3[1] - r[1], dk_inv * K3[2] - r[2],
                            dk - d};
      const float d_inv2 = d_inv * d_inv;
      const float si[4] = {prm.si0 * vq, prm.si0 * vq, prm.si0 * vq, prm.si1 * vq};
#pragma unroll
      for (int row = 0; row < 4; row++) {
        float drow[3];
        if (row < 3) {
#pragma unroll
          for (int c = 0; c < 3; c++)
            drow[c] = d_inv * ((row == c ? 1.f : 0.f) - d_inv2 * (P[row] * P[c]));
        } else {
          drow[0] = r[0];
          drow[1] = r[1];
          drow[2] = r[2];
        }
        float J[7];
        jac_row(drow, P, J);
        const float wr = si[row] * res[row];
        const float ws = si[row] * sqrtf(huber_w(wr, prm.huber_k));
        acc_row(acc, ws, J, res[row]);
      }
    } else {
      const float x = P[0], y = P[1], z = P[2];
      // p = K P / (K P)_z  (geometry.project_calib)
      const float pu = prm.fx * x + 0.f * y + prm.cx * z;
      const float pv = 0.f * x + prm.fy * y + prm.cy * z;
      const float pw = 0.f * x + 0.f * y + 1.f * z;
      const float u = pu / pw, v = pv / pw;
      const bool valid_u = (u > prm.border) && (u < (float)(prm.w - 1) - prm.border);
      const bool valid_v = (v > prm.border) && (v < (float)(prm.h - 1) - prm.border);
      const bool valid_z = z > prm.depth_eps;
      const float logz = valid_z ? logf(z) : 0.f;
      const float z_inv = 1.0f / z;
      const bool v2 = valid_u && valid_v && valid_z && (valid_meas[k] != 0);
      const float vq2 = v2 ? vq : 0.f;
      const float res[3] = {meas_k[3 * k] - u, meas_k[3 * k + 1] - v, meas_k[3 * k + 2] - logz};
      const float d0[3] = {prm.fx * z_inv, 0.f * z_inv, (-prm.fx * x * z_inv) * z_inv};
      const float d1[3] = {0.f * z_inv, prm.fy * z_inv, (-prm.fy * y * z_inv) * z_inv};
      const float d2[3] = {0.f, 0.f, z_inv};
      const float* drows[3] = {d0, d1, d2};
      const float si[3] = {prm.si0 * vq2, prm.si0 * vq2, prm.si1 * vq2};
#pragma unroll
      for (int row = 0; row < 3; row++) {
        float J[7];
        jac_row(drows[row], P, J);
        const float wr = si[row] * res[row];
        const float ws = si[row] * sqrtf(huber_w(wr, prm.huber_k));
        acc_row(acc, ws, J, res[row]);
      }
    }
  }
}

// Reduce-scatter of the 36 sums over a wave: each butterfly step halves the values a lane
// keeps (the lane's bit picks the half) and adds the partner's copy of that half — 32 + 16
// + 8 + 4 + 2 + 1 shuffles for the (zero-padded) 64 values instead of 36 x 6.  Lane l < 36
// then holds the wave's sum of value l (fixed order: deterministic).
template <typename F>
__device__ __forceinline__ F wave_reduce_scatter36(const F* acc) {
  const int lane = threadIdx.x & 63;
  F v[64];
#pragma unroll
  for (int j = 0; j < 64; j++) v[j] = j < kAcc ? acc[j] : F(0);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int j = 0; j < o; j++) {
      const F keep = hi ? v[j + o] : v[j];
      const F send = hi ? v[j] : v[j + o];
      v[j] = keep + __shfl_xor(send, o, 64);
    }
  }
  return v[0];   // lane l: value index l (bit k of l chose the half at step 2^k)
}

// the workgroup's 36 sums → out[0..35] (threads < kAcc write): per-wave reduce-scatter,
// then the waves' rows summed in wave order through LDS
template <int NT>
__device__ __forceinline__ void block_partial(const float* acc, float* out) {
  __shared__ float red[NT / M3S_WAVE][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  red[wid][lane] = wave_reduce_scatter36<float>(acc);
  __syncthreads();
  if (threadIdx.x < kAcc) {
    float v = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NT / M3S_WAVE; w++) v += red[w][threadIdx.x];
    out[threadIdx.x] = v;
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void track_iter_kernel(
    TrackState* __restrict__ st, TrackParams prm, const float* __restrict__ K,
    const float* __restrict__ Xf, const float* __restrict__ Xk, const float* __restrict__ Qk,
    const uint8_t* __restrict__ valid, const float* __restrict__ meas_k,
    const uint8_t* __restrict__ valid_meas, int64_t n, float* __restrict__ partial,
    float rel_error, float delta_norm) {
  if (st->done) return;
  if (MODE == TRACK_CALIB) {
    prm.fx = K[0];
    prm.fy = K[4];
    prm.cx = K[2];
    prm.cy = K[5];
  }
  float T[8];
#pragma unroll
  for (int i = 0; i < 8; i++) T[i] = st->T[i];
  float acc[kAcc];
#pragma unroll
  for (int l = 0; l < kAcc; l++) acc[l] = 0.f;

  track_points<MODE>(T, prm, Xf, Xk, Qk, valid, meas_k, valid_meas, n, acc,
                     (int64_t)blockIdx.x * kThreads + threadIdx.x, (int64_t)gridDim.x * kThreads);
  block_partial<kThreads>(acc, partial + blockIdx.x * kAcc);
  // publish this workgroup's partial row; the last to arrive reduces and solves
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  track_solve(st, partial, (int)gridDim.x, rel_error, delta_norm);
}

// f64 reduction of nblocks partial rows in fixed order (deterministic; every workgroup
// that runs it gets the same bits): thread (value l, group g) of the first 7 x 36 threads
// sums rows g, g + 7, ... of column l — all its loads in flight at once — then the 7 group
// sums of each value are added in group order.  The 36 sums land in sacc (shared).
__device__ void reduce_partials(const float* partial, int nblocks, double* sacc) {
  constexpr int G = kThreads / kAcc;   // 7
  const int tid = threadIdx.x;
  __shared__ double tmp[G][kAcc];
  if (tid < G * kAcc) {
    const int l = tid % kAcc, g = tid / kAcc;
    double v = 0.0;
    int b = g;
    for (; b + 3 * G < nblocks; b += 4 * G) {
      const float r0 = partial[(size_t)b * kAcc + l];
      const float r1 = partial[(size_t)(b + G) * kAcc + l];
      const float r2 = partial[(size_t)(b + 2 * G) * kAcc + l];
      const float r3 = partial[(size_t)(b + 3 * G) * kAcc + l];
      v += (double)r0;
      v += (double)r1;
      v += (double)r2;
      v += (double)r3;
    }
    for (; b < nblocks; b += G) v += (double)partial[(size_t)b * kAcc + l];
    tmp[g][l] = v;
  }
  __syncthreads();
  if (tid < kAcc) {
    double t = 0.0;
#pragma unroll
    for (int g = 0; g < G; g++) t += tmp[g][tid];
    sacc[tid] = t;
  }
  __syncthreads();
}

// One Gauss-Newton step on the reduced sums (one thread): 7x7 Cholesky (failure → the
// reference's CholeskyError, frame lost), tau = H^-1 g, T <- Exp(tau) * T (lietorch retr),
// check_convergence (nonlinear_optimizer.py:5-25; rel_dec is NaN on iteration 0).
// Returns 0 = continue, 1 = converged, 2 = Cholesky failure.
__device__ int gn_step(const double* sacc, float* T, double* old_cost, float rel_error,
                       float delta_norm) {
  double H[7][7], g[7];
  int l = 0;
  for (int n = 0; n < 7; n++)
    for (int m = 0; m <= n; m++) {
      H[n][m] = sacc[l];
      H[m][n] = sacc[l];
      l++;
    }
  for (int n = 0; n < 7; n++) g[n] = sacc[28 + n];
  const double new_cost = sacc[35];
  double L[7][7] = {};
  for (int j = 0; j < 7; j++) {
    double s = H[j][j];
    for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
    if (!(s > 0.0)) return 2;
    L[j][j] = sqrt(s);
    for (int i = j + 1; i < 7; i++) {
      double t = H[i][j];
      for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
      L[i][j] = t / L[j][j];
    }
  }
  double y[7], x[7];
  for (int i = 0; i < 7; i++) {
    double t = g[i];
    for (int k = 0; k < i; k++) t -= L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
  for (int i = 6; i >= 0; i--) {
    double t = y[i];
    for (int k = i + 1; k < 7; k++) t -= L[k][i] * x[k];
    x[i] = t / L[i][i];
  }
  float tau[7];
  for (int i = 0; i < 7; i++) tau[i] = (float)x[i];
  float t1[3], q1[4], s1;
  m3s_retr_sim3<float>(tau, T, T + 3, T[7], t1, q1, &s1);
  for (int i = 0; i < 3; i++) T[i] = t1[i];
  for (int i = 0; i < 4; i++) T[3 + i] = q1[i];
  T[7] = s1;
  const double rel_dec = fabs((*old_cost - new_cost) / *old_cost);
  float dn = 0.f;
  for (int i = 0; i < 7; i++) dn += tau[i] * tau[i];
  dn = sqrtf(dn);
  *old_cost = new_cost;
  return (rel_dec < (double)rel_error || dn < delta_norm) ? 1 : 0;
}

__device__ void track_solve(TrackState* st, const float* partial, int nblocks, float rel_error,
                            float delta_norm) {
  __shared__ double sacc[kAcc];
  reduce_partials(partial, nblocks, sacc);
  if (threadIdx.x != 0) return;
  st->ticket = 0;  // next iteration (next launch) counts from zero again
  float T[8];
  for (int i = 0; i < 8; i++) T[i] = st->T[i];
  double oc = st->old_cost;
  const int r = gn_step(sacc, T, &oc, rel_error, delta_norm);
  if (r == 2) {
    st->fail = 1;
    st->done = 1;
    return;
  }
  for (int i = 0; i < 8; i++) st->T[i] = T[i];
  st->old_cost = oc;
  st->iters += 1;
  if (r == 1) {
    st->conv = 1;
    st->done = 1;
  }
}

// All Gauss-Newton iterations in ONE launch: nb co-resident workgroups (nb <= 256, a few
// registers' worth of occupancy, so they fit beside whatever else runs) accumulate their
// points' 36 sums (per-wave reduce-scatter), publish them as tagged 8-byte granules
// (write-through atomic stores: the data is the flag — no fence, no barrier counter), and
// EVERY workgroup sweeps all granules until each carries this iteration's tag, sums them in
// the same fixed order and takes the same step — the pose never needs a broadcast and the
// next iteration starts straight away.  Granule slots alternate with the iteration parity
// (a workgroup can be at most one iteration ahead) and are zeroed per call (memset node).
// tools/track_bench.py --stamps: 38 → 11 µs per iteration at 384x512 (the fence-ordered
// barrier + a shuffle reduction per value were 27 µs of it).
// Exit: convergence, Cholesky failure, max_iters, or a sweep beyond `spin_limit` granule
// sweeps (co-residency broken; a sweep is up to one agent-scope load per producer workgroup,
// so the wait before recovery is spin_limit x one sweep's latency, not a fixed time) — that
// workgroup raises st->abort, every other workgroup sees it in its own sweep (or at entry,
// if it only got a CU after the others left) and leaves too.  Another workgroup may still
// see every granule of the iteration that timed out (the last one can land just as the
// waiter gives up) and take that step before it notices the abort one iteration later:
// correctness does not rest on "nobody completes it", but on workgroup 0 alone writing
// back ITS OWN consistent (pose, iteration, cost) with done = 0; track_finish_kernel then
// runs the remaining iterations from that state.
// `abort_at` >= 0 forces that exit at iteration abort_at (tests of the recovery path).
#ifdef M3S_TRACK_STAMPS
// debug build (tools/track_bench.py --stamps): workgroup 0, lane 0, s_memrealtime (100 MHz)
// at each phase boundary of the first 8 iterations
__device__ long long g_track_stamps[8 * 8];
#define M3S_TS(it, ph) \
  if (blockIdx.x == 0 && threadIdx.x == 0 && (it) < 8) \
    g_track_stamps[(it) * 8 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime();
#else
#define M3S_TS(it, ph)
#endif

template <int MODE>
__global__ __launch_bounds__(kThreads) void track_persistent_kernel(
    TrackState* __restrict__ st, TrackParams prm, const float* __restrict__ K,
    const float* __restrict__ Xf, const float* __restrict__ Xk, const float* __restrict__ Qk,
    const uint8_t* __restrict__ valid, const float* __restrict__ meas_k,
    const uint8_t* __restrict__ valid_meas, int64_t n, unsigned long long* __restrict__ gran,
    int max_iters, float rel_error, float delta_norm, long spin_limit, int abort_at) {
  if (MODE == TRACK_CALIB) {
    prm.fx = K[0];
    prm.fy = K[4];
    prm.cx = K[2];
    prm.cy = K[5];
  }
  constexpr int G = kThreads / kAcc;                      // 7 row groups per value
  constexpr int R = (kPersistentBlocks + G - 1) / G;      // rows per (value, group) thread
  __shared__ float sT[8];
  __shared__ float s_row[kAcc];
  __shared__ double tmp[G][kAcc];
  __shared__ double sacc[kAcc];
  __shared__ int s_status;
  const int nb = gridDim.x;
  const int tid = threadIdx.x;
  float T[8];
#pragma unroll
  for (int i = 0; i < 8; i++) T[i] = st->T[i];
  double old_cost = st->old_cost;
  int it = 0, status = 0;
  if (tid == 0)
    s_status = __hip_atomic_load(&st->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 3 : 0;
  __syncthreads();
  if (s_status == 3) return;  // started after the others gave up: nothing to contribute
  for (; it < max_iters; it++) {
    M3S_TS(it, 0);
    float acc[kAcc];
#pragma unroll
    for (int l = 0; l < kAcc; l++) acc[l] = 0.f;
    track_points<MODE>(T, prm, Xf, Xk, Qk, valid, meas_k, valid_meas, n, acc,
                       (int64_t)blockIdx.x * kThreads + tid, (int64_t)nb * kThreads);
    M3S_TS(it, 1);
    block_partial<kThreads>(acc, s_row);
    __syncthreads();
    M3S_TS(it, 2);
    // publish the 36 sums as granules {tag = iteration + 1, value}: the data is the flag —
    // one 8-byte relaxed agent-scope atomic store each (write-through), no fence, no counter
    // (cdna_hip_programming.md §6 Guideline 16, R2).  Slots alternate with the iteration
    // parity: a workgroup can be at most one iteration ahead of the slowest reader.
    unsigned long long* gslot = gran + (size_t)(it & 1) * kPersistentBlocks * kAcc;
    const unsigned long long tag = (unsigned long long)(it + 1) << 32;
    const bool forced = it == abort_at;
    if (tid < kAcc && !forced)
      __hip_atomic_store(&gslot[(size_t)blockIdx.x * kAcc + tid],
                         tag | __builtin_bit_cast(unsigned, s_row[tid]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    // sweep: thread (value l, group g) re-reads its rows g, g + 7, ... until every tag is this
    // iteration's, then sums them in row order (f64) — the same bits in every workgroup
    int timeout = forced ? 1 : 0;
    if (tid < G * kAcc && !forced) {
      const int l = tid % kAcc, g = tid / kAcc;
      unsigned long long x[R];
      for (long spins = 0;; spins++) {
        bool ok = true;
#pragma unroll
        for (int r = 0; r < R; r++) {
          const int b = g + r * G;
          x[r] = b < nb ? __hip_atomic_load(&gslot[(size_t)b * kAcc + l], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : tag;
          ok = ok && ((x[r] & 0xffffffff00000000ull) == tag);
        }
        if (ok) break;
        if (spins >= spin_limit ||
            __hip_atomic_load(&st->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          timeout = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < R; r++)
        if (g + r * G < nb) v += (double)__builtin_bit_cast(float, (unsigned)x[r]);
      tmp[g][l] = v;
    }
    if (__syncthreads_or(timeout)) {
      if (tid == 0) __hip_atomic_store(&st->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      status = 3;
      break;
    }
    M3S_TS(it, 3);
    if (tid < kAcc) {
      double t = 0.0;
#pragma unroll
      for (int g = 0; g < G; g++) t += tmp[g][tid];
      sacc[tid] = t;
    }
    __syncthreads();
    M3S_TS(it, 4);
    if (tid == 0) {
      const int r = gn_step(sacc, T, &old_cost, rel_error, delta_norm);
      M3S_TS(it, 5);
      s_status = r;
      if (r != 2)
        for (int i = 0; i < 8; i++) sT[i] = T[i];
    }
    __syncthreads();
    M3S_TS(it, 6);
    status = s_status;
    if (status == 2) break;
#pragma unroll
    for (int i = 0; i < 8; i++) T[i] = sT[i];
    if (status == 1) {
      it++;
      break;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    for (int i = 0; i < 8; i++) st->T[i] = T[i];
    st->old_cost = old_cost;
    st->iters = it;
    st->fail = status == 2 ? 1 : 0;
    st->conv = status == 1 ? 1 : 0;
    st->done = status == 3 ? 0 : 1;  // aborted: track_finish_kernel continues from here
  }
}

constexpr int kFinishThreads = 1024;

// Outputs T_WCf / T_CkCf / info.  If the iterations did not finish (persistent launch
// aborted, st->done == 0 with iterations left) this single workgroup runs the rest: same
// residuals and step, the points' sums in one 1024-thread partial (fp32 rounding differs
// from the multi-workgroup order, as between the two launch modes).
template <int MODE>
__global__ __launch_bounds__(kFinishThreads) void track_finish_kernel(
    const float* __restrict__ Twc_k, TrackState* st, TrackParams prm, const float* __restrict__ K,
    const float* __restrict__ Xf, const float* __restrict__ Xk, const float* __restrict__ Qk,
    const uint8_t* __restrict__ valid, const float* __restrict__ meas_k,
    const uint8_t* __restrict__ valid_meas, int64_t n, int max_iters, float rel_error,
    float delta_norm, float* __restrict__ T_WCf, float* __restrict__ T_CkCf,
    int* __restrict__ info) {
  __shared__ float srow[kAcc];
  __shared__ double sacc[kAcc];
  __shared__ float sT[8];
  __shared__ int s_go;
  if (threadIdx.x == 0) {
    s_go = !st->done && st->iters < max_iters;
    for (int i = 0; i < 8; i++) sT[i] = st->T[i];
  }
  __syncthreads();
  if (s_go) {
    if (MODE == TRACK_CALIB) {
      prm.fx = K[0];
      prm.fy = K[4];
      prm.cx = K[2];
      prm.cy = K[5];
    }
    int it = st->iters, status = 0, ran = 0;
    double old_cost = st->old_cost;
    for (; it < max_iters; it++) {
      float T[8];
#pragma unroll
      for (int i = 0; i < 8; i++) T[i] = sT[i];
      float acc[kAcc];
#pragma unroll
      for (int l = 0; l < kAcc; l++) acc[l] = 0.f;
      track_points<MODE>(T, prm, Xf, Xk, Qk, valid, meas_k, valid_meas, n, acc, threadIdx.x,
                         kFinishThreads);
      block_partial<kFinishThreads>(acc, srow);
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int l = 0; l < kAcc; l++) sacc[l] = (double)srow[l];
        status = gn_step(sacc, T, &old_cost, rel_error, delta_norm);
        if (status != 2)
          for (int i = 0; i < 8; i++) sT[i] = T[i];
        s_go = status;
      }
      __syncthreads();
      status = s_go;
      ran++;
      if (status == 2) break;
      if (status == 1) {
        it++;
        break;
      }
    }
    if (threadIdx.x == 0) {
      for (int i = 0; i < 8; i++) st->T[i] = sT[i];
      st->old_cost = old_cost;
      st->iters = it;
      st->fail = status == 2 ? 1 : 0;
      st->conv = status == 1 ? 1 : 0;
      st->recovered = ran;
      st->done = 1;
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  // T_WCf = T_WCk * T_CkCf: q = qk*q, s = sk*s, t = tk + sk * Rk t
  const float* Tk = Twc_k;
  float q[4], t[3];
  m3s_quat_comp<float>(Tk + 3, st->T + 3, q);
  m3s_act_so3<float>(Tk + 3, st->T, t);
  for (int i = 0; i < 3; i++) T_WCf[i] = Tk[i] + Tk[7] * t[i];
  for (int i = 0; i < 4; i++) T_WCf[3 + i] = q[i];
  T_WCf[7] = Tk[7] * st->T[7];
  for (int i = 0; i < 8; i++) T_CkCf[i] = st->T[i];
  info[0] = st->iters;
  info[1] = st->fail;
  info[2] = st->conv;
  info[3] = st->recovered;
}

struct Layout {
  size_t gran, state, partial, total;
};
Layout layout() {
  Layout L;
  L.gran = 0;  // zeroed per call by track_init_kernel: 2 parity slots of 256 x 36 granules
  L.state = sizeof(unsigned long long) * 2 * kPersistentBlocks * kAcc;
  L.partial = L.state + 512;
  L.total = L.partial + sizeof(float) * kBlocks * kAcc;
  return L;
}

template <int MODE>
int run_track(const float* Twc_k, const float* Twc_f, const float* Xf, const float* Xk,
              const float* Qk, const uint8_t* valid, const float* meas_k,
              const uint8_t* valid_meas, const float* K, int64_t n, TrackParams prm,
              int max_iters, float rel_error, float delta_norm, float* T_WCf, float* T_CkCf,
              int* info, void* ws, void* stream) {
  if (n < 1 || !Twc_k || !Twc_f || !Xf || !Qk || !valid || !T_WCf || !T_CkCf || !info || !ws)
    return M3S_ERR_INVALID_ARG;
  if (MODE == TRACK_RAYS && !Xk) return M3S_ERR_INVALID_ARG;
  if (MODE == TRACK_CALIB && (!meas_k || !valid_meas || !K)) return M3S_ERR_INVALID_ARG;
  hipStream_t s = m3s_stream(stream);
  const Layout L = layout();
  char* w = reinterpret_cast<char*>(ws);
  TrackState* st = reinterpret_cast<TrackState*>(w + L.state);
  float* partial = reinterpret_cast<float*>(w + L.partial);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(w + L.gran);
  const char* e = getenv("M3S_TRACK_PERSISTENT");  // A/B: 0 = one launch per iteration
  const bool persistent = !e || atoi(e) != 0;
  const int gran_vec = persistent && max_iters > 0 ? (int)((L.state - L.gran) / 16) : 0;
  hipLaunchKernelGGL(track_init_kernel, dim3(gran_vec ? 36 : 1), dim3(256), 0, s, Twc_k, Twc_f,
                     st, reinterpret_cast<uint4*>(w + L.gran), gran_vec);
  M3S_LAUNCH_CHECK();
  if (persistent) {
    int nb = (int)((n + kThreads - 1) / kThreads);
    if (nb > kPersistentBlocks) nb = kPersistentBlocks;
    if (const char* b = getenv("M3S_TRACK_BLOCKS"))  // tuning knob (tools/track_bench.py)
      nb = std::max(1, std::min(nb, atoi(b)));
    // debug knobs for the co-residency recovery path (tests): barrier poll limit, forced
    // abort at a given iteration
    const char* sl = getenv("M3S_TRACK_SPIN_LIMIT");
    const long spin_limit = sl ? atol(sl) : (1l << 22);
    const char* ab = getenv("M3S_TRACK_ABORT_AT");
    const int abort_at = ab ? atoi(ab) : -1;
    if (max_iters > 0) {
      hipLaunchKernelGGL(track_persistent_kernel<MODE>, dim3(nb), dim3(kThreads), 0, s, st, prm,
                         K, Xf, Xk, Qk, valid, meas_k, valid_meas, n, gran, max_iters,
                         rel_error, delta_norm, spin_limit, abort_at);
    }
    M3S_LAUNCH_CHECK();
  } else {
    int nb = (int)((n + kThreads - 1) / kThreads);
    if (nb > kBlocks) nb = kBlocks;
    for (int it = 0; it < max_iters; it++) {
      hipLaunchKernelGGL(track_iter_kernel<MODE>, dim3(nb), dim3(kThreads), 0, s, st, prm, K,
                         Xf, Xk, Qk, valid, meas_k, valid_meas, n, partial, rel_error,
                         delta_norm);
      M3S_LAUNCH_CHECK();
    }
  }
  hipLaunchKernelGGL(track_finish_kernel<MODE>, dim3(1), dim3(kFinishThreads), 0, s, Twc_k, st,
                     prm, K, Xf, Xk, Qk, valid, meas_k, valid_meas, n, max_iters, rel_error,
                     delta_norm, T_WCf, T_CkCf, info);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

}  // namespace

#ifdef M3S_TRACK_STAMPS
extern "C" int m3s_debug_track_stamps(long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_track_stamps), sizeof(long long) * 64) ==
                 hipSuccess ? 0 : -2;
}
#endif

extern "C" size_t m3s_track_workspace_bytes(int64_t n) {
  (void)n;
  return layout().total;
}

extern "C" int m3s_track_rays(const float* d_Twc_k, const float* d_Twc_f, const float* d_Xf,
                              const float* d_Xk, const float* d_Qk, const uint8_t* d_valid,
                              int64_t n, float sigma_ray, float sigma_dist, float huber_k,
                              int max_iters, float rel_error, float delta_norm, float* d_T_WCf,
                              float* d_T_CkCf, int* d_info, void* d_ws, void* stream) {
  TrackParams prm{};
  prm.si0 = 1.0f / sigma_ray;
  prm.si1 = 1.0f / sigma_dist;
  prm.huber_k = huber_k;
  return run_track<TRACK_RAYS>(d_Twc_k, d_Twc_f, d_Xf, d_Xk, d_Qk, d_valid, nullptr, nullptr,
                               nullptr, n, prm, max_iters, rel_error, delta_norm, d_T_WCf,
                               d_T_CkCf, d_info, d_ws, stream);
}

extern "C" int m3s_track_calib(const float* d_Twc_k, const float* d_Twc_f, const float* d_Xf,
                               const float* d_Qk, const uint8_t* d_valid, const float* d_meas_k,
                               const uint8_t* d_valid_meas_k, const float* d_K, int64_t n,
                               int64_t h, int64_t w, float sigma_pixel, float sigma_depth, float huber_k,
                               float pixel_border, float depth_eps, int max_iters,
                               float rel_error, float delta_norm, float* d_T_WCf,
                               float* d_T_CkCf, int* d_info, void* d_ws, void* stream) {
  TrackParams prm{};
  prm.si0 = 1.0f / sigma_pixel;
  prm.si1 = 1.0f / sigma_depth;
  prm.huber_k = huber_k;
  prm.border = pixel_border;
  prm.depth_eps = depth_eps;
  prm.h = (int)h;
  prm.w = (int)w;
  return run_track<TRACK_CALIB>(d_Twc_k, d_Twc_f, d_Xf, nullptr, d_Qk, d_valid, d_meas_k,
                                d_valid_meas_k, d_K, n, prm, max_iters, rel_error, delta_norm,
                                d_T_WCf, d_T_CkCf, d_info, d_ws, stream);
}
