// Backend Gauss-Newton over the keyframe graph, gfx950.
//
// Reference: gn_kernels.cu (ray_align_kernel :813-1138, calib_proj_kernel :1231-1543,
// point_align_kernel :455-723, drivers :725-811/:1140-1228/:1546-1638, Eigen host solve
// :57-159).  MI355X design:
//  * Algebra: every residual row has Ji = -Jj and Jj = M_i J' (M_i the reference's
//    apply_Sim3_adj_inv of pose i, linear in J').  So the 14x14 edge Hessian is
//    [[A,-A],[-A,A]] with A = M_i (sum w J'J'^T) M_i^T and g = (-M_i v', M_i v').
//    Per point we accumulate 28 + 7 f32 sums (not 105 + 14) and apply M_i once per
//    edge in f64 — the same quantity as the reference up to summation order.
//  * Parallelism: grid (E, S) — each edge's points split over S workgroups so that
//    E*S fills the 256 CUs; wave64 butterfly + LDS reduction per workgroup.
//  * Solve: a single-workgroup fp64 kernel assembles the dense 7(P-1) system, runs a
//    right-looking Cholesky, the two triangular solves, the retraction of poses 1..P-1
//    and the ||dx|| < delta test — all on device, no host round trip.  A device flag
//    makes later iterations' kernels exit at once, so max_iter launches need no sync.
#include <climits>
#include "common.h"
#include "sim3.h"

#pragma clang fp contract(off)

namespace {

constexpr int kEdgeThreads = 256;
constexpr int kSolveThreads = 1024;
constexpr int kAcc = 35;  // 28 upper-tri of sum w J'J'^T + 7 of sum w e J'

enum : int { MODE_RAYS = 0, MODE_CALIB = 1, MODE_POINTS = 2 };

struct GnParams {
  float s0_inv, s1_inv;  // sigma_ray_inv/sigma_dist_inv, pixel/depth, point/-
  float C_thresh, Q_thresh;
  int height, width, pixel_border;
  float z_eps;
};

struct GnWork {
  int* flags;          // [0] done, [1] not-PD seen, [2] unique count, [3] iterations
  int* rank_ii;        // [E]
  int* rank_jj;        // [E]
  float* partial;      // [E][S][kAcc]
  double* A;           // [n][n]
  double* bvec;        // [n]
  double* G;           // [E][kAcc] reduced per edge (scratch for the solve kernel)
};

// Huber weight (gn_kernels.cu:172-175).  The reference compares and divides in double
// (its 1.345 is a double literal); here the comparison is fp32 and exact (1.345f is the next
// float above 1.345, so r < 1.345 <=> r < 1.345f for every float r) and the weight is
// 1.345f * rcp(r) (v_rcp_f32, 1 ulp): six fp64 divisions per point were a third of the
// edge pass, and the correctly rounded fp32 division sequences another sixth.
__device__ __forceinline__ float huber_w(float r) {
  const float r_abs = fabsf(r);
  return r_abs < 1.345f ? 1.0f : 1.345f * __builtin_amdgcn_rcpf(r_abs);
}

// 1 / x and sqrt(x) of the residual normalisation.  These enter the residuals themselves
// (differences of unit rays ~1e-3): the 1-ulp v_rcp_f32 / v_sqrt_f32 bias them coherently
// over an edge's points (P = 19 chain: poses off by 8e-5), so they stay correctly rounded —
// the reference's 1.0 / x in double rounded to float differs from the fp32 quotient only
// where the double quotient rounds twice (<= 1 ulp, unbiased).
__device__ __forceinline__ float inv_f(float x) { return 1.0f / x; }
__device__ __forceinline__ float sqrt_f(float x) { return sqrtf(x); }

// Accumulate one weighted row into the 35 sums.  MASK (bit n: J[n] may be nonzero) is the
// row's compile-time sparsity: the zero entries' products are never formed (an exact zero
// added to a finite sum leaves it unchanged), which takes the rays rows from 35 to 15-19
// multiply-adds each.  Fused multiply-adds, as the reference's nvcc build contracts them.
template <int MASK>
__device__ __forceinline__ void acc_row(float* acc, float w, float e, const float* J) {
#pragma unroll
  for (int n = 0; n < 7; n++) {
    if (!((MASK >> n) & 1)) continue;
    const float wj = w * J[n];
#pragma unroll
    for (int m = 0; m <= n; m++)
      if ((MASK >> m) & 1) acc[n * (n + 1) / 2 + m] = __builtin_fmaf(wj, J[m], acc[n * (n + 1) / 2 + m]);
  }
  const float we = w * e;
#pragma unroll
  for (int n = 0; n < 7; n++)
    if ((MASK >> n) & 1) acc[28 + n] = __builtin_fmaf(we, J[n], acc[28 + n]);
}

// One point's residual rows accumulated into the 35 sums (per-point bodies of
// ray_align_kernel gn_kernels.cu:813-1138, calib_proj_kernel :1231-1543, point_align_kernel :455-723).
template <int MODE>
__device__ __forceinline__ void point_acc(float* acc, bool vm, int64_t ind, const float* Xi,
                                          float ci, const float* Xj, float q, float cj,
                                          const float* tij, const float* qij, float sij,
                                          const GnParams& prm, float fx, float fy, float cx,
                                          float cy) {
  float P[3];
  m3s_act_sim3<float>(tij, qij, sij, Xj, P);
  bool valid = vm & (q > prm.Q_thresh) & (ci > prm.C_thresh) & (cj > prm.C_thresh);

  if (MODE == MODE_RAYS) {
    const float n2i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
    const float n1i = sqrt_f(n2i);
    const float n1i_inv = inv_f(n1i);
    const float n2j = P[0] * P[0] + P[1] * P[1] + P[2] * P[2];
    const float n1j = sqrt_f(n2j);
    const float n1j_inv = inv_f(n1j);
    const float rj[3] = {n1j_inv * P[0], n1j_inv * P[1], n1j_inv * P[2]};
    const float err[4] = {rj[0] - n1i_inv * Xi[0], rj[1] - n1i_inv * Xi[1],
                          rj[2] - n1i_inv * Xi[2], n1j - n1i};
    const float sq = sqrt_f(q);
    const float swr = valid ? prm.s0_inv * sq : 0.f;
    const float swd = valid ? prm.s1_inv * sq : 0.f;
    const float cr = swr * swr, cd = swd * swd;
    const float w[4] = {huber_w(swr * err[0]) * cr, huber_w(swr * err[1]) * cr,
                        huber_w(swr * err[2]) * cr, huber_w(swd * err[3]) * cd};
    const float n3_inv = n1j_inv / n2j;
    const float dxx = n1j_inv - P[0] * P[0] * n3_inv;
    const float dyy = n1j_inv - P[1] * P[1] * n3_inv;
    const float dzz = n1j_inv - P[2] * P[2] * n3_inv;
    const float dxy = -P[0] * P[1] * n3_inv;
    const float dxz = -P[0] * P[2] * n3_inv;
    const float dyz = -P[1] * P[2] * n3_inv;
    const float J0[7] = {dxx, dxy, dxz, 0.f, rj[2], -rj[1], 0.f};
    const float J1[7] = {dxy, dyy, dyz, -rj[2], 0.f, rj[0], 0.f};
    const float J2[7] = {dxz, dyz, dzz, rj[1], -rj[0], 0.f, 0.f};
    const float J3[7] = {rj[0], rj[1], rj[2], 0.f, 0.f, 0.f, n1j};
    acc_row<0x37>(acc, w[0], err[0], J0);
    acc_row<0x2F>(acc, w[1], err[1], J1);
    acc_row<0x1F>(acc, w[2], err[2], J2);
    acc_row<0x47>(acc, w[3], err[3], J3);
  } else if (MODE == MODE_CALIB) {
    const int u_t = (int)ind % prm.width;  // ind < num_points < 2^31
    const int v_t = (int)ind / prm.width;
    const bool valid_z = (P[2] > prm.z_eps) && (Xi[2] > prm.z_eps);
    const float zj_inv = valid_z ? inv_f(P[2]) : 0.f;
    const float zj_log = valid_z ? logf(P[2]) : 0.f;
    const float zi_log = valid_z ? logf(Xi[2]) : 0.f;
    const float xz = P[0] * zj_inv;
    const float yz = P[1] * zj_inv;
    const float u = fx * xz + cx;
    const float v = fy * yz + cy;
    const bool valid_u = (u > (float)prm.pixel_border) &&
                         (u < (float)(prm.width - 1 - prm.pixel_border));
    const bool valid_v = (v > (float)prm.pixel_border) &&
                         (v < (float)(prm.height - 1 - prm.pixel_border));
    valid = valid & valid_u & valid_v & valid_z;
    const float err[3] = {u - (float)u_t, v - (float)v_t, zj_log - zi_log};
    const float sq = sqrt_f(q);
    const float swp = valid ? prm.s0_inv * sq : 0.f;
    const float swd = valid ? prm.s1_inv * sq : 0.f;
    const float cp = swp * swp, cd = swd * swd;
    const float w[3] = {huber_w(swp * err[0]) * cp, huber_w(swp * err[1]) * cp,
                        huber_w(swd * err[2]) * cd};
    const float J0[7] = {fx * zj_inv, 0.f, -fx * xz * zj_inv, -fx * xz * yz,
                         fx * (1.f + xz * xz), -fx * yz, 0.f};
    const float J1[7] = {0.f, fy * zj_inv, -fy * yz * zj_inv, -fy * (1.f + yz * yz),
                         fy * xz * yz, fy * xz, 0.f};
    const float J2[7] = {0.f, 0.f, zj_inv, yz, -xz, 0.f, 1.f};
    acc_row<0x3D>(acc, w[0], err[0], J0);
    acc_row<0x3E>(acc, w[1], err[1], J1);
    acc_row<0x5C>(acc, w[2], err[2], J2);
  } else {  // MODE_POINTS
    const float err[3] = {P[0] - Xi[0], P[1] - Xi[1], P[2] - Xi[2]};
    const float swp = valid ? prm.s0_inv * sqrt_f(q) : 0.f;
    const float cp = swp * swp;
    const float w[3] = {huber_w(swp * err[0]) * cp, huber_w(swp * err[1]) * cp,
                        huber_w(swp * err[2]) * cp};
    const float J0[7] = {1.f, 0.f, 0.f, 0.f, P[2], -P[1], P[0]};
    const float J1[7] = {0.f, 1.f, 0.f, -P[2], 0.f, P[0], P[1]};
    const float J2[7] = {0.f, 0.f, 1.f, P[1], -P[0], 0.f, P[2]};
    acc_row<0x71>(acc, w[0], err[0], J0);
    acc_row<0x6A>(acc, w[1], err[1], J1);
    acc_row<0x5C>(acc, w[2], err[2], J2);
  }
}

template <int MODE>
__global__ __launch_bounds__(kEdgeThreads) void gn_edge_kernel(
    const float* __restrict__ Twc, const float4* __restrict__ XC, const float* __restrict__ K,
    const int* __restrict__ rank_ii, const int* __restrict__ rank_jj,
    const int* __restrict__ MI, const float* __restrict__ Q,
    float* __restrict__ partial, int* __restrict__ flags, int64_t num_points, int S,
    GnParams prm, const int* __restrict__ edge_ids, const int* __restrict__ order, int rows) {
  if (flags[0]) return;  // converged in an earlier iteration
  // 1-D grid of rows x S blocks, dispatched round-robin over the 8 XCDs: block -> position v
  // in (row in `order`, split) sequence so that each XCD takes a contiguous run of the rows
  // sorted by pose i — its L2 then holds few keyframes' pointmaps for the scattered Xi / Ci
  // gathers instead of every keyframe's.  Same per-block work and partial slot either way.
  int e, s;
  {
    const int total = rows * S, lin = blockIdx.x, xcd = lin & 7, loc = lin >> 3;
    const int tq = total >> 3, tr = total & 7;
    const int v = xcd < tr ? xcd * (tq + 1) + loc : tr * (tq + 1) + (xcd - tr) * tq + loc;
    const int pos = v / S;
    s = v - pos * S;
    e = order[pos];             // row of this rank's edge data (idx / valid / Q / partial)
  }
  const int ge = edge_ids ? edge_ids[e] : e;   // the edge's id in the whole graph
  const int ix = rank_ii[ge], jx = rank_jj[ge];
  const float* Ti = Twc + 8 * ix;
  const float* Tj = Twc + 8 * jx;
  float tij[3], qij[4], sij;
  m3s_rel_sim3<float>(Ti, Ti + 3, Ti[7], Tj, Tj + 3, Tj[7], tij, qij, &sij);
  float fx = 0.f, fy = 0.f, cx = 0.f, cy = 0.f;
  if (MODE == MODE_CALIB) {
    fx = K[0];
    fy = K[4];
    cx = K[2];
    cy = K[5];
  }

  float acc[kAcc];
#pragma unroll
  for (int l = 0; l < kAcc; l++) acc[l] = 0.f;

  const int64_t chunk = (num_points + S - 1) / S;
  const int64_t k0 = (int64_t)s * chunk;
  const int64_t k1 = min(num_points, k0 + chunk);
  const float4* XCi = XC + (int64_t)ix * num_points;  // (X, C) records (gn_pack_kernel)
  const float4* XCj = XC + (int64_t)jx * num_points;
  const int64_t eoff = (int64_t)e * num_points;

  // U points per thread per trip: their independent loads (match, Q, record j) issue back to
  // back, then their gathers of record i at the match index, then the arithmetic — two
  // memory round trips per U points instead of per point, one 16-B gather per point.
  // Lanes past k1 load point k1 - 1 and accumulate it as invalid (weight 0).
  constexpr int U = 4;
  for (int64_t kb = k0 + threadIdx.x; kb < k1; kb += U * kEdgeThreads) {
    int mi[U];
    float qv[U];
    float4 rj[U], ri[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t k = min(kb + (int64_t)u * kEdgeThreads, k1 - 1);
      mi[u] = MI[eoff + k];
      qv[u] = Q[eoff + k];
      rj[u] = XCj[k];
    }
#pragma unroll
    for (int u = 0; u < U; u++) ri[u] = XCi[mi[u] >= 0 ? mi[u] : 0];
#pragma unroll
    for (int u = 0; u < U; u++) {  // unconditional (a branch would sink the loads into it)
      const bool in = kb + (int64_t)u * kEdgeThreads < k1;
      const float xi[3] = {ri[u].x, ri[u].y, ri[u].z}, xj[3] = {rj[u].x, rj[u].y, rj[u].z};
      point_acc<MODE>(acc, in && mi[u] >= 0, mi[u] >= 0 ? mi[u] : 0, xi, ri[u].w, xj, qv[u],
                      rj[u].w, tij, qij, sij, prm, fx, fy, cx, cy);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) flags[4] = 1;  // the records are packed (below)

  // workgroup reduction: wave butterfly, then 4 waves through LDS
  __shared__ float red[kEdgeThreads / M3S_WAVE][kAcc];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int l = 0; l < kAcc; l++) {
    const float v = m3s_wave_sum(acc[l]);
    if (lane == 0) red[wid][l] = v;
  }
  __syncthreads();
  if (threadIdx.x < kAcc) {
    float v = red[0][threadIdx.x];
#pragma unroll
    for (int wv = 1; wv < kEdgeThreads / M3S_WAVE; wv++) v += red[wv][threadIdx.x];
    partial[((int64_t)e * S + s) * kAcc + threadIdx.x] = v;
  }
}

// The rows of an edge pass sorted by the rank of pose i (counting sort in LDS, one
// workgroup; the order within a pose is immaterial: each row's partials are its own).
__global__ __launch_bounds__(kSolveThreads) void gn_order_kernel(
    const int* __restrict__ rank_ii, const int* __restrict__ edge_ids, int rows, int P,
    int* __restrict__ order, const int* __restrict__ flags) {
  // |unique(ii, jj)| != P (gn_rank_kernel set flags[0]): ranks may reach past the P + 1
  // counters, and every later kernel of the solve returns early anyway
  if (flags[0]) return;
  extern __shared__ int cnt[];  // [P + 1]
  for (int p = threadIdx.x; p <= P; p += blockDim.x) cnt[p] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < rows; r += blockDim.x)
    atomicAdd(&cnt[rank_ii[edge_ids ? edge_ids[r] : r] + 1], 1);
  __syncthreads();
  if (threadIdx.x == 0)
    for (int p = 1; p <= P; p++) cnt[p] += cnt[p - 1];
  __syncthreads();
  for (int r = threadIdx.x; r < rows; r += blockDim.x)
    order[atomicAdd(&cnt[rank_ii[edge_ids ? edge_ids[r] : r]], 1)] = r;
}

// The edge pass's inputs repacked once per solve (flags[4] = 0; the first edge pass sets
// it): XC f32x4 [P][N] = (X, C) of every point — one 16-B gather per matched point instead
// of a 12-B and a 4-B one — and MI i32 [rows][N] = the match index where valid, -1 where not
// (the reference's `valid ? idx : 0` with the flag folded in; 4 B streamed instead of 9).
__global__ __launch_bounds__(256) void gn_pack_kernel(const float* __restrict__ Xs,
                                                      const float* __restrict__ Cs,
                                                      const int64_t* __restrict__ idx,
                                                      const uint8_t* __restrict__ valid,
                                                      int64_t n_pts, int64_t n_match,
                                                      float4* __restrict__ XC,
                                                      int* __restrict__ MI,
                                                      const int* __restrict__ flags) {
  if (flags[4]) return;  // packed by an earlier edge pass of this solve
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_pts; i += stride)
    XC[i] = make_float4(Xs[3 * i], Xs[3 * i + 1], Xs[3 * i + 2], Cs[i]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_match; i += stride)
    MI[i] = valid[i] ? (int)idx[i] : -1;
}

// ranks of ii/jj in sorted unique(ii ∪ jj) (gn_kernels.cu:161-170, torch::_unique +
// searchsorted).  Single workgroup.  Keyframe ids span a small range in practice: a
// presence bitmap over [min, min + 2^17) in LDS, a popcount prefix per 32-bit word, then
// rank(v) = bits set below v — O(M + range / 32).  Ids spread wider than 2^17 fall back to
// the O(M^2) first-occurrence / count-below scan.
__global__ __launch_bounds__(kSolveThreads) void gn_rank_kernel(const int64_t* __restrict__ ii,
                                                               const int64_t* __restrict__ jj,
                                                               int E, int* __restrict__ rank_ii,
                                                               int* __restrict__ rank_jj,
                                                               int* __restrict__ flags, int P) {
  constexpr int kWords = (1 << 17) / 32;
  const int M = 2 * E;  // E <= 65535
  __shared__ unsigned bits[kWords];
  __shared__ int prefix[kWords + 1];
  __shared__ long long s_min, s_max;
  __shared__ int s_unique;
  if (threadIdx.x == 0) {
    s_min = LLONG_MAX;
    s_max = LLONG_MIN;
    s_unique = 0;
  }
  __syncthreads();
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (int p = threadIdx.x; p < M; p += blockDim.x) {
    const long long v = p < E ? ii[p] : jj[p - E];
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  atomicMin(&s_min, lo);
  atomicMax(&s_max, hi);
  __syncthreads();
  const long long base = s_min;
  if (s_max - base < (1ll << 17)) {
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) bits[w] = 0u;
    __syncthreads();
    for (int p = threadIdx.x; p < M; p += blockDim.x) {
      const int o = (int)((p < E ? ii[p] : jj[p - E]) - base);
      atomicOr(&bits[o >> 5], 1u << (o & 31));
    }
    __syncthreads();
    const int nw = (int)((s_max - base) >> 5) + 1;
    if (threadIdx.x == 0) {  // ≤ 4096 words: a serial exclusive scan is a few µs
      int acc = 0;
      for (int w = 0; w < nw; w++) {
        prefix[w] = acc;
        acc += __popc(bits[w]);
      }
      prefix[nw] = acc;
      s_unique = acc;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < M; p += blockDim.x) {
      const int o = (int)((p < E ? ii[p] : jj[p - E]) - base);
      const int rank = prefix[o >> 5] + __popc(bits[o >> 5] & ((1u << (o & 31)) - 1u));
      if (p < E) rank_ii[p] = rank;
      else rank_jj[p - E] = rank;
    }
    if (threadIdx.x == 0) {
      flags[2] = s_unique;
      if (s_unique != P) flags[0] = 1;  // invalid graph: no kernel of the solve runs (status)
    }
    return;
  }
  // wide id range: first occurrences (reusing the bitmap over positions), then count below
  for (int wd = threadIdx.x; wd < (M + 31) / 32; wd += blockDim.x) bits[wd] = 0u;
  __syncthreads();
  int local_unique = 0;
  for (int p = threadIdx.x; p < M; p += blockDim.x) {
    const int64_t v = p < E ? ii[p] : jj[p - E];
    bool first = true;
    for (int q = 0; q < p && first; q++) {
      const int64_t u = q < E ? ii[q] : jj[q - E];
      first = (u != v);
    }
    if (first) {
      atomicOr(&bits[p >> 5], 1u << (p & 31));
      local_unique++;
    }
  }
  atomicAdd(&s_unique, local_unique);
  __syncthreads();
  for (int p = threadIdx.x; p < M; p += blockDim.x) {
    const int64_t v = p < E ? ii[p] : jj[p - E];
    int rank = 0;
    for (int q = 0; q < M; q++) {
      const int64_t u = q < E ? ii[q] : jj[q - E];
      rank += ((u < v) && ((bits[q >> 5] >> (q & 31)) & 1u)) ? 1 : 0;
    }
    if (p < E) rank_ii[p] = rank;
    else rank_jj[p - E] = rank;
  }
  if (threadIdx.x == 0) {
    flags[2] = s_unique;
    if (s_unique != P) flags[0] = 1;
  }
}

// The S partials of each of this rank's E edges → G [E][kAcc] f64, in the solve kernel's
// fixed order (bit-identical to its step 1).
__global__ __launch_bounds__(256) void gn_reduce_kernel(const float* __restrict__ partial,
                                                        double* __restrict__ G,
                                                        const int* __restrict__ flags, int E,
                                                        int S) {
  if (flags[0]) return;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= E * kAcc) return;
  const int e = idx / kAcc, l = idx % kAcc;
  double v = 0.0;
  for (int s = 0; s < S; s++) v += (double)partial[((int64_t)e * S + s) * kAcc + l];
  G[idx] = v;
}

__device__ __forceinline__ int tri_idx(int n, int m) {  // n >= m
  return n * (n + 1) / 2 + m;
}

// Single-workgroup fp64 assemble + Cholesky + solve + retraction + convergence.
__global__ __launch_bounds__(kSolveThreads) void gn_solve_kernel(
    float* __restrict__ Twc, const float* __restrict__ partial, const int* __restrict__ rank_ii,
    const int* __restrict__ rank_jj, double* __restrict__ Ag, double* __restrict__ bg,
    double* __restrict__ Gs_ws, float* __restrict__ dx_out, int* __restrict__ flags, int E, int S,
    int P, float delta_thresh, const double* __restrict__ G_in) {
  if (flags[0]) return;
  const int tid = threadIdx.x;
  const int n = 7 * (P - 1);
  const int nt = blockDim.x;

  // 1) reduce the S partials of every edge (fixed order, f64) — or take them reduced
  //    (edge-sharded GN: gn_reduce_kernel on each rank, all-gathered in edge order)
  const double* Gs = G_in ? G_in : Gs_ws;
  if (!G_in) {
    for (int idx = tid; idx < E * kAcc; idx += nt) {
      const int e = idx / kAcc, l = idx % kAcc;
      double v = 0.0;
      for (int s = 0; s < S; s++) v += (double)partial[((int64_t)e * S + s) * kAcc + l];
      Gs_ws[idx] = v;
    }
  }
  for (int idx = tid; idx < n * n; idx += nt) Ag[idx] = 0.0;
  for (int idx = tid; idx < n; idx += nt) bg[idx] = 0.0;
  __syncthreads();

  // 2) per edge: A = M G M^T, vj = M v' (M from pose i), scatter into the system.
  __shared__ double sM[7][7];
  __shared__ double sG[7][7];
  __shared__ double sT[7][7];
  __shared__ double sA[7][7];
  __shared__ double sv[7];
  for (int e = 0; e < E; e++) {
    const int ix = rank_ii[e], jx = rank_jj[e];
    if (tid < 7) {
      // column tid of M = M applied to unit vector e_tid (M is linear, f64)
      const float* Ti = Twc + 8 * ix;
      const double t[3] = {Ti[0], Ti[1], Ti[2]};
      const double q[4] = {Ti[3], Ti[4], Ti[5], Ti[6]};
      const double s = Ti[7];
      double X[7] = {0, 0, 0, 0, 0, 0, 0};
      X[tid] = 1.0;
      double Y[7];
      m3s_adj_inv_apply<double>(t, q, s, X, Y);
      for (int r = 0; r < 7; r++) sM[r][tid] = Y[r];
    } else if (tid >= 64 && tid < 64 + 49) {
      const int r = (tid - 64) / 7, c = (tid - 64) % 7;
      sG[r][c] = Gs[e * kAcc + (r >= c ? tri_idx(r, c) : tri_idx(c, r))];
    }
    __syncthreads();
    if (tid < 49) {  // T = M G
      const int r = tid / 7, c = tid % 7;
      double v = 0.0;
      for (int k = 0; k < 7; k++) v += sM[r][k] * sG[k][c];
      sT[r][c] = v;
    } else if (tid >= 64 && tid < 71) {  // vj = M v'
      const int r = tid - 64;
      double v = 0.0;
      for (int k = 0; k < 7; k++) v += sM[r][k] * Gs[e * kAcc + 28 + k];
      sv[r] = v;
    }
    __syncthreads();
    if (tid < 49) {  // A = T M^T
      const int r = tid / 7, c = tid % 7;
      double v = 0.0;
      for (int k = 0; k < 7; k++) v += sT[r][k] * sM[c][k];
      sA[r][c] = v;
    }
    __syncthreads();
    // scatter: Hii += A, Hij -= A, Hji -= A, Hjj += A; b_i += -vj, b_j += vj
    // (one thread per entry handles all four blocks in order: no race even if i == j)
    const int oi = ix - 1, oj = jx - 1;  // rank 0 is the fixed pose
    if (tid < 49) {
      const int r = tid / 7, c = tid % 7;
      const double a = sA[r][c];
      if (oi >= 0) Ag[(int64_t)(7 * oi + r) * n + 7 * oi + c] += a;
      if (oi >= 0 && oj >= 0) Ag[(int64_t)(7 * oi + r) * n + 7 * oj + c] -= a;
      if (oi >= 0 && oj >= 0) Ag[(int64_t)(7 * oj + r) * n + 7 * oi + c] -= a;
      if (oj >= 0) Ag[(int64_t)(7 * oj + r) * n + 7 * oj + c] += a;
    } else if (tid >= 64 && tid < 71) {
      const int r = tid - 64;
      if (oi >= 0) bg[7 * oi + r] -= sv[r];
      if (oj >= 0) bg[7 * oj + r] += sv[r];
    }
    __syncthreads();
  }

  // 3) right-looking Cholesky, lower triangle in place (Eigen SimplicialLLT equivalent)
  // (column scaled by the reciprocal pivot; gn_solve_lds_kernel does the same operations)
  __shared__ int s_fail;
  __shared__ double s_rpiv;
  if (tid == 0) s_fail = 0;
  __syncthreads();
  for (int k = 0; k < n; k++) {
    if (tid == 0) {
      const double d = Ag[(int64_t)k * n + k];
      if (!(d > 0.0)) s_fail = 1;
      const double piv = sqrt(d);
      Ag[(int64_t)k * n + k] = piv;
      s_rpiv = 1.0 / piv;
    }
    __syncthreads();
    if (s_fail) break;
    const double rpiv = s_rpiv;
    for (int i = k + 1 + tid; i < n; i += nt) Ag[(int64_t)i * n + k] *= rpiv;
    __syncthreads();
    const int m = n - k - 1;  // trailing size
    const int64_t tot = (int64_t)m * (m + 1) / 2;
    for (int64_t idx = tid; idx < tot; idx += nt) {
      // map idx -> (i, j) with k < j <= i < n  (row-major lower triangle)
      int i = (int)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
      while ((int64_t)(i + 1) * (i + 2) / 2 <= idx) i++;
      while ((int64_t)i * (i + 1) / 2 > idx) i--;
      const int j = (int)(idx - (int64_t)i * (i + 1) / 2);
      const int gi = k + 1 + i, gj = k + 1 + j;
      Ag[(int64_t)gi * n + gj] -= Ag[(int64_t)gi * n + k] * Ag[(int64_t)gj * n + k];
    }
    __syncthreads();
  }

  // 4) solve L y = b, L^T x = y (column sweeps); x overwrites b.
  if (!s_fail) {
    for (int j = 0; j < n; j++) {
      if (tid == 0) bg[j] *= 1.0 / Ag[(int64_t)j * n + j];
      __syncthreads();
      const double yj = bg[j];
      for (int i = j + 1 + tid; i < n; i += nt) bg[i] -= Ag[(int64_t)i * n + j] * yj;
      __syncthreads();
    }
    for (int j = n - 1; j >= 0; j--) {
      if (tid == 0) bg[j] *= 1.0 / Ag[(int64_t)j * n + j];
      __syncthreads();
      const double xj = bg[j];
      for (int i = tid; i < j; i += nt) bg[i] -= Ag[(int64_t)j * n + i] * xj;
      __syncthreads();
    }
  }

  // 5) dx = -x (f32, zero on failure: gn_kernels.cu:147-150), retract poses 1..P-1
  for (int idx = tid; idx < n; idx += nt) dx_out[idx] = s_fail ? 0.f : (float)(-bg[idx]);
  __syncthreads();
  for (int p = 1 + tid; p < P; p += nt) {
    float* T = Twc + 8 * p;
    const float* xi = dx_out + 7 * (p - 1);
    float t1[3], q1[4], s1;
    m3s_retr_sim3<float>(xi, T, T + 3, T[7], t1, q1, &s1);
    T[0] = t1[0];
    T[1] = t1[1];
    T[2] = t1[2];
    T[3] = q1[0];
    T[4] = q1[1];
    T[5] = q1[2];
    T[6] = q1[3];
    T[7] = s1;
  }
  // 6) termination: ||dx|| < delta_thresh (gn_kernels.cu:1217-1222)
  __shared__ float s_red[kSolveThreads / M3S_WAVE];
  float ss = 0.f;
  for (int idx = tid; idx < n; idx += nt) ss += dx_out[idx] * dx_out[idx];
  ss = m3s_wave_sum(ss);
  if ((tid & 63) == 0) s_red[tid >> 6] = ss;
  __syncthreads();
  if (tid == 0) {
    float tot = 0.f;
    for (int w = 0; w < nt / 64; w++) tot += s_red[w];
    flags[3] += 1;
    if (s_fail) flags[1] = 1;
    if (sqrtf(tot) < delta_thresh) flags[0] = 1;
  }
}

// ---- the LDS-resident solve (n = 7(P-1) <= kLdsN) ----
// The system is small (P = 16 keyframes: n = 105, 88 KB of f64), so it lives in LDS for
// the whole solve instead of in global memory, and the per-edge serial assembly loop of
// gn_solve_kernel (four barriers and global read-modify-writes per edge) becomes:
//  * M of every pose once (apply_Sim3_adj_inv, f64), then per edge, in parallel over the
//    workgroup's 16 waves: the f64 reduction of its S partials (or its all-gathered G row;
//    the partials of four edges in flight at once), A = M G Mᵀ and v = M v' — the same
//    operations in the same order as gn_solve_kernel — written to EB;
//  * assembly by block row: wave w owns the system rows of pose w (+ 16, ...), walks the
//    edges in order, takes those touching its pose by ballot and applies their blocks
//    (Hii += A, Hij -= A, Hji -= A, Hjj += A; b_i -= v, b_j += v) — each entry's lane adds
//    the same contributions in the same order as the serial loop, so the system, and
//    everything after it, is bit-identical;
//  * blocked right-looking Cholesky in LDS (two barriers per 7-column panel), the two
//    triangular solves by one wave with the right-hand side in registers (no barriers,
//    each panel's operands read ahead of its dependent chain), retraction and the
//    convergence test as before.
constexpr int kLdsN = 140;            // P <= 21 (sA 153 KB of the 160 KB LDS)
constexpr int kLdsP = kLdsN / 7 + 1;
constexpr int kEB = 56;               // per edge: A (49) then v (7), f64

// LDS written by some lanes of a wave, then read by others of the same wave: wait for the
// writes and keep the compiler from moving accesses across (wave-scope fence on LDS only —
// a fence over all address spaces also waits for the wave's global stores)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
}

// keep a value in registers at this point: loads issued ahead of a dependent chain are not
// sunk by the compiler into the conditional updates that use them
__device__ __forceinline__ void pin_vgpr(double& v) { asm volatile("" : "+v"(v)); }

__device__ __forceinline__ double bcast_f64(double v, int l) {  // v of lane l, l uniform
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

#ifdef M3S_GN_STAMPS
// debug build (tools/gn_stamps.py): thread 0 of the LDS solve, s_memrealtime (100 MHz) at
// each phase boundary of the first 16 iterations
__device__ long long g_gn_stamps[16 * 8];
#define M3S_GS(ph) \
  if (tid == 0 && flags[3] < 16) \
    g_gn_stamps[flags[3] * 8 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime();
#else
#define M3S_GS(ph)
#endif

__global__ __launch_bounds__(kSolveThreads) void gn_solve_lds_kernel(
    float* __restrict__ Twc, const float* __restrict__ partial, const int* __restrict__ rank_ii,
    const int* __restrict__ rank_jj, double* __restrict__ EB, float* __restrict__ dx_out,
    int* __restrict__ flags, int E, int S, int P, float delta_thresh,
    const double* __restrict__ G_in) {
  if (flags[0]) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar edge indexing
  const int n = 7 * (P - 1);
  const int nt = blockDim.x;
  M3S_GS(0)
  constexpr int NW = kSolveThreads / 64;
  __shared__ double sA[kLdsN * kLdsN];
  __shared__ double sb[kLdsN];
  __shared__ double sR[kLdsN];          // 1 / L[k][k]
  __shared__ float s_red[NW];

  constexpr int CE = 4, CS = 8;  // edges per batch; partials per edge in flight
  // unconditional loads (indices clamped into range; what they fetch beyond the edge's
  // partials is not added): guarded loads became one branch and memory wait each.  The
  // next batch's first partials are requested before this batch's edges are processed.
  const int lc = lane < kAcc ? lane : kAcc - 1;
  float pv[CE][CS];
  auto load_partials = [&](int k0, int s0) {
#pragma unroll
    for (int u = 0; u < CE; u++) {
      const int e = min(wv + NW * (k0 + u), E - 1);
#pragma unroll
      for (int t = 0; t < CS; t++)
        pv[u][t] = partial[((int64_t)e * S + min(s0 + t, S - 1)) * kAcc + lc];
    }
  };
  if (!G_in && wv < E) load_partials(0, 0);  // in flight during 1a

  // 1a) M of every pose (column `lane` = M applied to the unit vector e_lane), into sA,
  //     which is free until the assembly
  double* sM = sA;  // [P][7][7], P * 49 <= kLdsN^2
  for (int p = wv; p < P; p += NW) {
    if (lane < 7) {
      const float* Ti = Twc + 8 * p;
      const double t[3] = {Ti[0], Ti[1], Ti[2]};
      const double q[4] = {Ti[3], Ti[4], Ti[5], Ti[6]};
      const double s = Ti[7];
      double X[7] = {0, 0, 0, 0, 0, 0, 0};
      X[lane] = 1.0;
      double Y[7];
      m3s_adj_inv_apply<double>(t, q, s, X, Y);
      for (int r = 0; r < 7; r++) sM[p * 49 + r * 7 + lane] = Y[r];
    }
  }
  __syncthreads();
  M3S_GS(6)

  // 1b) per edge (wave w: edges w, w + NW, ...): the 35 sums (the f64 reduction of
  //     gn_solve_kernel step 1, same order), T = M G, A = T Mᵀ, v = M v'
  // per-wave scratch for two edges at a time, in sA past the poses' M: edge h's G at
  // 147 h, T at 147 h + 49, v' at 147 h + 98
  double* scr = sA + 49 * kLdsP + wv * 294;  // past the poses' M; + 16 * 294 <= kLdsN^2
  const bool tl = lane < 49, vl = lane >= 56 && lane < 63;  // T / A lanes; v lanes
  const int r_l = tl ? lane / 7 : lane - 56, c_l = tl ? lane % 7 : 0;
  // pose ranks of this wave's edges k0 .. k0 + 63 (its k-th edge is wv + NW k), one per lane,
  // taken by v_readlane: no memory wait inside the loop (it would also wait for the prefetch)
  int rank_l = 0;
  for (int k0 = 0; wv + NW * k0 < E; k0 += CE) {
    if ((k0 & 63) == 0) rank_l = rank_ii[min(wv + NW * (k0 + lane), E - 1)];
    double g[CE];
    int ri[CE];
#pragma unroll
    for (int u = 0; u < CE; u++) {
      g[u] = 0.0;
      ri[u] = __builtin_amdgcn_readlane(rank_l, (k0 & 63) + u);
    }
    if (G_in) {
#pragma unroll
      for (int u = 0; u < CE; u++) {
        const int e = wv + NW * (k0 + u);
        if (lane < kAcc && e < E) g[u] = G_in[e * kAcc + lane];
      }
    } else {
      for (int s0 = 0;;) {
#pragma unroll
        for (int u = 0; u < CE; u++)
#pragma unroll
          for (int t = 0; t < CS; t++)
            if (s0 + t < S) g[u] += (double)pv[u][t];
        s0 += CS;
        if (s0 >= S) break;
        load_partials(k0, s0);
      }
      if (wv + NW * (k0 + CE) < E) load_partials(k0 + CE, 0);
    }
    // two edges per step, so the two dependent chains (T = M G, then A = T Mᵀ) of one
    // overlap the other's; v = M v' runs on lanes 56..62 in the same instructions as T
#pragma unroll
    for (int u = 0; u < CE; u += 2) {
      const int e0 = wv + NW * (k0 + u);
      if (e0 >= E) break;
      const bool two = e0 + NW < E;  // edge 1 is computed regardless, stored only if real
#pragma unroll
      for (int h = 0; h < 2; h++) {  // lanes 0..27: packed upper triangle → symmetric G
        double* G = scr + 147 * h;
        if (lane < 28) {
          int r = 0;
          while ((r + 1) * (r + 2) / 2 <= lane) r++;
          const int c = lane - r * (r + 1) / 2;
          G[r * 7 + c] = g[u + h];
          G[c * 7 + r] = g[u + h];
        } else if (lane < kAcc) {
          G[98 + lane - 28] = g[u + h];  // v'
        }
      }
      wave_lds_sync();                           // this wave's scratch writes visible
      const double* M0 = sM + 49 * ri[u];
      const double* M1 = sM + 49 * ri[u + 1];
      double v0 = 0.0, v1 = 0.0;
      if (tl || vl) {  // T = M G (lanes < 49), v = M v' (lanes 56..62)
        const int bo = tl ? c_l : 98, bs = tl ? 7 : 1;
        for (int k = 0; k < 7; k++) {
          v0 += M0[r_l * 7 + k] * scr[bo + k * bs];
          v1 += M1[r_l * 7 + k] * scr[147 + bo + k * bs];
        }
        if (tl) {
          scr[49 + lane] = v0;
          scr[147 + 49 + lane] = v1;
        }
      }
      wave_lds_sync();
      double* out0 = EB + (int64_t)e0 * kEB;
      double* out1 = EB + (int64_t)(e0 + NW) * kEB;
      if (tl) {  // A = T Mᵀ
        double a0 = 0.0, a1 = 0.0;
        for (int k = 0; k < 7; k++) {
          a0 += scr[49 + r_l * 7 + k] * M0[c_l * 7 + k];
          a1 += scr[147 + 49 + r_l * 7 + k] * M1[c_l * 7 + k];
        }
        out0[lane] = a0;
        if (two) out1[lane] = a1;
      } else if (vl) {
        out0[49 + lane - 56] = v0;
        if (two) out1[49 + lane - 56] = v1;
      }
      wave_lds_sync();                           // scratch reused by the next pair
    }
    if (k0 == 0) { M3S_GS(7) }
  }
  __threadfence_block();
  __syncthreads();
  M3S_GS(1)

  // 2) assembly by block row (see above): lane (r, c) < 49 owns entry (7 bi + r, 7 bj + c)
  //    of every block of the row, lanes 49..55 b[7 bi + r]; up to 8 touching edges' EB rows
  //    fetched per round trip, applied in edge order
  const int np = P - 1;
  for (int bi = wv; bi < np; bi += NW) {
    double* rowA = sA + 7 * bi * n;
    for (int x = lane; x < 7 * n; x += 64) rowA[x] = 0.0;
    if (lane < 7) sb[7 * bi + lane] = 0.0;
    wave_lds_sync();
    double* ent = lane < 49 ? rowA + (lane / 7) * n + lane % 7 : nullptr;
    for (int kb = 0; kb < E; kb += 64) {
      const int e_l = kb + lane;
      const int oi_l = e_l < E ? rank_ii[e_l] - 1 : -2;
      const int oj_l = e_l < E ? rank_jj[e_l] - 1 : -2;
      uint64_t mask = __ballot(oi_l == bi || oj_l == bi);
      while (mask) {
        constexpr int CB = 8;
        int eu[CB], oiu[CB], oju[CB];
        double v[CB];
#pragma unroll
        for (int u = 0; u < CB; u++) {
          eu[u] = -1;
          if (mask) {
            const int bit = __builtin_ctzll(mask);
            mask &= mask - 1;
            eu[u] = kb + bit;
            oiu[u] = __builtin_amdgcn_readlane(oi_l, bit);
            oju[u] = __builtin_amdgcn_readlane(oj_l, bit);
          }
        }
#pragma unroll
        for (int u = 0; u < CB; u++)  // unconditional (clamped) loads, all in flight
          v[u] = EB[(int64_t)max(eu[u], 0) * kEB + min(lane, kEB - 1)];
#pragma unroll
        for (int u = 0; u < CB; u++) {
          if (eu[u] < 0) break;
          const int oi = oiu[u], oj = oju[u];
          if (lane < 49) {
            if (oi == bi) {
              ent[7 * oi] += v[u];                 // Hii += A
              if (oj >= 0) ent[7 * oj] -= v[u];    // Hij -= A
            }
            if (oj == bi) {
              if (oi >= 0) ent[7 * oi] -= v[u];    // Hji -= A
              ent[7 * oj] += v[u];                 // Hjj += A
            }
          } else if (lane < kEB) {
            if (oi == bi) sb[7 * bi + lane - 49] -= v[u];
            if (oj == bi) sb[7 * bi + lane - 49] += v[u];
          }
        }
      }
    }
  }
  __syncthreads();
  M3S_GS(2)

  // 3) blocked right-looking Cholesky in LDS with look-ahead, one 7-column panel per pose.
  //    Wave 0 factors a panel with its rows in registers (row c0 + lane + 64 t; the pivot
  //    row and L[j][k] of the panel's rows come from lanes 0..6 by v_readlane).  Panel p's
  //    update of the trailing triangle is split: first the seven columns of panel p + 1 (all
  //    threads, one entry each), then — while wave 0 already factors panel p + 1 — waves
  //    1..15 apply panel p to the columns right of it, two entries per step.  Each entry
  //    still receives the unblocked algorithm's operations in the same order (A[i][j] -=
  //    L[i][k] L[j][k], k increasing; L[i][k] = A[i][k] · (1 / √A[k][k])), so the factor —
  //    and the poses — are bit-identical to gn_solve_kernel's.  L[., k] goes to the unused
  //    upper triangle (L[i][k] = sA[k n + i]), which neither update touches, 1 / L[k][k] to
  //    sR[k].  The panel factor (its 1 / √d chain) is the critical path; the wide update
  //    runs beside it.
  __shared__ int s_fail;
  bool fail = false;
  if (tid == 0) s_fail = 0;
  auto factor_panel = [&](int c0) {  // wave 0
    // rows c0 + lane + 64 t, t < 3: n - c0 <= 140 rows (the third only for the first panels)
    const int i0 = c0 + lane, i1 = c0 + 64 + lane, i2 = c0 + 128 + lane;
    double a0[7], a1[7], a2[7];
#pragma unroll
    for (int c = 0; c < 7; c++) {
      a0[c] = i0 < n ? sA[i0 * n + c0 + c] : 0.0;
      a1[c] = i1 < n ? sA[i1 * n + c0 + c] : 0.0;
      a2[c] = i2 < n ? sA[i2 * n + c0 + c] : 0.0;
    }
    bool f = false;
#pragma unroll
    for (int c = 0; c < 7; c++) {
      const int k = c0 + c;
      const double d = bcast_f64(a0[c], c);         // A[k][k]: row k is lane c
      if (!(d > 0.0)) {
        f = true;
        break;
      }
      const double rpiv = 1.0 / sqrt(d);
      const double l0 = a0[c] * rpiv, l1 = a1[c] * rpiv, l2 = a2[c] * rpiv;
      if (i0 > k && i0 < n) sA[k * n + i0] = l0;
      if (i1 > k && i1 < n) sA[k * n + i1] = l1;
      if (i2 < n) sA[k * n + i2] = l2;
      if (lane == 0) sR[k] = rpiv;
#pragma unroll
      for (int c2 = c + 1; c2 < 7; c2++) {
        const double lj = bcast_f64(l0, c2);        // L[c0 + c2][k]
        if (i0 >= c0 + c2) a0[c2] -= l0 * lj;
        if (i1 >= c0 + c2) a1[c2] -= l1 * lj;
        if (i2 < n) a2[c2] -= l2 * lj;
      }
    }
    if (lane == 0 && f) s_fail = 1;
  };
  if (wv == 0) factor_panel(0);
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += 7) {
    if (s_fail) {  // uniform: read after the barrier by every thread
      fail = true;
      break;
    }
    const int t0 = c0 + 7;
    if (t0 >= n) break;
    {  // panel p applied to panel p + 1's columns: entry (t0 + ri, t0 + cj), cj <= ri
      const int ri = tid / 7, cj = tid - 7 * ri;
      const int i = t0 + ri, j = t0 + cj;
      if (i < n && j <= i) {
        double a = sA[i * n + j];
#pragma unroll
        for (int c = 0; c < 7; c++) a -= sA[(c0 + c) * n + i] * sA[(c0 + c) * n + j];
        sA[i * n + j] = a;
      }
    }
    __syncthreads();
    if (wv == 0) {
      factor_panel(t0);
    } else {  // panel p applied to columns t0 + 7 .. i of row i = t0 + 7 + ri
      const int t1 = t0 + 7;
      const int cg = tid & 7;
      // 120 rows per pass (waves 1..15, 8 lanes a row); a second pass past row t1 + 119
      for (int i = t1 + ((tid - 64) >> 3); i < n; i += (kSolveThreads - 64) / 8) {
        double li[7];
#pragma unroll
        for (int c = 0; c < 7; c++) li[c] = sA[(c0 + c) * n + i];
        int j = t1 + cg;
        for (; j + 8 <= i; j += 16) {  // entries j and j + 8: two independent chains
          double a = sA[i * n + j], a8 = sA[i * n + j + 8];
          double lj[7], lj8[7];
#pragma unroll
          for (int c = 0; c < 7; c++) {
            lj[c] = sA[(c0 + c) * n + j];
            lj8[c] = sA[(c0 + c) * n + j + 8];
          }
#pragma unroll
          for (int c = 0; c < 7; c++) {
            a -= li[c] * lj[c];
            a8 -= li[c] * lj8[c];
          }
          sA[i * n + j] = a;
          sA[i * n + j + 8] = a8;
        }
        if (j <= i) {
          double a = sA[i * n + j];
#pragma unroll
          for (int c = 0; c < 7; c++) a -= li[c] * sA[(c0 + c) * n + j];
          sA[i * n + j] = a;
        }
      }
    }
    __syncthreads();
  }

  M3S_GS(3)
  // 4) L y = b, Lᵀ x = y by wave 0, rows i = lane + 64 t in registers (t < 3: n <= 192);
  //    the solved unknown goes to every lane by v_readlane (the owner lane is uniform).  The
  //    unknowns of rows [0, 64), [64, 128) and [128, n) are swept by separate loops, so the
  //    owner's register is known at compile time (a select between them was on every step's
  //    dependent chain), and each group of 8 steps reads its columns of L and 1 / L[j][j]
  //    (clamped, unconditional LDS loads; masked lanes do not use them) ahead of its chain;
  //    the masked updates are selects, so the compiler does not sink those loads into
  //    branches.  Every x_i receives x_i -= L[i][j] y_j (j increasing), then
  //    x_i -= L[j][i] x_j (j decreasing) — gn_solve_kernel's order.
  if (wv == 0 && !fail) {
    constexpr int G8 = 8;
    const int lc = min(lane, n - 1), lc1 = min(lane + 64, n - 1), lc2 = min(lane + 128, n - 1);
    const int n0 = min(n, 64), n1 = min(n, 128);
    double x0 = lane < n ? sb[lane] : 0.0, x1 = lane + 64 < n ? sb[lane + 64] : 0.0;
    double x2 = lane + 128 < n ? sb[lane + 128] : 0.0;
    for (int jb = 0; jb < n0; jb += G8) {       // forward, unknowns j < 64 (x0 of lane j)
      double c0[G8], c1[G8], c2[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = min(jb + u, n - 1);
        c0[u] = sA[j * n + lc];
        c1[u] = sA[j * n + lc1];
        c2[u] = sA[j * n + lc2];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c0[u]);
        pin_vgpr(c1[u]);
        pin_vgpr(c2[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jb + u;
        if (j >= n0) break;
        const double yj = bcast_f64(x0 * rr[u], j);
        if (lane == j) x0 = yj;
        x0 = lane > j && lane < n ? x0 - c0[u] * yj : x0;
        x1 = lane + 64 < n ? x1 - c1[u] * yj : x1;
        x2 = lane + 128 < n ? x2 - c2[u] * yj : x2;
      }
    }
    for (int jb = 64; jb < n1; jb += G8) {      // forward, unknowns 64 <= j < 128 (x1)
      double c1[G8], c2[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = min(jb + u, n - 1);
        c1[u] = sA[j * n + lc1];
        c2[u] = sA[j * n + lc2];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c1[u]);
        pin_vgpr(c2[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jb + u;
        if (j >= n1) break;
        const double yj = bcast_f64(x1 * rr[u], j - 64);
        if (lane == j - 64) x1 = yj;
        x1 = lane + 64 > j && lane + 64 < n ? x1 - c1[u] * yj : x1;
        x2 = lane + 128 < n ? x2 - c2[u] * yj : x2;
      }
    }
    for (int jb = 128; jb < n; jb += G8) {      // forward, unknowns j >= 128 (x2)
      double c2[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = min(jb + u, n - 1);
        c2[u] = sA[j * n + lc2];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c2[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jb + u;
        if (j >= n) break;
        const double yj = bcast_f64(x2 * rr[u], j - 128);
        if (lane == j - 128) x2 = yj;
        x2 = lane + 128 > j && lane + 128 < n ? x2 - c2[u] * yj : x2;
      }
    }
    for (int jt = n - 1; jt >= 128; jt -= G8) { // backward, unknowns j >= 128 (x2)
      double c0[G8], c1[G8], c2[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = max(jt - u, 0);
        c0[u] = sA[lc * n + j];
        c1[u] = sA[lc1 * n + j];
        c2[u] = sA[lc2 * n + j];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c0[u]);
        pin_vgpr(c1[u]);
        pin_vgpr(c2[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jt - u;
        if (j < 128) break;
        const double xj = bcast_f64(x2 * rr[u], j - 128);
        if (lane == j - 128) x2 = xj;
        x0 = lane < j ? x0 - c0[u] * xj : x0;
        x1 = lane + 64 < j ? x1 - c1[u] * xj : x1;
        x2 = lane + 128 < j ? x2 - c2[u] * xj : x2;
      }
    }
    for (int jt = n1 - 1; jt >= 64; jt -= G8) { // backward, unknowns 64 <= j < 128 (x1)
      double c0[G8], c1[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = max(jt - u, 0);
        c0[u] = sA[lc * n + j];
        c1[u] = sA[lc1 * n + j];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c0[u]);
        pin_vgpr(c1[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jt - u;
        if (j < 64) break;
        const double xj = bcast_f64(x1 * rr[u], j - 64);
        if (lane == j - 64) x1 = xj;
        x0 = lane < j ? x0 - c0[u] * xj : x0;
        x1 = lane + 64 < j ? x1 - c1[u] * xj : x1;
      }
    }
    for (int jt = n0 - 1; jt >= 0; jt -= G8) {  // backward, unknowns j < 64
      double c0[G8], rr[G8];
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = max(jt - u, 0);
        c0[u] = sA[lc * n + j];
        rr[u] = sR[j];
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        pin_vgpr(c0[u]);
        pin_vgpr(rr[u]);
      }
#pragma unroll
      for (int u = 0; u < G8; u++) {
        const int j = jt - u;
        if (j < 0) break;
        const double xj = bcast_f64(x0 * rr[u], j);
        if (lane == j) x0 = xj;
        x0 = lane < j ? x0 - c0[u] * xj : x0;
      }
    }
    if (lane < n) sb[lane] = x0;
    if (lane + 64 < n) sb[lane + 64] = x1;
    if (lane + 128 < n) sb[lane + 128] = x2;
  }
  __syncthreads();
  M3S_GS(4)

  // 5) dx = -x (zero on failure, gn_kernels.cu:147-150), retract poses 1..P-1
  for (int idx = tid; idx < n; idx += nt) dx_out[idx] = fail ? 0.f : (float)(-sb[idx]);
  __syncthreads();
  for (int p = 1 + tid; p < P; p += nt) {
    float* Tp = Twc + 8 * p;
    const float* xi = dx_out + 7 * (p - 1);
    float t1[3], q1[4], s1;
    m3s_retr_sim3<float>(xi, Tp, Tp + 3, Tp[7], t1, q1, &s1);
    Tp[0] = t1[0];
    Tp[1] = t1[1];
    Tp[2] = t1[2];
    Tp[3] = q1[0];
    Tp[4] = q1[1];
    Tp[5] = q1[2];
    Tp[6] = q1[3];
    Tp[7] = s1;
  }
  // 6) termination: ||dx|| < delta_thresh (gn_kernels.cu:1217-1222)
  float ss = 0.f;
  for (int idx = tid; idx < n; idx += nt) ss += dx_out[idx] * dx_out[idx];
  ss = m3s_wave_sum(ss);
  if (lane == 0) s_red[wv] = ss;
  __syncthreads();
  if (tid == 0) {
    float tot = 0.f;
    for (int w = 0; w < nt / 64; w++) tot += s_red[w];
    M3S_GS(5)
    flags[3] += 1;
    if (fail) flags[1] = 1;
    if (sqrtf(tot) < delta_thresh) flags[0] = 1;
  }
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// E x S ~ 3072 workgroups: four rounds of the 768 that fit the chip at once (3 waves per
// SIMD at the rays kernel's 126 VGPRs).  The 1-D grid gives each XCD a contiguous run of the
// edges sorted by pose i and dispatches it in order, so with four rounds an XCD works on
// about half of one keyframe's edges at a time and the scattered gathers of its (X, C)
// records (3.1 MB at 384 x 512) stay in its 4 MB L2; one round (768) had two keyframes'
// records in flight per XCD.  Measured per GN iteration at P = 16, E = 128 (debug builds,
// tools/gn_stamps.py, profiles/r04_gn_split_sweep.txt): random matches 376 → 294 µs, shifted
// 285 → 278, identity 273 → 271; 4608 / 6144 are slower again.
#ifndef M3S_GN_SPLIT_TARGET
#define M3S_GN_SPLIT_TARGET 3072
#endif
int choose_splits(int64_t E, int64_t N) {
  int64_t S = (M3S_GN_SPLIT_TARGET + E - 1) / E;
  const int64_t max_by_points = (N + 1023) / 1024;  // >= ~1024 points per workgroup
  if (S > max_by_points) S = max_by_points;
  if (S < 1) S = 1;
  if (S > 256) S = 256;
  return (int)S;
}

struct Layout {
  size_t flags, rank_ii, rank_jj, order, xc, mi, partial, A, b, G, EB, total;
};

// the LDS solve's per-edge blocks (EB) appended at `off`
template <class L>
size_t lds_regions(L& l, size_t off, int64_t E) {
  l.EB = off;
  return align_up(off + 8 * kEB * E, 256);
}

Layout make_layout(int64_t P, int64_t E, int S, int64_t N) {
  Layout L;
  const int64_t n = 7 * (P > 1 ? P - 1 : 0);
  size_t off = 0;
  L.flags = off;
  off = align_up(off + 64, 256);
  L.rank_ii = off;
  off = align_up(off + 4 * E, 256);
  L.rank_jj = off;
  off = align_up(off + 4 * E, 256);
  L.order = off;
  off = align_up(off + 4 * E, 256);
  L.xc = off;
  off = align_up(off + 16 * P * N, 256);
  L.mi = off;
  off = align_up(off + 4 * E * N, 256);
  L.partial = off;
  off = align_up(off + 4 * E * S * kAcc, 256);
  L.A = off;
  off = align_up(off + 8 * n * n, 256);
  L.b = off;
  off = align_up(off + 8 * n, 256);
  L.G = off;
  off = align_up(off + 8 * E * kAcc, 256);
  L.total = lds_regions(L, off, E);
  return L;
}

bool g_force_global_solve = false;   // m3s_gn_force_global_solve (diagnostic)
bool use_lds_solve(int64_t P) { return P > 1 && 7 * (P - 1) <= kLdsN && !g_force_global_solve; }

template <int MODE>
int run_gn(float* d_Twc, const float* d_Xs, const float* d_Cs, const float* d_K,
           const int64_t* d_ii, const int64_t* d_jj, const int64_t* d_idx,
           const uint8_t* d_valid, const float* d_Q, int64_t P, int64_t N, int64_t E,
           GnParams prm, int max_iter, float delta_thresh, float* d_dx, void* d_ws,
           int* h_status, void* stream) {
  if (P < 1 || N < 1 || E < 1) return M3S_ERR_INVALID_ARG;
  if (!d_Twc || !d_Xs || !d_Cs || !d_ii || !d_jj || !d_idx || !d_valid || !d_Q || !d_ws)
    return M3S_ERR_INVALID_ARG;
  if (MODE == MODE_CALIB && !d_K) return M3S_ERR_INVALID_ARG;
  if (E > 65535 || 7 * P > 46000 || N >= (1ll << 31)) return M3S_ERR_TOO_LARGE;
  hipStream_t st = m3s_stream(stream);
  const int S = choose_splits(E, N);
  const Layout L = make_layout(P, E, S, N);
  char* ws = reinterpret_cast<char*>(d_ws);
  int* flags = reinterpret_cast<int*>(ws + L.flags);
  int* rii = reinterpret_cast<int*>(ws + L.rank_ii);
  int* rjj = reinterpret_cast<int*>(ws + L.rank_jj);
  float* partial = reinterpret_cast<float*>(ws + L.partial);
  double* A = reinterpret_cast<double*>(ws + L.A);
  double* b = reinterpret_cast<double*>(ws + L.b);
  double* G = reinterpret_cast<double*>(ws + L.G);
  M3S_HIP_CHECK(hipMemsetAsync(flags, 0, 64, st));
  if (P > 1) M3S_HIP_CHECK(hipMemsetAsync(d_dx, 0, sizeof(float) * 7 * (P - 1), st));
  hipLaunchKernelGGL(gn_rank_kernel, dim3(1), dim3(kSolveThreads), 0, st, d_ii, d_jj, (int)E, rii,
                     rjj, flags, (int)P);
  M3S_LAUNCH_CHECK();
  int* order = reinterpret_cast<int*>(ws + L.order);
  hipLaunchKernelGGL(gn_order_kernel, dim3(1), dim3(kSolveThreads), sizeof(int) * (P + 1), st,
                     rii, nullptr, (int)E, (int)P, order, flags);
  M3S_LAUNCH_CHECK();
  float4* XC = reinterpret_cast<float4*>(ws + L.xc);
  int* MI = reinterpret_cast<int*>(ws + L.mi);
  hipLaunchKernelGGL(gn_pack_kernel, dim3(2048), dim3(256), 0, st, d_Xs, d_Cs, d_idx, d_valid,
                     P * N, E * N, XC, MI, flags);
  M3S_LAUNCH_CHECK();
  const bool lds = use_lds_solve(P);
  if (P > 1) {
    for (int it = 0; it < max_iter; it++) {
      hipLaunchKernelGGL(gn_edge_kernel<MODE>, dim3((unsigned)(E * S)), dim3(kEdgeThreads), 0,
                         st, d_Twc, XC, d_K, rii, rjj, MI, d_Q, partial, flags, N, S, prm,
                         nullptr, order, (int)E);
      M3S_LAUNCH_CHECK();
      if (lds)
        hipLaunchKernelGGL(gn_solve_lds_kernel, dim3(1), dim3(kSolveThreads), 0, st, d_Twc,
                           partial, rii, rjj, reinterpret_cast<double*>(ws + L.EB), d_dx,
                           flags, (int)E, S, (int)P, delta_thresh, nullptr);
      else
        hipLaunchKernelGGL(gn_solve_kernel, dim3(1), dim3(kSolveThreads), 0, st, d_Twc, partial,
                           rii, rjj, A, b, G, d_dx, flags, (int)E, S, (int)P, delta_thresh,
                           nullptr);
      M3S_LAUNCH_CHECK();
    }
  }
  if (h_status) {
    int hflags[4] = {0, 0, 0, 0};
    M3S_HIP_CHECK(hipMemcpyAsync(hflags, flags, sizeof(hflags), hipMemcpyDeviceToHost, st));
    M3S_HIP_CHECK(hipStreamSynchronize(st));
    if (hflags[2] != P) *h_status = M3S_ERR_INVALID_ARG;  // |unique(ii,jj)| != P
    else *h_status = hflags[1] ? M3S_ERR_NOT_PD : M3S_OK;
  }
  return M3S_OK;
}

// ---- edge-sharded GN ----
// Workspace: flags, ranks of ALL E_total two-way edges, partials of this rank's E_local
// edges, the dense system.  S comes from E_total, so every edge's partials — hence its G
// row — are those of the unsharded m3s_gauss_newton_* call, bit for bit.
struct ShardLayout {
  size_t flags, rank_ii, rank_jj, order, xc, mi, partial, A, b, EB, total;
  int S;
};

ShardLayout make_shard_layout(int64_t P, int64_t E_total, int64_t E_local, int64_t N) {
  ShardLayout L;
  L.S = choose_splits(E_total, N);
  const int64_t n = 7 * (P > 1 ? P - 1 : 0);
  size_t off = 0;
  L.flags = off;
  off = align_up(off + 64, 256);
  L.rank_ii = off;
  off = align_up(off + 4 * E_total, 256);
  L.rank_jj = off;
  off = align_up(off + 4 * E_total, 256);
  L.order = off;
  off = align_up(off + 4 * (E_local > 0 ? E_local : 1), 256);
  L.xc = off;
  off = align_up(off + 16 * P * N, 256);
  L.mi = off;
  off = align_up(off + 4 * (E_local > 0 ? E_local : 1) * N, 256);
  L.partial = off;
  off = align_up(off + 4 * (E_local > 0 ? E_local : 1) * L.S * kAcc, 256);
  L.A = off;
  off = align_up(off + 8 * n * n, 256);
  L.b = off;
  off = align_up(off + 8 * (n > 0 ? n : 1), 256);
  L.total = lds_regions(L, off, E_total);
  return L;
}

bool shard_sizes_ok(int64_t P, int64_t N, int64_t E_total, int64_t E_local) {
  return P >= 1 && N >= 1 && N < (1ll << 31) && E_total >= 1 && E_local >= 0 &&
         E_local <= E_total && E_total <= 65535 && 7 * P <= 46000;
}

template <int MODE>
int shard_edge_pass(const float* d_Twc, const float* d_Xs, const float* d_Cs, const float* d_K,
                    const int32_t* d_edge_ids, const int64_t* d_idx, const uint8_t* d_valid,
                    const float* d_Q, int64_t P, int64_t N, int64_t E_total, int64_t E_local,
                    GnParams prm, double* d_G, void* d_ws, void* stream) {
  if (!shard_sizes_ok(P, N, E_total, E_local) || !d_ws) return M3S_ERR_INVALID_ARG;
  if (E_local == 0 || P < 2) return M3S_OK;
  if (!d_Twc || !d_Xs || !d_Cs || !d_edge_ids || !d_idx || !d_valid || !d_Q || !d_G)
    return M3S_ERR_INVALID_ARG;
  if (MODE == MODE_CALIB && !d_K) return M3S_ERR_INVALID_ARG;
  const ShardLayout L = make_shard_layout(P, E_total, E_local, N);
  char* ws = reinterpret_cast<char*>(d_ws);
  int* flags = reinterpret_cast<int*>(ws + L.flags);
  float* partial = reinterpret_cast<float*>(ws + L.partial);
  hipStream_t st = m3s_stream(stream);
  float4* XC = reinterpret_cast<float4*>(ws + L.xc);
  int* MI = reinterpret_cast<int*>(ws + L.mi);
  hipLaunchKernelGGL(gn_pack_kernel, dim3(2048), dim3(256), 0, st, d_Xs, d_Cs, d_idx, d_valid,
                     P * N, E_local * N, XC, MI, flags);
  M3S_LAUNCH_CHECK();
  int* order = reinterpret_cast<int*>(ws + L.order);
  hipLaunchKernelGGL(gn_order_kernel, dim3(1), dim3(kSolveThreads), sizeof(int) * (P + 1), st,
                     reinterpret_cast<const int*>(ws + L.rank_ii),
                     reinterpret_cast<const int*>(d_edge_ids), (int)E_local, (int)P, order,
                     flags);
  M3S_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_edge_kernel<MODE>, dim3((unsigned)(E_local * L.S)), dim3(kEdgeThreads),
                     0, st, d_Twc, XC, d_K, reinterpret_cast<const int*>(ws + L.rank_ii),
                     reinterpret_cast<const int*>(ws + L.rank_jj), MI, d_Q, partial, flags, N,
                     L.S, prm, reinterpret_cast<const int*>(d_edge_ids), order, (int)E_local);
  M3S_LAUNCH_CHECK();
  hipLaunchKernelGGL(gn_reduce_kernel, dim3(m3s_div_up(E_local * kAcc, 256)), dim3(256), 0, st,
                     partial, d_G, flags, (int)E_local, L.S);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

}  // namespace

#ifdef M3S_GN_STAMPS
extern "C" int m3s_debug_gn_stamps(long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gn_stamps), sizeof(long long) * 16 * 8) ==
                 hipSuccess ? 0 : -2;
}
#endif

extern "C" int m3s_gn_force_global_solve(int on) {
  g_force_global_solve = on != 0;
  return M3S_OK;
}

extern "C" size_t m3s_gn_sharded_workspace_bytes(int64_t num_poses, int64_t num_edges_total,
                                                 int64_t num_edges_local, int64_t num_points) {
  if (!shard_sizes_ok(num_poses, num_points, num_edges_total, num_edges_local)) return 256;
  return make_shard_layout(num_poses, num_edges_total, num_edges_local, num_points).total;
}

extern "C" int m3s_gn_sharded_begin(const int64_t* d_ii, const int64_t* d_jj, int64_t num_poses,
                                    int64_t num_points, int64_t num_edges_total,
                                    int64_t num_edges_local, float* d_dx, void* d_ws,
                                    void* stream) {
  const int64_t P = num_poses, E = num_edges_total;
  if (!shard_sizes_ok(P, num_points, E, num_edges_local) || !d_ii || !d_jj || !d_ws ||
      (P > 1 && !d_dx))
    return M3S_ERR_INVALID_ARG;
  const ShardLayout L = make_shard_layout(P, E, num_edges_local, num_points);
  char* ws = reinterpret_cast<char*>(d_ws);
  hipStream_t st = m3s_stream(stream);
  M3S_HIP_CHECK(hipMemsetAsync(ws + L.flags, 0, 64, st));
  if (P > 1) M3S_HIP_CHECK(hipMemsetAsync(d_dx, 0, sizeof(float) * 7 * (P - 1), st));
  hipLaunchKernelGGL(gn_rank_kernel, dim3(1), dim3(kSolveThreads), 0, st, d_ii, d_jj, (int)E,
                     reinterpret_cast<int*>(ws + L.rank_ii), reinterpret_cast<int*>(ws + L.rank_jj),
                     reinterpret_cast<int*>(ws + L.flags), (int)P);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_gn_rays_edge_pass(const float* d_Twc, const float* d_Xs, const float* d_Cs,
                                     const int32_t* d_edge_ids, const int64_t* d_idx,
                                     const uint8_t* d_valid, const float* d_Q, int64_t P, int64_t N,
                                     int64_t E_total, int64_t E_local, float sigma_ray,
                                     float sigma_dist, float C_thresh, float Q_thresh, double* d_G,
                                     void* d_ws, void* stream) {
  GnParams prm{};
  prm.s0_inv = (float)(1.0 / (double)sigma_ray);
  prm.s1_inv = (float)(1.0 / (double)sigma_dist);
  prm.C_thresh = C_thresh;
  prm.Q_thresh = Q_thresh;
  return shard_edge_pass<MODE_RAYS>(d_Twc, d_Xs, d_Cs, nullptr, d_edge_ids, d_idx, d_valid, d_Q,
                                    P, N, E_total, E_local, prm, d_G, d_ws, stream);
}

extern "C" int m3s_gn_calib_edge_pass(const float* d_Twc, const float* d_Xs, const float* d_Cs,
                                      const float* d_K, const int32_t* d_edge_ids,
                                      const int64_t* d_idx, const uint8_t* d_valid,
                                      const float* d_Q, int64_t P, int64_t N, int64_t E_total,
                                      int64_t E_local, int height, int width, int pixel_border,
                                      float z_eps, float sigma_pixel, float sigma_depth,
                                      float C_thresh, float Q_thresh, double* d_G, void* d_ws,
                                      void* stream) {
  GnParams prm{};
  prm.s0_inv = (float)(1.0 / (double)sigma_pixel);
  prm.s1_inv = (float)(1.0 / (double)sigma_depth);
  prm.C_thresh = C_thresh;
  prm.Q_thresh = Q_thresh;
  prm.height = height;
  prm.width = width;
  prm.pixel_border = pixel_border;
  prm.z_eps = z_eps;
  if (width < 1 || height < 1) return M3S_ERR_INVALID_ARG;
  return shard_edge_pass<MODE_CALIB>(d_Twc, d_Xs, d_Cs, d_K, d_edge_ids, d_idx, d_valid, d_Q, P,
                                     N, E_total, E_local, prm, d_G, d_ws, stream);
}

extern "C" int m3s_gn_solve_step(float* d_Twc, const double* d_G, int64_t num_poses,
                                 int64_t num_points, int64_t num_edges_total,
                                 int64_t num_edges_local, float delta_thresh, float* d_dx,
                                 void* d_ws, void* stream) {
  const int64_t P = num_poses, E = num_edges_total;
  if (!shard_sizes_ok(P, num_points, E, num_edges_local) || !d_ws) return M3S_ERR_INVALID_ARG;
  if (P < 2) return M3S_OK;
  if (!d_Twc || !d_G || !d_dx) return M3S_ERR_INVALID_ARG;
  const ShardLayout L = make_shard_layout(P, E, num_edges_local, num_points);
  char* ws = reinterpret_cast<char*>(d_ws);
  if (use_lds_solve(P)) {
    hipLaunchKernelGGL(gn_solve_lds_kernel, dim3(1), dim3(kSolveThreads), 0, m3s_stream(stream),
                       d_Twc, nullptr, reinterpret_cast<const int*>(ws + L.rank_ii),
                       reinterpret_cast<const int*>(ws + L.rank_jj),
                       reinterpret_cast<double*>(ws + L.EB), d_dx,
                       reinterpret_cast<int*>(ws + L.flags), (int)E, L.S, (int)P, delta_thresh,
                       d_G);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
  }
  hipLaunchKernelGGL(gn_solve_kernel, dim3(1), dim3(kSolveThreads), 0, m3s_stream(stream), d_Twc,
                     nullptr, reinterpret_cast<const int*>(ws + L.rank_ii),
                     reinterpret_cast<const int*>(ws + L.rank_jj),
                     reinterpret_cast<double*>(ws + L.A), reinterpret_cast<double*>(ws + L.b),
                     nullptr, d_dx, reinterpret_cast<int*>(ws + L.flags), (int)E, L.S, (int)P,
                     delta_thresh, d_G);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_gn_sharded_status(const void* d_ws, int64_t num_poses, int* h_status,
                                     int* h_iters, void* stream) {
  if (!d_ws || !h_status) return M3S_ERR_INVALID_ARG;
  int hflags[4] = {0, 0, 0, 0};
  hipStream_t st = m3s_stream(stream);
  M3S_HIP_CHECK(hipMemcpyAsync(hflags, d_ws, sizeof(hflags), hipMemcpyDeviceToHost, st));
  M3S_HIP_CHECK(hipStreamSynchronize(st));
  if (hflags[2] != num_poses) *h_status = M3S_ERR_INVALID_ARG;
  else *h_status = hflags[1] ? M3S_ERR_NOT_PD : M3S_OK;
  if (h_iters) *h_iters = hflags[3];
  return M3S_OK;
}

extern "C" size_t m3s_gn_workspace_bytes(int64_t num_poses, int64_t num_edges,
                                         int64_t num_points) {
  if (num_poses < 1 || num_edges < 1 || num_points < 1) return 256;
  return make_layout(num_poses, num_edges, choose_splits(num_edges, num_points), num_points)
      .total;
}

extern "C" int m3s_gauss_newton_rays(float* d_Twc, const float* d_Xs, const float* d_Cs,
                                     const int64_t* d_ii, const int64_t* d_jj,
                                     const int64_t* d_idx, const uint8_t* d_valid,
                                     const float* d_Q, int64_t P, int64_t N, int64_t E,
                                     float sigma_ray, float sigma_dist, float C_thresh,
                                     float Q_thresh, int max_iter, float delta_thresh,
                                     float* d_dx, void* d_ws, int* h_status, void* stream) {
  GnParams prm{};
  prm.s0_inv = (float)(1.0 / (double)sigma_ray);
  prm.s1_inv = (float)(1.0 / (double)sigma_dist);
  prm.C_thresh = C_thresh;
  prm.Q_thresh = Q_thresh;
  return run_gn<MODE_RAYS>(d_Twc, d_Xs, d_Cs, nullptr, d_ii, d_jj, d_idx, d_valid, d_Q, P, N, E,
                           prm, max_iter, delta_thresh, d_dx, d_ws, h_status, stream);
}

extern "C" int m3s_gauss_newton_calib(float* d_Twc, const float* d_Xs, const float* d_Cs,
                                      const float* d_K, const int64_t* d_ii, const int64_t* d_jj,
                                      const int64_t* d_idx, const uint8_t* d_valid,
                                      const float* d_Q, int64_t P, int64_t N, int64_t E,
                                      int height, int width, int pixel_border, float z_eps,
                                      float sigma_pixel, float sigma_depth, float C_thresh,
                                      float Q_thresh, int max_iter, float delta_thresh,
                                      float* d_dx, void* d_ws, int* h_status, void* stream) {
  GnParams prm{};
  prm.s0_inv = (float)(1.0 / (double)sigma_pixel);
  prm.s1_inv = (float)(1.0 / (double)sigma_depth);
  prm.C_thresh = C_thresh;
  prm.Q_thresh = Q_thresh;
  prm.height = height;
  prm.width = width;
  prm.pixel_border = pixel_border;
  prm.z_eps = z_eps;
  if (width < 1 || height < 1) return M3S_ERR_INVALID_ARG;
  return run_gn<MODE_CALIB>(d_Twc, d_Xs, d_Cs, d_K, d_ii, d_jj, d_idx, d_valid, d_Q, P, N, E,
                            prm, max_iter, delta_thresh, d_dx, d_ws, h_status, stream);
}

extern "C" int m3s_gauss_newton_points(float* d_Twc, const float* d_Xs, const float* d_Cs,
                                       const int64_t* d_ii, const int64_t* d_jj,
                                       const int64_t* d_idx, const uint8_t* d_valid,
                                       const float* d_Q, int64_t P, int64_t N, int64_t E,
                                       float sigma_point, float C_thresh, float Q_thresh,
                                       int max_iter, float delta_thresh, float* d_dx, void* d_ws,
                                       int* h_status, void* stream) {
  GnParams prm{};
  prm.s0_inv = (float)(1.0 / (double)sigma_point);
  prm.C_thresh = C_thresh;
  prm.Q_thresh = Q_thresh;
  return run_gn<MODE_POINTS>(d_Twc, d_Xs, d_Cs, nullptr, d_ii, d_jj, d_idx, d_valid, d_Q, P, N,
                             E, prm, max_iter, delta_thresh, d_dx, d_ws, h_status, stream);
}
