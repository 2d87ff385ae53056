/*
 * ORACLE — test infrastructure only (never shipped, never on the product path).
 *
 * CPU restatement of the reference's backend Gauss-Newton
 * (/root/reference/MASt3R-SLAM/mast3r_slam/backend/src/gn_kernels.cu):
 *   Sim3 helpers                        gn_kernels.cu:178-413
 *   point_align_kernel                  :455-723
 *   ray_align_kernel                    :813-1138
 *   calib_proj_kernel                   :1231-1543
 *   SparseBlock (Eigen SimplicialLLT)   :57-159   → dense fp64 Cholesky (same system)
 *   gauss_newton_{points,rays,calib}    :725-811, :1140-1228, :1546-1638
 * Per point and residual row it builds the 14-vector Jx = [Ji, Jj] exactly as the
 * reference (Jj = apply_Sim3_adj_inv(pose i, row), Ji = -Jj) and accumulates the 105
 * upper-triangle products w*Jx[n]*Jx[m] and the 7+7 gradient terms — in double, one
 * point after another (the reference sums per thread then tree-reduces in f32; the
 * order differs, the quantity is the same).  Compile with -ffp-contract=off.
 * Parity with the CUDA original is unpinned by reference tests (none exist); it is
 * pinned here by restating the algorithm and by known-answer tests in tests/.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- Sim3 (gn_kernels.cu:178-413) ---------------------------------------- */
static void quat_comp(const float* qi, const float* qj, float* out) {
  out[0] = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  out[1] = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  out[2] = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  out[3] = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
}
static void quat_inv(const float* q, float* out) {
  out[0] = -q[0];
  out[1] = -q[1];
  out[2] = -q[2];
  out[3] = q[3];
}
static void actSO3(const float* q, const float* X, float* Y) {
  float uv[3];
  uv[0] = (float)(2.0 * (double)(q[1] * X[2] - q[2] * X[1]));
  uv[1] = (float)(2.0 * (double)(q[2] * X[0] - q[0] * X[2]));
  uv[2] = (float)(2.0 * (double)(q[0] * X[1] - q[1] * X[0]));
  float y0 = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  float y1 = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  float y2 = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}
static void actSim3(const float* t, const float* q, const float* s, const float* X, float* Y) {
  actSO3(q, X, Y);
  Y[0] *= s[0];
  Y[1] *= s[0];
  Y[2] *= s[0];
  Y[0] += t[0];
  Y[1] += t[1];
  Y[2] += t[2];
}
static void relSim3(const float* ti, const float* qi, const float* si, const float* tj,
                    const float* qj, const float* sj, float* tij, float* qij, float* sij) {
  float si_inv = (float)(1.0 / (double)si[0]);
  sij[0] = si_inv * sj[0];
  float qi_inv[4];
  quat_inv(qi, qi_inv);
  quat_comp(qi_inv, qj, qij);
  tij[0] = tj[0] - ti[0];
  tij[1] = tj[1] - ti[1];
  tij[2] = tj[2] - ti[2];
  actSO3(qi_inv, tij, tij);
  tij[0] *= si_inv;
  tij[1] *= si_inv;
  tij[2] *= si_inv;
}
static float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void apply_Sim3_adj_inv(const float* t, const float* q, const float* s, const float* X,
                               float* Y) {
  const float s_inv = (float)(1.0 / (double)s[0]);
  float Ra[3];
  actSO3(q, &X[0], Ra);
  Y[0] = s_inv * Ra[0];
  Y[1] = s_inv * Ra[1];
  Y[2] = s_inv * Ra[2];
  actSO3(q, &X[3], &Y[3]);
  Y[3] += s_inv * (t[1] * Ra[2] - t[2] * Ra[1]);
  Y[4] += s_inv * (t[2] * Ra[0] - t[0] * Ra[2]);
  Y[5] += s_inv * (t[0] * Ra[1] - t[1] * Ra[0]);
  Y[6] = X[6] + (s_inv * dot3(t, Ra));
}
#define EPS 1e-6
static void expSO3(const float* phi, float* q) {
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float imag, real;
  if (theta_sq < EPS) {
    float theta_p4 = theta_sq * theta_sq;
    imag = (float)(0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4);
    real = (float)(1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4);
  } else {
    float theta = sqrtf(theta_sq);
    imag = sinf((float)(0.5 * theta)) / theta;
    real = cosf((float)(0.5 * theta));
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}
static void crossInplace(const float* a, float* b) {
  float x[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  b[0] = x[0];
  b[1] = x[1];
  b[2] = x[2];
}
static void expSim3(const float* xi, float* t, float* q, float* s) {
  float tau[3] = {xi[0], xi[1], xi[2]};
  float phi[3] = {xi[3], xi[4], xi[5]};
  float sigma = xi[6];
  float scale = expf(sigma);
  expSO3(phi, q);
  s[0] = scale;
  float theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float theta = sqrtf(theta_sq);
  float A, B, C;
  const float one = 1.0f, half = 0.5f;
  if (fabsf(sigma) < EPS) {
    C = one;
    if (fabsf(theta) < EPS) {
      A = half;
      B = (float)(1.0 / 6.0);
    } else {
      A = (one - cosf(theta)) / theta_sq;
      B = (theta - sinf(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - one) / sigma;
    if (fabsf(theta) < EPS) {
      float sigma_sq = sigma * sigma;
      A = ((sigma - one) * scale + one) / sigma_sq;
      B = (scale * half * sigma_sq + scale - one - sigma * scale) / (sigma_sq * sigma);
    } else {
      float a = scale * sinf(theta);
      float b = scale * cosf(theta);
      float c = theta_sq + sigma * sigma;
      A = (a * sigma + (one - b) * theta) / (theta * c);
      B = (C - ((b - one) * sigma + a * theta) / (c)) / (theta_sq);
    }
  }
  t[0] = C * tau[0];
  t[1] = C * tau[1];
  t[2] = C * tau[2];
  crossInplace(phi, tau);
  t[0] += A * tau[0];
  t[1] += A * tau[1];
  t[2] += A * tau[2];
  crossInplace(phi, tau);
  t[0] += B * tau[0];
  t[1] += B * tau[1];
  t[2] += B * tau[2];
}
static void retrSim3(const float* xi, const float* t, const float* q, const float* s, float* t1,
                     float* q1, float* s1) {
  float dt[3] = {0, 0, 0}, dq[4] = {0, 0, 0, 1}, ds[1] = {0};
  expSim3(xi, dt, dq, ds);
  quat_comp(dq, q, q1);
  actSO3(dq, t, t1);
  t1[0] *= ds[0];
  t1[1] *= ds[0];
  t1[2] *= ds[0];
  t1[0] += dt[0];
  t1[1] += dt[1];
  t1[2] += dt[2];
  s1[0] = ds[0] * s[0];
}
void ref_retr_sim3(const float* xi, const float* pose, float* out) {
  retrSim3(xi, pose, pose + 3, pose + 7, out, out + 3, out + 7);
}
void ref_rel_sim3(const float* Ti, const float* Tj, float* out) {
  relSim3(Ti, Ti + 3, Ti + 7, Tj, Tj + 3, Tj + 7, out, out + 3, out + 7);
}
static float huber(float r) {
  const float r_abs = fabsf(r);
  return (double)r_abs < 1.345 ? 1.0f : (float)(1.345 / (double)r_abs);
}

/* ---- per-edge H, g --------------------------------------------------------- */
typedef struct {
  int mode; /* 0 rays, 1 calib, 2 points */
  float sig0, sig1;
  float C_thresh, Q_thresh;
  int height, width, pixel_border;
  float z_eps;
  float fx, fy, cx, cy;
} gn_params;

static void accumulate_row(double* hij, double* vi, double* vj, float w, float err, float* Jx,
                           const float* ti, const float* qi, const float* si) {
  float* Ji = &Jx[0];
  float* Jj = &Jx[7];
  apply_Sim3_adj_inv(ti, qi, si, Ji, Jj);
  for (int n = 0; n < 7; n++) Ji[n] = -Jj[n];
  int l = 0;
  for (int n = 0; n < 14; n++)
    for (int m = 0; m <= n; m++) {
      hij[l] += (double)(w * Jx[n] * Jx[m]);
      l++;
    }
  for (int n = 0; n < 7; n++) {
    vi[n] += (double)(w * err * Ji[n]);
    vj[n] += (double)(w * err * Jj[n]);
  }
}

/* Hs_out: [4][7][7], gs_out: [2][7] for this edge (reference layout, gn_kernels.cu:1114-1137) */
static void edge_system(const gn_params* prm, const float* Twc, const float* Xs, const float* Cs,
                        int ix, int jx, const int64_t* idx, const uint8_t* valid_match,
                        const float* Q, int64_t N, double* Hs_out, double* gs_out) {
  const float *ti = Twc + 8 * ix, *qi = Twc + 8 * ix + 3, *si = Twc + 8 * ix + 7;
  const float *tj = Twc + 8 * jx, *qj = Twc + 8 * jx + 3, *sj = Twc + 8 * jx + 7;
  float tij[3], qij[4], sij[1];
  relSim3(ti, qi, si, tj, qj, sj, tij, qij, sij);
  double hij[105], vi[7], vj[7];
  memset(hij, 0, sizeof(hij));
  memset(vi, 0, sizeof(vi));
  memset(vj, 0, sizeof(vj));
  const float s0_inv = (float)(1.0 / (double)prm->sig0);
  const float s1_inv = (float)(1.0 / (double)prm->sig1);
  for (int64_t k = 0; k < N; k++) {
    const int vm = valid_match[k] != 0;
    const int64_t ind = vm ? idx[k] : 0;
    const float* Xi = Xs + ((int64_t)ix * N + ind) * 3;
    const float* Xj = Xs + ((int64_t)jx * N + k) * 3;
    float P[3];
    actSim3(tij, qij, sij, Xj, P);
    const float q = Q[k];
    const float ci = Cs[(int64_t)ix * N + ind];
    const float cj = Cs[(int64_t)jx * N + k];
    int valid = vm & (q > prm->Q_thresh) & (ci > prm->C_thresh) & (cj > prm->C_thresh);
    float Jx[14];
    float* Ji = Jx;
    if (prm->mode == 0) {
      const float norm2_i = Xi[0] * Xi[0] + Xi[1] * Xi[1] + Xi[2] * Xi[2];
      const float norm1_i = sqrtf(norm2_i);
      const float norm1_i_inv = (float)(1.0 / (double)norm1_i);
      float ri[3];
      for (int i = 0; i < 3; i++) ri[i] = norm1_i_inv * Xi[i];
      const float norm2_j = P[0] * P[0] + P[1] * P[1] + P[2] * P[2];
      const float norm1_j = sqrtf(norm2_j);
      const float norm1_j_inv = (float)(1.0 / (double)norm1_j);
      float rj[3];
      for (int i = 0; i < 3; i++) rj[i] = norm1_j_inv * P[i];
      float err[4] = {rj[0] - ri[0], rj[1] - ri[1], rj[2] - ri[2], norm1_j - norm1_i};
      const float swr = valid ? s0_inv * sqrtf(q) : 0;
      const float swd = valid ? s1_inv * sqrtf(q) : 0;
      float w[4] = {huber(swr * err[0]), huber(swr * err[1]), huber(swr * err[2]),
                    huber(swd * err[3])};
      const float cr = swr * swr, cd = swd * swd;
      w[0] *= cr;
      w[1] *= cr;
      w[2] *= cr;
      w[3] *= cd;
      const float n3 = norm1_j_inv / norm2_j;
      const float drx_dPx = norm1_j_inv - P[0] * P[0] * n3;
      const float dry_dPy = norm1_j_inv - P[1] * P[1] * n3;
      const float drz_dPz = norm1_j_inv - P[2] * P[2] * n3;
      const float drx_dPy = -P[0] * P[1] * n3;
      const float drx_dPz = -P[0] * P[2] * n3;
      const float dry_dPz = -P[1] * P[2] * n3;
      float rows[4][7] = {{drx_dPx, drx_dPy, drx_dPz, 0.0f, rj[2], -rj[1], 0.0f},
                          {drx_dPy, dry_dPy, dry_dPz, -rj[2], 0.0f, rj[0], 0.0f},
                          {drx_dPz, dry_dPz, drz_dPz, rj[1], -rj[0], 0.0f, 0.0f},
                          {rj[0], rj[1], rj[2], 0.0f, 0.0f, 0.0f, norm1_j}};
      for (int r = 0; r < 4; r++) {
        memcpy(Ji, rows[r], sizeof(float) * 7);
        accumulate_row(hij, vi, vj, w[r], err[r], Jx, ti, qi, si);
      }
    } else if (prm->mode == 1) {
      const int u_target = (int)(ind % prm->width);
      const int v_target = (int)(ind / prm->width);
      const int valid_z = (P[2] > prm->z_eps) && (Xi[2] > prm->z_eps);
      const float zj_inv = valid_z ? (float)(1.0 / (double)P[2]) : 0.0f;
      const float zj_log = valid_z ? logf(P[2]) : 0.0f;
      const float zi_log = valid_z ? logf(Xi[2]) : 0.0f;
      const float x_div_z = P[0] * zj_inv;
      const float y_div_z = P[1] * zj_inv;
      const float u = prm->fx * x_div_z + prm->cx;
      const float v = prm->fy * y_div_z + prm->cy;
      const int valid_u = (u > prm->pixel_border) && (u < prm->width - 1 - prm->pixel_border);
      const int valid_v = (v > prm->pixel_border) && (v < prm->height - 1 - prm->pixel_border);
      float err[3] = {u - u_target, v - v_target, zj_log - zi_log};
      valid = valid & valid_u & valid_v & valid_z;
      const float swp = valid ? s0_inv * sqrtf(q) : 0;
      const float swd = valid ? s1_inv * sqrtf(q) : 0;
      float w[3] = {huber(swp * err[0]), huber(swp * err[1]), huber(swd * err[2])};
      w[0] *= swp * swp;
      w[1] *= swp * swp;
      w[2] *= swd * swd;
      const float fx = prm->fx, fy = prm->fy;
      float rows[3][7] = {
          {fx * zj_inv, 0.0f, -fx * x_div_z * zj_inv, -fx * x_div_z * y_div_z,
           fx * (1 + x_div_z * x_div_z), -fx * y_div_z, 0.0f},
          {0.0f, fy * zj_inv, -fy * y_div_z * zj_inv, -fy * (1 + y_div_z * y_div_z),
           fy * x_div_z * y_div_z, fy * x_div_z, 0.0f},
          {0.0f, 0.0f, zj_inv, y_div_z, -x_div_z, 0.0f, 1.0f}};
      for (int r = 0; r < 3; r++) {
        memcpy(Ji, rows[r], sizeof(float) * 7);
        accumulate_row(hij, vi, vj, w[r], err[r], Jx, ti, qi, si);
      }
    } else {
      float err[3] = {P[0] - Xi[0], P[1] - Xi[1], P[2] - Xi[2]};
      const float swp = valid ? s0_inv * sqrtf(q) : 0;
      float w[3] = {huber(swp * err[0]), huber(swp * err[1]), huber(swp * err[2])};
      for (int r = 0; r < 3; r++) w[r] *= swp * swp;
      float rows[3][7] = {{1.0f, 0.0f, 0.0f, 0.0f, P[2], -P[1], P[0]},
                          {0.0f, 1.0f, 0.0f, -P[2], 0, P[0], P[1]},
                          {0.0f, 0.0f, 1.0f, P[1], -P[0], 0, P[2]}};
      for (int r = 0; r < 3; r++) {
        memcpy(Ji, rows[r], sizeof(float) * 7);
        accumulate_row(hij, vi, vj, w[r], err[r], Jx, ti, qi, si);
      }
    }
  }
  int l = 0;
  for (int n = 0; n < 14; n++)
    for (int m = 0; m <= n; m++) {
      const double v = hij[l++];
      if (n < 7 && m < 7) {
        Hs_out[0 * 49 + n * 7 + m] = v;
        Hs_out[0 * 49 + m * 7 + n] = v;
      } else if (n >= 7 && m < 7) {
        Hs_out[1 * 49 + m * 7 + (n - 7)] = v;
        Hs_out[2 * 49 + (n - 7) * 7 + m] = v;
      } else {
        Hs_out[3 * 49 + (n - 7) * 7 + (m - 7)] = v;
        Hs_out[3 * 49 + (m - 7) * 7 + (n - 7)] = v;
      }
    }
  for (int n = 0; n < 7; n++) {
    gs_out[n] = vi[n];
    gs_out[7 + n] = vj[n];
  }
}

/* ranks in sorted unique(ii ∪ jj) — torch::_unique(sorted) + searchsorted */
static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}
static int64_t rank_of(const int64_t* uniq, int64_t nu, int64_t v) {
  int64_t lo = 0, hi = nu;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (uniq[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

/* Returns: number of iterations run; *not_pd set if any Cholesky failed.
 * H_first/g_first (optional): per-edge Hs [E][4][7][7] and gs [E][2][7] of iteration 0. */
int ref_gauss_newton(const gn_params* prm, float* Twc, const float* Xs, const float* Cs,
                     const int64_t* ii, const int64_t* jj, const int64_t* idx,
                     const uint8_t* valid_match, const float* Q, int64_t P, int64_t N, int64_t E,
                     int max_iter, float delta_thresh, float* dx_out, double* H_first,
                     double* g_first, int* not_pd) {
  *not_pd = 0;
  int64_t* vals = (int64_t*)malloc(sizeof(int64_t) * 2 * E);
  memcpy(vals, ii, sizeof(int64_t) * E);
  memcpy(vals + E, jj, sizeof(int64_t) * E);
  qsort(vals, 2 * E, sizeof(int64_t), cmp_i64);
  int64_t nu = 0;
  for (int64_t i = 0; i < 2 * E; i++)
    if (i == 0 || vals[i] != vals[i - 1]) vals[nu++] = vals[i];
  int* rii = (int*)malloc(sizeof(int) * E);
  int* rjj = (int*)malloc(sizeof(int) * E);
  for (int64_t e = 0; e < E; e++) {
    rii[e] = (int)rank_of(vals, nu, ii[e]);
    rjj[e] = (int)rank_of(vals, nu, jj[e]);
  }
  const int num_fix = 1;
  const int64_t n = 7 * (P - num_fix);
  double* Hs = (double*)malloc(sizeof(double) * E * 4 * 49);
  double* gs = (double*)malloc(sizeof(double) * E * 2 * 7);
  double* A = (double*)malloc(sizeof(double) * (n > 0 ? n * n : 1));
  double* b = (double*)malloc(sizeof(double) * (n > 0 ? n : 1));
  int itr;
  memset(dx_out, 0, sizeof(float) * (n > 0 ? n : 0));
  for (itr = 0; itr < max_iter; itr++) {
    /* edges are independent (each sums its own points in order): OpenMP over edges keeps
     * every per-edge sum, hence the result, identical to the serial loop */
#pragma omp parallel for schedule(dynamic)
    for (int64_t e = 0; e < E; e++)
      edge_system(prm, Twc, Xs, Cs, rii[e], rjj[e], idx + e * N, valid_match + e * N, Q + e * N,
                  N, Hs + e * 196, gs + e * 14);
    if (itr == 0 && H_first) memcpy(H_first, Hs, sizeof(double) * E * 196);
    if (itr == 0 && g_first) memcpy(g_first, gs, sizeof(double) * E * 14);
    /* assemble (setFromTriplets sums duplicates) — rows/cols of the fixed pose dropped */
    memset(A, 0, sizeof(double) * n * n);
    memset(b, 0, sizeof(double) * n);
    for (int64_t e = 0; e < E; e++) {
      const int oi = rii[e] - num_fix, oj = rjj[e] - num_fix;
      const int bi[4] = {oi, oi, oj, oj}, bj[4] = {oi, oj, oi, oj};
      for (int k = 0; k < 4; k++) {
        if (bi[k] < 0 || bj[k] < 0) continue;
        for (int r = 0; r < 7; r++)
          for (int c = 0; c < 7; c++)
            A[(7 * bi[k] + r) * n + 7 * bj[k] + c] += Hs[e * 196 + k * 49 + r * 7 + c];
      }
      if (oi >= 0)
        for (int r = 0; r < 7; r++) b[7 * oi + r] += gs[e * 14 + r];
      if (oj >= 0)
        for (int r = 0; r < 7; r++) b[7 * oj + r] += gs[e * 14 + 7 + r];
    }
    /* Cholesky (LL^T), fails on a non-positive pivot like SimplicialLLT */
    int ok = 1;
    for (int64_t j = 0; j < n && ok; j++) {
      double s = A[j * n + j];
      for (int64_t k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
      if (!(s > 0.0)) {
        ok = 0;
        break;
      }
      const double d = sqrt(s);
      A[j * n + j] = d;
      for (int64_t i = j + 1; i < n; i++) {
        double t = A[i * n + j];
        for (int64_t k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
        A[i * n + j] = t / d;
      }
    }
    if (ok) {
      for (int64_t i = 0; i < n; i++) {
        double t = b[i];
        for (int64_t k = 0; k < i; k++) t -= A[i * n + k] * b[k];
        b[i] = t / A[i * n + i];
      }
      for (int64_t i = n - 1; i >= 0; i--) {
        double t = b[i];
        for (int64_t k = i + 1; k < n; k++) t -= A[k * n + i] * b[k];
        b[i] = t / A[i * n + i];
      }
      for (int64_t i = 0; i < n; i++) dx_out[i] = (float)(-b[i]); /* dx = -A.solve() */
    } else {
      *not_pd = 1;
      for (int64_t i = 0; i < n; i++) dx_out[i] = 0.0f;
    }
    /* pose_retr_kernel (:415-453) */
    for (int64_t k = num_fix; k < P; k++) {
      float out[8];
      retrSim3(dx_out + 7 * (k - num_fix), Twc + 8 * k, Twc + 8 * k + 3, Twc + 8 * k + 7, out,
               out + 3, out + 7);
      memcpy(Twc + 8 * k, out, sizeof(out));
    }
    double ss = 0.0;
    for (int64_t i = 0; i < n; i++) ss += (double)dx_out[i] * (double)dx_out[i];
    if ((float)sqrt(ss) < delta_thresh) {
      itr++;
      break;
    }
  }
  free(vals);
  free(rii);
  free(rjj);
  free(Hs);
  free(gs);
  free(A);
  free(b);
  return itr;
}
