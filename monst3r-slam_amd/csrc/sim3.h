// Sim3 / SO3 device math (lietorch conventions: data = [t xyz, q xyzw, s]; tangent
// order (tau, omega, sigma); retraction = Exp(xi) * X from the left).
// Formulas follow lietorch's rxso3.h / sim3.h as restated in the reference's
// gn_kernels.cu:178-413 (quat_comp, actSO3, relSim3, apply_Sim3_adj_inv, expSO3,
// expSim3, retrSim3).  Templated on the scalar so the fp64 solve path can reuse it.
#pragma once
#include <hip/hip_runtime.h>

#define M3S_SIM3_EPS 1e-6

template <typename T>
__host__ __device__ __forceinline__ void m3s_quat_comp(const T* qi, const T* qj, T* out) {
  out[0] = qi[3] * qj[0] + qi[0] * qj[3] + qi[1] * qj[2] - qi[2] * qj[1];
  out[1] = qi[3] * qj[1] - qi[0] * qj[2] + qi[1] * qj[3] + qi[2] * qj[0];
  out[2] = qi[3] * qj[2] + qi[0] * qj[1] - qi[1] * qj[0] + qi[2] * qj[3];
  out[3] = qi[3] * qj[3] - qi[0] * qj[0] - qi[1] * qj[1] - qi[2] * qj[2];
}

template <typename T>
__host__ __device__ __forceinline__ void m3s_act_so3(const T* q, const T* X, T* Y) {
  T uv[3];
  uv[0] = T(2.0) * (q[1] * X[2] - q[2] * X[1]);
  uv[1] = T(2.0) * (q[2] * X[0] - q[0] * X[2]);
  uv[2] = T(2.0) * (q[0] * X[1] - q[1] * X[0]);
  T y0 = X[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  T y1 = X[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  T y2 = X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
  Y[0] = y0;
  Y[1] = y1;
  Y[2] = y2;
}

// Y = s R X + t
template <typename T>
__host__ __device__ __forceinline__ void m3s_act_sim3(const T* t, const T* q, T s, const T* X,
                                                      T* Y) {
  m3s_act_so3(q, X, Y);
  Y[0] *= s;
  Y[1] *= s;
  Y[2] *= s;
  Y[0] += t[0];
  Y[1] += t[1];
  Y[2] += t[2];
}

// T_ij = T_i^{-1} T_j  (gn_kernels.cu:258-277)
template <typename T>
__host__ __device__ __forceinline__ void m3s_rel_sim3(const T* ti, const T* qi, T si,
                                                      const T* tj, const T* qj, T sj, T* tij,
                                                      T* qij, T* sij) {
  const T si_inv = T(1.0) / si;
  *sij = si_inv * sj;
  T qi_inv[4] = {-qi[0], -qi[1], -qi[2], qi[3]};
  m3s_quat_comp(qi_inv, qj, qij);
  T d[3] = {tj[0] - ti[0], tj[1] - ti[1], tj[2] - ti[2]};
  m3s_act_so3(qi_inv, d, tij);
  tij[0] *= si_inv;
  tij[1] *= si_inv;
  tij[2] *= si_inv;
}

// Y = Adj(T)^{-T}-style action used by the reference (gn_kernels.cu:281-301):
// Y[0:3] = s^-1 R a; Y[3:6] = R b + s^-1 t x (R a); Y[6] = c + s^-1 t.(R a)
template <typename T>
__host__ __device__ __forceinline__ void m3s_adj_inv_apply(const T* t, const T* q, T s,
                                                           const T* X, T* Y) {
  const T s_inv = T(1.0) / s;
  T Ra[3];
  m3s_act_so3(q, X, Ra);
  Y[0] = s_inv * Ra[0];
  Y[1] = s_inv * Ra[1];
  Y[2] = s_inv * Ra[2];
  m3s_act_so3(q, X + 3, Y + 3);
  Y[3] += s_inv * (t[1] * Ra[2] - t[2] * Ra[1]);
  Y[4] += s_inv * (t[2] * Ra[0] - t[0] * Ra[2]);
  Y[5] += s_inv * (t[0] * Ra[1] - t[1] * Ra[0]);
  Y[6] = X[6] + s_inv * (t[0] * Ra[0] + t[1] * Ra[1] + t[2] * Ra[2]);
}

// SO3 exponential (gn_kernels.cu:303-325; lietorch so3.h)
template <typename T>
__host__ __device__ __forceinline__ void m3s_exp_so3(const T* phi, T* q) {
  const T theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  T imag, real;
  if (theta_sq < T(M3S_SIM3_EPS)) {
    const T theta_p4 = theta_sq * theta_sq;
    imag = T(0.5) - T(1.0 / 48.0) * theta_sq + T(1.0 / 3840.0) * theta_p4;
    real = T(1.0) - T(1.0 / 8.0) * theta_sq + T(1.0 / 384.0) * theta_p4;
  } else {
    const T theta = sqrt(theta_sq);
    imag = sin(T(0.5) * theta) / theta;
    real = cos(T(0.5) * theta);
  }
  q[0] = imag * phi[0];
  q[1] = imag * phi[1];
  q[2] = imag * phi[2];
  q[3] = real;
}

// Sim3 exponential (gn_kernels.cu:327-390; lietorch rxso3.h calcW):
// t = (C I + A Phi + B Phi^2) tau, q = exp_so3(phi), s = exp(sigma)
template <typename T>
__host__ __device__ __forceinline__ void m3s_exp_sim3(const T* xi, T* t, T* q, T* s) {
  const T tau[3] = {xi[0], xi[1], xi[2]};
  const T phi[3] = {xi[3], xi[4], xi[5]};
  const T sigma = xi[6];
  const T scale = exp(sigma);
  m3s_exp_so3(phi, q);
  *s = scale;
  const T theta_sq = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  const T theta = sqrt(theta_sq);
  T A, B, C;
  const T one = T(1.0), half = T(0.5);
  if (fabs(sigma) < T(M3S_SIM3_EPS)) {
    C = one;
    if (fabs(theta) < T(M3S_SIM3_EPS)) {
      A = half;
      B = T(1.0 / 6.0);
    } else {
      A = (one - cos(theta)) / theta_sq;
      B = (theta - sin(theta)) / (theta_sq * theta);
    }
  } else {
    C = (scale - one) / sigma;
    if (fabs(theta) < T(M3S_SIM3_EPS)) {
      const T sigma_sq = sigma * sigma;
      A = ((sigma - one) * scale + one) / sigma_sq;
      B = (scale * half * sigma_sq + scale - one - sigma * scale) / (sigma_sq * sigma);
    } else {
      const T a = scale * sin(theta);
      const T b = scale * cos(theta);
      const T c = theta_sq + sigma * sigma;
      A = (a * sigma + (one - b) * theta) / (theta * c);
      B = (C - ((b - one) * sigma + a * theta) / c) / theta_sq;
    }
  }
  t[0] = C * tau[0];
  t[1] = C * tau[1];
  t[2] = C * tau[2];
  // Phi tau = phi x tau
  T c1[3] = {phi[1] * tau[2] - phi[2] * tau[1], phi[2] * tau[0] - phi[0] * tau[2],
             phi[0] * tau[1] - phi[1] * tau[0]};
  t[0] += A * c1[0];
  t[1] += A * c1[1];
  t[2] += A * c1[2];
  T c2[3] = {phi[1] * c1[2] - phi[2] * c1[1], phi[2] * c1[0] - phi[0] * c1[2],
             phi[0] * c1[1] - phi[1] * c1[0]};
  t[0] += B * c2[0];
  t[1] += B * c2[1];
  t[2] += B * c2[2];
}

// Left retraction X1 = Exp(xi) * X  (gn_kernels.cu:392-413)
template <typename T>
__host__ __device__ __forceinline__ void m3s_retr_sim3(const T* xi, const T* t, const T* q, T s,
                                                       T* t1, T* q1, T* s1) {
  T dt[3], dq[4], ds;
  m3s_exp_sim3(xi, dt, dq, &ds);
  m3s_quat_comp(dq, q, q1);
  m3s_act_so3(dq, t, t1);
  t1[0] = t1[0] * ds + dt[0];
  t1[1] = t1[1] * ds + dt[1];
  t1[2] = t1[2] * ds + dt[2];
  *s1 = ds * s;
}
