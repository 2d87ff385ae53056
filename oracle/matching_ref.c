/*
 * ORACLE — test infrastructure only (never shipped, never on the product path).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * CPU restatement of the reference's projective-matching CUDA kernels
 * (/root/reference/MASt3R-SLAM/mast3r_slam/backend/src/matching_kernels.cu), written in
 * plain C from the reference's algorithm.  Numerical model (must be compiled with
 * -ffp-contract=off, see oracle/Makefile):
 *   iter_proj      — the source taken literally: f32 ops without contraction; the
 *                    sub-expressions the reference writes with double literals
 *                    (1.0/x, (1.0-du)*dv, lambda *= 0.1 / 10.0) are evaluated in f64.
 *   refine_matches — c10::Half arithmetic (torch Half-inl.h: operator* and operator+=
 *                    go through float and round to half, RNE); initial max score is the
 *                    value-initialised Half, +0.0 (cuda::std::numeric_limits has no
 *                    c10::Half specialisation).
 * The reference CUDA cannot be compiled here (no CUDA toolkit), so parity with it is
 * pinned by this restatement plus the known-answer tests in tests/ (identity pointmaps,
 * one-hot descriptors), and by goldens of the Python prep (tests/golden/).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <immintrin.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- IEEE half helpers (RNE, subnormals, inf/nan) ---------------------- */
static float half_to_float(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t exp = (h >> 10) & 0x1fu;
  const uint32_t man = h & 0x3ffu;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else { /* subnormal: value = man * 2^-24 */
      float f = (float)man * 5.9604644775390625e-08f;
      memcpy(&bits, &f, 4);
      bits |= sign;
    }
  } else if (exp == 31) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp + 112u) << 23) | (man << 13);
  }
  float out;
  memcpy(&out, &bits, 4);
  return out;
}

static uint16_t float_to_half(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  const uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) { /* inf or nan */
    return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
  }
  if (absx >= 0x477ff000u) { /* >= 65520 rounds to inf */
    return (uint16_t)(sign | 0x7c00u);
  }
  if (absx < 0x38800000u) { /* below smallest normal half (2^-14): subnormal or zero */
    /* value in units of 2^-24, rounded to nearest even */
    float a;
    memcpy(&a, &absx, 4);
    float scaled = a * 16777216.0f; /* exact (power of two) */
    /* nearbyintf uses the current rounding mode (RNE by default) */
    float r = nearbyintf(scaled);
    return (uint16_t)(sign | (uint16_t)r);
  }
  /* normal: keep 10 mantissa bits, RNE on the 13 dropped bits */
  uint32_t e = (absx >> 23) - 112u;
  uint32_t m = absx & 0x7fffffu;
  uint32_t hm = m >> 13;
  uint32_t rem = m & 0x1fffu;
  uint32_t hv = (e << 10) | hm;
  if (rem > 0x1000u || (rem == 0x1000u && (hm & 1u))) hv += 1u; /* may carry into exp */
  return (uint16_t)(sign | hv);
}

uint16_t ref_float_to_half(float f) { return float_to_half(f); }
float ref_half_to_float(uint16_t h) { return half_to_float(h); }

/* ---- iter_proj (matching_kernels.cu:119-275) ----------------------------- */
static float clampf_ref(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

static void bilinear(const float* img, int w, int C, float u, float v, int nch, float* out) {
  int u11 = (int)floorf(u);
  int v11 = (int)floorf(v);
  float du = u - (float)u11;
  float dv = v - (float)v11;
  float w11 = du * dv;
  float w12 = (float)((1.0 - (double)du) * (double)dv);
  float w21 = (float)((double)du * (1.0 - (double)dv));
  float w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
  const float* r11 = img + ((int64_t)(v11 + 1) * w + (u11 + 1)) * C; /* bottom right */
  const float* r12 = img + ((int64_t)(v11 + 1) * w + u11) * C;       /* bottom left */
  const float* r21 = img + ((int64_t)v11 * w + (u11 + 1)) * C;       /* top right */
  const float* r22 = img + ((int64_t)v11 * w + u11) * C;             /* top left */
  for (int j = 0; j < nch; j++) {
    float s = w11 * r11[j];
    s = s + w12 * r12[j];
    s = s + w21 * r21[j];
    s = s + w22 * r22[j];
    out[j] = s;
  }
}

void ref_iter_proj(const float* rays, const float* pts, const float* p_init, float* p_new,
                   uint8_t* converged, int64_t b, int64_t h, int64_t w, int64_t n, int C,
                   int max_iter, float lambda_init, float cost_thresh) {
  for (int64_t bi = 0; bi < b; bi++) {
    const float* img = rays + bi * h * w * C;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; i++) {
      const int64_t q = bi * n + i;
      float u = p_init[2 * q], v = p_init[2 * q + 1];
      u = clampf_ref(u, 1.0f, (float)(w - 2));
      v = clampf_ref(v, 1.0f, (float)(h - 2));
      float lambda = lambda_init;
      uint8_t conv = 0;
      for (int it = 0; it < max_iter; it++) {
        float s[9];
        bilinear(img, (int)w, C, u, v, 9, s);
        float r_norm = sqrtf(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
        float r_norm_inv = (float)(1.0 / (double)r_norm);
        float r[3] = {s[0] * r_norm_inv, s[1] * r_norm_inv, s[2] * r_norm_inv};
        float err[3] = {r[0] - pts[3 * q], r[1] - pts[3 * q + 1], r[2] - pts[3 * q + 2]};
        float cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        const float* gx = s + 3;
        const float* gy = s + 6;
        float A00 = gx[0] * gx[0] + gx[1] * gx[1] + gx[2] * gx[2];
        float A01 = gx[0] * gy[0] + gx[1] * gy[1] + gx[2] * gy[2];
        float A11 = gy[0] * gy[0] + gy[1] * gy[1] + gy[2] * gy[2];
        float b0 = -(err[0] * gx[0] + err[1] * gx[1] + err[2] * gx[2]);
        float b1 = -(err[0] * gy[0] + err[1] * gy[1] + err[2] * gy[2]);
        A00 += lambda;
        A11 += lambda;
        float det_inv = (float)(1.0 / (double)(A00 * A11 - A01 * A01));
        float delta_u = det_inv * (A11 * b0 - A01 * b1);
        float delta_v = det_inv * (-A01 * b0 + A00 * b1);
        float u_new = u + delta_u;
        float v_new = v + delta_v;
        u_new = clampf_ref(u_new, 1.0f, (float)(w - 2));
        v_new = clampf_ref(v_new, 1.0f, (float)(h - 2));
        bilinear(img, (int)w, C, u_new, v_new, 3, r);
        r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
        r_norm_inv = (float)(1.0 / (double)r_norm);
        for (int j = 0; j < 3; j++) r[j] *= r_norm_inv;
        for (int j = 0; j < 3; j++) err[j] = r[j] - pts[3 * q + j];
        float new_cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
        if (new_cost < cost) {
          u = u_new;
          v = v_new;
          lambda = (float)((double)lambda * 0.1);
          conv = new_cost < cost_thresh;
        } else {
          lambda = (float)((double)lambda * 10.0);
          conv = cost < cost_thresh;
        }
      }
      p_new[2 * q] = u;
      p_new[2 * q + 1] = v;
      converged[q] = conv;
    }
  }
}

/* ---- iter_proj, contracted model ----------------------
 * The reference is built by nvcc -O3 (setup.py:29-36), whose default --fmad=true lets the
 * compiler fuse a product into the add / subtract that consumes it.  This variant applies
 * the fusions LLVM's DAG combiner (NVPTX enables aggressive FMA fusion, no reassociation)
 * makes on matching_kernels.cu:154-228 as written — a sum of products a0*b0 + a1*b1 + ...
 * becomes fma(a_k, b_k, ... fma(a1, b1, a0*b0)) with the FIRST product fused into the
 * second add (fadd(fmul N0, fmul N1) -> fma(N0.x, N0.y, N1)), a difference of products
 * fma(x, y, -(z*w)), and the consumer of a single-use product is fused with it:
 *   bilinear   fma(w22,r22, fma(w21,r21, fma(w11,r11, w12*r12)))
 *   |r|^2      fma(r2,r2, fma(r0,r0, r1*r1))            (also cost, A00, A01, A11, b0, b1)
 *   err_j      fma(r_j, r_norm_inv, -pts_j)               (r *= inv then r - pts)
 *   det        fma(A00, A11, -(A01*A01))
 *   delta      fma(A11, b0, -(A01*b1)), fma(-A01, b0, A00*b1)
 *   u + delta  fma(det_inv, (A11 b0 - A01 b1), u)         (delta_u = det_inv * (...))
 * The f64 sub-expressions stay f64 (1.0/x, (1.0-du)*dv: a product of a difference, no
 * fusion).  Which fusions the proprietary nvcc front end actually emits cannot be checked
 * here (no CUDA toolkit); DESIGN §2 records how far the two models' results differ. */
static float dot3c(const float* a, const float* b) {
  return fmaf(a[2], b[2], fmaf(a[0], b[0], a[1] * b[1]));
}

static void bilinear_c(const float* img, int w, int C, float u, float v, int nch, float* out) {
  int u11 = (int)floorf(u);
  int v11 = (int)floorf(v);
  float du = u - (float)u11;
  float dv = v - (float)v11;
  float w11 = du * dv;
  float w12 = (float)((1.0 - (double)du) * (double)dv);
  float w21 = (float)((double)du * (1.0 - (double)dv));
  float w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
  const float* r11 = img + ((int64_t)(v11 + 1) * w + (u11 + 1)) * C;
  const float* r12 = img + ((int64_t)(v11 + 1) * w + u11) * C;
  const float* r21 = img + ((int64_t)v11 * w + (u11 + 1)) * C;
  const float* r22 = img + ((int64_t)v11 * w + u11) * C;
  for (int j = 0; j < nch; j++)
    out[j] = fmaf(w22, r22[j], fmaf(w21, r21[j], fmaf(w11, r11[j], w12 * r12[j])));
}

void ref_iter_proj_fma(const float* rays, const float* pts, const float* p_init, float* p_new,
                       uint8_t* converged, int64_t b, int64_t h, int64_t w, int64_t n, int C,
                       int max_iter, float lambda_init, float cost_thresh) {
  for (int64_t bi = 0; bi < b; bi++) {
    const float* img = rays + bi * h * w * C;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; i++) {
      const int64_t q = bi * n + i;
      const float* t = pts + 3 * q;
      float u = clampf_ref(p_init[2 * q], 1.0f, (float)(w - 2));
      float v = clampf_ref(p_init[2 * q + 1], 1.0f, (float)(h - 2));
      float lambda = lambda_init;
      uint8_t conv = 0;
      for (int it = 0; it < max_iter; it++) {
        float s[9], err[3], r[3];
        bilinear_c(img, (int)w, C, u, v, 9, s);
        float r_norm = sqrtf(dot3c(s, s));
        float r_norm_inv = (float)(1.0 / (double)r_norm);
        for (int j = 0; j < 3; j++) err[j] = fmaf(s[j], r_norm_inv, -t[j]);
        float cost = dot3c(err, err);
        const float* gx = s + 3;
        const float* gy = s + 6;
        float A00 = dot3c(gx, gx);
        float A01 = dot3c(gx, gy);
        float A11 = dot3c(gy, gy);
        float b0 = -dot3c(err, gx);
        float b1 = -dot3c(err, gy);
        A00 += lambda;
        A11 += lambda;
        float det_inv = (float)(1.0 / (double)fmaf(A00, A11, -(A01 * A01)));
        float u_new = fmaf(det_inv, fmaf(A11, b0, -(A01 * b1)), u);
        float v_new = fmaf(det_inv, fmaf(-A01, b0, A00 * b1), v);
        u_new = clampf_ref(u_new, 1.0f, (float)(w - 2));
        v_new = clampf_ref(v_new, 1.0f, (float)(h - 2));
        bilinear_c(img, (int)w, C, u_new, v_new, 3, r);
        r_norm = sqrtf(dot3c(r, r));
        r_norm_inv = (float)(1.0 / (double)r_norm);
        for (int j = 0; j < 3; j++) err[j] = fmaf(r[j], r_norm_inv, -t[j]);
        float new_cost = dot3c(err, err);
        if (new_cost < cost) {
          u = u_new;
          v = v_new;
          lambda = (float)((double)lambda * 0.1);
          conv = new_cost < cost_thresh;
        } else {
          lambda = (float)((double)lambda * 10.0);
          conv = cost < cost_thresh;
        }
      }
      p_new[2 * q] = u;
      p_new[2 * q + 1] = v;
      converged[q] = conv;
    }
  }
}

/* ---- refine_matches (matching_kernels.cu:25-81) --------------------------- */
static void refine_soft(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                        int64_t* p1_new, int64_t b, int64_t h, int64_t w, int64_t n,
                        int64_t fdim, int radius, int dilation_max) {
  for (int64_t bi = 0; bi < b; bi++) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256)
#endif
    for (int64_t i = 0; i < n; i++) {
      const int64_t q = bi * n + i;
      int64_t u0 = p1[2 * q], v0 = p1[2 * q + 1];
      uint16_t max_score = 0; /* value-initialised c10::Half: +0.0 */
      int64_t u_new = u0, v_new = v0;
      for (int d = dilation_max; d > 0; d--) {
        const int rd = radius * d;
        const int diam = 2 * rd + 1;
        for (int ii = 0; ii < diam; ii += d) {
          for (int jj = 0; jj < diam; jj += d) {
            const int64_t u = u0 - rd + ii;
            const int64_t v = v0 - rd + jj;
            if (v >= 0 && v < h && u >= 0 && u < w) {
              const uint16_t* a = D21 + q * fdim;
              const uint16_t* c = D11 + ((bi * h + v) * w + u) * fdim;
              uint16_t score = 0;
              for (int64_t k = 0; k < fdim; k++) {
                /* Half operator*: float product, converted to Half */
                uint16_t prod = float_to_half(half_to_float(a[k]) * half_to_float(c[k]));
                /* Half operator+=: float sum, converted to Half */
                score = float_to_half(half_to_float(score) + half_to_float(prod));
              }
              if (half_to_float(score) > half_to_float(max_score)) {
                max_score = score;
                u_new = u;
                v_new = v;
              }
            }
          }
        }
        u0 = u_new;
        v0 = v_new;
      }
      p1_new[2 * q] = u_new;
      p1_new[2 * q + 1] = v_new;
    }
  }
}

/* Same arithmetic with the x86 AVX2 + F16C conversions (VCVTPS2PH with explicit round-to-nearest-
 * even: the IEEE rounding float_to_half implements; VCVTPH2PS is exact) and the half
 * operands widened to float once.  Inputs of the conversions are never f32 denormals here
 * (products of two halves are >= 2^-48 in magnitude or exactly 0), so MXCSR.DAZ/FTZ do not
 * change results.  tests/test_oracle_matching.py checks both paths agree bit for bit. */
__attribute__((target("avx2,f16c"))) static inline __m256 rh8(__m256 x) {
  return _mm256_cvtph_ps(_mm256_cvtps_ph(x, _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC));
}

/* Eight candidates' sequential half chains side by side (each lane keeps its own k order);
 * the argmax then scans the scores in the reference's candidate order. */
__attribute__((target("avx2,f16c"))) static void refine_f16c(
    const uint16_t* D11, const uint16_t* D21, const int64_t* p1, int64_t* p1_new, int64_t b,
    int64_t h, int64_t w, int64_t n, int64_t fdim, int radius, int dilation_max) {
  float* F11 = (float*)malloc(sizeof(float) * (size_t)(b * h * w * fdim));
  float* F21 = (float*)malloc(sizeof(float) * (size_t)(b * n * fdim));
  for (int64_t i = 0; i < b * h * w * fdim; i++) F11[i] = _cvtsh_ss(D11[i]);
  for (int64_t i = 0; i < b * n * fdim; i++) F21[i] = _cvtsh_ss(D21[i]);
  const int maxc = (2 * radius + 1) * (2 * radius + 1) + 8;
  for (int64_t bi = 0; bi < b; bi++) {
    const float* F11b = F11 + bi * h * w * fdim;
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
      int* offs = (int*)malloc(sizeof(int) * (size_t)maxc);
      int* cu = (int*)malloc(sizeof(int) * (size_t)maxc);
      int* cv = (int*)malloc(sizeof(int) * (size_t)maxc);
      float* sc = (float*)malloc(sizeof(float) * (size_t)maxc);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
      for (int64_t i = 0; i < n; i++) {
        const int64_t q = bi * n + i;
        int64_t u0 = p1[2 * q], v0 = p1[2 * q + 1];
        float max_score = 0.0f; /* value-initialised c10::Half: +0.0 */
        int64_t u_new = u0, v_new = v0;
        const float* a = F21 + q * fdim;
        for (int d = dilation_max; d > 0; d--) {
          const int rd = radius * d;
          const int diam = 2 * rd + 1;
          int m = 0;
          for (int ii = 0; ii < diam; ii += d)
            for (int jj = 0; jj < diam; jj += d) {
              const int64_t u = u0 - rd + ii;
              const int64_t v = v0 - rd + jj;
              if (v >= 0 && v < h && u >= 0 && u < w) {
                offs[m] = (int)((v * w + u) * fdim);
                cu[m] = (int)u;
                cv[m] = (int)v;
                m++;
              }
            }
          for (int j = m; j < ((m + 7) & ~7); j++) offs[j] = m ? offs[0] : 0;
          for (int m0 = 0; m0 < m; m0 += 8) {
            const __m256i idx = _mm256_loadu_si256((const __m256i*)(offs + m0));
            __m256 score = _mm256_setzero_ps();
            for (int64_t k = 0; k < fdim; k++) {
              const __m256 c = _mm256_i32gather_ps(F11b + k, idx, 4);
              const __m256 prod = rh8(_mm256_mul_ps(_mm256_set1_ps(a[k]), c));
              score = rh8(_mm256_add_ps(score, prod));
            }
            _mm256_storeu_ps(sc + m0, score);
          }
          for (int j = 0; j < m; j++)
            if (sc[j] > max_score) {
              max_score = sc[j];
              u_new = cu[j];
              v_new = cv[j];
            }
          u0 = u_new;
          v0 = v_new;
        }
        p1_new[2 * q] = u_new;
        p1_new[2 * q + 1] = v_new;
      }
      free(offs);
      free(cu);
      free(cv);
      free(sc);
    }
  }
  free(F11);
  free(F21);
}

/* ORACLE_SOFT_HALF=1 (or a CPU without AVX2/F16C) selects the bit-level software path. */
void ref_refine_matches(const uint16_t* D11, const uint16_t* D21, const int64_t* p1,
                        int64_t* p1_new, int64_t b, int64_t h, int64_t w, int64_t n,
                        int64_t fdim, int radius, int dilation_max) {
  const char* e = getenv("ORACLE_SOFT_HALF");
  if ((!e || atoi(e) == 0) && __builtin_cpu_supports("f16c") && __builtin_cpu_supports("avx2"))
    refine_f16c(D11, D21, p1, p1_new, b, h, w, n, fdim, radius, dilation_max);
  else
    refine_soft(D11, D21, p1, p1_new, b, h, w, n, fdim, radius, dilation_max);
}

/* ---- matching prep (matching.py:25-49, image.py:5-38) ---------------------
 * Accumulation order pinned to the reference's torch-CPU run (tests/golden): vector
 * norms are a sequential FMA chain x0*x0 → fma(x1,x1,·) → fma(x2,x2,·); the depthwise
 * 3x3 conv is a sequential FMA over the 9 taps in row-major order (zero taps included). */
static void normalize3(const float* x, float* o) {
  float n = sqrtf(fmaf(x[2], x[2], fmaf(x[1], x[1], x[0] * x[0])));
  n = fmaxf(n, 1e-12f);
  o[0] = x[0] / n;
  o[1] = x[1] / n;
  o[2] = x[2] / n;
}

static int reflect1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

void ref_match_prep(const float* X11, const float* X21, const int64_t* idx_init, float* rwg,
                    float* pts, float* p_init, int64_t b, int64_t h, int64_t w) {
  const float W[3][3] = {{-3.0f / 32.0f, 0.0f, 3.0f / 32.0f},
                         {-10.0f / 32.0f, 0.0f, 10.0f / 32.0f},
                         {-3.0f / 32.0f, 0.0f, 3.0f / 32.0f}};
  const int64_t npix = h * w;
  for (int64_t bi = 0; bi < b; bi++) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < npix; i++) {
      const int y = (int)(i / w), x = (int)(i % w);
      float nb[3][3][3];
      for (int dy = 0; dy < 3; dy++)
        for (int dx = 0; dx < 3; dx++) {
          const int yy = reflect1(y + dy - 1, (int)h), xx = reflect1(x + dx - 1, (int)w);
          normalize3(X11 + ((bi * h + yy) * w + xx) * 3, nb[dy][dx]);
        }
      float* o = rwg + (bi * npix + i) * 9;
      for (int c = 0; c < 3; c++) {
        float gx = 0.0f, gy = 0.0f;
        for (int ky = 0; ky < 3; ky++)
          for (int kx = 0; kx < 3; kx++) {
            gx = fmaf(W[ky][kx], nb[ky][kx][c], gx);
            gy = fmaf(W[kx][ky], nb[ky][kx][c], gy); /* gy kernel = gx kernel transposed */
          }
        o[c] = nb[1][1][c];
        o[3 + c] = gx;
        o[6 + c] = gy;
      }
      normalize3(X21 + (bi * npix + i) * 3, pts + (bi * npix + i) * 3);
      const int64_t idx = idx_init ? idx_init[bi * npix + i] : i;
      p_init[(bi * npix + i) * 2] = (float)(idx % w);
      p_init[(bi * npix + i) * 2 + 1] = (float)(idx / w);
    }
  }
}

/* matching.py:67-76 */
void ref_match_occlusion(const float* X11, const float* X21, const float* p,
                         const uint8_t* conv, int64_t* p1, uint8_t* valid, int64_t b, int64_t h,
                         int64_t w, float dist_thresh) {
  const int64_t npix = h * w;
  for (int64_t q = 0; q < b * npix; q++) {
    const int64_t bi = q / npix;
    const int64_t u = (int64_t)p[2 * q], v = (int64_t)p[2 * q + 1];
    p1[2 * q] = u;
    p1[2 * q + 1] = v;
    const float* a = X11 + ((bi * h + v) * w + u) * 3;
    const float* c = X21 + q * 3;
    const float d0 = a[0] - c[0], d1 = a[1] - c[1], d2 = a[2] - c[2];
    const float d = sqrtf(fmaf(d2, d2, fmaf(d1, d1, d0 * d0)));
    valid[q] = (conv[q] && d < dist_thresh) ? 1 : 0;
  }
}

/* OpenMP thread count of the restatement (the CPU baseline uses every host core). */
void ref_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}
