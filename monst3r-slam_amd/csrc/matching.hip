// Projective matching kernels for gfx950 (MI355X).
//
// Compiled with -ffp-contract=off: every f32 product and sum is rounded on its own,
// exactly as the reference source is written (matching_kernels.cu), and the
// double-promoted sub-expressions of the reference are evaluated in f64.  The CPU
// oracle (oracle/matching_ref.c) follows the same model, so results are bit-exact.
//
// Layout: one lane per query pixel, 256-lane workgroups (4 waves), grid.y = batch.
// Unlike the reference (16-thread blocks, no tail guard, matching_kernels.cu:36,131,
// 290-293) any n is accepted.
#include <stdlib.h>
#include <string.h>
#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float clamp_ref(float x, float lo, float hi) {
  // matching_kernels.cu:22-24  x = fmin(fmax(x, min), max)
  return fminf(fmaxf(x, lo), hi);
}

// Bilinear weights of matching_kernels.cu:143-152 (and :201-209).
struct Bilin {
  int u11, v11;
  float w11, w12, w21, w22;
};

__device__ __forceinline__ Bilin bilin_weights(float u, float v) {
  Bilin r;
  r.u11 = (int)floorf(u);
  r.v11 = (int)floorf(v);
  const float du = u - (float)r.u11;
  const float dv = v - (float)r.v11;
  r.w11 = du * dv;                                             // top left
  r.w12 = (float)((1.0 - (double)du) * (double)dv);            // top right
  r.w21 = (float)((double)du * (1.0 - (double)dv));            // bottom left
  r.w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));    // bottom right
  return r;
}

// r[j] = w11*r11[j] + w12*r12[j] + w21*r21[j] + w22*r22[j], pixels opposite the area
// (matching_kernels.cu:154-158).  img points at the (b) image, row stride w*C floats.
template <int C, int NCH, bool FMA = false>
__device__ __forceinline__ void bilin_sample(const float* __restrict__ img, int w,
                                             const Bilin& bw, float* out) {
  const float* r22 = img + ((int64_t)bw.v11 * w + bw.u11) * C;        // top left
  const float* r21 = r22 + C;                                          // top right
  const float* r12 = r22 + (int64_t)w * C;                             // bottom left
  const float* r11 = r12 + C;                                          // bottom right
#pragma unroll
  for (int j = 0; j < NCH; j++) {
    if (FMA) {   // the contracted model (iter_proj_kernel<C, true>)
      out[j] = __builtin_fmaf(bw.w22, r22[j],
                              __builtin_fmaf(bw.w21, r21[j],
                                             __builtin_fmaf(bw.w11, r11[j], bw.w12 * r12[j])));
    } else {
      float s = bw.w11 * r11[j];
      s = s + bw.w12 * r12[j];
      s = s + bw.w21 * r21[j];
      s = s + bw.w22 * r22[j];
      out[j] = s;
    }
  }
}

// a0*b0 + a1*b1 + a2*b2: uncontracted, or as LLVM contracts it (the first product fused
// into the second add, the third into the result: oracle/matching_ref.c ref_iter_proj_fma)
template <bool FMA>
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
  if (FMA) return __builtin_fmaf(a2, b2, __builtin_fmaf(a0, b0, a1 * b1));
  return a0 * b0 + a1 * b1 + a2 * b2;
}

// FMA = false: the reference source taken literally (every product / sum rounded);
// FMA = true: the FMA-contracted model of nvcc's default --fmad=true (opt-in,
// m3s_iter_proj_fma; oracle/matching_ref.c ref_iter_proj_fma).
template <int C, bool FMA>
__global__ __launch_bounds__(kBlock) void iter_proj_kernel(
    const float* __restrict__ rays_img, const float* __restrict__ pts_3d_norm,
    const float* __restrict__ p_init, float* __restrict__ p_new,
    uint8_t* __restrict__ converged_out, int h, int w, int64_t n, int max_iter,
    float lambda_init, float cost_thresh) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= n) return;
  const float* img = rays_img + b * (int64_t)h * w * C;
  const int64_t q = b * n + i;

  float u = p_init[2 * q + 0];
  float v = p_init[2 * q + 1];
  const float umax = (float)(w - 2), vmax = (float)(h - 2);
  u = clamp_ref(u, 1.0f, umax);
  v = clamp_ref(v, 1.0f, vmax);

  const float t0 = pts_3d_norm[3 * q + 0];
  const float t1 = pts_3d_norm[3 * q + 1];
  const float t2 = pts_3d_norm[3 * q + 2];

  float lambda = lambda_init;
  bool conv = false;
  for (int it = 0; it < max_iter; it++) {
    float s[9];
    Bilin bw = bilin_weights(u, v);
    bilin_sample<C, 9, FMA>(img, w, bw, s);
    // normalise ray (:173-178); 1.0/r_norm is a double division in the reference
    float r_norm = sqrtf(dot3<FMA>(s[0], s[1], s[2], s[0], s[1], s[2]));
    float r_norm_inv = (float)(1.0 / (double)r_norm);
    // err = r * inv - pts (contracted: fma(r, inv, -pts))
    const float e0 = FMA ? __builtin_fmaf(s[0], r_norm_inv, -t0) : s[0] * r_norm_inv - t0;
    const float e1 = FMA ? __builtin_fmaf(s[1], r_norm_inv, -t1) : s[1] * r_norm_inv - t1;
    const float e2 = FMA ? __builtin_fmaf(s[2], r_norm_inv, -t2) : s[2] * r_norm_inv - t2;
    const float cost = dot3<FMA>(e0, e1, e2, e0, e1, e2);
    // J^T J + lambda I, -J^T r  (:187-197)
    float A00 = dot3<FMA>(s[3], s[4], s[5], s[3], s[4], s[5]);
    const float A01 = dot3<FMA>(s[3], s[4], s[5], s[6], s[7], s[8]);
    float A11 = dot3<FMA>(s[6], s[7], s[8], s[6], s[7], s[8]);
    const float b0 = -dot3<FMA>(e0, e1, e2, s[3], s[4], s[5]);
    const float b1 = -dot3<FMA>(e0, e1, e2, s[6], s[7], s[8]);
    A00 = A00 + lambda;
    A11 = A11 + lambda;
    float u_new, v_new;
    if (FMA) {
      const float det_inv = (float)(1.0 / (double)__builtin_fmaf(A00, A11, -(A01 * A01)));
      u_new = __builtin_fmaf(det_inv, __builtin_fmaf(A11, b0, -(A01 * b1)), u);
      v_new = __builtin_fmaf(det_inv, __builtin_fmaf(-A01, b0, A00 * b1), v);
    } else {
      const float det_inv = (float)(1.0 / (double)(A00 * A11 - A01 * A01));
      const float delta_u = det_inv * (A11 * b0 - A01 * b1);
      const float delta_v = det_inv * (-A01 * b0 + A00 * b1);
      u_new = u + delta_u;
      v_new = v + delta_v;
    }
    u_new = clamp_ref(u_new, 1.0f, umax);
    v_new = clamp_ref(v_new, 1.0f, vmax);
    // re-evaluate cost at the candidate (:200-228); only the ray channels are needed
    float s2[3];
    Bilin bw2 = bilin_weights(u_new, v_new);
    bilin_sample<C, 3, FMA>(img, w, bw2, s2);
    r_norm = sqrtf(dot3<FMA>(s2[0], s2[1], s2[2], s2[0], s2[1], s2[2]));
    r_norm_inv = (float)(1.0 / (double)r_norm);
    const float f0 = FMA ? __builtin_fmaf(s2[0], r_norm_inv, -t0) : s2[0] * r_norm_inv - t0;
    const float f1 = FMA ? __builtin_fmaf(s2[1], r_norm_inv, -t1) : s2[1] * r_norm_inv - t1;
    const float f2 = FMA ? __builtin_fmaf(s2[2], r_norm_inv, -t2) : s2[2] * r_norm_inv - t2;
    const float new_cost = dot3<FMA>(f0, f1, f2, f0, f1, f2);
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
  p_new[2 * q + 0] = u;
  p_new[2 * q + 1] = v;
  converged_out[q] = conv ? 1 : 0;
}

// ---------------------------------------------------------------------------
// refine_matches (matching_kernels.cu:25-81): descriptor argmax over a dilated
// (2r+1)^2 window, dilation d = dmax..1, window re-centred after each level.
// Score = Σ_k D21[k]*D11[k] in c10::Half arithmetic: each product and each partial
// sum rounded to f16 (correctly-rounded v_mul_f16 / v_add_f16 are exactly
// half(float(a)*float(b)) and half(float(s)+float(p)) — see DESIGN.md §Numerics).
// ---------------------------------------------------------------------------
template <int F>
__device__ __forceinline__ _Float16 desc_score(const _Float16* __restrict__ q,
                                               const _Float16* __restrict__ cand, int fdim) {
  _Float16 score = (_Float16)0.0f;
  const int nf = F > 0 ? F : fdim;
#pragma unroll
  for (int k = 0; k < (F > 0 ? F : 1); k++) {
    if (F == 0) break;
    _Float16 prod = q[k] * cand[k];
    score = score + prod;
  }
  if (F == 0) {
    for (int k = 0; k < nf; k++) {
      _Float16 prod = q[k] * cand[k];
      score = score + prod;
    }
  }
  return score;
}

// TILE2D: a workgroup takes a 16x16 tile of query pixels (n == h*w) instead of 256
// consecutive pixels of one row: the candidate windows of a tile's queries overlap far
// more (the union of the 31x31-pixel level-1 windows is 46x46 pixels instead of 31x286),
// so their descriptor rows are re-read from L1/L2 instead of fetched again; consecutive
// workgroups are neighbouring tiles of one direction.  Per-query work and results unchanged.
template <int F, bool TILE2D>
__global__ __launch_bounds__(kBlock) void refine_matches_kernel(
    const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
    const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w, int64_t n,
    int fdim, int radius, int dilation_max) {
  int64_t i;
  if constexpr (TILE2D) {
    const int tiles_w = (w + 15) >> 4;
    const int tx = blockIdx.x % tiles_w, ty = blockIdx.x / tiles_w;
    const int px = tx * 16 + (threadIdx.x & 15), py = ty * 16 + (threadIdx.x >> 4);
    if (px >= w || py >= h) return;
    i = (int64_t)py * w + px;
  } else {
    i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
  }
  const int64_t b = blockIdx.y;
  const int64_t q = b * n + i;
  constexpr int FMAX = F > 0 ? F : 64;
  _Float16 qd[FMAX];
  const int nf = F > 0 ? F : fdim;
  if (F == 24) {
    // 48-B descriptor row: three 16-B loads (rows are 16-B aligned: 48 = 3*16)
    const uint4* src = reinterpret_cast<const uint4*>(D21 + q * 24);
#pragma unroll
    for (int c = 0; c < 3; c++) {
      uint4 v = src[c];
      __builtin_memcpy(&qd[8 * c], &v, 16);
    }
  } else {
    for (int k = 0; k < nf; k++) qd[k] = D21[q * nf + k];
  }
  const _Float16* img = D11 + b * (int64_t)h * w * nf;

  int64_t u0 = p1[2 * q + 0];
  int64_t v0 = p1[2 * q + 1];
  // ::cuda::std::numeric_limits<c10::Half>::min() is the value-initialised Half (+0):
  // libcu++ has no specialisation for c10::Half.
  _Float16 max_score = (_Float16)0.0f;
  int64_t u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; d--) {
    const int rd = radius * d;
    const int diam = 2 * rd + 1;
    for (int ii = 0; ii < diam; ii += d) {
      const int64_t u = u0 - rd + ii;
      for (int jj = 0; jj < diam; jj += d) {
        const int64_t v = v0 - rd + jj;
        if (v >= 0 && v < h && u >= 0 && u < w) {
          const _Float16* cand = img + (v * w + u) * nf;
          _Float16 score;
          if (F == 24) {
            _Float16 cd[24];
            const uint4* src = reinterpret_cast<const uint4*>(cand);
#pragma unroll
            for (int c = 0; c < 3; c++) {
              uint4 vv = src[c];
              __builtin_memcpy(&cd[8 * c], &vv, 16);
            }
            score = desc_score<24>(qd, cd, 24);
          } else {
            score = desc_score<0>(qd, cand, nf);
          }
          if ((float)score > (float)max_score) {
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
  p1_new[2 * q + 0] = u_new;
  p1_new[2 * q + 1] = v_new;
}

// The reference configuration (F = 24, radius R = 3, n == h*w) as a latency-hiding variant
// of the TILE2D kernel above, same visiting order and arithmetic:
//  * the 2R+1 candidates of one window column (fixed u, the inner v loop) are loaded before
//    any of them is scored — 21 16-B loads in flight per lane instead of 3 — out-of-image
//    candidates load pixel 0 and are skipped when scoring, as the reference skips them;
//  * workgroups are dispatched round-robin over the 8 XCDs (linear id % 8): the tile order
//    is remapped so each XCD takes a contiguous band of tiles and its L2 holds one band's
//    windows instead of windows from all over the image;
//  * 32-bit in-image offsets (h*w < 2^31 is checked by the host).
template <int R>
__global__ __launch_bounds__(kBlock) void refine_matches_r_kernel(
    const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
    const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w,
    int dilation_max) {
  constexpr int S = 2 * R + 1;
  const int n = h * w;
  const int tiles_w = (w + 15) >> 4;
  const int tiles = tiles_w * ((h + 15) >> 4);
  const int lin = blockIdx.x, xcd = lin & 7, loc = lin >> 3;
  const int tq = tiles >> 3, tr = tiles & 7;
  const int t = xcd < tr ? xcd * (tq + 1) + loc : tr * (tq + 1) + (xcd - tr) * tq + loc;
  const int px = (t % tiles_w) * 16 + (threadIdx.x & 15);
  const int py = (t / tiles_w) * 16 + (threadIdx.x >> 4);
  if (px >= w || py >= h) return;
  const int64_t q = (int64_t)blockIdx.y * n + (int64_t)py * w + px;
  _Float16 qd[24];
  {
    const uint4* src = reinterpret_cast<const uint4*>(D21 + q * 24);
#pragma unroll
    for (int c = 0; c < 3; c++) {
      uint4 v = src[c];
      __builtin_memcpy(&qd[8 * c], &v, 16);
    }
  }
  const uint4* img = reinterpret_cast<const uint4*>(D11 + (int64_t)blockIdx.y * n * 24);
  int64_t u0 = p1[2 * q + 0];
  int64_t v0 = p1[2 * q + 1];
  _Float16 max_score = (_Float16)0.0f;
  int64_t u_new = u0, v_new = v0;
  for (int d = dilation_max; d > 0; d--) {
    const int rd = R * d;
    for (int ii = 0; ii < S; ii++) {
      const int64_t u = u0 - rd + ii * d;
      const bool uok = u >= 0 && u < w;
      uint4 buf[S][3];
      bool ok[S];
#pragma unroll
      for (int jj = 0; jj < S; jj++) {
        const int64_t v = v0 - rd + jj * d;
        ok[jj] = uok && v >= 0 && v < h;
        const int off = ok[jj] ? (int)v * w + (int)u : 0;
#pragma unroll
        for (int c = 0; c < 3; c++)
          buf[jj][c] = img[off * 3 + c];
      }
#pragma unroll
      for (int jj = 0; jj < S; jj++) {
        _Float16 cd[24];
        __builtin_memcpy(cd, buf[jj], 48);
        const _Float16 score = desc_score<24>(qd, cd, 24);
        if (ok[jj] && (float)score > (float)max_score) {
          max_score = score;
          u_new = u;
          v_new = v0 - rd + jj * d;
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
  }
  p1_new[2 * q + 0] = u_new;
  p1_new[2 * q + 1] = v_new;
}

// The same search with the window's columns split over lanes (round 5): lane ii of a group
// of 2R+1 lanes scores window column ii (its 2R+1 candidates, 3(2R+1) 16-B loads in flight)
// for one query, and the group merges the columns in the reference's visiting order.  The
// one-lane kernel above runs 3 waves per SIMD over 49 dependent candidate columns per
// query and stalls on the texture path; here a wave covers 9 queries (63 lanes, the last
// lane idle), 7x the waves for the same work.  Arithmetic per candidate is unchanged (each
// lane runs the full 24-term f16 chain); the merge is exact:
//   the sequential scan with strict > ends each dilation on the FIRST candidate holding the
//   window maximum, if that maximum beats the running max_score.  Lane ii scans its column
//   from the dilation's starting max_score, so it holds the column's first maximum (or
//   nothing); folding the columns in order ii = 0..2R with strict > then picks the same
//   candidate.  A column whose maximum does not beat the running value changes nothing in
//   either form.
// Every lane of a group computes the merge (7 shuffles of score and row), so the group
// agrees on (u0, v0) for the next dilation without a broadcast.
template <int R, bool BUF, bool TILE = false, int RB = kBlock / 64>
__global__ __launch_bounds__(64 * RB) void refine_matches_c_kernel(
    const _Float16* __restrict__ D11, const _Float16* __restrict__ D21,
    const int64_t* __restrict__ p1, int64_t* __restrict__ p1_new, int h, int w,
    int dilation_max) {
  constexpr int S = 2 * R + 1;
  constexpr int QW = 64 / S;                 // queries per wave
  constexpr int QB = QW * RB;                // queries per workgroup (RB waves)
  const int n = h * w;
  // TILE: a workgroup takes a QW x 4 pixel tile (one image row per wave) instead of QB
  // consecutive pixels, so its windows overlap in both directions
  const int tiles_x = (w + QW - 1) / QW;
  const int nblk = TILE ? tiles_x * ((h + RB - 1) / RB) : (n + QB - 1) / QB;
  const int lin = blockIdx.x, xcd = lin & 7, loc = lin >> 3;
  const int tq = nblk >> 3, tr = nblk & 7;
  const int t = xcd < tr ? xcd * (tq + 1) + loc : tr * (tq + 1) + (xcd - tr) * tq + loc;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane / S, ii = lane - grp * S, base = grp * S;
  // every lane takes part in the shuffles: the idle lane and queries past the end run a
  // clamped query and store nothing
  int qi;
  bool qok;
  if constexpr (TILE) {
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int px = tx * QW + grp, py = ty * RB + wv;
    qok = grp < QW && px < w && py < h;
    qi = qok ? py * w + px : 0;
  } else {
    qi = t * QB + wv * QW + grp;
    qok = grp < QW && qi < n;
  }
  const int64_t q = (int64_t)blockIdx.y * n + min(qi, n - 1);
  _Float16 qd[24];
  {
    const uint4* src = reinterpret_cast<const uint4*>(D21 + q * 24);
#pragma unroll
    for (int c = 0; c < 3; c++) {
      uint4 v = src[c];
      __builtin_memcpy(&qd[8 * c], &v, 16);
    }
  }
  const uint4* img = reinterpret_cast<const uint4*>(D11 + (int64_t)blockIdx.y * n * 24);
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(img), (short)0, 0x7ffffff0, 0x00020000);
  // the reference's coordinates are int64; h*w < 2^31 (host check) keeps in-image ones in
  // int; a start point beyond +-2^30 has no in-image candidate at any dilation, so it
  // never moves and the int arithmetic below stays clear of overflow
  const int64_t u0_64 = p1[2 * q + 0], v0_64 = p1[2 * q + 1];
  const bool far = u0_64 < -(1LL << 30) || u0_64 > (1LL << 30) || v0_64 < -(1LL << 30) ||
                   v0_64 > (1LL << 30);
  int u0 = far ? 0 : (int)u0_64;
  int v0 = far ? 0 : (int)v0_64;
  _Float16 max_score = (_Float16)0.0f;
  bool moved = false;
  for (int d = dilation_max; d > 0; d--) {
    const int rd = R * d;
    const int u = u0 - rd + ii * d;
    const bool uok = !far && u >= 0 && u < w;
    uint4 buf[S][3];
    bool ok[S];
#pragma unroll
    for (int jj = 0; jj < S; jj++) {
      const int v = v0 - rd + jj * d;
      ok[jj] = uok && v >= 0 && v < h;
      const int off = ok[jj] ? v * w + u : 0;
#pragma unroll
      for (int c = 0; c < 3; c++) {
        if constexpr (BUF) {
          buf[jj][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rD, (unsigned)(off * 3 + c) * 16u, 0, 0));
        } else {
          buf[jj][c] = img[off * 3 + c];
        }
      }
    }
    _Float16 best = max_score;
    int bj = -1;
#pragma unroll
    for (int jj = 0; jj < S; jj++) {
      _Float16 cd[24];
      __builtin_memcpy(cd, buf[jj], 48);
      const _Float16 score = desc_score<24>(qd, cd, 24);
      if (ok[jj] && (float)score > (float)best) {
        best = score;
        bj = jj;
      }
    }
    // merge the group's columns in visiting order
    const int mine = (int)__builtin_bit_cast(unsigned short, best) | ((bj + 1) << 16);
    int pick_i = -1, pick_j = -1;
#pragma unroll
    for (int k = 0; k < S; k++) {
      const int o = __shfl(mine, base + k);
      const int oj = (o >> 16) - 1;
      const _Float16 os = __builtin_bit_cast(_Float16, (unsigned short)(o & 0xFFFF));
      if (oj >= 0 && (float)os > (float)max_score) {
        max_score = os;
        pick_i = k;
        pick_j = oj;
      }
    }
    if (pick_i >= 0) {
      u0 = u0 - rd + pick_i * d;
      v0 = v0 - rd + pick_j * d;
      moved = true;
    }
  }
  if (qok && ii == 0) {
    p1_new[2 * q + 0] = moved ? (int64_t)u0 : u0_64;
    p1_new[2 * q + 1] = moved ? (int64_t)v0 : v0_64;
  }
}

// ---------------------------------------------------------------------------
// prep_for_iter_proj (matching.py:25-49) + img_gradient (image.py:5-38), fused.
// ---------------------------------------------------------------------------
// Accumulation orders pinned to the reference's torch run (tests/golden): the vector norm
// is the sequential FMA chain x0*x0 → fma(x1,x1,·) → fma(x2,x2,·); the depthwise 3x3
// conv is a sequential FMA over the 9 taps, row-major.
__device__ __forceinline__ void normalize3(const float* x, float* o) {
  // F.normalize(x, dim=-1): x / max(||x||_2, 1e-12)
  float nrm = sqrtf(__builtin_fmaf(x[2], x[2], __builtin_fmaf(x[1], x[1], x[0] * x[0])));
  nrm = fmaxf(nrm, 1e-12f);
  o[0] = x[0] / nrm;
  o[1] = x[1] / nrm;
  o[2] = x[2] / nrm;
}

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // F.pad(mode="reflect") with pad 1: -1 -> 1, n -> n-2
  return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

__global__ __launch_bounds__(kBlock) void match_prep_kernel(
    const float* __restrict__ X11, const float* __restrict__ X21,
    const int64_t* __restrict__ idx_init, float* __restrict__ rays_with_grad,
    float* __restrict__ pts_norm, float* __restrict__ p_init, int h, int w) {
  const int64_t npix = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= npix) return;
  const int y = (int)(i / w), x = (int)(i % w);
  const float* img = X11 + b * npix * 3;
  // 3x3 neighbourhood of normalised rays (reflect padding)
  float nb[3][3][3];
#pragma unroll
  for (int dy = 0; dy < 3; dy++) {
    const int yy = reflect_idx(y + dy - 1, h);
#pragma unroll
    for (int dx = 0; dx < 3; dx++) {
      const int xx = reflect_idx(x + dx - 1, w);
      normalize3(img + ((int64_t)yy * w + xx) * 3, nb[dy][dx]);
    }
  }
  float* out = rays_with_grad + (b * npix + i) * 9;
  // Scharr/32: gx = [[-3,0,3],[-10,0,10],[-3,0,3]]/32, gy = its transpose; taps in
  // row-major order (cross-correlation, as F.conv2d), zero taps included.
  const float W[3][3] = {{-3.0f / 32.0f, 0.0f, 3.0f / 32.0f},
                         {-10.0f / 32.0f, 0.0f, 10.0f / 32.0f},
                         {-3.0f / 32.0f, 0.0f, 3.0f / 32.0f}};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    out[c] = nb[1][1][c];
    float gx = 0.0f, gy = 0.0f;
#pragma unroll
    for (int ky = 0; ky < 3; ky++)
#pragma unroll
      for (int kx = 0; kx < 3; kx++) {
        gx = __builtin_fmaf(W[ky][kx], nb[ky][kx][c], gx);
        gy = __builtin_fmaf(W[kx][ky], nb[ky][kx][c], gy);
      }
    out[3 + c] = gx;
    out[6 + c] = gy;
  }
  float pn[3];
  normalize3(X21 + (b * npix + i) * 3, pn);
  float* po = pts_norm + (b * npix + i) * 3;
  po[0] = pn[0];
  po[1] = pn[1];
  po[2] = pn[2];
  int64_t idx = idx_init ? idx_init[b * npix + i] : i;
  p_init[(b * npix + i) * 2 + 0] = (float)(idx % w);
  p_init[(b * npix + i) * 2 + 1] = (float)(idx / w);
}

// matching.py:67-76: p1 = p.long(); d = ||X11[b,v,u] - X21[b,n]||; valid &= d < thresh
__global__ __launch_bounds__(kBlock) void match_occlusion_kernel(
    const float* __restrict__ X11, const float* __restrict__ X21, const float* __restrict__ p,
    const uint8_t* __restrict__ conv, int64_t* __restrict__ p1, uint8_t* __restrict__ valid,
    int h, int w, float dist_thresh) {
  const int64_t npix = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (i >= npix) return;
  const int64_t q = b * npix + i;
  const int64_t u = (int64_t)p[2 * q + 0];  // trunc toward zero, like Tensor.long()
  const int64_t v = (int64_t)p[2 * q + 1];
  p1[2 * q + 0] = u;
  p1[2 * q + 1] = v;
  const float* a = X11 + (b * npix + v * w + u) * 3;
  const float* c = X21 + q * 3;
  const float d0 = a[0] - c[0], d1 = a[1] - c[1], d2 = a[2] - c[2];
  const float dist = sqrtf(__builtin_fmaf(d2, d2, __builtin_fmaf(d1, d1, d0 * d0)));
  valid[q] = (conv[q] != 0 && dist < dist_thresh) ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void pixel_to_lin_kernel(const int64_t* __restrict__ p1,
                                                             int64_t* __restrict__ idx,
                                                             int64_t total, int64_t w) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= total) return;
  idx[i] = p1[2 * i + 0] + w * p1[2 * i + 1];
}

}  // namespace

namespace {
int iter_proj_launch(bool fma, const float* d_rays, const float* d_pts, const float* d_p_init,
                     float* d_p_new, uint8_t* d_conv, int64_t b, int64_t h, int64_t w, int64_t n,
                     int max_iter, float lambda_init, float cost_thresh, void* stream) {
  if (b < 0 || n < 0 || h < 3 || w < 3) return M3S_ERR_INVALID_ARG;
  if (b == 0 || n == 0) return M3S_OK;
  if (!d_rays || !d_pts || !d_p_init || !d_p_new || !d_conv) return M3S_ERR_INVALID_ARG;
  if (b > 65535) return M3S_ERR_TOO_LARGE;
  dim3 grid(m3s_div_up(n, kBlock), (unsigned)b);
  if (fma)
    hipLaunchKernelGGL((iter_proj_kernel<9, true>), grid, dim3(kBlock), 0, m3s_stream(stream),
                       d_rays, d_pts, d_p_init, d_p_new, d_conv, (int)h, (int)w, n, max_iter,
                       lambda_init, cost_thresh);
  else
    hipLaunchKernelGGL((iter_proj_kernel<9, false>), grid, dim3(kBlock), 0, m3s_stream(stream),
                       d_rays, d_pts, d_p_init, d_p_new, d_conv, (int)h, (int)w, n, max_iter,
                       lambda_init, cost_thresh);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
}  // namespace

extern "C" int m3s_iter_proj(const float* d_rays, const float* d_pts, const float* d_p_init,
                             float* d_p_new, uint8_t* d_conv, int64_t b, int64_t h, int64_t w,
                             int64_t n, int max_iter, float lambda_init, float cost_thresh,
                             void* stream) {
  return iter_proj_launch(false, d_rays, d_pts, d_p_init, d_p_new, d_conv, b, h, w, n, max_iter,
                          lambda_init, cost_thresh, stream);
}

extern "C" int m3s_iter_proj_fma(const float* d_rays, const float* d_pts, const float* d_p_init,
                                 float* d_p_new, uint8_t* d_conv, int64_t b, int64_t h, int64_t w,
                                 int64_t n, int max_iter, float lambda_init, float cost_thresh,
                                 void* stream) {
  return iter_proj_launch(true, d_rays, d_pts, d_p_init, d_p_new, d_conv, b, h, w, n, max_iter,
                          lambda_init, cost_thresh, stream);
}

extern "C" int m3s_refine_matches(const uint16_t* d_D11, const uint16_t* d_D21,
                                  const int64_t* d_p1, int64_t* d_p1_new, int64_t b, int64_t h,
                                  int64_t w, int64_t n, int64_t fdim, int radius,
                                  int dilation_max, void* stream) {
  if (b < 0 || n < 0 || h < 1 || w < 1 || fdim < 1) return M3S_ERR_INVALID_ARG;
  if (b == 0 || n == 0) return M3S_OK;
  if (!d_D11 || !d_D21 || !d_p1 || !d_p1_new) return M3S_ERR_INVALID_ARG;
  if (fdim > 64 || b > 65535) return M3S_ERR_TOO_LARGE;
  const _Float16* D11 = reinterpret_cast<const _Float16*>(d_D11);
  const _Float16* D21 = reinterpret_cast<const _Float16*>(d_D21);
  const bool aligned = ((uintptr_t)d_D11 % 16 == 0) && ((uintptr_t)d_D21 % 16 == 0);
  // A/B knob: M3S_REFINE_KERNEL = "rows" (1-D row blocks) | "tile" (plain 16x16 tiles)
  static const char* kind = getenv("M3S_REFINE_KERNEL");
  static const bool rows = kind && !strcmp(kind, "rows");
  static const bool tile = kind && !strcmp(kind, "tile");
  static const bool lane1 = kind && !strcmp(kind, "lane");  // the one-lane radius-3 kernel
  // the column-split kernel's buffer offsets (off * 3 + c) * 16 stay below the descriptor's
  // 0x7ffffff0-byte range: one image of D11 under 2 GB (h * w < 44.7 M)
  if (fdim == 24 && aligned && n == h * w && radius == 3 && h * w * 48 < 0x7ffffff0LL &&
      !rows && !tile && !lane1) {
    // 9-pixel-wide tiles per workgroup (one image row per wave), 8 rows by default: the
    // windows of a workgroup overlap in both directions (profiles/r05_refine_tile2_ab.txt);
    // "rowmajor" = 36 consecutive pixels per workgroup
    static const bool tile2 = !(kind && !strcmp(kind, "rowmajor"));
    dim3 gridq((unsigned)(tile2 ? m3s_div_up(w, 64 / 7) * m3s_div_up(h, kBlock / 64)
                                : m3s_div_up(h * w, (64 / 7) * (kBlock / 64))),
               (unsigned)b);
    if (tile2) {
      // rows per workgroup (M3S_REFINE_RB A/B: 4 | 8 | 16): 9 x 8 tiles of 512 threads
      // measured fastest (random 165 → 159.6 us, coherent 130.6 → 128.6;
      // profiles/r05_refine_tile2_ab.txt)
      static const int rbk = getenv("M3S_REFINE_RB") ? atoi(getenv("M3S_REFINE_RB")) : 8;
      if (rbk == 8 || rbk == 16) {
        dim3 g2((unsigned)(m3s_div_up(w, 64 / 7) * m3s_div_up(h, rbk)), (unsigned)b);
        if (rbk == 8)
          hipLaunchKernelGGL((refine_matches_c_kernel<3, true, true, 8>), g2, dim3(512), 0,
                             m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w,
                             dilation_max);
        else
          hipLaunchKernelGGL((refine_matches_c_kernel<3, true, true, 16>), g2, dim3(1024), 0,
                             m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w,
                             dilation_max);
        M3S_LAUNCH_CHECK();
        return M3S_OK;
      }
      hipLaunchKernelGGL((refine_matches_c_kernel<3, true, true>), gridq, dim3(kBlock), 0,
                         m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w,
                         dilation_max);
      M3S_LAUNCH_CHECK();
      return M3S_OK;
    }
    // buffer loads (32-bit offsets from one descriptor) by default: 168-172 vs 182-184 us on
    // a random match field, equal on a coherent one (profiles/r05_refine_buf_ab.txt);
    // "flat" = 64-bit per-lane addresses
    static const bool flat = kind && !strcmp(kind, "flat");
    hipLaunchKernelGGL(flat ? (refine_matches_c_kernel<3, false>) : (refine_matches_c_kernel<3, true>),
                       gridq, dim3(kBlock), 0, m3s_stream(stream),
                       D11, D21, d_p1, d_p1_new, (int)h, (int)w, dilation_max);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
  }
  if (fdim == 24 && aligned && n == h * w && radius == 3 && h * w < (1LL << 31) && !rows &&
      !tile) {
    dim3 grid2((unsigned)(m3s_div_up(w, 16) * m3s_div_up(h, 16)), (unsigned)b);
    hipLaunchKernelGGL(refine_matches_r_kernel<3>, grid2, dim3(kBlock), 0, m3s_stream(stream),
                       D11, D21, d_p1, d_p1_new, (int)h, (int)w, dilation_max);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
  }
  if (fdim == 24 && aligned && n == h * w && !rows) {
    dim3 grid2((unsigned)(m3s_div_up(w, 16) * m3s_div_up(h, 16)), (unsigned)b);
    hipLaunchKernelGGL((refine_matches_kernel<24, true>), grid2, dim3(kBlock), 0,
                       m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w, n, 24,
                       radius, dilation_max);
    M3S_LAUNCH_CHECK();
    return M3S_OK;
  }
  dim3 grid(m3s_div_up(n, kBlock), (unsigned)b);
  if (fdim == 24 && aligned) {
    hipLaunchKernelGGL((refine_matches_kernel<24, false>), grid, dim3(kBlock), 0,
                       m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w, n, 24,
                       radius, dilation_max);
  } else {
    hipLaunchKernelGGL((refine_matches_kernel<0, false>), grid, dim3(kBlock), 0,
                       m3s_stream(stream), D11, D21, d_p1, d_p1_new, (int)h, (int)w, n,
                       (int)fdim, radius, dilation_max);
  }
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_match_prep(const float* d_X11, const float* d_X21, const int64_t* d_idx_init,
                              float* d_rays_with_grad, float* d_pts_norm, float* d_p_init,
                              int64_t b, int64_t h, int64_t w, void* stream) {
  if (b < 0 || h < 2 || w < 2) return M3S_ERR_INVALID_ARG;
  if (b == 0) return M3S_OK;
  if (!d_X11 || !d_X21 || !d_rays_with_grad || !d_pts_norm || !d_p_init)
    return M3S_ERR_INVALID_ARG;
  dim3 grid(m3s_div_up(h * w, kBlock), (unsigned)b);
  hipLaunchKernelGGL(match_prep_kernel, grid, dim3(kBlock), 0, m3s_stream(stream), d_X11, d_X21,
                     d_idx_init, d_rays_with_grad, d_pts_norm, d_p_init, (int)h, (int)w);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_match_occlusion(const float* d_X11, const float* d_X21, const float* d_p,
                                   const uint8_t* d_conv, int64_t* d_p1, uint8_t* d_valid,
                                   int64_t b, int64_t h, int64_t w, float dist_thresh,
                                   void* stream) {
  if (b < 0 || h < 1 || w < 1) return M3S_ERR_INVALID_ARG;
  if (b == 0) return M3S_OK;
  if (!d_X11 || !d_X21 || !d_p || !d_conv || !d_p1 || !d_valid) return M3S_ERR_INVALID_ARG;
  dim3 grid(m3s_div_up(h * w, kBlock), (unsigned)b);
  hipLaunchKernelGGL(match_occlusion_kernel, grid, dim3(kBlock), 0, m3s_stream(stream), d_X11,
                     d_X21, d_p, d_conv, d_p1, d_valid, (int)h, (int)w, dist_thresh);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_pixel_to_lin(const int64_t* d_p1, int64_t* d_idx, int64_t b, int64_t n,
                                int64_t w, void* stream) {
  if (b < 0 || n < 0) return M3S_ERR_INVALID_ARG;
  if (b * n == 0) return M3S_OK;
  if (!d_p1 || !d_idx) return M3S_ERR_INVALID_ARG;
  hipLaunchKernelGGL(pixel_to_lin_kernel, dim3(m3s_div_up(b * n, kBlock)), dim3(kBlock), 0,
                     m3s_stream(stream), d_p1, d_idx, b * n, w);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
