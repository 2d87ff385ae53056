// Memory-bound ViT / DPT kernels (gfx950): LayerNorm, patch im2col, bilinear x2
// upsample (align_corners=True), the fused DPT output tail (1x1 conv 128→4 +
// reg_dense_depth/conf) and the MASt3R local-feature tail (pixel_shuffle(16) + desc
// normalisation + desc_conf).  All vectorised 16-B loads where the layout allows.
#include "vit_common.h"

namespace {

// ---- LayerNorm: one wave per row -----------------------------------------------------
// DUAL: the decoder's norm1(x) and norm_y of the other side read the same rows, so one
// pass writes y[b] = LN(x[b ^ xxor]; params b) and y2[b ^ 1] = LN(x[b]; params2 of b ^ 1)
// from one set of row statistics (y2 only with xxor == 0).
// YT: output type 0 bf16, 1 f32, 2 OCP e4m3 (the A operand of the fp8 GEMMs, unscaled).
// MAXV: float4 vectors per lane (dim <= 256 * MAXV).  gamma / beta are requested with the
// row, before the two reductions, so the launch pays one memory round trip, not two.
template <bool XBF, int YT, bool DUAL = false, int MAXV = 16>
__global__ __launch_bounds__(256) void layernorm_kernel(const void* __restrict__ x,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        void* __restrict__ y, int64_t rows,
                                                        int dim, float eps, int64_t sx,
                                                        int64_t sy, int64_t sp, int64_t pmod,
                                                        int xxor, const float* __restrict__ gamma2 = nullptr,
                                                        const float* __restrict__ beta2 = nullptr,
                                                        void* __restrict__ y2 = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t b = blockIdx.y;
  if (row >= rows) return;
  const int64_t pb = pmod > 0 ? b % pmod : b;
  const float* g = gamma + pb * sp;
  const float* be = beta + pb * sp;
  const int64_t b2 = b ^ 1;
  const int64_t pb2 = pmod > 0 ? b2 % pmod : b2;
  float v[MAXV][4];
  float4 gv[MAXV], bv[MAXV], gv2[DUAL ? MAXV : 1], bv2[DUAL ? MAXV : 1];
  const int nvec = dim / 4;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    const int c4 = lane + i * 64;
    if (c4 < nvec) {
      if (XBF) {
        const bf16_t* xr = reinterpret_cast<const bf16_t*>(x) + (b ^ xxor) * sx + row * dim;
        const uint2 raw = *reinterpret_cast<const uint2*>(xr + 4 * c4);
        const bf16_t* e = reinterpret_cast<const bf16_t*>(&raw);
#pragma unroll
        for (int k = 0; k < 4; k++) v[i][k] = bf2f(e[k]);
      } else {
        const float* xr = reinterpret_cast<const float*>(x) + (b ^ xxor) * sx + row * dim;
        const float4 f = *reinterpret_cast<const float4*>(xr + 4 * c4);
        v[i][0] = f.x;
        v[i][1] = f.y;
        v[i][2] = f.z;
        v[i][3] = f.w;
      }
      gv[i] = reinterpret_cast<const float4*>(g)[c4];
      bv[i] = reinterpret_cast<const float4*>(be)[c4];
      if constexpr (DUAL) {
        gv2[i] = reinterpret_cast<const float4*>(gamma2 + pb2 * sp)[c4];
        bv2[i] = reinterpret_cast<const float4*>(beta2 + pb2 * sp)[c4];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXV; i++)
    if (lane + i * 64 < nvec)
#pragma unroll
      for (int k = 0; k < 4; k++) s += v[i][k];
  s = m3s_wave_sum(s);
  const float mean = s / (float)dim;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    const int c4 = lane + i * 64;
    if (c4 < nvec) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const float d = v[i][k] - mean;
        ss += d * d;
      }
    }
  }
  ss = m3s_wave_sum(ss);
  const float rstd = 1.0f / sqrtf(ss / (float)dim + eps);
#pragma unroll
  for (int i = 0; i < MAXV; i++) {
    const int c4 = lane + i * 64;
    if (c4 < nvec) {
      const float gk[4] = {gv[i].x, gv[i].y, gv[i].z, gv[i].w};
      const float bk[4] = {bv[i].x, bv[i].y, bv[i].z, bv[i].w};
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; k++) o[k] = (v[i][k] - mean) * rstd * gk[k] + bk[k];
      if constexpr (YT == 1) {
        float* yr = reinterpret_cast<float*>(y) + b * sy + row * dim;
        *reinterpret_cast<float4*>(yr + 4 * c4) = make_float4(o[0], o[1], o[2], o[3]);
      } else if constexpr (YT == 2) {
        uint8_t* yr = reinterpret_cast<uint8_t*>(y) + b * sy + row * dim;
        *reinterpret_cast<uint32_t*>(yr + 4 * c4) = pack4_fp8(o[0], o[1], o[2], o[3]);
      } else {
        bf16_t* yr = reinterpret_cast<bf16_t*>(y) + b * sy + row * dim;
        bf16x4 ob;
#pragma unroll
        for (int k = 0; k < 4; k++) ob[k] = f2bf(o[k]);
        *reinterpret_cast<bf16x4*>(yr + 4 * c4) = ob;
      }
      if constexpr (DUAL) {
        const float gk2[4] = {gv2[i].x, gv2[i].y, gv2[i].z, gv2[i].w};
        const float bk2[4] = {bv2[i].x, bv2[i].y, bv2[i].z, bv2[i].w};
        float o2[4];
#pragma unroll
        for (int k = 0; k < 4; k++) o2[k] = (v[i][k] - mean) * rstd * gk2[k] + bk2[k];
        if constexpr (YT == 2) {
          *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(y2) + b2 * sy + row * dim +
                                       4 * c4) = pack4_fp8(o2[0], o2[1], o2[2], o2[3]);
        } else {
          bf16x4 ob;
#pragma unroll
          for (int k = 0; k < 4; k++) ob[k] = f2bf(o2[k]);
          *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16_t*>(y2) + b2 * sy + row * dim +
                                     4 * c4) = ob;
        }
      }
    }
  }
}

// ---- patch im2col: (c, ky, kx) K order, 8 values per thread ---------------------------
__global__ __launch_bounds__(256) void patchify_kernel(const float* __restrict__ img,
                                                       bf16_t* __restrict__ out, int h, int w,
                                                       int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int gw = w / 16, gh = h / 16;
  const int chunk = (int)(idx % 96);  // 768 / 8 chunks per patch
  int64_t t = idx / 96;
  const int pj = (int)(t % gw);
  t /= gw;
  const int pi = (int)(t % gh);
  const int64_t b = t / gh;
  const int k0 = chunk * 8;
  const int c = k0 / 256, ky = (k0 / 16) % 16, kx0 = k0 % 16;
  const float* src = img + ((b * 3 + c) * h + (pi * 16 + ky)) * (int64_t)w + pj * 16 + kx0;
  const float4 a = *reinterpret_cast<const float4*>(src);
  const float4 d = *reinterpret_cast<const float4*>(src + 4);
  bf16x8 o;
  o[0] = f2bf(a.x);
  o[1] = f2bf(a.y);
  o[2] = f2bf(a.z);
  o[3] = f2bf(a.w);
  o[4] = f2bf(d.x);
  o[5] = f2bf(d.y);
  o[6] = f2bf(d.z);
  o[7] = f2bf(d.w);
  *reinterpret_cast<bf16x8*>(out + idx * 8) = o;
}

// ---- bilinear x2, align_corners=True (torch upsample_bilinear2d formula) -------------
// IT: index type — 32-bit whenever the element count allows (the 64-bit div/mod of the
// index decomposition otherwise costs more than the memory traffic).
// F8OUT: the output is OCP e4m3 of v * inv_scale (the A operand of an fp8 implicit conv,
// C5; the conv's column scales carry the activation scale back).
template <typename IT, bool F8OUT = false>
__global__ __launch_bounds__(256) void upsample2x_kernel(const bf16_t* __restrict__ in,
                                                         void* __restrict__ out_,
                                                         const bf16_t* __restrict__ addend,
                                                         int h, int w, int c, int oh, int ow,
                                                         IT total, float inv_scale = 1.f) {
  const IT idx = (IT)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const IT c8 = (IT)(c / 8);
  const int cc = (int)(idx % c8) * 8;
  IT t = idx / c8;
  const int H2 = 2 * h, W2 = 2 * w;  // interpolation grid; the output keeps [0,oh)x[0,ow)
  const int ox = (int)(t % (IT)ow);
  t /= (IT)ow;
  const int oy = (int)(t % (IT)oh);
  const int64_t b = (int64_t)(t / (IT)oh);
  const float sh = H2 > 1 ? (float)(h - 1) / (float)(H2 - 1) : 0.f;
  const float sw = W2 > 1 ? (float)(w - 1) / (float)(W2 - 1) : 0.f;
  const float fy = sh * (float)oy, fx = sw * (float)ox;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 < h - 1 ? y0 + 1 : y0, x1 = x0 < w - 1 ? x0 + 1 : x0;
  const float ly = fy - (float)y0, lx = fx - (float)x0;
  const float hy = 1.f - ly, hx = 1.f - lx;
  const bf16_t* base = in + b * (int64_t)h * w * c;
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(base + ((int64_t)y0 * w + x0) * c + cc);
  const bf16x8 bb = *reinterpret_cast<const bf16x8*>(base + ((int64_t)y0 * w + x1) * c + cc);
  const bf16x8 cq = *reinterpret_cast<const bf16x8*>(base + ((int64_t)y1 * w + x0) * c + cc);
  const bf16x8 dq = *reinterpret_cast<const bf16x8*>(base + ((int64_t)y1 * w + x1) * c + cc);
  const int64_t oidx = (((b * oh + oy) * (int64_t)ow) + ox) * c + cc;
  bf16x8 ad = {};
  if (addend) ad = *reinterpret_cast<const bf16x8*>(addend + oidx);
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    v[k] = hy * (hx * bf2f(a[k]) + lx * bf2f(bb[k])) + ly * (hx * bf2f(cq[k]) + lx * bf2f(dq[k]));
    if (addend) v[k] += bf2f(ad[k]);
  }
  if constexpr (F8OUT) {
    uint2 o;
    o.x = pack4_fp8(v[0] * inv_scale, v[1] * inv_scale, v[2] * inv_scale, v[3] * inv_scale);
    o.y = pack4_fp8(v[4] * inv_scale, v[5] * inv_scale, v[6] * inv_scale, v[7] * inv_scale);
    *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(out_) + oidx) = o;
  } else {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = f2bf(v[k]);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16_t*>(out_) + oidx) = o;
  }
}

// ---- DPT output tail: 1x1 conv 128→4 + postprocess ------------------------------------
__global__ __launch_bounds__(256) void dpt_out_kernel(const bf16_t* __restrict__ t,
                                                      const float* __restrict__ w4,
                                                      const float* __restrict__ b4,
                                                      float* __restrict__ pts3d,
                                                      float* __restrict__ conf, int64_t pixels,
                                                      float conf_min, int64_t st, int64_t so,
                                                      int64_t pmod) {
  __shared__ float sw[4 * 128];
  const int64_t b = blockIdx.y;
  const int64_t pb = pmod > 0 ? b % pmod : b;
  w4 += pb * 512;  // per-head weights: w4 [B][4][128], b4 [B][4]
  b4 += pb * 4;
  for (int i = threadIdx.x; i < 512; i += 256) sw[i] = w4[i];
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= pixels) return;
  const bf16_t* row = t + b * st + p * 128;
  float acc[4] = {b4[0], b4[1], b4[2], b4[3]};
#pragma unroll 4
  for (int c8 = 0; c8 < 16; c8++) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(row + c8 * 8);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const float x = bf2f(v[k]);
#pragma unroll
      for (int o = 0; o < 4; o++) acc[o] += sw[o * 128 + c8 * 8 + k] * x;
    }
  }
  // reg_dense_depth('exp'): xyz / clip(|xyz|, 1e-8) * expm1(|xyz|)
  const float d = sqrtf(acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2]);
  const float sc = expm1f(d) / fmaxf(d, 1e-8f);
  float* P = pts3d + b * so * 3 + p * 3;
  P[0] = acc[0] * sc;
  P[1] = acc[1] * sc;
  P[2] = acc[2] * sc;
  conf[b * so + p] = conf_min + expf(acc[3]);
}

// ---- MASt3R local features: pixel_shuffle(16) + normalise + exp conf ---------------------
__global__ __launch_bounds__(256) void local_feat_kernel(const float* __restrict__ feats,
                                                         float* __restrict__ desc,
                                                         _Float16* __restrict__ desc16,
                                                         float* __restrict__ dconf, int h, int w,
                                                         int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int x = (int)(idx % w);
  int64_t t = idx / w;
  const int y = (int)(t % h);
  const int64_t b = t / h;
  const int gw = w / 16;
  const int64_t tok = (int64_t)(y / 16) * gw + (x / 16);
  const int sub = (y % 16) * 16 + (x % 16);
  const float* f = feats + (b * ((int64_t)(h / 16) * gw) + tok) * 6400 + sub;
  float v[24];
  float n2 = 0.f;
#pragma unroll
  for (int c = 0; c < 24; c++) {
    v[c] = f[c * 256];
    n2 += v[c] * v[c];
  }
  const float inv = 1.0f / sqrtf(n2);
  const int64_t pix = idx;
#pragma unroll
  for (int c = 0; c < 24; c++) v[c] *= inv;
  // 16-B vector stores (96 B f32 / 48 B f16 per pixel, pixels of a row are contiguous)
  if (desc) {
    float4* d4 = reinterpret_cast<float4*>(desc + pix * 24);
#pragma unroll
    for (int q = 0; q < 6; q++) d4[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  }
  if (desc16) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    h8* h = reinterpret_cast<h8*>(desc16 + pix * 24);
#pragma unroll
    for (int q = 0; q < 3; q++) {
      h8 o;
#pragma unroll
      for (int t = 0; t < 8; t++) o[t] = (_Float16)v[8 * q + t];
      h[q] = o;
    }
  }
  dconf[pix] = expf(f[24 * 256]);
}

}  // namespace

extern "C" int m3s_vit_layernorm(const void* d_x, int x_is_bf16, const float* d_gamma,
                                 const float* d_beta, void* d_y, int y_type, int64_t rows,
                                 int64_t dim, float eps, int64_t batch, int64_t stride_x,
                                 int64_t stride_y, int64_t stride_param, int64_t param_mod,
                                 int x_batch_xor, void* stream) {
  if (!d_x || !d_gamma || !d_beta || !d_y || rows <= 0 || batch <= 0) return M3S_ERR_INVALID_ARG;
  if (dim % 4 || dim > 4096 || dim <= 0 || y_type < 0 || y_type > 2) return M3S_ERR_INVALID_ARG;
  dim3 grid(m3s_div_up(rows, 4), (unsigned)batch);
  hipStream_t s = m3s_stream(stream);
  // float4 loads of gamma / beta: 16-byte aligned parameter rows
  if ((uintptr_t)d_gamma % 16 || (uintptr_t)d_beta % 16 || stride_param % 4)
    return M3S_ERR_INVALID_ARG;
  const bool narrow = dim <= 1024;
#define M3S_LN(XB, YT)                                                                        \
  do {                                                                                        \
  if (narrow)                                                                                 \
    hipLaunchKernelGGL((layernorm_kernel<XB, YT, false, 4>), grid, dim3(256), 0, s, d_x,      \
                       d_gamma, d_beta, d_y, rows, (int)dim, eps, stride_x, stride_y,         \
                       stride_param, param_mod, x_batch_xor);                                 \
  else                                                                                        \
    hipLaunchKernelGGL((layernorm_kernel<XB, YT, false, 16>), grid, dim3(256), 0, s, d_x,     \
                       d_gamma, d_beta, d_y, rows, (int)dim, eps, stride_x, stride_y,         \
                       stride_param, param_mod, x_batch_xor);                                 \
  } while (0)
  if (x_is_bf16) {
    if (y_type == 0) M3S_LN(true, 0);
    else if (y_type == 1) M3S_LN(true, 1);
    else M3S_LN(true, 2);
  } else {
    if (y_type == 0) M3S_LN(false, 0);
    else if (y_type == 1) M3S_LN(false, 1);
    else M3S_LN(false, 2);
  }
#undef M3S_LN
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_vit_layernorm_dual(const float* d_x, const float* d_gamma,
                                      const float* d_beta, void* d_y, const float* d_gamma2,
                                      const float* d_beta2, void* d_y2, int y_fp8, int64_t rows,
                                      int64_t dim, float eps, int64_t batch, int64_t stride_x,
                                      int64_t stride_y, int64_t stride_param, int64_t param_mod,
                                      void* stream) {
  if (!d_x || !d_gamma || !d_beta || !d_y || !d_gamma2 || !d_beta2 || !d_y2 || rows <= 0 ||
      batch <= 0 || batch % 2)
    return M3S_ERR_INVALID_ARG;
  if (dim % 4 || dim > 4096 || dim <= 0) return M3S_ERR_INVALID_ARG;
  if ((uintptr_t)d_gamma % 16 || (uintptr_t)d_beta % 16 || (uintptr_t)d_gamma2 % 16 ||
      (uintptr_t)d_beta2 % 16 || stride_param % 4)
    return M3S_ERR_INVALID_ARG;
  dim3 grid(m3s_div_up(rows, 4), (unsigned)batch);
  hipStream_t s = m3s_stream(stream);
#define M3S_LN2(YT, MV)                                                                       \
  hipLaunchKernelGGL((layernorm_kernel<false, YT, true, MV>), grid, dim3(256), 0, s, d_x,     \
                     d_gamma, d_beta, d_y, rows, (int)dim, eps, stride_x, stride_y,           \
                     stride_param, param_mod, 0, d_gamma2, d_beta2, d_y2)
  if (dim <= 1024) {
    if (y_fp8) M3S_LN2(2, 4);
    else M3S_LN2(0, 4);
  } else {
    if (y_fp8) M3S_LN2(2, 16);
    else M3S_LN2(0, 16);
  }
#undef M3S_LN2
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_vit_patchify(const float* d_img, void* d_out, int64_t batch, int64_t h,
                                int64_t w, void* stream) {
  if (!d_img || !d_out || batch <= 0 || h % 16 || w % 16 || h <= 0 || w <= 0)
    return M3S_ERR_INVALID_ARG;
  const int64_t total = batch * (h / 16) * (w / 16) * 96;
  hipLaunchKernelGGL(patchify_kernel, dim3(m3s_div_up(total, 256)), dim3(256), 0,
                     m3s_stream(stream), d_img, reinterpret_cast<bf16_t*>(d_out), (int)h, (int)w,
                     total);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

namespace {
// Strided row copy of `outer x inner` items (decoder input assembly, local-feature concat):
// item (o, i) copies `rows` rows of row_bytes from src + o·src_outer + i·src_inner + src_base
// (row stride src_row) to dst + o·dst_outer + i·dst_inner + dst_base (row stride dst_row),
// 16 B per thread (all sizes, strides and bases 16-B multiples: checked on the host).
__global__ __launch_bounds__(256) void copy_rows_kernel(
    const char* __restrict__ src, char* __restrict__ dst, int64_t rows, int64_t vpr,
    int64_t src_row, int64_t dst_row, int64_t inner, int64_t src_outer, int64_t src_inner,
    int64_t dst_outer, int64_t dst_inner, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int64_t v = t % vpr;
  const int64_t r = (t / vpr) % rows;
  const int64_t item = t / (vpr * rows);
  const int64_t o = item / inner, i = item - o * inner;
  const uint4 x = *reinterpret_cast<const uint4*>(src + o * src_outer + i * src_inner +
                                                  r * src_row + v * 16);
  *reinterpret_cast<uint4*>(dst + o * dst_outer + i * dst_inner + r * dst_row + v * 16) = x;
}
}  // namespace

extern "C" int m3s_copy_rows(const void* d_src, void* d_dst, int64_t rows, int64_t row_bytes,
                             int64_t src_row_stride, int64_t dst_row_stride, int64_t outer,
                             int64_t inner, int64_t src_outer, int64_t src_inner,
                             int64_t src_base, int64_t dst_outer, int64_t dst_inner,
                             int64_t dst_base, void* stream) {
  if (!d_src || !d_dst || rows < 0 || row_bytes < 0 || outer < 0 || inner <= 0)
    return M3S_ERR_INVALID_ARG;
  const int64_t total = outer * inner * rows * (row_bytes / 16);
  if (total == 0) return M3S_OK;
  const int64_t al = row_bytes | src_row_stride | dst_row_stride | src_outer | src_inner |
                     src_base | dst_outer | dst_inner | dst_base |
                     (int64_t)(uintptr_t)d_src | (int64_t)(uintptr_t)d_dst;
  if (al % 16) return M3S_ERR_INVALID_ARG;
  hipLaunchKernelGGL(copy_rows_kernel, dim3(m3s_div_up(total, 256)), dim3(256), 0,
                     m3s_stream(stream), reinterpret_cast<const char*>(d_src) + src_base,
                     reinterpret_cast<char*>(d_dst) + dst_base, rows, row_bytes / 16,
                     src_row_stride, dst_row_stride, inner, src_outer, src_inner, dst_outer,
                     dst_inner, total);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

namespace {
template <bool F8OUT>
int upsample2x_launch(const void* d_in, void* d_out, const void* d_add, int64_t batch, int64_t h,
                      int64_t w, int64_t c, int64_t oh, int64_t ow, float inv_scale,
                      void* stream) {
  if (!d_in || !d_out || batch <= 0 || h <= 0 || w <= 0 || c % 8) return M3S_ERR_INVALID_ARG;
  if (oh <= 0 || ow <= 0 || oh > 2 * h || ow > 2 * w) return M3S_ERR_INVALID_ARG;
  if (F8OUT && !(inv_scale > 0.f && inv_scale < 3.0e38f)) return M3S_ERR_INVALID_ARG;
  const int64_t total = batch * oh * ow * (c / 8);
  if (total < (int64_t(1) << 31) - 256)
    hipLaunchKernelGGL((upsample2x_kernel<uint32_t, F8OUT>), dim3(m3s_div_up(total, 256)),
                       dim3(256), 0, m3s_stream(stream), reinterpret_cast<const bf16_t*>(d_in),
                       d_out, reinterpret_cast<const bf16_t*>(d_add), (int)h, (int)w, (int)c,
                       (int)oh, (int)ow, (uint32_t)total, inv_scale);
  else
    hipLaunchKernelGGL((upsample2x_kernel<int64_t, F8OUT>), dim3(m3s_div_up(total, 256)),
                       dim3(256), 0, m3s_stream(stream), reinterpret_cast<const bf16_t*>(d_in),
                       d_out, reinterpret_cast<const bf16_t*>(d_add), (int)h, (int)w, (int)c,
                       (int)oh, (int)ow, total, inv_scale);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
}  // namespace

extern "C" int m3s_vit_upsample2x(const void* d_in, void* d_out, const void* d_add,
                                  int64_t batch, int64_t h, int64_t w, int64_t c, int64_t oh,
                                  int64_t ow, void* stream) {
  return upsample2x_launch<false>(d_in, d_out, d_add, batch, h, w, c, oh, ow, 1.f, stream);
}

extern "C" int m3s_vit_upsample2x_e4m3(const void* d_in, void* d_out, const void* d_add,
                                       int64_t batch, int64_t h, int64_t w, int64_t c, int64_t oh,
                                       int64_t ow, float inv_scale, void* stream) {
  return upsample2x_launch<true>(d_in, d_out, d_add, batch, h, w, c, oh, ow, inv_scale, stream);
}

extern "C" int m3s_vit_dpt_out(const void* d_t, const float* d_w4, const float* d_b4,
                               float* d_pts3d, float* d_conf, int64_t pixels, float conf_min,
                               int64_t batch, int64_t stride_t, int64_t stride_out,
                               int64_t param_mod, void* stream) {
  if (!d_t || !d_w4 || !d_b4 || !d_pts3d || !d_conf || pixels <= 0 || batch <= 0)
    return M3S_ERR_INVALID_ARG;
  dim3 grid(m3s_div_up(pixels, 256), (unsigned)batch);
  hipLaunchKernelGGL(dpt_out_kernel, grid, dim3(256), 0, m3s_stream(stream),
                     reinterpret_cast<const bf16_t*>(d_t), d_w4, d_b4, d_pts3d, d_conf, pixels,
                     conf_min, stride_t, stride_out, param_mod);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_vit_local_features(const float* d_feats, float* d_desc, uint16_t* d_desc_f16,
                                      float* d_desc_conf, int64_t batch, int64_t h, int64_t w,
                                      void* stream) {
  if (!d_feats || !d_desc_conf || (!d_desc && !d_desc_f16) || batch <= 0 || h % 16 || w % 16)
    return M3S_ERR_INVALID_ARG;
  const int64_t total = batch * h * w;
  hipLaunchKernelGGL(local_feat_kernel, dim3(m3s_div_up(total, 256)), dim3(256), 0,
                     m3s_stream(stream), d_feats, d_desc,
                     reinterpret_cast<_Float16*>(d_desc_f16), d_desc_conf, (int)h, (int)w, total);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
