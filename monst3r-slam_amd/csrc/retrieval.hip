// Keyframe retrieval / loop-closure candidate search (gfx950): the MASt3R retrieval head
// (Whitener + projector + how_select_local) and the binary ASMK inverted-file search that
// RetrievalDatabase.update runs once per new keyframe
// (mast3r_slam/retrieval_database.py:25-166; asmk/kernel.py:26-68; asmk/inverted_file.py:156-208;
//  asmk/cython/hamming.pyx; mast3r/retrieval/model.py:55-104).
//
//   m3s_retr_affine       Y = (X[rows] - mu) W + b, fp32 FMA tiles (whitening / projector)
//   m3s_retr_rownorm      ||Y_r||_2 (the 'l2norm' attention, model.py:133)
//   m3s_topk_select       sorted top-k of <= 4096 keys in one workgroup (bitonic in LDS)
//   m3s_retr_quantize     ||q||^2 + ||c||^2 - 2 q.c against the codebook on the f32 MFMA, the
//                         k smallest per row and 256-centroid chunk, merged by a second pass
//   m3s_asmk_aggregate    unique visual words, residual sums, sign binarisation packed MSB-first
//   m3s_ivf_search        per-image ASMK scores over a flat image-major inverted file
//
// Numerics: fp32 like the reference's torch/numpy code, except the scores (fp64, as numpy's
// `scores = np.zeros(n_images)` accumulates them).  Residual sums add descriptors in index order
// (numpy's axis-0 sum), so the packed codes are bit-exact given identical descriptors.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------------------------
// fp32 affine: Y[M][N] = (X[row(i)][:] - mu) * W[K][N] + bias on the f32 MFMA (32x32x2).
// 64x64 tile, 4 waves of 32x32, K slices of 32 staged through LDS with the next slice
// prefetched into registers during the MFMAs (the sizes here, M <= 768, give < 1 block per
// CU, so latency hiding inside the block is what matters).  X may be bf16 or fp32.
constexpr int ABK = 32, APAD = ABK + 1, ABN = 64, ABNP = ABN + 4;

template <typename XT>
__global__ __launch_bounds__(256) void affine_kernel(const XT* __restrict__ X, int64_t ldx,
                                                     const int64_t* __restrict__ rows,
                                                     const float* __restrict__ mu,
                                                     const float* __restrict__ W,
                                                     const float* __restrict__ bias, int M, int N,
                                                     int K, float* __restrict__ Y) {
  __shared__ float As[64 * APAD];
  __shared__ float Bs[ABK * ABNP];
  typedef float f32x16_t __attribute__((ext_vector_type(16)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * ABN;
  f32x16_t acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.f;
  // A: 64 rows x 32 k = 512 float4 (2 per thread, f = tid + 256u: row f>>3, k (f&7)*4)
  // B: 32 k x 64 n = 512 float4 (2 per thread, f: k f>>4, n (f&15)*4)
  int64_t src[2];
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const int r = m0 + ((tid + u * 256) >> 3);
    src[u] = r < M ? (rows ? rows[r] : r) : -1;
  }
  float4 ra[2], rb[2];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int f = tid + u * 256;
      const int k = k0 + (f & 7) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (src[u] >= 0 && k < K) {
        if constexpr (sizeof(XT) == 2) {
          const uint2 q = *reinterpret_cast<const uint2*>(X + src[u] * ldx + k);
          v = make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                          __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
        } else {
          v = *reinterpret_cast<const float4*>(X + src[u] * ldx + k);
        }
        if (mu) {
          const float4 mm = *reinterpret_cast<const float4*>(mu + k);
          v.x = v.x - mm.x; v.y = v.y - mm.y; v.z = v.z - mm.z; v.w = v.w - mm.w;
        }
      }
      ra[u] = v;
      const int kb = k0 + (f >> 4), n = n0 + (f & 15) * 4;
      float4 w = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kb < K) {
        if (n + 3 < N) {
          w = *reinterpret_cast<const float4*>(W + (int64_t)kb * N + n);
        } else {
          const float* wp = W + (int64_t)kb * N;
          w.x = n < N ? wp[n] : 0.f;
          w.y = n + 1 < N ? wp[n + 1] : 0.f;
          w.z = n + 2 < N ? wp[n + 2] : 0.f;
        }
      }
      rb[u] = w;
    }
  };
  fetch(0);
  const float* ap = As + (wm * 32 + (lane & 31)) * APAD + (lane >> 5);
  const float* bp = Bs + (lane >> 5) * ABNP + wn * 32 + (lane & 31);
  for (int k0 = 0; k0 < K; k0 += ABK) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int f = tid + u * 256;
      float* d = As + (f >> 3) * APAD + (f & 7) * 4;
      d[0] = ra[u].x; d[1] = ra[u].y; d[2] = ra[u].z; d[3] = ra[u].w;
      float* e = Bs + (f >> 4) * ABNP + (f & 15) * 4;
      e[0] = rb[u].x; e[1] = rb[u].y; e[2] = rb[u].z; e[3] = rb[u].w;
    }
    __syncthreads();
    if (k0 + ABK < K) fetch(k0 + ABK);
#pragma unroll
    for (int kk = 0; kk < ABK; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[kk], bp[kk * ABNP], acc, 0, 0, 0);
    __syncthreads();
  }
  const int col = n0 + wn * 32 + (lane & 31);
  if (col < N) {
    const float bb = bias ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) Y[(int64_t)row * N + col] = acc[r] + bb;
    }
  }
}

// One wave per row: sqrt(sum x^2) (sq = 0) or sum x^2 (sq = 1).
__global__ __launch_bounds__(256) void rownorm_kernel(const float* __restrict__ Y, int64_t M,
                                                      int N, int sq, float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  const float* y = Y + r * N;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s = fmaf(y[c], y[c], s);
  s = m3s_wave_sum(s);
  if (lane == 0) out[r] = sq ? s : sqrtf(s);
}

// ---------------------------------------------------------------------------------------------
// Sorted top-k of n <= 4096 keys (descending, ties to the lower index) by a bitonic sort of
// (key, index) pairs in LDS; one workgroup of 1024 threads.  fp32 keys are widened exactly.
constexpr int TOPK_MAX_N = 4096;

template <typename KT>
__global__ __launch_bounds__(1024) void topk_kernel(const KT* __restrict__ keys, int n, int k,
                                                    int largest, int64_t* __restrict__ idx_out,
                                                    KT* __restrict__ val_out) {
  __shared__ double sk[TOPK_MAX_N];
  __shared__ int si[TOPK_MAX_N];
  int P = 1;
  while (P < n) P <<= 1;
  const double pad = largest ? -INFINITY : INFINITY;
  for (int i = threadIdx.x; i < P; i += 1024) {
    sk[i] = i < n ? (double)keys[i] : pad;
    si[i] = i < n ? i : 0x7fffffff;
  }
  __syncthreads();
  // "a before b": larger key first (or smaller when !largest), ties by lower index
  auto before = [largest](double ka, int ia, double kb, int ib) {
    if (ka != kb) return largest ? ka > kb : ka < kb;
    return ia < ib;
  };
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += 1024) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const double ka = sk[lo], kb = sk[hi];
        const int ia = si[lo], ib = si[hi];
        const bool swap = up ? before(kb, ib, ka, ia) : before(ka, ia, kb, ib);
        if (swap) {
          sk[lo] = kb; sk[hi] = ka;
          si[lo] = ib; si[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k; i += 1024) {
    idx_out[i] = si[i];
    if (val_out) val_out[i] = (KT)sk[i];
  }
}

// ---------------------------------------------------------------------------------------------
// Codebook quantisation (retrieval_database.py:96-105): d = (|q|^2 + |c|^2) - 2 q.c, the k
// smallest per query row, ascending, ties to the lower centroid index.
// Grid (chunks, ceil(M/64)); a block covers 64 query rows x `chunk` centroids in 128-wide tiles.
constexpr int QK_MAX = 8;

__device__ __forceinline__ bool qless(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

__device__ __forceinline__ void qinsert(float* bd, int* bi, int k, float d, int i) {
  float wd = bd[0];
  int wi = bi[0];
#pragma unroll
  for (int s = 1; s < QK_MAX; s++)
    if (s == k - 1) {
      wd = bd[s];
      wi = bi[s];
    }
  if (!qless(d, i, wd, wi)) return;
  bool placed = false;
#pragma unroll
  for (int s = QK_MAX - 1; s >= 0; s--) {
    if (s >= k || placed) continue;
    if (s > 0 && qless(d, i, bd[s - 1], bi[s - 1])) {
      bd[s] = bd[s - 1];
      bi[s] = bi[s - 1];
    } else {
      bd[s] = d;
      bi[s] = i;
      placed = true;
    }
  }
}

// f32-input MFMA (v_mfma_f32_32x32x2_f32: exact fp32 products, k-ordered fp32 accumulation).
// Block: 64 query rows x 256 centroids (one chunk), 4 waves in 2 (rows) x 2 (cols), each wave
// 32 rows x 128 cols = 4 accumulators of 32x32.  K staged through LDS 32 at a time, operands
// kept row-major with a 1-float pad (fragment reads conflict-free).  The distance tile then
// goes through LDS: 4 threads per row scan 64 columns each keeping the k smallest, merged by a
// 2-step butterfly.  1-D grid, XCD-aware: the row blocks of one chunk run on one XCD so the
// chunk's 1 MB of centroids is fetched from HBM once and re-read from that XCD's L2.
constexpr int QBM = 64, QBN = 256, QBK = 32, QPAD = QBK + 1;
constexpr int QDST = QBN + 1;
constexpr int Q_LDS_FLOATS = (QBM * QDST > (QBM + QBN) * QPAD) ? QBM * QDST : (QBM + QBN) * QPAD;

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256, 2) void quantize_kernel(const float* __restrict__ Q,
                                                          const float* __restrict__ qn,
                                                          const float* __restrict__ C,
                                                          const float* __restrict__ cn, int M,
                                                          int NC, int D, int nchunk, int nrb,
                                                          int k, float* __restrict__ part_d,
                                                          int* __restrict__ part_i) {
  __shared__ float lds[Q_LDS_FLOATS];
  float* As = lds;                 // [QBM][QPAD]
  float* Bs = lds + QBM * QPAD;    // [QBN][QPAD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // blockIdx -> (chunk, row block); same chunk on the same XCD when nchunk % 8 == 0
  int chunk, rb;
  {
    const int L = blockIdx.x;
    if ((nchunk & 7) == 0) {
      const int xcd = L & 7, j = L >> 3;
      chunk = (j / nrb) * 8 + xcd;
      rb = j % nrb;
    } else {
      chunk = L / nrb;
      rb = L % nrb;
    }
  }
  const int m0 = rb * QBM, c0 = chunk * QBN;
  const int wm = wave >> 1, wn = wave & 1;
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[t][r] = 0.f;
  // loaders: A 64 rows x 32 k = 512 float4 (2 per thread); B 256 x 32 = 2048 float4 (8 each).
  // The next K slice is fetched into registers while the MFMAs consume the current one.
  float4 ra[2], rb4[8];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int f = tid + u * 256;
      const int m = m0 + (f >> 3);
      ra[u] = m < M ? *reinterpret_cast<const float4*>(Q + (int64_t)m * D + k0 + (f & 7) * 4)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int f = tid + u * 256;
      const int c = c0 + (f >> 3);
      rb4[u] = c < NC ? *reinterpret_cast<const float4*>(C + (int64_t)c * D + k0 + (f & 7) * 4)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  fetch(0);
  const float* ap = As + (wm * 32 + (lane & 31)) * QPAD + (lane >> 5);
  const float* bp = Bs + (wn * 128 + (lane & 31)) * QPAD + (lane >> 5);
  for (int k0 = 0; k0 < D; k0 += QBK) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int f = tid + u * 256;
      float* d = As + (f >> 3) * QPAD + (f & 7) * 4;
      d[0] = ra[u].x; d[1] = ra[u].y; d[2] = ra[u].z; d[3] = ra[u].w;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int f = tid + u * 256;
      float* d = Bs + (f >> 3) * QPAD + (f & 7) * 4;
      d[0] = rb4[u].x; d[1] = rb4[u].y; d[2] = rb4[u].z; d[3] = rb4[u].w;
    }
    __syncthreads();
    if (k0 + QBK < D) fetch(k0 + QBK);
#pragma unroll
    for (int kk = 0; kk < QBK; kk += 2) {
      const float a = ap[kk];
#pragma unroll
      for (int t = 0; t < 4; t++)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bp[t * 32 * QPAD + kk], acc[t], 0, 0, 0);
    }
    __syncthreads();
  }
  // distances into LDS: d = (|q|^2 + |c|^2) - 2 q.c
  float* dst = lds;  // [QBM][QDST]
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int col = wn * 128 + t * 32 + (lane & 31);
      dst[row * QDST + col] = acc[t][r];
    }
  __syncthreads();
  const int row = tid >> 2, part = tid & 3;
  const int m = m0 + row;
  const float q2 = m < M ? qn[m] : 0.f;
  float bd[QK_MAX];
  int bi[QK_MAX];
#pragma unroll
  for (int s = 0; s < QK_MAX; s++) {
    bd[s] = INFINITY;
    bi[s] = 0x7fffffff;
  }
  for (int j = 0; j < QBN / 4; j++) {
    const int cl = part + 4 * j;  // increasing per thread: ties keep the earlier index
    const int c = c0 + cl;
    if (c < NC) qinsert(bd, bi, k, (q2 + cn[c]) - 2.0f * dst[row * QDST + cl], c);
  }
#pragma unroll
  for (int off = 1; off < 4; off <<= 1) {
    float od[QK_MAX];
    int oi[QK_MAX];
#pragma unroll
    for (int s = 0; s < QK_MAX; s++) {
      od[s] = __shfl_xor(bd[s], off, 64);
      oi[s] = __shfl_xor(bi[s], off, 64);
    }
#pragma unroll
    for (int s = 0; s < QK_MAX; s++)
      if (s < k) qinsert(bd, bi, k, od[s], oi[s]);
  }
  if (part == 0 && m < M) {
    const int64_t o = ((int64_t)m * nchunk + chunk) * k;
#pragma unroll
    for (int s = 0; s < QK_MAX; s++)
      if (s < k) {
        part_d[o + s] = bd[s];
        part_i[o + s] = bi[s];
      }
  }
}

// One 64-thread block (one wave) per query row: each lane merges a strided subset of the chunk
// partials, then a 6-step butterfly over the wave (lanes hold disjoint candidate sets).
__global__ __launch_bounds__(64) void quantize_merge_kernel(const float* __restrict__ part_d,
                                                            const int* __restrict__ part_i,
                                                            int nchunk, int k,
                                                            int32_t* __restrict__ codes,
                                                            float* __restrict__ dists) {
  const int m = blockIdx.x, t = threadIdx.x;
  float rd[QK_MAX];
  int ri[QK_MAX];
#pragma unroll
  for (int s = 0; s < QK_MAX; s++) {
    rd[s] = INFINITY;
    ri[s] = 0x7fffffff;
  }
  const int64_t base = (int64_t)m * nchunk * k;
  for (int c = t; c < nchunk; c += 64)
    for (int s = 0; s < k; s++) qinsert(rd, ri, k, part_d[base + c * k + s], part_i[base + c * k + s]);
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    float od[QK_MAX];
    int oi[QK_MAX];
#pragma unroll
    for (int s = 0; s < QK_MAX; s++) {
      od[s] = __shfl_xor(rd[s], off, 64);
      oi[s] = __shfl_xor(ri[s], off, 64);
    }
#pragma unroll
    for (int s = 0; s < QK_MAX; s++)
      if (s < k) qinsert(rd, ri, k, od[s], oi[s]);
  }
  if (t == 0) {
#pragma unroll
    for (int s = 0; s < QK_MAX; s++)
      if (s < k) {
        codes[(int64_t)m * k + s] = ri[s];
        if (dists) dists[(int64_t)m * k + s] = rd[s];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// ASMK aggregation (kernel.py:26-39): unique words of the codes (sorted, np.unique), per word
// the sum over descriptors having that word among their k codes of (des - centroid), then
// binarize_and_pack_2D (hamming.pyx:77-110): bit = sum > 0, element 0 of each 32 in the MSB.
__global__ __launch_bounds__(256) void mark_words_kernel(const int32_t* __restrict__ codes,
                                                         int64_t n, int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) flags[codes[i]] = 1;
}

// One workgroup of 16 waves: ordered compaction of the flag array -> sorted unique words +
// count; wave w owns a contiguous range, lane l four consecutive flags per step (int4).
// Pass 1 counts per wave, pass 2 writes at wave offset + lane prefix.  Clears the flags.
__global__ __launch_bounds__(1024) void compact_words_kernel(int32_t* __restrict__ flags, int NC,
                                                             int32_t* __restrict__ words,
                                                             int32_t* __restrict__ count) {
  __shared__ int wtot[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int per = ((NC + 16 * 256 - 1) / (16 * 256)) * 256;  // multiple of 256 flags per wave
  const int b0 = w * per, b1 = min(NC, b0 + per);
  auto load4 = [&](int i) {
    int4 v = make_int4(0, 0, 0, 0);
    if (i + 3 < b1) {
      v = *reinterpret_cast<const int4*>(flags + i);
    } else {
      v.x = i < b1 ? flags[i] : 0;
      v.y = i + 1 < b1 ? flags[i + 1] : 0;
      v.z = i + 2 < b1 ? flags[i + 2] : 0;
    }
    return v;
  };
  int cnt = 0;
  for (int i0 = b0; i0 < b1; i0 += 256) {
    const int4 v = load4(i0 + lane * 4);
    cnt += (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
  }
  cnt = m3s_wave_sum_int(cnt);
  if (lane == 0) wtot[w] = cnt;
  __syncthreads();
  int off = 0;
  for (int u = 0; u < w; u++) off += wtot[u];
  for (int i0 = b0; i0 < b1; i0 += 256) {
    const int i = i0 + lane * 4;
    const int4 v = load4(i);
    const int c = (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
    int incl = c;  // inclusive prefix over lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(incl, d, 64);
      if (lane >= d) incl += t;
    }
    int p = off + incl - c;
    if (v.x) { words[p++] = i; flags[i] = 0; }
    if (v.y) { words[p++] = i + 1; flags[i + 1] = 0; }
    if (v.z) { words[p++] = i + 2; flags[i + 2] = 0; }
    if (v.w) { words[p++] = i + 3; flags[i + 3] = 0; }
    off += __shfl(incl, 63, 64);
  }
  if (threadIdx.x == 0) {
    int s = 0;
    for (int u = 0; u < 16; u++) s += wtot[u];
    *count = s;
  }
}

// One workgroup per unique word (blocks past the count exit): thread t owns elements
// t, t+256, ... of the residual sum; packed with a wave ballot (lane l = element base + l).
__global__ __launch_bounds__(256) void aggregate_kernel(const float* __restrict__ des, int n,
                                                        int D, const int32_t* __restrict__ codes,
                                                        int k, const float* __restrict__ C,
                                                        const int32_t* __restrict__ words,
                                                        const int32_t* __restrict__ count,
                                                        uint32_t* __restrict__ packed) {
  const int u = blockIdx.x;
  if (u >= *count) return;
  const int word = words[u];
  const int W32 = D / 32;
  // ordered list of the member descriptors (ballot compaction keeps index order)
  extern __shared__ int member[];
  __shared__ int wcnt[4];
  __shared__ int nmem;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (threadIdx.x == 0) nmem = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + threadIdx.x;
    int hit = 0;
    if (i < n)
      for (int s = 0; s < k; s++) hit |= codes[(int64_t)i * k + s] == word;
    const uint64_t b = __ballot(hit);
    if (ln == 0) wcnt[wv] = __popcll(b);
    __syncthreads();
    int off = nmem;
    for (int w = 0; w < wv; w++) off += wcnt[w];
    if (hit) member[off + __popcll(b & ((1ull << ln) - 1ull))] = i;
    __syncthreads();
    if (threadIdx.x == 0) nmem += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
  const int nm = nmem;
  const float* c = C + (int64_t)word * D;
  const int lane = threadIdx.x & 63;
  for (int e0 = 0; e0 < D; e0 += 256) {
    const int e = e0 + threadIdx.x;
    float acc = 0.f;
    if (e < D) {
      const float ce = c[e];
      for (int j = 0; j < nm; j++) acc = acc + (des[(int64_t)member[j] * D + e] - ce);
    }
    const uint64_t b = __ballot(e < D && acc > 0.f);
    // elements e0 + wave*64 + [0,32) -> word (e0 + wave*64)/32, [32,64) -> the next
    const int wbase = (e0 + (threadIdx.x & ~63)) / 32;
    if (lane == 0 && wbase < W32)
      packed[(int64_t)u * W32 + wbase] = __builtin_bitreverse32((uint32_t)(b & 0xffffffffull));
    if (lane == 32 && wbase + 1 < W32)
      packed[(int64_t)u * W32 + wbase + 1] = __builtin_bitreverse32((uint32_t)(b >> 32));
  }
}

// ---------------------------------------------------------------------------------------------
// IVF search (inverted_file.py:186-208 + kernel.py:56-68 + functional.py:96-100) over a flat
// image-major inverted file: image g owns entries [img_start[g], img_start[g+1]).  Per entry
// whose word the query holds: sim = 1 - 2 hamming/bits (fp32), kept if sim >= thr, sim^alpha,
// divided by sqrt(norm_factor[g]) (= entries of g without idf) in fp64; per-image sums in a
// fixed order; the total / sqrt(#query words).
__global__ __launch_bounds__(256) void word_map_kernel(const int32_t* __restrict__ qwords,
                                                       const int32_t* __restrict__ qcount,
                                                       int32_t* __restrict__ map, int set) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < *qcount) map[qwords[i]] = set ? i : -1;
}

__global__ __launch_bounds__(256) void ivf_score_kernel(
    const uint32_t* __restrict__ qpacked, const int32_t* __restrict__ qcount,
    const int32_t* __restrict__ map, const uint32_t* __restrict__ db_packed,
    const int32_t* __restrict__ db_words, const int32_t* __restrict__ img_start, int W32,
    float alpha, float thr, double* __restrict__ scores) {
  __shared__ float contrib[256];
  const int g = blockIdx.x;
  const int b = img_start[g], e = img_start[g + 1];
  const float nbits = (float)(W32 * 32);
  const double rnorm = sqrt((double)(e - b));  // norm_factor[g] without idf
  double s = 0.0;
  for (int j0 = b; j0 < e; j0 += 256) {
    const int j = j0 + threadIdx.x;
    float c = 0.f;
    if (j < e) {
      const int q = map[db_words[j]];
      if (q >= 0) {
        int hd = 0;
        for (int w = 0; w < W32; w++)
          hd += __popc(qpacked[(int64_t)q * W32 + w] ^ db_packed[(int64_t)j * W32 + w]);
        const float h = (float)hd / nbits;
        const float sim = -2.0f * h + 1.0f;  // hamming -> similarity in [-1, 1] (fp32)
        if (sim >= thr) {
          // sim ** alpha (fp32), *= idf (1), /= sqrt(norm_factor) in fp64 stored back to fp32
          c = (float)((double)powf(sim, alpha) / rnorm);
        }
      }
    }
    contrib[threadIdx.x] = c;
    __syncthreads();
    // entries of an image are in ascending word order, the order the reference's loop over
    // the query's (sorted) words adds them: sum sequentially in fp64
    if (threadIdx.x == 0) {
      const int m = min(256, e - j0);
      for (int u = 0; u < m; u++) s += (double)contrib[u];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) scores[g] = s / (double)sqrtf((float)*qcount);
}

}  // namespace

extern "C" int m3s_retr_affine(const void* d_X, int X_is_bf16, int64_t ldx, const int64_t* d_rows,
                               const float* d_mu, const float* d_W, const float* d_bias, int64_t M,
                               int64_t N, int64_t K, float* d_Y, void* stream) {
  if (!d_X || !d_W || !d_Y || M < 0 || N <= 0 || K <= 0 || ldx < K || K % 4 || ldx % 4 || N % 4)
    return M3S_ERR_INVALID_ARG;
  if (M == 0) return M3S_OK;
  dim3 grid(m3s_div_up(N, ABN), m3s_div_up(M, 64));
  hipStream_t s = m3s_stream(stream);
  if (X_is_bf16)
    hipLaunchKernelGGL((affine_kernel<__bf16>), grid, dim3(256), 0, s,
                       reinterpret_cast<const __bf16*>(d_X), ldx, d_rows, d_mu, d_W, d_bias,
                       (int)M, (int)N, (int)K, d_Y);
  else
    hipLaunchKernelGGL((affine_kernel<float>), grid, dim3(256), 0, s,
                       reinterpret_cast<const float*>(d_X), ldx, d_rows, d_mu, d_W, d_bias,
                       (int)M, (int)N, (int)K, d_Y);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_retr_rownorm(const float* d_Y, int64_t M, int64_t N, int squared, float* d_out,
                                void* stream) {
  if (!d_Y || !d_out || M < 0 || N <= 0) return M3S_ERR_INVALID_ARG;
  if (M == 0) return M3S_OK;
  hipLaunchKernelGGL(rownorm_kernel, dim3(m3s_div_up(M, 4)), dim3(256), 0, m3s_stream(stream),
                     d_Y, M, (int)N, squared, d_out);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_topk_select(const void* d_keys, int keys_f64, int64_t n, int64_t k, int largest,
                               int64_t* d_idx, void* d_vals, void* stream) {
  if (!d_keys || !d_idx || n <= 0 || n > TOPK_MAX_N || k < 0 || k > n) return M3S_ERR_INVALID_ARG;
  if (k == 0) return M3S_OK;
  hipStream_t s = m3s_stream(stream);
  if (keys_f64)
    hipLaunchKernelGGL((topk_kernel<double>), dim3(1), dim3(1024), 0, s,
                       reinterpret_cast<const double*>(d_keys), (int)n, (int)k, largest, d_idx,
                       reinterpret_cast<double*>(d_vals));
  else
    hipLaunchKernelGGL((topk_kernel<float>), dim3(1), dim3(1024), 0, s,
                       reinterpret_cast<const float*>(d_keys), (int)n, (int)k, largest, d_idx,
                       reinterpret_cast<float*>(d_vals));
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" size_t m3s_retr_quantize_workspace_bytes(int64_t M, int64_t ncent, int64_t k) {
  const int64_t nchunk = (ncent + QBN - 1) / QBN;
  return (size_t)(M * nchunk * k) * (sizeof(float) + sizeof(int));
}

extern "C" int m3s_retr_quantize(const float* d_Q, const float* d_qnorm2, int64_t M,
                                 const float* d_C, const float* d_cnorm2, int64_t ncent, int64_t D,
                                 int64_t k, int32_t* d_codes, float* d_dists, void* d_workspace,
                                 void* stream) {
  if (!d_Q || !d_qnorm2 || !d_C || !d_cnorm2 || !d_codes || !d_workspace) return M3S_ERR_INVALID_ARG;
  if (M < 0 || ncent <= 0 || D <= 0 || D % QBK || k < 1 || k > QK_MAX || k > ncent)
    return M3S_ERR_INVALID_ARG;
  if (M == 0) return M3S_OK;
  const int nchunk = (int)((ncent + QBN - 1) / QBN);
  const int nrb = (int)((M + QBM - 1) / QBM);
  float* pd = reinterpret_cast<float*>(d_workspace);
  int* pi = reinterpret_cast<int*>(pd + M * nchunk * k);
  hipStream_t s = m3s_stream(stream);
  hipLaunchKernelGGL(quantize_kernel, dim3((unsigned)(nchunk * nrb)), dim3(256), 0, s, d_Q,
                     d_qnorm2, d_C, d_cnorm2, (int)M, (int)ncent, (int)D, nchunk, nrb, (int)k,
                     pd, pi);
  hipLaunchKernelGGL(quantize_merge_kernel, dim3((unsigned)M), dim3(64), 0, s, pd, pi, nchunk,
                     (int)k, d_codes, d_dists);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_asmk_aggregate(const float* d_des, int64_t n, int64_t D, const int32_t* d_codes,
                                  int64_t k, const float* d_C, int64_t ncent, int32_t* d_flags,
                                  int32_t* d_words, int32_t* d_count, uint32_t* d_packed,
                                  void* stream) {
  if (!d_des || !d_codes || !d_C || !d_flags || !d_words || !d_count || !d_packed)
    return M3S_ERR_INVALID_ARG;
  if (n <= 0 || D <= 0 || D % 32 || k < 1 || ncent <= 0 || n > 16384) return M3S_ERR_INVALID_ARG;
  hipStream_t s = m3s_stream(stream);
  hipLaunchKernelGGL(mark_words_kernel, dim3(m3s_div_up(n * k, 256)), dim3(256), 0, s, d_codes,
                     n * k, d_flags);
  hipLaunchKernelGGL(compact_words_kernel, dim3(1), dim3(1024), 0, s, d_flags, (int)ncent, d_words,
                     d_count);
  hipLaunchKernelGGL(aggregate_kernel, dim3((unsigned)(n * k)), dim3(256), n * sizeof(int), s,
                     d_des, (int)n, (int)D, d_codes, (int)k, d_C, d_words, d_count, d_packed);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}

extern "C" int m3s_ivf_search(const uint32_t* d_qpacked, const int32_t* d_qwords,
                              const int32_t* d_qcount, int64_t max_qwords,
                              const uint32_t* d_db_packed, const int32_t* d_db_words,
                              const int32_t* d_img_start, int64_t n_images, int64_t D, float alpha,
                              float similarity_threshold, int32_t* d_word_map, double* d_scores,
                              void* stream) {
  if (!d_qpacked || !d_qwords || !d_qcount || !d_db_packed || !d_db_words || !d_img_start ||
      !d_word_map || !d_scores || D % 32 || max_qwords <= 0)
    return M3S_ERR_INVALID_ARG;
  if (n_images <= 0) return M3S_OK;
  hipStream_t s = m3s_stream(stream);
  const unsigned gq = m3s_div_up(max_qwords, 256);
  hipLaunchKernelGGL(word_map_kernel, dim3(gq), dim3(256), 0, s, d_qwords, d_qcount, d_word_map, 1);
  hipLaunchKernelGGL(ivf_score_kernel, dim3((unsigned)n_images), dim3(256), 0, s, d_qpacked,
                     d_qcount, d_word_map, d_db_packed, d_db_words, d_img_start, (int)(D / 32),
                     alpha, similarity_threshold, d_scores);
  hipLaunchKernelGGL(word_map_kernel, dim3(gq), dim3(256), 0, s, d_qwords, d_qcount, d_word_map, 0);
  M3S_LAUNCH_CHECK();
  return M3S_OK;
}
