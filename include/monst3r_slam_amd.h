/*
 * monst3r_slam_amd.h — C ABI of the MI355X-native MonST3R/MASt3R-SLAM hot path.
 *
 * Plain pointers, sizes and scalars only (no torch types). Every pointer named
 * `d_*` is a DEVICE pointer (HBM, hipMalloc'd or a torch CUDA tensor's data_ptr);
 * `stream` is a hipStream_t passed as void* (NULL = legacy default stream, which is
 * what the reference launches on: matching_kernels.cu:104,303; gn_kernels.cu:767,...).
 * All tensors are dense, C-contiguous, in the reference's layouts (cited per call).
 * Calls are asynchronous on `stream` unless the comment says otherwise.
 *
 * Return value: M3S_OK (0) or a negative M3S_ERR_* code; m3s_status_string() names it.
 * The Python drop-in (monst3r-slam_amd/mast3r_slam_backends) maps non-zero to
 * RuntimeError, like the reference's TORCH_CHECK (gn.h:5, gn.cpp:14-21,92-94,108-110).
 *
 * Numerical model (shared with oracle/):
 *   - iter_proj: the reference source taken literally — f32 ops, no FMA contraction,
 *     double-promoted sub-expressions (`1.0/x`, `(1.0-du)*dv`, `lambda*=0.1`) in f64.
 *   - refine_matches: c10::Half arithmetic (Half-inl.h operator*, operator+=):
 *     each product and each partial sum rounded to f16 (RNE), k = 0..F-1 in order;
 *     initial best score = value-initialised half (+0.0) — see DESIGN.md.
 */
#ifndef MONST3R_SLAM_AMD_H
#define MONST3R_SLAM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  M3S_OK = 0,
  M3S_ERR_INVALID_ARG = -1,   /* null pointer / bad size (reference: TORCH_CHECK) */
  M3S_ERR_HIP = -2,           /* a HIP runtime call or kernel launch failed        */
  M3S_ERR_TOO_LARGE = -3,     /* a size exceeds a kernel's static capacity          */
  M3S_ERR_NOT_PD = -4,        /* Cholesky failed; reference semantics kept (zero step) */
  M3S_ERR_NO_DEVICE = -5
};

const char* m3s_status_string(int status);
int m3s_version(void);                 /* (major<<16)|(minor<<8)|patch */
int m3s_device_count(void);

/* Step timeline (diagnostic; bench.py step_timeline).  m3s_timeline_set(d_buf, capacity)
 * arms it: every GEMM (m3s_vit_gemm) and attention (m3s_vit_attention) launch issued
 * afterwards — eager or captured into a graph — takes the next of `capacity` slots of
 * d_buf (u64 [capacity][132]: per slot 64 pairs {earliest block start, latest wave end}
 * in s_memrealtime ticks of 100 MHz, block b stamping pair b % 64; the launch spans
 * [min of the starts, max of the ends]; the caller fills every pair with {UINT64_MAX, 0}
 * before a run; then a 4-u64 header {block-log buffer or 0, pointer to its u32 record
 * counter, capacity in records, 0}, zeroed by m3s_timeline_set (call it outside any stream
 * capture; it synchronises the device) and filled by the caller afterwards: when set, the
 * first wave of every block appends
 * {start, end, slot address, HW_ID | XCC_ID << 32, 4 phase marks} (8 u64) at the counter — the busy
 * intervals of every CU).  A null d_buf
 * disarms it (later launches carry no slot).  m3s_timeline_count() = slots taken since the
 * last set; m3s_timeline_meta() copies their kinds (1 GEMM, 2 attention, 3 implicit 3x3
 * conv GEMM), algorithmic
 * FLOPs (2·M·N·K·batch; 4·Sq·Sk·64·heads·batch) and dims ({M, N, K, batch};
 * {Sq, Sk, heads, batch}) to host arrays of `capacity` entries (dims: [capacity][4]). */
int m3s_timeline_set(void* d_buf, int capacity);
int m3s_timeline_count(void);
int m3s_timeline_meta(int* kinds, double* flops, int64_t* dims, int capacity);

/* ------------------------------------------------------------------------- *
 * Projective matching.
 * ------------------------------------------------------------------------- */

/* Replaces mast3r_slam_backends.iter_proj  (gn.cpp:84-99 → matching_kernels.cu:279-316,
 * kernel :119-275).  rays_img_with_grad f32[b,h,w,c] (c = 9: ray xyz, d/dx xyz, d/dy xyz),
 * pts_3d_norm f32[b,n,3], p_init f32[b,n,2]  →  p_new f32[b,n,2], converged u8[b,n].
 * Any n ≥ 0 (the reference needs n % 16 == 0 — it has no tail guard). */
int m3s_iter_proj(const float* d_rays_img_with_grad, const float* d_pts_3d_norm,
                  const float* d_p_init, float* d_p_new, uint8_t* d_converged,
                  int64_t b, int64_t h, int64_t w, int64_t n,
                  int max_iter, float lambda_init, float cost_thresh, void* stream);

/* m3s_iter_proj under the FMA-contracted numeric model (opt-in): the products fused into
 * the adds that consume them as nvcc's default --fmad=true contraction does under LLVM's
 * rules (sums of products as fma chains, a*b - c*d as fma(a, b, -(c*d)), r*inv - pts and
 * u + det_inv*(...) fused).  Bit-exact to oracle/matching_ref.c ref_iter_proj_fma; same
 * arguments and errors as m3s_iter_proj.  DESIGN §2 records how far the models differ. */
int m3s_iter_proj_fma(const float* d_rays_img_with_grad, const float* d_pts_3d_norm,
                      const float* d_p_init, float* d_p_new, uint8_t* d_converged,
                      int64_t b, int64_t h, int64_t w, int64_t n,
                      int max_iter, float lambda_init, float cost_thresh, void* stream);

/* Replaces mast3r_slam_backends.refine_matches (gn.cpp:101-114 → matching_kernels.cu:84-116,
 * kernel :25-81).  D11 f16[b,h,w,fdim], D21 f16[b,n,fdim] (raw IEEE half bits),
 * p1 i64[b,n,2] (u,v)  →  p1_new i64[b,n,2].  fdim ≤ 64. */
int m3s_refine_matches(const uint16_t* d_D11, const uint16_t* d_D21, const int64_t* d_p1,
                       int64_t* d_p1_new, int64_t b, int64_t h, int64_t w, int64_t n,
                       int64_t fdim, int radius, int dilation_max, void* stream);

/* Fused replacement for matching.prep_for_iter_proj (matching.py:25-49) and
 * image.img_gradient (image.py:5-38): rays = X11/max(|X11|,1e-12);
 * g{x,y} = 3×3 Scharr/32 on reflect-padded rays;  pts = X21/max(|X21|,1e-12);
 * p_init = (idx % w, idx / w) (identity when d_idx_init == NULL).
 * X11,X21 f32[b,h,w,3] → rays_with_grad f32[b,h,w,9], pts f32[b,h*w,3], p_init f32[b,h*w,2]. */
int m3s_match_prep(const float* d_X11, const float* d_X21, const int64_t* d_idx_init,
                   float* d_rays_with_grad, float* d_pts_norm, float* d_p_init,
                   int64_t b, int64_t h, int64_t w, void* stream);

/* Occlusion test + truncation of matching.match_iterative_proj (matching.py:67-76):
 * p1 = trunc(p) (int64); valid = converged & (|X11[b,p1v,p1u] - X21[b,n]| < dist_thresh).
 * p f32[b,n,2], converged u8[b,n] → p1 i64[b,n,2], valid u8[b,n]. */
int m3s_match_occlusion(const float* d_X11, const float* d_X21, const float* d_p,
                        const uint8_t* d_converged, int64_t* d_p1, uint8_t* d_valid,
                        int64_t b, int64_t h, int64_t w, float dist_thresh, void* stream);

/* pixel_to_lin (matching.py:13-15,88): idx = u + w*v.  p1 i64[b,n,2] → idx i64[b,n]. */
int m3s_pixel_to_lin(const int64_t* d_p1, int64_t* d_idx, int64_t b, int64_t n, int64_t w,
                     void* stream);

/* ------------------------------------------------------------------------- *
 * Backend Gauss-Newton over the keyframe graph (gn_kernels.cu).
 * Twc f32[P,8] (t xyz, q xyzw, s — lietorch Sim3 layout) is UPDATED IN PLACE, exactly
 * like the reference (gn_kernels.cu:1212 pose_retr_kernel writes Twc).  ii,jj i64[E]
 * are global keyframe ids; Twc/Xs/Cs are indexed by rank in sorted unique(ii ∪ jj)
 * (gn_kernels.cu:161-170); the rank-0 pose is fixed (num_fix = 1, :1157).
 * Xs f32[P,N,3], Cs f32[P,N,1], idx_ii2jj i64[E,N], valid_match u8[E,N,1], Q f32[E,N,1].
 * dx_out f32[P-1,7] receives the last step (the reference's return value).
 * The solve (Eigen SimplicialLLT on the host in the reference, :57-159) runs on the
 * GPU in fp64; no host round trip and no per-iteration sync.  If the Cholesky fails
 * the step is zero (reference :142-150) and M3S_ERR_NOT_PD is reported through
 * *h_status_out after the call completes (it is written by a final D2H copy; the call
 * synchronises `stream` only when h_status_out != NULL).
 * workspace: d_workspace of m3s_gn_workspace_bytes(P, E, N) bytes (device); it includes a
 * packed copy of the inputs (16-B (X, C) records, 32-bit match indices: 16 P N + 4 E N B).
 * N < 2^31.
 * ------------------------------------------------------------------------- */
size_t m3s_gn_workspace_bytes(int64_t num_poses, int64_t num_edges, int64_t num_points);

/* Replaces mast3r_slam_backends.gauss_newton_rays (gn.cpp:28-50 → gn_kernels.cu:1140-1228). */
int m3s_gauss_newton_rays(float* d_Twc, const float* d_Xs, const float* d_Cs,
                          const int64_t* d_ii, const int64_t* d_jj, const int64_t* d_idx_ii2jj,
                          const uint8_t* d_valid_match, const float* d_Q,
                          int64_t num_poses, int64_t num_points, int64_t num_edges,
                          float sigma_ray, float sigma_dist, float C_thresh, float Q_thresh,
                          int max_iter, float delta_thresh, float* d_dx_out,
                          void* d_workspace, int* h_status_out, void* stream);

/* Replaces mast3r_slam_backends.gauss_newton_calib (gn.cpp:52-82 → gn_kernels.cu:1546-1638).
 * K f32[3,3] (device). */
int m3s_gauss_newton_calib(float* d_Twc, const float* d_Xs, const float* d_Cs, const float* d_K,
                           const int64_t* d_ii, const int64_t* d_jj, const int64_t* d_idx_ii2jj,
                           const uint8_t* d_valid_match, const float* d_Q,
                           int64_t num_poses, int64_t num_points, int64_t num_edges,
                           int height, int width, int pixel_border, float z_eps,
                           float sigma_pixel, float sigma_depth, float C_thresh, float Q_thresh,
                           int max_iter, float delta_thresh, float* d_dx_out,
                           void* d_workspace, int* h_status_out, void* stream);

/* Replaces mast3r_slam_backends.gauss_newton_points (gn.cpp:3-26 → gn_kernels.cu:725-811). */
int m3s_gauss_newton_points(float* d_Twc, const float* d_Xs, const float* d_Cs,
                            const int64_t* d_ii, const int64_t* d_jj, const int64_t* d_idx_ii2jj,
                            const uint8_t* d_valid_match, const float* d_Q,
                            int64_t num_poses, int64_t num_points, int64_t num_edges,
                            float sigma_point, float C_thresh, float Q_thresh,
                            int max_iter, float delta_thresh, float* d_dx_out,
                            void* d_workspace, int* h_status_out, void* stream);

/* Diagnostic: 1 = run every backend GN solve on the global-memory dense path instead of the
 * LDS-resident one used while 7(P-1) <= 140 (both give bit-identical poses; tests compare
 * them).  Not thread-scoped; returns M3S_OK. */
int m3s_gn_force_global_solve(int on);

/* Edge-sharded backend GN (the iteration of gn_kernels.cu:1140-1228 split at
 * its reduction).  Each rank holds the data rows of ITS two-way edges only (idx / valid /
 * Q [E_local,...], global edge ids d_edge_ids i32 [E_local]) plus the replicated poses
 * and pointmaps; per iteration:
 *   m3s_gn_{rays,calib}_edge_pass  → d_G f64 [E_local][35]: the per-edge sums
 *                                    (28 of Σ w J'J'ᵀ + 7 of Σ w e J')
 *   (caller) all-gather the rows into d_G_all [E_total][35] in global edge order
 *   m3s_gn_solve_step              → assemble + fp64 Cholesky + retract + convergence flag
 * m3s_gn_sharded_begin once before (ranks of all E_total edges, flags, dx = 0); the first
 * edge pass after it packs Xs / Cs / idx / valid into the workspace, later ones (until the
 * next begin) read that copy — the points and matches are fixed during a solve;
 * m3s_gn_sharded_status after (synchronises; status as h_status_out of the calls above,
 * iterations taken).  The split count S follows E_total, so every edge's sums — and the
 * poses — are bit-identical to the unsharded call's.  After convergence the kernels exit
 * at once (device flag), so a fixed max_iter loop needs no host sync. */
size_t m3s_gn_sharded_workspace_bytes(int64_t num_poses, int64_t num_edges_total,
                                      int64_t num_edges_local, int64_t num_points);
int m3s_gn_sharded_begin(const int64_t* d_ii, const int64_t* d_jj, int64_t num_poses,
                         int64_t num_points, int64_t num_edges_total, int64_t num_edges_local,
                         float* d_dx_out, void* d_workspace, void* stream);
int m3s_gn_rays_edge_pass(const float* d_Twc, const float* d_Xs, const float* d_Cs,
                          const int32_t* d_edge_ids, const int64_t* d_idx_local,
                          const uint8_t* d_valid_local, const float* d_Q_local,
                          int64_t num_poses, int64_t num_points, int64_t num_edges_total,
                          int64_t num_edges_local, float sigma_ray, float sigma_dist,
                          float C_thresh, float Q_thresh, double* d_G_local, void* d_workspace,
                          void* stream);
int m3s_gn_calib_edge_pass(const float* d_Twc, const float* d_Xs, const float* d_Cs,
                           const float* d_K, const int32_t* d_edge_ids,
                           const int64_t* d_idx_local, const uint8_t* d_valid_local,
                           const float* d_Q_local, int64_t num_poses, int64_t num_points,
                           int64_t num_edges_total, int64_t num_edges_local, int height,
                           int width, int pixel_border, float z_eps, float sigma_pixel,
                           float sigma_depth, float C_thresh, float Q_thresh, double* d_G_local,
                           void* d_workspace, void* stream);
int m3s_gn_solve_step(float* d_Twc, const double* d_G_all, int64_t num_poses,
                      int64_t num_points, int64_t num_edges_total, int64_t num_edges_local,
                      float delta_thresh, float* d_dx_out, void* d_workspace, void* stream);
int m3s_gn_sharded_status(const void* d_workspace, int64_t num_poses, int* h_status_out,
                          int* h_iters_out, void* stream);

/* ------------------------------------------------------------------------- *
 * Frontend tracker: 7-dof Sim3 Gauss-Newton of FrameTracker2.opt_pose_ray_dist_sim3
 * (tracker2.py:316-357, solve :299-314, check_convergence nonlinear_optimizer.py:5-25)
 * and opt_pose_calib_sim3 (tracker2.py:359-409), fused: residual + Jacobian + Huber
 * weights + 7×7 normal equations per point, reduced on device; 7×7 Cholesky, lietorch
 * left retraction and the convergence test on device (no .item() per iteration).
 * Twc_k, Twc_f f32[8] (lietorch Sim3 data).  Xf, Xk f32[N,3]; Qk f32[N]; valid u8[N].
 * Out: T_WCf f32[8] and T_CkCf f32[8] (device), info i32[4] (device):
 *   info[0] iterations run, info[1] 1 if Cholesky failed (frame lost, tracker2.py:234),
 *   info[2] 1 if converged, info[3] iterations run by the single-workgroup recovery path
 *   (0 normally; > 0 when the persistent launch lost co-residency next to concurrent
 *   kernels and stopped at a barrier timeout — the result is still the GN solution, never
 *   a Cholesky failure).
 * workspace: m3s_track_workspace_bytes(N) bytes.
 * ------------------------------------------------------------------------- */
size_t m3s_track_workspace_bytes(int64_t n);

int m3s_track_rays(const float* d_Twc_k, const float* d_Twc_f, const float* d_Xf,
                   const float* d_Xk, const float* d_Qk, const uint8_t* d_valid, int64_t n,
                   float sigma_ray, float sigma_dist, float huber_k, int max_iters,
                   float rel_error, float delta_norm, float* d_T_WCf_out, float* d_T_CkCf_out,
                   int* d_info, void* d_workspace, void* stream);

/* Frontend tracking glue around m3s_track_rays (FrameTracker2.track, tracker2.py:127-257,
 * use_calib False): replaces the reference's torch ops between matching and the pose solve
 * and after it.  X, C, Q: the pair outputs [2][n] (x3 for X; row 0 = frame, 1 = keyframe),
 * idx i64[n] / valid_match u8[n]: matching.match's result, kf_C f32[n], kf_N f32[1]: the
 * keyframe's accumulated confidence / update count.  workspace: m3s_glue_workspace_bytes(n),
 * 16-B aligned, shared by the pre / post calls of one frame.
 *   pre:  Xf = X[0][idx], Qk = sqrt(Q[0][idx] Q[1]), valid_opt (u8) as tracker2.py:130-193
 *   post: lost = match_frac < min_match_frac | info[1]; unless lost, X_canon / C / N of the
 *         keyframe take the weighted fusion with T_CkCf.act(X[1]) (frame.py:105-109);
 *         flags u8[2] = {new_kf, lost} (tracker2.py:246-257), fracs f32[3] = {match_frac,
 *         match_frac_k, unique_frac}. */
size_t m3s_glue_workspace_bytes(int64_t n);
int m3s_track_glue_pre(const float* d_X, const float* d_C, const float* d_Q, const int64_t* d_idx,
                       const uint8_t* d_valid_match, const float* d_kf_C, const float* d_kf_N,
                       int64_t n, float Q_conf, float C_conf, float* d_Xf, float* d_Qk,
                       uint8_t* d_valid_opt, void* d_workspace, void* stream);
int m3s_track_glue_post(const float* d_X, const float* d_C, const int64_t* d_idx,
                        const uint8_t* d_valid_match, const int* d_info, const float* d_T_CkCf,
                        int64_t n, float min_match_frac, float match_frac_thresh, float* d_kf_X,
                        float* d_kf_C, float* d_kf_N, uint8_t* d_flags, float* d_fracs,
                        void* d_workspace, void* stream);

/* Calibrated variant.  K f32[3,3] device; n points; img h,w; meas_k f32[n,3];
 * valid_meas_k u8[n]. */
int m3s_track_calib(const float* d_Twc_k, const float* d_Twc_f, const float* d_Xf,
                    const float* d_Qk, const uint8_t* d_valid, const float* d_meas_k,
                    const uint8_t* d_valid_meas_k, const float* d_K, int64_t n, int64_t h, int64_t w,
                    float sigma_pixel, float sigma_depth, float huber_k, float pixel_border,
                    float depth_eps, int max_iters, float rel_error, float delta_norm,
                    float* d_T_WCf_out, float* d_T_CkCf_out, int* d_info, void* d_workspace,
                    void* stream);

/* ------------------------------------------------------------------------- *
 * ViT / DPT building blocks (bf16 MFMA).  The reference runs these as PyTorch ops
 * (cuBLAS/cuDNN, fp32/TF32: croco/blocks.py, croco/dpt_block.py, d3r/heads/dpt_head.py,
 * mast3r/catmlp_dpt_head.py); they have no FFI in the reference, so this is the
 * native surface the host-side model (monst3r_slam_amd/model.py) drives.
 * Activations: bf16 row-major [rows][channels] (tokens, or NHWC pixels);
 * residual stream f32; weights bf16 [N][K] (torch Linear layout; convs repacked
 * [Cout][ky][kx][Cin]; ConvTranspose repacked [(a,b,Cout)][Cin]).
 * ------------------------------------------------------------------------- */
enum {
  M3S_EPI_BIAS = 1,       /* + bias[n] (f32)                                  */
  M3S_EPI_GELU = 2,       /* exact-erf GELU                                    */
  M3S_EPI_RELU = 4,       /* ReLU on the output                                */
  M3S_EPI_RES_F32 = 8,    /* + R[m][n] (f32 residual)                          */
  M3S_EPI_RES_BF16 = 16,  /* + R[m][n] (bf16 residual)                         */
  M3S_EPI_OUT_F32 = 32,   /* store f32 (default bf16)                          */
  M3S_PRO_RELU = 64,      /* ReLU applied to A while loading (conv prologue)   */
  M3S_EPI_CONVT = 128,    /* scatter rows/cols as ConvTranspose(k=s, stride=s) */
  M3S_EPI_ROPE = 256,     /* 2D RoPE on columns < rope_cols (head dim 64), after bias;
                             not combined with a residual or CONVT                   */
  M3S_EPI_DPT_OUT = 512,  /* DPT regression tail fused into a conv with N = 128 (one tile
                             spans the row): relu(acc + bias) · W4ᵀ + b4 (1x1, 128 → 4), then
                             reg_dense_depth / conf (d3r/heads/postprocess.py:10-58) written
                             to dpt_pts / dpt_conf; C is not written               */
  M3S_IN_FP8 = 1024,      /* A and B are OCP fp8 e4m3 (1 byte; K, lda, ldb, strides % 16
                             == 0; GEMM mode only): scaled-MFMA 32x32x64 path; the f32
                             accumulator is multiplied by col_scale[n] before the epilogue */
  M3S_EPI_OUT_FP8 = 2048, /* store C as OCP fp8 e4m3 (saturated to ±448)           */
  M3S_EPI_LN_STATS = 4096, /* producer of a LayerNorm input (the f32 residual stream; GEMM
                             mode, N % 128 == 0, f32 out): also stores a bf16 copy of C to
                             C2 and, per row and 128-column group, (mean, M2) of the stored
                             values to stats — the row statistics a LN_FOLD consumer needs */
  M3S_EPI_LN_FOLD = 8192  /* consumer: A is the bf16 copy of LayerNorm's INPUT x and B the
                             weight with gamma folded in (B[n][k] = W[n][k] gamma[k]); the
                             epilogue forms LN(x) W^T + b = rstd (acc - mean c1[n]) + c2[n]
                             with mean / rstd from the producer's stats (Chan's combination
                             of the groups, fixed order), c1 = ln_c1 (row sums of B) and
                             bias = c2 = b + W beta.  GEMM mode.  On e4m3 operands (IN_FP8,
                             ABI 0.5) A is the producer's shifted e4m3 copy (ln_shift) and
                             ln_c3 restores the shift before the fold                 */
};

typedef struct {
  const void* A; int64_t lda, strideA;     /* bf16 [M][lda]; per-batch element stride */
  const void* B; int64_t ldb, strideB;     /* bf16 [N][ldb]                         */
  void* C; int64_t ldc, strideC;           /* bf16 or f32 [M][ldc]                  */
  const float* bias; int64_t strideBias;   /* f32 [N] (or [Cout] for CONVT)          */
  const void* R; int64_t ldr, strideR;     /* residual [M][ldr]                     */
  int32_t M, N, K, batch;
  int32_t flags;                           /* OR of M3S_EPI_x / M3S_PRO_x bits       */
  int32_t mode;                            /* 0: GEMM; 1: implicit 3x3 conv, pad 1  */
  int32_t Hin, Win, Cin, Hout, Wout, stride; /* conv geometry (mode 1); K = 9*Cin   */
  int32_t ct_s, ct_cout, ct_gw;            /* CONVT: kernel=stride=s, Cout, grid w  */
  void* workspace; int64_t workspace_bytes; /* optional f32 split-K scratch (device) */
  int32_t split_k;                         /* 0 = auto (uses workspace if it pays)  */
  const float* rope_table;                 /* ROPE: m3s_vit_rope_table output        */
  int32_t rope_cols, rope_tokens;          /* ROPE: rotated columns; row m → token m % rope_tokens */
  int32_t weight_mod;                      /* >0: batch g reads B / bias of batch g % weight_mod
                                              (P problem groups sharing one weight stack) */
  const float* dpt_w4;                     /* DPT_OUT: f32 [heads][4][128] (head g % weight_mod) */
  const float* dpt_b4;                     /* DPT_OUT: f32 [heads][4]                  */
  float* dpt_pts;                          /* DPT_OUT: f32 [batch][M][3]               */
  float* dpt_conf;                         /* DPT_OUT: f32 [batch][M]                  */
  float dpt_conf_min;                      /* DPT_OUT: conf = conf_min + exp(c)        */
  const float* col_scale;                  /* IN_FP8: f32 [N] per weight batch (dequant of
                                              A·B: activation scale x weight row scale) */
  int64_t stride_col_scale;                /* IN_FP8: elements between batches (weight_mod) */
  void* C2;                                /* LN_STATS: bf16 copy of C (ldc / strideC)  */
  float* stats;                            /* LN_STATS out / LN_FOLD in: f32 [batch][M][groups][2]
                                              (mean, M2) per 128-column group of a row     */
  int32_t stats_groups;                    /* LN_FOLD: groups per row (LayerNorm dim / 128, ≤ 8) */
  int32_t a_batch_xor;                     /* LN_FOLD: batch g reads A and stats of g ^ this
                                              (the decoder's norm_y of the other side)     */
  const float* ln_c1;                      /* LN_FOLD: f32 [N] per weight batch (strideBias) */
  float ln_eps;                            /* LN_FOLD: LayerNorm eps                       */
  int32_t* tile_counters;                  /* split-K: i32 per (batch, output tile), all zero
                                              on entry and left zero (device; the caller
                                              zeroes it once; one per concurrent stream)   */
  int32_t tile_counters_len;               /* entries; split-K needs batch x tiles of them  */
  int32_t tile_hint;                       /* 0: the per-shape tuned table / heuristic; > 0: this
                                              tile configuration (vit_gemm_kern.h TileCfg) with
                                              split_k (0 → 1) — a caller that knows the launch
                                              shares the chip (the prefetched encoder) */
  /* ABI 0.5: the LayerNorm fold on e4m3 operands (fp8 mode) */
  const float* ln_c3;                      /* LN_FOLD + IN_FP8: f32 [N] per weight batch
                                              (strideBias) added to the dequantised accumulator
                                              before the fold: Σ_k shift[k] B[n][k] for an A
                                              copy written with ln_shift                    */
  const float* ln_shift;                   /* LN_STATS: null → C2 is the bf16 copy; else C2 is
                                              e4m3((C[m][n] − shift[n]) · ln_qscale[g]), shift
                                              f32 [N] per weight batch (strideBias)          */
  const float* ln_qscale;                  /* LN_STATS with ln_shift: f32 e4m3 scale per weight
                                              batch (device memory, > 0)                    */
} m3s_gemm_desc;

/* C = epilogue(A · Bᵀ), batched over desc->batch.  K % 8 == 0; conv: Cin % 32 == 0.
 * A, B 16-B aligned, lda/ldb/batch strides % 8 == 0; per-batch operand spans < 2 GiB.
 * With a workspace and tile counters, GEMMs whose tile grid cannot fill the chip (M = 768
 * tokens) split K over workgroups into f32 partials; the last split of each tile sums them
 * in split order (deterministic) and applies the epilogue — one launch.
 * ROPE (croco/pos_embed.py RoPE2D as applied in croco/blocks.py:64-66, 110-112) rotates
 * the q / k columns in the epilogue, replacing a separate pass over q and k. */
int m3s_vit_gemm(const m3s_gemm_desc* desc, void* stream);

/* RoPE2D cos/sin table for the GEMM epilogue: pos int64 [tokens][2] (y, x) →
 * table f32 [tokens][2][2][16] = {cos, sin}(pos[t][h] · base^(−i/16)), i < 16. */
int m3s_vit_rope_table(const int64_t* d_pos, int64_t tokens, float base, float* d_table,
                       void* stream);

/* LayerNorm over the last dim (eps), x f32/bf16 [rows][dim] → y (x_is_bf16 flag;
 * y_type 0 bf16, 1 f32, 2 OCP fp8 e4m3 saturated to ±448 — the A operand of the
 * M3S_IN_FP8 GEMMs); batch strides in elements.  dim ≤ 4096, dim % 4 == 0; gamma / beta
 * 16-byte aligned, stride_param % 4 == 0 (else M3S_ERR_INVALID_ARG).
 * param_mod > 0: batch b uses gamma/beta of batch b % param_mod.
 * Batch b of y normalises batch (b ^ x_batch_xor) of x: with x_batch_xor = 1 the
 * decoder's norm_y(other side) (croco/blocks.py:187) runs for both sides in one launch. */
int m3s_vit_layernorm(const void* d_x, int x_is_bf16, const float* d_gamma,
                      const float* d_beta, void* d_y, int y_type, int64_t rows, int64_t dim,
                      float eps, int64_t batch, int64_t stride_x, int64_t stride_y,
                      int64_t stride_param, int64_t param_mod, int x_batch_xor, void* stream);

/* Two LayerNorms of the same f32 rows in one pass (the decoder's norm1 of x and norm_y of
 * the other side, croco/blocks.py:184-187): y[b] = LN(x[b]; gamma/beta of b) and
 * y2[b ^ 1] = LN(x[b]; gamma2/beta2 of b ^ 1), both bf16 (y_fp8 = 0) or both e4m3
 * (y_fp8 = 1); batch even; param_mod and the parameter alignment as above. */
int m3s_vit_layernorm_dual(const float* d_x, const float* d_gamma, const float* d_beta,
                           void* d_y, const float* d_gamma2, const float* d_beta2, void* d_y2,
                           int y_fp8, int64_t rows, int64_t dim, float eps, int64_t batch,
                           int64_t stride_x, int64_t stride_y, int64_t stride_param,
                           int64_t param_mod, void* stream);

/* In-place 2-D RoPE (curope kernels.cu:17-82; pos_embed.py:106-158) on a bf16 view
 * t [B][S] rows of ld (head h at column h*64): dims [0,32) rotate by pos y, [32,64) by
 * pos x, pairs (i, i+16), angle = pos * base^(-i/16).  pos int64 [B][S][2] (y, x). */
int m3s_vit_rope(void* d_t, int64_t ld, int64_t stride, const int64_t* d_pos,
                 int64_t stride_pos, int64_t batch, int64_t S, int64_t heads, float base,
                 void* stream);

/* Multi-head attention, head dim 64 (croco/blocks.py:81-112 self, :132-169 cross):
 * o = softmax(q k^T / 8) v.  q [B][Sq] rows of ld_q bf16 (head h at column h*64), k,v
 * [B][Sk] rows of ld_kv; RoPE already applied (m3s_vit_rope).  o [B][Sq][ld_o]: bf16,
 * or OCP e4m3 bytes saturated to ±448 when o_fp8 (the fp8 output projection's A operand).
 * The pos/rope arguments are reserved (must be NULL/0).  With a device workspace (16-B
 * aligned, optional) a small (query tile x head x batch) grid is split along the keys
 * (flash-decoding): per-split unnormalised O, max and sum in f32, merged by a second
 * kernel; up to splits x B x heads x sq x 68 floats of workspace are used.
 * kv_batch_xor = 1 (B even): batch b attends to the k / v rows of batch b ^ 1 (the
 * decoder's cross-attention reading the other side's k / v from a fused projection). */
int m3s_vit_attention(const void* d_q, int64_t ld_q, int64_t stride_q, const void* d_k,
                      const void* d_v, int64_t ld_kv, int64_t stride_kv, const int64_t* d_qpos,
                      const int64_t* d_kpos, int64_t stride_pos, void* d_o, int64_t ld_o,
                      int64_t stride_o, int o_fp8, int64_t batch, int64_t heads, int64_t sq,
                      int64_t sk, float rope_base, void* d_workspace, int64_t workspace_bytes,
                      int kv_batch_xor, void* stream);

/* Patch-embed im2col: img f32 NCHW [B][3][H][W] → bf16 [B][(H/16)(W/16)][3*16*16]
 * with K ordered (c, ky, kx) like the conv weight [1024][3][16][16]. */
int m3s_vit_patchify(const float* d_img, void* d_out, int64_t batch, int64_t h, int64_t w,
                     void* stream);

/* Strided row copy (decoder input assembly, the local-feature concat): for o < outer,
 * i < inner, copy `rows` rows of row_bytes from src + o·src_outer + i·src_inner + src_base
 * (row stride src_row_stride) to dst + o·dst_outer + i·dst_inner + dst_base (row stride
 * dst_row_stride); every size, stride, base and pointer a multiple of 16 bytes. */
int m3s_copy_rows(const void* d_src, void* d_dst, int64_t rows, int64_t row_bytes,
                  int64_t src_row_stride, int64_t dst_row_stride, int64_t outer, int64_t inner,
                  int64_t src_outer, int64_t src_inner, int64_t src_base, int64_t dst_outer,
                  int64_t dst_inner, int64_t dst_base, void* stream);

/* Bilinear x2 upsample, align_corners=True (dpt_block.py:215-216), NHWC bf16
 * [B][h][w][C] → [B][oh][ow][C] (oh ≤ 2h, ow ≤ 2w: the DPT crop of dpt_head.py:57);
 * optional d_add [B][oh][ow][C] is added (fuses the fusion block's skip add). C % 8 == 0. */
int m3s_vit_upsample2x(const void* d_in, void* d_out, const void* d_add, int64_t batch,
                       int64_t h, int64_t w, int64_t c, int64_t oh, int64_t ow, void* stream);
/* The same upsample with an OCP e4m3 output of v * inv_scale (d_out: uint8 [b][oh][ow][c]):
 * the A operand of an fp8 implicit conv (C5 fp8 heads; the conv's per-column scales carry
 * 1 / inv_scale).  inv_scale must be finite and > 0.  (ABI 0.3) */
int m3s_vit_upsample2x_e4m3(const void* d_in, void* d_out, const void* d_add, int64_t batch,
                            int64_t h, int64_t w, int64_t c, int64_t oh, int64_t ow,
                            float inv_scale, void* stream);

/* DPT regression head tail, fused: t = relu(conv3x3 output) [B][P][128] bf16 is reduced
 * by the final 1x1 conv (128 → 4, per-head W4 f32 [B][4][128], b4 [B][4]) and post-processed
 * (d3r/heads/postprocess.py:10-58): pts3d = xyz/max(|xyz|,1e-8) * expm1(|xyz|),
 * conf = conf_min + exp(c).  pts3d f32 [P][3], conf f32 [P].
 * param_mod > 0: batch b uses W4/b4 of head b % param_mod. */
int m3s_vit_dpt_out(const void* d_t, const float* d_w4, const float* d_b4, float* d_pts3d,
                    float* d_conf, int64_t pixels, float conf_min, int64_t batch,
                    int64_t stride_t, int64_t stride_out, int64_t param_mod, void* stream);

/* MASt3R local-feature tail (catmlp_dpt_head.py:25-39,84-96): feats bf16 or f32
 * [B][S][25*256] (fc2 output, per token) → pixel_shuffle(16) → desc = normalise(ch 0..23)
 * as f32 [B][H][W][24] and f16 [B][H][W][24], desc_conf = 0 + exp(ch 24) f32 [B][H][W].
 * gw = W/16 token-grid width. */
int m3s_vit_local_features(const float* d_feats, float* d_desc, uint16_t* d_desc_f16,
                           float* d_desc_conf, int64_t batch, int64_t h, int64_t w,
                           void* stream);

/* ------------------------------------------------------------------------- *
 * Dynamic-mask arithmetic (MonST3R dynamic-object filtering).
 * ------------------------------------------------------------------------- */

/* Error map + threshold of get_dynamic_mask (mast3r_slam/monst3r_utils.py:625-637):
 * err = |flow - ego_flow[:2]| per pixel, norm = (err - min)/(max - min) (0 if max == min),
 * mask = norm > threshold.  flow, ego_flow f32 [2][n] (channel-major, n = H*W; only the
 * first 2 ego channels are read) → mask u8 [n].  workspace: (n + 64) floats (device). */
int m3s_flow_error_mask(const float* d_flow, const float* d_ego_flow, int64_t n,
                        float threshold, uint8_t* d_mask, float* d_workspace, void* stream);

/* Ego-motion flow of get_dynamic_mask (monst3r_utils.py:566-614): pixel (x, y) of frame i
 * at depth pts[p].z (the mono decode's res_i pts3d, f32 [h][w][3]; inv_depth =
 * 1/(z + 1e-6) as :586) maps to K_j (R_ji d K_i^-1 [x y 1]^T + t_ji) in frame j.
 * params (device, 30 f32): R_ji row-major 9, t_ji 3, K_j 9, K_i^-1 9.  Out ego f32 [3][h*w]:
 * flow x, flow y (projection - pixel), valid (projected depth > 1e-6; flow 0 otherwise).
 * DepthBasedWarping itself is absent from the reference checkout: restated, parity
 * unpinned. */
int m3s_ego_flow(const float* d_pts, const float* d_params, int64_t h, int64_t w,
                 float* d_ego, void* stream);

/* apply_dynamic_mask_to_pointmaps (monst3r_utils.py:300-341), in place: where mask[p]
 * (u8 [hw], shared by the batch) C[b][p] = value, Q[b][p] = value (Q optional) and
 * D[b][p][:] = 0 (D optional, f32 or f16 [b][hw][fdim]).  The reference zeroes D whenever
 * it is given, whatever zero_descriptors says (:333-335); the flag is accepted and ignored. */
int m3s_apply_dynamic_mask(const uint8_t* d_mask, float* d_C, float* d_Q, void* d_D,
                           int D_is_f16, int64_t batch, int64_t hw, int64_t fdim,
                           float value, int zero_descriptors, void* stream);

/* ---- Keyframe retrieval / loop-closure candidates (RetrievalDatabase, 8(f) row 3) --------
 * Replaces the per-keyframe work of mast3r_slam/retrieval_database.py:25-166 (prep_features,
 * quantize_custom, accumulate_scores / aggregate_image, add_to_ivf_custom, ivf.search) and
 * the Cython asmk/cython/hamming.pyx it calls.  Host bookkeeping (kf_counter, kf_ids, the
 * inverted file's growth) stays in monst3r_slam_amd/retrieval.py.                          */

/* Y[M][N] = (X[rows[i]][:K] - mu) W + bias (fp32; W [K][N] row-major, mu [K] and bias [N]
 * optional, rows optional = identity).  X is f32 or bf16 with row stride ldx.  Whitener
 * (mast3r/retrieval/model.py:55-76, fp64 in the reference) and the projector Linear.
 * K, N and ldx multiples of 4 (vector loads); f32 MFMA (exact fp32 products). */
int m3s_retr_affine(const void* d_X, int X_is_bf16, int64_t ldx, const int64_t* d_rows,
                    const float* d_mu, const float* d_W, const float* d_bias, int64_t M,
                    int64_t N, int64_t K, float* d_Y, void* stream);

/* Per-row L2 norm (squared = 0; the 'l2norm' attention, model.py:133) or squared norm. */
int m3s_retr_rownorm(const float* d_Y, int64_t M, int64_t N, int squared, float* d_out,
                     void* stream);

/* Sorted top-k of n <= 4096 keys (f32 or f64): largest first (largest = 1) or smallest
 * first, ties to the lower index.  torch.topk as used by how_select_local (model.py:101)
 * and RetrievalDatabase.update (retrieval_database.py:63).  d_vals optional. */
int m3s_topk_select(const void* d_keys, int keys_f64, int64_t n, int64_t k, int largest,
                    int64_t* d_idx, void* d_vals, void* stream);

/* quantize_custom (retrieval_database.py:96-105): d = (|q|^2 + |c|^2) - 2 q.c against the
 * codebook C [ncent][D] f32 (|c|^2 precomputed: m3s_retr_rownorm squared), the k <= 8
 * smallest per query row, ascending (ties: lower index) -> codes i32 [M][k], dists f32
 * (optional).  D % 32 == 0.  workspace: m3s_retr_quantize_workspace_bytes(M, ncent, k). */
size_t m3s_retr_quantize_workspace_bytes(int64_t M, int64_t ncent, int64_t k);
int m3s_retr_quantize(const float* d_Q, const float* d_qnorm2, int64_t M, const float* d_C,
                      const float* d_cnorm2, int64_t ncent, int64_t D, int64_t k,
                      int32_t* d_codes, float* d_dists, void* d_workspace, void* stream);

/* ASMKKernel.aggregate_image + binarize_and_pack_2D (asmk/kernel.py:26-39,
 * hamming.pyx:77-110): unique words of codes [n][k] (sorted, as np.unique) -> d_words
 * (capacity n*k) and *d_count (device); per word the index-order sum of des[i] - C[word]
 * over descriptors holding the word, packed as D/32 u32 with element 0 in bit 31
 * -> d_packed [n*k][D/32].  d_flags: i32 [ncent] zeroed once by the caller, left zeroed.
 * n <= 16384, D % 32 == 0. */
int m3s_asmk_aggregate(const float* d_des, int64_t n, int64_t D, const int32_t* d_codes,
                       int64_t k, const float* d_C, int64_t ncent, int32_t* d_flags,
                       int32_t* d_words, int32_t* d_count, uint32_t* d_packed, void* stream);

/* IVF.search with the binary ASMK similarity (inverted_file.py:186-208, kernel.py:56-68,
 * functional.py:96-100; use_idf = False): the inverted file is flat and image-major (image g
 * owns entries [img_start[g], img_start[g+1]) in ascending word order, as add() receives
 * them).  scores f64 [n_images] = sum over entries whose word the query holds of
 * f32(sim^alpha / sqrt(entries of g)) where sim = 1 - 2 hamming/D >= threshold, divided by
 * sqrt(#query words).  d_word_map: i32 [ncent] all -1 (caller initialises once; restored). */
int m3s_ivf_search(const uint32_t* d_qpacked, const int32_t* d_qwords, const int32_t* d_qcount,
                   int64_t max_qwords, const uint32_t* d_db_packed, const int32_t* d_db_words,
                   const int32_t* d_img_start, int64_t n_images, int64_t D, float alpha,
                   float similarity_threshold, int32_t* d_word_map, double* d_scores,
                   void* stream);

/* ------------------------------------------------------------------------- *
 * Streaming tracking-loop plumbing (configs[2], the main loop main_monster_slam.py:247-332
 * with FrameTracker2.track, tracker2.py:70-270), graph-replayable: the frame index
 * d_frame and the keyframe's frame index d_kf_frame live on the device.
 *
 * m3s_seq_gather: frame min(*d_frame + offset, nframes-1) of a staged sequence
 *   (frame_bytes per frame, 16-B multiple, 16-B aligned) -> d_dst.
 * m3s_seq_pair_outputs: the synthetic scene's stand-in for the pair inference outputs of
 *   monst3r_asymmetric_inference (monst3r_utils.py:255-297) — trained weights are absent,
 *   random weights carry no geometry.  Staged per frame f: Xcam f32[F][n][3] (own camera),
 *   C_own/C_other/Q_own/Q_other f32[F][n], D16 f16[F][n][24], T_gt f32[F][8] (camera to
 *   world).  Writes X f32[2][n][3] = {Xcam[t], T_gt[t]^-1 T_gt[j] Xcam[j]},
 *   C = {C_own[t], C_other[t]}, Q likewise, D16 f16[2][n][24] = {D16[t], D16[j]} with
 *   t = *d_frame, j = *d_kf_frame.
 * m3s_seq_advance: after the tracking glue (flags u8[2] = {new_kf, lost}, info i32[4] of
 *   m3s_track_rays, T_WCf f32[8]): log row t (i32[8] = iterations, new_kf, lost,
 *   keyframe frame, Cholesky failure, recovered iterations; f32[8] T_WCf) if t < nlog;
 *   T_prev = T_WCf unless lost; on new_kf the frame becomes the keyframe
 *   (keyframes.append(frame), main_monster_slam.py:319-321): kf_X = Xff f32[n][3],
 *   kf_C = Cff f32[n], kf_N = 1, kf_T = T_WCf, kf_feat = feat_i (feat_bytes), idx_f2k =
 *   identity (reset_idx_f2k, tracker2.py:256-257), *d_kf_frame = t; then *d_frame = t + 1.
 * ------------------------------------------------------------------------- */
int m3s_seq_gather(const void* d_src, int64_t frame_bytes, const int* d_frame, int offset,
                   int nframes, void* d_dst, void* stream);

int m3s_seq_pair_outputs(const float* d_Xcam, const float* d_C_own, const float* d_C_other,
                         const float* d_Q_own, const float* d_Q_other, const void* d_D16,
                         const float* d_T_gt, const int* d_frame, const int* d_kf_frame,
                         int nframes, int64_t n, float* d_X, float* d_C, void* d_D16_out,
                         float* d_Q, void* stream);

int m3s_seq_advance(const uint8_t* d_flags, const int* d_info, const float* d_T_WCf,
                    const float* d_Xff, const float* d_Cff, const void* d_feat_i,
                    int64_t feat_bytes, int64_t n, float* d_kf_X, float* d_kf_C, float* d_kf_N,
                    float* d_kf_T, void* d_kf_feat, int64_t* d_idx_f2k, float* d_T_prev,
                    int* d_frame, int* d_kf_frame, int* d_log_i, float* d_log_T, int nlog,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MONST3R_SLAM_AMD_H */
