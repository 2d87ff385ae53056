// Batched bf16 MFMA GEMM with fused epilogues for the ViT / DPT path (gfx950).
//
//   C[g] = epi(A[g] · B[g]^T)       A [M][K] (or implicit 3x3-conv rows of an NHWC image),
//                                   B [N][K] weights (K contiguous: torch Linear layout)
//
// Main loop (cdna_hip_programming.md §5 "Pipelining across barriers"):
//  * operands go HBM → LDS with 16-B LDS-DMA buffer loads (buffer_load_dwordx4 … lds), a
//    ring of STAGES K-tiles in one __shared__ array; tile t+STAGES-1 is issued right after
//    the barrier that retires tile t, so STAGES-1 tiles are in flight during each MFMA
//    phase; counted `s_waitcnt vmcnt(N)` + raw s_barrier (never __syncthreads, whose fence
//    would drain the DMA queue).
//  * out-of-range rows, K tails and conv zero padding are buffer out-of-bounds reads
//    (voffset ≥ num_records → the hardware writes zeros): no branches around loads.
//  * LDS image is lane-linear per wave instruction (what the DMA writes); bank conflicts of
//    the ds_read_b128 fragment reads are removed by XOR-swizzling the 16-B chunk index with
//    the row (applied to the per-lane GLOBAL address at load time and to the read address).
//  * 4 waves, each a grid of 32x32 v_mfma_f32_32x32x16_bf16 accumulators.
// Epilogue: accumulators → LDS f32 tile → row-contiguous 8-column vectors per thread:
//   bias, GELU(erf), 2D RoPE (croco RoPE2D, via a per-token cos/sin table), f32/bf16
//   residual, ReLU, f32/bf16 store, ConvTranspose(k=s) scatter — 16-B loads/stores.
// Split-K (tile grids that cannot fill 256 CUs): batch x splits groups of workgroups; each
//   writes its f32 partial tile to a workspace and bumps the tile's counter (agent-scope
//   release); the LAST split of a tile (acquire) sums the partials in split order — fixed,
//   so deterministic whichever workgroup finishes last — and runs the normal epilogue (any
//   flag set, LayerNorm fold included).  One launch; counters return to zero.
// Implicit conv (MODE 1, MODE 2 = ReLU on A): per K-tile the tap (ky, kx) and channel
//   offset are block-uniform (Cin % BK == 0); ReLU is applied to the A fragments in
//   registers (v_pk_max_i16 on the bf16 bits).
// XCD-aware bijective tile order (cdna_hip_programming.md T1).
#include <stdlib.h>
#include <algorithm>
#include "vit_gemm_kern.h"

// the launchers are instantiated in vit_gemm_i*.hip (parallel compilation)
#ifndef M3S_GEMM_STAMPS
namespace m3s_gemm {
extern template int launch<128, 128, 64, 2, 2, 3, 1>(Args&, int, hipStream_t);
extern template int launch<128, 128, 32, 2, 2, 4, 2>(Args&, int, hipStream_t);
extern template int launch<256, 128, 64, 2, 2, 3, 1>(Args&, int, hipStream_t);
extern template int launch<256, 128, 64, 4, 2, 3, 1>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 2, 2, 2, 2>(Args&, int, hipStream_t);
extern template int launch<96, 128, 64, 1, 4, 3, 1>(Args&, int, hipStream_t);
extern template int launch<96, 128, 64, 1, 4, 2, 2>(Args&, int, hipStream_t);
extern template int launch<64, 128, 64, 2, 2, 6, 1>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 2, 2, 4, 1>(Args&, int, hipStream_t);
extern template int launch<64, 128, 64, 2, 2, 3, 2>(Args&, int, hipStream_t);
extern template int launch<64, 128, 64, 2, 2, 3, 2, true>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 4, 2, 3, 1, true>(Args&, int, hipStream_t);
extern template int launch<256, 128, 64, 4, 2, 3, 1, true>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 2, 2, 2, 2, true>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 2, 2, 3, 1, true>(Args&, int, hipStream_t);
extern template int launch<128, 128, 64, 4, 2, 3, 1>(Args&, int, hipStream_t);
extern template int launch<256, 256, 64, 2, 4, 2, 1>(Args&, int, hipStream_t);
extern template int launch_pp<0>(Args&, int, hipStream_t);
extern template int launch_pp<1>(Args&, int, hipStream_t);
extern template int launch_pp<2>(Args&, int, hipStream_t);
extern template int launch_pp<0, 192>(Args&, int, hipStream_t);
extern template int launch_pp<1, 192>(Args&, int, hipStream_t);
extern template int launch_pp<2, 192>(Args&, int, hipStream_t);
}  // namespace m3s_gemm
#endif

namespace {
using namespace m3s_gemm;

// Per-shape launch choices measured on MI355X (tools/gemm_autotune.py): exact match on the
// descriptor's (M, N, K, batch, flags, mode); everything else takes the heuristic below.
struct TunedShape {
  int M, N, K, batch, flags, mode, cfg, splits, fused;
};
const TunedShape kTuned[] = {
#include "gemm_table.inc"
    {0, 0, 0, 0, 0, 0, 0, 0, 0}};

const TunedShape* tuned_for(const m3s_gemm_desc* d) {
  static const bool off = getenv("M3S_GEMM_NO_TABLE") != nullptr;
  static const int maxcfg = getenv("M3S_GEMM_TABLE_MAXCFG") ? atoi(getenv("M3S_GEMM_TABLE_MAXCFG"))
                                                            : 99;  // A/B knob
  if (off) return nullptr;
  for (const TunedShape& t : kTuned)
    if (t.cfg <= maxcfg && t.M == d->M && t.N == d->N && t.K == d->K && t.batch == d->batch && t.flags == d->flags &&
        t.mode == d->mode)
      return &t;
  return nullptr;
}

int forced_tile() {
  const char* s = getenv("M3S_GEMM_TILE");  // tuning override (tools/gemm_bench.py)
  return s ? atoi(s) : 0;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

#ifdef M3S_GEMM_STAMPS
extern "C" int m3s_debug_set_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(m3s_gemm::g_m3s_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int m3s_vit_gemm(const m3s_gemm_desc* d, void* stream) {
  if (!d || !d->A || !d->B || !d->C) return M3S_ERR_INVALID_ARG;
  if (d->M <= 0 || d->N <= 0 || d->K <= 0 || d->batch <= 0) return M3S_ERR_INVALID_ARG;
  if (d->K % 8 != 0) return M3S_ERR_INVALID_ARG;
  if (d->mode == 1 && (d->Cin % 32 != 0 || d->K != 9 * d->Cin)) return M3S_ERR_INVALID_ARG;
  if ((d->flags & (M3S_EPI_RES_F32 | M3S_EPI_RES_BF16)) && !d->R) return M3S_ERR_INVALID_ARG;
  if ((d->flags & M3S_EPI_CONVT) && (d->ct_s <= 0 || d->ct_cout <= 0 || d->ct_gw <= 0))
    return M3S_ERR_INVALID_ARG;
  if ((d->flags & M3S_EPI_ROPE) &&
      (!d->rope_table || d->rope_tokens <= 0 ||
       (d->flags & (M3S_EPI_CONVT | M3S_EPI_RES_F32 | M3S_EPI_RES_BF16)) ||
       d->rope_cols % 64 != 0 || !aligned16(d->rope_table)))
    return M3S_ERR_INVALID_ARG;
  if (!aligned16(d->A) || !aligned16(d->B)) return M3S_ERR_INVALID_ARG;
  if ((d->mode == 0 && d->lda % 8) || d->ldb % 8 || d->strideA % 8 || d->strideB % 8)
    return M3S_ERR_INVALID_ARG;
  if (d->batch > 65535) return M3S_ERR_TOO_LARGE;
  const bool f8 = d->flags & M3S_IN_FP8;
  // fp8 implicit conv (mode 1): e4m3 NHWC input whose channel count fills whole K-tiles in
  // 2-byte units (Cin % 128); no ReLU prologue (the e4m3 fragments are not rectified)
  if (f8 && (d->mode > 1 || (d->mode == 0 && d->lda % 16) || d->K % 16 || d->ldb % 16 ||
             d->strideA % 16 || d->strideB % 16 || !d->col_scale ||
             (d->flags & (M3S_EPI_CONVT | M3S_PRO_RELU)) || (d->mode == 1 && d->Cin % 128)))
    return M3S_ERR_INVALID_ARG;
  if ((d->flags & M3S_EPI_OUT_FP8) && (d->flags & M3S_EPI_OUT_F32)) return M3S_ERR_INVALID_ARG;
  // fp8 operands are addressed in 2-byte units (the bf16 kernel's byte layout, §F8)
  const int64_t eK = f8 ? d->K / 2 : d->K, elda = f8 ? d->lda / 2 : d->lda;
  const int64_t eldb = f8 ? d->ldb / 2 : d->ldb;
  // buffer addressing: each operand's per-batch span must fit a 31-bit byte offset
  const int64_t spanA = d->mode == 0 ? ((int64_t)(d->M - 1) * elda + eK) * 2
                                     : (int64_t)d->Hin * d->Win * (f8 ? d->Cin / 2 : d->Cin) * 2;
  const int64_t spanB = ((int64_t)(d->N - 1) * eldb + eK) * 2;
  if (spanA >= NUM_RECORDS || spanB >= NUM_RECORDS) return M3S_ERR_TOO_LARGE;
  Args a;
  a.A = reinterpret_cast<const bf16_t*>(d->A);
  a.lda = d->lda;
  a.sA = d->strideA;
  a.B = reinterpret_cast<const bf16_t*>(d->B);
  a.ldb = d->ldb;
  a.sB = d->strideB;
  a.C = d->C;
  a.ldc = d->ldc;
  a.sC = d->strideC;
  a.bias = d->bias;
  a.sBias = d->strideBias;
  a.R = d->R;
  a.ldr = d->ldr;
  a.sR = d->strideR;
  a.M = d->M;
  a.N = d->N;
  a.K = d->K;
  a.flags = d->flags;
  a.mode = d->mode;
  a.Hin = d->Hin;
  a.Win = d->Win;
  a.Cin = d->Cin;
  a.Hout = d->Hout;
  a.Wout = d->Wout;
  a.stride = d->stride;
  a.ct_s = d->ct_s;
  a.ct_cout = d->ct_cout;
  a.ct_gw = d->ct_gw;
  a.splits = 1;
  a.ws = reinterpret_cast<float*>(d->workspace);
  a.cnt = d->tile_counters;
  a.rope_tab = d->rope_table;
  a.rope_cols = d->rope_cols;
  a.rope_tokens = d->rope_tokens;
  a.wmod = d->weight_mod > 0 ? d->weight_mod : 0;
  a.dpt_w4 = d->dpt_w4;
  a.dpt_b4 = d->dpt_b4;
  a.dpt_pts = d->dpt_pts;
  a.dpt_conf = d->dpt_conf;
  a.dpt_conf_min = d->dpt_conf_min;
  a.cscale = d->col_scale;
  a.sCscale = d->stride_col_scale;
  a.C2 = reinterpret_cast<bf16_t*>(d->C2);
  a.stats = d->stats;
  a.a_xor = 0;
  a.ln_c1 = d->ln_c1;
  a.ln_eps = d->ln_eps;
  a.ln_groups = d->stats_groups;
  a.ln_c3 = d->ln_c3;
  a.ln_shift = d->ln_shift;
  a.ln_qscale = d->ln_qscale;
  const bool ln_stats = d->flags & M3S_EPI_LN_STATS, ln_fold = d->flags & M3S_EPI_LN_FOLD;
  if (ln_stats || ln_fold) {
    // GEMM mode, biased, 128-column groups, 16-B aligned row vectors (bf16 or e4m3 operands)
    if (d->mode != 0 || !d->stats || !d->bias || !(d->flags & M3S_EPI_BIAS) ||
        (d->flags & M3S_EPI_CONVT) || (ln_stats && (d->flags & M3S_EPI_OUT_FP8)) ||
        !aligned16(d->stats))
      return M3S_ERR_INVALID_ARG;
  }
  if (ln_stats && (d->N % 128 || !(d->flags & M3S_EPI_OUT_F32) || !d->C2 || !aligned16(d->C2) ||
                   (d->flags & (M3S_EPI_GELU | M3S_EPI_ROPE | M3S_EPI_RELU))))
    return M3S_ERR_INVALID_ARG;
  // the shifted e4m3 copy (fp8 consumer) / the consumer's shift term: fp8 fold only
  if (d->ln_shift && (!ln_stats || !aligned16(d->ln_shift) || !d->ln_qscale ||
                      d->strideBias % 4))
    return M3S_ERR_INVALID_ARG;
  if (d->ln_c3 && (!ln_fold || !f8 || !aligned16(d->ln_c3)))
    return M3S_ERR_INVALID_ARG;
  if (!ln_stats) a.ln_shift = nullptr;
  if (!ln_fold) a.ln_c3 = nullptr;
  if (ln_fold) {
    if (d->K % 128 || d->K / 128 != d->stats_groups || d->stats_groups > 8 || !d->ln_c1 ||
        !aligned16(d->ln_c1) || d->a_batch_xor < 0 || d->a_batch_xor > 1 ||
        (d->a_batch_xor && d->batch % 2) || (d->flags & (M3S_EPI_RES_F32 | M3S_EPI_RES_BF16)) ||
        !(d->ln_eps > 0.f))
      return M3S_ERR_INVALID_ARG;
    a.a_xor = d->a_batch_xor;
  }
  if (f8) {
    a.K = (int)eK;
    a.lda = elda;
    a.ldb = eldb;
    a.sA = d->strideA / 2;
    a.sB = d->strideB / 2;
    a.Cin = d->Cin / 2;
  }
  const bool out32 = d->flags & M3S_EPI_OUT_F32;
  const bool has_bias = d->bias && (d->flags & M3S_EPI_BIAS);
  a.vec = d->N % 8 == 0 && d->ldc % 8 == 0 && d->strideC % 8 == 0 && aligned16(d->C) &&
          (!(d->flags & M3S_EPI_CONVT) || d->ct_cout % 8 == 0) &&
          (!has_bias || (aligned16(d->bias) && d->strideBias % 4 == 0)) &&
          (!d->R || (d->ldr % 8 == 0 && d->strideR % 8 == 0 && aligned16(d->R)));
  (void)out32;
  if ((d->flags & M3S_EPI_ROPE) && !a.vec) return M3S_ERR_INVALID_ARG;
  if ((ln_stats || ln_fold) && !a.vec) return M3S_ERR_INVALID_ARG;
  if (d->flags & M3S_EPI_DPT_OUT) {
    // compiled only as the conv variant BIAS? | RELU | DPT_OUT on the 8-wide vector path
    const int rest = d->flags & ~(M3S_EPI_DPT_OUT | M3S_EPI_RELU | M3S_EPI_BIAS | M3S_IN_FP8);
    if (d->mode != 1 || d->N != 128 || rest != 0 || !(d->flags & M3S_EPI_RELU) || !a.vec ||
        !d->dpt_w4 || !d->dpt_b4 || !d->dpt_pts || !d->dpt_conf)
      return M3S_ERR_INVALID_ARG;
  }
  // the step-timeline slot (if armed) is taken only once every check has passed, so a
  // rejected launch never holds a slot that no kernel stamps
  a.tl = m3s_timeline_take(d->mode != 0 ? M3S_TL_CONV : M3S_TL_GEMM,
                           2.0 * d->M * d->N * d->K * d->batch, d->M, d->N, d->K, d->batch);
  hipStream_t s = m3s_stream(stream);

  // Tile choice (measured on the pair shapes, tools/gemm_tune.py): 128x128 tiles (one
  // workgroup per CU, K split while the grid stays within one wave of 256 CUs) unless the
  // grid is tiny, K is short, or a large grid with short K favours 64x128 at 2/CU; convs
  // 64x128, or 256x128 once the grid has several waves of workgroups.
  const bool conv = d->mode == 1;
  const int64_t tiles128 = (int64_t)((d->M + 127) / 128) * ((d->N + 127) / 128) * d->batch;
  const int nk = (int)((eK + 63) / 64);     // K-tiles of 128 bytes per row
  int cfg = forced_tile();
  const bool hinted = cfg == 0 && d->tile_hint > 0;  // the caller's choice (header)
  if (hinted) cfg = d->tile_hint;
  const TunedShape* tuned = (cfg == 0 && !getenv("M3S_GEMM_SPLITS")) ? tuned_for(d) : nullptr;
  if (tuned) cfg = tuned->cfg;
  if (cfg == 0 && f8) {
    // fp8 (tools/fp8_tune.py, S = 768 / 1024 shapes): a K-tile holds 128 e4m3 values, so
    // the short-K latency regime comes sooner; 64x128 tiles at 2/CU win below ~1.5 waves
    // of 128^2 tiles, 2 x 128^2 per CU above (1.96 PFLOP/s on 4096^3)
    cfg = tiles128 >= 400 ? T128O2 : T64;
  } else if (cfg == 0 && !conv && eK >= 512 &&
             (int64_t)((d->M + 255) / 256) * ((d->N + 255) / 256) * d->batch >= 256 &&
             !(d->flags & (M3S_EPI_DPT_OUT | M3S_EPI_CONVT | M3S_EPI_OUT_FP8))) {
    // a GEMM with at least a full wave of 256^2 tiles and K >= 512 that the table does not
    // name: the ping-pong tile (tools/gemm_pp_bench.py, r06_pp_orders.txt: 4096^3 1083 ->
    // 1431 TF/s, 8192^3 892 -> 1511 TF/s; every model shape of that size is in the table)
    cfg = T256PP;
  } else if (cfg == 0) {
    // measured on the pair shapes (tools/gemm_tune.py): 2 x 128^2 blocks per CU win for
    // wide convs with several waves of tiles, for one-to-two waves of short-K GEMM tiles,
    // and for large square-ish GEMMs
    // (2 x 128^2 per CU beat 256x128 on the 128-channel head convs too: head.2 + DPT tail
    // 348 → 311 us, tools/gemm_depth.py conv sweep)
    if (conv) cfg = tiles128 < 1536 ? T64 : T128O2;
    else if (nk >= 32) cfg = tiles128 >= 1024 ? T128O2 : T128;
    else if (tiles128 < 64 || nk < 8 || (tiles128 > 512 && nk < 16)) cfg = T64;
    // under one wave of 128^2 tiles with K ≤ 1024 (the encoder's qkv / fc1, the decoder's
    // N = 768 projections): 64x128 tiles spread the grid over more CUs (graph-replayed
    // sweep, tools/gemm_depth.py: enc qkv 18.4 → 15.1 us, enc fc1 18.9 → 16.2 us)
    else if (tiles128 < 256 && nk <= 16) cfg = T64;
    else if (tiles128 >= 256 && tiles128 <= 512 && nk <= 16) cfg = T128O2;
    else cfg = T128;
    // (96-row tiles, 768 tokens = 8 bands, measured faster launch by launch but slower in
    // the pipelined step: 182 vs 184.6 frames/s, DESIGN §2 — reachable by tile hint only)
  }
  if (cfg < 1 || cfg > 16 || cfg == 4 || cfg == 5) cfg = T128;
  if (conv && (cfg == T64D || cfg == T128D)) cfg = T64;
  if (conv && d->Cin % 64 != 0) cfg = T128K32;  // tap-uniform K-tiles need Cin % BK == 0
  if (!conv && cfg == T128K32) cfg = T128;
  if (conv && d->Cin % 64 == 0 && cfg == T128K32) cfg = T128;
  int splits = d->split_k;
  if (tuned && splits <= 0) splits = tuned->splits;
  if (const char* e = getenv("M3S_GEMM_SPLITS")) splits = atoi(e);  // tuning override
  if (splits <= 0) {
    splits = 1;
    if (!hinted && !conv && (cfg == T128 || cfg == T128O2))
      while (tiles128 * splits * 2 <= 256 && nk / (splits * 2) >= 8) splits *= 2;
    // the small DPT levels (24x32, 12x16 convs: 24-96 tiles of 64x128 with K = 2304-6912)
    // split K while the grid stays within one round of 2 blocks per CU
    if (!hinted && conv && cfg == T64 && !(d->flags & M3S_EPI_DPT_OUT)) {
      const int64_t tiles64 = (int64_t)((d->M + 63) / 64) * ((d->N + 127) / 128) * d->batch;
      while (tiles64 * splits * 2 <= 512 && nk / (splits * 2) >= 8) splits *= 2;
    }
  }
  // fused split-K: 128^2 GEMM tiles or 64x128 GEMM / conv tiles, a workspace for the f32
  // partials and one zeroed counter per (batch, tile)
  const int bm = (cfg == T64 || cfg == T64D) ? 64
                 : (cfg == T256 || cfg == T256W8 || cfg == T256SQ || cfg == T256PP) ? 256
                 : cfg == T192PP ? 192 : 128;
  const int64_t tiles_cfg = (int64_t)((d->M + bm - 1) / bm) * ((d->N + 127) / 128) * d->batch;
  const bool split_cfg = (!conv && (cfg == T128 || cfg == T128O2 || cfg == T64 || cfg == T64D ||
                                    cfg == T128D || cfg == T128W8 || cfg == T256 ||
                                    cfg == T256W8)) ||
                         (conv && cfg == T64);
  // fused (last split reduces the tile on its CU: one launch, but that CU streams all the
  // partials) vs a separate reduce kernel spread over the chip; the LayerNorm-fold epilogue
  // needs the fused path (the reduce kernel has no fold)
  int fused = ln_fold ? 1 : (tuned ? tuned->fused : 0);
  if (const char* e = getenv("M3S_GEMM_FUSED")) fused = atoi(e) != 0 || ln_fold;  // tuning
  // (fp8: GEMM mode; the e4m3 tile set T64 / T128O2 / T128W8 / T256W8 / T128 all split)
  const bool can_split = split_cfg && !(f8 && conv) &&
                         !(d->flags & (M3S_EPI_CONVT | M3S_EPI_DPT_OUT)) &&
                         d->workspace &&
                         (!fused || (d->tile_counters && tiles_cfg <= (int64_t)d->tile_counters_len)) &&
                         (int64_t)splits * d->batch * d->M * d->N * 4 <= d->workspace_bytes;
  a.fused = fused;
  if (splits > 1 && can_split) a.splits = splits;
  if (f8) {
    switch (cfg) {
      case T64: return launch<64, 128, 64, 2, 2, 3, 2, true>(a, d->batch, s);
      case T128O2: return launch<128, 128, 64, 2, 2, 2, 2, true>(a, d->batch, s);
      case T128W8: return launch<128, 128, 64, 4, 2, 3, 1, true>(a, d->batch, s);
      case T256W8: return launch<256, 128, 64, 4, 2, 3, 1, true>(a, d->batch, s);
      default: return launch<128, 128, 64, 2, 2, 3, 1, true>(a, d->batch, s);
    }
  }
  switch (cfg) {
    case T128: return launch<128, 128, 64, 2, 2, 3, 1>(a, d->batch, s);
    case T128K32: return launch<128, 128, 32, 2, 2, 4, 2>(a, d->batch, s);
    case T256: return launch<256, 128, 64, 2, 2, 3, 1>(a, d->batch, s);
    case T128O2: return launch<128, 128, 64, 2, 2, 2, 2>(a, d->batch, s);
    // 96 x 128 tiles (waves 1 x 4, each 96 x 32): 768-token problems tile to 8 bands
    case T96: return launch<96, 128, 64, 1, 4, 3, 1>(a, d->batch, s);
    case T96O2: return launch<96, 128, 64, 1, 4, 2, 2>(a, d->batch, s);
    case T64D: return launch<64, 128, 64, 2, 2, 6, 1>(a, d->batch, s);
    case T128D: return launch<128, 128, 64, 2, 2, 4, 1>(a, d->batch, s);
    case T128W8: return launch<128, 128, 64, 4, 2, 3, 1>(a, d->batch, s);
    case T256W8: return launch<256, 128, 64, 4, 2, 3, 1>(a, d->batch, s);
    // 256x256: unsplit only (two-pass epilogue), no DPT tail (128-channel rows); the RoPE
    // and the run-time-flag epilogues spill at 256 VGPRs (-Rpass-analysis) → 256x128
    case T256SQ:
      if (a.splits > 1 || !a.vec ||
          (d->flags & (M3S_EPI_DPT_OUT | M3S_EPI_ROPE | M3S_EPI_CONVT | M3S_EPI_OUT_FP8)))
        return launch<256, 128, 64, 4, 2, 3, 1>(a, d->batch, s);
      return launch<256, 256, 64, 2, 4, 2, 1>(a, d->batch, s);
    // 256x256 ping-pong (unsplit; no DPT tail / ConvTranspose scatter / e4m3 output):
    // otherwise the 256x128 8-wave tile
    case T256PP:
      if (a.splits > 1 || (d->flags & (M3S_EPI_DPT_OUT | M3S_EPI_CONVT | M3S_EPI_OUT_FP8)))
        return launch<256, 128, 64, 4, 2, 3, 1>(a, d->batch, s);
      if (!conv) return launch_pp<0>(a, d->batch, s);
      return (d->flags & M3S_PRO_RELU) ? launch_pp<2>(a, d->batch, s) : launch_pp<1>(a, d->batch, s);
    // 192x256 ping-pong: the grids a 256-row tile leaves on a partial wave (same fallbacks)
    case T192PP:
      if (a.splits > 1 || (d->flags & (M3S_EPI_DPT_OUT | M3S_EPI_CONVT | M3S_EPI_OUT_FP8)))
        return launch<256, 128, 64, 4, 2, 3, 1>(a, d->batch, s);
      if (!conv) return launch_pp<0, 192>(a, d->batch, s);
      return (d->flags & M3S_PRO_RELU) ? launch_pp<2, 192>(a, d->batch, s)
                                       : launch_pp<1, 192>(a, d->batch, s);
    default: return launch<64, 128, 64, 2, 2, 3, 2>(a, d->batch, s);
  }
}
