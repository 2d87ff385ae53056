"""Tile / split-K sweep of the pair's skinny (M = 768 tokens) GEMMs with their real
epilogues, graph-replayed (20 back-to-back launches x 5 replays, HIP events on the replay
stream), plus torch.bmm (hipBLASLt) on the same operands as a reference point.
One JSON line per (shape, tile, splits, fused).
  python tools/gemm_sweep.py [--shapes enc|dec|all] > out.jsonl"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd import _lib  # noqa: E402
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)

# (name, M, N, K, batch, epilogue): "res" = bias + f32 residual + LN statistics (the
# residual producers), "gelu" = bias + GELU, "bias" = plain
SHAPES = {
    "enc": [("enc_qkv", 768, 3072, 1024, 1, "bias"), ("enc_proj", 768, 1024, 1024, 1, "res"),
            ("enc_fc1", 768, 4096, 1024, 1, "gelu"), ("enc_fc2", 768, 1024, 4096, 1, "res")],
    "dec": [("dec_qkvkv", 768, 3840, 768, 2, "bias"), ("dec_proj", 768, 768, 768, 2, "res"),
            ("dec_fc1", 768, 3072, 768, 2, "gelu"), ("dec_fc2", 768, 768, 3072, 2, "res")],
    # the MASt3R local-feature MLP (per pair: the two MASt3R views)
    "lf": [("lf_fc1", 768, 7168, 1792, 2, "gelu"), ("lf_fc2", 768, 6400, 7168, 2, "f32")],
}


def timed(fn, reps=20, replays=5):
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(replays):
            g.replay()
        e1.record(s)
        e1.synchronize()
    del g
    return e0.elapsed_time(e1) / (replays * reps) * 1e3


# DPT head convs (H, W, Cin, Cout, batch): implicit-GEMM 3x3, bias (+ bf16 residual)
CONVS = [("rn1_rcu", 96, 128, 256, 256, 2), ("rn2_rcu", 48, 64, 256, 256, 2),
         ("rn3_rcu", 24, 32, 256, 256, 2), ("head0", 192, 256, 256, 128, 2),
         ("head2", 384, 512, 128, 128, 2)]


def sweep_convs(tiles):
    from monst3r_slam_amd.model import _conv_pack
    for name, H, W, cin, cout, b in CONVS:
        g = torch.Generator(device=dev).manual_seed(3)
        x = torch.randn(b, H, W, cin, device=dev, generator=g).bfloat16()
        w = _conv_pack(torch.randn(cout, cin, 3, 3, device=dev, generator=g) /
                       (9 * cin) ** 0.5).bfloat16().contiguous()
        bias = torch.randn(cout, device=dev, generator=g)
        out = torch.empty(b, H, W, cout, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * H * W * cout * 9 * cin * b

        def run(tile=None):
            ops.gemm(x, w, out, H * W, cout, 9 * cin, b, sA=H * W * cin, sB=0,
                     sC=H * W * cout, bias=bias, sBias=0, conv=(H, W, cin, H, W, 1), tile=tile)
        us = timed(run)
        print(json.dumps({"shape": name, "impl": "default", "us": us, "tflops": fl / us / 1e6}),
              flush=True)
        for t in tiles:
            us = timed(lambda: run((t, 1)))
            print(json.dumps({"shape": name, "impl": "m3s", "tile": t, "splits": 1, "fused": 0,
                              "us": us, "tflops": fl / us / 1e6}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--tiles", default="1,2,7,10,11,12,13")
    ap.add_argument("--splits", default="1,2,3,4,6,8")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    if a.shapes == "conv":
        sweep_convs(tiles)
        return
    shapes = SHAPES["enc"] + SHAPES["dec"] if a.shapes == "all" else SHAPES[a.shapes]
    splits = [int(t) for t in a.splits.split(",")]
    for name, M, N, K, b, epi in shapes:
        A = torch.randn(b, M, K, device=dev).bfloat16()
        B = (torch.randn(b, N, K, device=dev) / K ** 0.5).bfloat16()
        bias = torch.randn(b, N, device=dev)
        x = torch.randn(b, M, N, device=dev)
        C2 = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(b, M, N // 128, 2, device=dev)
        fl = 2.0 * M * N * K * b
        ref = timed(lambda: torch.bmm(A, B.transpose(1, 2)))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "batch": b, "impl": "hipblaslt",
                          "us": ref, "tflops": fl / ref / 1e6}), flush=True)
        os.environ.pop("M3S_GEMM_TILE", None)
        os.environ.pop("M3S_GEMM_SPLITS", None)

        def run(tile=None):
            kw = dict(sA=M * K, sB=N * K, sC=M * N, sBias=N, tile=tile)
            if epi == "res":
                ops.gemm(A, B, x, M, N, K, b, bias=bias, R=x, sR=M * N, ln_stats=(C2, stats),
                         flags=_lib.EPI_OUT_F32 | _lib.EPI_RES_F32, **kw)
            elif epi == "gelu":
                ops.gemm(A, B, C2, M, N, K, b, bias=bias, flags=_lib.EPI_GELU, **kw)
            elif epi == "f32":
                ops.gemm(A, B, x, M, N, K, b, bias=bias, flags=_lib.EPI_OUT_F32, **kw)
            else:
                ops.gemm(A, B, C2, M, N, K, b, bias=bias, **kw)
        us = timed(run)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "batch": b, "impl": "default",
                          "us": us, "tflops": fl / us / 1e6}), flush=True)
        for t in tiles:
            for sp in splits:
                for fused in ((0, 1) if sp > 1 else (0,)):
                    os.environ["M3S_GEMM_FUSED"] = str(fused)
                    try:
                        us = timed(lambda: run((t, sp)))
                    except RuntimeError as e:
                        print(json.dumps({"shape": name, "tile": t, "splits": sp, "fused": fused,
                                          "error": str(e)}), flush=True)
                        continue
                    print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "batch": b,
                                      "impl": "m3s", "tile": t, "splits": sp, "fused": fused,
                                      "us": us, "tflops": fl / us / 1e6}), flush=True)
        os.environ.pop("M3S_GEMM_FUSED", None)


if __name__ == "__main__":
    main()
