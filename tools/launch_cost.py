"""Fixed cost of a kernel boundary on the replayed graph: 50 back-to-back launches of one
kernel captured in a HIP graph, time per launch.  Separates launch/boundary overhead from
the GEMM's own block lifetime (tools/gemm_stamps.py)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops  # noqa: E402

dev = torch.device("cuda:0")
ops = Ops(dev)
N_L = 50


def graph_us(fn):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(N_L):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream(dev)
    e0.record(st)
    for _ in range(5):
        g.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * N_L)


x = torch.randn(4, 1024, device=dev)
g1 = torch.ones(1024, device=dev)
b1 = torch.zeros(1024, device=dev)
y = torch.empty(4, 1024, device=dev, dtype=torch.bfloat16)
print(f"layernorm 1 row          : {graph_us(lambda: ops.ln(x, g1, b1, y, 1, 1024)):7.2f} us", flush=True)
xl = torch.randn(4 * 768, 768, device=dev)
yl = torch.empty(4 * 768, 768, device=dev, dtype=torch.bfloat16)
g2, b2 = torch.ones(768, device=dev), torch.zeros(768, device=dev)
print(f"layernorm 3072x768       : {graph_us(lambda: ops.ln(xl, g2, b2, yl, 3072, 768)):7.2f} us", flush=True)
for (M, N, K, b, out32) in [(128, 128, 64, 1, False), (768, 4096, 64, 1, False), (768, 4096, 64, 1, True),
                            (768, 4096, 256, 1, False), (768, 4096, 1024, 1, False),
                            (768, 768, 64, 4, True), (768, 768, 768, 4, True), (768, 3072, 768, 4, False)]:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = torch.randn(b, N, K, device=dev).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.float32 if out32 else torch.bfloat16)
    fl = 32 if out32 else 0
    us = graph_us(lambda: ops.gemm(A, B, C, M, N, K, b, sA=M * K, sB=N * K, sC=M * N, flags=fl,
                                   split_k=1))
    print(f"gemm {M}x{N}x{K}x{b} {'f32' if out32 else 'bf16'} out: {us:7.2f} us "
          f"({2.0 * M * N * K * b / us / 1e6:6.0f} TF/s)", flush=True)
print(torch.cuda.get_device_properties(dev))
