"""Microbench of the HIP GEMM on the pair-inference shapes vs torch.matmul (hipBLASLt,
reference point only)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monst3r-slam_amd")]
from monst3r_slam_amd.model import Ops
from monst3r_slam_amd import _lib
dev = torch.device("cuda:0"); ops = Ops(dev)
def t_ms(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); [fn() for _ in range(n)]; e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / n
shapes = [("enc qkv", 768, 3072, 1024, 1), ("enc proj", 768, 1024, 1024, 1), ("enc fc1", 768, 4096, 1024, 1),
          ("enc fc2", 768, 1024, 4096, 1), ("dec qkv x4", 768, 2304, 768, 4), ("dec fc2 x4", 768, 768, 3072, 4),
          ("dec fc1 x4", 768, 3072, 768, 4), ("lf fc2 x2", 768, 6400, 7168, 2), ("big 4096^3", 4096, 4096, 4096, 1)]
for name, M, N, K, b in shapes:
    A = torch.randn(b, M, K, device=dev).bfloat16(); B = torch.randn(b, N, K, device=dev).bfloat16()
    C = torch.empty(b, M, N, device=dev, dtype=torch.bfloat16)
    ms = t_ms(lambda: ops.gemm(A, B, C, M, N, K, b, sA=M*K, sB=N*K, sC=M*N))
    ms_ref = t_ms(lambda: torch.bmm(A, B.transpose(1, 2)))
    fl = 2.0 * M * N * K * b
    print(f"{name:12s} {M}x{N}x{K}x{b}: hip {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s | torch {ms_ref*1e3:8.1f} us {fl/ms_ref/1e9:7.1f} TF/s")
convs = [("head.2", 384, 512, 128, 128, 4), ("head.0", 192, 256, 256, 128, 4), ("rcu r1", 192, 256, 256, 256, 4),
         ("rcu r2", 96, 128, 256, 256, 4), ("layer1_rn", 96, 128, 96, 256, 4)]
for name, H, W, cin, cout, b in convs:
    x = torch.randn(b, H, W, cin, device=dev).bfloat16(); w = torch.randn(cout, 9 * cin, device=dev).bfloat16()
    out = torch.empty(b, H, W, cout, device=dev, dtype=torch.bfloat16)
    ms = t_ms(lambda: ops.gemm(x, w, out, H * W, cout, 9 * cin, b, sA=H*W*cin, sB=0, sC=H*W*cout, conv=(H, W, cin, H, W, 1)))
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last); wn = w.reshape(cout, 3, 3, cin).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    ms_ref = t_ms(lambda: torch.nn.functional.conv2d(xn, wn, padding=1))
    fl = 2.0 * H * W * cout * 9 * cin * b
    print(f"conv {name:10s} {H}x{W} {cin}->{cout} x{b}: hip {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s | torch {ms_ref*1e3:8.1f} us {fl/ms_ref/1e9:7.1f} TF/s")
