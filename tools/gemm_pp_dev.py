"""Bench + check of the 256x256 ping-pong GEMM prototype (tools/gemm_pp_dev.hip, built as
tools/_build/libgemm_pp_dev.so) against torch.matmul (hipBLASLt) on the same random bf16
operands, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes, os, sys, statistics
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libgemm_pp_dev.so"))
lib.pp_gemm.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 7 + [ctypes.c_long] * 3 + \
    [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")


def run(A, B, C, M, N, K, b, group_m=0, prio=0):
    st = torch.cuda.current_stream().cuda_stream
    r = lib.pp_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, b, K, K, N, M * K, N * K,
                    M * N, group_m, prio, st)
    assert r == 0, r


def t_us(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


shapes = [(4096, 4096, 4096, 1), (8192, 8192, 8192, 1), (768, 6400, 7168, 2),
          (6144, 3072, 768, 4), (6144, 768, 3072, 4), (1536, 3072, 1024, 1), (1000, 1000, 1000, 1),
          (264, 200, 72, 3)]
if len(sys.argv) > 1:
    shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
BLAS_OK = {(4096, 4096, 4096, 1), (8192, 8192, 8192, 1), (768, 6400, 7168, 2),
           (6144, 3072, 768, 4), (6144, 768, 3072, 4)}
torch.manual_seed(0)
for (M, N, K, b) in shapes:
    A = (torch.rand(b, M, K, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(b, N, K, device=dev) * 2 - 1).bfloat16()
    C = torch.zeros(b, M, N, device=dev, dtype=torch.bfloat16)
    run(A, B, C, M, N, K, b)
    torch.cuda.synchronize()
    ref = torch.bmm(A.float(), B.float().transpose(1, 2))
    err = (C.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    ok = err <= 1e-2 * scale + 1e-2
    fl = 2.0 * M * N * K * b
    best = {}
    for rnd in range(3):   # interleaved rounds
        for pr in (0, 1, 2):
            for g in (0, 4, 8):
                t = t_us(lambda: run(A, B, C, M, N, K, b, g, pr))
                best[(pr, g)] = min(best.get((pr, g), 1e30), t)
    # hipBLASLt only on the shapes it has run cleanly on this image (a torch.bmm on
    # 6144x3840x768x4 left a memory-access fault, gpurun_out/pp1.txt)
    tr = min(t_us(lambda: torch.bmm(A, B.transpose(1, 2))) for _ in range(3)) \
        if (M, N, K, b) in BLAS_OK else float("nan")
    k = min(best, key=best.get)
    print(f"{M}x{N}x{K}x{b}: err {err:.3e} (scale {scale:.1f}) {'OK' if ok else 'FAIL'} | "
          f"pp {best[k]:8.1f} us {fl / best[k] / 1e6:7.1f} TF/s (prio {k[0]} group {k[1]}; "
          f"{' '.join(f'p{a}g{c}={v:.1f}' for (a, c), v in best.items())}) | "
          f"hipBLASLt {tr:8.1f} us {fl / tr / 1e6:7.1f} TF/s", flush=True)
