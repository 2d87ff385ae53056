"""Which hipBLASLt kernels torch picks for the pair's GEMM shapes (run under rocprofv3
--kernel-trace: the kernel names encode macro tile / waves / split)."""
import torch

dev = torch.device("cuda:0")
for (M, N, K, b) in [(768, 4096, 1024, 1), (768, 1024, 4096, 1), (768, 3072, 768, 4),
                     (768, 768, 3072, 4), (768, 6400, 7168, 2), (4096, 4096, 4096, 1)]:
    A = torch.randn(b, M, K, device=dev).bfloat16()
    B = torch.randn(b, N, K, device=dev).bfloat16()
    for _ in range(5):
        torch.bmm(A, B.transpose(1, 2))
    torch.cuda.synchronize()
    print("done", M, N, K, b, flush=True)
