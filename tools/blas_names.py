"""hipBLASLt (torch.matmul) on the encoder GEMM shapes, for rocprofv3 --kernel-trace: the kernel
names encode the vendor's macro tile / MFMA / depth choices (a known-good reference, guide §5.4 rule 10)."""
import torch

SHAPES = [("qkv", 12608, 2304, 768), ("o", 12608, 768, 768), ("fc1", 12608, 3072, 768), ("fc2", 12608, 768, 3072),
          ("4096^3", 4096, 4096, 4096)]
dev = torch.device("cuda")
for name, M, N, K in SHAPES:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(10):
        torch.matmul(A, B.t())
    torch.cuda.synchronize()
    print(name, flush=True)
