"""Which library kernel torch.mm (hipBLASLt) picks for the encoder GEMM shapes
(GPU box; a reference point only)."""
import torch
dev = torch.device("cuda")
for N, K in ((768, 256), (256, 256), (256, 1024), (1024, 256)):
    a = torch.randn(12032, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(3):
        torch.mm(a, w.t())
torch.cuda.synchronize()
