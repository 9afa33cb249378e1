"""Which library kernel does torch's fp64 GEMM (n=4096 x 8192 x 4096) run on gfx950, and how fast?  (context for
the trmm kernel's tiling; run under rocprofv3 --kernel-trace to read the Tensile/hipBLASLt kernel name.)"""
import torch, time
dev = torch.device("cuda", 0)
A = torch.rand(4096, 4096, device=dev, dtype=torch.float64)
B = torch.rand(4096, 8192, device=dev, dtype=torch.float64)
for _ in range(3):
    C = A.T @ B
torch.cuda.synchronize()
a = time.perf_counter()
for _ in range(5):
    C = A.T @ B
torch.cuda.synchronize()
t = (time.perf_counter() - a) / 5
print(f"A^T B 4096x4096x8192 fp64: {t * 1e3:.3f} ms, {2 * 4096 * 4096 * 8192 / t / 1e12:.1f} TF/s")
