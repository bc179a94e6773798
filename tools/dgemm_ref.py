"""Times torch's f64 matmul (the ROCm library DGEMM) as a ceiling reference for the
hand-written gemm_tn_kernel. Diagnostic only; not part of the product path."""
import time
import torch

for (m, n, k) in [(8192, 8192, 8192), (16384, 16384, 768), (32768, 8192, 768), (4096, 4096, 4096)]:
    a = torch.randn(k, m, dtype=torch.float64, device="cuda")
    b = torch.randn(k, n, dtype=torch.float64, device="cuda")
    c = a.t() @ b
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        c = a.t() @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print(f"torch f64 TN GEMM m={m} n={n} k={k}: {2*m*n*k/dt/1e12:.2f} TFLOP/s")
