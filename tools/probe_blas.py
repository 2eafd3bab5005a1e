"""Calibration probe (not product): the MFMA utilisation a vendor library GEMM (torch.matmul ->
hipBLASLt) reaches on the tower's shapes, as a yardstick for the hand-written split GEMM.
bf16 A (M x K) @ B (K x N), fp32 accumulate; prints TFLOP/s per shape."""
import json
import time

import torch


def bench(M, K, N, dtype=torch.bfloat16, reps=50):
    a = torch.randn(M, K, device="cuda", dtype=dtype)
    b = torch.randn(K, N, device="cuda", dtype=dtype)
    for _ in range(10):
        c = a @ b
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"M": M, "K": K, "N": N, "dtype": str(dtype).split(".")[-1], "us": round(dt * 1e6, 2),
            "tflops": round(2.0 * M * K * N / dt / 1e12, 1)}


res = []
for (M, K, N) in [(65536, 640, 416), (65536, 416, 416), (65536, 624, 400), (65536, 400, 400),
                  (262144, 7808, 208), (65536, 1376, 400)]:
    res.append(bench(M, K, N))
    res.append(bench(M, K, N, torch.float32, reps=10))
print(json.dumps(res))
