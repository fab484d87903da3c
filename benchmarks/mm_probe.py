"""Library reference point for the MFMA GEMMs: torch.matmul (hipBLASLt) bf16 on GEMM shapes
of the ResNet-50 convolutions (implicit-GEMM M x N x K), against gemm_probe.py's numbers.

    python benchmarks/mm_probe.py [--f32] M N K [M N K ...]

--f32: fp32 operands (hipBLASLt's fp32 path), the library point for the fp32 (bf16x6) GEMMs.
"""
import json
import sys

import torch


def main():
    args = sys.argv[1:]
    f32 = "--f32" in args
    dt = torch.float32 if f32 else torch.bfloat16
    a = [int(v) for v in args if v != "--f32"]
    for i in range(0, len(a), 3):
        M, N, K = a[i:i + 3]
        x = torch.randn(M, K, device="cuda").to(dt)
        w = torch.randn(K, N, device="cuda").to(dt)
        for _ in range(5):
            y = x @ w
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 50
        s.record()
        for _ in range(it):
            y = x @ w
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / it
        print(json.dumps({"mm": [M, N, K], "dtype": "fp32" if f32 else "bf16", "ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
