"""Library reference point for the MFMA GEMMs: torch.matmul (hipBLASLt) bf16 on GEMM shapes
of the ResNet-50 convolutions (implicit-GEMM M x N x K), against gemm_probe.py's numbers.

    python benchmarks/mm_probe.py M N K [M N K ...]
"""
import json
import sys

import torch


def main():
    a = list(map(int, sys.argv[1:]))
    for i in range(0, len(a), 3):
        M, N, K = a[i:i + 3]
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(K, N, device="cuda").to(torch.bfloat16)
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
        print(json.dumps({"mm": [M, N, K], "ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
