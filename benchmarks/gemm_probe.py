"""Time the MFMA GEMM / implicit-GEMM conv kernels on one shape (for rocprofv3 counter
runs and tile experiments).

    python benchmarks/gemm_probe.py nt M N K [iters]
    python benchmarks/gemm_probe.py conv N H W C Co R stride [iters]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd._ext import native


def timeit(fn, it):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    m = native()
    st = torch.cuda.current_stream().cuda_stream
    kind = sys.argv[1]
    if kind == "nt":
        M, N, K = map(int, sys.argv[2:5])
        it = int(sys.argv[5]) if len(sys.argv) > 5 else 50
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ms = timeit(lambda: m.gemm_nt(0, st, M, N, K, a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, 0), it)
        fl = 2.0 * M * N * K
        by = 2.0 * (M * K + N * K + M * N)
    else:
        Nb, H, W, C, Co, R, S = map(int, sys.argv[2:9])
        it = int(sys.argv[9]) if len(sys.argv) > 9 else 50
        pad = R // 2
        x = torch.randn(Nb, H, W, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Co, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        Ho, Wo = (H + 2 * pad - R) // S + 1, (W + 2 * pad - R) // S + 1
        y = torch.empty(Nb, Ho, Wo, Co, device="cuda", dtype=torch.bfloat16)
        ms = timeit(lambda: m.conv_fwd(0, st, Nb, H, W, C, Co, R, R, S, pad, x.data_ptr(), w.data_ptr(),
                                       y.data_ptr()), it)
        fl = 2.0 * Nb * Ho * Wo * Co * R * R * C
        by = 2.0 * (x.numel() + w.numel() + y.numel())
    print(json.dumps({"args": sys.argv[1:], "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                      "hbm_tbs": round(by / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
