"""Probe: the short-K 1x1 forward GEMMs of ResNet-50 (memory-bound: the output write
dominates) — gemm_nt with and without the BN-statistics epilogue, fp32 (fp16x3) and bf16,
against PyTorch's matmul and a plain copy of the output's bytes, so the achieved bandwidth
of each can be compared.

    python benchmarks/nt_shortk_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

SHAPES = [(802816, 256, 64), (802816, 64, 256), (200704, 512, 128), (50176, 1024, 256), (3211264, 64, 256)]


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3  # us


def main():
    from mpit_amd._ext import native
    from mpit_amd.ops import conv as C

    m = native()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    for dt in (torch.float32, torch.bfloat16):
        f32 = dt == torch.float32
        es = 4 if f32 else 2
        for M, N, K in SHAPES:
            a = torch.randn(M, K, device=dev).to(dt)
            b = (torch.randn(N, K, device=dev) * 0.05).to(dt)
            c = torch.empty(M, N, device=dev, dtype=dt)
            keep = []
            if f32:
                bp = C.f16_planes(b.contiguous(), C.bound_of_value(torch.linalg.vector_norm(b, float("inf"))))
                C.set_amax(a, C.bound_of_value(torch.linalg.vector_norm(a, float("inf"))))
                kw = C._split_kw(a, bp, True, keep)
                bb = bp
            else:
                kw, bb = {}, b
            stats = torch.empty(m.gemm_nt_stats_floats(M, N), dtype=torch.float32, device=dev)
            t0 = timeit(lambda: m.gemm_nt(0, st, M, N, K, a.data_ptr(), K, bb.data_ptr(), K, c.data_ptr(), N, 0,
                                          f32=f32, **kw))
            t1 = timeit(lambda: m.gemm_nt(0, st, M, N, K, a.data_ptr(), K, bb.data_ptr(), K, c.data_ptr(), N,
                                          stats.data_ptr(), f32=f32, **kw))
            tm = timeit(lambda: torch.mm(a, b.t(), out=c))
            c2 = torch.empty_like(c)
            tc = timeit(lambda: c2.copy_(c))
            by = (M * K + N * K + M * N) * es
            print(json.dumps({"dtype": str(dt)[6:], "M": M, "N": N, "K": K, "nt_us": round(t0, 1),
                              "nt_TBs": round(by / t0 / 1e6, 2), "nt_stats_us": round(t1, 1),
                              "torch_mm_us": round(tm, 1), "torch_mm_TBs": round(by / tm / 1e6, 2),
                              "copy_out_TBs": round(2 * M * N * es / tc / 1e6, 2)}), flush=True)
            del a, b, c, c2, keep


if __name__ == "__main__":
    main()
