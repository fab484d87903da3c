"""HBM bandwidth of the BN normalise(+add)(+ReLU) apply kernel (csrc/kernels/bn_act.hip),
fp32 and bf16, next to PyTorch's own elementwise kernels moving the same bytes.
Graph-replayed (device time, not launch time).

    python benchmarks/bn_bw_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd._ext import native


def timeit(fn, per_graph=10, reps=5):
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * per_graph)


def main():
    m = native()
    for (M, C) in [(802816, 256), (200704, 512), (802816, 64)]:
        for dt in (torch.float32, torch.bfloat16):
            es = 4 if dt == torch.float32 else 2
            x = torch.randn(M, C, device="cuda").to(dt)
            r = torch.randn(M, C, device="cuda").to(dt)
            y = torch.empty_like(x)
            coef = torch.randn(2 * C, device="cuda")

            def apply_res():
                m.bn_act_apply(0, torch.cuda.current_stream().cuda_stream, dt == torch.bfloat16, x.data_ptr(),
                               r.data_ptr(), y.data_ptr(), M, C, coef.data_ptr(), True)

            def apply_plain():
                m.bn_act_apply(0, torch.cuda.current_stream().cuda_stream, dt == torch.bfloat16, x.data_ptr(), 0,
                               y.data_ptr(), M, C, coef.data_ptr(), True)

            cases = {"bn_apply+res+relu": (apply_res, 3), "bn_apply+relu": (apply_plain, 2),
                     "torch add (x+r)": (lambda: torch.add(x, r, out=y), 3), "torch copy": (lambda: y.copy_(x), 2)}
            for name, (fn, passes) in cases.items():
                ms = timeit(fn)
                print(json.dumps({"M": M, "C": C, "dtype": str(dt).split(".")[-1], "op": name, "us": round(ms * 1e3, 1),
                                  "TBps": round(passes * M * C * es / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
