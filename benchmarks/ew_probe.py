"""Bandwidth of the fused update kernels (csrc/kernels/ew.h engine) on PS-sized shards.

    python benchmarks/ew_probe.py [n_millions ...]

Each case is captured 20 times into one HIP graph and the graph is replayed, so the
number is device time (a Python-issued launch costs more host time than a 3.2 M-element
kernel runs: timing eager calls measures the launcher, not the kernel). The parameter
server issues these kernels from its native progress thread, not from Python.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd import ops


def timeit(fn, per_graph=20, reps=10):
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(3):
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


for nm in [float(a) for a in sys.argv[1:]] or [25.6, 3.2]:
    n = int(nm * 1e6) // 64 * 64
    p, g, w = (torch.randn(n, device="cuda") for _ in range(3))
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    cases = {
        "apply(p+=a*g, w=p) 16B/elem": (lambda: ops.apply_(p, g, 0.5, out=w), 16),
        "apply(p+=a*g) 12B/elem": (lambda: ops.apply_(p, g, 0.5), 12),
        "adam 28B/elem": (lambda: ops.adam_(p, g, m, v, 0.9, 0.999, 1e-8, 1e-3), 28),
        "copy 8B/elem": (lambda: ops.copy_(w, p), 8),
        "torch add_ 12B/elem": (lambda: p.add_(g, alpha=0.5), 12),
    }
    for name, (fn, bpe) in cases.items():
        ms = timeit(fn)
        print(json.dumps({"n": n, "op": name, "us": round(ms * 1e3, 2), "tb_s": round(n * bpe / ms / 1e9, 2),
                          "unroll": os.environ.get("MPIT_EW_UNROLL", "auto"),
                          "grid": os.environ.get("MPIT_EW_GRID", "auto")}), flush=True)

# K shard pieces due at once (a server at N = K with 3.2 M-element pieces): one apply_ per
# piece vs ONE multi-segment launch (ops.apply_multi_), same bytes
if os.environ.get("EW_MULTI", "1") != "0":
    for k, nm in ((8, 3.2), (8, 0.8), (16, 0.8)):
        n = int(nm * 1e6) // 64 * 64
        ps = [torch.randn(n, device="cuda") for _ in range(k)]
        gs = [torch.randn(n, device="cuda") for _ in range(k)]
        ws = [torch.empty(n, device="cuda") for _ in range(k)]

        def one_by_one():
            for p, g, w in zip(ps, gs, ws):
                ops.apply_(p, g, 0.5, out=w)

        for name, fn in (("apply x%d launches 16B/elem" % k, one_by_one),
                         ("apply_multi %d segments 16B/elem" % k, lambda: ops.apply_multi_(ps, gs, 0.5, outs=ws))):
            ms = timeit(fn, per_graph=10)
            print(json.dumps({"n": k * n, "pieces": k, "op": name, "us": round(ms * 1e3, 2),
                              "tb_s": round(k * n * 16 / ms / 1e9, 2)}), flush=True)
