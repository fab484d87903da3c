"""Probe: the fp32 (fp16x3) backward-weight GEMMs of ResNet-50 at batch 256 — plain 1x1 shapes
through gemm_tn and the 3x3 implicit-conv wgrads through conv_wgrad — timed and saved, so two
processes with different kernel knobs (MPIT_TN_F16S=0/1: per-use split FM 11 vs split-once FM 12)
can be compared for speed and agreement.

    python benchmarks/wgrad_f16x3_probe.py OUT.pt        (one JSON line per shape on stdout)
    python benchmarks/wgrad_f16x3_probe.py --compare A.pt B.pt
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

# (kind, M or (n, hw), N (co), K (c), taps): the wgrad shapes of gemm_calls_fp32 (r04h)
SHAPES = [("tn", 802816, 256, 64), ("tn", 802816, 64, 256), ("tn", 200704, 512, 128), ("tn", 200704, 128, 512),
          ("tn", 50176, 1024, 256), ("tn", 50176, 256, 1024), ("tn", 12544, 2048, 512), ("tn", 12544, 512, 2048),
          ("conv", 56, 64, 64), ("conv", 28, 128, 128), ("conv", 14, 256, 256), ("conv", 7, 512, 512)]


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
    return s.elapsed_time(e) / it


def run(out_path):
    from mpit_amd._ext import native
    from mpit_amd.ops import conv as C

    m = native()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    res = {}
    for sh in SHAPES:
        if sh[0] == "tn":
            _, M, N, K = sh
            y = torch.randn(M, N, device=dev, generator=g) * 1e-3
            x = torch.relu(torch.randn(M, K, device=dev, generator=g))
            fl = 2.0 * M * N * K
            out = C.gemm_tn(y, x, f16x3=True)
            ms = timeit(lambda: C.gemm_tn(y, x, f16x3=True))
        else:
            _, hw, co, c = sh
            n = 256
            x = torch.relu(torch.randn(n, hw, hw, c, device=dev, generator=g))
            y = torch.randn(n, hw, hw, co, device=dev, generator=g) * 1e-3
            ay, ax = [C.bound_of_value(torch.linalg.vector_norm(t, float("inf"))) for t in (y, x)]
            out = torch.empty(co, 9 * c, device=dev)
            nws = m.conv_wgrad_ws_floats(0, n, hw, hw, c, co, 3, 3, 1, 1)
            ws = torch.empty(max(nws, 1), device=dev)
            st = torch.cuda.current_stream().cuda_stream

            def f():
                m.conv_wgrad(0, st, n, hw, hw, c, co, 3, 3, 1, 1, y.data_ptr(), x.data_ptr(), out.data_ptr(),
                             ws.data_ptr(), 0.0, True, ay.data_ptr(), ax.data_ptr())
            f()
            ms = timeit(f)
            M, N, K = n * hw * hw, co, 9 * c
            fl = 2.0 * M * N * K
        key = "_".join(str(v) for v in sh)
        res[key] = out.detach().cpu()
        print(json.dumps({"shape": key, "ms": round(ms, 4), "TFLOPs": round(fl / ms / 1e9, 1),
                          "f16s": os.environ.get("MPIT_TN_F16S", "default")}), flush=True)
    torch.save(res, out_path)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    for k in A:
        d = ((A[k].double() - B[k].double()).norm() / B[k].double().norm()).item()
        print(json.dumps({"shape": k, "rel_diff": d, "bitwise": bool(torch.equal(A[k], B[k]))}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
