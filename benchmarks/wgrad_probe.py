"""Probe: backward-weight GEMM (gemm_tn) in plain vs implicit-conv (CONV) mode on the same
problem sizes, to separate the im2col addressing cost from the GEMM itself."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd._ext import native


def timeit(fn, it=20):
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
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    for (n, c, hw, co, k) in [(256, 256, 14, 256, 3), (256, 256, 14, 256, 1), (256, 2304, 14, 256, 1),
                              (256, 64, 56, 64, 3), (256, 576, 56, 64, 1), (256, 512, 7, 512, 3),
                              (256, 4608, 7, 512, 1), (256, 128, 28, 128, 3), (256, 1152, 28, 128, 1)]:
        x = torch.randn(n, hw, hw, c, device=dev).to(torch.bfloat16)
        dy = torch.randn(n, hw, hw, co, device=dev).to(torch.bfloat16)
        M = n * hw * hw
        fl = 2.0 * M * co * c * k * k
        p = k // 2
        nws = m.conv_wgrad_ws_floats(0, n, hw, hw, c, co, k, k, 1, p)
        ws = torch.empty(max(nws, 1), device=dev)
        dw = torch.empty(co, k * k * c, device=dev)
        t_conv = timeit(lambda: m.conv_wgrad(0, st, n, hw, hw, c, co, k, k, 1, p, dy.data_ptr(), x.data_ptr(),
                                             dw.data_ptr(), ws.data_ptr(), 0.0))
        rec = {"n": n, "c": c, "hw": hw, "co": co, "k": k, "conv_ms": round(t_conv, 4),
               "conv_tflops": round(fl / t_conv / 1e9, 1)}
        if k == 1:
            nws2 = m.gemm_tn_ws_floats(0, M, co, c)
            ws2 = torch.empty(max(nws2, 1), device=dev)
            t_g = timeit(lambda: m.gemm_tn(0, st, M, co, c, dy.data_ptr(), co, x.data_ptr(), c, dw.data_ptr(),
                                           ws2.data_ptr(), 0.0))
            rec.update(gemm_ms=round(t_g, 4), gemm_tflops=round(fl / t_g / 1e9, 1))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
