"""Time the MFMA GEMM / implicit-GEMM conv kernels on one shape (for rocprofv3 counter
runs and tile experiments), bf16 or fp32 (``--f32``: v_mfma_f32_32x32x2_f32).

    python benchmarks/gemm_probe.py [--f32] nt M N K [iters]
    python benchmarks/gemm_probe.py [--f32] tn M N K [iters]
    python benchmarks/gemm_probe.py [--f32] conv N H W C Co R stride [iters]
    python benchmarks/gemm_probe.py [--f32] wgrad N H W C Co R stride [iters]
    python benchmarks/gemm_probe.py [--f32] dgrad N H W C Co R 1 [iters]      (stride-1 backward-data)

``--f32 --bsplit``: the weight operand as three bf16 planes (bf16x6, FM 9); ``--f32 --f16x3``:
the fp16x3 split products (FM 11: weight as two fp16 planes, operand bounds from reductions);
``--f32 --f16x3 --planes``: the activation / gradient operands arrive as fp16 planes too (FM 13,
what the BN apply passes write in an fp32 step: nothing split in the kernel).
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
    args = sys.argv[1:]
    f32 = "--f32" in args
    bsplit = "--bsplit" in args  # fp32: weight operand as three pre-split bf16 planes (FM 4)
    f16x3 = "--f16x3" in args
    pl = "--planes" in args and f32 and f16x3
    args = [a for a in args if a not in ("--f32", "--bsplit", "--f16x3", "--planes")]
    from mpit_amd.ops import conv as cops

    def bound(t):
        return cops.bound_of_value(torch.linalg.vector_norm(t.float(), float("inf")))
    keep = []

    def planes(t):
        t = t.float()
        h = t.to(torch.bfloat16)
        r = t - h.float()
        m_ = r.to(torch.bfloat16)
        return torch.stack([h, m_, (r - m_.float()).to(torch.bfloat16)]).contiguous()

    def act(t, bnd):  # (operand, plane stride) of an activation operand: fp16 planes with --planes
        if not pl:
            return t, 0
        p = cops.f16_planes(t.reshape(-1).contiguous(), bnd)
        keep.append(p)
        return p, p[0].numel()

    def bp(t):  # (operand, bps) of a weight operand
        if f32 and f16x3:
            p = cops.f16_planes(t.contiguous(), bound(t))
            keep.append(p)
            return p, p[0].numel()
        if f32 and bsplit:
            p = planes(t)
            return p, p[0].numel()
        return t, 0
    dt = torch.float32 if f32 else torch.bfloat16
    es = 4 if f32 else 2
    kind = args[0]
    if kind in ("nt", "tn"):
        M, N, K = map(int, args[1:4])
        it = int(args[4]) if len(args) > 4 else 50
        if kind == "nt":
            a = torch.randn(M, K, device="cuda").to(dt)
            b, bps = bp((torch.randn(N, K, device="cuda") * 0.05).to(dt))
            c = torch.empty(M, N, device="cuda", dtype=dt)
            ab = bound(a)
            keep.append(ab)
            a, aps = act(a, ab)
            kw = dict(amax_a=ab.data_ptr(), amax_b=b._mpit_wamax.data_ptr()) if (f32 and f16x3) else {}
            if aps:
                kw["aps"] = aps
            ms = timeit(lambda: m.gemm_nt(0, st, M, N, K, a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N, 0,
                                          f32=f32, bps=bps, **kw), it)
            by = es * (M * K + N * K + M * N)
        else:
            y = torch.randn(M, N, device="cuda").to(dt)
            x = torch.randn(M, K, device="cuda").to(dt)
            out = torch.empty(N, K, device="cuda")
            nws = m.gemm_tn_ws_floats(0, M, N, K)
            ws = torch.empty(max(1, nws), device="cuda")
            yb, xb = bound(y), bound(x)
            keep += [yb, xb]
            kw = dict(amax_y=yb.data_ptr(), amax_x=xb.data_ptr()) if (f32 and f16x3) else {}
            y, yps = act(y, yb)
            x, xps = act(x, xb)
            if yps:
                kw.update(yps=yps, xps=xps)
            ms = timeit(lambda: m.gemm_tn(0, st, M, N, K, y.data_ptr(), N, x.data_ptr(), K, out.data_ptr(),
                                          ws.data_ptr(), 0.0, f32=f32, **kw), it)
            by = es * (M * K + M * N) + 4 * N * K
        fl = 2.0 * M * N * K
    else:
        Nb, H, W, C, Co, R, S = map(int, args[1:8])
        it = int(args[8]) if len(args) > 8 else 50
        pad = R // 2
        Ho, Wo = (H + 2 * pad - R) // S + 1, (W + 2 * pad - R) // S + 1
        x = torch.randn(Nb, H, W, C, device="cuda").to(dt)
        w, wbps = bp((torch.randn(Co, R, R, C, device="cuda") * 0.05).to(dt))
        y = torch.randn(Nb, Ho, Wo, Co, device="cuda").to(dt)
        keep += [bound(x), bound(y)]
        fx = f32 and f16x3
        xb, yb = keep[-2], keep[-1]
        x, xps = act(x, xb)
        y, yps = act(y, yb)
        if kind == "conv":
            kw = dict(amax_a=xb.data_ptr(), amax_b=w._mpit_wamax.data_ptr()) if fx else {}
            if xps:
                kw["aps"] = xps
            ms = timeit(lambda: m.conv_fwd(0, st, Nb, H, W, C, Co, R, R, S, pad, x.data_ptr(), w.data_ptr(),
                                           y.data_ptr(), f32=f32, bps=wbps, **kw), it)
        elif kind == "dgrad":  # stride-1 backward-data = forward conv of dy with the transposed weight
            wt, tbps = bp((torch.randn(C, R, R, Co, device="cuda") * 0.05).to(dt))
            dx = torch.empty(Nb, H, W, C, device="cuda", dtype=dt)
            kw = dict(amax_a=yb.data_ptr(), amax_b=wt._mpit_wamax.data_ptr()) if fx else {}
            if yps:
                kw["aps"] = yps
            ms = timeit(lambda: m.conv_fwd(0, st, Nb, Ho, Wo, Co, C, R, R, 1, R - 1 - pad, y.data_ptr(),
                                           wt.data_ptr(), dx.data_ptr(), f32=f32, bps=tbps, **kw), it)
        else:
            dw = torch.empty(Co, R, R, C, device="cuda")
            nws = m.conv_wgrad_ws_floats(0, Nb, H, W, C, Co, R, R, S, pad)
            ws = torch.empty(max(1, nws), device="cuda")
            kw = dict(amax_y=yb.data_ptr(), amax_x=xb.data_ptr()) if fx else {}
            if yps:
                kw.update(yps=yps, xps=xps)
            ms = timeit(lambda: m.conv_wgrad(0, st, Nb, H, W, C, Co, R, R, S, pad, y.data_ptr(), x.data_ptr(),
                                             dw.data_ptr(), ws.data_ptr(), 0.0, f32=f32, **kw), it)
        fl = 2.0 * Nb * Ho * Wo * Co * R * R * C
        by = es * (Nb * H * W * C + (w[0].numel() if wbps else w.numel()) + Nb * Ho * Wo * Co)
    print(json.dumps({"args": sys.argv[1:], "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                      "hbm_tbs": round(by / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
