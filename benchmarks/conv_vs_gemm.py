"""Micro-benchmark: every convolution of ResNet-50 at batch 256 (bf16, channels_last) as
MIOpen runs it (fwd, bwd-data, bwd-weight) versus the equivalent plain GEMMs on
hipBLASLt for the 1x1 convolutions (NHWC 1x1 conv == [N*H*W, Cin] x [Cin, Cout]).

Prints one JSON line per unique conv shape with its multiplicity in the network, and a
final line with the per-step totals. Used to decide which convolutions the ResNet
blocks route to GEMMs (mpit_amd/ops/conv.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mpit_amd.models import get_model


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


def collect(batch):
    dev = torch.device("cuda")
    m = get_model("resnet50").to(dev).to(memory_format=torch.channels_last)
    seen = {}

    def hook(mod, inp, out):
        x = inp[0]
        key = (tuple(x.shape), mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0])
        seen[key] = seen.get(key, 0) + 1

    hs = [mm.register_forward_hook(hook) for mm in m.modules() if isinstance(mm, torch.nn.Conv2d)]
    x = torch.randn(batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        m(x)
    for h in hs:
        h.remove()
    return seen


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dev = torch.device("cuda")
    tot = {"miopen": 0.0, "gemm_or_miopen": 0.0}
    for (xs, cout, k, s, p), mult in collect(batch).items():
        n, cin, h, w = xs
        x = torch.randn(xs, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, wt, stride=s, padding=p)
        gy = torch.randn_like(y)
        t_f = timeit(lambda: F.conv2d(x, wt, stride=s, padding=p))
        t_b = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                                  [0, 0], 1, [True, True, False]))
        rec = {"x": xs, "cout": cout, "k": k, "stride": s, "mult": mult, "miopen_fwd_ms": round(t_f, 4),
               "miopen_bwd_ms": round(t_b, 4)}
        fl = 2.0 * y.numel() * cin * k * k
        rec["miopen_fwd_tflops"] = round(fl / t_f / 1e9, 1)
        rec["miopen_bwd_tflops"] = round(2 * fl / t_b / 1e9, 1)
        best = t_f + t_b
        if k == 1 and s == 1 and cin % 64 == 0 and cout % 64 == 0:
            from mpit_amd.ops import conv as MC

            X = x.permute(0, 2, 3, 1).reshape(-1, cin)
            GY = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            W = wt.view(cout, cin)
            Wt = W.t().contiguous()
            t_md = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                                       [0, 0], 1, [True, False, False]))
            t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                                       [0, 0], 1, [False, True, False]))
            k_f = timeit(lambda: MC.gemm_nt(X, W))
            k_fs = timeit(lambda: MC.gemm_nt(X, W, stats=True))
            k_d = timeit(lambda: MC.gemm_nt(GY, Wt))
            k_w = timeit(lambda: MC.gemm_tn(GY, X))
            rec.update(miopen_dgrad_ms=round(t_md, 4), miopen_wgrad_ms=round(t_mw, 4), mfma_fwd_ms=round(k_f, 4),
                       mfma_fwd_stats_ms=round(k_fs, 4), mfma_dgrad_ms=round(k_d, 4), mfma_wgrad_ms=round(k_w, 4),
                       mfma_fwd_tflops=round(fl / k_f / 1e9, 1), mfma_wgrad_tflops=round(fl / k_w / 1e9, 1),
                       fwd_hbm_tbs=round((X.numel() + y.numel()) * 2 / k_f / 1e9, 2))
            tot.setdefault("mfma_1x1", 0.0)
            tot.setdefault("miopen_1x1", 0.0)
            tot["mfma_1x1"] += mult * (k_f + k_d + k_w)
            tot["miopen_1x1"] += mult * (t_f + t_md + t_mw)
        if k > 1 and cin % 64 == 0 and cout % 64 == 0:
            from mpit_amd.ops import conv as MC
            from mpit_amd._ext import native

            nm = native()
            wf = wt.float().contiguous(memory_format=torch.channels_last)
            wb, wtt = MC.conv_weights(wf, dgrad=True)
            dev_, st_ = x.device.index, torch.cuda.current_stream().cuda_stream
            yk = torch.empty_like(y)
            dxk = torch.empty_like(x)
            ho = y.shape[2]
            nws = nm.conv_wgrad_ws_floats(dev_, n, h, w, cin, cout, k, k, s, p)
            ws = torch.empty(max(nws, 1), device=dev, dtype=torch.float32)
            dwk = torch.empty(cout, k, k, cin, device=dev, dtype=torch.float32)
            k_f = timeit(lambda: nm.conv_fwd(dev_, st_, n, h, w, cin, cout, k, k, s, p, x.data_ptr(), wb.data_ptr(),
                                             yk.data_ptr(), 0, 0))
            k_w = timeit(lambda: nm.conv_wgrad(dev_, st_, n, h, w, cin, cout, k, k, s, p, gy.data_ptr(), x.data_ptr(),
                                               dwk.data_ptr(), ws.data_ptr(), 0.0))
            t_md = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                                       [0, 0], 1, [True, False, False]))
            t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [p, p], [1, 1], False,
                                                                       [0, 0], 1, [False, True, False]))
            if s == 1:
                k_d = timeit(lambda: nm.conv_fwd(dev_, st_, n, ho, ho, cout, cin, k, k, 1, k - 1 - p, gy.data_ptr(),
                                                 wtt.data_ptr(), dxk.data_ptr(), 0, 0))
            else:
                k_d = t_md
            rec.update(miopen_dgrad_ms=round(t_md, 4), miopen_wgrad_ms=round(t_mw, 4), mfma_fwd_ms=round(k_f, 4),
                       mfma_dgrad_ms=round(k_d, 4), mfma_wgrad_ms=round(k_w, 4),
                       mfma_fwd_tflops=round(fl / k_f / 1e9, 1), mfma_dgrad_tflops=round(fl / k_d / 1e9, 1),
                       mfma_wgrad_tflops=round(fl / k_w / 1e9, 1))
            tot.setdefault("mfma_kxk", 0.0)
            tot.setdefault("miopen_kxk", 0.0)
            tot["mfma_kxk"] += mult * (k_f + k_d + k_w)
            tot["miopen_kxk"] += mult * (t_f + t_md + t_mw)
            best = min(best, k_f + k_d + k_w)
        if k == 1:
            xin = x if s == 1 else x[:, :, ::s, ::s].contiguous(memory_format=torch.channels_last)
            X = xin.permute(0, 2, 3, 1).reshape(-1, cin)
            W = wt.view(cout, cin)
            GY = gy.permute(0, 2, 3, 1).reshape(-1, cout)
            g_f = timeit(lambda: X @ W.t()) + (timeit(lambda: x[:, :, ::s, ::s].contiguous(
                memory_format=torch.channels_last)) if s != 1 else 0.0)
            g_b = timeit(lambda: (GY @ W, GY.t() @ X))
            rec.update(gemm_fwd_ms=round(g_f, 4), gemm_bwd_ms=round(g_b, 4),
                       gemm_fwd_tflops=round(fl / g_f / 1e9, 1), gemm_bwd_tflops=round(2 * fl / g_b / 1e9, 1))
            best = min(best, g_f + g_b)
        tot["miopen"] += mult * (t_f + t_b)
        tot["gemm_or_miopen"] += mult * best
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_ms_per_step": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
