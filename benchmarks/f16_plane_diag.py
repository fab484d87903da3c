"""Diagnostic: the weight plan's fp16x3 planes (cast_batch_kernel, split1h) against the same
split on PyTorch ops (ops/conv.py f16_planes), element by element with the exact residual.

    python benchmarks/f16_plane_diag.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd.ops import conv as C


def main():
    torch.manual_seed(5)
    net = torch.nn.Sequential(C.Conv1x1(256, 128)).cuda().to(memory_format=torch.channels_last)
    plan = C.WeightCastPlan(net, torch.float32)
    plan.run()
    torch.cuda.synchronize()
    mod, _, (wb, wt) = plan.mods[0]
    w = mod.weight.detach().reshape(128, 256)
    amax = wb._mpit_wamax
    e = int(C._f16_exp(amax).item())
    ref = C.f16_planes(w, amax)
    for name, got, want, src in (("wb", wb, ref, w), ("wt", wt, C.f16_planes(w.t().contiguous(), amax), w.t())):
        bad = (got != want).reshape(2, -1)
        print(name, "amax", amax.item(), "e", e, "h mismatches", int(bad[0].sum()), "l mismatches", int(bad[1].sum()))
        idx = torch.nonzero(bad[1])[:8, 0]
        for i in idx.tolist():
            v = src.reshape(-1)[i].item()
            s = v * 2.0 ** e
            h = float(got.reshape(2, -1)[0, i].item())
            print(f"  v={v!r} s={s!r} h={h!r} exact_l={(s - h) * 2048!r} got_l={got.reshape(2, -1)[1, i].item()!r} "
                  f"torch_l={want.reshape(2, -1)[1, i].item()!r}")


if __name__ == "__main__":
    main()
