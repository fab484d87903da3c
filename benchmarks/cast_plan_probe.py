"""Time the per-step weight cast launch (ops/conv.py WeightCastPlan, gemm.hip cast_batch_kernel)
of VGG-16's bf16 plan: the whole model, the convolutions only, the classifier only.

    python benchmarks/cast_plan_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


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
    return s.elapsed_time(e) / it * 1e3


def main():
    from mpit_amd.models import get_model
    from mpit_amd.ops.conv import WeightCastPlan

    m = get_model("vgg16").cuda().to(memory_format=torch.channels_last)
    for name, mod in (("all", m), ("features", m.features), ("classifier", m.classifier)):
        plan = WeightCastPlan(mod, torch.bfloat16)
        nbytes = sum(p.numel() for mm, _, _ in plan.mods for p in [mm.weight]) * 6
        t = timeit(plan.run)
        print(json.dumps({"plan": name, "jobs": plan.njobs, "blocks": plan.nblocks, "us": round(t, 1),
                          "TBs_fp32_in_2x_bf16_out": round(nbytes / t / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
