"""fp32 training parity: the mpit_amd ResNet-50 on its hand-written gfx950 kernels (fp16x3 or
bf16x6 split-product GEMMs through the trainer's weight plan, fused BN) vs the same network in stock PyTorch fp32 (MIOpen / hipBLASLt)
on the GPU, both against an fp64 CPU reference — same initial weights, same fixed synthetic
batch, plain SGD for ``--steps`` steps. Reports the step-0 gradients' error against fp64
(the precision measure: same weights, same batch) and the per-step losses / final
parameters (later steps amplify any fp32 rounding chaotically, for PyTorch's own fp32 too).

    python benchmarks/loss_parity.py [--batch 16] [--size 96] [--steps 20] [--lr 0.02] [--out f.json]
"""
import argparse
import copy
import json
import os
import sys
import threading
import time

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "benchmarks"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def train(model, x, y, steps, lr, plan=None):
    """(losses, final parameters, first-step gradients) of plain SGD on one fixed batch; with
    ``plan`` (the trainer's per-step WeightCastPlan) the GEMMs read its weight planes, as in
    training (fp16x3: every GEMM on the split products)"""
    losses, g0 = [], None
    params = [p for p in model.parameters()]
    for _ in range(steps):
        for p in params:
            p.grad = None
        if plan is not None:
            plan.run()
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        if plan is not None:
            plan.invalidate()
        if g0 is None:
            g0 = [p.grad.detach().double().cpu() for p in params]
        with torch.no_grad():
            for p in params:
                p.add_(p.grad, alpha=-lr)
        losses.append(float(loss.item()))
    return losses, [p.detach().double().cpu() for p in params], g0


def run(batch=16, size=96, steps=20, lr=0.02, classes=100, seed=0, use_plan=True):
    from mpit_amd.models.resnet import resnet50
    from torch_stock_resnet50 import ResNet50

    torch.manual_seed(seed)
    ours = resnet50(num_classes=classes)
    stock = ResNet50(classes)
    po, ps = list(ours.parameters()), list(stock.parameters())
    assert len(po) == len(ps), (len(po), len(ps))
    with torch.no_grad():
        for a, b in zip(po, ps):
            assert a.shape == b.shape, (a.shape, b.shape)
            b.copy_(a)
    ref = copy.deepcopy(stock).double()
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(batch, 3, size, size, generator=g)
    y = torch.randint(0, classes, (batch,), generator=g)
    dev = torch.device("cuda")
    cl = torch.channels_last
    t0 = time.perf_counter()
    l_ref, p_ref, g_ref = train(ref, x.double(), y, steps, lr)
    t_ref = time.perf_counter() - t0
    from mpit_amd.ops.conv import WeightCastPlan

    ours = ours.to(dev).to(memory_format=cl)
    plan = WeightCastPlan(ours, torch.float32) if use_plan else None
    l_ours, p_ours, g_ours = train(ours, x.to(dev).contiguous(memory_format=cl), y.to(dev), steps, lr, plan)
    l_stock, p_stock, g_stock = train(stock.to(dev).to(memory_format=cl), x.to(dev).contiguous(memory_format=cl),
                                      y.to(dev), steps, lr)

    def dev_loss(ls):
        return max(abs(a - b) / abs(b) for a, b in zip(ls, l_ref))

    def dev_param(ps_, ref_=None):
        ref_ = p_ref if ref_ is None else ref_
        num = sum(float((a - b).norm() ** 2) for a, b in zip(ps_, ref_)) ** 0.5
        den = sum(float(b.norm() ** 2) for b in ref_) ** 0.5
        return num / den

    def worst_tensor(gs):  # largest per-tensor relative gradient error
        return max(float((a - b).norm() / (b.norm() + 1e-30)) for a, b in zip(gs, g_ref))

    from mpit_amd.ops import conv as C

    return {"batch": batch, "size": size, "steps": steps, "lr": lr, "classes": classes,
            "split": C._F32_SPLIT, "weight_plan": bool(use_plan),
            "loss_fp64_cpu": l_ref, "loss_mpit_fp32": l_ours, "loss_stock_fp32": l_stock,
            "max_rel_loss_dev": {"mpit_fp32": dev_loss(l_ours), "stock_fp32": dev_loss(l_stock)},
            "final_param_rel_err": {"mpit_fp32": dev_param(p_ours), "stock_fp32": dev_param(p_stock)},
            # the step-0 gradients (same weights, same batch) are the precision measure; later
            # steps amplify fp32 rounding chaotically (CPU fp32 vs fp64 differs ~0.4 % in loss
            # after one step at lr 0.02 on this problem)
            "step0_grad_rel_err": {"mpit_fp32": dev_param(g_ours, g_ref), "stock_fp32": dev_param(g_stock, g_ref)},
            "step0_grad_worst_tensor_rel_err": {"mpit_fp32": worst_tensor(g_ours), "stock_fp32": worst_tensor(g_stock)},
            "fp64_cpu_s": round(t_ref, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=96)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-plan", action="store_true", help="GEMMs split the fp32 weights per call (no weight plan)")
    a = ap.parse_args()
    done = threading.Event()

    def heartbeat():  # MIOpen's first-call kernel builds / the fp64 CPU run print nothing for a while
        t0 = time.perf_counter()
        while not done.wait(30):
            print(f"... {time.perf_counter() - t0:.0f} s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    r = run(a.batch, a.size, a.steps, a.lr, use_plan=not a.no_plan)
    done.set()
    s = json.dumps(r)
    print(s, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
