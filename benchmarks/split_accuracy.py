"""Accuracy of the fp32 GEMM paths on the ResNet-50 GEMM shapes: relative Frobenius error
against an fp64 CPU reference of PyTorch fp32 (hipBLASLt), the bf16x6 split products (6 bf16
MFMAs per product, weight as three bf16 planes) and the fp16x3 split products (3 fp16 MFMAs,
weight as two fp16 planes of the power-of-two-scaled weight). Operands like the network's:
ReLU'd activations x weights (forward), gradients (1e-6 scale) x weights (backward-data),
gradients x activations reduced over M (backward-weight).

    python benchmarks/split_accuracy.py
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpit_amd._ext import native
from mpit_amd.ops import conv as C


def rel(a, ref):
    a = a.double().cpu()
    return float((a - ref).norm() / ref.norm())


def bf16_planes(t):
    t = t.float()
    h = t.to(torch.bfloat16)
    r = t - h.float()
    m = r.to(torch.bfloat16)
    return torch.stack([h, m, (r - m.float()).to(torch.bfloat16)]).contiguous()


def nt(a, b, mode):
    m = native()
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty(M, N, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    if mode == "bf16x6":
        p = bf16_planes(b)
        m.gemm_nt(0, st, M, N, K, a.data_ptr(), K, p.data_ptr(), K, c.data_ptr(), N, 0, f32=True, bps=p[0].numel())
    else:
        c = C.gemm_nt(a, b, f16x3=True)
    return c


def main():
    torch.manual_seed(0)
    out = []
    for kind, M, N, K in [("fwd", 50176, 256, 2304), ("fwd", 802816 // 4, 64, 576), ("fwd", 12544, 512, 4608),
                          ("fwd", 200704, 512, 128), ("dgrad", 50176, 256, 2304), ("dgrad", 12544, 1024, 2048),
                          ("wgrad", 50176, 256, 1024), ("wgrad", 200704, 64, 576)]:
        if kind == "wgrad":
            y = torch.randn(M, N, device="cuda") * 1e-6
            x = torch.relu(torch.randn(M, K, device="cuda"))
            ref = y.double().cpu().t() @ x.double().cpu()
            res = {"torch_fp32": rel(y.t() @ x, ref), "bf16x6": rel(C.gemm_tn(y, x), ref),
                   "fp16x3": rel(C.gemm_tn(y, x, f16x3=True), ref)}
        else:
            a = torch.relu(torch.randn(M, K, device="cuda")) if kind == "fwd" else torch.randn(M, K, device="cuda") * 1e-6
            b = torch.randn(N, K, device="cuda") * math.sqrt(2.0 / K)
            ref = a.double().cpu() @ b.double().cpu().t()
            res = {"torch_fp32": rel(a @ b.t(), ref), "bf16x6": rel(nt(a, b, "bf16x6"), ref),
                   "fp16x3": rel(nt(a, b, "fp16x3"), ref)}
        r = {"kind": kind, "M": M, "N": N, "K": K, **{k: float(f"{v:.3e}") for k, v in res.items()}}
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
