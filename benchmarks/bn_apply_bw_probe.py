"""Probe: bandwidth of the BatchNorm apply passes (forward apply with residual + ReLU mask,
backward apply with and without the mask) on the ResNet-50 batch-256 activation shapes, against a PyTorch
elementwise pass moving the same bytes (addcmul: two reads, one write). Run it twice with
MPIT_BN_SPLIT=0/1 to compare the fp32 lane layouts (csrc/kernels/bn_act.hip, Slot).

    python benchmarks/bn_apply_bw_probe.py [fp32|bf16]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

SHAPES = [(112 * 112, 64), (56 * 56, 64), (56 * 56, 256), (28 * 28, 128), (28 * 28, 512), (14 * 14, 256),
          (14 * 14, 1024), (7 * 7, 512), (7 * 7, 2048)]


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
    dt = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    from mpit_amd._ext import native

    m = native()
    dev = torch.device("cuda")
    bf16 = dt == "bf16"
    ty = torch.bfloat16 if bf16 else torch.float32
    es = 2 if bf16 else 4
    st = torch.cuda.current_stream().cuda_stream
    tot = {"bwd_ms": 0.0, "fwd_ms": 0.0, "torch_ms": 0.0}
    for hw, C in SHAPES:
        M = 256 * hw
        x = torch.randn(M, C, device=dev).to(ty)
        dy = torch.randn(M, C, device=dev).to(ty)
        res = torch.randn(M, C, device=dev).to(ty)
        dx = torch.empty_like(x)
        mask = torch.randint(0, 256, (M * C // 8,), device=dev, dtype=torch.uint8)
        coef = torch.randn(3 * C, device=dev)
        amax = torch.zeros(512, device=dev)
        ws = torch.empty(m.bn_workspace_floats(C), device=dev)

        def bwd():
            m.bn_act_bwd(0, st, bf16, dy.data_ptr(), mask.data_ptr(), x.data_ptr(), dx.data_ptr(), 0, M, C, 0, 0, 0,
                         0, 0, ws.data_ptr(), True, coef=coef.data_ptr(), amax=amax.data_ptr())

        def bwd_nomask():
            m.bn_act_bwd(0, st, bf16, dy.data_ptr(), 0, x.data_ptr(), dx.data_ptr(), 0, M, C, 0, 0, 0,
                         0, 0, ws.data_ptr(), False, coef=coef.data_ptr(), amax=amax.data_ptr())

        def fwd():
            m.bn_act_apply(0, st, bf16, x.data_ptr(), res.data_ptr(), dx.data_ptr(), M, C, coef.data_ptr(), True)

        def ref():
            torch.addcmul(x, dy, x, out=dx)

        tb, tn, tf, tr = timeit(bwd), timeit(bwd_nomask), timeit(fwd), timeit(ref)
        nb = M * C * (3 * es) + M * C // 8
        tot["bwd_ms"] += tb
        tot["fwd_ms"] += tf
        tot["torch_ms"] += tr
        print(json.dumps({"dtype": dt, "M": M, "C": C, "bwd_ms": round(tb, 4), "bwd_TBs": round(nb / tb / 1e9, 2),
                          "bwd_nomask_TBs": round(M * C * 3 * es / tn / 1e9, 2),
                          "fwd_ms": round(tf, 4), "fwd_TBs": round(M * C * 3 * es / tf / 1e9, 2),
                          "torch_addcmul_TBs": round(M * C * 3 * es / tr / 1e9, 2),
                          "split": os.environ.get("MPIT_BN_SPLIT", "default")}), flush=True)
        del x, dy, res, dx, mask
    print(json.dumps({"dtype": dt, "total": {k: round(v, 3) for k, v in tot.items()},
                      "split": os.environ.get("MPIT_BN_SPLIT", "default")}), flush=True)


if __name__ == "__main__":
    main()
