"""Micro-benchmark: fused BN(+add)(+ReLU) HIP kernels vs MIOpen batch-norm + PyTorch
add/ReLU, ResNet-50 activation shapes at batch 256, bf16 channels_last, fwd+bwd.
Prints one JSON line per shape with ms and effective TB/s of the fused version."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mpit_amd.ops.bn import BatchNormAct2d

SHAPES = [(256, 64, 112, 112), (256, 64, 56, 56), (256, 256, 56, 56), (256, 128, 28, 28), (256, 512, 28, 28),
          (256, 256, 14, 14), (256, 1024, 14, 14), (256, 512, 7, 7), (256, 2048, 7, 7)]


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
    dev = torch.device("cuda")
    for (n, c, h, w) in SHAPES:
        for res in (False, True):
            x = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
            r = torch.randn_like(x) if res else None
            gy = torch.randn_like(x)
            fused = BatchNormAct2d(c).to(dev)
            plain = torch.nn.BatchNorm2d(c).to(dev)

            def f_fused():
                xx = x.detach().requires_grad_(True)
                y = fused(xx, r)
                y.backward(gy)

            def f_plain():
                xx = x.detach().requires_grad_(True)
                y = plain(xx)
                if r is not None:
                    y = y + r
                y = F.relu(y)
                y.backward(gy)

            tf, tp = timeit(f_fused), timeit(f_plain)
            elems = n * c * h * w
            # fused bytes: fwd 2 reads (+res) + 1 write; bwd 2x(dy,y,x) reads + dx (+dres) write
            passes = (3 + (1 if res else 0)) + (6 + 1 + (1 if res else 0))
            print(json.dumps({"shape": [n, c, h, w], "residual": res, "fused_ms": round(tf, 3),
                              "miopen_plus_eltwise_ms": round(tp, 3), "speedup": round(tp / tf, 2),
                              "fused_TBps": round(passes * elems * 2 / tf / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
