"""Probe: where the host's time goes in a ResNet-50 Downpour step (N = 1). cProfile around a
few steady steps, the functions sorted by their own time; with the GPU step at ~47 ms (fp32) /
~22 ms (bf16), the host is only on the critical path where it falls behind the GPU, which the
trace shows as gaps (scripts/step_gaps.py).

    python benchmarks/host_profile.py [fp32|bf16] [steps]
"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    dt = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import mpit_amd as mp
    from mpit_amd.train import TrainConfig, Trainer

    mp.Init()
    tr = Trainer(TrainConfig(model="resnet50", batch=256, amp=dt == "bf16"))
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(steps):
        tr.step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    print(f"host {1e3 * (t1 - t0) / steps:.2f} ms/step (profiled), wall incl. drain {1e3 * (t2 - t0) / steps:.2f}")
    print(s.getvalue())
    tr.stop()
    mp.Finalize()


if __name__ == "__main__":
    main()
