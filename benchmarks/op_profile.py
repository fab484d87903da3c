"""torch.profiler operator table of the training step (which PyTorch ops launch the
non-mpit kernels of a kernel trace).

    python benchmarks/op_profile.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --dtype bf16

Prints the top operators by self device time over 3 profiled steps (after 3 warmup steps)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg16")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--optimizer", default="eamsgd")
    ap.add_argument("--su", type=int, default=2)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rows", type=int, default=45)
    a = ap.parse_args()
    mp.Init()
    mva = 0.9 if a.optimizer in ("eamsgd", "easgd") else 0.0  # bench.py's single-rank settings
    tr = Trainer(TrainConfig(model=a.model, batch=a.batch, optimizer=a.optimizer, su=a.su, mva=mva, mom=0.0,
                             amp=a.dtype == "bf16"))
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts) as prof:
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_device_time_total", row_limit=a.rows, max_name_column_width=60))
    tr.stop()
    mp.Finalize()


if __name__ == "__main__":
    main()
