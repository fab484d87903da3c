"""Downpour steps with and without the side-stream backward are bitwise identical at N=1:
prints a checksum of the parameters after a few steps (run under MPIT_WGRAD_STREAM=0 / 1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp
from mpit_amd.ops.conv import WgradStream
from mpit_amd.train import TrainConfig, Trainer

mp.Init()
tr = Trainer(TrainConfig(model="resnet50", batch=32, num_classes=100, lr=0.01))
for _ in range(4):
    loss = tr.step()
tr.sync()
w = tr.flat.flat.double()
print(f"side={WgradStream.enabled} loss={float(loss):.6f} sum={w.sum().item():.10e} "
      f"l2={w.norm().item():.10e} absmax={w.abs().max().item():.6e}", flush=True)
tr.stop()
mp.Finalize()
