"""Metrics / logging: JSON-lines logs per rank (the reference's optim.Logger train.log /
test.log with gnuplot plots, asyncsgd/goot.lua:96-97,236-244), a confusion matrix
(optim.ConfusionMatrix, :93,209,232) and a running-average loss printer
(BiCNN/bicnn.lua:412-418)."""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import torch


class JsonLogger:
    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = path
        self.rank = rank
        self._f = None
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._f = open(path, "a", buffering=1)

    def log(self, **kv):
        kv.setdefault("time", time.time())
        kv.setdefault("rank", self.rank)
        line = json.dumps({k: (float(v) if isinstance(v, torch.Tensor) else v) for k, v in kv.items()})
        if self._f:
            self._f.write(line + "\n")
        return line

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class ConfusionMatrix:
    def __init__(self, nclasses: int):
        self.n = nclasses
        self.mat = torch.zeros(nclasses, nclasses, dtype=torch.int64)

    def add(self, pred: torch.Tensor, target: torch.Tensor):
        p = pred.reshape(-1).cpu().long()
        t = target.reshape(-1).cpu().long()
        self.mat.index_put_((t, p), torch.ones_like(t), accumulate=True)

    def batch_add(self, logits: torch.Tensor, target: torch.Tensor):
        self.add(logits.argmax(dim=-1), target)

    @property
    def total_valid(self) -> float:
        s = self.mat.sum().item()
        return self.mat.diag().sum().item() / s if s else 0.0

    def zero(self):
        self.mat.zero_()

    def __str__(self):
        return f"ConfusionMatrix(n={self.n}, global correct {100 * self.total_valid:.2f}%)"


class RunningAverage:
    def __init__(self, every: int = 2000):
        self.every, self.sum, self.cnt = every, 0.0, 0

    def add(self, v: float) -> Optional[float]:
        self.sum += float(v)
        self.cnt += 1
        if self.cnt == self.every:
            avg = self.sum / self.cnt
            self.sum, self.cnt = 0.0, 0
            return avg
        return None
