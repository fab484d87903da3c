"""Checkpoint / resume for workers AND parameter-server shards.

The reference saves only the worker model every ``saveep`` epochs
(asyncsgd/goot.lua:246-254) or the tester's flat parameters (BiCNN/bicnn.lua:590-594),
and never the server shards or server optimizer state. Here every rank
writes one file per checkpoint step:

* worker: flat parameters, local optimizer state (tensors in ``state``), step counters;
* server: its shard, offset/size, server optimizer state, update version.

Files are written atomically (tmp + rename) with ``torch.save`` and read back with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def _atomic_save(obj, path: str):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _tensors_only(state: dict) -> dict:
    out = {}
    for k, v in state.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.detach().cpu()
        elif isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
    return out


def save(directory: str, step: int, rank: int, flat=None, opt_state: Optional[dict] = None, server=None,
         extra: Optional[dict] = None) -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f"ckpt_step{step:08d}_rank{rank:03d}.pt")
    obj = {"step": step, "rank": rank}
    if flat is not None:
        obj["params"] = flat.flat[: flat.numel].detach().cpu()
    if opt_state is not None:
        obj["opt_state"] = _tensors_only(opt_state)
    if server is not None:
        obj["server"] = server.state_dict()
    if extra:
        obj["extra"] = extra
    _atomic_save(obj, path)
    return path


def latest(directory: str, rank: int) -> Optional[str]:
    if not os.path.isdir(directory):
        return None
    c = sorted(f for f in os.listdir(directory) if f.endswith(f"_rank{rank:03d}.pt"))
    return os.path.join(directory, c[-1]) if c else None


def load(path: str, flat=None, opt_state: Optional[dict] = None, server=None) -> dict:
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if flat is not None and "params" in obj:
        with torch.no_grad():
            flat.flat[: flat.numel].copy_(obj["params"].to(flat.flat.device))
    if opt_state is not None and "opt_state" in obj:
        for k, v in obj["opt_state"].items():
            if isinstance(v, torch.Tensor) and isinstance(opt_state.get(k), torch.Tensor):
                opt_state[k].copy_(v.to(opt_state[k].device))
            else:
                opt_state[k] = v
    if server is not None and "server" in obj:
        server.load_state_dict(obj["server"])
    return obj
