"""Object (de)serialisation for sending arbitrary objects (mpiT.serialize / deserialize,
init.lua:111-132, which went through torch.MemoryFile). Here: ``torch.save`` into a byte
buffer and back with ``weights_only=True`` — no code runs while loading a received blob.
Tensors, numbers, strings, lists, tuples and dicts round-trip."""
from __future__ import annotations

import io

import torch


def serialize(obj) -> torch.Tensor:
    buf = io.BytesIO()
    torch.save(obj, buf)
    return torch.frombuffer(bytearray(buf.getvalue()), dtype=torch.uint8)


def deserialize(t: torch.Tensor):
    data = t.detach().cpu().contiguous().numpy().tobytes()
    return torch.load(io.BytesIO(data), weights_only=True)
