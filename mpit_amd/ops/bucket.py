"""K12: gradient bucketing / unbucketing — many tensors <-> one flat buffer in one launch.

A :class:`PackPlan` is built once for a list of tensors and a flat buffer (offsets are
element offsets into the flat buffer). ``pack()`` gathers the tensors into the buffer
(optionally scaling — K14's ``g /= B`` fused in — and casting fp32<->bf16); ``unpack()``
scatters back. The chunk table lives on the device, so each call is a single kernel
launch (csrc/kernels/multi_copy.hip) regardless of the number of tensors.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from .._ext import native

_CHUNK = 1 << 15  # elements per workgroup work item


class PackPlan:
    def __init__(self, tensors: Sequence[torch.Tensor], flat: torch.Tensor, offsets: Sequence[int] | None = None):
        if offsets is None:
            offsets, o = [], 0
            for t in tensors:
                offsets.append(o)
                o += t.numel()
        total = max((o + t.numel() for o, t in zip(offsets, tensors)), default=0)
        if total > flat.numel():
            raise ValueError("flat buffer too small for the tensors")
        for t in tensors:
            if not t.is_contiguous():
                raise ValueError("PackPlan needs contiguous tensors")
            if t.device != flat.device:
                raise ValueError("tensors and flat buffer must share a device")
        self.tensors: List[torch.Tensor] = list(tensors)
        self.flat = flat
        self.offsets = list(offsets)
        self._tables = {}

    def _table(self, to_flat: bool) -> torch.Tensor:
        tab = self._tables.get(to_flat)
        if tab is not None:
            return tab
        fes = self.flat.element_size()
        rows = []
        for t, off in zip(self.tensors, self.offsets):
            n, tes = t.numel(), t.element_size()
            tb = t.dtype == torch.bfloat16
            fb = self.flat.dtype == torch.bfloat16
            for s in range(0, n, _CHUNK):
                m = min(_CHUNK, n - s)
                ta = t.data_ptr() + s * tes
                fa = self.flat.data_ptr() + (off + s) * fes
                if to_flat:
                    rows.append((ta, fa, m, (1 if tb else 0) | (2 if fb else 0)))
                else:
                    rows.append((fa, ta, m, (1 if fb else 0) | (2 if tb else 0)))
        # CopyChunk = {u64 src, u64 dst, i64 n, i32 flags, i32 pad}; user-space addresses
        # are < 2^47 so they fit int64; flags land in the low (little-endian) half.
        arr = np.array(rows, dtype=np.int64).reshape(-1, 4)
        assert native().COPY_CHUNK_BYTES == 32
        tab = torch.from_numpy(arr).to(self.flat.device)
        self._tables[to_flat] = tab
        return tab

    def _run(self, to_flat: bool, scale: float):
        tab = self._table(to_flat)
        m = native()
        if self.flat.is_cuda:
            dev = self.flat.device.index
            stream = torch.cuda.current_stream(self.flat.device).cuda_stream
        else:
            dev, stream = -1, 0
        m.multi_copy(dev, stream, tab.data_ptr(), tab.shape[0], float(scale))

    def pack(self, scale: float = 1.0):
        """flat[off_i : off_i+n_i] = scale * tensors[i] for all i (one launch)."""
        self._run(True, scale)
        return self.flat

    def unpack(self, scale: float = 1.0):
        """tensors[i] = scale * flat[off_i : off_i+n_i] for all i (one launch)."""
        self._run(False, scale)
        return self.tensors
