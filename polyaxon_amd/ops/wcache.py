"""Per-step bf16 copies of every convolution weight, made by ONE launch (``plx_weight_prep_all``).

The native convolutions (:mod:`polyaxon_amd.ops.conv1x1`, :mod:`polyaxon_amd.ops.conv`) need each fp32 master
weight as a bf16 forward operand ``Wf[Cout][taps][Cin]`` and a bf16 data-gradient operand ``Wd[Cin][taps][Cout]``.
Made per layer, that is 52 small launches per ResNet-50 step, each too small to fill the chip (≈0.33 ms of the
main stream in ``profiles/r2_resnet50_*``).  The resident executor instead refreshes this cache once at the top of
every step: one launch over a segment table that covers every native conv weight of the model (one block per
32×32 tile of one tap, so ≈23k blocks), writing into two persistent bf16 buffers whose addresses never change —
the captured hipGraph replays it like any other node.  While the cache is active (between :meth:`activate` and
:meth:`deactivate`) the conv ops take their operands from it instead of preparing them.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from polyaxon_amd.ops import _native

_ACTIVE: Optional["ConvWeightCache"] = None


class _WSeg(ctypes.Structure):
    _fields_ = [("src", ctypes.c_int64), ("dst_f", ctypes.c_int64), ("dst_d", ctypes.c_int64),
                ("cout", ctypes.c_int32), ("cin", ctypes.c_int32), ("taps", ctypes.c_int32), ("tile0", ctypes.c_int32)]


assert ctypes.sizeof(_WSeg) == 40  # csrc/conv_gemm.hip WSeg


def lookup(weight: torch.Tensor) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """(Wf, Wd) bf16 views for ``weight`` from the active cache, or None (the op prepares its own)."""
    c = _ACTIVE
    if c is None:
        return None
    return c.views.get(weight.data_ptr())


class ConvWeightCache:
    def __init__(self, model: nn.Module, params: torch.Tensor):
        """``params``: the flat fp32 buffer the conv weights are views of (ops.flat.FlatParams.params)."""
        from polyaxon_amd.ops.conv import ConvKxK
        from polyaxon_amd.ops.conv1x1 import Conv1x1

        self.params = params
        dev = params.device
        base = params.data_ptr()
        end = base + params.numel() * 4
        segs, metas = [], []
        nf = tiles = 0
        for mod in model.modules():
            if not isinstance(mod, (Conv1x1, ConvKxK)) or not mod.native:
                continue
            w = mod.weight
            cout, cin, kh, kw = w.shape
            if kh != kw or cin % 64 or cout % 64 or w.dtype != torch.float32:
                continue
            # the flat buffer keeps conv weights channels_last: memory order [cout][kh][kw][cin] = [cout][tap][cin]
            if kh > 1 and w.stride() != (kh * kw * cin, 1, kw * cin, cin):
                continue
            if not (base <= w.data_ptr() < end):
                continue
            taps = kh * kw
            n = w.numel()
            segs.append(_WSeg((w.data_ptr() - base) // 4, nf, nf, cout, cin, taps, tiles))
            metas.append((w.data_ptr(), cout, cin, taps, nf))
            nf += n
            tiles += taps * ((cout + 31) // 32) * ((cin + 31) // 32)
        self.total_tiles = tiles
        self.nseg = len(segs)
        self.wf = torch.empty(max(nf, 1), dtype=torch.bfloat16, device=dev)
        self.wd = torch.empty(max(nf, 1), dtype=torch.bfloat16, device=dev)
        raw = (_WSeg * max(len(segs), 1))(*segs)
        table = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
        self.table = table.to(dev)
        self.views: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        for ptr, cout, cin, taps, off in metas:
            n = cout * cin * taps
            wf = self.wf[off: off + n]
            wd = self.wd[off: off + n]
            if taps == 1:
                self.views[ptr] = (wf.view(cout, cin), wd.view(cin, cout))
            else:
                self.views[ptr] = (wf.view(cout, taps, cin), wd.view(cin, taps, cout))

    def __len__(self) -> int:
        return self.nseg

    def refresh(self) -> None:
        """Re-derive every cached operand from the current fp32 weights (one launch on the current stream)."""
        if self.nseg == 0:
            return
        rc = _native.lib("plx_conv").plx_weight_prep_all(
            self.params.data_ptr(), self.wf.data_ptr(), self.wd.data_ptr(), self.table.data_ptr(), self.nseg,
            self.total_tiles, torch.cuda.current_stream(self.params.device).cuda_stream)
        _native.check(rc, "plx_weight_prep_all")

    def activate(self) -> None:
        """Refresh and let the conv ops read from the cache (until :meth:`deactivate`)."""
        global _ACTIVE
        self.refresh()
        _ACTIVE = self

    @staticmethod
    def deactivate() -> None:
        global _ACTIVE
        _ACTIVE = None
