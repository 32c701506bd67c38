"""Flat parameter storage: every parameter of a module becomes a view into ONE fp32 buffer.

Why (MI355X-first): the optimizer step then touches three contiguous buffers (params, grads, state) with
one vectorised HIP kernel (``plx_sgd_flat`` / ``plx_adamw_flat``) instead of ~160 tensors × several
foreach launches; re-initialising a trial's weights is one ``plx_init_flat`` launch; snapshotting a trial
for Hyperband *resume* is one device-to-device copy of a contiguous buffer; and every pointer is fixed for
the life of the executor, so a captured hipGraph stays valid across trials.

Layout: parameters that take weight decay (ndim > 1: conv / linear weights) come first, the rest
(BN affine, biases) after, each segment padded to 4 floats so the kernels can use float4 accesses.
4-D conv weights get channels_last strides inside the flat buffer so MIOpen's NHWC kernels read them
without a layout transform, and their ``.grad`` aliases the flat gradient buffer with the same strides.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn as nn

_KIND = {"normal": 0, "const": 1, "uniform": 2}
CHUNK = 16384


def _contig_strides(shape) -> Tuple[int, ...]:
    strides, acc = [], 1
    for s in reversed(shape):
        strides.append(acc)
        acc *= s
    return tuple(reversed(strides))


def _cl_strides(shape) -> Tuple[int, ...]:
    n, c, h, w = shape
    return (h * w * c, 1, w * c, c)


def _pad4(n: int) -> int:
    return (n + 3) & ~3


@dataclass
class Segment:
    name: str
    offset: int
    numel: int
    shape: Tuple[int, ...]
    strides: Tuple[int, ...]
    decay: bool


def direct_grad(p: torch.Tensor):
    """The flat gradient slot a native op may accumulate ``p``'s gradient into itself, or None (autograd's)."""
    if getattr(p, "_plx_direct_grad", False):
        return p.grad
    return None


class FlatParams:
    """Re-home ``module``'s parameters into flat fp32 ``params``/``grads`` buffers on ``device``.

    ``lp_dtype=torch.bfloat16`` (the language models): the weight-decayed segment (every matrix: embeddings,
    projections) is presented to the model as bf16 views into ``lp_params`` with bf16 gradients in
    ``lp_grads``; ``params`` stays the fp32 master copy the optimizer updates (``plx_adamw_mixed`` rewrites
    ``lp_params`` in the same pass).  The 1-D tail (norm weights, biases) keeps fp32 params and fp32 grads
    (``grads`` then holds only that tail: ``grad_view`` maps flat offsets).  Autocast then has no weight to
    cast and autograd no gradient to cast back: per Llama-3 8B step that removes ~580 cast kernels and a
    fp32 read-modify-write of every gradient (profiles/r1_llama3_8b_*), and DP all-reduces move bf16.
    """

    def __init__(self, module: nn.Module, device: torch.device, channels_last: bool = True,
                 lp_dtype: torch.dtype = None):
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        decay = [(n, p) for n, p in named if p.dim() > 1]
        no_decay = [(n, p) for n, p in named if p.dim() <= 1]
        self.segments: List[Segment] = []
        off = 0
        for group, is_decay in ((decay, True), (no_decay, False)):
            for n, p in group:
                strides = (_cl_strides(p.shape) if (channels_last and p.dim() == 4)
                           else _contig_strides(p.shape))
                self.segments.append(Segment(n, off, p.numel(), tuple(p.shape), strides, is_decay))
                off += _pad4(p.numel())
            if is_decay:
                self.n_decay = off
        if not decay:
            self.n_decay = 0
        self.numel = off
        self.device = torch.device(device)
        self.lp_dtype = lp_dtype
        self.params = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        if lp_dtype is not None:
            self.lp_params = torch.zeros(self.n_decay, dtype=lp_dtype, device=self.device)
            self.lp_grads = torch.zeros(self.n_decay, dtype=lp_dtype, device=self.device)
            self.grad_base = self.n_decay
        else:
            self.lp_params = self.lp_grads = None
            self.grad_base = 0
        self.grads = torch.zeros(self.numel - self.grad_base, dtype=torch.float32, device=self.device)
        by_name: Dict[str, nn.Parameter] = dict(named)
        self._views: Dict[str, torch.Tensor] = {}
        self._master: Dict[str, torch.Tensor] = {}
        with torch.no_grad():
            for seg in self.segments:
                old = by_name[seg.name]
                master = self.params.as_strided(seg.shape, seg.strides, seg.offset)
                master.copy_(old.detach().to(self.device))
                self._master[seg.name] = master
                if lp_dtype is not None and seg.decay:
                    newp = nn.Parameter(self.lp_params.as_strided(seg.shape, seg.strides, seg.offset))
                    newp.grad = self.lp_grads.as_strided(seg.shape, seg.strides, seg.offset)
                else:
                    newp = nn.Parameter(master)
                    newp.grad = self.grads.as_strided(seg.shape, seg.strides, seg.offset - self.grad_base)
                newp._plx_flat = self
                self._set(module, seg.name, newp)
                self._views[seg.name] = newp
        self._written = set()
        self.sync_lp()
        module.to(self.device)  # buffers (BN running stats)

    # ------------------------------------------------------------------ mixed precision (lp mode)
    def sync_lp(self) -> None:
        """Refresh the bf16 model weights from the fp32 master (after init / load / broadcast)."""
        if self.lp_params is None or self.n_decay == 0:
            return
        if self.params.is_cuda:
            from polyaxon_amd.ops import _native

            _native.check(_native.lib("plx_train").plx_cast_lp(
                self.params.data_ptr(), self.lp_params.data_ptr(), self.n_decay,
                torch.cuda.current_stream(self.device).cuda_stream), "plx_cast_lp")
        else:
            with torch.no_grad():
                self.lp_params.copy_(self.params[: self.n_decay])

    def grad_view(self, lo: int, hi: int) -> torch.Tensor:
        """Gradient elements [lo, hi) of the flat layout (never straddling the bf16 / fp32 boundary)."""
        if self.lp_grads is None:
            return self.grads[lo:hi]
        if hi <= self.n_decay:
            return self.lp_grads[lo:hi]
        if lo >= self.n_decay:
            return self.grads[lo - self.n_decay: hi - self.n_decay]
        raise ValueError(f"grad range [{lo}, {hi}) straddles the bf16/fp32 boundary at {self.n_decay}")

    def zero_grads(self) -> None:
        self.grads.zero_()
        if self.lp_grads is not None:
            self.lp_grads.zero_()
        self._written.clear()

    def mark_written(self, slot: torch.Tensor) -> bool:
        """Direct-gradient GEMMs (ops/lm.py): record that ``slot`` holds this step's gradient; True if it
        already did (then the GEMM accumulates)."""
        key = slot.data_ptr()
        seen = key in self._written
        self._written.add(key)
        return seen

    def grads_consumed(self) -> None:
        """The optimizer zeroed the gradient buffers: the next direct write of every slot overwrites."""
        self._written.clear()

    def master(self, name: str) -> torch.Tensor:
        return self._master[name]

    @staticmethod
    def _set(module: nn.Module, dotted: str, value: nn.Parameter) -> None:
        parts = dotted.split(".")
        for part in parts[:-1]:
            module = getattr(module, part)
        setattr(module, parts[-1], value)

    def enable_direct_grads(self, on: bool = True) -> None:
        """Let the native ops accumulate weight gradients straight into the flat gradient buffer (their backward
        then returns None for the weight, so autograd runs no per-parameter ``grad += g`` kernel: ~160 launches and
        a read-modify-write of every gradient per ResNet-50 step).  Off for :class:`FlatDDP`, whose bucket
        readiness rides on autograd's post-accumulate hooks."""
        for p in self._views.values():
            p._plx_direct_grad = on

    def parameter(self, name: str) -> nn.Parameter:
        return self._views[name]

    def segment_of(self, param: torch.Tensor) -> Segment:
        for seg in self.segments:
            if self._views[seg.name] is param:
                return seg
        raise KeyError("parameter is not part of this FlatParams")

    # ------------------------------------------------------------------ fused re-init tables
    def init_tables(self, init_spec) -> Dict[str, torch.Tensor]:
        """Chunk tables for ``plx_init_flat`` from (param, kind, scale) triples (model.init_spec())."""
        kinds, scales, lo, hi, seg_id = [], [], [], [], []
        for i, (p, kind, scale) in enumerate(init_spec):
            seg = self.segment_of(p)
            kinds.append(_KIND[kind])
            scales.append(float(scale))
            start, end = seg.offset, seg.offset + seg.numel
            for c in range(start, end, CHUNK):
                lo.append(c)
                hi.append(min(c + CHUNK, end))
                seg_id.append(i)
        dev = self.device
        return {
            "chunk_lo": torch.tensor(lo, dtype=torch.int64, device=dev),
            "chunk_hi": torch.tensor(hi, dtype=torch.int64, device=dev),
            "chunk_seg": torch.tensor(seg_id, dtype=torch.int32, device=dev),
            "seg_kind": torch.tensor(kinds, dtype=torch.int32, device=dev),
            "seg_scale": torch.tensor(scales, dtype=torch.float32, device=dev),
        }

    def init_reference(self, init_spec, seed: int) -> None:
        """CPU / numerics-reference re-initialiser (torch RNG; distributions match the kernel)."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        with torch.no_grad():
            for p, kind, scale in init_spec:
                if kind == "normal":
                    v = torch.randn(p.shape, generator=g) * scale
                elif kind == "const":
                    v = torch.full(p.shape, float(scale))
                else:
                    v = (torch.rand(p.shape, generator=g) * 2 - 1) * scale
                self._master[self.segment_of(p).name].copy_(v.to(p.device))
        self.sync_lp()
