"""Fused flat-buffer optimizers with device-resident hyper-parameters.

The hyper-parameters (lr, momentum, weight decay, ...) live in a small fp32 device tensor that the kernel
reads at run time.  A trial executor therefore changes a trial's hyper-parameters with one 32-byte H2D
copy and keeps replaying the SAME captured hipGraph — the graph never has to be re-captured per trial,
which is what makes a warm per-GPU trial executor cheap (SURVEY.md §7.1 polyflow; BASELINE.md "reference
design constants": every reference trial pays pod start + 1 s task hops instead).

On CPU (no native library) the same update is computed with torch ops; tests compare the two.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.flat import FlatParams


def _stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class _PinnedRing:
    """Preallocated pinned staging slots for the per-trial hyper-parameter H2D copies.  ``tensor.pin_memory()``
    per call went through the caching host allocator, which allocates fresh pinned memory (a synchronising
    hipHostMalloc) while earlier copies are still queued -- with the host running trials ahead of the GPU that
    stalled it, and the GPU then idled at every trial start waiting for the host's next launches.  A slot is
    reused only after the event recorded behind its copy has completed (it nearly always has: 64 trials later)."""

    def __init__(self, slots: int = 64, width: int = 8):
        self.buf = torch.zeros(slots, width, dtype=torch.float32).pin_memory()
        self.events = [None] * slots
        self.i = 0

    def copy_to(self, dst: torch.Tensor, values) -> None:
        i = self.i
        self.i = (i + 1) % len(self.events)
        ev = self.events[i]
        if ev is not None:
            ev.synchronize()
        self.buf[i, : len(values)] = torch.tensor(values, dtype=torch.float32)
        dst.copy_(self.buf[i, : dst.numel()], non_blocking=True)
        ev = self.events[i] or torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dst.device))
        self.events[i] = ev


def _set_hp(opt, values) -> None:
    if not opt.hp.is_cuda:
        opt.hp.copy_(torch.tensor(values, dtype=torch.float32))
        return
    ring = getattr(opt, "_ring", None)
    if ring is None:
        ring = opt._ring = _PinnedRing(width=opt.hp.numel())
    ring.copy_to(opt.hp, values)


class FusedSGD:
    """SGD with momentum / nesterov / dampening and weight decay on the decay segment only."""

    HP = ("lr", "momentum", "weight_decay", "nesterov", "dampening")

    def __init__(self, flat: FlatParams, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4,
                 nesterov: bool = False, dampening: float = 0.0, step_counter: Optional[torch.Tensor] = None):
        self.flat = flat
        dev = flat.device
        self.momentum_buf = torch.zeros_like(flat.params)
        self.hp = torch.zeros(8, dtype=torch.float32, device=dev)
        # step counter shared with the metric ring: 0 right after reset() => momentum := grad
        self.step = step_counter if step_counter is not None else torch.zeros(1, dtype=torch.int32, device=dev)
        self.set_hparams(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov,
                         dampening=dampening)

    def set_hparams(self, **hp) -> None:
        vals = getattr(self, "_hp_host", {k: 0.0 for k in self.HP})
        for k, v in hp.items():
            if k not in self.HP:
                raise KeyError(f"unknown SGD hyper-parameter {k!r}")
            vals[k] = float(v)
        self._hp_host = vals
        _set_hp(self, [vals[k] for k in self.HP] + [0.0] * (8 - len(self.HP)))

    def reset_state(self) -> None:
        if self.flat.params.is_cuda:
            _native.check(_native.lib("plx_train").plx_zero_flat(
                self.momentum_buf.data_ptr(), self.momentum_buf.numel(), _stream_ptr(self.hp)), "plx_zero_flat")
        else:
            self.momentum_buf.zero_()

    def step_(self) -> None:
        f = self.flat
        f.grads_consumed()
        if f.lp_params is not None:
            raise NotImplementedError("FusedSGD has no mixed-precision (lp) flat mode; use FusedAdamW")
        if f.params.is_cuda:
            rc = _native.lib("plx_train").plx_sgd_flat(
                f.params.data_ptr(), f.grads.data_ptr(), self.momentum_buf.data_ptr(), f.numel, f.n_decay,
                self.hp.data_ptr(), self.step.data_ptr(), _stream_ptr(f.params))
            _native.check(rc, "plx_sgd_flat")
        else:
            self._step_reference()

    @torch.no_grad()
    def _step_reference(self) -> None:
        f = self.flat
        lr, mom, wd, nest, damp = (float(self.hp[i]) for i in range(5))
        g = f.grads.clone()
        g[: f.n_decay] += wd * f.params[: f.n_decay]
        if int(self.step.item()) == 0:
            self.momentum_buf.copy_(g)
        else:
            self.momentum_buf.mul_(mom).add_(g, alpha=1.0 - damp)
        d = g + mom * self.momentum_buf if nest else self.momentum_buf
        f.params.sub_(lr * d)
        f.grads.zero_()

    def state_buffers(self) -> Dict[str, torch.Tensor]:
        return {"momentum": self.momentum_buf}


class FusedAdamW:
    HP = ("lr", "beta1", "beta2", "eps", "weight_decay")

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, step_counter: Optional[torch.Tensor] = None):
        self.flat = flat
        dev = flat.device
        self.exp_avg = torch.zeros_like(flat.params)
        self.exp_avg_sq = torch.zeros_like(flat.params)
        self.hp = torch.zeros(8, dtype=torch.float32, device=dev)
        self.step = step_counter if step_counter is not None else torch.zeros(1, dtype=torch.int32, device=dev)
        self.set_hparams(lr=lr, beta1=betas[0], beta2=betas[1], eps=eps, weight_decay=weight_decay)

    def set_hparams(self, **hp) -> None:
        vals = getattr(self, "_hp_host", {k: 0.0 for k in self.HP})
        for k, v in hp.items():
            if k not in self.HP:
                raise KeyError(f"unknown AdamW hyper-parameter {k!r}")
            vals[k] = float(v)
        self._hp_host = vals
        _set_hp(self, [vals[k] for k in self.HP] + [0.0] * (8 - len(self.HP)))

    def reset_state(self) -> None:
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()

    def shard_state(self, numel: int) -> None:
        """ZeRO-1 (FlatDDP(shard_optimizer=True)): keep the moments only for the ``numel`` flat elements this rank
        updates, packed; every update then names its range's offset in that packed state (``step_range_(state_off=)``).
        The full-size moments are released."""
        dev = self.flat.device
        self.exp_avg = torch.zeros(numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(numel, dtype=torch.float32, device=dev)
        self.sharded = True

    sharded = False

    # set by FlatDDP(optimizer=...): the update runs per gradient bucket during the backward (step_range_), and
    # step_() only closes the step's bookkeeping
    in_backward = False

    def step_(self) -> None:
        f = self.flat
        f.grads_consumed()  # every kernel below zeroes the gradients it reads
        if self.in_backward:
            return  # every bucket was already updated (FlatDDP.finish joined the optimizer stream)
        if self.sharded:
            raise RuntimeError("sharded AdamW state is updated per bucket by FlatDDP; step_() alone would skip it")
        if not f.params.is_cuda:
            self._step_reference()
            return
        lib = _native.lib("plx_train")
        st = _stream_ptr(f.params)
        if f.lp_params is None:
            rc = lib.plx_adamw_flat(
                f.params.data_ptr(), f.grads.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                f.numel, f.n_decay, self.hp.data_ptr(), self.step.data_ptr(), st)
            _native.check(rc, "plx_adamw_flat")
            return
        # lp mode: bf16 decay segment (master fp32 + bf16 model copy) and the fp32 tail
        nd = f.n_decay
        if nd:
            _native.check(lib.plx_adamw_mixed(
                f.params.data_ptr(), f.lp_grads.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                f.lp_params.data_ptr(), nd, 1, self.hp.data_ptr(), self.step.data_ptr(), st), "plx_adamw_mixed")
        if f.numel > nd:
            off = nd * 4
            _native.check(lib.plx_adamw_flat(
                f.params.data_ptr() + off, f.grads.data_ptr(), self.exp_avg.data_ptr() + off,
                self.exp_avg_sq.data_ptr() + off, f.numel - nd, 0, self.hp.data_ptr(), self.step.data_ptr(), st),
                "plx_adamw_flat")

    def step_range_(self, lo: int, hi: int, stream: Optional[int] = None, state_off: Optional[int] = None) -> None:
        """AdamW over flat elements [lo, hi) on ``stream`` (a FlatDDP bucket: 4-aligned, and in lp mode entirely
        inside the bf16 decay segment or entirely inside the fp32 tail).  The same per-element update as
        :meth:`step_`; weight decay applies to the elements below ``n_decay``; the range's gradients are zeroed.
        ``state_off``: where the range's moments start in the packed (sharded) state; default ``lo``."""
        f = self.flat
        so = lo if state_off is None else state_off
        if not f.params.is_cuda:
            self._step_reference_range(lo, hi, so)
            return
        lib = _native.lib("plx_train")
        st = stream if stream is not None else _stream_ptr(f.params)
        nd, n = f.n_decay, hi - lo
        p, m, v = f.params.data_ptr() + 4 * lo, self.exp_avg.data_ptr() + 4 * so, self.exp_avg_sq.data_ptr() + 4 * so
        if f.lp_params is None:
            rc = lib.plx_adamw_flat(p, f.grads.data_ptr() + 4 * lo, m, v, n, max(0, min(hi, nd) - lo),
                                    self.hp.data_ptr(), self.step.data_ptr(), st)
            _native.check(rc, "plx_adamw_flat")
        elif hi <= nd:
            rc = lib.plx_adamw_mixed(p, f.lp_grads.data_ptr() + 2 * lo, m, v, f.lp_params.data_ptr() + 2 * lo, n, 1,
                                     self.hp.data_ptr(), self.step.data_ptr(), st)
            _native.check(rc, "plx_adamw_mixed")
        elif lo >= nd:
            rc = lib.plx_adamw_flat(p, f.grads.data_ptr() + 4 * (lo - nd), m, v, n, 0, self.hp.data_ptr(),
                                    self.step.data_ptr(), st)
            _native.check(rc, "plx_adamw_flat")
        else:
            raise ValueError(f"range [{lo}, {hi}) straddles the bf16/fp32 boundary at {nd}")

    @torch.no_grad()
    def _step_reference(self, lo: int = 0, hi: Optional[int] = None) -> None:
        f = self.flat
        if lo != 0 or (hi is not None and hi != f.numel):
            self._step_reference_range(lo, f.numel if hi is None else hi)
            return
        lr, b1, b2, eps, wd = (float(self.hp[i]) for i in range(5))
        t = int(self.step.item()) + 1
        g = f.grads if f.lp_grads is None else torch.cat([f.lp_grads.float(), f.grads])
        f.params[: f.n_decay].mul_(1.0 - lr * wd)
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        denom = (self.exp_avg_sq.sqrt() / bc2 ** 0.5).add_(eps)
        f.params.addcdiv_(self.exp_avg, denom, value=-lr / bc1)
        f.zero_grads()
        f.sync_lp()

    @torch.no_grad()
    def _step_reference_range(self, lo: int, hi: int, so: Optional[int] = None) -> None:
        """The reference update restricted to [lo, hi) (CPU).  It runs inside the backward (FlatDDP optimizer mode),
        so it writes through ``.data``: the parameters are views of the flat buffers and share their autograd version
        counter, which an in-place op on any slice would bump under the tensors other layers saved for backward (the
        native kernels write through pointers and never touch it)."""
        f = self.flat
        lr, b1, b2, eps, wd = (float(self.hp[i]) for i in range(5))
        t = int(self.step.item()) + 1
        so = lo if so is None else so
        g = f.grad_view(lo, hi).data
        p, m, v = f.params.data[lo:hi], self.exp_avg[so:so + hi - lo], self.exp_avg_sq[so:so + hi - lo]
        nd = max(0, min(hi, f.n_decay) - lo)
        if nd:
            p[:nd].mul_(1.0 - lr * wd)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        p.addcdiv_(m, (v.sqrt() / bc2 ** 0.5).add_(eps), value=-lr / bc1)
        g.zero_()
        if f.lp_params is not None and hi <= f.n_decay:
            f.lp_params.data[lo:hi].copy_(p)

    def state_buffers(self) -> Dict[str, torch.Tensor]:
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}
