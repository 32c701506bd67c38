"""Weight-gradient GEMMs on a side HIP stream, overlapped with the memory-bound BatchNorm / data-gradient chain.

In a ResNet backward the data gradient of layer L is on the critical path (layer L-1 needs it) while layer L's
weight gradient is only needed by the optimizer at the end of the step.  The direct-gradient convolutions
(ops/conv.py, ops/conv1x1.py) hand their weight-gradient launch to :func:`run`: it forks from the current
stream with an event, runs the launch on the device's side stream, and pins the operand tensors to that stream
(``record_stream``) so the caching allocator does not recycle them early.  :func:`join`, queued as an autograd
end-of-backward callback (and called again by the executor before the optimizer), makes the main stream wait
for every side launch.  Inside hipGraph capture the fork and join are captured as graph edges.  ``PLX_WGRAD_STREAM=0``
runs every launch inline (A/B: the serialized backward, profiles/r5_backward_contention.md).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable

import torch

_side: Dict[int, "torch.cuda.Stream"] = {}
_pending: Dict[int, bool] = {}


_ENABLED = os.environ.get("PLX_WGRAD_STREAM", "1") != "0"


def enabled() -> bool:
    return _ENABLED


def capturing() -> bool:
    return torch.cuda.is_current_stream_capturing()


def priority_stream(idx: int, priority: int) -> "torch.cuda.Stream":
    """A HIP stream created with ``hipStreamCreateWithPriority`` (lower = higher priority; HIP maps -1 / 0 / 1 to
    the high / normal / low hardware-queue priority, which the command processor uses when it picks the next queue
    to dispatch workgroups from).  torch clamps ``torch.cuda.Stream(priority=)`` to the range HIP reports, which is
    not the full one on every ROCm release, hence the direct call."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    handle = ctypes.c_void_p()
    with torch.cuda.device(idx):
        # hipStreamNonBlocking (1), as torch's own streams: a blocking stream would synchronise with every launch on
        # the null stream, the main stream of the step when it is the caller's
        rc = hip.hipStreamCreateWithPriority(ctypes.byref(handle), ctypes.c_uint(1), ctypes.c_int(priority))
    if rc != 0:
        raise RuntimeError(f"hipStreamCreateWithPriority failed ({rc})")
    return torch.cuda.ExternalStream(handle.value, device=torch.device("cuda", idx))


# The side stream is created with low HIP priority (1).  HIP keeps a hardware-queue pool per priority level, so a low-priority side stream gets a queue
# of its own even when the compute stream, RCCL's streams and torch's share the box's 4 (GPU_MAX_HW_QUEUES) normal
# queues: with a live communicator and 4 queues the default-priority side stream landed on the compute stream's queue
# and the two serialised (ResNet-50 bench 10.65k / 10.68k trials/h), low priority 11.52k, 8 queues 11.54k
# (profiles/r5_hw_queues.md)
_WGRAD_PRIORITY = 1


def _stream_for(dev: torch.device) -> "torch.cuda.Stream":
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        # (a CU-masked side stream, hipExtStreamCreateWithCUMask, was removed in round 5: it cannot take a priority,
        # so it shares the compute stream's hardware queue and serialises with it, -29 %,
        # profiles/r5_wgrad_cumask_ab.jsonl; round 3 measured it slower too)
        s = _side[idx] = priority_stream(idx, _WGRAD_PRIORITY)
    return s


def stream_for(dev: torch.device) -> "torch.cuda.Stream":
    """The device's side stream (created on first use)."""
    return _stream_for(dev)


def run(fn: Callable[[], None], tensors: Iterable[torch.Tensor], dev: torch.device) -> None:
    if not enabled() or dev.type != "cuda":
        fn()
        return
    main = torch.cuda.current_stream(dev)
    side = _stream_for(dev)
    side.wait_stream(main)  # operands (dy, x) and the gradient slot are ready in main-stream order
    with torch.cuda.stream(side):
        fn()
    # the operands must not be recycled before the side stream has read them -- during hipGraph capture too: the
    # capture's private pool DOES hand a block freed by the main stream to a later allocation of the same capture, and
    # in the graph that later kernel then overwrote dy / x under the concurrently replayed weight gradient (garbage
    # gradients, the graph check's NaN since round 3).  A recorded block freed during capture is held until the
    # capture ends (the allocator defers its reuse), which is what the graph needs.
    for t in tensors:
        t.record_stream(side)
    idx = side.device.index
    if not _pending.get(idx):
        _pending[idx] = True
        # join at the end of this backward pass, so every caller (executor, tests, user loops) reads complete
        # gradients; the executor's explicit join() before the optimizer is then a no-op
        torch.autograd.Variable._execution_engine.queue_callback(lambda d=dev: join(d))


def busy(dev: torch.device) -> bool:
    """Has this backward queued side-stream work that the end-of-backward join has not yet covered?"""
    if dev.type != "cuda":
        return False
    return bool(_pending.get(dev.index if dev.index is not None else torch.cuda.current_device()))


def fence(stream: "torch.cuda.Stream", dev: torch.device) -> None:
    """``stream`` waits for every side-stream launch queued so far on this device, without stalling the main stream:
    a consumer of flat-slot gradients that runs before the end-of-backward join (FlatDDP's bucket all-reduce, fired by
    the parameter's post-accumulate hook as soon as the op that queued its weight gradient returns) must not read the
    slot before the side stream has written it."""
    if dev.type != "cuda":
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if _pending.get(idx):
        stream.wait_stream(_side[idx])


def join(dev: torch.device) -> None:
    """Main stream waits for every side-stream weight-gradient launch of this device."""
    if dev.type != "cuda":
        return
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if _pending.get(idx):
        torch.cuda.current_stream(dev).wait_stream(_side[idx])
        _pending[idx] = False
