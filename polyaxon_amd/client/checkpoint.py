"""Asynchronous checkpointing for trials.

``AsyncCheckpointer.save(tensors, name)`` snapshots device tensors into pinned host buffers on a side
stream (the training stream is not blocked; the buffers are reused between saves), and a background
thread waits for the copy event and writes a safetensors file into POLYAXON_RUN_OUTPUTS_PATH atomically
(write to ``.tmp`` then rename).  With Hyperband ``resume: true`` the promoted experiment shares the
original's outputs path, so ``load`` picks up where the lower rung stopped.
"""
from __future__ import annotations

import os
import queue
import threading
from typing import Dict, Optional

import torch


class AsyncCheckpointer:
    def __init__(self, directory: Optional[str] = None):
        self.dir = directory or os.environ.get("POLYAXON_RUN_OUTPUTS_PATH") or "."
        os.makedirs(self.dir, exist_ok=True)
        self._pinned: Dict[str, torch.Tensor] = {}
        self._q: "queue.Queue" = queue.Queue()
        self._stream = None
        self._thread = threading.Thread(target=self._writer, name="plx-ckpt", daemon=True)
        self._thread.start()
        self.saved = []

    def _buf(self, key: str, t: torch.Tensor) -> torch.Tensor:
        b = self._pinned.get(key)
        if b is None or b.shape != t.shape or b.dtype != t.dtype:
            b = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
            self._pinned[key] = b
        return b

    def save(self, tensors: Dict[str, torch.Tensor], name: str = "checkpoint", meta: Optional[Dict] = None) -> None:
        self.wait()  # one checkpoint in flight keeps the pinned buffers single-buffered
        host = {}
        event = None
        cuda = [t for t in tensors.values() if t.is_cuda]
        if cuda:
            dev = cuda[0].device
            if self._stream is None:
                self._stream = torch.cuda.Stream(dev)
            self._stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self._stream):
                for k, t in tensors.items():
                    b = self._buf(k, t)
                    b.copy_(t.detach(), non_blocking=True)
                    host[k] = b
                event = torch.cuda.Event()
                event.record(self._stream)
        else:
            host = {k: t.detach().clone() for k, t in tensors.items()}
        self._q.put((event, host, name, dict(meta or {})))

    def _writer(self) -> None:
        from safetensors.torch import save_file

        while True:
            event, host, name, meta = self._q.get()
            try:
                if event is not None:
                    event.synchronize()
                path = os.path.join(self.dir, f"{name}.safetensors")
                tmp = path + ".tmp"
                save_file({k: v.contiguous() for k, v in host.items()}, tmp,
                          metadata={k: str(v) for k, v in meta.items()})
                os.replace(tmp, path)
                self.saved.append(path)
            finally:
                self._q.task_done()

    def wait(self) -> None:
        self._q.join()

    def load(self, name: str = "checkpoint", device=None) -> Optional[Dict[str, torch.Tensor]]:
        from safetensors.torch import load_file

        path = os.path.join(self.dir, f"{name}.safetensors")
        if not os.path.exists(path):
            return None
        return load_file(path, device=str(device) if device is not None else "cpu")

    def meta(self, name: str = "checkpoint") -> Dict[str, str]:
        from safetensors import safe_open

        path = os.path.join(self.dir, f"{name}.safetensors")
        with safe_open(path, framework="pt") as f:
            return dict(f.metadata() or {})
