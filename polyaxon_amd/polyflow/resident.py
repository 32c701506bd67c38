"""Resident trial executors: warm per-GPU worker processes that polyflow feeds Hyperband brackets over a socket.

Reference behaviour being replaced: every Hyperband trial -- including every promotion, which
the reference models as a *new* experiment resumed from the previous rung's outputs
(polyaxon/hpsearch/iteration_managers/hyperband.py:79-113) -- is a pod: build check, pod create, container start,
framework import, CUDA context, then user code, with a 1 s Celery hop per step and a 30 s poll at every rung
barrier (polyaxon/hpsearch/tasks/hyperband.py:48-83).  On one 8×MI355X node everything trial-invariant can stay
warm, so polyflow keeps **one resident executor per GPU**:

* the worker process (``python -m polyaxon_amd.polyflow.resident``) builds its *program* once
  (polyflow/programs.py: model, flat fp32 weights, fused optimizer, device data stream, optional hipGraph) and
  then trains trial after trial, re-initialising weights/optimizer state in place (polyflow/executor.py);
* the scheduler assigns whole **brackets** to executors (brackets are independent successive-halving runs, so
  they spread over GPUs with no cross-GPU barrier); an executor interleaves up to ``max_active_brackets`` of
  them in *rounds*: the current rung of every active bracket, then ONE ``plx_topk_brackets`` launch over the
  device-resident ``[brackets × configs]`` metric tensor decides every promotion of the round (and one
  ``plx_early_stop_any`` launch per rule set evaluates early stopping), with a single small D2H read;
* promotions with ``resume: true`` restore the config's HBM snapshot (the reference RESUME clone,
  db/models/experiments.py:225-316) instead of a checkpoint file round trip -- 288 GB of HBM holds hundreds of
  ResNet-50 trial states;
* ASHA groups (``hptuning.asha``) come as *shards*: an independent asynchronous successive-halving search over a
  set of configs, no rung barrier.  Every round a shard runs ONE job -- the best not-yet-promoted config in the
  top 1/eta of the highest rung that has one (RESUME from its HBM snapshot), else a new config at rung 0 -- and the
  round's single top-k launch (over the shard's ``[rungs × configs]`` device metric table, beside the Hyperband
  brackets' rows) gives the next round its rung rankings;
* a bracket or shard whose executor died can be re-sent with its progress (``start_rung``/``active`` for a
  bracket, ``history`` for a shard): the new executor continues from the last completed decision, re-training
  promoted configs from scratch (their snapshots died with the old process);
* every trial is still a Polyaxon experiment: the worker streams ``trial_start``/``trial_end``/``rung_done``
  events, and the scheduler thread (polyflow/groups.py ``ResidentHyperbandDriver``) writes the experiment rows,
  RESUME clones, FSM status history, metrics/``last_metric`` and iteration rows, while the GPU keeps running.

Protocol (length-prefixed JSON over a stream socket; ``Channel``):

  scheduler -> worker  {"op": "init", "program", "params", "max_active"} | {"op": "bracket", ...} |
                       {"op": "asha", ...} | {"op": "stop_bracket", "key"} | {"op": "pause", "tag"} | {"op": "shutdown"}
  worker -> scheduler  {"ev": "ready", ...} | {"ev": "trial_start", ...} | {"ev": "trial_end", ...} |
                       {"ev": "rung_done", ...} | {"ev": "bracket_done", ...} | {"ev": "paused", "tag"} |
                       {"ev": "error", ...}
"""
from __future__ import annotations

import argparse
import json
import math
import os
import select
import socket
import struct
import sys
import threading
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

_HDR = struct.Struct("!I")


class ChannelClosed(EOFError):
    pass


class Channel:
    """Length-prefixed JSON messages over a connected stream socket.  ``send`` is thread-safe; ``recv`` is meant
    for one reader."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self._wlock = threading.Lock()
        self._buf = b""
        self.closed = False

    @classmethod
    def connect(cls, host: str, port: int, timeout: float = 60.0) -> "Channel":
        end = time.time() + timeout
        while True:
            try:
                s = socket.create_connection((host, port), timeout=5.0)
                s.settimeout(None)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                return cls(s)
            except OSError:
                if time.time() > end:
                    raise
                time.sleep(0.1)

    def fileno(self) -> int:
        return self.sock.fileno()

    def send(self, msg: Dict[str, Any]) -> None:
        data = json.dumps(msg, allow_nan=True).encode()
        with self._wlock:
            self.sock.sendall(_HDR.pack(len(data)) + data)

    def _read_exact(self, n: int, timeout: Optional[float]) -> Optional[bytes]:
        while len(self._buf) < n:
            if timeout is not None:
                r, _, _ = select.select([self.sock], [], [], timeout)
                if not r:
                    return None
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                self.closed = True
                raise ChannelClosed("peer closed the channel")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def recv(self, timeout: Optional[float] = None) -> Optional[Dict[str, Any]]:
        """Next message; None if ``timeout`` (seconds, 0 = poll) passed without a complete header.  Once a
        header has arrived the body is read to completion.  Raises ChannelClosed at EOF."""
        hdr = self._read_exact(_HDR.size, timeout)
        if hdr is None:
            return None
        (n,) = _HDR.unpack(hdr)
        body = self._read_exact(n, None)
        return json.loads(body)

    def close(self) -> None:
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass


# ============================================================================ worker side
@dataclass
class _Bracket:
    key: str
    manager: Any                      # HyperbandSearchManager of the owning group (reference-exact arithmetic)
    iteration: int                    # Hyperband iteration = bracket index (bracket s = s_max - iteration)
    configs: Dict[int, Dict[str, Any]]
    resource_name: str
    resource: Any                     # ResourceConfig (cast_value)
    maximize: bool
    resume: bool
    seed: int
    rules: List[Tuple[int, float, bool]] = field(default_factory=list)   # early stopping on the program metric
    rung: int = 0
    active: List[int] = field(default_factory=list)
    prev_r: Dict[int, float] = field(default_factory=dict)
    stopped: bool = False
    early_stopped: bool = False


class _FixedBudget:
    """The manager of a ``trials`` unit (a BO batch, or any list of independent fixed-budget trials): one rung of
    ``units`` resource units, no promotion -- the bracket machinery runs it like a one-rung bracket."""

    def __init__(self, units: float):
        self.units = units

    def get_n_resources_for_iteration(self, iteration: int, rung: int) -> float:
        return self.units

    def get_n_config_to_keep_for_iteration(self, iteration: int, rung: int) -> int:
        return 0

    def should_reschedule(self, iteration: int, rung: int) -> bool:
        return True


class _Units:
    """Resource declaration of a ``trials`` unit: whole units stay ints in the trial's declarations."""

    @staticmethod
    def cast_value(v: float):
        return int(round(v)) if abs(v - round(v)) < 1e-9 else float(v)


@dataclass
class _AshaShard:
    """One asynchronous successive-halving search (Li et al. 2018, "Massively parallel hyperparameter tuning") over
    ``configs``: rungs k = 0..K-1 with resource min_r * eta^k (capped at max_r); a config enters rung k+1 once it is
    in the top floor(n_k / eta) of rung k's n_k results -- decided from the device top-k order of the rung table."""
    key: str
    configs: Dict[int, Dict[str, Any]]
    pending: List[int]                # configs not started yet (in suggestion order)
    n_rungs: int
    eta: float
    min_r: float
    max_r: float
    resource_name: str
    resource: Any
    maximize: bool
    resume: bool
    seed: int
    rules: List[Tuple[int, float, bool]] = field(default_factory=list)
    row0: int = -1                    # first row of this shard in the worker's ASHA metric table
    results: List[Dict[int, float]] = field(default_factory=list)      # rung -> {cid: metric} (host mirror)
    promoted: List[set] = field(default_factory=list)                  # rung -> cids promoted out of it
    snap_rung: Dict[int, int] = field(default_factory=dict)            # cid -> rung of its HBM snapshot
    order: List[List[int]] = field(default_factory=list)               # rung -> cids best first (last top-k)
    stopped: bool = False
    early_stopped: bool = False

    def r(self, rung: int):
        return self.resource.cast_value(min(self.min_r * self.eta ** rung, self.max_r))

    def next_job(self) -> Optional[Tuple[int, int]]:
        """(cid, rung) to run next, or None when the search has nothing runnable (it is then finished: jobs of a
        round all complete before the next decision)."""
        for rung in range(self.n_rungs - 2, -1, -1):
            k = int(len(self.results[rung]) / self.eta)
            for cid in self.order[rung][:k]:
                if cid not in self.promoted[rung]:
                    self.promoted[rung].add(cid)
                    return cid, rung + 1
        if self.pending:
            return self.pending.pop(0), 0
        return None


class ResidentWorker:
    """The GPU side.  Owns one TrialProgram; runs the brackets (and ASHA shards) it is handed, in rounds."""

    def __init__(self, program: str, params: Optional[Dict[str, Any]] = None, device=None, max_active: int = 8):
        # ASHA jobs per shard per round (A/B knob PLX_ASHA_JOBS): each round ends in one device->host read of the
        # round's results; one job per shard per round made that read a quarter of an ASHA sweep's wall time
        self.asha_jobs = max(1, int(os.environ.get("PLX_ASHA_JOBS", "4")))
        self.program_name = program
        self.params = dict(params or {})
        self.device = device
        self.max_active = max(1, int(max_active))
        self.program = None
        self.queue: List[_Bracket] = []
        self.active: List[_Bracket] = []
        self.asha_queue: List[_AshaShard] = []
        self.asha_active: List[_AshaShard] = []
        self.asha_metrics = None          # BracketMetrics: rung rows of every active shard
        self.pause_tag: Optional[str] = None
        self.metrics = None
        self.stats = {"trials": 0, "train_steps": 0, "rounds": 0, "topk_launches": 0, "early_stop_launches": 0,
                      "asha_jobs": 0,
                      # wall seconds: blocked waiting for work, inside rounds, and in each round's synchronising
                      # D2H read (host waiting for the GPU to finish the round's queued work)
                      "idle_s": 0.0, "round_s": 0.0, "sync_s": 0.0}
        self._base_ev = None
        self._base_wall = 0.0
        self._shutdown: Optional[str] = None
        self.gang: Optional[_GangGroup] = None

    def join_gang(self, rank: int, world: int, group=None) -> None:
        """Become rank ``rank`` of a DP gang (before ``build``): the program trains with FlatDDP over the gang,
        each rank on its own slice of the data stream.  ``group``: an existing process (sub)group of the ``world``
        ranks (bench.py's gangs inside its own world group); None: the gang's own rendezvous from the pool's env."""
        import torch

        if self.device is None:
            self.device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        if torch.device(self.device).type == "cuda":
            torch.cuda.set_device(self.device)
        self.gang = _GangGroup(rank, world, self.device, group=group)

    def close_gang(self) -> None:
        """Release the gang's framework communicator (the executor's FlatDDP hold and the metric mean's) and the
        rendezvous; a no-op outside a gang."""
        if self.gang is None:
            return
        ex = getattr(getattr(self, "program", None), "executor", None)
        if ex is not None and ex.ddp is not None:
            ex.ddp.close()
        self.gang.close()
        self.gang = None

    # ------------------------------------------------------------------ build
    def build(self) -> Dict[str, Any]:
        import torch

        from polyaxon_amd.polyflow.programs import build_program
        from polyaxon_amd.polytune.kernels import BracketMetrics

        from polyaxon_amd.client.budget import apply_hbm_budget

        t0 = time.time()
        if self.device is None:
            self.device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        if torch.device(self.device).type == "cuda":
            apply_hbm_budget(self.device)
        params = dict(self.params)
        if self.gang is not None:  # each rank draws its own batches of the same task
            params["data_seed"] = int(params.get("data_seed", 0)) + 1000003 * self.gang.rank
            params["graph"] = False  # the DP step runs eagerly (its collectives ride RCCL's own streams)
        self.program = build_program(self.program_name, params, self.device)
        if self.gang is not None:
            self.program.executor.enable_dp(process_group=self.gang.group)
        self.program.warm()
        ex = self.program.executor
        self.metrics = BracketMetrics(self.max_active, 32, ex.device)
        self._reset_clock()
        return {"ev": "ready", "program": self.program_name, "device": str(ex.device), "pid": os.getpid(),
                "dp_world": self.gang.world if self.gang is not None else 1,
                "build_s": round(time.time() - t0, 3), "snapshot_bytes": ex.snapshot_bytes(),
                "metric": self.program.metric, "unit_steps": self.program.unit_steps, "info": self.program.info,
                "hip_graph": ex.graph is not None, "graph_check_error": ex.graph_check_error,
                "device_name": torch.cuda.get_device_name(ex.device) if ex.is_cuda else "cpu"}

    def _reset_clock(self) -> None:
        import torch

        ex = self.program.executor
        if ex.is_cuda:
            torch.cuda.synchronize(ex.device)
            self._base_ev = torch.cuda.Event(enable_timing=True)
            self._base_ev.record()
            torch.cuda.synchronize(ex.device)
        self._base_wall = time.time()

    def _event(self):
        import torch

        if not self.program.executor.is_cuda:
            return time.time()
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _wall(self, ev) -> float:
        if isinstance(ev, float):
            return ev
        return self._base_wall + self._base_ev.elapsed_time(ev) / 1000.0

    # ------------------------------------------------------------------ messages
    def handle(self, msg: Dict[str, Any], chan: Channel) -> Optional[str]:
        op = msg.get("op")
        if op == "bracket":
            self.queue.append(self._make_bracket(msg))
        elif op == "asha":
            self.asha_queue.append(self._make_shard(msg))
        elif op == "trials":
            self.queue.append(self._make_trials(msg))
        elif op == "stop_bracket":
            for q in (self.queue, self.asha_queue):
                for br in list(q):
                    if br.key == msg["key"]:
                        q.remove(br)
                        chan.send({"ev": "bracket_done", "key": br.key, "status": "stopped"})
            for br in self.active + self.asha_active:
                if br.key == msg["key"]:
                    br.stopped = True
        elif op == "pause":
            self.pause_tag = str(msg.get("tag", ""))
        elif op == "shutdown":
            return "shutdown"
        elif op == "ping":
            chan.send({"ev": "pong", "stats": dict(self.stats)})
        elif op == "bo_suggest":
            # a DP gang's followers see every control message too, but only the leader's reply reaches the scheduler:
            # only rank 0 fits the GP and searches the acquisition
            if self.gang is None or self.gang.rank == 0:
                chan.send(self._bo_suggest(msg))
        elif op == "init":
            if msg.get("program") != self.program_name:
                chan.send({"ev": "error", "fatal": True,
                           "message": f"worker runs {self.program_name}, asked for {msg.get('program')}"})
                return "shutdown"
            chan.send(self._ready_info)
        else:
            chan.send({"ev": "error", "fatal": False, "message": f"unknown op {op!r}"})
        return None

    def _bo_suggest(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        """A BO group's next batch: GP fit + acquisition search with the HIP kernels on this executor's device (the
        scheduler that asks stays GPU-free), numpy on a CPU executor."""
        from polyaxon_amd.polytune.bo import suggest
        from polyaxon_amd.spec.hptuning import HPTuningConfig

        t0 = time.perf_counter()
        ex = self.program.executor
        backend = "hip" if ex.is_cuda else "numpy"
        out = suggest(HPTuningConfig.from_dict(msg["hptuning"]), list(msg["configs"]), list(msg["metrics"]),
                      int(msg["n"]), backend=backend)
        plain = [{k: (v.item() if hasattr(v, "item") else v) for k, v in s.items()} for s in out]
        return {"ev": "bo_suggestions", "key": msg["key"], "suggestions": plain, "backend": backend,
                "ms": round((time.perf_counter() - t0) * 1e3, 2)}

    def _make_bracket(self, msg: Dict[str, Any]) -> _Bracket:
        from polyaxon_amd.polytune.managers import HyperbandSearchManager
        from polyaxon_amd.spec.hptuning import HPTuningConfig, Optimization

        hp = HPTuningConfig.from_dict(msg["hptuning"])
        hb = hp.hyperband
        m = HyperbandSearchManager(hp)
        rules = []
        for r in msg.get("early_stopping") or []:
            if r["metric"] == self.program.metric:
                rules.append((0, float(r["value"]), Optimization.maximize(r["optimization"])))
        if hb.metric.name != self.program.metric:
            raise ValueError(f"hyperband metric {hb.metric.name!r} is not what program {self.program_name} "
                             f"reports ({self.program.metric!r})")
        configs = {int(c["cid"]): dict(c["params"]) for c in msg["configs"]}
        br = _Bracket(key=msg["key"], manager=m, iteration=int(msg["iteration"]), configs=configs,
                      resource_name=hb.resource.name, resource=hb.resource,
                      maximize=Optimization.maximize(hb.metric.optimization), resume=hb.resume,
                      seed=int(msg.get("seed", 0)), rules=rules)
        # a re-dispatched bracket starts at the rung after its last completed one, with that rung's promotions;
        # no snapshot exists here, so those configs re-train from scratch with the full resource of the rung
        br.rung = int(msg.get("start_rung", 0))
        br.active = [int(c) for c in msg["active"]] if msg.get("active") is not None else sorted(configs)
        return br

    def _make_trials(self, msg: Dict[str, Any]) -> _Bracket:
        """``{"op": "trials", "key", "configs": [{cid, params}], "units", "maximize", "seed", "early_stopping"}``:
        independent trials of ``units`` resource units each (a BO batch), run as a one-rung bracket."""
        from polyaxon_amd.spec.hptuning import Optimization

        if msg.get("metric", self.program.metric) != self.program.metric:
            raise ValueError(f"metric {msg.get('metric')!r} is not what program {self.program_name} reports "
                             f"({self.program.metric!r})")
        rules = [(0, float(r["value"]), Optimization.maximize(r["optimization"]))
                 for r in msg.get("early_stopping") or [] if r["metric"] == self.program.metric]
        configs = {int(c["cid"]): dict(c["params"]) for c in msg["configs"]}
        return _Bracket(key=msg["key"], manager=_FixedBudget(float(msg["units"])), iteration=0, configs=configs,
                        resource_name=str(msg.get("resource", "units")), resource=_Units(),
                        maximize=bool(msg.get("maximize", False)), resume=False, seed=int(msg.get("seed", 0)),
                        rules=rules, active=sorted(configs))

    def _make_shard(self, msg: Dict[str, Any]) -> _AshaShard:
        from polyaxon_amd.spec.hptuning import HPTuningConfig, Optimization

        hp = HPTuningConfig.from_dict(msg["hptuning"])
        a = hp.asha
        if a.metric.name != self.program.metric:
            raise ValueError(f"asha metric {a.metric.name!r} is not what program {self.program_name} "
                             f"reports ({self.program.metric!r})")
        rules = [(0, float(r["value"]), Optimization.maximize(r["optimization"]))
                 for r in msg.get("early_stopping") or [] if r["metric"] == self.program.metric]
        configs = {int(c["cid"]): dict(c["params"]) for c in msg["configs"]}
        n_rungs = int(math.floor(math.log(a.max_resource / a.min_resource) / math.log(a.eta) + 1e-9)) + 1
        sh = _AshaShard(key=msg["key"], configs=configs, pending=sorted(configs), n_rungs=n_rungs, eta=float(a.eta),
                        min_r=float(a.min_resource), max_r=float(a.max_resource), resource_name=a.resource.name,
                        resource=a.resource, maximize=Optimization.maximize(a.metric.optimization), resume=a.resume,
                        seed=int(msg.get("seed", 0)), rules=rules)
        sh.results = [dict() for _ in range(n_rungs)]
        sh.promoted = [set() for _ in range(n_rungs)]
        sh.order = [[] for _ in range(n_rungs)]
        # re-dispatch: the results the scheduler recorded before the old executor died ([rung, cid, metric])
        for rung, cid, v in msg.get("history") or []:
            rung, cid = int(rung), int(cid)
            if cid in sh.pending:
                sh.pending.remove(cid)
            if v is not None and not (isinstance(v, float) and math.isnan(v)):
                sh.results[rung][cid] = float(v)
            if rung > 0:
                sh.promoted[rung - 1].add(cid)
        for rung in range(n_rungs):
            sh.order[rung] = sorted(sh.results[rung], key=lambda c: (-sh.results[rung][c] if sh.maximize
                                                                     else sh.results[rung][c], c))
        return sh

    # ------------------------------------------------------------------ serve loop
    def serve(self, chan: Channel) -> str:
        """Process messages and run rounds until paused (returns ``pause:<tag>``), shut down or disconnected."""
        self._ready_info = getattr(self, "_ready_info", None) or {"ev": "ready", "program": self.program_name}
        while True:
            busy = bool(self.active or self.queue or self.asha_active or self.asha_queue)
            try:
                t_wait = time.perf_counter()
                msg = chan.recv(timeout=0 if busy else (None if self.pause_tag is None else 0))
                if not busy:
                    self.stats["idle_s"] += time.perf_counter() - t_wait
            except ChannelClosed:
                return "eof"
            if msg is not None:
                try:
                    r = self.handle(msg, chan)
                except Exception as e:  # bad bracket message: report, keep serving
                    chan.send({"ev": "error", "fatal": False, "key": msg.get("key"), "message": repr(e),
                               "traceback": traceback.format_exc()})
                    if msg.get("op") in ("bracket", "trials"):
                        chan.send({"ev": "bracket_done", "key": msg.get("key"), "status": "failed"})
                    r = None
                if r is not None:
                    return r
                continue
            if self.active or self.queue or self.asha_active or self.asha_queue:
                self._shutdown = None
                t_round = time.perf_counter()
                self.run_round(chan)
                self.stats["round_s"] += time.perf_counter() - t_round
                if self._shutdown is not None:
                    return self._shutdown
            elif self.pause_tag is not None:
                tag, self.pause_tag = self.pause_tag, None
                chan.send({"ev": "paused", "tag": tag, "stats": dict(self.stats)})
                return f"pause:{tag}"

    def _poll_control(self, chan: Channel) -> None:
        """Between trials: take in new brackets, stop requests and pauses without blocking, in arrival order
        (a shutdown is honoured at the end of the round)."""
        while True:
            try:
                msg = chan.recv(timeout=0)
            except ChannelClosed:
                self._shutdown = "eof"
                return
            if msg is None:
                return
            try:
                r = self.handle(msg, chan)
            except Exception as e:
                chan.send({"ev": "error", "fatal": False, "key": msg.get("key"), "message": repr(e),
                           "traceback": traceback.format_exc()})
                if msg.get("op") in ("bracket", "trials"):
                    chan.send({"ev": "bracket_done", "key": msg.get("key"), "status": "failed"})
                r = None
            if r is not None:
                self._shutdown = r

    # ------------------------------------------------------------------ one round
    def _asha_rows(self, sh: _AshaShard) -> None:
        """Give an admitted shard ``n_rungs`` contiguous rows of the ASHA metric table (grown, values kept)."""
        from polyaxon_amd.polytune.kernels import BracketMetrics

        dev = self.program.executor.device
        width = max(len(sh.configs), 1)
        used = sorted((o.row0, o.row0 + o.n_rungs) for o in self.asha_active if o is not sh and o.row0 >= 0)
        row0, prev = 0, 0
        for lo, hi in used:
            if lo - prev >= sh.n_rungs:
                break
            prev = hi
        row0 = prev
        need_rows, cur = row0 + sh.n_rungs, self.asha_metrics
        if cur is None or cur.values.shape[0] < need_rows or cur.values.shape[1] < width:
            rows = max(need_rows, cur.values.shape[0] if cur is not None else 0, 4 * sh.n_rungs)
            cols = max(width, cur.values.shape[1] if cur is not None else 0)
            grown = BracketMetrics(rows, cols, dev)
            if cur is not None:
                r, c = cur.values.shape
                grown.values[:r, :c].copy_(cur.values)
                grown.counts[:r].copy_(cur.counts)
                grown._host_counts[:r] = cur._host_counts
            self.asha_metrics = grown
        sh.row0 = row0
        for rung in range(sh.n_rungs):
            self.asha_metrics.reset_bracket(row0 + rung, len(sh.configs))
        # a re-dispatched shard brings its recorded results back onto the device table
        cols = sorted(sh.configs)
        for rung in range(sh.n_rungs):
            for cid, v in sh.results[rung].items():
                self.asha_metrics.values[row0 + rung, cols.index(cid)] = v

    def run_round(self, chan: Channel) -> None:
        import torch

        from polyaxon_amd.polytune.kernels import BracketMetrics, early_stop_any

        while len(self.active) + len(self.asha_active) < self.max_active and (self.queue or self.asha_queue):
            if self.queue:
                self.active.append(self.queue.pop(0))
            if self.asha_queue and len(self.active) + len(self.asha_active) < self.max_active:
                sh = self.asha_queue.pop(0)
                self.asha_active.append(sh)
                self._asha_rows(sh)
        brs = list(self.active)
        shards = list(self.asha_active)
        ex = self.program.executor
        if brs:
            width = max(len(br.active) for br in brs)
            if self.metrics.values.shape[1] < width or self.metrics.values.shape[0] < len(brs):
                self.metrics = BracketMetrics(max(self.max_active, len(brs)), max(width, self.metrics.values.shape[1]),
                                              ex.device)
            for row, br in enumerate(brs):
                self.metrics.reset_bracket(row, len(br.active))
        records = []
        for row, br in enumerate(brs):
            m = br.manager
            r = br.resource.cast_value(m.get_n_resources_for_iteration(br.iteration, br.rung))
            more = m.get_n_config_to_keep_for_iteration(br.iteration, br.rung) > 0
            for slot, cid in enumerate(br.active):
                self._poll_control(chan)
                if br.stopped:
                    break
                params = dict(br.configs[cid])
                params[br.resource_name] = r
                resumed = br.resume and br.rung > 0 and cid in br.prev_r
                chan.send({"ev": "trial_start", "key": br.key, "rung": br.rung, "cid": cid, "params": params,
                           "resumed": resumed, "t": time.time()})
                t_start = self._event()
                if resumed:
                    ex.restore((br.key, cid))
                    steps = int(round((r - br.prev_r[cid]) * self.program.unit_steps))
                else:
                    ex.reset(seed=(br.seed * 1000003 + br.iteration * 1009 + cid) & 0x7FFFFFFF)
                    steps = int(round(r * self.program.unit_steps))
                ex.set_hparams(**{k: v for k, v in params.items() if k in self.program.hp_keys})
                ex.run(steps)
                ex.commit(self.metrics.values[row], slot, self.program.window)
                if br.resume and more:
                    ex.snapshot((br.key, cid))
                records.append((row, br, slot, cid, steps, t_start, self._event()))
        # ---- ASHA shards: up to asha_jobs jobs each, decided from the previous round's device rankings (next_job marks
        # a promotion as taken when it hands it out, so a round never runs one twice; a shard is finished only when
        # its first job of a round finds nothing runnable -- later ones may wait for this round's results)
        asha_records = []
        finished = []
        jobs = []
        for sh in shards:
            for j in range(self.asha_jobs):
                job = None if (sh.stopped or sh.early_stopped) else sh.next_job()
                if job is None:
                    if j == 0:
                        finished.append(sh)
                    break
                jobs.append((sh, job))
        for sh, job in jobs:
            self._poll_control(chan)
            if sh.stopped:
                continue
            cid, rung = job
            col = sorted(sh.configs).index(cid)
            r = sh.r(rung)
            params = dict(sh.configs[cid])
            params[sh.resource_name] = r
            resumed = sh.resume and rung > 0 and sh.snap_rung.get(cid) == rung - 1
            chan.send({"ev": "trial_start", "key": sh.key, "rung": rung, "cid": cid, "params": params,
                       "resumed": resumed, "t": time.time()})
            t_start = self._event()
            if resumed:
                ex.restore((sh.key, cid))
                steps = int(round((r - sh.r(rung - 1)) * self.program.unit_steps))
            else:
                ex.reset(seed=(sh.seed * 1000003 + cid) & 0x7FFFFFFF)
                steps = int(round(r * self.program.unit_steps))
            ex.set_hparams(**{k: v for k, v in params.items() if k in self.program.hp_keys})
            ex.run(steps)
            ex.commit(self.asha_metrics.values[sh.row0 + rung], col, self.program.window)
            if rung < sh.n_rungs - 1 and self._snapshot_room():
                # over the snapshot budget the config is not snapshotted: a later promotion re-trains it (RESTART)
                ex.snapshot((sh.key, cid))
                sh.snap_rung[cid] = rung
            self.stats["asha_jobs"] += 1
            asha_records.append((sh, rung, cid, col, steps, t_start, self._event()))
        # ---- the round's decision: one top-k launch per optimisation direction over every active bracket
        n = len(brs)
        if self.gang is not None:  # DP gang: every rank decides from the cross-rank mean of the round's metrics
            if n:
                self.gang.mean_(self.metrics.values[:n])
            if self.asha_metrics is not None and asha_records:
                self.gang.mean_(self.asha_metrics.values)
        orders = {}
        if n:
            vals_dev = self.metrics.values[:n]
            for mx in sorted({br.maximize for br in brs}):
                orders[mx] = self.metrics.order(mx, rows=n)
                self.stats["topk_launches"] += 1
        # ... and one per direction over every ASHA rung row (the shards' rankings for the next round)
        a_orders = {}
        live = [sh for sh in shards if sh not in finished]
        a_rows = max((sh.row0 + sh.n_rungs for sh in live), default=0)
        if live:
            for mx in sorted({sh.maximize for sh in live}):
                a_orders[mx] = self.asha_metrics.order(mx, rows=a_rows)
                self.stats["topk_launches"] += 1
        early = {}
        by_rules: Dict[Tuple, List[int]] = {}
        for row, br in enumerate(brs):
            if br.rules:
                by_rules.setdefault(tuple(br.rules), []).append(row)
        for rules, rows in by_rules.items():
            idx = torch.tensor(rows, device=self.metrics.values.device)
            flags = early_stop_any(self.metrics.values[:n].index_select(0, idx).reshape(-1, 1), list(rules))
            self.stats["early_stop_launches"] += 1
            for row in rows:
                early[row] = any(flags)
        a_early = {}
        for sh in live:
            if sh.rules:
                flags = early_stop_any(self.asha_metrics.values[sh.row0: sh.row0 + sh.n_rungs].reshape(-1, 1),
                                       list(sh.rules))
                self.stats["early_stop_launches"] += 1
                a_early[sh.key] = any(flags)
        # the round's D2H reads (the first one synchronises)
        t_sync = time.perf_counter()
        vals = self.metrics.values[:n].detach().cpu().tolist() if n else []
        orders_h = {mx: o[:n].cpu().tolist() for mx, o in orders.items()}
        a_vals = self.asha_metrics.values[:a_rows].detach().cpu().tolist() if live else []
        a_orders_h = {mx: o[:a_rows].cpu().tolist() for mx, o in a_orders.items()}
        self.stats["sync_s"] += time.perf_counter() - t_sync
        for row, br, slot, cid, steps, t0, t1 in records:
            v = vals[row][slot]
            self.stats["trials"] += 1
            self.stats["train_steps"] += steps
            chan.send({"ev": "trial_end", "key": br.key, "rung": br.rung, "cid": cid, "steps": steps,
                       "metric": None if math.isnan(v) else v, "t_start": self._wall(t0), "t_end": self._wall(t1)})
        for sh, rung, cid, col, steps, t0, t1 in asha_records:
            v = a_vals[sh.row0 + rung][col]
            self.stats["trials"] += 1
            self.stats["train_steps"] += steps
            if not math.isnan(v):
                sh.results[rung][cid] = v
            chan.send({"ev": "trial_end", "key": sh.key, "rung": rung, "cid": cid, "steps": steps,
                       "metric": None if math.isnan(v) else v, "t_start": self._wall(t0), "t_end": self._wall(t1)})
        self.stats["rounds"] += 1
        for row, br in enumerate(brs):
            m = br.manager
            ran = [rec for rec in records if rec[1] is br]
            metrics = [[cid, vals[row][slot]] for (_, _, slot, cid, _, _, _) in ran if not math.isnan(vals[row][slot])]
            # bracket ends where the reference's create_iteration reschedules (hpsearch/iteration_managers/
            # hyperband.py:25-36): only the last bracket takes reduce steps past its own rung count
            keep = (0 if m.should_reschedule(br.iteration, br.rung)
                    else m.get_n_config_to_keep_for_iteration(br.iteration, br.rung))
            ranked = [br.active[i] for i in orders_h[br.maximize][row]
                      if 0 <= i < len(br.active) and not math.isnan(vals[row][i])]
            br.early_stopped = br.early_stopped or early.get(row, False)
            stop = br.stopped or br.early_stopped or len(ran) < len(br.active)
            promoted = [] if stop else ranked[:keep]
            chan.send({"ev": "rung_done", "key": br.key, "rung": br.rung, "metrics": metrics, "promoted": promoted,
                       "early_stop": br.early_stopped})
            for cid in br.active:
                if cid not in promoted:
                    ex.drop((br.key, cid))
            if promoted:
                br.prev_r = {cid: br.resource.cast_value(m.get_n_resources_for_iteration(br.iteration, br.rung))
                             for cid in promoted}
                br.active = promoted
                br.rung += 1
            else:
                self.active.remove(br)
                status = "stopped" if (br.stopped or br.early_stopped) else "succeeded"
                chan.send({"ev": "bracket_done", "key": br.key, "status": status})
        # ASHA: refresh every live shard's rung rankings from the device order (NaN results sort last and are not
        # in ``results``, so they never enter a top set)
        for sh in live:
            cols = sorted(sh.configs)
            order = a_orders_h[sh.maximize]
            for rung in range(sh.n_rungs):
                sh.order[rung] = [cols[i] for i in order[sh.row0 + rung]
                                  if 0 <= i < len(cols) and cols[i] in sh.results[rung]]
            if a_early.get(sh.key):
                sh.early_stopped = True
            self._drop_hopeless_snapshots(sh)
        for sh in finished:
            self._finish_shard(sh, chan)

    def _snapshot_room(self) -> bool:
        """HBM budget of the resume snapshots (PLX_SNAPSHOT_GB, default 40 % of the device): one more fits?"""
        import torch

        ex = self.program.executor
        if self._snap_budget is None:
            gb = os.environ.get("PLX_SNAPSHOT_GB")
            if gb:
                self._snap_budget = float(gb) * 2 ** 30
            elif ex.is_cuda:
                self._snap_budget = 0.4 * torch.cuda.get_device_properties(ex.device).total_memory
            else:
                self._snap_budget = float("inf")
        return (len(ex.snapshots) + 1) * ex.snapshot_bytes() <= self._snap_budget

    _snap_budget = None

    def _drop_hopeless_snapshots(self, sh: _AshaShard) -> None:
        """Release the HBM snapshots of configs that can no longer be promoted: rung 0's result set is final
        once no config is pending (every job of a round completes within the round), rung k+1's once rung k is final
        and its whole top floor(n_k / eta) has been promoted; a config below its final rung's top set never resumes."""
        final = not sh.pending
        for rung in range(sh.n_rungs - 1):
            if not final:
                break
            k = int(len(sh.results[rung]) / sh.eta)
            top = set(sh.order[rung][:k])
            for cid, r in list(sh.snap_rung.items()):
                if r == rung and cid not in top:
                    self.program.executor.drop((sh.key, cid))
                    del sh.snap_rung[cid]
            final = top <= sh.promoted[rung]

    def _finish_shard(self, sh: _AshaShard, chan: Channel) -> None:
        """Rung summaries (one ``rung_done`` per rung: its results and the configs promoted out of it), snapshots
        released, rows freed, ``bracket_done``."""
        for rung in range(sh.n_rungs):
            if not sh.results[rung] and rung > 0:
                continue
            chan.send({"ev": "rung_done", "key": sh.key, "rung": rung,
                       "metrics": [[cid, v] for cid, v in sorted(sh.results[rung].items())],
                       "promoted": sorted(sh.promoted[rung]) if rung < sh.n_rungs - 1 else [],
                       "early_stop": sh.early_stopped})
        for cid in list(sh.snap_rung):
            self.program.executor.drop((sh.key, cid))
        self.asha_active.remove(sh)
        sh.row0 = -1
        status = "stopped" if (sh.stopped or sh.early_stopped) else "succeeded"
        chan.send({"ev": "bracket_done", "key": sh.key, "status": status})


class _GangGroup:
    """A DP gang of resident workers (``environment.resources.gpu: N`` with a resident executor): one process per
    device, ranks from the pool's env (PLX_RESIDENT_RANK / _WORLD, MASTER_ADDR / MASTER_PORT).  The process group is a
    gloo rendezvous: it carries the control stream -- the scheduler messages rank 0 receives, re-broadcast to the other
    ranks so every rank handles the same messages at the same program points and runs the same trials in the same
    order -- and ships the RCCL unique id.  Every device collective (the executor's gradient buckets, the metric-table
    mean before each rung decision) runs on the process's one framework communicator (parallel/comm.py)."""

    def __init__(self, rank: int, world: int, device, group=None):
        import datetime

        import torch
        import torch.distributed as dist

        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.comm = None  # acquired on first use (collective: every rank reaches it at the same program point)
        if group is not None:  # a subgroup of an existing world (bench.py): its rank 0 leads, as a GLOBAL rank
            from polyaxon_amd.parallel.comm import group_rank0

            if dist.get_world_size(group) != world or dist.get_rank(group) != rank:
                raise ValueError("gang group does not match (rank, world)")
            self.group, self.src, self.owns = group, group_rank0(group), False
            return
        self.group, self.src, self.owns = None, 0, True
        long = datetime.timedelta(days=7)  # an idle executor blocks in the control broadcast between groups
        # rank 0 serves the store on the pool's already-listening socket (polyflow/pool.py _spawn_gang); every rank
        # builds its store explicitly so all of them see the same (unprefixed) key space
        fd = os.environ.get("PLX_MASTER_LISTEN_FD") if rank == 0 else None
        kw = {"master_listen_fd": int(fd)} if fd else {}
        store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                              rank == 0, timeout=long, **kw)
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world, timeout=long)

    def broadcast(self, obj):
        import torch.distributed as dist

        box = [obj]
        dist.broadcast_object_list(box, src=self.src, group=self.group)
        return box[0]

    def mean_(self, t) -> None:
        """In-place cross-rank mean of a metric table (every rank then takes the same promotion decisions)."""
        from polyaxon_amd.parallel import comm as _comm

        if self.comm is None:
            self.comm = _comm.acquire(self.group, t.device)
        if self.comm.native_avg:
            self.comm.all_reduce(t, op="avg")
        else:
            self.comm.all_reduce(t, op="sum").div_(self.world)

    def close(self) -> None:
        import torch.distributed as dist

        from polyaxon_amd.parallel import comm as _comm

        if self.comm is not None:
            _comm.release(self.comm)
            self.comm = None
        if self.owns and dist.is_initialized():
            dist.destroy_process_group()


class _LeaderChannel:
    """Rank 0's scheduler channel: every ``recv`` result (or its absence) is re-broadcast to the followers."""

    def __init__(self, chan: Channel, gang: _GangGroup):
        self.chan, self.gang = chan, gang

    def recv(self, timeout: Optional[float] = None):
        try:
            msg = self.chan.recv(timeout)
        except ChannelClosed:
            self.gang.broadcast({"__eof__": True})
            raise
        self.gang.broadcast(msg)
        return msg

    def send(self, msg: Dict[str, Any]) -> None:
        self.chan.send(msg)

    def close(self) -> None:
        self.chan.close()


class _FollowerChannel:
    """A follower rank's view of the control stream: rank 0's broadcasts; its events go nowhere (rank 0 reports)."""

    def __init__(self, gang: _GangGroup):
        self.gang = gang

    def recv(self, timeout: Optional[float] = None):
        msg = self.gang.broadcast(None)
        if isinstance(msg, dict) and msg.get("__eof__"):
            raise ChannelClosed("leader closed the control stream")
        return msg

    def send(self, msg: Dict[str, Any]) -> None:
        pass

    def close(self) -> None:
        pass


def serve_forever(worker: ResidentWorker, chan: Channel) -> str:
    """Worker process main loop: first message must be ``init``; then serve until shutdown / EOF."""
    msg = chan.recv()
    if msg is None or msg.get("op") != "init":
        chan.send({"ev": "error", "fatal": True, "message": "expected init"})
        return "error"
    worker.program_name = msg.get("program", worker.program_name)
    worker.params = dict(msg.get("params") or {})
    worker.max_active = int(msg.get("max_active", worker.max_active))
    world = int(os.environ.get("PLX_RESIDENT_WORLD", "1"))
    try:
        if world > 1:
            worker.join_gang(int(os.environ["PLX_RESIDENT_RANK"]), world)
        worker._ready_info = worker.build()
    except Exception as e:
        chan.send({"ev": "error", "fatal": True, "message": f"program build failed: {e!r}",
                   "traceback": traceback.format_exc()})
        return "error"
    chan.send(worker._ready_info)
    if worker.gang is not None:
        # the scheduler talks to rank 0; the other ranks follow its control stream (their own channel only carries
        # the init handshake, and their exit is how the pool notices a lost rank)
        chan = _LeaderChannel(chan, worker.gang) if worker.gang.rank == 0 else _FollowerChannel(worker.gang)
    try:
        while True:
            r = worker.serve(chan)
            if r in ("shutdown", "eof"):
                return r
    finally:
        worker.close_gang()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="polyaxon_amd.polyflow.resident")
    ap.add_argument("--fd", type=int, help="inherited connected socket")
    ap.add_argument("--connect", help="host:port of the scheduler")
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args(argv)
    if args.fd is not None:
        chan = Channel(socket.socket(fileno=args.fd))
    elif args.connect:
        host, _, port = args.connect.rpartition(":")
        chan = Channel.connect(host, int(port))
    else:
        ap.error("need --fd or --connect")
    device = "cpu" if args.cpu or os.environ.get("PLX_CPU_ONLY") == "1" else None
    worker = ResidentWorker("", device=device)
    r = serve_forever(worker, chan)
    chan.close()
    return 0 if r in ("shutdown", "eof") else 1


if __name__ == "__main__":
    sys.exit(main())
