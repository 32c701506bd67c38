"""Scheduler-side pool of resident executors (one warm worker process per GPU, see polyflow/resident.py).

The pool lives on the polyflow thread.  It

* spawns workers on demand for a program (``environment.executor``), each on a device it reserves in the
  allocator under owner ``resident:<wid>`` (whole GPU, or a fraction + HBM budget for small programs), pinned
  with ``HIP_VISIBLE_DEVICES`` and the NUMA-local CPUs like any trial replica;
* accepts externally started workers (``attach``: bench.py's ranks, or a worker on a GPU another launcher owns);
* balances brackets over the workers of a program by outstanding training units (longest-processing-time
  greedy: every new bracket goes to the least-loaded executor the group may use);
* turns worker messages into calls on the owning group driver (reader thread per worker -> ``flow.post``), and
  a lost worker (process died, socket closed) into failed trials and released devices;
* shuts idle spawned workers down after ``idle_s`` so their GPUs return to process-mode runs -- at once when a
  multi-device run (a DP gang) waits for devices the idle executors hold, and spawns none into a gang's
  reservation (the reference counts concurrency against the cluster's capacity the same way for every run,
  polyaxon/db/models/experiment_groups.py:193-197; warm executors must not starve a DP=8 job).
"""
from __future__ import annotations

import logging
import os
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from polyaxon_amd.polyflow.env import hw_queue_env
from polyaxon_amd.polyflow.resident import Channel, ChannelClosed

log = logging.getLogger("polyaxon_amd.polyflow.pool")


@dataclass
class WorkerHandle:
    wid: int
    key: str                          # program key (name + params)
    program: str
    params: Dict[str, Any]
    devices: List[int]
    chan: Channel
    proc: Optional[subprocess.Popen] = None
    external: bool = False
    ready: bool = False
    alive: bool = True
    info: Dict[str, Any] = field(default_factory=dict)
    brackets: Dict[str, Any] = field(default_factory=dict)   # bracket key -> driver
    units: Dict[str, float] = field(default_factory=dict)    # bracket key -> outstanding units
    idle_since: float = field(default_factory=time.time)
    closing: bool = False
    assigned_units: float = 0.0                              # cumulative training units / units of work assigned
    assigned_count: int = 0
    waiters: Dict[str, Callable[[Dict[str, Any]], None]] = field(default_factory=dict)
    peers: List[Any] = field(default_factory=list)             # DP gang: (Popen, Channel) of ranks 1..N-1

    @property
    def owner(self) -> str:
        return f"resident:{self.wid}"

    @property
    def load(self) -> float:
        return sum(self.units.values())


class ResidentPool:
    def __init__(self, flow, idle_s: float = 300.0):
        self.flow = flow
        self.idle_s = idle_s
        self.workers: Dict[int, WorkerHandle] = {}
        self._next = 1
        self._reaper_armed = False
        # why the last spawn could NEVER succeed on this node (allocator ValueError: no such device, a fraction or
        # HBM request larger than a device); None when it merely found every device busy
        self.placement_error: Optional[str] = None

    # ------------------------------------------------------------------ queries
    def workers_for(self, key: str) -> List[WorkerHandle]:
        return [w for w in self.workers.values() if w.alive and w.key == key]

    def snapshot(self) -> List[Dict[str, Any]]:
        return [{"wid": w.wid, "program": w.program, "devices": w.devices, "external": w.external, "ready": w.ready,
                 "alive": w.alive, "brackets": sorted(w.brackets), "load_units": w.load,
                 "assigned_units": w.assigned_units, "assigned": w.assigned_count,
                 "pid": w.proc.pid if w.proc else w.info.get("pid")} for w in self.workers.values()]

    # ------------------------------------------------------------------ creation
    @staticmethod
    def dp_world(gpu: float) -> int:
        """Devices of one executor for a ``resources.gpu`` request: a DP gang for an integer > 1, else one."""
        return int(round(gpu)) if gpu > 1.0 + 1e-9 else 1

    def ensure(self, key: str, program: str, params: Dict[str, Any], want: int, gpu: float = 1.0,
               hbm_gb: float = 0.0, max_active: int = 8) -> List[WorkerHandle]:
        """Make sure up to ``want`` workers run ``program`` on ``dp_world(gpu)`` devices each (spawning on free
        devices); returns the live ones.  An executor of another DP world never serves the request (a DP=2 trial
        must not silently train on one device)."""
        world = self.dp_world(gpu)
        have = [w for w in self.workers_for(key) if len(w.devices) == world]
        self.placement_error = None
        while len(have) < want:
            h = self._spawn(key, program, params, gpu, hbm_gb, max_active)
            if h is None:
                break
            have.append(h)
        return have

    def _spawn(self, key, program, params, gpu, hbm_gb, max_active) -> Optional[WorkerHandle]:
        wid = self._next
        owner = f"resident:{wid}"
        reserve = self.flow._gang_reservation()
        if reserve is not None:  # a gang holds a reservation: a new executor must leave its devices free
            need = int(round(gpu)) if gpu >= 1.0 - 1e-9 else 0
            if len(self.flow.alloc.free_whole()) - need < reserve[1]:
                return None
        try:
            a = self.flow.alloc.allocate(owner, gpu, hbm_gb)
        except ValueError as e:
            log.warning("resident executor allocation rejected: %s", e)
            self.placement_error = str(e)
            return None
        if a is None:
            devs = self.flow.alloc.devices
            if not devs:
                self.placement_error = "no devices on this node"
            elif not any(d.healthy and d.memory_gb >= hbm_gb for d in devs):
                self.placement_error = f"no healthy device with {hbm_gb} GB of HBM"
            return None
        self._next += 1
        world = len(a.devices) if gpu > 1.0 + 1e-9 else 1
        if world > 1:
            return self._spawn_gang(wid, owner, a, key, program, params, max_active)
        parent, child = socket.socketpair()
        env = self._worker_env(a.devices)
        if hbm_gb > 0:  # the executor's HBM budget (client/budget.py, applied in ResidentWorker.build)
            env["PLX_HBM_GB"] = f"{hbm_gb:g}"
        elif 0 < gpu < 1:
            env["PLX_HBM_FRACTION"] = f"{gpu:g}"
        log_dir = os.path.join(self.flow.paths.root, "executors")
        os.makedirs(log_dir, exist_ok=True)
        log_path = os.path.join(log_dir, f"worker{wid}.log")
        argv = [self.flow.python, "-m", "polyaxon_amd.polyflow.resident", "--fd", str(child.fileno())]
        if self.flow.alloc.n_devices and os.environ.get("PLX_CPU_ONLY") == "1":
            argv.append("--cpu")
        try:
            with open(log_path, "ab") as logf:
                proc = subprocess.Popen(argv, env=env, pass_fds=(child.fileno(),), stdout=logf,
                                        stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL, start_new_session=True)
        except OSError as e:
            child.close()
            parent.close()
            self.flow.alloc.release(owner)
            log.error("cannot start resident executor: %s", e)
            self.flow.store.add_cluster_event("resident_executor", "error", f"spawn failed: {e}")
            return None
        child.close()
        if a.devices and getattr(self.flow, "numa_bind", False):
            self.flow._bind_cpus(proc.pid, a.devices)
        h = WorkerHandle(wid, key, program, dict(params), list(a.devices), Channel(parent), proc=proc)
        h.info["log_path"] = log_path
        self.workers[wid] = h
        h.chan.send({"op": "init", "program": program, "params": params, "max_active": max_active})
        self._start_reader(h)
        self._arm_reaper()
        self.flow.auditor.record("resident_executor.started", "executor", wid, devices=a.devices, program=program)
        return h

    def _worker_env(self, devices: List[int]) -> Dict[str, str]:
        env = dict(os.environ)
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
        env.pop("ROCR_VISIBLE_DEVICES", None)
        env["PYTHONUNBUFFERED"] = "1"
        env.pop("PLX_HBM_GB", None)
        env.pop("PLX_HBM_FRACTION", None)
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        hw_queue_env(env)
        return env

    def _spawn_gang(self, wid, owner, a, key, program, params, max_active) -> Optional[WorkerHandle]:
        """A resident executor spanning a DP gang (``resources.gpu: N``): one worker process per device, ranks wired
        with the torch.distributed env contract (MASTER_ADDR / MASTER_PORT / rank / world, as polyflow/env.py gives a
        process-mode PyTorch job); rank 0's channel is the executor's, the others only carry the init handshake.
        The rendezvous port is bound and listening HERE and rank 0 inherits the listening socket
        (PLX_MASTER_LISTEN_FD, the TCPStore's master_listen_fd): picking a free port and closing it before rank 0
        binds it again would race with any other process binding ports on the node."""
        world = len(a.devices)
        listener = socket.socket()
        listener.bind(("127.0.0.1", 0))
        listener.listen(128)
        port = listener.getsockname()[1]
        log_dir = os.path.join(self.flow.paths.root, "executors")
        os.makedirs(log_dir, exist_ok=True)
        ranks = []
        argv = [self.flow.python, "-m", "polyaxon_amd.polyflow.resident", "--fd"]
        cpu = self.flow.alloc.n_devices and os.environ.get("PLX_CPU_ONLY") == "1"
        try:
            for r, dev in enumerate(a.devices):
                parent, child = socket.socketpair()
                env = self._worker_env([dev])
                env.update(PLX_RESIDENT_RANK=str(r), PLX_RESIDENT_WORLD=str(world), MASTER_ADDR="127.0.0.1",
                           MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0")
                fds = (child.fileno(),)
                if r == 0:
                    env["PLX_MASTER_LISTEN_FD"] = str(listener.fileno())
                    fds += (listener.fileno(),)
                path = os.path.join(log_dir, f"worker{wid}.rank{r}.log")
                with open(path, "ab") as logf:
                    proc = subprocess.Popen(argv + [str(child.fileno())] + (["--cpu"] if cpu else []), env=env,
                                            pass_fds=fds, stdout=logf, stderr=subprocess.STDOUT,
                                            stdin=subprocess.DEVNULL, start_new_session=True)
                child.close()
                ranks.append((proc, Channel(parent), path))
        except OSError as e:
            for proc, ch, _ in ranks:
                ch.close()
                try:
                    os.killpg(proc.pid, 9)
                except OSError:
                    pass
            self.flow.alloc.release(owner)
            log.error("cannot start resident DP gang: %s", e)
            self.flow.store.add_cluster_event("resident_executor", "error", f"gang spawn failed: {e}")
            return None
        finally:
            listener.close()  # rank 0 holds its own copy
        if getattr(self.flow, "numa_bind", False):
            for (proc, _, _), dev in zip(ranks, a.devices):
                self.flow._bind_cpus(proc.pid, [dev])
        proc0, chan0, path0 = ranks[0]
        h = WorkerHandle(wid, key, program, dict(params), list(a.devices), chan0, proc=proc0)
        h.info["log_path"] = path0
        h.peers = [(proc, ch) for proc, ch, _ in ranks[1:]]
        self.workers[wid] = h
        init = {"op": "init", "program": program, "params": params, "max_active": max_active}
        for _, ch, _ in ranks:
            ch.send(init)
        self._start_reader(h)
        for proc, ch in h.peers:
            self._start_peer_reader(h, proc, ch)
        self._arm_reaper()
        self.flow.auditor.record("resident_executor.started", "executor", wid, devices=a.devices, program=program,
                                 dp_world=world)
        return h

    def _start_peer_reader(self, h: WorkerHandle, proc, chan: Channel) -> None:
        """A gang's rank > 0: its only messages are the ready handshake or a fatal error; its exit loses the gang."""
        def reader():
            while True:
                try:
                    msg = chan.recv()
                except (ChannelClosed, OSError, ValueError):
                    break
                if msg is not None and msg.get("ev") == "error" and msg.get("fatal"):
                    self.flow.post(self._lost, h, f"gang rank failed: {msg.get('message')}")
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                proc.kill()
            self.flow.post(self._lost, h, f"gang rank exited ({proc.returncode})")

        threading.Thread(target=reader, name=f"resident-peer-{h.wid}", daemon=True).start()

    def attach(self, chan: Channel, device, program: str, params: Optional[Dict[str, Any]] = None,
               max_active: int = 8, gpu: float = 1.0) -> WorkerHandle:
        """Register an already running worker (it was built by another launcher, e.g. a bench.py rank) that owns
        ``device`` -- one index, or the list of a DP gang's devices (its leader attaches; the other ranks follow
        the leader's control stream).  Runs on the scheduler thread."""
        from polyaxon_amd.polyflow.programs import program_key

        devices = [int(d) for d in device] if isinstance(device, (list, tuple)) else [int(device)]
        wid = self._next
        self._next += 1
        owner = f"resident:{wid}"
        if self.flow.alloc.allocate_on(owner, devices, gpu) is None:
            raise RuntimeError(f"devices {devices} are not free for a resident executor")
        h = WorkerHandle(wid, program_key(program, params), program, dict(params or {}), devices, chan,
                         external=True)
        self.workers[wid] = h
        chan.send({"op": "init", "program": program, "params": params or {}, "max_active": max_active})
        self._start_reader(h)
        return h

    # ------------------------------------------------------------------ dispatch
    def assign(self, driver, msg: Dict[str, Any], units: float,
               allowed: Optional[List[int]] = None, key: Optional[str] = None,
               world: Optional[int] = None) -> Optional[WorkerHandle]:
        cands = [w for w in self.workers.values() if w.alive and (key is None or w.key == key)
                 and (allowed is None or w.wid in allowed) and (world is None or len(w.devices) == world)]
        if not cands:
            return None
        w = min(cands, key=lambda h: (h.load, h.wid))
        w.brackets[msg["key"]] = driver
        w.units[msg["key"]] = units
        w.assigned_units += units
        w.assigned_count += 1
        try:
            w.chan.send(msg)
        except OSError:
            self._lost(w, "send failed")
            return None
        return w

    def request(self, driver, msg: Dict[str, Any], key: Optional[str] = None,
                allowed: Optional[List[int]] = None) -> Optional[WorkerHandle]:
        """Send a one-shot request (``bo_suggest``) to the least-loaded live executor of ``key``; its reply (same
        ``key`` field) is routed to ``driver.on_resident_event``, and a lost executor to ``on_bracket_lost``."""
        cands = [w for w in self.workers.values() if w.alive and w.ready and (key is None or w.key == key)
                 and (allowed is None or w.wid in allowed)]
        if not cands and allowed is not None:
            cands = [w for w in self.workers.values() if w.alive and w.ready and (key is None or w.key == key)]
        if not cands:
            return None
        w = min(cands, key=lambda h: (h.load, h.wid))
        w.brackets[msg["key"]] = driver
        try:
            w.chan.send(msg)
        except OSError:
            self._lost(w, "send failed")
            return None
        return w

    def send(self, wid: int, msg: Dict[str, Any]) -> bool:
        w = self.workers.get(wid)
        if w is None or not w.alive:
            return False
        try:
            w.chan.send(msg)
            return True
        except OSError:
            self._lost(w, "send failed")
            return False

    def pause_all(self, tag: str, on_paused: Optional[Callable[[Dict[str, Any]], None]] = None,
                  key: Optional[str] = None) -> int:
        n = 0
        for w in self.workers.values():
            if w.alive and (key is None or w.key == key):
                if on_paused is not None:
                    w.waiters[f"paused:{tag}"] = on_paused
                self.send(w.wid, {"op": "pause", "tag": tag})
                n += 1
        return n

    def shutdown(self, wid: Optional[int] = None) -> None:
        for w in list(self.workers.values()):
            if wid is not None and w.wid != wid:
                continue
            if w.alive:
                w.closing = True
                self.send(w.wid, {"op": "shutdown"})

    def close(self, timeout: float = 10.0) -> None:
        """Scheduler shutdown: ask every worker to exit, wait for the spawned ones, release every device."""
        self.shutdown()
        end = time.time() + timeout
        for w in list(self.workers.values()):
            if w.proc is not None:
                try:
                    w.proc.wait(timeout=max(0.1, end - time.time()))
                except subprocess.TimeoutExpired:
                    pass
            w.closing = True
            self._lost(w, "scheduler shutdown")

    # ------------------------------------------------------------------ messages (scheduler thread)
    def _start_reader(self, h: WorkerHandle) -> None:
        def reader():
            while True:
                try:
                    msg = h.chan.recv()
                except (ChannelClosed, OSError, ValueError):
                    break
                if msg is None:
                    continue
                self.flow.post(self._on_message, h, msg)
            if h.proc is not None:
                try:
                    h.proc.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    h.proc.kill()
            self.flow.post(self._lost, h, "worker exited" if h.proc is None else f"worker exited ({h.proc.returncode})")

        threading.Thread(target=reader, name=f"resident-reader-{h.wid}", daemon=True).start()

    def _on_message(self, h: WorkerHandle, msg: Dict[str, Any]) -> None:
        ev = msg.get("ev")
        if ev == "ready":
            h.ready = True
            h.info.update(msg)
            self.flow.store.kv_set(f"resident:{h.wid}", {k: v for k, v in msg.items() if k != "ev"})
            return
        if ev == "paused":
            cb = h.waiters.pop(f"paused:{msg.get('tag')}", None)
            if cb is not None:
                cb(dict(msg, wid=h.wid))
            return
        if ev == "pong":
            cb = h.waiters.pop("pong", None)
            if cb is not None:
                cb(dict(msg, wid=h.wid))
            return
        if ev == "error" and msg.get("fatal"):
            log.error("resident executor %d failed: %s", h.wid, msg.get("message"))
            self.flow.store.add_cluster_event("resident_executor", "error",
                                              f"executor {h.wid} on devices {h.devices}: {msg.get('message')}",
                                              {"traceback": msg.get("traceback")})
            self._lost(h, msg.get("message") or "fatal error")
            return
        key = msg.get("key")
        driver = h.brackets.get(key) if key is not None else None
        if driver is None:
            if ev == "error":
                log.warning("resident executor %d: %s", h.wid, msg.get("message"))
            return
        try:
            driver.on_resident_event(h, msg)
        finally:
            if ev == "trial_end":
                # outstanding work shrinks as trials finish (keeps the balancing estimate honest)
                h.units[key] = max(0.0, h.units.get(key, 0.0) - float(msg.get("steps", 0)) /
                                   max(1.0, float(h.info.get("unit_steps", 1) or 1)))
            if ev == "bo_suggestions" or (ev == "error" and key.endswith(".suggest")):
                h.brackets.pop(key, None)  # one-shot request answered
            if ev == "bracket_done":
                h.brackets.pop(key, None)
                h.units.pop(key, None)
                if not h.brackets:
                    h.idle_since = time.time()

    def _lost(self, h: WorkerHandle, reason: str) -> None:
        if not h.alive:
            return
        h.alive = False
        self.flow.alloc.release(h.owner)
        try:
            h.chan.close()
        except Exception:
            pass
        for proc in [h.proc] + [p for p, _ in h.peers]:
            if proc is not None and proc.poll() is None:
                try:
                    os.killpg(proc.pid, 9)
                except OSError:
                    pass
        for _, ch in h.peers:
            try:
                ch.close()
            except Exception:
                pass
        lost = dict(h.brackets)
        h.brackets.clear()
        h.units.clear()
        if lost or not (h.external or h.closing):
            self.flow.store.add_cluster_event("resident_executor", "warning" if not lost else "error",
                                              f"executor {h.wid} on devices {h.devices} gone: {reason}",
                                              {"brackets": sorted(lost)})
        for key, driver in lost.items():
            try:
                driver.on_bracket_lost(h, key, reason)
            except Exception:
                log.exception("bracket loss handler failed")

    def yield_to_gangs(self) -> int:
        """A multi-device run waits for devices: shut down idle spawned executors (no brackets) until it would fit,
        if releasing them is enough to place it.  Returns the number of executors asked to exit."""
        g = self.flow.waiting_gang()
        if g is None:
            return 0
        _, whole = g
        free = len(self.flow.alloc.free_whole())
        if free >= whole:
            return 0
        idle = [w for w in sorted(self.workers.values(), key=lambda h: h.wid)
                if w.alive and not w.external and not w.brackets and not w.closing]
        if free + sum(len(w.devices) for w in idle) < whole:
            return 0  # not enough even with every idle executor gone: keep them warm for now
        n = 0
        for w in idle:
            if free >= whole:
                break
            self.shutdown(w.wid)
            free += len(w.devices)
            n += 1
            self.flow.auditor.record("resident_executor.yielded", "executor", w.wid, devices=w.devices,
                                     gang=g[0])
        return n

    # ------------------------------------------------------------------ idle reaping
    def _arm_reaper(self) -> None:
        if self._reaper_armed or self.idle_s <= 0:
            return
        self._reaper_armed = True
        self.flow.after(min(self.idle_s, 30.0), self._reap)

    def _reap(self) -> None:
        self._reaper_armed = False
        now = time.time()
        for w in list(self.workers.values()):
            if w.alive and not w.external and not w.brackets and now - w.idle_since > self.idle_s:
                self.shutdown(w.wid)
        if any(w.alive and not w.external for w in self.workers.values()):
            self._arm_reaper()
