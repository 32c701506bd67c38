#!/usr/bin/env python3
"""Headline benchmark: HPO trials/hour (whole node) + wall-clock-to-target, ResNet-50 Hyperband sweep.

BASELINE.json config 3 ("Hyperband/ASHA sweep of ResNet-50 on synthetic ImageNet-shape data, 8×MI355X,
64 brackets"), measured through the real control plane:

* one rank per GPU (``torchrun``, or ``--gpus N`` spawns the N ranks itself before anything touches a GPU);
  every rank builds a **resident trial executor** (polyflow/resident.py) for the ResNet-50 program, pinned to the
  CPUs local to its GPU, and attaches it to the **polyflow scheduler**;
* the scheduler (SQLite store, FSMs, group drivers) runs in a process of its own that never touches a GPU -- the
  ``--gpus N`` launcher itself, or a control process rank 0 starts before its own GPU initialisation under
  torchrun -- so no rank shares its interpreter (and GIL) with the scheduler's store writes and event handling;
* the timed work is ``--steps K`` complete sweeps **per GPU**: ``K × N`` Polyaxonfile groups with
  ``environment.executor: resident``.  ``--search hyperband`` (default; ``max_iter 9, eta 3, resume: true``:
  3 brackets and 23 trials each, reference-exact bracket arithmetic) spreads its ``3·K·N`` brackets over the N
  executors, each executor interleaves its brackets and decides each round's promotions with one HIP top-k launch;
  ``--search asha`` runs each sweep as one asynchronous successive-halving search (min 1, max 27, eta 3 resource
  units -- 27 is the largest budget the reference's Hyperband arithmetic gives one trial of a max_iter 9 sweep --
  and ``--asha-n`` 29 configs, about the 87 units of a Hyperband sweep; no rung barrier).  Every trial is an experiment row with its status history, metric
  and RESUME lineage.  The timed region starts after a barrier (after ``--warmup W`` untimed sweeps per GPU through
  the same path) and ends when every group has SUCCEEDED and every rank passed the final barrier: only whole sweeps
  are timed, never a prefix;
* one resource unit = ``--unit-steps`` full training steps (bf16 forward + backward + fused SGD) at ``--batch``
  224×224 images; the data is a fresh, learnable synthetic batch generated on the device every step
  (ops/synth.py).  A trial's metric is its mean loss over its last 4 steps, each measured on a batch the weights
  had never seen (the forward of a fresh batch precedes its update), so it is a held-out estimate;
  ``wall_clock_to_target_s`` = time from the start of the timed region to the first trial whose metric is below
  ``--target`` (set near the synthetic task's floor at this budget, so reaching it separates search strategies).

``value`` = trials completed in the timed region (all GPUs) / elapsed (max over ranks) × 3600.
Data: synthetic ImageNet-shape tensors generated on the device, random-init weights (no datasets available).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

# The box's own hardware-queue count is used (HIP's default 4): the trial process's streams fit it (one RCCL
# communicator; the weight-gradient side stream on a priority level of its own, ops/side_stream.py).  PLX_HW_QUEUES=n
# is an explicit opt-in to raise GPU_MAX_HW_QUEUES before any GPU call (the round-4 setting was 8).
if int(os.environ.get("PLX_HW_QUEUES", "0") or 0) > int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0):
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(int(os.environ.get("PLX_HW_QUEUES")), 32))

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

T0 = time.perf_counter()
METRIC = "HPO trials/hour (whole node) + wall-clock-to-target, ResNet-50 Hyperband sweep"
METRIC_BO = "HPO trials/hour (whole node) + best loss, GPT-2 125M Bayesian-GP search"
MAX_ITER, ETA = 9, 3
# ASHA's largest rung: the reference's Hyperband (r_i = r * eta^i, polytune/managers.py) trains its last bracket's
# survivor 27 units at max_iter 9, so ASHA gets the same top budget to be comparable
ASHA_MAX = MAX_ITER * ETA


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed sweeps per GPU (hyperband: 3 brackets, 23 trials)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed sweeps per GPU through the same path")
    ap.add_argument("--search", choices=("hyperband", "asha"), default="hyperband")
    ap.add_argument("--config", choices=("resnet50_hb", "gpt2_bo"), default="resnet50_hb",
                    help="gpt2_bo: BASELINE config 4 on one node -- a Bayesian-GP search over GPT-2 125M AdamW "
                         "hyper-parameters on resident executors (each timed step = one BO group of "
                         "--bo-initial + --bo-iterations x --bo-concurrency trials per GPU)")
    ap.add_argument("--trial-gpus", type=int, default=1,
                    help="GPUs per trial: > 1 runs every trial data-parallel on a resident DP gang of that many ranks "
                         "(FlatDDP over the framework RCCL communicator; BASELINE config 4: 2).  Must divide --gpus")
    ap.add_argument("--bo-initial", type=int, default=4)
    ap.add_argument("--bo-iterations", type=int, default=3)
    ap.add_argument("--bo-concurrency", type=int, default=4, help="trials per BO batch (constant liar) per GPU")
    ap.add_argument("--trial-units", type=int, default=25, help="gpt2_bo: resource units (x --unit-steps) per trial")
    ap.add_argument("--task", choices=("chain", "copy"), default="chain",
                    help="gpt2_bo: the synthetic objective.  chain (default): x_{t+1} = (a x_t + b) mod 4093, a transition "
                         "table to memorise -- within a 100-step trial the loss ends between ~0.01 and ~8 nats by learning "
                         "rate; copy: repeated 64-token phrases, whose copying is not learned within a trial budget (every "
                         "trial ends near the unigram loss: profiles/r5_config4_search.md)")
    ap.add_argument("--active-vocab", type=int, default=4096,
                    help="gpt2_bo copy task: token ids the phrases draw from (0 = the whole vocabulary)")
    ap.add_argument("--asha-n", type=int, default=29,
                    help="configs per ASHA sweep (29 at min 1 / max 27 / eta 3 with resume ~ the 87 units of a "
                         "Hyperband sweep)")
    ap.add_argument("--batch", type=int, default=256, help="per-trial batch (one trial per GPU at a time)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--unit-steps", type=int, default=4, help="training steps per resource unit")
    ap.add_argument("--target", type=float, default=None,
                    help="loss target for wall-clock-to-target (default 0.03 for resnet50_hb, 0.5 for gpt2_bo): "
                         "near the synthetic task's floor at a sweep's budget "
                         "(Hyperband sweeps reach 0.015-0.1), so only some sweeps reach it")
    ap.add_argument("--signal", type=float, default=0.5, help="class-pattern amplitude of the synthetic data")
    ap.add_argument("--active-classes", type=int, default=100, help="classes the synthetic task draws from")
    ap.add_argument("--max-active", type=int, default=8, help="brackets one executor interleaves")
    ap.add_argument("--graph", type=int, default=int(os.environ.get("PLX_BENCH_GRAPH", "0")),
                    help="replay each training step as a captured (and verified) hipGraph; measured 8 %% slower than eager "
                         "launches for this step on ROCm 7.2 (10.5k vs 11.4k trials/h, same box)")
    ap.add_argument("--cpu", action="store_true", help="CPU rehearsal (gloo, small ResNet, tiny images)")
    ap.add_argument("--control-only", action="store_true", help=argparse.SUPPRESS)  # internal: the scheduler process
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args(argv)
    if args.target is None:
        args.target = 0.5 if args.config == "gpt2_bo" else 0.03
    if args.trial_gpus < 1 or args.gpus % args.trial_gpus:
        ap.error("--trial-gpus must divide --gpus")
    return args


def program_params(args):
    if args.config == "gpt2_bo":
        if args.cpu:
            return "gpt2_tiny", {"batch": 2, "seq": 32, "unit_steps": 1, "trial_units": 2, "data_seed": 1234,
                                 "task": args.task}
        return "gpt2", {"batch": 16, "seq": 1024, "unit_steps": args.unit_steps, "trial_units": args.trial_units,
                        "graph": bool(args.graph), "data_seed": 1234, "active_vocab": args.active_vocab,
                        "task": args.task}
    if args.cpu:
        return "resnet_tiny", {"batch": min(args.batch, 8), "image": min(args.image, 32),
                               "unit_steps": min(args.unit_steps, 1), "grid": 4, "signal": args.signal,
                               "active_classes": min(args.active_classes, 10), "data_seed": 1234}
    return "resnet50", {"batch": args.batch, "image": args.image, "unit_steps": args.unit_steps, "signal": args.signal,
                        "active_classes": args.active_classes, "graph": bool(args.graph), "data_seed": 1234}


def bo_group_spec(seed: int, program: str, params: dict, args, world: int) -> dict:
    """BASELINE config 4: GP-UCB over GPT-2's AdamW learning rate, weight decay and beta2.  ``world``: executors (one
    per GPU, or one per DP gang of ``--trial-gpus`` GPUs); every trial asks for ``--trial-gpus`` devices."""
    hp = {"seed": seed, "concurrency": args.bo_concurrency * world,
          "matrix": {"lr": {"loguniform": [math.log(1e-5), math.log(3e-3)]},
                     "weight_decay": {"uniform": [0.0, 0.2]},
                     "beta2": {"uniform": [0.9, 0.999]}},
          "bo": {"n_initial_trials": args.bo_initial * world, "n_iterations": args.bo_iterations,
                 "space": "unit",  # lr over decades: the GP works in log-lr, every dimension scaled to [0, 1]
                 "metric": {"name": "loss", "optimization": "minimize"},
                 "utility_function": {"acquisition_function": "ucb", "kappa": 1.5,
                                      "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 2.5},
                                      "n_warmup": 10000, "n_iter": 8}}}
    return {"version": 1, "kind": "group", "project": "bench_gpt2_bo", "hptuning": hp,
            "environment": {"resources": {"gpu": args.trial_gpus},
                            "executor": {"kind": "resident", "program": program, "params": params,
                                         "max_active_brackets": args.max_active}}}


def group_spec(seed: int, program: str, params: dict, concurrency: int, max_active: int, search: str = "hyperband",
               asha_n: int = 29, trial_gpus: int = 1) -> dict:
    matrix = {"lr": {"loguniform": [math.log(0.02), math.log(1.0)]},
              "momentum": {"uniform": [0.8, 0.95]},
              "weight_decay": {"loguniform": [math.log(1e-5), math.log(1e-3)]}}
    metric = {"name": "loss", "optimization": "minimize"}
    resource = {"name": "units", "type": "int"}
    if search == "asha":
        hp = {"seed": seed, "concurrency": concurrency, "matrix": matrix,
              "asha": {"min_resource": 1, "max_resource": ASHA_MAX, "eta": ETA, "n_experiments": asha_n,
                       "resource": resource, "metric": metric, "resume": True}}
    else:
        hp = {"seed": seed, "concurrency": concurrency, "matrix": matrix,
              "hyperband": {"max_iter": MAX_ITER, "eta": ETA, "resource": resource, "metric": metric, "resume": True}}
    return {"version": 1, "kind": "group", "project": "bench_resnet50_" + search, "hptuning": hp,
            "environment": {"resources": {"gpu": trial_gpus},
                            "executor": {"kind": "resident", "program": program, "params": params,
                                         "max_active_brackets": max_active}}}


# ----------------------------------------------------------------------------- control (no GPU calls here)
class ControlServer:
    """The polyflow scheduler of the benchmark, in a process that never touches a GPU.  Accepts ``world`` executor
    channels (hello ``{"rank": r}``) and rank 0's bench channel (hello ``{"bench": 1}``), runs the warm-up sweeps,
    pauses the executors, waits for rank 0's ``go``, runs the timed sweeps, pauses again and sends the summary."""

    def __init__(self, args, world: int, log=None):
        from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
        from polyaxon_amd.polyflow.scheduler import Polyflow

        self.args, self.world = args, world
        self.n_exec = world // args.trial_gpus  # resident executors: one per GPU, or one per DP gang
        self.program, self.params = program_params(args)
        self.log = log or (lambda m: print(f"[control +{time.perf_counter() - T0:.1f}s] {m}", file=sys.stderr,
                                           flush=True))
        self.listener = socket.socket()
        self.listener.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.listener.bind(("127.0.0.1", 0))
        self.listener.listen(world + 2)
        self.port = self.listener.getsockname()[1]
        self.root = tempfile.mkdtemp(prefix="plx_bench_")
        self.flow = Polyflow(self.root, allocator=DeviceAllocator([Device(i) for i in range(world)]),
                             reconcile_s=0, clean_on_start=False).start()
        self.bench = None

    def _accept(self) -> None:
        from polyaxon_amd.polyflow.resident import Channel

        execs = 0
        self.listener.settimeout(900)
        while execs < self.n_exec or self.bench is None:
            sock, _ = self.listener.accept()
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            chan = Channel(sock)
            hello = chan.recv(timeout=900)
            if hello is None:
                raise TimeoutError("a benchmark peer connected but sent no hello")
            if hello.get("bench"):
                self.bench = chan
                continue
            devices = hello.get("devices") or [int(hello["rank"])]  # a DP gang's leader brings the gang's devices
            self.flow.attach_resident(chan, devices, self.program, self.params, max_active=self.args.max_active)
            execs += 1
        end = time.time() + 900
        while time.time() < end:
            snap = self.flow.call(lambda: self.flow.resident_pool().snapshot())
            if sum(1 for w in snap if w["ready"]) == self.n_exec:
                return
            time.sleep(0.05)
        raise TimeoutError("resident executors did not become ready")

    def _sweeps(self, n: int, seed0: int):
        gids = []
        n_groups = n // self.world if self.args.config == "gpt2_bo" else n  # one BO group spans every GPU
        for i in range(n_groups):
            if self.args.config == "gpt2_bo":
                spec = bo_group_spec(seed0 + i, self.program, self.params, self.args, self.n_exec)
            else:
                spec = group_spec(seed0 + i, self.program, self.params, self.n_exec, self.args.max_active,
                                  self.args.search, self.args.asha_n, self.args.trial_gpus)
            gids.append(self.flow.submit(spec)["id"])
        t_log = time.time()
        for g in gids:
            end = time.time() + 7200
            while True:  # a progress line at least every 30 s (a silent multi-minute region looks hung)
                try:
                    st = self.flow.wait("group", g, timeout=min(30.0, max(0.1, end - time.time())), poll_s=0.05)
                    break
                except TimeoutError:
                    st = "timeout"
                    if time.time() >= end:
                        break
                if time.time() - t_log >= 30:
                    t_log = time.time()
                    done = sum(1 for x in self.flow.store.list_experiments(group_id=g) if x["status"] == "succeeded")
                    self.log(f"group {g}: {done} trials done")
            if st != "succeeded":
                raise RuntimeError(f"group {g} ended {st}")
        return gids

    def _pause(self, tag: str) -> None:
        done = threading.Event()
        left = [self.n_exec]

        def on_paused(_msg):
            left[0] -= 1
            if left[0] == 0:
                done.set()

        self.flow.call(lambda: self.flow.resident_pool().pause_all(tag, on_paused))
        if not done.wait(900):
            raise TimeoutError(f"executors did not pause ({tag})")

    def serve(self) -> int:
        rc = 0
        try:
            self._accept()
            self.log(f"{self.n_exec} resident executors ready ({self.args.trial_gpus} GPU(s) each); warm-up: "
                     f"{self.args.warmup} sweep(s)/GPU")
            if self.args.warmup:
                self._sweeps(self.args.warmup * self.world, 10_000)
            base = self.flow.call(lambda: self.flow.resident_pool().snapshot())
            self._pause("warm")
            go = self.bench.recv(timeout=900)
            if go is None or go.get("op") != "go":
                raise RuntimeError(f"expected go from rank 0, got {go!r}")
            t0_wall = float(go["t0"])
            gids = self._sweeps(self.args.steps * self.world, 1)
            self._pause("timed")
            self.bench.send({"ev": "result", "result": self._summarise(gids, t0_wall, base)})
        except BaseException as e:  # rank 0 raises it; every executor is released so no rank hangs
            rc = 1
            try:
                self.flow.call(lambda: self.flow.resident_pool().pause_all("abort"))
            except Exception:
                pass
            if self.bench is not None:
                try:
                    self.bench.send({"ev": "error", "message": repr(e)})
                except OSError:
                    pass
            self.log(f"control failed: {e!r}")
        finally:
            self.flow.shutdown(stop_running=False, timeout=10)
            self.listener.close()
        return rc

    def _summarise(self, gids, t0_wall: float, base) -> dict:
        from polyaxon_amd.polyflow.scheduler import device_footprint

        st = self.flow.store
        q = ",".join("?" * len(gids))
        xs = st.list_experiments(ids=[r["id"] for r in st.execute(
            f"SELECT id FROM experiments WHERE group_id IN ({q})", gids).fetchall()])
        trials = len(xs)
        ok = sum(1 for x in xs if x["status"] == "succeeded")
        steps = sum(int(r["step"] or 0) for r in st.execute(
            f"SELECT m.step FROM experiment_metrics m JOIN experiments e ON e.id = m.experiment_id "
            f"WHERE e.group_id IN ({q})", gids).fetchall())
        target = self.args.target
        hit = [x["finished_at"] for x in xs
               if (x.get("last_metric") or {}).get("loss") is not None and x["last_metric"]["loss"] <= target]
        ttt = (min(hit) - t0_wall) if hit else None
        best = min((x["last_metric"]["loss"] for x in xs if (x.get("last_metric") or {}).get("loss") is not None),
                   default=None)
        # per sweep: its best metric and when that sweep first reached the target (the calibration of --target:
        # a target near the task's floor is reached by a minority of sweeps, so the time to it spans several)
        # training steps each trial ran (its metric rows' last step: resumed trials train only the increment)
        trial_steps = {int(r["experiment_id"]): int(r["s"] or 0) for r in st.execute(
            f"SELECT m.experiment_id, MAX(m.step) AS s FROM experiment_metrics m JOIN experiments e "
            f"ON e.id = m.experiment_id WHERE e.group_id IN ({q}) GROUP BY m.experiment_id", gids).fetchall()}
        per_sweep = []
        for g in gids:
            gx = [x for x in xs if x["group_id"] == g and (x.get("last_metric") or {}).get("loss") is not None]
            b = min((x["last_metric"]["loss"] for x in gx), default=None)
            h = [x["finished_at"] for x in gx if x["last_metric"]["loss"] <= target]
            hit = min(h) if h else None
            # the sweep's own training up to (and including) the trial that first reached the target: a time to
            # target that does not depend on how many sweeps share the GPU (they are submitted together)
            to_hit = sum(trial_steps.get(x["id"], 0) for x in gx if hit is not None and x["finished_at"] <= hit)
            per_sweep.append({"group": g, "best": round(b, 4) if b is not None else None,
                              "hit_s": round(hit - t0_wall, 2) if hit is not None else None,
                              "steps_to_hit": to_hit if hit is not None else None,
                              "steps": sum(trial_steps.get(x["id"], 0) for x in gx)})
        # per training budget (resource units): trials and their best / median metric -- what each rung bought
        by_units: dict = {}
        for x in xs:
            u = (x.get("declarations") or {}).get("units")
            v = (x.get("last_metric") or {}).get("loss")
            if u is not None and v is not None:
                by_units.setdefault(str(u), []).append(float(v))
        per_units = {u: {"trials": len(v), "best": round(min(v), 4), "median": round(sorted(v)[len(v) // 2], 4)}
                     for u, v in sorted(by_units.items(), key=lambda kv: float(kv[0]))}
        # the status history every trial must show (reference ExperimentLifeCycle)
        want = ["created", "scheduled", "starting", "running", "succeeded"]
        sample = xs[:: max(1, len(xs) // 50)]
        fsm_ok = all([s["status"] for s in st.experiment_statuses(x["id"])] == want
                     for x in sample if x["status"] == "succeeded")
        resumed = sum(1 for x in xs if x["cloning_strategy"] == "resume")
        units = sum(1 for it in st.execute(
            f"SELECT data FROM experiment_group_iterations WHERE group_id IN ({q})", gids).fetchall()
            if json.loads(it["data"]).get("bracket_iteration") == 0)
        # devices held by every trial's job (a DP=2 trial: both of its gang's devices)
        trial_devices: dict = {}
        for x in xs:
            for j in st.experiment_jobs(x["id"]):
                n = str(len(j.get("devices") or []))
                trial_devices[n] = trial_devices.get(n, 0) + 1
        pool = self.flow.call(lambda: self.flow.resident_pool().snapshot())
        b = {w["wid"]: w for w in base}
        execs = []
        for w in pool:
            w0 = b.get(w["wid"], {})
            execs.append({"wid": w["wid"], "devices": w["devices"], "pid": w["pid"],
                          "load_units": round(w["assigned_units"] - w0.get("assigned_units", 0.0), 3),
                          "units_of_work": w["assigned"] - w0.get("assigned", 0)})
        bo_groups = []
        if self.args.config == "gpt2_bo":  # per BO group: the random batch's best vs the GP iterations' best
            for g in gids:
                its = sorted(st.iterations(g), key=lambda i: i["data"]["iteration"])
                loss = {x["id"]: x["last_metric"]["loss"] for x in xs
                        if x["group_id"] == g and (x.get("last_metric") or {}).get("loss") is not None}
                rnd = [loss[i] for i in (its[0]["data"]["experiment_ids"] if its else []) if i in loss]
                bo = [loss[i] for it in its[1:] for i in it["data"]["experiment_ids"] if i in loss]
                allv = list(loss.values())
                bo_groups.append({"group": g, "random_best": round(min(rnd), 4) if rnd else None,
                                  "bo_best": round(min(bo), 4) if bo else None,
                                  "bo_beats_random": bool(rnd and bo and min(bo) < min(rnd)),
                                  "spread": round(max(allv) - min(allv), 4) if allv else None,
                                  "suggest": [it["data"].get("suggest") for it in its[1:]]})
        return {"trials": trials, "succeeded": ok, "train_steps": steps, "ttt": ttt, "best": best, "per_sweep": per_sweep,
                "bo_groups": bo_groups,
                "per_units": per_units, "trial_devices": trial_devices,
                "fsm_ok": fsm_ok, "resumed": resumed, "brackets": units, "groups": len(gids), "executors": execs,
                "control_pid": os.getpid(), "control_device_footprint": device_footprint()}


def control_main(args) -> int:
    """``--control-only``: the scheduler process rank 0 starts under torchrun (or a single-GPU run)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    srv = ControlServer(args, world)
    print(f"PLX_BENCH_CONTROL 127.0.0.1:{srv.port}", flush=True)
    return srv.serve()


def _spawn_control(argv):
    """Start the control process (no GPU), return (Popen, "host:port")."""
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv, "--control-only"],
                         stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if not line.startswith("PLX_BENCH_CONTROL "):
        p.kill()
        raise RuntimeError(f"control process did not start: {line!r}")
    return p, line.split()[1]


# ----------------------------------------------------------------------------- launcher (no GPU calls here)
def _median(v):
    v = sorted(v)
    if not v:
        return None
    return v[len(v) // 2] if len(v) % 2 else round((v[len(v) // 2 - 1] + v[len(v) // 2]) / 2, 3)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, args, argv) -> int:
    """``--gpus N`` without torchrun: host the scheduler here (this process never initialises the GPU runtime) and
    start N rank processes, one per GPU."""
    srv = ControlServer(args, n)
    ctl = threading.Thread(target=srv.serve, name="bench-control", daemon=True)
    ctl.start()
    env = dict(os.environ)
    env.update({"WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()),
                "LOCAL_WORLD_SIZE": str(n), "PLX_BENCH_CONTROL": f"127.0.0.1:{srv.port}"})
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=e))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    ctl.join(timeout=60)
    return rc


def _physical_gpu(local_rank: int, world: int):
    """KFD index of this rank's GPU, or None when it cannot be known before the GPU runtime starts.  The KFD topology
    lists every GPU of the machine whatever this process may use: with HIP/ROCR_VISIBLE_DEVICES the rank's GPU is
    that list's entry; without it the ranks own the node's GPUs in order only when they use all of them (the
    driver's whole-node runs).  A 1-GPU lease on a shared machine is neither: pinning it to GPU 0's CPUs measured
    20 % slower (remote NUMA node for the launch path), so it is left unpinned."""
    from polyaxon_amd.obs.nodes import kfd_gpus

    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        ids = [v for v in vis.split(",") if v.strip()]
        return int(ids[local_rank]) if local_rank < len(ids) and ids[local_rank].strip().isdigit() else None
    n = len(kfd_gpus())
    return local_rank if n and n == world else None


def _pin_cpus(local_rank: int, world: int) -> list:
    """Bind this rank to the CPUs local to its GPU (NUMA node of the PCIe root) before torch starts its threads."""
    from polyaxon_amd.polyflow.devices import device_cpus

    phys = _physical_gpu(local_rank, world)
    if phys is None:
        return []
    cpus = device_cpus(phys)
    if cpus:
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            return []
    return cpus or []


def main() -> int:
    args = _args()
    if args.control_only:
        return control_main(args)
    argv = sys.argv[1:]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus, args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    pinned = [] if args.cpu else _pin_cpus(local, world)
    # The result is ONE JSON line on stdout.  Native libraries print to fd 1 on their own (RCCL's version banner at
    # communicator init), so fd 1 is pointed at stderr for the rest of the run and the JSON goes to a saved copy
    # of the original stdout.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ctl_addr = os.environ.get("PLX_BENCH_CONTROL")
    ctl_proc = None
    if ctl_addr is None and rank == 0:  # torchrun / single GPU: the scheduler gets a process of its own
        ctl_proc, ctl_addr = _spawn_control(argv)

    import torch
    import torch.distributed as dist

    from polyaxon_amd.polyflow.resident import Channel, ResidentWorker, _FollowerChannel, _LeaderChannel

    def log(msg):
        if rank == 0:
            print(f"[bench +{time.perf_counter() - T0:.1f}s] {msg}", file=sys.stderr, flush=True)

    program, params = program_params(args)
    if args.cpu:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // (2 * world)))  # ranks must not oversubscribe the CPU
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        # The process group is the gloo rendezvous: the ranks' control traffic (control address, barriers around the
        # timed region) and the RCCL unique id; the per-rank gather runs on the framework RCCL communicator
        # (parallel/comm.py), alive for the whole run (below).
        dist.init_process_group("gloo")
        addr = [ctl_addr]
        dist.broadcast_object_list(addr, src=0)
        ctl_addr = addr[0]
    host, _, port = ctl_addr.rpartition(":")
    # --trial-gpus T > 1: ranks [g T, (g + 1) T) form DP gang g -- one resident executor whose trials train
    # data-parallel over the gang's subgroup (FlatDDP on the gang's framework RCCL communicator); its rank 0 talks to
    # the scheduler and re-broadcasts the control stream to the others (polyflow/resident.py _GangGroup)
    tg = args.trial_gpus
    gang_group = None
    if tg > 1:
        groups = [dist.new_group(list(range(g * tg, (g + 1) * tg))) for g in range(world // tg)]
        gang_group = groups[rank // tg]
    leader = rank % tg == 0

    def barrier():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    # The framework's RCCL communicator is alive for the whole run, as in a DP trial (round 4: with 4 hardware queues
    # its streams pushed the side stream onto the compute stream's queue, -17 %, profiles/r4_rccl_slowdown.md; the
    # side stream now has a queue of its own, profiles/r5_hw_queues.md)
    early_comm = None
    if dev.type == "cuda":
        from polyaxon_amd.parallel.rccl import RcclComm

        try:
            if world > 1:
                from polyaxon_amd.parallel import comm as _comm

                early_comm = _comm.acquire(None, dev)
            else:
                early_comm = RcclComm(RcclComm.new_unique_id(), 1, 0, local)
        except Exception as e:  # built again after the timed region (or gloo) rather than fail the run
            print(f"bench: early RCCL communicator unavailable ({e})", file=sys.stderr)
    worker = ResidentWorker(program, params, device=dev, max_active=args.max_active)
    if gang_group is not None:
        worker.join_gang(rank % tg, tg, group=gang_group)
    log(f"building {program} executors (batch {params['batch']}, image {params.get('image')}, config {args.config}, "
        f"{tg} GPU(s) per trial)")
    worker._ready_info = worker.build()
    log(f"executor ready in {worker._ready_info['build_s']} s")
    chan = ctl = None
    if leader:
        chan = Channel.connect(host, int(port), timeout=300)
        first = local if world > 1 else 0
        chan.send({"rank": first, "devices": list(range(first, first + tg))})
        ctl = _LeaderChannel(chan, worker.gang) if worker.gang is not None else chan
    else:
        ctl = _FollowerChannel(worker.gang)
    bench = None
    if rank == 0:
        bench = Channel.connect(host, int(port), timeout=300)
        bench.send({"bench": 1})

    r = worker.serve(ctl)                       # warm-up sweeps, until paused
    if r != "pause:warm":
        raise RuntimeError(f"executor stopped during warm-up: {r}")
    s0 = dict(worker.stats)
    barrier()
    t0 = time.perf_counter()
    if bench is not None:
        bench.send({"op": "go", "t0": time.time()})
        log("timed region")
    r = worker.serve(ctl)                       # timed sweeps, until paused
    barrier()
    elapsed = time.perf_counter() - t0
    if r != "pause:timed":
        raise RuntimeError(f"executor stopped during the timed region: {r}")
    ex = worker.program.executor
    with torch.no_grad():  # fingerprint of the final weights: the ranks of one DP gang must hold identical ones
        p64 = ex.flat.params.detach().double()
        w_sum = float(p64.sum())
        w_mix = float((p64 * torch.arange(p64.numel(), device=p64.device, dtype=torch.float64).remainder_(97).add_(1))
                      .sum())
    mine = [elapsed, worker.stats["trials"] - s0["trials"], worker.stats["train_steps"] - s0["train_steps"],
            float(os.getpid())] + [worker.stats[k] - s0[k] for k in ("idle_s", "round_s", "sync_s")] + [
            float(ex.ddp.launched if ex.ddp is not None else 0),
            float(ex.ddp._comm is not None) if ex.ddp is not None else 0.0, w_sum, w_mix]
    # framework-owned collective (csrc/rccl_comm.cpp) for the per-rank gather on the GPU path (the early communicator,
    # or one created now).
    comm = early_comm
    if comm is None and dev.type == "cuda":
        from polyaxon_amd.parallel.rccl import RcclComm

        try:
            comm = (RcclComm.from_torch_distributed() if world > 1
                    else RcclComm(RcclComm.new_unique_id(), 1, 0, local))
        except Exception as e:  # a communicator that cannot be built must not cost the measured result
            print(f"bench: RCCL communicator unavailable ({e}); per-rank gather over gloo", file=sys.stderr)
            comm = None
    if comm is not None:
        t = torch.tensor(mine, dtype=torch.float64, device=dev)
        per_rank = comm.all_gather(t).cpu().tolist()
        torch.cuda.synchronize(dev)
    elif world > 1:
        g = [torch.zeros(len(mine), dtype=torch.float64) for _ in range(world)]
        dist.all_gather(g, torch.tensor(mine, dtype=torch.float64))
        per_rank = [x.tolist() for x in g]
    else:
        per_rank = [mine]
    elapsed_max = max(p[0] for p in per_rank)
    rc = 0
    if rank == 0:
        msg = bench.recv(timeout=900)
        if msg is None or msg.get("ev") != "result":
            raise RuntimeError(f"control process failed: {msg}")
        res = msg["result"]
        value = res["trials"] / elapsed_max * 3600.0
        n_exec = world // tg
        search = (f"hyperband max_iter={MAX_ITER} eta={ETA} resume=true, 3 brackets / 23 trials per sweep"
                  if args.search == "hyperband" else
                  f"asha min_resource=1 max_resource={ASHA_MAX} eta={ETA} resume=true, {args.asha_n} configs per sweep")
        gpt2 = args.config == "gpt2_bo"
        if gpt2:
            search = (f"bo (GP-UCB, matern 2.5, unit space: log-lr) over lr / weight_decay / beta2: "
                      f"{args.bo_initial * n_exec} random + "
                      f"{args.bo_iterations} x {args.bo_concurrency * n_exec} constant-liar suggestions per group, "
                      f"{params['trial_units'] * params['unit_steps']} AdamW steps per trial")
        out = {
            "metric": METRIC_BO if gpt2 else METRIC,
            "value": round(value, 2),
            "unit": "trials/hour",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": (("synthetic chain tokens (x_{t+1} = (a x_t + b) mod 4093 from a random start, 1024 per sequence, "
                      "vocab 50257; ops/synth.py SyntheticChain)" if args.task == "chain" else
                      "synthetic copy-task tokens (64-token phrases repeated to 1024, vocab 50257; ops/synth.py "
                      "SyntheticTokens)") + ", fresh batch generated on the device every step; random-init weights"
                     if gpt2
                     else "synthetic ImageNet-shape (224x224x3, 1000 classes), fresh learnable batch generated on "
                          "the device every step (ops/synth.py); random-init weights"),
            "config": {
                "model": (("gpt2_125m" if dev.type == "cuda" else "gpt2 tiny (CPU rehearsal)") if gpt2 else
                          ("resnet50" if dev.type == "cuda" else "resnet18ish (CPU rehearsal)")),
                "global_batch": params["batch"] * world,
                "per_trial_batch": params["batch"] * tg,
                "per_trial_world": tg,
                "seq_len": params.get("seq"),
                "image_size": params.get("image"),
                "parallelism": (f"trial-parallel x{world} (resident executor per GPU, brackets balanced by polyflow)"
                                if tg == 1 else
                                f"trial-parallel x{n_exec}, each trial dp{tg} (resident executor per DP gang: FlatDDP "
                                f"over the framework RCCL communicator)"),
                "search": search,
                "unit_steps": params["unit_steps"],
                "step": "one complete sweep per GPU",
                "sweeps": res["groups"],
                "brackets": res["brackets"],
                "signal": args.signal,
                "active_classes": params.get("active_classes"),
            },
            "trials": res["trials"],
            "trials_succeeded": res["succeeded"],
            "trials_resumed": res["resumed"],
            # every rank of a DP=T trial trains its own per-rank batch each step
            "train_images_per_s": round(res["train_steps"] * params["batch"] * tg / elapsed_max, 1),
            "wall_clock_to_target_s": round(res["ttt"], 3) if res["ttt"] is not None else None,
            "target_loss": args.target,
            "best_loss": round(res["best"], 4) if res["best"] is not None else None,
            "sweeps_reaching_target": sum(1 for p in res["per_sweep"] if p["hit_s"] is not None),
            "sweep_best_loss": [p["best"] for p in res["per_sweep"]],
            # time to target as a distribution over the timed sweeps: wall seconds from the timed region's start
            # (sweeps share the GPU, so these grow with the number submitted together) and the sweep's own training
            # up to its first hit converted at the measured step rate (comparable across search strategies)
            "sweep_hit_s": [p["hit_s"] for p in res["per_sweep"]],
            "target_hit_fraction": round(sum(1 for p in res["per_sweep"] if p["hit_s"] is not None)
                                         / max(1, len(res["per_sweep"])), 3),
            "median_time_to_target_s": _median([p["hit_s"] for p in res["per_sweep"] if p["hit_s"] is not None]),
            "median_train_s_to_target": _median([round(p["steps_to_hit"] * elapsed_max / max(1, res["train_steps"])
                                                       * world, 3)
                                                 for p in res["per_sweep"] if p["steps_to_hit"] is not None]),
            "sweep_steps_to_target": [p["steps_to_hit"] for p in res["per_sweep"]],
            "loss_by_units": res["per_units"],
            **({"bo_groups": res["bo_groups"],
                "bo_beats_random_fraction": round(sum(1 for b in res["bo_groups"] if b["bo_beats_random"])
                                                  / max(1, len(res["bo_groups"])), 3),
                "trial_loss_spread_median": _median([b["spread"] for b in res["bo_groups"] if b["spread"] is not None]),
                "chance_loss": round(math.log(50257), 4)} if gpt2 else {}),
            "store_fsm_history_ok": res["fsm_ok"],
            "path": "polyflow scheduler (own process) + SQLite store + resident executors (same path as plx run)",
            "hip_graph": bool(worker._ready_info.get("hip_graph")),
            "per_rank": [{"rank": i, "pid": int(p[3]), "elapsed_s": round(p[0], 3), "trials": int(p[1]),
                          "train_steps": int(p[2]), "idle_s": round(p[4], 3), "round_s": round(p[5], 3),
                          "sync_s": round(p[6], 3), "gang": i // tg, "ddp_collectives": int(p[7]),
                          "ddp_on_framework_comm": bool(p[8]), "weights_fingerprint": [p[9], p[10]]}
                         for i, p in enumerate(per_rank)],
            "trial_devices": res["trial_devices"],
            "executors": res["executors"],
            "control_pid": res["control_pid"],
            # the scheduler process (polyflow + BO GP requests to the executors) holds no GPU state
            "control_device_footprint": res.get("control_device_footprint"),
            "cpus_pinned": len(pinned),
        }
        print(json.dumps(out), file=result_out, flush=True)
    if chan is not None:
        chan.close()
    if bench is not None:
        bench.close()
    worker.close_gang()
    if comm is not None:
        if comm is early_comm and world > 1:
            from polyaxon_amd.parallel import comm as _comm

            _comm.release(comm)  # acquired from the registry above
        else:
            comm.close()
    if world > 1:
        dist.destroy_process_group()
    if ctl_proc is not None:
        try:
            rc = max(rc, ctl_proc.wait(timeout=60))
        except subprocess.TimeoutExpired:
            ctl_proc.kill()
    return rc


if __name__ == "__main__":
    sys.exit(main())
