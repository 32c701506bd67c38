"""``environment`` section: resources, outputs refs, persistence, scheduling hints and distributed topologies.

Contract: docs/templates/polyaxonfile_specification/sections.md:292-714 and the spawners that consume it
(polyaxon/scheduler/spawners/{pytorch,horovod,tensorflow,mxnet}_spawner.py, experiment_scheduler.py:93-385).

MI355X-native meaning of the fields (no Kubernetes): ``resources.gpu`` is a count of HIP devices the
polyflow allocator reserves per replica; ``cpu``/``memory`` are admission budgets; ``node_selector``,
``tolerations`` and ``affinity`` are accepted and recorded (single node) — ``node_selector: {xgmi: pair}``
asks the allocator for xGMI-adjacent devices.  Framework sections define the replica topology:
pytorch/horovod = master + n_workers; tensorflow/mxnet = master + n_workers + n_ps (parameter servers
run as extra DP ranks — documented deviation).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from polyaxon_amd.spec.matrix import MatrixValidationError

FRAMEWORKS = ("tensorflow", "mxnet", "pytorch", "horovod")


@dataclass
class ResourceSpec:
    requests: Optional[float] = None
    limits: Optional[float] = None

    @classmethod
    def from_dict(cls, d):
        if d is None:
            return None
        if isinstance(d, (int, float)):
            return cls(requests=d, limits=d)
        req = d.get("requests", d.get("request"))
        lim = d.get("limits", d.get("limit"))
        if req is not None and lim is not None and float(req) > float(lim):
            raise MatrixValidationError(f"resource requests {req} > limits {lim}")
        return cls(requests=req, limits=lim)

    def to_dict(self):
        return {k: v for k, v in (("requests", self.requests), ("limits", self.limits)) if v is not None}

    @property
    def value(self) -> float:
        v = self.limits if self.limits is not None else self.requests
        return float(v or 0)


@dataclass
class PodResources:
    cpu: Optional[ResourceSpec] = None
    memory: Optional[ResourceSpec] = None
    gpu: Optional[ResourceSpec] = None
    # MI355X extension: HBM budget (GB) a replica reserves on each of its devices, so fractional-GPU trials
    # (``gpu: 0.25``) are packed by memory as well as by compute share (288 GB per MI355X)
    hbm: Optional[ResourceSpec] = None

    KEYS = ("cpu", "memory", "gpu", "hbm")

    @classmethod
    def from_dict(cls, d):
        if not d:
            return None
        unknown = set(d) - set(cls.KEYS)
        if unknown:
            raise MatrixValidationError(f"unknown resources {sorted(unknown)}")
        out = cls(cpu=ResourceSpec.from_dict(d.get("cpu")), memory=ResourceSpec.from_dict(d.get("memory")),
                  gpu=ResourceSpec.from_dict(d.get("gpu")), hbm=ResourceSpec.from_dict(d.get("hbm")))
        if out.gpu is not None:
            g = out.gpu.value
            if g < 0 or (g > 1 and abs(g - round(g)) > 1e-9):
                # a fraction shares one device; more than one device is a gang of whole devices
                raise MatrixValidationError(f"resources.gpu must be a fraction <= 1 or a whole number, got {g}")
        if out.hbm is not None and out.hbm.value < 0:
            raise MatrixValidationError("resources.hbm must be >= 0 (GB)")
        return out

    def to_dict(self):
        return {k: getattr(self, k).to_dict() for k in self.KEYS if getattr(self, k) is not None}

    @property
    def hbm_gb(self) -> float:
        return self.hbm.value if self.hbm else 0.0

    @property
    def gpus(self) -> int:
        return int(self.gpu.value) if self.gpu else 0

    def __add__(self, other: "PodResources") -> "PodResources":
        if other is None:
            return self

        def total(x, y):
            return None if x is None and y is None else float(x or 0) + float(y or 0)

        def add(a, b):
            if a is None or b is None:
                return a if b is None else b
            return ResourceSpec(requests=total(a.requests, b.requests), limits=total(a.limits, b.limits))

        return PodResources(cpu=add(self.cpu, other.cpu), memory=add(self.memory, other.memory),
                            gpu=add(self.gpu, other.gpu), hbm=add(self.hbm, other.hbm))


@dataclass
class ReplicaSpec:
    """Per-replica overrides (``default_worker``, ``worker: [{index, ...}]`` ...)."""
    index: Optional[int] = None
    resources: Optional[PodResources] = None
    node_selector: Optional[Dict[str, Any]] = None
    affinity: Optional[Dict[str, Any]] = None
    tolerations: Optional[List[Dict[str, Any]]] = None

    @classmethod
    def from_dict(cls, d):
        if d is None:
            return None
        return cls(index=d.get("index"), resources=PodResources.from_dict(d.get("resources")),
                   node_selector=d.get("node_selector"), affinity=d.get("affinity"), tolerations=d.get("tolerations"))

    def to_dict(self):
        out = {}
        if self.index is not None:
            out["index"] = self.index
        if self.resources:
            out["resources"] = self.resources.to_dict()
        for k in ("node_selector", "affinity", "tolerations"):
            if getattr(self, k) is not None:
                out[k] = getattr(self, k)
        return out


@dataclass
class FrameworkSpec:
    framework: str
    n_workers: int = 0
    n_ps: int = 0
    default_worker: Optional[ReplicaSpec] = None
    default_ps: Optional[ReplicaSpec] = None
    worker: List[ReplicaSpec] = field(default_factory=list)
    ps: List[ReplicaSpec] = field(default_factory=list)

    @classmethod
    def from_dict(cls, framework: str, d: Dict[str, Any]):
        d = d or {}
        if framework in ("pytorch", "horovod") and d.get("n_ps"):
            raise MatrixValidationError(f"{framework} has no parameter servers (n_ps)")
        workers = [ReplicaSpec.from_dict(w) for w in d.get("worker") or []]
        ps = [ReplicaSpec.from_dict(p) for p in d.get("ps") or []]
        # legacy keys from the docs example
        for w in d.get("worker_resources") or []:
            workers.append(ReplicaSpec(index=w.get("index"), resources=PodResources.from_dict(
                {k: v for k, v in w.items() if k != "index"})))
        for p in d.get("ps_resources") or []:
            ps.append(ReplicaSpec(index=p.get("index"), resources=PodResources.from_dict(
                {k: v for k, v in p.items() if k != "index"})))
        spec = cls(framework=framework, n_workers=int(d.get("n_workers", 0) or 0), n_ps=int(d.get("n_ps", 0) or 0),
                   default_worker=ReplicaSpec.from_dict(d.get("default_worker")),
                   default_ps=ReplicaSpec.from_dict(d.get("default_ps")), worker=workers, ps=ps)
        for r in spec.worker:
            if r.index is None or not 0 <= r.index < spec.n_workers:
                raise MatrixValidationError(f"worker index {r.index} out of range [0, {spec.n_workers})")
        for r in spec.ps:
            if r.index is None or not 0 <= r.index < spec.n_ps:
                raise MatrixValidationError(f"ps index {r.index} out of range [0, {spec.n_ps})")
        return spec

    def to_dict(self):
        out: Dict[str, Any] = {"n_workers": self.n_workers}
        if self.framework in ("tensorflow", "mxnet"):
            out["n_ps"] = self.n_ps
        if self.default_worker:
            out["default_worker"] = self.default_worker.to_dict()
        if self.default_ps:
            out["default_ps"] = self.default_ps.to_dict()
        if self.worker:
            out["worker"] = [w.to_dict() for w in self.worker]
        if self.ps:
            out["ps"] = [p.to_dict() for p in self.ps]
        return out

    def _replica(self, role: str, index: int) -> Optional[ReplicaSpec]:
        specific = {r.index: r for r in (self.worker if role == "worker" else self.ps)}
        default = self.default_worker if role == "worker" else self.default_ps
        return specific.get(index, default)

    def replica_resources(self, role: str, index: int) -> Optional[PodResources]:
        r = self._replica(role, index)
        return r.resources if r else None


@dataclass
class ExecutorSpec:
    """``environment.executor`` (MI355X extension): how polyflow runs the trials of an experiment or group.

    * ``kind: process`` (default) -- every experiment is a fresh process tree running ``run.cmd``, exactly the
      reference's one-pod-per-trial model.
    * ``kind: resident`` -- trials run on warm resident executors (polyflow/resident.py): one long-lived worker
      process per GPU holds the model, its flat weights, the captured step and the HBM snapshots, and receives
      trials over a socket.  ``program`` names the trial program (polyflow/programs.py registry or
      ``module:callable``), ``params`` are its build arguments (batch, image size, ``unit_steps`` = training steps
      per Hyperband resource unit ...), ``max_active_brackets`` bounds how many brackets (or ASHA shards) one
      executor interleaves (each keeps its promotion snapshots in HBM), ``shards`` cuts an ASHA group into that many
      independent asynchronous searches, one per executor (default 1).
    """
    kind: str = "process"
    program: Optional[str] = None
    params: Dict[str, Any] = field(default_factory=dict)
    max_active_brackets: int = 8
    shards: int = 1

    @classmethod
    def from_dict(cls, d):
        if d is None:
            return None
        if isinstance(d, str):
            d = {"kind": d}
        unknown = set(d) - {"kind", "program", "params", "max_active_brackets", "shards"}
        if unknown:
            raise MatrixValidationError(f"unknown executor keys {sorted(unknown)}")
        kind = d.get("kind", "process")
        if kind not in ("process", "resident"):
            raise MatrixValidationError(f"executor.kind must be process or resident, got {kind!r}")
        if kind == "resident" and not d.get("program"):
            raise MatrixValidationError("a resident executor needs `program`")
        n = int(d.get("max_active_brackets", 8))
        if n < 1:
            raise MatrixValidationError("executor.max_active_brackets must be >= 1")
        shards = int(d.get("shards", 1))
        if shards < 1:
            raise MatrixValidationError("executor.shards must be >= 1")
        return cls(kind=kind, program=d.get("program"), params=dict(d.get("params") or {}), max_active_brackets=n,
                   shards=shards)

    def to_dict(self):
        out: Dict[str, Any] = {"kind": self.kind}
        if self.program:
            out["program"] = self.program
        if self.params:
            out["params"] = dict(self.params)
        if self.max_active_brackets != 8:
            out["max_active_brackets"] = self.max_active_brackets
        if self.shards != 1:
            out["shards"] = self.shards
        return out

    @property
    def resident(self) -> bool:
        return self.kind == "resident"


@dataclass
class EnvironmentSpec:
    resources: Optional[PodResources] = None
    outputs: Dict[str, List[Any]] = field(default_factory=dict)
    persistence: Dict[str, Any] = field(default_factory=dict)
    node_selector: Optional[Dict[str, Any]] = None
    tolerations: Optional[List[Dict[str, Any]]] = None
    affinity: Optional[Dict[str, Any]] = None
    secret_refs: List[str] = field(default_factory=list)
    configmap_refs: List[str] = field(default_factory=list)
    env_vars: List[List[str]] = field(default_factory=list)
    framework: Optional[FrameworkSpec] = None
    # MI355X extensions: opt-in trial retry and a heartbeat deadline for hung trials
    max_restarts: int = 0
    heartbeat_timeout: Optional[float] = None
    # wrap every replica in `rocprofv3 --kernel-trace --stats` (outputs/rocprof/<role>.<index>)
    profile: bool = False
    executor: Optional[ExecutorSpec] = None

    @classmethod
    def from_dict(cls, d: Optional[Dict[str, Any]]):
        d = dict(d or {})
        fws = [f for f in FRAMEWORKS if d.get(f) is not None]
        if len(fws) > 1:
            raise MatrixValidationError(f"environment defines more than one framework: {fws}")
        # the reference docs also place the per-replica sections next to the framework section
        # (docs/templates/customization/customize_node_scheduling.md): fold them into it
        replica_keys = [k for k in ("worker", "ps", "default_worker", "default_ps") if k in d]
        if replica_keys:
            if not fws:
                raise MatrixValidationError(f"{replica_keys} need a distributed framework section")
            fw = dict(d[fws[0]] or {})
            for k in replica_keys:
                fw.setdefault(k, d.pop(k))
            d[fws[0]] = fw
        known = {"resources", "outputs", "persistence", "node_selector", "tolerations", "affinity", "secret_refs",
                 "configmap_refs", "env_vars", "max_restarts", "heartbeat_timeout", "profile", "executor", *FRAMEWORKS}
        unknown = set(d) - known
        if unknown:
            raise MatrixValidationError(f"unknown environment keys {sorted(unknown)}")
        if not isinstance(d.get("profile", False), bool):
            raise MatrixValidationError("environment.profile must be true or false")
        outputs = d.get("outputs") or {}
        bad = set(outputs) - {"jobs", "experiments"}
        if bad:
            raise MatrixValidationError(f"environment.outputs only accepts jobs/experiments, got {sorted(bad)}")
        return cls(resources=PodResources.from_dict(d.get("resources")), outputs=outputs,
                   persistence=d.get("persistence") or {}, node_selector=d.get("node_selector"),
                   tolerations=d.get("tolerations"), affinity=d.get("affinity"),
                   secret_refs=list(d.get("secret_refs") or []), configmap_refs=list(d.get("configmap_refs") or []),
                   env_vars=[list(e) for e in d.get("env_vars") or []],
                   framework=FrameworkSpec.from_dict(fws[0], d[fws[0]]) if fws else None,
                   max_restarts=int(d.get("max_restarts") or 0),
                   heartbeat_timeout=float(d["heartbeat_timeout"]) if d.get("heartbeat_timeout") else None,
                   profile=bool(d.get("profile", False)),
                   executor=ExecutorSpec.from_dict(d.get("executor")))

    def to_dict(self):
        out: Dict[str, Any] = {}
        if self.resources:
            out["resources"] = self.resources.to_dict()
        for k in ("outputs", "persistence", "secret_refs", "configmap_refs", "env_vars"):
            if getattr(self, k):
                out[k] = getattr(self, k)
        for k in ("node_selector", "tolerations", "affinity"):
            if getattr(self, k) is not None:
                out[k] = getattr(self, k)
        if self.framework:
            out[self.framework.framework] = self.framework.to_dict()
        if self.max_restarts:
            out["max_restarts"] = self.max_restarts
        if self.heartbeat_timeout:
            out["heartbeat_timeout"] = self.heartbeat_timeout
        if self.profile:
            out["profile"] = True
        if self.executor is not None:
            out["executor"] = self.executor.to_dict()
        return out
