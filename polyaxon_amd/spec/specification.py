"""Polyaxonfile specifications: experiment, group, job, build, notebook, tensorboard, pipeline.

Re-creates the external ``polyaxon_schemas`` specification layer the reference imports
(polyaxon/schemas/specifications.py:1-14, used through polyaxon/libs/spec_validation.py:19-128) from its
documentation (docs/templates/polyaxonfile_specification/{introduction,sections}.md) and call sites:
``ExperimentSpecification.read/cluster_def/total_resources/get_worker_resources/patch``,
``GroupSpecification.get_experiment_spec(matrix_declaration)/hptuning/matrix_space``.

Reading accepts a path, a YAML/JSON string, a dict, or a list of those merged in order (later files
override earlier ones key by key, like multi-file ``polyaxon run -f a.yml -f b.yml``).
"""
from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, List, Optional, Sequence, Union

import numpy as np
import yaml

from polyaxon_amd.spec.environment import EnvironmentSpec, PodResources
from polyaxon_amd.spec.hptuning import HPTuningConfig
from polyaxon_amd.spec.matrix import MatrixValidationError, space_size
from polyaxon_amd.spec.templating import TemplateError, has_template, render


class PolyaxonfileError(ValueError):
    pass


class Kinds:
    EXPERIMENT = "experiment"
    GROUP = "group"
    JOB = "job"
    BUILD = "build"
    NOTEBOOK = "notebook"
    TENSORBOARD = "tensorboard"
    PIPELINE = "pipeline"
    VALUES = (EXPERIMENT, GROUP, JOB, BUILD, NOTEBOOK, TENSORBOARD, PIPELINE)


SECTIONS = ("version", "kind", "project", "name", "description", "tags", "logging", "declarations", "build", "run",
            "environment", "hptuning", "settings", "ops", "concurrency", "schedule", "image", "trigger", "model",
            "train", "eval")


def _deep_merge(a: Dict[str, Any], b: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(a)
    for k, v in (b or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _load_one(value: Any) -> Dict[str, Any]:
    if isinstance(value, dict):
        return copy.deepcopy(value)
    if isinstance(value, (str, os.PathLike)):
        s = str(value)
        if "\n" not in s and os.path.exists(s):
            with open(s) as f:
                s = f.read()
        try:
            data = yaml.safe_load(s)
        except yaml.YAMLError as e:
            try:
                data = json.loads(s)
            except ValueError:
                raise PolyaxonfileError(f"cannot parse Polyaxonfile: {e}") from None
        if not isinstance(data, dict):
            raise PolyaxonfileError("a Polyaxonfile must be a mapping")
        return data
    raise PolyaxonfileError(f"unsupported Polyaxonfile value {type(value)}")


def read_raw(values: Union[Any, Sequence[Any]]) -> Dict[str, Any]:
    if isinstance(values, (list, tuple)):
        data: Dict[str, Any] = {}
        for v in values:
            data = _deep_merge(data, _load_one(v))
        return data
    return _load_one(values)


class BuildConfig:
    def __init__(self, d: Dict[str, Any]):
        if not isinstance(d, dict):
            raise PolyaxonfileError("build must be a mapping")
        self.image = d.get("image")
        self.build_steps: List[str] = list(d.get("build_steps") or [])
        self.env_vars: List[List[str]] = [list(e) for e in d.get("env_vars") or []]
        self.git = d.get("git")
        self.ref = d.get("ref")
        self.nocache = bool(d.get("nocache", False))
        self.dockerfile = d.get("dockerfile")
        if not self.image and not self.dockerfile and not self.git:
            raise PolyaxonfileError("build requires an `image` (or a `dockerfile`, or a `git` source)")
        for e in self.env_vars:
            if len(e) != 2:
                raise PolyaxonfileError(f"build.env_vars entries are [key, value] pairs, got {e}")

    def to_dict(self):
        out = {"image": self.image}
        for k in ("build_steps", "env_vars", "git", "ref", "dockerfile"):
            if getattr(self, k):
                out[k] = getattr(self, k)
        if self.nocache:
            out["nocache"] = True
        return out


class RunConfig:
    def __init__(self, d: Dict[str, Any]):
        if not isinstance(d, dict) or "cmd" not in d:
            raise PolyaxonfileError("run requires `cmd`")
        self.cmd = d["cmd"]
        if not isinstance(self.cmd, (str, list)):
            raise PolyaxonfileError("run.cmd must be a string or a list of strings")

    def to_dict(self):
        return {"cmd": self.cmd}

    @property
    def commands(self) -> List[str]:
        return [self.cmd] if isinstance(self.cmd, str) else list(self.cmd)


class BaseSpecification:
    KIND: Optional[str] = None

    def __init__(self, data: Dict[str, Any], render_templates: bool = True):
        if not isinstance(data, dict):
            raise PolyaxonfileError("specification must be a mapping")
        self.raw_data = copy.deepcopy(data)
        version = data.get("version")
        if version is None:
            raise PolyaxonfileError("the Polyaxonfile must define `version`")
        if int(version) != 1:
            raise PolyaxonfileError(f"unsupported Polyaxonfile version {version}")
        kind = data.get("kind")
        if kind not in Kinds.VALUES:
            raise PolyaxonfileError(f"unknown kind `{kind}`; expected one of {Kinds.VALUES}")
        if self.KIND and kind != self.KIND:
            raise PolyaxonfileError(f"expected kind `{self.KIND}`, got `{kind}`")
        unknown = set(data) - set(SECTIONS)
        if unknown:
            raise PolyaxonfileError(f"unknown sections {sorted(unknown)}")
        self.declarations: Dict[str, Any] = copy.deepcopy(data.get("declarations") or {})
        if not isinstance(self.declarations, dict):
            raise PolyaxonfileError("declarations must be a mapping")
        parsed = data
        if render_templates:
            try:
                parsed = render(data, self.template_context())
            except TemplateError as e:
                raise PolyaxonfileError(str(e)) from None
        self.parsed_data = parsed
        self._parse(parsed)

    def template_context(self) -> Dict[str, Any]:
        return dict(self.declarations)

    def _parse(self, d: Dict[str, Any]) -> None:
        self.version = int(d["version"])
        self.kind = d["kind"]
        self.project = d.get("project")
        self.name = d.get("name")
        self.description = d.get("description")
        tags = d.get("tags") or []
        if isinstance(tags, str):
            tags = [t.strip() for t in tags.split(",") if t.strip()]
        self.tags: List[str] = list(tags)
        self.logging = d.get("logging") or {}
        if self.logging and self.logging.get("level") not in (None, "DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL"):
            raise PolyaxonfileError(f"invalid logging level {self.logging.get('level')}")
        self.build = BuildConfig(d["build"]) if d.get("build") is not None else None
        self.run = RunConfig(d["run"]) if d.get("run") is not None else None
        try:
            self.environment = EnvironmentSpec.from_dict(d.get("environment"))
        except MatrixValidationError as e:
            raise PolyaxonfileError(str(e)) from None

    # ------------------------------------------------------------------ construction helpers
    @classmethod
    def read(cls, values, **kw) -> "BaseSpecification":
        data = read_raw(values)
        if cls is BaseSpecification:
            return specification_for(data, **kw)
        return cls(data, **kw)

    def patch(self, values: Dict[str, Any]) -> "BaseSpecification":
        return type(self)(_deep_merge(self.raw_data, values))

    def to_dict(self) -> Dict[str, Any]:
        return copy.deepcopy(self.parsed_data)

    # ------------------------------------------------------------------ environment helpers
    @property
    def resources(self) -> Optional[PodResources]:
        return self.environment.resources

    @property
    def framework(self) -> Optional[str]:
        return self.environment.framework.framework if self.environment.framework else None

    @property
    def is_distributed(self) -> bool:
        fw = self.environment.framework
        return bool(fw and (fw.n_workers or fw.n_ps))

    @property
    def cluster_def(self):
        """({role: count}, is_distributed) — reference ExperimentSpecification.cluster_def."""
        fw = self.environment.framework
        cluster = {"master": 1}
        if fw:
            if fw.n_workers:
                cluster["worker"] = fw.n_workers
            if fw.n_ps:
                cluster["ps"] = fw.n_ps
        return cluster, self.is_distributed

    def get_worker_resources(self, index: int) -> Optional[PodResources]:
        fw = self.environment.framework
        return fw.replica_resources("worker", index) if fw else None

    def get_ps_resources(self, index: int) -> Optional[PodResources]:
        fw = self.environment.framework
        return fw.replica_resources("ps", index) if fw else None

    @property
    def total_resources(self) -> Optional[PodResources]:
        total = self.resources
        fw = self.environment.framework
        if fw:
            for i in range(fw.n_workers):
                r = self.get_worker_resources(i)
                total = r if total is None else total + r
            for i in range(fw.n_ps):
                r = self.get_ps_resources(i)
                total = r if total is None else total + r
        return total

    @property
    def total_gpus(self) -> int:
        t = self.total_resources
        return t.gpus if t else 0


class ExperimentSpecification(BaseSpecification):
    KIND = Kinds.EXPERIMENT

    def __init__(self, data: Dict[str, Any], render_templates: bool = True, group_trial: bool = False):
        # group_trial: the spec of one trial of a group (GroupSpecification.get_experiment_spec).  Only such a spec
        # may name a resident executor without a `run`: the group's resident driver trains it; the scheduler has no
        # resident path for a standalone experiment, so one would only fail later, at spawn ("nothing to run").
        self._group_trial = group_trial
        super().__init__(data, render_templates=render_templates)

    def _parse(self, d):
        super()._parse(d)
        if d.get("hptuning") is not None:
            raise PolyaxonfileError("an experiment cannot define `hptuning`; use kind: group")
        ex = self.environment.executor
        if ex is not None and ex.resident and not getattr(self, "_group_trial", False):
            raise PolyaxonfileError("`environment.executor: resident` runs the trials of a group (kind: group); "
                                    "a standalone experiment uses executor: process with a `run` section")
        if self.run is None and d.get("model") is None and not (ex is not None and ex.resident):
            raise PolyaxonfileError("an experiment requires a `run` section")


class JobSpecification(BaseSpecification):
    KIND = Kinds.JOB

    def _parse(self, d):
        super()._parse(d)
        if self.run is None:
            raise PolyaxonfileError("a job requires a `run` section")
        if self.environment.framework:
            raise PolyaxonfileError("a job cannot define a distributed framework")


class BuildSpecification(BaseSpecification):
    KIND = Kinds.BUILD

    def _parse(self, d):
        super()._parse(d)
        if self.build is None:
            raise PolyaxonfileError("a build specification requires a `build` section")


class NotebookSpecification(BaseSpecification):
    KIND = Kinds.NOTEBOOK

    def _parse(self, d):
        super()._parse(d)
        if self.build is None:
            self.build = BuildConfig({"image": "python:3"})


class TensorboardSpecification(BaseSpecification):
    KIND = Kinds.TENSORBOARD

    def _parse(self, d):
        super()._parse(d)
        if self.build is None:
            self.build = BuildConfig({"image": "tensorflow/tensorflow"})


class GroupSpecification(BaseSpecification):
    KIND = Kinds.GROUP

    def __init__(self, data: Dict[str, Any], render_templates: bool = True):
        if not data.get("hptuning"):
            raise PolyaxonfileError("a group requires an `hptuning` section with a `matrix`")
        try:
            self.hptuning = HPTuningConfig.from_dict(data["hptuning"])
        except (MatrixValidationError, KeyError, TypeError) as e:
            raise PolyaxonfileError(f"invalid hptuning: {e}") from None
        if not self.hptuning.matrix:
            raise PolyaxonfileError("hptuning requires a non-empty `matrix`")
        super().__init__(data, render_templates=False)
        # validate the templates with one matrix sample, as experiments will render them
        sample = {k: _first_value(v) for k, v in self.hptuning.matrix.items()}
        for algo in (self.hptuning.hyperband, self.hptuning.asha):
            if algo is not None:  # the resource is injected into every suggestion
                sample[algo.resource.name] = algo.resource.cast_value(1)
        try:
            self.get_experiment_spec(sample)
        except PolyaxonfileError as e:
            raise PolyaxonfileError(f"group template does not render with a matrix sample: {e}") from None

    @property
    def matrix(self):
        return self.hptuning.matrix

    @property
    def search_algorithm(self) -> str:
        return self.hptuning.search_algorithm

    @property
    def concurrency(self) -> int:
        return self.hptuning.concurrency

    @property
    def early_stopping(self):
        return self.hptuning.early_stopping

    @property
    def matrix_space(self) -> Optional[int]:
        return space_size(self.hptuning.matrix)

    def experiment_data(self, matrix_declaration: Dict[str, Any]) -> Dict[str, Any]:
        data = {k: v for k, v in copy.deepcopy(self.raw_data).items() if k != "hptuning"}
        data["kind"] = Kinds.EXPERIMENT
        decl = dict(data.get("declarations") or {})
        decl.update(matrix_declaration)
        data["declarations"] = decl
        return data

    def get_experiment_spec(self, matrix_declaration: Dict[str, Any]) -> ExperimentSpecification:
        return ExperimentSpecification(self.experiment_data(matrix_declaration), group_trial=True)


def _first_value(m):
    if m.is_discrete:
        v = m.to_numpy()[0]
        return v.item() if hasattr(v, "item") else v
    return m.sample(rand_generator=np.random.RandomState(0))


class PipelineSpecification(BaseSpecification):
    """``kind: pipeline`` — a DAG of operations (reference pipelines/ + operations/, db/models/pipelines.py).

    ops: [{name, upstream: [names], trigger: all_succeeded|all_failed|all_done|one_succeeded|one_failed|one_done,
           max_retries, retry_delay, retry_exponential_backoff, max_retry_delay, timeout, concurrency,
           template: <inline Polyaxonfile of kind experiment|job|group>}]
    plus pipeline-level ``concurrency`` and optional ``schedule: {frequency | cron, start_at, end_at,
    depends_on_past, max_runs}`` (polyflow/schedules.py).
    """
    KIND = Kinds.PIPELINE
    TRIGGERS = ("all_succeeded", "all_failed", "all_done", "one_succeeded", "one_failed", "one_done")

    def _parse(self, d):
        super()._parse(d)
        ops = d.get("ops")
        if not ops or not isinstance(ops, list):
            raise PolyaxonfileError("a pipeline requires a non-empty `ops` list")
        names = set()
        self.ops = []
        for op in ops:
            if "name" not in op:
                raise PolyaxonfileError("every pipeline op needs a `name`")
            if op["name"] in names:
                raise PolyaxonfileError(f"duplicate op name {op['name']}")
            names.add(op["name"])
            trig = op.get("trigger", "all_succeeded")
            if trig not in self.TRIGGERS:
                raise PolyaxonfileError(f"unknown trigger policy {trig}")
            tmpl = op.get("template")
            if tmpl is not None:
                specification_for(tmpl)
            self.ops.append(dict(op, trigger=trig, upstream=list(op.get("upstream") or op.get("dependencies") or [])))
        for op in self.ops:
            missing = [u for u in op["upstream"] if u not in names]
            if missing:
                raise PolyaxonfileError(f"op {op['name']} depends on unknown ops {missing}")
        self.concurrency = int(d.get("concurrency") or 0) or None
        self.schedule = d.get("schedule")
        if self.schedule is not None:
            from polyaxon_amd.polyflow.schedules import Schedule, ScheduleError

            try:
                Schedule.from_dict(self.schedule)
            except (ScheduleError, ValueError, TypeError) as e:
                raise PolyaxonfileError(f"invalid schedule: {e}") from None


_KIND_TO_SPEC = {
    Kinds.EXPERIMENT: ExperimentSpecification,
    Kinds.GROUP: GroupSpecification,
    Kinds.JOB: JobSpecification,
    Kinds.BUILD: BuildSpecification,
    Kinds.NOTEBOOK: NotebookSpecification,
    Kinds.TENSORBOARD: TensorboardSpecification,
    Kinds.PIPELINE: PipelineSpecification,
}


def specification_for(values, **kw) -> BaseSpecification:
    data = read_raw(values)
    kind = data.get("kind")
    if kind not in _KIND_TO_SPEC:
        raise PolyaxonfileError(f"unknown kind `{kind}`; expected one of {Kinds.VALUES}")
    return _KIND_TO_SPEC[kind](data, **kw)


def validate(values) -> BaseSpecification:
    """``polyaxon check`` equivalent."""
    return specification_for(values)


__all__ = ["BaseSpecification", "ExperimentSpecification", "GroupSpecification", "JobSpecification",
           "BuildSpecification", "NotebookSpecification", "TensorboardSpecification", "PipelineSpecification",
           "PolyaxonfileError", "Kinds", "specification_for", "validate", "read_raw", "has_template"]
