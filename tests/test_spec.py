"""Polyaxonfile parsing, matrix distributions and templating."""
import math

import numpy as np
import pytest

from polyaxon_amd.spec import (ExperimentSpecification, GroupSpecification, MatrixConfig, PolyaxonfileError,
                               specification_for)
from polyaxon_amd.spec.hptuning import HPTuningConfig
from polyaxon_amd.spec.matrix import MatrixValidationError, space_size
from polyaxon_amd.spec.templating import render

GROUP = """
version: 1
kind: group
project: mnist
tags: [fixtures, hb]
declarations:
  batch_size: 64
hptuning:
  seed: 7
  concurrency: 2
  hyperband:
    max_iter: 10
    eta: 3
    resource: {name: steps, type: int}
    metric: {name: loss, optimization: minimize}
    resume: true
  early_stopping:
    - {metric: precision, value: 0.9}
    - {metric: loss, value: 0.1, optimization: minimize}
  matrix:
    lr: {logspace: '0.01:0.1:5'}
    dropout: {linspace: [0.1, 0.5, 5]}
    optimizer: {values: [adam, sgd]}
build:
  image: rocm/pytorch
  build_steps: [pip install -r requirements.txt]
run:
  cmd: python train.py --lr={{ lr }} --bs={{ batch_size }} --opt={{ optimizer }} --steps={{ steps }}
"""


def test_matrix_discrete_options():
    assert list(MatrixConfig.from_dict({"values": [1, 2, 3]}).to_numpy()) == [1, 2, 3]
    assert list(MatrixConfig.from_dict({"range": [1, 5, 1]}).to_numpy()) == [1, 2, 3, 4]
    assert list(MatrixConfig.from_dict({"range": "1:10:3"}).to_numpy()) == [1, 4, 7]
    assert list(MatrixConfig.from_dict({"range": {"start": 0, "stop": 4, "step": 2}}).to_numpy()) == [0, 2]
    np.testing.assert_allclose(MatrixConfig.from_dict({"linspace": [1, 2, 5]}).to_numpy(),
                               [1., 1.25, 1.5, 1.75, 2.])
    np.testing.assert_allclose(MatrixConfig.from_dict({"logspace": "0:2:3"}).to_numpy(), [1, 10, 100])
    np.testing.assert_allclose(MatrixConfig.from_dict({"geomspace": [1, 8, 4]}).to_numpy(), [1, 2, 4, 8])
    m = MatrixConfig.from_dict({"values": ["a", "b"]})
    assert m.is_categorical and m.is_discrete and not m.is_continuous and m.min is None
    n = MatrixConfig.from_dict({"values": [1, 2, 3]})
    assert not n.is_categorical and n.min == 1 and n.max == 3


def test_matrix_distributions_sample_in_support():
    rng = np.random.RandomState(0)
    u = MatrixConfig.from_dict({"uniform": [1, 5]})
    assert u.is_continuous and u.is_uniform and (u.min, u.max) == (1.0, 5.0)
    xs = [u.sample(rand_generator=rng) for _ in range(200)]
    assert all(1 <= x < 5 for x in xs)
    q = MatrixConfig.from_dict({"quniform": {"low": 0, "high": 10, "q": 2}})
    assert all(v % 2 == 0 for v in (q.sample(rand_generator=rng) for _ in range(50)))
    lu = MatrixConfig.from_dict({"loguniform": [math.log(1e-4), math.log(1e-1)]})
    assert all(1e-4 <= v <= 1e-1 for v in (lu.sample(rand_generator=rng) for _ in range(100)))
    ln = MatrixConfig.from_dict({"lognormal": "0:1"})
    assert all(v > 0 for v in (ln.sample(rand_generator=rng) for _ in range(50)))
    pv = MatrixConfig.from_dict({"pvalues": [["a", 0.2], ["b", 0.8]]})
    draws = [pv.sample(rand_generator=rng) for _ in range(400)]
    assert 0.7 < draws.count("b") / 400 < 0.9


@pytest.mark.parametrize("bad", [{"uniform": [5, 1]}, {"pvalues": [["a", 0.5], ["b", 0.2]]}, {"nope": [1]},
                                 {"range": [1, 2]}, {"values": []}, {"normal": [0, -1]}])
def test_matrix_validation(bad):
    with pytest.raises(MatrixValidationError):
        MatrixConfig.from_dict(bad)


def test_space_size():
    m = HPTuningConfig.from_dict({"matrix": {"a": {"values": [1, 2]}, "b": {"range": [0, 3, 1]}}}).matrix
    assert space_size(m) == 6
    m = HPTuningConfig.from_dict({"matrix": {"a": {"values": [1, 2]}, "b": {"uniform": [0, 1]}},
                                  "random_search": {"n_experiments": 3}}).matrix
    assert space_size(m) is None


def test_grid_rejects_continuous():
    with pytest.raises(MatrixValidationError):
        HPTuningConfig.from_dict({"matrix": {"b": {"uniform": [0, 1]}}})


def test_group_spec_and_experiment_rendering():
    g = specification_for(GROUP)
    assert isinstance(g, GroupSpecification)
    assert g.search_algorithm == "hyperband" and g.concurrency == 2 and g.hptuning.seed == 7
    assert len(g.early_stopping) == 2 and g.early_stopping[0].optimization == "maximize"
    assert g.matrix_space == 5 * 5 * 2
    e = g.get_experiment_spec({"lr": 0.01, "dropout": 0.1, "optimizer": "adam", "steps": 3})
    assert isinstance(e, ExperimentSpecification)
    assert e.run.cmd == "python train.py --lr=0.01 --bs=64 --opt=adam --steps=3"
    assert e.declarations["lr"] == 0.01 and e.declarations["batch_size"] == 64
    assert e.tags == ["fixtures", "hb"] and e.build.image == "rocm/pytorch"
    assert "hptuning" not in e.parsed_data


def test_group_rejects_unrenderable_template():
    bad = GROUP.replace("{{ optimizer }}", "{{ missing_name }}")
    with pytest.raises(PolyaxonfileError):
        specification_for(bad)


def test_experiment_distributed_cluster_def_and_resources():
    spec = specification_for({
        "version": 1, "kind": "experiment",
        "environment": {
            "resources": {"gpu": {"requests": 1, "limits": 1}, "cpu": {"requests": 2, "limits": 4}},
            "pytorch": {"n_workers": 3, "default_worker": {"resources": {"gpu": {"limits": 1}}},
                        "worker": [{"index": 2, "resources": {"gpu": {"limits": 2}}}]}},
        "run": {"cmd": "python -m train"}})
    assert spec.cluster_def == ({"master": 1, "worker": 3}, True)
    assert spec.framework == "pytorch" and spec.is_distributed
    assert spec.get_worker_resources(0).gpus == 1 and spec.get_worker_resources(2).gpus == 2
    assert spec.total_gpus == 1 + 1 + 1 + 2


def test_tensorflow_ps_and_validation_errors():
    spec = specification_for({"version": 1, "kind": "experiment", "run": {"cmd": "x"},
                              "environment": {"tensorflow": {"n_workers": 2, "n_ps": 1}}})
    assert spec.cluster_def[0] == {"master": 1, "worker": 2, "ps": 1}
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 1, "kind": "experiment", "run": {"cmd": "x"},
                           "environment": {"pytorch": {"n_workers": 1, "n_ps": 1}}})
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 1, "kind": "experiment", "run": {"cmd": "x"},
                           "environment": {"pytorch": {"n_workers": 1}, "horovod": {"n_workers": 1}}})
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 2, "kind": "experiment", "run": {"cmd": "x"}})
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 1, "kind": "experiment", "run": {"cmd": "x"}, "bogus": 1})
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 1, "kind": "experiment", "hptuning": {"matrix": {}}, "run": {"cmd": "x"}})


def test_other_kinds():
    assert specification_for({"version": 1, "kind": "job", "run": {"cmd": "echo hi"}}).kind == "job"
    assert specification_for({"version": 1, "kind": "build", "build": {"image": "img"}}).build.image == "img"
    assert specification_for({"version": 1, "kind": "notebook"}).build.image
    assert specification_for({"version": 1, "kind": "tensorboard"}).kind == "tensorboard"
    p = specification_for({"version": 1, "kind": "pipeline", "concurrency": 2, "ops": [
        {"name": "a", "template": {"version": 1, "kind": "job", "run": {"cmd": "true"}}},
        {"name": "b", "upstream": ["a"], "trigger": "all_done", "max_retries": 2}]})
    assert [o["name"] for o in p.ops] == ["a", "b"] and p.ops[1]["upstream"] == ["a"]
    with pytest.raises(PolyaxonfileError):
        specification_for({"version": 1, "kind": "pipeline", "ops": [{"name": "a", "upstream": ["zz"]}]})


def test_patch_and_multi_file_merge(tmp_path):
    f1 = tmp_path / "a.yml"
    f1.write_text("version: 1\nkind: experiment\ndeclarations: {lr: 0.1}\nrun: {cmd: 'train --lr={{ lr }}'}\n")
    f2 = tmp_path / "b.yml"
    f2.write_text("declarations: {lr: 0.5}\n")
    e = ExperimentSpecification.read([str(f1), str(f2)])
    assert e.run.cmd == "train --lr=0.5"
    e2 = e.patch({"declarations": {"lr": 0.7}})
    assert e2.run.cmd == "train --lr=0.7"


def test_templating_types_and_expressions():
    ctx = {"lr": 0.1, "layers": [1, 2], "cfg": {"a": 3}, "name": "x"}
    assert render("{{ lr }}", ctx) == 0.1
    assert render("{{ lr * 10 }}", ctx) == 1.0
    assert render("n={{ layers[1] }} a={{ cfg.a }} {{ name | upper }}", ctx) == "n=2 a=3 X"
    assert render({"k": ["{{ cfg['a'] + 1 }}"]}, ctx) == {"k": [4]}
    assert render("{{ 'big' if lr > 0.05 else 'small' }}", ctx) == "big"
