"""Golden parse tests against the reference's own Polyaxonfiles: every ``*_content`` spec of
polyaxon/factories/fixtures.py:11-461 and every complete example in docs/templates/polyaxonfile_specification.

The fixtures are read from the reference tree with ``ast`` (string literals only -- nothing of the reference is
imported or executed); the tests skip when the reference tree is not mounted."""
import ast
import os
import re

import pytest

from polyaxon_amd.spec import specification_for
from polyaxon_amd.spec.specification import GroupSpecification, Kinds

REF = "/root/reference"
FIXTURES = os.path.join(REF, "polyaxon", "factories", "fixtures.py")

pytestmark = pytest.mark.skipif(not os.path.exists(FIXTURES), reason="reference tree not mounted")


def _fixture_strings():
    tree = ast.parse(open(FIXTURES).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and isinstance(node.value, ast.Constant) and isinstance(node.value.value, str):
            for t in node.targets:
                if isinstance(t, ast.Name) and "_content" in t.id:
                    out[t.id] = node.value.value
    return out


def test_every_reference_fixture_parses():
    specs = _fixture_strings()
    assert len(specs) >= 13
    kinds = {}
    for name, content in specs.items():
        spec = specification_for(content)
        kinds[name] = spec.kind
    assert kinds["experiment_group_spec_content"] == Kinds.GROUP
    assert kinds["build_spec_content"] == Kinds.BUILD
    assert kinds["notebook_spec_content"] == Kinds.NOTEBOOK and kinds["tensorboard_spec_content"] == Kinds.TENSORBOARD
    assert kinds["job_spec_content"] == Kinds.JOB


def test_fixture_semantics():
    s = _fixture_strings()
    g = specification_for(s["experiment_group_spec_content"])
    assert isinstance(g, GroupSpecification) and g.search_algorithm == "grid_search" and g.tags == ["fixtures"]
    assert g.matrix_space == 5  # logspace 0.01:0.1:5

    hb = specification_for(s["experiment_group_spec_content_hyperband"]).hptuning.hyperband
    assert hb is not None and hb.max_iter > 0 and hb.eta > 1 and hb.resource.name and hb.metric.name

    es = specification_for(s["experiment_group_spec_content_early_stopping"]).hptuning.early_stopping
    assert es and all(r.metric and r.optimization in ("maximize", "minimize") for r in es)

    bo = specification_for(s["experiment_group_spec_content_bo"]).hptuning.bo
    assert bo is not None and bo.n_iterations > 0 and bo.utility_function.acquisition_function in ("ucb", "ei", "poi")

    res = specification_for(s["exec_experiment_resources_content"])
    cluster, distributed = res.cluster_def
    assert distributed and sum(cluster.values()) > 1
    assert res.total_resources is not None

    refs = specification_for(s["exec_experiment_outputs_refs_content"])
    assert refs.environment.outputs.get("jobs") or refs.environment.outputs.get("experiments")

    job = specification_for(s["job_spec_resources_content"])
    assert job.resources is not None
    build = specification_for(s["build_spec_content"])
    assert build.build.image


def _doc_yaml_blocks():
    import glob
    import textwrap

    for fn in sorted(glob.glob(os.path.join(REF, "docs", "templates", "**", "*.md"), recursive=True)):
        txt = open(fn).read()
        for block in re.findall(r"```yaml\n(.*?)```", txt, flags=re.S):
            block = textwrap.dedent(block)
            if re.search(r"^version:", block, flags=re.M) and re.search(r"^kind:", block, flags=re.M):
                yield fn, block


def test_complete_doc_examples_parse():
    blocks = list(_doc_yaml_blocks())
    if not blocks:
        pytest.skip("no complete examples in the docs")
    assert len(blocks) >= 10
    for fn, block in blocks:
        spec = specification_for(block)
        assert spec.kind in Kinds.VALUES, fn
