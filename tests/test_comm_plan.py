"""Gradient-bucket planning over xGMI (parallel/comm_plan.py) and its use by FlatDDP / the LM trainer."""
import json

import pytest
import torch

from polyaxon_amd.parallel import comm_plan as cp


def _rows(world, alpha_s, busbw_GBps, sizes_mb=(1, 8, 64, 256, 1024)):
    m = cp.FittedModel(world, alpha_s, busbw_GBps)
    out = []
    for mb in sizes_mb:
        b = mb * cp.MB
        t = cp.allreduce_seconds(b, world, m)
        out.append({"bytes": b, "algbw_GBps": b / t / 1e9, "busbw_GBps": b / t / 1e9 * 2 * (world - 1) / world})
    return out


def test_fit_recovers_latency_and_bandwidth():
    for world, alpha, bw in ((2, 8e-6, 110.0), (8, 5e-6, 780.0)):
        f = cp.fit_table(_rows(world, alpha, bw), world)
        assert f.alpha_s_ == pytest.approx(alpha, rel=1e-6)
        assert f.busbw == pytest.approx(bw, rel=1e-6)


def test_fit_rejects_tables_that_are_not_all_reduces():
    with pytest.raises(ValueError):
        cp.fit_table([{"bytes": 1 << 20, "algbw_GBps": 10.0}], 2)
    with pytest.raises(ValueError):  # time falls with size
        cp.fit_table([{"bytes": 1 << 20, "algbw_GBps": 1.0}, {"bytes": 1 << 30, "algbw_GBps": 1e9}], 2)


def test_plan_meets_the_efficiency_target_and_grows_with_the_links():
    big = 16e9  # Llama-3 8B bf16 gradients: never capped
    plans = {w: cp.plan(big, w) for w in (2, 4, 8)}
    for w, p in plans.items():
        assert p["reason"] == "efficiency target"
        assert p["efficiency"] == pytest.approx(0.9, abs=1e-3)
        t = cp.allreduce_seconds(p["bucket_bytes"], w)
        assert p["per_bucket_ms"] == pytest.approx(t * 1e3, rel=1e-2)
    # more ranks -> more xGMI links per ring step -> bigger buckets for the same efficiency
    assert plans[2]["bucket_bytes"] < plans[4]["bucket_bytes"] < plans[8]["bucket_bytes"]
    assert plans[8]["busbw_GBps"] == pytest.approx(7 * 153.0 * 0.75, rel=1e-3)


def test_plan_caps_small_models_for_overlap_and_floors_tiny_ones():
    p = cp.plan(100e6, 8)  # ResNet-50 fp32 gradients: the efficiency bucket would be one bucket
    assert p["reason"].startswith("capped") and p["buckets"] >= 4
    assert p["bucket_bytes"] == int(100e6 / 4)
    q = cp.plan(1e6, 8)
    assert q["bucket_bytes"] == 4 * cp.MB and q["reason"].startswith("floor")  # min_mb floor
    w1 = cp.plan(1e9, 1)
    assert w1["source"] == "world-1"


def test_measured_table_overrides_the_link_model(tmp_path, monkeypatch):
    path = tmp_path / "busbw.jsonl"
    path.write_text("\n".join(json.dumps({"world": w, "all_reduce": _rows(w, 20e-6, 200.0)}) for w in (2, 8)))
    monkeypatch.setenv("PLX_COMM_TABLE", str(path))
    p = cp.plan(16e9, 8)
    assert p["source"] == "table"
    assert p["alpha_us"] == pytest.approx(20.0, rel=1e-3) and p["busbw_GBps"] == pytest.approx(200.0, rel=1e-3)
    assert p["bucket_bytes"] == pytest.approx(9 * 20e-6 * 8 * 200e9, rel=1e-6)
    assert cp.plan(16e9, 4)["source"] == "link-model"  # no row for world 4


def test_cli_prints_one_plan_per_world(capsys):
    assert cp.main(["--params", "8.03e9", "--world", "2", "8"]) == 0
    lines = [json.loads(x) for x in capsys.readouterr().out.strip().splitlines()]
    assert [x["world"] for x in lines] == [2, 8] and all(x["bucket_MB"] > 0 for x in lines)


def test_flat_ddp_auto_buckets():
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP

    model = torch.nn.Sequential(torch.nn.Linear(256, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10))
    flat = FlatParams(model, torch.device("cpu"))
    ddp = FlatDDP(flat)  # default "auto"
    assert ddp.plan is not None and ddp.plan["world"] == 1
    assert sum(hi - lo for lo, hi, _ in ddp.buckets) >= flat.numel - 16
    fixed = FlatDDP(flat, bucket_mb=0.01)
    assert fixed.plan is None and len(fixed.buckets) > len(ddp.buckets)
