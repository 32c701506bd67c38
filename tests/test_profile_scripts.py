"""The rocprofv3 trace summarisers in scripts/ (the profiles/ evidence is made with them) on a small synthetic kernel
trace: step phases split at the loss kernel (torch NLL or the fused class cross entropy), all-stream idle gaps, and
the launch window around a kernel."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, loss="xent_fwd_kernel<true>"):
    # two steps bracketed by the SGD kernel; stream 0 = main, 7 = side (a weight-gradient kernel overlapping)
    rows, t = [], 0
    for _ in range(3):
        seq = [("gemm_nt_kernel<128>", 0, 100), ("bn_apply_kernel<true>", 0, 50), (loss, 0, 10),
               ("bn_bwd_dx_kernel<false>", 0, 60), ("wgrad_kernel<2,2>", 7, 200), ("sgd_flat_kernel", 0, 20)]
        for name, stream, dur in seq:
            start = t if stream == 0 else t - 50  # the side-stream kernel starts under the previous main kernel
            rows.append({"Kernel_Name": name, "Stream_Id": stream, "Start_Timestamp": start * 1000,
                         "End_Timestamp": (start + dur) * 1000, "Correlation_Id": len(rows)})
            if stream == 0:
                t += dur + 5  # 5 us gap between main-stream kernels
            else:
                t = max(t, start + dur + 30)  # a 30 us idle after the side kernel before the optimizer
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def _run(script, *args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script), *map(str, args)],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    return out.stdout


def test_step_phases_splits_at_the_class_cross_entropy(tmp_path):
    p = tmp_path / "t.csv"
    _trace(p)
    out = _run("step_phases.py", p, "--steps", 2, "--markdown")
    assert "steps averaged: 2" in out
    assert "| bwd | 7 | wgrad |" in out  # the v2 weight-gradient kernel is classed as wgrad


def test_step_phases_accepts_torch_nll(tmp_path):
    p = tmp_path / "t.csv"
    _trace(p, loss="nll_loss_forward_reduce")
    assert "steps averaged: 2" in _run("step_phases.py", p, "--steps", 2)


def test_gap_report_groups_idle_intervals(tmp_path):
    p = tmp_path / "t.csv"
    _trace(p)
    lines = [json.loads(x) for x in _run("gap_report.py", p, "--min-us", 20, "--skip-first", 0).splitlines()]
    head, groups = lines[0], lines[1:]
    assert head["idle_ms_over_threshold"] > 0 and 0 < head["idle_share"] < 1
    assert any(g["before"].startswith("wgrad_kernel") and g["after"].startswith("sgd_flat_kernel") for g in groups)


def test_trace_window_prints_the_neighbourhood(tmp_path):
    p = tmp_path / "t.csv"
    _trace(p)
    out = _run("trace_window.py", p, "--match", "xent_fwd", "--occurrence", -1, "--before", 2, "--after", 2)
    assert len(out.splitlines()) == 4 and "xent_fwd_kernel" in out
