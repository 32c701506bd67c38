"""Trial runtime plumbing: RCCL watchdog env for multi-rank trials, GPU -> local CPU (NUMA) binding from the KFD
topology, the rocprofv3 trial wrapper, and ``environment.profile`` in the Polyaxonfile."""
import pytest

from polyaxon_amd.polyflow.devices import device_cpus, parse_cpulist
from polyaxon_amd.polyflow.env import trial_env
from polyaxon_amd.polyflow.scheduler import profile_argv


def _env(cluster, devices):
    return trial_env(base_env={}, experiment={"id": 1, "uuid": "u"}, project="p", user="u", group=None,
                     role="master", index=0, framework="pytorch", cluster=cluster, devices=devices,
                     outputs_path="/o", logs_path="/l", declarations={}, data_paths={}, refs_outputs={},
                     log_level=None, store_path=None, api_host=None, ephemeral_token=None, master_port=1234,
                     local_rank=0)


def test_rccl_watchdog_only_for_multi_rank():
    one = _env({"master": ["127.0.0.1:1234"]}, [0])
    assert "TORCH_NCCL_ASYNC_ERROR_HANDLING" not in one
    two = _env({"master": ["127.0.0.1:1234"], "worker": ["127.0.0.1:1235"]}, [0])
    assert two["TORCH_NCCL_ASYNC_ERROR_HANDLING"] == "1" and float(two["PLX_COLLECTIVE_TIMEOUT_S"]) > 0


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


def test_device_cpus_from_fake_sysfs(tmp_path):
    nodes = tmp_path / "class" / "kfd" / "kfd" / "topology" / "nodes"
    for i, (simd, minor) in enumerate([(0, 0), (1216, 128), (1216, 136)]):
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor}\n")
    for minor, cpus in ((128, "0-3,96-99"), (136, "48-51")):
        p = tmp_path / "class" / "drm" / f"renderD{minor}" / "device"
        p.mkdir(parents=True)
        (p / "local_cpulist").write_text(cpus + "\n")
    assert device_cpus(0, sysfs=str(tmp_path)) == [0, 1, 2, 3, 96, 97, 98, 99]
    assert device_cpus(1, sysfs=str(tmp_path)) == [48, 49, 50, 51]
    assert device_cpus(2, sysfs=str(tmp_path)) is None
    assert device_cpus(0, sysfs=str(tmp_path / "missing")) is None


def test_profile_argv():
    argv = profile_argv("python -m polyaxon_amd.trainers lm --lr 0.1", "/out/rocprof/master.0")
    assert argv[0].endswith("rocprofv3") and "--kernel-trace" in argv and "--stats" in argv
    i = argv.index("--")
    assert argv[i + 1:] == ["python", "-m", "polyaxon_amd.trainers", "lm", "--lr", "0.1"]
    assert argv[argv.index("-d") + 1] == "/out/rocprof/master.0"
    # the profiler must launch the program itself: shell constructs are not wrapped
    for cmd in ("pip install x && python t.py", "python t.py > log", "A=1 python t.py", "echo $(date)"):
        assert profile_argv(cmd, "/o") is None


def test_environment_profile_flag():
    from polyaxon_amd.spec.environment import EnvironmentSpec

    env = EnvironmentSpec.from_dict({"profile": True, "resources": {"gpu": {"limits": 1}}})
    assert env.profile is True and env.to_dict()["profile"] is True
    assert EnvironmentSpec.from_dict({}).profile is False
    with pytest.raises(Exception):
        EnvironmentSpec.from_dict({"profile": "sometimes"})
