"""HIP stream priorities for the training step (ops/side_stream.py ``priority_stream``, executor
``PLX_MAIN_PRIORITY``): the step on a high-priority stream is the same computation as on the caller's stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_priority_streams_run_work(cuda):
    from polyaxon_amd.ops import side_stream

    x = torch.arange(1 << 20, device=cuda, dtype=torch.float32)
    for prio in (-1, 0, 1):
        s = side_stream.priority_stream(cuda.index or 0, prio)
        s.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(s):
            y = x * 2 + 1
        torch.cuda.current_stream(cuda).wait_stream(s)
        torch.testing.assert_close(y, x * 2 + 1)


def test_executor_high_priority_main_stream_matches_default(cuda, monkeypatch):
    from polyaxon_amd.models.resnet import resnet50
    from polyaxon_amd.ops.synth import SyntheticImages
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    out = {}
    for prio in ("", "-1"):
        monkeypatch.setenv("PLX_MAIN_PRIORITY", prio)
        torch.manual_seed(0)
        data = SyntheticImages(4, 64, cuda, classes=1000, active_classes=100, grid=7, signal=0.5, seed=5)
        ex = ResidentTrialExecutor(resnet50(), data, cuda, use_graph=False)
        ex.reset(seed=1)
        ex.set_hparams(lr=0.05, momentum=0.9, weight_decay=1e-4)
        ex.run(2)
        ex.run(2)  # a second call re-forks from the caller's stream
        torch.cuda.synchronize()
        out[prio] = (ex.losses(), ex.flat.params.detach().float().clone())
        assert (ex._main_stream is not None) == bool(prio)
        del ex
    torch.testing.assert_close(out["-1"][0], out[""][0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out["-1"][1], out[""][1], rtol=1e-4, atol=1e-5)
