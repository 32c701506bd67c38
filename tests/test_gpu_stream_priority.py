"""HIP stream priorities (ops/side_stream.py ``priority_stream``: the weight-gradient side stream is a low-priority
stream, which gives it a hardware queue of its own)."""
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
