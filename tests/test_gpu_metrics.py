"""MetricStream on a GPU: preallocated pinned ring + low-priority side stream, no training-stream sync, FIFO,
nothing dropped when the ring wraps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Sink:
    def __init__(self):
        self.rows = []

    def log_metrics(self, xid, rows):
        self.rows.extend(rows)


def test_metric_stream_ring_wraps_without_loss(cuda):
    from polyaxon_amd.client.tracking import MetricStream

    sink = _Sink()
    ms = MetricStream(sink, 1, flush_every_s=0.01, ring_floats=16)
    ring = None
    for i in range(500):
        loss = torch.full((), float(i), device=cuda)
        acc = torch.full((1,), float(-i), device=cuda)
        ms.put({"loss": loss, "acc": acc, "lr": 0.1}, step=i)
        if ring is None:
            ring = ms._ring
    ms.close()
    assert ms._ring is ring and ring.is_pinned() and ring.numel() == 16  # allocated once, never grown
    assert [r[1] for r in sink.rows] == list(range(500))
    assert all(r[0]["loss"] == float(r[1]) and r[0]["acc"] == -float(r[1]) and r[0]["lr"] == 0.1 for r in sink.rows)
    lo = torch.cuda.Stream.priority_range()[0]
    assert ms._side.priority == lo
