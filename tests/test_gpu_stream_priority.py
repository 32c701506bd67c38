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


def test_fence_orders_a_consumer_after_queued_side_stream_work(cuda):
    """side_stream.fence: a consumer stream (FlatDDP's collective / optimizer stream) waits for the weight gradients
    already queued on the side stream, without the main stream waiting -- the bucket all-reduce fired by a parameter's
    post-accumulate hook must read the slot after the side stream wrote it."""
    from polyaxon_amd.ops import side_stream

    slot = torch.zeros(1 << 20, device=cuda)
    out = torch.empty_like(slot)
    side = side_stream.stream_for(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):  # what side_stream.run queues (outside a backward: no end-of-backward callback)
        torch.cuda._sleep(200_000_000)
        slot.fill_(3.0)
    side_stream._pending[cuda.index or 0] = True
    consumer = torch.cuda.Stream(device=cuda)
    side_stream.fence(consumer, cuda)
    with torch.cuda.stream(consumer):
        out.copy_(slot)
    done = torch.cuda.Event()
    done.record(consumer)
    assert not done.query()  # still behind the side stream's sleep
    main_free = torch.cuda.Event()
    main_free.record(torch.cuda.current_stream(cuda))
    main_free.synchronize()  # the main stream did not wait for the side stream
    torch.cuda.synchronize(cuda)
    assert torch.all(out == 3.0)
    side_stream.join(cuda)
