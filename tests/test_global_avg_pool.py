"""ops/pool.py global_avg_pool: the NHWC-native mean over H x W (forward column means of the NHWC view, backward one
broadcast write in channels_last) against x.mean((2, 3)) -- values, gradient, and the gradient's memory format."""
import pytest
import torch

from polyaxon_amd.ops.pool import global_avg_pool


@pytest.mark.parametrize("shape", [(4, 16, 7, 5), (2, 2048, 7, 7), (3, 8, 1, 9)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_avg_pool_matches_mean(shape, dtype):
    torch.manual_seed(0)
    x = torch.randn(shape).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    y = global_avg_pool(x)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    yr = xr.mean((2, 3))
    yr.backward(g.float())
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol, atol=tol)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
