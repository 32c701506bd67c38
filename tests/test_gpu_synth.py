"""Device-generated synthetic learnable batches (csrc/train_kernels.hip ``plx_synth_images``) against the
fp32 PyTorch definition of the same distribution: x = signal * upsample(proto[y]) + N(0, 1)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_synth_images_distribution(cuda):
    from polyaxon_amd.ops.synth import SyntheticImages

    d = SyntheticImages(64, 56, cuda, classes=1000, active_classes=100, grid=7, signal=0.5, seed=3)
    d.next()
    torch.cuda.synchronize()
    assert int(d.counter.item()) == 1
    y = d.y.cpu()
    assert y.min() >= 0 and y.max() < 100
    assert len(set(y.tolist())) > 20  # labels are spread over the active classes
    x = d.x.float().cpu()
    assert d.x.is_contiguous(memory_format=torch.channels_last)
    noise = x - d.expected_mean(y).cpu()  # fp32 reference of the noise-free image
    assert abs(float(noise.mean())) < 0.02
    assert abs(float(noise.std()) - 1.0) < 0.02
    # the noise is independent of the pattern and across channels / pixels
    c = torch.corrcoef(torch.stack([noise[:, 0].flatten(), noise[:, 1].flatten()]))[0, 1]
    assert abs(float(c)) < 0.02


def test_synth_images_fresh_and_deterministic(cuda):
    from polyaxon_amd.ops.synth import SyntheticImages

    a = SyntheticImages(8, 32, cuda, classes=10, active_classes=10, grid=4, signal=1.0, seed=9)
    b = SyntheticImages(8, 32, cuda, classes=10, active_classes=10, grid=4, signal=1.0, seed=9)
    a.next()
    x1, y1 = a.x.clone(), a.y.clone()
    a.next()
    assert not torch.equal(x1, a.x)  # a new batch every step
    b.next()
    assert torch.equal(x1, b.x) and torch.equal(y1, b.y)  # same seed + position -> same batch


def test_executor_learns_fresh_synthetic_task(cuda):
    """A small ResNet trained on the fresh-batch stream must beat chance clearly (labels are learnable)."""
    from polyaxon_amd.models.resnet import resnet18ish
    from polyaxon_amd.ops.synth import SyntheticImages
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    data = SyntheticImages(64, 32, cuda, classes=10, active_classes=10, grid=4, signal=1.0, seed=1)
    ex = ResidentTrialExecutor(resnet18ish(), data, cuda, use_graph=False)
    ex.reset(seed=0)
    ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4)
    ex.run(60)
    torch.cuda.synchronize()
    losses = ex.losses()
    assert float(losses[:5].mean()) > 1.8
    assert float(losses[-10:].mean()) < 1.0, losses[-10:]


def test_executor_batch_prefetch_matches_inline(cuda):
    """Side-stream prefetch of the next batch (executor._prefetch, eager path): the same batch stream, the same
    training trajectory and the same per-step losses as generating each batch inline on the main stream."""
    from polyaxon_amd.models.resnet import resnet50
    from polyaxon_amd.ops.synth import SyntheticImages
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    out = {}
    for mode in ("inline", "end"):  # generated inline / prefetched after the backward
        torch.manual_seed(0)
        data = SyntheticImages(4, 64, cuda, classes=1000, active_classes=100, grid=7, signal=0.5, seed=5)
        ex = ResidentTrialExecutor(resnet50(), data, cuda, use_graph=False)
        ex._prefetch = mode != "inline"
        ex.reset(seed=1)
        ex.set_hparams(lr=0.05, momentum=0.9, weight_decay=1e-4)
        ex.run(4)
        torch.cuda.synchronize()
        out[mode] = (ex.losses(), ex.flat.params.detach().float().clone(), int(data.counter.item()))
        if mode != "inline":
            assert ex._ready is not None and ex._bufs is not None  # the prefetch path really ran
        del ex
    for mode in ("end",):
        assert out[mode][2] == out["inline"][2] + 1  # one batch generated ahead
        torch.testing.assert_close(out[mode][0], out["inline"][0], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(out[mode][1], out["inline"][1], rtol=1e-4, atol=1e-5)


def test_synth_images_odd_sizes_match_the_pattern(cuda):
    """Image sides that the pattern grid does not divide, chunks that cross pixel rows (H*W*3 % 8 == 0 only):
    the incremental (h, w) walk and the LDS cell table give the same noise-free image as the fp32 reference."""
    from polyaxon_amd.ops.synth import SyntheticImages

    for image, grid in ((40, 7), (24, 5), (56, 3)):
        d = SyntheticImages(32, image, cuda, classes=10, active_classes=10, grid=grid, signal=4.0, seed=11)
        d.next()
        torch.cuda.synchronize()
        noise = d.x.float().cpu() - d.expected_mean(d.y.cpu()).cpu()
        # a wrong cell would leave pattern residue of variance ~ signal^2 in the noise
        assert abs(float(noise.std()) - 1.0) < 0.03, (image, grid, float(noise.std()))
        assert abs(float(noise.mean())) < 0.03
