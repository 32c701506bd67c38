"""Synthetic, learnable ImageNet-shape data generated on the device, a fresh batch every training step.

BASELINE.json config 3 runs on "synthetic ImageNet-shape data".  A fixed random batch (what round 1 used) is
memorised within a few steps, so wall-clock-to-target said nothing.  Here the task is fixed but the samples are
not: every class owns a coarse ``G x G x 3`` pattern (``proto``, drawn once from the task seed) and each step's
images are ``signal * upsample(proto[y]) + N(0, 1)`` with fresh labels and fresh noise.  Reaching a low loss
needs real learning (the network must find the class pattern under unit noise), and a trial never sees the same
batch twice.

On the GPU the batch is produced in place by ``plx_synth_images`` (csrc/train_kernels.hip: Philox4x32-10 noise,
16-B bf16 stores, one launch + a counter bump, graph-capturable).  The CPU path draws the same distribution with
torch's generator (not bit-identical) for the unit tests.
"""
from __future__ import annotations

import math

import torch

from polyaxon_amd.ops import _native


class SyntheticImages:
    def __init__(self, batch: int, image: int, device, classes: int = 1000, active_classes: int = 100,
                 grid: int = 7, signal: float = 0.5, seed: int = 0, channels_last: bool = True,
                 dtype: torch.dtype = torch.bfloat16):
        self.device = torch.device(device)
        self.is_cuda = self.device.type == "cuda"
        self.batch, self.image, self.classes = batch, image, classes
        self.active = min(active_classes, classes)
        self.grid, self.signal, self.seed = grid, float(signal), int(seed)
        if self.is_cuda and (image * image * 3) % 8:
            raise ValueError("the device generator needs image*image*3 to be a multiple of 8")
        g = torch.Generator().manual_seed(self.seed ^ 0x7a5c)
        # [active, G, G, 3] fp32, channel innermost (matches the NHWC image layout)
        self.proto = torch.randn(self.active, grid, grid, 3, generator=g).to(self.device)
        dt = dtype if self.is_cuda else torch.float32
        x = torch.empty(batch, 3, image, image, dtype=dt, device=self.device)
        self.x = x.contiguous(memory_format=torch.channels_last) if channels_last else x
        self.y = torch.zeros(batch, dtype=torch.int64, device=self.device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._cpu_gen = torch.Generator().manual_seed(self.seed)

    def next(self) -> None:
        """Refill ``x``/``y`` in place with the next batch of the stream."""
        if self.is_cuda:
            self.next_into(self.x, self.y, torch.cuda.current_stream(self.device))
            return
        y = torch.randint(0, self.active, (self.batch,), generator=self._cpu_gen)
        mean = self.expected_mean(y)
        noise = torch.randn(mean.shape, generator=self._cpu_gen)
        self.x.copy_(mean + noise)
        self.y.copy_(y)
        self.counter += 1

    def next_into(self, x: torch.Tensor, y: torch.Tensor, stream: "torch.cuda.Stream") -> None:
        """Device path: write the next batch of the stream into ``x``/``y`` (shaped as ``self.x``/``self.y``) on
        ``stream``.  The batch counter advances on that stream, so every launch of one stream of batches must be
        ordered after the previous one (the executor's prefetch keeps them all on one side stream after the first)."""
        if not self.is_cuda:
            raise RuntimeError("next_into is the device generator's path")
        if not x.is_contiguous(memory_format=torch.channels_last):
            raise ValueError("device generator writes NHWC (channels_last) images")
        if x.shape != self.x.shape or x.dtype != self.x.dtype or y.shape != self.y.shape or y.dtype != self.y.dtype:
            raise ValueError("batch buffers must match the generator's x / y")
        rc = _native.lib("plx_train").plx_synth_images(
            x.data_ptr(), y.data_ptr(), self.batch, self.image, self.image, self.proto.data_ptr(),
            self.active, self.grid, self.signal, self.seed & 0xFFFFFFFFFFFFFFFF, self.counter.data_ptr(),
            stream.cuda_stream)
        _native.check(rc, "plx_synth_images")

    def expected_mean(self, y: torch.Tensor) -> torch.Tensor:
        """``signal * upsample(proto[y])`` as an NCHW fp32 tensor (the noise-free image of each label)."""
        p = self.proto.to(y.device)[y].permute(0, 3, 1, 2).float()  # [B, 3, G, G]
        idx = (torch.arange(self.image, device=p.device) * self.grid) // self.image
        up = p[:, :, idx][:, :, :, idx]
        return self.signal * up

    @property
    def chance_loss(self) -> float:
        return math.log(self.classes)


class SyntheticTokens:
    """Synthetic, learnable token batches for the language-model trial programs, a fresh batch every step.

    Each sequence is a random ``period``-token phrase repeated to ``seq`` tokens: the first period is noise (loss
    ln V per token) and every later token is predictable by copying from ``period`` positions back, so the loss
    floor is about ``period / seq * ln V`` and reaching it needs the model to learn induction -- hyper-parameter
    sensitive (learning rate, warm-up, weight decay), unlike uniform random tokens whose loss never leaves ln V.
    The phrases come from a counter-based integer hash of (seed, step counter, position) computed with plain tensor
    ops on the device: graph-capturable (the counter is device data, bumped in place), identical on CPU and GPU.
    ``y`` is ``x`` (next-token targets are the shifted tokens, ``models.transformer.lm_loss``)."""

    M32 = 0xFFFFFFFF

    def __init__(self, batch: int, seq: int, vocab: int, device, period: int = 64, seed: int = 0,
                 active_vocab: int = 0):
        """``active_vocab`` (0 = all): the phrases draw from the first ``active_vocab`` token ids only, so a model
        also has a unigram distribution to learn (ln V -> ln active_vocab within tens of steps at a good learning
        rate) before the copying: a budget of ~100 steps separates learning rates by nats, not hundredths."""
        if seq % period:
            raise ValueError("seq must be a multiple of period")
        self.device = torch.device(device)
        self.batch, self.seq, self.vocab, self.period, self.seed = batch, seq, vocab, period, int(seed)
        self.active_vocab = int(active_vocab) if 0 < int(active_vocab) < vocab else vocab
        self.x = torch.zeros(batch, seq, dtype=torch.int64, device=self.device)
        self.y = self.x
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._idx = torch.arange(batch * period, dtype=torch.int64, device=self.device)
        self._h = torch.empty_like(self._idx)
        self._t = torch.empty_like(self._idx)

    def next(self) -> None:
        """Refill ``x`` in place with the next batch of the stream (and advance the device counter)."""
        m, h, t = self.M32, self._h, self._t
        torch.mul(self._idx, 0x9E3779B1, out=h)
        h.add_(self.counter * 0x85EBCA77 + (self.seed * 0xC2B2AE3D) % (1 << 32))
        h.bitwise_and_(m)
        for mult in (0x7FEB352D, 0x846CA68B):  # lowbias32 finaliser
            torch.bitwise_right_shift(h, 16, out=t)
            h.bitwise_xor_(t)
            h.mul_(mult).bitwise_and_(m)
        torch.bitwise_right_shift(h, 15, out=t)
        h.bitwise_xor_(t)
        h.remainder_(self.active_vocab)
        self.x.view(self.batch, self.seq // self.period, self.period).copy_(
            h.view(self.batch, 1, self.period).expand(self.batch, self.seq // self.period, self.period))
        self.counter.add_(1)

    @property
    def floor_loss(self) -> float:
        """Expected loss of a perfect copier: only the first period (minus its first token) is unpredictable."""
        return (self.period - 1) / (self.seq - 1) * math.log(self.active_vocab)

    @property
    def unigram_loss(self) -> float:
        """Loss of a model that learned which tokens occur but does not copy."""
        return math.log(self.active_vocab)

    @property
    def chance_loss(self) -> float:
        return math.log(self.vocab)


class SyntheticChain:
    """A deterministic token chain for the language-model trial programs (config 4's objective): each sequence starts
    at a random token x0 of [0, p) (p prime) and continues x_{t+1} = (a x_t + b) mod p, so every target is a fixed
    function of the previous token -- a p-entry transition table the model has to memorise.  Each transition occurs
    ~batch * seq / p times per step, so within ~100 steps the loss falls from ln V by several nats at a good
    learning rate and stays near ln p at a poor one (the copy task's induction is not learned within a trial budget:
    profiles/r5_config4_search.md).  The chain has a closed form, x_t = (A_t x0 + B_t) mod p with A_t = a^t and
    B_t = b (a^t - 1) / (a - 1) tabulated on the host, so a batch is four tensor ops on the device: graph-capturable
    (the start tokens come from the same counter hash as SyntheticTokens), identical on CPU and GPU."""

    M32 = 0xFFFFFFFF

    def __init__(self, batch: int, seq: int, vocab: int, device, p: int = 4093, a: int = 1103, b: int = 12345,
                 seed: int = 0):
        if not (2 < p <= vocab) or any(p % d == 0 for d in range(2, int(p ** 0.5) + 1)):
            raise ValueError("p must be a prime <= vocab")
        self.device = torch.device(device)
        self.batch, self.seq, self.vocab, self.p, self.seed = batch, seq, vocab, p, int(seed)
        self.active_vocab = p
        A, B = [1], [0]
        for _ in range(seq - 1):  # x_{t+1} = a x_t + b: A_{t+1} = a A_t, B_{t+1} = a B_t + b
            A.append(A[-1] * a % p)
            B.append((B[-1] * a + b) % p)
        self._A = torch.tensor(A, dtype=torch.int64, device=self.device).view(1, seq)
        self._B = torch.tensor(B, dtype=torch.int64, device=self.device).view(1, seq)
        self.x = torch.zeros(batch, seq, dtype=torch.int64, device=self.device)
        self.y = self.x
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._idx = torch.arange(batch, dtype=torch.int64, device=self.device).view(batch, 1)
        self._h = torch.empty_like(self._idx)
        self._t = torch.empty_like(self._idx)

    def next(self) -> None:
        """Refill ``x`` in place with the next batch of the stream (and advance the device counter)."""
        m, h, t = self.M32, self._h, self._t
        torch.mul(self._idx, 0x9E3779B1, out=h)
        h.add_(self.counter * 0x85EBCA77 + (self.seed * 0xC2B2AE3D) % (1 << 32))
        h.bitwise_and_(m)
        for mult in (0x7FEB352D, 0x846CA68B):  # lowbias32 finaliser
            torch.bitwise_right_shift(h, 16, out=t)
            h.bitwise_xor_(t)
            h.mul_(mult).bitwise_and_(m)
        torch.bitwise_right_shift(h, 15, out=t)
        h.bitwise_xor_(t)
        h.remainder_(self.p)
        torch.mul(self._A, h, out=self.x)
        self.x.add_(self._B).remainder_(self.p)
        self.counter.add_(1)

    @property
    def floor_loss(self) -> float:
        """A model that knows the table predicts every target but none for the first token (it has none)."""
        return 0.0

    @property
    def unigram_loss(self) -> float:
        """Loss of a model that learned which tokens occur but not the transitions."""
        return math.log(self.p)

    @property
    def chance_loss(self) -> float:
        return math.log(self.vocab)
