"""plx_philox_sample (csrc/polytune_kernels.hip) vs its numpy twin: the same counter-based stream."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_sampler_matches_host_twin(cuda):
    from polyaxon_amd.polytune.sampler import PhiloxSampler, philox_random_suggestions
    from polyaxon_amd.spec.matrix import parse_matrix

    m = parse_matrix({"u": {"uniform": [2, 5]}, "lu": {"qloguniform": [-3, 0, 0.01]}, "n": {"normal": [1, 2]},
                      "ln": {"lognormal": [0, 0.5]}, "v": {"linspace": [0, 1, 11]},
                      "pv": {"pvalues": [["a", 0.1], ["b", 0.6], ["c", 0.3]]}})
    s = PhiloxSampler(m)
    for n, row0, seed in ((1, 0, 1), (1000, 0, 7), (4097, 123456, 2 ** 40 + 9)):
        dev = s.draw_device(n, seed, row0, cuda).cpu().numpy()
        host = s.draw_host(n, seed, row0)
        exact = [i for i, k in enumerate(s.keys) if k in ("u", "v", "pv")]
        np.testing.assert_array_equal(dev[:, exact], host[:, exact])          # integer / affine maps: bit exact
        np.testing.assert_allclose(dev, host, rtol=1e-12, atol=1e-12)         # libm log / cos / exp: ulps
    got = philox_random_suggestions(m, 64, seed=3, device="cuda")
    assert got == philox_random_suggestions(m, 64, seed=3, device=None) or \
        all(abs(a[k] - b[k]) < 1e-9 if isinstance(a[k], float) else a[k] == b[k]
            for a, b in zip(got, philox_random_suggestions(m, 64, seed=3, device=None)) for k in a)
