import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # pytest-xdist: every worker's torch defaults to one intra-op thread per core, so N workers oversubscribe the
    # CPUs N-fold and the spinning OpenMP pools slowed the resident-worker tests ~40x (past their 300 s stall
    # timeout).  Give each worker its share; subprocesses (torchrun tests) inherit it through the environment.
    n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "0") or 0)
    if n > 1:
        share = str(max(1, (os.cpu_count() or 1) // n))
        os.environ.setdefault("OMP_NUM_THREADS", share)
        import torch

        torch.set_num_threads(int(os.environ["OMP_NUM_THREADS"]))


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
