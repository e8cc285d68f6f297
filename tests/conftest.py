import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rp-style-transfer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The GPU torch runs of the oracle (the reference's algorithm on MIOpen / rocBLAS) measure the
# reference's fp32 noise on the platform it trains on, which the attention models' gradient
# bars include (helpers.check_grads_rms_vs_fp64). MIOpen's default find mode benchmarks
# candidate algorithms at the first call, so which one runs -- and the rounding it brings --
# changed from box to box (that floor read 0.7-1.8e-4 on SAModel's decoder.1.weight over six
# boxes). The immediate-mode heuristic (FAST) picks from the problem, the arch and the MIOpen
# version alone. Our kernels do not use MIOpen.
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and librpst.so")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
