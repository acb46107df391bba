import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "marl-sat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def c_precision():
    """Setter for the library's weight-gradient path (msat_set_precision: 'fp16x2' | 'bf16x3' | 'fp32');
    restores the process's validated MARLSAT_PRECISION after the test."""
    from marlsat import _lib
    from marlsat.learners import gnn

    def set_(name):
        _lib.check(_lib.lib.msat_set_precision(gnn.PRECISION_CODES[name]), "msat_set_precision")

    yield set_
    set_(gnn.PRECISION)
