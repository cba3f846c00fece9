import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
        return cache[name]
    return load


@pytest.fixture(params=["k28", "auto"])
def conv_path(request, monkeypatch):
    """The explicit CNN trunk's conv choice: "k28" forces K28 / K29 for every conv they take and the first fc layer's
    split GEMMs (K40G, r05) — the C3 update's path at any batch; "auto" keeps the size rules (MIOpen below
    fused_cnn._Trunk.igemm_min_rows output pixels, hipBLASLt for the fc layer below fc_split_min_rows)."""
    from xuanpolicy_amd import fused_cnn
    if request.param == "k28":
        monkeypatch.setattr(fused_cnn._Trunk, "igemm_min_rows", 0)
        monkeypatch.setattr(fused_cnn._Trunk, "fc_split_min_rows", 0)
    return request.param
