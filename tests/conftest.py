import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "speech-enhancement-clskd_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


def check_summary(prefix, x, fx, rtol=1e-4, atol=1e-5, sample_atol=None):
    """Compare a full tensor x with the checksum+sample summary ``prefix`` in fixture fx."""
    x = np.asarray(x, np.float64)
    assert tuple(x.shape) == tuple(fx[prefix + "/shape"]), (prefix, x.shape, fx[prefix + "/shape"])
    flat = x.ravel()
    samp = flat[fx[prefix + "/idx"]]
    ref = fx[prefix + "/sample"].astype(np.float64)
    scale = max(np.abs(ref).max(), 1e-6)
    sa = sample_atol if sample_atol is not None else max(atol, rtol * scale)
    err = np.abs(samp - ref).max()
    assert err <= sa, f"{prefix}: max sample err {err:.3e} > {sa:.3e} (scale {scale:.3e})"
    n = flat.size
    for key, val in (("abssum", np.abs(flat).sum()), ("sqsum", (flat ** 2).sum())):
        r = float(fx[prefix + "/" + key])
        assert abs(val - r) <= rtol * abs(r) + atol * n, f"{prefix}/{key}: {val} vs {r}"


@pytest.fixture
def gold():
    return golden
