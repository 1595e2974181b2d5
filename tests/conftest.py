import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ml-depth-pro-video_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libdp_mi355x.so")
    config.addinivalue_line("markers", "slow: full-size oracle forward on the CPU (tens of seconds)")


_METRICS = []


@pytest.fixture
def record(request):
    """record(name, value): keep a measured figure (parity error, margin) of this test; written
    as JSON to $DP_TEST_METRICS at the end of the session (DESIGN.md section 4 quotes them)."""
    def _rec(name, value):
        _METRICS.append({"test": request.node.nodeid, "name": name, "value": float(value)})
    return _rec


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("DP_TEST_METRICS")
    if path and _METRICS:
        import json
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_METRICS, f, indent=1)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def synth_sd():
    from depth_pro.weights import synthetic_state_dict

    return synthetic_state_dict(0)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
