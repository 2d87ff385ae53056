import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "monst3r-slam_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built library")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def parity_log():
    """Append measured parity statistics (one JSON object per call) to
    $M3S_PARITY_LOG (default gpurun_out/parity_stats.jsonl) so the numbers behind each
    tolerance survive `pytest -q`; copied into profiles/ per round."""
    import json
    import time
    path = os.environ.get("M3S_PARITY_LOG", os.path.join(ROOT, "gpurun_out",
                                                          "parity_stats.jsonl"))

    def log(test, **stats):
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "a") as f:
                f.write(json.dumps(dict(test=test, time=time.strftime("%Y-%m-%dT%H:%M:%S"),
                                        **stats), default=float) + "\n")
        except OSError:
            pass
    return log
