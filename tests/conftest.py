"""pytest configuration: the `gpu` marker, import paths, shared helpers.

`-m "not gpu"` (run in the build container, no GPU): oracle vs golden vectors,
host logic, C-ABI load/export checks, gloo multi-process plumbing.
`-m gpu` (run on an MI355X): HIP path vs the oracle through the C ABI.
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device); run with -m gpu")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def coracle():
    import nf4_oracle as O

    return O.COracle()


@pytest.fixture(scope="session")
def gpu():
    import torch

    # No skip: a -m gpu run without a device must fail, not pass vacuously.
    assert torch.cuda.is_available(), "gpu-marked test needs a ROCm device"
    return torch.device("cuda", 0)
