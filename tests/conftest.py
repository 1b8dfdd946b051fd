import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "humanoid-walking-with-sac_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libsacmi.so)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN

# the world-1 RCCL tests exercise the data-parallel phase sequence itself (sacmi_step_dp
# takes the fused update at world 1 unless asked; the bench does not ask)
os.environ.setdefault("SACMI_DP_PHASES_AT_WORLD1", "1")
