import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "k8s-spot-rescheduler_amd")
for p in (PKG, os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X (HIP device); parity tests of the HIP path")
    # Build the in-tree libraries once if they are missing (cross-compiles without a GPU).
    need = [os.path.join(PKG, "lib", "libsrplanner.so"), os.path.join(PKG, "lib", "libsrsynth.so"),
            os.path.join(REPO, "oracle", "build", "libsroracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True)
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True)


@pytest.fixture(scope="session")
def checker():
    from spotplanner.planner import PredicateChecker
    c = PredicateChecker(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def podorder_checker():
    """A planner with SR_K2_MODE=1: K2's pod-order path for every candidate
    (the A/B arm of the node-order window kernel)."""
    from spotplanner.planner import PredicateChecker
    os.environ["SR_K2_MODE"] = "1"
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_K2_MODE"]
    yield c
    c.close()
