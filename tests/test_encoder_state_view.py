"""The encoder's persistent state view (csrc/encode.cpp `refresh_state`,
DESIGN.md §5) patched node by node across ticks equals the view rebuilt from
scratch: node records, free values, their sorted values with multiplicity and
the distinct ones (the T-row thresholds come from these), and the pod-count
row.  Host only: tools/encode_stats.cpp in `check` mode runs 300 consecutive
fresh snapshots with pods added to and removed from random spot nodes."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "k8s-spot-rescheduler_amd")


@pytest.fixture(scope="module")
def encode_stats():
    subprocess.run(["make", "-C", PKG, "tools"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(PKG, "bin", "encode_stats")


@pytest.mark.parametrize("config", [2, 5])
def test_patched_state_view_equals_rebuilt(encode_stats, config):
    out = subprocess.run([encode_stats, str(config), "24", "check"], check=True, capture_output=True, text=True,
                         timeout=300).stdout
    assert "state views consistent: 300 ticks (300 patched node by node)" in out, out
