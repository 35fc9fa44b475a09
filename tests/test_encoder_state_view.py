"""The encoder's persistent state view (csrc/encode.cpp `refresh_state`,
DESIGN.md §5) patched node by node across ticks equals the view rebuilt from
scratch: node records, free values, their sorted values with multiplicity and
the distinct ones (the T-row thresholds come from these), and the pod-count
row.  Host only: tools/encode_stats.cpp in `check` mode runs 300 consecutive
fresh snapshots with pods added to and removed from random spot nodes."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "k8s-spot-rescheduler_amd")


@pytest.fixture(scope="module")
def encode_stats():
    subprocess.run(["make", "-C", PKG, "tools"], check=True, stdout=subprocess.DEVNULL)
    return os.path.join(PKG, "bin", "encode_stats")


@pytest.mark.parametrize("config", [2, 5])
@pytest.mark.parametrize("mode", ["check", "check-perm"])
def test_patched_state_view_equals_rebuilt(encode_stats, config, mode):
    """`check-perm`: pods on spot nodes also change requests, so the spot order
    moves between ticks; each moved node's records follow it to its new
    position and only the nodes whose own state changed are patched."""
    out = subprocess.run([encode_stats, str(config), "24", mode], check=True, capture_output=True, text=True,
                         timeout=300).stdout
    m = re.search(r"state views consistent: 300 ticks \(300 patched node by node, spot order moved (\d+)\)", out)
    assert m, out
    if mode == "check-perm":
        assert int(m.group(1)) >= 100, out
