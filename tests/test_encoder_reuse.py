"""Candidate-side reuse of the persistent encoder (host only, no GPU).

A housekeeping tick whose candidate input (lists, global indices, stamped
pods) equals the previous tick's keeps the previous encoding and brings only
its capacity-dependent parts up to date: pod-count / composite atom rows, the
T-row thresholds and the records of the pods asking within a moved threshold
interval (host.hpp CandReuse).  tools/encode_stats' `reuse`
mode drives tick after tick of fresh snapshots with pods added on random spot
nodes (bursts included, and the extra pods leaving again) and compares every
reused workload with one encoded from scratch on the same snapshot: atoms,
class programs and request words equal, per pod the same dead flag, class and
threshold per dimension.  Reference: nodes/nodes.go:63-145 (the tick's model,
rebuilt by run() every tick, rescheduler.go:195,215)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "k8s-spot-rescheduler_amd")
TOOL = os.path.join(PKG, "bin", "encode_stats")


@pytest.fixture(scope="module")
def tool():
    subprocess.run(["make", "-C", PKG, "-j8", "tools"], check=True, stdout=subprocess.DEVNULL)
    return TOOL


def run_check(tool, config, ticks, burst=24, env=None, mode="reuse"):
    e = dict(os.environ)
    e.update(env or {})
    out = subprocess.run([tool, str(config), "100000", mode, str(ticks), str(burst)], env=e, check=True,
                         capture_output=True, text=True, timeout=600).stdout
    m = re.search(r"reuse check: (\d+) ticks \((\d+) reused, (\d+) full\), (\d+) pod patches.*mismatches (\d+)", out)
    assert m, out
    ticks_, reused, full, patches, bad = map(int, m.groups())
    one = re.search(r"one-node-changed encode .*reused (\d), pod patches (\d+)", out)
    moved = re.search(r"spot order moved (\d+)", out)
    return dict(ticks=ticks_, reused=reused, full=full, patches=patches, bad=bad,
                one_node_reused=int(one.group(1)), moved=int(moved.group(1)), out=out)


@pytest.mark.parametrize("config", [1, 2, 3])
def test_reuse_matches_fresh_encode(tool, config):
    """Every tick after the index is built reuses the candidate side, and the
    reused workload plans like a fresh encode (zero mismatches)."""
    r = run_check(tool, config, 120 if config < 3 else 60)
    assert r["bad"] == 0, r["out"]
    assert r["reused"] == r["ticks"] and r["full"] == 0, r["out"]
    assert r["one_node_reused"] == 1
    assert r["patches"] > 0, r["out"]  # thresholds moved under some pods and their records were re-pointed


def test_spare_rows_exhausted_falls_back_to_full_encode(tool):
    """No spare T row (SR_T_SPARE=0): a threshold that needs a new row ends
    the reuse, the tick is encoded in full and the next one reuses again."""
    r = run_check(tool, 2, 80, burst=60, env={"SR_T_SPARE": "0"})
    assert r["bad"] == 0, r["out"]
    assert r["full"] >= 1 and r["reused"] >= 1, r["out"]


def test_host_port_cluster_is_reused(tool):
    """C5's candidates ask for host ports: their candidate side reads the spot
    pods' ports only through the base conflict rows of the port queries, which
    a reuse encode recomputes (kept by query, patched per changed node); the
    candidates' pods go onto spot nodes tick after tick, so those rows move."""
    r = run_check(tool, 5, 40)
    assert r["bad"] == 0, r["out"]
    assert r["reused"] == r["ticks"] and r["full"] == 0, r["out"]


@pytest.mark.parametrize("config", [2, 3, 5])
def test_reuse_survives_spot_order_moves(tool, config):
    """Pods on spot nodes change their cpu requests between ticks, so
    NewNodeMap re-sorts the spot list and the snapshot holds the same nodes in
    another order (nodes/nodes.go:95-97).  The encoder permutes its static view
    and the kept atom rows (encode.cpp permute_static) instead of rebuilding:
    every tick stays reused and equals a fresh encode."""
    r = run_check(tool, config, 60, mode="reuse-perm")
    assert r["bad"] == 0, r["out"]
    assert r["moved"] >= 30, r["out"]
    assert r["reused"] == r["ticks"] and r["full"] == 0, r["out"]


@pytest.mark.parametrize("mode", ["reuse", "reuse-perm"])
def test_realistic_variant_reuse(tool, mode):
    """The realistic variant (scalar resources, attachable volumes, init
    containers): a reuse recomputes the scalar / volume-limit atom rows and the
    shared scalar rows, and rechecks the fallback decisions that read the
    snapshot (a planned candidate's attachable volume now on a changed spot node
    ends the reuse).  Compared with a full encode by a copy of the encoder taken
    before the call (class and atom numbering follow its dictionaries' history)."""
    r = run_check(tool, 3, 40, env={"SR_SYNTH_REALISTIC": "1"}, mode=mode)
    assert r["bad"] == 0, r["out"]
    assert r["reused"] >= 3, r["out"]


def test_scalar_rows_turning_non_empty_flip_classes(tool):
    """a scalar-resource query row that goes from empty to
    non-empty (a spot node's extended-resource usage drops) must flip the
    classes built on it out of the certainly-empty class in the same reuse
    encode.  `reuse-scalar` fills every spot node allocating a GPU past its
    allocatable for two ticks in six, then frees it; every tick stays reused
    (the attachable-volume recheck scans every node when the state view was
    rebuilt) and equals a fresh encode, with class flips recorded."""
    r = run_check(tool, 3, 24, env={"SR_SYNTH_REALISTIC": "1"}, mode="reuse-scalar")
    assert r["bad"] == 0, r["out"]
    assert r["reused"] == r["ticks"], r["out"]
    flips = int(re.search(r"class flips (\d+)", r["out"]).group(1))
    assert flips >= 4, r["out"]


@pytest.mark.parametrize("config", [2, 3])
def test_affinity_variant_reuse(tool, config):
    """The affinity variant (hostname anti-affinity, zone DoNotSchedule
    spread): a reuse patches the DA / DB rows (AntiReuse: per node the pods'
    (term, side) codes, per value the counts), the spread rows and the domain
    path's base-count tables (SpreadReuse: per selector the nodes' counts) for
    the changed nodes only.  The added pods are the candidates' own replicas,
    so rows and tables move; every tick stays reused and equals a fresh encode
    (its kept terms numbered by their words, so the atom layout is the same)."""
    r = run_check(tool, config, 30, env={"SR_SYNTH_AFFINITY": "1"})
    assert r["bad"] == 0, r["out"]
    assert r["reused"] >= r["ticks"] * 3 // 4, r["out"]  # a DA / DB row turning (non-)empty re-encodes


def test_affinity_variant_reuse_survives_spot_order_moves(tool):
    """The affinity variant with the spot order moving between ticks: the
    AntiReuse / SpreadReuse states, the node-local base tables and the domain
    path's node domains are permuted with the atom rows (anti_reuse_permute,
    spread_reuse_permute), then patched for the nodes whose own pods changed."""
    r = run_check(tool, 2, 40, env={"SR_SYNTH_AFFINITY": "1"}, mode="reuse-perm")
    assert r["bad"] == 0, r["out"]
    assert r["moved"] >= 20, r["out"]
    assert r["reused"] >= r["ticks"] * 3 // 4, r["out"]
