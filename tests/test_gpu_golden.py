"""The reference's own test vectors (rescheduler_test.go) through the product's
GPU path, written like the reference tests."""
import pytest

from helpers import fixture_node, fixture_pod, golden
from spotplanner import nodes as N
from spotplanner.model import Container, Pod
from spotplanner.planner import NewBasicClusterSnapshot, NewTestPredicateChecker
from spotplanner.rescheduler import canDrainNode, findSpotNodeForPod

pytestmark = pytest.mark.gpu
G = golden()


def _create_snapshot(node_infos):
    """_createSnapshot (rescheduler_test.go:31-38)."""
    snapshot = NewBasicClusterSnapshot()
    for ni in node_infos:
        snapshot.AddNodeWithPods(ni.Node, ni.Pods)
    return snapshot


def _node_infos(fx):
    out = []
    for s in fx["spot"]:
        pods = [fixture_pod(p) for p in s["pods"]]
        req = sum(p.cpu_sort_milli() for p in pods)
        node = fixture_node(s["node"])
        out.append(N.NodeInfo(node, pods, req, node.cpu_milli - req))
    return N.NodeInfoArray(out)


def test_find_spot_node_for_pod():
    fx = G["TestFindSpotNodeForPod"]
    predicate_checker, _ = NewTestPredicateChecker()
    node_infos = _node_infos(fx)
    snapshot = _create_snapshot(node_infos)
    for q in fx["queries"]:
        assert findSpotNodeForPod(predicate_checker, snapshot, node_infos, fixture_pod(q["pod"])) == q["expect"]


def test_can_drain_node():
    fx = G["TestCanDrainNode"]
    predicate_checker, _ = NewTestPredicateChecker()
    spot_node_infos = _node_infos(fx)
    snapshot = _create_snapshot(spot_node_infos)
    c1, c2 = fx["calls"]
    err1 = canDrainNode(predicate_checker, snapshot, spot_node_infos, [fixture_pod(p) for p in c1["pods"]])
    assert err1 is None, "canDrainNode should be successful with podsForDeletion1"
    assert canDrainNode.last_mapping == c1["derived_mapping"]
    pods2 = [fixture_pod(p) for p in c2["pods"]]
    err2 = canDrainNode(predicate_checker, snapshot, spot_node_infos, pods2)
    assert err2 is not None, "canDrainNode should fail with podsForDeletion2, too much requested CPU."
    assert str(err2) == "pod kube-system/%s can't be rescheduled on any existing spot node" % \
        pods2[c2["derived_fail_pod"]].name


def test_can_drain_node_fork_revert_like_run():
    # run() brackets canDrainNode with Fork / Revert (rescheduler.go:269-274).
    fx = G["TestCanDrainNode"]
    checker, _ = NewTestPredicateChecker()
    infos = _node_infos(fx)
    snapshot = _create_snapshot(infos)
    c1, c2 = fx["calls"]
    for _ in range(3):
        snapshot.Fork()
        assert canDrainNode(checker, snapshot, infos, [fixture_pod(p) for p in c1["pods"]]) is None
        snapshot.Revert()
    snapshot.Fork()
    assert canDrainNode(checker, snapshot, infos, [fixture_pod(p) for p in c2["pods"]]) is not None
    snapshot.Revert()
    assert snapshot.node_state("node3") == ((1300, 0, 0), 3)


def test_find_spot_node_sets_node_name_empty():
    fx = G["TestFindSpotNodeForPod"]
    checker, _ = NewTestPredicateChecker()
    infos = _node_infos(fx)
    snapshot = _create_snapshot(infos)
    pod = Pod("bound", node_name="elsewhere", containers=[Container(100)])
    assert findSpotNodeForPod(checker, snapshot, infos, pod) == "node1"
    assert pod.node_name == ""
