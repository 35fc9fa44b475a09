"""The Python mirror of the reference API (findSpotNodeForPod / canDrainNode /
ClusterSnapshot.AddPod) on the GPU when the query pods come in a cluster of
their own: the snapshot must keep what InterPodAffinity reads from the pods it
holds (namespace, labels, anti-affinity terms), not indices into the cluster
it was built from."""
import pytest

from spotplanner import nodes as N
from spotplanner.model import Container, GiB, LabelSelector, Node, Pod, PodAffinityTerm
from spotplanner.planner import NewBasicClusterSnapshot, NewTestPredicateChecker
from spotplanner.rescheduler import canDrainNode, findSpotNodeForPod

pytestmark = pytest.mark.gpu
HOST = "kubernetes.io/hostname"


def _spot(names, pods_per_node):
    infos = []
    snap = NewBasicClusterSnapshot()
    for name, pods in zip(names, pods_per_node):
        node = Node(name, cpu_milli=4000, memory=8 * GiB, pods=110, labels={HOST: name})
        req = sum(p.cpu_sort_milli() for p in pods)
        infos.append(N.NodeInfo(node, pods, req, node.cpu_milli - req))
        snap.AddNodeWithPods(node, pods)
    return N.NodeInfoArray(infos), snap


def _pod(name, app, anti_app=None):
    terms = [PodAffinityTerm(HOST, LabelSelector({"app": anti_app}))] if anti_app else None
    return Pod(name, namespace="default", labels={"app": app}, containers=[Container(cpu_milli=100)],
               pod_anti_affinity=terms)


def test_existing_pod_anti_affinity_selects_a_plain_incoming_pod():
    # db on node1 refuses web pods on its host; the web pod has no terms itself
    checker, _ = NewTestPredicateChecker()
    infos, snap = _spot(["node1", "node2"], [[_pod("db", "db", anti_app="web")], []])
    assert findSpotNodeForPod(checker, snap, infos, _pod("w", "web")) == "node2"
    assert findSpotNodeForPod(checker, snap, infos, _pod("x", "other")) == "node1"


def test_incoming_pod_anti_affinity_against_the_snapshot_pods():
    checker, _ = NewTestPredicateChecker()
    infos, snap = _spot(["node1", "node2", "node3"], [[_pod("db", "db")], [_pod("c", "cache")], []])
    assert findSpotNodeForPod(checker, snap, infos, _pod("w", "web", anti_app="db")) == "node2"
    assert findSpotNodeForPod(checker, snap, infos, _pod("w2", "web", anti_app="cache")) == "node1"


def test_can_drain_node_sees_existing_anti_affinity_and_added_pods():
    checker, _ = NewTestPredicateChecker()
    infos, snap = _spot(["node1", "node2", "node3"], [[_pod("db", "db", anti_app="web")], [], []])
    pods = [_pod("w1", "web", anti_app="web"), _pod("w2", "web", anti_app="web"), _pod("o", "other")]
    assert canDrainNode(checker, snap, infos, pods) is None
    assert canDrainNode.last_mapping == ["node2", "node3", "node1"]
    # the snapshot now holds w1 and w2 (rescheduler.go:366): a third replica fits nowhere
    err = canDrainNode(checker, snap, infos, [_pod("w3", "web", anti_app="web")])
    assert str(err) == "pod default/w3 can't be rescheduled on any existing spot node"


def test_add_pod_from_another_cluster_keeps_its_terms():
    checker, _ = NewTestPredicateChecker()
    infos, snap = _spot(["node1", "node2"], [[], []])
    snap.AddPod(_pod("guard", "guard", anti_app="web"), "node1")
    assert findSpotNodeForPod(checker, snap, infos, _pod("w", "web")) == "node2"
    snap.Fork()
    snap.AddPod(_pod("guard2", "guard", anti_app="web"), "node2")
    assert findSpotNodeForPod(checker, snap, infos, _pod("w", "web")) == ""
    snap.Revert()  # guard2 is gone again
    assert findSpotNodeForPod(checker, snap, infos, _pod("w", "web")) == "node2"


def test_can_drain_node_clears_node_name_of_evaluated_pods_only():
    # rescheduler.go:341 runs inside findSpotNodeForPod, which canDrainNode stops
    # calling after the first pod that fits nowhere
    checker, _ = NewTestPredicateChecker()
    infos, snap = _spot(["node1"], [[]])
    pods = [Pod("a", node_name="od1", containers=[Container(cpu_milli=1000)]),
            Pod("b", node_name="od1", containers=[Container(cpu_milli=5000)]),
            Pod("c", node_name="od1", containers=[Container(cpu_milli=10)])]
    assert canDrainNode(checker, snap, infos, pods) is not None
    assert [p.node_name for p in pods] == ["", "", "od1"]
