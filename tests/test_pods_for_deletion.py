"""The candidate lists of run() (rescheduler.go:228-264): GetPodsForDeletionOnNodeDrain
with the reference's arguments, then the DaemonSet-owner filter.

The drain rules live in cluster-autoscaler utils/drain (@03f60a4c3818), which
the reference does not vendor and no reference test exercises (its test pods
have no owner references and never reach run()).  Parity here is UNPINNED:
the oracle (oracle_pods_for_deletion) restates the published CA algorithm,
the known-answer cases below are derived by hand from it, one per rule, and
the product (sr_pods_for_deletion, host C++) must agree with the oracle on
every case and on random pod mixes.  CPU only: no device work on this step."""
import ctypes
import random

import numpy as np
import pytest

from oracle_lib import load_oracle
from spotplanner import capi
from spotplanner.model import (Container, EncodedDrain, NilControllerPanic, Node, OwnerReference, Pod,
                               PodDisruptionBudget, encode_cluster)
from spotplanner.rescheduler import podsForDeletion, updateSpotNodeMetrics
from spotplanner.synth import SynthCluster, build_candidates, new_node_map, pods_for_deletion

B = capi
RS = [OwnerReference("ReplicaSet")]


def mk(name, **kw):
    kw.setdefault("owner_references", RS)
    kw.setdefault("containers", [Container(100)])
    return Pod(name, **kw)


def names(pods):
    return [p.name for p in pods]


# ------------------------------------------------------------- known answers
def test_mirror_and_daemonset_pods_are_skipped():
    pods = [mk("m", annotations={"kubernetes.io/config.mirror": "x"}, owner_references=[]),
            mk("ds", owner_references=[OwnerReference("DaemonSet")]),
            mk("dsa", owner_references=[], annotations={"cluster-autoscaler.kubernetes.io/daemonset-pod": "true"}),
            mk("a")]
    out, blocking, err = podsForDeletion(pods, [])
    assert names(out) == ["a"] and blocking is None and err is None


def test_replication_controller_ref_wins_over_daemonset_annotation():
    # the CA checks the ReplicationController kind before IsDaemonSetPod
    p = mk("rc", owner_references=[OwnerReference("ReplicationController")],
           annotations={"cluster-autoscaler.kubernetes.io/daemonset-pod": "true"})
    assert names(podsForDeletion([p], [])[0]) == ["rc"]


@pytest.mark.parametrize("kind", ["ReplicationController", "Job", "ReplicaSet", "StatefulSet"])
def test_replicated_controller_kinds(kind):
    assert names(podsForDeletion([mk("p", owner_references=[OwnerReference(kind)])], [])[0]) == ["p"]


@pytest.mark.parametrize("owners", [[], [OwnerReference("Deployment")], [OwnerReference("ReplicaSet", controller=False)]])
def test_not_replicated_blocks_the_node(owners):
    pods = [mk("a"), mk("lonely", owner_references=owners), mk("b")]
    out, blocking, err = podsForDeletion(pods, [])
    assert out == [] and blocking.Pod.name == "lonely" and blocking.Reason == B.SR_BLOCK_NOT_REPLICATED
    assert str(err) == "kube-system/lonely is not replicated"


def test_first_blocking_pod_in_list_order():
    pods = [mk("x", owner_references=[]), mk("y", local_storage=True)]
    _, blocking, _ = podsForDeletion(pods, [])
    assert blocking.Pod.name == "x"


def test_safe_to_evict_and_terminal_pods_are_movable_without_a_controller():
    pods = [mk("s", owner_references=[], annotations={"cluster-autoscaler.kubernetes.io/safe-to-evict": "true"}),
            mk("t1", owner_references=[], phase="Succeeded", restart_policy="Never"),
            mk("t2", owner_references=[], phase="Failed", restart_policy="Never"),
            mk("t3", owner_references=[], phase="Succeeded", restart_policy="OnFailure"),
            mk("t4", owner_references=[], phase="Failed", restart_policy="Always")]
    assert names(podsForDeletion(pods, [])[0]) == ["s", "t1", "t2", "t3", "t4"]


def test_succeeded_with_restart_always_is_not_terminal():
    _, blocking, _ = podsForDeletion([mk("t", owner_references=[], phase="Succeeded", restart_policy="Always")], [])
    assert blocking is not None and blocking.Reason == B.SR_BLOCK_NOT_REPLICATED


@pytest.mark.parametrize("age,grace,skipped", [(61, None, True), (60, None, False), (41, 10, True), (40, 10, False),
                                               (5, 0, False), (30.5, 0, True)])
def test_long_terminating_pods_are_skipped(age, grace, skipped):
    # deletionTimestamp + grace (default 30 s) + 30 s strictly before now
    p = mk("d", owner_references=[], deletion_age_s=age, grace_seconds=grace)
    out, blocking, _ = podsForDeletion([p], [])
    if skipped:
        assert out == [] and blocking is None
    else:
        assert blocking is not None and blocking.Pod.name == "d"


def test_kube_system_pods_need_a_pdb_only_when_skipping_system_pods():
    p = mk("sys", labels={"app": "dns"})
    assert names(podsForDeletion([p], [], deleteNonReplicatedPods=False)[0]) == ["sys"]
    out, blocking, err = podsForDeletion([p], [], deleteNonReplicatedPods=True)
    assert blocking.Reason == B.SR_BLOCK_UNMOVABLE_KUBE_SYSTEM
    assert str(err) == "non-daemonset, non-mirrored, non-pdb-assigned kube-system pod present: sys"
    pdb = PodDisruptionBudget(match_labels={"app": "dns"})
    assert names(podsForDeletion([p], [pdb], deleteNonReplicatedPods=True)[0]) == ["sys"]
    other_ns = PodDisruptionBudget(namespace="default", match_labels={})
    assert podsForDeletion([p], [other_ns], deleteNonReplicatedPods=True)[1].Reason == B.SR_BLOCK_UNMOVABLE_KUBE_SYSTEM
    assert names(podsForDeletion([mk("n", namespace="default")], [], deleteNonReplicatedPods=True)[0]) == ["n"]


def test_kube_system_pdb_selector_error_only_before_a_match():
    p = mk("sys", labels={"app": "dns"})
    match, bad = PodDisruptionBudget(match_labels={"app": "dns"}), PodDisruptionBudget(invalid=True)
    assert podsForDeletion([p], [bad, match], True)[1].Reason == B.SR_BLOCK_UNEXPECTED_ERROR
    assert names(podsForDeletion([p], [match, bad], True)[0]) == ["sys"]
    assert podsForDeletion([p], [PodDisruptionBudget(match_labels=None)], True)[1].Reason == \
        B.SR_BLOCK_UNMOVABLE_KUBE_SYSTEM  # nil selector selects nothing
    assert names(podsForDeletion([p], [PodDisruptionBudget(match_labels={})], True)[0]) == ["sys"]


def test_local_storage_is_not_checked_with_the_reference_arguments():
    # skipNodesWithLocalStorage is false at rescheduler.go:231
    assert names(podsForDeletion([mk("ls", local_storage=True)], [])[0]) == ["ls"]


def test_not_safe_to_evict_annotation_blocks():
    p = mk("n", annotations={"cluster-autoscaler.kubernetes.io/safe-to-evict": "false"})
    out, blocking, err = podsForDeletion([p], [])
    assert blocking.Reason == B.SR_BLOCK_NOT_SAFE_TO_EVICT
    assert str(err) == "pod annotated as not safe to evict present: n"


def test_daemonset_owner_filter_and_nil_controller_panic():
    # a non-controller DaemonSet owner does not make IsDaemonSetPod true, and the
    # reference's own filter needs *Controller && Kind == DaemonSet
    p = mk("p", owner_references=[OwnerReference("DaemonSet", controller=False), OwnerReference("ReplicaSet")])
    assert names(podsForDeletion([p], [])[0]) == ["p"]
    with pytest.raises(NilControllerPanic):
        podsForDeletion([mk("q", owner_references=[OwnerReference("ReplicaSet"), OwnerReference("Foo", controller=None)])],
                        [])
    # the owner loop breaks at a DaemonSet controller before reaching the nil one;
    # the pod is a DaemonSet pod for the CA anyway
    ok = mk("r", owner_references=[OwnerReference("DaemonSet"), OwnerReference("Foo", controller=None)])
    assert podsForDeletion([ok], [])[0] == []
    # a blocked node never reaches the filter
    blocked = [mk("x", owner_references=[]), mk("q", owner_references=[OwnerReference("Foo", controller=None)])]
    assert podsForDeletion(blocked, [])[1].Pod.name == "x"


# ------------------------------------------------------------ product == oracle
def rand_pod(r: random.Random, i: int) -> Pod:
    kinds = ["ReplicaSet", "Job", "StatefulSet", "ReplicationController", "DaemonSet", "Deployment", None]
    owners = []
    for _ in range(r.choice([0, 1, 1, 1, 2])):
        k = r.choice(kinds)
        if k is not None:
            owners.append(OwnerReference(k, controller=r.choice([True, True, False, None if r.random() < 0.05 else True])))
    ann = {}
    if r.random() < 0.1:
        ann["cluster-autoscaler.kubernetes.io/safe-to-evict"] = r.choice(["true", "false", "maybe"])
    if r.random() < 0.05:
        ann["cluster-autoscaler.kubernetes.io/daemonset-pod"] = r.choice(["true", "false"])
    if r.random() < 0.05:
        ann["kubernetes.io/config.mirror"] = "m"
    return Pod("p%d" % i, namespace=r.choice(["kube-system", "default"]), containers=[Container(100)],
               labels={"app": r.choice(["a", "b", "c"])}, annotations=ann, owner_references=owners,
               phase=r.choice(["Running", "Running", "Succeeded", "Failed", "Pending"]),
               restart_policy=r.choice(["Always", "OnFailure", "Never"]),
               deletion_age_s=None if r.random() < 0.8 else r.choice([10.0, 59.9, 60.1, 100.0]),
               grace_seconds=None if r.random() < 0.5 else r.choice([0, 10, 30, 120]),
               local_storage=r.random() < 0.1)


@pytest.mark.parametrize("seed", range(30))
def test_product_matches_oracle_on_random_pods(seed):
    r = random.Random(9000 + seed)
    n_nodes = 12
    pods, pod_node = [], []
    for node in range(n_nodes):
        for _ in range(r.randint(0, 9)):
            pods.append(rand_pod(r, len(pods)))
            pod_node.append(node)
    pdbs = [PodDisruptionBudget(namespace=r.choice(["kube-system", "default"]),
                                match_labels=r.choice([{"app": "a"}, {"app": "b"}, {}, None]),
                                invalid=r.random() < 0.15) for _ in range(r.randint(0, 3))]
    enc = encode_cluster([Node("n%d" % i, 1000) for i in range(n_nodes)], pods, pod_node=pod_node)
    drain = EncodedDrain(pods, pdbs)
    off = np.zeros(n_nodes + 1, np.int32)
    for node in pod_node:
        off[node + 1] += 1
    off = np.cumsum(off).astype(np.int32)
    idx = np.argsort(np.asarray(pod_node, np.int32), kind="stable").astype(np.int32)
    order = np.array(r.sample(range(n_nodes), n_nodes), np.int32)
    for dnr, owner_filter in ((False, True), (True, True), (False, False), (True, False)):
        got = pods_for_deletion(capi.load_planner().sr_pods_for_deletion, enc.ptr, drain.ptr, order, off, idx, dnr,
                                owner_filter)
        want = pods_for_deletion(load_oracle().oracle_pods_for_deletion, enc.ptr, drain.ptr, order, off, idx, dnr,
                                 owner_filter)
        assert got[4] == want[4]
        if got[4] == capi.SR_OK:
            for a, b in zip(got[:4], want[:4]):
                assert np.array_equal(a, b), (seed, dnr)


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_synthetic_candidates(config):
    # every synthetic pod is ReplicaSet- or DaemonSet-controlled: the lists are
    # NodeInfo.Pods minus the DaemonSet pods, nothing blocks
    sc = SynthCluster(config)
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    got = pods_for_deletion(lib.sr_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain), nm.on_demand, nm.node_pod_off,
                            nm.node_pod_idx)
    want = pods_for_deletion(load_oracle().oracle_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain), nm.on_demand,
                             nm.node_pod_off, nm.node_pod_idx)
    off, pods = build_candidates(nm, sc.pod_flags())
    assert got[4] == want[4] == capi.SR_OK
    assert np.array_equal(got[0], off) and np.array_equal(got[1], pods)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    assert np.all(got[2] == -1)


def test_update_spot_node_metrics_counts():
    # rescheduler.go:388-399: counts of GetPodsForDeletionOnNodeDrain per spot
    # node; no DaemonSet-owner filter and no panic on nil controllers there;
    # a node whose call errors is skipped
    from spotplanner.nodes import NodeInfo
    n1 = NodeInfo(Node("s1", 4000), [mk("a"), mk("ds", owner_references=[OwnerReference("DaemonSet")]),
                                     mk("q", owner_references=[OwnerReference("ReplicaSet"),
                                                               OwnerReference("Foo", controller=None)])], 0, 0)
    n2 = NodeInfo(Node("s2", 4000), [mk("b"), mk("lonely", owner_references=[])], 0, 0)
    n3 = NodeInfo(Node("s3", 4000), [], 0, 0)
    assert updateSpotNodeMetrics([n1, n2, n3], []) == {"s1": 2, "s3": 0}


def test_repeated_nodes_match_oracle():
    # a node named twice in the input (the ABI does not forbid it)
    # gets its list twice, computed without two threads sharing its scratch
    # range (the repeated input runs serially): more than 256 nodes so the
    # parallel pass would otherwise be taken
    sc = SynthCluster(2)
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    order = np.concatenate([nm.on_demand, nm.on_demand[:40], nm.on_demand[::-1][:7]]).astype(np.int32)
    got = pods_for_deletion(lib.sr_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain), order, nm.node_pod_off,
                            nm.node_pod_idx)
    want = pods_for_deletion(load_oracle().oracle_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain), order,
                             nm.node_pod_off, nm.node_pod_idx)
    assert got[4] == want[4] == capi.SR_OK
    for a, b in zip(got[:4], want[:4]):
        assert np.array_equal(a, b)
