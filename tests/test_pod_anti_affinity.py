"""Required inter-pod anti-affinity (k8s v1.19.2 InterPodAffinity filter; SURVEY
§8f row 3): hand-derived known answers for the CPU oracle, one per rule of the
upstream filter, and the product's host-side fallback decisions.  The GPU
parity of the same cases (and of random clusters carrying anti-affinity) is in
test_gpu_parity.py.  Parity unpinned: the filter lives in k8s.io/kubernetes
v1.19.2, which the reference tree does not vendor; every expected answer
below is derived by hand from the rule it names."""
import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import load_oracle, oracle_plan
from spotplanner import capi
from spotplanner.model import (Container, GiB, LabelSelector, LabelSelectorRequirement, Node, Pod,
                               PodAffinityTerm)

HOST = "kubernetes.io/hostname"
ZONE = "topology.kubernetes.io/zone"


def node(name, zone=None, cpu=4000, pods=110):
    labels = {HOST: name}
    if zone is not None:
        labels[ZONE] = zone
    return Node(name=name, cpu_milli=cpu, memory=8 * GiB, pods=pods, labels=labels)


def pod(name, labels=None, ns="default", anti=None, cpu=100):
    return Pod(name=name, namespace=ns, containers=[Container(cpu_milli=cpu)], labels=dict(labels or {}),
               pod_anti_affinity=anti)


def term(tk=HOST, ml=None, me=None, namespaces=None, nil=False):
    sel = None if nil else LabelSelector(dict(ml or {}), list(me or []))
    return PodAffinityTerm(tk, sel, list(namespaces or []))


def find(nodes, spot_pods, query):
    """oracle findSpotNodeForPod for each query pod: node name or ""."""
    sc = Scenario(nodes, spot_pods, query)
    snap = sc.oracle_snapshot()
    lib = load_oracle()
    out = []
    for i in range(len(query)):
        pos = lib.oracle_find_spot_node_for_pod(snap.h, sc.ptr, sc.qidx(i))
        out.append({-1: "", -2: "FALLBACK"}.get(pos, None) if pos < 0 else nodes[pos].name)
    return out


def plan(nodes, spot_pods, cands):
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cp = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    return oracle_plan(sc.oracle_snapshot(), sc.ptr, off, cp, mode=1), off


def test_existing_pod_anti_affinity_rejects_its_node():
    # existing pod on n0 refuses app=web on its hostname
    nodes = [node("n0"), node("n1")]
    spot = [[pod("e", anti=[term(ml={"app": "web"})])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"}), pod("q", {"app": "db"})]) == ["n1", "n0"]


def test_existing_term_selects_in_its_own_namespace_only():
    nodes = [node("n0"), node("n1")]
    spot = [[pod("e", ns="a", anti=[term(ml={"app": "web"})])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"}, ns="b"), pod("q", {"app": "web"}, ns="a")]) == ["n0", "n1"]


def test_term_namespaces_list():
    nodes = [node("n0"), node("n1")]
    spot = [[pod("e", ns="a", anti=[term(ml={"app": "web"}, namespaces=["b", "c"])])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"}, ns="b"), pod("q", {"app": "web"}, ns="a")]) == ["n1", "n0"]


def test_incoming_pod_anti_affinity_against_existing_pods():
    nodes = [node("n0"), node("n1"), node("n2")]
    spot = [[pod("e0", {"app": "db"})], [pod("e1", {"app": "db"}, ns="other")], []]
    # the incoming term selects app=db in the incoming pod's namespace ("default")
    assert find(nodes, spot, [pod("p", anti=[term(ml={"app": "db"})])]) == ["n1"]


def test_zone_topology_rejects_the_whole_zone():
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b")]
    spot = [[pod("e", anti=[term(ZONE, ml={"app": "web"})])], [], []]
    assert find(nodes, spot, [pod("p", {"app": "web"})]) == ["n2"]


def test_node_without_topology_key_counts_no_pair():
    # the existing pod's node has no zone label: its term adds no topology pair;
    # the incoming pod's node must also carry the key for a conflict
    nodes = [node("n0"), node("n1", "a")]
    spot = [[pod("e", anti=[term(ZONE, ml={"app": "web"})])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"})]) == ["n0"]
    nodes = [node("n0", "a"), node("n1")]
    spot = [[pod("e", anti=[term(ZONE, ml={"app": "web"})])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"})]) == ["n1"]


def test_nil_selector_selects_nothing_empty_selects_everything():
    nodes = [node("n0"), node("n1")]
    spot = [[pod("e", anti=[term(nil=True)])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"})]) == ["n0"]
    spot = [[pod("e", anti=[term()])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"}), pod("q")]) == ["n1", "n1"]


def test_match_expressions():
    nodes = [node("n0"), node("n1")]
    R = LabelSelectorRequirement
    cases = [(R("tier", "In", ["fe", "be"]), {"tier": "be"}, "n1"),
             (R("tier", "In", ["fe"]), {"tier": "be"}, "n0"),
             (R("tier", "NotIn", ["fe"]), {}, "n1"),
             (R("tier", "NotIn", ["fe"]), {"tier": "fe"}, "n0"),
             (R("tier", "Exists"), {"tier": "x"}, "n1"),
             (R("tier", "DoesNotExist"), {"tier": "x"}, "n0"),
             (R("tier", "DoesNotExist"), {}, "n1")]
    for req, labels, want in cases:
        spot = [[pod("e", anti=[term(me=[req])])], []]
        assert find(nodes, spot, [pod("p", labels)]) == [want], req


def test_match_labels_and_expressions_are_anded():
    nodes = [node("n0"), node("n1")]
    t = term(ml={"app": "web"}, me=[LabelSelectorRequirement("tier", "In", ["fe"])])
    spot = [[pod("e", anti=[t])], []]
    assert find(nodes, spot, [pod("p", {"app": "web"}), pod("q", {"app": "web", "tier": "fe"})]) == ["n0", "n1"]


def test_replicas_with_self_anti_affinity_spread_inside_one_candidate():
    # canDrainNode places r0 on n0; r1 (same labels, same term) is then refused
    # on n0 by both directions of the filter and goes to n1; r2 to n2
    nodes = [node("n0"), node("n1"), node("n2")]
    t = [term(ml={"app": "web"})]
    cands = [[pod("r%d" % i, {"app": "web"}, anti=t) for i in range(3)]]
    o, off = plan(nodes, [[], [], []], cands)
    assert int(o["status"][0]) == capi.SR_CAND_OK
    assert list(o["node_of_pod"][:3]) == [0, 1, 2]
    # a fourth replica finds no node
    cands = [[pod("r%d" % i, {"app": "web"}, anti=t) for i in range(4)]]
    o, off = plan(nodes, [[], [], []], cands)
    assert int(o["status"][0]) == 3


def test_candidates_start_from_the_base_snapshot():
    # candidate 0 fails after placing a pod that would block candidate 1; the
    # Revert between candidates means candidate 1 does not see it
    nodes = [node("n0", cpu=1000)]
    blocker = pod("b", {"app": "x"}, anti=[term(ml={"app": "y"})])
    big = pod("big", cpu=5000)
    cands = [[blocker, big], [pod("y", {"app": "y"})]]
    o, off = plan(nodes, [[]], cands)
    assert int(o["status"][0]) == 1 and int(o["status"][1]) == capi.SR_CAND_OK


def test_opaque_or_invalid_anti_affinity_falls_back():
    nodes = [node("n0"), node("n1")]
    opaque = Pod(name="e", containers=[Container(cpu_milli=10)], required_pod_anti_affinity=True)
    assert find(nodes, [[opaque], []], [pod("p")]) == ["FALLBACK"]
    bad = [term(me=[LabelSelectorRequirement("app", "In", [])])]
    assert find(nodes, [[pod("e", anti=bad)], []], [pod("p")]) == ["FALLBACK"]
    assert find(nodes, [[], []], [pod("p", anti=bad), pod("q")]) == ["FALLBACK", "n0"]
    odd = [term(me=[LabelSelectorRequirement("app", "Gt", ["1"])])]
    assert find(nodes, [[], []], [pod("p", anti=odd)]) == ["FALLBACK"]
