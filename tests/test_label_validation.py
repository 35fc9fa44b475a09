"""labels.NewRequirement's key / value validation (apimachinery v0.19.2
labels/selector.go validateLabelKey / validateLabelValue), which the
reference's predicate checker (call site rescheduler.go:344) runs through
NodeSelectorRequirementsAsSelector (required node affinity) and
metav1.LabelSelectorAsSelector (inter-pod terms).

The planner sees interned ids only; the shim passes each string's validity
(sr_cluster.str_label).  The node-affinity consequences are pinned by
tests/known_answer.py (a term with an invalid key or value matches nothing,
on the oracle and on the GPU).  Here: the shim's validity functions against a
hand-derived table of the published regular expressions and lengths, the
synthetic generator's table against the same functions, and the inter-pod
consequence (the term fails to build: the pod goes to the reference path) on
the oracle and the product.  Parity unpinned beyond the reference's own tests:
the rules live in k8s.io/apimachinery, which the reference tree does not
vendor; every expectation below is derived by hand from the rule it names."""
import ctypes

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import load_oracle, oracle_plan
from spotplanner import capi
from spotplanner.model import (Container, GiB, LabelSelector, LabelSelectorRequirement, Node, NodeSelectorRequirement,
                               NodeSelectorTerm, Pod, PodAffinityTerm, is_qualified_name, is_valid_label_value)

# IsValidLabelValue: empty, or <= 63 characters of ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]
VALUES = [("", True), ("a", True), ("A-b_c.9", True), ("0", True), ("012", True), ("v" * 63, True),
          ("v" * 64, False), ("-3", False), ("+012", False), ("a.", False), ("_a", False), ("a b", False),
          ("a/b", False), ("é", False), ("a\n", False), ("x" * 62 + "-", False), ("1.5", True)]
# IsQualifiedName: [DNS-1123 subdomain "/"] name, name 1..63 characters of the same pattern
KEYS = [("zone", True), ("kubernetes.io/hostname", True), ("topology.kubernetes.io/zone", True),
        ("example.com/Zone_1", True), ("", False), ("bad key", False), ("/zone", False), ("a/b/c", False),
        ("Example.com/zone", False), ("example.com/", False), ("-a", False), ("a" * 63, True), ("a" * 64, False),
        ("x.y-z/a", True), ("x..y/a", False), ("-x.com/a", False), ("x." * 126 + "y/a", True),
        ("x" * 254 + "/a", False)]


@pytest.mark.parametrize("s,ok", VALUES)
def test_is_valid_label_value(s, ok):
    assert is_valid_label_value(s) == ok


@pytest.mark.parametrize("s,ok", KEYS)
def test_is_qualified_name(s, ok):
    assert is_qualified_name(s) == ok


def test_synthetic_generator_table_matches_shim():
    """libsrsynth computes str_label itself (C++): the same answers as the shim's functions."""
    from spotplanner.synth import SynthCluster
    sc = SynthCluster(3, n_on_demand=20, n_spot=30)
    c = sc.cluster
    n = c.n_strings
    assert n == sc.lib.sr_synth_num_strings(sc.handle) and n > 10
    for i in range(n):
        s = sc.lib.sr_synth_string(sc.handle, i).decode()
        want = (capi.SR_STR_LABEL_VALUE if is_valid_label_value(s) else 0) | \
               (capi.SR_STR_LABEL_KEY if is_qualified_name(s) else 0)
        assert c.str_label[i] == want, s


def test_synthetic_generator_flags_like_shim_on_edge_strings():
    """The C++ restatement (synth.cpp label_flags) on the hand-derived table."""
    from spotplanner.synth import synth_label_flags
    for s, ok in VALUES:
        assert bool(synth_label_flags(s) & capi.SR_STR_LABEL_VALUE) == ok, s
    for s, ok in KEYS:
        assert bool(synth_label_flags(s) & capi.SR_STR_LABEL_KEY) == ok, s


HOST = "kubernetes.io/hostname"


def _nodes():
    return [Node("n%d" % i, cpu_milli=4000, memory=8 * GiB, labels={HOST: "n%d" % i, "zone": "a"}) for i in range(3)]


def _pod(name, labels=None, anti=None, aff=None):
    return Pod(name, namespace="default", containers=[Container(cpu_milli=100)], labels=dict(labels or {}),
               pod_anti_affinity=anti, pod_affinity=aff)


INVALID_SELECTORS = {
    "match_labels_value": LabelSelector({"app": "-web"}),
    "match_labels_key": LabelSelector({"bad key": "web"}),
    "expression_value": LabelSelector({}, [LabelSelectorRequirement("app", "In", ["web", "v" * 64])]),
    "expression_key": LabelSelector({}, [LabelSelectorRequirement("Example.com/app", "Exists", [])]),
}


@pytest.mark.parametrize("which", sorted(INVALID_SELECTORS))
def test_oracle_invalid_selector_routes_to_reference_path(which):
    """LabelSelectorAsSelector fails: the incoming pod's terms cannot be built
    (InterPodAffinity PreFilter: parse error), and an existing spot pod's
    anti-affinity terms cannot be read -- both leave the encoded set."""
    sel = INVALID_SELECTORS[which]
    lib = load_oracle()
    # the incoming pod's anti-affinity / affinity term
    for kw in ({"anti": [PodAffinityTerm(HOST, sel)]}, {"aff": [PodAffinityTerm("zone", sel)]}):
        sc = Scenario(_nodes(), [[], [], []], [_pod("p", {"app": "web"}, **kw)])
        assert lib.oracle_find_spot_node_for_pod(sc.oracle_snapshot().h, sc.ptr, sc.qidx(0)) == -2
    # an existing pod's anti-affinity: every candidate falls back
    base = [[_pod("e", {"app": "db"}, anti=[PodAffinityTerm(HOST, sel)])], [], []]
    sc = Scenario(_nodes(), base, [_pod("p", {"app": "web"})])
    assert lib.oracle_find_spot_node_for_pod(sc.oracle_snapshot().h, sc.ptr, sc.qidx(0)) == -2
    # the valid twin of the same selector is evaluated
    good = LabelSelector({"app": "web"})
    sc = Scenario(_nodes(), [[_pod("e", {"app": "db"}, anti=[PodAffinityTerm(HOST, good)])], [], []],
                  [_pod("p", {"app": "web"})])
    assert lib.oracle_find_spot_node_for_pod(sc.oracle_snapshot().h, sc.ptr, sc.qidx(0)) == 1


def _without_label_table(sc):
    sc.enc.struct.str_label = ctypes.cast(None, capi.PU8)
    return sc


def test_oracle_without_label_table_routes_node_affinity_to_fallback():
    """Without str_label the strings' validity is unknown: a pod with
    node-affinity matchExpressions, or an inter-pod term with a label
    requirement, is routed to the reference path; other pods are evaluated."""
    lib = load_oracle()
    na = Pod("p", containers=[Container(cpu_milli=100)],
             required_node_affinity=[NodeSelectorTerm([NodeSelectorRequirement("zone", "In", ["a"])])])
    fields_only = Pod("q", containers=[Container(cpu_milli=100)],
                      required_node_affinity=[NodeSelectorTerm([], [NodeSelectorRequirement("metadata.name", "In",
                                                                                             ["n1"])])])
    anti = _pod("r", {"app": "web"}, anti=[PodAffinityTerm(HOST, LabelSelector({"app": "web"}))])
    plain = Pod("s", containers=[Container(cpu_milli=100)], node_selector={"zone": "a"})
    sc = _without_label_table(Scenario(_nodes(), [[], [], []], [na, fields_only, anti, plain]))
    snap = sc.oracle_snapshot()
    got = [lib.oracle_find_spot_node_for_pod(snap.h, sc.ptr, sc.qidx(i)) for i in range(4)]
    assert got == [-2, 1, -2, 0]


def test_oracle_plan_marks_invalid_selector_candidates():
    sel = INVALID_SELECTORS["match_labels_value"]
    cands = [[_pod("a", {"app": "web"})], [_pod("b", {"app": "web"}, anti=[PodAffinityTerm(HOST, sel)])],
             [_pod("c", {"app": "web"})]]
    flat = [p for c in cands for p in c]
    sc = Scenario(_nodes(), [[], [], []], flat)
    off = np.array([0, 1, 2, 3], np.int32)
    o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, np.arange(sc.q0, sc.q0 + 3, dtype=np.int32), mode=1)
    assert list(o["status"]) == [capi.SR_CAND_OK, capi.SR_CAND_FALLBACK, capi.SR_CAND_OK]


@pytest.mark.gpu
@pytest.mark.parametrize("which", sorted(INVALID_SELECTORS))
def test_gpu_invalid_selector_routes_to_reference_path(checker, which):
    from spotplanner.rescheduler import plan_arrays
    sel = INVALID_SELECTORS[which]
    lib = capi.load_planner()
    scen = [  # (spot pods, candidate pods): incoming anti, incoming affinity, existing anti
        ([[], [], []], [_pod("p", {"app": "web"}, anti=[PodAffinityTerm(HOST, sel)])]),
        ([[], [], []], [_pod("p", {"app": "web"}, aff=[PodAffinityTerm("zone", sel)])]),
        ([[_pod("e", {"app": "db"}, anti=[PodAffinityTerm(HOST, sel)])], [], []], [_pod("p", {"app": "web"})]),
    ]
    for base, pods in scen:
        sc = Scenario(_nodes(), base, pods)
        h = sc.product_snapshot()
        try:
            p = plan_arrays(checker, h, sc.ptr, np.array([0, 1], np.int32), np.array([sc.qidx(0)], np.int32))
        finally:
            lib.sr_snapshot_destroy(h)
        assert list(p.status) == [capi.SR_CAND_FALLBACK] and p.first_fallback == 0 and p.winner == -1


@pytest.mark.gpu
def test_gpu_without_label_table_routes_node_affinity_to_fallback(checker):
    from spotplanner.rescheduler import plan_arrays
    lib = capi.load_planner()
    na = Pod("p", containers=[Container(cpu_milli=100)],
             required_node_affinity=[NodeSelectorTerm([NodeSelectorRequirement("zone", "In", ["a"])])])
    fields_only = Pod("q", containers=[Container(cpu_milli=100)],
                      required_node_affinity=[NodeSelectorTerm([], [NodeSelectorRequirement("metadata.name", "In",
                                                                                             ["n1"])])])
    anti = _pod("r", {"app": "web"}, anti=[PodAffinityTerm(HOST, LabelSelector({"app": "web"}))])
    plain = Pod("s", containers=[Container(cpu_milli=100)], node_selector={"zone": "a"})
    sc = _without_label_table(Scenario(_nodes(), [[], [], []], [na, fields_only, anti, plain]))
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, np.arange(5, dtype=np.int32), np.arange(sc.q0, sc.q0 + 4,
                                                                                    dtype=np.int32))
    finally:
        lib.sr_snapshot_destroy(h)
    FB = capi.SR_CAND_FALLBACK
    assert list(p.status) == [FB, capi.SR_CAND_OK, FB, capi.SR_CAND_OK]
    assert list(p.node_of_pod) == [-1, 1, -1, 0]
