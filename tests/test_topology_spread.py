"""PodTopologySpread (whenUnsatisfiable: DoNotSchedule), the filter CheckPredicates
runs (rescheduler.go:344; k8s v1.19.2 plugins/podtopologyspread/filtering.go,
upstream, not vendored in the reference: parity unpinned beyond the
hand-derived answers here).

Rules the answers below are derived from: the pairs (key, value) come from
the spot nodes passing the pod's nodeSelector / required node affinity and
carrying every constraint's key; each pair counts the pods (the pod's
namespace, not terminating, selected) on every node with that value -- a node
lacking the key counts into the pair of the empty value; constraints on one key
share their pairs' counts; no pair at all passes every node; otherwise a node
lacking a key fails, and count + self-match - the key's minimum > maxSkew
fails.

The planner encodes a pod's constraints as one static row against the base
snapshot; a candidate with a pod whose constraint counts an earlier pod of the
candidate goes to the reference path, as does a selector that fails to build.
Checked on the oracle (CPU) and the GPU (C-ABI), plus random clusters on the
GPU against the oracle."""
import random

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import oracle_plan
from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import (Container, LabelSelector, LabelSelectorRequirement, Node, NodeSelectorRequirement,
                               NodeSelectorTerm, Pod, TopologySpreadConstraint)

OK, FB = capi.SR_CAND_OK, capi.SR_CAND_FALLBACK
Z = "topology.kubernetes.io/zone"
H = "kubernetes.io/hostname"
WEB = LabelSelector(match_labels={"app": "web"})


def zone_nodes():
    return [Node("a", cpu_milli=4000, labels={Z: "z1", H: "a"}),
            Node("b", cpu_milli=4000, labels={Z: "z1", H: "b"}),
            Node("c", cpu_milli=4000, labels={Z: "z2", H: "c"}),
            Node("d", cpu_milli=4000, labels={H: "d"})]


def web(name, ns="default", cpu=100, **kw):
    return Pod(name, namespace=ns, containers=[Container(cpu_milli=cpu)], labels={"app": "web"}, **kw)


def other(name, ns="default", cpu=100, labels=None):
    return Pod(name, namespace=ns, containers=[Container(cpu_milli=cpu)], labels=labels or {"app": "other"})


def spread(pod, *cs):
    pod.topology_spread = list(cs)
    return pod


def zc(skew=1, sel=WEB, key=Z, when="DoNotSchedule"):
    return TopologySpreadConstraint(skew, key, when, sel)


def cases():
    """(name, nodes, spot pods, candidates, expected oracle statuses, expected mappings)"""
    N = zone_nodes
    yield ("less_loaded_zone", N(), [[web("e")], [], [], []], [[spread(web("p"), zc())]], [OK], [[2]])
    yield ("balanced_first_node", N(), [[], [], [], []], [[spread(web("p"), zc())]], [OK], [[0]])
    yield ("equal_zones_first_node", N(), [[web("e")], [], [web("f")], []], [[spread(web("p"), zc())]], [OK], [[0]])
    yield ("node_without_key_refused", N(), [[other("x", cpu=2000)], [other("y", cpu=2000)], [other("z", cpu=2000)], []],
           [[spread(web("p", cpu=3000), zc())]], [0], [[-1]])
    yield ("no_constraint_same_pod_fits_keyless_node", N(),
           [[other("x", cpu=2000)], [other("y", cpu=2000)], [other("z", cpu=2000)], []],
           [[web("p", cpu=3000)]], [OK], [[3]])
    yield ("selector_not_matching_self", N(), [[web("e")], [], [], []], [[spread(other("p"), zc())]], [OK], [[0]])
    yield ("other_namespace_not_counted", N(), [[web("e", ns="other")], [], [], []],
           [[spread(web("p"), zc())]], [OK], [[0]])
    yield ("terminating_not_counted", N(), [[web("e", deletion_age_s=5.0)], [], [], []],
           [[spread(web("p"), zc())]], [OK], [[0]])
    # the pods of one candidate counted by each other: planned on the domain path
    yield ("earlier_pod_counted", N(), [[], [], [], []],
           [[web("q"), spread(web("p"), zc())]], [OK], [[0, 2]])
    yield ("three_replicas_zone", N(), [[], [], [], []],
           [[spread(web("p%d" % i), zc()) for i in range(3)]], [OK], [[0, 2, 0]])
    yield ("replicas_zone_min_moves", N(), [[web("e")], [], [], []],
           [[spread(web("p%d" % i), zc()) for i in range(3)]], [OK], [[2, 0, 2]])
    yield ("replicas_zone_skew_two", N(), [[web("e")], [], [], []],
           [[spread(web("p%d" % i), zc(skew=2)) for i in range(4)]], [OK], [[0, 2, 0, 2]])
    yield ("replicas_hostname", N(), [[], [], [], []],
           [[spread(web("p%d" % i), zc(key=H)) for i in range(3)]], [OK], [[0, 1, 2]])
    yield ("replicas_hostname_with_base", N(), [[web("e")], [], [], []],
           [[spread(web("p%d" % i), zc(key=H)) for i in range(3)]], [OK], [[1, 2, 3]])
    yield ("replicas_hostname_skew_two", N(), [[], [], [], []],
           [[spread(web("p%d" % i), zc(key=H, skew=2)) for i in range(3)]], [OK], [[0, 0, 1]])
    # the 5th replica counts 4 earlier ones and only 4 nodes hold the minimum:
    # the minimum could move, the planner leaves it to the reference path
    yield ("replicas_hostname_min_could_move_falls_back", N(), [[], [], [], []],
           [[spread(web("p%d" % i), zc(key=H)) for i in range(5)]], [FB], [[-1] * 5])
    yield ("replicas_zone_and_hostname", N(), [[], [], [], []],
           [[spread(web("p%d" % i), zc(), zc(key=H)) for i in range(3)]], [OK], [[0, 2, 1]])
    yield ("interacting_constraint_sharing_a_key_falls_back", N(), [[], [], [], []],
           [[web("q"), spread(web("p"), zc(), zc(sel=LabelSelector(match_labels={"tier": "fe"})))]], [FB], [[-1, -1]])
    yield ("earlier_pod_other_namespace_planned", N(), [[web("e")], [], [], []],
           [[web("q", ns="other"), spread(web("p"), zc())]], [OK], [[0, 2]])
    yield ("earlier_pod_not_selected_planned", N(), [[web("e")], [], [], []],
           [[other("q"), spread(web("p"), zc())]], [OK], [[0, 2]])
    yield ("later_pod_counted_is_planned", N(), [[web("e")], [], [], []],
           [[spread(web("p"), zc()), web("q")]], [OK], [[2, 0]])
    yield ("node_selector_restricts_pairs", N(), [[web("e")], [], [], []],
           [[spread(Pod("p", namespace="default", containers=[Container(cpu_milli=100)], labels={"app": "web"},
                        node_selector={Z: "z1"}), zc())]], [OK], [[0]])
    yield ("required_affinity_restricts_pairs", N(), [[web("e")], [], [], []],
           [[spread(Pod("p", namespace="default", containers=[Container(cpu_milli=100)], labels={"app": "web"},
                        required_node_affinity=[NodeSelectorTerm([NodeSelectorRequirement(Z, "In", ["z1"])])]),
                    zc())]], [OK], [[0]])
    # v1.19.2 calPreFilterState: the pairs come from the nodes passing the pod's
    # node affinity, but processNode then counts the matching pods of EVERY node
    # whose value names an existing pair.  p refuses node a by affinity, yet e on
    # a counts into (zone, z1): z1 = 1, z2 = 0, so b (1 + 1 - 0 > 1) fails and c
    # is the first fit.  (Counting only passing nodes would give z1 = 0 and b.)
    yield ("pods_on_node_failing_affinity_still_counted", N(), [[web("e")], [], [], []],
           [[spread(Pod("p", namespace="default", containers=[Container(cpu_milli=100)], labels={"app": "web"},
                        required_node_affinity=[NodeSelectorTerm([NodeSelectorRequirement(H, "NotIn", ["a"])])]),
                    zc())]], [OK], [[2]])
    yield ("no_pairs_pass_every_node", N(), [[web("e"), web("f")], [], [], []],
           [[spread(web("p"), zc(key="example.com/rack"))]], [OK], [[0]])
    yield ("nil_selector_counts_nothing", N(), [[web("e"), web("f")], [], [], []],
           [[spread(web("p"), zc(sel=None))]], [OK], [[0]])
    yield ("schedule_anyway_never_filters", N(), [[web("e"), web("f")], [], [], []],
           [[spread(web("p"), zc(when="ScheduleAnyway"))]], [OK], [[0]])
    yield ("max_skew_two", N(), [[web("e")], [], [], []], [[spread(web("p"), zc(skew=2))]], [OK], [[0]])
    yield ("hostname_key", N(), [[web("e")], [], [], []], [[spread(web("p"), zc(key=H))]], [OK], [[1]])
    # constraints on one key share their pairs: z1 counts e (app=web) and f (tier=fe)
    yield ("same_key_constraints_share_counts", N(),
           [[web("e")], [other("f", labels={"tier": "fe"})], [], []],
           [[spread(web("p"), zc(skew=2), zc(skew=1, sel=LabelSelector(match_labels={"tier": "fe"})))]], [OK], [[2]])
    yield ("two_keys_both_bind", N(), [[web("e")], [], [], []],
           [[spread(web("p"), zc(), zc(key=H))]], [OK], [[2]])
    yield ("expression_selector", N(), [[web("e")], [], [], []],
           [[spread(web("p"), zc(sel=LabelSelector(match_expressions=[
               LabelSelectorRequirement("app", "In", ["web", "api"])])))]], [OK], [[2]])
    bare = [Pod("e%d" % i, namespace="default", containers=[Container(cpu_milli=1)]) for i in range(2)]
    yield ("not_in_selector_counts_unlabelled", N(), [bare, [], [], []],
           [[spread(web("p"), zc(sel=LabelSelector(match_expressions=[
               LabelSelectorRequirement("app", "NotIn", ["web"])])))]], [OK], [[2]])
    yield ("invalid_selector_falls_back", N(), [[], [], [], []],
           [[spread(web("p"), zc(sel=LabelSelector(match_labels={"bad key!": "x"})))]], [FB], [[-1]])
    # maxSkew <= 0 fails API validation; the C ABI accepts it and sends the pod to the reference path
    yield ("max_skew_zero_falls_back", N(), [[web("e")], [], [], []], [[spread(web("p"), zc(skew=0))]], [FB], [[-1]])
    yield ("max_skew_negative_falls_back", N(), [[], [], [], []],
           [[web("q"), spread(web("p"), zc(skew=-1, key=H))]], [FB], [[-1, -1]])
    yield ("in_without_values_falls_back", N(), [[], [], [], []],
           [[spread(web("p"), zc(sel=LabelSelector(match_expressions=[LabelSelectorRequirement("app", "In", [])])))]],
           [FB], [[-1]])
    # a node lacking the key counts into the pair of the empty value: d's two
    # pods raise (zone, "") to 2, so the minimum is z1's 1 and a passes
    empty_zone = [Node("a", cpu_milli=4000, labels={Z: "z1"}), Node("e", cpu_milli=4000, labels={Z: ""}),
                  Node("d", cpu_milli=4000)]
    yield ("keyless_node_counts_into_empty_value", empty_zone, [[web("x")], [], [web("y"), web("z")]],
           [[spread(web("p"), zc())]], [OK], [[0]])
    # the same on the domain path: q (too big for a and e) lands on the keyless
    # d and counts into (zone, ""), so the minimum is 1 and p fits a
    small_e = [Node("a", cpu_milli=4000, labels={Z: "z1"}), Node("e", cpu_milli=1000, labels={Z: ""}),
               Node("d", cpu_milli=4000)]
    yield ("earlier_pod_on_keyless_node_counts_into_empty_value", small_e, [[web("x")], [], []],
           [[web("q", cpu=3950), spread(web("p"), zc())]], [OK], [[2, 0]])


def run_oracle(nodes, spot_pods, cands):
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32), mode=1)
    return off, o


@pytest.mark.parametrize("case", list(cases()), ids=lambda c: c[0])
def test_oracle_spread_cases(case):
    _, nodes, spot_pods, cands, want_status, want_map = case
    off, o = run_oracle(nodes, spot_pods, cands)
    assert [int(x) for x in o["status"]] == want_status
    for k, m in enumerate(want_map):
        if want_status[k] != FB:
            assert [int(x) for x in o["node_of_pod"][off[k]:off[k + 1]]] == m


def test_spread_without_tables_flags_pod():
    """A shim without spread tables flags the pod (SR_POD_FB_TOPOLOGY_SPREAD)."""
    from spotplanner.model import encode_cluster
    p = spread(web("p"), zc())
    enc = encode_cluster(zone_nodes(), [p], spread_tables=False)
    assert enc.a["flags"][0] & capi.SR_POD_FB_TOPOLOGY_SPREAD
    enc = encode_cluster(zone_nodes(), [p])
    assert not enc.a["flags"][0] & capi.SR_POD_FB_TOPOLOGY_SPREAD
    q = spread(web("q"), zc(when="ScheduleAnyway"))
    assert not encode_cluster(zone_nodes(), [q], spread_tables=False).a["flags"][0] & capi.SR_POD_FB_TOPOLOGY_SPREAD


def rand_spread_scenario(seed):
    """Random zone / rack clusters with web / api pods in two namespaces,
    some terminating, and spread constraints on a share of the candidate
    pods (several per pod, shared keys, selectors of every operator, nil)."""
    r = random.Random(5150 + seed)
    nodes, spot_pods, cands = rand_scenario(6600 + seed, n_spot=6 + seed % 25, n_cand=12, max_pods=5,
                                            features=False)
    zones = ["z%d" % i for i in range(1 + seed % 4)]
    for i, n in enumerate(nodes):
        n.labels = dict(n.labels)
        n.labels[H] = n.name
        if r.random() < 0.85:
            n.labels[Z] = r.choice(zones + [""] if seed % 5 == 0 else zones)
        if r.random() < 0.5:
            n.labels["example.com/rack"] = "r%d" % r.randrange(3)
    apps = ["web", "api", "db"]
    for ps in spot_pods:
        for p in ps:
            p.namespace = r.choice(["default", "default", "other"])
            p.labels = {"app": r.choice(apps)} if r.random() < 0.9 else {}
            if r.random() < 0.1:
                p.deletion_age_s = 3.0

    def rand_sel():
        x = r.random()
        if x < 0.1:
            return None
        if x < 0.6:
            return LabelSelector(match_labels={"app": r.choice(apps)})
        op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
        vals = r.sample(apps, r.randint(1, 2)) if op in ("In", "NotIn") else []
        return LabelSelector(match_expressions=[LabelSelectorRequirement("app", op, vals)])

    for c in cands:
        for p in c:
            p.namespace = "default" if r.random() < 0.8 else "other"
            p.labels = {"app": r.choice(apps)}
            if r.random() < 0.5:
                p.topology_spread = [zc(skew=r.choice([1, 1, 2]), sel=rand_sel(),
                                        key=r.choice([Z, Z, H, "example.com/rack"]))
                                     for _ in range(r.choice([1, 1, 2]))]
                if r.random() < 0.2:
                    p.node_selector = {Z: r.choice(zones)}
    return nodes, spot_pods, cands


def rand_spread_replicas(seed):
    """Large candidates of Deployment replicas spread over zones (65-230 pods
    per candidate: 2-4 pod groups of the domain path), with a hostname
    constraint on some, over pools whose nodes already run replicas."""
    r = random.Random(8080 + seed)
    zones = ["z%d" % i for i in range(2 + seed % 4)]
    n_spot = 30 + seed % 40
    nodes = [Node("s%d" % i, cpu_milli=64000, memory=256 * 2 ** 30, pods=110,
                  labels={Z: r.choice(zones), H: "s%d" % i}) for i in range(n_spot)]
    apps = ["web", "api"]
    spot_pods = [[Pod("b%d_%d" % (i, j), namespace="default", containers=[Container(cpu_milli=r.choice([100, 250]))],
                      labels={"app": r.choice(apps)}) for j in range(r.randrange(4))] for i in range(n_spot)]
    cands = []
    for ci in range(3):
        n = 65 + r.randrange(166)
        app = r.choice(apps)
        cs = [zc(skew=r.choice([1, 2, 3]), sel=LabelSelector(match_labels={"app": app}))]
        if r.random() < 0.3:
            cs.append(zc(skew=r.choice([2, 4]), sel=LabelSelector(match_labels={"app": app}), key=H))
        cands.append([spread(Pod("c%d_%d" % (ci, j), namespace="default",
                                 containers=[Container(cpu_milli=r.choice([50, 100, 250, 500]))],
                                 labels={"app": app}), *cs) for j in range(n)])
    return nodes, spot_pods, cands


@pytest.mark.parametrize("seed", range(6))
def test_oracle_random_spread_runs(seed):
    """The random generator exercises planned, failing and fallback candidates."""
    nodes, spot_pods, cands = rand_spread_scenario(seed)
    _, o = run_oracle(nodes, spot_pods, cands)
    assert len(o["status"]) == len(cands)


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(cases()), ids=lambda c: c[0])
def test_gpu_spread_cases(checker, case):
    from spotplanner.rescheduler import plan_arrays
    _, nodes, spot_pods, cands, want_status, want_map = case
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, off, np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32))
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    assert [int(x) for x in p.status] == want_status
    _, o = run_oracle(nodes, spot_pods, cands)
    for k, m in enumerate(want_map):
        if want_status[k] != FB:
            assert list(p.node_of_pod[off[k]:off[k + 1]]) == list(o["node_of_pod"][off[k]:off[k + 1]])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_gpu_random_spread_clusters(checker, seed):
    """Every candidate the device plans equals the oracle; the fallback
    candidates are the oracle's."""
    from test_gpu_parity import run_scenario
    nodes, spot_pods, cands = rand_spread_scenario(seed)
    _, o, p = run_scenario(checker, nodes, spot_pods, cands)
    assert sum(int(s) != FB for s in p.status) >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_spread_replica_candidates(checker, seed):
    """65-230 replicas per candidate spread over zones (and hostnames): the
    domain path's pod groups against the oracle."""
    from test_gpu_parity import run_scenario
    nodes, spot_pods, cands = rand_spread_replicas(seed)
    _, o, p = run_scenario(checker, nodes, spot_pods, cands)
    assert sum(int(s) != FB for s in p.status) >= 1
