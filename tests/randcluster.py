"""Random small clusters exercising every encoded predicate and its edge cases
(zero requests, overcommitted nodes, pod-count limits, every taint effect,
every toleration shape, selectors, node affinity incl. invalid / empty terms
and matchFields, host ports incl. intra-candidate conflicts, fallback features).
Seeded; sized so the oracle finishes in milliseconds."""
from __future__ import annotations

import random

from spotplanner.model import (Container, ContainerPort, GiB, LabelSelector, LabelSelectorRequirement, MiB, Node,
                               NodeSelectorRequirement, NodeSelectorTerm, OwnerReference, Pod, PodAffinityTerm,
                               Taint, Toleration)

KEYS = ["zone", "type", "team", "disk", "gpu"]
GENS = ["1", "2", "10", "-3", "+4", "07", "x", ""]  # node label values (some do not parse as int64)
VALS = ["a", "b", "c", ""]
EFFECTS = ["NoSchedule", "NoExecute", "PreferNoSchedule"]


def rand_node(r: random.Random, name: str, features: bool) -> Node:
    labels = {"kubernetes.io/hostname": name}
    if features:
        for k in KEYS:
            if r.random() < 0.5:
                labels[k] = r.choice(VALS)
        if r.random() < 0.6:  # an integer-ish label for node-affinity Gt / Lt
            labels["gen"] = r.choice(GENS)
    taints = []
    if features and r.random() < 0.3:
        for _ in range(r.randint(1, 2)):
            taints.append(Taint(r.choice(["dedicated", "team", "x"]), r.choice(VALS), r.choice(EFFECTS)))
    scalar = {}
    if features and r.random() < 0.3:  # extended resources / hugepages (NodeResourcesFit's scalar loop)
        scalar["nvidia.com/gpu"] = r.choice([0, 1, 2, 4])
        if r.random() < 0.3:
            scalar["hugepages-2Mi"] = r.choice([0, 4 * MiB])
    return Node(name=name, cpu_milli=r.choice([500, 1000, 2000, 4000]), memory=r.choice([1, 2, 4]) * GiB,
                pods=r.choice([3, 5, 110]), ephemeral=r.choice([0, 10 * GiB]), labels=labels, taints=taints,
                unschedulable=features and r.random() < 0.1, scalar=scalar)


def rand_pod(r: random.Random, name: str, features: bool, fallback: bool = False) -> Pod:
    cpu = r.choice([0, 0, 50, 100, 250, 500, 1000])
    mem = r.choice([0, 64 * MiB, 256 * MiB, 1 * GiB])
    eph = r.choice([0, 0, 0, 1 * GiB])
    conts = [Container(cpu_milli=cpu, memory=mem, ephemeral=eph)]
    if r.random() < 0.2:
        conts.append(Container(cpu_milli=r.choice([0, 100]), memory=r.choice([0, 128 * MiB])))
    init = [Container(cpu_milli=r.choice([0, 800]), memory=r.choice([0, 2 * GiB]))] if r.random() < 0.15 else []
    overhead = Container(cpu_milli=50, memory=32 * MiB) if r.random() < 0.1 else None
    p = Pod(name=name, containers=conts, init_containers=init, overhead=overhead,
            owner_references=[OwnerReference("ReplicaSet")])
    if features:
        if r.random() < 0.12:  # scalar resources (sometimes also on an init container)
            p.containers[0].scalar = {"nvidia.com/gpu": r.choice([0, 1, 1, 2])}
            if r.random() < 0.2:
                p.containers[0].scalar["hugepages-2Mi"] = r.choice([2 * MiB, 4 * MiB])
            if init and r.random() < 0.5:
                init[0].scalar = {"nvidia.com/gpu": r.choice([1, 3])}
        if r.random() < 0.3:
            p.node_selector = {r.choice(KEYS): r.choice(VALS)}
        if r.random() < 0.25:
            terms = []
            for _ in range(r.randint(0, 3)):
                exprs = []
                for _ in range(r.randint(0, 2)):
                    op = r.choice(["In", "NotIn", "Exists", "DoesNotExist", "Bogus", "Gt", "Lt"])
                    key = r.choice(KEYS)
                    if op in ("Gt", "Lt"):  # integer compares on the "gen" label (some values invalid)
                        key = "gen" if r.random() < 0.8 else key
                        vals = [r.choice(["2", "-1", "07", "+3", "x"])]
                    else:
                        vals = [] if op in ("Exists", "DoesNotExist") else r.sample(VALS, r.randint(1, 2))
                    if r.random() < 0.05:  # invalid arity
                        vals = [] if vals else ["a"]
                    exprs.append(NodeSelectorRequirement(key, op, vals))
                fields = []
                if r.random() < 0.2:
                    fields.append(NodeSelectorRequirement(r.choice(["metadata.name", "metadata.uid"]),
                                                          r.choice(["In", "NotIn"]),
                                                          ["n%d" % r.randint(0, 5)]))
                terms.append(NodeSelectorTerm(exprs, fields))
            p.required_node_affinity = terms
        if r.random() < 0.35:
            for _ in range(r.randint(1, 2)):
                p.tolerations.append(Toleration(r.choice(["", "dedicated", "team", "x",
                                                          "node.kubernetes.io/unschedulable"]),
                                                r.choice(["", "Equal", "Exists", "Weird"]), r.choice(VALS),
                                                r.choice(["", "NoSchedule", "NoExecute", "PreferNoSchedule"])))
        if r.random() < 0.2:
            p.containers[0].ports.append(ContainerPort(host_port=r.choice([80, 443, 9100]),
                                                       protocol=r.choice(["TCP", "UDP", ""]),
                                                       host_ip=r.choice(["", "", "0.0.0.0", "10.0.0.1",
                                                                         "10.0.0.2"])))
    if fallback and r.random() < 0.1:
        kind = r.randint(0, 4)
        if kind == 0:
            p.has_pvc = True
        elif kind == 1:
            p.containers[0].scalar = {"nvidia.com/gpu": 1}
        elif kind == 2:
            p.required_pod_affinity = True
        elif kind == 3:
            p.containers[0].ports.append(ContainerPort(host_port=8080, host_ip="10.0.0.1"))
        else:
            p.required_node_affinity = [NodeSelectorTerm([NodeSelectorRequirement("zone", "Gt", ["1"])])]
    return p


HOST = "kubernetes.io/hostname"
APPS = ["web", "db", "cache"]
NAMESPACES = ["default", "default", "other"]


def rand_selector(r: random.Random, valid_only: bool = False):
    k = r.random() * (0.95 if valid_only else 1.0)
    if k < 0.55:
        return LabelSelector({"app": r.choice(APPS)})
    if k < 0.75:
        op = r.choice(["In", "NotIn", "Exists", "DoesNotExist"])
        vals = [] if op in ("Exists", "DoesNotExist") else r.sample(["fe", "be"], r.randint(1, 2))
        return LabelSelector({"app": r.choice(APPS)} if r.random() < 0.5 else {},
                             [LabelSelectorRequirement("tier", op, vals)])
    if k < 0.85:
        return LabelSelector()  # selects every pod of the namespaces
    if k < 0.95:
        return None  # nil: selects nothing
    return LabelSelector({}, [LabelSelectorRequirement("tier", "In", [])])  # invalid: fallback


def rand_anti(r: random.Random, p: Pod, rate: float, hostname_only: bool = False, shared_keys: bool = False,
              valid_only: bool = False):
    """Labels and namespace for every pod; required anti-affinity for some.
    Topology keys: the hostname (node-local) mostly, zone / team (shared or
    missing on some nodes) otherwise (always with shared_keys)."""
    p.namespace = r.choice(NAMESPACES)
    p.labels = {"app": r.choice(APPS)}
    if r.random() < 0.5:
        p.labels["tier"] = r.choice(["fe", "be"])
    if r.random() < rate:
        p.pod_anti_affinity = []
        for _ in range(r.randint(1, 2)):
            tk = HOST if hostname_only or (not shared_keys and r.random() < 0.7) else r.choice(["zone", "team"])
            ns = [] if r.random() < 0.7 else r.sample(["default", "other"], r.randint(1, 2))
            p.pod_anti_affinity.append(PodAffinityTerm(tk, rand_selector(r, hostname_only or valid_only), ns))


def rand_aff(r: random.Random, p: Pod, rate: float, shared_keys: bool = False):
    """Required pod affinity for some pods: one or two terms on the hostname or
    a shared key (zone / team), valid selectors mostly on the app label."""
    if r.random() < rate:
        p.pod_affinity = []
        for _ in range(r.randint(1, 2)):
            tk = r.choice(["zone", "zone", "team"] if shared_keys else [HOST, "zone", "zone", "team"])
            ns = [] if r.random() < 0.8 else r.sample(["default", "other"], r.randint(1, 2))
            p.pod_affinity.append(PodAffinityTerm(tk, rand_selector(r, True), ns))


def rand_scenario(seed: int, n_spot: int = 12, n_cand: int = 8, max_pods: int = 8, features: bool = True,
                  fallback: bool = False, anti: float = 0.0, hostname_only: bool = False, aff: float = 0.0,
                  shared_keys: bool = False, valid_selectors: bool = False):
    """Returns (spot_nodes, spot_pods, candidates) with candidates a list of pod lists.
    anti > 0: pods carry namespaces / labels and that share required pod anti-affinity
    (hostname_only: every term on kubernetes.io/hostname with a valid selector).
    aff > 0: that share of the pods (spot and candidate) carries required pod affinity.
    shared_keys: every inter-pod term on zone / team (shared domains).
    valid_selectors: no selector that LabelSelectorAsSelector rejects (those send candidates to fallback)."""
    r = random.Random(seed)
    nodes = [rand_node(r, "n%d" % i, features) for i in range(n_spot)]
    spot_pods = []
    for i, n in enumerate(nodes):
        ps = [rand_pod(r, "s%d_%d" % (i, k), features) for k in range(r.randint(0, 4))]
        if r.random() < 0.15:  # overcommitted node
            ps.append(Pod(name="big%d" % i, containers=[Container(cpu_milli=n.cpu_milli + 100)]))
        spot_pods.append(ps)
    cands = [[rand_pod(r, "c%d_%d" % (c, k), features, fallback) for k in range(r.randint(0, max_pods))]
             for c in range(n_cand)]
    if anti > 0 or aff > 0:
        for ps in spot_pods + cands:
            for p in ps:
                rand_anti(r, p, anti, hostname_only, shared_keys, valid_selectors)
    if aff > 0:
        for ps in spot_pods + cands:
            for p in ps:
                rand_aff(r, p, aff, shared_keys)
    return nodes, spot_pods, cands


def term_selects(owner: Pod, t: PodAffinityTerm, target: Pod) -> bool:
    """Namespace + label selector of an anti-affinity term (test-side restatement)."""
    if target.namespace not in (t.namespaces or [owner.namespace]):
        return False
    sel = t.label_selector
    if sel is None:
        return False
    if any(target.labels.get(k) != v for k, v in sel.match_labels.items()):
        return False
    for e in sel.match_expressions:
        v = target.labels.get(e.key)
        ok = {"In": v is not None and v in e.values, "NotIn": v is None or v not in e.values,
              "Exists": v is not None, "DoesNotExist": v is None}[e.operator]
        if not ok:
            return False
    return True


def anti_interacts_off_node(nodes, pods) -> bool:
    """Two pods of one candidate interact through an anti-affinity term whose
    topology key is not node-local on the spot pool (some node lacks it or two
    nodes share a value): the product plans such a candidate on K2's domain
    path (antiaff.cpp, kernels.hip k2_domain)."""
    def node_local(tk):
        vals = [n.labels.get(tk) for n in nodes]
        return all(v is not None for v in vals) and len(set(vals)) == len(vals)
    for i, a in enumerate(pods):
        for t in a.pod_anti_affinity or []:
            if node_local(t.topology_key):
                continue
            if any(j != i and term_selects(a, t, b) for j, b in enumerate(pods)):
                return True
    return False


def aff_interacts(pods) -> bool:
    """An earlier pod of the candidate matches every required affinity term of a
    later one: that pod's allowed domains change while the candidate is
    planned; the product plans such a candidate on K2's domain path."""
    for k, p in enumerate(pods):
        terms = p.pod_affinity or []
        if terms and any(all(term_selects(p, t, q) for t in terms) for q in pods[:k]):
            return True
    return False
