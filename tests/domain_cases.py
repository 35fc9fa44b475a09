"""Hand-derived drain plans for candidates whose pods interact through
inter-pod (anti-)affinity across nodes: the K2 domain path (antiaff.cpp,
kernels.hip k2_domain).  Each case is one candidate planned by canDrainNode
(rescheduler.go:357-370) on four spot nodes

    n1 zone=a   n2 zone=a   n3 zone=b   n4 (no zone)

in NodeInfoArray order, every node roomy enough that only inter-pod terms
decide.  Rules (InterPodAffinity.Filter, k8s v1.19.2
plugins/interpodaffinity/filtering.go; the candidate's placed pods count as
existing pods, rescheduler.go:366):
  anti  (1) an existing pod's term (key K) that selects the incoming pod
            refuses every node sharing the existing pod's node's K value;
        (2) an incoming pod's term (key K) refuses every node sharing the K
            value of a node hosting a pod the term selects;
        a node without K is never refused by a K term.
  aff   every term's key must be on the node, and per term a pod matching ALL
        the incoming pod's terms must run in the node's K domain; when no such
        pod runs on any node carrying one of the keys (empty pair map) and the
        pod matches its own terms, every node with the keys passes.
`want` is the expected node index per pod (-1 from the failing pod on), and
`fail` the failing pod index (-1: drainable)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

from spotplanner.model import Container, LabelSelector, Node, Pod, PodAffinityTerm

Z, H = "zone", "kubernetes.io/hostname"


@dataclass
class DomainCase:
    name: str
    why: str
    pods: List[Pod]
    want: List[int]
    fail: int = -1


def nodes() -> List[Node]:
    return [Node("n1", cpu_milli=8000, pods=110, labels={Z: "a", H: "n1"}),
            Node("n2", cpu_milli=8000, pods=110, labels={Z: "a", H: "n2"}),
            Node("n3", cpu_milli=8000, pods=110, labels={Z: "b", H: "n3"}),
            Node("n4", cpu_milli=8000, pods=110, labels={H: "n4"})]


def pod(name, app, anti=None, aff=None, on=None) -> Pod:
    p = Pod(name, labels={"app": app}, containers=[Container(cpu_milli=10)], pod_anti_affinity=anti,
            pod_affinity=aff)
    if on is not None:
        p.node_selector = {H: on}
    return p


def sel(app) -> LabelSelector:
    return LabelSelector({"app": app})


def term(key, app) -> PodAffinityTerm:
    return PodAffinityTerm(key, sel(app), [])


def cases() -> List[DomainCase]:
    return [
        DomainCase("anti_zone_both_have_the_term",
                   "w1 -> n1; w2: w1's term selects it (1) and its term selects w1 (2): zone a refused -> n3",
                   [pod("w1", "web", anti=[term(Z, "web")]), pod("w2", "web", anti=[term(Z, "web")])],
                   [0, 2]),
        DomainCase("anti_zone_three_pods_spill_to_the_zoneless_node",
                   "w1 -> n1 (zone a), w2 -> n3 (zone b), w3: zones a and b refused, n4 has no zone key -> n4",
                   [pod("w%d" % i, "web", anti=[term(Z, "web")]) for i in (1, 2, 3)],
                   [0, 2, 3]),
        DomainCase("anti_zone_incoming_term_only",
                   "d -> n1; w's term selects d in zone a (2) -> n3",
                   [pod("d", "db"), pod("w", "web", anti=[term(Z, "db")])],
                   [0, 2]),
        DomainCase("anti_zone_existing_term_only",
                   "w (term against db) -> n1; d is selected by w's term (1): zone a refused -> n3",
                   [pod("w", "web", anti=[term(Z, "db")]), pod("d", "db")],
                   [0, 2]),
        DomainCase("anti_zone_from_the_zoneless_node_refuses_nothing",
                   "w1 pinned to n4 (no zone): its zone term has no pair; w2 -> n1",
                   [pod("w1", "web", anti=[term(Z, "web")], on="n4"), pod("w2", "web", anti=[term(Z, "web")])],
                   [3, 0]),
        DomainCase("anti_zone_four_pods_two_on_the_zoneless_node",
                   "w1 -> n1, w2 -> n3, w3 -> n4 (no zone); w4: zones a and b refused, and on n4 neither w3's "
                   "zone term nor w4's own has a pair -> n4",
                   [pod("w%d" % i, "web", anti=[term(Z, "web")]) for i in (1, 2, 3, 4)],
                   [0, 2, 3, 3]),
        DomainCase("aff_zone_follows_an_earlier_pod",
                   "c pinned to n3 (zone b); w needs a cache pod in its zone: only zone b -> n3",
                   [pod("c", "cache", on="n3"), pod("w", "web", aff=[term(Z, "cache")])],
                   [2, 2]),
        DomainCase("aff_zone_first_node_of_the_domain",
                   "c pinned to n2 (zone a); w: zone a -> first node of zone a is n1",
                   [pod("c", "cache", on="n2"), pod("w", "web", aff=[term(Z, "cache")])],
                   [1, 0]),
        DomainCase("aff_hostname_follows_an_earlier_pod",
                   "c pinned to n2; w needs a cache pod on its own node -> n2",
                   [pod("c", "cache", on="n2"), pod("w", "web", aff=[term(H, "cache")])],
                   [1, 1]),
        DomainCase("aff_self_affine_group",
                   "w1: empty map, matches itself -> any node with zone: n1; w2: w1 in zone a -> n1",
                   [pod("w1", "web", aff=[term(Z, "web")]), pod("w2", "web", aff=[term(Z, "web")])],
                   [0, 0]),
        DomainCase("aff_self_affine_group_pinned",
                   "w1 pinned to n3: zone b; w2 follows into zone b -> n3",
                   [pod("w1", "web", aff=[term(Z, "web")], on="n3"), pod("w2", "web", aff=[term(Z, "web")])],
                   [2, 2]),
        DomainCase("aff_match_on_zoneless_node_keeps_the_map_empty",
                   "c pinned to n4 (no zone) adds no pair; w (not matching its own term) fails everywhere",
                   [pod("c", "cache", on="n4"), pod("w", "web", aff=[term(Z, "cache")])],
                   [3, -1], fail=1),
        DomainCase("aff_match_on_zoneless_node_self_exception",
                   "w1 pinned to n4 adds no pair; w2 matches its own term with an empty map -> n1",
                   [pod("w1", "web", on="n4"), pod("w2", "web", aff=[term(Z, "web")])],
                   [3, 0]),
        DomainCase("aff_two_terms_need_both_domains",
                   "c pinned to n2 matches both terms; w: zone a and host n2 -> n2",
                   [pod("c", "cache", on="n2"), pod("w", "web", aff=[term(Z, "cache"), term(H, "cache")])],
                   [1, 1]),
        DomainCase("aff_and_anti_together",
                   "c -> n1; w: cache in its zone (zone a) but no cache pod on its node -> n2",
                   [pod("c", "cache"), pod("w", "web", aff=[term(Z, "cache")], anti=[term(H, "cache")])],
                   [0, 1]),
        DomainCase("anti_zone_then_aff_zone",
                   "c -> n1; d (anti zone vs cache) -> n3; w (aff zone cache) -> n1",
                   [pod("c", "cache"), pod("d", "db", anti=[term(Z, "cache")]),
                    pod("w", "web", aff=[term(Z, "cache")])],
                   [0, 2, 0]),
    ]
