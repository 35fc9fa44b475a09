"""Hand-derived known-answer cases for the scheduler filters behind
CheckPredicates (call site rescheduler.go:344).  The reference's own tests pin
only CPU fit (rescheduler_test.go:40-151); every other filter rule comes from
the pinned upstream modules, which are not in the reference tree:

  k8s.io/kubernetes v1.19.2  pkg/scheduler/framework/plugins/
      noderesources/fit.go          fitsRequest, computePodResourceRequest
      tainttoleration/taint_toleration.go  Filter (NoSchedule / NoExecute only)
      nodeunschedulable/node_unschedulable.go  Filter
      nodeaffinity/node_affinity.go -> helper/node_affinity.go
                                    PodMatchesNodeSelectorAndAffinityTerms
      nodeports/node_ports.go       fitsPorts -> framework/types.go
                                    HostPortInfo.CheckConflict
      interpodaffinity/filtering.go satisfyPodAffinity, satisfyPodAntiAffinity,
                                    satisfyExistingPodsAntiAffinity
  k8s.io/api v0.19.2 core/v1/toleration.go  Toleration.ToleratesTaint
  k8s.io/api v0.19.2 core/v1/helper MatchNodeSelectorTerms

Each case gives one pod, spot nodes (with the pods already on them) and the
answer of the filter chain for the pod on each node, derived by hand from the
rule quoted in `rule`.  tests/test_known_answer.py checks every answer on the
oracle (CPU) and, one node at a time through sr_find_spot_nodes, on the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

from spotplanner.model import (Container, ContainerPort, GiB, LabelSelector, LabelSelectorRequirement, MiB, Node,
                               NodeSelectorRequirement, NodeSelectorTerm, Pod, PodAffinityTerm, Taint, Toleration)


@dataclass
class Case:
    name: str
    rule: str
    pod: Pod
    nodes: List[Node]
    base: List[List[Pod]]
    fits: List[bool]
    tags: List[str] = field(default_factory=list)


def P(name="p", cpu=100, mem=0, eph=0, **kw) -> Pod:
    return Pod(name, containers=[Container(cpu_milli=cpu, memory=mem, ephemeral=eph)], **kw)


def N(name, cpu=4000, mem=8 * GiB, pods=110, eph=0, **kw) -> Node:
    return Node(name, cpu_milli=cpu, memory=mem, pods=pods, ephemeral=eph, **kw)


def used(cpu=0, mem=0, eph=0, name="used") -> Pod:
    return P(name, cpu=cpu, mem=mem, eph=eph)


def _resources():
    fit = "fitsRequest: fail iff allocatable < podRequest + nodeInfo.Requested (per resource)"
    yield Case("memory_exact_fit", fit, P(cpu=0, mem=512 * MiB),
               [N("a", mem=2 * GiB), N("b", mem=2 * GiB)], [[used(mem=1536 * MiB)], [used(mem=1537 * MiB)]],
               [True, False])
    yield Case("ephemeral_exact_fit", fit, P(cpu=0, eph=1 * GiB),
               [N("a", eph=10 * GiB), N("b", eph=10 * GiB), N("c", eph=0)],
               [[used(eph=9 * GiB)], [used(eph=9 * GiB + 1)], []], [True, False, False])
    yield Case("cpu_exact_fit", fit, P(cpu=700), [N("a", cpu=1000), N("b", cpu=1000)],
               [[used(cpu=300)], [used(cpu=301)]], [True, False])
    yield Case("pod_count", "fitsRequest: len(nodeInfo.Pods)+1 > allowedPodNumber fails, before the zero-request "
               "shortcut", P(cpu=0), [N("a", pods=2), N("b", pods=2), N("c", pods=0)],
               [[used(), used()], [used()], []], [False, True, False])
    yield Case("zero_request_skips_resources", "fitsRequest: an all-zero request returns after the pod-count check",
               P(cpu=0, mem=0, eph=0), [N("a", cpu=1000, mem=1 * GiB)], [[used(cpu=5000, mem=4 * GiB)]], [True])
    yield Case("nonzero_request_on_overcommitted_node", fit + " (memory checked for a cpu-only pod too)",
               P(cpu=1, mem=0), [N("a", cpu=1000, mem=1 * GiB), N("b", cpu=1000, mem=1 * GiB)],
               [[used(mem=1 * GiB + 1)], [used(mem=1 * GiB)]], [False, True])
    ic = Pod("p", containers=[Container(cpu_milli=100, memory=64 * MiB)],
             init_containers=[Container(cpu_milli=800), Container(cpu_milli=50, memory=1 * GiB)])
    yield Case("init_container_max", "computePodResourceRequest: max(sum(containers), each init container) per "
               "resource: cpu 800, memory 1Gi", ic,
               [N("a", cpu=1000, mem=8 * GiB), N("b", cpu=1000, mem=8 * GiB), N("c", cpu=1000, mem=2 * GiB)],
               [[used(cpu=201)], [used(cpu=200)], [used(mem=1 * GiB + 1)]], [False, True, False])
    oh = Pod("p", containers=[Container(cpu_milli=400), Container(cpu_milli=0, memory=0)],
             overhead=Container(cpu_milli=200, memory=100 * MiB))
    yield Case("pod_overhead", "computePodResourceRequest: + Spec.Overhead: cpu 600, memory 100Mi", oh,
               [N("a", cpu=1000), N("b", cpu=1000), N("c", cpu=1000, mem=1 * GiB)],
               [[used(cpu=401)], [used(cpu=400)], [used(mem=1 * GiB - 100 * MiB + 1)]], [False, True, False])
    yield Case("sum_of_containers", "computePodResourceRequest: regular containers add up",
               Pod("p", containers=[Container(cpu_milli=300), Container(cpu_milli=300)]),
               [N("a", cpu=1000), N("b", cpu=1000)], [[used(cpu=401)], [used(cpu=400)]], [False, True])


def _scalar():
    sr = ("fitsRequest: for each scalar resource the pod lists, Allocatable.ScalarResources[name] (0 when the node "
          "has none) < request + Requested.ScalarResources[name] fails")
    G = "nvidia.com/gpu"

    def gp(name="p", gpu=1, cpu=100, **kw):
        return Pod(name, containers=[Container(cpu_milli=cpu, scalar={G: gpu} if gpu is not None else {})], **kw)
    yield Case("scalar_request_needs_the_resource", sr, gp(gpu=1),
               [N("a", scalar={G: 2}), N("b"), N("c", scalar={G: 1}), N("d", scalar={G: 2})],
               [[], [], [gp("u", gpu=1)], [gp("u", gpu=1)]], [True, False, False, True])
    yield Case("scalar_zero_request_listed", sr + " (0 < 0 + 0 is false: a listed zero fits anywhere)", gp(gpu=0),
               [N("a"), N("b", scalar={G: 1})], [[], [gp("u", gpu=1)]], [True, True])
    hp = "hugepages-2Mi"
    yield Case("hugepages_exact_fit", sr,
               Pod("p", containers=[Container(cpu_milli=10, scalar={hp: 2 * MiB})]),
               [N("a", scalar={hp: 4 * MiB}), N("b", scalar={hp: 4 * MiB})],
               [[Pod("u", containers=[Container(cpu_milli=10, scalar={hp: 2 * MiB})])],
                [Pod("u", containers=[Container(cpu_milli=10, scalar={hp: 2 * MiB + 1})])]], [True, False])
    ini = Pod("p", containers=[Container(cpu_milli=100, scalar={G: 1})],
              init_containers=[Container(cpu_milli=0, scalar={G: 3})])
    yield Case("scalar_init_container_max", sr + "; computePodResourceRequest: max(sum, each init container) = 3",
               ini, [N("a", scalar={G: 2}), N("b", scalar={G: 3})], [[], []], [False, True])
    oh = Pod("p", containers=[Container(cpu_milli=100, scalar={G: 1})], overhead=Container(scalar={G: 1}))
    yield Case("scalar_overhead", sr + "; + Spec.Overhead", oh, [N("a", scalar={G: 1}), N("b", scalar={G: 2})],
               [[], []], [False, True])
    yield Case("scalar_and_cpu_both_checked", sr + "; cpu is checked as well", gp(gpu=1, cpu=900),
               [N("a", cpu=1000, scalar={G: 1}), N("b", cpu=1000, scalar={G: 1})],
               [[used(cpu=200)], [used(cpu=100)]], [False, True])
    acc = ("NodeInfo.AddPod (calculateResource, k8s v1.19.2 framework/v1alpha1/types.go): Requested adds the "
           "regular containers and Overhead, not init containers")
    base_ini = Pod("u", containers=[Container(cpu_milli=100, scalar={G: 1})],
                   init_containers=[Container(cpu_milli=800, scalar={G: 2})])
    yield Case("node_accounting_skips_init_containers", acc + " (parity unpinned: the module is not vendored)",
               gp(gpu=1, cpu=500), [N("a", cpu=1000, scalar={G: 2})], [[base_ini]], [True])


def _taints():
    flt = "TaintToleration.Filter: FindMatchingUntoleratedTaint over NoSchedule / NoExecute taints"
    tt = "Toleration.ToleratesTaint: effect empty or equal, key empty or equal, Exists or Equal with equal value"
    yield Case("no_schedule_and_no_execute_filter", flt, P(),
               [N("a", taints=[Taint("k", "v", "NoSchedule")]), N("b", taints=[Taint("k", "v", "NoExecute")]),
                N("c")], [[], [], []], [False, False, True])
    yield Case("prefer_no_schedule_never_filters", flt, P(),
               [N("a", taints=[Taint("k", "v", "PreferNoSchedule")])], [[]], [True])
    yield Case("empty_effect_tolerates_every_effect", tt, P(tolerations=[Toleration("k", "Equal", "v", "")]),
               [N("a", taints=[Taint("k", "v", "NoSchedule")]), N("b", taints=[Taint("k", "v", "NoExecute")]),
                N("c", taints=[Taint("k", "w", "NoSchedule")])], [[], [], []], [True, True, False])
    yield Case("effect_must_match", tt, P(tolerations=[Toleration("k", "Exists", "", "NoSchedule")]),
               [N("a", taints=[Taint("k", "v", "NoExecute")]), N("b", taints=[Taint("k", "v", "NoSchedule")])],
               [[], []], [False, True])
    yield Case("empty_key_exists_tolerates_everything", tt, P(tolerations=[Toleration("", "Exists")]),
               [N("a", taints=[Taint("k", "v", "NoSchedule"), Taint("j", "", "NoExecute")])], [[]], [True])
    yield Case("empty_key_equal_matches_empty_values_only", tt, P(tolerations=[Toleration("", "Equal", "")]),
               [N("a", taints=[Taint("k", "", "NoSchedule")]), N("b", taints=[Taint("k", "v", "NoSchedule")])],
               [[], []], [True, False])
    yield Case("equal_with_empty_value", tt + " (operator \"\" is Equal)", P(tolerations=[Toleration("k", "", "")]),
               [N("a", taints=[Taint("k", "", "NoSchedule")]), N("b", taints=[Taint("k", "v", "NoSchedule")])],
               [[], []], [True, False])
    yield Case("unknown_operator_tolerates_nothing", tt, P(tolerations=[Toleration("k", "Weird", "v")]),
               [N("a", taints=[Taint("k", "v", "NoSchedule")])], [[]], [False])
    yield Case("every_taint_must_be_tolerated", flt,
               P(tolerations=[Toleration("k", "Exists", "", "NoSchedule")]),
               [N("a", taints=[Taint("k", "v", "NoSchedule"), Taint("j", "v", "NoSchedule")]),
                N("b", taints=[Taint("k", "v", "NoSchedule"), Taint("j", "v", "PreferNoSchedule")])],
               [[], []], [False, True])


def _unschedulable():
    r = ("NodeUnschedulable.Filter: Spec.Unschedulable and the pod does not tolerate "
         "node.kubernetes.io/unschedulable:NoSchedule")
    k = "node.kubernetes.io/unschedulable"
    yield Case("unschedulable_without_toleration", r, P(), [N("a", unschedulable=True), N("b")], [[], []],
               [False, True])
    yield Case("unschedulable_tolerated_exists", r, P(tolerations=[Toleration(k, "Exists", "", "NoSchedule")]),
               [N("a", unschedulable=True)], [[]], [True])
    yield Case("unschedulable_tolerated_equal_empty_value", r, P(tolerations=[Toleration(k, "Equal", "")]),
               [N("a", unschedulable=True)], [[]], [True])
    yield Case("unschedulable_tolerated_by_wildcard", r, P(tolerations=[Toleration("", "Exists")]),
               [N("a", unschedulable=True)], [[]], [True])
    yield Case("unschedulable_wrong_effect", r, P(tolerations=[Toleration(k, "Exists", "", "NoExecute")]),
               [N("a", unschedulable=True)], [[]], [False])


def _affinity():
    sel = "PodMatchesNodeSelectorAndAffinityTerms: every nodeSelector pair must equal the node label"
    mt = ("MatchNodeSelectorTerms: terms ORed; an empty term or a term that fails to build selects nothing; "
          "requirements ANDed")
    z = lambda v: {"zone": v}  # noqa: E731
    nodes3 = [N("a", labels=z("a")), N("b", labels=z("b")), N("c", labels={})]

    def aff(*terms):
        return P(required_node_affinity=list(terms))

    def T(*exprs, fields=()):
        return NodeSelectorTerm([NodeSelectorRequirement(*e) for e in exprs],
                                [NodeSelectorRequirement(*f) for f in fields])

    yield Case("node_selector", sel, P(node_selector={"zone": "a"}), nodes3, [[], [], []], [True, False, False])
    yield Case("in", mt, aff(T(("zone", "In", ["b", "x"]))), nodes3, [[], [], []], [False, True, False])
    yield Case("not_in_missing_key", mt + "; NotIn holds when the key is absent", aff(T(("zone", "NotIn", ["a"]))),
               nodes3, [[], [], []], [False, True, True])
    yield Case("does_not_exist_missing_key", mt, aff(T(("zone", "DoesNotExist", []))), nodes3, [[], [], []],
               [False, False, True])
    yield Case("exists", mt, aff(T(("zone", "Exists", []))), nodes3, [[], [], []], [True, True, False])
    yield Case("empty_term_list_matches_nothing", mt, aff(), nodes3, [[], [], []], [False, False, False])
    yield Case("empty_term_matches_nothing", mt, aff(T()), nodes3, [[], [], []], [False, False, False])
    yield Case("empty_term_or_valid_term", mt, aff(T(), T(("zone", "In", ["a"]))), nodes3, [[], [], []],
               [True, False, False])
    yield Case("terms_ored", mt, aff(T(("zone", "In", ["a"])), T(("zone", "DoesNotExist", []))), nodes3,
               [[], [], []], [True, False, True])
    yield Case("requirements_anded", mt,
               aff(T(("zone", "Exists", []), ("disk", "In", ["ssd"]))),
               [N("a", labels={"zone": "a", "disk": "ssd"}), N("b", labels={"zone": "b"}),
                N("c", labels={"disk": "ssd"})], [[], [], []], [True, False, False])
    yield Case("node_selector_and_terms", sel + "; then the required terms",
               P(node_selector={"zone": "a"}, required_node_affinity=[T(("disk", "In", ["ssd"]))]),
               [N("a", labels={"zone": "a"}), N("b", labels={"zone": "b", "disk": "ssd"}),
                N("c", labels={"zone": "a", "disk": "ssd"})], [[], [], []], [False, False, True])
    yield Case("invalid_requirement_fails_its_term", mt + "; In without values fails NewRequirement",
               aff(T(("zone", "In", [])), T(("zone", "In", ["b"]))), nodes3, [[], [], []], [False, True, False])
    yield Case("match_fields_name_in", mt + "; fields.Set{metadata.name: node.Name}",
               aff(T(fields=[("metadata.name", "In", ["b"])])), nodes3, [[], [], []], [False, True, False])
    yield Case("match_fields_name_not_in", mt, aff(T(fields=[("metadata.name", "NotIn", ["b"])])), nodes3,
               [[], [], []], [True, False, True])
    yield Case("match_fields_two_values_invalid", mt + "; In on a field needs exactly one value",
               aff(T(fields=[("metadata.name", "In", ["a", "b"])])), nodes3, [[], [], []], [False, False, False])
    yield Case("match_fields_and_expressions", mt,
               aff(T(("zone", "Exists", []), fields=[("metadata.name", "NotIn", ["a"])])), nodes3, [[], [], []],
               [False, True, False])
    # Gt / Lt: Requirement.Matches parses the node's value with strconv.ParseInt(v, 10, 64) (a value that
    # does not parse, or a missing key, fails); NewRequirement needs exactly one value that parses
    gt = mt + "; Gt/Lt: ParseInt of the node's label value against the single integer value"
    gen = [N("g1", labels={"gen": "7"}), N("g2", labels={"gen": "+12"}), N("g3", labels={"gen": "-3"}),
           N("g4", labels={"gen": "x9"}), N("g5", labels={})]
    none = [[] for _ in gen]
    yield Case("gt_integer_labels", gt, aff(T(("gen", "Gt", ["6"]))), gen, none, [True, True, False, False, False])
    yield Case("lt_integer_labels", gt, aff(T(("gen", "Lt", ["7"]))), gen, none, [False, False, True, False, False])
    yield Case("gt_is_strict", gt, aff(T(("gen", "Gt", ["7"]))), gen, none, [False, True, False, False, False])
    yield Case("lt_value_with_leading_zero", gt + "; ParseInt(\"012\") = 12", aff(T(("gen", "Lt", ["012"]))), gen,
               none, [True, False, True, False, False])
    # labels.NewRequirement runs validateLabelValue (validation.IsValidLabelValue: <= 63 characters of
    # ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9], or empty) on every value after the operator checks, and
    # validateLabelKey (validation.IsQualifiedName) on the key: a requirement that fails makes
    # NodeSelectorRequirementsAsSelector return an error, and MatchNodeSelectorTerms skips the term
    lv = mt + "; NewRequirement: validateLabelKey / validateLabelValue on the key and every value"
    yield Case("gt_signed_value_fails_label_validation", lv + " (\"-3\" starts with '-')",
               aff(T(("gen", "Gt", ["-3"]))), gen, none, [False, False, False, False, False])
    yield Case("lt_plus_sign_fails_label_validation", lv + " (\"+012\" starts with '+')",
               aff(T(("gen", "Lt", ["+012"]))), gen, none, [False, False, False, False, False])
    yield Case("not_in_invalid_value_fails_its_term", lv + "; NotIn [\"-x\"] would hold on every node",
               aff(T(("zone", "NotIn", ["-x"]))), nodes3, [[], [], []], [False, False, False])
    yield Case("not_in_invalid_value_other_term_holds", lv, aff(T(("zone", "NotIn", ["b", "a."])),
                                                               T(("zone", "In", ["b"]))), nodes3, [[], [], []],
               [False, True, False])
    yield Case("in_64_character_value_fails_its_term", lv + " (63 characters at most)",
               aff(T(("zone", "In", ["a", "v" * 64]))), nodes3 + [N("d", labels=z("v" * 64))], [[], [], [], []],
               [False, False, False, False])
    yield Case("in_63_character_value_is_valid", lv,
               aff(T(("zone", "In", ["a", "v" * 63]))), nodes3 + [N("d", labels=z("v" * 63))], [[], [], [], []],
               [True, False, False, True])
    yield Case("exists_invalid_key_fails_its_term", lv + " (\"bad key\" is not a qualified name)",
               aff(T(("bad key", "DoesNotExist", [])), T(("zone", "Exists", []))), nodes3, [[], [], []],
               [True, True, False])
    yield Case("prefixed_key_is_valid", lv + " (DNS-1123 subdomain prefix)",
               aff(T(("example.com/zone", "DoesNotExist", []))), nodes3, [[], [], []], [True, True, True])
    yield Case("uppercase_prefix_fails_key_validation", lv + " (the prefix is lower case)",
               aff(T(("Example.com/zone", "DoesNotExist", []))), nodes3, [[], [], []], [False, False, False])
    yield Case("empty_value_is_valid", lv + " (an empty label value is valid)", aff(T(("zone", "NotIn", [""]))),
               nodes3, [[], [], []], [True, True, True])
    yield Case("node_selector_values_not_validated", sel + "; labels.SelectorFromSet does not validate in v0.19",
               P(node_selector={"zone": "-x"}), [N("a", labels=z("-x")), N("b", labels=z("a"))], [[], []],
               [True, False])
    yield Case("gt_non_integer_value_fails_its_term", gt + "; a value that does not parse fails NewRequirement",
               aff(T(("gen", "Gt", ["six"])), T(("gen", "Lt", ["0"]))), gen, none,
               [False, False, True, False, False])
    yield Case("gt_two_values_fails_its_term", gt + "; exactly one value", aff(T(("gen", "Gt", ["1", "2"]))), gen,
               none, [False, False, False, False, False])
    yield Case("gt_anded_with_in", gt, aff(T(("gen", "Gt", ["0"]), ("gen", "NotIn", ["7"]))), gen, none,
               [False, True, False, False, False])


def _ports():
    r = ("HostPortInfo.CheckConflict: port <= 0 never conflicts; 0.0.0.0 (or \"\") conflicts with every IP of the "
         "same (protocol, port); a specific IP with 0.0.0.0 and itself")

    def hp(name, port, ip="", proto="TCP"):
        return Pod(name, containers=[Container(cpu_milli=10, ports=[ContainerPort(port, protocol=proto,
                                                                                   host_ip=ip)])])
    nodes = [N("a"), N("b"), N("c"), N("d"), N("e")]
    base = [[hp("x", 80, "10.0.0.1")], [hp("y", 80)], [hp("z", 80, "10.0.0.2")], [hp("u", 80, proto="UDP")],
            [hp("v", 8080)]]
    yield Case("wildcard_against_specific", r, hp("p", 80), nodes, base, [False, False, False, True, True])
    yield Case("specific_against_wildcard_and_itself", r, hp("p", 80, "10.0.0.1"), nodes, base,
               [False, False, True, True, True])
    yield Case("explicit_0000_is_wildcard", r, hp("p", 80, "0.0.0.0"), nodes, base,
               [False, False, False, True, True])
    yield Case("protocol_separates", r, hp("p", 80, proto="UDP"), nodes, base, [True, True, True, False, True])
    yield Case("zero_host_port_ignored", r, hp("p", 0), nodes, base, [True, True, True, True, True])


def _interpod():
    aff = ("satisfyPodAffinity: the node carries every term's topology key and, per term, an existing pod that "
           "matches ALL the pod's terms runs in the node's domain; else, when no such pod runs on a node with any of "
           "the keys and the pod matches its own terms, every node carrying the keys")
    anti = ("satisfyPodAntiAffinity / satisfyExistingPodsAntiAffinity: no pod selected by the pod's term (or whose "
            "term selects the pod) in the node's domain of the term's key; a node without the key passes")
    Z, H = "zone", "kubernetes.io/hostname"

    def nodes():
        return [N("n1", labels={Z: "a", H: "n1"}), N("n2", labels={Z: "a", H: "n2"}),
                N("n3", labels={Z: "b", H: "n3"}), N("n4", labels={H: "n4"})]

    def pod(name, labels, ns="default", affinity=None, anti_affinity=None):
        return Pod(name, namespace=ns, labels=dict(labels), containers=[Container(cpu_milli=10)],
                   pod_affinity=affinity, pod_anti_affinity=anti_affinity)

    def term(key, sel, namespaces=()):
        return PodAffinityTerm(key, sel, list(namespaces))

    cache = LabelSelector({"app": "cache"})
    web = LabelSelector({"app": "web"})
    yield Case("aff_zone_existing_pod", aff, pod("w", {"app": "web"}, affinity=[term(Z, cache)]), nodes(),
               [[], [], [pod("c", {"app": "cache"})], []], [False, False, True, False])
    yield Case("aff_zone_whole_domain", aff, pod("w", {"app": "web"}, affinity=[term(Z, cache)]), nodes(),
               [[pod("c", {"app": "cache"})], [], [], []], [True, True, False, False])
    yield Case("aff_hostname", aff, pod("w", {"app": "web"}, affinity=[term(H, cache)]), nodes(),
               [[], [pod("c", {"app": "cache"})], [], []], [False, True, False, False])
    yield Case("aff_first_pod_of_self_affine_group", aff, pod("w", {"app": "web"}, affinity=[term(Z, web)]),
               nodes(), [[], [], [], []], [True, True, True, False])
    yield Case("aff_nothing_matches", aff, pod("w", {"app": "web"}, affinity=[term(Z, cache)]), nodes(),
               [[pod("x", {"app": "db"})], [], [], []], [False, False, False, False])
    yield Case("aff_match_on_node_without_key_not_self", aff, pod("w", {"app": "web"}, affinity=[term(Z, cache)]),
               nodes(), [[], [], [], [pod("c", {"app": "cache"})]], [False, False, False, False])
    yield Case("aff_match_on_node_without_key_self", aff + " (the pair map stays empty)",
               pod("w", {"app": "web"}, affinity=[term(Z, web)]), nodes(),
               [[], [], [], [pod("w0", {"app": "web"})]], [True, True, True, False])
    yield Case("aff_self_affine_group_already_placed", aff, pod("w", {"app": "web"}, affinity=[term(Z, web)]),
               nodes(), [[], [], [pod("w0", {"app": "web"})], []], [False, False, True, False])
    two = [term(Z, cache), term(H, LabelSelector({"tier": "be"}))]
    yield Case("aff_existing_pod_must_match_all_terms", aff, pod("w", {"app": "web"}, affinity=two), nodes(),
               [[pod("x", {"app": "cache", "tier": "be"})], [], [pod("y", {"app": "cache"})], []],
               [True, False, False, False])
    yield Case("aff_term_namespace_defaults_to_pod", aff, pod("w", {"app": "web"}, affinity=[term(Z, cache)]),
               nodes(), [[], [], [pod("c", {"app": "cache"}, ns="other")], []], [False, False, False, False])
    yield Case("aff_term_namespaces_listed", aff,
               pod("w", {"app": "web"}, affinity=[term(Z, cache, ["other", "default"])]), nodes(),
               [[], [], [pod("c", {"app": "cache"}, ns="other")], []], [False, False, True, False])
    yield Case("aff_nil_selector_matches_nothing", aff, pod("w", {"app": "web"}, affinity=[term(Z, None)]),
               nodes(), [[pod("c", {"app": "cache"})], [], [], []], [False, False, False, False])
    yield Case("aff_match_expressions", aff,
               pod("w", {"app": "web"}, affinity=[term(Z, LabelSelector({}, [LabelSelectorRequirement(
                   "app", "In", ["cache", "db"])]))]), nodes(),
               [[], [], [pod("d", {"app": "db"})], []], [False, False, True, False])
    yield Case("anti_zone_existing_pod_refuses", anti, pod("w", {"app": "web"}), nodes(),
               [[pod("d", {"app": "db"}, anti_affinity=[term(Z, web)])], [], [], []], [False, False, True, True])
    yield Case("anti_zone_incoming_pod_refuses", anti,
               pod("w", {"app": "web"}, anti_affinity=[term(Z, LabelSelector({"app": "db"}))]), nodes(),
               [[], [], [pod("d", {"app": "db"})], []], [True, True, False, True])
    yield Case("aff_and_anti_together", aff + "; " + anti,
               pod("w", {"app": "web"}, affinity=[term(Z, cache)], anti_affinity=[term(H, cache)]), nodes(),
               [[pod("c", {"app": "cache"})], [], [], []], [False, True, False, False])


def cases() -> List[Case]:
    out = []
    for gen in (_resources, _scalar, _taints, _unschedulable, _affinity, _ports, _interpod):
        out.extend(gen())
    names = [c.name for c in out]
    assert len(names) == len(set(names))
    return out
