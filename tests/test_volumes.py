"""The volume filters behind CheckPredicates (rescheduler.go:344; k8s v1.19.2
plugins volumebinding, volumezone, volumerestrictions, nodevolumelimits --
upstream, not vendored in the reference: parity unpinned beyond the
hand-derived answers here).  The shim resolves every claim through the
scheduler's listers (spotplanner.model.resolve_volumes); the planner encodes:

- VolumeBinding PreFilter failing (a missing claim or volume, an unbound claim
  with Immediate binding): the pod fits no node;
- VolumeBinding Filter on bound claims (volumeutil.CheckNodeAffinity =
  MatchNodeSelectorTerms(PV terms, node labels, nil fields)): requirement
  atoms, terms ORed, a matchFields requirement reading "";
- VolumeZone (a node without any of the four zone / region labels passes, else
  the node's value of each PV zone label's key, "" when absent, must be one of
  LabelZonesToSet's values): REQ_ZONE requirement atoms;
- VolumeRestrictions (isVolumeConflict: the same GCE PD / ISCSI IQN unless both
  mounts are read-only, the same EBS VolumeID always): pseudo host ports, state
  bits inside a candidate;
- the volume limits (per limit key, the node's unique attachable volumes plus
  the pod's new ones against the node's limit; non-CSI keys default to 39 EBS /
  16 GCE PD / 16 Azure Disk unless Allocatable lists the key, CSI keys come
  from CSINode): scalar-like capacity per key, running counts inside a
  candidate (extension records).

The reference path takes: claims with WaitForFirstConsumer binding still
unbound, RBD volumes, a pod whose attachable volume a spot node already holds,
two pods of one candidate sharing one, more than two shared limit keys / scalar
names per candidate.  Checked on the oracle (CPU) and the GPU (C-ABI)."""
import random

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import oracle_plan
from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import (Container, Node, NodeSelectorRequirement, NodeSelectorTerm, PersistentVolume,
                               PersistentVolumeClaim, Pod, Volume, VolumeWorld)

OK, FB = capi.SR_CAND_OK, capi.SR_CAND_FALLBACK
TZ, TR = "topology.kubernetes.io/zone", "topology.kubernetes.io/region"
BZ = "failure-domain.beta.kubernetes.io/zone"
EBS_CSI = "ebs.csi.aws.com"



@pytest.fixture(params=["node_order", "pod_order"])
def checker(request, checker):
    """Every GPU case of this module under both K2 settings: the default
    (extension-record candidates on the node-order window kernel) and
    SR_K2_MODE=1 (pod order)."""
    return checker if request.param == "node_order" else request.getfixturevalue("podorder_checker")

def nodes4():
    return [Node("a", cpu_milli=4000, labels={TZ: "z1", TR: "r1", "disk": "ssd"},
                 scalar={"attachable-volumes-aws-ebs": 1}),
            Node("b", cpu_milli=4000, labels={TZ: "z2", TR: "r1"}),
            Node("c", cpu_milli=4000, labels={TR: "r1"}),
            Node("d", cpu_milli=4000)]


def pod(name, *vols, cpu=100):
    return Pod(name, containers=[Container(cpu_milli=cpu)], volumes=list(vols))


def claim(c):
    return Volume(name=c, claim=c)


def world(*pairs, csi=None):
    """(claim name, PV or None (unbound Immediate) or "wffc") pairs -> VolumeWorld."""
    pvcs, pvs = [], []
    for name, pv in pairs:
        if pv == "wffc":
            pvcs.append(PersistentVolumeClaim(name, binding_mode="WaitForFirstConsumer"))
        elif pv is None:
            pvcs.append(PersistentVolumeClaim(name))
        elif pv == "dangling":
            pvcs.append(PersistentVolumeClaim(name, volume_name="pv-missing"))
        else:
            pvcs.append(PersistentVolumeClaim(name, volume_name=pv.name))
            pvs.append(pv)
    return VolumeWorld(pvcs=pvcs, pvs=pvs,
                       csi_limits=csi if csi is not None else {"a": {EBS_CSI: 1}, "b": {EBS_CSI: 3}})


def pv(name, zone=None, labels=None, terms=None, kind="csi", vid=None):
    lab = dict(labels or {})
    if zone is not None:
        lab[TZ] = zone
    return PersistentVolume(name, kind=kind, volume_id=vid or name, labels=lab, node_affinity=terms)


def term(*reqs, fields=()):
    return NodeSelectorTerm(list(reqs), list(fields))


def req(k, op, *vals):
    return NodeSelectorRequirement(k, op, list(vals))


def cases():
    """(name, volume world, spot pods, candidates, expected statuses, expected mappings, upstream rule)"""
    E = [[], [], [], []]
    # ---- VolumeZone
    yield ("zone_other_zone", world(("q", pv("v1", zone="z2"))), E, [[pod("p", claim("q"))]], [OK], [[1]],
           "zone z2: a (z1) and c (region only: zone reads \"\") fail, b passes")
    yield ("zone_multi_value", world(("q", pv("v1", zone="z3__z2"))), E, [[pod("p", claim("q"))]], [OK], [[1]],
           "LabelZonesToSet splits \"z3__z2\" into {z3, z2}")
    yield ("zone_no_node_matches_but_zoneless_node", world(("q", pv("v1", zone="z9"))), E,
           [[pod("p", claim("q"))]], [OK], [[3]], "a node without any zone / region label passes")
    yield ("zone_region_label", world(("q", pv("v1", labels={TR: "r1"}))), E, [[pod("p", claim("q"))]], [OK],
           [[0]], "region r1 on a")
    yield ("zone_empty_part_skipped", world(("q", pv("v1", zone="z2__"))), E, [[pod("p", claim("q"))]], [OK],
           [[0]], "LabelZonesToSet fails on an empty zone: the filter skips the label")
    yield ("zone_beta_key_absent_on_labelled_nodes", world(("q", pv("v1", labels={BZ: "z1"}))), E,
           [[pod("p", claim("q"))]], [OK], [[3]],
           "a, b, c carry some zone / region key but not the beta zone key: \"\" is never in the set")
    # ---- VolumeBinding Filter (bound PVs' node affinity)
    yield ("pv_affinity_in", world(("q", pv("v1", terms=[term(req("disk", "In", "ssd"))]))), E,
           [[pod("p", claim("q"))]], [OK], [[0]], "term disk In [ssd]")
    yield ("pv_affinity_second_node", world(("q", pv("v1", terms=[term(req(TZ, "In", "z2"))]))), E,
           [[pod("p", claim("q"))]], [OK], [[1]], "term zone In [z2]")
    yield ("pv_affinity_terms_ored", world(("q", pv("v1", terms=[term(req(TZ, "In", "z9")),
                                                                  term(req(TR, "Exists"))]))), E,
           [[pod("p", claim("q"))]], [OK], [[0]], "terms ORed: region Exists matches a")
    yield ("pv_affinity_two_pvs_anded", world(("q", pv("v1", terms=[term(req("disk", "In", "ssd"))])),
                                              ("r", pv("v2", terms=[term(req(TZ, "In", "z2"))]))), E,
           [[pod("p", claim("q"), claim("r"))]], [0], [[-1]], "every bound PV must match: a and b exclude each other")
    yield ("pv_affinity_two_multi_term_pvs", world(
        ("q", pv("v1", terms=[term(req("disk", "In", "ssd")), term(req(TZ, "In", "z2"))])),
        ("r", pv("v2", terms=[term(req(TZ, "In", "z9")), term(req(TZ, "NotIn", "z1"))]))), E,
           [[pod("p", claim("q"), claim("r"))]], [OK], [[1]], "(a or b) and (not z1): b")
    yield ("pv_affinity_match_fields_read_empty", world(
        ("q", pv("v1", terms=[term(fields=[req("metadata.name", "In", "a")])]))), E,
           [[pod("p", claim("q"))]], [0], [[-1]], "CheckNodeAffinity passes no fields: metadata.name reads \"\"")
    yield ("pv_affinity_match_fields_not_in", world(
        ("q", pv("v1", terms=[term(req(TZ, "In", "z2"), fields=[req("metadata.name", "NotIn", "b")])]))), E,
           [[pod("p", claim("q"))]], [OK], [[1]], "\"\" NotIn [b] holds on every node")
    yield ("pv_affinity_empty_term_list", world(("q", pv("v1", terms=[]))), E, [[pod("p", claim("q"))]], [0],
           [[-1]], "MatchNodeSelectorTerms over no terms is false")
    yield ("pv_affinity_invalid_value", world(("q", pv("v1", terms=[term(req("disk", "In", "-x"))]))), E,
           [[pod("p", claim("q"))]], [0], [[-1]], "a value failing IsValidLabelValue fails the only term")
    # ---- VolumeBinding PreFilter
    yield ("unbound_immediate_claim", world(("q", None)), E, [[pod("p", claim("q"))]], [0], [[-1]],
           "an unbound claim with Immediate binding fails PreFilter: no node")
    yield ("missing_claim", world(), E, [[pod("p", claim("nope"))]], [0], [[-1]], "GetPodVolumes errors")
    yield ("dangling_volume", world(("q", "dangling")), E, [[pod("p", claim("q"))]], [0], [[-1]],
           "the bound PV is missing")
    yield ("wait_for_first_consumer_falls_back", world(("q", "wffc")), E, [[pod("p", claim("q"))]], [FB], [[-1]],
           "claims to bind need the binder: reference path")
    yield ("rbd_falls_back", world(), E, [[pod("p", Volume(rbd_image="img"))]], [FB], [[-1]],
           "RBD (monitor overlap) is not encoded")
    # ---- VolumeRestrictions
    iq = lambda i, ro=False: Volume(name="i" + i, iscsi_iqn=i, read_only=ro)  # noqa: E731
    yield ("iscsi_rw_meets_rw", world(), [[pod("e", iq("t1"))], [], [], []], [[pod("p", iq("t1"))]], [OK], [[1]],
           "same IQN, not both read-only")
    yield ("iscsi_ro_meets_rw", world(), [[pod("e", iq("t1"))], [], [], []], [[pod("p", iq("t1", True))]], [OK],
           [[1]], "a read-only mount meets a read-write one")
    yield ("iscsi_both_read_only", world(), [[pod("e", iq("t1", True))], [], [], []],
           [[pod("p", iq("t1", True))]], [OK], [[0]], "both read-only: no conflict")
    yield ("iscsi_other_iqn", world(), [[pod("e", iq("t1"))], [], [], []], [[pod("p", iq("t2"))]], [OK], [[0]],
           "different IQN")
    yield ("iscsi_inside_candidate", world(), E, [[pod("p", iq("t3")), pod("q", iq("t3", True))]], [OK], [[0, 1]],
           "q meets p's read-write mount on a")
    yield ("iscsi_read_only_pair_in_candidate", world(), E, [[pod("p", iq("t3", True)), pod("q", iq("t3", True))]],
           [OK], [[0, 0]], "two read-only mounts share a")
    yield ("iscsi_three_in_candidate", world(), E,
           [[pod("p", iq("t3", True)), pod("q", iq("t3")), pod("r", iq("t3", True))]], [OK], [[0, 1, 0]],
           "q (rw) avoids p (ro) on a; r (ro) shares a with p")
    yield ("gce_pd_on_a_spot_node_falls_back", world(),
           [[pod("e", Volume(gce_pd="pd1", read_only=True))], [], [], []],
           [[pod("p", Volume(gce_pd="pd1", read_only=True))]], [FB], [[-1]],
           "planner limit: the attachable volume is already on a spot node")
    # ---- volume limits
    csi = lambda n: claim(n)  # noqa: E731
    w_lim = world(("e1", pv("ve1")), ("q1", pv("vq1")), ("q2", pv("vq2")), ("q3", pv("vq3")), ("q4", pv("vq4")),
                  ("q5", pv("vq5")))
    yield ("csi_limit_full_node", w_lim, [[pod("e", csi("e1"))], [], [], []], [[pod("p", csi("q1"))]], [OK], [[1]],
           "a: 1 attached + 1 new > CSINode count 1")
    yield ("csi_limit_candidate_fills_nodes", w_lim, [[pod("e", csi("e1"))], [], [], []],
           [[pod("p%d" % i, csi("q%d" % i)) for i in range(1, 6)]], [OK], [[1, 1, 1, 2, 2]],
           "b takes 3 (count 3), c has no CSINode limit")
    yield ("csi_limit_without_volume_on_full_node", w_lim, [[pod("e", csi("e1"))], [], [], []],
           [[pod("p")]], [OK], [[0]], "no new volume: no check")
    yield ("csi_limit_over_limit_node_no_new_volume", w_lim, [[pod("e", csi("e1")), pod("f", csi("q5"))], [], [], []],
           [[pod("p")]], [OK], [[0]],
           "a holds 2 > CSINode count 1, but p brings no new volume: csi.go returns before counting (DESIGN 2.11)")
    w_ebs = world(("q1", pv("ve", kind="aws-ebs", vid="vol-9")))
    yield ("ebs_allocatable_limit", w_ebs, [[pod("e", Volume(aws_ebs="vol-1"))], [], [], []],
           [[pod("p", Volume(aws_ebs="vol-2"))]], [OK], [[1]],
           "a's Allocatable attachable-volumes-aws-ebs is 1 and holds vol-1; b: default 39")
    yield ("ebs_pv_counts_too", w_ebs, [[pod("e", Volume(aws_ebs="vol-1"))], [], [], []],
           [[pod("p", claim("q1"))]], [OK], [[1]], "an EBS PV counts under the same key")
    yield ("shared_claim_in_candidate_falls_back", w_lim, E, [[pod("p", csi("q1")), pod("q", csi("q1"))]], [FB],
           [[-1, -1]], "planner limit: two pods of a candidate sharing an attachable volume")
    yield ("attached_volume_falls_back", w_lim, [[pod("e", csi("e1"))], [], [], []], [[pod("p", csi("e1"))]], [FB],
           [[-1]], "planner limit: a spot node already holds the pod's attachable volume")
    w3 = world(("q1", pv("vq1")), ("q2", pv("vq2")), ("g1", pv("vg1", kind="gce-pd")),
               ("g2", pv("vg2", kind="gce-pd")), ("z1", pv("vz1", kind="azure-disk")),
               ("z2", pv("vz2", kind="azure-disk")))
    yield ("three_shared_limit_keys_fall_back", w3, E,
           [[pod("p", claim("q1"), claim("g1"), claim("z1")), pod("q", claim("q2"), claim("g2"), claim("z2"))]],
           [FB], [[-1, -1]], "planner limit: two running slots per candidate")
    yield ("two_shared_limit_keys_planned", w3, E,
           [[pod("p", claim("q1"), claim("g1")), pod("q", claim("q2"), claim("g2"))]], [OK], [[0, 1]],
           "CSI (a: count 1, taken by p) and GCE PD (default 16): q goes to b")
    # combined: zone + CSI limit
    w_zl = world(("e1", pv("ve1")), ("q1", pv("vq1", zone="z1")), ("q2", pv("vq2", zone="z1")))
    yield ("zone_and_limit", w_zl, [[pod("e", csi("e1"))], [], [], []],
           [[pod("p", csi("q1")), pod("q", csi("q2"))]], [OK], [[3, 3]],
           "z1 only on a, which is full: d (no zone labels, no limit)")


CASES = list(cases())


def plan(case, use_gpu, checker=None):
    name, w, spot_pods, cands, _, _, _ = case
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes4(), spot_pods, flat, volumes=w)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    if not use_gpu:
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, cand_pods, mode=1)
        return [int(x) for x in o["status"]], [int(x) for x in o["node_of_pod"]], off
    from spotplanner.rescheduler import plan_arrays
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, off, cand_pods)
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    return [int(x) for x in p.status], [int(x) for x in p.node_of_pod], off


def check(case, got):
    status, nodes, off = got
    want_status, want_map = case[4], case[5]
    assert status == want_status, (case[0], case[6])
    for k, m in enumerate(want_map):
        if want_status[k] != FB:
            assert nodes[off[k]:off[k + 1]] == m, (case[0], case[6])


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_volume_cases(case):
    check(case, plan(case, False))


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_gpu_volume_cases(checker, case):
    check(case, plan(case, True, checker))


def test_volume_tables_absent_flag_pods():
    """A shim without sr_volumes flags every pod with volumes (SR_POD_FB_VOLUMES)."""
    from spotplanner.model import encode_cluster
    p = pod("p", claim("q"))
    enc = encode_cluster(nodes4(), [p], volume_tables=False)
    assert enc.a["flags"][0] & capi.SR_POD_FB_VOLUMES
    enc = encode_cluster(nodes4(), [p], volumes=world(("q", pv("v1"))))
    assert not enc.a["flags"][0] & capi.SR_POD_FB_VOLUMES


def rand_volume_scenario(seed):
    """Random clusters whose pods carry claims (CSI / EBS / GCE PD PVs with zone
    labels and node affinity), inline ISCSI / GCE PD / EBS disks, under CSINode
    and Allocatable limits; some claims unbound or waiting for a consumer."""
    r = random.Random(seed)
    nodes, spot_pods, cands = rand_scenario(9500 + seed, n_spot=6 + seed % 14, n_cand=10, max_pods=3 + seed % 6,
                                            features=seed % 3 == 0)
    zones = ["z1", "z2", "z3"]
    for i, n in enumerate(nodes):
        if r.random() < 0.8:
            n.labels[TZ] = r.choice(zones)
        if r.random() < 0.5:
            n.labels[TR] = "r1"
        if r.random() < 0.3:
            n.scalar["attachable-volumes-aws-ebs"] = r.choice([0, 1, 2, 3])
    pvcs, pvs, vid = [], [], [0]

    def new_claim(ns):
        vid[0] += 1
        name = "c%d" % vid[0]
        x = r.random()
        if x < 0.05:
            pvcs.append(PersistentVolumeClaim(name, namespace=ns))
        elif x < 0.1:
            pvcs.append(PersistentVolumeClaim(name, namespace=ns, binding_mode="WaitForFirstConsumer"))
        else:
            kind = r.choice(["csi", "csi", "aws-ebs", "gce-pd", "nfs"])
            labels = {TZ: r.choice(zones + ["z1__z2"])} if r.random() < 0.5 else {}
            terms = None
            if r.random() < 0.3:
                terms = [term(req(TZ, "In", *r.sample(zones, r.choice([1, 2]))))]
                if r.random() < 0.3:
                    terms.append(term(req(TR, "Exists")))
            pvs.append(PersistentVolume("pv" + name, kind=kind, volume_id="v%d" % vid[0], labels=labels,
                                        node_affinity=terms))
            pvcs.append(PersistentVolumeClaim(name, namespace=ns, volume_name="pv" + name))
        return Volume(name=name, claim=name)

    iqns = ["iq1", "iq2", "iq3"]
    for ps in spot_pods + cands:
        for p in ps:
            if r.random() < 0.35:
                p.volumes.append(new_claim(p.namespace))
            if r.random() < 0.15:
                p.volumes.append(Volume(name="isc", iscsi_iqn=r.choice(iqns), read_only=r.random() < 0.5))
            if r.random() < 0.05:
                p.volumes.append(Volume(name="pd", gce_pd="pd%d" % r.randrange(1000), read_only=r.random() < 0.5))
    csi = {n.name: {EBS_CSI: r.choice([1, 2, 4])} for n in nodes if r.random() < 0.6}
    return nodes, spot_pods, cands, VolumeWorld(pvcs=pvcs, pvs=pvs, csi_limits=csi)


def run_volume_scenario(checker, seed):
    nodes, spot_pods, cands, w = rand_volume_scenario(seed)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat, volumes=w)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, cand_pods, mode=1)
    if checker is None:
        return o
    from spotplanner.rescheduler import plan_arrays
    from test_gpu_parity import compare_plans
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, off, cand_pods)
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    compare_plans(o, p, off, None)
    return o


def test_random_volume_scenarios_are_mostly_planned():
    planned = failed = 0
    for seed in range(30):
        o = run_volume_scenario(None, seed)
        planned += int(np.sum(o["status"] != FB))
        failed += int(np.sum(o["status"] >= 0))
    assert planned >= 200 and failed >= 20, (planned, failed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_gpu_random_volume_clusters(checker, seed):
    """Every candidate's status and every pod's node equal to the oracle."""
    run_volume_scenario(checker, seed)
