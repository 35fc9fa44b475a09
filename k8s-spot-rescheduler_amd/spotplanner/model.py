"""Kubernetes object model + the shim's encoding into the C-ABI cluster arrays.

The dataclasses mirror the fields of k8s.io/api/core/v1 Pod / Node that the
reference's hot path reads (rescheduler.go:338-370, nodes/nodes.go:63-165 and
the k8s v1.19.2 scheduler filters behind CheckPredicates).  `encode_cluster`
is what the Go shim of INTEGRATION.md does before crossing the C-ABI: intern
strings into ids, convert quantities, compute the scheduler request of each
pod and set fallback flags for features the encoded predicate set lacks.
"""
from __future__ import annotations

import ctypes
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import capi

GiB = 1024 * 1024 * 1024
MiB = 1024 * 1024

EFFECTS = {"": capi.SR_EFFECT_EMPTY, "NoSchedule": capi.SR_EFFECT_NO_SCHEDULE,
           "PreferNoSchedule": capi.SR_EFFECT_PREFER_NO_SCHEDULE, "NoExecute": capi.SR_EFFECT_NO_EXECUTE}
TOL_OPS = {"": capi.SR_TOL_EQUAL, "Equal": capi.SR_TOL_EQUAL, "Exists": capi.SR_TOL_EXISTS}
SEL_OPS = {"In": capi.SR_OP_IN, "NotIn": capi.SR_OP_NOT_IN, "Exists": capi.SR_OP_EXISTS,
           "DoesNotExist": capi.SR_OP_DOES_NOT_EXIST, "Gt": capi.SR_OP_GT, "Lt": capi.SR_OP_LT}
PROTOS = {"": capi.SR_PROTO_TCP, "TCP": capi.SR_PROTO_TCP, "UDP": capi.SR_PROTO_UDP,
          "SCTP": capi.SR_PROTO_SCTP}
MIRROR_ANNOTATION = "kubernetes.io/config.mirror"
UNSCHEDULABLE_TAINT_KEY = "node.kubernetes.io/unschedulable"


@dataclass
class ContainerPort:
    host_port: int
    container_port: int = 0
    protocol: str = "TCP"
    host_ip: str = ""


@dataclass
class Container:
    cpu_milli: int = 0          # Requests.Cpu().MilliValue()
    memory: int = 0             # Requests.Memory().Value()
    ephemeral: int = 0          # Requests.StorageEphemeral().Value()
    scalar: Dict[str, int] = field(default_factory=dict)   # extended / hugepages requests
    ports: List[ContainerPort] = field(default_factory=list)


@dataclass
class Toleration:
    key: str = ""
    operator: str = ""
    value: str = ""
    effect: str = ""


@dataclass
class Taint:
    key: str
    value: str = ""
    effect: str = "NoSchedule"


@dataclass
class NodeSelectorRequirement:
    key: str
    operator: str
    values: List[str] = field(default_factory=list)


@dataclass
class NodeSelectorTerm:
    match_expressions: List[NodeSelectorRequirement] = field(default_factory=list)
    match_fields: List[NodeSelectorRequirement] = field(default_factory=list)


@dataclass
class LabelSelectorRequirement:
    key: str
    operator: str
    values: List[str] = field(default_factory=list)


@dataclass
class LabelSelector:
    match_labels: Dict[str, str] = field(default_factory=dict)
    match_expressions: List[LabelSelectorRequirement] = field(default_factory=list)


@dataclass
class PodAffinityTerm:
    topology_key: str
    label_selector: Optional[LabelSelector] = None   # None = nil: selects nothing
    namespaces: List[str] = field(default_factory=list)  # [] = the term's own pod's namespace


@dataclass
class TopologySpreadConstraint:
    max_skew: int
    topology_key: str
    when_unsatisfiable: str = "DoNotSchedule"   # ScheduleAnyway never filters
    label_selector: Optional[LabelSelector] = None  # None = nil: matches nothing


@dataclass
class Volume:
    """A Spec.Volumes entry the volume filters read (the rest: local_storage)."""
    name: str = "data"
    claim: Optional[str] = None        # PersistentVolumeClaim.ClaimName
    gce_pd: Optional[str] = None       # GCEPersistentDisk.PDName
    aws_ebs: Optional[str] = None      # AWSElasticBlockStore.VolumeID
    iscsi_iqn: Optional[str] = None    # ISCSI.IQN
    azure_disk: Optional[str] = None   # AzureDisk.DiskName
    rbd_image: Optional[str] = None    # RBD (not encoded: the shim flags the pod)
    read_only: bool = False


@dataclass
class PersistentVolume:
    name: str
    kind: str = "csi"                  # csi | aws-ebs | gce-pd | azure-disk | nfs (not attachable)
    volume_id: str = ""                # CSI VolumeHandle / EBS VolumeID / PD name / DiskName
    driver: str = "ebs.csi.aws.com"    # CSI driver
    labels: Dict[str, str] = field(default_factory=dict)        # zone / region labels (VolumeZone)
    node_affinity: Optional[List[NodeSelectorTerm]] = None      # Spec.NodeAffinity.Required.NodeSelectorTerms


@dataclass
class PersistentVolumeClaim:
    name: str
    namespace: str = "kube-system"
    volume_name: str = ""              # Spec.VolumeName of a bound claim ("" unbound)
    binding_mode: str = "Immediate"    # its StorageClass's VolumeBindingMode


ZONE_KEYS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
             "topology.kubernetes.io/zone", "topology.kubernetes.io/region")
NONCSI_KEYS = {"aws-ebs": "attachable-volumes-aws-ebs", "gce-pd": "attachable-volumes-gce-pd",
               "azure-disk": "attachable-volumes-azure-disk"}
NONCSI_DEFAULT = {"attachable-volumes-aws-ebs": 39, "attachable-volumes-gce-pd": 16,
                  "attachable-volumes-azure-disk": 16}  # nodevolumelimits defaults (KUBE_MAX_PD_VOLS unset)


@dataclass
class VolumeWorld:
    """The listers the volume filters read: claims, volumes, and per node the
    CSINode drivers' allocatable counts (CSI limits; the non-CSI limits come
    from Node.scalar attachable-volumes-* or the filter default)."""
    pvcs: List[PersistentVolumeClaim] = field(default_factory=list)
    pvs: List[PersistentVolume] = field(default_factory=list)
    csi_limits: Dict[str, Dict[str, int]] = field(default_factory=dict)  # node name -> {driver: count}


def _att_key(pv_kind: str, driver: str) -> Optional[str]:
    if pv_kind == "csi":
        return "attachable-volumes-csi-" + driver
    return NONCSI_KEYS.get(pv_kind)


def resolve_volumes(pod: "Pod", world: VolumeWorld):
    """What the Go shim derives from a pod's volumes through the scheduler's
    listers [upstream k8s v1.19.2]: (prefilter_fail, fallback, disks, attachable,
    zones, pv_terms).  VolumeBinding's GetPodVolumes: a missing claim or
    volume, or an unbound claim with Immediate binding, fails PreFilter; an
    unbound claim with WaitForFirstConsumer needs the binder (not encoded).  RBD
    volumes are not encoded."""
    pvcs = {(c.namespace, c.name): c for c in world.pvcs}
    pvs = {v.name: v for v in world.pvs}
    pf, fb = False, False
    disks, att, zones, pv_terms = [], [], [], []
    for v in pod.volumes:
        if v.rbd_image is not None:
            fb = True
        if v.gce_pd is not None:
            disks.append((capi.SR_DISK_GCE_PD, v.gce_pd, v.read_only))
            att.append(("attachable-volumes-gce-pd", "gce-pd/" + v.gce_pd, True))
        if v.aws_ebs is not None:
            disks.append((capi.SR_DISK_AWS_EBS, v.aws_ebs, v.read_only))
            att.append(("attachable-volumes-aws-ebs", "aws-ebs/" + v.aws_ebs, True))
        if v.iscsi_iqn is not None:
            disks.append((capi.SR_DISK_ISCSI, v.iscsi_iqn, v.read_only))
        if v.azure_disk is not None:
            att.append(("attachable-volumes-azure-disk", "azure-disk/" + v.azure_disk, True))
        if v.claim is None:
            continue
        pvc = pvcs.get((pod.namespace, v.claim))
        if pvc is None:
            pf = True
            continue
        if not pvc.volume_name:
            if pvc.binding_mode == "WaitForFirstConsumer":
                fb = True
            else:
                pf = True
            continue
        pv = pvs.get(pvc.volume_name)
        if pv is None:
            pf = True
            continue
        for k in ZONE_KEYS:
            if k in pv.labels:
                zs = [z.strip() for z in pv.labels[k].split("__")]
                if all(zs):  # LabelZonesToSet fails on an empty zone: the filter skips the label
                    zones.append((k, zs))
        if pv.node_affinity is not None:
            pv_terms.append(pv.node_affinity)
        key = _att_key(pv.kind, pv.driver)
        if key is not None:
            uid = ("csi/%s/%s" % (pv.driver, pv.volume_id)) if pv.kind == "csi" else "%s/%s" % (pv.kind, pv.volume_id)
            att.append((key, uid, pv.kind != "csi"))
    seen, uatt = set(), []
    for a in att:  # each (key, unique name) once per pod
        if (a[0], a[1]) not in seen:
            seen.add((a[0], a[1]))
            uatt.append(a)
    return pf, fb, disks, uatt, zones, pv_terms


@dataclass
class OwnerReference:
    kind: str
    name: str = ""
    controller: Optional[bool] = True


@dataclass
class Pod:
    name: str
    namespace: str = "kube-system"
    node_name: str = ""
    containers: List[Container] = field(default_factory=list)
    init_containers: List[Container] = field(default_factory=list)
    overhead: Optional[Container] = None
    priority: Optional[int] = 0
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)
    node_selector: Dict[str, str] = field(default_factory=dict)
    # Affinity.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution.NodeSelectorTerms;
    # None = the pointer is nil (no requirement).
    required_node_affinity: Optional[List[NodeSelectorTerm]] = None
    tolerations: List[Toleration] = field(default_factory=list)
    owner_references: List[OwnerReference] = field(default_factory=list)
    # features outside the encoded predicate set
    has_pvc: bool = False
    required_pod_affinity: bool = False
    required_pod_anti_affinity: bool = False  # opaque anti-affinity (no terms given): fallback
    # Affinity.PodAntiAffinity.RequiredDuringSchedulingIgnoredDuringExecution (encoded)
    pod_anti_affinity: Optional[List[PodAffinityTerm]] = None
    # Affinity.PodAffinity.RequiredDuringSchedulingIgnoredDuringExecution (encoded)
    pod_affinity: Optional[List[PodAffinityTerm]] = None
    hard_topology_spread: bool = False  # opaque DoNotSchedule spread (no constraints given): fallback
    # Spec.TopologySpreadConstraints (encoded)
    topology_spread: List[TopologySpreadConstraint] = field(default_factory=list)
    # drain attributes (cluster-autoscaler utils/drain)
    phase: str = "Running"                    # Status.Phase
    restart_policy: str = "Always"            # Spec.RestartPolicy
    deletion_age_s: Optional[float] = None    # now - DeletionTimestamp; None = not being deleted
    grace_seconds: Optional[int] = None       # Spec.TerminationGracePeriodSeconds (None = nil)
    local_storage: bool = False               # an EmptyDir or HostPath volume
    volumes: List[Volume] = field(default_factory=list)  # resolved through encode_cluster's VolumeWorld

    def cpu_sort_milli(self) -> int:
        """getPodCPURequests (nodes/nodes.go:159-165): Σ regular containers' CPU."""
        return sum(c.cpu_milli for c in self.containers)

    def scheduler_request(self):
        """computePodResourceRequest (k8s v1.19 noderesources/fit.go):
        max(Σ containers, each init container) + Overhead, per resource."""
        cpu = sum(c.cpu_milli for c in self.containers)
        mem = sum(c.memory for c in self.containers)
        eph = sum(c.ephemeral for c in self.containers)
        for ic in self.init_containers:
            cpu, mem, eph = max(cpu, ic.cpu_milli), max(mem, ic.memory), max(eph, ic.ephemeral)
        if self.overhead is not None:
            cpu += self.overhead.cpu_milli
            mem += self.overhead.memory
            eph += self.overhead.ephemeral
        return cpu, mem, eph

    def scalar_request(self) -> Dict[str, int]:
        """computePodResourceRequest's ScalarResources: max(Σ containers, each
        init container) + Overhead per name (every name listed anywhere)."""
        out: Dict[str, int] = {}
        for c in self.containers:
            for k, v in c.scalar.items():
                out[k] = out.get(k, 0) + v
        for ic in self.init_containers:
            for k, v in ic.scalar.items():
                out[k] = max(out.get(k, 0), v)
        if self.overhead is not None:
            for k, v in self.overhead.scalar.items():
                out[k] = out.get(k, 0) + v
        return out

    def node_accounting(self):
        """What NodeInfo.AddPod adds to the node's Requested in k8s v1.19.2
        (framework/v1alpha1/types.go calculateResource): the regular containers'
        sum plus Overhead -- init containers are not counted there, unlike in
        the fit request (parity unpinned: the module is not in the reference
        tree; the Go shim takes both from the pinned scheduler itself).
        Returns (cpu, memory, ephemeral, {scalar name: amount})."""
        cpu = sum(c.cpu_milli for c in self.containers)
        mem = sum(c.memory for c in self.containers)
        eph = sum(c.ephemeral for c in self.containers)
        sc: Dict[str, int] = {}
        for c in self.containers:
            for k, v in c.scalar.items():
                sc[k] = sc.get(k, 0) + v
        if self.overhead is not None:
            cpu += self.overhead.cpu_milli
            mem += self.overhead.memory
            eph += self.overhead.ephemeral
            for k, v in self.overhead.scalar.items():
                sc[k] = sc.get(k, 0) + v
        return cpu, mem, eph, sc

    def host_ports(self):
        return [p for c in self.containers for p in c.ports if p.host_port > 0]


@dataclass
class Node:
    name: str
    cpu_milli: int
    memory: int = 2 * GiB
    pods: int = 100
    ephemeral: int = 0
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    unschedulable: bool = False
    scalar: Dict[str, int] = field(default_factory=dict)  # Allocatable extended / hugepages resources


def pod_id(pod: Pod) -> str:
    """podID (rescheduler.go:402-404)."""
    return "%s/%s" % (pod.namespace, pod.name)


class Interner:
    """String -> int32 id, shared by every encoding that talks to one snapshot."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.strings: List[str] = []

    def id(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.strings)
            self.ids[s] = i
            self.strings.append(s)
        return i

    def peek(self, s: str) -> int:
        return self.ids.get(s, -1)


def _i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32).reshape(-1))


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64).reshape(-1))


def _u8(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint8).reshape(-1))


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))


class NilControllerPanic(RuntimeError):
    """rescheduler.go:244 dereferences *owner.Controller: the reference panics on nil."""


def _daemonset_owner_walk(pod: Pod):
    """The owner loop of rescheduler.go:243-248: (controlledByDaemonSet, derefs a nil Controller)."""
    for o in pod.owner_references:
        if o.controller is None:
            return False, True
        if o.controller and o.kind == "DaemonSet":
            return True, False
    return False, False


def pod_flags(pod: Pod, scalar_tables: bool = True, spread_tables: bool = True, volume_tables: bool = True) -> int:
    f = 0
    if _daemonset_owner_walk(pod)[0]:
        f |= capi.SR_POD_DAEMONSET_CONTROLLER
    if MIRROR_ANNOTATION in pod.annotations:
        f |= capi.SR_POD_MIRROR
    if pod.required_pod_anti_affinity or pod.pod_anti_affinity:
        f |= capi.SR_POD_HAS_REQ_ANTI_AFFINITY
    conts = list(pod.containers) + list(pod.init_containers) + ([pod.overhead] if pod.overhead else [])
    if not scalar_tables and any(c.scalar for c in conts):  # the shim passes no scalar tables
        f |= capi.SR_POD_FB_SCALAR_RESOURCES
    if pod.has_pvc or (pod.volumes and not volume_tables):
        f |= capi.SR_POD_FB_VOLUMES
    if pod.hard_topology_spread or (not spread_tables and any(c.when_unsatisfiable == "DoNotSchedule"
                                                              for c in pod.topology_spread)):
        f |= capi.SR_POD_FB_TOPOLOGY_SPREAD
    if pod.required_pod_affinity or (pod.required_pod_anti_affinity and not pod.pod_anti_affinity):
        f |= capi.SR_POD_FB_POD_AFFINITY
    return f


_INT64 = re.compile(r"[+-]?[0-9]+\Z")


def parse_int64(s: str):
    """strconv.ParseInt(s, 10, 64): optional sign, decimal digits, in range; None otherwise."""
    if not _INT64.match(s):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def string_ints(interner: Interner):
    """sr_cluster.str_int / str_int_ok over the interner's strings (node-affinity Gt / Lt)."""
    vals = [parse_int64(s) for s in interner.strings]
    return (np.ascontiguousarray([0 if v is None else v for v in vals], dtype=np.int64).reshape(-1),
            np.ascontiguousarray([v is not None for v in vals], dtype=np.uint8).reshape(-1))


# apimachinery v0.19.2 util/validation [upstream]: qualifiedNameFmt is
# ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]; a label value is empty or such a
# name of at most 63 characters; a qualified name is [DNS-1123 subdomain "/"]
# name, the name part non-empty and at most 63 characters, the prefix at most
# 253 characters of [a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*.
# Go's regexp `$` matches at the end of the text only: fullmatch.
_QNAME = re.compile(r"([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]")
_DNS1123_SUBDOMAIN = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")


def is_valid_label_value(s: str) -> bool:
    """validation.IsValidLabelValue: labels.NewRequirement's validateLabelValue."""
    return len(s.encode()) <= 63 and (s == "" or _QNAME.fullmatch(s) is not None)


def is_qualified_name(s: str) -> bool:
    """validation.IsQualifiedName: labels.NewRequirement's validateLabelKey."""
    parts = s.split("/")
    if len(parts) > 2:
        return False
    if len(parts) == 2:
        prefix = parts[0]
        if not prefix or len(prefix.encode()) > 253 or _DNS1123_SUBDOMAIN.fullmatch(prefix) is None:
            return False
    name = parts[-1]
    return 0 < len(name.encode()) <= 63 and _QNAME.fullmatch(name) is not None


def string_label_flags(interner: Interner):
    """sr_cluster.str_label over the interner's strings (labels.NewRequirement validation)."""
    return np.ascontiguousarray([(capi.SR_STR_LABEL_VALUE if is_valid_label_value(s) else 0) |
                                 (capi.SR_STR_LABEL_KEY if is_qualified_name(s) else 0)
                                 for s in interner.strings], dtype=np.uint8).reshape(-1)


class EncodedCluster:
    """numpy arrays in the sr_cluster layout + the ctypes struct pointing at them."""

    def __init__(self, arrays: dict, interner: Interner):
        self.a = arrays
        self.interner = interner
        self.a["str_int"], self.a["str_int_ok"] = string_ints(interner)
        self.a["str_label"] = string_label_flags(interner)
        self.struct = capi.make_cluster_struct(self.a)

    @property
    def ptr(self):
        return ctypes.byref(self.struct)


def _encode_pod_affinity(pods: List[Pod], it: Interner) -> dict:
    """sr_pod_affinity arrays: namespaces, labels, required anti-affinity terms,
    then required affinity terms (one term table, anti-affinity terms first)."""
    ns, lo, lk, lv, ao = [], [0], [], [], [0]
    tk, nso, nsi, nil, mlo, mlk, mlv, meo, mek, mep, mevo, mev = [], [0], [], [], [0], [], [], [0], [], [], [0], []

    def add_term(t):
        tk.append(it.id(t.topology_key))
        nsi.extend(it.id(x) for x in t.namespaces)
        nso.append(len(nsi))
        sel = t.label_selector
        nil.append(1 if sel is None else 0)
        for k, v in (sel.match_labels.items() if sel else []):
            mlk.append(it.id(k))
            mlv.append(it.id(v))
        mlo.append(len(mlk))
        for r in (sel.match_expressions if sel else []):
            mek.append(it.id(r.key))
            mep.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER) if r.operator not in ("Gt", "Lt")
                       else capi.SR_OP_OTHER)
            mev.extend(it.id(v) for v in r.values)
            mevo.append(len(mev))
        meo.append(len(mek))

    for p in pods:
        ns.append(it.id(p.namespace))
        for k, v in p.labels.items():
            lk.append(it.id(k))
            lv.append(it.id(v))
        lo.append(len(lk))
        for t in (p.pod_anti_affinity or []):
            add_term(t)
        ao.append(len(tk))
    fo = [len(tk)]  # affinity terms are numbered after every anti-affinity term
    for p in pods:
        for t in (p.pod_affinity or []):
            add_term(t)
        fo.append(len(tk))
    return dict(pa_ns=_i32(ns), pa_label_off=_i32(lo), pa_label_key=_i32(lk), pa_label_val=_i32(lv),
                pa_anti_off=_i32(ao), pa_topology_key=_i32(tk), pa_ns_off=_i32(nso), pa_ns_ids=_i32(nsi),
                pa_selector_nil=_u8(nil), pa_ml_off=_i32(mlo), pa_ml_key=_i32(mlk), pa_ml_val=_i32(mlv),
                pa_me_off=_i32(meo), pa_me_key=_i32(mek), pa_me_op=_i32(mep), pa_me_val_off=_i32(mevo),
                pa_me_vals=_i32(mev), pa_aff_off=_i32(fo))


def _encode_spread(pods: List[Pod], it: Interner) -> dict:
    """sr_spread arrays: the DoNotSchedule constraints of every pod."""
    off, skew, tk, nil, mlo, mlk, mlv, meo, mek, mep, mevo, mev, term = \
        [0], [], [], [], [0], [], [], [0], [], [], [0], [], []
    for p in pods:
        for c in p.topology_spread:
            if c.when_unsatisfiable != "DoNotSchedule":
                continue
            skew.append(c.max_skew)
            tk.append(it.id(c.topology_key))
            sel = c.label_selector
            nil.append(1 if sel is None else 0)
            for k, v in (sel.match_labels.items() if sel else []):
                mlk.append(it.id(k))
                mlv.append(it.id(v))
            mlo.append(len(mlk))
            for r in (sel.match_expressions if sel else []):
                mek.append(it.id(r.key))
                mep.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER) if r.operator not in ("Gt", "Lt")
                           else capi.SR_OP_OTHER)
                mev.extend(it.id(v) for v in r.values)
                mevo.append(len(mev))
            meo.append(len(mek))
        off.append(len(skew))
        term.append(1 if p.deletion_age_s is not None else 0)
    return dict(ts_off=_i32(off), ts_max_skew=_i32(skew), ts_topology_key=_i32(tk), ts_selector_nil=_u8(nil),
                ts_ml_off=_i32(mlo), ts_ml_key=_i32(mlk), ts_ml_val=_i32(mlv), ts_me_off=_i32(meo),
                ts_me_key=_i32(mek), ts_me_op=_i32(mep), ts_me_val_off=_i32(mevo), ts_me_vals=_i32(mev),
                ts_terminating=_u8(term))


def _encode_volumes(nodes: List[Node], pods: List[Pod], world: VolumeWorld, it: Interner, flags: List[int]) -> dict:
    """sr_volumes arrays (the shim's resolution of every pod's volumes)."""
    pf, do, dk, di, dr = [], [0], [], [], []
    ao, ak, ai, an = [0], [], [], []
    zo, zk, zvo, zv = [0], [], [0], []
    pvo, pto, teo, tfo = [0], [0], [0], [0]
    ek, eo, evo, ev, fk, fo, fvo, fv = [], [], [0], [], [], [], [0], []
    for i, p in enumerate(pods):
        fail, fb, disks, att, zones, pv_terms = resolve_volumes(p, world)
        if fb:
            flags[i] |= capi.SR_POD_FB_VOLUMES
        pf.append(1 if fail else 0)
        for kind, vid, ro in disks:
            dk.append(kind)
            di.append(it.id(vid))
            dr.append(1 if ro else 0)
        do.append(len(dk))
        for key, uid, noncsi in att:
            ak.append(it.id(key))
            ai.append(it.id(uid))
            an.append(1 if noncsi else 0)
        ao.append(len(ak))
        for key, vals in zones:
            zk.append(it.id(key))
            zv.extend(it.id(v) for v in vals)
            zvo.append(len(zv))
        zo.append(len(zk))
        for terms in pv_terms:
            for term in terms:
                for r in term.match_expressions:
                    ek.append(it.id(r.key))
                    eo.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER))
                    ev.extend(it.id(v) for v in r.values)
                    evo.append(len(ev))
                teo.append(len(ek))
                for r in term.match_fields:
                    fk.append(it.id(r.key))
                    fo.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER))
                    fv.extend(it.id(v) for v in r.values)
                    fvo.append(len(fv))
                tfo.append(len(fk))
            pto.append(len(teo) - 1)
        pvo.append(len(pto) - 1)
    lo, lk, lv = [0], [], []
    for n in nodes:
        lim = {}
        for key, default in NONCSI_DEFAULT.items():  # non-CSI: Allocatable, else the filter's default
            lim[key] = n.scalar.get(key, default)
        for driver, count in world.csi_limits.get(n.name, {}).items():
            lim["attachable-volumes-csi-" + driver] = count
        for key in sorted(lim):
            lk.append(it.id(key))
            lv.append(lim[key])
        lo.append(len(lk))
    return dict(vol_prefilter_fail=_u8(pf), vol_disk_off=_i32(do), vol_disk_kind=_i32(dk), vol_disk_id=_i32(di),
                vol_disk_ro=_u8(dr), vol_att_off=_i32(ao), vol_att_key=_i32(ak), vol_att_id=_i32(ai),
                vol_att_noncsi=_u8(an), vol_limit_off=_i32(lo), vol_limit_key=_i32(lk), vol_limit=_i64(lv),
                vol_zone_off=_i32(zo), vol_zone_key=_i32(zk), vol_zone_val_off=_i32(zvo), vol_zone_vals=_i32(zv),
                vol_zone_keys=[it.peek(k) for k in ZONE_KEYS], vol_pv_off=_i32(pvo), vol_pv_term_off=_i32(pto),
                vol_term_expr_off=_i32(teo), vol_term_field_off=_i32(tfo), vol_expr_key=_i32(ek),
                vol_expr_op=_i32(eo), vol_expr_val_off=_i32(evo), vol_expr_vals=_i32(ev), vol_field_key=_i32(fk),
                vol_field_op=_i32(fo), vol_field_val_off=_i32(fvo), vol_field_vals=_i32(fv))


def encode_cluster(nodes: List[Node], pods: List[Pod], interner: Optional[Interner] = None,
                   pod_node: Optional[List[int]] = None, scalar_tables: bool = True,
                   accounting: bool = True, spread_tables: bool = True,
                   volumes: Optional[VolumeWorld] = None, volume_tables: bool = True,
                   stamps: Optional[List[int]] = None) -> EncodedCluster:
    """Encode nodes and pods.  pod_node[i] is the node index of pods[i] (default:
    looked up by pod.node_name; -1 when unbound).  Pods of one node keep their
    relative order (= the per-node LIST order).  scalar_tables=False: no scalar
    resource tables (pods listing scalars are flagged for the fallback path);
    accounting=False: no acc_* table (NodeInfo.AddPod adds the fit request)."""
    it = interner or Interner()
    e = it.id("")
    mn = it.id("metadata.name")
    uk = it.id(UNSCHEDULABLE_TAINT_KEY)
    name_idx = {n.name: i for i, n in enumerate(nodes)}
    A = {}
    A["node_name"] = _i32([it.id(n.name) for n in nodes])
    A["alloc_cpu"] = _i64([n.cpu_milli for n in nodes])
    A["alloc_mem"] = _i64([n.memory for n in nodes])
    A["alloc_eph"] = _i64([n.ephemeral for n in nodes])
    A["alloc_pods"] = _i64([n.pods for n in nodes])
    A["unsched"] = _u8([1 if n.unschedulable else 0 for n in nodes])
    lo, lk, lv = [0], [], []
    to, tk, tv, te = [0], [], [], []
    for n in nodes:
        for k, v in n.labels.items():
            lk.append(it.id(k))
            lv.append(it.id(v))
        lo.append(len(lk))
        for t in n.taints:
            tk.append(it.id(t.key))
            tv.append(it.id(t.value))
            te.append(EFFECTS.get(t.effect, capi.SR_EFFECT_OTHER))
        to.append(len(tk))
    A.update(label_off=_i32(lo), label_key=_i32(lk), label_val=_i32(lv),
             taint_off=_i32(to), taint_key=_i32(tk), taint_val=_i32(tv), taint_eff=_i32(te))

    pn, sortc, rc, rm, re, pr, hp, fl = [], [], [], [], [], [], [], []
    so, sk, sv = [0], [], []
    aff, term_off = [], [0]
    texpr, tfield = [0], [0]
    ek, eo, evo, ev = [], [], [0], []
    fk, fo, fvo, fv = [], [], [0], []
    tolo, tolk, tolop, tolv, tole = [0], [], [], [], []
    po, pp, pnum, pip = [0], [], [], []
    for i, p in enumerate(pods):
        if pod_node is not None:
            pn.append(pod_node[i])
        else:
            pn.append(name_idx.get(p.node_name, -1))
        sortc.append(p.cpu_sort_milli())
        c, m, eph = p.scheduler_request()
        rc.append(c)
        rm.append(m)
        re.append(eph)
        hp.append(0 if p.priority is None else 1)
        pr.append(0 if p.priority is None else p.priority)
        fl.append(pod_flags(p, scalar_tables, spread_tables, volume_tables))
        for k, v in p.node_selector.items():
            sk.append(it.id(k))
            sv.append(it.id(v))
        so.append(len(sk))
        aff.append(0 if p.required_node_affinity is None else 1)
        for term in (p.required_node_affinity or []):
            for r in term.match_expressions:
                ek.append(it.id(r.key))
                eo.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER))
                ev.extend(it.id(v) for v in r.values)
                evo.append(len(ev))
            texpr.append(len(ek))
            for r in term.match_fields:
                fk.append(it.id(r.key))
                fo.append(SEL_OPS.get(r.operator, capi.SR_OP_OTHER))
                fv.extend(it.id(v) for v in r.values)
                fvo.append(len(fv))
            tfield.append(len(fk))
        term_off.append(len(texpr) - 1)
        for t in p.tolerations:
            tolk.append(it.id(t.key))
            tolop.append(TOL_OPS.get(t.operator, capi.SR_TOL_OTHER))
            tolv.append(it.id(t.value))
            tole.append(EFFECTS.get(t.effect, capi.SR_EFFECT_OTHER))
        tolo.append(len(tolk))
        for hpz in p.host_ports():
            pp.append(PROTOS.get(hpz.protocol, capi.SR_PROTO_TCP))
            pnum.append(hpz.host_port)
            pip.append(-1 if hpz.host_ip in ("", "0.0.0.0") else it.id(hpz.host_ip))
        po.append(len(pp))
    A.update(pod_node=_i32(pn), cpu_sort=_i64(sortc), req_cpu=_i64(rc), req_mem=_i64(rm),
             req_eph=_i64(re), priority=_i32(pr), has_priority=_u8(hp), flags=_u32(fl),
             sel_off=_i32(so), sel_key=_i32(sk), sel_val=_i32(sv), aff_required=_u8(aff),
             term_off=_i32(term_off), term_expr_off=_i32(texpr), term_field_off=_i32(tfield),
             expr_key=_i32(ek), expr_op=_i32(eo), expr_val_off=_i32(evo), expr_vals=_i32(ev),
             field_key=_i32(fk), field_op=_i32(fo), field_val_off=_i32(fvo), field_vals=_i32(fv),
             tol_off=_i32(tolo), tol_key=_i32(tolk), tol_op=_i32(tolop), tol_val=_i32(tolv),
             tol_eff=_i32(tole), port_off=_i32(po), port_proto=_i32(pp), port_num=_i32(pnum),
             port_ip=_i32(pip))
    if volume_tables:
        for k in ZONE_KEYS:  # interned up front: nodes carrying them match the keys' ids
            it.id(k)
        A.update(_encode_volumes(nodes, pods, volumes or VolumeWorld(), it, fl))
        A["flags"] = _u32(fl)
    A.update(_encode_pod_affinity(pods, it))
    if spread_tables:
        A.update(_encode_spread(pods, it))
    if scalar_tables:
        so_, sn_, sr_, sa_ = [0], [], [], []
        for p in pods:
            req = p.scalar_request()
            acc = p.node_accounting()[3]
            for name in sorted(req):
                sn_.append(it.id(name))
                sr_.append(req[name])
                sa_.append(acc.get(name, 0))
            so_.append(len(sn_))
        no_, nn_, na_ = [0], [], []
        for n in nodes:
            for name in sorted(n.scalar):
                nn_.append(it.id(name))
                na_.append(n.scalar[name])
            no_.append(len(nn_))
        A.update(pod_scalar_off=_i32(so_), pod_scalar_name=_i32(sn_), pod_scalar_req=_i64(sr_),
                 pod_scalar_acc=_i64(sa_), node_scalar_off=_i32(no_), node_scalar_name=_i32(nn_),
                 node_scalar_alloc=_i64(na_))
    if accounting:
        accs = [p.node_accounting() for p in pods]
        A.update(acc_cpu=_i64([a[0] for a in accs]), acc_mem=_i64([a[1] for a in accs]),
                 acc_eph=_i64([a[2] for a in accs]))
    if stamps is not None:  # sr_cluster.pod_stamp (the shim: a hash of UID and ResourceVersion)
        A["pod_stamp"] = np.ascontiguousarray(np.asarray(stamps, dtype=np.uint64).reshape(-1))
    A["n_nodes"] = len(nodes)
    A["n_pods"] = len(pods)
    A["id_empty"] = e
    A["id_metadata_name"] = mn
    A["id_unschedulable_key"] = uk
    return EncodedCluster(A, it)


def label_flag(flag: str, interner: Interner) -> capi.sr_node_label:
    """Parse a node-label flag the way isSpotNode does (strings.SplitN(label, "=", 2))."""
    parts = flag.split("=", 1)
    if len(parts) == 1:
        return capi.sr_node_label(interner.id(parts[0]), -1, 0)
    return capi.sr_node_label(interner.id(parts[0]), interner.id(parts[1]), 1)


# ------------------------------------------------------------ drain attributes
SAFE_TO_EVICT_ANNOTATION = "cluster-autoscaler.kubernetes.io/safe-to-evict"
DAEMONSET_POD_ANNOTATION = "cluster-autoscaler.kubernetes.io/daemonset-pod"
CONTROLLER_KINDS = {"ReplicationController": capi.SR_DRAIN_CTRL_REPLICATION_CONTROLLER,
                    "DaemonSet": capi.SR_DRAIN_CTRL_DAEMONSET, "Job": capi.SR_DRAIN_CTRL_JOB,
                    "ReplicaSet": capi.SR_DRAIN_CTRL_REPLICASET, "StatefulSet": capi.SR_DRAIN_CTRL_STATEFULSET}
PHASES = {"Pending": capi.SR_PHASE_PENDING, "Running": capi.SR_PHASE_RUNNING, "Succeeded": capi.SR_PHASE_SUCCEEDED,
          "Failed": capi.SR_PHASE_FAILED}
RESTART = {"Always": capi.SR_RESTART_ALWAYS, "OnFailure": capi.SR_RESTART_ON_FAILURE, "Never": capi.SR_RESTART_NEVER}


@dataclass
class PodDisruptionBudget:
    namespace: str = "kube-system"
    match_labels: Optional[Dict[str, str]] = field(default_factory=dict)  # None = nil selector (selects nothing)
    invalid: bool = False  # LabelSelectorAsSelector fails


def _kube_system_pdb(pod: Pod, pdbs: List[PodDisruptionBudget]):
    """checkKubeSystemPDBs over the kube-system PDBs in list order: (matched, error)."""
    for pdb in pdbs:
        if pdb.namespace != "kube-system":
            continue
        if pdb.invalid:
            return False, True
        if pdb.match_labels is not None and all(pod.labels.get(k) == v for k, v in pdb.match_labels.items()):
            return True, False
    return False, False


class EncodedDrain:
    """numpy arrays in the sr_pod_drain layout + the ctypes struct pointing at them."""

    def __init__(self, pods: List[Pod], pdbs: List[PodDisruptionBudget]):
        fl, ph, rp, age, gr = [], [], [], [], []
        for p in pods:
            f = 0
            ctrl = next((o for o in p.owner_references if o.controller), None)  # metav1.GetControllerOf
            if ctrl is not None:
                f |= CONTROLLER_KINDS.get(ctrl.kind, capi.SR_DRAIN_CTRL_OTHER)
            if p.annotations.get(DAEMONSET_POD_ANNOTATION) == "true":
                f |= capi.SR_DRAIN_DAEMONSET_ANNOTATION
            ste = p.annotations.get(SAFE_TO_EVICT_ANNOTATION)
            if ste == "true":
                f |= capi.SR_DRAIN_SAFE_TO_EVICT
            elif ste == "false":
                f |= capi.SR_DRAIN_NOT_SAFE_TO_EVICT
            if p.deletion_age_s is not None:
                f |= capi.SR_DRAIN_DELETING
            if p.namespace == "kube-system":
                f |= capi.SR_DRAIN_KUBE_SYSTEM
                matched, err = _kube_system_pdb(p, pdbs)
                f |= (capi.SR_DRAIN_KUBE_SYSTEM_PDB if matched else 0) | (capi.SR_DRAIN_PDB_ERROR if err else 0)
            if p.local_storage:
                f |= capi.SR_DRAIN_LOCAL_STORAGE
            if _daemonset_owner_walk(p)[1]:
                f |= capi.SR_DRAIN_NIL_CONTROLLER
            fl.append(f)
            ph.append(PHASES.get(p.phase, capi.SR_PHASE_UNKNOWN))
            rp.append(RESTART.get(p.restart_policy, capi.SR_RESTART_ALWAYS))
            age.append(0 if p.deletion_age_s is None else int(round(p.deletion_age_s * 1e9)))
            gr.append(-1 if p.grace_seconds is None else p.grace_seconds)
        self.a = dict(flags=_u32(fl), phase=_u8(ph), restart=_u8(rp), age=_i64(age), grace=_i64(gr))
        self.struct = capi.sr_pod_drain(len(pods), capi.ptr(self.a["flags"], capi.PU32),
                                        capi.ptr(self.a["phase"], capi.PU8), capi.ptr(self.a["restart"], capi.PU8),
                                        capi.ptr(self.a["age"], capi.P64), capi.ptr(self.a["grace"], capi.P64))

    @property
    def ptr(self):
        return ctypes.byref(self.struct)
