/*
 * sr_planner.h — C-ABI of the MI355X drain planner (k8s-spot-rescheduler hot path).
 *
 * The reference (Go, github.com/pusher/k8s-spot-rescheduler) has no FFI: the hot
 * path sits behind unexported Go functions plus cluster-autoscaler interfaces.
 * Every entry point below names the reference interface it replaces (file:line
 * into the reference tree).  A cgo binding for these entry points is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only; no torch / HIP types cross this boundary.
 *  - Strings never cross.  The caller (the Go shim) interns every string it
 *    needs (label keys/values, taint keys/values, node names, host IPs) into
 *    int32 ids; the planner only compares ids.  `sr_cluster.id_empty`,
 *    `id_metadata_name` and `id_unschedulable_key` tell the planner which ids
 *    stand for "", "metadata.name" and "node.kubernetes.io/unschedulable".
 *  - Quantities arrive already converted the way the reference converts them:
 *    CPU via Quantity.MilliValue(), memory / ephemeral storage / pods via
 *    Quantity.Value().
 *  - Input buffers are owned by the caller for the duration of a call only;
 *    nothing is retained after return (handles copy what they keep).
 *  - Output buffers are caller-allocated.
 *  - Handles are not thread-safe: one owner at a time.
 */
#ifndef SR_PLANNER_H
#define SR_PLANNER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SR_ABI_VERSION 9

/* ------------------------------------------------------------------ status */
typedef int32_t sr_status;
#define SR_OK                 0
#define SR_ERR_INVALID_ARG    1  /* malformed input (bad CSR, index out of range) */
#define SR_ERR_HIP            2  /* HIP runtime error (message in sr_last_error) */
#define SR_ERR_CAPACITY       3  /* a planner limit was exceeded */
#define SR_ERR_NIL_PRIORITY   4  /* nodes/nodes.go:139 dereferences *Spec.Priority: the reference panics */
#define SR_ERR_RCCL           5  /* RCCL error */
#define SR_ERR_NO_DEVICE      6  /* no HIP device: the planner never falls back to the CPU */
#define SR_ERR_STATE          7  /* call sequence error (e.g. Revert without Fork) */
#define SR_ERR_NIL_CONTROLLER 8  /* rescheduler.go:244 dereferences a nil OwnerReference.Controller: the reference panics */

/* -------------------------------------------------------------- enumerations */
/* Taint / toleration effects (k8s.io/api/core/v1 TaintEffect). */
#define SR_EFFECT_EMPTY               0  /* toleration only: "" = every effect */
#define SR_EFFECT_NO_SCHEDULE         1
#define SR_EFFECT_PREFER_NO_SCHEDULE  2
#define SR_EFFECT_NO_EXECUTE          3
#define SR_EFFECT_OTHER               4  /* any other string */

/* Toleration operators. */
#define SR_TOL_EQUAL   0  /* "" or "Equal" */
#define SR_TOL_EXISTS  1
#define SR_TOL_OTHER   2  /* unknown operator: never tolerates */

/* Node selector requirement operators (v1.NodeSelectorOperator). */
#define SR_OP_IN              0
#define SR_OP_NOT_IN          1
#define SR_OP_EXISTS          2
#define SR_OP_DOES_NOT_EXIST  3
#define SR_OP_GT              4
#define SR_OP_LT              5
#define SR_OP_OTHER           6  /* unknown operator: the term fails to build */

/* Host-port protocols ("" is sanitised to TCP by the shim, as HostPortInfo does). */
#define SR_PROTO_TCP   0
#define SR_PROTO_UDP   1
#define SR_PROTO_SCTP  2

/* Pod flags (sr_pods.flags). */
#define SR_POD_DAEMONSET_CONTROLLER (1u << 0)  /* an owner ref with *Controller && Kind=="DaemonSet" (rescheduler.go:243-248) */
#define SR_POD_MIRROR               (1u << 1)  /* mirror pod (config.mirror annotation) */
#define SR_POD_HAS_REQ_ANTI_AFFINITY (1u << 2) /* carries required pod anti-affinity terms (matters when it sits on a spot node);
                                                  without sr_cluster.pod_affinity, or with the flag but no terms
                                                  there, the terms are opaque and every candidate falls back */
/* Fallback reasons set by the shim: features the encoded predicate set does not cover. */
#define SR_POD_FB_SCALAR_RESOURCES  (1u << 8)  /* extended / hugepages / attachable-volume requests */
#define SR_POD_FB_VOLUMES           (1u << 9)  /* PVCs or volumes inspected by volume filters */
#define SR_POD_FB_TOPOLOGY_SPREAD   (1u << 10) /* DoNotSchedule topology spread constraints */
#define SR_POD_FB_POD_AFFINITY      (1u << 11) /* required pod (anti-)affinity the shim does not pass in
                                                  sr_cluster.pod_affinity */
#define SR_POD_FB_OTHER             (1u << 12) /* anything else the shim cannot encode */
#define SR_POD_FB_MASK              (0xff00u)

/* Candidate status codes (sr_plan_out.status).  >= 0: index of the first pod
 * that fits on no spot node ("pod %s can't be rescheduled on any existing spot
 * node", rescheduler.go:363). */
#define SR_CAND_OK        (-1)
#define SR_CAND_FALLBACK  (-2)  /* outside the encoded predicate set: evaluate with the reference path */
#define SR_CAND_EMPTY     (-3)  /* no pods to move: run() skips it (rescheduler.go:260-264) */
#define SR_CAND_SKIPPED   (-4)  /* sr_plan_first: after the first drainable candidate, never evaluated
                                   (run() drains it and breaks, rescheduler.go:280-286) */

/* ------------------------------------------------------------- cluster model */
/* Nodes (k8s.io/api/core/v1 Node), in the order the node lister returned them
 * (rescheduler.go:186).  CSR arrays: x_off has n+1 entries. */
typedef struct {
  int32_t        n;
  const int32_t *name;             /* interned ObjectMeta.Name (matchFields metadata.name) */
  const int64_t *alloc_milli_cpu;  /* Status.Allocatable.Cpu().MilliValue() */
  const int64_t *alloc_memory;     /* Status.Allocatable.Memory().Value() */
  const int64_t *alloc_ephemeral;  /* Status.Allocatable.StorageEphemeral().Value() */
  const int64_t *alloc_pods;       /* Status.Allocatable.Pods().Value() */
  const uint8_t *unschedulable;    /* Spec.Unschedulable */
  const int32_t *label_off;        /* ObjectMeta.Labels (keys unique per node) */
  const int32_t *label_key;
  const int32_t *label_val;
  const int32_t *taint_off;        /* Spec.Taints */
  const int32_t *taint_key;
  const int32_t *taint_val;
  const int32_t *taint_effect;     /* SR_EFFECT_* */
} sr_nodes;

/* Pods (k8s.io/api/core/v1 Pod).  Pods bound to one node appear in the order
 * the per-node LIST returned them (nodes/nodes.go:130). */
typedef struct {
  int32_t        n;
  const int32_t *node;             /* index into sr_nodes of Spec.NodeName, -1 if unbound */
  const int64_t *cpu_sort_milli;   /* Σ regular containers Requests.Cpu().MilliValue() (nodes/nodes.go:159-165) */
  const int64_t *req_milli_cpu;    /* scheduler request: max(Σ containers, each init container) + Overhead */
  const int64_t *req_memory;       /*   (k8s v1.19 noderesources computePodResourceRequest) */
  const int64_t *req_ephemeral;
  const int32_t *priority;         /* *Spec.Priority */
  const uint8_t *has_priority;     /* Spec.Priority != nil */
  const uint32_t *flags;           /* SR_POD_* */
  /* Spec.NodeSelector (key, value) pairs */
  const int32_t *sel_off, *sel_key, *sel_val;
  /* Spec.Affinity.NodeAffinity.RequiredDuringSchedulingIgnoredDuringExecution:
   * aff_required[i] != 0 iff that pointer is non-nil.  Terms are ORed; a term
   * ANDs its matchExpressions and its matchFields. */
  const uint8_t *aff_required;
  const int32_t *term_off;         /* [n+1]       pods  -> terms */
  const int32_t *term_expr_off;    /* [terms+1]   terms -> matchExpressions */
  const int32_t *term_field_off;   /* [terms+1]   terms -> matchFields */
  const int32_t *expr_key, *expr_op, *expr_val_off, *expr_vals;     /* expr_val_off [exprs+1] */
  const int32_t *field_key, *field_op, *field_val_off, *field_vals; /* field_val_off [fields+1] */
  /* Spec.Tolerations */
  const int32_t *tol_off, *tol_key, *tol_op, *tol_val, *tol_effect;  /* "" key/value = id_empty */
  /* container host ports with HostPort > 0 (regular containers only) */
  const int32_t *port_off, *port_proto, *port_num, *port_ip /* -1 = "" or "0.0.0.0" */;
} sr_pods;

/* Required inter-pod (anti-)affinity: the InterPodAffinity filter of k8s
 * v1.19.2 [upstream plugins/interpodaffinity] for
 * Spec.Affinity.PodAntiAffinity.RequiredDuringSchedulingIgnoredDuringExecution
 * and Spec.Affinity.PodAffinity.RequiredDuringSchedulingIgnoredDuringExecution,
 * and the pod namespaces and labels their terms select on.  CSR arrays over
 * sr_pods; terms are numbered across all pods.  A term's Namespaces list is
 * empty when the API object's is (the term then selects in its own pod's
 * namespace).  Selector operators: SR_OP_IN / NOT_IN / EXISTS / DOES_NOT_EXIST;
 * anything else (or In/NotIn without values, Exists/DoesNotExist with values,
 * a key that is not a qualified name, a value that is not a valid label value:
 * sr_cluster.str_label) fails LabelSelectorAsSelector, and a pod carrying such
 * a term is routed to the fallback path (on a spot node: every candidate). */
typedef struct {
  const int32_t *ns;                                /* [pods.n] interned ObjectMeta.Namespace */
  const int32_t *label_off, *label_key, *label_val; /* [pods.n+1] ObjectMeta.Labels (keys unique per pod) */
  const int32_t *anti_off;                          /* [pods.n+1] pods -> required anti-affinity terms */
  const int32_t *topology_key;                      /* [terms] interned TopologyKey */
  const int32_t *ns_off, *ns_ids;                   /* [terms+1] Namespaces */
  const uint8_t *selector_nil;                      /* [terms] LabelSelector == nil: selects nothing */
  const int32_t *ml_off, *ml_key, *ml_val;          /* [terms+1] MatchLabels */
  const int32_t *me_off, *me_key, *me_op;           /* [terms+1] MatchExpressions */
  const int32_t *me_val_off, *me_vals;              /* [exprs+1] their values */
  /* Spec.Affinity.PodAffinity.RequiredDuringSchedulingIgnoredDuringExecution:
   * [pods.n+1] pods -> required pod AFFINITY terms, in the same term tables
   * (numbered after every anti-affinity term).  NULL: none given.  A pod whose
   * affinity the shim cannot pass carries SR_POD_FB_POD_AFFINITY instead. */
  const int32_t *aff_off;
} sr_pod_affinity;

/* Spec.TopologySpreadConstraints with WhenUnsatisfiable = DoNotSchedule: the
 * PodTopologySpread filter of k8s v1.19.2 [upstream
 * plugins/podtopologyspread/filtering.go].  ScheduleAnyway constraints never
 * filter and are not passed.  For each constraint: the nodes of the snapshot
 * that pass the pod's nodeSelector / required node affinity and carry every
 * constraint's topology key define the topology pairs; a pair counts the
 * snapshot pods in the pod's own namespace, not terminating, matching the
 * selector; a node passes when it carries every key and, per constraint,
 * count(pair) + (the pod matches the selector) - min over the pairs <= maxSkew.
 * Selector tables in the sr_pod_affinity term format; a selector that fails
 * LabelSelectorAsSelector (or any pod with constraints when the cluster passes
 * no sr_spread) goes to the fallback path. */
typedef struct {
  const int32_t *off;            /* [pods.n+1] pods -> DoNotSchedule constraints */
  const int32_t *max_skew;       /* [constraints] */
  const int32_t *topology_key;   /* [constraints] interned TopologyKey */
  const uint8_t *selector_nil;   /* [constraints] LabelSelector == nil: matches nothing */
  const int32_t *ml_off, *ml_key, *ml_val;  /* [constraints+1] MatchLabels */
  const int32_t *me_off, *me_key, *me_op;   /* [constraints+1] MatchExpressions */
  const int32_t *me_val_off, *me_vals;      /* [exprs+1] their values */
  const uint8_t *terminating;    /* [pods.n] DeletionTimestamp != nil: never counted */
} sr_spread;

/* The volume filters of CheckPredicates (rescheduler.go:344) [upstream k8s
 * v1.19.2 plugins volumebinding, volumezone, volumerestrictions and
 * nodevolumelimits: EBSLimits, GCEPDLimits, AzureDiskLimits (non-CSI) and
 * NodeVolumeLimits (CSI)], with every PersistentVolumeClaim already resolved by
 * the shim through the scheduler's own listers (PVC -> PV, StorageClass,
 * CSINode).  A pod whose volumes the shim cannot describe here (an unbound
 * claim with WaitForFirstConsumer binding, an RBD volume, a lister error) keeps
 * SR_POD_FB_VOLUMES; without this table every pod with such volumes does. */
#define SR_DISK_GCE_PD   0  /* GCEPersistentDisk.PDName: two mounts conflict unless both are read-only */
#define SR_DISK_AWS_EBS  1  /* AWSElasticBlockStore.VolumeID: two mounts always conflict */
#define SR_DISK_ISCSI    2  /* ISCSI.IQN: two mounts conflict unless both are read-only */
typedef struct {
  /* VolumeBinding PreFilter fails (an unbound claim with Immediate binding, a
   * claim or volume the listers do not find): the pod fits no node. [pods.n] */
  const uint8_t *prefilter_fail;
  /* VolumeRestrictions: the pod's inline GCE PD / AWS EBS / ISCSI volumes */
  const int32_t *disk_off;         /* [pods.n+1] */
  const int32_t *disk_kind;        /* SR_DISK_* */
  const int32_t *disk_id;          /* interned PDName / VolumeID / IQN */
  const uint8_t *disk_ro;          /* ReadOnly */
  /* volume limits: the pod's attachable volumes, each (limit key, unique volume
   * name) once per pod -- the filters' unique names of inline and PV-backed
   * volumes (a claim without a volume counts as one unique name of its own) */
  const int32_t *att_off;          /* [pods.n+1] */
  const int32_t *att_key;          /* interned limit key: attachable-volumes-aws-ebs, -gce-pd, -azure-disk, -csi-<driver> */
  const int32_t *att_id;           /* interned unique volume name */
  const uint8_t *att_noncsi;       /* non-CSI filter key: checked whenever the pod has such a volume, even one already attached */
  /* the limit of each key per node (non-CSI: Allocatable or the filter's
   * default; CSI: the CSINode driver's allocatable count).  A key without an
   * entry on a node never refuses there. */
  const int32_t *limit_off;        /* [nodes.n+1] */
  const int32_t *limit_key;
  const int64_t *limit;
  /* VolumeZone: per bound PV, each zone / region label (one of zone_keys) with
   * the values volumehelpers.LabelZonesToSet parses ("a__b" -> {a, b}; a label
   * that fails to parse is skipped by the filter and not passed) */
  const int32_t *zone_off;         /* [pods.n+1] */
  const int32_t *zone_key;
  const int32_t *zone_val_off;     /* [zones+1] */
  const int32_t *zone_vals;
  int32_t zone_keys[4];            /* interned failure-domain.beta.kubernetes.io/zone, .../region,
                                      topology.kubernetes.io/zone, .../region (-1: never interned) */
  /* VolumeBinding: Spec.NodeAffinity.Required of each bound PV
   * (volumeutil.CheckNodeAffinity: MatchNodeSelectorTerms on the node's labels
   * with no fields, so a matchFields requirement reads "") */
  const int32_t *pv_off;           /* [pods.n+1] pods -> PVs with a Required node affinity */
  const int32_t *pv_term_off;      /* [pvs+1] PVs -> NodeSelectorTerms */
  const int32_t *term_expr_off;    /* [terms+1] */
  const int32_t *term_field_off;   /* [terms+1] */
  const int32_t *expr_key, *expr_op, *expr_val_off, *expr_vals;
  const int32_t *field_key, *field_op, *field_val_off, *field_vals;
} sr_volumes;

typedef struct {
  sr_nodes nodes;
  sr_pods  pods;
  int32_t  id_empty;          /* interned id of "" (-1 if never interned) */
  int32_t  id_metadata_name;  /* interned id of "metadata.name" (-1 if never interned) */
  int32_t  id_unschedulable_key; /* interned id of "node.kubernetes.io/unschedulable" (-1 if never interned) */
  const sr_pod_affinity *pod_affinity; /* NULL: required anti-affinity stays on the fallback path */
  /* Integer values of the interned strings, for node-affinity Gt / Lt
   * (labels.Requirement.Matches: strconv.ParseInt(s, 10, 64) of the node's label
   * value and of the requirement's single value).  str_int_ok[id] = 1 when string
   * `id` parses, str_int[id] its value; ids >= n_strings never parse.  NULL: a pod
   * with Gt / Lt is routed to the fallback path. */
  int32_t        n_strings;
  const int64_t *str_int;
  const uint8_t *str_int_ok;
  /* labels.NewRequirement's validation of the interned strings [upstream
   * apimachinery v0.19.2 labels/selector.go: validateLabelKey =
   * validation.IsQualifiedName, validateLabelValue = validation.IsValidLabelValue],
   * which NodeSelectorRequirementsAsSelector (required node affinity) and
   * metav1.LabelSelectorAsSelector (inter-pod terms) run on every key and value:
   * str_label[id] & SR_STR_LABEL_VALUE when string `id` is a valid label value,
   * & SR_STR_LABEL_KEY when it is a qualified name; ids >= n_strings are neither.
   * The Go shim fills it with apimachinery's own functions.  A node-affinity term
   * with an invalid key or value matches nothing; a pod (anti-)affinity term with
   * one is opaque (fallback).  NULL: validity unknown -- a pod with node-affinity
   * matchExpressions, or an inter-pod term with a label requirement, is routed to
   * the fallback path.  (Spec.NodeSelector goes through labels.SelectorFromSet,
   * which does not validate in v0.19.) */
  const uint8_t *str_label;
  /* Scalar resources (v1helper.IsScalarResourceName: extended resources,
   * hugepages-*, attachable-volumes-*): the ScalarResources loop of
   * NodeResourcesFit fitsRequest [upstream k8s v1.19.2 noderesources/fit.go]:
   * a pod fits when alloc[s] >= req[s] + requested[s] for every name s it
   * lists (a node without s allocates 0; a listed name, even with 0, disables
   * the all-zero-request shortcut).  CSR per pod / per node, names interned;
   * Value() quantities.  pod_scalar_req: computePodResourceRequest (max of the
   * containers' sum and each init container, plus Overhead); pod_scalar_acc:
   * what NodeInfo.AddPod adds to Requested for the same name.  NULL
   * pod_scalar_off: no scalar tables (the shim flags such pods
   * SR_POD_FB_SCALAR_RESOURCES). */
  const int32_t *pod_scalar_off;   /* [pods.n+1] */
  const int32_t *pod_scalar_name;
  const int64_t *pod_scalar_req;
  const int64_t *pod_scalar_acc;
  const int32_t *node_scalar_off;  /* [nodes.n+1] Status.Allocatable scalar resources */
  const int32_t *node_scalar_name;
  const int64_t *node_scalar_alloc;
  /* NodeInfo.AddPod's accounting of cpu / memory / ephemeral storage
   * (calculateResource) for each pod; it can differ from the fit request
   * req_* (init containers).  The snapshot's Requested sums these.  NULL: the
   * same as req_*.  The Go shim fills both sides from the pinned scheduler
   * (framework.NewNodeInfo(pod).Requested). */
  const int64_t *acc_milli_cpu;
  const int64_t *acc_memory;
  const int64_t *acc_ephemeral;
  /* DoNotSchedule topology spread constraints (NULL: a pod that has them
   * carries SR_POD_FB_TOPOLOGY_SPREAD).  Pod labels and namespaces come from
   * pod_affinity, which must be given with it. */
  const sr_spread *spread;
  /* Volume filters (ABI 5).  NULL: pods with volumes carry SR_POD_FB_VOLUMES. */
  const sr_volumes *volumes;
  /* [pods.n] A value the shim changes whenever the pod object changes (e.g. a
   * hash of UID and ResourceVersion; 0 = unknown).  The planner's encoder keeps
   * what it derived from a pod's spec keyed by (pod index, stamp) across calls
   * and re-derives it only for pods whose stamp changed, so the string ids a
   * stamped pod's spec uses must stay the same across calls (one interner per
   * process).  A stamp also covers what the pod's spec resolves through (its
   * PVCs' bound PVs).  With every candidate pod stamped, a call whose
   * candidate input (cand_pod_off, cand_pods, cand_global, stamps) equals the
   * previous call's keeps that call's candidate side (sr_timing.enc_reused).
   * NULL: no stamps (every call re-reads every pod's spec).  ABI 5. */
  const uint64_t *pod_stamp;
} sr_cluster;
#define SR_STR_LABEL_VALUE 1u
#define SR_STR_LABEL_KEY   2u

/* ------------------------------------------------------------- NewNodeMap */
/* A node-label flag: "key" (has_value = 0) or "key=value" (has_value = 1). */
typedef struct {
  int32_t key;
  int32_t value;
  int32_t has_value;
} sr_node_label;

typedef struct {
  sr_node_label on_demand;     /* nodes.OnDemandNodeLabel  (nodes/nodes.go:33) */
  sr_node_label spot;          /* nodes.SpotNodeLabel      (nodes/nodes.go:35) */
  int32_t priority_threshold;  /* nodes.PriorityThreshold  (nodes/nodes.go:41) */
} sr_node_map_params;

/* Output of NewNodeMap; every array is caller-allocated. */
typedef struct {
  int32_t *spot;           /* [nodes.n] out: nodeMap[Spot], RequestedCPU desc (nodes/nodes.go:95-97) */
  int32_t *n_spot;         /* [1] */
  int32_t *on_demand;      /* [nodes.n] out: nodeMap[OnDemand], RequestedCPU asc (nodes/nodes.go:99-101) */
  int32_t *n_on_demand;    /* [1] */
  int32_t *node_pod_off;   /* [nodes.n+1] NodeInfo.Pods per node index (every node, mapped or not) */
  int32_t *node_pod_idx;   /* [pods.n]    pod indices, CPU-desc sort order (nodes/nodes.go:76-80) */
  int64_t *requested_cpu;  /* [nodes.n] NodeInfo.RequestedCPU */
  int64_t *free_cpu;       /* [nodes.n] NodeInfo.FreeCPU */
} sr_node_map;

/* Replaces nodes.NewNodeMap (nodes/nodes.go:63-104) with the pod LIST already
 * done by the caller (pods carry their node index).  Sorting reproduces Go
 * 1.16 sort.Slice exactly, ties included.  Host-only: needs no GPU. */
sr_status sr_new_node_map(const sr_cluster *cluster, const sr_node_map_params *params,
                          sr_node_map *out);

/* NewNodeMap of consecutive housekeeping ticks (rescheduler.go:195): the cache
 * keeps each node's pod sort (by node name) and reuses it for a node whose
 * LISTed pods carry the same non-zero pod_stamp values in the same order under
 * the same params and node kind.  Output identical to sr_new_node_map;
 * cache NULL = sr_new_node_map.  out_sorted (optional): nodes whose pods were
 * sorted anew.  Not thread-safe per cache. */
typedef struct sr_node_map_cache sr_node_map_cache;
sr_status sr_node_map_cache_create(sr_node_map_cache **out);
void      sr_node_map_cache_destroy(sr_node_map_cache *cache);
sr_status sr_new_node_map_cached(sr_node_map_cache *cache, const sr_cluster *cluster,
                                 const sr_node_map_params *params, sr_node_map *out, int32_t *out_sorted);

/* Replaces isSpotNode / isOnDemandNode (nodes/nodes.go:168-209).  Host-only. */
int32_t sr_node_has_label(const sr_cluster *cluster, int32_t node, const sr_node_label *label);

/* --------------------------------------------------- pods to move per candidate */
/* Drain attributes of a pod for cluster-autoscaler utils/drain
 * GetPodsForDeletionOnNodeDrain (@03f60a4c3818 [upstream, not in the reference
 * tree]; call rescheduler.go:231), derived by the shim from the Pod object. */
#define SR_DRAIN_CTRL_MASK          0x7u   /* kind of the ControllerRef (first owner ref with Controller == true): */
#define SR_DRAIN_CTRL_NONE          0u
#define SR_DRAIN_CTRL_REPLICATION_CONTROLLER 1u
#define SR_DRAIN_CTRL_DAEMONSET     2u
#define SR_DRAIN_CTRL_JOB           3u
#define SR_DRAIN_CTRL_REPLICASET    4u
#define SR_DRAIN_CTRL_STATEFULSET   5u
#define SR_DRAIN_CTRL_OTHER         6u
#define SR_DRAIN_DAEMONSET_ANNOTATION (1u << 3)  /* annotation cluster-autoscaler.kubernetes.io/daemonset-pod == "true" */
#define SR_DRAIN_SAFE_TO_EVICT      (1u << 4)  /* annotation cluster-autoscaler.kubernetes.io/safe-to-evict == "true" */
#define SR_DRAIN_NOT_SAFE_TO_EVICT  (1u << 5)  /*   ... == "false" */
#define SR_DRAIN_DELETING           (1u << 6)  /* DeletionTimestamp != nil */
#define SR_DRAIN_KUBE_SYSTEM        (1u << 7)  /* Namespace == "kube-system" */
#define SR_DRAIN_KUBE_SYSTEM_PDB    (1u << 8)  /* checkKubeSystemPDBs(pod, kube-system PDBs in list order) == true */
#define SR_DRAIN_PDB_ERROR          (1u << 9)  /* checkKubeSystemPDBs returns an error (a selector failing to
                                                  convert before the first matching PDB) */
#define SR_DRAIN_LOCAL_STORAGE      (1u << 10) /* an EmptyDir or HostPath volume */
#define SR_DRAIN_NIL_CONTROLLER     (1u << 11) /* rescheduler.go:243-248 run on this pod dereferences a nil Controller */

/* Pod phases (Status.Phase) and restart policies (Spec.RestartPolicy). */
#define SR_PHASE_PENDING    0
#define SR_PHASE_RUNNING    1
#define SR_PHASE_SUCCEEDED  2
#define SR_PHASE_FAILED     3
#define SR_PHASE_UNKNOWN    4
#define SR_RESTART_ALWAYS     0
#define SR_RESTART_ON_FAILURE 1
#define SR_RESTART_NEVER      2

typedef struct {
  int32_t         n;               /* = sr_pods.n */
  const uint32_t *flags;           /* SR_DRAIN_* */
  const uint8_t  *phase;           /* SR_PHASE_* */
  const uint8_t  *restart_policy;  /* SR_RESTART_* */
  const int64_t  *deletion_age_ns; /* now - DeletionTimestamp (read with SR_DRAIN_DELETING) */
  const int64_t  *grace_seconds;   /* *Spec.TerminationGracePeriodSeconds, -1 = nil (30 s default) */
} sr_pod_drain;

typedef struct {
  int32_t skip_nodes_with_system_pods;   /* argument 3 at rescheduler.go:231 / :391: *deleteNonReplicatedPods */
  int32_t skip_nodes_with_local_storage; /* argument 4 at rescheduler.go:231 / :391: false */
  int32_t owner_filter;                  /* 1: then the DaemonSet-owner filter of run() (:240-256);
                                            0: GetPodsForDeletionOnNodeDrain alone, as updateSpotNodeMetrics (:388-399) */
} sr_drain_params;

/* drain.BlockingPodReason */
#define SR_BLOCK_NONE                 0
#define SR_BLOCK_NOT_REPLICATED       1
#define SR_BLOCK_UNMOVABLE_KUBE_SYSTEM 2
#define SR_BLOCK_LOCAL_STORAGE        3
#define SR_BLOCK_NOT_SAFE_TO_EVICT    4
#define SR_BLOCK_UNEXPECTED_ERROR     5

/* The candidate lists of run() (rescheduler.go:228-264): for each node of
 * `nodes` (on-demand NodeInfoArray order), GetPodsForDeletionOnNodeDrain over
 * NodeInfo.Pods (node_pod_off / node_pod_idx, sr_node_map layout) with the
 * reference's arguments, then (owner_filter) the DaemonSet-owner filter
 * (:240-256).  With owner_filter = 0 over the spot nodes, the list lengths are
 * updateSpotNodeMetrics' pod counts (:388-399; blocked nodes are skipped).
 * out_cand_off [n_nodes + 1], out_cand_pods [<= all pods of the nodes]: the
 * podsForDeletion of each node, in order.  A node with a blocking pod gets an
 * empty list, its pod in out_block_pod (else -1) and the reason in
 * out_block_reason (run() logs and `continue`s, :232-238).  Host-only. */
sr_status sr_pods_for_deletion(const sr_cluster *cluster, const sr_pod_drain *drain, const sr_drain_params *params,
                               const int32_t *nodes, int32_t n_nodes, const int32_t *node_pod_off,
                               const int32_t *node_pod_idx, int32_t *out_cand_off, int32_t *out_cand_pods,
                               int32_t *out_block_pod, int32_t *out_block_reason);

/* ------------------------------------------------------------ cluster snapshot */
typedef struct sr_snapshot sr_snapshot;

/* Replaces NodeInfoArray.GetClusterSnapshot (nodes/nodes.go:226-232):
 * AddNodeWithPods(node, pods) per spot node, in NodeInfoArray order.
 * node_pod_off/node_pod_idx: CSR indexed by node index (sr_node_map layout).
 *
 * Ownership: the snapshot COPIES what it needs of every pod it holds (requests,
 * host ports, namespace, labels, anti-affinity terms) when the pod is added, by
 * sr_snapshot_create or sr_snapshot_add_pod.  Later calls may pass any
 * sr_cluster (e.g. one holding only the pods being queried): pod indices in a
 * call always index that call's cluster, never the one the snapshot was built
 * from.  A pod added from a cluster without sr_pod_affinity has unknown labels;
 * a candidate whose own inter-pod terms would have to match it is routed to the
 * fallback path. */
sr_status sr_snapshot_create(const sr_cluster *cluster, const int32_t *spot_nodes, int32_t n_spot,
                             const int32_t *node_pod_off, const int32_t *node_pod_idx,
                             sr_snapshot **out);
/* GetClusterSnapshot of the next housekeeping tick (nodes/nodes.go:226-232,
 * rescheduler.go:215) into a snapshot built by an earlier tick: afterwards
 * `snap` holds what sr_snapshot_create on these arguments would build.  A spot
 * node (matched by name) whose pod list carries the same non-zero pod_stamp
 * values in the same order as the snapshot's keeps its state and pod copies;
 * the other nodes are rebuilt.  Without stamps, or after the cluster's optional
 * tables changed, the whole snapshot is rebuilt.  SR_ERR_STATE while forked;
 * SR_ERR_INVALID_ARG leaves `snap` unchanged.  out_rebuilt (optional): spot
 * nodes whose state was rebuilt. */
sr_status sr_snapshot_refresh(sr_snapshot *snap, const sr_cluster *cluster, const int32_t *spot_nodes,
                              int32_t n_spot, const int32_t *node_pod_off, const int32_t *node_pod_idx,
                              int32_t *out_rebuilt);
/* sr_snapshot_refresh when this tick's node map came from sr_new_node_map_cached(cache, ...) and `snap` was
 * last refreshed (or rebuilt) by this call from the cache's previous node map and not changed since: a spot node
 * whose LISTed pods that node map found unchanged (same non-zero stamps, same order) keeps its state without its
 * pods' stamps being gathered again.  Otherwise (another cache, a skipped tick, an AddPod since) exactly
 * sr_snapshot_refresh.  Either way `snap` ends up as sr_snapshot_create would build it. */
sr_status sr_snapshot_refresh_cached(sr_snapshot *snap, const sr_node_map_cache *cache, const sr_cluster *cluster,
                                     const int32_t *spot_nodes, int32_t n_spot, const int32_t *node_pod_off,
                                     const int32_t *node_pod_idx, int32_t *out_rebuilt);
void      sr_snapshot_destroy(sr_snapshot *snap);
/* ClusterSnapshot.AddPod(pod, nodeName) (rescheduler.go:366); spot_pos = position in the NodeInfoArray. */
sr_status sr_snapshot_add_pod(sr_snapshot *snap, const sr_cluster *cluster, int32_t pod, int32_t spot_pos);
/* ClusterSnapshot.Fork / Revert (rescheduler.go:269,273): one level deep. */
sr_status sr_snapshot_fork(sr_snapshot *snap);
sr_status sr_snapshot_revert(sr_snapshot *snap);
/* Introspection (tests, metrics): requested cpu/mem/eph, pod count of a spot node. */
sr_status sr_snapshot_node_state(const sr_snapshot *snap, int32_t spot_pos, int64_t out_requested[3],
                                 int32_t *out_num_pods);
int32_t   sr_snapshot_num_nodes(const sr_snapshot *snap);

/* ---------------------------------------------------------------- planner */
typedef struct sr_ctx sr_ctx;

/* Created once per process like the predicate checker (rescheduler.go:149).
 * device: HIP device ordinal.  Returns SR_ERR_NO_DEVICE without a GPU. */
sr_status   sr_create(int32_t device, sr_ctx **out);
void        sr_destroy(sr_ctx *ctx);
const char *sr_last_error(const sr_ctx *ctx);
const char *sr_build_info(void);
/* SR_ABI_VERSION the library was built with.  The sr_cluster layout grows at
 * its end between versions (ABI 4 added str_label, the scalar tables, acc_*
 * and spread): a binding compares this with the SR_ABI_VERSION it was built
 * against before its first call and refuses to run on a mismatch, since the
 * library would otherwise read fields past the end of a shorter struct (ABI 5
 * added sr_cluster.volumes and pod_stamp; ABI 6 the sr_timing enc_reused /
 * enc_pod_patches counters, which sr_get_timing writes; ABI 7 sr_timing.ms_collective; ABI 8
 * sr_snapshot_refresh_cached; ABI 9 the sr_timing K2 launch fields). */
int32_t     sr_abi_version(void);

/* Batched findSpotNodeForPod (rescheduler.go:338-353): for each pod, the first
 * spot node (NodeInfoArray order) whose predicates pass against the snapshot
 * as it is; the snapshot is not modified.  out_spot_pos[i] = -1 is "".
 * out_fallback[i] = 1: pod outside the encoded predicate set (not evaluated). */
sr_status sr_find_spot_nodes(sr_ctx *ctx, const sr_snapshot *snap, const sr_cluster *cluster,
                             const int32_t *pods, int32_t n, int32_t *out_spot_pos,
                             uint8_t *out_fallback);

/* canDrainNode (rescheduler.go:357-370): sequential first fit of `pods` in
 * order; each placed pod is added to the snapshot (also on failure, for the
 * pods placed before the failing one — exactly like the reference).
 * *out_fail_pod = -1 (nil error) or the index of the first unplaceable pod.
 * *out_fallback = 1: outside the encoded set; nothing evaluated or modified. */
sr_status sr_can_drain_node(sr_ctx *ctx, sr_snapshot *snap, const sr_cluster *cluster,
                            const int32_t *pods, int32_t n, int32_t *out_node_of_pod,
                            int32_t *out_fail_pod, uint8_t *out_fallback);

/* A batch of on-demand candidates in NodeInfoArray order (rescheduler.go:228),
 * each with its podsForDeletion list (rescheduler.go:231-256). */
typedef struct {
  int32_t        n_cand;
  const int32_t *cand_pod_off;  /* [n_cand+1] */
  const int32_t *cand_pods;     /* pod indices, podsForDeletion order */
  const int32_t *cand_global;   /* optional: global candidate index (sharded runs); NULL = 0..n-1 */
} sr_candidates;

typedef struct {
  /* All indices are global candidate indices. */
  int32_t  winner;          /* the node run() drains: first OK candidate with no unresolved
                               fallback candidate before it; -1 = none (or unresolved) */
  int32_t  first_ok;        /* first candidate whose plan succeeds on the GPU; -1 none */
  int32_t  first_fallback;  /* first candidate flagged SR_CAND_FALLBACK; -1 none */
  int32_t  winner_npods;    /* pods in winner_map (0 if the winner is not local) */
  uint64_t checks;          /* CheckPredicates calls (rescheduler.go:344) the reference's loop makes to reach
                               the same plan of the evaluated candidates: per pod its spot position + 1
                               (findSpotNodeForPod returns at the first fit), the spot-node count for a pod
                               that fits nowhere (canDrainNode returns there).  The device does not evaluate
                               pairs one by one; this is the reference-equivalent work.  Known after a run
                               with status or node_of_pod outputs since the last prepare (0 before). */
  uint64_t fallback_pods;   /* pods of fallback candidates */
  /* optional outputs (NULL = not wanted) */
  int32_t *status;          /* [n_cand] SR_CAND_* or failing pod index */
  int32_t *node_of_pod;     /* [cand_pod_off[n_cand] - cand_pod_off[0]] spot position, -1 not placed */
  int32_t *winner_map;      /* [max pods of a candidate] spot position per pod of first_ok */
  uint64_t checks_dense;    /* candidate pods x spot nodes of the evaluated candidates (dense-equivalent pairs) */
} sr_plan_out;

/* One housekeeping tick's planning segment (rescheduler.go:228-287): every
 * candidate is evaluated from the same base snapshot (Fork / canDrainNode /
 * Revert), all in parallel on the GPU.  The snapshot is not modified. */
sr_status sr_plan(sr_ctx *ctx, const sr_snapshot *snap, const sr_cluster *cluster,
                  const sr_candidates *cands, sr_plan_out *out);

/* The planning segment as run() executes it (rescheduler.go:228-287): the
 * candidates in order until the first whose plan succeeds (drain + break,
 * :280-286).  The device plans prefix batches of 16, 32, 64, ... candidates
 * (the environment variable SR_PREFIX_BATCH sets the first size) and stops
 * after the batch holding the first drainable candidate; a batch's host
 * encoding costs in proportion to its pods, so a tick whose winner comes early
 * encodes little.  Outputs as sr_plan for the evaluated candidates and
 * SR_CAND_SKIPPED for the rest; `checks` / `checks_dense` cover the evaluated
 * ones.  With a communicator every rank passes its shard (cand_global, any
 * partition) and plans the same number of batches: a batch's drainable
 * candidate is the winner once every global index below it has been planned
 * on some rank (the reduced smallest unplanned index lies above it). */
sr_status sr_plan_first(sr_ctx *ctx, const sr_snapshot *snap, const sr_cluster *cluster,
                        const sr_candidates *cands, sr_plan_out *out);

/* Split form of sr_plan for a resident workload (bench): prepare = host
 * encoding + upload; run = device-only tick over the resident buffers
 * (kernels + result download).  The planner keeps what it derived from the
 * spot pool and the pod specs across calls: a prepare encodes
 * only what changed since the previous one. */
sr_status sr_plan_prepare(sr_ctx *ctx, const sr_snapshot *snap, const sr_cluster *cluster,
                          const sr_candidates *cands);
sr_status sr_plan_run(sr_ctx *ctx, sr_plan_out *out);

/* Kernel timing (HIP events on the planner's stream). */
typedef struct {
  int32_t  n_runs;          /* timed runs accumulated */
  double   ms_tables;       /* K0: class / threshold row tables */
  double   ms_placement;    /* K2: feasibility rows + per-candidate first-fit placement */
  double   ms_winner;       /* K3, which writes the result to mapped host memory (ABI 7: without the
                               collective, which is ms_collective) */
  double   ms_pack_host;    /* last sr_plan_prepare host encoding */
  double   ms_upload;       /* last sr_plan_prepare upload */
  uint64_t bytes_tables;    /* algorithmic bytes per K0 launch */
  uint64_t bytes_placement; /* bytes K2 moved in its last launch, counted by the kernel per candidate (records,
                               row heads and scans, node-record windows, outputs); read back by a run with
                               status or node_of_pod outputs (0 before) */
  int32_t  n_pods, n_spot, n_cand, n_words;
  int32_t  n_rows_static, n_rows_threshold, n_classes;
  uint64_t bytes_uploaded;     /* last prepare's H2D bytes (the spot nodes' records only when their state changed) */
  int32_t  enc_new_specs;      /* pod specs the last prepare had never seen (canonicalised) */
  int32_t  enc_static_rebuilt; /* 1: the last prepare rebuilt the spot pool's static view (order, labels, taints) */
  int32_t  enc_state_nodes;    /* spot nodes whose capacity state the last prepare re-encoded */
  int32_t  prefix_batches;     /* batches the last sr_plan_first ran */
  int32_t  enc_memo_pods;      /* candidate pods the last prepare found in its per-pod memo (sr_cluster.pod_stamp) */
  int32_t  enc_reused;         /* 1: the last prepare kept the candidate side of the call before (same stamped
                                * candidate input; ABI 6), updating only capacity-dependent rows and records */
  int32_t  enc_pod_patches;    /* ... and re-pointed this many pod records (uploaded as patches) */
  int32_t  k0_columns;         /* word columns K0 rewrites for the last prepare (-1: every row; -2: no K0, the
                                * tables stand and K2 recomputes the changed nodes' bits; ABI 6) */
  int32_t  k0_rows_moved;      /* ... and threshold rows it rewrites whole */
  int32_t  k0_dirty_nodes;     /* no K0: spot nodes changed since the tables were written */
  double   ms_collective;      /* multi-GPU: the allreduce(min) between K2 and K3 (ABI 7) */
  int32_t  k2_launches;        /* K2 kernels of the last run: 2 = the split launch (domain-path candidates on a
                                * second stream beside the node-order kernel; ABI 9) */
  int32_t  k2_list_by_cost;    /* 1: the last prepare's work list runs in the order of the previous run's K2
                                * wave durations (reused candidate side of a long list; ABI 9) */
  int32_t  k2_coop;            /* candidates of the last run planned by a block of cooperating waves (ABI 9) */
} sr_timing;
/* mask: which kernels sr_plan_run brackets with HIP events (resets the sums):
 * 1 = K0, 2 = K2, 4 = collective (multi-GPU) and K3, timed apart; 0 = no events.  Events are read back lazily, by
 * sr_get_timing / sr_set_timing, so timed runs do not synchronise.  Timestamped dispatches
 * lengthen a tick, so SR_TIME_EVERY(n) samples every n-th run only (n_runs counts sampled runs). */
#define SR_TIME_TABLES      1
#define SR_TIME_PLACEMENT   2
#define SR_TIME_WINNER      4
#define SR_TIME_EVERY(n)    ((n) << 8)
sr_status sr_set_timing(sr_ctx *ctx, int32_t mask);
sr_status sr_get_timing(sr_ctx *ctx, sr_timing *out);

/* Multi-GPU: one process per GPU; candidates sharded by the caller (use
 * cand_global: any partition of the global candidate indices; interleaved
 * c % nranks keeps every rank busy on the early candidates sr_plan_first
 * needs).  With a communicator attached, sr_plan_run reduces first_ok /
 * first_fallback (and, for sr_plan_first, the smallest global index any rank
 * has not planned yet) with one allreduce(min) of three 64-bit words: RCCL
 * over xGMI, or the caller's own collective (sr_comm_init_host). */
#define SR_UNIQUE_ID_BYTES 128
sr_status sr_comm_unique_id(uint8_t out[SR_UNIQUE_ID_BYTES]);
sr_status sr_comm_init(sr_ctx *ctx, const uint8_t id[SR_UNIQUE_ID_BYTES], int32_t nranks, int32_t rank);
/* A caller-provided collective instead of RCCL (the orchestrator's own
 * transport, ranks on several hosts, or tests): fn(user, words, n) replaces
 * words[0..n) by their elementwise minimum over the ranks (every rank calls it
 * with the same n, in the same order) and returns 0 (nonzero: the call fails
 * with SR_ERR_RCCL).  It is called from the thread that called the planner. */
typedef int32_t (*sr_allreduce_min_fn)(void *user, uint64_t *words, int32_t n);
sr_status sr_comm_init_host(sr_ctx *ctx, int32_t nranks, int32_t rank, sr_allreduce_min_fn fn, void *user);
/* The ranks of ONE node reduce through host memory instead (ABI 9): every
 * rank's K2 writes its candidates' outcomes into one POSIX shared-memory
 * segment (`name`, e.g. "/sr-<job>", identical on every rank), mapped into
 * every rank's GPU, and each rank's host walks them in global candidate order
 * up to the first drainable candidate -- no collective call and no K3
 * (rescheduler.go:280-286 stops at the first drainable candidate, whichever
 * rank planned it).  `session`: identical on every rank, fresh
 * for the job (it tags the shared words).  Shards must be interleaved:
 * cand_global[i] = (first + i) * nranks + rank (SR_ERR_INVALID_ARG
 * otherwise); max_cand bounds the candidates of one rank's call
 * (SR_ERR_CAPACITY).  Every rank calls it before any rank plans and plans the
 * same sequence of calls; rank 0's sr_destroy removes the name. */
sr_status sr_comm_init_shm(sr_ctx *ctx, const char *name, uint32_t session, int32_t nranks, int32_t rank,
                           int32_t max_cand);

#ifdef __cplusplus
}
#endif
#endif /* SR_PLANNER_H */
