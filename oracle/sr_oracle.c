/*
 * sr_oracle.c — CPU ORACLE (test infrastructure only; see sr_oracle.h).
 *
 * Deliberately written as a direct, unoptimised restatement: objects are
 * walked one (pod, node) pair at a time exactly as the reference's predicate
 * loop does, with no bitmask encoding, no interning tables and no code shared
 * with the product.
 */
#include "sr_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ===================================================================== */
/* Go 1.16 sort.Slice -> quickSort_func  [upstream: go/src/sort/zfuncversion.go,
 * sort/sort.go]; Go 1.15/1.16 per go.mod:3 and Dockerfile:3. */
typedef struct {
  int32_t *a;
  oracle_less_fn less;
  const void *ctx;
} o_ls;

static int o_less(const o_ls *d, int i, int j) { return d->less(d->ctx, d->a[i], d->a[j]); }
static void o_swap(o_ls *d, int i, int j) {
  int32_t t = d->a[i];
  d->a[i] = d->a[j];
  d->a[j] = t;
}

static void o_insertion_sort(o_ls *d, int a, int b) {
  for (int i = a + 1; i < b; i++)
    for (int j = i; j > a && o_less(d, j, j - 1); j--) o_swap(d, j, j - 1);
}

static void o_sift_down(o_ls *d, int lo, int hi, int first) {
  int root = lo;
  for (;;) {
    int child = 2 * root + 1;
    if (child >= hi) break;
    if (child + 1 < hi && o_less(d, first + child, first + child + 1)) child++;
    if (!o_less(d, first + root, first + child)) return;
    o_swap(d, first + root, first + child);
    root = child;
  }
}

static void o_heap_sort(o_ls *d, int a, int b) {
  int first = a, lo = 0, hi = b - a;
  for (int i = (hi - 1) / 2; i >= 0; i--) o_sift_down(d, i, hi, first);
  for (int i = hi - 1; i >= 0; i--) {
    o_swap(d, first, first + i);
    o_sift_down(d, lo, i, first);
  }
}

/* medianOfThree moves the median of data[m0], data[m1], data[m2] into data[m1]. */
static void o_median_of_three(o_ls *d, int m1, int m0, int m2) {
  if (o_less(d, m1, m0)) o_swap(d, m1, m0);
  if (o_less(d, m2, m1)) {
    o_swap(d, m2, m1);
    if (o_less(d, m1, m0)) o_swap(d, m1, m0);
  }
}

static void o_do_pivot(o_ls *d, int lo, int hi, int *midlo, int *midhi) {
  int m = (int)(((unsigned)lo + (unsigned)hi) >> 1);
  if (hi - lo > 40) {
    int s = (hi - lo) / 8;
    o_median_of_three(d, lo, lo + s, lo + 2 * s);
    o_median_of_three(d, m, m - s, m + s);
    o_median_of_three(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
  }
  o_median_of_three(d, lo, m, hi - 1);

  int pivot = lo;
  int a = lo + 1, c = hi - 1;
  for (; a < c && o_less(d, a, pivot); a++) {
  }
  int b = a;
  for (;;) {
    for (; b < c && !o_less(d, pivot, b); b++) {
    }
    for (; b < c && o_less(d, pivot, c - 1); c--) {
    }
    if (b >= c) break;
    o_swap(d, b, c - 1);
    b++;
    c--;
  }
  int protect = hi - c < 5;
  if (!protect && hi - c < (hi - lo) / 4) {
    int dups = 0;
    if (!o_less(d, pivot, hi - 1)) {
      o_swap(d, c, hi - 1);
      c++;
      dups++;
    }
    if (!o_less(d, b - 1, pivot)) {
      b--;
      dups++;
    }
    if (!o_less(d, m, pivot)) {
      o_swap(d, m, b - 1);
      b--;
      dups++;
    }
    protect = dups > 1;
  }
  if (protect) {
    for (;;) {
      for (; a < b && !o_less(d, b - 1, pivot); b--) {
      }
      for (; a < b && o_less(d, a, pivot); a++) {
      }
      if (a >= b) break;
      o_swap(d, a, b - 1);
      a++;
      b--;
    }
  }
  o_swap(d, pivot, b - 1);
  *midlo = b - 1;
  *midhi = c;
}

static void o_quick_sort(o_ls *d, int a, int b, int max_depth) {
  while (b - a > 12) {
    if (max_depth == 0) {
      o_heap_sort(d, a, b);
      return;
    }
    max_depth--;
    int mlo, mhi;
    o_do_pivot(d, a, b, &mlo, &mhi);
    if (mlo - a < b - mhi) {
      o_quick_sort(d, a, mlo, max_depth);
      a = mhi;
    } else {
      o_quick_sort(d, mhi, b, max_depth);
      b = mlo;
    }
  }
  if (b - a > 1) {
    for (int i = a + 6; i < b; i++)
      if (o_less(d, i, i - 6)) o_swap(d, i, i - 6);
    o_insertion_sort(d, a, b);
  }
}

static int o_max_depth(int n) {
  int depth = 0;
  for (int i = n; i > 0; i >>= 1) depth++;
  return depth * 2;
}

void oracle_go_sort_slice(int32_t *a, int32_t n, oracle_less_fn less, const void *ctx) {
  o_ls d = {a, less, ctx};
  o_quick_sort(&d, 0, n, o_max_depth(n));
}

typedef struct {
  const int64_t *key;
} o_keyctx;
static int o_less_desc(const void *ctx, int32_t x, int32_t y) {
  const int64_t *k = ((const o_keyctx *)ctx)->key;
  return k[x] > k[y];
}
static int o_less_asc(const void *ctx, int32_t x, int32_t y) {
  const int64_t *k = ((const o_keyctx *)ctx)->key;
  return k[x] < k[y];
}
void oracle_go_sort_by_key(int32_t *a, int32_t n, const int64_t *key, int32_t desc) {
  o_keyctx k = {key};
  oracle_go_sort_slice(a, n, desc ? o_less_desc : o_less_asc, &k);
}

/* ===================================================================== */
/* Labels */

/* labels[key] lookup; returns 1 and *val when present. */
static int o_node_label(const sr_cluster *c, int32_t node, int32_t key, int32_t *val) {
  const sr_nodes *N = &c->nodes;
  for (int32_t i = N->label_off[node]; i < N->label_off[node + 1]; i++)
    if (N->label_key[i] == key) {
      *val = N->label_val[i];
      return 1;
    }
  return 0;
}

/* isSpotNode / isOnDemandNode (nodes/nodes.go:168-209): "k" tests presence;
 * "k=v" tests labels[k] == v where a missing key reads as "". */
int32_t oracle_node_has_label(const sr_cluster *c, int32_t node, const sr_node_label *l) {
  int32_t v;
  int found = o_node_label(c, node, l->key, &v);
  if (!l->has_value) return found;
  if (!found) v = c->id_empty;
  return v == l->value;
}

/* validateArgs (rescheduler.go:407-417): more than one '=' is an error. */
int32_t oracle_validate_label_flag(int32_t n_equals_parts) { return n_equals_parts > 2 ? 0 : 1; }

/* ===================================================================== */
/* NewNodeMap (nodes/nodes.go:63-104) */

int32_t oracle_new_node_map(const sr_cluster *c, const sr_node_map_params *p, sr_node_map *out) {
  const sr_nodes *N = &c->nodes;
  const sr_pods *P = &c->pods;
  int32_t nn = N->n, np = P->n;
  /* group pods per node in LIST order */
  int32_t *cnt = (int32_t *)calloc((size_t)nn + 1, sizeof(int32_t));
  for (int32_t i = 0; i < np; i++)
    if (P->node[i] >= 0) cnt[P->node[i] + 1]++;
  for (int32_t i = 0; i < nn; i++) cnt[i + 1] += cnt[i];
  int32_t *listed = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np ? np : 1));
  int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nn ? nn : 1));
  for (int32_t i = 0; i < nn; i++) fill[i] = cnt[i];
  for (int32_t i = 0; i < np; i++)
    if (P->node[i] >= 0) listed[fill[P->node[i]]++] = i;

  int32_t kept = 0, ns = 0, nod = 0;
  int32_t rc = SR_OK;
  for (int32_t node = 0; node < nn; node++) {
    int spot = oracle_node_has_label(c, node, &p->spot);
    out->node_pod_off[node] = kept;
    int64_t requested = 0;
    int32_t start = kept;
    /* getPodsOnNode (nodes/nodes.go:129-145) */
    for (int32_t j = cnt[node]; j < cnt[node + 1]; j++) {
      int32_t pod = listed[j];
      if (!P->has_priority[pod]) { /* int(*Spec.Priority) panics on nil */
        rc = SR_ERR_NIL_PRIORITY;
        goto done;
      }
      if (P->priority[pod] < p->priority_threshold && spot) continue;
      out->node_pod_idx[kept++] = pod;
      requested += P->cpu_sort_milli[pod]; /* calculateRequestedCPU (:149-156) */
    }
    out->requested_cpu[node] = requested;
    out->free_cpu[node] = N->alloc_milli_cpu[node] - requested; /* newNodeInfo (:117) */
    /* sort.Slice(pods, cpu(i) > cpu(j)) (:76-80) */
    oracle_go_sort_by_key(out->node_pod_idx + start, kept - start, P->cpu_sort_milli, 1);
    /* switch: spot first, then on-demand, else dropped (:82-91) */
    if (spot)
      out->spot[ns++] = node;
    else if (oracle_node_has_label(c, node, &p->on_demand))
      out->on_demand[nod++] = node;
  }
  out->node_pod_off[nn] = kept;
  oracle_go_sort_by_key(out->spot, ns, out->requested_cpu, 1);      /* :95-97 */
  oracle_go_sort_by_key(out->on_demand, nod, out->requested_cpu, 0); /* :99-101 */
  *out->n_spot = ns;
  *out->n_on_demand = nod;
done:
  free(cnt);
  free(listed);
  free(fill);
  return rc;
}

void oracle_build_candidates(const sr_cluster *c, const sr_node_map *m, int32_t *cand_off,
                             int32_t *cand_pods) {
  int32_t k = 0;
  for (int32_t i = 0; i < *m->n_on_demand; i++) {
    int32_t node = m->on_demand[i];
    cand_off[i] = k;
    for (int32_t j = m->node_pod_off[node]; j < m->node_pod_off[node + 1]; j++) {
      int32_t pod = m->node_pod_idx[j];
      uint32_t f = c->pods.flags[pod];
      if (f & (SR_POD_MIRROR | SR_POD_DAEMONSET_CONTROLLER)) continue;
      cand_pods[k++] = pod;
    }
  }
  cand_off[*m->n_on_demand] = k;
}

/* ===================================================================== */
/* GetPodsForDeletionOnNodeDrain [upstream CA utils/drain/drain.go @03f60a4c3818]
 * as called at rescheduler.go:231 (checkReferences = false, no listers,
 * minReplica 0), and the loop of rescheduler.go:240-256. */

/* pod_util.IsDaemonSetPod: a DaemonSet ControllerRef, or the annotation */
static int o_is_daemonset_pod(uint32_t f) {
  return (f & SR_DRAIN_CTRL_MASK) == SR_DRAIN_CTRL_DAEMONSET || (f & SR_DRAIN_DAEMONSET_ANNOTATION) != 0;
}

/* drain.IsPodLongTerminating: deletionTimestamp + grace (default 30 s) + 30 s before now */
static int o_long_terminating(const sr_pod_drain *d, int32_t pod) {
  if (!(d->flags[pod] & SR_DRAIN_DELETING)) return 0;
  long double grace = d->grace_seconds[pod] < 0 ? 30.0L : (long double)d->grace_seconds[pod];
  return (long double)d->deletion_age_ns[pod] > (grace + 30.0L) * 1e9L;
}

/* drain.isPodTerminal */
static int o_terminal(const sr_pod_drain *d, int32_t pod) {
  int ph = d->phase[pod], rp = d->restart_policy[pod];
  if (rp == SR_RESTART_NEVER && (ph == SR_PHASE_SUCCEEDED || ph == SR_PHASE_FAILED)) return 1;
  if (rp == SR_RESTART_ON_FAILURE && ph == SR_PHASE_SUCCEEDED) return 1;
  return ph == SR_PHASE_FAILED;
}

/* GetPodsForDeletionOnNodeDrain over one node's pods: returns the blocking pod
 * (its reason in *reason) or -1 with the pods appended to out[*n]. */
static int32_t o_get_pods_for_deletion(const sr_cluster *c, const sr_pod_drain *d, const sr_drain_params *prm,
                                       const int32_t *pods, int32_t np, int32_t *out, int32_t *n, int32_t *reason) {
  *n = 0;
  *reason = SR_BLOCK_NONE;
  for (int32_t i = 0; i < np; i++) {
    int32_t pod = pods[i];
    uint32_t f = d->flags[pod];
    if (c->pods.flags[pod] & SR_POD_MIRROR) continue;
    if (o_long_terminating(d, pod)) continue;
    int replicated = 0, is_ds = 0;
    uint32_t kind = f & SR_DRAIN_CTRL_MASK;
    if (kind == SR_DRAIN_CTRL_REPLICATION_CONTROLLER) {
      replicated = 1;
    } else if (o_is_daemonset_pod(f)) {
      is_ds = 1;
    } else if (kind == SR_DRAIN_CTRL_JOB) {
      replicated = 1;
    } else if (kind == SR_DRAIN_CTRL_REPLICASET) {
      replicated = 1;
    } else if (kind == SR_DRAIN_CTRL_STATEFULSET) {
      replicated = 1;
    }
    if (is_ds) continue;
    if (!(f & SR_DRAIN_SAFE_TO_EVICT) && !o_terminal(d, pod)) {
      if (!replicated) {
        *reason = SR_BLOCK_NOT_REPLICATED;
        return pod;
      }
      if ((f & SR_DRAIN_KUBE_SYSTEM) && prm->skip_nodes_with_system_pods) {
        if (f & SR_DRAIN_PDB_ERROR) {
          *reason = SR_BLOCK_UNEXPECTED_ERROR;
          return pod;
        }
        if (!(f & SR_DRAIN_KUBE_SYSTEM_PDB)) {
          *reason = SR_BLOCK_UNMOVABLE_KUBE_SYSTEM;
          return pod;
        }
      }
      if ((f & SR_DRAIN_LOCAL_STORAGE) && prm->skip_nodes_with_local_storage) {
        *reason = SR_BLOCK_LOCAL_STORAGE;
        return pod;
      }
      if (f & SR_DRAIN_NOT_SAFE_TO_EVICT) {
        *reason = SR_BLOCK_NOT_SAFE_TO_EVICT;
        return pod;
      }
    }
    out[(*n)++] = pod;
  }
  return -1;
}

int32_t oracle_pods_for_deletion(const sr_cluster *c, const sr_pod_drain *d, const sr_drain_params *prm,
                                 const int32_t *nodes, int32_t n_nodes, const int32_t *node_pod_off,
                                 const int32_t *node_pod_idx, int32_t *cand_off, int32_t *cand_pods,
                                 int32_t *block_pod, int32_t *block_reason) {
  if (d->n != c->pods.n) return SR_ERR_INVALID_ARG;
  int32_t k = 0;
  int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(c->pods.n > 0 ? c->pods.n : 1));
  for (int32_t i = 0; i < n_nodes; i++) {
    int32_t node = nodes[i], n = 0;
    cand_off[i] = k;
    block_pod[i] = o_get_pods_for_deletion(c, d, prm, node_pod_idx + node_pod_off[node],
                                           node_pod_off[node + 1] - node_pod_off[node], tmp, &n, &block_reason[i]);
    if (block_pod[i] >= 0) continue; /* glog + continue (rescheduler.go:232-238) */
    if (!prm->owner_filter) { /* updateSpotNodeMetrics counts the CA's list as is (rescheduler.go:391-396) */
      for (int32_t q = 0; q < n; q++) cand_pods[k++] = tmp[q];
      continue;
    }
    for (int32_t q = 0; q < n; q++) {
      int32_t pod = tmp[q];
      if (d->flags[pod] & SR_DRAIN_NIL_CONTROLLER) { /* *owner.Controller with Controller == nil */
        free(tmp);
        return SR_ERR_NIL_CONTROLLER;
      }
      if (c->pods.flags[pod] & SR_POD_DAEMONSET_CONTROLLER) continue; /* controlledByDaemonSet */
      cand_pods[k++] = pod;
    }
  }
  cand_off[n_nodes] = k;
  free(tmp);
  return SR_OK;
}

/* ===================================================================== */
/* Cluster snapshot [upstream CA simulator BasicClusterSnapshot/DeltaClusterSnapshot
 * over scheduler NodeInfo]: per node Requested (cpu, mem, eph), len(Pods),
 * UsedPorts, and whether any pod carries required anti-affinity. */
typedef struct {
  int32_t ip, proto, port;
} o_port;

typedef struct {
  int64_t req[3];
  int32_t npods;
  int32_t anti;  /* pods with SR_POD_HAS_REQ_ANTI_AFFINITY */
  int32_t opaque; /* of those, pods whose terms the planner cannot read (o_anti_opaque) */
  int32_t nports, cap;
  o_port *ports;
  int32_t nlist, lcap; /* NodeInfo.Pods (InterPodAffinity matches against them) */
  int32_t *list;
  int32_t nsc, sccap;  /* Requested.ScalarResources as (name, amount) entries, one per AddPod entry */
  int32_t *sc_name;
  int64_t *sc_val;
  int32_t sc_unknown;  /* pods added without scalar tables that carry scalar requests */
} o_state;

struct oracle_snapshot {
  int32_t n;
  int32_t *node; /* cluster node index per position */
  o_state *st;
  o_state *saved;
  int32_t forked;
  int32_t anti_total;
  int32_t opaque_total;
  int32_t sc_unknown_total;
  /* Allocatable scalar resources per position, copied at AddNodeWithPods */
  int32_t *alloc_off, *alloc_name;
  int64_t *alloc_val;
  /* the attachable volumes (limit key << 32 | unique name) of every pod the
   * snapshot holds, sorted; rebuilt on demand after a change (planner limit:
   * a candidate pod whose attachable volume is already on a spot node) */
  uint64_t *vb;
  int32_t vb_n, vb_valid;
};

/* labels.NewRequirement's validateLabelKey (validation.IsQualifiedName) /
 * validateLabelValue (validation.IsValidLabelValue) [upstream apimachinery
 * v0.19.2 labels/selector.go], through the shim's table (sr_cluster.str_label).
 * Without a table the strings' validity is unknown: callers treat the
 * requirement as unverifiable (fallback). */
static int o_label_ok(const sr_cluster *c, int32_t id, uint8_t what) {
  return c->str_label && id >= 0 && id < c->n_strings && (c->str_label[id] & what) == what;
}

static int o_req_strings_ok(const sr_cluster *c, int32_t key, const int32_t *vals, int32_t lo, int32_t hi) {
  if (!o_label_ok(c, key, SR_STR_LABEL_KEY)) return 0;
  for (int32_t v = lo; v < hi; v++)
    if (!o_label_ok(c, vals[v], SR_STR_LABEL_VALUE)) return 0;
  return 1;
}

/* A term whose label selector fails metav1.LabelSelectorAsSelector [upstream
 * apimachinery v0.19.2]: NewRequirement(key, op, values) on every matchLabels
 * pair (Equals) and matchExpression -- the key a qualified name, every value a
 * valid label value, In/NotIn with values, Exists/DoesNotExist without, no
 * other operator. */
static int o_term_invalid(const sr_cluster *c, int32_t t) {
  const sr_pod_affinity *A = c->pod_affinity;
  if (A->selector_nil[t]) return 0;
  for (int32_t i = A->ml_off[t]; i < A->ml_off[t + 1]; i++) {
    if (A->ml_key[i] == c->id_empty && c->id_empty != -1) return 1;
    if (!o_req_strings_ok(c, A->ml_key[i], A->ml_val, i, i + 1)) return 1;
  }
  for (int32_t e = A->me_off[t]; e < A->me_off[t + 1]; e++) {
    int32_t nv = A->me_val_off[e + 1] - A->me_val_off[e], op = A->me_op[e];
    if (A->me_key[e] == c->id_empty && c->id_empty != -1) return 1;
    if (!o_req_strings_ok(c, A->me_key[e], A->me_vals, A->me_val_off[e], A->me_val_off[e + 1])) return 1;
    if ((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 0) return 1;
    if ((op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) && nv != 0) return 1;
    if (op != SR_OP_IN && op != SR_OP_NOT_IN && op != SR_OP_EXISTS && op != SR_OP_DOES_NOT_EXIST) return 1;
  }
  return 0;
}

/* A pod whose required anti-affinity the encoded set cannot evaluate: no
 * sr_pod_affinity at all, the flag without terms, or a term whose label
 * selector fails LabelSelectorAsSelector [upstream apimachinery
 * metav1.LabelSelectorAsSelector: In/NotIn need values, Exists/DoesNotExist
 * take none, other operators and empty keys are errors]. */
static int o_anti_opaque(const sr_cluster *c, int32_t pod) {
  if (!(c->pods.flags[pod] & SR_POD_HAS_REQ_ANTI_AFFINITY)) return 0;
  const sr_pod_affinity *A = c->pod_affinity;
  if (!A || A->anti_off[pod] == A->anti_off[pod + 1]) return 1;
  for (int32_t t = A->anti_off[pod]; t < A->anti_off[pod + 1]; t++)
    if (o_term_invalid(c, t)) return 1;
  return 0;
}

/* Required pod affinity the planner cannot evaluate: a selector that fails to build. */
static int o_aff_opaque(const sr_cluster *c, int32_t pod) {
  const sr_pod_affinity *A = c->pod_affinity;
  if (!A || !A->aff_off) return 0;
  for (int32_t t = A->aff_off[pod]; t < A->aff_off[pod + 1]; t++)
    if (o_term_invalid(c, t)) return 1;
  return 0;
}

static int64_t o_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* What NodeInfo.AddPod adds to Requested (calculateResource [upstream k8s
 * v1.19.2 framework/v1alpha1/types.go]); the shim's acc_* table, else the
 * fit request. */
static int64_t o_acc(const sr_cluster *c, int32_t pod, int r) {
  const sr_pods *P = &c->pods;
  if (r == 0) return c->acc_milli_cpu ? c->acc_milli_cpu[pod] : P->req_milli_cpu[pod];
  if (r == 1) return c->acc_memory ? c->acc_memory[pod] : P->req_memory[pod];
  return c->acc_ephemeral ? c->acc_ephemeral[pod] : P->req_ephemeral[pod];
}

static int o_has_scalars(const sr_cluster *c, int32_t pod) {
  return c->pod_scalar_off && c->pod_scalar_off[pod + 1] > c->pod_scalar_off[pod];
}

static void o_state_add_pod(o_state *st, const sr_cluster *c, int32_t pod) {
  const sr_pods *P = &c->pods;
  for (int r = 0; r < 3; r++) st->req[r] = o_add(st->req[r], o_acc(c, pod, r));
  if (o_has_scalars(c, pod)) {
    for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; i++) {
      if (st->nsc == st->sccap) {
        st->sccap = st->sccap ? st->sccap * 2 : 4;
        st->sc_name = (int32_t *)realloc(st->sc_name, sizeof(int32_t) * (size_t)st->sccap);
        st->sc_val = (int64_t *)realloc(st->sc_val, sizeof(int64_t) * (size_t)st->sccap);
      }
      st->sc_name[st->nsc] = c->pod_scalar_name[i];
      st->sc_val[st->nsc] = c->pod_scalar_acc[i];
      st->nsc++;
    }
  } else if (!c->pod_scalar_off && (P->flags[pod] & SR_POD_FB_SCALAR_RESOURCES)) {
    st->sc_unknown++;
  }
  st->npods++;
  if ((P->flags[pod] & SR_POD_HAS_REQ_ANTI_AFFINITY) ||
      (c->pod_affinity && c->pod_affinity->anti_off[pod + 1] > c->pod_affinity->anti_off[pod]))
    st->anti++;
  if (o_anti_opaque(c, pod)) st->opaque++;
  if (st->nlist == st->lcap) {
    st->lcap = st->lcap ? st->lcap * 2 : 8;
    st->list = (int32_t *)realloc(st->list, sizeof(int32_t) * (size_t)st->lcap);
  }
  st->list[st->nlist++] = pod;
  for (int32_t i = P->port_off[pod]; i < P->port_off[pod + 1]; i++) {
    if (P->port_num[i] <= 0) continue; /* HostPortInfo.Add ignores port <= 0 */
    if (st->nports == st->cap) {
      st->cap = st->cap ? st->cap * 2 : 4;
      st->ports = (o_port *)realloc(st->ports, sizeof(o_port) * (size_t)st->cap);
    }
    st->ports[st->nports].ip = P->port_ip[i];
    st->ports[st->nports].proto = P->port_proto[i];
    st->ports[st->nports].port = P->port_num[i];
    st->nports++;
  }
}

oracle_snapshot *oracle_snapshot_create(const sr_cluster *c, const int32_t *spot, int32_t n_spot,
                                        const int32_t *node_pod_off, const int32_t *node_pod_idx) {
  oracle_snapshot *s = (oracle_snapshot *)calloc(1, sizeof(*s));
  s->n = n_spot;
  s->node = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_spot ? n_spot : 1));
  s->st = (o_state *)calloc((size_t)(n_spot ? n_spot : 1), sizeof(o_state));
  for (int32_t i = 0; i < n_spot; i++) {
    int32_t node = spot[i];
    s->node[i] = node;
    /* AddNodeWithPods(node.Node, node.Pods) (nodes/nodes.go:229) */
    for (int32_t j = node_pod_off[node]; j < node_pod_off[node + 1]; j++)
      o_state_add_pod(&s->st[i], c, node_pod_idx[j]);
    s->anti_total += s->st[i].anti;
    s->opaque_total += s->st[i].opaque;
    s->sc_unknown_total += s->st[i].sc_unknown;
  }
  s->alloc_off = (int32_t *)calloc((size_t)n_spot + 1, sizeof(int32_t));
  int32_t total = 0;
  for (int32_t i = 0; i < n_spot; i++) {
    s->alloc_off[i] = total;
    if (c->node_scalar_off) total += c->node_scalar_off[spot[i] + 1] - c->node_scalar_off[spot[i]];
  }
  s->alloc_off[n_spot] = total;
  s->alloc_name = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total ? total : 1));
  s->alloc_val = (int64_t *)malloc(sizeof(int64_t) * (size_t)(total ? total : 1));
  for (int32_t i = 0; i < n_spot && c->node_scalar_off; i++)
    for (int32_t j = c->node_scalar_off[spot[i]], k = s->alloc_off[i]; j < c->node_scalar_off[spot[i] + 1]; j++, k++) {
      s->alloc_name[k] = c->node_scalar_name[j];
      s->alloc_val[k] = c->node_scalar_alloc[j];
    }
  return s;
}

static void o_free_states(o_state *st, int32_t n) {
  if (!st) return;
  for (int32_t i = 0; i < n; i++) {
    free(st[i].ports);
    free(st[i].list);
    free(st[i].sc_name);
    free(st[i].sc_val);
  }
  free(st);
}

static o_state *o_copy_states(const o_state *src, int32_t n) {
  o_state *dst = (o_state *)calloc((size_t)(n ? n : 1), sizeof(o_state));
  for (int32_t i = 0; i < n; i++) {
    dst[i] = src[i];
    dst[i].ports = NULL;
    if (src[i].nports) {
      dst[i].ports = (o_port *)malloc(sizeof(o_port) * (size_t)src[i].cap);
      memcpy(dst[i].ports, src[i].ports, sizeof(o_port) * (size_t)src[i].nports);
    }
    dst[i].list = NULL;
    if (src[i].nlist) {
      dst[i].list = (int32_t *)malloc(sizeof(int32_t) * (size_t)src[i].lcap);
      memcpy(dst[i].list, src[i].list, sizeof(int32_t) * (size_t)src[i].nlist);
    }
    dst[i].sc_name = NULL;
    dst[i].sc_val = NULL;
    if (src[i].nsc) {
      dst[i].sc_name = (int32_t *)malloc(sizeof(int32_t) * (size_t)src[i].sccap);
      dst[i].sc_val = (int64_t *)malloc(sizeof(int64_t) * (size_t)src[i].sccap);
      memcpy(dst[i].sc_name, src[i].sc_name, sizeof(int32_t) * (size_t)src[i].nsc);
      memcpy(dst[i].sc_val, src[i].sc_val, sizeof(int64_t) * (size_t)src[i].nsc);
    }
  }
  return dst;
}

void oracle_snapshot_destroy(oracle_snapshot *s) {
  if (!s) return;
  o_free_states(s->st, s->n);
  o_free_states(s->saved, s->n);
  free(s->node);
  free(s->alloc_off);
  free(s->alloc_name);
  free(s->alloc_val);
  free(s->vb);
  free(s);
}

void oracle_snapshot_add_pod(oracle_snapshot *s, const sr_cluster *c, int32_t pod, int32_t pos) {
  int32_t before = s->st[pos].anti, obefore = s->st[pos].opaque, ubefore = s->st[pos].sc_unknown;
  s->vb_valid = 0;
  o_state_add_pod(&s->st[pos], c, pod);
  s->anti_total += s->st[pos].anti - before;
  s->opaque_total += s->st[pos].opaque - obefore;
  s->sc_unknown_total += s->st[pos].sc_unknown - ubefore;
}

int32_t oracle_snapshot_fork(oracle_snapshot *s) {
  if (s->forked) return SR_ERR_STATE; /* DeltaClusterSnapshot: one level */
  s->saved = o_copy_states(s->st, s->n);
  s->forked = 1;
  return SR_OK;
}

int32_t oracle_snapshot_revert(oracle_snapshot *s) {
  if (!s->forked) return SR_OK; /* Revert without Fork is a no-op in the CA snapshot */
  o_free_states(s->st, s->n);
  s->st = s->saved;
  s->saved = NULL;
  s->forked = 0;
  s->vb_valid = 0;
  s->anti_total = s->opaque_total = s->sc_unknown_total = 0;
  for (int32_t i = 0; i < s->n; i++) {
    s->anti_total += s->st[i].anti;
    s->opaque_total += s->st[i].opaque;
    s->sc_unknown_total += s->st[i].sc_unknown;
  }
  return SR_OK;
}

void oracle_snapshot_node_state(const oracle_snapshot *s, int32_t pos, int64_t req[3], int32_t *npods) {
  req[0] = s->st[pos].req[0];
  req[1] = s->st[pos].req[1];
  req[2] = s->st[pos].req[2];
  *npods = s->st[pos].npods;
}

/* ===================================================================== */
/* Predicates: k8s v1.19.2 filter plugins [upstream], one (pod, node) pair. */

/* v1.Toleration.ToleratesTaint [upstream k8s.io/api/core/v1/toleration.go] */
static int o_tolerates(const sr_cluster *c, int32_t pod, int32_t key, int32_t val, int32_t effect) {
  const sr_pods *P = &c->pods;
  for (int32_t t = P->tol_off[pod]; t < P->tol_off[pod + 1]; t++) {
    int32_t te = P->tol_effect[t];
    if (te != SR_EFFECT_EMPTY && (te != effect || te == SR_EFFECT_OTHER)) continue;
    int32_t tk = P->tol_key[t];
    if (tk != c->id_empty && tk != key) continue; /* len(t.Key) > 0 && t.Key != taint.Key */
    switch (P->tol_op[t]) {
      case SR_TOL_EQUAL:
        if (P->tol_val[t] == val) return 1;
        break;
      case SR_TOL_EXISTS:
        return 1;
      default:
        break;
    }
  }
  return 0;
}

/* NodeUnschedulable.Filter [upstream plugins/nodeunschedulable] */
static int o_unschedulable_ok(const sr_cluster *c, int32_t pod, int32_t node) {
  if (!c->nodes.unschedulable[node]) return 1;
  return o_tolerates(c, pod, c->id_unschedulable_key, c->id_empty, SR_EFFECT_NO_SCHEDULE);
}

/* TaintToleration.Filter: FindMatchingUntoleratedTaint over NoSchedule/NoExecute taints. */
static int o_taints_ok(const sr_cluster *c, int32_t pod, int32_t node) {
  const sr_nodes *N = &c->nodes;
  for (int32_t t = N->taint_off[node]; t < N->taint_off[node + 1]; t++) {
    int32_t e = N->taint_effect[t];
    if (e != SR_EFFECT_NO_SCHEDULE && e != SR_EFFECT_NO_EXECUTE) continue;
    if (!o_tolerates(c, pod, N->taint_key[t], N->taint_val[t], e)) return 0;
  }
  return 1;
}

static int o_in_values(const int32_t *vals, int32_t lo, int32_t hi, int32_t v) {
  for (int32_t i = lo; i < hi; i++)
    if (vals[i] == v) return 1;
  return 0;
}

/* strconv.ParseInt(string id, 10, 64), through the shim's table of the
 * interned strings' integer values (sr_cluster.str_int). */
static int o_str_int(const sr_cluster *c, int32_t id, int64_t *v) {
  if (!c->str_int || !c->str_int_ok || id < 0 || id >= c->n_strings || !c->str_int_ok[id]) return 0;
  *v = c->str_int[id];
  return 1;
}

/* labels.NewRequirement validation + Requirement.Matches [upstream apimachinery labels]. */
static int o_expr_valid(const sr_cluster *c, int32_t e) {
  const sr_pods *P = &c->pods;
  int32_t nv = P->expr_val_off[e + 1] - P->expr_val_off[e];
  if (P->expr_key[e] == c->id_empty && c->id_empty != -1) return 0; /* empty key fails validateLabelKey */
  /* validateLabelKey(key), then (after the operator's arity / integer checks)
   * validateLabelValue on every value: any failure fails the term */
  if (!o_req_strings_ok(c, P->expr_key[e], P->expr_vals, P->expr_val_off[e], P->expr_val_off[e + 1])) return 0;
  switch (P->expr_op[e]) {
    case SR_OP_IN:
    case SR_OP_NOT_IN:
      return nv > 0;
    case SR_OP_EXISTS:
    case SR_OP_DOES_NOT_EXIST:
      return nv == 0;
    case SR_OP_GT:
    case SR_OP_LT: {
      /* labels.NewRequirement: exactly one value, and it parses as an int64 */
      int64_t x;
      return nv == 1 && o_str_int(c, P->expr_vals[P->expr_val_off[e]], &x);
    }
    default:
      return 0; /* unknown operator: the term fails to build */
  }
}

static int o_expr_match(const sr_cluster *c, int32_t e, int32_t node) {
  const sr_pods *P = &c->pods;
  int32_t v;
  int has = o_node_label(c, node, P->expr_key[e], &v);
  int32_t lo = P->expr_val_off[e], hi = P->expr_val_off[e + 1];
  int64_t lv, rv;
  switch (P->expr_op[e]) {
    case SR_OP_GT: /* labels.Requirement.Matches: the node's value must parse too */
      return has && o_str_int(c, v, &lv) && o_str_int(c, P->expr_vals[lo], &rv) && lv > rv;
    case SR_OP_LT:
      return has && o_str_int(c, v, &lv) && o_str_int(c, P->expr_vals[lo], &rv) && lv < rv;
    case SR_OP_IN:
      return has && o_in_values(P->expr_vals, lo, hi, v);
    case SR_OP_NOT_IN:
      return !has || !o_in_values(P->expr_vals, lo, hi, v);
    case SR_OP_EXISTS:
      return has;
    case SR_OP_DOES_NOT_EXIST:
      return !has;
    default:
      return 0;
  }
}

/* NodeSelectorRequirementsAsFieldSelector: In/NotIn with exactly one value
 * against fields.Set{"metadata.name": node.Name}. */
static int o_field_valid(const sr_cluster *c, int32_t f) {
  const sr_pods *P = &c->pods;
  int32_t nv = P->field_val_off[f + 1] - P->field_val_off[f];
  int32_t op = P->field_op[f];
  return (op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 1;
}

static int o_field_match(const sr_cluster *c, int32_t f, int32_t node) {
  const sr_pods *P = &c->pods;
  int32_t fv = (P->field_key[f] == c->id_metadata_name && c->id_metadata_name != -1)
                   ? c->nodes.name[node]
                   : c->id_empty;
  int32_t want = P->field_vals[P->field_val_off[f]];
  int eq = (fv == want) && fv != -1;
  return P->field_op[f] == SR_OP_IN ? eq : !eq;
}

/* NodeAffinity.Filter = PodMatchesNodeSelectorAndAffinityTerms [upstream
 * pkg/scheduler/framework/plugins/helper/node_affinity.go]. */
static int o_affinity_ok(const sr_cluster *c, int32_t pod, int32_t node) {
  const sr_pods *P = &c->pods;
  for (int32_t i = P->sel_off[pod]; i < P->sel_off[pod + 1]; i++) {
    int32_t v;
    if (!o_node_label(c, node, P->sel_key[i], &v) || v != P->sel_val[i]) return 0;
  }
  if (!P->aff_required[pod]) return 1;
  for (int32_t t = P->term_off[pod]; t < P->term_off[pod + 1]; t++) {
    int32_t e0 = P->term_expr_off[t], e1 = P->term_expr_off[t + 1];
    int32_t f0 = P->term_field_off[t], f1 = P->term_field_off[t + 1];
    if (e0 == e1 && f0 == f1) continue; /* nil or empty term selects no objects */
    int ok = 1;
    if (e1 > e0) {
      for (int32_t e = e0; e < e1 && ok; e++)
        if (!o_expr_valid(c, e)) ok = 0;
      for (int32_t e = e0; e < e1 && ok; e++)
        if (!o_expr_match(c, e, node)) ok = 0;
    }
    if (ok && f1 > f0) {
      for (int32_t f = f0; f < f1 && ok; f++)
        if (!o_field_valid(c, f)) ok = 0;
      for (int32_t f = f0; f < f1 && ok; f++)
        if (!o_field_match(c, f, node)) ok = 0;
    }
    if (ok) return 1;
  }
  return 0;
}

/* NodePorts.Filter: HostPortInfo.CheckConflict [upstream framework/types.go]. */
static int o_ports_ok(const o_state *st, const sr_cluster *c, int32_t pod) {
  const sr_pods *P = &c->pods;
  for (int32_t i = P->port_off[pod]; i < P->port_off[pod + 1]; i++) {
    int32_t ip = P->port_ip[i], proto = P->port_proto[i], port = P->port_num[i];
    if (port <= 0) continue;
    for (int32_t j = 0; j < st->nports; j++) {
      const o_port *u = &st->ports[j];
      if (u->proto != proto || u->port != port) continue;
      if (ip == -1) return 0;                    /* 0.0.0.0 conflicts with any IP */
      if (u->ip == -1 || u->ip == ip) return 0;  /* else 0.0.0.0 or the same IP */
    }
  }
  return 1;
}

/* NodeResourcesFit.Filter: fitsRequest [upstream k8s v1.19.2
 * plugins/noderesources/fit.go]: the pod count, then -- unless cpu, memory,
 * ephemeral storage are all zero and no scalar resource is listed -- every
 * resource: Allocatable < request + Requested fails; for each listed scalar
 * resource the node's Allocatable.ScalarResources (0 when absent) against
 * the request plus Requested.ScalarResources. */
static int o_resources_ok(const oracle_snapshot *s, const o_state *st, const sr_cluster *c, int32_t pod, int32_t pos,
                          int32_t node) {
  const sr_pods *P = &c->pods;
  const sr_nodes *N = &c->nodes;
  if ((int64_t)st->npods + 1 > N->alloc_pods[node]) return 0;
  int64_t rc = P->req_milli_cpu[pod], rm = P->req_memory[pod], re = P->req_ephemeral[pod];
  if (rc == 0 && rm == 0 && re == 0 && !o_has_scalars(c, pod)) return 1;
  if (N->alloc_milli_cpu[node] < o_add(rc, st->req[0])) return 0;
  if (N->alloc_memory[node] < o_add(rm, st->req[1])) return 0;
  if (N->alloc_ephemeral[node] < o_add(re, st->req[2])) return 0;
  if (o_has_scalars(c, pod))
    for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; i++) {
      int32_t name = c->pod_scalar_name[i];
      int64_t alloc = 0, used = 0;
      for (int32_t k = s->alloc_off[pos]; k < s->alloc_off[pos + 1]; k++)
        if (s->alloc_name[k] == name) alloc = s->alloc_val[k];
      for (int32_t k = 0; k < st->nsc; k++)
        if (st->sc_name[k] == name) used = o_add(used, st->sc_val[k]);
      if (alloc < o_add(c->pod_scalar_req[i], used)) return 0;
    }
  return 1;
}

/* labels.Selector.Matches over a pod's labels for term t (MatchLabels are
 * Equals requirements; MatchExpressions In / NotIn / Exists / DoesNotExist;
 * a nil selector selects nothing, an empty one everything). */
static int o_pod_label(const sr_cluster *c, int32_t pod, int32_t key, int32_t *val) {
  const sr_pod_affinity *A = c->pod_affinity;
  for (int32_t i = A->label_off[pod]; i < A->label_off[pod + 1]; i++)
    if (A->label_key[i] == key) {
      *val = A->label_val[i];
      return 1;
    }
  return 0;
}

static int o_selector_matches(const sr_cluster *c, int32_t t, int32_t pod) {
  const sr_pod_affinity *A = c->pod_affinity;
  if (A->selector_nil[t]) return 0;
  for (int32_t i = A->ml_off[t]; i < A->ml_off[t + 1]; i++) {
    int32_t v;
    if (!o_pod_label(c, pod, A->ml_key[i], &v) || v != A->ml_val[i]) return 0;
  }
  for (int32_t e = A->me_off[t]; e < A->me_off[t + 1]; e++) {
    int32_t v;
    int has = o_pod_label(c, pod, A->me_key[e], &v);
    int32_t lo = A->me_val_off[e], hi = A->me_val_off[e + 1];
    int ok;
    switch (A->me_op[e]) {
      case SR_OP_IN: ok = has && o_in_values(A->me_vals, lo, hi, v); break;
      case SR_OP_NOT_IN: ok = !has || !o_in_values(A->me_vals, lo, hi, v); break;
      case SR_OP_EXISTS: ok = has; break;
      case SR_OP_DOES_NOT_EXIST: ok = !has; break;
      default: ok = 0; break;
    }
    if (!ok) return 0;
  }
  return 1;
}

/* schedutil.PodMatchesTermsNamespaceAndSelector for the term t of `owner`
 * against `target`: namespace in the term's Namespaces (none: the owner's
 * namespace, getNamespacesFromPodAffinityTerm) and the selector matches. */
static int o_term_matches(const sr_cluster *c, int32_t owner, int32_t t, int32_t target) {
  const sr_pod_affinity *A = c->pod_affinity;
  int32_t tns = A->ns[target];
  if (A->ns_off[t] == A->ns_off[t + 1]) {
    if (tns != A->ns[owner]) return 0;
  } else if (!o_in_values(A->ns_ids, A->ns_off[t], A->ns_off[t + 1], tns)) {
    return 0;
  }
  return o_selector_matches(c, t, target);
}

/* InterPodAffinity.Filter, required anti-affinity part [upstream k8s v1.19.2
 * plugins/interpodaffinity/filtering.go]: PreFilter counts topology pairs
 * (key, value of the existing pod's node) for (1) every existing pod's
 * anti-affinity term that matches the incoming pod and (2) every anti-affinity
 * term of the incoming pod that matches an existing pod; Filter rejects a node
 * whose value for such a pair's key equals the pair's value.  Existing pods =
 * NodeInfo.Pods of every snapshot node.  (Required pod *affinity* stays on the
 * fallback path.) */
static int o_interpod_ok(const o_state *st, const int32_t *node, int32_t n, const sr_cluster *c, int32_t pod,
                         int32_t nnode) {
  const sr_pod_affinity *A = c->pod_affinity;
  if (!A || A->anti_off[c->pods.n] == 0) return 1; /* no term anywhere */
  for (int32_t m = 0; m < n; m++) {
    if (st[m].anti == 0) continue;
    for (int32_t j = 0; j < st[m].nlist; j++) {
      int32_t e = st[m].list[j];
      for (int32_t t = A->anti_off[e]; t < A->anti_off[e + 1]; t++) {
        int32_t vm, vn;
        if (!o_node_label(c, node[m], A->topology_key[t], &vm)) continue;
        if (!o_node_label(c, nnode, A->topology_key[t], &vn) || vn != vm) continue;
        if (o_term_matches(c, e, t, pod)) return 0;
      }
    }
  }
  for (int32_t t = A->anti_off[pod]; t < A->anti_off[pod + 1]; t++) {
    int32_t vn;
    if (!o_node_label(c, nnode, A->topology_key[t], &vn)) continue;
    for (int32_t m = 0; m < n; m++) {
      int32_t vm;
      if (!o_node_label(c, node[m], A->topology_key[t], &vm) || vm != vn) continue;
      for (int32_t j = 0; j < st[m].nlist; j++)
        if (o_term_matches(c, pod, t, st[m].list[j])) return 0;
    }
  }
  return 1;
}

/* InterPodAffinity.Filter, required affinity part [upstream k8s v1.19.2
 * plugins/interpodaffinity filtering.go satisfyPodAffinity]: PreFilter counts
 * topology pairs (key, value of the existing pod's node) over every term of
 * the incoming pod, for each existing pod that matches ALL of its terms
 * (updateWithAffinityTerms / podMatchesAllAffinityTerms).  A node passes when
 * it carries every term's topology key and each term's pair has a count; or,
 * when no pair was counted at all and the pod matches its own terms (the
 * first pod of a group with affinity to itself), when it carries every key. */
static int o_pod_affinity_ok(const o_state *st, const int32_t *node, int32_t n, const sr_cluster *c, int32_t pod,
                             int32_t nnode) {
  const sr_pod_affinity *A = c->pod_affinity;
  if (!A || !A->aff_off || A->aff_off[pod] == A->aff_off[pod + 1]) return 1;
  int32_t t0 = A->aff_off[pod], t1 = A->aff_off[pod + 1];
  int32_t vn[64];
  if (t1 - t0 > 64) return 0; /* never reached: the shim's terms per pod are few */
  for (int32_t t = t0; t < t1; t++)
    if (!o_node_label(c, nnode, A->topology_key[t], &vn[t - t0])) return 0; /* all topology labels must exist */
  int map_empty = 1, all_sat = 1;
  for (int32_t t = t0; t < t1 && all_sat; t++) {
    int sat = 0;
    for (int32_t m = 0; m < n && !sat; m++) {
      int32_t vm;
      if (!o_node_label(c, node[m], A->topology_key[t], &vm) || vm != vn[t - t0]) continue;
      for (int32_t j = 0; j < st[m].nlist && !sat; j++) {
        int32_t e = st[m].list[j], all = 1;
        for (int32_t u = t0; u < t1 && all; u++) all = o_term_matches(c, pod, u, e);
        sat = all;
      }
    }
    all_sat = sat;
  }
  if (all_sat) return 1;
  /* podsExist is false: the self-affinity exception needs an empty pair map */
  for (int32_t m = 0; m < n && map_empty; m++) {
    int has_key = 0;
    for (int32_t t = t0; t < t1 && !has_key; t++) {
      int32_t v;
      has_key = o_node_label(c, node[m], A->topology_key[t], &v);
    }
    if (!has_key) continue;
    for (int32_t j = 0; j < st[m].nlist && map_empty; j++) {
      int32_t e = st[m].list[j], all = 1;
      for (int32_t u = t0; u < t1 && all; u++) all = o_term_matches(c, pod, u, e);
      if (all) map_empty = 0;
    }
  }
  if (!map_empty) return 0;
  for (int32_t u = t0; u < t1; u++)
    if (!o_term_matches(c, pod, u, pod)) return 0;
  return 1;
}

/* ---- PodTopologySpread (DoNotSchedule) [upstream k8s v1.19.2
 * plugins/podtopologyspread/filtering.go]. */

/* labels.Selector.Matches of constraint k's selector over a pod's labels. */
static int o_spread_sel(const sr_cluster *c, int32_t k, int32_t pod) {
  const sr_spread *S = c->spread;
  if (S->selector_nil[k]) return 0; /* LabelSelectorAsSelector(nil) = labels.Nothing() */
  for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1]; i++) {
    int32_t v;
    if (!o_pod_label(c, pod, S->ml_key[i], &v) || v != S->ml_val[i]) return 0;
  }
  for (int32_t e = S->me_off[k]; e < S->me_off[k + 1]; e++) {
    int32_t v;
    int has = o_pod_label(c, pod, S->me_key[e], &v), ok;
    int32_t lo = S->me_val_off[e], hi = S->me_val_off[e + 1];
    switch (S->me_op[e]) {
      case SR_OP_IN: ok = has && o_in_values(S->me_vals, lo, hi, v); break;
      case SR_OP_NOT_IN: ok = !has || !o_in_values(S->me_vals, lo, hi, v); break;
      case SR_OP_EXISTS: ok = has; break;
      case SR_OP_DOES_NOT_EXIST: ok = !has; break;
      default: ok = 0; break;
    }
    if (!ok) return 0;
  }
  return 1;
}

/* filterTopologySpreadConstraints -> metav1.LabelSelectorAsSelector: a
 * constraint selector that fails to build (NewRequirement's rules). */
static int o_spread_invalid(const sr_cluster *c, int32_t k) {
  const sr_spread *S = c->spread;
  /* maxSkew < 1 fails API validation and never reaches the scheduler: the
   * planner's C ABI accepts it but routes it to the reference path */
  if (S->max_skew[k] < 1) return 1;
  if (S->selector_nil[k]) return 0;
  for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1]; i++)
    if (!o_req_strings_ok(c, S->ml_key[i], S->ml_val, i, i + 1)) return 1;
  for (int32_t e = S->me_off[k]; e < S->me_off[k + 1]; e++) {
    int32_t nv = S->me_val_off[e + 1] - S->me_val_off[e], op = S->me_op[e];
    if (!o_req_strings_ok(c, S->me_key[e], S->me_vals, S->me_val_off[e], S->me_val_off[e + 1])) return 1;
    if ((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 0) return 1;
    if ((op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) && nv != 0) return 1;
    if (op != SR_OP_IN && op != SR_OP_NOT_IN && op != SR_OP_EXISTS && op != SR_OP_DOES_NOT_EXIST) return 1;
  }
  return 0;
}

static int o_affinity_ok(const sr_cluster *c, int32_t pod, int32_t node);

/* node.Labels[key] with Go's zero value: "" when the key is absent. */
static int32_t o_label_or_empty(const sr_cluster *c, int32_t node, int32_t key) {
  int32_t v;
  return o_node_label(c, node, key, &v) ? v : c->id_empty;
}

/* PreFilter (calPreFilterState) + Filter for `pod` on snapshot position `pos`:
 * the pairs (topology key, value) of the nodes passing the pod's nodeSelector
 * / required affinity and carrying every constraint's key; per pair the
 * matching pods (the pod's namespace, not terminating, the constraint's
 * selector) on every node whose value of that key is the pair's -- counted
 * into the pair itself, so two constraints on one key share their pairs'
 * counts, as TpPairToMatchNum does; min per key over its pairs. */
static int o_spread_ok(const o_state *st, const int32_t *node, int32_t n, const sr_cluster *c, int32_t pod,
                       int32_t pos) {
  const sr_spread *S = c->spread;
  if (!S || S->off[pod] == S->off[pod + 1]) return 1;
  const sr_pod_affinity *A = c->pod_affinity;
  int32_t k0 = S->off[pod], k1 = S->off[pod + 1], nk = k1 - k0;
  if (nk > 16) return 0; /* never reached: the shim's constraints per pod are few */
  /* pairs: up to one per distinct (key, value) over the map nodes */
  int32_t cap = n * nk + 1, np_ = 0;
  int32_t *pkey = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
  int32_t *pval = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
  int64_t *pcnt = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
  for (int32_t m = 0; m < n; m++) {
    if (!o_affinity_ok(c, pod, node[m])) continue;
    int all = 1;
    for (int32_t k = k0; k < k1 && all; k++) {
      int32_t v;
      all = o_node_label(c, node[m], S->topology_key[k], &v);
    }
    if (!all) continue;
    for (int32_t k = k0; k < k1; k++) {
      int32_t key = S->topology_key[k], v = o_label_or_empty(c, node[m], key), found = 0;
      for (int32_t q = 0; q < np_ && !found; q++) found = pkey[q] == key && pval[q] == v;
      if (!found) {
        pkey[np_] = key;
        pval[np_] = v;
        pcnt[np_] = 0;
        np_++;
      }
    }
  }
  int ok = 1;
  if (np_ > 0) {
    /* processNode: every node, every constraint, the pair of the node's value */
    for (int32_t m = 0; m < n; m++)
      for (int32_t k = k0; k < k1; k++) {
        int32_t key = S->topology_key[k], v = o_label_or_empty(c, node[m], key), q = 0;
        while (q < np_ && !(pkey[q] == key && pval[q] == v)) q++;
        if (q == np_) continue;
        for (int32_t j = 0; j < st[m].nlist; j++) {
          int32_t e = st[m].list[j];
          if (S->terminating[e] || A->ns[e] != A->ns[pod]) continue;
          if (o_spread_sel(c, k, e)) pcnt[q]++;
        }
      }
    for (int32_t k = k0; k < k1 && ok; k++) {
      int32_t key = S->topology_key[k], v;
      if (!o_node_label(c, node[pos], key, &v)) {
        ok = 0; /* the node lacks the key: UnschedulableAndUnresolvable */
        break;
      }
      int64_t minc = INT64_MAX, match = 0;
      for (int32_t q = 0; q < np_; q++)
        if (pkey[q] == key) {
          if (pcnt[q] < minc) minc = pcnt[q];
          if (pval[q] == v) match = pcnt[q];
        }
      int64_t self = o_spread_sel(c, k, pod);
      if (match + self - minc > S->max_skew[k]) ok = 0;
    }
  }
  free(pkey);
  free(pval);
  free(pcnt);
  return ok;
}

/* ===================================================================== */
/* Volume filters [upstream k8s v1.19.2 plugins volumebinding, volumezone,
 * volumerestrictions, nodevolumelimits], over the shim's resolved
 * sr_volumes.  Not pinned by any reference test. */

static uint64_t o_att_word(int32_t key, int32_t id) { return (uint64_t)(uint32_t)key << 32 | (uint32_t)id; }

static int o_cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

/* the snapshot's attachable volumes, sorted (s->vb) */
static void o_vol_base_build(oracle_snapshot *s, const sr_cluster *c) {
  const sr_volumes *V = c->volumes;
  int32_t n = 0, cap = 0;
  free(s->vb);
  s->vb = NULL;
  for (int32_t i = 0; i < s->n && V; i++)
    for (int32_t q = 0; q < s->st[i].nlist; q++) {
      int32_t pod = s->st[i].list[q];
      for (int32_t a = V->att_off[pod]; a < V->att_off[pod + 1]; a++) {
        if (n == cap) {
          cap = cap ? 2 * cap : 64;
          s->vb = (uint64_t *)realloc(s->vb, sizeof(uint64_t) * (size_t)cap);
        }
        s->vb[n++] = o_att_word(V->att_key[a], V->att_id[a]);
      }
    }
  if (n) qsort(s->vb, (size_t)n, sizeof(uint64_t), o_cmp_u64);
  s->vb_n = n;
  s->vb_valid = 1;
}

/* labels.NewRequirement validation + Requirement.Matches over a PV term's expressions */
static int o_vexpr_valid(const sr_cluster *c, const sr_volumes *V, int32_t e) {
  int32_t nv = V->expr_val_off[e + 1] - V->expr_val_off[e];
  if (V->expr_key[e] == c->id_empty && c->id_empty != -1) return 0;
  if (!o_req_strings_ok(c, V->expr_key[e], V->expr_vals, V->expr_val_off[e], V->expr_val_off[e + 1])) return 0;
  switch (V->expr_op[e]) {
    case SR_OP_IN:
    case SR_OP_NOT_IN:
      return nv > 0;
    case SR_OP_EXISTS:
    case SR_OP_DOES_NOT_EXIST:
      return nv == 0;
    case SR_OP_GT:
    case SR_OP_LT: {
      int64_t x;
      return nv == 1 && o_str_int(c, V->expr_vals[V->expr_val_off[e]], &x);
    }
    default:
      return 0;
  }
}

static int o_vexpr_match(const sr_cluster *c, const sr_volumes *V, int32_t e, int32_t node) {
  int32_t v;
  int has = o_node_label(c, node, V->expr_key[e], &v);
  int32_t lo = V->expr_val_off[e], hi = V->expr_val_off[e + 1];
  int64_t lv, rv;
  switch (V->expr_op[e]) {
    case SR_OP_GT:
      return has && o_str_int(c, v, &lv) && o_str_int(c, V->expr_vals[lo], &rv) && lv > rv;
    case SR_OP_LT:
      return has && o_str_int(c, v, &lv) && o_str_int(c, V->expr_vals[lo], &rv) && lv < rv;
    case SR_OP_IN:
      return has && o_in_values(V->expr_vals, lo, hi, v);
    case SR_OP_NOT_IN:
      return !has || !o_in_values(V->expr_vals, lo, hi, v);
    case SR_OP_EXISTS:
      return has;
    case SR_OP_DOES_NOT_EXIST:
      return !has;
    default:
      return 0;
  }
}

/* VolumeBinding.Filter on the bound claims: volumeutil.CheckNodeAffinity =
 * v1helper.MatchNodeSelectorTerms(terms, node labels, nil fields) per PV with
 * a Required node affinity: terms ORed, an empty term matches nothing, a term
 * failing to build matches nothing, a field requirement reads "" */
static int o_pv_affinity_ok(const sr_cluster *c, int32_t pod, int32_t node) {
  const sr_volumes *V = c->volumes;
  for (int32_t pv = V->pv_off[pod]; pv < V->pv_off[pod + 1]; pv++) {
    int matched = 0;
    for (int32_t t = V->pv_term_off[pv]; t < V->pv_term_off[pv + 1] && !matched; t++) {
      int32_t e0 = V->term_expr_off[t], e1 = V->term_expr_off[t + 1];
      int32_t f0 = V->term_field_off[t], f1 = V->term_field_off[t + 1];
      if (e0 == e1 && f0 == f1) continue;
      int ok = 1;
      for (int32_t e = e0; e < e1 && ok; e++)
        if (!o_vexpr_valid(c, V, e)) ok = 0;
      for (int32_t e = e0; e < e1 && ok; e++)
        if (!o_vexpr_match(c, V, e, node)) ok = 0;
      for (int32_t f = f0; f < f1 && ok; f++) {
        int32_t nv = V->field_val_off[f + 1] - V->field_val_off[f], op = V->field_op[f];
        if (!((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 1)) ok = 0;
      }
      for (int32_t f = f0; f < f1 && ok; f++) {
        int eq = V->field_vals[V->field_val_off[f]] == c->id_empty && c->id_empty != -1; /* fields.Set(nil) */
        if (!(V->field_op[f] == SR_OP_IN ? eq : !eq)) ok = 0;
      }
      if (ok) matched = 1;
    }
    if (!matched) return 0;
  }
  return 1;
}

/* VolumeZone.Filter: a node without any of the four zone / region labels
 * passes; otherwise, per PV zone label, the node's value of its key ("" when
 * absent) must be in the label's LabelZonesToSet values */
static int o_volume_zone_ok(const sr_cluster *c, int32_t pod, int32_t node) {
  const sr_volumes *V = c->volumes;
  if (V->zone_off[pod] == V->zone_off[pod + 1]) return 1;
  int any = 0;
  for (int z = 0; z < 4; z++) {
    int32_t v;
    if (V->zone_keys[z] >= 0 && o_node_label(c, node, V->zone_keys[z], &v)) any = 1;
  }
  if (!any) return 1;
  for (int32_t z = V->zone_off[pod]; z < V->zone_off[pod + 1]; z++) {
    int32_t v;
    if (!o_node_label(c, node, V->zone_key[z], &v)) return 0; /* "" is never in the set */
    if (!o_in_values(V->zone_vals, V->zone_val_off[z], V->zone_val_off[z + 1], v)) return 0;
  }
  return 1;
}

/* VolumeRestrictions.Filter: isVolumeConflict of each inline disk against the
 * disks of every pod on the node (same GCE PD / ISCSI IQN unless both mounts
 * are read-only; the same EBS VolumeID always) */
static int o_disks_ok(const o_state *st, const sr_cluster *c, int32_t pod) {
  const sr_volumes *V = c->volumes;
  for (int32_t d = V->disk_off[pod]; d < V->disk_off[pod + 1]; d++)
    for (int32_t q = 0; q < st->nlist; q++) {
      int32_t e = st->list[q];
      for (int32_t f = V->disk_off[e]; f < V->disk_off[e + 1]; f++) {
        if (V->disk_kind[f] != V->disk_kind[d] || V->disk_id[f] != V->disk_id[d]) continue;
        if (V->disk_kind[d] == SR_DISK_AWS_EBS || !(V->disk_ro[d] && V->disk_ro[f])) return 0;
      }
    }
  return 1;
}

/* nodevolumelimits: per limit key the node's unique attachable volumes plus
 * the pod's volumes not already among them, against the node's limit (none:
 * no check).  Non-CSI filters check whenever the pod has such a volume; the
 * CSI filter only when some volume is new. */
static int o_volume_limits_ok(const o_state *st, const sr_cluster *c, int32_t pod, int32_t node) {
  const sr_volumes *V = c->volumes;
  for (int32_t a = V->att_off[pod]; a < V->att_off[pod + 1]; a++) {
    int32_t key = V->att_key[a], first = 1;
    for (int32_t b = V->att_off[pod]; b < a; b++)
      if (V->att_key[b] == key) first = 0;
    if (!first) continue;
    int64_t limit = -1;
    for (int32_t l = V->limit_off[node]; l < V->limit_off[node + 1]; l++)
      if (V->limit_key[l] == key) limit = V->limit[l];
    if (limit < 0) continue; /* no limit for the key on this node */
    /* existing unique volumes of the key: count each id once */
    int64_t existing = 0;
    for (int32_t q = 0; q < st->nlist; q++) {
      int32_t e = st->list[q];
      for (int32_t f = V->att_off[e]; f < V->att_off[e + 1]; f++) {
        if (V->att_key[f] != key) continue;
        int seen = 0;
        for (int32_t q2 = 0; q2 <= q && !seen; q2++) {
          int32_t e2 = st->list[q2];
          int32_t end = q2 == q ? f : V->att_off[e2 + 1];
          for (int32_t g = V->att_off[e2]; g < end && !seen; g++)
            seen = V->att_key[g] == key && V->att_id[g] == V->att_id[f];
        }
        if (!seen) existing++;
      }
    }
    int64_t fresh = 0;
    for (int32_t b = V->att_off[pod]; b < V->att_off[pod + 1]; b++) {
      if (V->att_key[b] != key) continue;
      int on = 0;
      for (int32_t q = 0; q < st->nlist && !on; q++) {
        int32_t e = st->list[q];
        for (int32_t f = V->att_off[e]; f < V->att_off[e + 1] && !on; f++)
          on = V->att_key[f] == key && V->att_id[f] == V->att_id[b];
      }
      if (!on) fresh++;
    }
    if (!V->att_noncsi[a] && fresh == 0) continue;
    if (existing + fresh > limit) return 0;
  }
  return 1;
}

int32_t oracle_pod_needs_fallback(const oracle_snapshot *s, const sr_cluster *c, int32_t pod) {
  const sr_pods *P = &c->pods;
  if (P->flags[pod] & SR_POD_FB_MASK) return 1;
  /* planner limit: an attachable volume some spot node already holds (the
   * device counts a pod's volumes as all new) */
  if (c->volumes && c->volumes->att_off[pod + 1] > c->volumes->att_off[pod]) {
    if (!s->vb_valid) o_vol_base_build((oracle_snapshot *)s, c);
    for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1]; a++) {
      uint64_t w = o_att_word(c->volumes->att_key[a], c->volumes->att_id[a]);
      if (s->vb_n && bsearch(&w, s->vb, (size_t)s->vb_n, sizeof(uint64_t), o_cmp_u64)) return 1;
    }
  }
  /* outside the encoded set: scalar resources on an all-zero
   * cpu / memory / ephemeral request, or while some snapshot pod's scalar
   * usage is unknown */
  if (o_has_scalars(c, pod) &&
      ((P->req_milli_cpu[pod] == 0 && P->req_memory[pod] == 0 && P->req_ephemeral[pod] == 0) || s->sc_unknown_total > 0))
    return 1;
  /* topology spread constraints the planner cannot read: no pod metadata or
   * validation table, or a selector that fails to build (PreFilter errors) */
  if (c->spread && c->spread->off[pod + 1] > c->spread->off[pod]) {
    if (!c->pod_affinity || !c->str_label) return 1;
    for (int32_t k = c->spread->off[pod]; k < c->spread->off[pod + 1]; k++)
      if (o_spread_invalid(c, k)) return 1;
  }
  /* an existing pod's required anti-affinity may select the incoming pod:
   * opaque terms (o_anti_opaque) keep every pod on the fallback path */
  if (s->opaque_total > 0 || o_anti_opaque(c, pod) || o_aff_opaque(c, pod)) return 1;
  if (P->aff_required[pod])
    for (int32_t t = P->term_off[pod]; t < P->term_off[pod + 1]; t++)
      for (int32_t e = P->term_expr_off[t]; e < P->term_expr_off[t + 1]; e++)
        if (((P->expr_op[e] == SR_OP_GT || P->expr_op[e] == SR_OP_LT) && !c->str_int) || !c->str_label) return 1;
  return 0;
}

static int o_check(const oracle_snapshot *s, const o_state *st, const int32_t *node, int32_t n, const sr_cluster *c, int32_t pod,
                   int32_t pos) {
  /* Filter order of the default provider; the result is their conjunction. */
  const o_state *sp = &st[pos];
  int32_t nd = node[pos];
  if (!o_unschedulable_ok(c, pod, nd)) return 0;
  if (!o_resources_ok(s, sp, c, pod, pos, nd)) return 0;
  /* NodeName: passes, findSpotNodeForPod clears Spec.NodeName (rescheduler.go:341) */
  if (!o_ports_ok(sp, c, pod)) return 0;
  if (!o_affinity_ok(c, pod, nd)) return 0;
  if (!o_taints_ok(c, pod, nd)) return 0;
  if (!o_spread_ok(st, node, n, c, pod, pos)) return 0;
  if (!o_interpod_ok(st, node, n, c, pod, nd)) return 0;
  if (!o_pod_affinity_ok(st, node, n, c, pod, nd)) return 0;
  if (c->volumes) {
    if (c->volumes->prefilter_fail[pod]) return 0; /* VolumeBinding PreFilter */
    if (!o_disks_ok(sp, c, pod)) return 0;
    if (!o_volume_limits_ok(sp, c, pod, nd)) return 0;
    if (!o_pv_affinity_ok(c, pod, nd)) return 0;
    if (!o_volume_zone_ok(c, pod, nd)) return 0;
  }
  return 1;
}

int32_t oracle_check_predicates(const oracle_snapshot *s, const sr_cluster *c, int32_t pod, int32_t pos) {
  if (oracle_pod_needs_fallback(s, c, pod)) return -1;
  return o_check(s, s->st, s->node, s->n, c, pod, pos);
}

/* findSpotNodeForPod (rescheduler.go:338-353) */
static int32_t o_find(const oracle_snapshot *s, const o_state *st, const int32_t *node, int32_t n, const sr_cluster *c,
                      int32_t pod, uint64_t *checks) {
  for (int32_t pos = 0; pos < n; pos++) {
    if (checks) (*checks)++;
    if (o_check(s, st, node, n, c, pod, pos)) return pos;
  }
  return -1;
}

int32_t oracle_find_spot_node_for_pod(const oracle_snapshot *s, const sr_cluster *c, int32_t pod) {
  if (oracle_pod_needs_fallback(s, c, pod)) return -2;
  return o_find(s, s->st, s->node, s->n, c, pod, NULL);
}

static int o_cand_fallback(const oracle_snapshot *s, const sr_cluster *c, const int32_t *pods, int32_t np);

/* canDrainNode (rescheduler.go:357-370) */
int32_t oracle_can_drain_node(oracle_snapshot *s, const sr_cluster *c, const int32_t *pods, int32_t n,
                              int32_t *node_of_pod) {
  if (o_cand_fallback(s, c, pods, n)) return -2;
  for (int32_t i = 0; i < n; i++) node_of_pod[i] = -1;
  for (int32_t i = 0; i < n; i++) {
    int32_t pos = o_find(s, s->st, s->node, s->n, c, pods[i], NULL);
    if (pos < 0) return i;
    node_of_pod[i] = pos;
    oracle_snapshot_add_pod(s, c, pods[i], pos);
  }
  return -1;
}

/* ===================================================================== */
/* The planning loop of run() (rescheduler.go:228-287). */

typedef struct {
  int32_t pos;
  int64_t req[3];
  int32_t npods, nports, anti, opaque, nlist, nsc;
} o_undo;

/* Evaluate one candidate from the base state `st` (Fork), then restore it (Revert). */
static int32_t o_eval_candidate(const oracle_snapshot *s, o_state *st, const int32_t *node, int32_t n, const sr_cluster *c,
                                const int32_t *pods, int32_t np, int32_t *map, o_undo *undo,
                                uint64_t *checks) {
  int32_t nu = 0, status = SR_CAND_OK;
  for (int32_t i = 0; i < np; i++) map[i] = -1;
  for (int32_t i = 0; i < np; i++) {
    int32_t pos = o_find(s, st, node, n, c, pods[i], checks);
    if (pos < 0) {
      status = i;
      break;
    }
    map[i] = pos;
    o_undo *u = &undo[nu++];
    u->pos = pos;
    memcpy(u->req, st[pos].req, sizeof(u->req));
    u->npods = st[pos].npods;
    u->nports = st[pos].nports;
    u->anti = st[pos].anti;
    u->opaque = st[pos].opaque;
    u->nlist = st[pos].nlist;
    u->nsc = st[pos].nsc;
    o_state_add_pod(&st[pos], c, pods[i]);
  }
  while (nu > 0) { /* Revert, newest first */
    o_undo *u = &undo[--nu];
    memcpy(st[u->pos].req, u->req, sizeof(u->req));
    st[u->pos].npods = u->npods;
    st[u->pos].nports = u->nports;
    st[u->pos].anti = u->anti;
    st[u->pos].opaque = u->opaque;
    st[u->pos].nlist = u->nlist;
    st[u->pos].nsc = u->nsc;
  }
  return status;
}

/* Topology spread between the pods of one candidate beyond what the planner
 * plans on its domain path: a pod whose constraint counts an
 * earlier pod of the candidate (its namespace, not terminating, selected),
 * when the pod has pairs at all, makes the candidate a fallback if it has
 * more than 512 pods, if the pod has another constraint on that key or more
 * than 2 such constraints, if the key is shared (not on every spot node with
 * distinct values) and has more than 64 values, or if the key is node-local
 * and no more of the pairs' nodes hold the minimum count than the constraint
 * counts earlier pods. */
static int o_spread_counted(const sr_cluster *c, int32_t k, int32_t pod, int32_t q) {
  return !c->spread->terminating[q] && c->pod_affinity->ns[q] == c->pod_affinity->ns[pod] && o_spread_sel(c, k, q);
}

static int o_spread_dyn_fallback(const oracle_snapshot *s, const sr_cluster *c, const int32_t *pods, int32_t np) {
  const sr_spread *S = c->spread;
  if (!S || !c->pod_affinity) return 0;
  int any = 0;
  for (int32_t i = 1; i < np && !any; i++)
    for (int32_t k = S->off[pods[i]]; k < S->off[pods[i] + 1] && !any; k++)
      for (int32_t j = 0; j < i && !any; j++) any = o_spread_counted(c, k, pods[i], pods[j]);
  if (!any) return 0;
  if (np > 512) return 1;
  const int32_t n = s->n;
  uint8_t *pair = (uint8_t *)malloc((size_t)n + 1);
  int fb = 0;
  for (int32_t i = 1; i < np && !fb; i++) {
    const int32_t pod = pods[i];
    int npair = 0, slots = 0;
    for (int32_t m = 0; m < n; m++) {
      int all = o_affinity_ok(c, pod, s->node[m]);
      for (int32_t k = S->off[pod]; k < S->off[pod + 1] && all; k++) {
        int32_t v;
        all = o_node_label(c, s->node[m], S->topology_key[k], &v);
      }
      pair[m] = (uint8_t)all;
      npair += all;
    }
    for (int32_t k = S->off[pod]; k < S->off[pod + 1] && !fb; k++) {
      int32_t counted = 0;
      for (int32_t j = 0; j < i; j++) counted += o_spread_counted(c, k, pod, pods[j]);
      if (counted == 0) continue;
      if (npair == 0) break; /* no pair: the filter passes every node */
      for (int32_t k2 = S->off[pod]; k2 < S->off[pod + 1]; k2++)
        if (k2 != k && S->topology_key[k2] == S->topology_key[k]) fb = 1;
      if (fb || ++slots > 2) {
        fb = 1;
        break;
      }
      /* node-local: every spot node carries the key, values pairwise distinct */
      int32_t key = S->topology_key[k], nvals = 0, local = 1;
      int32_t *vals = (int32_t *)malloc(sizeof(int32_t) * ((size_t)n + 1));
      for (int32_t m = 0; m < n; m++) {
        int32_t v;
        if (!o_node_label(c, s->node[m], key, &v)) {
          local = 0;
          continue;
        }
        int32_t seen = 0;
        for (int32_t q = 0; q < nvals && !seen; q++) seen = vals[q] == v;
        if (seen) local = 0;
        else vals[nvals++] = v;
      }
      free(vals);
      if (!local) {
        if (nvals > 64) fb = 1;
        continue;
      }
      /* the pairs' minimum count and how many nodes hold it */
      int64_t m0 = INT64_MAX, n0 = 0;
      for (int32_t m = 0; m < n; m++) {
        if (!pair[m]) continue;
        int64_t cnt = 0;
        for (int32_t j = 0; j < s->st[m].nlist; j++) {
          int32_t e = s->st[m].list[j];
          if (!S->terminating[e] && c->pod_affinity->ns[e] == c->pod_affinity->ns[pod] && o_spread_sel(c, k, e)) cnt++;
        }
        if (cnt < m0) {
          m0 = cnt;
          n0 = 0;
        }
        if (cnt == m0) n0++;
      }
      if (n0 <= counted) fb = 1;
    }
  }
  free(pair);
  return fb;
}

static int o_cand_fallback(const oracle_snapshot *s, const sr_cluster *c, const int32_t *pods, int32_t np) {
  for (int32_t i = 0; i < np; i++)
    if (oracle_pod_needs_fallback(s, c, pods[i])) return 1;
  if (o_spread_dyn_fallback(s, c, pods, np)) return 1;
  /* planner limit: two pods of the candidate sharing an attachable volume */
  if (c->volumes)
    for (int32_t i = 0; i < np; i++)
      for (int32_t a = c->volumes->att_off[pods[i]]; a < c->volumes->att_off[pods[i] + 1]; a++)
        for (int32_t j = i + 1; j < np; j++)
          for (int32_t b = c->volumes->att_off[pods[j]]; b < c->volumes->att_off[pods[j] + 1]; b++)
            if (c->volumes->att_key[a] == c->volumes->att_key[b] && c->volumes->att_id[a] == c->volumes->att_id[b])
              return 1;
  /* scalar resources and volume limit keys: the planner's per-candidate table
   * holds 64 distinct names, and it keeps a running state for at most 2 names
   * listed by more than one pod of the candidate (the later pods see the
   * earlier ones' AddPod); beyond that, the reference path */
  if (c->pod_scalar_off || c->volumes) {
    int32_t names[64], cnt[64], nn = 0, shared = 0;
    for (int32_t i = 0; i < np; i++) {
      int32_t n_here = 0, here[64];
      if (c->pod_scalar_off)
        for (int32_t a = c->pod_scalar_off[pods[i]]; a < c->pod_scalar_off[pods[i] + 1] && n_here < 64; a++)
          here[n_here++] = c->pod_scalar_name[a];
      if (c->volumes)
        for (int32_t a = c->volumes->att_off[pods[i]]; a < c->volumes->att_off[pods[i] + 1] && n_here < 64; a++) {
          int32_t name = -(c->volumes->att_key[a] + 1), dup = 0; /* each limit key once per pod */
          for (int32_t h = 0; h < n_here; h++) dup |= here[h] == name;
          if (!dup) here[n_here++] = name;
        }
      for (int32_t h = 0; h < n_here; h++) {
        int32_t u = 0;
        while (u < nn && names[u] != here[h]) u++;
        if (u < nn) {
          if (++cnt[u] == 2) shared++;
        } else {
          if (nn == 64) return 1;
          names[nn] = here[h];
          cnt[nn++] = 1;
        }
      }
    }
    if (shared > 2) return 1;
  }
  return 0;
}

int32_t oracle_plan(const oracle_snapshot *s, const sr_cluster *c, const sr_candidates *cands,
                    int32_t mode, int32_t threads, sr_plan_out *out) {
  int32_t nc = cands->n_cand;
  const int32_t *off = cands->cand_pod_off;
  int32_t maxp = 0;
  for (int32_t i = 0; i < nc; i++)
    if (off[i + 1] - off[i] > maxp) maxp = off[i + 1] - off[i];
  int32_t *status = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nc ? nc : 1));
  int32_t total = off[nc];
  int32_t *map = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total ? total : 1));
  for (int32_t i = 0; i < nc; i++) status[i] = ORACLE_NOT_EVALUATED;
  for (int32_t i = 0; i < total; i++) map[i] = -1;
  uint64_t checks = 0, fb_pods = 0;
  if (c->volumes && !s->vb_valid) o_vol_base_build((oracle_snapshot *)s, c); /* before any worker reads it */

  if (mode == 0 || threads <= 1) {
    o_state *st = o_copy_states(s->st, s->n);
    o_undo *undo = (o_undo *)malloc(sizeof(o_undo) * (size_t)(maxp ? maxp : 1));
    for (int32_t i = 0; i < nc; i++) {
      const int32_t *pods = cands->cand_pods + off[i];
      int32_t np = off[i + 1] - off[i];
      if (np < 1) {
        status[i] = SR_CAND_EMPTY;
        continue;
      }
      if (o_cand_fallback(s, c, pods, np)) {
        status[i] = SR_CAND_FALLBACK;
        fb_pods += (uint64_t)np;
        continue;
      }
      status[i] = o_eval_candidate(s, st, s->node, s->n, c, pods, np, map + off[i], undo, &checks);
      if (mode == 0 && status[i] == SR_CAND_OK) break; /* drain + break (rescheduler.go:286) */
    }
    free(undo);
    o_free_states(st, s->n);
  } else {
#ifdef _OPENMP
    omp_set_num_threads(threads);
#endif
#pragma omp parallel reduction(+ : checks, fb_pods)
    {
      o_state *st = o_copy_states(s->st, s->n);
      o_undo *undo = (o_undo *)malloc(sizeof(o_undo) * (size_t)(maxp ? maxp : 1));
#pragma omp for schedule(dynamic, 4)
      for (int32_t i = 0; i < nc; i++) {
        const int32_t *pods = cands->cand_pods + off[i];
        int32_t np = off[i + 1] - off[i];
        if (np < 1) {
          status[i] = SR_CAND_EMPTY;
          continue;
        }
        if (o_cand_fallback(s, c, pods, np)) {
          status[i] = SR_CAND_FALLBACK;
          fb_pods += (uint64_t)np;
          continue;
        }
        status[i] = o_eval_candidate(s, st, s->node, s->n, c, pods, np, map + off[i], undo, &checks);
      }
      free(undo);
      o_free_states(st, s->n);
    }
  }

  int32_t first_ok = -1, first_fb = -1;
  for (int32_t i = 0; i < nc; i++) {
    int32_t g = cands->cand_global ? cands->cand_global[i] : i;
    if (status[i] == SR_CAND_OK && (first_ok < 0 || g < first_ok)) first_ok = g;
    if (status[i] == SR_CAND_FALLBACK && (first_fb < 0 || g < first_fb)) first_fb = g;
  }
  out->first_ok = first_ok;
  out->first_fallback = first_fb;
  out->winner = (first_ok >= 0 && (first_fb < 0 || first_fb > first_ok)) ? first_ok : -1;
  out->checks = checks;
  out->fallback_pods = fb_pods;
  out->checks_dense = 0;
  for (int32_t i = 0; i < nc; i++)
    if (status[i] >= SR_CAND_OK) out->checks_dense += (uint64_t)(off[i + 1] - off[i]) * (uint64_t)s->n;
  out->winner_npods = 0;
  for (int32_t i = 0; i < nc; i++) {
    int32_t g = cands->cand_global ? cands->cand_global[i] : i;
    if (g == first_ok) {
      out->winner_npods = off[i + 1] - off[i];
      if (out->winner_map) memcpy(out->winner_map, map + off[i], sizeof(int32_t) * (size_t)out->winner_npods);
    }
  }
  if (out->status) memcpy(out->status, status, sizeof(int32_t) * (size_t)nc);
  if (out->node_of_pod) memcpy(out->node_of_pod, map, sizeof(int32_t) * (size_t)total);
  free(status);
  free(map);
  return SR_OK;
}
