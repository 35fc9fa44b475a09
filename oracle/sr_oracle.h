/*
 * sr_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference drain planner
 * (github.com/pusher/k8s-spot-rescheduler @ /root/reference) and of the
 * third-party semantics it calls, used ONLY as the checker in tests/, in
 * __graft_entry__.smoke() and as bench.py's cpu_baseline leg.  The product
 * (k8s-spot-rescheduler_amd/) never links, loads or calls it.
 *
 * What it restates (file:line into /root/reference unless marked [upstream]):
 *   nodes/nodes.go:63-104    NewNodeMap (pod sort, spot/on-demand split, node sorts)
 *   nodes/nodes.go:106-165   newNodeInfo / getPodsOnNode / calculateRequestedCPU
 *   nodes/nodes.go:168-209   isSpotNode / isOnDemandNode
 *   nodes/nodes.go:226-232   GetClusterSnapshot
 *   rescheduler.go:228-287   the planning loop of run() (Fork / canDrainNode / Revert)
 *   rescheduler.go:338-370   findSpotNodeForPod / canDrainNode
 *   [upstream] Go 1.16 sort.Slice = quickSort_func (sort/zfuncversion.go)
 *   [upstream] k8s v1.19.2 scheduler filters NodeResourcesFit, NodePorts,
 *              NodeAffinity, NodeUnschedulable, TaintToleration, NodeName
 *   [upstream] cluster-autoscaler 03f60a4c3818 ClusterSnapshot AddPod/Fork/Revert
 *
 * Parity pinning: checked against every golden vector of the reference's own
 * tests (tests/golden/reference_tests.json, transcribed from
 * rescheduler_test.go and nodes/nodes_test.go).  Behaviour those tests do not
 * cover (memory, ephemeral storage, pod count, taints, selectors, affinity,
 * host ports, sort ties) is restated from the pinned upstream versions and is
 * "parity unpinned" by any reference-run vector.
 */
#ifndef SR_ORACLE_H
#define SR_ORACLE_H

#include <stdint.h>
#include "../include/sr_planner.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_NOT_EVALUATED (-4)

/* Go 1.16 sort.Slice over an array of element ids; less(ctx, x, y) compares
 * two element ids (the closure sees the slice as it is being permuted). */
typedef int (*oracle_less_fn)(const void *ctx, int32_t x, int32_t y);
void oracle_go_sort_slice(int32_t *a, int32_t n, oracle_less_fn less, const void *ctx);
/* Convenience: sort ids by key[id] descending (desc=1) or ascending (desc=0)
 * with the reference's strict comparison (ties left to Go's algorithm). */
void oracle_go_sort_by_key(int32_t *a, int32_t n, const int64_t *key, int32_t desc);

int32_t oracle_node_has_label(const sr_cluster *c, int32_t node, const sr_node_label *l);
int32_t oracle_validate_label_flag(int32_t n_equals_parts);

/* NewNodeMap; same output layout as sr_new_node_map.  Returns SR_OK or SR_ERR_*. */
int32_t oracle_new_node_map(const sr_cluster *c, const sr_node_map_params *p, sr_node_map *out);

/* podsForDeletion for every on-demand node: NodeInfo.Pods minus mirror and
 * DaemonSet-controlled pods (rescheduler.go:231-256; GetPodsForDeletionOnNodeDrain
 * blocking rules are not modelled).  cand_off[n_on_demand+1], cand_pods[<=pods.n]. */
void oracle_build_candidates(const sr_cluster *c, const sr_node_map *m, int32_t *cand_off,
                             int32_t *cand_pods);

/* Candidate lists of run() (rescheduler.go:228-264) with the CA drain rules:
 * GetPodsForDeletionOnNodeDrain (cluster-autoscaler utils/drain @03f60a4c3818,
 * un-vendored: restated, parity unpinned) then the DaemonSet-owner filter.
 * Same contract as sr_pods_for_deletion; returns SR_OK, SR_ERR_NIL_CONTROLLER
 * or SR_ERR_INVALID_ARG. */
int32_t oracle_pods_for_deletion(const sr_cluster *c, const sr_pod_drain *d, const sr_drain_params *prm,
                                 const int32_t *nodes, int32_t n_nodes, const int32_t *node_pod_off,
                                 const int32_t *node_pod_idx, int32_t *cand_off, int32_t *cand_pods,
                                 int32_t *block_pod, int32_t *block_reason);

typedef struct oracle_snapshot oracle_snapshot;
oracle_snapshot *oracle_snapshot_create(const sr_cluster *c, const int32_t *spot, int32_t n_spot,
                                        const int32_t *node_pod_off, const int32_t *node_pod_idx);
void    oracle_snapshot_destroy(oracle_snapshot *s);
void    oracle_snapshot_add_pod(oracle_snapshot *s, const sr_cluster *c, int32_t pod, int32_t pos);
int32_t oracle_snapshot_fork(oracle_snapshot *s);
int32_t oracle_snapshot_revert(oracle_snapshot *s);
void    oracle_snapshot_node_state(const oracle_snapshot *s, int32_t pos, int64_t req[3], int32_t *npods);

/* 1 fits, 0 does not, -1 outside what the oracle can evaluate (fallback). */
int32_t oracle_check_predicates(const oracle_snapshot *s, const sr_cluster *c, int32_t pod, int32_t pos);
/* 1 if the pod must be routed to the reference path. */
int32_t oracle_pod_needs_fallback(const oracle_snapshot *s, const sr_cluster *c, int32_t pod);
/* spot position, -1 = "", -2 = fallback. */
int32_t oracle_find_spot_node_for_pod(const oracle_snapshot *s, const sr_cluster *c, int32_t pod);
/* returns -1 (nil), failing pod index, or -2 fallback; mutates s like the reference. */
int32_t oracle_can_drain_node(oracle_snapshot *s, const sr_cluster *c, const int32_t *pods,
                              int32_t n, int32_t *node_of_pod);

/* The planning segment of one tick.  mode 0 = reference-faithful (serial,
 * stop at the first drainable candidate); mode 1 = evaluate every candidate.
 * threads > 1 parallelises mode 1 over candidates (OpenMP).  Fills the same
 * fields as sr_plan_out (status entries never evaluated = ORACLE_NOT_EVALUATED). */
int32_t oracle_plan(const oracle_snapshot *s, const sr_cluster *c, const sr_candidates *cands,
                    int32_t mode, int32_t threads, sr_plan_out *out);

#ifdef __cplusplus
}
#endif
#endif
