// drain.cpp — the candidate lists of run() (rescheduler.go:228-264).
//
// Per on-demand node, in NodeInfoArray order: GetPodsForDeletionOnNodeDrain
// over NodeInfo.Pods (cluster-autoscaler utils/drain @03f60a4c3818 [upstream,
// not in the reference tree]) with the reference's arguments
// (rescheduler.go:231: skipNodesWithSystemPods = *deleteNonReplicatedPods,
// skipNodesWithLocalStorage = false, checkReferences = false, no listers,
// minReplica 0, now), then the DaemonSet-owner filter (:240-256).  Host code:
// one pass over the on-demand pods, no device work.
#include <climits>

#include "host.hpp"

namespace {

// DefaultTerminationGracePeriodSeconds and PodLongTerminatingExtraThreshold [upstream].
constexpr int64_t kDefaultGraceSeconds = 30;
constexpr int64_t kLongTerminatingExtraSeconds = 30;

// drain.IsPodLongTerminating: DeletionTimestamp + grace + 30 s is before now.
bool long_terminating(const sr_pod_drain* D, int32_t pod) {
  if (!(D->flags[pod] & SR_DRAIN_DELETING)) return false;
  const int64_t grace = D->grace_seconds[pod] >= 0 ? D->grace_seconds[pod] : kDefaultGraceSeconds;
  if (grace > INT64_MAX / 1000000000 - kLongTerminatingExtraSeconds) return false;  // beyond ~292 years
  return D->deletion_age_ns[pod] > (grace + kLongTerminatingExtraSeconds) * 1000000000;
}

// drain.isPodTerminal: will never run again.
bool terminal(const sr_pod_drain* D, int32_t pod) {
  const int phase = D->phase[pod], restart = D->restart_policy[pod];
  if (restart == SR_RESTART_NEVER && (phase == SR_PHASE_SUCCEEDED || phase == SR_PHASE_FAILED)) return true;
  if (restart == SR_RESTART_ON_FAILURE && phase == SR_PHASE_SUCCEEDED) return true;
  return phase == SR_PHASE_FAILED;  // the kubelet rejected it
}

}  // namespace

extern "C" sr_status sr_pods_for_deletion(const sr_cluster* c, const sr_pod_drain* D, const sr_drain_params* prm,
                                          const int32_t* nodes, int32_t n_nodes, const int32_t* node_pod_off,
                                          const int32_t* node_pod_idx, int32_t* out_cand_off, int32_t* out_cand_pods,
                                          int32_t* out_block_pod, int32_t* out_block_reason) {
  if (!c || !D || !prm || n_nodes < 0 || (n_nodes > 0 && (!nodes || !node_pod_off || !node_pod_idx)) ||
      !out_cand_off || !out_cand_pods || !out_block_pod || !out_block_reason || D->n != c->pods.n)
    return SR_ERR_INVALID_ARG;
  const sr_pods& P = c->pods;
  int32_t k = 0;
  for (int32_t i = 0; i < n_nodes; ++i) {
    out_cand_off[i] = k;
    out_block_pod[i] = -1;
    out_block_reason[i] = SR_BLOCK_NONE;
    const int32_t node = nodes[i];
    if (node < 0 || node >= c->nodes.n || node_pod_off[node] > node_pod_off[node + 1]) return SR_ERR_INVALID_ARG;
    const int32_t k0 = k;
    for (int32_t j = node_pod_off[node]; j < node_pod_off[node + 1]; ++j) {
      const int32_t pod = node_pod_idx[j];
      if (pod < 0 || pod >= P.n) return SR_ERR_INVALID_ARG;
      if (P.flags[pod] & SR_POD_MIRROR) continue;  // pod_util.IsMirrorPod
      if (long_terminating(D, pod)) continue;
      const uint32_t f = D->flags[pod];
      const uint32_t ctrl = f & SR_DRAIN_CTRL_MASK;
      // ControllerRef kinds in the order the CA checks them: ReplicationController,
      // then IsDaemonSetPod (DaemonSet ref or the daemonset-pod annotation), then
      // Job / ReplicaSet / StatefulSet.
      bool replicated = false, daemonset = false;
      if (ctrl == SR_DRAIN_CTRL_REPLICATION_CONTROLLER) replicated = true;
      else if (ctrl == SR_DRAIN_CTRL_DAEMONSET || (f & SR_DRAIN_DAEMONSET_ANNOTATION)) daemonset = true;
      else if (ctrl == SR_DRAIN_CTRL_JOB || ctrl == SR_DRAIN_CTRL_REPLICASET || ctrl == SR_DRAIN_CTRL_STATEFULSET)
        replicated = true;
      if (daemonset) continue;
      int32_t reason = SR_BLOCK_NONE;
      if (!(f & SR_DRAIN_SAFE_TO_EVICT) && !terminal(D, pod)) {
        if (!replicated) {
          reason = SR_BLOCK_NOT_REPLICATED;
        } else if ((f & SR_DRAIN_KUBE_SYSTEM) && prm->skip_nodes_with_system_pods &&
                   ((f & SR_DRAIN_PDB_ERROR) || !(f & SR_DRAIN_KUBE_SYSTEM_PDB))) {
          reason = (f & SR_DRAIN_PDB_ERROR) ? SR_BLOCK_UNEXPECTED_ERROR : SR_BLOCK_UNMOVABLE_KUBE_SYSTEM;
        } else if ((f & SR_DRAIN_LOCAL_STORAGE) && prm->skip_nodes_with_local_storage) {
          reason = SR_BLOCK_LOCAL_STORAGE;
        } else if (f & SR_DRAIN_NOT_SAFE_TO_EVICT) {
          reason = SR_BLOCK_NOT_SAFE_TO_EVICT;
        }
      }
      if (reason != SR_BLOCK_NONE) {  // the whole node is skipped (rescheduler.go:232-238)
        out_block_pod[i] = pod;
        out_block_reason[i] = reason;
        k = k0;
        break;
      }
      out_cand_pods[k++] = pod;
    }
    if (out_block_pod[i] >= 0 || !prm->owner_filter) continue;
    // rescheduler.go:240-256: drop DaemonSet-controlled pods; *owner.Controller
    // is dereferenced for every owner reference it reaches
    int32_t kept = k0;
    for (int32_t q = k0; q < k; ++q) {
      const int32_t pod = out_cand_pods[q];
      if (D->flags[pod] & SR_DRAIN_NIL_CONTROLLER) return SR_ERR_NIL_CONTROLLER;
      if (P.flags[pod] & SR_POD_DAEMONSET_CONTROLLER) continue;
      out_cand_pods[kept++] = pod;
    }
    k = kept;
  }
  out_cand_off[n_nodes] = k;
  return SR_OK;
}
