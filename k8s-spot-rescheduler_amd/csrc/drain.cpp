// drain.cpp — the candidate lists of run() (rescheduler.go:228-264).
//
// Per on-demand node, in NodeInfoArray order: GetPodsForDeletionOnNodeDrain
// over NodeInfo.Pods (cluster-autoscaler utils/drain @03f60a4c3818 [upstream,
// not in the reference tree]) with the reference's arguments
// (rescheduler.go:231: skipNodesWithSystemPods = *deleteNonReplicatedPods,
// skipNodesWithLocalStorage = false, checkReferences = false, no listers,
// minReplica 0, now), then the DaemonSet-owner filter (:240-256).  Host code:
// two parallel passes over the on-demand pods, no device work.
#include <algorithm>
#include <atomic>
#include <climits>
#include <vector>

#include "host.hpp"
#include "pool.hpp"

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


// One node's podsForDeletion (rescheduler.go:231-256): writes the list to
// `out` (when given) and returns its length, or -1 with *block_pod /
// *block_reason when a pod blocks the node; *status reports malformed input
// or a nil ControllerRef the owner filter would dereference.
int32_t node_list(const sr_cluster* c, const sr_pod_drain* D, const sr_drain_params* prm, int32_t node,
                  const int32_t* node_pod_off, const int32_t* node_pod_idx, int32_t* out, int32_t* block_pod,
                  int32_t* block_reason, sr_status* status) {
  const sr_pods& P = c->pods;
  *block_pod = -1;
  *block_reason = SR_BLOCK_NONE;
  if (node < 0 || node >= c->nodes.n || node_pod_off[node] > node_pod_off[node + 1]) {
    *status = SR_ERR_INVALID_ARG;
    return 0;
  }
  thread_local std::vector<int32_t> kept;  // GetPodsForDeletionOnNodeDrain's list, before the owner filter
  kept.clear();
  for (int32_t j = node_pod_off[node]; j < node_pod_off[node + 1]; ++j) {
    const int32_t pod = node_pod_idx[j];
    if (pod < 0 || pod >= P.n) {
      *status = SR_ERR_INVALID_ARG;
      return 0;
    }
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
      *block_pod = pod;
      *block_reason = reason;
      return -1;
    }
    kept.push_back(pod);
  }
  // rescheduler.go:240-256: drop DaemonSet-controlled pods; *owner.Controller
  // is dereferenced for every owner reference it reaches
  int32_t k = 0;
  for (int32_t pod : kept) {
    if (prm->owner_filter) {
      if (D->flags[pod] & SR_DRAIN_NIL_CONTROLLER) {
        *status = SR_ERR_NIL_CONTROLLER;
        return 0;
      }
      if (P.flags[pod] & SR_POD_DAEMONSET_CONTROLLER) continue;
    }
    if (out) out[k] = pod;
    ++k;
  }
  return k;
}

}  // namespace

// One pass over the nodes on the pool writes each node's list into a scratch
// copy of the LIST layout (a list never outgrows its node's pods), then the
// lists move to their prefix offsets.
extern "C" sr_status sr_pods_for_deletion(const sr_cluster* c, const sr_pod_drain* D, const sr_drain_params* prm,
                                          const int32_t* nodes, int32_t n_nodes, const int32_t* node_pod_off,
                                          const int32_t* node_pod_idx, int32_t* out_cand_off, int32_t* out_cand_pods,
                                          int32_t* out_block_pod, int32_t* out_block_reason) {
  if (!c || !D || !prm || n_nodes < 0 || (n_nodes > 0 && (!nodes || !node_pod_off || !node_pod_idx)) ||
      !out_cand_off || !out_cand_pods || !out_block_pod || !out_block_reason || D->n != c->pods.n)
    return SR_ERR_INVALID_ARG;
  // the scratch is indexed by the nodes' LIST offsets (a malformed node is
  // reported by node_list, in input order, and writes nothing)
  auto well_formed = [&](int32_t node) {
    return node >= 0 && node < c->nodes.n && node_pod_off[node] >= 0 && node_pod_off[node] <= node_pod_off[node + 1];
  };
  int32_t span = 0;
  for (int32_t i = 0; i < n_nodes; ++i)
    if (well_formed(nodes[i])) span = std::max(span, node_pod_off[nodes[i] + 1]);
  thread_local std::vector<int32_t> scratch;  // kept per calling thread: a fresh buffer page-faults every call
  if (scratch.size() < static_cast<size_t>(span)) scratch.resize(static_cast<size_t>(span));
  int32_t* const lists = scratch.data();  // (the pool's threads name their own thread_local)
  // the error of the first failing node in input order (what the serial loop returned)
  std::atomic<int64_t> first_err{INT64_MAX};
  auto body = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      sr_status st = SR_OK;
      int32_t* out = well_formed(nodes[i]) ? lists + node_pod_off[nodes[i]] : nullptr;
      const int32_t k = node_list(c, D, prm, nodes[i], node_pod_off, node_pod_idx, out, &out_block_pod[i],
                                  &out_block_reason[i], &st);
      if (st != SR_OK) {
        const int64_t v = static_cast<int64_t>(i) << 8 | st;
        int64_t cur = first_err.load();
        while (v < cur && !first_err.compare_exchange_weak(cur, v)) {
        }
        return;
      }
      out_cand_off[i + 1] = k < 0 ? 0 : k;  // lengths, summed below
    }
  };
  // a node named twice would have two pool threads write its scratch range:
  // such an input runs the pass serially (same lists, no concurrent writes)
  bool repeats = false;
  if (n_nodes > 256) {
    thread_local std::vector<uint32_t> seen;
    thread_local uint32_t epoch = 0;
    if (seen.size() < static_cast<size_t>(c->nodes.n)) seen.assign(static_cast<size_t>(c->nodes.n), 0);
    if (++epoch == 0) {
      std::fill(seen.begin(), seen.end(), 0u);
      epoch = 1;
    }
    for (int32_t i = 0; i < n_nodes && !repeats; ++i)
      if (well_formed(nodes[i])) {
        repeats = seen[nodes[i]] == epoch;
        seen[nodes[i]] = epoch;
      }
  }
  if (n_nodes > 256 && !repeats) sr::parallel_for(static_cast<size_t>(n_nodes), 64, body);
  else body(0, static_cast<size_t>(n_nodes));
  if (first_err.load() != INT64_MAX) return static_cast<sr_status>(first_err.load() & 0xff);
  out_cand_off[0] = 0;
  for (int32_t i = 0; i < n_nodes; ++i) out_cand_off[i + 1] += out_cand_off[i];
  auto move = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i)
      std::copy(lists + node_pod_off[nodes[i]], lists + node_pod_off[nodes[i]] + (out_cand_off[i + 1] - out_cand_off[i]),
                out_cand_pods + out_cand_off[i]);
  };
  if (n_nodes > 256) sr::parallel_for(static_cast<size_t>(n_nodes), 256, move);
  else move(0, static_cast<size_t>(n_nodes));
  return SR_OK;
}
