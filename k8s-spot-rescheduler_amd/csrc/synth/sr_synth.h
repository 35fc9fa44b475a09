/*
 * sr_synth.h — deterministic synthetic clusters for the BASELINE.json configs
 * (bench / test infrastructure; the generator spec is in DESIGN.md §Workloads).
 * Output is a cluster in the sr_cluster layout of include/sr_planner.h, with
 * nodes and pods in a fixed "API list" order.
 */
#ifndef SR_SYNTH_H
#define SR_SYNTH_H

#include <stdint.h>

#include "../../../include/sr_planner.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t config;          /* 1..5 = BASELINE.json configs[0..4] */
  uint64_t seed;           /* 0 = 0x5EED0000 + config */
  int32_t n_on_demand;     /* 0 = config default */
  int32_t n_spot;          /* 0 = config default */
  double pinned_fraction;  /* < 0 = default; share of on-demand pods pinned to on-demand nodes */
  /* "realistic" variant (all 0 = the BASELINE config as specified): */
  double stateful_fraction; /* share of ReplicaSet-slot pods that are StatefulSet pods with one EBS CSI claim,
                               its PV in the pod's zone (zone label + node affinity), CSINode count 25 per node */
  double init_fraction;     /* share of pods with an init container (fit request != AddPod accounting) */
  double gpu_fraction;      /* share of pods on GPU nodes (1 in 8 nodes, 4 nvidia.com/gpu) asking for one GPU */
  /* "affinity" variant (both 0 = none): every pod belongs to a Deployment (label app=<name>, one of 16
   * namespaces; ~5 replicas per Deployment, spot and on-demand alike, never two replicas of an anti-affinity
   * Deployment on one node); a share of the Deployments carries required pod anti-affinity on the hostname
   * key, another share a zone DoNotSchedule topology spread constraint (maxSkew 1), both selecting their own
   * replicas.  Drawn from a separate stream: the cluster is otherwise the config's. */
  double anti_fraction;     /* share of Deployments with hostname anti-affinity */
  double spread_fraction;   /* share of Deployments with a zone DoNotSchedule spread constraint */
} sr_synth_params;

typedef struct sr_synth sr_synth;

sr_synth *sr_synth_generate(const sr_synth_params *params);
void sr_synth_destroy(sr_synth *s);
/* Pointers stay valid until sr_synth_destroy. */
void sr_synth_view(const sr_synth *s, sr_cluster *out);
/* The --on-demand-node-label / --spot-node-label flags of the cluster (defaults of rescheduler.go:98-105). */
void sr_synth_labels(const sr_synth *s, sr_node_label *on_demand, sr_node_label *spot);
/* Drain attributes: ReplicaSet-controlled running pods, DaemonSet pods DaemonSet-controlled. */
void sr_synth_drain(const sr_synth *s, sr_pod_drain *out);
const char *sr_synth_string(const sr_synth *s, int32_t id);
int32_t sr_synth_num_strings(const sr_synth *s);
/* The generator's sr_cluster.str_label entry for one string (SR_STR_LABEL_*). */
uint8_t sr_synth_label_flags(const char *s);

#ifdef __cplusplus
}
#endif
#endif
