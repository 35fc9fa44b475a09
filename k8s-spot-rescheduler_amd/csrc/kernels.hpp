// kernels.hpp — device view of the workload and the kernel launchers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "progops.hpp"

namespace sr {

constexpr int kResultHeader = 8;           // words before the winner's mapping in `result`
constexpr size_t kK0ProfWaves = 32768;  // K0 waves profiled after K2's [n_cand][16] records
constexpr int kDevDynG = 8;             // domain path: groups of 64 pods (<= 512 pods per candidate)
constexpr int kDevSpreadSlots = 2;     // spread constraints per pod on the domain path (host.hpp kSpreadSlots)
constexpr int kDevDynU64 = 5 * kDevDynG + 1 + kDevSpreadSlots * (kDevDynG + 3);
                                        // domain-path pod record words (host.hpp kDynU64): per key slot
                                        // kDevDynG mask words, kDevDynG affinity mask words, the set word,
                                        // per spread slot kDevDynG mask words and 3 info words (SpreadDyn)
constexpr int kDevDomKeys = 4;          // key slots (host.hpp kDomKeys)
constexpr int kNodePatchU64 = 12;       // node patch: {node, node_rec[8], node_free[3]}
constexpr int kPodPatchU64 = 3;         // pod patch: {active pod, pod_rec[4], pod_rec[5]}
constexpr int64_t kTPad = INT64_MAX - 1;  // threshold of a spare T row (no pod points at it; K0 skips it)
constexpr int kDevDynTerms = 4;         // terms per domain-path affinity set (host.hpp kDynTerms)
constexpr int kDevExtU64 = 8;           // extension record words (host.hpp kExtU64)
constexpr int kListInline = 128;  // work-list entries also carried in the kernel arguments

// Pointers into the device arena (layout: DESIGN.md §HBM layout).
struct DevWorkload {
  int32_t n_spot, n_pad, Wp;
  const int64_t* node_free;    // [3][n_pad] free cpu / memory / ephemeral per spot node (pads: INT64_MIN)
  const uint64_t* node_rec;    // [n_pad][8] AoS {free cpu, mem, eph, state bits, pods_left, 0, 0, 0} for K2
  const uint64_t* node_patch;  // [n_node_patch][kNodePatchU64]: records of nodes changed since the generation the
  int32_t n_node_patch;        //   node section holds; K0 writes them there (T rows use them directly)
  const uint64_t* pod_patch;   // [n_pod_patch][kPodPatchU64]: row words of the pod records a candidate-side
  int32_t n_pod_patch;         //   reuse encode re-pointed (K0 writes them into pod_rec for K2)
  int32_t k0_skip;             // no K0 this run: the tables and the node section are those of the slot's device
                               //   generation; node_patch lists every spot node changed since (K2 takes their
                               //   records from it and recomputes their bits of T rows, skip_mode: DESIGN §4)
  int32_t n_dirty;             // K0-less runs: the changed nodes and their free cpu / memory / ephemeral, in the
  int32_t dirty_node[16];      //   kernel arguments (K2's first loads need them: no memory round trip)
  int64_t dirty_free[16][3];
  int32_t* d_min_next;         // the next run's d_min buffer (runs alternate): K2 resets its first word
  int32_t first_fallback_local;  // d_min[1] of the run (K2 sets it too: K0 may not run)
  int32_t k0_inc;              // K0 rewrites only the word columns k0_cols of every row and the rows k0_rows
  int32_t n_k0_cols, n_k0_rows;  //   whole (the tables hold this candidate generation's rows otherwise current)
  const int32_t* k0_cols;
  const int32_t* k0_rows;
  int32_t n_atoms;
  const uint64_t* atoms;       // [n_atoms][Wp] node bitsets (encode.cpp)
  const int32_t* cls_prog_off; // class atom programs (CSR): ops atom << 2 | {AND, AND NOT,
  const int32_t* cls_prog;     //   open an ORed term, AND into the open term}
  const int32_t* cls_prog8;    // [n_classes][8] programs of <= 8 ops (-1 pad, -2: use cls_prog)
  int32_t n_classes;
  uint32_t s_empty_off;     // word offset of the all-zero S row pods with a certainly empty F row point
                            // at (encode.cpp), 0xffffffff if there is none
  int32_t n_t;              // threshold rows: row 0 = every node, then cpu, memory,
  int32_t t_off[5];         //   ephemeral rows [t_off[d + 1], t_off[d + 2]) (any order; kTPad: spare)
  const int64_t* t_thr;
  int32_t n_pods;
  uint64_t swap_mask;       // state bits [0, 2 * pairs): anti-affinity pairs; a pod conflicts with the
                            // pair-swapped image of the bits it sets (swap_pairs), host ports above
  const uint64_t* pod_rec;  // [n_pods + 128][6] AoS {cpu, memory, ephemeral, state bits, S | T cpu row word
                            //  offset, T mem | T eph row word offset} (48 B, padded for K2's window reads)
  int32_t n_cand;
  const int32_t* cand_off;
  const int32_t* cand_global;
  const int4* list;         // [n_list] {candidate, first pod, end pod, global index}, longest first
  int32_t n_list;
  int32_t max_np;       // most pods in one candidate of this call
  int32_t k2_node_kernel; // launch the node-order-only K2 when every candidate takes that path (SR_K2_NODE_KERNEL=0: never)
  int32_t s_head_only;    // K0 writes only the head words of S rows; K2 evaluates S words beyond them from the
                          // class programs (wide rows, node-order kernel, every program <= 8 operations)
  // domain path (k2_domain): candidates whose pods interact through shared-domain
  // topology keys (antiaff.cpp); null when the call has none
  const int32_t* dyn_cand;  // [n_cand] first record in dyn_pod, -1: node / pod order
  const uint64_t* dyn_pod;  // [..][kDevDynU64] {anti-affinity masks per key slot (4 x kDevDynG words),
                            //  affinity masks (kDevDynG words), set << 1 | self or ~0}; masks over the
                            //  candidate's earlier pods, 64 per word
  int32_t n_dk;             // key slots
  const int32_t* dk_dom;    // [n_dk][n_spot] domain of each spot node (node-local key: the node), -1 absent
  int32_t dk_row[4];        // atom of domain 0 per table key slot, -1: node-local key
  const int32_t* sp_tab;    // spread base counts per domain / caps per node (host.hpp SpreadDyn)
  const int32_t* ds_info;   // [set][2 + 2 * 4] {terms, map_empty, (key slot, base-row atom) per term}
  // extension records (pod-order and domain paths; null when the call has none):
  // candidates whose AddPod accounting differs from the fit request or whose
  // pods share a scalar resource
  const int32_t* ext_cand;   // [n_cand] first record in pod_ext, -1: none
  const uint64_t* pod_ext;   // [..][kDevExtU64] {acc cpu, acc mem, acc eph, req s0, req s1 (INT64_MIN: not
                             //  listed), acc s0, acc s1, node_scal row of s0 | of s1 << 32 (-1: no slot)}
  const int64_t* node_scal;  // [rows][n_pad] base free value (allocatable - requested) of a shared scalar
  const int4* list_ext;      // [n_list] per work-list entry {first record in pod_ext (-1: none), node_scal row of
                             //  slot 0, of slot 1 (-1: no slot), 0}
  // outputs / scratch
  uint64_t* S;         // [n_classes][Wp] static-class rows, followed by
  uint64_t* T;         // [n_t][Wp] capacity threshold rows (one table)
  int32_t* out_node;   // [n_pods] spot position or -1
  int32_t* out_status; // [n_cand]
  uint32_t* out_bytes; // [n_cand] bytes K2 moved for the candidate (the roofline's algorithmic bytes)
  uint32_t* out_cycles; // [n_cand] the candidate's wave duration in cycles (null: not recorded): the next
                        // ticks' work list runs longest first by it (planner.cpp, list_cost)
  int32_t* d_min;      // 3 x u64, reduced (min) over the ranks: packed {global << 32 | local} first ok,
                       // first fallback (~0 = none), and the smallest global candidate index a rank has
                       // not planned yet (rank_next; ~0 = none)
  uint64_t rank_next;  // this rank's d_min[2] (sr_plan_first's prefix batches; ~0 otherwise)
  uint64_t* result;    // mapped host memory [kResultHeader + max pods] words seq << 32 | value:
                       //   {winner, local, npods, first_fallback, reduced rank_next (-1: none), -, -, -,
                       //    mapping...}
  uint64_t* res_stat;  // single-rank runs: mapped host memory [n_cand] words seq << 32 | drainable, one
                       // stored by K2 per finished candidate, and
  uint64_t* res_map;   // [n_pods] words seq << 32 | spot position: a candidate's mapping, stored by K2
                       // when the candidate was the first drainable one so far as it finished (no K3);
                       // both null on runs that end with K3
  uint32_t seq;        // run sequence number: the tag of every result word (wraps)
  int32_t k2_narrow;   // node order: 32-bit scaled window visits where every request allows (SR_K2_NARROW=0: never)
  int32_t k2_wpb;      // K2 waves per block (SR_K2_WPB: 1, 2 or 4; 0 = 1 up to 2,048 entries, else 4)
  int32_t k2_excl;     // node order: exclusive candidates placed with the taken-mask step (SR_K2_EXCL=0: never)
  int32_t n_coop;      // node-order kernel, four waves per block: the first n_coop work-list entries (the costliest)
                       // are planned by one block each, its other waves scanning far resolutions with the chain
  int32_t k2_mode;     // 0: node-order first fit where it applies (<= 64 pods, <= 64-word rows);
                       // 1: pod order everywhere (SR_K2_MODE=1, A/B measurement)
  uint64_t* prof;      // optional [n_cand][16] K2 + [kK0ProfWaves][2] K0 per-wave profile
                       // (SR_K2_PROFILE), else null
  // the first kListInline work-list entries (the longest candidates, whose
  // chains set K2's time): a wave li < n_list_head reads its entry with the
  // other kernel arguments instead of one memory round trip later
  int32_t n_list_head;
  int4 list_head[kListInline];
};

// K0: S and T rows (also resets d_min: d_min[1] = local first fallback).
// ev0 / ev1 (optional): HIP events the dispatch records around the kernel.
hipError_t launch_tables(const DevWorkload& w, int32_t local_first_fallback, hipStream_t s,
                         hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// K2: per-candidate feasibility rows + first-fit placement; atomicMin of first_ok into d_min[0].
hipError_t launch_placement(const DevWorkload& w, hipStream_t s, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// K3: winner mapping into `result` (after the collective when ranks > 1), then the run's seq.
// Not launched when K2 writes res_stat / res_map itself (single rank).
hipError_t launch_winner(const DevWorkload& w, hipStream_t s, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

}  // namespace sr
