// host.hpp — host-side model of the drain planner (C++).
//
// Mirrors the reference's cluster model (nodes/nodes.go NodeInfo /
// NodeInfoArray) and the cluster-autoscaler ClusterSnapshot the predicate
// checker reads [upstream CA simulator @03f60a4c3818], and declares the
// encoder that turns a snapshot + candidate pod lists into the SoA workload
// the gfx950 kernels consume (layout: DESIGN.md §HBM layout).
#pragma once

#include <algorithm>
#include <climits>
#include <deque>
#include <memory>
#include <utility>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/sr_planner.h"
#include "progops.hpp"
#include "worddict.hpp"

namespace sr {

struct Port {
  int32_t ip;  // -1 = 0.0.0.0 / ""
  int32_t proto;
  int32_t port;
};

struct TaintRec {
  int32_t key, val, effect;
};

// Static part of one spot node, copied out of the caller's cluster when the
// snapshot is created (AddNodeWithPods, nodes/nodes.go:229).
struct SpotNode {
  uint64_t static_fp = 0;  // node_static_fp
  uint64_t copy_fp = 0;    // fingerprint of the cluster fields it was copied from (0: copied anew every refresh)
  int32_t name = -1;
  int64_t alloc[3] = {0, 0, 0};  // milli-cpu, memory, ephemeral
  int64_t alloc_pods = 0;
  uint8_t unschedulable = 0;
  std::vector<std::pair<int32_t, int32_t>> labels;  // (key, value)
  std::vector<TaintRec> taints;
  std::vector<std::pair<int32_t, int64_t>> scalar_alloc;  // Allocatable scalar resources (name, value), by name
  std::vector<std::pair<int32_t, int64_t>> vol_limit;     // volume limits (limit key, count), by key
};

// The snapshot's own copy of what InterPodAffinity reads from a pod it holds
// (scheduler NodeInfo.Pods): namespace, labels and required anti-affinity
// terms (resolved words, anti_term_words).  Copied when the pod enters the
// snapshot, so later calls may pass any cluster encoded with the same string
// interner: pod indices of the creating cluster are never kept.
// Trivial (no member initializers): the snapshot's pod arena grows without a
// zero fill and snap_pod_from writes every field.
struct SnapPod {
  int32_t ns;
  uint8_t meta;    // ns / labels / terms known (the cluster passed sr_pod_affinity)
  uint8_t anti;    // carries required anti-affinity
  uint8_t opaque;  // ... that the encoder cannot read (anti_opaque)
  uint8_t term;    // DeletionTimestamp set (countPodsMatchSelector skips it); 2: unknown (no sr_spread)
  uint32_t lab, nlab;       // labels: sr_snapshot::lkey / lval [lab, lab + nlab)
  uint32_t terms, nterms;   // anti-affinity terms: sr_snapshot::term_words [terms, terms + nterms),
                            // {n words, words...} per term (rare)
  uint64_t meta_fp;         // fingerprint of what the inter-pod and spread filters read of it: namespace,
                            // deletion state, labels, terms (order-independent)
};

// std::allocator that default-initializes on resize() / emplace_back(): the
// snapshot's pod and label arenas (a million entries at C4) are filled in
// parallel right after they grow, so the serial zero fill is skipped.
template <class T>
struct UninitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = UninitAlloc<U>;
  };
  UninitAlloc() = default;
  template <class U>
  UninitAlloc(const UninitAlloc<U>&) {}
  template <class U>
  void construct(U* p) {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};

// Mutable part: scheduler NodeInfo.Requested, len(Pods), UsedPorts, the pods
// themselves (indices into sr_snapshot::pods; InterPodAffinity matches against
// them), the number carrying required anti-affinity, of those the opaque ones,
// and the pods whose metadata is unknown.
struct NodeState {
  int64_t requested[3] = {0, 0, 0};
  int64_t npods = 0;
  int32_t anti = 0;
  int32_t opaque = 0;
  int32_t unknown = 0;
  std::vector<Port> ports;
  std::vector<int32_t> pods;
  std::vector<std::pair<int32_t, int64_t>> scalar_req;  // Requested scalar resources (name, value), by name
  int32_t scalar_unknown = 0;  // pods added without scalar tables that carry scalar requests
  int32_t term_unknown = 0;    // pods added without sr_spread (deletion state unknown)
  std::vector<std::pair<int32_t, int32_t>> att;  // attachable volumes (limit key, unique name) of its pods, sorted
  uint64_t meta_sum = 0;       // sum of its pods' SnapPod::meta_fp (node_state_fp: a reuse encode's
                               // inter-pod and spread rows follow the nodes whose pods changed)
};

// ---- volume filters (sr_volumes)
// VolumeRestrictions' inline disks ride the host-port machinery as pseudo
// ports: protocol kDiskProto + SR_DISK_*, port = disk id + 1, ip = -1 for a
// read-write mount (it conflicts with every mount of the disk) or
// kReadOnlyMount (it conflicts with read-write mounts only; an EBS mount is
// always read-write: any two conflict).
constexpr int32_t kDiskProto = 16;
constexpr int32_t kReadOnlyMount = -2;
// A limit key without an entry on a node never refuses there.
constexpr int64_t kVolUnlimited = int64_t(1) << 61;
// The volume limit keys ride the scalar-resource machinery under negative
// names: key k -> -(k + 1) (real scalar names are interned ids >= 0).
inline int32_t vol_name(int32_t key) { return -(key + 1); }
inline int32_t vol_key_of(int32_t name) { return -name - 1; }
// Host ports (port > 0) then inline disks of a pod as (protocol, port, ip).
template <class F>
inline void for_each_port(const sr_cluster* c, int32_t pod, F&& f) {
  const sr_pods& P = c->pods;
  for (int32_t i = P.port_off[pod]; i < P.port_off[pod + 1]; ++i)
    if (P.port_num[i] > 0) f(P.port_proto[i], P.port_num[i], P.port_ip[i]);
  if (const sr_volumes* V = c->volumes)
    for (int32_t i = V->disk_off[pod]; i < V->disk_off[pod + 1]; ++i)
      f(kDiskProto + V->disk_kind[i], V->disk_id[i] + 1,
        V->disk_ro[i] && V->disk_kind[i] != SR_DISK_AWS_EBS ? kReadOnlyMount : -1);
}
inline bool has_ports(const sr_cluster* c, int32_t pod) {
  bool any = false;
  for_each_port(c, pod, [&](int32_t, int32_t, int32_t) { any = true; });
  return any;
}
// The pod's attachable volumes (sr_volumes.att_*), count of entries.
inline int32_t att_count(const sr_cluster* c, int32_t pod) {
  return c->volumes ? c->volumes->att_off[pod + 1] - c->volumes->att_off[pod] : 0;
}
// The pod carries anything the volume filters read beyond its inline disks.
inline bool has_volume_spec(const sr_cluster* c, int32_t pod) {
  const sr_volumes* V = c->volumes;
  return V && (V->prefilter_fail[pod] || V->att_off[pod + 1] > V->att_off[pod] ||
               V->zone_off[pod + 1] > V->zone_off[pod] || V->pv_off[pod + 1] > V->pv_off[pod]);
}
// Unique attachable volumes of limit key `key` on a node.
inline int64_t vol_used(const NodeState& st, int32_t key) {
  auto lo = std::lower_bound(st.att.begin(), st.att.end(), std::make_pair(key, INT32_MIN));
  auto hi = std::lower_bound(lo, st.att.end(), std::make_pair(key + 1, INT32_MIN));
  return hi - lo;
}
inline int64_t vol_limit_of(const SpotNode& sn, int32_t key) {
  auto it = std::lower_bound(sn.vol_limit.begin(), sn.vol_limit.end(), std::make_pair(key, INT64_MIN));
  return it != sn.vol_limit.end() && it->first == key ? it->second : kVolUnlimited;
}
// Allocatable and Requested of a scalar-machinery name on a node: a scalar
// resource (0 when absent), or a volume limit key (limit or kVolUnlimited, and
// the node's unique attachable volumes of the key).
inline int64_t scalar_alloc_of(const SpotNode& sn, int32_t name) {
  if (name < 0) return vol_limit_of(sn, vol_key_of(name));
  auto it = std::lower_bound(sn.scalar_alloc.begin(), sn.scalar_alloc.end(), std::make_pair(name, INT64_MIN));
  return it != sn.scalar_alloc.end() && it->first == name ? it->second : 0;
}
inline int64_t scalar_used_of(const NodeState& st, int32_t name) {
  if (name < 0) return vol_used(st, vol_key_of(name));
  auto it = std::lower_bound(st.scalar_req.begin(), st.scalar_req.end(), std::make_pair(name, INT64_MIN));
  return it != st.scalar_req.end() && it->first == name ? it->second : 0;
}

}  // namespace sr

// The opaque handle of the C-ABI.
struct sr_snapshot {
  int32_t id_empty = -1, id_metadata_name = -1, id_unschedulable_key = -1;
  std::vector<sr::SpotNode> nodes;
  std::vector<sr::NodeState> state;
  std::vector<sr::NodeState> saved;
  // per spot node, contiguous (the encoder compares them with its cached views
  // every call): name, static fingerprint (node_static_fp), state
  // fingerprint (node_state_fp, kept current by AddPod / Revert)
  std::vector<int32_t> node_names;
  std::vector<uint64_t> node_sfp, node_dfp, saved_dfp;
  std::vector<sr::SnapPod, sr::UninitAlloc<sr::SnapPod>> pods;  // every pod ever added (NodeState::pods index it)
  std::vector<uint64_t, sr::UninitAlloc<uint64_t>> stamps;       // ... their sr_cluster.pod_stamp (0: unknown),
                                                                 // read by sr_snapshot_refresh
  std::vector<int32_t, sr::UninitAlloc<int32_t>> lkey, lval;     // the pods' labels (one arena: no allocation per pod)
  std::vector<int32_t> term_words;  // the pods' anti-affinity terms (one arena)
  size_t fork_pods = 0;           // pods.size() at Fork: Revert drops the rest
  size_t fork_labels = 0;         // lkey.size() at Fork
  size_t fork_terms = 0;          // term_words.size() at Fork
  bool forked = false;
  int64_t anti_total = 0;
  int64_t opaque_total = 0;   // pods whose anti-affinity the encoder cannot read: every candidate falls back
  int64_t unknown_total = 0;  // pods without metadata: candidates whose own terms need it fall back
  int64_t scalar_unknown_total = 0;  // pods whose scalar requests are unknown: candidates asking for any fall back
  int64_t term_unknown_total = 0;    // pods whose deletion state is unknown: pods with spread constraints fall back
  uint64_t version = 0;  // bumped on every mutation
  // sr_snapshot_refresh: the cluster shape the store was built under
  // (cluster_shape) and a scratch map node name -> previous spot position
  uint64_t shape = 0;
  std::vector<int32_t> pos_of_name;
  // sr_snapshot_refresh_cached: the node map cache call this snapshot was last
  // refreshed from, and the version it had then (null: none)
  const void* map_cache = nullptr;
  uint64_t map_calls = 0, map_version = 0;
  // the spot node indices of the last create / refresh, and a scratch map
  // node index -> previous position (sr_snapshot_refresh: nodes keep their
  // cluster index from tick to tick; the name is still checked)
  std::vector<int32_t> spot_prev, pos_of_node;
};

namespace sr {

// Pod accessors over the caller's arrays.
inline bool add_overflows(int64_t a, int64_t b) {
  int64_t r;
  return __builtin_add_overflow(a, b, &r);
}

void snapshot_add_pod(sr_snapshot* s, const sr_cluster* c, int32_t pod, int32_t pos);

// The pod carries required anti-affinity terms.
// strconv.ParseInt(string `id`, 10, 64) through the shim's table (false: does not parse / no table).
inline bool str_int(const sr_cluster* c, int32_t id, int64_t* v) {
  if (!c->str_int || !c->str_int_ok || id < 0 || id >= c->n_strings || !c->str_int_ok[id]) return false;
  *v = c->str_int[id];
  return true;
}
// labels.NewRequirement's key / value validation through the shim's table
// (sr_cluster.str_label; false without a table: callers route to fallback first).
inline bool label_str_ok(const sr_cluster* c, int32_t id, uint8_t what) {
  return c->str_label && id >= 0 && id < c->n_strings && (c->str_label[id] & what) == what;
}
// Every key / value of requirement (key, vals[lo, hi)) passes NewRequirement's validation.
inline bool label_req_strings_ok(const sr_cluster* c, int32_t key, const int32_t* vals, int32_t lo, int32_t hi) {
  if (!label_str_ok(c, key, SR_STR_LABEL_KEY)) return false;
  for (int32_t v = lo; v < hi; ++v)
    if (!label_str_ok(c, vals[v], SR_STR_LABEL_VALUE)) return false;
  return true;
}
// The pod lists scalar resources (sr_cluster.pod_scalar_*).
inline bool has_scalars(const sr_cluster* c, int32_t pod) {
  return c->pod_scalar_off && c->pod_scalar_off[pod + 1] > c->pod_scalar_off[pod];
}
// NodeInfo.AddPod's accounting of resource r (0 cpu, 1 memory, 2 ephemeral) for the pod.
// Which optional tables the cluster passes: what a stamped pod derives depends
// on them too, so memos keyed by pod_stamp are valid under one shape only.
inline uint64_t cluster_shape(const sr_cluster* c) {
  return 1 | (c->str_int ? 2u : 0u) | (c->str_label ? 4u : 0u) | (c->pod_affinity ? 8u : 0u) |
         (c->spread ? 16u : 0u) | (c->pod_scalar_off ? 32u : 0u) | (c->volumes ? 64u : 0u) |
         (c->acc_milli_cpu ? 128u : 0u);
}

inline int64_t pod_acc(const sr_cluster* c, int32_t pod, int r) {
  const sr_pods& P = c->pods;
  switch (r) {
    case 0: return c->acc_milli_cpu ? c->acc_milli_cpu[pod] : P.req_milli_cpu[pod];
    case 1: return c->acc_memory ? c->acc_memory[pod] : P.req_memory[pod];
    default: return c->acc_ephemeral ? c->acc_ephemeral[pod] : P.req_ephemeral[pod];
  }
}
// The pod carries DoNotSchedule topology spread constraints (sr_cluster.spread).
inline bool has_spread(const sr_cluster* c, int32_t pod) {
  return c->spread && c->spread->off[pod + 1] > c->spread->off[pod];
}
// PodTopologySpread (spread.cpp): constraint k's selector fails to build
// (LabelSelectorAsSelector); the pod's constraints as canonical words
// {namespace, n, per constraint {maxSkew, topologyKey, selects the pod itself,
// nil, n matchLabels, (key, value)*, n matchExpressions, (key, op, n, values)*}};
// the node row of such words against the base snapshot, given the pod's
// NodeAffinity row (nodes passing its nodeSelector / required affinity).
bool spread_invalid(const sr_cluster* c, int32_t k);
bool spread_selects(const sr_cluster* c, int32_t k, int32_t pod);
void spread_words(const sr_cluster* c, int32_t pod, std::vector<int32_t>& out);
// One encode's view of the snapshot for the spread rows (spread.cpp), built
// lazily: per topology key the spot nodes' values and a node bitset per value,
// and the snapshot pods per (label key, value), so a constraint with a
// matchLabels pair counts only the pods carrying it (a Deployment's replicas)
// instead of every snapshot pod.
struct SpreadIndex {
  struct KeyView {
    std::vector<int32_t> val;     // [n_spot] the node's value (INT32_MIN: no such label)
    std::vector<int32_t> values;  // distinct values
    std::vector<uint64_t> bits;   // [values][Wp] nodes carrying each value
    std::vector<uint64_t> has;    // [Wp] nodes carrying the key
    std::vector<int32_t> slot;    // [n_spot] the value slot of the node's pair (a node without the key: the
                                  // slot of "" when some node carries ""), -1 none
  };
  explicit SpreadIndex(const sr_snapshot* s);
  const KeyView& key(int32_t k);
  // snapshot pods carrying label (k, v): (spot position, SnapPod index); null: none
  const std::vector<std::pair<int32_t, int32_t>>* pods_with(int32_t k, int32_t v);
  const sr_snapshot* snap;
  int32_t n_spot, Wp;
  std::unordered_map<int32_t, KeyView> keys;
  // the label values the call's constraints select on, registered before the
  // first query (want); a query finds its pods in a per-key column built by
  // one parallel pass over the snapshot's pods for every wanted value of the
  // key (an unregistered value rebuilds the column with it)
  void want(int32_t k, int32_t v) { wanted[k].push_back(v); }
  std::unordered_map<int32_t, std::vector<int32_t>> wanted;
  struct LabelCol {
    std::unordered_map<int32_t, std::vector<std::pair<int32_t, int32_t>>> pods;  // value -> (spot position, pod)
  };
  std::unordered_map<int32_t, LabelCol> by_key;
};
// The snapshot-side state of one encode's spread rows and domain-path tables
// that a reuse encode (CandReuse) brings up to date node by node (spread.cpp):
// per distinct selector (namespace + selector words) the spot nodes' counts of
// the snapshot pods it counts, and per row / table entry the selectors and
// static inputs it was computed from.
struct SpreadReuse;
struct AntiReuse;  // antiaff.cpp
std::shared_ptr<SpreadReuse> spread_reuse_new(const sr_snapshot* snap, int32_t Wp);
// Constraints in `dmask` (bit k: the k-th) keep only their key check
// (SpreadDyn).  `keep`: registers the row as atom `atom` of the workload.
void spread_row(SpreadIndex& ix, const int32_t* words, const uint64_t* aff_row, uint32_t dmask, uint64_t* row,
                SpreadReuse* keep = nullptr, int32_t atom = -1);
// {namespace, nil, n matchLabels, (key, value)* sorted, n matchExpressions,
// (key, op, n, values sorted)*}: constraint k's counting selector for a pod of
// namespace `ns` (the counters' key).
void spread_selector_words(const sr_cluster* c, int32_t ns, int32_t k, std::vector<int32_t>& out);
// A domain-path table entry of analyse_spread (node-local key: tab[off + n]
// for every spot node, `pairs` its pairs; table key: tab[off + d] per domain).
void spread_reuse_slot(SpreadReuse& R, const std::vector<int32_t>& sel_words, const std::vector<int32_t>& node_cnt,
                       uint32_t off, bool node_local, const std::vector<uint64_t>& pairs, int32_t skew, int32_t self,
                       int32_t n_counted, const std::vector<int32_t>& dom, uint64_t pm, int32_t edom);
// Brings the rows (atoms) and tables to the snapshot after the pods of `nodes`
// changed; the atoms whose rows changed and the row words touched are
// appended.  False: a table's minimum could now move under the candidate
// (the full encode would send it to the reference path).
bool spread_reuse_patch(SpreadReuse& R, const sr_snapshot* snap, const std::vector<int32_t>& nodes, uint64_t* A,
                        std::vector<int32_t>& tab, bool* tab_changed, std::vector<int32_t>& atoms,
                        std::vector<int32_t>& words);
// The spot order moved: the per-position state and the node-local table
// entries of `tab` follow their nodes.
void spread_reuse_permute(SpreadReuse& R, const std::vector<int32_t>& src, const std::vector<int32_t>& moved,
                          std::vector<int32_t>& tab);
// Position-indexed helpers of the permutations (src[i]: the previous position
// of the node now at i; moved: the positions with src[i] != i).
template <class T>
void permute_positions(T* v, const std::vector<int32_t>& src, const std::vector<int32_t>& moved) {
  std::vector<T> tmp(moved.size());
  for (size_t q = 0; q < moved.size(); ++q) tmp[q] = std::move(v[src[moved[q]]]);
  for (size_t q = 0; q < moved.size(); ++q) v[moved[q]] = std::move(tmp[q]);
}
// A [Wp] row whose bits follow their nodes: through the moved positions, or,
// for a row with fewer set bits than that, through its set bits (`to`: new
// position of every previous one).
inline void permute_bits(uint64_t* row, int32_t Wp, const std::vector<int32_t>& src, const std::vector<int32_t>& moved,
                         const std::vector<int32_t>& to) {
  if (moved.size() <= 256) {  // few moved positions: through them
    uint8_t tmp[256];
    for (size_t q = 0; q < moved.size(); ++q) tmp[q] = static_cast<uint8_t>(row[src[moved[q]] >> 6] >> (src[moved[q]] & 63) & 1);
    for (size_t q = 0; q < moved.size(); ++q) {
      const int32_t i = moved[q];
      const uint64_t bit = 1ull << (i & 63);
      row[i >> 6] = tmp[q] ? (row[i >> 6] | bit) : (row[i >> 6] & ~bit);
    }
    return;
  }
  size_t pop = 0;
  for (int32_t i = 0; i < Wp; ++i) pop += static_cast<size_t>(__builtin_popcountll(row[i]));
  if (pop == 0) return;
  if (pop < moved.size()) {
    int32_t set[64];
    size_t k = 0;
    bool small = pop <= 64;
    if (small) {
      for (int32_t i = 0; i < Wp; ++i)
        for (uint64_t m = row[i]; m; m &= m - 1) set[k++] = i * 64 + __builtin_ctzll(m);
      for (int32_t i = 0; i < Wp; ++i) row[i] = 0;
      for (size_t q = 0; q < k; ++q) row[to[set[q]] >> 6] |= 1ull << (to[set[q]] & 63);
      return;
    }
    std::vector<int32_t> bits;
    bits.reserve(pop);
    for (int32_t i = 0; i < Wp; ++i)
      for (uint64_t m = row[i]; m; m &= m - 1) bits.push_back(i * 64 + __builtin_ctzll(m));
    for (int32_t i = 0; i < Wp; ++i) row[i] = 0;
    for (int32_t b : bits) row[to[b] >> 6] |= 1ull << (to[b] & 63);
    return;
  }
  std::vector<uint8_t> tmp(moved.size());
  for (size_t q = 0; q < moved.size(); ++q) tmp[q] = static_cast<uint8_t>(row[src[moved[q]] >> 6] >> (src[moved[q]] & 63) & 1);
  for (size_t q = 0; q < moved.size(); ++q) {
    const int32_t i = moved[q];
    const uint64_t bit = 1ull << (i & 63);
    row[i >> 6] = tmp[q] ? (row[i >> 6] | bit) : (row[i >> 6] & ~bit);
  }
}
// new position of every previous position
inline std::vector<int32_t> permute_targets(int32_t n, const std::vector<int32_t>& src, const std::vector<int32_t>& moved) {
  std::vector<int32_t> to(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; ++i) to[i] = i;
  for (int32_t i : moved) to[src[i]] = i;
  return to;
}
// The same by a scan of every snapshot pod (SR_SPREAD_CHECK=1 compares both).
void spread_row_scan(const sr_snapshot* snap, const int32_t* words, const uint64_t* aff_row, uint32_t dmask,
                     uint64_t* row);
// Per spot node, the snapshot pods constraint k counts (namespace `ns`, not terminating, selected).
void spread_node_counts(SpreadIndex& ix, const sr_cluster* c, int32_t k, int32_t ns, std::vector<int32_t>& out);
inline bool has_anti_terms(const sr_cluster* c, int32_t pod) {
  return (c->pods.flags[pod] & SR_POD_HAS_REQ_ANTI_AFFINITY) ||
         (c->pod_affinity && c->pod_affinity->anti_off[pod + 1] > c->pod_affinity->anti_off[pod]);
}
// Its required anti-affinity is outside the encoded set: no sr_pod_affinity,
// the flag without terms, or a selector LabelSelectorAsSelector rejects.
bool anti_opaque(const sr_cluster* c, int32_t pod);
// Its required pod affinity has a selector LabelSelectorAsSelector rejects.
bool aff_opaque(const sr_cluster* c, int32_t pod);
// The words of the pod's anti-affinity term t (antiaff.cpp): topology key,
// namespaces (defaulted to the owner's), selector; equal words = equal terms.
void anti_term_words(const sr_cluster* c, int32_t owner, int32_t t, std::vector<int32_t>& out);
// The snapshot's copy of a pod of `c` (SnapPod).
// The snapshot's copy of a pod's metadata; its labels go to (*k, *v)
// [lab, lab + their count), which the caller sized, its anti-affinity terms
// (rare) to `terms` (appended; callers on several threads pass their own).
void snap_pod_from(const sr_cluster* c, int32_t pod, SnapPod* out, int32_t* k, int32_t* v, uint32_t lab,
                   std::vector<int32_t>* terms);
inline uint32_t pod_label_count(const sr_cluster* c, int32_t pod) {
  const sr_pod_affinity* A = c->pod_affinity;
  return A ? static_cast<uint32_t>(A->label_off[pod + 1] - A->label_off[pod]) : 0u;
}

// Class descriptor flags.
enum : int32_t { CLS_AFF_REQUIRED = 1, CLS_IMPOSSIBLE = 2 };

// K2 domain path limits (antiaff.cpp, kernels.hip k2_domain)
constexpr int kDomKeys = 4;   // key slots per encode
constexpr int kDomMax = 64;   // domains of a table key (one bit each in a 64-bit mask)
constexpr int kDynTerms = 4;  // terms of an affinity set planned on the domain path
constexpr int kDynG = 8;      // domain path: mask words per pod set (64 pods each)
constexpr int kDynPods = 64 * kDynG;  // pods of a candidate planned on the domain path
constexpr int kSpreadSlots = 2;  // topology spread constraints per pod planned on the domain path
constexpr int kSpreadU64 = kSpreadSlots * (kDynG + 3);  // their words in the pod record
constexpr int kDynU64 = 5 * kDynG + 1 + kSpreadU64;  // words per pod record (kernels.hpp)
// K2 extension records (pod-order and domain paths): AddPod accounting that
// differs from the fit request, scalar resources shared inside a candidate
constexpr int kExtScalars = 2;      // shared scalar names per candidate
constexpr int kExtScalarNames = 8;  // shared scalar names per call (node_scal rows)
constexpr int kExtU64 = 8;          // {acc cpu, mem, eph, req s0, req s1, acc s0, acc s1, row s0 | row s1 << 32}
constexpr int kPodPatchWords = 3;   // {active pod, rec[4], rec[5]} (kernels.hpp kPodPatchU64)
constexpr int64_t kTSpare = INT64_MAX - 1;  // threshold of a spare T row (kernels.hpp kTPad)

// Candidate-side reuse (encode.cpp reuse_encode), one per Workload.  When a
// call's candidate input (lists, global indices, every pod stamped and
// unchanged) equals the one the Workload was last encoded for, and that side
// reads nothing from the snapshot but
// node capacities, pod counts, the spot pods' host ports, scalar usage and
// attachable volumes (no topology spread or inter-pod terms, no existing pod
// with anti-affinity), the Workload is kept: only the pod-count, composite,
// host-port conflict and scalar atom rows, the shared scalar rows, the T-row
// thresholds and the records of the pods whose T rows or dead flag moved are
// updated.  T rows are slots keyed by threshold value
// (a dimension's group has spare rows, kTPad), so a threshold that moves
// re-points only the pods asking within the moved interval.  The index is
// built by the second consecutive full encode of one input.
struct CandReuse {
  bool have_input = false;  // the last call's candidate input
  std::vector<int32_t> pod_off, pods, glob;
  std::vector<uint64_t> stamps;
  uint64_t shape = 0;
  bool indexed = false;  // the index below describes the Workload holding it
  uint64_t content_gen = 0;  // EncoderCache::content_gen it was built under (the classes name its ids)
  uint64_t static_gen = 0;
  int32_t n_spot = -1, Wp = 0;
  int32_t a_comp = 0;                          // first composite atom
  std::vector<int32_t> comp_sets;              // untolerated-taint set of each composite atom
  int32_t a_port = 0;                          // first host-port query atom
  std::vector<int32_t> port_q;                 // the queries {proto, port, ip}* of those atoms
  std::vector<uint64_t> port_scratch;          // their rows, recomputed by each reuse encode
  int32_t a_scalar = 0;                        // first scalar-resource / volume-limit query atom
  std::vector<std::pair<int64_t, int64_t>> scalar_q;  // their (name, request): rows recomputed by each reuse
  std::vector<int32_t> scal_names;             // shared scalar names of the extension records (node_scal rows)
  bool scalars = false;                        // some candidate pod lists scalar resources
  std::vector<uint64_t> att_words;             // attachable volumes of the planned candidates' pods: a spot node
                                               // that comes to hold one sends its candidate to the fallback path
  std::shared_ptr<AntiReuse> anti;             // DA / DB rows at a_anti (null: no inter-pod term in the call)
  int32_t a_anti = 0;
  std::shared_ptr<SpreadReuse> spread;         // spread rows and domain-path tables (null: no constraint)
  std::vector<uint8_t> atom_empty, atom_full;  // [n_atoms]
  std::vector<uint8_t> cls_empty;              // [classes before the empty class]
  std::vector<int32_t> pod_cls;                // [active pod] class before the dead check
  std::vector<int32_t> pod_ri;                 // [active pod][3] distinct request (-1: zero-request pod)
  std::vector<int64_t> vals[3];                // the node values the thresholds below were taken from
  std::vector<int64_t> dreq[3], dthr[3];       // distinct requests, their threshold (node value >= it)
  std::vector<int32_t> drow[3];                // ... and T row
  std::vector<int32_t> dpod_off[3], dpod[3];   // CSR distinct request -> active pods
  std::vector<int32_t> cls_pod_off, cls_pod;   // CSR class -> active pods
  std::unordered_map<int64_t, int32_t> row_of[3];  // threshold -> T row
  std::vector<int32_t> row_refs;               // [T row] distinct requests on it
  std::vector<int32_t> spare[3];               // free T rows of each dimension's group
  std::vector<uint32_t> mark;                  // [active pod] epoch of the last patch
  uint32_t epoch = 0;
  void drop() {
    have_input = indexed = false;
    anti.reset();
    spread.reset();
  }
};

// The encoded workload of one planning call (host copy; uploaded as one
// arena).  The spot nodes' state (capacity records, free values) lives in the
// EncoderCache and is uploaded only when it changes.
struct Workload {
  // ---- dimensions
  int32_t n_spot = 0;   // spot nodes
  int32_t n_pad = 0;    // node arrays padded to Wp*64 entries
  int32_t Wp = 0;       // 64-bit words per bitmask row (even)
  uint64_t state_gen = 0;  // EncoderCache state the workload refers to (node_rec / node_free)
  uint64_t layout_gen = 0; // EncoderCache node order its atom rows follow
  // ---- atom rows [n_atoms][Wp]: node bitsets every static predicate is built from
  //   atom 0                 len(pods)+1 <= allowed pods
  //   atoms 1 .. R           node matches requirement r (nodeSelector pair, matchExpression, matchField)
  //   atoms R+1 .. R+T       node carries NoSchedule/NoExecute taint t (incl. the unschedulable pseudo-taint)
  //   atoms R+T+1 .. +Q      node's base UsedPorts conflict with host port query q
  //   then anti-affinity DA/DB pairs and composite (pod count AND NOT untolerated taints) atoms
  int32_t n_atoms = 0;
  std::vector<uint64_t> atoms;
  // ---- static pod classes as atom programs:
  //   S[c] = AND(and atoms) & AND(~not atoms) & [OR over terms of AND(term atoms)]
  int32_t n_classes = 0;
  int32_t empty_class = -1;  // all-zero S row for pods whose F row is certainly empty (-1: none)
  std::vector<int32_t> cls_prog_off, cls_prog;  // CSR class -> ops (atom << 2 | PROG_*)
  std::vector<int32_t> cls_prog8;               // [n_classes][8] the same ops, -1 padded; -2: longer program
  // ---- T rows: capacity thresholds.  Row 0 = every node (zero-request pods
  // skip the resource checks); other rows: free_<dim>[n] >= thr.
  std::vector<int32_t> t_dim;   // 0 cpu, 1 memory, 2 ephemeral, 3 all
  std::vector<int64_t> t_thr;
  int32_t t_off[5] = {0, 0, 0, 0, 0};  // rows [t_off[i], t_off[i+1]): all, cpu, memory, ephemeral
  // ---- active pods, grouped by candidate, in podsForDeletion order
  std::vector<int32_t> pod_rows;  // [n][4]: S row (class), T rows for cpu, memory, ephemeral
  std::vector<uint64_t> pod_rec;  // [n + 128][6] AoS {cpu, memory, ephemeral, state bits, rows} for K2
  // state bits of a node / the bits a pod sets: anti-affinity pairs and host-port
  // pairs in [0, swap region) (pair-swapped to get the bits a pod conflicts with),
  // single host-port bits above them
  uint64_t swap_mask = 0;
  std::vector<int32_t> pod_src;  // index into the caller's cand_pods array
  // ---- active candidates
  std::vector<int32_t> cand_off;     // [n_active+1] into active pods
  std::vector<int32_t> cand_global;  // global candidate index
  std::vector<int32_t> cand_src;     // index in the caller's candidate list
  std::vector<int32_t> list;  // [n][4] K2 work list {candidate, first pod, end pod, global}, longest first
  int32_t max_cand_pods = 0;
  // A large work list with domain-path candidates in two parts (planner.cpp
  // k2_split): the first n_list_node entries are node-order candidates
  // (max_np_node their largest pod count), then the rest (domain path, more
  // than 256 pods: the general kernel).  0: one part, the list in plain order.
  int32_t n_list_node = 0, max_np_node = 0;
  // reorder_list_by_cost moved the costliest entries of the first part to the
  // front of the list (the node-order kernel's cooperative blocks take them)
  int32_t n_coop_front = 0;
  // ---- domain path: candidates whose pods interact through a topology key
  // with shared domains (antiaff.cpp), planned by K2's k2_domain
  std::vector<int32_t> dyn_cand;  // [n_active] first record in dyn_pod, -1: other paths (empty: none)
  std::vector<uint64_t> dyn_pod;  // [pods of those candidates][kDynU64]: anti-affinity masks per
                                  // key slot (earlier pods of the candidate it interacts with),
                                  // affinity mask (earlier pods matching every term of its set),
                                  // set << 1 | matches its own terms (~0: none), then per spread
                                  // slot the earlier pods its constraint counts and 3 info words
                                  // (SpreadDyn)
  std::vector<int32_t> sp_tab;    // spread base counts per domain / caps per node (SpreadDyn::tab)
  int32_t n_dk = 0;               // key slots in use
  std::vector<int32_t> dk_dom;    // [n_dk][n_spot] domain of each spot node (node-local key: the node), -1 absent
  int32_t dk_row[kDomKeys] = {-1, -1, -1, -1};  // atom of domain 0 of each table key (-1: node-local key)
  std::vector<int32_t> ds_info;   // [set][2 + 2 * kDynTerms] {terms, map_empty, (key slot, base atom) per term}
  // ---- extension records (kExtU64 per pod of the candidates that need them)
  std::vector<int32_t> ext_cand;  // [n_active] first record in pod_ext, -1: none (empty: no such candidate)
  std::vector<uint64_t> pod_ext;
  std::vector<int32_t> list_ext;  // [n][4] per work-list entry {first record (-1: none), node_scal row of slot 0,
                                  // of slot 1 (-1: no slot), 0}: K2 reads it with the entry (no dependent loads)
  int32_t n_scal_names = 0;
  std::vector<int64_t> node_scal; // [n_scal_names][n_pad] alloc - requested of each shared scalar name
  // ---- host-decided outcomes for every input candidate
  std::vector<int32_t> status_host;  // SR_CAND_EMPTY / SR_CAND_FALLBACK / PENDING
  int32_t first_fallback = -1;       // global index
  uint64_t fallback_pods = 0;
  int32_t n_input_cand = 0;
  int32_t n_input_pods = 0;
  int32_t pod_base = 0;  // cand_pod_off[0] of the call: pod_src - pod_base indexes its pods
  // ---- candidate-side reuse (EncoderCache::CandReuse): every array above
  // except atoms, t_thr and the node state belongs to candidate generation
  // cand_gen; a reuse encode keeps them and lists the pod records it changed
  uint64_t cand_gen = 0;
  bool reused = false;
  bool class_flip = false;          // a reuse encode moved some pod to or from the empty class
  std::vector<uint64_t> pod_patch;  // [n][kPodPatchWords] {active pod, rec[4], rec[5]} (reuse encodes)
  std::vector<int32_t> atom_cols;   // row words a reuse encode changed in the inter-pod / spread atoms (beyond the
                                    // changed nodes' own words: a zone's nodes, a moved minimum), sorted
  bool tab_changed = false;         // a reuse encode rewrote sp_tab entries
  // version of `atoms` (a new one per encode that changes any row); a reuse
  // encode that moved rows lists them (atom_rows_all: too many to list, or a
  // permutation) against the version it started from
  uint64_t atoms_ver = 0, atoms_prev_ver = 0;
  std::vector<int32_t> atom_rows;
  bool atom_rows_all = false;
  CandReuse reuse;                  // kept by reset(): the encoder rebuilds or drops it

  // Back to the default state, keeping every buffer's capacity: a planner
  // encodes one tick after another, and fresh multi-MB buffers page-fault.
  void reset() {
    t_thr.clear();
    for (auto* v : {&cls_prog_off, &cls_prog, &cls_prog8, &t_dim, &pod_src, &cand_off, &cand_global, &cand_src, &list,
                    &status_host, &dyn_cand, &dk_dom, &ds_info, &sp_tab, &ext_cand, &list_ext})
      v->clear();
    dyn_pod.clear();
    pod_ext.clear();
    node_scal.clear();
    n_scal_names = 0;
    n_dk = 0;
    for (int32_t& r : dk_row) r = -1;
    atoms.clear();
    // pod_rows / pod_rec keep their size: the encoder resizes them and writes
    // every field, so a steady-state encode does not zero-fill them first
    n_spot = n_pad = Wp = n_atoms = n_classes = 0;
    state_gen = 0;
    empty_class = -1;
    swap_mask = 0;
    for (int32_t& t : t_off) t = 0;
    max_cand_pods = 0;
    n_list_node = max_np_node = 0;
    n_coop_front = 0;
    first_fallback = -1;
    fallback_pods = 0;
    n_input_cand = n_input_pods = pod_base = 0;
    reused = false;
    class_flip = false;
    pod_patch.clear();
    atom_cols.clear();
    tab_changed = false;
  }
};

// A distinct static pod spec (nodeSelector, required node affinity,
// tolerations, host ports), canonical and independent of the nodes.
struct SpecInfo {
  int32_t flags = 0;           // CLS_AFF_REQUIRED, CLS_IMPOSSIBLE
  std::vector<int32_t> sel;    // requirement ids of the nodeSelector pairs, sorted
  std::vector<int32_t> terms;  // per buildable required term: {n, requirement ids sorted}
  int32_t n_terms = 0;
  std::vector<int32_t> tol;    // Spec.Tolerations {key, op, value, effect}*
  std::vector<int32_t> ports;  // host ports {protocol, port, ip}* with port > 0
  std::vector<int64_t> scalars;  // scalar resources {name, fit request}*, sorted by name
  std::vector<int32_t> spread;   // DoNotSchedule topology spread constraints (spread_words), empty: none
  std::vector<int32_t> vsel;     // volume filters: requirement ids ANDed (VolumeZone REQ_ZONE, one-term PV affinity)
  std::vector<int32_t> vpv;      // PV selectors with several terms (EncoderCache::pvsel_dict ids), sorted
  uint64_t untol_gen = ~0ull;  // static generation `untol` was computed for
  int32_t untol = -1;          // set of spot-pool taints it does not tolerate (EncoderCache::untol_dict)
  uint64_t psig_gen = ~0ull;   // static generation `psig` was interned for
  int32_t psig = -1;           // its class signature (EncoderCache::psig_dict) when it asks for no host port
};

// What the encoder keeps across calls (one per sr_ctx).  The spot pool is
// compared position by position against the last call's view through two
// fingerprints per node: the static one (name, labels, taints, unschedulable)
// and the state one (allocatable, requested, pod count, host ports).  Data
// derived from an unchanged view is reused: label columns, requirement rows
// and taint rows (static), capacity records, free values and their sorted
// distinct values (state).  Specs, requirements and untolerated-taint sets are
// interned by content; all of it is dropped when the interned ids of "",
// "metadata.name" or the unschedulable key change, or when the dictionaries
// grow past their bounds.
struct EncoderCache {
  // ---- per-context settings (sr_create reads them from the environment)
  int32_t list_head = 512;    // SR_LIST_HEAD: candidates dispatched ahead of the longest-first rest (round 6:
                              //   512 instead of 1,024 -- C4 step 44.7 -> 42.6 us, C4 / affinity C4 latency -3 us)
  int32_t split_min = 4096;   // SR_K2_SPLIT_MIN: a work list with domain-path candidates and more entries than
                              //   this goes in two parts (planner.cpp k2_split)
  int32_t id_empty = INT32_MIN, id_metadata_name = INT32_MIN, id_unschedulable_key = INT32_MIN;
  // ---- static view
  int32_t n_spot = -1, Wp = 0, n_pad = 0;
  std::vector<int32_t> names;       // spot order (interned node names)
  std::vector<uint64_t> static_fp;  // per position
  uint64_t static_gen = 0;
  std::deque<std::pair<int32_t, std::vector<int32_t>>> label_col;  // key -> value per position (INT32_MIN: absent);
                                                                  // a deque: columns stay put while more are added
  std::vector<TaintRec> taints;     // NoSchedule / NoExecute taints of the pool + the unschedulable pseudo-taint
  std::vector<uint64_t> taint_rows; // [taint][Wp]
  std::vector<uint64_t> req_row_gen;             // [req] static generation of its row (~0: none)
  std::vector<std::vector<uint64_t>> req_rows;   // [req][Wp]
  // The same nodes (names, static fingerprints) in another order: the view is
  // permuted, not rebuilt (the spot order follows RequestedCPU, which moves
  // whenever pods come or go).  layout_gen counts permutations; perm_src[i] is
  // the previous position of the node now at i, perm_k the positions that
  // moved; perm_dirty hands them to the state view as changed nodes.
  uint64_t layout_gen = 0;
  std::vector<int32_t> perm_src, perm_k, perm_dirty, pos_scratch;
  std::vector<int32_t> perm_to;  // new position of every previous one
  // ---- state view
  std::vector<uint64_t> state_fp;
  bool state_valid = false;  // the arrays below describe the current static view
  uint64_t state_gen = 0;
  std::vector<uint64_t> node_rec;      // [n_pad][8] {free cpu, mem, eph, state bits (0), pods left, 0, 0, 0}
  std::vector<int64_t> node_free;      // [3][n_pad] free cpu / memory / ephemeral (pads: INT64_MIN)
  std::vector<uint64_t> podcount_row;  // [Wp] len(pods)+1 <= allowed pods
  std::vector<int64_t> sorted_free[3]; // every node's free value, sorted
  std::vector<int64_t> node_vals[3];   // distinct free values, sorted
  // base UsedPorts conflict rows by query (proto, port, ip), valid for state
  // generation port_rows_gen (patched node by node when few nodes changed)
  std::unordered_map<uint64_t, std::vector<uint64_t>> port_rows;
  uint64_t port_rows_gen = ~0ull;
  // ---- content-interned, node independent
  struct SpecShard {
    WordDict dict;               // static spec words -> local id
    std::vector<int32_t> global; // local id -> spec id
  };
  std::vector<SpecShard> spec_shards;  // by spec-word hash (a fixed count: ids do not depend on threads)
  std::vector<SpecInfo> spec;          // [spec id]; spec 0 = no static constraints
  std::vector<uint32_t> spec_req_off{0};  // [spec id + 1] the specs' requirement ids (selector, then
  std::vector<int32_t> spec_req;          //   terms), flat: the per-call key pass reads them in key order
  WordDict req_dict;                   // requirement words {type, key, op, vals...} -> requirement id
  WordDict pvsel_dict;                 // PV selectors {n terms, per term {n, requirement ids}} -> id
  WordDict untol_dict;                 // untolerated-taint sets (valid for untol_gen)
  uint64_t untol_gen = ~0ull;
  WordDict psig_dict;                  // class signatures of port-free specs (valid for psig_gen)
  uint64_t psig_gen = ~0ull;
  // ---- per-call scratch (kept: fresh multi-MB buffers page-fault on every call)
  struct Scratch {
    std::vector<uint8_t> cand_ports, spec_shard, key_seen, cand_ext;
    std::vector<int32_t> cand_sname;
    std::vector<int32_t> active_pod, active_src, act_of, pod_spec, pod_key, key_slot, psig_class;
    std::vector<uint64_t> spec_hash;
    std::vector<int64_t> req_flat;  // [input candidate pod][3] requests (cpu, memory, ephemeral)
    std::vector<uint32_t> spec_woff;
    std::vector<std::vector<int32_t>> spec_words, chunk_shard;
  } scratch;
  // ---- per-pod memo by (pod index, sr_cluster.pod_stamp): the spec id and
  // the snapshot-independent part of the candidate checks of pods the shim
  // stamped, valid while the stamp, the content dictionaries (spec ids) and
  // the cluster's table shape are unchanged
  struct PodMemo {
    uint64_t stamp_spec = 0;  // stamp `spec` was derived for (0: none)
    uint64_t stamp_bits = 0;  // stamp `bits` were derived for (0: none)
    int32_t spec = 0;
    uint32_t bits = 0;        // MEMO_* (encode.cpp)
  };
  std::vector<PodMemo> pod_memo;
  uint64_t memo_shape = 0;
  int32_t last_memo_hits = 0;
  // ---- per-call counters (bench: what the last call had to rebuild)
  int32_t last_new_specs = 0, last_static_changed = 0, last_state_changed = 0;
  // the last state refresh patched these nodes' records on top of generation
  // patched_from (~0: it rebuilt them all); the planner uploads only those
  std::vector<int32_t> patched_nodes;
  uint64_t patched_from = ~0ull;
  std::vector<int32_t> content_nodes;  // ... of which these changed their own state (not only their position)
  uint64_t content_from = ~0ull;
  uint64_t cand_gen_next = 1;
  uint64_t atoms_ver_next = 1;  // Workload::atoms_ver
  int32_t last_reused = 0, last_pod_patches = 0;

  uint64_t content_gen = 0;  // bumped by clear_content (a Workload's CandReuse is valid for one value)

  void clear_content() {  // drops every content-interned dictionary
    ++content_gen;        // reuse indices: their classes and atoms name them
    pod_memo.clear();     // its spec ids index them
    spec_shards.clear();
    spec.clear();
    spec_req_off.assign(1, 0);
    spec_req.clear();
    req_dict.clear();
    pvsel_dict.clear();
    req_rows.clear();
    req_row_gen.clear();
    untol_dict.clear();
    untol_gen = ~0ull;
    psig_dict.clear();
    psig_gen = ~0ull;
  }
};

constexpr int32_t STATUS_PENDING = -100;
constexpr int32_t MAX_CAND_PODS = 512;  // pods per candidate on the device (K2 kMaxPods)
constexpr int32_t MAX_WORDS = 64 * 32; // spot nodes <= 131072

// Required pod anti-affinity of one encode (antiaff.cpp).
// Topology keys through which the pods of one candidate interact with
// shared domains (zone-style keys; node-local keys for affinity): K2's domain
// path tracks, per candidate, the domains its placed pods occupy.

struct DomKeys {
  std::vector<int32_t> key;               // [slot] label key id
  std::vector<uint8_t> node_local;        // [slot] every spot node carries it, values pairwise distinct
  std::vector<std::vector<int32_t>> dom;  // [slot][n_spot] domain id (node-local: the node), -1 absent
  std::vector<int32_t> n_dom;             // [slot] domains (node-local: n_spot)
  // The slot of `key`, registered (its domains computed) on first use; -1
  // when the slots are full or a shared-domain key has more than kDomMax values.
  int32_t slot(const sr_snapshot* snap, int32_t key);
};

struct AntiTerms {
  bool active = false;
  int32_t base = 0;                      // cand_pod_off[0]: per-pod arrays are indexed by flat index - base
  int32_t n_terms = 0;
  std::vector<uint8_t> node_local;       // [term] every spot node has the key, values pairwise distinct
  std::vector<uint64_t> da, db;          // [term][Wp] base conflicts: pods having / selected by the term
  std::vector<uint8_t> da_any, db_any;   // [term] the set is not empty
  std::vector<int32_t> pod_off, pod_ids; // [flat candidate pod - base + 1] -> ids: term << 1 (selects it) | 1 (it has)
  std::vector<uint64_t> pod_bits;         // [flat candidate pod] state-bit pairs it sets, numbered per
                                         // candidate (A = 2p: it has term p, B = 2p + 1: term p selects it)
  int32_t n_pairs = 0;                   // most pairs any candidate uses (<= 32)
  // domain path: candidates interacting through shared-domain keys, and per
  // flat pod of those, the earlier pods of its candidate it interacts with
  // through each key slot ([flat - base][kDomKeys]; empty: no such candidate)
  std::vector<uint8_t> cand_dyn;         // [candidate]
  std::vector<uint64_t> amask;          // [flat - base][kDomKeys][kDynG]
};

// Collects the terms of the snapshot's pods and of the pending candidates,
// builds the static node sets and decides which candidates fall back
// (status -> SR_CAND_FALLBACK) or need state bits.
// `keep`: also builds the state a reuse encode patches (AntiReuse).
struct AntiReuse;
void analyse_anti(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands, int32_t Wp,
                  std::vector<int32_t>& status, DomKeys* dk, AntiTerms* out,
                  std::shared_ptr<AntiReuse>* keep = nullptr);
// Brings the DA / DB atom rows (DA(t) at a_anti + 2t, DB(t) at a_anti + 2t + 1)
// to the snapshot after the pods of `nodes` changed; the atoms whose rows
// changed and the row words touched are appended.  False: a change the reuse
// cannot follow -- a term it never saw that may select a candidate pod, or a
// set that was empty when the class programs were emitted and no longer is.
bool anti_reuse_patch(AntiReuse& R, const sr_snapshot* snap, const std::vector<int32_t>& nodes, uint64_t* A,
                      int32_t a_anti, std::vector<int32_t>& atoms, std::vector<int32_t>& words);
// The spot order moved (EncoderCache::perm_src / perm_k): the per-position
// state follows its nodes.
void anti_reuse_permute(AntiReuse& R, const std::vector<int32_t>& src, const std::vector<int32_t>& moved);

// Required pod affinity of one encode (antiaff.cpp).
struct AffTerms {
  bool active = false;
  int32_t base = 0;                 // per-pod arrays: flat index - base
  int32_t n_sets = 0;               // distinct term sets of the pending pods
  std::vector<uint64_t> sat, keys;  // [set][Wp] SAT(S) (keys and a matching pod in every term's domain), KEYS(S)
  std::vector<uint8_t> map_empty;   // [set] no matching pod on a node carrying any of the keys
  std::vector<int32_t> pod_code;    // [flat - base] -1 none, else 2 * set + (the pod matches its own terms)
  // domain path: candidates in which an earlier pod matches every term of a
  // later pod's set; per flat pod the mask of those earlier pods (0: static
  // SAT(S) is exact); per set planned there, each term's key slot and base row
  std::vector<uint8_t> cand_dyn;    // [candidate]
  std::vector<uint64_t> mmask;      // [flat - base][kDynG] (empty: no such candidate)
  std::vector<uint8_t> set_dyn;     // [set]
  std::vector<std::vector<int32_t>> set_slots;     // [set][term] key slot (sets planned dynamically)
  std::vector<std::vector<uint64_t>> term_rows;    // [set][term * Wp] nodes whose domain hosts a base pod of M(S)
};

// The sets, their node rows, and the candidates whose pods interact through
// them (status -> SR_CAND_FALLBACK).
void analyse_affinity(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands, int32_t Wp,
                      std::vector<int32_t>& status, DomKeys* dk, AffTerms* out);

// DoNotSchedule topology spread between the pods of one candidate (encode.cpp
// analyse_spread): a pod whose constraint counts earlier pods
// of its candidate is planned on the domain path.  Per such constraint (at
// most kSpreadSlots per pod) the record holds the mask of those earlier pods
// and three info words:
//   w0 = key slot | node-local << 2 | selects itself << 3 | maxSkew << 32
//   w1 = offset in `tab` | domain of the value "" << 32 (-1: none)  [table key]
//   w2 = the pairs' domains (bit per domain id)                        [table key]
// Table key: tab[offset + d] = the base count of domain d's pair; the device
// adds the earlier pods' domains, takes the minimum over the pairs and refuses
// the domains over maxSkew (the pod's atom keeps only the key check).
// Node-local key: tab[offset + n] = maxSkew - self + minimum - base count of
// node n (INT32_MAX off the pairs); the minimum cannot move (more nodes at it
// than the constraint counts pods in the candidate), so the pod's atom keeps
// the full base check and the device refuses the nodes whose count of earlier
// pods exceeds that cap.
struct SpreadDyn {
  bool active = false;
  int32_t base = 0;                // per-pod arrays: flat index - base
  std::vector<uint8_t> cand_dyn;   // [candidate]
  std::vector<uint64_t> rec;       // [flat - base][kSpreadU64] (empty: no such candidate)
  std::vector<uint8_t> dmask;      // [flat - base] bit k: the pod's k-th constraint is a device-planned table key
  std::vector<int32_t> tab;
  bool state_fb = false;           // a candidate went to the reference path on the base counts (n0 <= counted)
};

// The work list of a reused workload in the order of each candidate's wave
// duration in its last run (`cycles`, by active candidate), longest first,
// within the parts the list was built in (the head, the rest; the split
// launch's two kernels), after the n_front longest entries of the first part
// (the node-order kernel's), which go to the front (Workload::n_coop_front);
// list_ext follows.
void reorder_list_by_cost(Workload& w, const uint32_t* cycles, int32_t list_head, int32_t n_front);

// Builds the workload; returns SR_OK or an error with *err filled.  `cache`
// carries what the previous calls derived (and is updated).
sr_status encode_workload(EncoderCache* cache, const sr_snapshot* snap, const sr_cluster* c,
                          const sr_candidates* cands, Workload* w, std::string* err);

// Fingerprint of a spot node's static part (name, unschedulable, labels,
// taints): computed when the snapshot is created.
uint64_t node_static_fp(const SpotNode& n, const sr_cluster* c);
uint64_t node_state_fp(const SpotNode& sn, const NodeState& st);

}  // namespace sr
