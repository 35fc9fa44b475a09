// nodemap.cpp — nodes.NewNodeMap and the cluster snapshot (host side).
//
// NewNodeMap (nodes/nodes.go:63-104) with the per-node pod LIST
// (nodes/nodes.go:129-145) already resolved by the caller: pods carry their
// node index and arrive in LIST order.  Sorting uses the Go-exact sort.Slice of
// gosort.hpp.  GetClusterSnapshot (nodes/nodes.go:226-232) and the
// ClusterSnapshot operations the planner needs (AddPod / Fork / Revert,
// rescheduler.go:269,273,366) live here too.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <functional>
#include <vector>

#include "gosort.hpp"
#include "host.hpp"
#include "pool.hpp"
#include "worddict.hpp"

// Per-node pod sorts of earlier NewNodeMap calls (sr_new_node_map_cached),
// by node name: the stamps of the node's LISTed pods in list order, its kind,
// and the sorted kept pods as positions in that list.
struct sr_node_map_cache {
  struct Entry {
    int8_t kind = -1;
    uint32_t epoch = 0;             // the call that last claimed it (a repeated name is not cached)
    int64_t requested = 0;
    std::vector<uint64_t> stamps;   // every LISTed pod, list order
    std::vector<int32_t> perm;      // kept pods, sorted: positions in the list
  };
  // per-call buffers kept across calls (fresh multi-MB buffers page-fault)
  // and the last call's spot / on-demand sort: its input (key, node) pairs in
  // node order and its output
  struct Scratch {
    std::vector<int32_t> start, listed, cnt, nkept;
    std::vector<int8_t> kind;
    std::vector<uint8_t> hit;
  } scratch;
  std::vector<std::pair<int64_t, int32_t>> list_in[2], list_out[2];
  uint64_t shape = 0;
  sr_node_map_params params{};
  uint32_t epoch = 0;
  // calls made (sr_snapshot_refresh_cached links a snapshot to one call), and
  // whether the last one completed (scratch.hit: its nodes whose LISTed pods
  // equal the previous call's)
  uint64_t calls = 0;
  bool hit_valid = false;
  std::vector<int32_t> slot_of_name;  // [n_strings] -> entries, -1
  std::vector<Entry> entries;
  std::vector<int32_t> names, slot;   // the last call's node names and their entries (-1: none)
  void clear() {
    std::fill(slot_of_name.begin(), slot_of_name.end(), -1);
    entries.clear();
    names.clear();
    slot.clear();
    for (int k = 0; k < 2; ++k) list_in[k].clear(), list_out[k].clear();
  }
};

namespace sr {

// Phase timestamps of NewNodeMap / the snapshot refresh for tools/refresh_check's
// profiling build (-DSR_NM_PROFILE); compiled out otherwise.
#ifdef SR_NM_PROFILE
double nm_phase_ms[10];
#define NM_MARK(i)                                                                                     \
  do {                                                                                                 \
    const auto now_ = std::chrono::steady_clock::now();                                               \
    nm_phase_ms[i] = std::chrono::duration<double, std::milli>(now_ - nm_t_).count();                 \
    nm_t_ = now_;                                                                                      \
  } while (0)
#define NM_START() auto nm_t_ = std::chrono::steady_clock::now()
#else
#define NM_MARK(i) \
  do {             \
  } while (0)
#define NM_START() \
  do {             \
  } while (0)
#endif

// isSpotNode / isOnDemandNode (nodes/nodes.go:168-209).
static bool node_has_label(const sr_cluster* c, int32_t node, const sr_node_label* l) {
  const sr_nodes& N = c->nodes;
  int32_t val = c->id_empty;
  bool found = false;
  for (int32_t i = N.label_off[node]; i < N.label_off[node + 1]; ++i) {
    if (N.label_key[i] == l->key) {
      found = true;
      val = N.label_val[i];
      break;
    }
  }
  if (!l->has_value) return found;   // old label schema: key presence
  return val == l->value;            // labels[k] == v, missing key reads as ""
}

static bool same_label(const sr_node_label& a, const sr_node_label& b) {
  return a.key == b.key && a.value == b.value && a.has_value == b.has_value;
}

static sr_status new_node_map(const sr_cluster* c, const sr_node_map_params* p, sr_node_map* out,
                              sr_node_map_cache* cache, int32_t* out_sorted) {
  const sr_nodes& N = c->nodes;
  const sr_pods& P = c->pods;
  const int32_t nn = N.n, np = P.n;
  NM_START();
  if (cache) {
    ++cache->calls;
    cache->hit_valid = false;
  }
  // Per-node LIST results: counting sort by node index keeps list order.
  // Large clusters: K pod ranges counted and scattered in parallel, range k's
  // pods of a node placed after those of ranges < k (still list order).
  sr_node_map_cache::Scratch local;
  sr_node_map_cache::Scratch& W = cache ? cache->scratch : local;
  std::vector<int32_t>& start = W.start;
  std::vector<int32_t>& listed = W.listed;
  start.assign(static_cast<size_t>(nn) + 1, 0);
  if (listed.size() < static_cast<size_t>(np > 0 ? np : 1)) listed.resize(static_cast<size_t>(np > 0 ? np : 1));
  const size_t K = std::min<size_t>(pool_threads(), np >= (1 << 17) ? static_cast<size_t>(np) >> 16 : 1);
  if (K <= 1) {
    for (int32_t i = 0; i < np; ++i) {
      if (P.node[i] < -1 || P.node[i] >= nn) return SR_ERR_INVALID_ARG;
      if (P.node[i] >= 0) ++start[P.node[i] + 1];
    }
    for (int32_t i = 0; i < nn; ++i) start[i + 1] += start[i];
    std::vector<int32_t> cursor(start.begin(), start.end() - 1);
    for (int32_t i = 0; i < np; ++i)
      if (P.node[i] >= 0) listed[cursor[P.node[i]]++] = i;
  } else {
    std::vector<int32_t>& cnt = W.cnt;  // [range][node], then the range's cursor
    if (cnt.size() < K * static_cast<size_t>(nn)) cnt.resize(K * static_cast<size_t>(nn));
    std::atomic<bool> bad{false};
    auto range = [&](size_t k, int32_t* lo, int32_t* hi) {
      *lo = static_cast<int32_t>(static_cast<size_t>(np) * k / K);
      *hi = static_cast<int32_t>(static_cast<size_t>(np) * (k + 1) / K);
    };
    parallel_for(K, 1, [&](size_t a, size_t b) {
      for (size_t k = a; k < b; ++k) {
        int32_t lo, hi;
        range(k, &lo, &hi);
        int32_t* c = &cnt[k * static_cast<size_t>(nn)];
        std::fill(c, c + nn, 0);  // each range zeroes its own row
        for (int32_t i = lo; i < hi; ++i) {
          const int32_t nd = P.node[i];
          if (nd < -1 || nd >= nn) bad.store(true, std::memory_order_relaxed);
          else if (nd >= 0) ++c[nd];
        }
      }
    });
    if (bad.load()) return SR_ERR_INVALID_ARG;
    // per node: the per-range offsets and the total, a block of nodes at a
    // time with each range's row read in sequence (the rows lie nn apart)
    parallel_for(static_cast<size_t>(nn), 2048, [&](size_t a, size_t b) {
      int32_t acc[2048];
      std::fill(acc, acc + (b - a), 0);
      for (size_t k = 0; k < K; ++k) {
        int32_t* c = &cnt[k * static_cast<size_t>(nn)];
        for (size_t nd = a; nd < b; ++nd) {
          const int32_t x = c[nd];
          c[nd] = acc[nd - a];
          acc[nd - a] += x;
        }
      }
      for (size_t nd = a; nd < b; ++nd) start[nd + 1] = acc[nd - a];
    });
    for (int32_t i = 0; i < nn; ++i) start[i + 1] += start[i];
    parallel_for(K, 1, [&](size_t a, size_t b) {
      for (size_t k = a; k < b; ++k) {
        int32_t lo, hi;
        range(k, &lo, &hi);
        int32_t* c = &cnt[k * static_cast<size_t>(nn)];
        for (int32_t i = lo; i < hi; ++i) {
          const int32_t nd = P.node[i];
          if (nd >= 0) listed[start[nd] + c[nd]++] = i;
        }
      }
    });
  }

  const int64_t* cpu = P.cpu_sort_milli;
  NM_MARK(0);
  // the reference's less functions (nodes/nodes.go:76-80, 95-101) on (key, id) pairs: the same
  // comparisons, so Go's sort makes the same swaps
  using KV = std::pair<int64_t, int32_t>;
  auto by_key_desc = [](const KV& x, const KV& y) { return x.first > y.first; };
  auto by_key_asc = [](const KV& x, const KV& y) { return x.first < y.first; };
  std::vector<int8_t>& kind = W.kind;  // 1 spot, 2 on-demand
  kind.assign(static_cast<size_t>(nn), 0);
  parallel_for(static_cast<size_t>(nn), 256, [&](size_t lo, size_t hi) {
    for (size_t node = lo; node < hi; ++node) {
      const bool spot = node_has_label(c, static_cast<int32_t>(node), &p->spot);
      kind[node] = spot ? 1 : node_has_label(c, static_cast<int32_t>(node), &p->on_demand) ? 2 : 0;
    }
  });
  // The cache's entry per node (-1: none): valid for one cluster shape and
  // one set of params, stamped pods only.
  const uint64_t* stamps = c->pod_stamp;
  std::vector<int32_t> no_slot;
  const std::vector<int32_t>* slot_v = &no_slot;
  if (cache && stamps) {
    const uint64_t shape = cluster_shape(c);
    bool fresh = false;
    if (cache->shape != shape || !same_label(cache->params.spot, p->spot) ||
        !same_label(cache->params.on_demand, p->on_demand) ||
        cache->params.priority_threshold != p->priority_threshold ||
        cache->entries.size() > 2 * static_cast<size_t>(nn) + 1024) {
      cache->clear();
      cache->shape = shape;
      cache->params = *p;
      fresh = true;
    }
    const int32_t ns_str = c->n_strings;
    // the same node names in the same order as the last call: the same slots
    if (fresh || cache->names.size() != static_cast<size_t>(nn) ||
        !std::equal(N.name, N.name + nn, cache->names.begin())) {
      if (cache->slot_of_name.size() < static_cast<size_t>(ns_str))
        cache->slot_of_name.resize(static_cast<size_t>(ns_str), -1);
      const uint32_t ep = ++cache->epoch;
      std::vector<int32_t>& slot = cache->slot;
      slot.assign(static_cast<size_t>(nn), -1);
      for (int32_t node = 0; node < nn; ++node) {
        const int32_t nm = N.name[node];
        if (nm < 0 || nm >= ns_str) continue;
        int32_t& e = cache->slot_of_name[nm];
        if (e < 0) {
          e = static_cast<int32_t>(cache->entries.size());
          cache->entries.emplace_back();
        }
        auto& en = cache->entries[static_cast<size_t>(e)];
        if (en.epoch == ep) {  // a second node of this name: neither is cached
          en.kind = -1;
          for (int32_t m = 0; m < node; ++m)
            if (slot[m] == e) slot[m] = -1;
          continue;
        }
        en.epoch = ep;
        slot[node] = e;
      }
      cache->names.assign(N.name, N.name + nn);
    }
    slot_v = &cache->slot;
  }
  const std::vector<int32_t>& slot = *slot_v;
  NM_MARK(1);
  // Per node (independent, on the pool): the priority filter of
  // getPodsOnNode, RequestedCPU and the pod sort, or the cached sort of the
  // same stamped pods.  Pass 1 counts the kept pods, pass 2 writes them at
  // their prefix offsets.
  std::vector<int32_t>& nkept = W.nkept;
  std::vector<uint8_t>& hit = W.hit;
  nkept.assign(static_cast<size_t>(nn) + 1, 0);
  hit.assign(static_cast<size_t>(nn), 0);
  std::atomic<bool> nil_priority{false};
  parallel_for(static_cast<size_t>(nn), 64, [&](size_t lo, size_t hi) {
    for (size_t node = lo; node < hi; ++node) {
      const bool spot = kind[node] == 1;
      if (!slot.empty() && slot[node] >= 0) {
        const auto& en = cache->entries[static_cast<size_t>(slot[node])];
        const int32_t n = start[node + 1] - start[node];
        bool same = en.kind == kind[node] && static_cast<int32_t>(en.stamps.size()) == n;
        for (int32_t k = 0; k < n && same; ++k) {
          const uint64_t st = stamps[listed[start[node] + k]];
          same = st != 0 && st == en.stamps[static_cast<size_t>(k)];
        }
        if (same) {
          hit[node] = 1;
          nkept[node + 1] = static_cast<int32_t>(en.perm.size());
          continue;
        }
      }
      int32_t k = 0;
      for (int32_t j = start[node]; j < start[node + 1]; ++j) {
        const int32_t pod = listed[j];
        // int(*Spec.Priority) < PriorityThreshold && isSpotNode(node)  (:139);
        // the dereference comes first, so a nil priority panics on any node.
        if (!P.has_priority[pod]) nil_priority.store(true, std::memory_order_relaxed);
        else if (!(P.priority[pod] < p->priority_threshold && spot)) ++k;
      }
      nkept[node + 1] = k;
    }
  });
  if (nil_priority.load()) return SR_ERR_NIL_PRIORITY;
  for (int32_t node = 0; node < nn; ++node) nkept[node + 1] += nkept[node];
  NM_MARK(2);
  std::atomic<int32_t> sorted{0};
  parallel_for(static_cast<size_t>(nn), 64, [&](size_t lo, size_t hi) {
    std::vector<std::pair<int64_t, int32_t>> kv;  // (cpu, position in the node's list): the sort compares keys held in place
    int32_t my_sorted = 0;
    for (size_t node = lo; node < hi; ++node) {
      const bool spot = kind[node] == 1;
      const int32_t s0 = start[node];
      out->node_pod_off[node] = nkept[node];
      int32_t* dst = out->node_pod_idx + nkept[node];
      if (hit[node]) {
        const auto& en = cache->entries[static_cast<size_t>(slot[node])];
        for (size_t k = 0; k < en.perm.size(); ++k) dst[k] = listed[s0 + en.perm[k]];
        out->requested_cpu[node] = en.requested;
        out->free_cpu[node] = N.alloc_milli_cpu[node] - en.requested;
        continue;
      }
      ++my_sorted;
      int64_t requested = 0;
      kv.clear();
      for (int32_t j = s0; j < start[node + 1]; ++j) {
        const int32_t pod = listed[j];
        if (P.priority[pod] < p->priority_threshold && spot) continue;
        kv.emplace_back(cpu[pod], j - s0);
        requested += cpu[pod];
      }
      out->requested_cpu[node] = requested;
      out->free_cpu[node] = N.alloc_milli_cpu[node] - requested;
      go_sort_slice(kv.data(), static_cast<int>(kv.size()), by_key_desc);
      for (size_t k = 0; k < kv.size(); ++k) dst[k] = listed[s0 + kv[k].second];
      if (!slot.empty() && slot[node] >= 0) {  // remember this sort
        auto& en = cache->entries[static_cast<size_t>(slot[node])];
        const int32_t n = start[node + 1] - s0;
        en.kind = kind[node];
        en.stamps.resize(static_cast<size_t>(n));
        for (int32_t k = 0; k < n; ++k) {
          en.stamps[static_cast<size_t>(k)] = stamps[listed[s0 + k]];
          if (!en.stamps[static_cast<size_t>(k)]) en.kind = -1;  // an unstamped pod: never a hit
        }
        en.perm.resize(kv.size());
        for (size_t k = 0; k < kv.size(); ++k) en.perm[k] = kv[k].second;
        en.requested = requested;
      }
    }
    sorted.fetch_add(my_sorted, std::memory_order_relaxed);
  });
  if (out_sorted) *out_sorted = sorted.load();
  NM_MARK(3);
  int32_t ns = 0, nod = 0;
  for (int32_t node = 0; node < nn; ++node) {
    if (kind[node] == 1)
      out->spot[ns++] = node;
    else if (kind[node] == 2)
      out->on_demand[nod++] = node;
  }
  out->node_pod_off[nn] = nkept[nn];
  const int64_t* req = out->requested_cpu;
  auto par = [](int n, const std::function<void(int)>& fn) {
    parallel_for(static_cast<size_t>(n), 1, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; ++i) fn(static_cast<int>(i));
    });
  };
  // The on-demand list sorts on ~RequestedCPU with the spot list's less
  // function (x < y exactly when ~x > ~y: every comparison, so every swap, is
  // by_key_asc's), so both split over the pool together.  A list whose input
  // pairs equal the cache's last ones takes its last output.
  (void)by_key_asc;
  std::vector<KV> in[2], sorted_v[2];
  const int32_t len[2] = {ns, nod};
  const int32_t* ids[2] = {out->spot, out->on_demand};
  std::vector<std::pair<KV*, int>> todo;
  bool reuse[2] = {false, false};
  for (int k = 0; k < 2; ++k) {
    in[k].resize(static_cast<size_t>(len[k]));
    for (int32_t i = 0; i < len[k]; ++i) {
      const int64_t r = req[ids[k][i]];
      in[k][static_cast<size_t>(i)] = KV(k == 0 ? r : ~r, ids[k][i]);
    }
    reuse[k] = cache && cache->list_in[k] == in[k];
    if (!reuse[k]) {
      sorted_v[k] = in[k];
      todo.emplace_back(sorted_v[k].data(), len[k]);
    }
  }
  if (!todo.empty()) go_sort_slices_parallel(todo, by_key_desc, par);
  int32_t* dst[2] = {out->spot, out->on_demand};
  for (int k = 0; k < 2; ++k) {
    const std::vector<KV>& res = reuse[k] ? cache->list_out[k] : sorted_v[k];
    for (int32_t i = 0; i < len[k]; ++i) dst[k][i] = res[static_cast<size_t>(i)].second;
    if (cache && !reuse[k]) {
      cache->list_in[k].swap(in[k]);
      cache->list_out[k].swap(sorted_v[k]);
    }
  }
  *out->n_spot = ns;
  *out->n_on_demand = nod;
  if (cache) cache->hit_valid = stamps != nullptr && W.hit.size() == static_cast<size_t>(nn);
  NM_MARK(4);
  return SR_OK;
}

static inline uint64_t pod_meta_mix(uint64_t h, uint64_t x) {
  h = (h ^ x) * 0xff51afd7ed558ccdull;
  return h ^ (h >> 32);
}

void snap_pod_from(const sr_cluster* c, int32_t pod, SnapPod* out, int32_t* k, int32_t* v, uint32_t lab,
                   std::vector<int32_t>* terms) {
  *out = SnapPod{};
  out->ns = -1;
  out->anti = has_anti_terms(c, pod) ? 1 : 0;
  out->opaque = anti_opaque(c, pod) ? 1 : 0;
  out->term = c->spread ? (c->spread->terminating[pod] ? 1 : 0) : 2;
  out->meta_fp = pod_meta_mix(0x5EEDull, out->term);
  const sr_pod_affinity* A = c->pod_affinity;
  if (!A) return;
  out->meta = 1;
  out->ns = A->ns[pod];
  out->lab = lab;
  out->nlab = pod_label_count(c, pod);
  std::copy(A->label_key + A->label_off[pod], A->label_key + A->label_off[pod + 1], k + lab);
  std::copy(A->label_val + A->label_off[pod], A->label_val + A->label_off[pod + 1], v + lab);
  uint64_t fp = pod_meta_mix(pod_meta_mix(0x3E7Aull, static_cast<uint32_t>(out->ns)), out->term);
  for (int32_t i = A->label_off[pod]; i < A->label_off[pod + 1]; ++i)  // labels: a map (order-independent)
    fp += pod_meta_mix(pod_meta_mix(0x1AB7ull, static_cast<uint32_t>(A->label_key[i])), static_cast<uint32_t>(A->label_val[i]));
  out->meta_fp = fp;
  if (out->opaque || !out->anti) return;  // opaque: never read, every candidate falls back while it is there
  std::vector<int32_t> words;
  out->terms = static_cast<uint32_t>(terms->size());
  for (int32_t t = A->anti_off[pod]; t < A->anti_off[pod + 1]; ++t) {
    anti_term_words(c, pod, t, words);
    terms->push_back(static_cast<int32_t>(words.size()));
    terms->insert(terms->end(), words.begin(), words.end());
  }
  out->nterms = static_cast<uint32_t>(terms->size()) - out->terms;
  for (uint32_t i = out->terms; i < out->terms + out->nterms; i += 1 + static_cast<uint32_t>((*terms)[i]))
    out->meta_fp += pod_meta_mix(0x7E4Dull, hash_words(terms->data() + i + 1, static_cast<size_t>((*terms)[i])));
}

// scheduler NodeInfo.AddPod [upstream k8s v1.19 framework/types.go]: Requested +=
// the pod's request, Pods += pod, UsedPorts += container host ports.  `sp` is
// the snapshot's copy of the pod (index `store` in sr_snapshot::pods).
static void state_add_pod(NodeState& st, const sr_cluster* c, int32_t pod, const SnapPod& sp, int32_t store) {
  const sr_pods& P = c->pods;
  // int64 addition wraps in Go; do the same without signed-overflow UB.
  auto wrap_add = [](int64_t a, int64_t b) {
    return static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(b));
  };
  for (int r = 0; r < 3; ++r) st.requested[r] = wrap_add(st.requested[r], pod_acc(c, pod, r));
  if (has_scalars(c, pod)) {  // Requested.ScalarResources[name] += value (kept sorted by name)
    for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; ++i) {
      const int32_t name = c->pod_scalar_name[i];
      auto it = std::lower_bound(st.scalar_req.begin(), st.scalar_req.end(), std::make_pair(name, INT64_MIN));
      if (it == st.scalar_req.end() || it->first != name) it = st.scalar_req.insert(it, {name, 0});
      it->second = wrap_add(it->second, c->pod_scalar_acc[i]);
    }
  } else if (!c->pod_scalar_off && (P.flags[pod] & SR_POD_FB_SCALAR_RESOURCES)) {
    st.scalar_unknown += 1;  // its scalar requests are not in the call: unknown to the planner
  }
  st.npods += 1;
  st.meta_sum += sp.meta_fp;
  st.anti += sp.anti;
  st.opaque += sp.opaque;
  st.unknown += sp.meta ? 0 : 1;
  st.term_unknown += sp.term == 2 ? 1 : 0;
  st.pods.push_back(store);
  // UsedPorts += container host ports; the inline disks VolumeRestrictions
  // compares as pseudo ports (host.hpp for_each_port)
  for_each_port(c, pod, [&](int32_t proto, int32_t port, int32_t ip) { st.ports.push_back(Port{ip, proto, port}); });
  if (const sr_volumes* V = c->volumes)  // the node's unique attachable volumes per limit key
    for (int32_t i = V->att_off[pod]; i < V->att_off[pod + 1]; ++i) {
      const std::pair<int32_t, int32_t> a(V->att_key[i], V->att_id[i]);
      auto it = std::lower_bound(st.att.begin(), st.att.end(), a);
      if (it == st.att.end() || *it != a) st.att.insert(it, a);
    }
}

// A term whose label selector metav1.LabelSelectorAsSelector rejects: a key
// that is not a qualified name (the empty key included), a value that is not
// a valid label value (labels.NewRequirement on every matchLabels pair and
// matchExpression), In / NotIn without values, Exists / DoesNotExist with
// values, any other operator [upstream apimachinery v0.19.2].  Without the
// shim's validity table (sr_cluster.str_label) any label requirement counts
// as rejected: the planner cannot tell.
static bool term_invalid(const sr_cluster* c, int32_t t) {
  const sr_pod_affinity* A = c->pod_affinity;
  const int32_t e_id = c->id_empty;
  if (A->selector_nil[t]) return false;
  for (int32_t i = A->ml_off[t]; i < A->ml_off[t + 1]; ++i) {
    if (A->ml_key[i] == e_id && e_id != -1) return true;
    if (!label_req_strings_ok(c, A->ml_key[i], A->ml_val, i, i + 1)) return true;
  }
  for (int32_t e = A->me_off[t]; e < A->me_off[t + 1]; ++e) {
    const int32_t nv = A->me_val_off[e + 1] - A->me_val_off[e], op = A->me_op[e];
    if (A->me_key[e] == e_id && e_id != -1) return true;
    if (!label_req_strings_ok(c, A->me_key[e], A->me_vals, A->me_val_off[e], A->me_val_off[e + 1])) return true;
    if (op == SR_OP_IN || op == SR_OP_NOT_IN) {
      if (nv == 0) return true;
    } else if (op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) {
      if (nv != 0) return true;
    } else {
      return true;
    }
  }
  return false;
}

bool anti_opaque(const sr_cluster* c, int32_t pod) {
  if (!has_anti_terms(c, pod)) return false;
  const sr_pod_affinity* A = c->pod_affinity;
  if (!A || A->anti_off[pod] == A->anti_off[pod + 1]) return true;
  for (int32_t t = A->anti_off[pod]; t < A->anti_off[pod + 1]; ++t)
    if (term_invalid(c, t)) return true;
  return false;
}

bool aff_opaque(const sr_cluster* c, int32_t pod) {
  const sr_pod_affinity* A = c->pod_affinity;
  if (!A || !A->aff_off) return false;
  for (int32_t t = A->aff_off[pod]; t < A->aff_off[pod + 1]; ++t)
    if (term_invalid(c, t)) return true;
  return false;
}

void snapshot_add_pod(sr_snapshot* s, const sr_cluster* c, int32_t pod, int32_t pos) {
  const int32_t store = static_cast<int32_t>(s->pods.size());
  s->pods.emplace_back();
  s->stamps.push_back(c->pod_stamp ? c->pod_stamp[pod] : 0);
  const uint32_t lab = static_cast<uint32_t>(s->lkey.size());
  s->lkey.resize(lab + pod_label_count(c, pod));
  s->lval.resize(s->lkey.size());
  snap_pod_from(c, pod, &s->pods.back(), s->lkey.data(), s->lval.data(), lab, &s->term_words);
  const SnapPod& sp = s->pods.back();
  state_add_pod(s->state[pos], c, pod, sp, store);
  s->node_dfp[pos] = node_state_fp(s->nodes[pos], s->state[pos]);
  s->anti_total += sp.anti;
  s->opaque_total += sp.opaque;
  s->unknown_total += sp.meta ? 0 : 1;
  s->scalar_unknown_total += !c->pod_scalar_off && (c->pods.flags[pod] & SR_POD_FB_SCALAR_RESOURCES) ? 1 : 0;
  s->term_unknown_total += sp.term == 2 ? 1 : 0;
  s->version++;
}

// The input of GetClusterSnapshot: spot node indices and each node's pod list
// in range (checked before anything is built, so a build cannot fail).
static bool snapshot_input_ok(const sr_cluster* c, const int32_t* spot, int32_t n_spot, const int32_t* off,
                              const int32_t* idx) {
  if (n_spot < 0 || (n_spot > 0 && (!spot || !off || !idx))) return false;
  std::atomic<bool> bad{false};
  parallel_for(static_cast<size_t>(n_spot), 512, [&](size_t lo, size_t hi) {
    const int32_t np = c->pods.n, nn = c->nodes.n;
    bool b = false;
    for (size_t i = lo; i < hi && !b; ++i) {
      const int32_t node = spot[i];
      if (node < 0 || node >= nn) {
        b = true;
        break;
      }
      for (int32_t j = off[node]; j < off[node + 1]; ++j) b |= static_cast<uint32_t>(idx[j]) >= static_cast<uint32_t>(np);
    }
    if (b) bad.store(true, std::memory_order_relaxed);
  });
  return !bad.load();
}

// The node AddNodeWithPods copies (nodes/nodes.go:229): allocatable,
// labels, taints, scalar and volume limits.
static inline uint64_t fp_mix(uint64_t h, uint64_t x) {
  h = (h ^ x) * 0xff51afd7ed558ccdull;
  return h ^ (h >> 32);
}

// Fingerprint of everything a snapshot's SpotNode copies from the cluster's
// node (0: a node with scalar resources or volume limits, copied anew).
static uint64_t cluster_node_fp(const sr_cluster* c, int32_t node) {
  const sr_nodes& N = c->nodes;
  if (c->node_scalar_off && c->node_scalar_off[node + 1] != c->node_scalar_off[node]) return 0;
  if (c->volumes && c->volumes->limit_off[node + 1] != c->volumes->limit_off[node]) return 0;
  uint64_t h = fp_mix(fp_mix(0xC0DEull, static_cast<uint32_t>(N.name[node])), N.unschedulable[node]);
  h = fp_mix(fp_mix(fp_mix(h, static_cast<uint64_t>(N.alloc_milli_cpu[node])), static_cast<uint64_t>(N.alloc_memory[node])),
             static_cast<uint64_t>(N.alloc_ephemeral[node]));
  h = fp_mix(h, static_cast<uint64_t>(N.alloc_pods[node]));
  h = fp_mix(h, static_cast<uint64_t>(N.label_off[node + 1] - N.label_off[node]));
  for (int32_t j = N.label_off[node]; j < N.label_off[node + 1]; ++j)  // in order, as the copy holds them
    h = fp_mix(h, static_cast<uint64_t>(static_cast<uint32_t>(N.label_key[j])) << 32 | static_cast<uint32_t>(N.label_val[j]));
  h = fp_mix(h, static_cast<uint64_t>(N.taint_off[node + 1] - N.taint_off[node]));
  for (int32_t j = N.taint_off[node]; j < N.taint_off[node + 1]; ++j)
    h = fp_mix(fp_mix(h, static_cast<uint64_t>(static_cast<uint32_t>(N.taint_key[j])) << 32 | static_cast<uint32_t>(N.taint_val[j])),
               static_cast<uint64_t>(N.taint_effect[j]));
  return h | 1;  // never 0
}

static void spot_node_from(const sr_cluster* c, int32_t node, SpotNode& sn) {
  const sr_nodes& N = c->nodes;
  sn = SpotNode{};
  sn.name = N.name[node];
  sn.alloc[0] = N.alloc_milli_cpu[node];
  sn.alloc[1] = N.alloc_memory[node];
  sn.alloc[2] = N.alloc_ephemeral[node];
  sn.alloc_pods = N.alloc_pods[node];
  sn.unschedulable = N.unschedulable[node];
  sn.labels.reserve(static_cast<size_t>(N.label_off[node + 1] - N.label_off[node]));
  for (int32_t j = N.label_off[node]; j < N.label_off[node + 1]; ++j) sn.labels.emplace_back(N.label_key[j], N.label_val[j]);
  for (int32_t j = N.taint_off[node]; j < N.taint_off[node + 1]; ++j)
    sn.taints.push_back(TaintRec{N.taint_key[j], N.taint_val[j], N.taint_effect[j]});
  if (c->node_scalar_off) {
    for (int32_t j = c->node_scalar_off[node]; j < c->node_scalar_off[node + 1]; ++j)
      sn.scalar_alloc.emplace_back(c->node_scalar_name[j], c->node_scalar_alloc[j]);
    std::sort(sn.scalar_alloc.begin(), sn.scalar_alloc.end());
  }
  if (const sr_volumes* V = c->volumes) {
    for (int32_t j = V->limit_off[node]; j < V->limit_off[node + 1]; ++j) sn.vol_limit.emplace_back(V->limit_key[j], V->limit[j]);
    std::sort(sn.vol_limit.begin(), sn.vol_limit.end());
  }
  sn.static_fp = node_static_fp(sn, c);
  sn.copy_fp = cluster_node_fp(c, node);
}

// AddNodeWithPods' pods for the spot positions `pos` (empty states): each
// position's pods are appended to the snapshot's store, their labels to the
// label arena, on the pool; the rare anti-affinity terms go to per-chunk
// arenas, concatenated afterwards.
static void build_states(sr_snapshot* s, const sr_cluster* c, const int32_t* spot, const int32_t* off,
                         const int32_t* idx, const std::vector<int32_t>& pos) {
  const size_t n = pos.size();
  if (n == 0) return;
  // position pos[q]'s pods at [base[q], base[q + 1]) of the store, labels at [lbase[q], lbase[q + 1])
  std::vector<int32_t> base(n + 1, static_cast<int32_t>(s->pods.size()));
  for (size_t q = 0; q < n; ++q) base[q + 1] = base[q] + (off[spot[pos[q]] + 1] - off[spot[pos[q]]]);
  std::vector<uint32_t> lbase(n + 1, static_cast<uint32_t>(s->lkey.size()));
  if (c->pod_affinity) {
    std::vector<uint32_t> cnt(n, 0);
    parallel_for(n, 256, [&](size_t lo, size_t hi) {
      for (size_t q = lo; q < hi; ++q) {
        const int32_t node = spot[pos[q]];
        uint32_t k = 0;
        for (int32_t j = off[node]; j < off[node + 1]; ++j) k += pod_label_count(c, idx[j]);
        cnt[q] = k;
      }
    });
    for (size_t q = 0; q < n; ++q) lbase[q + 1] = lbase[q] + cnt[q];
  }
  s->pods.resize(static_cast<size_t>(base[n]));
  s->stamps.resize(static_cast<size_t>(base[n]));
  s->lkey.resize(lbase[n]);
  s->lval.resize(lbase[n]);
  constexpr size_t kNodeChunk = 32;
  std::vector<std::vector<int32_t>> chunk_terms((n + kNodeChunk - 1) / kNodeChunk);
  parallel_for(n, kNodeChunk, [&](size_t lo, size_t hi) {
    for (size_t q = lo; q < hi; ++q) {
      std::vector<int32_t>* terms = &chunk_terms[q / kNodeChunk];
      const int32_t node = spot[pos[q]];
      NodeState& st = s->state[pos[q]];
      st.pods.reserve(static_cast<size_t>(off[node + 1] - off[node]));
      uint32_t lab = lbase[q];
      for (int32_t j = off[node]; j < off[node + 1]; ++j) {
        const int32_t store = base[q] + (j - off[node]);
        snap_pod_from(c, idx[j], &s->pods[store], s->lkey.data(), s->lval.data(), lab, terms);
        s->stamps[store] = c->pod_stamp ? c->pod_stamp[idx[j]] : 0;
        lab += s->pods[store].nlab;
        state_add_pod(st, c, idx[j], s->pods[store], store);
      }
    }
  });
  for (size_t ch = 0; ch < chunk_terms.size(); ++ch) {
    if (chunk_terms[ch].empty()) continue;
    const uint32_t shift = static_cast<uint32_t>(s->term_words.size());
    s->term_words.insert(s->term_words.end(), chunk_terms[ch].begin(), chunk_terms[ch].end());
    const size_t q1 = std::min(n, (ch + 1) * kNodeChunk);
    for (int32_t e = base[ch * kNodeChunk]; e < base[q1]; ++e)
      if (s->pods[e].nterms) s->pods[e].terms += shift;
  }
}

// Per-position views the encoder compares (names, fingerprints) and the totals.
static void finish_snapshot(sr_snapshot* s) {
  const size_t n = s->nodes.size();
  s->node_names.resize(n);
  s->node_sfp.resize(n);
  s->node_dfp.resize(n);
  parallel_for(n, 256, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      s->node_names[i] = s->nodes[i].name;
      s->node_sfp[i] = s->nodes[i].static_fp;
      s->node_dfp[i] = node_state_fp(s->nodes[i], s->state[i]);
    }
  });
  s->anti_total = s->opaque_total = s->unknown_total = s->scalar_unknown_total = s->term_unknown_total = 0;
  for (const NodeState& st : s->state) {
    s->anti_total += st.anti;
    s->opaque_total += st.opaque;
    s->unknown_total += st.unknown;
    s->scalar_unknown_total += st.scalar_unknown;
    s->term_unknown_total += st.term_unknown;
  }
}

static sr_status snapshot_create(const sr_cluster* c, const int32_t* spot, int32_t n_spot,
                                 const int32_t* off, const int32_t* idx, sr_snapshot** out) {
  if (!snapshot_input_ok(c, spot, n_spot, off, idx)) return SR_ERR_INVALID_ARG;
  auto* s = new sr_snapshot();
  s->id_empty = c->id_empty;
  s->id_metadata_name = c->id_metadata_name;
  s->id_unschedulable_key = c->id_unschedulable_key;
  s->shape = cluster_shape(c);
  s->nodes.resize(n_spot);
  s->state.resize(n_spot);
  parallel_for(static_cast<size_t>(n_spot), 64, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) spot_node_from(c, spot[i], s->nodes[i]);
  });
  std::vector<int32_t> pos(static_cast<size_t>(n_spot));
  for (int32_t i = 0; i < n_spot; ++i) pos[i] = i;
  build_states(s, c, spot, off, idx, pos);
  finish_snapshot(s);
  s->spot_prev.assign(spot, spot + n_spot);
  *out = s;
  return SR_OK;
}

// The snapshot's copy of `node` still equals the cluster's (nodes with scalar
// resources or volume limits are copied anew): the fingerprint rejects most
// changed nodes, and a match is confirmed field by field, so a fingerprint
// collision can never keep a stale copy.
static inline bool spot_node_same(const sr_cluster* c, int32_t node, const SpotNode& sn) {
  if (sn.copy_fp == 0 || sn.copy_fp != cluster_node_fp(c, node)) return false;
  const sr_nodes& N = c->nodes;
  if (sn.name != N.name[node] || sn.unschedulable != N.unschedulable[node] || sn.alloc[0] != N.alloc_milli_cpu[node] ||
      sn.alloc[1] != N.alloc_memory[node] || sn.alloc[2] != N.alloc_ephemeral[node] || sn.alloc_pods != N.alloc_pods[node])
    return false;
  const int32_t l0 = N.label_off[node], nl = N.label_off[node + 1] - l0;
  if (static_cast<size_t>(nl) != sn.labels.size()) return false;
  for (int32_t j = 0; j < nl; ++j)
    if (sn.labels[j].first != N.label_key[l0 + j] || sn.labels[j].second != N.label_val[l0 + j]) return false;
  const int32_t t0 = N.taint_off[node], nt = N.taint_off[node + 1] - t0;
  if (static_cast<size_t>(nt) != sn.taints.size()) return false;
  for (int32_t j = 0; j < nt; ++j) {
    const TaintRec& t = sn.taints[j];
    if (t.key != N.taint_key[t0 + j] || t.val != N.taint_val[t0 + j] || t.effect != N.taint_effect[t0 + j]) return false;
  }
  return true;
}

// GetClusterSnapshot again on a snapshot built from an earlier call's cluster:
// afterwards it holds what snapshot_create on these arguments would build.
// A spot node (by name) whose pod list carries the same non-zero stamps in the
// same order as its state in the snapshot keeps that state and its pods in the
// store (a stamp covers everything a pod contributes, sr_cluster.pod_stamp);
// the others are rebuilt, their pods appended to the store.  A node whose
// static part equals the cluster's keeps its copy too.  The store is rebuilt
// whole once dead entries outnumber live ones, or when the cluster's shape
// changed.
static sr_status snapshot_refresh(sr_snapshot* s, const sr_cluster* c, const int32_t* spot, int32_t n_spot,
                                  const int32_t* off, const int32_t* idx, int32_t* out_rebuilt,
                                  const sr_node_map_cache* cache = nullptr) {
  if (s->forked) return SR_ERR_STATE;  // a forked snapshot is mid-simulation
  // Linked to the node map cache (sr_snapshot_refresh_cached): the snapshot
  // was last refreshed from the output of the cache's previous call and not
  // changed since, so a node whose LISTed pods that call found unchanged
  // (same non-zero stamps, same order: the same kept pods in the same sort)
  // holds exactly those pods -- their stamps are not gathered again.
  const bool linked = cache && cache->hit_valid && s->map_cache == cache && s->map_calls + 1 == cache->calls &&
                      s->map_version == s->version && cache->scratch.hit.size() == static_cast<size_t>(c->nodes.n);
  const uint8_t* hit = linked ? cache->scratch.hit.data() : nullptr;
  s->map_cache = nullptr;
  if (n_spot < 0 || (n_spot > 0 && (!spot || !off || !idx))) return SR_ERR_INVALID_ARG;
  const uint64_t* stamps = c->pod_stamp;
  auto rebuild = [&]() {
    sr_snapshot* t = nullptr;
    const sr_status st = snapshot_create(c, spot, n_spot, off, idx, &t);
    if (st != SR_OK) return st;
    const uint64_t v = s->version;
    std::vector<int32_t> scratch, scratch2;
    scratch.swap(s->pos_of_name);
    scratch2.swap(s->pos_of_node);
    *s = std::move(*t);
    delete t;
    s->pos_of_name.swap(scratch);
    s->pos_of_node.swap(scratch2);
    s->version = v + 1;
    if (cache && cache->hit_valid) {
      s->map_cache = cache;
      s->map_calls = cache->calls;
      s->map_version = s->version;
    }
    if (out_rebuilt) *out_rebuilt = n_spot;
    return SR_OK;
  };
  if (!stamps || s->shape != cluster_shape(c) || s->id_empty != c->id_empty ||
      s->id_metadata_name != c->id_metadata_name || s->id_unschedulable_key != c->id_unschedulable_key)
    return rebuild();
  // previous position of each node, by name (unique per cluster; a repeated
  // name claims the previous state once)
  const int32_t ns_str = c->n_strings, nn = c->nodes.n, np = c->pods.n;
  NM_START();
  const int32_t n_old = static_cast<int32_t>(s->nodes.size());
  std::vector<int32_t> from(static_cast<size_t>(n_spot), -1);
  std::vector<uint8_t> claimed(static_cast<size_t>(n_old), 0);
  bool bad = false, missed = false;
  for (int32_t i = 0; i < n_spot && !bad; ++i) bad = spot[i] < 0 || spot[i] >= nn;
  if (bad) return SR_ERR_INVALID_ARG;
  // by cluster node index first (a node keeps its index from tick to tick;
  // an [nn] map instead of one over every string), the name checked
  if (s->spot_prev.size() == static_cast<size_t>(n_old)) {
    std::vector<int32_t>& pon = s->pos_of_node;
    if (pon.size() < static_cast<size_t>(nn)) pon.resize(static_cast<size_t>(nn), -1);
    for (int32_t o = 0; o < n_old; ++o)
      if (s->spot_prev[o] >= 0 && s->spot_prev[o] < nn) pon[s->spot_prev[o]] = o;
    for (int32_t i = 0; i < n_spot; ++i) {
      const int32_t o = pon[spot[i]];
      if (o >= 0 && s->node_names[o] == c->nodes.name[spot[i]] && c->nodes.name[spot[i]] >= 0) {
        from[i] = o;
        claimed[o] = 1;
        pon[spot[i]] = -1;
      } else {
        missed = true;
      }
    }
    for (int32_t o = 0; o < n_old; ++o)
      if (s->spot_prev[o] >= 0 && s->spot_prev[o] < nn) pon[s->spot_prev[o]] = -1;
  } else {
    missed = n_spot > 0;
  }
  if (missed) {  // the rest by name (unique per cluster; a repeated name claims a previous state once)
    if (s->pos_of_name.size() < static_cast<size_t>(ns_str)) s->pos_of_name.resize(static_cast<size_t>(ns_str), -1);
    for (int32_t o = 0; o < n_old; ++o) {
      const int32_t nm = s->node_names[o];
      if (!claimed[o] && nm >= 0 && nm < ns_str) s->pos_of_name[nm] = o;
    }
    for (int32_t i = 0; i < n_spot; ++i) {
      if (from[i] >= 0) continue;
      const int32_t nm = c->nodes.name[spot[i]];
      if (nm < 0 || nm >= ns_str) continue;
      const int32_t o = s->pos_of_name[nm];
      if (o >= 0) {
        from[i] = o;
        claimed[o] = 1;
        s->pos_of_name[nm] = -1;  // claimed
      }
    }
    for (int32_t o = 0; o < n_old; ++o) {
      const int32_t nm = s->node_names[o];
      if (nm >= 0 && nm < ns_str) s->pos_of_name[nm] = -1;
    }
  }
  NM_MARK(5);
  // Pass 1 (reads only): the input validated, per position whether the pods
  // and the static part stand
  std::vector<uint8_t> keep(static_cast<size_t>(n_spot), 0);  // bit 0: state, bit 1: static part
  std::atomic<bool> bad_pod{false};
  std::atomic<size_t> live{0};
  parallel_for(static_cast<size_t>(n_spot), 64, [&](size_t lo, size_t hi) {
    bool b = false;
    size_t my_live = 0;
    // the stamps are a gather (a node's pods lie anywhere in the cluster's
    // arrays): the next node's are requested while this one is compared
    auto prefetch_node = [&](size_t i) {
      const int32_t nd = spot[i];
      for (int32_t j = off[nd]; j < off[nd + 1]; ++j)
        if (static_cast<uint32_t>(idx[j]) < static_cast<uint32_t>(np)) __builtin_prefetch(&stamps[idx[j]]);
    };
    if (lo < hi) prefetch_node(lo);
    for (size_t i = lo; i < hi && !b; ++i) {
      if (i + 1 < hi && !(hit && hit[spot[i + 1]])) prefetch_node(i + 1);
      const int32_t node = spot[i], j0 = off[node], n = off[node + 1] - j0;
      my_live += static_cast<size_t>(n);
      const int32_t o = from[i];
      const NodeState* prev = o >= 0 ? &s->state[static_cast<size_t>(o)] : nullptr;
      bool same = prev && static_cast<int64_t>(prev->pods.size()) == n && prev->npods == n;
      if (same && hit && hit[node]) {  // unchanged since the previous node map (linked): kept as it is
        keep[i] = static_cast<uint8_t>(1 | (spot_node_same(c, node, s->nodes[static_cast<size_t>(o)]) ? 2 : 0));
        continue;
      }
      for (int32_t k = 0; k < n; ++k) {  // the pods validated and, while equal, their stamps compared
        const int32_t pod = idx[j0 + k];
        if (static_cast<uint32_t>(pod) >= static_cast<uint32_t>(np)) {
          b = true;
          break;
        }
        if (same) {
          const uint64_t st = stamps[pod];
          same = st != 0 && s->stamps[static_cast<size_t>(prev->pods[k])] == st;
        }
      }
      if (b || !prev) continue;
      keep[i] = static_cast<uint8_t>((same ? 1 : 0) | (spot_node_same(c, node, s->nodes[static_cast<size_t>(o)]) ? 2 : 0));
    }
    if (b) bad_pod.store(true, std::memory_order_relaxed);
    live.fetch_add(my_live, std::memory_order_relaxed);
  });
  if (bad_pod.load()) return SR_ERR_INVALID_ARG;
  if (s->pods.size() > 2 * live.load() + 4096) return rebuild();  // mostly dead entries: compact
  NM_MARK(6);
  // the totals follow the states: those not kept leave them (the rebuilt
  // ones join below)
  {
    std::vector<uint8_t> state_kept(static_cast<size_t>(n_old), 0);
    for (int32_t i = 0; i < n_spot; ++i)
      if (keep[i] & 1) state_kept[from[i]] = 1;
    for (int32_t o = 0; o < n_old; ++o) {
      if (state_kept[o]) continue;
      const NodeState& st = s->state[o];
      s->anti_total -= st.anti;
      s->opaque_total -= st.opaque;
      s->unknown_total -= st.unknown;
      s->scalar_unknown_total -= st.scalar_unknown;
      s->term_unknown_total -= st.term_unknown;
    }
  }
  // Pass 2: kept states and copies move to their new positions (most stay
  // where they are: only the moved ones go through a side buffer), the rest
  // is built
  std::vector<int32_t> moved;
  for (int32_t i = 0; i < n_spot; ++i)
    if (keep[i] && from[i] != i) moved.push_back(i);
  std::vector<NodeState> side_state(moved.size());
  std::vector<SpotNode> side_node(moved.size());
  std::vector<uint64_t> side_dfp(moved.size());
  for (size_t q = 0; q < moved.size(); ++q) {
    const int32_t i = moved[q], o = from[i];
    if (keep[i] & 1) side_state[q] = std::move(s->state[o]);
    if (keep[i] & 2) side_node[q] = std::move(s->nodes[o]);
    side_dfp[q] = s->node_dfp[o];
  }
  s->state.resize(static_cast<size_t>(n_spot));
  s->nodes.resize(static_cast<size_t>(n_spot));
  s->node_names.resize(static_cast<size_t>(n_spot));
  s->node_sfp.resize(static_cast<size_t>(n_spot));
  s->node_dfp.resize(static_cast<size_t>(n_spot));
  for (size_t q = 0; q < moved.size(); ++q) {
    const int32_t i = moved[q];
    if (keep[i] & 1) s->state[i] = std::move(side_state[q]);
    if (keep[i] & 2) s->nodes[i] = std::move(side_node[q]);
    s->node_dfp[i] = side_dfp[q];
  }
  parallel_for(static_cast<size_t>(n_spot), 256, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      if (!(keep[i] & 1)) {  // rebuilt below: empty, its vectors' storage kept
        NodeState& st = s->state[i];
        std::vector<Port> ports(std::move(st.ports));
        std::vector<int32_t> pods(std::move(st.pods));
        ports.clear();
        pods.clear();
        st = NodeState{};
        st.ports = std::move(ports);
        st.pods = std::move(pods);
      }
      if (!(keep[i] & 2)) spot_node_from(c, spot[i], s->nodes[i]);
      s->node_names[i] = s->nodes[i].name;
      s->node_sfp[i] = s->nodes[i].static_fp;
    }
  });
  NM_MARK(7);
  std::vector<int32_t> pos;
  for (int32_t i = 0; i < n_spot; ++i)
    if (!(keep[i] & 1)) pos.push_back(i);
  build_states(s, c, spot, off, idx, pos);
  for (int32_t i = 0; i < n_spot; ++i)  // the state fingerprint of every node not kept whole
    if (keep[i] != 3) s->node_dfp[i] = node_state_fp(s->nodes[i], s->state[i]);
  s->saved.clear();
  s->saved_dfp.clear();
  for (int32_t i : pos) {
    const NodeState& st = s->state[i];
    s->anti_total += st.anti;
    s->opaque_total += st.opaque;
    s->unknown_total += st.unknown;
    s->scalar_unknown_total += st.scalar_unknown;
    s->term_unknown_total += st.term_unknown;
  }
  s->spot_prev.assign(spot, spot + n_spot);
  s->version++;
  if (cache && cache->hit_valid) {  // the next cached refresh may skip this call's unchanged nodes
    s->map_cache = cache;
    s->map_calls = cache->calls;
    s->map_version = s->version;
  }
  NM_MARK(8);
  if (out_rebuilt) *out_rebuilt = static_cast<int32_t>(pos.size());
  return SR_OK;
}

}  // namespace sr

extern "C" {

sr_status sr_new_node_map(const sr_cluster* cluster, const sr_node_map_params* params, sr_node_map* out) {
  if (!cluster || !params || !out) return SR_ERR_INVALID_ARG;
  return sr::new_node_map(cluster, params, out, nullptr, nullptr);
}

sr_status sr_node_map_cache_create(sr_node_map_cache** out) {
  if (!out) return SR_ERR_INVALID_ARG;
  *out = new sr_node_map_cache();
  return SR_OK;
}

void sr_node_map_cache_destroy(sr_node_map_cache* cache) { delete cache; }

sr_status sr_new_node_map_cached(sr_node_map_cache* cache, const sr_cluster* cluster, const sr_node_map_params* params,
                                 sr_node_map* out, int32_t* out_sorted) {
  if (!cluster || !params || !out) return SR_ERR_INVALID_ARG;
  return sr::new_node_map(cluster, params, out, cache, out_sorted);
}

int32_t sr_node_has_label(const sr_cluster* cluster, int32_t node, const sr_node_label* label) {
  if (!cluster || !label || node < 0 || node >= cluster->nodes.n) return 0;
  return sr::node_has_label(cluster, node, label) ? 1 : 0;
}

sr_status sr_snapshot_create(const sr_cluster* cluster, const int32_t* spot_nodes, int32_t n_spot,
                             const int32_t* node_pod_off, const int32_t* node_pod_idx, sr_snapshot** out) {
  if (!cluster || !out) return SR_ERR_INVALID_ARG;
  return sr::snapshot_create(cluster, spot_nodes, n_spot, node_pod_off, node_pod_idx, out);
}

sr_status sr_snapshot_refresh_cached(sr_snapshot* snap, const sr_node_map_cache* cache, const sr_cluster* cluster,
                                     const int32_t* spot_nodes, int32_t n_spot, const int32_t* node_pod_off,
                                     const int32_t* node_pod_idx, int32_t* out_rebuilt) {
  if (!snap || !cluster) return SR_ERR_INVALID_ARG;
  return sr::snapshot_refresh(snap, cluster, spot_nodes, n_spot, node_pod_off, node_pod_idx, out_rebuilt, cache);
}

sr_status sr_snapshot_refresh(sr_snapshot* snap, const sr_cluster* cluster, const int32_t* spot_nodes,
                              int32_t n_spot, const int32_t* node_pod_off, const int32_t* node_pod_idx,
                              int32_t* out_rebuilt) {
  if (!snap || !cluster) return SR_ERR_INVALID_ARG;
  return sr::snapshot_refresh(snap, cluster, spot_nodes, n_spot, node_pod_off, node_pod_idx, out_rebuilt);
}

void sr_snapshot_destroy(sr_snapshot* snap) { delete snap; }

sr_status sr_snapshot_add_pod(sr_snapshot* snap, const sr_cluster* cluster, int32_t pod, int32_t spot_pos) {
  if (!snap || !cluster || pod < 0 || pod >= cluster->pods.n || spot_pos < 0 ||
      spot_pos >= static_cast<int32_t>(snap->nodes.size()))
    return SR_ERR_INVALID_ARG;
  sr::snapshot_add_pod(snap, cluster, pod, spot_pos);
  return SR_OK;
}

sr_status sr_snapshot_fork(sr_snapshot* snap) {
  if (!snap) return SR_ERR_INVALID_ARG;
  if (snap->forked) return SR_ERR_STATE;  // DeltaClusterSnapshot forks one level deep
  snap->saved = snap->state;
  snap->saved_dfp = snap->node_dfp;
  snap->fork_pods = snap->pods.size();
  snap->fork_labels = snap->lkey.size();
  snap->fork_terms = snap->term_words.size();
  snap->forked = true;
  return SR_OK;
}

sr_status sr_snapshot_revert(sr_snapshot* snap) {
  if (!snap) return SR_ERR_INVALID_ARG;
  if (!snap->forked) return SR_OK;  // Revert with nothing forked leaves the snapshot as is
  snap->state.swap(snap->saved);
  snap->saved.clear();
  snap->node_dfp.swap(snap->saved_dfp);
  snap->pods.resize(snap->fork_pods);  // pods added since Fork are referenced by no state any more
  snap->stamps.resize(snap->fork_pods);
  snap->lkey.resize(snap->fork_labels);
  snap->lval.resize(snap->fork_labels);
  snap->term_words.resize(snap->fork_terms);
  snap->forked = false;
  snap->anti_total = snap->opaque_total = snap->unknown_total = snap->scalar_unknown_total = 0;
  snap->term_unknown_total = 0;
  for (const auto& st : snap->state) {
    snap->anti_total += st.anti;
    snap->opaque_total += st.opaque;
    snap->unknown_total += st.unknown;
    snap->scalar_unknown_total += st.scalar_unknown;
    snap->term_unknown_total += st.term_unknown;
  }
  snap->version++;
  return SR_OK;
}

sr_status sr_snapshot_node_state(const sr_snapshot* snap, int32_t spot_pos, int64_t out_requested[3],
                                 int32_t* out_num_pods) {
  if (!snap || spot_pos < 0 || spot_pos >= static_cast<int32_t>(snap->nodes.size())) return SR_ERR_INVALID_ARG;
  const auto& st = snap->state[spot_pos];
  if (out_requested) std::memcpy(out_requested, st.requested, sizeof(st.requested));
  if (out_num_pods) *out_num_pods = static_cast<int32_t>(st.npods);
  return SR_OK;
}

int32_t sr_snapshot_num_nodes(const sr_snapshot* snap) {
  return snap ? static_cast<int32_t>(snap->nodes.size()) : 0;
}

}  // extern "C"
