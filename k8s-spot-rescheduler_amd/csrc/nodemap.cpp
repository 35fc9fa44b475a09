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
#include <cstring>
#include <functional>
#include <vector>

#include "gosort.hpp"
#include "host.hpp"
#include "pool.hpp"

namespace sr {

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

static sr_status new_node_map(const sr_cluster* c, const sr_node_map_params* p, sr_node_map* out) {
  const sr_nodes& N = c->nodes;
  const sr_pods& P = c->pods;
  const int32_t nn = N.n, np = P.n;
  // Per-node LIST results: counting sort by node index keeps list order.
  // Large clusters: K pod ranges counted and scattered in parallel, range k's
  // pods of a node placed after those of ranges < k (still list order).
  std::vector<int32_t> start(static_cast<size_t>(nn) + 1, 0);
  std::vector<int32_t> listed(np > 0 ? np : 1);
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
    std::vector<int32_t> cnt(K * static_cast<size_t>(nn), 0);  // [range][node], then the range's cursor
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
        for (int32_t i = lo; i < hi; ++i) {
          const int32_t nd = P.node[i];
          if (nd < -1 || nd >= nn) bad.store(true, std::memory_order_relaxed);
          else if (nd >= 0) ++c[nd];
        }
      }
    });
    if (bad.load()) return SR_ERR_INVALID_ARG;
    parallel_for(static_cast<size_t>(nn), 4096, [&](size_t a, size_t b) {  // per node: total, then per-range offsets
      for (size_t nd = a; nd < b; ++nd) {
        int32_t acc = 0;
        for (size_t k = 0; k < K; ++k) {
          const int32_t x = cnt[k * static_cast<size_t>(nn) + nd];
          cnt[k * static_cast<size_t>(nn) + nd] = acc;
          acc += x;
        }
        start[nd + 1] = acc;
      }
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
  // the reference's less functions (nodes/nodes.go:76-80, 95-101) on (key, id) pairs: the same
  // comparisons, so Go's sort makes the same swaps
  using KV = std::pair<int64_t, int32_t>;
  auto by_key_desc = [](const KV& x, const KV& y) { return x.first > y.first; };
  auto by_key_asc = [](const KV& x, const KV& y) { return x.first < y.first; };
  // Per node (independent, on the pool): the spot / on-demand test, the
  // priority filter of getPodsOnNode, RequestedCPU and the pod sort.  Pass 1
  // counts the kept pods, pass 2 writes them at their prefix offsets.
  std::vector<int8_t> kind(static_cast<size_t>(nn), 0);  // 1 spot, 2 on-demand
  std::vector<int32_t> nkept(static_cast<size_t>(nn) + 1, 0);
  std::atomic<bool> nil_priority{false};
  parallel_for(static_cast<size_t>(nn), 64, [&](size_t lo, size_t hi) {
    for (size_t node = lo; node < hi; ++node) {
      const bool spot = node_has_label(c, static_cast<int32_t>(node), &p->spot);
      kind[node] = spot ? 1 : node_has_label(c, static_cast<int32_t>(node), &p->on_demand) ? 2 : 0;
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
  parallel_for(static_cast<size_t>(nn), 64, [&](size_t lo, size_t hi) {
    std::vector<std::pair<int64_t, int32_t>> kv;  // (cpu, pod): the sort compares keys held in place
    for (size_t node = lo; node < hi; ++node) {
      const bool spot = kind[node] == 1;
      out->node_pod_off[node] = nkept[node];
      int64_t requested = 0;
      kv.clear();
      for (int32_t j = start[node]; j < start[node + 1]; ++j) {
        const int32_t pod = listed[j];
        if (P.priority[pod] < p->priority_threshold && spot) continue;
        kv.emplace_back(cpu[pod], pod);
        requested += cpu[pod];
      }
      out->requested_cpu[node] = requested;
      out->free_cpu[node] = N.alloc_milli_cpu[node] - requested;
      go_sort_slice(kv.data(), static_cast<int>(kv.size()), by_key_desc);
      for (size_t k = 0; k < kv.size(); ++k) out->node_pod_idx[nkept[node] + static_cast<int32_t>(k)] = kv[k].second;
    }
  });
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
  std::vector<KV> kv_spot(static_cast<size_t>(ns)), kv_od(static_cast<size_t>(nod));
  for (int32_t i = 0; i < ns; ++i) kv_spot[i] = KV(req[out->spot[i]], out->spot[i]);
  for (int32_t i = 0; i < nod; ++i) kv_od[i] = KV(req[out->on_demand[i]], out->on_demand[i]);
  go_sort_slice_parallel(kv_spot.data(), ns, by_key_desc, par);
  go_sort_slice_parallel(kv_od.data(), nod, by_key_asc, par);
  for (int32_t i = 0; i < ns; ++i) out->spot[i] = kv_spot[i].second;
  for (int32_t i = 0; i < nod; ++i) out->on_demand[i] = kv_od[i].second;
  *out->n_spot = ns;
  *out->n_on_demand = nod;
  return SR_OK;
}

void snap_pod_from(const sr_cluster* c, int32_t pod, SnapPod* out, int32_t* k, int32_t* v, uint32_t lab,
                   std::vector<int32_t>* terms) {
  *out = SnapPod{};
  out->ns = -1;
  out->anti = has_anti_terms(c, pod) ? 1 : 0;
  out->opaque = anti_opaque(c, pod) ? 1 : 0;
  out->term = c->spread ? (c->spread->terminating[pod] ? 1 : 0) : 2;
  const sr_pod_affinity* A = c->pod_affinity;
  if (!A) return;
  out->meta = 1;
  out->ns = A->ns[pod];
  out->lab = lab;
  out->nlab = pod_label_count(c, pod);
  std::copy(A->label_key + A->label_off[pod], A->label_key + A->label_off[pod + 1], k + lab);
  std::copy(A->label_val + A->label_off[pod], A->label_val + A->label_off[pod + 1], v + lab);
  if (out->opaque || !out->anti) return;  // opaque: never read, every candidate falls back while it is there
  std::vector<int32_t> words;
  out->terms = static_cast<uint32_t>(terms->size());
  for (int32_t t = A->anti_off[pod]; t < A->anti_off[pod + 1]; ++t) {
    anti_term_words(c, pod, t, words);
    terms->push_back(static_cast<int32_t>(words.size()));
    terms->insert(terms->end(), words.begin(), words.end());
  }
  out->nterms = static_cast<uint32_t>(terms->size()) - out->terms;
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

static sr_status snapshot_create(const sr_cluster* c, const int32_t* spot, int32_t n_spot,
                                 const int32_t* off, const int32_t* idx, sr_snapshot** out) {
  if (n_spot < 0 || (n_spot > 0 && (!spot || !off || !idx))) return SR_ERR_INVALID_ARG;
  auto* s = new sr_snapshot();
  s->id_empty = c->id_empty;
  s->id_metadata_name = c->id_metadata_name;
  s->id_unschedulable_key = c->id_unschedulable_key;
  s->nodes.resize(n_spot);
  s->state.resize(n_spot);
  s->node_names.resize(n_spot);
  s->node_sfp.resize(n_spot);
  s->node_dfp.resize(n_spot);
  const sr_nodes& N = c->nodes;
  std::atomic<bool> bad{false};  // validate first: the build below cannot fail
  parallel_for(static_cast<size_t>(n_spot), 512, [&](size_t lo, size_t hi) {
    const int32_t np = c->pods.n, nn = N.n;
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
  if (bad.load()) {
    delete s;
    return SR_ERR_INVALID_ARG;
  }
  // the snapshot's pod store: the pods of spot node i at [base[i], base[i + 1])
  std::vector<int32_t> base(static_cast<size_t>(n_spot) + 1, 0);
  for (int32_t i = 0; i < n_spot; ++i) base[i + 1] = base[i] + (off[spot[i] + 1] - off[spot[i]]);
  s->pods.resize(static_cast<size_t>(base[n_spot]));
  // their labels: node i's at [lbase[i], lbase[i + 1])
  std::vector<uint32_t> lbase(static_cast<size_t>(n_spot) + 1, 0);
  if (c->pod_affinity) {
    parallel_for(static_cast<size_t>(n_spot), 256, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        uint32_t n = 0;
        for (int32_t j = off[spot[i]]; j < off[spot[i] + 1]; ++j) n += pod_label_count(c, idx[j]);
        lbase[i + 1] = n;
      }
    });
    for (int32_t i = 0; i < n_spot; ++i) lbase[i + 1] += lbase[i];
  }
  s->lkey.resize(lbase[n_spot]);
  s->lval.resize(lbase[n_spot]);
  // AddNodeWithPods per spot node: independent nodes, on the pool; the rare
  // anti-affinity terms go to per-chunk arenas, concatenated afterwards
  constexpr size_t kNodeChunk = 32;
  std::vector<std::vector<int32_t>> chunk_terms((static_cast<size_t>(n_spot) + kNodeChunk - 1) / kNodeChunk);
  parallel_for(static_cast<size_t>(n_spot), kNodeChunk, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      std::vector<int32_t>* terms = &chunk_terms[i / kNodeChunk];
      const int32_t node = spot[i];
      SpotNode& sn = s->nodes[i];
      sn.name = N.name[node];
      sn.alloc[0] = N.alloc_milli_cpu[node];
      sn.alloc[1] = N.alloc_memory[node];
      sn.alloc[2] = N.alloc_ephemeral[node];
      sn.alloc_pods = N.alloc_pods[node];
      sn.unschedulable = N.unschedulable[node];
      sn.labels.reserve(static_cast<size_t>(N.label_off[node + 1] - N.label_off[node]));
      for (int32_t j = N.label_off[node]; j < N.label_off[node + 1]; ++j)
        sn.labels.emplace_back(N.label_key[j], N.label_val[j]);
      for (int32_t j = N.taint_off[node]; j < N.taint_off[node + 1]; ++j)
        sn.taints.push_back(TaintRec{N.taint_key[j], N.taint_val[j], N.taint_effect[j]});
      if (c->node_scalar_off) {
        for (int32_t j = c->node_scalar_off[node]; j < c->node_scalar_off[node + 1]; ++j)
          sn.scalar_alloc.emplace_back(c->node_scalar_name[j], c->node_scalar_alloc[j]);
        std::sort(sn.scalar_alloc.begin(), sn.scalar_alloc.end());
      }
      if (const sr_volumes* V = c->volumes) {
        for (int32_t j = V->limit_off[node]; j < V->limit_off[node + 1]; ++j)
          sn.vol_limit.emplace_back(V->limit_key[j], V->limit[j]);
        std::sort(sn.vol_limit.begin(), sn.vol_limit.end());
      }
      sn.static_fp = node_static_fp(sn, c);
      s->state[i].pods.reserve(static_cast<size_t>(off[node + 1] - off[node]));
      uint32_t lab = lbase[i];
      for (int32_t j = off[node]; j < off[node + 1]; ++j) {
        const int32_t store = base[i] + (j - off[node]);
        snap_pod_from(c, idx[j], &s->pods[store], s->lkey.data(), s->lval.data(), lab, terms);
        lab += s->pods[store].nlab;
        state_add_pod(s->state[i], c, idx[j], s->pods[store], store);
      }
      s->node_names[i] = sn.name;
      s->node_sfp[i] = sn.static_fp;
      s->node_dfp[i] = node_state_fp(sn, s->state[i]);
    }
  });
  for (size_t ch = 0; ch < chunk_terms.size(); ++ch) {
    if (chunk_terms[ch].empty()) continue;
    const uint32_t shift = static_cast<uint32_t>(s->term_words.size());
    s->term_words.insert(s->term_words.end(), chunk_terms[ch].begin(), chunk_terms[ch].end());
    const size_t i1 = std::min(static_cast<size_t>(n_spot), (ch + 1) * kNodeChunk);
    for (int32_t q = base[ch * kNodeChunk]; q < base[i1]; ++q)
      if (s->pods[q].nterms) s->pods[q].terms += shift;
  }
  for (int32_t i = 0; i < n_spot; ++i) {
    s->anti_total += s->state[i].anti;
    s->opaque_total += s->state[i].opaque;
    s->unknown_total += s->state[i].unknown;
    s->scalar_unknown_total += s->state[i].scalar_unknown;
    s->term_unknown_total += s->state[i].term_unknown;
  }
  *out = s;
  return SR_OK;
}

}  // namespace sr

extern "C" {

sr_status sr_new_node_map(const sr_cluster* cluster, const sr_node_map_params* params, sr_node_map* out) {
  if (!cluster || !params || !out) return SR_ERR_INVALID_ARG;
  return sr::new_node_map(cluster, params, out);
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
