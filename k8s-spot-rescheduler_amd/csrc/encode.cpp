// encode.cpp — snapshot + candidate pod lists -> SoA workload for gfx950.
//
// The predicate of one (pod, spot node) pair against the *base* snapshot
// (k8s v1.19.2 NodeUnschedulable, NodeResourcesFit, NodeName, NodePorts,
// NodeAffinity, TaintToleration [upstream]; call site rescheduler.go:344)
// factors into a conjunction of terms that each depend on a low-cardinality
// projection of the pod:
//
//   fits(p, n) = S[class(p)](n) & T[cpu(p)](n) & T[mem(p)](n) & T[eph(p)](n)
//
//   S = static(class, n)            selector / affinity / taints / base ports
//       AND len(pods)+1 <= allowed  (pod-count part of NodeResourcesFit)
//   T = free_dim(n) >= threshold    (zero-request pods use row 0 = all nodes:
//                                    fitsRequest skips the resource checks)
//
// where "class" interns everything static about a pod.  S and T are bitmask
// rows over spot nodes in NodeInfoArray order, built on the GPU (K0); the dense
// pod's feasibility row is their AND, formed inside K2.  Everything that changes while a
// candidate's pods are placed (capacity, pod count, host ports) is rechecked
// exactly on the nodes the candidate touched (K2).  Features outside this set
// route the whole candidate to the reference path (SR_CAND_FALLBACK).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "host.hpp"
#include "pool.hpp"
#include "worddict.hpp"

namespace sr {

double encode_phase_ms[16];  // host-side profile of the last encode (tools/encode_stats)

namespace {

constexpr int64_t kQuantityLimit = int64_t(1) << 62;

bool in_range(int64_t v) { return v >= 0 && v < kQuantityLimit; }

enum : int32_t { REQ_LABEL_EQ = 0, REQ_LABEL_EXPR = 1, REQ_FIELD = 2 };

// A node-side requirement: nodeSelector pair, matchExpression or matchField.
struct Requirement {
  int32_t type, key, op;
  std::vector<int32_t> vals;  // sorted, unique
};

// v1.Toleration.ToleratesTaint [upstream k8s.io/api/core/v1/toleration.go].
bool tolerates(const sr_pods& P, int32_t pod, int32_t id_empty, const TaintRec& t) {
  for (int32_t i = P.tol_off[pod]; i < P.tol_off[pod + 1]; ++i) {
    const int32_t eff = P.tol_effect[i];
    if (eff != SR_EFFECT_EMPTY && (eff == SR_EFFECT_OTHER || eff != t.effect)) continue;
    const int32_t key = P.tol_key[i];
    if (key != id_empty && key != t.key) continue;
    const int32_t op = P.tol_op[i];
    if (op == SR_TOL_EXISTS) return true;
    if (op == SR_TOL_EQUAL && P.tol_val[i] == t.val) return true;
  }
  return false;
}

// lower_bound over a sorted array of distinct values, with a bucket index on
// top: bucket b = (x - lo) >> shift holds the lower bound of its first value,
// so a lookup is one table read plus a short scan (binary searches over
// distinct memory requests mispredict on every level).
class LowerBound {
 public:
  void build(const std::vector<int64_t>& v) {
    v_ = &v;
    table_.clear();
    if (v.empty()) return;
    lo_ = v.front();
    const uint64_t span = static_cast<uint64_t>(v.back() - lo_) + 1;
    shift_ = 0;
    while ((span >> shift_) > (1u << 16)) ++shift_;
    const size_t nb = static_cast<size_t>(span >> shift_) + 2;
    table_.resize(nb);
    size_t pos = 0;
    for (size_t b = 0; b < nb; ++b) {
      const int64_t start = lo_ + static_cast<int64_t>(static_cast<uint64_t>(b) << shift_);
      while (pos < v.size() && v[pos] < start) ++pos;
      table_[b] = static_cast<uint32_t>(pos);
    }
  }
  size_t operator()(int64_t x) const {
    const std::vector<int64_t>& v = *v_;
    if (v.empty() || x <= lo_) return 0;
    if (x > v.back()) return v.size();
    size_t pos = table_[static_cast<size_t>(static_cast<uint64_t>(x - lo_) >> shift_)];
    while (v[pos] < x) ++pos;  // stays inside x's bucket: v.back() >= x
    return pos;
  }

 private:
  const std::vector<int64_t>* v_ = nullptr;
  std::vector<uint32_t> table_;
  int64_t lo_ = 0;
  int shift_ = 0;
};

// The raw static spec of a pod: nodeSelector, required node affinity,
// tolerations, host ports.  Hash 0 is reserved for "no static constraints".
template <class F>
void for_each_spec_word(const sr_pods& P, int32_t pod, F&& f) {
  const int32_t s0 = P.sel_off[pod], s1 = P.sel_off[pod + 1];
  f(s1 - s0);
  for (int32_t i = s0; i < s1; ++i) {
    f(P.sel_key[i]);
    f(P.sel_val[i]);
  }
  const bool aff = P.aff_required[pod] != 0;
  f(aff ? P.term_off[pod + 1] - P.term_off[pod] : -1);
  if (aff)
    for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t) {
      f(P.term_expr_off[t + 1] - P.term_expr_off[t]);
      for (int32_t e = P.term_expr_off[t]; e < P.term_expr_off[t + 1]; ++e) {
        f(P.expr_key[e]);
        f(P.expr_op[e]);
        f(P.expr_val_off[e + 1] - P.expr_val_off[e]);
        for (int32_t v = P.expr_val_off[e]; v < P.expr_val_off[e + 1]; ++v) f(P.expr_vals[v]);
      }
      f(P.term_field_off[t + 1] - P.term_field_off[t]);
      for (int32_t g = P.term_field_off[t]; g < P.term_field_off[t + 1]; ++g) {
        f(P.field_key[g]);
        f(P.field_op[g]);
        f(P.field_val_off[g + 1] - P.field_val_off[g]);
        for (int32_t v = P.field_val_off[g]; v < P.field_val_off[g + 1]; ++v) f(P.field_vals[v]);
      }
    }
  const int32_t t0 = P.tol_off[pod], t1 = P.tol_off[pod + 1];
  f(t1 - t0);
  for (int32_t i = t0; i < t1; ++i) {
    f(P.tol_key[i]);
    f(P.tol_op[i]);
    f(P.tol_val[i]);
    f(P.tol_effect[i]);
  }
  for (int32_t i = P.port_off[pod]; i < P.port_off[pod + 1]; ++i) {
    f(P.port_proto[i]);
    f(P.port_num[i]);
    f(P.port_ip[i]);
  }
}

bool has_static_spec(const sr_pods& P, int32_t pod) {
  return P.sel_off[pod] != P.sel_off[pod + 1] || P.tol_off[pod] != P.tol_off[pod + 1] ||
         P.port_off[pod] != P.port_off[pod + 1] || P.aff_required[pod] != 0;
}


}  // namespace

sr_status encode_workload(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                          Workload* w, std::string* err) {
  const sr_pods& P = c->pods;
  const int32_t nc = cands->n_cand;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](int i) {
    auto now = std::chrono::steady_clock::now();
    encode_phase_ms[i] = std::chrono::duration<double, std::milli>(now - t_last).count();
    t_last = now;
  };
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  w->reset();
  w->n_input_cand = nc;
  w->n_input_pods = nc > 0 ? cands->cand_pod_off[nc] : 0;
  if (!snap->nodes.empty() &&
      (c->id_empty != snap->id_empty || c->id_metadata_name != snap->id_metadata_name ||
       c->id_unschedulable_key != snap->id_unschedulable_key)) {
    *err = "cluster string ids differ from the snapshot's (one interner per snapshot)";
    return SR_ERR_INVALID_ARG;
  }

  // ---- spot node dimensions
  const int32_t W = (n_spot + 63) / 64;
  w->n_spot = n_spot;
  w->Wp = std::max(2, (W + 1) & ~1);
  if (w->Wp > MAX_WORDS) {
    *err = "too many spot nodes for one device plan";
    return SR_ERR_CAPACITY;
  }
  w->n_pad = w->Wp * 64;

  phase(0);
  // ---- pass 1: candidate-level fallback (host-decided)
  w->status_host.assign(static_cast<size_t>(nc), STATUS_PENDING);
  auto pod_fallback = [&](int32_t pod) {
    if (P.flags[pod] & SR_POD_FB_MASK) return true;
    if (!in_range(P.req_milli_cpu[pod]) || !in_range(P.req_memory[pod]) || !in_range(P.req_ephemeral[pod]))
      return true;
    if (P.aff_required[pod])
      for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t)
        for (int32_t e = P.term_expr_off[t]; e < P.term_expr_off[t + 1]; ++e)
          if (P.expr_op[e] == SR_OP_GT || P.expr_op[e] == SR_OP_LT) return true;
    return anti_opaque(c, pod);  // required anti-affinity the encoded set cannot read
  };
  for (int32_t i = 0; i < nc; ++i) {
    if (cands->cand_pod_off[i + 1] < cands->cand_pod_off[i]) {
      *err = "cand_pod_off not monotone";
      return SR_ERR_INVALID_ARG;
    }
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j)
      if (cands->cand_pods[j] < 0 || cands->cand_pods[j] >= P.n) {
        *err = "candidate pod index out of range";
        return SR_ERR_INVALID_ARG;
      }
  }
  parallel_for(static_cast<size_t>(nc), 64, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
      if (e == b) {
        w->status_host[i] = SR_CAND_EMPTY;
        continue;
      }
      // an existing pod's opaque anti-affinity may select any incoming pod
      bool fb = (c->pod_affinity ? snap->opaque_total : snap->anti_total) > 0 || (e - b) > MAX_CAND_PODS;
      for (int32_t j = b; j < e && !fb; ++j) fb = pod_fallback(cands->cand_pods[j]);
      if (fb) w->status_host[i] = SR_CAND_FALLBACK;
    }
  });

  phase(8);
  // ---- required pod anti-affinity: static node sets, state-bit pairs and
  // the candidates it sends to the fallback path (antiaff.cpp)
  AntiTerms anti;
  analyse_anti(snap, c, cands, w->Wp, w->status_host, &anti);
  const int32_t bit_shift = 2 * anti.n_pairs;  // host-port bits sit above the pairs

  // ---- host ports: HostPortInfo.CheckConflict [upstream k8s v1.19
  // framework/types.go] as state bits.  A (protocol, port) group whose active
  // pods all bind 0.0.0.0 ("" is 0.0.0.0) is one bit a pod sets and conflicts
  // with.  A group with specific host IPs gets a swapped pair (W, S) plus one
  // bit I(ip) per IP: a 0.0.0.0 pod sets W and S, a pod on ip sets S and
  // I(ip); the conflict bits are the pair-swapped image of the set bits (W <->
  // S, I(ip) fixed), so 0.0.0.0 conflicts with every IP of the group and an
  // IP with 0.0.0.0 and itself only.  Layout: anti-affinity pairs, port pairs
  // (the swapped region), then the single bits.  Pass A classifies the groups,
  // pass B numbers the bits in candidate order; a candidate that would take
  // the state word past 64 bits falls back.
  auto port_key = [](int32_t proto, int32_t port) { return (static_cast<int64_t>(proto) << 32) | uint32_t(port); };
  std::unordered_map<int64_t, uint8_t> group_specific;  // (proto, port) -> has a specific IP
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING) continue;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      for (int32_t k = P.port_off[pod]; k < P.port_off[pod + 1]; ++k)
        if (P.port_num[k] > 0) group_specific[port_key(P.port_proto[k], P.port_num[k])] |= P.port_ip[k] != -1;
    }
  }
  struct PortGroup {
    int32_t pair = -1;                            // pair index (specific IPs), else
    int32_t single = -1;                          // single-bit index (0.0.0.0 only)
    std::unordered_map<int32_t, int32_t> ip_bit;  // specific IP -> single-bit index
  };
  std::unordered_map<int64_t, PortGroup> groups;
  int32_t n_port_pairs = 0, n_port_single = 0;
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING) continue;
    const int32_t pairs0 = n_port_pairs, single0 = n_port_single;
    std::vector<std::pair<int64_t, int32_t>> added_ips;  // undone if the candidate overflows
    std::vector<int64_t> added_groups;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      for (int32_t k = P.port_off[pod]; k < P.port_off[pod + 1]; ++k) {
        if (P.port_num[k] <= 0) continue;
        const int64_t key = port_key(P.port_proto[k], P.port_num[k]);
        auto ins = groups.emplace(key, PortGroup{});
        PortGroup& g = ins.first->second;
        if (ins.second) {
          added_groups.push_back(key);
          if (group_specific[key]) g.pair = n_port_pairs++;
          else g.single = n_port_single++;
        }
        if (P.port_ip[k] != -1 && g.ip_bit.emplace(P.port_ip[k], n_port_single).second) {
          ++n_port_single;
          added_ips.emplace_back(key, P.port_ip[k]);
        }
      }
    }
    if (bit_shift + 2 * n_port_pairs + n_port_single > 64) {  // overflow: undo, fall back
      for (const auto& ki : added_ips) groups[ki.first].ip_bit.erase(ki.second);
      for (int64_t key : added_groups) groups.erase(key);
      n_port_pairs = pairs0;
      n_port_single = single0;
      w->status_host[i] = SR_CAND_FALLBACK;
    }
  }
  const int32_t single_base = bit_shift + 2 * n_port_pairs;
  w->swap_mask = single_base >= 64 ? ~0ull : (1ull << single_base) - 1;
  // Static conflicts with the base snapshot's UsedPorts: one atom per
  // (protocol, port, ip) a pod can ask for, addressed by the bit that stands
  // for the query (single bits: 0.0.0.0 of a single group or I(ip); the W bit
  // of a pair: 0.0.0.0 of that group).
  struct PortQuery {
    int32_t proto, port, ip;
  };
  std::vector<PortQuery> port_query;
  int32_t bit_query[64];
  for (int32_t& b : bit_query) b = -1;
  for (const auto& kv : groups) {
    const int32_t proto = static_cast<int32_t>(kv.first >> 32), port = static_cast<int32_t>(kv.first & 0xffffffff);
    const PortGroup& g = kv.second;
    const int32_t wbit = g.pair >= 0 ? bit_shift + 2 * g.pair : single_base + g.single;
    bit_query[wbit] = static_cast<int32_t>(port_query.size());
    port_query.push_back(PortQuery{proto, port, -1});
    for (const auto& ib : g.ip_bit) {
      bit_query[single_base + ib.second] = static_cast<int32_t>(port_query.size());
      port_query.push_back(PortQuery{proto, port, ib.first});
    }
  }
  // The state bits a pod sets (absolute positions).
  auto pod_port_mask = [&](int32_t pod) {
    uint64_t m = 0;
    for (int32_t k = P.port_off[pod]; k < P.port_off[pod + 1]; ++k) {
      if (P.port_num[k] <= 0) continue;
      auto it = groups.find(port_key(P.port_proto[k], P.port_num[k]));
      if (it == groups.end()) continue;  // a fallback candidate's pod
      const PortGroup& g = it->second;
      if (g.pair < 0) {
        m |= 1ull << (single_base + g.single);
      } else if (P.port_ip[k] == -1) {
        m |= 3ull << (bit_shift + 2 * g.pair);  // W and S
      } else {
        auto ib = g.ip_bit.find(P.port_ip[k]);
        if (ib == g.ip_bit.end()) continue;
        m |= (2ull << (bit_shift + 2 * g.pair)) | (1ull << (single_base + ib->second));  // S and I(ip)
      }
    }
    return m;
  };

  // ---- outcome bookkeeping for non-active candidates
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != SR_CAND_FALLBACK) continue;
    const int32_t g = cands->cand_global ? cands->cand_global[i] : i;
    if (w->first_fallback < 0 || g < w->first_fallback) w->first_fallback = g;
    w->fallback_pods += static_cast<uint64_t>(cands->cand_pod_off[i + 1] - cands->cand_pod_off[i]);
  }

  // ---- taint dictionary over spot nodes (NoSchedule / NoExecute only; the
  // unschedulable flag is the pseudo-taint node.kubernetes.io/unschedulable:NoSchedule)
  std::vector<TaintRec> taints;
  WordDict taint_dict;
  auto taint_id = [&](const TaintRec& t) {
    const int32_t k[3] = {t.key, t.val, t.effect};
    bool ins = false;
    const int32_t id = taint_dict.intern(k, 3, &ins);
    if (ins) taints.push_back(t);
    return id;
  };
  std::vector<int32_t> node_taint_off(static_cast<size_t>(n_spot) + 1, 0), node_taint_ids;
  for (int32_t n = 0; n < n_spot; ++n) {
    const SpotNode& sn = snap->nodes[n];
    for (const TaintRec& t : sn.taints)
      if (t.effect == SR_EFFECT_NO_SCHEDULE || t.effect == SR_EFFECT_NO_EXECUTE) node_taint_ids.push_back(taint_id(t));
    if (sn.unschedulable)
      node_taint_ids.push_back(taint_id(TaintRec{snap->id_unschedulable_key, snap->id_empty, SR_EFFECT_NO_SCHEDULE}));
    node_taint_off[n + 1] = static_cast<int32_t>(node_taint_ids.size());
  }
  const int32_t n_taints = static_cast<int32_t>(taints.size());

  phase(1);
  // Active pods in candidate order.
  std::vector<int32_t> active_pod;   // cluster pod index
  std::vector<int32_t> active_src;   // flat index into cand_pods
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING) continue;
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    w->cand_off.push_back(static_cast<int32_t>(active_pod.size()));
    w->cand_global.push_back(cands->cand_global ? cands->cand_global[i] : i);
    w->cand_src.push_back(i);
    w->max_cand_pods = std::max(w->max_cand_pods, e - b);
    for (int32_t j = b; j < e; ++j) {
      active_pod.push_back(cands->cand_pods[j]);
      active_src.push_back(j);
    }
  }
  w->cand_off.push_back(static_cast<int32_t>(active_pod.size()));
  const int32_t na = static_cast<int32_t>(active_pod.size());

  // ---- distinct static specs.  Pods with word-identical static specs
  // (selector, affinity, tolerations, host ports) share one spec; pods with no
  // static constraints at all share spec 0.  The raw spec is hashed once per
  // pod; the dictionaries are sharded by hash over the pool, and spec ids are
  // assigned in first-occurrence order afterwards, so they do not depend on
  // the thread count.
  std::vector<int32_t> pod_spec(static_cast<size_t>(na), 0);
  std::vector<uint64_t> spec_hash(static_cast<size_t>(na), 0);
  std::vector<uint8_t> spec_shard(static_cast<size_t>(na), 0);
  // The spec words are gathered once per pod (the pod arrays are read at
  // scattered indices) into one buffer per 2048-pod chunk.
  constexpr size_t kChunk = 2048;
  std::vector<std::vector<int32_t>> spec_words((static_cast<size_t>(na) + kChunk - 1) / kChunk);
  std::vector<uint32_t> spec_woff(static_cast<size_t>(na), 0);  // offset in its chunk's buffer
  const size_t n_shards = std::min<size_t>(pool_threads(), 255);
  auto shard_of = [n_shards](uint64_t h) { return static_cast<size_t>(((h >> 32) * n_shards) >> 32); };
  parallel_for(spec_words.size(), 1, [&](size_t lo, size_t hi) {
    for (size_t ch = lo; ch < hi; ++ch) {
      std::vector<int32_t>& buf = spec_words[ch];
      const size_t q1 = std::min(static_cast<size_t>(na), (ch + 1) * kChunk);
      for (size_t q = ch * kChunk; q < q1; ++q) {
        const size_t b0 = buf.size();
        spec_woff[q] = static_cast<uint32_t>(b0);
        const int32_t pod = active_pod[q];
        // anti-affinity ids (term << 1 | has) of the pod, a suffix of its spec
        const int32_t* aid = nullptr;
        size_t nai = 0;
        if (anti.active) {
          const int32_t j = active_src[q];
          aid = anti.pod_ids.data() + anti.pod_off[j];
          nai = static_cast<size_t>(anti.pod_off[j + 1] - anti.pod_off[j]);
        }
        if (!has_static_spec(P, pod) && nai == 0) {
          spec_shard[q] = 255;  // spec 0
          continue;
        }
        for_each_spec_word(P, pod, [&](int32_t x) { buf.push_back(x); });
        if (nai) {
          buf.push_back(static_cast<int32_t>(nai));
          buf.insert(buf.end(), aid, aid + nai);
        }
        const uint64_t h = hash_words(buf.data() + b0, buf.size() - b0);
        spec_hash[q] = h;
        spec_shard[q] = static_cast<uint8_t>(shard_of(h));
      }
    }
  });
  auto words_of = [&](size_t q, size_t* n) {
    const std::vector<int32_t>& buf = spec_words[q / kChunk];
    const size_t e = (q + 1) % kChunk == 0 || q + 1 == static_cast<size_t>(na) ? buf.size() : spec_woff[q + 1];
    *n = e - spec_woff[q];
    return buf.data() + spec_woff[q];
  };
  phase(14);
  struct Shard {
    WordDict dict;
    std::vector<int32_t> rep_q;  // local id -> first active pod
  };
  std::vector<Shard> shards(n_shards);
  parallel_for(n_shards, 1, [&](size_t lo, size_t hi) {
    for (size_t sh = lo; sh < hi; ++sh) {
      Shard& S = shards[sh];
      S.dict.clear();
      for (int32_t q = 0; q < na; ++q) {
        if (spec_shard[q] != sh) continue;
        size_t n = 0;
        const int32_t* p = words_of(static_cast<size_t>(q), &n);
        bool ins = false;
        pod_spec[q] = S.dict.intern(p, n, spec_hash[q], &ins);
        if (ins) S.rep_q.push_back(q);
      }
    }
  });
  phase(15);
  std::vector<int32_t> spec_rep{-1}, spec_rep_q{-1};  // first pod of each spec (cluster / active index)
  {
    struct Rep {
      int32_t q, shard, local;
    };
    std::vector<Rep> reps;
    std::vector<std::vector<int32_t>> global(n_shards);
    for (size_t sh = 0; sh < n_shards; ++sh) {
      global[sh].resize(shards[sh].rep_q.size());
      for (size_t l = 0; l < shards[sh].rep_q.size(); ++l)
        reps.push_back(Rep{shards[sh].rep_q[l], static_cast<int32_t>(sh), static_cast<int32_t>(l)});
    }
    std::sort(reps.begin(), reps.end(), [](const Rep& x, const Rep& y) { return x.q < y.q; });
    for (const Rep& r : reps) {
      global[r.shard][r.local] = static_cast<int32_t>(spec_rep.size());
      spec_rep.push_back(active_pod[r.q]);
      spec_rep_q.push_back(r.q);
    }
    parallel_for(static_cast<size_t>(na), 4096, [&](size_t lo, size_t hi) {
      for (size_t q = lo; q < hi; ++q)
        if (spec_shard[q] != 255) pod_spec[q] = global[spec_shard[q]][pod_spec[q]];
    });
  }
  const size_t n_specs = spec_rep.size();
  phase(7);

  // ---- per spec (parallel): canonical requirements, untolerated taints, ports.
  // A requirement is the word group {len, type, key, op, sorted unique vals}.
  struct SpecCanon {
    int32_t flags = 0;
    std::vector<int32_t> sel;    // nodeSelector requirement groups
    std::vector<int32_t> terms;  // per valid term: {n_req, groups...}
    int32_t n_terms = 0;
    std::vector<int32_t> untol;  // taint ids the spec does not tolerate
    uint64_t ports = 0;          // host-port state bits it sets (pod_port_mask)
    std::vector<int32_t> anti_da, anti_db;  // anti-affinity terms: ANDNOT DA(t) / DB(t)
  };
  std::vector<SpecCanon> canon(n_specs);
  auto put_req = [](std::vector<int32_t>& out, int32_t type, int32_t key, int32_t op, const int32_t* v, int32_t nv) {
    const size_t at = out.size();
    out.push_back(0);
    out.push_back(type);
    out.push_back(key);
    out.push_back(op);
    const size_t vb = out.size();
    out.insert(out.end(), v, v + nv);
    std::sort(out.begin() + vb, out.end());
    out.erase(std::unique(out.begin() + vb, out.end()), out.end());
    out[at] = static_cast<int32_t>(out.size() - at - 1);
  };
  parallel_for(n_specs, 64, [&](size_t lo, size_t hi) {
    std::vector<int32_t> term;
    for (size_t sp = lo; sp < hi; ++sp) {
      SpecCanon& sc = canon[sp];
      if (sp == 0) {  // unconstrained: tolerates nothing
        for (int32_t t = 0; t < n_taints; ++t) sc.untol.push_back(t);
        continue;
      }
      const int32_t pod = spec_rep[sp];
      // Spec.NodeSelector: labels.SelectorFromSet -> Equals requirements.
      for (int32_t i = P.sel_off[pod]; i < P.sel_off[pod + 1]; ++i)
        put_req(sc.sel, REQ_LABEL_EQ, P.sel_key[i], SR_OP_IN, &P.sel_val[i], 1);
      // Required node affinity: MatchNodeSelectorTerms.
      if (P.aff_required[pod]) {
        sc.flags |= CLS_AFF_REQUIRED;
        for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t) {
          const int32_t e0 = P.term_expr_off[t], e1 = P.term_expr_off[t + 1];
          const int32_t f0 = P.term_field_off[t], f1 = P.term_field_off[t + 1];
          if (e0 == e1 && f0 == f1) continue;  // an empty term selects nothing
          bool valid = true;
          term.clear();
          for (int32_t e = e0; e < e1 && valid; ++e) {
            const int32_t nv = P.expr_val_off[e + 1] - P.expr_val_off[e];
            const int32_t op = P.expr_op[e];
            if (P.expr_key[e] == c->id_empty) valid = false;  // validateLabelKey("") fails
            else if ((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 0) valid = false;
            else if ((op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) && nv != 0) valid = false;
            else if (op != SR_OP_IN && op != SR_OP_NOT_IN && op != SR_OP_EXISTS && op != SR_OP_DOES_NOT_EXIST)
              valid = false;
            if (valid) put_req(term, REQ_LABEL_EXPR, P.expr_key[e], op, P.expr_vals + P.expr_val_off[e], nv);
          }
          for (int32_t f = f0; f < f1 && valid; ++f) {
            const int32_t nv = P.field_val_off[f + 1] - P.field_val_off[f];
            const int32_t op = P.field_op[f];
            valid = (op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 1;
            if (valid) put_req(term, REQ_FIELD, P.field_key[f], op, &P.field_vals[P.field_val_off[f]], 1);
          }
          if (!valid) continue;  // a term that fails to build matches nothing
          sc.terms.push_back(static_cast<int32_t>(f1 - f0 + e1 - e0));
          sc.terms.insert(sc.terms.end(), term.begin(), term.end());
          ++sc.n_terms;
        }
        if (sc.n_terms == 0) sc.flags |= CLS_IMPOSSIBLE;
      }
      // Spec.Tolerations against the spot pool's taints.
      for (int32_t t = 0; t < n_taints; ++t)
        if (!tolerates(P, pod, c->id_empty, taints[t])) sc.untol.push_back(t);
      sc.ports = pod_port_mask(pod);
      if (anti.active) {
        const int32_t j = active_src[spec_rep_q[sp]];
        for (int32_t k = anti.pod_off[j]; k < anti.pod_off[j + 1]; ++k) {
          const int32_t t = anti.pod_ids[k] >> 1;
          if (anti.pod_ids[k] & 1) {  // it has t: refuses domains hosting pods t selects
            if (anti.db_any[t]) sc.anti_db.push_back(t);
          } else {  // t selects it: refused by domains hosting pods that have t
            if (anti.da_any[t]) sc.anti_da.push_back(t);
          }
        }
      }
    }
  });

  // ---- requirement ids and class signatures (serial: ids in spec order).
  // Signature: {flags, n_sel, sel ids (sorted), n_terms, per term {n, ids (sorted)},
  // untolerated-set id, ports lo, ports hi}.
  WordDict rdict;      // requirement words {type, key, op, vals...}
  WordDict untol_dict;  // untolerated taint sets
  std::vector<int32_t> sig_words, sig_off{0}, ids;
  for (size_t sp = 0; sp < n_specs; ++sp) {
    const SpecCanon& sc = canon[sp];
    auto intern_groups = [&](const int32_t* g, int32_t n_groups, size_t* used) {
      ids.clear();
      size_t i = 0;
      for (int32_t k = 0; k < n_groups; ++k) {
        ids.push_back(rdict.intern(g + i + 1, static_cast<size_t>(g[i])));
        i += 1 + static_cast<size_t>(g[i]);
      }
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      sig_words.push_back(static_cast<int32_t>(ids.size()));
      sig_words.insert(sig_words.end(), ids.begin(), ids.end());
      if (used) *used = i;
    };
    sig_words.push_back(sc.flags);
    int32_t n_sel = 0;
    for (size_t i = 0; i < sc.sel.size(); i += 1 + static_cast<size_t>(sc.sel[i])) ++n_sel;
    intern_groups(sc.sel.data(), n_sel, nullptr);
    sig_words.push_back(sc.n_terms);
    for (size_t i = 0, k = 0; k < static_cast<size_t>(sc.n_terms); ++k) {
      size_t used = 0;
      intern_groups(sc.terms.data() + i + 1, sc.terms[i], &used);
      i += 1 + used;
    }
    sig_words.push_back(untol_dict.intern(sc.untol));
    sig_words.push_back(static_cast<int32_t>(sc.ports & 0xffffffffu));
    sig_words.push_back(static_cast<int32_t>(sc.ports >> 32));
    sig_words.push_back(static_cast<int32_t>(sc.anti_da.size()));
    sig_words.insert(sig_words.end(), sc.anti_da.begin(), sc.anti_da.end());
    sig_words.push_back(static_cast<int32_t>(sc.anti_db.size()));
    sig_words.insert(sig_words.end(), sc.anti_db.begin(), sc.anti_db.end());
    sig_off.push_back(static_cast<int32_t>(sig_words.size()));
  }
  const int32_t n_reqs = static_cast<int32_t>(rdict.size());
  const int32_t n_ports = static_cast<int32_t>(port_query.size());
  const int32_t A_REQ = 1, A_TAINT = 1 + n_reqs, A_PORT = 1 + n_reqs + n_taints;
  // Composite atoms, one per distinct untolerated-taint set U of the pods:
  // atom 0 AND NOT (OR of U's taint atoms) -- the pod-count check and
  // TaintToleration / NodeUnschedulable in one row, so a class program opens
  // with a single AND instead of 1 + |U| operations.
  const int32_t A_ANTI = A_PORT + n_ports;  // DA(t) at A_ANTI + 2t, DB(t) at A_ANTI + 2t + 1
  const int32_t A_COMP = A_ANTI + 2 * anti.n_terms;
  std::vector<int32_t> comp_of(untol_dict.size(), -1), comp_sets;  // untolerated-set ids
  auto comp_atom = [&](int32_t u) {
    if (untol_dict.len(u) == 0) return 0;  // tolerates every taint: the pod-count atom alone
    if (comp_of[u] < 0) {
      comp_of[u] = static_cast<int32_t>(comp_sets.size());
      comp_sets.push_back(u);
    }
    return A_COMP + comp_of[u];
  };

  phase(2);
  // ---- intern classes (atom programs), once per distinct signature
  WordDict class_dict;
  std::vector<int32_t> spec_class(n_specs);
  w->cls_prog_off.push_back(0);
  auto emit = [&](int32_t atom, int32_t kind) { w->cls_prog.push_back(atom << 2 | kind); };
  for (size_t sp = 0; sp < n_specs; ++sp) {
    const int32_t* g = sig_words.data() + sig_off[sp];
    bool ins = false;
    spec_class[sp] = class_dict.intern(g, static_cast<size_t>(sig_off[sp + 1] - sig_off[sp]), &ins);
    if (!ins) continue;
    // program: AND atoms, AND-NOT atoms, then the ORed terms (TERM_START
    // opens a term, TERM_AND extends it); an impossible class ANDs atom 0
    // with its complement
    const int32_t flags = g[0], n_sel = g[1];
    const int32_t* sel = g + 2;
    const int32_t* tp = sel + n_sel;
    const int32_t n_terms = *tp++;
    const int32_t* term_words = tp;
    for (int32_t k = 0; k < n_terms; ++k) tp += 1 + *tp;
    const int32_t untol = tp[0];
    const uint64_t ports = static_cast<uint32_t>(tp[1]) | static_cast<uint64_t>(static_cast<uint32_t>(tp[2])) << 32;
    emit(comp_atom(untol), PROG_AND);  // len(pods)+1 <= allowed pods, untolerated taints
    for (int32_t k = 0; k < n_sel; ++k) emit(A_REQ + sel[k], PROG_AND);
    for (int32_t b = 0; b < 64; ++b)  // the base UsedPorts conflicting with each host port it asks for
      if ((ports >> b & 1) && bit_query[b] >= 0) emit(A_PORT + bit_query[b], PROG_ANDNOT);
    {  // anti-affinity base conflicts
      const int32_t* ad = tp + 3;
      const int32_t nda = ad[0];
      for (int32_t k = 0; k < nda; ++k) emit(A_ANTI + 2 * ad[1 + k], PROG_ANDNOT);
      const int32_t* bd = ad + 1 + nda;
      for (int32_t k = 0; k < bd[0]; ++k) emit(A_ANTI + 2 * bd[1 + k] + 1, PROG_ANDNOT);
    }
    if (flags & CLS_IMPOSSIBLE) {
      emit(0, PROG_ANDNOT);
    } else {
      for (int32_t k = 0; k < n_terms; ++k) {
        const int32_t n = *term_words++;
        for (int32_t i = 0; i < n; ++i) emit(A_REQ + term_words[i], i == 0 ? PROG_TERM_START : PROG_TERM_AND);
        term_words += n;
      }
    }
    w->cls_prog_off.push_back(static_cast<int32_t>(w->cls_prog.size()));
    w->n_classes++;
  }
  w->n_atoms = A_COMP + static_cast<int32_t>(comp_sets.size());
  phase(3);
  // ---- spot nodes: base capacity state and the atom rows
  const int32_t NP = w->n_pad, Wp = w->Wp;
  w->free_cpu.assign(NP, 0);
  w->free_mem.assign(NP, 0);
  w->free_eph.assign(NP, 0);
  w->pods_left.assign(NP, 0);
  w->port_bits.assign(NP, 0);
  w->atoms.assign(static_cast<size_t>(w->n_atoms) * Wp, 0);
  auto set_atom = [&](int32_t atom, int32_t n) {
    w->atoms[static_cast<size_t>(atom) * Wp + (n >> 6)] |= 1ull << (n & 63);
  };
  for (int32_t n = 0; n < n_spot; ++n) {
    const SpotNode& sn = snap->nodes[n];
    const NodeState& st = snap->state[n];
    for (int r = 0; r < 3; ++r) {
      if (!in_range(sn.alloc[r]) || !in_range(st.requested[r])) {
        *err = "spot node quantity outside [0, 2^62)";
        return SR_ERR_CAPACITY;
      }
    }
    w->free_cpu[n] = sn.alloc[0] - st.requested[0];
    w->free_mem[n] = sn.alloc[1] - st.requested[1];
    w->free_eph[n] = sn.alloc[2] - st.requested[2];
    const int64_t left = sn.alloc_pods - st.npods;
    w->pods_left[n] = static_cast<int32_t>(std::max<int64_t>(-(1 << 30), std::min<int64_t>(left, 1 << 30)));
    if (left >= 1) set_atom(0, n);
    // base UsedPorts: static conflicts (atoms A_PORT + q, in the F rows); the
    // state word starts empty (it only carries the candidate's own pods)
    w->port_bits[n] = 0;
    for (const Port& u : st.ports)
      for (int32_t q = 0; q < n_ports; ++q) {
        const PortQuery& pq = port_query[q];
        if (pq.proto == u.proto && pq.port == u.port && (pq.ip == -1 || u.ip == -1 || u.ip == pq.ip))
          set_atom(A_PORT + q, n);
      }
    for (int32_t k = node_taint_off[n]; k < node_taint_off[n + 1]; ++k) set_atom(A_TAINT + node_taint_ids[k], n);
  }
  w->node_rec.assign(static_cast<size_t>(NP) * 8, 0);
  for (int32_t n = 0; n < n_spot; ++n) {
    uint64_t* r = &w->node_rec[static_cast<size_t>(n) * 8];
    r[0] = static_cast<uint64_t>(w->free_cpu[n]);
    r[1] = static_cast<uint64_t>(w->free_mem[n]);
    r[2] = static_cast<uint64_t>(w->free_eph[n]);
    r[3] = w->port_bits[n];
    r[4] = static_cast<uint64_t>(static_cast<int64_t>(w->pods_left[n]));
  }
  // anti-affinity base conflicts: DA(t), DB(t)
  for (int32_t t = 0; t < anti.n_terms; ++t) {
    std::copy_n(&anti.da[static_cast<size_t>(t) * Wp], Wp, &w->atoms[static_cast<size_t>(A_ANTI + 2 * t) * Wp]);
    std::copy_n(&anti.db[static_cast<size_t>(t) * Wp], Wp, &w->atoms[static_cast<size_t>(A_ANTI + 2 * t + 1) * Wp]);
  }
  // composite atoms: atom 0 AND NOT (any taint of the set)
  for (size_t k = 0; k < comp_sets.size(); ++k) {
    uint64_t* row = &w->atoms[static_cast<size_t>(A_COMP + static_cast<int32_t>(k)) * Wp];
    for (int32_t i = 0; i < Wp; ++i) {
      uint64_t any = 0;
      const int32_t* u = untol_dict.data(comp_sets[k]);
      for (size_t j = 0; j < untol_dict.len(comp_sets[k]); ++j) any |= w->atoms[static_cast<size_t>(A_TAINT + u[j]) * Wp + i];
      row[i] = w->atoms[i] & ~any;
    }
  }
  phase(9);
  // requirement atoms: one label-value column per distinct key
  std::unordered_map<int32_t, std::vector<int32_t>> col;  // key -> value per node (INT32_MIN absent)
  for (int32_t ri = 0; ri < n_reqs; ++ri) {
    const int32_t* r = rdict.data(ri);  // {type, key, op, vals...}
    if (r[0] != REQ_FIELD && !col.count(r[1])) col.emplace(r[1], std::vector<int32_t>(n_spot, INT32_MIN));
  }
  for (int32_t n = 0; n < n_spot; ++n)
    for (const auto& kv : snap->nodes[n].labels) {
      auto it = col.find(kv.first);
      if (it != col.end()) it->second[n] = kv.second;
    }
  parallel_for(static_cast<size_t>(n_reqs), 1, [&](size_t rlo, size_t rhi) {
  for (size_t ri = rlo; ri < rhi; ++ri) {  // one atom row per requirement: disjoint writes
    const int32_t* rw = rdict.data(static_cast<int32_t>(ri));
    const Requirement r{rw[0], rw[1], rw[2], std::vector<int32_t>(rw + 3, rw + rdict.len(static_cast<int32_t>(ri)))};
    const int32_t atom = A_REQ + static_cast<int32_t>(ri);
    if (r.type == REQ_FIELD) {
      // fields.Set{"metadata.name": node.Name}; any other key reads as "".
      const bool is_name = r.key == c->id_metadata_name && c->id_metadata_name != -1;
      for (int32_t n = 0; n < n_spot; ++n) {
        const int32_t fv = is_name ? snap->nodes[n].name : c->id_empty;
        const bool eq = fv == r.vals[0];
        if (r.op == SR_OP_IN ? eq : !eq) set_atom(atom, n);
      }
      continue;
    }
    const std::vector<int32_t>& v = col.at(r.key);
    for (int32_t n = 0; n < n_spot; ++n) {
      const bool has = v[n] != INT32_MIN;
      bool m;
      switch (r.op) {
        case SR_OP_IN:
          m = has && std::binary_search(r.vals.begin(), r.vals.end(), v[n]);
          break;
        case SR_OP_NOT_IN:
          m = !has || !std::binary_search(r.vals.begin(), r.vals.end(), v[n]);
          break;
        case SR_OP_EXISTS:
          m = has;
          break;
        default:  // DoesNotExist
          m = !has;
          break;
      }
      if (m) set_atom(atom, n);
    }
  }
  });

  phase(4);
  // ---- T row descriptors.  A pod asking r in one dimension uses the row of the
  // smallest node free value v >= r: it selects exactly the nodes with
  // free >= r (no node value lies in [r, v)), and there are at most
  // min(distinct requests, distinct node values) such rows.  A request above
  // every node's free capacity maps to the empty row.
  w->t_dim.push_back(3);
  w->t_thr.push_back(0);  // row 0: every node
  const int64_t kNever = INT64_MAX;  // free >= INT64_MAX never holds (free < 2^62)
  std::vector<int64_t> node_vals[3];
  const std::vector<int64_t>* frees[3] = {&w->free_cpu, &w->free_mem, &w->free_eph};
  std::vector<int32_t> t_index[3];  // lower-bound position -> T row
  LowerBound lb[3];
  parallel_for(3, 1, [&](size_t lo, size_t hi) {
    for (size_t d = lo; d < hi; ++d) {
      node_vals[d].assign(frees[d]->begin(), frees[d]->begin() + n_spot);
      std::sort(node_vals[d].begin(), node_vals[d].end());
      node_vals[d].erase(std::unique(node_vals[d].begin(), node_vals[d].end()), node_vals[d].end());
      t_index[d].assign(node_vals[d].size() + 1, -1);
      lb[d].build(node_vals[d]);
    }
  });
  // every field of pod_rows / pod_rec is written below (only the padding is
  // cleared here): the vectors keep their size across encodes, so this is
  // no zero fill in the steady state
  w->pod_rows.resize(static_cast<size_t>(na) * 4);
  w->pod_rec.resize(static_cast<size_t>(na + 128) * 6);  // padded: K2 stages 64-pod halves
  std::fill(w->pod_rec.begin() + static_cast<size_t>(na) * 6, w->pod_rec.end(), 0);
  w->pod_src = active_src;
  // Pods whose F row is certainly empty point at one all-zero class (atom 0
  // AND NOT atom 0), so K2 knows them without reading their rows: a class
  // that ANDs an empty atom, ANDs the complement of a full one, or whose
  // terms each hold an empty atom; or a request above every node's free
  // value in some dimension (the never-row).  Sound, not complete: the rest
  // is found exactly on the device.
  std::vector<uint8_t> cls_empty(static_cast<size_t>(w->n_classes), 0);
  {
    std::vector<uint8_t> atom_empty(static_cast<size_t>(w->n_atoms)), atom_full(static_cast<size_t>(w->n_atoms));
    for (int32_t a = 0; a < w->n_atoms; ++a) {
      const uint64_t* row = &w->atoms[static_cast<size_t>(a) * Wp];
      int64_t pop = 0;
      for (int32_t i = 0; i < Wp; ++i) pop += __builtin_popcountll(row[i]);
      atom_empty[a] = pop == 0;
      atom_full[a] = pop == n_spot;
    }
    for (int32_t c = 0; c < w->n_classes; ++c) {
      bool empty = false, has_terms = false, all_terms_empty = true, term_empty = false;
      for (int32_t o = w->cls_prog_off[c]; o < w->cls_prog_off[c + 1]; ++o) {
        const int32_t atom = w->cls_prog[o] >> 2, kind = w->cls_prog[o] & 3;
        if (kind == PROG_AND) {
          empty = empty || atom_empty[atom];
        } else if (kind == PROG_ANDNOT) {
          empty = empty || atom_full[atom];
        } else {
          if (kind == PROG_TERM_START) {
            if (has_terms) all_terms_empty = all_terms_empty && term_empty;
            has_terms = true;
            term_empty = false;
          }
          term_empty = term_empty || atom_empty[atom];
        }
      }
      if (has_terms) all_terms_empty = all_terms_empty && term_empty;
      cls_empty[c] = empty || (has_terms && all_terms_empty);
    }
  }
  std::atomic<bool> any_dead{false};
  // per pod (parallel): requests, records and the lower-bound position of each
  // request among the node values (stored in pod_rows[1..3] for now)
  parallel_for(static_cast<size_t>(na), 2048, [&](size_t lo, size_t hi) {
    for (size_t q = lo; q < hi; ++q) {
      const int32_t pod = active_pod[q];
      const int64_t rc = P.req_milli_cpu[pod], rm = P.req_memory[pod], re = P.req_ephemeral[pod];
      const bool zero = rc == 0 && rm == 0 && re == 0;
      int32_t* r = &w->pod_rows[q * 4];
      r[0] = spec_class[pod_spec[q]];
      r[1] = zero ? -1 : static_cast<int32_t>(lb[0](rc));
      r[2] = zero ? -1 : static_cast<int32_t>(lb[1](rm));
      r[3] = zero ? -1 : static_cast<int32_t>(lb[2](re));
      uint64_t* rec = &w->pod_rec[q * 6];
      rec[0] = static_cast<uint64_t>(rc);
      rec[1] = static_cast<uint64_t>(rm);
      rec[2] = static_cast<uint64_t>(re);
      rec[3] = canon[pod_spec[q]].ports |
               (anti.active ? anti.pod_bits[active_src[q]] : 0);
      bool dead = cls_empty[r[0]] != 0;
      for (int d = 0; d < 3; ++d) dead = dead || (r[1 + d] >= 0 && static_cast<size_t>(r[1 + d]) == node_vals[d].size());
      if (dead) {
        r[0] = -1;  // the empty class, appended below
        any_dead.store(true, std::memory_order_relaxed);
      }
    }
  });
  phase(10);
  if (any_dead.load(std::memory_order_relaxed)) {
    emit(0, PROG_AND);
    emit(0, PROG_ANDNOT);
    w->cls_prog_off.push_back(static_cast<int32_t>(w->cls_prog.size()));
    w->empty_class = w->n_classes++;
  }
  phase(11);
  // positions -> T rows: row 0 = every node, then the used positions of each
  // dimension in increasing threshold order (rows grouped by dimension, so
  // K0 compares one dimension per wave)
  std::vector<uint8_t> used[3];
  for (int d = 0; d < 3; ++d) used[d].assign(node_vals[d].size() + 1, 0);
  for (int32_t q = 0; q < na; ++q) {
    const int32_t* r = &w->pod_rows[static_cast<size_t>(q) * 4];
    for (int d = 0; d < 3; ++d)
      if (r[1 + d] >= 0) used[d][static_cast<size_t>(r[1 + d])] = 1;
  }
  w->t_off[0] = 0;
  w->t_off[1] = 1;
  for (int d = 0; d < 3; ++d) {
    for (size_t pos = 0; pos < used[d].size(); ++pos) {
      if (!used[d][pos]) continue;
      t_index[d][pos] = static_cast<int32_t>(w->t_dim.size());
      w->t_dim.push_back(d);
      w->t_thr.push_back(pos == node_vals[d].size() ? kNever : node_vals[d][pos]);
    }
    w->t_off[d + 2] = static_cast<int32_t>(w->t_dim.size());
  }
  phase(12);
  // Node ranks: the dimension-d rows are in threshold order, so the rows a
  // node belongs to (threshold <= its free value) are a prefix of them; K0
  // sets bit n of the dimension's row r exactly when r < rank(n).
  w->node_rank.assign(static_cast<size_t>(3) * NP, 0);
  for (int d = 0; d < 3; ++d) {
    std::vector<int32_t> below(used[d].size() + 1, 0);  // used positions in [0, pos)
    for (size_t pos = 0; pos < used[d].size(); ++pos) below[pos + 1] = below[pos] + used[d][pos];
    const std::vector<int64_t>& fr = *frees[d];
    int32_t* rk = &w->node_rank[static_cast<size_t>(d) * NP];
    for (int32_t n = 0; n < n_spot; ++n) rk[n] = below[lb[d](fr[n]) + 1];  // fr[n] is node_vals[d][pos]
  }
  phase(13);
  parallel_for(static_cast<size_t>(na), 4096, [&](size_t lo, size_t hi) {
    auto off = [&](int32_t table_row) { return static_cast<uint64_t>(table_row) * static_cast<uint64_t>(w->Wp); };
    for (size_t q = lo; q < hi; ++q) {
      int32_t* r = &w->pod_rows[q * 4];
      if (r[0] < 0) r[0] = w->empty_class;
      for (int d = 0; d < 3; ++d) r[1 + d] = r[1 + d] < 0 ? 0 : t_index[d][static_cast<size_t>(r[1 + d])];
      uint64_t* rec = &w->pod_rec[q * 6];
      rec[4] = off(r[0]) | off(w->n_classes + r[1]) << 32;
      rec[5] = off(w->n_classes + r[2]) | off(w->n_classes + r[3]) << 32;
    }
  });
  if ((static_cast<uint64_t>(w->n_classes) + w->t_dim.size()) * static_cast<uint64_t>(w->Wp) >= (1ull << 32)) {
    *err = "bitmask tables exceed 2^32 words";
    return SR_ERR_CAPACITY;
  }

  // ---- class programs of <= 8 operations in fixed 8-slot records (K0 reads
  // one record with one scalar load); -1 pads, -2 in slot 0 marks a longer
  // program (read through cls_prog_off)
  w->cls_prog8.assign(static_cast<size_t>(w->n_classes) * 8, -1);
  for (int32_t c = 0; c < w->n_classes; ++c) {
    const int32_t o = w->cls_prog_off[c], len = w->cls_prog_off[c + 1] - o;
    int32_t* slot = &w->cls_prog8[static_cast<size_t>(c) * 8];
    if (len > 8) {
      slot[0] = -2;
      continue;
    }
    for (int32_t i = 0; i < len; ++i) slot[i] = w->cls_prog[o + i];
  }

  phase(5);
  // ---- K2 work list: longest candidates first (counting sort, stable)
  {
    const size_t nc = w->cand_off.size() - 1;
    std::vector<int32_t> cnt(MAX_CAND_PODS + 2, 0);
    for (size_t i = 0; i < nc; ++i) ++cnt[MAX_CAND_PODS - (w->cand_off[i + 1] - w->cand_off[i])];
    for (int32_t v = 0, acc = 0; v <= MAX_CAND_PODS + 1; ++v) {
      const int32_t c = cnt[v];
      cnt[v] = acc;
      acc += c;
    }
    w->list.assign(nc * 4, 0);
    for (size_t i = 0; i < nc; ++i) {
      const int32_t b = w->cand_off[i], e = w->cand_off[i + 1];
      int32_t* l = &w->list[static_cast<size_t>(cnt[MAX_CAND_PODS - (e - b)]++) * 4];
      l[0] = static_cast<int32_t>(i);
      l[1] = b;
      l[2] = e;
      l[3] = w->cand_global[i];
    }
  }
  phase(6);
  return SR_OK;
}

}  // namespace sr
