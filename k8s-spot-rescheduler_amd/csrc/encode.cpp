// encode.cpp — snapshot + candidate pod lists -> SoA workload for gfx950.
//
// The predicate of one (pod, spot node) pair against the *base* snapshot
// (k8s v1.19.2 NodeUnschedulable, NodeResourcesFit, NodeName, NodePorts,
// NodeAffinity, TaintToleration, InterPodAffinity [upstream]; call site
// rescheduler.go:344) factors into a conjunction of terms that each depend on
// a low-cardinality projection of the pod:
//
//   fits(p, n) = S[class(p)](n) & T[cpu(p)](n) & T[mem(p)](n) & T[eph(p)](n)
//
//   S = static(class, n)            selector / affinity / taints / base ports
//       AND len(pods)+1 <= allowed  (pod-count part of NodeResourcesFit)
//   T = free_dim(n) >= threshold    (zero-request pods use row 0 = all nodes:
//                                    fitsRequest skips the resource checks)
//
// where "class" interns everything static about a pod.  S and T are bitmask
// rows over spot nodes in NodeInfoArray order, built on the GPU (K0); the
// pod's feasibility row is their AND, formed inside K2.  Everything that
// changes while a candidate's pods are placed (capacity, pod count, host
// ports, anti-affinity pairs) is state K2 carries per candidate.  Features
// outside this set route the whole candidate to the reference path
// (SR_CAND_FALLBACK).
//
// Persistence (EncoderCache, one per sr_ctx): a planner sees one snapshot
// after another, mostly identical.  The spot pool is compared with the last
// call's view by per-node fingerprints; label columns, requirement rows and
// taint rows survive while the static view does, capacity records and sorted
// free values while the state view does (a few changed nodes are patched in
// place).  Pod specs and requirements are interned by content across calls,
// so a call canonicalises only specs it has never seen.
#include <algorithm>
#include <array>
#include <map>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "host.hpp"
#include "pool.hpp"
#include "worddict.hpp"

namespace sr {

double encode_phase_ms[16];  // host-side profile of the last encode (tools/encode_stats)

namespace {

constexpr int64_t kQuantityLimit = int64_t(1) << 62;
constexpr size_t kSpecShards = 16;             // fixed: spec ids do not depend on the thread count
constexpr size_t kMaxSpecs = size_t(1) << 21;  // content dictionaries are dropped beyond these
constexpr size_t kMaxReqs = size_t(1) << 18;
// below this many pods, per-pod passes run on the calling thread (SR_SERIAL_PODS)
int32_t serial_pods() {
  static const int32_t v = [] {
    const char* e = std::getenv("SR_SERIAL_PODS");
    return e ? std::max(0, std::atoi(e)) : 4096;
  }();
  return v;
}

bool in_range(int64_t v) { return v >= 0 && v < kQuantityLimit; }

// HostPortInfo.CheckConflict of one (protocol, port) entry pair by their IPs
// (0.0.0.0 = -1 meets every IP, an IP meets 0.0.0.0 and itself), and
// VolumeRestrictions' isVolumeConflict for disks (-1: read-write, meets every
// mount; kReadOnlyMount: meets read-write mounts only).
bool port_conflict(int32_t a, int32_t b) { return a == -1 || b == -1 || (a == b && a != kReadOnlyMount); }

// A host-port query (protocol, port, IP) whose base conflicts make an atom row.
struct PortQuery {
  int32_t proto, port, ip;
};
static_assert(sizeof(PortQuery) == 3 * sizeof(int32_t), "CandReuse::port_q holds queries as int32 triples");


// (limit key, unique volume name) as one word.
inline uint64_t att_word(int32_t key, int32_t id) {
  return static_cast<uint64_t>(static_cast<uint32_t>(key)) << 32 | static_cast<uint32_t>(id);
}
// The pod's attachable volumes of limit key `key`.
int32_t pod_att_of(const sr_cluster* c, int32_t pod, int32_t key) {
  int32_t n = 0;
  for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1]; ++a) n += c->volumes->att_key[a] == key;
  return n;
}
constexpr int32_t kNoName = INT32_MIN;  // no shared scalar name (volume keys are negative names)
// EncoderCache::PodMemo::bits
enum : uint32_t { MEMO_PLAIN = 1, MEMO_FB = 2, MEMO_ACC_BAD = 4, MEMO_ACC_DIFF = 8, MEMO_PORTS = 16 };

// REQ_ZONE: VolumeZone's check of one PV zone / region label {key, zone keys
// [4], values}: a node passes when it carries none of the four zone keys, or
// its value of `key` ("" when absent) is one of the values.
enum : int32_t { REQ_LABEL_EQ = 0, REQ_LABEL_EXPR = 1, REQ_FIELD = 2, REQ_ZONE = 3 };

inline uint64_t mix(uint64_t h, uint64_t x) {
  h = (h ^ x) * 0xff51afd7ed558ccdull;
  return h ^ (h >> 32);
}

// NodeResourcesFit's ScalarResources check of one (name, request) against the
// base snapshot: bit n set when alloc[s] >= request + requested[s] on spot node
// n (a node without s allocates 0; volume limit keys under negative names: the
// node's limit, or unlimited, against its unique attachable volumes of the key
// plus the pod's count).  row: [Wp] words, zeroed by the caller.
inline bool scalar_query_node(const sr_snapshot* snap, int32_t n, int64_t name64, int64_t req) {
  const int32_t name = static_cast<int32_t>(name64);
  const int64_t alloc = scalar_alloc_of(snap->nodes[n], name);
  const int64_t used = scalar_used_of(snap->state[n], name);
  // Go int64 arithmetic: request + requested wraps like the reference's
  const int64_t need = static_cast<int64_t>(static_cast<uint64_t>(req) + static_cast<uint64_t>(used));
  return !(alloc < need);
}
void scalar_query_row(const sr_snapshot* snap, int64_t name64, int64_t req, uint64_t* row) {
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  for (int32_t n = 0; n < n_spot; ++n)
    if (scalar_query_node(snap, n, name64, req)) row[n >> 6] |= 1ull << (n & 63);
}

// The base free value (alloc - requested) of each shared scalar name on every
// spot node: the extension records' node_scal rows, [names][n_pad].
inline int64_t node_scal_value(const sr_snapshot* snap, int32_t n, int32_t name) {
  // Go int64 arithmetic: alloc - requested wraps like the reference's
  return static_cast<int64_t>(static_cast<uint64_t>(scalar_alloc_of(snap->nodes[n], name)) -
                              static_cast<uint64_t>(scalar_used_of(snap->state[n], name)));
}
void node_scal_rows(const sr_snapshot* snap, const std::vector<int32_t>& names, int32_t n_pad, int64_t* out) {
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  for (size_t u = 0; u < names.size(); ++u)
    for (int32_t n = 0; n < n_spot; ++n)
      out[u * static_cast<size_t>(n_pad) + static_cast<size_t>(n)] = node_scal_value(snap, n, names[u]);
}

// HostPortInfo.CheckConflict of each query against every spot node's base
// UsedPorts, row q written to dst + q * Wp.  Rows are kept in C.port_rows by
// query across calls: a state refresh that patched a few nodes patches their
// bits, any other refresh drops them.
void port_conflict_rows(EncoderCache& C, const sr_snapshot* snap, const PortQuery* queries, int32_t n_ports,
                        int32_t Wp, uint64_t* dst) {
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  auto conflicts = [&](int32_t n, const PortQuery& pq) {
    for (const Port& u : snap->state[n].ports)
      if (pq.proto == u.proto && pq.port == u.port && port_conflict(pq.ip, u.ip)) return true;
    return false;
  };
  auto qkey = [](const PortQuery& pq) {
    return mix(mix(mix(0x51ull, static_cast<uint32_t>(pq.proto)), static_cast<uint32_t>(pq.port)),
               static_cast<uint32_t>(pq.ip));
  };
  if (C.port_rows_gen != C.state_gen) {
    const bool patch = C.patched_from != ~0ull && C.port_rows_gen == C.patched_from && !C.patched_nodes.empty() &&
                       C.port_rows.size() < 4096;
    if (patch) {
      for (auto& kv : C.port_rows) {
        // the key does not carry the query: rebuild it from the row's stored tail
        const std::vector<uint64_t>& row = kv.second;
        const PortQuery pq{static_cast<int32_t>(row[Wp]), static_cast<int32_t>(row[Wp + 1]),
                           static_cast<int32_t>(row[Wp + 2])};
        for (int32_t n : C.patched_nodes) {
          uint64_t& wd = kv.second[static_cast<size_t>(n >> 6)];
          const uint64_t bit = 1ull << (n & 63);
          wd = conflicts(n, pq) ? (wd | bit) : (wd & ~bit);
        }
      }
    } else {
      C.port_rows.clear();
    }
    C.port_rows_gen = C.state_gen;
  }
  std::vector<int32_t> missing;
  std::vector<std::vector<uint64_t>*> rows(static_cast<size_t>(n_ports), nullptr);
  for (int32_t q = 0; q < n_ports; ++q) {
    const PortQuery& pq = queries[q];
    auto it = C.port_rows.find(qkey(pq));
    if (it != C.port_rows.end() && static_cast<int32_t>(it->second[Wp]) == pq.proto &&
        static_cast<int32_t>(it->second[Wp + 1]) == pq.port && static_cast<int32_t>(it->second[Wp + 2]) == pq.ip) {
      rows[q] = &it->second;
    } else {
      missing.push_back(q);
    }
  }
  if (!missing.empty()) {  // one pass over the nodes for every query not cached
    std::vector<std::vector<uint64_t>> fresh(missing.size(), std::vector<uint64_t>(static_cast<size_t>(Wp) + 3, 0));
    for (int32_t n = 0; n < n_spot; ++n)
      for (const Port& u : snap->state[n].ports)
        for (size_t m = 0; m < missing.size(); ++m) {
          const PortQuery& pq = queries[missing[m]];
          if (pq.proto == u.proto && pq.port == u.port && port_conflict(pq.ip, u.ip))
            fresh[m][static_cast<size_t>(n >> 6)] |= 1ull << (n & 63);
        }
    for (size_t m = 0; m < missing.size(); ++m) {
      const PortQuery& pq = queries[missing[m]];
      fresh[m][Wp] = static_cast<uint64_t>(static_cast<uint32_t>(pq.proto));
      fresh[m][Wp + 1] = static_cast<uint64_t>(static_cast<uint32_t>(pq.port));
      fresh[m][Wp + 2] = static_cast<uint64_t>(static_cast<uint32_t>(pq.ip));
      if (C.port_rows.size() < 4096 && C.port_rows.find(qkey(pq)) == C.port_rows.end()) {
        auto& slot = C.port_rows[qkey(pq)];
        slot = std::move(fresh[m]);
        rows[missing[m]] = &slot;
      } else {  // full, or another query under the same key: not cached
        std::copy_n(fresh[m].begin(), Wp, dst + static_cast<size_t>(missing[m]) * Wp);
      }
    }
  }
  for (int32_t q = 0; q < n_ports; ++q)
    if (rows[q]) std::copy_n(rows[q]->begin(), Wp, dst + static_cast<size_t>(q) * Wp);
}

// v1.Toleration.ToleratesTaint [upstream k8s.io/api/core/v1/toleration.go]
// over a spec's toleration words {key, op, value, effect}.
bool tolerates(const std::vector<int32_t>& tol, int32_t id_empty, const TaintRec& t) {
  for (size_t i = 0; i + 4 <= tol.size(); i += 4) {
    const int32_t key = tol[i], op = tol[i + 1], val = tol[i + 2], eff = tol[i + 3];
    if (eff != SR_EFFECT_EMPTY && (eff == SR_EFFECT_OTHER || eff != t.effect)) continue;
    if (key != id_empty && key != t.key) continue;
    if (op == SR_TOL_EXISTS) return true;
    if (op == SR_TOL_EQUAL && val == t.val) return true;
  }
  return false;
}

// lower_bound over a sorted array of distinct values with a bucket index on
// top (bucket b = (x - lo) >> shift holds the position of its first value):
// one table read plus a binary search inside the bucket.  Lookups over
// scattered requests mispredict on every level of a plain binary search.
class LowerBound {
 public:
  void build(const std::vector<int64_t>& v) {
    v_ = &v;
    table_.clear();
    if (v.empty()) return;
    lo_ = v.front();
    const uint64_t span = static_cast<uint64_t>(v.back() - lo_) + 1;
    const uint64_t want = std::max<uint64_t>(64, 2 * v.size());
    shift_ = 0;
    while ((span >> shift_) > want) ++shift_;
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
    const size_t b = static_cast<size_t>(static_cast<uint64_t>(x - lo_) >> shift_);
    return static_cast<size_t>(std::lower_bound(v.begin() + table_[b], v.begin() + table_[b + 1], x) - v.begin());
  }

 private:
  const std::vector<int64_t>* v_ = nullptr;
  std::vector<uint32_t> table_;
  int64_t lo_ = 0;
  int shift_ = 0;
};

// The raw static spec of a pod: nodeSelector, required node affinity,
// tolerations, host ports (with their host IP).
template <class F>
void for_each_spec_word(const sr_cluster* c, const sr_pods& P, int32_t pod, F&& f) {
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
        // the strings' validity (labels.NewRequirement), not only their ids
        f(label_req_strings_ok(c, P.expr_key[e], P.expr_vals, P.expr_val_off[e], P.expr_val_off[e + 1]) ? 1 : 0);
        if (P.expr_op[e] == SR_OP_GT || P.expr_op[e] == SR_OP_LT)  // the values' integers, not only their ids
          for (int32_t v = P.expr_val_off[e]; v < P.expr_val_off[e + 1]; ++v) {
            int64_t x = 0;
            f(str_int(c, P.expr_vals[v], &x) ? 1 : 0);
            f(static_cast<int32_t>(static_cast<uint64_t>(x)));
            f(static_cast<int32_t>(static_cast<uint64_t>(x) >> 32));
          }
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
  for_each_port(c, pod, [&](int32_t proto, int32_t port, int32_t ip) {  // host ports and inline disks
    f(proto);
    f(port);
    f(ip);
  });
  if (has_volume_spec(c, pod)) {  // the volume filters' static part (attachable volumes: counts per key)
    const sr_volumes* V = c->volumes;
    f(-9);
    f(V->prefilter_fail[pod]);
    f(V->zone_off[pod + 1] - V->zone_off[pod]);
    for (int32_t z = V->zone_off[pod]; z < V->zone_off[pod + 1]; ++z) {
      f(V->zone_key[z]);
      f(V->zone_val_off[z + 1] - V->zone_val_off[z]);
      for (int32_t v = V->zone_val_off[z]; v < V->zone_val_off[z + 1]; ++v) f(V->zone_vals[v]);
    }
    for (int i = 0; i < 4; ++i) f(V->zone_keys[i]);
    f(V->pv_off[pod + 1] - V->pv_off[pod]);
    for (int32_t pv = V->pv_off[pod]; pv < V->pv_off[pod + 1]; ++pv) {
      f(V->pv_term_off[pv + 1] - V->pv_term_off[pv]);
      for (int32_t t = V->pv_term_off[pv]; t < V->pv_term_off[pv + 1]; ++t) {
        f(V->term_expr_off[t + 1] - V->term_expr_off[t]);
        for (int32_t e = V->term_expr_off[t]; e < V->term_expr_off[t + 1]; ++e) {
          f(V->expr_key[e]);
          f(V->expr_op[e]);
          f(V->expr_val_off[e + 1] - V->expr_val_off[e]);
          for (int32_t v = V->expr_val_off[e]; v < V->expr_val_off[e + 1]; ++v) f(V->expr_vals[v]);
          f(label_req_strings_ok(c, V->expr_key[e], V->expr_vals, V->expr_val_off[e], V->expr_val_off[e + 1]) ? 1 : 0);
          if (V->expr_op[e] == SR_OP_GT || V->expr_op[e] == SR_OP_LT)
            for (int32_t v = V->expr_val_off[e]; v < V->expr_val_off[e + 1]; ++v) {
              int64_t x = 0;
              f(str_int(c, V->expr_vals[v], &x) ? 1 : 0);
              f(static_cast<int32_t>(static_cast<uint64_t>(x)));
              f(static_cast<int32_t>(static_cast<uint64_t>(x) >> 32));
            }
        }
        f(V->term_field_off[t + 1] - V->term_field_off[t]);
        for (int32_t g = V->term_field_off[t]; g < V->term_field_off[t + 1]; ++g) {
          f(V->field_key[g]);
          f(V->field_op[g]);
          f(V->field_val_off[g + 1] - V->field_val_off[g]);
          for (int32_t v = V->field_val_off[g]; v < V->field_val_off[g + 1]; ++v) f(V->field_vals[v]);
        }
      }
    }
    std::vector<std::pair<int32_t, int32_t>> per_key;  // (key, count), the ids themselves are not static
    for (int32_t a = V->att_off[pod]; a < V->att_off[pod + 1]; ++a) {
      auto it = std::find_if(per_key.begin(), per_key.end(), [&](const auto& x) { return x.first == V->att_key[a]; });
      if (it == per_key.end()) per_key.emplace_back(V->att_key[a], 1);
      else ++it->second;
    }
    std::sort(per_key.begin(), per_key.end());
    f(static_cast<int32_t>(per_key.size()));
    for (const auto& kc : per_key) {
      f(kc.first);
      f(kc.second);
    }
  }
  if (has_spread(c, pod)) {  // topology spread constraints (with the pod's namespace and self-match)
    f(-8);
    std::vector<int32_t> w;
    spread_words(c, pod, w);
    for (int32_t x : w) f(x);
  }
  if (has_scalars(c, pod)) {  // scalar resources: (name, fit request)
    f(-7);
    for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; ++i) {
      f(c->pod_scalar_name[i]);
      f(static_cast<int32_t>(static_cast<uint64_t>(c->pod_scalar_req[i])));
      f(static_cast<int32_t>(static_cast<uint64_t>(c->pod_scalar_req[i]) >> 32));
    }
  }
}

bool has_static_spec(const sr_cluster* c, const sr_pods& P, int32_t pod) {
  return P.sel_off[pod] != P.sel_off[pod + 1] || P.tol_off[pod] != P.tol_off[pod + 1] ||
         P.port_off[pod] != P.port_off[pod + 1] || P.aff_required[pod] != 0 || has_scalars(c, pod) ||
         has_spread(c, pod) || has_ports(c, pod) || has_volume_spec(c, pod);
}

// Requirement word group {len, type, key, op, sorted unique values}.
void put_req(std::vector<int32_t>& out, int32_t type, int32_t key, int32_t op, const int32_t* v, int32_t nv) {
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
}

// A new spec's canonical form before its requirements are interned.
struct SpecDraft {
  int32_t flags = 0;
  std::vector<int32_t> sel;    // nodeSelector requirement groups
  std::vector<int32_t> terms;  // per buildable term: {n groups, groups...}
  int32_t n_terms = 0;
  std::vector<int32_t> tol, ports;
  std::vector<int64_t> scalars;  // {name, fit request}*, sorted by name
  std::vector<int32_t> spread;   // spread_words
  // volume filters: requirement groups ANDed (VolumeZone, single-term PV node
  // affinity) and the PV selectors with several terms ({n terms, per term
  // {n groups, groups...}} each)
  std::vector<int32_t> vsel;
  std::vector<std::vector<int32_t>> vpv;
};

// Drafts one NodeSelectorTerm (MatchNodeSelectorTerms [upstream core/v1/helper]:
// NodeSelectorRequirementsAsSelector over the expressions, As-FieldSelector
// over the fields) into requirement groups; false when it fails to build
// (it matches nothing).  `no_fields`: the PV form (volumeutil.CheckNodeAffinity
// passes no fields, so a field requirement reads "" and is decided here).
bool draft_term(const sr_cluster* c, const int32_t* expr_key, const int32_t* expr_op, const int32_t* expr_val_off,
                const int32_t* expr_vals, int32_t e0, int32_t e1, const int32_t* field_key, const int32_t* field_op,
                const int32_t* field_val_off, const int32_t* field_vals, int32_t f0, int32_t f1, bool no_fields,
                std::vector<int32_t>& term, int32_t* n_groups) {
  bool valid = true;
  term.clear();
  int32_t n = 0;
  for (int32_t e = e0; e < e1 && valid; ++e) {
    const int32_t nv = expr_val_off[e + 1] - expr_val_off[e];
    const int32_t op = expr_op[e];
    if (expr_key[e] == c->id_empty) valid = false;  // validateLabelKey("") fails
    // validateLabelKey / validateLabelValue on every value (every operator)
    else if (!label_req_strings_ok(c, expr_key[e], expr_vals, expr_val_off[e], expr_val_off[e + 1]))
      valid = false;
    else if ((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 0) valid = false;
    else if ((op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) && nv != 0) valid = false;
    else if (op == SR_OP_GT || op == SR_OP_LT) {  // exactly one value, an integer (labels.NewRequirement)
      int64_t x;
      valid = nv == 1 && str_int(c, expr_vals[expr_val_off[e]], &x);
    } else if (op != SR_OP_IN && op != SR_OP_NOT_IN && op != SR_OP_EXISTS && op != SR_OP_DOES_NOT_EXIST) {
      valid = false;
    }
    if (valid && (op == SR_OP_GT || op == SR_OP_LT)) {  // {value id, its integer (lo, hi)}
      int64_t x = 0;
      str_int(c, expr_vals[expr_val_off[e]], &x);
      const int32_t w[3] = {expr_vals[expr_val_off[e]], static_cast<int32_t>(static_cast<uint64_t>(x)),
                            static_cast<int32_t>(static_cast<uint64_t>(x) >> 32)};
      term.insert(term.end(), {6, REQ_LABEL_EXPR, expr_key[e], op, w[0], w[1], w[2]});
      ++n;
    } else if (valid) {
      put_req(term, REQ_LABEL_EXPR, expr_key[e], op, expr_vals + expr_val_off[e], nv);
      ++n;
    }
  }
  for (int32_t f = f0; f < f1 && valid; ++f) {  // NodeSelectorRequirementsAsFieldSelector
    const int32_t nv = field_val_off[f + 1] - field_val_off[f];
    const int32_t op = field_op[f];
    valid = (op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 1;
    if (valid && no_fields) {  // fields.Set(nil): every key reads ""
      const bool eq = field_vals[field_val_off[f]] == c->id_empty && c->id_empty != -1;
      valid = op == SR_OP_IN ? eq : !eq;
    } else if (valid) {
      put_req(term, REQ_FIELD, field_key[f], op, &field_vals[field_val_off[f]], 1);
      ++n;
    }
  }
  *n_groups = n;
  return valid;
}

void draft_spec(const sr_cluster* c, int32_t pod, SpecDraft* d) {
  const sr_pods& P = c->pods;
  // Spec.NodeSelector: labels.SelectorFromSet -> Equals requirements.
  for (int32_t i = P.sel_off[pod]; i < P.sel_off[pod + 1]; ++i)
    put_req(d->sel, REQ_LABEL_EQ, P.sel_key[i], SR_OP_IN, &P.sel_val[i], 1);
  // Required node affinity: MatchNodeSelectorTerms [upstream core/v1/helper].
  if (P.aff_required[pod]) {
    d->flags |= CLS_AFF_REQUIRED;
    std::vector<int32_t> term;
    for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t) {
      const int32_t e0 = P.term_expr_off[t], e1 = P.term_expr_off[t + 1];
      const int32_t f0 = P.term_field_off[t], f1 = P.term_field_off[t + 1];
      if (e0 == e1 && f0 == f1) continue;  // an empty term selects nothing
      int32_t n = 0;
      if (!draft_term(c, P.expr_key, P.expr_op, P.expr_val_off, P.expr_vals, e0, e1, P.field_key, P.field_op,
                      P.field_val_off, P.field_vals, f0, f1, false, term, &n))
        continue;  // a term that fails to build matches nothing
      d->terms.push_back(n);
      d->terms.insert(d->terms.end(), term.begin(), term.end());
      ++d->n_terms;
    }
    if (d->n_terms == 0) d->flags |= CLS_IMPOSSIBLE;
  }
  for (int32_t i = P.tol_off[pod]; i < P.tol_off[pod + 1]; ++i) {
    d->tol.push_back(P.tol_key[i]);
    d->tol.push_back(P.tol_op[i]);
    d->tol.push_back(P.tol_val[i]);
    d->tol.push_back(P.tol_effect[i]);
  }
  // HostPortInfo ignores port <= 0; inline disks as pseudo ports (VolumeRestrictions)
  for_each_port(c, pod, [&](int32_t proto, int32_t port, int32_t ip) {
    d->ports.push_back(proto);
    d->ports.push_back(port);
    d->ports.push_back(ip);
  });
  if (has_spread(c, pod)) spread_words(c, pod, d->spread);
  std::vector<std::pair<int64_t, int64_t>> sc;
  if (has_volume_spec(c, pod)) {
    const sr_volumes* V = c->volumes;
    // VolumeBinding PreFilter failing: the pod fits no node
    if (V->prefilter_fail[pod]) d->flags |= CLS_IMPOSSIBLE;
    // VolumeZone: each PV zone / region label a REQ_ZONE requirement
    for (int32_t z = V->zone_off[pod]; z < V->zone_off[pod + 1]; ++z) {
      std::vector<int32_t> vals(V->zone_vals + V->zone_val_off[z], V->zone_vals + V->zone_val_off[z + 1]);
      std::sort(vals.begin(), vals.end());
      vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
      d->vsel.push_back(static_cast<int32_t>(7 + vals.size()));
      d->vsel.insert(d->vsel.end(), {REQ_ZONE, V->zone_key[z], SR_OP_IN, V->zone_keys[0], V->zone_keys[1],
                                     V->zone_keys[2], V->zone_keys[3]});
      d->vsel.insert(d->vsel.end(), vals.begin(), vals.end());
    }
    // VolumeBinding Filter: every bound PV's Required node affinity (terms ORed)
    std::vector<int32_t> term, sel;
    for (int32_t pv = V->pv_off[pod]; pv < V->pv_off[pod + 1]; ++pv) {
      sel.assign(1, 0);
      int32_t n_terms = 0, one = -1;
      for (int32_t t = V->pv_term_off[pv]; t < V->pv_term_off[pv + 1]; ++t) {
        const int32_t e0 = V->term_expr_off[t], e1 = V->term_expr_off[t + 1];
        const int32_t f0 = V->term_field_off[t], f1 = V->term_field_off[t + 1];
        if (e0 == e1 && f0 == f1) continue;  // an empty term selects nothing
        int32_t n = 0;
        if (!draft_term(c, V->expr_key, V->expr_op, V->expr_val_off, V->expr_vals, e0, e1, V->field_key,
                        V->field_op, V->field_val_off, V->field_vals, f0, f1, true, term, &n))
          continue;
        if (n_terms == 0) one = static_cast<int32_t>(sel.size());
        sel.push_back(n);
        sel.insert(sel.end(), term.begin(), term.end());
        ++n_terms;
      }
      sel[0] = n_terms;
      if (n_terms == 0) {
        d->flags |= CLS_IMPOSSIBLE;  // no term can match
      } else if (n_terms == 1) {  // its requirements ANDed with the others
        d->vsel.insert(d->vsel.end(), sel.begin() + one + 1, sel.end());
        if (sel[one] == 0) continue;  // a term of decided fields only: every node
      } else {
        d->vpv.push_back(sel);
      }
    }
    // volume limits: attachable volumes per limit key ride the scalar
    // machinery (alloc = the node's limit, requested = its unique attachable
    // volumes of the key), one (key, count) check each
    for (int32_t a = V->att_off[pod]; a < V->att_off[pod + 1]; ++a) {
      const int64_t name = vol_name(V->att_key[a]);
      auto it = std::find_if(sc.begin(), sc.end(), [&](const auto& x) { return x.first == name; });
      if (it == sc.end()) sc.emplace_back(name, 1);
      else ++it->second;
    }
  }
  if (has_scalars(c, pod) || !sc.empty()) {  // fitsRequest's ScalarResources loop: one (name, request) check each
    if (has_scalars(c, pod))
      for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; ++i)
        sc.emplace_back(c->pod_scalar_name[i], c->pod_scalar_req[i]);
    std::sort(sc.begin(), sc.end());
    for (const auto& x : sc) {
      d->scalars.push_back(x.first);
      d->scalars.push_back(x.second);
    }
  }
}

// Interns a draft's requirement groups; returns the sorted unique ids.
void intern_groups(WordDict& dict, const int32_t* g, int32_t n_groups, std::vector<int32_t>& ids, size_t* used) {
  ids.clear();
  size_t i = 0;
  for (int32_t k = 0; k < n_groups; ++k) {
    ids.push_back(dict.intern(g + i + 1, static_cast<size_t>(g[i])));
    i += 1 + static_cast<size_t>(g[i]);
  }
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  if (used) *used = i;
}

// Moves the bits at the positions perm_k of a [Wp] row to where their nodes went.
void permute_row(const EncoderCache& C, uint64_t* row, std::vector<uint8_t>& tmp) {
  const std::vector<int32_t>& k = C.perm_k;
  tmp.resize(k.size());
  for (size_t q = 0; q < k.size(); ++q) {
    const int32_t o = C.perm_src[k[q]];
    tmp[q] = static_cast<uint8_t>(row[o >> 6] >> (o & 63) & 1);
  }
  for (size_t q = 0; q < k.size(); ++q) {
    const int32_t i = k[q];
    const uint64_t bit = 1ull << (i & 63);
    row[i >> 6] = tmp[q] ? (row[i >> 6] | bit) : (row[i >> 6] & ~bit);
  }
}

// The spot pool holds the same nodes as the cached view (names and static
// fingerprints), some at other positions: permute the position-indexed static
// data (label columns, taint and requirement rows) instead of rebuilding it.
// The moved positions count as changed nodes for the state view.
bool permute_static(EncoderCache& C, const sr_snapshot* snap) {
  const int32_t n = C.n_spot;
  int32_t max_name = -1;
  for (int32_t i = 0; i < n; ++i) {
    if (C.names[i] < 0 || snap->node_names[i] < 0) return false;
    max_name = std::max(max_name, std::max(C.names[i], snap->node_names[i]));
  }
  std::vector<int32_t>& pos = C.pos_scratch;
  if (pos.size() < static_cast<size_t>(max_name) + 1) pos.resize(static_cast<size_t>(max_name) + 1, -1);
  for (int32_t i = 0; i < n; ++i) pos[C.names[i]] = i;
  C.perm_src.assign(static_cast<size_t>(n), -1);
  bool ok = true;
  for (int32_t i = 0; i < n && ok; ++i) {
    const int32_t nm = snap->node_names[i], o = pos[nm];
    ok = o >= 0 && C.static_fp[o] == snap->node_sfp[i];
    C.perm_src[i] = o;
    pos[nm] = -1;  // claimed: a repeated name fails
  }
  for (int32_t i = 0; i < n; ++i) pos[C.names[i]] = -1;
  if (!ok) return false;
  C.perm_k.clear();
  for (int32_t i = 0; i < n; ++i)
    if (C.perm_src[i] != i) C.perm_k.push_back(i);
  C.perm_to = permute_targets(n, C.perm_src, C.perm_k);
  std::vector<int32_t> vals(C.perm_k.size());
  for (auto& kc : C.label_col) {
    std::vector<int32_t>& col = kc.second;
    for (size_t q = 0; q < C.perm_k.size(); ++q) vals[q] = col[C.perm_src[C.perm_k[q]]];
    for (size_t q = 0; q < C.perm_k.size(); ++q) col[C.perm_k[q]] = vals[q];
  }
  std::vector<uint8_t> tmp;
  for (size_t t = 0; t < C.taints.size(); ++t) permute_row(C, &C.taint_rows[t * static_cast<size_t>(C.Wp)], tmp);
  for (size_t r = 0; r < C.req_rows.size(); ++r)
    if (C.req_row_gen[r] == C.static_gen) permute_row(C, C.req_rows[r].data(), tmp);
  C.names = snap->node_names;
  C.static_fp = snap->node_sfp;
  C.perm_dirty.insert(C.perm_dirty.end(), C.perm_k.begin(), C.perm_k.end());
  ++C.layout_gen;
  return true;
}

// ---- static view: names, labels, taints of the spot pool in NodeInfoArray order
void refresh_static(EncoderCache& C, const sr_snapshot* snap, int32_t Wp) {
  const int32_t n = static_cast<int32_t>(snap->nodes.size());
  bool same = C.n_spot == n && C.Wp == Wp;
  same = same && std::equal(C.names.begin(), C.names.end(), snap->node_names.begin()) &&
         std::equal(C.static_fp.begin(), C.static_fp.end(), snap->node_sfp.begin());
  C.last_static_changed = same ? 0 : 1;
  if (same) return;
  if (C.n_spot == n && C.Wp == Wp && n > 0 && permute_static(C, snap)) {
    C.last_static_changed = 2;
    return;
  }
  C.perm_dirty.clear();
  ++C.layout_gen;
  ++C.static_gen;
  C.n_spot = n;
  C.Wp = Wp;
  C.n_pad = Wp * 64;
  C.names = snap->node_names;
  C.static_fp = snap->node_sfp;
  C.label_col.clear();
  // taints: NoSchedule / NoExecute only (TaintToleration.Filter); the
  // unschedulable flag is the pseudo-taint node.kubernetes.io/unschedulable:NoSchedule
  WordDict taint_dict;
  C.taints.clear();
  std::vector<std::pair<int32_t, int32_t>> hits;  // (taint, node)
  auto add = [&](const TaintRec& t, int32_t node) {
    const int32_t k[3] = {t.key, t.val, t.effect};
    bool ins = false;
    const int32_t id = taint_dict.intern(k, 3, &ins);
    if (ins) C.taints.push_back(t);
    hits.emplace_back(id, node);
  };
  for (int32_t i = 0; i < n; ++i) {
    const SpotNode& sn = snap->nodes[i];
    for (const TaintRec& t : sn.taints)
      if (t.effect == SR_EFFECT_NO_SCHEDULE || t.effect == SR_EFFECT_NO_EXECUTE) add(t, i);
    if (sn.unschedulable) add(TaintRec{snap->id_unschedulable_key, snap->id_empty, SR_EFFECT_NO_SCHEDULE}, i);
  }
  C.taint_rows.assign(C.taints.size() * static_cast<size_t>(Wp), 0);
  for (const auto& h : hits)
    C.taint_rows[static_cast<size_t>(h.first) * Wp + (h.second >> 6)] |= 1ull << (h.second & 63);
  C.state_valid = false;  // positions may have moved: the state view is rebuilt too
}

// ---- state view: capacity records, free values (sorted), pod-count atom
sr_status refresh_state(EncoderCache& C, const sr_snapshot* snap, std::string* err) {
  const int32_t n = C.n_spot, NP = C.n_pad, Wp = C.Wp;
  const std::vector<uint64_t>& fp = snap->node_dfp;  // kept current by the snapshot
  std::vector<int32_t> changed, moved;
  const bool full = !C.state_valid || C.state_fp.size() != static_cast<size_t>(n);
  if (!full && !C.perm_dirty.empty()) {
    // the spot order moved (permute_static): each moved node's records and
    // fingerprint follow it to its new position (the multiset of free values
    // is unchanged); only nodes whose own state changed are patched below,
    // but every moved position is a changed record for the device
    moved = C.perm_dirty;
    const std::vector<int32_t>& K = C.perm_k;
    std::vector<uint64_t> rec(K.size() * 8), sfp(K.size());
    std::vector<int64_t> fr(K.size() * 3);
    std::vector<uint8_t> pc(K.size());
    for (size_t q = 0; q < K.size(); ++q) {
      const int32_t o = C.perm_src[K[q]];
      std::copy_n(&C.node_rec[static_cast<size_t>(o) * 8], 8, &rec[q * 8]);
      for (int d = 0; d < 3; ++d) fr[q * 3 + d] = C.node_free[static_cast<size_t>(d) * NP + o];
      pc[q] = static_cast<uint8_t>(C.podcount_row[static_cast<size_t>(o >> 6)] >> (o & 63) & 1);
      sfp[q] = C.state_fp[o];
    }
    for (size_t q = 0; q < K.size(); ++q) {
      const int32_t i = K[q];
      std::copy_n(&rec[q * 8], 8, &C.node_rec[static_cast<size_t>(i) * 8]);
      for (int d = 0; d < 3; ++d) C.node_free[static_cast<size_t>(d) * NP + i] = fr[q * 3 + d];
      uint64_t& word = C.podcount_row[static_cast<size_t>(i >> 6)];
      const uint64_t bit = 1ull << (i & 63);
      word = pc[q] ? (word | bit) : (word & ~bit);
      C.state_fp[i] = sfp[q];
    }
  }
  C.perm_dirty.clear();
  if (!full)
    for (int32_t i = 0; i < n; ++i)
      if (fp[i] != C.state_fp[i]) changed.push_back(i);
  C.last_state_changed = full ? n : static_cast<int32_t>(changed.size() + moved.size());
  if (!full && changed.empty() && moved.empty()) return SR_OK;
  C.patched_from = ~0ull;
  C.patched_nodes.clear();
  ++C.state_gen;
  // the nodes whose own state changed (a moved node's follows it): the
  // reuse's inter-pod and spread states are permuted, then patched only there
  C.content_from = full ? ~0ull : C.state_gen - 1;
  C.content_nodes = changed;
  auto node_values = [&](int32_t i, int64_t out[3], int64_t* left) -> bool {
    const SpotNode& sn = snap->nodes[i];
    const NodeState& st = snap->state[i];
    for (int r = 0; r < 3; ++r) {
      if (!in_range(sn.alloc[r]) || !in_range(st.requested[r])) return false;
      out[r] = sn.alloc[r] - st.requested[r];
    }
    *left = sn.alloc_pods - st.npods;
    return true;
  };
  auto write_node = [&](int32_t i, const int64_t f[3], int64_t left) {
    uint64_t* r = &C.node_rec[static_cast<size_t>(i) * 8];
    for (int d = 0; d < 3; ++d) {
      r[d] = static_cast<uint64_t>(f[d]);
      C.node_free[static_cast<size_t>(d) * NP + i] = f[d];
    }
    r[3] = 0;  // state bits: the base UsedPorts are static conflicts (F rows)
    const int32_t pl = static_cast<int32_t>(std::max<int64_t>(-(1 << 30), std::min<int64_t>(left, 1 << 30)));
    r[4] = static_cast<uint64_t>(static_cast<int64_t>(pl));
    uint64_t& word = C.podcount_row[static_cast<size_t>(i >> 6)];
    const uint64_t bit = 1ull << (i & 63);
    word = left >= 1 ? (word | bit) : (word & ~bit);
  };
  auto fail = [&]() {
    C.state_valid = false;
    *err = "spot node quantity outside [0, 2^62)";
    return SR_ERR_CAPACITY;
  };
  if (full || changed.size() * 8 > static_cast<size_t>(n)) {
    C.node_rec.assign(static_cast<size_t>(NP) * 8, 0);
    C.node_free.assign(static_cast<size_t>(3) * NP, INT64_MIN);  // pads never pass a threshold
    C.podcount_row.assign(static_cast<size_t>(Wp), 0);
    for (int d = 0; d < 3; ++d) C.sorted_free[d].resize(static_cast<size_t>(n));
    for (int32_t i = 0; i < n; ++i) {
      int64_t f[3], left;
      if (!node_values(i, f, &left)) return fail();
      write_node(i, f, left);
      for (int d = 0; d < 3; ++d) C.sorted_free[d][i] = f[d];
    }
    for (int d = 0; d < 3; ++d) std::sort(C.sorted_free[d].begin(), C.sorted_free[d].end());
  } else {  // a few nodes changed: patch their records and the sorted values
    C.patched_from = C.state_gen - 1;
    C.patched_nodes = changed;
    if (!moved.empty()) {  // and the moved records
      C.patched_nodes.insert(C.patched_nodes.end(), moved.begin(), moved.end());
      std::sort(C.patched_nodes.begin(), C.patched_nodes.end());
      C.patched_nodes.erase(std::unique(C.patched_nodes.begin(), C.patched_nodes.end()), C.patched_nodes.end());
    }
    for (int32_t i : changed) {
      int64_t f[3], left;
      if (!node_values(i, f, &left)) return fail();
      for (int d = 0; d < 3; ++d) {  // the sorted values with multiplicity, and the distinct ones
        std::vector<int64_t>& s = C.sorted_free[d];
        std::vector<int64_t>& v = C.node_vals[d];
        const int64_t old = C.node_free[static_cast<size_t>(d) * NP + i], nv = f[d];
        if (old == nv) continue;
        // old leaves the distinct values when it was its only copy; nv enters them when absent
        const bool old_goes = std::upper_bound(s.begin(), s.end(), old) - std::lower_bound(s.begin(), s.end(), old) == 1;
        const bool nv_comes = !std::binary_search(s.begin(), s.end(), nv);
        // one value replaced by another in a sorted array: only the span between
        // their places moves (a node's free value usually moves a little)
        auto replace_sorted = [](std::vector<int64_t>& a, int64_t from, int64_t to) {
          const auto at = std::lower_bound(a.begin(), a.end(), from);
          if (to > from) {
            const auto ub = std::upper_bound(at + 1, a.end(), to);
            std::move(at + 1, ub, at);
            *(ub - 1) = to;
          } else {
            const auto ub = std::upper_bound(a.begin(), at, to);
            std::move_backward(ub, at, at + 1);
            *ub = to;
          }
        };
        replace_sorted(s, old, nv);
        if (old_goes && nv_comes) replace_sorted(v, old, nv);
        else if (old_goes) v.erase(std::lower_bound(v.begin(), v.end(), old));
        else if (nv_comes) v.insert(std::lower_bound(v.begin(), v.end(), nv), nv);
      }
      write_node(i, f, left);
    }
  }
  if (full || changed.size() * 8 > static_cast<size_t>(n))
    for (int d = 0; d < 3; ++d) {
      C.node_vals[d].assign(C.sorted_free[d].begin(), C.sorted_free[d].end());
      C.node_vals[d].erase(std::unique(C.node_vals[d].begin(), C.node_vals[d].end()), C.node_vals[d].end());
    }
  C.state_fp = fp;
  C.state_valid = true;
  return SR_OK;
}

// Label value column of `key` over the static view (built on first use).
const std::vector<int32_t>& label_column(EncoderCache& C, const sr_snapshot* snap, int32_t key) {
  for (const auto& kc : C.label_col)
    if (kc.first == key) return kc.second;
  std::vector<int32_t> col(static_cast<size_t>(C.n_spot), INT32_MIN);
  for (int32_t n = 0; n < C.n_spot; ++n)
    for (const auto& kv : snap->nodes[n].labels)
      if (kv.first == key) {
        col[n] = kv.second;
        break;
      }
  C.label_col.emplace_back(key, std::move(col));
  return C.label_col.back().second;
}

// Node row of requirement `rw` = {type, key, op, vals...} over the static view:
// Requirement.Matches on the node's labels, or the metadata.name field.
void build_req_row(const EncoderCache& C, const sr_snapshot* snap, const sr_cluster* c, const int32_t* rw,
                   size_t len, const std::vector<int32_t>* col, std::vector<uint64_t>& row,
                   const std::vector<int32_t>* const* zcols = nullptr) {
  const int32_t type = rw[0], key = rw[1], op = rw[2];
  const int32_t* vals = rw + 3;
  const size_t nv = len - 3;
  row.assign(static_cast<size_t>(C.Wp), 0);
  auto set = [&](int32_t n) { row[static_cast<size_t>(n >> 6)] |= 1ull << (n & 63); };
  if (type == REQ_ZONE) {
    // VolumeZone.Filter [upstream k8s v1.19.2 plugins/volumezone]: a node
    // without any of the four zone / region labels passes; otherwise its value
    // of the PV label's key ("" when absent: never in a LabelZonesToSet set)
    // must be one of the PV's values
    const int32_t* zv = rw + 7;
    const size_t nz = len - 7;
    for (int32_t n = 0; n < C.n_spot; ++n) {
      bool any = false;
      for (int z = 0; z < 4; ++z) any = any || (zcols && zcols[z] && (*zcols[z])[n] != INT32_MIN);
      const int32_t v = (*col)[n];
      if (!any || (v != INT32_MIN && std::binary_search(zv, zv + nz, v))) set(n);
    }
    return;
  }
  if (type == REQ_FIELD) {
    // fields.Set{"metadata.name": node.Name}; any other key reads as "".
    const bool is_name = key == C.id_metadata_name && C.id_metadata_name != -1;
    for (int32_t n = 0; n < C.n_spot; ++n) {
      const int32_t fv = is_name ? snap->nodes[n].name : C.id_empty;
      const bool eq = fv == vals[0];
      if (op == SR_OP_IN ? eq : !eq) set(n);
    }
    return;
  }
  // Gt / Lt: {value id, its integer (lo, hi)}, validated when the spec was drafted
  const int64_t bound = (op == SR_OP_GT || op == SR_OP_LT) && nv == 3
                            ? static_cast<int64_t>(static_cast<uint64_t>(static_cast<uint32_t>(vals[1])) |
                                                   static_cast<uint64_t>(static_cast<uint32_t>(vals[2])) << 32)
                            : 0;
  for (int32_t n = 0; n < C.n_spot; ++n) {
    const int32_t v = (*col)[n];
    const bool has = v != INT32_MIN;
    bool m;
    int64_t x;
    switch (op) {
      case SR_OP_IN: m = has && std::binary_search(vals, vals + nv, v); break;
      case SR_OP_NOT_IN: m = !has || !std::binary_search(vals, vals + nv, v); break;
      case SR_OP_EXISTS: m = has; break;
      case SR_OP_GT: m = has && str_int(c, v, &x) && x > bound; break;  // a label that does not parse: false
      case SR_OP_LT: m = has && str_int(c, v, &x) && x < bound; break;
      default: m = !has; break;  // DoesNotExist
    }
    if (m) set(n);
  }
}

// The NodeAffinity row of a pod (nodeSelector AND, OR of the required
// terms), from its drafted spec's requirements over the static view.
void pod_affinity_row(EncoderCache& C, const sr_snapshot* snap, const sr_cluster* c, int32_t pod,
                      std::vector<uint64_t>& out) {
  SpecDraft d;
  draft_spec(c, pod, &d);
  const int32_t Wp = C.Wp, n_spot = C.n_spot;
  out.assign(static_cast<size_t>(Wp), 0);
  if (d.flags & CLS_IMPOSSIBLE) return;
  for (int32_t n = 0; n < n_spot; ++n) out[n >> 6] |= 1ull << (n & 63);
  std::vector<uint64_t> r;
  auto group_row = [&](const int32_t* g) {  // {len, type, key, op, vals...}
    const int32_t* rw = g + 1;
    build_req_row(C, snap, c, rw, static_cast<size_t>(g[0]), rw[0] != REQ_FIELD ? &label_column(C, snap, rw[1]) : nullptr,
                  r);
  };
  for (size_t i = 0; i < d.sel.size(); i += 1 + static_cast<size_t>(d.sel[i])) {
    group_row(&d.sel[i]);
    for (int32_t x = 0; x < Wp; ++x) out[x] &= r[x];
  }
  if (!(d.flags & CLS_AFF_REQUIRED)) return;
  std::vector<uint64_t> any(static_cast<size_t>(Wp), 0), t(static_cast<size_t>(Wp));
  for (size_t i = 0; i < d.terms.size();) {
    const int32_t ng = d.terms[i++];
    std::fill(t.begin(), t.end(), ~0ull);
    for (int32_t q = 0; q < ng; ++q) {
      group_row(&d.terms[i]);
      for (int32_t x = 0; x < Wp; ++x) t[x] &= r[x];
      i += 1 + static_cast<size_t>(d.terms[i]);
    }
    for (int32_t x = 0; x < Wp; ++x) any[x] |= t[x];
  }
  for (int32_t x = 0; x < Wp; ++x) out[x] &= any[x];
}

// Topology spread between the pods of one candidate (SpreadDyn, DESIGN.md
// §2.9): a pod whose DoNotSchedule constraint counts earlier pods of its
// candidate (its namespace, not terminating, selected) sends the candidate to
// the domain path, or to the reference path beyond its limits -- more than
// kDynPods pods, more than kSpreadSlots such constraints in a pod, another
// constraint of the pod on the same key, a key without a domain slot, or a
// node-local key whose minimum could move (no more nodes at the minimum than
// the constraint counts pods of the candidate).
void analyse_spread(EncoderCache& C, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                    std::vector<int32_t>& status, DomKeys* dk, SpreadDyn* out, SpreadIndex& six, SpreadReuse* keep) {
  SpreadDyn& sd = *out;
  sd = SpreadDyn{};
  const sr_spread* S = c->spread;
  const sr_pod_affinity* A = c->pod_affinity;
  const int32_t nc = cands->n_cand;
  if (!S || !A || nc == 0) return;
  const int32_t base = cands->cand_pod_off[0];
  sd.base = base;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  auto counted = [&](int32_t k, int32_t pod, int32_t q) {  // earlier pod q counted by pod's constraint k
    return !S->terminating[q] && A->ns[q] == A->ns[pod] && spread_selects(c, k, q);
  };
  std::vector<uint64_t> aff, words;
  // replicas share their NodeAffinity and their constraints' counts: both are
  // computed once per distinct content (the nodeSelector / affinity words; the
  // namespace and selector)
  std::map<std::vector<int32_t>, std::vector<uint64_t>> aff_rows;
  std::map<std::vector<int32_t>, std::vector<int32_t>> counts;  // spread_selector_words -> node counts
  std::vector<int32_t> key_words;
  struct PendingSlot {  // a table entry for the reuse state (SpreadReuse), once the candidate is planned
    std::vector<int32_t> sel;
    uint32_t off;
    bool local;
    std::vector<uint64_t> pairs;
    int32_t skew, self, n_counted, slot;
    uint64_t pm;
    int32_t edom;
  };
  std::vector<PendingSlot> pend;
  for (int32_t i = 0; i < nc; ++i) {
    if (status[i] != STATUS_PENDING) continue;
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    bool any = false;
    for (int32_t u = b + 1; u < e && !any; ++u) {
      const int32_t pod = cands->cand_pods[u];
      for (int32_t k = S->off[pod]; k < S->off[pod + 1] && !any; ++k)
        for (int32_t t = b; t < u && !any; ++t) any = counted(k, pod, cands->cand_pods[t]);
    }
    if (!any) continue;
    bool fb = e - b > kDynPods;
    pend.clear();
    words.assign(static_cast<size_t>(e - b) * kSpreadU64, 0);
    std::vector<uint8_t> dm(static_cast<size_t>(e - b), 0);
    const size_t tab0 = sd.tab.size();
    for (int32_t u = b; u < e && !fb; ++u) {
      const int32_t pod = cands->cand_pods[u];
      uint64_t* rec = &words[static_cast<size_t>(u - b) * kSpreadU64];
      for (int s2 = 0; s2 < kSpreadSlots; ++s2) rec[s2 * (kDynG + 3) + kDynG] = ~0ull;  // slot unused
      if (S->off[pod + 1] == S->off[pod]) continue;
      // the pairs: nodes passing the pod's NodeAffinity and carrying every key
      bool affd = false;
      int32_t slots = 0;
      for (int32_t k = S->off[pod]; k < S->off[pod + 1] && !fb; ++k) {
        uint64_t mk[kDynG] = {0, 0, 0, 0};
        int32_t n_counted = 0;
        for (int32_t t = b; t < u; ++t)
          if (counted(k, pod, cands->cand_pods[t])) {
            mk[(t - b) >> 6] |= 1ull << ((t - b) & 63);
            ++n_counted;
          }
        if (n_counted == 0) continue;
        if (!affd) {
          key_words.clear();
          for_each_spec_word(c, c->pods, pod, [&](int32_t x) { key_words.push_back(x); });
          auto it = aff_rows.find(key_words);
          if (it == aff_rows.end()) {
            pod_affinity_row(C, snap, c, pod, aff);
            it = aff_rows.emplace(key_words, aff).first;
          }
          aff = it->second;
          for (int32_t k2 = S->off[pod]; k2 < S->off[pod + 1]; ++k2) {
            const std::vector<int32_t>& col = label_column(C, snap, S->topology_key[k2]);
            for (int32_t n = 0; n < n_spot; ++n)
              if (col[n] == INT32_MIN) aff[n >> 6] &= ~(1ull << (n & 63));
          }
          affd = true;
        }
        bool pairs = false;
        for (uint64_t x : aff) pairs = pairs || x != 0;
        if (!pairs) break;  // no pair at all: the filter passes every node (the static row says so)
        const int32_t key = S->topology_key[k];
        for (int32_t k2 = S->off[pod]; k2 < S->off[pod + 1]; ++k2)
          fb = fb || (k2 != k && S->topology_key[k2] == key);  // shared pair counts: not on the device
        if (fb || slots == kSpreadSlots) {
          fb = true;
          break;
        }
        const int32_t slot = dk->slot(snap, key);
        if (slot < 0) {
          fb = true;
          break;
        }
        const int32_t self = spread_selects(c, k, pod) ? 1 : 0, skew = S->max_skew[k];
        spread_selector_words(c, A->ns[pod], k, key_words);
        auto ci = counts.find(key_words);
        if (ci == counts.end()) {
          std::vector<int32_t> v;
          spread_node_counts(six, c, k, A->ns[pod], v);
          ci = counts.emplace(key_words, std::move(v)).first;
        }
        const std::vector<int32_t>& cnt = ci->second;
        const std::vector<int32_t>& dom = dk->dom[slot];
        uint64_t* sw = rec + slots * (kDynG + 3);
        for (int g = 0; g < kDynG; ++g) sw[g] = mk[g];
        const uint32_t off = static_cast<uint32_t>(sd.tab.size());
        if (dk->node_local[slot]) {
          // the minimum over the pairs and how many nodes hold it
          int64_t m0 = INT64_MAX, n0 = 0;
          for (int32_t n = 0; n < n_spot; ++n) {
            if (!((aff[n >> 6] >> (n & 63)) & 1)) continue;
            if (cnt[n] < m0) {
              m0 = cnt[n];
              n0 = 0;
            }
            n0 += cnt[n] == m0 ? 1 : 0;
          }
          if (n0 <= n_counted) {
            fb = true;
            sd.state_fb = true;  // decided by the base counts
            break;
          }
          for (int32_t n = 0; n < n_spot; ++n) {
            const bool in = (aff[n >> 6] >> (n & 63)) & 1;
            sd.tab.push_back(in ? static_cast<int32_t>(std::max<int64_t>(INT32_MIN, std::min<int64_t>(
                                      INT32_MAX - 1, static_cast<int64_t>(skew) - self + m0 - cnt[n])))
                                : INT32_MAX);
          }
          sw[kDynG] = static_cast<uint64_t>(slot) | 1ull << 2 | static_cast<uint64_t>(self) << 3 |
                      static_cast<uint64_t>(static_cast<uint32_t>(skew)) << 32;
          sw[kDynG + 1] = off;
          sw[kDynG + 2] = 0;
          if (keep) pend.push_back(PendingSlot{key_words, off, true, aff, skew, self, n_counted, slot, 0, -1});
        } else {
          // pairs by domain; a node lacking the key counts into the pair of ""
          int32_t edom = -1;
          for (int32_t n = 0; n < n_spot && edom < 0; ++n) {
            int32_t v = INT32_MIN;
            for (const auto& kv : snap->nodes[n].labels)
              if (kv.first == key) v = kv.second;
            if (v == snap->id_empty && v != INT32_MIN) edom = dom[n];
          }
          uint64_t pm = 0;
          for (int32_t n = 0; n < n_spot; ++n)
            if (((aff[n >> 6] >> (n & 63)) & 1) && dom[n] >= 0) pm |= 1ull << dom[n];
          int64_t bc[kDomMax] = {0};
          for (int32_t n = 0; n < n_spot; ++n) {
            const int32_t d = dom[n] >= 0 ? dom[n] : edom;
            if (d >= 0 && ((pm >> d) & 1)) bc[d] += cnt[n];
          }
          for (int32_t d = 0; d < kDomMax; ++d)
            sd.tab.push_back(static_cast<int32_t>(std::min<int64_t>(bc[d], INT32_MAX / 4)));
          sw[kDynG] = static_cast<uint64_t>(slot) | static_cast<uint64_t>(self) << 3 |
                      static_cast<uint64_t>(static_cast<uint32_t>(skew)) << 32;
          sw[kDynG + 1] = off | static_cast<uint64_t>(static_cast<uint32_t>(edom)) << 32;
          sw[kDynG + 2] = pm;
          if (keep) pend.push_back(PendingSlot{key_words, off, false, {}, skew, self, n_counted, slot, pm, edom});
          dm[u - b] |= static_cast<uint8_t>(1u << (k - S->off[pod]));
        }
        ++slots;
      }
    }
    if (fb) {
      status[i] = SR_CAND_FALLBACK;
      sd.tab.resize(tab0);
      continue;
    }
    if (sd.cand_dyn.empty()) {
      sd.cand_dyn.assign(static_cast<size_t>(nc), 0);
      sd.rec.assign(static_cast<size_t>(cands->cand_pod_off[nc] - base) * kSpreadU64, 0);
      sd.dmask.assign(static_cast<size_t>(cands->cand_pod_off[nc] - base), 0);
    }
    sd.cand_dyn[i] = 1;
    sd.active = true;
    for (const PendingSlot& ps : pend)
      spread_reuse_slot(*keep, ps.sel, counts.find(ps.sel)->second, ps.off, ps.local, ps.pairs, ps.skew, ps.self,
                        ps.n_counted, dk->dom[ps.slot], ps.pm, ps.edom);
    std::copy(words.begin(), words.end(), sd.rec.begin() + static_cast<size_t>(b - base) * kSpreadU64);
    std::copy(dm.begin(), dm.end(), sd.dmask.begin() + (b - base));
  }
}

}  // namespace

void reorder_list_by_cost(Workload& w, const uint32_t* cycles, int32_t head, int32_t n_front) {
  const size_t n = w.list.size() / 4;
  auto cost = [&](size_t j) { return cycles[w.list[j * 4]]; };
  std::vector<int8_t> front(n, 0);
  std::vector<int32_t> first;  // entries of the first part (the node-order kernel's when the list is split)
  for (size_t j = 0; j < n; ++j)
    if (w.n_list_node == 0 || static_cast<int32_t>(j) < w.n_list_node) first.push_back(static_cast<int32_t>(j));
  const size_t nf = std::min(first.size(), static_cast<size_t>(std::max(0, n_front)));
  std::nth_element(first.begin(), first.begin() + static_cast<std::ptrdiff_t>(nf), first.end(),
                   [&](int32_t a, int32_t b) { return cost(static_cast<size_t>(a)) > cost(static_cast<size_t>(b)); });
  for (size_t i = 0; i < nf; ++i) front[static_cast<size_t>(first[i])] = 1;
  w.n_coop_front = static_cast<int32_t>(nf);
  auto part = [&](size_t j) {
    if (front[j]) return -1;
    return (w.n_list_node > 0 && static_cast<int32_t>(j) >= w.n_list_node ? 2 : 0) + (w.list[j * 4] < head ? 0 : 1);
  };
  std::vector<int32_t> order(n);
  for (size_t j = 0; j < n; ++j) order[j] = static_cast<int32_t>(j);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
    const int pa = part(static_cast<size_t>(a)), pb = part(static_cast<size_t>(b));
    if (pa != pb) return pa < pb;
    return cycles[w.list[static_cast<size_t>(a) * 4]] > cycles[w.list[static_cast<size_t>(b) * 4]];
  });
  std::vector<int32_t> l(w.list.size()), x(w.list_ext.size());
  for (size_t j = 0; j < n; ++j) {
    std::copy_n(&w.list[static_cast<size_t>(order[j]) * 4], 4, &l[j * 4]);
    if (!x.empty()) std::copy_n(&w.list_ext[static_cast<size_t>(order[j]) * 4], 4, &x[j * 4]);
  }
  w.list.swap(l);
  if (!x.empty()) w.list_ext.swap(x);
}

uint64_t node_static_fp(const SpotNode& n, const sr_cluster* c) {
  uint64_t h = mix(mix(0xC0FFEEull, static_cast<uint32_t>(n.name)), n.unschedulable);
  uint64_t labels = 0, taints = 0;  // order-independent sums (Go map iteration order varies)
  for (const auto& kv : n.labels) {
    int64_t x = 0;  // Gt / Lt read the value's integer: part of the node's static content
    const uint64_t iv = str_int(c, kv.second, &x) ? mix(0x17ull, static_cast<uint64_t>(x)) : 0;
    labels += mix(mix(mix(0x1AB3ull, static_cast<uint32_t>(kv.first)), static_cast<uint32_t>(kv.second)), iv);
  }
  for (const TaintRec& t : n.taints)
    taints += mix(mix(mix(0x7A1Eull, static_cast<uint32_t>(t.key)), static_cast<uint32_t>(t.val)),
                  static_cast<uint32_t>(t.effect));
  return mix(mix(h, labels), taints);
}

uint64_t node_state_fp(const SpotNode& sn, const NodeState& st) {
  uint64_t h = 0x51ED270B7A1DE5ull;
  for (int r = 0; r < 3; ++r) h = mix(mix(h, static_cast<uint64_t>(sn.alloc[r])), static_cast<uint64_t>(st.requested[r]));
  h = mix(mix(h, static_cast<uint64_t>(sn.alloc_pods)), static_cast<uint64_t>(st.npods));
  for (const auto& a : sn.scalar_alloc)  // sorted by name: the order is canonical
    h = mix(mix(mix(h, 0x5CA1ull), static_cast<uint32_t>(a.first)), static_cast<uint64_t>(a.second));
  for (const auto& r : st.scalar_req)
    h = mix(mix(mix(h, 0x5CA2ull), static_cast<uint32_t>(r.first)), static_cast<uint64_t>(r.second));
  for (const auto& l : sn.vol_limit)
    h = mix(mix(mix(h, 0x5CA3ull), static_cast<uint32_t>(l.first)), static_cast<uint64_t>(l.second));
  for (const auto& a : st.att)  // sorted
    h = mix(mix(mix(h, 0x5CA4ull), static_cast<uint32_t>(a.first)), static_cast<uint32_t>(a.second));
  h = mix(mix(h, 0x3E7Aull), st.meta_sum);
  uint64_t ports = 0;  // order-independent
  for (const Port& u : st.ports)
    ports += mix(mix(mix(0x9E37ull, static_cast<uint32_t>(u.ip)), static_cast<uint32_t>(u.proto)),
                 static_cast<uint32_t>(u.port));
  return mix(h, ports);
}

namespace {

// A class whose S row is certainly empty: it ANDs an empty atom, ANDs the
// complement of a full one, or each of its ORed terms holds an empty atom.
bool class_empty(const Workload& w, int32_t k, const uint8_t* atom_empty, const uint8_t* atom_full) {
  bool empty = false, has_terms = false, all_terms_empty = true, term_empty = false;
  for (int32_t o = w.cls_prog_off[k]; o < w.cls_prog_off[k + 1]; ++o) {
    const int32_t atom = w.cls_prog[o] >> 2, kind = w.cls_prog[o] & 3;
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
  return empty || (has_terms && all_terms_empty);
}

// Composite atom rows: the pod-count atom AND NOT (any taint of the set).
void composite_rows(const EncoderCache& C, const std::vector<int32_t>& comp_sets, int32_t a_comp, int32_t Wp,
                    uint64_t* A) {
  for (size_t k = 0; k < comp_sets.size(); ++k) {
    uint64_t* row = A + static_cast<size_t>(a_comp + static_cast<int32_t>(k)) * Wp;
    const int32_t* u = C.untol_dict.data(comp_sets[k]);
    const size_t nu = C.untol_dict.len(comp_sets[k]);
    for (int32_t i = 0; i < Wp; ++i) {
      uint64_t any = 0;
      for (size_t j = 0; j < nu; ++j) any |= C.taint_rows[static_cast<size_t>(u[j]) * Wp + i];
      row[i] = A[i] & ~any;
    }
  }
}

void atom_flags(const uint64_t* row, int32_t Wp, int32_t n_spot, uint8_t* empty, uint8_t* full) {
  int64_t pop = 0;
  for (int32_t i = 0; i < Wp; ++i) pop += __builtin_popcountll(row[i]);
  *empty = pop == 0;
  *full = pop == n_spot;
}

// The call's candidate input equals the one CandReuse saved, every pod stamped.
bool same_cand_input(const CandReuse& R, const sr_candidates* cands, const uint64_t* stamps) {
  const int32_t nc = cands->n_cand;
  if (!R.have_input || !stamps || static_cast<size_t>(nc) + 1 != R.pod_off.size() ||
      (cands->cand_global != nullptr) != !R.glob.empty())
    return false;
  if (std::memcmp(cands->cand_pod_off, R.pod_off.data(), sizeof(int32_t) * (static_cast<size_t>(nc) + 1)) != 0)
    return false;
  if (cands->cand_global && std::memcmp(cands->cand_global, R.glob.data(), sizeof(int32_t) * nc) != 0) return false;
  const int32_t b = cands->cand_pod_off[0];
  const size_t n = R.pods.size();
  std::atomic<bool> same{true};
  auto cmp = [&](size_t lo, size_t hi) {
    bool ok = std::memcmp(cands->cand_pods + b + lo, R.pods.data() + lo, sizeof(int32_t) * (hi - lo)) == 0;
    for (size_t j = lo; j < hi && ok; ++j) {
      if (j + 32 < hi) __builtin_prefetch(stamps + R.pods[j + 32]);  // scattered reads: keep many in flight
      ok = stamps[R.pods[j]] != 0 && stamps[R.pods[j]] == R.stamps[j];
    }
    if (!ok) same.store(false, std::memory_order_relaxed);
  };
  if (n > (size_t(1) << 18)) parallel_for(n, 65536, cmp);  // a sequential pass is ~0.1 ns per byte compared
  else cmp(0, n);
  return same.load(std::memory_order_relaxed);
}

void save_cand_input(CandReuse& R, const sr_candidates* cands, const uint64_t* stamps, int32_t n_pods) {
  R.drop();
  const int32_t nc = cands->n_cand;
  const int32_t b = nc > 0 ? cands->cand_pod_off[0] : 0, e = nc > 0 ? cands->cand_pod_off[nc] : 0;
  for (int32_t j = b; j < e; ++j)
    if (cands->cand_pods[j] < 0 || cands->cand_pods[j] >= n_pods || stamps[cands->cand_pods[j]] == 0) return;
  R.pod_off.assign(cands->cand_pod_off, cands->cand_pod_off + nc + 1);
  if (nc == 0) R.pod_off.assign(1, 0);
  R.glob.assign(cands->cand_global ? cands->cand_global : nullptr, cands->cand_global ? cands->cand_global + nc : nullptr);
  R.pods.assign(cands->cand_pods + b, cands->cand_pods + e);
  R.stamps.resize(R.pods.size());
  for (size_t j = 0; j < R.pods.size(); ++j) R.stamps[j] = stamps[R.pods[j]];
  R.have_input = true;
}

// The candidate-side reuse encode (CandReuse): the Workload of
// the last call, its state-dependent parts brought up to the current state
// view.  False when a dimension ran out of spare T rows (the caller encodes in
// full; the index is rebuilt).
bool reuse_encode(EncoderCache& C, const sr_snapshot* snap, Workload* w, uint64_t prev_state_gen) {
  CandReuse& R = w->reuse;
  const int32_t Wp = w->Wp, n_spot = w->n_spot;
  uint64_t* A = w->atoms.data();
  w->atom_cols.clear();
  w->tab_changed = false;
  w->atoms_prev_ver = w->atoms_ver;
  w->atom_rows.clear();
  w->atom_rows_all = false;
  std::vector<int32_t>& rows_moved = w->atom_rows;

  // the host-decided outcomes that read the snapshot must still hold: scalar
  // usage known on every node, no planned candidate's attachable volume on a
  // spot node (only the nodes changed since the last encode can have one now;
  // every node when the state view was rebuilt rather than patched)
  if (R.scalars && snap->scalar_unknown_total > 0) return false;
  if (!R.att_words.empty() && prev_state_gen != C.state_gen) {
    auto holds = [&](int32_t n) {
      for (const auto& a : snap->state[n].att)
        if (std::binary_search(R.att_words.begin(), R.att_words.end(), att_word(a.first, a.second))) return true;
      return false;
    };
    if (C.patched_from == prev_state_gen) {
      for (int32_t n : C.patched_nodes)
        if (holds(n)) return false;
    } else {
      for (int32_t n = 0; n < n_spot; ++n)
        if (holds(n)) return false;
    }
  }
  if (w->layout_gen != C.layout_gen) {  // the spot order moved (permute_static): every atom row follows
    auto rows = [&](size_t lo, size_t hi) {
      for (size_t a = lo; a < hi; ++a) permute_bits(A + a * Wp, Wp, C.perm_src, C.perm_k, C.perm_to);
    };
    if (w->n_atoms > 512) parallel_for(static_cast<size_t>(w->n_atoms), 256, rows);  // (inter-pod atoms: thousands)
    else rows(0, static_cast<size_t>(w->n_atoms));
    w->layout_gen = C.layout_gen;
    w->atom_rows_all = true;
    // the inter-pod and spread states, the domain path's node domains and
    // node-local base tables are kept per spot position too
    if (R.anti) anti_reuse_permute(*R.anti, C.perm_src, C.perm_k);
    if (R.spread) {
      spread_reuse_permute(*R.spread, C.perm_src, C.perm_k, w->sp_tab);
      w->tab_changed = true;
    }
    for (int32_t k = 0; k < w->n_dk; ++k)  // (a node-local key's domain is the position itself)
      if (w->dk_row[k] >= 0) permute_positions(w->dk_dom.data() + static_cast<size_t>(k) * n_spot, C.perm_src, C.perm_k);
  }
  // pod count and the composites built on it, in the words where it changed
  std::vector<int32_t> words;
  for (int32_t i = 0; i < Wp; ++i)
    if (A[i] != C.podcount_row[i]) words.push_back(i);
  for (int32_t i : words) {
    A[i] = C.podcount_row[i];
    for (size_t k = 0; k < R.comp_sets.size(); ++k) {
      const int32_t* u = C.untol_dict.data(R.comp_sets[k]);
      const size_t nu = C.untol_dict.len(R.comp_sets[k]);
      uint64_t any = 0;
      for (size_t j = 0; j < nu; ++j) any |= C.taint_rows[static_cast<size_t>(u[j]) * Wp + i];
      A[static_cast<size_t>(R.a_comp + static_cast<int32_t>(k)) * Wp + i] = A[i] & ~any;
    }
  }
  if (!words.empty()) {
    rows_moved.push_back(0);
    for (size_t k = 0; k < R.comp_sets.size(); ++k) rows_moved.push_back(R.a_comp + static_cast<int32_t>(k));
  }
  bool flags_moved = false;
  auto refresh_flags = [&](int32_t a) {
    uint8_t e = 0, f = 0;
    atom_flags(A + static_cast<size_t>(a) * Wp, Wp, n_spot, &e, &f);
    flags_moved = flags_moved || e != R.atom_empty[a] || f != R.atom_full[a];
    R.atom_empty[a] = e;
    R.atom_full[a] = f;
  };
  if (!words.empty()) {
    refresh_flags(0);
    for (size_t k = 0; k < R.comp_sets.size(); ++k) refresh_flags(R.a_comp + static_cast<int32_t>(k));
  }
  // host-port queries: their base conflict rows follow the spot pods' ports
  const int32_t n_ports = static_cast<int32_t>(R.port_q.size() / 3);
  if (n_ports > 0) {
    std::vector<uint64_t>& rows = R.port_scratch;
    rows.resize(static_cast<size_t>(n_ports) * Wp);
    port_conflict_rows(C, snap, reinterpret_cast<const PortQuery*>(R.port_q.data()), n_ports, Wp, rows.data());
    for (int32_t q = 0; q < n_ports; ++q) {
      uint64_t* a = A + static_cast<size_t>(R.a_port + q) * Wp;
      const uint64_t* r = rows.data() + static_cast<size_t>(q) * Wp;
      if (!std::equal(r, r + Wp, a)) {
        std::copy_n(r, Wp, a);
        refresh_flags(R.a_port + q);
        rows_moved.push_back(R.a_port + q);
      }
    }
  }
  // scalar-resource / volume-limit queries and the shared scalar rows follow
  // the spot nodes' usage: only the changed nodes' bits and values when the
  // state view was patched node by node since this workload's last encode
  // (its moved positions included: the rows were permuted above), every node
  // otherwise
  if (prev_state_gen != C.state_gen && C.patched_from == prev_state_gen) {
    for (size_t q = 0; q < R.scalar_q.size(); ++q) {
      uint64_t* a = A + static_cast<size_t>(R.a_scalar + static_cast<int32_t>(q)) * Wp;
      bool moved_bit = false;
      for (int32_t n : C.patched_nodes) {
        uint64_t& wd = a[n >> 6];
        const uint64_t bit = 1ull << (n & 63), old = wd;
        wd = scalar_query_node(snap, n, R.scalar_q[q].first, R.scalar_q[q].second) ? (wd | bit) : (wd & ~bit);
        moved_bit = moved_bit || wd != old;
      }
      if (moved_bit) {
        refresh_flags(R.a_scalar + static_cast<int32_t>(q));
        rows_moved.push_back(R.a_scalar + static_cast<int32_t>(q));
      }
    }
    if (!R.scal_names.empty())
      for (size_t u = 0; u < R.scal_names.size(); ++u)
        for (int32_t n : C.patched_nodes)
          w->node_scal[u * static_cast<size_t>(w->n_pad) + static_cast<size_t>(n)] =
              node_scal_value(snap, n, R.scal_names[u]);
  } else if (prev_state_gen != C.state_gen) {
    for (size_t q = 0; q < R.scalar_q.size(); ++q) {
      uint64_t* a = A + static_cast<size_t>(R.a_scalar + static_cast<int32_t>(q)) * Wp;
      std::vector<uint64_t>& row = R.port_scratch;
      row.assign(static_cast<size_t>(Wp), 0);
      scalar_query_row(snap, R.scalar_q[q].first, R.scalar_q[q].second, row.data());
      if (!std::equal(row.begin(), row.end(), a)) {
        std::copy(row.begin(), row.end(), a);
        refresh_flags(R.a_scalar + static_cast<int32_t>(q));
        rows_moved.push_back(R.a_scalar + static_cast<int32_t>(q));
      }
    }
    if (!R.scal_names.empty()) node_scal_rows(snap, R.scal_names, w->n_pad, w->node_scal.data());
  }
  // required anti-affinity and topology spread: the DA / DB rows, the spread
  // rows and the domain-path tables follow the nodes whose pods changed
  // (every node when the state view was rebuilt since this workload's encode)
  if ((R.anti || R.spread) && prev_state_gen != C.state_gen) {
    std::vector<int32_t> every;
    const std::vector<int32_t>* nodes = &C.content_nodes;
    if (C.content_from != prev_state_gen) {
      every.resize(static_cast<size_t>(n_spot));
      for (int32_t n = 0; n < n_spot; ++n) every[n] = n;
      nodes = &every;
    }
    std::vector<int32_t> moved_atoms;
    if (R.anti && !anti_reuse_patch(*R.anti, snap, *nodes, A, R.a_anti, moved_atoms, w->atom_cols)) return false;
    if (R.spread &&
        !spread_reuse_patch(*R.spread, snap, *nodes, A, w->sp_tab, &w->tab_changed, moved_atoms, w->atom_cols))
      return false;
    std::sort(moved_atoms.begin(), moved_atoms.end());
    moved_atoms.erase(std::unique(moved_atoms.begin(), moved_atoms.end()), moved_atoms.end());
    for (int32_t a : moved_atoms) refresh_flags(a);
    rows_moved.insert(rows_moved.end(), moved_atoms.begin(), moved_atoms.end());
    std::sort(w->atom_cols.begin(), w->atom_cols.end());
    w->atom_cols.erase(std::unique(w->atom_cols.begin(), w->atom_cols.end()), w->atom_cols.end());
  }
  std::sort(rows_moved.begin(), rows_moved.end());
  rows_moved.erase(std::unique(rows_moved.begin(), rows_moved.end()), rows_moved.end());
  if (w->atom_rows_all || !rows_moved.empty()) w->atoms_ver = C.atoms_ver_next++;
  // classes whose certain emptiness changed: after every atom row above was
  // refreshed (pod count, composites, ports, scalar / volume-limit queries,
  // inter-pod and spread rows)
  std::vector<int32_t> flipped;
  if (flags_moved)
    for (int32_t k = 0; k < static_cast<int32_t>(R.cls_empty.size()); ++k) {
      const uint8_t e = class_empty(*w, k, R.atom_empty.data(), R.atom_full.data()) ? 1 : 0;
      if (e != R.cls_empty[k]) {
        R.cls_empty[k] = e;
        flipped.push_back(k);
      }
    }
  // thresholds: a distinct request whose smallest node value >= it moved
  constexpr int64_t kNever = INT64_MAX;
  // Only requests in the interval (previous value, value] of a node value
  // that appeared or disappeared since the last update can move: the two
  // sorted value lists are merged, and each such interval's requests found
  // by binary search.
  std::vector<std::pair<int32_t, int64_t>> moved[3];  // (distinct request, new threshold)
  std::vector<int32_t> cand_u;
  for (int d = 0; d < 3; ++d) {
    const std::vector<int64_t>& v = C.node_vals[d];
    const std::vector<int64_t>& old = R.vals[d];
    const std::vector<int64_t>& dr = R.dreq[d];
    cand_u.clear();
    auto interval = [&](int64_t lo, int64_t hi) {  // requests in (lo, hi]
      const size_t a = static_cast<size_t>(std::upper_bound(dr.begin(), dr.end(), lo) - dr.begin());
      const size_t b = static_cast<size_t>(std::upper_bound(dr.begin(), dr.end(), hi) - dr.begin());
      for (size_t u = a; u < b; ++u) cand_u.push_back(static_cast<int32_t>(u));
    };
    size_t i = 0, j = 0;
    while (i < old.size() || j < v.size()) {
      if (j == v.size() || (i < old.size() && old[i] < v[j])) {  // gone
        interval(i == 0 ? INT64_MIN : old[i - 1], old[i]);
        ++i;
      } else if (i == old.size() || v[j] < old[i]) {  // new
        interval(j == 0 ? INT64_MIN : v[j - 1], v[j]);
        ++j;
      } else {
        ++i;
        ++j;
      }
    }
    std::sort(cand_u.begin(), cand_u.end());
    cand_u.erase(std::unique(cand_u.begin(), cand_u.end()), cand_u.end());
    for (int32_t u : cand_u) {
      const size_t pos = static_cast<size_t>(std::lower_bound(v.begin(), v.end(), dr[u]) - v.begin());
      const int64_t thr = pos == v.size() ? kNever : v[pos];
      if (thr != R.dthr[d][u]) moved[d].emplace_back(u, thr);
    }
    R.vals[d] = v;
  }
  for (int d = 0; d < 3; ++d)  // rows left without requests become spare ...
    for (const auto& m : moved[d]) {
      const int32_t row = R.drow[d][m.first];
      if (--R.row_refs[row] == 0) {
        R.row_of[d].erase(R.dthr[d][m.first]);
        w->t_thr[row] = kTSpare;
        R.spare[d].push_back(row);
      }
    }
  for (int d = 0; d < 3; ++d)  // ... before the new thresholds take rows
    for (const auto& m : moved[d]) {
      int32_t row;
      auto it = R.row_of[d].find(m.second);
      if (it != R.row_of[d].end()) {
        row = it->second;
      } else {
        if (R.spare[d].empty()) {
          R.indexed = false;
          return false;
        }
        row = R.spare[d].back();
        R.spare[d].pop_back();
        R.row_of[d].emplace(m.second, row);
        w->t_thr[row] = m.second;
        R.row_refs[row] = 0;
      }
      ++R.row_refs[row];
      R.drow[d][m.first] = row;
      R.dthr[d][m.first] = m.second;
    }
  // the records of the pods asking within a moved interval or of a flipped class
  if (++R.epoch == 0) {
    std::fill(R.mark.begin(), R.mark.end(), 0u);
    R.epoch = 1;
  }
  w->pod_patch.clear();
  w->class_flip = false;
  const uint64_t Wp64 = static_cast<uint64_t>(Wp);
  auto off = [&](int32_t table_row) { return static_cast<uint64_t>(table_row) * Wp64; };
  auto repoint = [&](int32_t q) {
    if (R.mark[q] == R.epoch) return;
    R.mark[q] = R.epoch;
    const int32_t* ri = &R.pod_ri[static_cast<size_t>(q) * 3];
    const bool zero = ri[0] < 0;
    int32_t cls = R.pod_cls[q], row[3] = {0, 0, 0};
    bool dead = R.cls_empty[cls] != 0;
    if (!zero)
      for (int d = 0; d < 3; ++d) {
        row[d] = R.drow[d][ri[d]];
        dead = dead || R.dthr[d][ri[d]] == kNever;
      }
    if (dead) cls = w->empty_class;
    int32_t* r = &w->pod_rows[static_cast<size_t>(q) * 4];
    if (r[0] != cls) w->class_flip = true;
    r[0] = cls;
    for (int d = 0; d < 3; ++d) r[1 + d] = row[d];
    uint64_t* rec = &w->pod_rec[static_cast<size_t>(q) * 6];
    const uint64_t r4 = off(cls) | off(w->n_classes + row[0]) << 32;
    const uint64_t r5 = off(w->n_classes + row[1]) | off(w->n_classes + row[2]) << 32;
    if (rec[4] == r4 && rec[5] == r5) return;
    rec[4] = r4;
    rec[5] = r5;
    w->pod_patch.insert(w->pod_patch.end(), {static_cast<uint64_t>(q), r4, r5});
  };
  for (int d = 0; d < 3; ++d)
    for (const auto& m : moved[d])
      for (int32_t i = R.dpod_off[d][m.first]; i < R.dpod_off[d][m.first + 1]; ++i) repoint(R.dpod[d][i]);
  for (int32_t k : flipped)
    for (int32_t i = R.cls_pod_off[k]; i < R.cls_pod_off[k + 1]; ++i) repoint(R.cls_pod[i]);
  w->reused = true;
  return true;
}

}  // namespace

namespace {
sr_status encode_impl(EncoderCache& C, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                      Workload* w, std::string* err);
}  // namespace

sr_status encode_workload(EncoderCache* cache, const sr_snapshot* snap, const sr_cluster* c,
                          const sr_candidates* cands, Workload* w, std::string* err) {
  const sr_status st = encode_impl(*cache, snap, c, cands, w, err);
  if (st != SR_OK) w->reuse.drop();  // the Workload no longer holds the input it saved
  return st;
}

namespace {
sr_status encode_impl(EncoderCache& C, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
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
  if (!snap->nodes.empty() &&
      (c->id_empty != snap->id_empty || c->id_metadata_name != snap->id_metadata_name ||
       c->id_unschedulable_key != snap->id_unschedulable_key)) {
    *err = "cluster string ids differ from the snapshot's (one interner per snapshot)";
    return SR_ERR_INVALID_ARG;
  }
  // content dictionaries are a function of the interned ids of these strings
  if (C.id_empty != c->id_empty || C.id_metadata_name != c->id_metadata_name ||
      C.id_unschedulable_key != c->id_unschedulable_key || C.spec.size() > kMaxSpecs ||
      C.req_dict.size() > kMaxReqs) {
    C.clear_content();
    C.id_empty = c->id_empty;
    C.id_metadata_name = c->id_metadata_name;
    C.id_unschedulable_key = c->id_unschedulable_key;
    C.n_spot = -1;  // and the node views
  }
  if (C.spec.empty()) {  // spec 0: no static constraints
    C.spec.emplace_back();
    C.spec_shards.assign(kSpecShards, EncoderCache::SpecShard{});
  }

  // ---- spot node dimensions and the cached node views
  const int32_t W = (n_spot + 63) / 64;
  const int32_t Wp = std::max(2, (W + 1) & ~1);
  if (Wp > MAX_WORDS) {
    *err = "too many spot nodes for one device plan";
    return SR_ERR_CAPACITY;
  }
  refresh_static(C, snap, Wp);
  sr_status st = refresh_state(C, snap, err);
  if (st != SR_OK) return st;
  phase(0);

  // ---- per-pod memo (sr_cluster.pod_stamp): valid for the cluster's table
  // shape it was derived under
  const uint64_t* stamps = c->pod_stamp;
  if (stamps) {
    const uint64_t shape = cluster_shape(c);
    if (C.memo_shape != shape) {
      C.pod_memo.clear();
      C.memo_shape = shape;
    }
    if (C.pod_memo.size() < static_cast<size_t>(P.n)) C.pod_memo.resize(static_cast<size_t>(P.n));
  }
  std::atomic<int32_t> memo_hits{0};

  // ---- candidate-side reuse (CandReuse): the same stamped
  // candidate input as the last call
  CandReuse& R = w->reuse;
  const bool same_input = stamps && R.shape == C.memo_shape && same_cand_input(R, cands, stamps);
  if (same_input && R.indexed && R.content_gen == C.content_gen && R.static_gen == C.static_gen && R.n_spot == n_spot && R.Wp == Wp &&
      (w->layout_gen == C.layout_gen || w->layout_gen + 1 == C.layout_gen) && snap->opaque_total == 0 &&
      (snap->anti_total == 0 || R.anti) &&
      (!(R.anti || R.spread) || (snap->unknown_total == 0 && snap->term_unknown_total == 0))) {
    const uint64_t prev_state_gen = w->state_gen;
    w->state_gen = C.state_gen;
    if (reuse_encode(C, snap, w, prev_state_gen)) {
      C.last_new_specs = 0;
      C.last_memo_hits = w->n_input_pods;
      C.last_reused = 1;
      C.last_pod_patches = static_cast<int32_t>(w->pod_patch.size() / kPodPatchWords);
      for (int i = 1; i < 16; ++i) encode_phase_ms[i] = 0;
      phase(11);
      return SR_OK;
    }
  }
  C.last_reused = 0;
  C.last_pod_patches = 0;
  R.indexed = false;
  if (!same_input) {
    if (stamps) {
      save_cand_input(R, cands, stamps, P.n);
      R.shape = C.memo_shape;
    } else {
      R.drop();
    }
  }
  // the second consecutive encode of one input builds the index (below,
  // when the candidate side turns out to read no other snapshot state)
  const bool want_index = same_input;
  w->reset();
  w->cand_gen = C.cand_gen_next++;
  w->atoms_ver = C.atoms_ver_next++;
  w->atoms_prev_ver = 0;
  w->atom_rows.clear();
  w->atom_rows_all = true;
  w->n_input_cand = nc;
  w->pod_base = nc > 0 ? cands->cand_pod_off[0] : 0;
  w->n_input_pods = nc > 0 ? cands->cand_pod_off[nc] - w->pod_base : 0;
  w->n_spot = n_spot;
  w->Wp = Wp;
  w->n_pad = Wp * 64;
  w->state_gen = C.state_gen;
  w->layout_gen = C.layout_gen;

  // ---- pass 1: candidate-level fallback (host-decided)
  w->status_host.assign(static_cast<size_t>(nc), STATUS_PENDING);
  // the candidate pods' requests, gathered once in input order (the per-pod
  // pass later reads them sequentially instead of from the cluster arrays)
  std::vector<int64_t>& req_flat = C.scratch.req_flat;
  req_flat.resize(static_cast<size_t>(w->n_input_pods) * 3);
  auto pod_fallback = [&](int32_t pod, int32_t j, bool last) {
    if (P.flags[pod] & SR_POD_FB_MASK) return true;
    int64_t* rq = &req_flat[static_cast<size_t>(j - w->pod_base) * 3];
    rq[0] = P.req_milli_cpu[pod];
    rq[1] = P.req_memory[pod];
    rq[2] = P.req_ephemeral[pod];
    if (!in_range(rq[0]) || !in_range(rq[1]) || !in_range(rq[2])) return true;
    // NodeInfo.AddPod's accounting (init containers: it can differ from the
    // fit request; the candidate's extension records carry it, see below)
    for (int r = 0; r < 3 && !last; ++r)
      if (!in_range(pod_acc(c, pod, r))) return true;
    if (has_scalars(c, pod)) {
      // a listed scalar keeps an all-zero cpu / memory / ephemeral request
      // from skipping the resource checks: not encoded (the volume limit keys
      // are other filters: they do not)
      if (rq[0] == 0 && rq[1] == 0 && rq[2] == 0) return true;
      if (snap->scalar_unknown_total > 0) return true;  // some node's scalar usage is unknown
      for (int32_t i = c->pod_scalar_off[pod]; i < c->pod_scalar_off[pod + 1]; ++i)
        if (!in_range(c->pod_scalar_req[i]) || !in_range(c->pod_scalar_acc[i])) return true;
    }
    if (P.aff_required[pod])
      for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t)
        for (int32_t e = P.term_expr_off[t]; e < P.term_expr_off[t + 1]; ++e) {
          if ((P.expr_op[e] == SR_OP_GT || P.expr_op[e] == SR_OP_LT) && !c->str_int) return true;
          if (!c->str_label) return true;  // NewRequirement's validation unknown
        }
    if (has_spread(c, pod)) {
      // the counts need every snapshot pod's namespace, labels and deletion
      // state; a selector that fails to build errors PreFilter
      if (!c->pod_affinity || !c->str_label || snap->unknown_total > 0 || snap->term_unknown_total > 0) return true;
      for (int32_t k = c->spread->off[pod]; k < c->spread->off[pod + 1]; ++k)
        if (spread_invalid(c, k)) return true;
    }
    return anti_opaque(c, pod) || aff_opaque(c, pod);  // required (anti-)affinity the encoded set cannot read
  };
  // The same checks through the memo: for a "plain" pod (no scalar resources,
  // spread constraints or attachable volumes: nothing snapshot-dependent) the
  // answer is a function of the pod alone; MEMO_ACC_DIFF and MEMO_PORTS feed
  // the extension and host-port passes.
  auto pod_bits = [&](int32_t pod) -> uint32_t {
    uint32_t b = 0;
    const bool plain = !has_scalars(c, pod) && !has_spread(c, pod) && att_count(c, pod) == 0;
    if (plain) {
      b |= MEMO_PLAIN;
      const int64_t rq[3] = {P.req_milli_cpu[pod], P.req_memory[pod], P.req_ephemeral[pod]};
      bool fb = (P.flags[pod] & SR_POD_FB_MASK) || !in_range(rq[0]) || !in_range(rq[1]) || !in_range(rq[2]);
      if (!fb && P.aff_required[pod])
        for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1] && !fb; ++t)
          for (int32_t e = P.term_expr_off[t]; e < P.term_expr_off[t + 1] && !fb; ++e)
            fb = ((P.expr_op[e] == SR_OP_GT || P.expr_op[e] == SR_OP_LT) && !c->str_int) || !c->str_label;
      fb = fb || anti_opaque(c, pod) || aff_opaque(c, pod);
      if (fb) b |= MEMO_FB;
      for (int r = 0; r < 3; ++r)
        if (!in_range(pod_acc(c, pod, r))) b |= MEMO_ACC_BAD;
    }
    if (pod_acc(c, pod, 0) != P.req_milli_cpu[pod] || pod_acc(c, pod, 1) != P.req_memory[pod] ||
        pod_acc(c, pod, 2) != P.req_ephemeral[pod])
      b |= MEMO_ACC_DIFF;
    if (has_ports(c, pod)) b |= MEMO_PORTS;
    return b;
  };
  auto memo_bits = [&](int32_t pod) -> uint32_t {
    if (!stamps || stamps[pod] == 0) return pod_bits(pod);
    EncoderCache::PodMemo& m = C.pod_memo[static_cast<size_t>(pod)];
    if (m.stamp_bits == stamps[pod]) return m.bits;
    m.bits = pod_bits(pod);
    m.stamp_bits = stamps[pod];
    return m.bits;
  };
  for (int32_t i = 0; i < nc; ++i)
    if (cands->cand_pod_off[i + 1] < cands->cand_pod_off[i]) {
      *err = "cand_pod_off not monotone";
      return SR_ERR_INVALID_ARG;
    }
  // attachable volumes the spot nodes already hold (limit key, unique name),
  // when some candidate pod has attachable volumes
  std::unordered_set<uint64_t> vol_base_set;
  const std::unordered_set<uint64_t>* vol_base = nullptr;
  if (c->volumes) {
    bool any = false;
    for (int32_t i = 0; i < nc && !any; ++i)
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1] && !any; ++j)
        any = cands->cand_pods[j] >= 0 && cands->cand_pods[j] < P.n && att_count(c, cands->cand_pods[j]) > 0;
    if (any) {
      for (const NodeState& st : snap->state)
        for (const auto& a : st.att) vol_base_set.insert(att_word(a.first, a.second));
      vol_base = &vol_base_set;
    }
  }
  std::vector<uint8_t>& cand_ports = C.scratch.cand_ports;  // the candidate's pods ask for host ports
  cand_ports.assign(static_cast<size_t>(nc), 0);
  std::vector<uint8_t>& cand_ext = C.scratch.cand_ext;       // bit 0: accounting differs, bit 1: shared scalars
  cand_ext.assign(static_cast<size_t>(nc), 0);
  std::vector<int32_t>& cand_sname = C.scratch.cand_sname;   // [2 * candidate] its shared scalar names (-1: none)
  cand_sname.resize(static_cast<size_t>(2 * nc));
  std::atomic<bool> bad_index{false};
  auto pass1 = [&](size_t lo, size_t hi) {
    bool bad = false;
    for (size_t i = lo; i < hi; ++i)
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j)
        bad = bad || cands->cand_pods[j] < 0 || cands->cand_pods[j] >= P.n;
    if (bad) {
      bad_index.store(true, std::memory_order_relaxed);
      return;
    }
    for (size_t i = lo; i < hi; ++i) {
      const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
      if (e == b) {
        w->status_host[i] = SR_CAND_EMPTY;
        continue;
      }
      // an existing pod's opaque anti-affinity may select any incoming pod
      bool fb = (c->pod_affinity ? snap->opaque_total : snap->anti_total) > 0 || (e - b) > MAX_CAND_PODS;
      // Extension records (K2's pod-order and domain paths): a pod followed by
      // others whose AddPod accounting differs from its fit request (the
      // running state subtracts the accounting), and scalar resources listed
      // by two or more pods of the candidate (the later ones see the earlier
      // ones' AddPod: a running scalar state per touched node, at most
      // kExtScalars names per candidate)
      uint8_t ext = 0;
      bool ports = false;
      int32_t hits = 0;
      for (int32_t j = b; j < e && !fb; ++j) {
        const int32_t pod = cands->cand_pods[j];
        const bool last = j + 1 == e;
        const uint32_t mb = memo_bits(pod);
        hits += stamps && stamps[pod] != 0 ? 1 : 0;
        if (mb & MEMO_PLAIN) {
          fb = (mb & MEMO_FB) || (!last && (mb & MEMO_ACC_BAD));
          int64_t* rq = &req_flat[static_cast<size_t>(j - w->pod_base) * 3];
          rq[0] = P.req_milli_cpu[pod];
          rq[1] = P.req_memory[pod];
          rq[2] = P.req_ephemeral[pod];
        } else {
          fb = pod_fallback(pod, j, last);
        }
        if (!last && (mb & MEMO_ACC_DIFF)) ext |= 1;
        ports = ports || (mb & MEMO_PORTS);
      }
      if (stamps) memo_hits.fetch_add(hits, std::memory_order_relaxed);
      cand_sname[2 * i] = cand_sname[2 * i + 1] = kNoName;
      if (!fb && c->volumes && vol_base && !vol_base->empty()) {
        // an attachable volume some spot node already holds, or two pods of
        // the candidate sharing one: the volume counts stop being additive
        for (int32_t j = b; j < e && !fb; ++j) {
          const int32_t pod = cands->cand_pods[j];
          for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1] && !fb; ++a)
            fb = vol_base->count(att_word(c->volumes->att_key[a], c->volumes->att_id[a])) != 0;
        }
      }
      bool any_att = false;
      for (int32_t j = b; j < e && !fb && c->volumes && !any_att; ++j) any_att = att_count(c, cands->cand_pods[j]) > 0;
      if (!fb && any_att) {
        std::vector<uint64_t> ids;
        for (int32_t j = b; j < e; ++j) {
          const int32_t pod = cands->cand_pods[j];
          for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1]; ++a)
            ids.push_back(att_word(c->volumes->att_key[a], c->volumes->att_id[a]));
        }
        std::sort(ids.begin(), ids.end());
        fb = std::adjacent_find(ids.begin(), ids.end()) != ids.end();
      }
      if (!fb && (c->pod_scalar_off || c->volumes)) {
        // names listed by the candidate's pods: scalar resources, then the
        // volume limit keys (negative names, one per pod with such volumes)
        int32_t names[64], cnt[64], nn = 0;
        auto count_name = [&](int32_t name) {
          int32_t u = 0;
          while (u < nn && names[u] != name) ++u;
          if (u < nn) {
            ++cnt[u];
          } else if (nn == 64) {
            fb = true;  // more scalar entries than the candidate's table holds
          } else {
            names[nn] = name;
            cnt[nn++] = 1;
          }
        };
        for (int32_t j = b; j < e && !fb; ++j) {
          const int32_t pod = cands->cand_pods[j];
          if (c->pod_scalar_off)
            for (int32_t k = c->pod_scalar_off[pod]; k < c->pod_scalar_off[pod + 1] && !fb; ++k)
              count_name(c->pod_scalar_name[k]);
          if (c->volumes)
            for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1] && !fb; ++a) {
              bool first = true;  // each key once per pod
              for (int32_t a2 = c->volumes->att_off[pod]; a2 < a; ++a2) first = first && c->volumes->att_key[a2] != c->volumes->att_key[a];
              if (first) count_name(vol_name(c->volumes->att_key[a]));
            }
        }
        int32_t shared = 0;
        for (int32_t u = 0; u < nn && !fb; ++u)
          if (cnt[u] >= 2) {
            if (shared == kExtScalars) fb = true;
            else cand_sname[2 * i + shared++] = names[u];
          }
        if (shared > 0) ext |= 2;
      }
      cand_ext[i] = fb ? 0 : ext;
      if (fb) w->status_host[i] = SR_CAND_FALLBACK;
      cand_ports[i] = !fb && ports;
    }
  };
  if (w->n_input_pods > serial_pods()) parallel_for(static_cast<size_t>(nc), 64, pass1);
  else pass1(0, static_cast<size_t>(nc));
  if (bad_index.load(std::memory_order_relaxed)) {
    *err = "candidate pod index out of range";
    return SR_ERR_INVALID_ARG;
  }
  phase(5);

  // ---- required pod anti-affinity: static node sets, state-bit pairs and
  // the candidates it sends to the fallback path (antiaff.cpp)
  DomKeys dk;  // topology keys of the domain path (K2 k2_domain)
  AntiTerms anti;
  // the index build (want_index) keeps the snapshot-side state a reuse encode patches
  std::shared_ptr<AntiReuse> anti_keep;
  analyse_anti(snap, c, cands, Wp, w->status_host, &dk, &anti, want_index ? &anti_keep : nullptr);
  const int32_t bit_shift = 2 * anti.n_pairs;  // host-port bits sit above the pairs
  // ---- required pod affinity: term sets, their node rows, and the
  // candidates whose pods interact through them (antiaff.cpp)
  AffTerms aff;
  analyse_affinity(snap, c, cands, Wp, w->status_host, &dk, &aff);
  // ---- topology spread between the pods of one candidate (domain path)
  SpreadDyn sdyn;
  SpreadIndex six(snap);  // spread rows: node values per key, snapshot pods per label (built lazily)
  if (c->spread) {  // the label values the call's constraints select on (SpreadIndex::want)
    const sr_spread* S = c->spread;
    for (int32_t i = 0; i < nc; ++i) {
      if (w->status_host[i] != STATUS_PENDING) continue;
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j)
        for (int32_t k = S->off[cands->cand_pods[j]]; k < S->off[cands->cand_pods[j] + 1]; ++k) {
          if (S->selector_nil[k] || S->ml_off[k] == S->ml_off[k + 1]) continue;
          int32_t f = S->ml_off[k];
          for (int32_t x = S->ml_off[k] + 1; x < S->ml_off[k + 1]; ++x)
            if (S->ml_key[x] < S->ml_key[f]) f = x;
          six.want(S->ml_key[f], S->ml_val[f]);
        }
    }
  }
  std::shared_ptr<SpreadReuse> spread_keep = want_index && c->spread ? spread_reuse_new(snap, Wp) : nullptr;
  analyse_spread(C, snap, c, cands, w->status_host, &dk, &sdyn, six, spread_keep.get());
  auto spread_dm = [&](int32_t flat) -> int32_t { return sdyn.dmask.empty() ? 0 : sdyn.dmask[flat - sdyn.base]; };
  // affinity planned on the domain path: the pod's class carries KEYS(S), the
  // device the rest (an earlier pod of its candidate matches all its terms)
  auto aff_dyn = [&](int32_t flat) {
    if (aff.mmask.empty()) return false;
    for (int g = 0; g < kDynG; ++g)
      if (aff.mmask[static_cast<size_t>(flat - aff.base) * kDynG + g] != 0) return true;
    return false;
  };

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
    if (w->status_host[i] != STATUS_PENDING || !cand_ports[i]) continue;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j)
      for_each_port(c, cands->cand_pods[j], [&](int32_t proto, int32_t port, int32_t ip) {
        group_specific[port_key(proto, port)] |= ip != -1;
      });
  }
  struct PortGroup {
    int32_t pair = -1;                            // pair index (specific IPs), else
    int32_t single = -1;                          // single-bit index (0.0.0.0 only)
    std::unordered_map<int32_t, int32_t> ip_bit;  // specific IP -> single-bit index
  };
  std::unordered_map<int64_t, PortGroup> groups;
  int32_t n_port_pairs = 0, n_port_single = 0;
  if (!group_specific.empty())
    for (int32_t i = 0; i < nc; ++i) {
      if (w->status_host[i] != STATUS_PENDING || !cand_ports[i]) continue;
      const int32_t pairs0 = n_port_pairs, single0 = n_port_single;
      std::vector<std::pair<int64_t, int32_t>> added_ips;  // undone if the candidate overflows
      std::vector<int64_t> added_groups;
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j)
        for_each_port(c, cands->cand_pods[j], [&](int32_t proto, int32_t port, int32_t ip) {
          const int64_t key = port_key(proto, port);
          auto ins = groups.emplace(key, PortGroup{});
          PortGroup& g = ins.first->second;
          if (ins.second) {
            added_groups.push_back(key);
            if (group_specific[key]) g.pair = n_port_pairs++;
            else g.single = n_port_single++;
          }
          // a read-only disk mount sets S only: it meets read-write mounts (W)
          // and never another read-only one
          if (ip != -1 && ip != kReadOnlyMount && g.ip_bit.emplace(ip, n_port_single).second) {
            ++n_port_single;
            added_ips.emplace_back(key, ip);
          }
        });
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
  std::vector<PortQuery> port_query;
  int32_t bit_query[64];
  for (int32_t& b : bit_query) b = -1;
  for (const auto& kv : groups) {
    const int32_t proto = static_cast<int32_t>(kv.first >> 32), port = static_cast<int32_t>(kv.first & 0xffffffff);
    const PortGroup& g = kv.second;
    const int32_t wbit = g.pair >= 0 ? bit_shift + 2 * g.pair : single_base + g.single;
    bit_query[wbit] = static_cast<int32_t>(port_query.size());
    port_query.push_back(PortQuery{proto, port, -1});
    if (g.pair >= 0 && proto >= kDiskProto) {  // a disk's S bit: the read-only mount's base conflicts
      bit_query[wbit + 1] = static_cast<int32_t>(port_query.size());
      port_query.push_back(PortQuery{proto, port, kReadOnlyMount});
    }
    for (const auto& ib : g.ip_bit) {
      bit_query[single_base + ib.second] = static_cast<int32_t>(port_query.size());
      port_query.push_back(PortQuery{proto, port, ib.first});
    }
  }
  // The state bits a spec's host ports {proto, port, ip}* set (absolute positions).
  auto port_mask = [&](const std::vector<int32_t>& ports) {
    uint64_t m = 0;
    for (size_t k = 0; k + 3 <= ports.size(); k += 3) {
      auto it = groups.find(port_key(ports[k], ports[k + 1]));
      if (it == groups.end()) continue;  // a fallback candidate's pod
      const PortGroup& g = it->second;
      if (g.pair < 0) {
        m |= 1ull << (single_base + g.single);
      } else if (ports[k + 2] == -1) {
        m |= 3ull << (bit_shift + 2 * g.pair);  // W and S
      } else if (ports[k + 2] == kReadOnlyMount) {
        m |= 2ull << (bit_shift + 2 * g.pair);  // S: a read-only disk mount
      } else {
        auto ib = g.ip_bit.find(ports[k + 2]);
        if (ib == g.ip_bit.end()) continue;
        m |= (2ull << (bit_shift + 2 * g.pair)) | (1ull << (single_base + ib->second));  // S and I(ip)
      }
    }
    return m;
  };

  // ---- shared scalar names of this call (extension records): a table row of
  // base free values per name, at most kExtScalarNames per call, the
  // candidates needing another one go to the reference path
  std::vector<int32_t> scal_names;
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING || !(cand_ext[i] & 2)) continue;
    int32_t need = 0;
    for (int j = 0; j < 2; ++j) {
      const int32_t nm = cand_sname[2 * i + j];
      need += nm != kNoName && std::find(scal_names.begin(), scal_names.end(), nm) == scal_names.end();
    }
    if (static_cast<int32_t>(scal_names.size()) + need > kExtScalarNames) {
      w->status_host[i] = SR_CAND_FALLBACK;
      continue;
    }
    for (int j = 0; j < 2; ++j) {
      const int32_t nm = cand_sname[2 * i + j];
      if (nm != kNoName && std::find(scal_names.begin(), scal_names.end(), nm) == scal_names.end())
        scal_names.push_back(nm);
    }
  }

  // ---- outcome bookkeeping for non-active candidates
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != SR_CAND_FALLBACK) continue;
    const int32_t g = cands->cand_global ? cands->cand_global[i] : i;
    if (w->first_fallback < 0 || g < w->first_fallback) w->first_fallback = g;
    w->fallback_pods += static_cast<uint64_t>(cands->cand_pod_off[i + 1] - cands->cand_pod_off[i]);
  }
  phase(1);

  // Active pods in candidate order: offsets per candidate, then a parallel fill.
  std::vector<int32_t>& active_pod = C.scratch.active_pod;  // cluster pod index
  std::vector<int32_t>& active_src = C.scratch.active_src;  // flat index into cand_pods
  std::vector<int32_t>& act_of = C.scratch.act_of;          // input candidate -> active candidate (-1)
  act_of.assign(static_cast<size_t>(nc), -1);
  for (int32_t i = 0, acc = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING) continue;
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    act_of[i] = static_cast<int32_t>(w->cand_src.size());
    w->cand_off.push_back(acc);
    w->cand_global.push_back(cands->cand_global ? cands->cand_global[i] : i);
    w->cand_src.push_back(i);
    w->max_cand_pods = std::max(w->max_cand_pods, e - b);
    acc += e - b;
  }
  const int32_t n_act = static_cast<int32_t>(w->cand_src.size());
  const int32_t na = n_act > 0 ? w->cand_off.back() + (cands->cand_pod_off[w->cand_src.back() + 1] -
                                                        cands->cand_pod_off[w->cand_src.back()]) : 0;
  w->cand_off.push_back(na);
  active_pod.resize(static_cast<size_t>(na));
  active_src.resize(static_cast<size_t>(na));
  const bool big = na > serial_pods();
  auto pfor = [&](size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
    if (big) parallel_for(n, grain, fn);
    else fn(0, n);
  };
  pfor(static_cast<size_t>(n_act), 256, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const int32_t i = w->cand_src[k], b = cands->cand_pod_off[i];
      for (int32_t q = w->cand_off[k]; q < w->cand_off[k + 1]; ++q) {
        active_pod[q] = cands->cand_pods[b + (q - w->cand_off[k])];
        active_src[q] = b + (q - w->cand_off[k]);
      }
    }
  });

  // ---- static specs, interned by content across calls.  Each pod's raw spec
  // words are gathered once into per-chunk buffers and hashed; the hash picks
  // one of kSpecShards persistent dictionaries, each scanned by one thread;
  // specs never seen before get their ids serially afterwards (in shard,
  // first-occurrence order: independent of the thread count) and are
  // canonicalised in parallel.
  EncoderCache::Scratch& X = C.scratch;
  std::vector<int32_t>& pod_spec = X.pod_spec;
  std::vector<uint64_t>& spec_hash = X.spec_hash;
  std::vector<uint8_t>& spec_shard = X.spec_shard;
  pod_spec.assign(static_cast<size_t>(na), 0);
  spec_hash.resize(static_cast<size_t>(na));
  spec_shard.assign(static_cast<size_t>(na), 0xff);
  constexpr size_t kChunk = 2048;
  const size_t n_chunks = (static_cast<size_t>(na) + kChunk - 1) / kChunk;
  std::vector<std::vector<int32_t>>& spec_words = X.spec_words;
  if (spec_words.size() < n_chunks) spec_words.resize(n_chunks);
  std::vector<uint32_t>& spec_woff = X.spec_woff;
  spec_woff.resize(static_cast<size_t>(na));
  // per chunk and shard, the chunk's pods of the shard (in order): each shard
  // then scans only its own pods
  std::vector<std::vector<int32_t>>& chunk_shard = X.chunk_shard;  // [chunk * kSpecShards + shard]
  if (chunk_shard.size() < n_chunks * kSpecShards) chunk_shard.resize(n_chunks * kSpecShards);
  pfor(n_chunks, 1, [&](size_t lo, size_t hi) {
    for (size_t ch = lo; ch < hi; ++ch) {
      // fill stack-held vectors (swapped in and out): the vector headers in
      // spec_words / chunk_shard share cache lines with the neighbouring
      // chunks' headers, which other threads update
      std::vector<int32_t> buf;
      buf.swap(spec_words[ch]);
      buf.clear();
      std::vector<int32_t> mine[kSpecShards];
      for (size_t sh = 0; sh < kSpecShards; ++sh) {
        mine[sh].swap(chunk_shard[ch * kSpecShards + sh]);
        mine[sh].clear();
      }
      const size_t q1 = std::min(static_cast<size_t>(na), (ch + 1) * kChunk);
      for (size_t q = ch * kChunk; q < q1; ++q) {
        const size_t b0 = buf.size();
        spec_woff[q] = static_cast<uint32_t>(b0);
        const int32_t pod = active_pod[q];
        if (stamps && stamps[pod] != 0 && C.pod_memo[static_cast<size_t>(pod)].stamp_spec == stamps[pod]) {
          pod_spec[q] = C.pod_memo[static_cast<size_t>(pod)].spec;  // a global id already
          spec_shard[q] = 0xfe;
          continue;
        }
        if (!has_static_spec(c, P, pod)) continue;  // spec 0
        for_each_spec_word(c, P, pod, [&](int32_t x) { buf.push_back(x); });
        const uint64_t h = hash_words(buf.data() + b0, buf.size() - b0);
        spec_hash[q] = h;
        const size_t sh = static_cast<size_t>(((h >> 32) * kSpecShards) >> 32);
        spec_shard[q] = static_cast<uint8_t>(sh);
        // known specs resolve here, read-only, while the words are hot; the
        // shard pass below interns the rest
        const int32_t local = C.spec_shards[sh].dict.find(buf.data() + b0, buf.size() - b0, h);
        if (local >= 0) pod_spec[q] = local;
        else mine[sh].push_back(static_cast<int32_t>(q));
      }
      buf.swap(spec_words[ch]);
      for (size_t sh = 0; sh < kSpecShards; ++sh) mine[sh].swap(chunk_shard[ch * kSpecShards + sh]);
    }
  });
  phase(9);
  auto words_of = [&](size_t q, size_t* n) {
    const std::vector<int32_t>& buf = spec_words[q / kChunk];
    const size_t e = (q + 1) % kChunk == 0 || q + 1 == static_cast<size_t>(na) ? buf.size() : spec_woff[q + 1];
    *n = e - spec_woff[q];
    return buf.data() + spec_woff[q];
  };
  std::vector<std::vector<int32_t>> shard_new(kSpecShards);  // first pod of each new local id
  pfor(kSpecShards, 1, [&](size_t lo, size_t hi) {
    for (size_t sh = lo; sh < hi; ++sh) {
      EncoderCache::SpecShard& S = C.spec_shards[sh];
      shard_new[sh].clear();
      for (size_t ch = 0; ch < n_chunks; ++ch)
        for (int32_t q : chunk_shard[ch * kSpecShards + sh]) {
          size_t n = 0;
          const int32_t* p = words_of(static_cast<size_t>(q), &n);
          bool ins = false;
          const int32_t local = S.dict.intern(p, n, spec_hash[q], &ins);
          if (ins) {
            S.global.push_back(-1);
            shard_new[sh].push_back(q);
          }
          pod_spec[q] = local;  // local for now
        }
    }
  });
  phase(14);
  std::vector<int32_t> new_spec_pod;  // representative pod of each new spec
  const int32_t spec0 = static_cast<int32_t>(C.spec.size());
  for (size_t sh = 0; sh < kSpecShards; ++sh)
    for (int32_t q : shard_new[sh]) {
      EncoderCache::SpecShard& S = C.spec_shards[sh];
      S.global[pod_spec[q]] = spec0 + static_cast<int32_t>(new_spec_pod.size());
      new_spec_pod.push_back(active_pod[q]);
    }
  C.last_new_specs = static_cast<int32_t>(new_spec_pod.size());
  C.last_memo_hits = memo_hits.load(std::memory_order_relaxed);
  const int32_t n_spec_ids = spec0 + static_cast<int32_t>(new_spec_pod.size());
  const bool combos = anti.active || aff.active || sdyn.active;
  // keys present in this call (pods without inter-pod terms: the spec id),
  // flagged here with the global ids; read first: a shared line written by
  // every thread would bounce
  std::vector<uint8_t>& key_seen = X.key_seen;
  key_seen.assign(static_cast<size_t>(n_spec_ids), 0);
  pfor(static_cast<size_t>(na), 4096, [&](size_t lo, size_t hi) {
    for (size_t q = lo; q < hi; ++q) {
      const uint8_t sh = spec_shard[q];
      const int32_t g = sh == 0xff ? 0 : sh == 0xfe ? pod_spec[q] : C.spec_shards[sh].global[pod_spec[q]];
      pod_spec[q] = g;
      if (stamps && sh != 0xfe) {
        const int32_t pod = active_pod[q];
        if (stamps[pod] != 0) {
          C.pod_memo[static_cast<size_t>(pod)].spec = g;
          C.pod_memo[static_cast<size_t>(pod)].stamp_spec = stamps[pod];
        }
      }
      if (!combos && !__atomic_load_n(&key_seen[g], __ATOMIC_RELAXED)) __atomic_store_n(&key_seen[g], uint8_t(1), __ATOMIC_RELAXED);
    }
  });
  if (!new_spec_pod.empty()) {
    std::vector<SpecDraft> drafts(new_spec_pod.size());
    auto draft = [&](size_t lo, size_t hi) {
      for (size_t k = lo; k < hi; ++k) draft_spec(c, new_spec_pod[k], &drafts[k]);
    };
    if (drafts.size() > 256) parallel_for(drafts.size(), 64, draft);
    else draft(0, drafts.size());
    C.spec.resize(static_cast<size_t>(spec0) + drafts.size());
    std::vector<int32_t> ids;
    for (size_t k = 0; k < drafts.size(); ++k) {  // requirement ids: serial
      SpecDraft& d = drafts[k];
      SpecInfo& sp = C.spec[static_cast<size_t>(spec0) + k];
      sp.flags = d.flags;
      int32_t n_sel = 0;
      for (size_t i = 0; i < d.sel.size(); i += 1 + static_cast<size_t>(d.sel[i])) ++n_sel;
      intern_groups(C.req_dict, d.sel.data(), n_sel, sp.sel, nullptr);
      sp.n_terms = d.n_terms;
      for (size_t i = 0, t = 0; t < static_cast<size_t>(d.n_terms); ++t) {
        size_t used = 0;
        intern_groups(C.req_dict, d.terms.data() + i + 1, d.terms[i], ids, &used);
        sp.terms.push_back(static_cast<int32_t>(ids.size()));
        sp.terms.insert(sp.terms.end(), ids.begin(), ids.end());
        i += 1 + used;
      }
      sp.tol.swap(d.tol);
      sp.ports.swap(d.ports);
      sp.scalars.swap(d.scalars);
      sp.spread.swap(d.spread);
      int32_t n_vsel = 0;
      for (size_t i = 0; i < d.vsel.size(); i += 1 + static_cast<size_t>(d.vsel[i])) ++n_vsel;
      intern_groups(C.req_dict, d.vsel.data(), n_vsel, sp.vsel, nullptr);
      for (const std::vector<int32_t>& pv : d.vpv) {  // canonical {n terms, per term {n, requirement ids}}
        std::vector<int32_t> words(1, pv[0]);
        for (size_t i = 1, t = 0; t < static_cast<size_t>(pv[0]); ++t) {
          size_t used = 0;
          intern_groups(C.req_dict, pv.data() + i + 1, pv[i], ids, &used);
          words.push_back(static_cast<int32_t>(ids.size()));
          words.insert(words.end(), ids.begin(), ids.end());
          i += 1 + used;
        }
        sp.vpv.push_back(C.pvsel_dict.intern(words));
      }
      std::sort(sp.vpv.begin(), sp.vpv.end());
      sp.vpv.erase(std::unique(sp.vpv.begin(), sp.vpv.end()), sp.vpv.end());
    }
  }
  for (size_t id = C.spec_req_off.size() - 1; id < C.spec.size(); ++id) {
    const SpecInfo& sp = C.spec[id];
    C.spec_req.insert(C.spec_req.end(), sp.sel.begin(), sp.sel.end());
    for (size_t i = 0; i < sp.terms.size(); i += 1 + static_cast<size_t>(sp.terms[i]))
      C.spec_req.insert(C.spec_req.end(), sp.terms.begin() + i + 1, sp.terms.begin() + i + 1 + sp.terms[i]);
    C.spec_req.insert(C.spec_req.end(), sp.vsel.begin(), sp.vsel.end());
    for (int32_t pv : sp.vpv) {  // the PV selectors' requirements
      const int32_t* w = C.pvsel_dict.data(pv);
      for (size_t i = 1, t = 0; t < static_cast<size_t>(w[0]); ++t) {
        C.spec_req.insert(C.spec_req.end(), w + i + 1, w + i + 1 + w[i]);
        i += 1 + static_cast<size_t>(w[i]);
      }
    }
    C.spec_req_off.push_back(static_cast<uint32_t>(C.spec_req.size()));
  }
  phase(7);

  // ---- class keys: the static spec, plus (with inter-pod affinity) the pod's
  // anti-affinity term ids and affinity set of this call.  Pods without either
  // use their spec id as key.
  std::vector<int32_t>& pod_key_buf = X.pod_key;
  std::vector<int32_t> key_spec;               // keys >= n_spec_ids: spec of the combined key,
  std::vector<std::vector<int32_t>> key_anti;  // ... its anti-affinity term ids
  std::vector<int32_t> key_aff;                // ... and its affinity code (AffTerms::pod_code; 1 << 30: domain path)
  std::vector<int32_t> key_sdm;                // ... and its device-planned spread constraints (SpreadDyn::dmask)
  if (combos) {
    pod_key_buf.resize(static_cast<size_t>(na));
    WordDict combo;
    std::vector<int32_t> kw;
    for (int32_t q = 0; q < na; ++q) {
      const int32_t j = active_src[q] - anti.base;
      const int32_t n_ids = anti.active ? anti.pod_off[j + 1] - anti.pod_off[j] : 0;
      const int32_t code = aff.active ? aff.pod_code[active_src[q] - aff.base] : -1;
      const int32_t sdm = spread_dm(active_src[q]);
      if (n_ids == 0 && code < 0 && sdm == 0) {
        pod_key_buf[q] = pod_spec[q];
        continue;
      }
      const int32_t kcode = code < 0 ? code : code | (aff_dyn(active_src[q]) ? 1 << 30 : 0);
      kw.assign(1, pod_spec[q]);
      kw.push_back(kcode);
      kw.push_back(sdm);
      if (n_ids) kw.insert(kw.end(), anti.pod_ids.begin() + anti.pod_off[j], anti.pod_ids.begin() + anti.pod_off[j + 1]);
      bool ins = false;
      const int32_t id = combo.intern(kw, &ins);
      if (ins) {
        key_spec.push_back(pod_spec[q]);
        key_aff.push_back(kcode);
        key_sdm.push_back(sdm);
        key_anti.emplace_back(kw.begin() + 3, kw.end());
      }
      pod_key_buf[q] = n_spec_ids + id;
    }
  }
  const std::vector<int32_t>& pod_key = combos ? pod_key_buf : pod_spec;
  // distinct keys of this call, in key order: flags set in parallel, slots serially
  const size_t n_key_ids = static_cast<size_t>(n_spec_ids) + key_spec.size();
  if (combos) {
    key_seen.assign(n_key_ids, 0);
    pfor(static_cast<size_t>(na), 8192, [&](size_t lo, size_t hi) {
      for (size_t q = lo; q < hi; ++q) {
        uint8_t* f = &key_seen[pod_key[q]];
        if (!__atomic_load_n(f, __ATOMIC_RELAXED)) __atomic_store_n(f, uint8_t(1), __ATOMIC_RELAXED);
      }
    });
  }
  std::vector<int32_t>& key_slot = X.key_slot;
  key_slot.assign(n_key_ids, -1);
  std::vector<int32_t> keys;
  for (size_t k = 0; k < n_key_ids; ++k)
    if (key_seen[k]) {
      key_slot[k] = static_cast<int32_t>(keys.size());
      keys.push_back(static_cast<int32_t>(k));
    }

  // ---- per key: untolerated taints (cached per spec and static view), host
  // ports of this call, anti-affinity atoms; the requirement atoms in use
  if (C.untol_gen != C.static_gen) {
    C.untol_dict.clear();
    C.untol_gen = C.static_gen;
  }
  const int32_t n_taints = static_cast<int32_t>(C.taints.size());
  std::vector<int32_t> untol_scratch;
  auto untol_of = [&](int32_t spec_id) {
    SpecInfo& sp = C.spec[spec_id];
    if (sp.untol_gen != C.static_gen) {
      untol_scratch.clear();
      for (int32_t t = 0; t < n_taints; ++t)  // spec 0 (no tolerations) tolerates nothing
        if (!tolerates(sp.tol, c->id_empty, C.taints[t])) untol_scratch.push_back(t);
      sp.untol = C.untol_dict.intern(untol_scratch);
      sp.untol_gen = C.static_gen;
    }
    return sp.untol;
  };
  std::vector<int32_t> req_atom(C.req_dict.size(), -1), used_reqs;
  auto use_req = [&](int32_t r) {
    if (req_atom[r] < 0) {
      req_atom[r] = static_cast<int32_t>(used_reqs.size());
      used_reqs.push_back(r);
    }
  };
  // scalar resource checks of this call: one atom per distinct (name, request)
  std::vector<std::pair<int64_t, int64_t>> scalar_query;
  std::map<std::pair<int64_t, int64_t>, int32_t> scalar_index;
  auto scalar_atom_index = [&](int64_t name, int64_t req) {
    auto ins = scalar_index.emplace(std::make_pair(name, req), static_cast<int32_t>(scalar_query.size()));
    if (ins.second) scalar_query.emplace_back(name, req);
    return ins.first->second;
  };
  // topology spread of this call: one atom per spec carrying constraints and
  // set of device-planned constraints
  std::vector<std::pair<int32_t, int32_t>> spread_query;
  std::unordered_map<int64_t, int32_t> spread_index;
  auto spread_atom_index = [&](int32_t spec_id, int32_t dm) {
    auto ins = spread_index.emplace(static_cast<int64_t>(spec_id) << 32 | static_cast<uint32_t>(dm),
                                    static_cast<int32_t>(spread_query.size()));
    if (ins.second) spread_query.emplace_back(spec_id, dm);
    return ins.first->second;
  };
  auto key_dm = [&](int32_t k) { return k < n_spec_ids ? 0 : key_sdm[k - n_spec_ids]; };
  // PV selectors with several terms (VolumeBinding): one atom each
  std::vector<int32_t> pvsel_atom(C.pvsel_dict.size(), -1), used_pvsel;
  for (int32_t k : keys) {
    const int32_t id = k < n_spec_ids ? k : key_spec[k - n_spec_ids];
    for (uint32_t i = C.spec_req_off[id]; i < C.spec_req_off[id + 1]; ++i) use_req(C.spec_req[i]);
    for (int32_t pv : C.spec[id].vpv)
      if (pvsel_atom[pv] < 0) {
        pvsel_atom[pv] = static_cast<int32_t>(used_pvsel.size());
        used_pvsel.push_back(pv);
      }
    const std::vector<int64_t>& sc = C.spec[id].scalars;
    for (size_t i = 0; i + 2 <= sc.size(); i += 2) scalar_atom_index(sc[i], sc[i + 1]);
    if (!C.spec[id].spread.empty()) spread_atom_index(id, key_dm(k));
  }
  const int32_t n_reqs = static_cast<int32_t>(used_reqs.size());
  const int32_t n_ports = static_cast<int32_t>(port_query.size());
  const int32_t n_scalars = static_cast<int32_t>(scalar_query.size());
  const int32_t A_REQ = 1, A_TAINT = 1 + n_reqs, A_PORT = A_TAINT + n_taints;
  const int32_t n_spreads = static_cast<int32_t>(spread_query.size());
  const int32_t A_SCALAR = A_PORT + n_ports;
  const int32_t A_SPREAD = A_SCALAR + n_scalars;  // scalar and spread atoms: the class's `sc_` list
  const int32_t A_ANTI = A_SPREAD + n_spreads;  // DA(t) at A_ANTI + 2t, DB(t) at A_ANTI + 2t + 1
  const int32_t A_AFF = A_ANTI + 2 * anti.n_terms;  // SAT(S) at A_AFF + 2s, KEYS(S) at A_AFF + 2s + 1
  const int32_t A_VOL = A_AFF + 2 * aff.n_sets;  // PV selector atoms
  const int32_t A_COMP = A_VOL + static_cast<int32_t>(used_pvsel.size());
  // Composite atoms, one per distinct untolerated-taint set U of the pods:
  // atom 0 AND NOT (OR of U's taint atoms) -- the pod-count check and
  // TaintToleration / NodeUnschedulable in one row, so a class program opens
  // with a single AND instead of 1 + |U| operations.
  std::vector<int32_t> comp_of, comp_sets;
  auto comp_atom = [&](int32_t u) {
    if (C.untol_dict.len(u) == 0) return 0;  // tolerates every taint: the pod-count atom alone
    if (static_cast<size_t>(u) >= comp_of.size()) comp_of.resize(static_cast<size_t>(u) + 1, -1);
    if (comp_of[u] < 0) {
      comp_of[u] = static_cast<int32_t>(comp_sets.size());
      comp_sets.push_back(u);
    }
    return A_COMP + comp_of[u];
  };
  phase(2);

  // ---- classes: one program per distinct signature.  A spec without host
  // ports and without inter-pod terms has a signature that only depends on
  // the spec and the static view {flags, selector ids, terms, untolerated
  // set}: it is interned once per static view (SpecInfo::psig) and its class
  // found by one table lookup per call.  Other keys add this call's host-port
  // bits, anti-affinity atoms and affinity atom and are interned per call.
  if (C.psig_gen != C.static_gen) {
    C.psig_dict.clear();
    C.psig_gen = C.static_gen;
  }
  std::vector<int32_t> sig, da, db, call_class, scq;
  auto static_sig = [&](const SpecInfo& sp, int32_t untol, std::vector<int32_t>& out) {
    out.clear();
    out.push_back(sp.flags);
    out.push_back(static_cast<int32_t>(sp.sel.size()));
    out.insert(out.end(), sp.sel.begin(), sp.sel.end());
    out.push_back(sp.n_terms);
    out.insert(out.end(), sp.terms.begin(), sp.terms.end());
    out.push_back(static_cast<int32_t>(sp.vsel.size()));
    out.insert(out.end(), sp.vsel.begin(), sp.vsel.end());
    out.push_back(static_cast<int32_t>(sp.vpv.size()));
    out.insert(out.end(), sp.vpv.begin(), sp.vpv.end());
    out.push_back(untol);
  };
  w->cls_prog_off.push_back(0);
  auto emit = [&](int32_t atom, int32_t kind) { w->cls_prog.push_back(atom << 2 | kind); };
  // program: AND atoms, AND-NOT atoms, then the ORed terms (TERM_START opens a
  // term, TERM_AND extends it); an impossible class ANDs atom 0 with its
  // complement.  `sw` = static signature words.
  auto emit_class = [&](const int32_t* sw, uint64_t ports, const std::vector<int32_t>* da_, const std::vector<int32_t>* db_,
                        int32_t aff_atom, const std::vector<int32_t>* sc_ = nullptr) {
    const int32_t flags = sw[0], n_sel = sw[1];
    const int32_t* sel = sw + 2;
    const int32_t* tp = sel + n_sel;
    const int32_t n_terms = *tp++;
    const int32_t* term_words = tp;
    for (int32_t k = 0; k < n_terms; ++k) tp += 1 + *tp;
    const int32_t n_vsel = *tp++;
    const int32_t* vsel = tp;
    tp += n_vsel;
    const int32_t n_vpv = *tp++;
    const int32_t* vpv = tp;
    tp += n_vpv;
    const int32_t untol = *tp;
    emit(comp_atom(untol), PROG_AND);  // len(pods)+1 <= allowed pods, untolerated taints
    for (int32_t k = 0; k < n_sel; ++k) emit(A_REQ + req_atom[sel[k]], PROG_AND);
    for (int32_t k = 0; k < n_vsel; ++k) emit(A_REQ + req_atom[vsel[k]], PROG_AND);  // VolumeZone, PV affinity
    for (int32_t k = 0; k < n_vpv; ++k) emit(A_VOL + pvsel_atom[vpv[k]], PROG_AND);
    for (uint64_t m = ports; m; m &= m - 1) {  // the base UsedPorts conflicting with each host port it asks for
      const int32_t b = __builtin_ctzll(m);
      if (bit_query[b] >= 0) emit(A_PORT + bit_query[b], PROG_ANDNOT);
    }
    if (sc_)
      for (int32_t q : *sc_) emit(A_SCALAR + q, PROG_AND);  // alloc[s] >= request + requested[s]; spread rows
    if (da_)
      for (int32_t t : *da_) emit(A_ANTI + 2 * t, PROG_ANDNOT);  // anti-affinity base conflicts
    if (db_)
      for (int32_t t : *db_) emit(A_ANTI + 2 * t + 1, PROG_ANDNOT);
    if (aff_atom >= 0) emit(aff_atom, PROG_AND);
    if ((flags & CLS_IMPOSSIBLE) || aff_atom == -2) {
      emit(0, PROG_ANDNOT);
    } else {
      for (int32_t k = 0; k < n_terms; ++k) {
        const int32_t n = *term_words++;
        for (int32_t i = 0; i < n; ++i)
          emit(A_REQ + req_atom[term_words[i]], i == 0 ? PROG_TERM_START : PROG_TERM_AND);
        term_words += n;
      }
    }
    w->cls_prog_off.push_back(static_cast<int32_t>(w->cls_prog.size()));
    return w->n_classes++;
  };
  WordDict class_dict;
  std::vector<int32_t> key_class(keys.size());
  std::vector<uint64_t> key_ports(keys.size(), 0);
  std::vector<int32_t>& psig_class = X.psig_class;  // static signature -> class of this call
  psig_class.assign(C.psig_dict.size(), -1);
  for (size_t ki = 0; ki < keys.size(); ++ki) {
    const int32_t k = keys[ki];
    const int32_t spec_id = k < n_spec_ids ? k : key_spec[k - n_spec_ids];
    SpecInfo& sp = C.spec[spec_id];
    const int32_t untol = untol_of(spec_id);
    if (k < n_spec_ids && sp.ports.empty() && sp.scalars.empty() && sp.spread.empty()) {
      if (sp.psig_gen != C.static_gen) {
        static_sig(sp, untol, sig);
        sp.psig = C.psig_dict.intern(sig);
        sp.psig_gen = C.static_gen;
      }
      if (static_cast<size_t>(sp.psig) >= psig_class.size()) psig_class.resize(C.psig_dict.size(), -1);
      int32_t& cls = psig_class[sp.psig];
      if (cls < 0) cls = emit_class(C.psig_dict.data(sp.psig), 0, nullptr, nullptr, -1);
      key_class[ki] = cls;
      continue;
    }
    const uint64_t ports = port_mask(sp.ports);
    key_ports[ki] = ports;
    da.clear();
    db.clear();
    // pod affinity: SAT(S); with an empty pair map KEYS(S) for a pod matching
    // its own terms, nothing otherwise (-2)
    int32_t aff_atom = -1;
    if (k >= n_spec_ids && key_aff[k - n_spec_ids] >= 0) {
      const int32_t code = key_aff[k - n_spec_ids] & ~(1 << 30), set = code >> 1;
      if (key_aff[k - n_spec_ids] & (1 << 30)) aff_atom = A_AFF + 2 * set + 1;  // domain path: the device adds SAT
      else aff_atom = !aff.map_empty[set] ? A_AFF + 2 * set : (code & 1) ? A_AFF + 2 * set + 1 : -2;
    }
    if (k >= n_spec_ids)
      for (int32_t id : key_anti[k - n_spec_ids]) {
        const int32_t t = id >> 1;
        if (id & 1) {  // it has t: refuses domains hosting pods t selects
          if (anti.db_any[t]) db.push_back(t);
        } else {  // t selects it: refused by domains hosting pods that have t
          if (anti.da_any[t]) da.push_back(t);
        }
      }
    scq.clear();
    for (size_t i = 0; i + 2 <= sp.scalars.size(); i += 2) scq.push_back(scalar_atom_index(sp.scalars[i], sp.scalars[i + 1]));
    if (!sp.spread.empty()) scq.push_back(n_scalars + spread_atom_index(spec_id, key_dm(k)));
    static_sig(sp, untol, sig);
    const size_t n_static = sig.size();
    sig.push_back(static_cast<int32_t>(scq.size()));
    sig.insert(sig.end(), scq.begin(), scq.end());
    sig.push_back(static_cast<int32_t>(ports & 0xffffffffu));
    sig.push_back(static_cast<int32_t>(ports >> 32));
    sig.push_back(static_cast<int32_t>(da.size()));
    sig.insert(sig.end(), da.begin(), da.end());
    sig.push_back(static_cast<int32_t>(db.size()));
    sig.insert(sig.end(), db.begin(), db.end());
    sig.push_back(aff_atom);
    bool ins = false;
    const int32_t id = class_dict.intern(sig, &ins);
    if (ins) {
      sig.resize(n_static);
      call_class.push_back(emit_class(sig.data(), ports, &da, &db, aff_atom, &scq));
    }
    key_class[ki] = call_class[id];
  }
  // domain path rows, named by no class program: each domain of a table key
  // slot, then each term's base row of the sets planned there
  const int32_t A_DOM = A_COMP + static_cast<int32_t>(comp_sets.size());
  int32_t n_dom_rows = 0;
  for (size_t k = 0; k < dk.key.size(); ++k)
    if (!dk.node_local[k]) {
      w->dk_row[k] = A_DOM + n_dom_rows;
      n_dom_rows += dk.n_dom[k];
    }
  const int32_t A_TERM = A_DOM + n_dom_rows;
  std::vector<int32_t> term_atom(static_cast<size_t>(aff.n_sets), -1);
  int32_t n_term_rows = 0;
  for (int32_t s2 = 0; s2 < static_cast<int32_t>(aff.set_dyn.size()); ++s2)
    if (aff.set_dyn[s2]) {
      term_atom[s2] = A_TERM + n_term_rows;
      n_term_rows += static_cast<int32_t>(aff.set_slots[s2].size());
    }
  w->n_atoms = A_TERM + n_term_rows;
  phase(3);

  // ---- atom rows: pod count (state), requirements and taints (static view,
  // requirement rows cached), base port conflicts, anti-affinity, composites
  w->atoms.assign(static_cast<size_t>(w->n_atoms) * Wp, 0);
  uint64_t* A = w->atoms.data();
  std::copy(C.podcount_row.begin(), C.podcount_row.end(), A);
  {
    if (C.req_rows.size() < C.req_dict.size()) {
      C.req_rows.resize(C.req_dict.size());
      C.req_row_gen.resize(C.req_dict.size(), ~0ull);
    }
    std::vector<int32_t> stale;
    for (int32_t r : used_reqs)
      if (C.req_row_gen[r] != C.static_gen) stale.push_back(r);
    std::vector<const std::vector<int32_t>*> cols(stale.size(), nullptr);
    std::vector<std::array<const std::vector<int32_t>*, 4>> zcols(stale.size());
    for (size_t i = 0; i < stale.size(); ++i) {  // label columns: serial (the cache is not thread-safe)
      const int32_t* rw = C.req_dict.data(stale[i]);
      if (rw[0] != REQ_FIELD) cols[i] = &label_column(C, snap, rw[1]);
      for (int z = 0; z < 4; ++z)
        zcols[i][z] = rw[0] == REQ_ZONE && rw[3 + z] >= 0 ? &label_column(C, snap, rw[3 + z]) : nullptr;
    }
    auto build = [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        const int32_t r = stale[i];
        build_req_row(C, snap, c, C.req_dict.data(r), C.req_dict.len(r), cols[i], C.req_rows[r], zcols[i].data());
        C.req_row_gen[r] = C.static_gen;
      }
    };
    if (stale.size() > 8 && n_spot > 1024) parallel_for(stale.size(), 1, build);
    else build(0, stale.size());
    for (int32_t i = 0; i < n_reqs; ++i)
      std::copy(C.req_rows[used_reqs[i]].begin(), C.req_rows[used_reqs[i]].end(),
                A + static_cast<size_t>(A_REQ + i) * Wp);
    // PV selectors: OR over the terms of the AND of their requirement rows
    for (size_t i = 0; i < used_pvsel.size(); ++i) {
      const int32_t* pw = C.pvsel_dict.data(used_pvsel[i]);
      uint64_t* row = A + static_cast<size_t>(A_VOL + static_cast<int32_t>(i)) * Wp;
      std::vector<uint64_t> t(static_cast<size_t>(Wp));
      for (size_t j = 1, term = 0; term < static_cast<size_t>(pw[0]); ++term) {
        for (int32_t n = 0; n < n_spot; ++n) t[n >> 6] |= 1ull << (n & 63);
        for (int32_t g = 0; g < pw[j]; ++g) {
          const std::vector<uint64_t>& rr = C.req_rows[pw[j + 1 + g]];
          for (int32_t x = 0; x < Wp; ++x) t[x] &= rr[x];
        }
        for (int32_t x = 0; x < Wp; ++x) row[x] |= t[x];
        std::fill(t.begin(), t.end(), 0);
        j += 1 + static_cast<size_t>(pw[j]);
      }
    }
  }
  std::copy(C.taint_rows.begin(), C.taint_rows.end(), A + static_cast<size_t>(A_TAINT) * Wp);
  if (n_ports > 0) port_conflict_rows(C, snap, port_query.data(), n_ports, Wp, A + static_cast<size_t>(A_PORT) * Wp);
  // NodeResourcesFit's ScalarResources loop against the base snapshot:
  // alloc[s] < request + requested[s] fails (a node without s allocates 0)
  // (volume limit keys under negative names: the node's limit, or unlimited,
  // against its unique attachable volumes of the key plus the pod's count)
  for (int32_t q = 0; q < n_scalars; ++q)
    scalar_query_row(snap, scalar_query[q].first, scalar_query[q].second, A + static_cast<size_t>(A_SCALAR + q) * Wp);
  // PodTopologySpread against the base snapshot, over the spec's NodeAffinity
  // row (nodeSelector AND, OR of the required terms) built from its requirement rows
  for (int32_t q = 0; q < n_spreads; ++q) {
    const SpecInfo& sp = C.spec[spread_query[q].first];
    std::vector<uint64_t> aff_row(static_cast<size_t>(Wp), (sp.flags & CLS_IMPOSSIBLE) ? 0ull : ~0ull);
    for (int32_t r : sp.sel)
      for (int32_t i = 0; i < Wp; ++i) aff_row[i] &= A[static_cast<size_t>(A_REQ + req_atom[r]) * Wp + i];
    if ((sp.flags & CLS_AFF_REQUIRED) && !(sp.flags & CLS_IMPOSSIBLE)) {
      std::vector<uint64_t> any(static_cast<size_t>(Wp), 0), t_row(static_cast<size_t>(Wp));
      for (size_t i = 0; i < sp.terms.size(); i += 1 + static_cast<size_t>(sp.terms[i])) {
        std::fill(t_row.begin(), t_row.end(), ~0ull);
        for (int32_t j = 0; j < sp.terms[i]; ++j) {
          const uint64_t* rr = A + static_cast<size_t>(A_REQ + req_atom[sp.terms[i + 1 + j]]) * Wp;
          for (int32_t x = 0; x < Wp; ++x) t_row[x] &= rr[x];
        }
        for (int32_t x = 0; x < Wp; ++x) any[x] |= t_row[x];
      }
      for (int32_t x = 0; x < Wp; ++x) aff_row[x] &= any[x];
    }
    spread_row(six, sp.spread.data(), aff_row.data(), static_cast<uint32_t>(spread_query[q].second),
               A + static_cast<size_t>(A_SPREAD + q) * Wp, spread_keep.get(), A_SPREAD + q);
  }
  for (int32_t t = 0; t < anti.n_terms; ++t) {
    std::copy_n(&anti.da[static_cast<size_t>(t) * Wp], Wp, A + static_cast<size_t>(A_ANTI + 2 * t) * Wp);
    std::copy_n(&anti.db[static_cast<size_t>(t) * Wp], Wp, A + static_cast<size_t>(A_ANTI + 2 * t + 1) * Wp);
  }
  for (int32_t t = 0; t < aff.n_sets; ++t) {
    std::copy_n(&aff.sat[static_cast<size_t>(t) * Wp], Wp, A + static_cast<size_t>(A_AFF + 2 * t) * Wp);
    std::copy_n(&aff.keys[static_cast<size_t>(t) * Wp], Wp, A + static_cast<size_t>(A_AFF + 2 * t + 1) * Wp);
  }
  composite_rows(C, comp_sets, A_COMP, Wp, A);  // atom 0 AND NOT (any taint of the set)
  for (size_t k = 0; k < dk.key.size(); ++k)
    if (!dk.node_local[k])
      for (int32_t n = 0; n < n_spot; ++n)
        if (dk.dom[k][n] >= 0)
          A[static_cast<size_t>(w->dk_row[k] + dk.dom[k][n]) * Wp + (n >> 6)] |= 1ull << (n & 63);
  for (int32_t s2 = 0; s2 < static_cast<int32_t>(term_atom.size()); ++s2)
    if (term_atom[s2] >= 0)
      std::copy(aff.term_rows[s2].begin(), aff.term_rows[s2].end(), A + static_cast<size_t>(term_atom[s2]) * Wp);
  // domain path: key slots, sets, and the candidates' pod records
  const bool dyn_any = !anti.cand_dyn.empty() || !aff.cand_dyn.empty() || !sdyn.cand_dyn.empty();
  if (dyn_any) {
    w->n_dk = static_cast<int32_t>(dk.key.size());
    w->sp_tab = sdyn.tab;
    for (const auto& d : dk.dom) w->dk_dom.insert(w->dk_dom.end(), d.begin(), d.end());
    constexpr int32_t kInfo = 2 + 2 * kDynTerms;
    w->ds_info.assign(static_cast<size_t>(std::max(1, aff.n_sets)) * kInfo, 0);
    for (int32_t s2 = 0; s2 < static_cast<int32_t>(term_atom.size()); ++s2) {
      if (term_atom[s2] < 0) continue;
      int32_t* info = &w->ds_info[static_cast<size_t>(s2) * kInfo];
      info[0] = static_cast<int32_t>(aff.set_slots[s2].size());
      info[1] = aff.map_empty[s2];
      for (int32_t t = 0; t < info[0]; ++t) {
        info[2 + 2 * t] = aff.set_slots[s2][t];
        info[3 + 2 * t] = term_atom[s2] + t;
      }
    }
    const int32_t n_act = static_cast<int32_t>(w->cand_src.size());
    w->dyn_cand.assign(static_cast<size_t>(n_act), -1);
    for (int32_t k = 0; k < n_act; ++k) {
      const int32_t i = w->cand_src[k];
      const bool dyn = (!anti.cand_dyn.empty() && anti.cand_dyn[i]) || (!aff.cand_dyn.empty() && aff.cand_dyn[i]) ||
                       (!sdyn.cand_dyn.empty() && sdyn.cand_dyn[i]);
      if (!dyn) continue;
      w->dyn_cand[k] = static_cast<int32_t>(w->dyn_pod.size() / kDynU64);
      for (int32_t q = w->cand_off[k]; q < w->cand_off[k + 1]; ++q) {
        const int32_t j = active_src[q];
        for (int32_t sl = 0; sl < kDomKeys; ++sl)
          for (int g = 0; g < kDynG; ++g)
            w->dyn_pod.push_back(anti.amask.empty()
                                     ? 0
                                     : anti.amask[(static_cast<size_t>(j - anti.base) * kDomKeys + sl) * kDynG + g]);
        uint64_t any_mm = 0;
        for (int g = 0; g < kDynG; ++g) {
          const uint64_t mm = aff.mmask.empty() ? 0 : aff.mmask[static_cast<size_t>(j - aff.base) * kDynG + g];
          any_mm |= mm;
          w->dyn_pod.push_back(mm);
        }
        w->dyn_pod.push_back(any_mm != 0 ? static_cast<uint64_t>(aff.pod_code[j - aff.base]) : ~0ull);
        if (!sdyn.cand_dyn.empty() && sdyn.cand_dyn[i]) {
          const uint64_t* sw = &sdyn.rec[static_cast<size_t>(j - sdyn.base) * kSpreadU64];
          w->dyn_pod.insert(w->dyn_pod.end(), sw, sw + kSpreadU64);
        } else {
          for (int s2 = 0; s2 < kSpreadSlots; ++s2) {
            for (int g = 0; g < kDynG; ++g) w->dyn_pod.push_back(0);
            w->dyn_pod.insert(w->dyn_pod.end(), {~0ull, 0ull, 0ull});
          }
        }
      }
    }
  }
  // extension records: per pod of such a candidate {AddPod accounting of
  // cpu / memory / ephemeral, per scalar slot the fit request (INT64_MIN: the
  // pod does not list it) and the accounting, the slots' name rows}; per
  // shared scalar name of the call, the base free value of every spot node
  {
    const int32_t n_act = static_cast<int32_t>(w->cand_src.size());
    bool any_ext = false;
    for (int32_t k = 0; k < n_act && !any_ext; ++k) any_ext = cand_ext[w->cand_src[k]] != 0;
    if (any_ext) {
      w->ext_cand.assign(static_cast<size_t>(n_act), -1);
      for (int32_t k = 0; k < n_act; ++k) {
        const int32_t i = w->cand_src[k];
        if (!cand_ext[i]) continue;
        w->ext_cand[k] = static_cast<int32_t>(w->pod_ext.size() / kExtU64);
        int32_t row[2] = {-1, -1};
        for (int j = 0; j < 2; ++j)
          if (cand_sname[2 * i + j] != kNoName)
            row[j] = static_cast<int32_t>(std::find(scal_names.begin(), scal_names.end(), cand_sname[2 * i + j]) -
                                          scal_names.begin());
        for (int32_t q = w->cand_off[k]; q < w->cand_off[k + 1]; ++q) {
          const int32_t pod = active_pod[q];
          uint64_t x[kExtU64];
          for (int r = 0; r < 3; ++r) x[r] = static_cast<uint64_t>(pod_acc(c, pod, r));
          for (int j = 0; j < 2; ++j) {
            int64_t rq = INT64_MIN, ac = 0;
            const int32_t nm = cand_sname[2 * i + j];
            if (row[j] >= 0 && nm >= 0) {
              for (int32_t a = c->pod_scalar_off[pod]; a < c->pod_scalar_off[pod + 1]; ++a)
                if (c->pod_scalar_name[a] == nm) {
                  rq = c->pod_scalar_req[a];
                  ac = c->pod_scalar_acc[a];
                }
            } else if (row[j] >= 0) {  // a volume limit key: the pod's attachable volumes of it (distinct)
              const int32_t n_att = pod_att_of(c, pod, vol_key_of(nm));
              if (n_att > 0) rq = ac = n_att;
            }
            x[3 + j] = static_cast<uint64_t>(rq);
            x[5 + j] = static_cast<uint64_t>(ac);
          }
          x[7] = static_cast<uint64_t>(static_cast<uint32_t>(row[0])) |
                 static_cast<uint64_t>(static_cast<uint32_t>(row[1])) << 32;
          w->pod_ext.insert(w->pod_ext.end(), x, x + kExtU64);
        }
      }
      w->n_scal_names = static_cast<int32_t>(scal_names.size());
      w->node_scal.assign(std::max<size_t>(1, scal_names.size()) * static_cast<size_t>(w->n_pad), 0);
      node_scal_rows(snap, scal_names, w->n_pad, w->node_scal.data());
    }
  }
  phase(4);

  // ---- T rows.  A pod asking r in one dimension uses the row of the
  // smallest node free value v >= r: it selects exactly the nodes with
  // free >= r (no node value lies in [r, v)), and there are at most
  // min(distinct requests, distinct node values) such rows.  A request above
  // every node's free capacity maps to the empty row.
  w->t_dim.push_back(3);
  w->t_thr.push_back(0);  // row 0: every node
  const int64_t kNever = INT64_MAX;  // free >= INT64_MAX never holds (free < 2^62)
  LowerBound lb[3];
  if (big)
    for (int d = 0; d < 3; ++d) lb[d].build(C.node_vals[d]);
  auto lower = [&](int d, int64_t x) -> size_t {
    if (big) return lb[d](x);
    const std::vector<int64_t>& v = C.node_vals[d];
    return static_cast<size_t>(std::lower_bound(v.begin(), v.end(), x) - v.begin());
  };
  // every field of pod_rows / pod_rec is written below (only the padding is
  // cleared here): the vectors keep their size across encodes
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
  std::vector<uint8_t> atom_empty(static_cast<size_t>(w->n_atoms)), atom_full(static_cast<size_t>(w->n_atoms));
  for (int32_t a = 0; a < w->n_atoms; ++a)
    atom_flags(A + static_cast<size_t>(a) * Wp, Wp, n_spot, &atom_empty[a], &atom_full[a]);
  for (int32_t k = 0; k < w->n_classes; ++k) cls_empty[k] = class_empty(*w, k, atom_empty.data(), atom_full.data());
  phase(8);
  std::vector<uint8_t> used[3];  // lower-bound positions some pod asks for, per dimension
  for (int d = 0; d < 3; ++d) used[d].assign(C.node_vals[d].size() + 1, 0);
  std::vector<int32_t> used_list[3];  // the same positions, listed (serial runs: no scan of `used`)
  std::atomic<bool> any_dead{false};
  // per pod: requests, records and the lower-bound position of each request
  // among the node values (stored in pod_rows[1..3] for now)
  pfor(static_cast<size_t>(na), 2048, [&](size_t lo, size_t hi) {
    bool chunk_dead = false;  // one shared store per chunk, not per pod
    for (size_t q = lo; q < hi; ++q) {
      const int64_t* rq = &req_flat[static_cast<size_t>(active_src[q] - w->pod_base) * 3];
      const int64_t rc = rq[0], rm = rq[1], re = rq[2];
      const bool zero = rc == 0 && rm == 0 && re == 0;
      const int32_t ki = key_slot[pod_key[q]];
      int32_t* r = &w->pod_rows[q * 4];
      r[0] = key_class[ki];
      r[1] = zero ? -1 : static_cast<int32_t>(lower(0, rc));
      r[2] = zero ? -1 : static_cast<int32_t>(lower(1, rm));
      r[3] = zero ? -1 : static_cast<int32_t>(lower(2, re));
      uint64_t* rec = &w->pod_rec[q * 6];
      rec[0] = static_cast<uint64_t>(rc);
      rec[1] = static_cast<uint64_t>(rm);
      rec[2] = static_cast<uint64_t>(re);
      rec[3] = key_ports[ki] | (anti.active ? anti.pod_bits[active_src[q] - anti.base] : 0);
      bool dead = cls_empty[r[0]] != 0;
      for (int d = 0; d < 3; ++d) {
        if (r[1 + d] < 0) continue;
        uint8_t* u = &used[d][static_cast<size_t>(r[1 + d])];  // read first (see key_seen)
        if (!__atomic_load_n(u, __ATOMIC_RELAXED)) {
          __atomic_store_n(u, uint8_t(1), __ATOMIC_RELAXED);
          if (!big) used_list[d].push_back(r[1 + d]);
        }
        dead = dead || static_cast<size_t>(r[1 + d]) == C.node_vals[d].size();
      }
      if (dead) {
        r[0] = -1;  // the empty class, appended below
        chunk_dead = true;
      }
    }
    if (chunk_dead) any_dead.store(true, std::memory_order_relaxed);
  });
  phase(10);
  if (any_dead.load(std::memory_order_relaxed) || want_index) {  // (a reuse encode may need it later)
    emit(0, PROG_AND);
    emit(0, PROG_ANDNOT);
    w->cls_prog_off.push_back(static_cast<int32_t>(w->cls_prog.size()));
    w->empty_class = w->n_classes++;
  }
  // positions -> T rows: row 0 = every node, then the used positions of each
  // dimension in increasing threshold order (rows grouped by dimension, so
  // K0 compares one dimension per wave)
  std::vector<int32_t> t_index[3];
  {
    w->t_off[0] = 0;
    w->t_off[1] = 1;
    for (int d = 0; d < 3; ++d) {
      t_index[d].assign(used[d].size(), -1);
      auto add_row = [&](size_t pos) {
        t_index[d][pos] = static_cast<int32_t>(w->t_dim.size());
        w->t_dim.push_back(d);
        w->t_thr.push_back(pos == C.node_vals[d].size() ? kNever : C.node_vals[d][pos]);
      };
      if (big) {
        for (size_t pos = 0; pos < used[d].size(); ++pos)
          if (used[d][pos]) add_row(pos);
      } else {
        std::sort(used_list[d].begin(), used_list[d].end());
        for (int32_t pos : used_list[d]) add_row(static_cast<size_t>(pos));
      }
      if (want_index) {  // spare rows for thresholds a reuse encode adds: up to the next 64 (K0's row groups;
                         // SR_T_SPARE=n: exactly n, tests of the spare-exhausted path)
        static const int spare_env = std::getenv("SR_T_SPARE") ? std::atoi(std::getenv("SR_T_SPARE")) : -1;
        const size_t n_used = w->t_dim.size() - static_cast<size_t>(w->t_off[d + 1]);
        const size_t n_rows = spare_env >= 0 ? n_used + static_cast<size_t>(spare_env) : (n_used + 4 + 63) / 64 * 64;
        for (size_t i = n_used; i < n_rows; ++i) {
          w->t_dim.push_back(d);
          w->t_thr.push_back(kTSpare);
        }
      }
      w->t_off[d + 2] = static_cast<int32_t>(w->t_dim.size());
    }
  }
  phase(12);
  pfor(static_cast<size_t>(na), 4096, [&](size_t lo, size_t hi) {
    auto off = [&](int32_t table_row) { return static_cast<uint64_t>(table_row) * static_cast<uint64_t>(Wp); };
    for (size_t q = lo; q < hi; ++q) {
      int32_t* r = &w->pod_rows[q * 4];
      if (r[0] < 0) r[0] = w->empty_class;
      for (int d = 0; d < 3; ++d) r[1 + d] = r[1 + d] < 0 ? 0 : t_index[d][static_cast<size_t>(r[1 + d])];
      uint64_t* rec = &w->pod_rec[q * 6];
      rec[4] = off(r[0]) | off(w->n_classes + r[1]) << 32;
      rec[5] = off(w->n_classes + r[2]) | off(w->n_classes + r[3]) << 32;
    }
  });
  if ((static_cast<uint64_t>(w->n_classes) + w->t_dim.size()) * static_cast<uint64_t>(Wp) >= (1ull << 32)) {
    *err = "bitmask tables exceed 2^32 words";
    return SR_ERR_CAPACITY;
  }
  phase(13);

  // ---- class programs of <= 8 operations in fixed 8-slot records (K0 reads
  // one record with one scalar load); -1 pads, -2 in slot 0 marks a longer
  // program (read through cls_prog_off)
  w->cls_prog8.assign(static_cast<size_t>(w->n_classes) * 8, -1);
  for (int32_t k = 0; k < w->n_classes; ++k) {
    const int32_t o = w->cls_prog_off[k], len = w->cls_prog_off[k + 1] - o;
    int32_t* slot = &w->cls_prog8[static_cast<size_t>(k) * 8];
    if (len > 8) {
      slot[0] = -2;
      continue;
    }
    for (int32_t i = 0; i < len; ++i) slot[i] = w->cls_prog[o + i];
  }

  // ---- K2 work list: the first kListHead candidates, then the rest, each part
  // longest first (counting sort, stable).  Longest first shortens the grid's
  // makespan; the head goes first because a winner-only tick returns once the
  // candidates up to the winner are planned, and run() drains the first
  // drainable one (rescheduler.go:280-286) -- on a grid larger than the chip
  // holds at once, low indices must not wait for a later dispatch round.  A
  // list longer than the chip holds at once, with domain-path candidates, goes
  // in two parts, each in that order (Workload::n_list_node): planned by two
  // kernels side by side.
  {
    const size_t n_act = w->cand_off.size() - 1;
    const int32_t kListHead = C.list_head;
    const int32_t split_min = C.split_min;
    auto part_of = [&](size_t i) {  // 1: node order; 2: the rest (domain path, more than 256 pods)
      const int32_t len = w->cand_off[i + 1] - w->cand_off[i];
      return (!w->dyn_cand.empty() && w->dyn_cand[i] >= 0) || len > 256 ? 2 : 1;
    };
    const bool split = static_cast<int64_t>(n_act) > split_min && !w->dyn_cand.empty();
    auto bucket = [&](size_t i) {
      const int32_t len = w->cand_off[i + 1] - w->cand_off[i];
      const int32_t part = (split ? 2 * part_of(i) : 0) + (static_cast<int32_t>(i) < kListHead ? 0 : 1);
      return part * (MAX_CAND_PODS + 1) + MAX_CAND_PODS - len;
    };
    w->n_list_node = w->max_np_node = 0;
    if (split)
      for (size_t i = 0; i < n_act; ++i)
        if (part_of(i) == 1) {
          ++w->n_list_node;
          w->max_np_node = std::max(w->max_np_node, w->cand_off[i + 1] - w->cand_off[i]);
        }
    std::vector<int32_t> cnt(6 * (MAX_CAND_PODS + 1) + 1, 0);
    for (size_t i = 0; i < n_act; ++i) ++cnt[bucket(i)];
    for (size_t v = 0, acc = 0; v < cnt.size(); ++v) {
      const int32_t k = cnt[v];
      cnt[v] = static_cast<int32_t>(acc);
      acc += static_cast<size_t>(k);
    }
    w->list.assign(n_act * 4, 0);
    for (size_t i = 0; i < n_act; ++i) {
      const int32_t b = w->cand_off[i], e = w->cand_off[i + 1];
      int32_t* l = &w->list[static_cast<size_t>(cnt[bucket(i)]++) * 4];
      l[0] = static_cast<int32_t>(i);
      l[1] = b;
      l[2] = e;
      l[3] = w->cand_global[i];
    }
    if (!w->ext_cand.empty()) {  // the entries' extension-record heads, in list order
      w->list_ext.assign(n_act * 4, -1);
      for (size_t j = 0; j < n_act; ++j) {
        const int32_t e = w->ext_cand[static_cast<size_t>(w->list[j * 4])];
        int32_t* x = &w->list_ext[j * 4];
        x[0] = e;
        x[3] = 0;
        if (e >= 0) {
          const uint64_t erow = w->pod_ext[static_cast<size_t>(e) * kExtU64 + 7];
          x[1] = static_cast<int32_t>(static_cast<uint32_t>(erow));
          x[2] = static_cast<int32_t>(erow >> 32);
        }
      }
    }
  }
  phase(6);

  // ---- the reuse index (CandReuse), when this input was also
  // the last call's and its candidate side reads nothing from the snapshot but
  // node capacities and pod counts
  if (want_index) {
    // host ports, scalar resources and volume limits read the snapshot through
    // atom rows a reuse encode recomputes (CandReuse::port_q, scalar_q) and the
    // shared scalar rows (scal_names)
    // inter-pod anti-affinity and topology spread read the snapshot through
    // the DA / DB rows, the spread rows and the domain-path tables, which a
    // reuse patches node by node (AntiReuse, SpreadReuse), and through host
    // decisions that must not be able to turn: no opaque or unknown pods
    // (pass 1), no candidate sent to the reference path on the base counts
    // (analyse_spread); required pod affinity is not followed
    bool state_free = snap->opaque_total == 0 && (snap->anti_total == 0 || anti_keep) && !aff.active &&
                      !sdyn.state_fb && w->empty_class >= 0;
    if ((anti_keep || spread_keep) && (snap->unknown_total > 0 || snap->term_unknown_total > 0)) state_free = false;
    if (!c->pod_affinity && snap->anti_total > 0) state_free = false;  // pass 1 sent everything back on it
    const sr_pod_affinity* PA = c->pod_affinity;
    for (int32_t j = w->pod_base; j < w->pod_base + w->n_input_pods && state_free; ++j) {
      const int32_t pod = cands->cand_pods[j];
      // scalar resources and attachable volumes read the snapshot through
      // their atom rows and the shared scalar rows (recomputed by a reuse) and
      // through the fallback checks (rechecked by a reuse)
      if (PA) state_free = !PA->aff_off || PA->aff_off[pod] == PA->aff_off[pod + 1];
      // a fallback decided by the snapshot must not be able to turn back:
      // scalar usage unknown on some node, or an attachable volume of a
      // fallback candidate (a spot node may hold it)
      if (has_scalars(c, pod) && snap->scalar_unknown_total > 0) state_free = false;
    }
    for (int32_t i = 0; i < nc && state_free && c->volumes; ++i)
      if (w->status_host[i] == SR_CAND_FALLBACK)
        for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1] && state_free; ++j)
          state_free = att_count(c, cands->cand_pods[j]) == 0;
    if (state_free) {
      const size_t NA = static_cast<size_t>(na);
      const int32_t n_base_cls = static_cast<int32_t>(cls_empty.size());
      R.content_gen = C.content_gen;
      R.static_gen = C.static_gen;
      R.n_spot = n_spot;
      R.Wp = Wp;
      R.a_comp = A_COMP;
      R.comp_sets = comp_sets;
      R.a_scalar = A_SCALAR;
      R.scalar_q = scalar_query;
      R.scal_names = w->ext_cand.empty() ? std::vector<int32_t>() : scal_names;
      R.scalars = false;
      R.att_words.clear();
      for (int32_t i = 0; i < nc; ++i) {
        const bool planned = w->status_host[i] == STATUS_PENDING;
        for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
          const int32_t pod = cands->cand_pods[j];
          R.scalars = R.scalars || has_scalars(c, pod);
          if (planned && c->volumes)
            for (int32_t a = c->volumes->att_off[pod]; a < c->volumes->att_off[pod + 1]; ++a)
              R.att_words.push_back(att_word(c->volumes->att_key[a], c->volumes->att_id[a]));
        }
      }
      std::sort(R.att_words.begin(), R.att_words.end());
      R.anti = anti_keep;
      R.a_anti = A_ANTI;
      R.spread = spread_keep;
      R.a_port = A_PORT;
      R.port_q.clear();
      for (const PortQuery& pq : port_query) R.port_q.insert(R.port_q.end(), {pq.proto, pq.port, pq.ip});
      R.atom_empty = atom_empty;
      R.atom_full = atom_full;
      R.cls_empty = cls_empty;
      R.pod_cls.resize(NA);
      R.pod_ri.assign(NA * 3, -1);
      auto req_of = [&](size_t q) { return &req_flat[static_cast<size_t>(active_src[q] - w->pod_base) * 3]; };
      auto is_zero = [&](size_t q) {
        const int64_t* rq = req_of(q);
        return rq[0] == 0 && rq[1] == 0 && rq[2] == 0;
      };
      for (size_t q = 0; q < NA; ++q) R.pod_cls[q] = key_class[key_slot[pod_key[q]]];
      pfor(3, 1, [&](size_t lo, size_t hi) {
        for (size_t d = lo; d < hi; ++d) {
          std::vector<int64_t>& dr = R.dreq[d];
          dr.clear();
          for (size_t q = 0; q < NA; ++q)
            if (!is_zero(q)) dr.push_back(req_of(q)[d]);
          std::sort(dr.begin(), dr.end());
          dr.erase(std::unique(dr.begin(), dr.end()), dr.end());
          const std::vector<int64_t>& v = C.node_vals[d];
          R.vals[d] = v;
          R.dthr[d].resize(dr.size());
          R.drow[d].resize(dr.size());
          for (size_t u = 0; u < dr.size(); ++u) {
            const size_t pos = static_cast<size_t>(std::lower_bound(v.begin(), v.end(), dr[u]) - v.begin());
            R.dthr[d][u] = pos == v.size() ? INT64_MAX : v[pos];
            R.drow[d][u] = t_index[d][pos];
          }
          std::vector<int32_t>& po = R.dpod_off[d];
          po.assign(dr.size() + 1, 0);
          for (size_t q = 0; q < NA; ++q) {
            if (is_zero(q)) continue;
            const int32_t u = static_cast<int32_t>(std::lower_bound(dr.begin(), dr.end(), req_of(q)[d]) - dr.begin());
            R.pod_ri[q * 3 + d] = u;
            ++po[u + 1];
          }
          for (size_t u = 0; u < dr.size(); ++u) po[u + 1] += po[u];
          R.dpod[d].resize(static_cast<size_t>(po.back()));
          std::vector<int32_t> fill(po.begin(), po.end() - 1);
          for (size_t q = 0; q < NA; ++q)
            if (R.pod_ri[q * 3 + d] >= 0) R.dpod[d][fill[R.pod_ri[q * 3 + d]]++] = static_cast<int32_t>(q);
        }
      });
      R.row_refs.assign(w->t_dim.size(), 0);
      for (int d = 0; d < 3; ++d) {
        R.row_of[d].clear();
        R.spare[d].clear();
        for (size_t u = 0; u < R.dreq[d].size(); ++u) {
          ++R.row_refs[R.drow[d][u]];
          R.row_of[d][R.dthr[d][u]] = R.drow[d][u];
        }
        for (int32_t row = w->t_off[d + 1]; row < w->t_off[d + 2]; ++row)
          if (w->t_thr[row] == kTSpare) R.spare[d].push_back(row);
      }
      R.cls_pod_off.assign(static_cast<size_t>(n_base_cls) + 1, 0);
      for (size_t q = 0; q < NA; ++q) ++R.cls_pod_off[R.pod_cls[q] + 1];
      for (int32_t k = 0; k < n_base_cls; ++k) R.cls_pod_off[k + 1] += R.cls_pod_off[k];
      R.cls_pod.resize(NA);
      std::vector<int32_t> fill(R.cls_pod_off.begin(), R.cls_pod_off.end() - 1);
      for (size_t q = 0; q < NA; ++q) R.cls_pod[fill[R.pod_cls[q]]++] = static_cast<int32_t>(q);
      R.mark.assign(NA, 0);
      R.epoch = 0;
      R.indexed = true;
    }
  }
  return SR_OK;
}

}  // namespace

}  // namespace sr
