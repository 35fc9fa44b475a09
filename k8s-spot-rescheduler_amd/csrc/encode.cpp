// encode.cpp — snapshot + candidate pod lists -> SoA workload for gfx950.
//
// The predicate of one (pod, spot node) pair against the *base* snapshot
// (k8s v1.19.2 NodeUnschedulable, NodeResourcesFit, NodeName, NodePorts,
// NodeAffinity, TaintToleration [upstream]; call site rescheduler.go:344)
// factors into a conjunction of terms that each depend on a low-cardinality
// projection of the pod:
//
//   fits(p, n) = A[class(p), cpu(p), eph(p), zero(p)](n)  AND  B[mem(p)](n)
//
//   A = static(class, n)            selector / affinity / taints / base ports
//       AND len(pods)+1 <= allowed  (pod-count part of NodeResourcesFit)
//       AND (zero-request OR (cpu <= free_cpu AND eph <= free_eph))
//   B = zero-request OR mem <= free_mem
//
// where "class" interns everything static about a pod.  Both tables are bitmask
// rows over spot nodes in NodeInfoArray order, built on the GPU (K0); the dense
// pod x node bitmask is their AND (K1).  Everything that changes while a
// candidate's pods are placed (capacity, pod count, host ports) is rechecked
// exactly on the nodes the candidate touched (K2).  Features outside this set
// route the whole candidate to the reference path (SR_CAND_FALLBACK).
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "host.hpp"

namespace sr {
namespace {

constexpr int64_t kQuantityLimit = int64_t(1) << 62;

bool in_range(int64_t v) { return v >= 0 && v < kQuantityLimit; }

enum : int32_t { REQ_LABEL_EQ = 0, REQ_LABEL_EXPR = 1, REQ_FIELD = 2 };

// A node-side requirement: nodeSelector pair, matchExpression or matchField.
struct Requirement {
  int32_t type, key, op;
  std::vector<int32_t> vals;  // sorted, unique
};

std::string bytes_of(const int32_t* p, size_t n) {
  return std::string(reinterpret_cast<const char*>(p), n * sizeof(int32_t));
}

class RequirementDict {
 public:
  int32_t intern(Requirement r) {
    std::sort(r.vals.begin(), r.vals.end());
    r.vals.erase(std::unique(r.vals.begin(), r.vals.end()), r.vals.end());
    std::vector<int32_t> k = {r.type, r.key, r.op};
    k.insert(k.end(), r.vals.begin(), r.vals.end());
    auto ins = index_.emplace(bytes_of(k.data(), k.size()), static_cast<int32_t>(reqs_.size()));
    if (ins.second) reqs_.push_back(std::move(r));
    return ins.first->second;
  }
  const std::vector<Requirement>& all() const { return reqs_; }

 private:
  std::unordered_map<std::string, int32_t> index_;
  std::vector<Requirement> reqs_;
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

struct TupleKey {
  int32_t cls, zero;
  int64_t cpu, eph;
  bool operator==(const TupleKey& o) const {
    return cls == o.cls && zero == o.zero && cpu == o.cpu && eph == o.eph;
  }
};
struct TupleHash {
  size_t operator()(const TupleKey& k) const {
    uint64_t h = static_cast<uint64_t>(k.cls) * 0x9E3779B97F4A7C15ull;
    h ^= static_cast<uint64_t>(k.cpu) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
    h ^= static_cast<uint64_t>(k.eph) + 0x8CB92BA72F3D8DD7ull + (h << 6) + (h >> 2);
    return static_cast<size_t>(h ^ static_cast<uint64_t>(k.zero));
  }
};

}  // namespace

sr_status encode_workload(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                          Workload* w, std::string* err) {
  const sr_pods& P = c->pods;
  const int32_t nc = cands->n_cand;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  *w = Workload();
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
    for (int32_t i = P.port_off[pod]; i < P.port_off[pod + 1]; ++i)
      if (P.port_ip[i] != -1 && P.port_num[i] > 0) return true;  // specific hostIP
    return false;
  };
  for (int32_t i = 0; i < nc; ++i) {
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    if (e < b) {
      *err = "cand_pod_off not monotone";
      return SR_ERR_INVALID_ARG;
    }
    if (e == b) {
      w->status_host[i] = SR_CAND_EMPTY;
      continue;
    }
    bool fb = snap->anti_total > 0 || (e - b) > SLOTS_LARGE;
    for (int32_t j = b; j < e && !fb; ++j) {
      const int32_t pod = cands->cand_pods[j];
      if (pod < 0 || pod >= P.n) {
        *err = "candidate pod index out of range";
        return SR_ERR_INVALID_ARG;
      }
      fb = pod_fallback(pod);
    }
    if (fb) w->status_host[i] = SR_CAND_FALLBACK;
  }

  // ---- host-port dictionary: (protocol, port) pairs of active pods, <= 64
  std::unordered_map<int64_t, int32_t> port_dict;
  auto port_key = [](int32_t proto, int32_t port) { return (static_cast<int64_t>(proto) << 32) | uint32_t(port); };
  for (int32_t i = 0; i < nc; ++i) {
    if (w->status_host[i] != STATUS_PENDING) continue;
    bool overflow = false;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      for (int32_t k = P.port_off[pod]; k < P.port_off[pod + 1]; ++k) {
        if (P.port_num[k] <= 0) continue;
        const int64_t key = port_key(P.port_proto[k], P.port_num[k]);
        if (port_dict.count(key)) continue;
        if (port_dict.size() >= 64) {
          overflow = true;
          continue;
        }
        port_dict.emplace(key, static_cast<int32_t>(port_dict.size()));
      }
    }
    if (overflow) w->status_host[i] = SR_CAND_FALLBACK;
  }
  auto pod_port_mask = [&](int32_t pod) {
    uint64_t m = 0;
    for (int32_t k = P.port_off[pod]; k < P.port_off[pod + 1]; ++k) {
      if (P.port_num[k] <= 0) continue;
      auto it = port_dict.find(port_key(P.port_proto[k], P.port_num[k]));
      if (it != port_dict.end()) m |= 1ull << it->second;
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
  std::unordered_map<std::string, int32_t> taint_index;
  auto taint_id = [&](const TaintRec& t) {
    const int32_t k[3] = {t.key, t.val, t.effect};
    auto ins = taint_index.emplace(bytes_of(k, 3), static_cast<int32_t>(taints.size()));
    if (ins.second) taints.push_back(t);
    return ins.first->second;
  };
  std::vector<std::vector<int32_t>> node_taints(static_cast<size_t>(n_spot));
  for (int32_t n = 0; n < n_spot; ++n) {
    const SpotNode& sn = snap->nodes[n];
    for (const TaintRec& t : sn.taints)
      if (t.effect == SR_EFFECT_NO_SCHEDULE || t.effect == SR_EFFECT_NO_EXECUTE)
        node_taints[n].push_back(taint_id(t));
    if (sn.unschedulable)
      node_taints[n].push_back(taint_id(TaintRec{snap->id_unschedulable_key, snap->id_empty, SR_EFFECT_NO_SCHEDULE}));
  }
  w->WT = std::max<int32_t>(1, (static_cast<int32_t>(taints.size()) + 63) / 64);

  // ---- classes of active pods
  RequirementDict rdict;
  struct PodStatic {
    std::vector<int32_t> sel;                 // requirement ids
    std::vector<std::vector<int32_t>> terms;  // valid terms only
    int32_t flags = 0;
    std::vector<uint64_t> tol;
    uint64_t ports = 0;
  };
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

  std::vector<PodStatic> pstat(static_cast<size_t>(na));
  for (int32_t q = 0; q < na; ++q) {
    const int32_t pod = active_pod[q];
    PodStatic& ps = pstat[q];
    // Spec.NodeSelector: labels.SelectorFromSet -> Equals requirements.
    for (int32_t i = P.sel_off[pod]; i < P.sel_off[pod + 1]; ++i)
      ps.sel.push_back(rdict.intern(Requirement{REQ_LABEL_EQ, P.sel_key[i], SR_OP_IN, {P.sel_val[i]}}));
    std::sort(ps.sel.begin(), ps.sel.end());
    ps.sel.erase(std::unique(ps.sel.begin(), ps.sel.end()), ps.sel.end());
    // Required node affinity: MatchNodeSelectorTerms.
    if (P.aff_required[pod]) {
      ps.flags |= CLS_AFF_REQUIRED;
      for (int32_t t = P.term_off[pod]; t < P.term_off[pod + 1]; ++t) {
        const int32_t e0 = P.term_expr_off[t], e1 = P.term_expr_off[t + 1];
        const int32_t f0 = P.term_field_off[t], f1 = P.term_field_off[t + 1];
        if (e0 == e1 && f0 == f1) continue;  // an empty term selects nothing
        bool valid = true;
        std::vector<int32_t> term;
        for (int32_t e = e0; e < e1 && valid; ++e) {
          const int32_t nv = P.expr_val_off[e + 1] - P.expr_val_off[e];
          const int32_t op = P.expr_op[e];
          if (P.expr_key[e] == c->id_empty) valid = false;  // validateLabelKey("") fails
          else if ((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 0) valid = false;
          else if ((op == SR_OP_EXISTS || op == SR_OP_DOES_NOT_EXIST) && nv != 0) valid = false;
          else if (op != SR_OP_IN && op != SR_OP_NOT_IN && op != SR_OP_EXISTS && op != SR_OP_DOES_NOT_EXIST)
            valid = false;
          if (!valid) break;
          Requirement r{REQ_LABEL_EXPR, P.expr_key[e], op,
                        std::vector<int32_t>(P.expr_vals + P.expr_val_off[e], P.expr_vals + P.expr_val_off[e + 1])};
          term.push_back(rdict.intern(std::move(r)));
        }
        for (int32_t f = f0; f < f1 && valid; ++f) {
          const int32_t nv = P.field_val_off[f + 1] - P.field_val_off[f];
          const int32_t op = P.field_op[f];
          if (!((op == SR_OP_IN || op == SR_OP_NOT_IN) && nv == 1)) {
            valid = false;
            break;
          }
          term.push_back(rdict.intern(Requirement{REQ_FIELD, P.field_key[f], op, {P.field_vals[P.field_val_off[f]]}}));
        }
        if (!valid) continue;  // a term that fails to build matches nothing
        std::sort(term.begin(), term.end());
        term.erase(std::unique(term.begin(), term.end()), term.end());
        ps.terms.push_back(std::move(term));
      }
      if (ps.terms.empty()) ps.flags |= CLS_IMPOSSIBLE;
    }
    ps.tol.assign(static_cast<size_t>(w->WT), 0);
    if (P.tol_off[pod + 1] > P.tol_off[pod])
      for (size_t t = 0; t < taints.size(); ++t)
        if (tolerates(P, pod, c->id_empty, taints[t])) ps.tol[t >> 6] |= 1ull << (t & 63);
    ps.ports = pod_port_mask(pod);
  }
  const std::vector<Requirement>& reqs = rdict.all();
  w->WR = std::max<int32_t>(1, (static_cast<int32_t>(reqs.size()) + 63) / 64);
  const int32_t WR = w->WR, WT = w->WT;

  // intern classes
  std::unordered_map<std::string, int32_t> class_index;
  std::vector<int32_t> pod_class(static_cast<size_t>(na));
  w->cls_term_off.push_back(0);
  std::vector<uint64_t> sig;
  for (int32_t q = 0; q < na; ++q) {
    const PodStatic& ps = pstat[q];
    sig.assign(static_cast<size_t>(WR), 0);
    for (int32_t r : ps.sel) sig[r >> 6] |= 1ull << (r & 63);
    sig.push_back(static_cast<uint64_t>(ps.flags));
    sig.push_back(ps.terms.size());
    for (const auto& t : ps.terms) {
      const size_t base = sig.size();
      sig.resize(base + WR, 0);
      for (int32_t r : t) sig[base + (r >> 6)] |= 1ull << (r & 63);
    }
    sig.insert(sig.end(), ps.tol.begin(), ps.tol.end());
    sig.push_back(ps.ports);
    std::string key(reinterpret_cast<const char*>(sig.data()), sig.size() * sizeof(uint64_t));
    auto ins = class_index.emplace(std::move(key), w->n_classes);
    if (ins.second) {
      w->cls_sel.insert(w->cls_sel.end(), sig.begin(), sig.begin() + WR);
      w->cls_flags.push_back(ps.flags);
      for (const auto& t : ps.terms) {
        const size_t base = w->term_mask.size();
        w->term_mask.resize(base + WR, 0);
        for (int32_t r : t) w->term_mask[base + (r >> 6)] |= 1ull << (r & 63);
      }
      w->cls_term_off.push_back(static_cast<int32_t>(w->term_mask.size() / WR));
      w->cls_tol.insert(w->cls_tol.end(), ps.tol.begin(), ps.tol.end());
      w->cls_port.push_back(ps.ports);
      w->n_classes++;
    }
    pod_class[q] = ins.first->second;
  }

  // ---- spot nodes: dynamic base state, requirement / taint / port bitsets
  const int32_t NP = w->n_pad;
  w->free_cpu.assign(NP, 0);
  w->free_mem.assign(NP, 0);
  w->free_eph.assign(NP, 0);
  w->pods_left.assign(NP, 0);
  w->port_bits.assign(NP, 0);
  w->req_bits.assign(static_cast<size_t>(WR) * NP, 0);
  w->taint_bits.assign(static_cast<size_t>(WT) * NP, 0);
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
    uint64_t pb = 0;
    for (const Port& u : st.ports) {
      auto it = port_dict.find(port_key(u.proto, u.port));
      if (it != port_dict.end()) pb |= 1ull << it->second;  // incoming pods bind 0.0.0.0
    }
    w->port_bits[n] = pb;
    for (int32_t t : node_taints[n]) w->taint_bits[static_cast<size_t>(t >> 6) * NP + n] |= 1ull << (t & 63);
  }
  // requirement bits: one label-value column per distinct key
  std::unordered_map<int32_t, std::vector<int32_t>> col;  // key -> value per node (INT32_MIN absent)
  for (const Requirement& r : reqs)
    if (r.type != REQ_FIELD && !col.count(r.key)) col.emplace(r.key, std::vector<int32_t>(n_spot, INT32_MIN));
  for (int32_t n = 0; n < n_spot; ++n)
    for (const auto& kv : snap->nodes[n].labels) {
      auto it = col.find(kv.first);
      if (it != col.end()) it->second[n] = kv.second;
    }
  for (size_t ri = 0; ri < reqs.size(); ++ri) {
    const Requirement& r = reqs[ri];
    uint64_t* dst = w->req_bits.data() + (ri >> 6) * NP;
    const uint64_t bit = 1ull << (ri & 63);
    if (r.type == REQ_FIELD) {
      // fields.Set{"metadata.name": node.Name}; any other key reads as "".
      const bool is_name = r.key == c->id_metadata_name && c->id_metadata_name != -1;
      for (int32_t n = 0; n < n_spot; ++n) {
        const int32_t fv = is_name ? snap->nodes[n].name : c->id_empty;
        const bool eq = fv == r.vals[0];
        if (r.op == SR_OP_IN ? eq : !eq) dst[n] |= bit;
      }
      continue;
    }
    const std::vector<int32_t>& v = col[r.key];
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
      if (m) dst[n] |= bit;
    }
  }

  // ---- A / B row descriptors and per-pod arrays
  std::unordered_map<TupleKey, int32_t, TupleHash> a_index;
  std::unordered_map<int64_t, int32_t> b_index;
  w->b_mem.push_back(0);
  w->b_all.push_back(1);  // row 0: every node (zero-request pods skip the memory check)
  w->pod_a.resize(na);
  w->pod_b.resize(na);
  w->pod_zero.resize(na);
  w->pod_cpu.resize(na);
  w->pod_mem.resize(na);
  w->pod_eph.resize(na);
  w->pod_ports.resize(na);
  w->pod_src = active_src;
  for (int32_t q = 0; q < na; ++q) {
    const int32_t pod = active_pod[q];
    const int64_t rc = P.req_milli_cpu[pod], rm = P.req_memory[pod], re = P.req_ephemeral[pod];
    const int32_t zero = (rc == 0 && rm == 0 && re == 0) ? 1 : 0;
    TupleKey k{pod_class[q], zero, zero ? 0 : rc, zero ? 0 : re};
    auto ia = a_index.emplace(k, static_cast<int32_t>(w->a_class.size()));
    if (ia.second) {
      w->a_class.push_back(k.cls);
      w->a_zero.push_back(k.zero);
      w->a_cpu.push_back(k.cpu);
      w->a_eph.push_back(k.eph);
    }
    int32_t b = 0;
    if (!zero) {
      auto ib = b_index.emplace(rm, static_cast<int32_t>(w->b_mem.size()));
      if (ib.second) {
        w->b_mem.push_back(rm);
        w->b_all.push_back(0);
      }
      b = ib.first->second;
    }
    w->pod_a[q] = ia.first->second;
    w->pod_b[q] = b;
    w->pod_zero[q] = zero;
    w->pod_cpu[q] = rc;
    w->pod_mem[q] = rm;
    w->pod_eph[q] = re;
    w->pod_ports[q] = pstat[q].ports;
  }

  // ---- K2 variants by pod count (touched-node slots per wave)
  for (size_t i = 0; i + 1 < w->cand_off.size(); ++i) {
    const int32_t np = w->cand_off[i + 1] - w->cand_off[i];
    (np <= SLOTS_SMALL ? w->list_small : w->list_large).push_back(static_cast<int32_t>(i));
  }
  return SR_OK;
}

}  // namespace sr
