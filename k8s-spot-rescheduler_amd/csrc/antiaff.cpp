// antiaff.cpp — required inter-pod anti-affinity for the encoder.
//
// InterPodAffinity.Filter of k8s v1.19.2 [upstream
// plugins/interpodaffinity/filtering.go], anti-affinity part: a pod P is
// refused on node n when (1) an existing pod E on a node m carries a term t
// that selects P (E's term namespaces, selector on P's labels) and m, n carry
// the same value of t's topology key, or (2) P carries a term t that selects
// an existing pod E on such a node m.  "Existing" = NodeInfo.Pods of every
// snapshot node, which during canDrainNode includes the candidate's pods
// already placed (rescheduler.go:366).
//
// Encoding:
//  - static part, against the base snapshot: per distinct term t two node
//    sets, DA(t) = nodes sharing a t-domain with a base pod that has t, and
//    DB(t) = nodes sharing a t-domain with a base pod that t selects; a pod
//    ANDs NOT DA(t) for every t it matches and NOT DB(t) for every t it has
//    (atoms of its class program, so they land in its S row);
//  - dynamic part, between the pods of one candidate: a term through which
//    two of its pods interact must have a node-local topology key (every spot
//    node carries it, values pairwise distinct, e.g. kubernetes.io/hostname);
//    it then gets a pair of state bits of that candidate's own numbering (A:
//    a pod having t is here, B: a pod t selects is here).  A pod sets A for
//    its terms and B for the terms selecting it; it conflicts with a node
//    whose state holds B for its terms or A for the terms selecting it -- the
//    pair-swapped image of what it sets.  K2 keeps these bits with the
//    host-port bits; the base snapshot needs none (its conflicts are the
//    static part).  Interaction through a key whose domains span several
//    nodes (zone-style) puts the candidate on K2's domain path: each pod
//    records, per key slot, the earlier pods of its candidate it interacts
//    with, and the device refuses it the domains those pods were placed in
//    (DomKeys: <= kDomKeys keys of <= kDomMax domains, <= kDynPods pods;
//    beyond that the candidate takes the fallback path).
#include <algorithm>
#include <climits>
#include <cstring>
#include <unordered_map>
#include <unordered_set>

#include "host.hpp"
#include "pool.hpp"
#include "worddict.hpp"

namespace sr {

namespace {

struct Expr {
  int32_t key, op;
  std::vector<int32_t> vals;  // sorted
};

// One distinct term, resolved against its owner (namespaces defaulted).
struct Term {
  int32_t tk = -1;
  std::vector<int32_t> ns;  // sorted
  bool nil = false;
  std::vector<std::pair<int32_t, int32_t>> ml;  // sorted by key
  std::vector<Expr> me;
};

}  // namespace

void anti_term_words(const sr_cluster* c, int32_t owner, int32_t t, std::vector<int32_t>& out) {
  const sr_pod_affinity& A = *c->pod_affinity;
  out.clear();
  out.push_back(A.topology_key[t]);
  const size_t ns_at = out.size();
  out.push_back(0);
  if (A.ns_off[t] == A.ns_off[t + 1]) {
    out.push_back(A.ns[owner]);  // getNamespacesFromPodAffinityTerm: the owner's namespace
  } else {
    out.insert(out.end(), A.ns_ids + A.ns_off[t], A.ns_ids + A.ns_off[t + 1]);
    std::sort(out.begin() + ns_at + 1, out.end());
    out.erase(std::unique(out.begin() + ns_at + 1, out.end()), out.end());
  }
  out[ns_at] = static_cast<int32_t>(out.size() - ns_at - 1);
  out.push_back(A.selector_nil[t] ? 1 : 0);
  if (A.selector_nil[t]) return;
  std::vector<std::pair<int32_t, int32_t>> ml;
  for (int32_t i = A.ml_off[t]; i < A.ml_off[t + 1]; ++i) ml.emplace_back(A.ml_key[i], A.ml_val[i]);
  std::sort(ml.begin(), ml.end());
  out.push_back(static_cast<int32_t>(ml.size()));
  for (const auto& kv : ml) {
    out.push_back(kv.first);
    out.push_back(kv.second);
  }
  out.push_back(A.me_off[t + 1] - A.me_off[t]);
  for (int32_t e = A.me_off[t]; e < A.me_off[t + 1]; ++e) {
    out.push_back(A.me_key[e]);
    out.push_back(A.me_op[e]);
    const size_t at = out.size();
    out.push_back(0);
    out.insert(out.end(), A.me_vals + A.me_val_off[e], A.me_vals + A.me_val_off[e + 1]);
    std::sort(out.begin() + at + 1, out.end());
    out.erase(std::unique(out.begin() + at + 1, out.end()), out.end());
    out[at] = static_cast<int32_t>(out.size() - at - 1);
  }
}

int32_t DomKeys::slot(const sr_snapshot* snap, int32_t k) {
  for (size_t i = 0; i < key.size(); ++i)
    if (key[i] == k) return static_cast<int32_t>(i);
  if (key.size() >= static_cast<size_t>(kDomKeys)) return -1;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  std::vector<int32_t> d(static_cast<size_t>(n_spot), -1);
  std::unordered_map<int32_t, int32_t> id_of;
  bool local = true;
  for (int32_t n = 0; n < n_spot; ++n) {
    const auto& lb = snap->nodes[n].labels;
    auto it = std::find_if(lb.begin(), lb.end(), [k](const std::pair<int32_t, int32_t>& kv) { return kv.first == k; });
    if (it == lb.end()) {
      local = false;
      continue;
    }
    auto ins = id_of.emplace(it->second, static_cast<int32_t>(id_of.size()));
    if (!ins.second) local = false;
    d[n] = ins.first->second;
  }
  if (local) {
    for (int32_t n = 0; n < n_spot; ++n) d[n] = n;
  } else if (id_of.size() > static_cast<size_t>(kDomMax)) {
    return -1;
  }
  key.push_back(k);
  node_local.push_back(local ? 1 : 0);
  dom.push_back(std::move(d));
  n_dom.push_back(local ? n_spot : static_cast<int32_t>(id_of.size()));
  return static_cast<int32_t>(key.size() - 1);
}

namespace {

Term parse_term(const int32_t* w) {
  Term t;
  size_t i = 0;
  t.tk = w[i++];
  const int32_t nns = w[i++];
  t.ns.assign(w + i, w + i + nns);
  i += nns;
  t.nil = w[i++] != 0;
  if (t.nil) return t;
  const int32_t nml = w[i++];
  for (int32_t k = 0; k < nml; ++k, i += 2) t.ml.emplace_back(w[i], w[i + 1]);
  const int32_t nme = w[i++];
  for (int32_t k = 0; k < nme; ++k) {
    Expr e;
    e.key = w[i++];
    e.op = w[i++];
    const int32_t nv = w[i++];
    e.vals.assign(w + i, w + i + nv);
    i += nv;
    t.me.push_back(std::move(e));
  }
  return t;
}

// A pod's namespace and labels, from the caller's cluster or the snapshot's copy.
struct PodMeta {
  int32_t ns;
  const int32_t *key, *val;
  int32_t n;
};

PodMeta meta_of(const sr_pod_affinity& A, int32_t pod) {
  return PodMeta{A.ns[pod], A.label_key + A.label_off[pod], A.label_val + A.label_off[pod],
                 A.label_off[pod + 1] - A.label_off[pod]};
}

PodMeta meta_of(const sr_snapshot* s, const SnapPod& p) {
  return PodMeta{p.ns, s->lkey.data() + p.lab, s->lval.data() + p.lab, static_cast<int32_t>(p.nlab)};
}

bool pod_label(const PodMeta& m, int32_t key, int32_t* val) {
  for (int32_t i = 0; i < m.n; ++i)
    if (m.key[i] == key) {
      *val = m.val[i];
      return true;
    }
  return false;
}

// schedutil.PodMatchesTermsNamespaceAndSelector: namespace, then
// labels.Selector.Matches (MatchLabels = Equals; In / NotIn / Exists /
// DoesNotExist; nil selects nothing, empty everything).
bool term_selects(const Term& t, const PodMeta& m) {
  if (!std::binary_search(t.ns.begin(), t.ns.end(), m.ns)) return false;
  if (t.nil) return false;
  int32_t v;
  for (const auto& kv : t.ml)
    if (!pod_label(m, kv.first, &v) || v != kv.second) return false;
  for (const Expr& e : t.me) {
    const bool has = pod_label(m, e.key, &v);
    bool ok;
    switch (e.op) {
      case SR_OP_IN: ok = has && std::binary_search(e.vals.begin(), e.vals.end(), v); break;
      case SR_OP_NOT_IN: ok = !has || !std::binary_search(e.vals.begin(), e.vals.end(), v); break;
      case SR_OP_EXISTS: ok = has; break;
      default: ok = !has; break;  // DoesNotExist (anything else is opaque: never encoded)
    }
    if (!ok) return false;
  }
  return true;
}

inline uint64_t label_key(int32_t k, int32_t v) {
  return static_cast<uint64_t>(static_cast<uint32_t>(k)) << 32 | static_cast<uint32_t>(v);
}

using LabelIndex = std::unordered_map<uint64_t, std::vector<int32_t>>;

// The terms selecting a pod: an index on each term's first MatchLabels pair
// (a pod can only be selected through one of its own labels); terms without
// MatchLabels are tried on every pod, nil selectors never.
template <class F>
void for_each_selecting(const std::vector<Term>& terms, const LabelIndex& by_label, const std::vector<int32_t>& unindexed,
                        const PodMeta& m, F&& f) {
  for (int32_t t : unindexed)
    if (term_selects(terms[t], m)) f(t);
  for (int32_t i = 0; i < m.n; ++i) {
    auto it = by_label.find(label_key(m.key[i], m.val[i]));
    if (it == by_label.end()) continue;
    for (int32_t t : it->second)
      if (term_selects(terms[t], m)) f(t);
  }
}

}  // namespace

// The snapshot-side state of one encode's DA / DB rows (analyse_anti with
// `keep`): per spot node the (term, side) of each of its pods -- side 0: the
// pod has the term, 1: the term selects it -- and per (term, side, value of
// the term's key) the pods counted, so a reuse encode moves only the rows of
// the values whose count went to or from zero.
struct AntiReuse {
  int32_t n_spot = 0, Wp = 0;
  WordDict all;                           // every term the full encode interned
  std::vector<int32_t> nid;               // [all id] kept term, -1: selects no pending candidate pod
  std::unordered_set<uint64_t> cand_labels;
  std::vector<Term> terms;                // kept
  LabelIndex by_label;
  std::vector<int32_t> unindexed;
  struct KeyVals {
    std::vector<int32_t> val;                                 // [n_spot] INT_MIN: absent
    std::unordered_map<int32_t, std::vector<int32_t>> nodes;  // value -> spot nodes
  };
  std::vector<KeyVals> keys;
  std::vector<int32_t> kidx;              // [term] key
  std::vector<uint8_t> any_built;         // [2t + side] the class programs AND NOT the row
  std::vector<int64_t> total;             // [2t + side] pods counted (on nodes carrying the key)
  std::unordered_map<uint64_t, int32_t> cnt;   // (2t + side) << 32 | value -> pods
  std::vector<std::vector<int32_t>> contrib;   // [node] 2t + side per pod and term, sorted
};

namespace {

// Node n's codes 2t + side; false: a term the full encode never interned that
// passes its filter (it may select a candidate pod).
bool node_contrib(const AntiReuse& R, const sr_snapshot* snap, int32_t n, std::vector<int32_t>& out) {
  out.clear();
  for (int32_t e : snap->state[n].pods) {
    const SnapPod& sp = snap->pods[e];
    const int32_t* tw = snap->term_words.data() + sp.terms;
    for (size_t i = 0; i < sp.nterms; i += 1 + static_cast<size_t>(tw[i])) {
      const int32_t* w = tw + i + 1;  // {tk, n ns, ns..., nil, n ml, (k, v)...}
      const int32_t* p = w + 2 + w[1];
      if (p[0] != 0) continue;  // nil: selects nothing
      if (p[1] > 0 && !R.cand_labels.count(label_key(p[2], p[3]))) continue;
      const size_t len = static_cast<size_t>(tw[i]);
      const int32_t id = R.all.find(w, len, hash_words(w, len));
      if (id < 0) return false;
      if (R.nid[id] >= 0) out.push_back(2 * R.nid[id]);
    }
    for_each_selecting(R.terms, R.by_label, R.unindexed, meta_of(snap, sp), [&](int32_t t) { out.push_back(2 * t + 1); });
  }
  std::sort(out.begin(), out.end());
  return true;
}

}  // namespace

bool anti_reuse_patch(AntiReuse& R, const sr_snapshot* snap, const std::vector<int32_t>& nodes, uint64_t* A,
                      int32_t a_anti, std::vector<int32_t>& atoms, std::vector<int32_t>& words) {
  if (static_cast<int32_t>(snap->nodes.size()) != R.n_spot) return false;
  const int32_t Wp = R.Wp;
  std::vector<int32_t> now;
  std::vector<std::pair<int32_t, int32_t>> delta;  // (code, +1 / -1)
  for (int32_t n : nodes) {
    if (!node_contrib(R, snap, n, now)) return false;
    std::vector<int32_t>& was = R.contrib[n];
    if (now == was) continue;
    delta.clear();
    size_t i = 0, j = 0;  // sorted multisets: what left, what came
    while (i < was.size() || j < now.size()) {
      if (j == now.size() || (i < was.size() && was[i] < now[j])) delta.emplace_back(was[i++], -1);
      else if (i == was.size() || now[j] < was[i]) delta.emplace_back(now[j++], +1);
      else ++i, ++j;
    }
    was.swap(now);
    for (const auto& d : delta) {
      const int32_t code = d.first, t = code >> 1;
      const AntiReuse::KeyVals& K = R.keys[R.kidx[t]];
      const int32_t v = K.val[n];
      if (v == INT_MIN) continue;
      // the class programs AND NOT the row exactly when it is not empty
      R.total[code] += d.second;
      if ((R.total[code] > 0) != (R.any_built[code] != 0)) return false;
      const uint64_t key = static_cast<uint64_t>(code) << 32 | static_cast<uint32_t>(v);
      int32_t& c = R.cnt[key];
      const int32_t before = c;
      c += d.second;
      if ((before == 0) == (c == 0)) continue;
      // the value's domain joins or leaves the row
      uint64_t* row = A + static_cast<size_t>(a_anti + code) * Wp;
      auto it = K.nodes.find(v);
      if (it != K.nodes.end())
        for (int32_t m : it->second) {
          if (c != 0) row[m >> 6] |= 1ull << (m & 63);
          else row[m >> 6] &= ~(1ull << (m & 63));
          words.push_back(m >> 6);
        }
      if (c == 0) R.cnt.erase(key);
      atoms.push_back(a_anti + code);
    }
  }
  return true;
}

void anti_reuse_permute(AntiReuse& R, const std::vector<int32_t>& src, const std::vector<int32_t>& moved) {
  permute_positions(R.contrib.data(), src, moved);
  const std::vector<int32_t> to = permute_targets(R.n_spot, src, moved);
  for (AntiReuse::KeyVals& K : R.keys) {
    permute_positions(K.val.data(), src, moved);
    for (auto& vn : K.nodes)
      for (int32_t& m : vn.second) m = to[m];
  }
}

void analyse_anti(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands, int32_t Wp,
                  std::vector<int32_t>& status, DomKeys* dk, AntiTerms* out, std::shared_ptr<AntiReuse>* keep_state) {
  AntiTerms& at = *out;
  at = AntiTerms{};
  const sr_pod_affinity* PA = c->pod_affinity;
  const int32_t nc = cands->n_cand;
  const int32_t base = nc > 0 ? cands->cand_pod_off[0] : 0;  // per-pod arrays: flat index - base
  const int32_t n_flat = nc > 0 ? cands->cand_pod_off[nc] - base : 0;
  at.base = base;
  at.pod_off.assign(static_cast<size_t>(n_flat) + 1, 0);
  // Without sr_pod_affinity a candidate pod's labels are unknown: if the
  // snapshot holds anti-affinity, pass 1 already sent every candidate to the
  // fallback path.
  if (!PA) return;
  if (PA->anti_off[c->pods.n] == 0 && snap->anti_total == 0) return;  // no term anywhere
  const sr_pod_affinity& A = *PA;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  AntiReuse* R = nullptr;
  if (keep_state) {
    *keep_state = std::make_shared<AntiReuse>();
    R = keep_state->get();
    R->n_spot = n_spot;
    R->Wp = Wp;
    R->contrib.resize(static_cast<size_t>(n_spot));
  }

  // ---- distinct terms: base pods (every snapshot node; the snapshot's own
  // copies) and pending candidates (the call's cluster)
  WordDict dict;
  std::vector<int32_t> words;
  std::vector<std::pair<int32_t, int32_t>> base_has;  // (node, term)
  // A base pod's term matters here only when it selects some pending
  // candidate pod (its DA row), so a term whose first matchLabels pair no
  // pending pod carries is not even interned; nil selectors select nothing.
  // The snapshot's pods are scanned in parallel, the kept terms interned in
  // node order.
  std::unordered_set<uint64_t> cand_labels;
  for (int32_t i = 0; i < nc; ++i) {
    if (status[i] != STATUS_PENDING) continue;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      for (int32_t l = A.label_off[pod]; l < A.label_off[pod + 1]; ++l)
        cand_labels.insert(static_cast<uint64_t>(static_cast<uint32_t>(A.label_key[l])) << 32 |
                           static_cast<uint32_t>(A.label_val[l]));
    }
  }
  {
    constexpr int32_t kNodes = 256;
    const size_t n_parts = (static_cast<size_t>(n_spot) + kNodes - 1) / kNodes;
    std::vector<std::vector<std::pair<int32_t, const int32_t*>>> part(n_parts);  // (node, term words)
    parallel_for(n_parts, 1, [&](size_t lo, size_t hi) {
      for (size_t ch = lo; ch < hi; ++ch)
        for (int32_t n = static_cast<int32_t>(ch) * kNodes; n < std::min<int32_t>(n_spot, (ch + 1) * kNodes); ++n)
          for (int32_t e : snap->state[n].pods) {
            const SnapPod& sp = snap->pods[e];
            const int32_t* tw = snap->term_words.data() + sp.terms;
            for (size_t i = 0; i < sp.nterms; i += 1 + static_cast<size_t>(tw[i])) {
              const int32_t* w = tw + i + 1;  // {tk, n ns, ns..., nil, n ml, (k, v)...}
              const int32_t* p = w + 2 + w[1];
              if (p[0] != 0) continue;  // nil: selects nothing
              if (p[1] > 0 && !cand_labels.count(static_cast<uint64_t>(static_cast<uint32_t>(p[2])) << 32 |
                                                 static_cast<uint32_t>(p[3])))
                continue;
              part[ch].emplace_back(n, tw + i);
            }
          }
    });
    for (const auto& pc : part)
      for (const auto& nt : pc) base_has.emplace_back(nt.first, dict.intern(nt.second + 1, static_cast<size_t>(nt.second[0])));
  }
  std::vector<std::vector<int32_t>> has(static_cast<size_t>(n_flat));  // term ids per flat candidate pod
  for (int32_t i = 0; i < nc; ++i) {
    if (status[i] != STATUS_PENDING) continue;
    bool own_terms = false;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      for (int32_t t = A.anti_off[pod]; t < A.anti_off[pod + 1]; ++t) {
        anti_term_words(c, pod, t, words);
        has[j - base].push_back(dict.intern(words));
        own_terms = true;
      }
      std::sort(has[j - base].begin(), has[j - base].end());
      has[j - base].erase(std::unique(has[j - base].begin(), has[j - base].end()), has[j - base].end());
    }
    // its terms would have to be matched against snapshot pods whose labels
    // are unknown (added from a cluster without sr_pod_affinity)
    if (own_terms && snap->unknown_total > 0) status[i] = SR_CAND_FALLBACK;
  }
  // ---- the terms that matter to this call: InterPodAffinity for a pod P
  // reads only the existing pods' terms that select P and P's own terms, so a
  // term no pending candidate pod has or is selected by constrains nothing
  // here (a prefix batch of 16 candidates keeps a handful of the snapshot's
  // thousands of Deployment terms).  Kept terms are renumbered densely.
  std::vector<Term> terms;
  {
    const int32_t T_all = static_cast<int32_t>(dict.size());
    std::vector<Term> all(static_cast<size_t>(T_all));
    for (int32_t t = 0; t < T_all; ++t) all[t] = parse_term(dict.data(t));
    std::vector<uint8_t> keep(static_cast<size_t>(T_all), 0);
    std::unordered_map<uint64_t, std::vector<int32_t>> idx;
    std::vector<int32_t> unidx;
    for (int32_t t = 0; t < T_all; ++t) {
      if (all[t].nil) continue;
      if (all[t].ml.empty()) unidx.push_back(t);
      else idx[static_cast<uint64_t>(static_cast<uint32_t>(all[t].ml[0].first)) << 32 |
               static_cast<uint32_t>(all[t].ml[0].second)].push_back(t);
    }
    for (int32_t i = 0; i < nc; ++i) {
      if (status[i] != STATUS_PENDING) continue;
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
        for (int32_t t : has[j - base]) keep[t] = 1;
        const PodMeta m = meta_of(A, cands->cand_pods[j]);
        for (int32_t t : unidx)
          if (!keep[t] && term_selects(all[t], m)) keep[t] = 1;
        for (int32_t l = 0; l < m.n; ++l) {
          auto it = idx.find(static_cast<uint64_t>(static_cast<uint32_t>(m.key[l])) << 32 | static_cast<uint32_t>(m.val[l]));
          if (it == idx.end()) continue;
          for (int32_t t : it->second)
            if (!keep[t] && term_selects(all[t], m)) keep[t] = 1;
        }
      }
    }
    // numbered in the order of their words: the numbering (atoms, state-bit
    // pairs) is a function of the kept set, not of the order the snapshot's
    // pods were met in (a reuse encode's rows stay where a fresh encode puts them)
    std::vector<int32_t> order;
    for (int32_t t = 0; t < T_all; ++t)
      if (keep[t]) order.push_back(t);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      return std::lexicographical_compare(dict.data(a), dict.data(a) + dict.len(a), dict.data(b), dict.data(b) + dict.len(b));
    });
    std::vector<int32_t> nid(static_cast<size_t>(T_all), -1);
    for (int32_t t : order) {
      nid[t] = static_cast<int32_t>(terms.size());
      terms.push_back(std::move(all[t]));
    }
    size_t w2 = 0;
    for (const auto& nt : base_has)
      if (nid[nt.second] >= 0) base_has[w2++] = {nt.first, nid[nt.second]};
    base_has.resize(w2);
    for (auto& h : has)
      for (int32_t& t : h) t = nid[t];  // every term a pending pod has is kept
    if (R) {
      R->cand_labels = cand_labels;
      R->nid = std::move(nid);
      R->all = std::move(dict);
    }
  }
  const int32_t T = static_cast<int32_t>(terms.size());
  if (T == 0) return;
  at.active = true;
  at.n_terms = T;

  // ---- topology keys (few distinct: hostname, zone, ...): each spot node's
  // value, the nodes of every value, node-local keys (every node carries the
  // key, values pairwise distinct)
  struct Key {
    int32_t key;
    std::vector<int32_t> val;                                 // [n_spot], INT_MIN: absent
    std::unordered_map<int32_t, std::vector<int32_t>> nodes;  // value -> spot nodes
    bool node_local = true;
  };
  std::vector<Key> keys;
  std::vector<int32_t> kidx(static_cast<size_t>(T));
  {
    std::unordered_map<int32_t, int32_t> key_of;
    for (int32_t t = 0; t < T; ++t) {
      auto ins = key_of.emplace(terms[t].tk, static_cast<int32_t>(keys.size()));
      if (ins.second) keys.push_back(Key{terms[t].tk, {}, {}, true});
      kidx[t] = ins.first->second;
    }
  }
  parallel_for(keys.size(), 1, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      Key& K = keys[k];
      K.val.assign(static_cast<size_t>(n_spot), INT_MIN);
      for (int32_t n = 0; n < n_spot; ++n) {
        for (const auto& kv : snap->nodes[n].labels)
          if (kv.first == K.key) {
            K.val[n] = kv.second;
            break;
          }
        if (K.val[n] == INT_MIN) {
          K.node_local = false;
          continue;
        }
        std::vector<int32_t>& ns = K.nodes[K.val[n]];
        ns.push_back(n);
        if (ns.size() > 1) K.node_local = false;
      }
    }
  });
  at.node_local.assign(static_cast<size_t>(T), 0);
  for (int32_t t = 0; t < T; ++t) at.node_local[t] = keys[kidx[t]].node_local;

  // ---- which terms select a pod: an index on each term's first MatchLabels
  // pair (a pod can only be selected through one of its own labels); terms
  // without MatchLabels are tried on every pod, nil selectors never
  LabelIndex by_label;
  std::vector<int32_t> unindexed;
  for (int32_t t = 0; t < T; ++t) {
    if (terms[t].nil) continue;
    if (terms[t].ml.empty()) unindexed.push_back(t);
    else by_label[label_key(terms[t].ml[0].first, terms[t].ml[0].second)].push_back(t);
  }
  auto selecting = [&](const PodMeta& m, auto&& f) { for_each_selecting(terms, by_label, unindexed, m, f); };

  // ---- domains of the base pods: SA(t) values hosting a pod that has t,
  // SB(t) values hosting a pod t selects
  std::vector<std::vector<int32_t>> sa(static_cast<size_t>(T)), sb(static_cast<size_t>(T));
  for (const auto& nt : base_has) {
    const int32_t v = keys[kidx[nt.second]].val[nt.first];
    if (v != INT_MIN) sa[nt.second].push_back(v);
  }
  {
    constexpr size_t kNodes = 64;
    std::vector<std::vector<std::pair<int32_t, int32_t>>> part((static_cast<size_t>(n_spot) + kNodes - 1) / kNodes);
    parallel_for(part.size(), 1, [&](size_t lo, size_t hi) {
      for (size_t ch = lo; ch < hi; ++ch)
        for (int32_t n = static_cast<int32_t>(ch * kNodes); n < std::min<int32_t>(n_spot, (ch + 1) * kNodes); ++n)
          for (int32_t e : snap->state[n].pods)
            selecting(meta_of(snap, snap->pods[e]), [&](int32_t t) { part[ch].emplace_back(t, n); });
    });
    for (const auto& pc : part)
      for (const auto& tn : pc) {
        const int32_t v = keys[kidx[tn.first]].val[tn.second];
        if (v != INT_MIN) sb[tn.first].push_back(v);
      }
    if (R) {  // per node: the pods' (term, side) codes, and the counts per value
      R->total.assign(static_cast<size_t>(2 * T), 0);
      for (const auto& nt : base_has) R->contrib[nt.first].push_back(2 * nt.second);
      for (const auto& pc : part)
        for (const auto& tn : pc) R->contrib[tn.second].push_back(2 * tn.first + 1);
      for (int32_t n = 0; n < n_spot; ++n) {
        std::sort(R->contrib[n].begin(), R->contrib[n].end());
        for (int32_t code : R->contrib[n]) {
          const int32_t v = keys[kidx[code >> 1]].val[n];
          if (v == INT_MIN) continue;
          ++R->total[code];
          ++R->cnt[static_cast<uint64_t>(code) << 32 | static_cast<uint32_t>(v)];
        }
      }
    }
  }
  at.da.assign(static_cast<size_t>(T) * Wp, 0);
  at.db.assign(static_cast<size_t>(T) * Wp, 0);
  at.da_any.assign(static_cast<size_t>(T), 0);
  at.db_any.assign(static_cast<size_t>(T), 0);
  parallel_for(static_cast<size_t>(T), 8, [&](size_t lo, size_t hi) {
    for (size_t t = lo; t < hi; ++t) {
      const Key& K = keys[kidx[t]];
      for (int side = 0; side < 2; ++side) {
        std::vector<int32_t>& s = side ? sb[t] : sa[t];
        std::sort(s.begin(), s.end());
        s.erase(std::unique(s.begin(), s.end()), s.end());
        uint64_t* row = (side ? at.db.data() : at.da.data()) + t * Wp;
        for (int32_t v : s) {
          auto it = K.nodes.find(v);
          if (it == K.nodes.end()) continue;
          for (int32_t n : it->second) row[n >> 6] |= 1ull << (n & 63);
        }
        (side ? at.db_any : at.da_any)[t] = !s.empty();
      }
    }
  });
  if (R) {
    R->terms = terms;
    R->by_label = by_label;
    R->unindexed = unindexed;
    R->kidx = kidx;
    R->keys.resize(keys.size());
    for (size_t k = 0; k < keys.size(); ++k) {
      R->keys[k].val = keys[k].val;
      R->keys[k].nodes = keys[k].nodes;
    }
    R->any_built.resize(static_cast<size_t>(2 * T));
    for (int32_t t = 0; t < T; ++t) {
      R->any_built[2 * t] = at.da_any[t];
      R->any_built[2 * t + 1] = at.db_any[t];
    }
  }

  // ---- per pending candidate pod: ids t << 1 (t selects it) | t << 1 | 1 (it has t)
  std::vector<std::vector<int32_t>> ids(static_cast<size_t>(n_flat));
  parallel_for(static_cast<size_t>(nc), 16, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      if (status[i] != STATUS_PENDING) continue;
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
        const int32_t pod = cands->cand_pods[j];
        std::vector<int32_t>& v = ids[j - base];
        selecting(meta_of(A, pod), [&](int32_t t) { v.push_back(t << 1); });
        for (int32_t t : has[j - base]) v.push_back(t << 1 | 1);
        std::sort(v.begin(), v.end());
      }
    }
  });

  // ---- interactions inside each candidate: terms one pod has and another
  // pod matches.  Node-local ones get a bit pair of the candidate's own (the
  // state is per candidate; base conflicts are in the F rows already), at most
  // 32; the others ("far" terms) put the candidate on the domain path.
  at.pod_bits.assign(static_cast<size_t>(n_flat), 0);
  std::vector<int32_t> pairs(static_cast<size_t>(nc), 0);
  std::vector<std::vector<int32_t>> far_of(static_cast<size_t>(nc));
  parallel_for(static_cast<size_t>(nc), 16, [&](size_t lo, size_t hi) {
    std::vector<int32_t> nh(static_cast<size_t>(T)), nm(static_cast<size_t>(T)), nb(static_cast<size_t>(T));
    std::vector<int32_t> pair(static_cast<size_t>(T), -1), touched, need, far;
    for (size_t i = lo; i < hi; ++i) {
      if (status[i] != STATUS_PENDING) continue;
      touched.clear();
      need.clear();
      far.clear();
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
        const std::vector<int32_t>& v = ids[j - base];
        for (size_t k = 0; k < v.size(); ++k) {
          const int32_t t = v[k] >> 1;
          if (nh[t] == 0 && nm[t] == 0) touched.push_back(t);
          if (v[k] & 1) {
            ++nh[t];
            if (k > 0 && v[k - 1] == (t << 1)) ++nb[t];  // sorted: "selects" precedes "has"
          } else {
            ++nm[t];
          }
        }
      }
      std::sort(touched.begin(), touched.end());
      for (int32_t t : touched) {
        const bool interacts = nh[t] >= 1 && nm[t] >= 1 && !(nh[t] == 1 && nm[t] == 1 && nb[t] == 1);
        if (interacts) {
          if (!at.node_local[t]) far.push_back(t);
          else need.push_back(t);
        }
        nh[t] = nm[t] = nb[t] = 0;
      }
      if (need.size() > 32 || (!far.empty() && cands->cand_pod_off[i + 1] - cands->cand_pod_off[i] > kDynPods)) {
        status[i] = SR_CAND_FALLBACK;
        continue;
      }
      if (!far.empty()) far_of[i] = far;
      for (size_t p = 0; p < need.size(); ++p) pair[need[p]] = static_cast<int32_t>(p);
      for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
        uint64_t bits = 0;
        for (int32_t id : ids[j - base]) {
          const int32_t p = pair[id >> 1];
          if (p >= 0) bits |= 1ull << (2 * p + ((id & 1) ? 0 : 1));  // A: it has t, B: t selects it
        }
        at.pod_bits[j - base] = bits;
      }
      for (int32_t t : need) pair[t] = -1;
      pairs[i] = static_cast<int32_t>(need.size());
    }
  });
  for (int32_t i = 0; i < nc; ++i) at.n_pairs = std::max(at.n_pairs, pairs[i]);

  // ---- domain path: per pod, the earlier pods of its candidate it interacts
  // with through each far term's key (either has the term and the other one
  // matches it): the device refuses it the domains they were placed in
  std::vector<int32_t> fslot;
  for (int32_t i = 0; i < nc; ++i) {
    if (far_of[i].empty() || status[i] != STATUS_PENDING) continue;
    fslot.clear();
    bool ok = true;
    for (int32_t t : far_of[i]) {
      const int32_t sl = dk->slot(snap, terms[t].tk);
      ok = ok && sl >= 0;
      fslot.push_back(sl);
    }
    if (!ok) {
      status[i] = SR_CAND_FALLBACK;
      continue;
    }
    if (at.amask.empty()) {
      at.amask.assign(static_cast<size_t>(n_flat) * kDomKeys * kDynG, 0);
      at.cand_dyn.assign(static_cast<size_t>(nc), 0);
    }
    at.cand_dyn[i] = 1;
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    auto has = [&](int32_t j, int32_t id) { return std::binary_search(ids[j - base].begin(), ids[j - base].end(), id); };
    for (int32_t q = b + 1; q < e; ++q)
      for (int32_t p = b; p < q; ++p)
        for (size_t f = 0; f < far_of[i].size(); ++f) {
          const int32_t t = far_of[i][f];
          if ((has(p, t << 1 | 1) && has(q, t << 1)) || (has(q, t << 1 | 1) && has(p, t << 1)))
            at.amask[(static_cast<size_t>(q - base) * kDomKeys + fslot[f]) * kDynG + (p - b) / 64] |=
                1ull << ((p - b) % 64);
        }
  }

  // ---- CSR of the ids
  for (int32_t j = 0; j < n_flat; ++j) at.pod_off[j + 1] = at.pod_off[j] + static_cast<int32_t>(ids[j].size());
  at.pod_ids.reserve(static_cast<size_t>(at.pod_off[n_flat]));
  for (int32_t j = 0; j < n_flat; ++j) at.pod_ids.insert(at.pod_ids.end(), ids[j].begin(), ids[j].end());
}

// Required pod affinity (InterPodAffinity.Filter, satisfyPodAffinity [upstream
// k8s v1.19.2 plugins/interpodaffinity/filtering.go]).  A pod's terms form a
// set S (canonical words of its resolved terms); M(S) = the snapshot pods that
// match every term of S (updateWithAffinityTerms counts only those).  Per set:
// KEYS(S) = nodes carrying every term's topology key; SAT(S) = KEYS(S) and,
// per term, a pod of M(S) in the node's domain of the term's key; map_empty =
// no pod of M(S) runs on a node carrying any of the keys.  A pod passes a node
// of SAT(S) -- or, with map_empty and the pod matching its own terms (the
// first pod of a self-affine group), a node of KEYS(S).  A candidate in which
// an earlier pod matches every term of a later pod's set changes that pod's
// pair map while it is planned: it takes K2's domain path, where the later
// pod's class carries KEYS(S) and the device adds, per term, the domains of
// the earlier matching pods' nodes to the base row (and drops the map-empty
// exception once one of them sits on a node with a key).
void analyse_affinity(const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands, int32_t Wp,
                      std::vector<int32_t>& status, DomKeys* dk, AffTerms* out) {
  AffTerms& af = *out;
  af = AffTerms{};
  const sr_pod_affinity* PA = c->pod_affinity;
  const int32_t nc = cands->n_cand;
  const int32_t base = nc > 0 ? cands->cand_pod_off[0] : 0;
  const int32_t n_flat = nc > 0 ? cands->cand_pod_off[nc] - base : 0;
  af.base = base;
  af.pod_code.assign(static_cast<size_t>(n_flat), -1);
  if (!PA || !PA->aff_off) return;
  const sr_pod_affinity& A = *PA;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());

  // ---- distinct sets of the pending candidates' pods
  WordDict set_dict;
  std::vector<std::vector<Term>> sets;
  std::vector<std::vector<int32_t>> tws;
  std::vector<int32_t> words, setw;
  for (int32_t i = 0; i < nc; ++i) {
    if (status[i] != STATUS_PENDING) continue;
    bool any = false;
    for (int32_t j = cands->cand_pod_off[i]; j < cands->cand_pod_off[i + 1]; ++j) {
      const int32_t pod = cands->cand_pods[j];
      if (A.aff_off[pod] == A.aff_off[pod + 1]) continue;
      any = true;
      tws.clear();
      for (int32_t t = A.aff_off[pod]; t < A.aff_off[pod + 1]; ++t) {
        anti_term_words(c, pod, t, words);
        tws.push_back(words);
      }
      std::sort(tws.begin(), tws.end());
      tws.erase(std::unique(tws.begin(), tws.end()), tws.end());
      setw.assign(1, static_cast<int32_t>(tws.size()));
      for (const auto& tw : tws) {
        setw.push_back(static_cast<int32_t>(tw.size()));
        setw.insert(setw.end(), tw.begin(), tw.end());
      }
      bool ins = false;
      const int32_t sid = set_dict.intern(setw, &ins);
      if (ins) {
        sets.emplace_back();
        for (const auto& tw : tws) sets.back().push_back(parse_term(tw.data()));
      }
      bool self = true;  // podMatchesAllAffinityTerms(pod, its own terms)
      for (const Term& t : sets[sid]) self = self && term_selects(t, meta_of(A, pod));
      af.pod_code[j - base] = 2 * sid + (self ? 1 : 0);
    }
    // snapshot pods whose labels are unknown may match its terms
    if (any && snap->unknown_total > 0) status[i] = SR_CAND_FALLBACK;
  }
  const int32_t S = static_cast<int32_t>(sets.size());
  if (S == 0) return;
  af.active = true;
  af.n_sets = S;

  // ---- topology key values of the spot nodes (few distinct keys)
  std::vector<int32_t> key_ids;
  std::vector<std::vector<int32_t>> key_val;  // [key][node], INT_MIN: absent
  auto key_slot = [&](int32_t key) {
    for (size_t k = 0; k < key_ids.size(); ++k)
      if (key_ids[k] == key) return static_cast<int32_t>(k);
    key_ids.push_back(key);
    key_val.emplace_back(static_cast<size_t>(n_spot), INT_MIN);
    std::vector<int32_t>& v = key_val.back();
    for (int32_t n = 0; n < n_spot; ++n)
      for (const auto& kv : snap->nodes[n].labels)
        if (kv.first == key) {
          v[n] = kv.second;
          break;
        }
    return static_cast<int32_t>(key_ids.size() - 1);
  };
  std::vector<std::vector<int32_t>> set_keys(static_cast<size_t>(S));
  for (int32_t s = 0; s < S; ++s)
    for (const Term& t : sets[s]) set_keys[s].push_back(key_slot(t.tk));

  // ---- M(S) over the snapshot pods: per set and term, the key values of
  // the nodes hosting a matching pod; map_empty
  std::vector<std::vector<std::vector<int32_t>>> vals(static_cast<size_t>(S));
  for (int32_t s = 0; s < S; ++s) vals[s].resize(sets[s].size());
  af.map_empty.assign(static_cast<size_t>(S), 1);
  for (int32_t n = 0; n < n_spot; ++n)
    for (int32_t e : snap->state[n].pods) {
      const SnapPod& sp = snap->pods[e];
      if (!sp.meta) continue;  // candidates with terms already fell back
      const PodMeta m = meta_of(snap, sp);
      for (int32_t s = 0; s < S; ++s) {
        bool all = true;
        for (const Term& t : sets[s]) all = all && term_selects(t, m);
        if (!all) continue;
        for (size_t t = 0; t < sets[s].size(); ++t) {
          const int32_t v = key_val[set_keys[s][t]][n];
          if (v == INT_MIN) continue;
          vals[s][t].push_back(v);
          af.map_empty[s] = 0;
        }
      }
    }
  af.sat.assign(static_cast<size_t>(S) * Wp, 0);
  af.keys.assign(static_cast<size_t>(S) * Wp, 0);
  for (int32_t s = 0; s < S; ++s) {
    for (auto& v : vals[s]) {
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
    }
    for (int32_t n = 0; n < n_spot; ++n) {
      bool keys = true, sat = true;
      for (size_t t = 0; t < sets[s].size(); ++t) {
        const int32_t v = key_val[set_keys[s][t]][n];
        keys = keys && v != INT_MIN;
        sat = sat && v != INT_MIN && std::binary_search(vals[s][t].begin(), vals[s][t].end(), v);
      }
      if (keys) af.keys[static_cast<size_t>(s) * Wp + (n >> 6)] |= 1ull << (n & 63);
      if (sat) af.sat[static_cast<size_t>(s) * Wp + (n >> 6)] |= 1ull << (n & 63);
    }
  }

  // ---- interactions inside a candidate: an earlier pod matching every term
  // of a later pod's set adds its domains to that pod's pair map while the
  // candidate is planned: the candidate takes K2's domain path (per pod, the
  // mask of those earlier pods), or the fallback path beyond its limits
  std::vector<uint64_t> masks;  // [pod of the candidate][kDynG]
  for (int32_t i = 0; i < nc; ++i) {
    if (status[i] != STATUS_PENDING) continue;
    const int32_t b = cands->cand_pod_off[i], e = cands->cand_pod_off[i + 1];
    masks.assign(static_cast<size_t>(e - b) * kDynG, 0);
    bool any = false;
    for (int32_t k = b + 1; k < e; ++k) {
      const int32_t code = af.pod_code[k - base];
      if (code < 0) continue;
      for (int32_t q = b; q < k; ++q) {
        const PodMeta m = meta_of(A, cands->cand_pods[q]);
        bool all = true;
        for (const Term& t : sets[code >> 1]) all = all && term_selects(t, m);
        if (all && q - b < kDynPods) masks[static_cast<size_t>(k - b) * kDynG + (q - b) / 64] |= 1ull << ((q - b) % 64);
        any = any || all;
      }
    }
    if (!any) continue;
    bool ok = e - b <= kDynPods;
    auto masked = [&](int32_t k) {
      for (int g = 0; g < kDynG; ++g)
        if (masks[static_cast<size_t>(k - b) * kDynG + g] != 0) return true;
      return false;
    };
    for (int32_t k = b; k < e && ok; ++k) {
      if (!masked(k)) continue;
      const int32_t set = af.pod_code[k - base] >> 1;
      ok = sets[set].size() <= static_cast<size_t>(kDynTerms);
      for (size_t t = 0; t < sets[set].size() && ok; ++t) ok = dk->slot(snap, sets[set][t].tk) >= 0;
    }
    if (!ok) {
      status[i] = SR_CAND_FALLBACK;
      continue;
    }
    if (af.mmask.empty()) {
      af.mmask.assign(static_cast<size_t>(n_flat) * kDynG, 0);
      af.cand_dyn.assign(static_cast<size_t>(nc), 0);
      af.set_dyn.assign(static_cast<size_t>(S), 0);
      af.set_slots.resize(static_cast<size_t>(S));
      af.term_rows.resize(static_cast<size_t>(S));
    }
    af.cand_dyn[i] = 1;
    for (int32_t k = b; k < e; ++k) {
      std::copy_n(&masks[static_cast<size_t>(k - b) * kDynG], kDynG, &af.mmask[static_cast<size_t>(k - base) * kDynG]);
      if (masked(k)) af.set_dyn[af.pod_code[k - base] >> 1] = 1;
    }
  }
  // per set planned there: each term's key slot, and its base row (nodes
  // whose domain of the term's key hosts a snapshot pod of M(S))
  for (int32_t s = 0; s < static_cast<int32_t>(af.set_dyn.size()); ++s) {
    if (!af.set_dyn[s]) continue;
    const size_t nt = sets[s].size();
    af.set_slots[s].resize(nt);
    af.term_rows[s].assign(nt * Wp, 0);
    for (size_t t = 0; t < nt; ++t) {
      af.set_slots[s][t] = dk->slot(snap, sets[s][t].tk);
      const std::vector<int32_t>& kv = key_val[set_keys[s][t]];
      for (int32_t n = 0; n < n_spot; ++n)
        if (kv[n] != INT_MIN && std::binary_search(vals[s][t].begin(), vals[s][t].end(), kv[n]))
          af.term_rows[s][t * Wp + (n >> 6)] |= 1ull << (n & 63);
    }
  }
}

}  // namespace sr
