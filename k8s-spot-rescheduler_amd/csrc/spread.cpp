// spread.cpp — PodTopologySpread (whenUnsatisfiable: DoNotSchedule) for the encoder.
//
// k8s v1.19.2 plugins/podtopologyspread/filtering.go [upstream, not vendored;
// run by CheckPredicates, rescheduler.go:344]:
//  - PreFilter (calPreFilterState): the pairs (topologyKey, value) of the
//    snapshot nodes that pass the pod's nodeSelector / required node affinity
//    and carry every constraint's key; per pair the pods on every node whose
//    value of that key is the pair's, counted per constraint when they are in
//    the pod's namespace, not terminating and selected by the constraint's
//    selector (two constraints on one key add into one pair); per key the
//    minimum over its pairs (TpKeyToCriticalPaths[0]);
//  - Filter: no pair at all passes every node; otherwise a node lacking a
//    constraint's key fails, and a node whose pair count + (the pod selects
//    itself) - the key's minimum exceeds maxSkew fails.
//
// Encoding: with the counts taken over the base snapshot,
// the result for a pod is one node row -- a static atom of its class, one per
// spec carrying constraints.  That is exact while no earlier pod of the same
// candidate is counted by the pod's constraints.  A candidate with such pods
// is planned on K2's domain path (encode.cpp analyse_spread, kernels.hip
// k2_domain): the device adds the earlier pods to the pair counts; the pod's
// atom keeps only the key check of a device-planned table-key constraint
// (`dmask`), and the full base check of a node-local one, whose minimum the
// encoder proved cannot move.  Selectors that fail to build go to the
// reference path.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <unordered_map>

#include "host.hpp"
#include "pool.hpp"

namespace sr {

namespace {

bool cluster_label(const sr_cluster* c, int32_t pod, int32_t key, int32_t* val) {
  const sr_pod_affinity* A = c->pod_affinity;
  for (int32_t i = A->label_off[pod]; i < A->label_off[pod + 1]; ++i)
    if (A->label_key[i] == key) {
      *val = A->label_val[i];
      return true;
    }
  return false;
}

bool in_sorted(const int32_t* v, int32_t n, int32_t x) { return std::binary_search(v, v + n, x); }

// One constraint parsed from its words.
struct Constraint {
  int32_t max_skew, key, self;
  bool nil;
  const int32_t* ml;  // (key, value)*
  int32_t n_ml;
  std::vector<const int32_t*> me;  // {key, op, n, values...} each
};

// {nil, n matchLabels, (key, value)*, n matchExpressions, (key, op, n, values)*}
const int32_t* parse_sel(const int32_t* w, Constraint* c) {
  c->nil = *w++ != 0;
  c->n_ml = *w++;
  c->ml = w;
  w += 2 * c->n_ml;
  const int32_t n_me = *w++;
  c->me.clear();
  for (int32_t e = 0; e < n_me; ++e) {
    c->me.push_back(w);
    w += 3 + w[2];
  }
  return w;
}

const int32_t* parse(const int32_t* w, Constraint* c) {
  c->max_skew = *w++;
  c->key = *w++;
  c->self = *w++;
  return parse_sel(w, c);
}

// labels.Selector.Matches over a snapshot pod's labels (the namespace is the caller's check).
bool selects(const Constraint& k, const int32_t* lk, const int32_t* lv, int32_t nl) {
  if (k.nil) return false;  // LabelSelectorAsSelector(nil) = labels.Nothing()
  auto label = [&](int32_t key, int32_t* v) {
    for (int32_t i = 0; i < nl; ++i)
      if (lk[i] == key) {
        *v = lv[i];
        return true;
      }
    return false;
  };
  int32_t v;
  for (int32_t i = 0; i < k.n_ml; ++i)
    if (!label(k.ml[2 * i], &v) || v != k.ml[2 * i + 1]) return false;
  for (const int32_t* e : k.me) {
    const bool has = label(e[0], &v);
    bool ok;
    switch (e[1]) {
      case SR_OP_IN: ok = has && in_sorted(e + 3, e[2], v); break;
      case SR_OP_NOT_IN: ok = !has || !in_sorted(e + 3, e[2], v); break;
      case SR_OP_EXISTS: ok = has; break;
      default: ok = !has; break;  // DoesNotExist (anything else fails to build: never encoded)
    }
    if (!ok) return false;
  }
  return true;
}

inline uint64_t pair_key(int32_t key, int32_t val) {
  return static_cast<uint64_t>(static_cast<uint32_t>(key)) << 32 | static_cast<uint32_t>(val);
}

}  // namespace

bool spread_invalid(const sr_cluster* c, int32_t k) {
  const sr_spread* S = c->spread;
  // maxSkew < 1 never reaches the scheduler (API validation rejects it); the
  // encoded forms (domain path, node-local caps) assume maxSkew >= 1, so the
  // C ABI routes such a constraint to the reference path instead of guessing
  if (S->max_skew[k] < 1) return true;
  if (S->selector_nil[k]) return false;
  for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1]; ++i)
    if (!label_req_strings_ok(c, S->ml_key[i], S->ml_val, i, i + 1)) return true;
  for (int32_t e = S->me_off[k]; e < S->me_off[k + 1]; ++e) {
    const int32_t nv = S->me_val_off[e + 1] - S->me_val_off[e], op = S->me_op[e];
    if (!label_req_strings_ok(c, S->me_key[e], S->me_vals, S->me_val_off[e], S->me_val_off[e + 1])) return true;
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

bool spread_selects(const sr_cluster* c, int32_t k, int32_t pod) {
  const sr_spread* S = c->spread;
  if (S->selector_nil[k]) return false;
  int32_t v;
  for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1]; ++i)
    if (!cluster_label(c, pod, S->ml_key[i], &v) || v != S->ml_val[i]) return false;
  for (int32_t e = S->me_off[k]; e < S->me_off[k + 1]; ++e) {
    const bool has = cluster_label(c, pod, S->me_key[e], &v);
    const int32_t* vals = S->me_vals + S->me_val_off[e];
    const int32_t nv = S->me_val_off[e + 1] - S->me_val_off[e];
    const bool in = has && std::find(vals, vals + nv, v) != vals + nv;
    bool ok;
    switch (S->me_op[e]) {
      case SR_OP_IN: ok = in; break;
      case SR_OP_NOT_IN: ok = !in; break;
      case SR_OP_EXISTS: ok = has; break;
      case SR_OP_DOES_NOT_EXIST: ok = !has; break;
      default: ok = false; break;
    }
    if (!ok) return false;
  }
  return true;
}

SpreadIndex::SpreadIndex(const sr_snapshot* s)
    : snap(s), n_spot(static_cast<int32_t>(s->nodes.size())), Wp(std::max(2, ((n_spot + 63) / 64 + 1) & ~1)) {}

const SpreadIndex::KeyView& SpreadIndex::key(int32_t k) {
  auto it = keys.find(k);
  if (it != keys.end()) return it->second;
  KeyView& v = keys[k];
  v.val.assign(static_cast<size_t>(n_spot), INT32_MIN);
  v.has.assign(static_cast<size_t>(Wp), 0);
  std::unordered_map<int32_t, int32_t> slot;
  for (int32_t n = 0; n < n_spot; ++n)
    for (const auto& kv : snap->nodes[n].labels)
      if (kv.first == k) {
        v.val[n] = kv.second;
        v.has[n >> 6] |= 1ull << (n & 63);
        auto ins = slot.emplace(kv.second, static_cast<int32_t>(v.values.size()));
        if (ins.second) {
          v.values.push_back(kv.second);
          v.bits.resize(v.values.size() * static_cast<size_t>(Wp), 0);
        }
        v.bits[static_cast<size_t>(ins.first->second) * Wp + (n >> 6)] |= 1ull << (n & 63);
      }
  // processNode's pair of each node: its value's, "" for a node without the key
  const auto e = slot.find(snap->id_empty);
  const int32_t empty_slot = e == slot.end() ? -1 : e->second;
  v.slot.assign(static_cast<size_t>(n_spot), -1);
  for (int32_t n = 0; n < n_spot; ++n) v.slot[n] = v.val[n] == INT32_MIN ? empty_slot : slot[v.val[n]];
  return v;
}

const std::vector<std::pair<int32_t, int32_t>>* SpreadIndex::pods_with(int32_t k, int32_t v) {
  auto it = by_key.find(k);
  if (it == by_key.end() || !it->second.pods.count(v)) {  // (re)build the column of key k
    std::vector<int32_t>& vals = wanted[k];
    if (std::find(vals.begin(), vals.end(), v) == vals.end()) vals.push_back(v);
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    // snapshot pods in node chunks on the pool; each chunk keeps the (value,
    // node, pod) of wanted values in node order
    constexpr int32_t kNodes = 256;
    const size_t n_parts = (static_cast<size_t>(n_spot) + kNodes - 1) / kNodes;
    struct Hit {
      int32_t v, n, e;
    };
    std::vector<std::vector<Hit>> part(n_parts);
    parallel_for(n_parts, 1, [&](size_t lo, size_t hi) {
      for (size_t ch = lo; ch < hi; ++ch)
        for (int32_t n = static_cast<int32_t>(ch) * kNodes; n < std::min<int32_t>(n_spot, (ch + 1) * kNodes); ++n)
          for (int32_t e : snap->state[n].pods) {
            const SnapPod& sp = snap->pods[e];
            for (uint32_t i = 0; i < sp.nlab; ++i)
              if (snap->lkey[sp.lab + i] == k) {
                const int32_t x = snap->lval[sp.lab + i];
                if (std::binary_search(vals.begin(), vals.end(), x)) part[ch].push_back(Hit{x, n, e});
                break;  // keys are unique per pod
              }
          }
    });
    LabelCol& col = by_key[k];
    col.pods.clear();
    for (int32_t x : vals) col.pods[x];  // wanted values without pods: an empty list
    for (const auto& pc : part)
      for (const Hit& h : pc) col.pods[h.v].emplace_back(h.n, h.e);
    it = by_key.find(k);
  }
  const auto& lst = it->second.pods.find(v)->second;
  return lst.empty() ? nullptr : &lst;
}

void spread_node_counts(SpreadIndex& ix, const sr_cluster* c, int32_t k, int32_t ns, std::vector<int32_t>& out) {
  const sr_snapshot* snap = ix.snap;
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  const sr_spread* S = c->spread;
  out.assign(static_cast<size_t>(n_spot), 0);
  if (S->selector_nil[k]) return;
  // a matchLabels pair bounds the pods to test: those carrying it
  std::vector<std::pair<int32_t, int32_t>> all;
  const std::vector<std::pair<int32_t, int32_t>>* list = nullptr;
  if (S->ml_off[k + 1] > S->ml_off[k]) {
    int32_t f = S->ml_off[k];  // the pair with the smallest key (spread_words' first)
    for (int32_t i = S->ml_off[k] + 1; i < S->ml_off[k + 1]; ++i)
      if (S->ml_key[i] < S->ml_key[f]) f = i;
    list = ix.pods_with(S->ml_key[f], S->ml_val[f]);
    if (!list) return;
  } else {
    for (int32_t n = 0; n < n_spot; ++n)
      for (int32_t e : snap->state[n].pods) all.emplace_back(n, e);
    list = &all;
  }
  for (const auto& ne : *list) {
    const int32_t n = ne.first, e = ne.second;
    {
      const SnapPod& sp = snap->pods[e];
      if (sp.term || sp.ns != ns) continue;
      const int32_t *lk = snap->lkey.data() + sp.lab, *lv = snap->lval.data() + sp.lab;
      const int32_t nl = static_cast<int32_t>(sp.nlab);
      auto label = [&](int32_t key, int32_t* v) {
        for (int32_t i = 0; i < nl; ++i)
          if (lk[i] == key) {
            *v = lv[i];
            return true;
          }
        return false;
      };
      bool ok = true;
      int32_t v;
      for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1] && ok; ++i) ok = label(S->ml_key[i], &v) && v == S->ml_val[i];
      for (int32_t x = S->me_off[k]; x < S->me_off[k + 1] && ok; ++x) {
        const bool has = label(S->me_key[x], &v);
        const int32_t* vals = S->me_vals + S->me_val_off[x];
        const int32_t nv = S->me_val_off[x + 1] - S->me_val_off[x];
        const bool in = has && std::find(vals, vals + nv, v) != vals + nv;
        switch (S->me_op[x]) {
          case SR_OP_IN: ok = in; break;
          case SR_OP_NOT_IN: ok = !in; break;
          case SR_OP_EXISTS: ok = has; break;
          default: ok = !has; break;  // DoesNotExist (anything else fails to build: never encoded)
        }
      }
      if (ok) ++out[n];
    }
  }
}

namespace {

// {nil, n matchLabels, (key, value)* sorted, n matchExpressions, (key, op, n, values sorted)*} of constraint k
void append_selector(const sr_cluster* c, int32_t k, std::vector<int32_t>& out) {
  const sr_spread* S = c->spread;
  out.push_back(S->selector_nil[k] ? 1 : 0);
  std::vector<std::pair<int32_t, int32_t>> ml;
  if (!S->selector_nil[k])
    for (int32_t i = S->ml_off[k]; i < S->ml_off[k + 1]; ++i) ml.emplace_back(S->ml_key[i], S->ml_val[i]);
  std::sort(ml.begin(), ml.end());
  out.push_back(static_cast<int32_t>(ml.size()));
  for (const auto& kv : ml) {
    out.push_back(kv.first);
    out.push_back(kv.second);
  }
  const int32_t e0 = S->selector_nil[k] ? 0 : S->me_off[k], e1 = S->selector_nil[k] ? 0 : S->me_off[k + 1];
  out.push_back(e1 - e0);
  for (int32_t e = e0; e < e1; ++e) {
    out.push_back(S->me_key[e]);
    out.push_back(S->me_op[e]);
    const size_t at = out.size();
    out.push_back(0);
    out.insert(out.end(), S->me_vals + S->me_val_off[e], S->me_vals + S->me_val_off[e + 1]);
    std::sort(out.begin() + at + 1, out.end());
    out.erase(std::unique(out.begin() + at + 1, out.end()), out.end());
    out[at] = static_cast<int32_t>(out.size() - at - 1);
  }
}

}  // namespace

void spread_selector_words(const sr_cluster* c, int32_t ns, int32_t k, std::vector<int32_t>& out) {
  out.clear();
  out.push_back(ns);
  append_selector(c, k, out);
}

void spread_words(const sr_cluster* c, int32_t pod, std::vector<int32_t>& out) {
  const sr_spread* S = c->spread;
  out.clear();
  out.push_back(c->pod_affinity->ns[pod]);
  out.push_back(S->off[pod + 1] - S->off[pod]);
  for (int32_t k = S->off[pod]; k < S->off[pod + 1]; ++k) {
    out.push_back(S->max_skew[k]);
    out.push_back(S->topology_key[k]);
    out.push_back(spread_selects(c, k, pod) ? 1 : 0);
    append_selector(c, k, out);
  }
}

struct SpreadReuse {
  int32_t n_spot = 0, Wp = 0;
  struct Counter {
    std::vector<int32_t> words;                 // spread_selector_words
    std::vector<std::pair<int32_t, int32_t>> nz;  // (spot node, pods) where it counts any
    bool changed = false;
    int32_t get(int32_t n) const {
      for (const auto& e : nz)
        if (e.first == n) return e.second;
      return 0;
    }
    void set(int32_t n, int32_t x) {
      for (size_t i = 0; i < nz.size(); ++i)
        if (nz[i].first == n) {
          if (x) nz[i].second = x;
          else nz.erase(nz.begin() + static_cast<std::ptrdiff_t>(i));
          return;
        }
      if (x) nz.emplace_back(n, x);
    }
  };
  std::vector<Counter> ctr;
  std::map<std::vector<int32_t>, int32_t> ctr_of;
  // the counters a pod can be counted by: through the first matchLabels pair
  // of their words (the pod must carry it), or tried on every pod
  std::unordered_map<uint64_t, std::vector<int32_t>> by_label;
  std::vector<int32_t> unindexed;
  std::vector<std::vector<int32_t>> node_nz;   // [spot node] counters with pods there
  std::unordered_map<int32_t, SpreadIndex::KeyView> keys;  // copies of the encode's key views
  struct Query {
    int32_t atom;
    std::vector<int32_t> words;  // spread_words
    std::vector<uint64_t> aff;   // [Wp] NodeAffinity row
    uint32_t dmask;
    std::vector<int32_t> ctr;    // [constraint] counter (-1: nil selector)
  };
  std::vector<Query> queries;
  struct Slot {
    int32_t ctr;
    uint32_t off;
    bool local;
    std::vector<uint64_t> pairs;  // node-local key: the pairs
    int32_t skew, self, n_counted;
    int32_t dom;                  // table key: index into doms
    uint64_t pm;
    int32_t edom;
  };
  std::vector<Slot> slots;
  std::vector<std::vector<int32_t>> doms;

  int32_t counter(const int32_t* w, size_t n, const std::vector<std::pair<int32_t, int32_t>>& nz) {
    std::vector<int32_t> key(w, w + n);
    auto it = ctr_of.find(key);
    if (it != ctr_of.end()) return it->second;
    const int32_t id = static_cast<int32_t>(ctr.size());
    ctr.push_back(Counter{key, nz, false});
    ctr_of.emplace(std::move(key), id);
    if (w[1] == 0) {  // not nil (a nil selector counts nothing)
      if (w[2] > 0) by_label[static_cast<uint64_t>(static_cast<uint32_t>(w[3])) << 32 | static_cast<uint32_t>(w[4])].push_back(id);
      else unindexed.push_back(id);
    }
    for (const auto& e : nz) node_nz[e.first].push_back(id);
    return id;
  }
};

std::shared_ptr<SpreadReuse> spread_reuse_new(const sr_snapshot* snap, int32_t Wp) {
  auto r = std::make_shared<SpreadReuse>();
  r->n_spot = static_cast<int32_t>(snap->nodes.size());
  r->Wp = Wp;
  r->node_nz.resize(static_cast<size_t>(r->n_spot));
  return r;
}

void spread_reuse_permute(SpreadReuse& R, const std::vector<int32_t>& src, const std::vector<int32_t>& moved,
                          std::vector<int32_t>& tab) {
  permute_positions(R.node_nz.data(), src, moved);
  const std::vector<int32_t> to = permute_targets(R.n_spot, src, moved);
  for (SpreadReuse::Counter& C : R.ctr)
    for (auto& e : C.nz) e.first = to[e.first];
  for (auto& kv : R.keys) {
    SpreadIndex::KeyView& v = kv.second;
    permute_positions(v.val.data(), src, moved);
    permute_positions(v.slot.data(), src, moved);
    permute_bits(v.has.data(), R.Wp, src, moved, to);
    auto rows = [&](size_t lo, size_t hi) {
      for (size_t j = lo; j < hi; ++j) permute_bits(v.bits.data() + j * static_cast<size_t>(R.Wp), R.Wp, src, moved, to);
    };
    if (v.values.size() > 512) parallel_for(v.values.size(), 256, rows);  // a node-local key: a row per node
    else rows(0, v.values.size());
  }
  auto aff_rows = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) permute_bits(R.queries[i].aff.data(), R.Wp, src, moved, to);
  };
  if (R.queries.size() > 512) parallel_for(R.queries.size(), 256, aff_rows);
  else aff_rows(0, R.queries.size());
  for (SpreadReuse::Slot& sl : R.slots)
    if (sl.local) {
      permute_bits(sl.pairs.data(), R.Wp, src, moved, to);
      permute_positions(tab.data() + sl.off, src, moved);
    }
  for (auto& d : R.doms) permute_positions(d.data(), src, moved);
}

void spread_reuse_slot(SpreadReuse& R, const std::vector<int32_t>& sel_words, const std::vector<int32_t>& node_cnt,
                       uint32_t off, bool node_local, const std::vector<uint64_t>& pairs, int32_t skew, int32_t self,
                       int32_t n_counted, const std::vector<int32_t>& dom, uint64_t pm, int32_t edom) {
  SpreadReuse::Slot s;
  std::vector<std::pair<int32_t, int32_t>> nz;
  for (int32_t n = 0; n < static_cast<int32_t>(node_cnt.size()); ++n)
    if (node_cnt[n]) nz.emplace_back(n, node_cnt[n]);
  s.ctr = R.counter(sel_words.data(), sel_words.size(), nz);
  s.off = off;
  s.local = node_local;
  if (node_local) s.pairs = pairs;
  s.skew = skew;
  s.self = self;
  s.n_counted = n_counted;
  s.dom = -1;
  if (!node_local) {
    for (size_t i = 0; i < R.doms.size() && s.dom < 0; ++i)
      if (R.doms[i] == dom) s.dom = static_cast<int32_t>(i);
    if (s.dom < 0) {
      R.doms.push_back(dom);
      s.dom = static_cast<int32_t>(R.doms.size() - 1);
    }
  }
  s.pm = pm;
  s.edom = edom;
  R.slots.push_back(std::move(s));
}

namespace {

using KeyView = SpreadIndex::KeyView;
using Counts = std::unordered_map<int32_t, std::vector<int64_t>>;  // key -> per value slot (-1: no such pair)

// PreFilter: the nodes passing NodeAffinity and carrying every key define the
// pairs (per key of the constraints, per value slot 0 = a pair, -1 none).
// False: no pair at all (Filter passes every node).
bool pair_slots(const std::vector<Constraint>& cs, const std::vector<const KeyView*>& kv, const uint64_t* aff_row,
                int32_t Wp, Counts& count) {
  const int32_t nk = static_cast<int32_t>(cs.size());
  std::vector<uint64_t> elig(aff_row, aff_row + Wp);
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t i = 0; i < Wp; ++i) elig[i] &= kv[k]->has[i];
  bool any = false;
  for (int32_t i = 0; i < Wp && !any; ++i) any = elig[i] != 0;
  if (!any) return false;
  // two constraints on one key add into the same pairs: counted by key
  for (int32_t k = 0; k < nk; ++k) {
    auto ins = count.emplace(cs[k].key, std::vector<int64_t>());
    if (!ins.second) continue;
    const KeyView& v = *kv[k];
    ins.first->second.assign(v.values.size(), -1);
    for (size_t j = 0; j < v.values.size(); ++j)
      for (int32_t i = 0; i < Wp; ++i)
        if (v.bits[j * Wp + i] & elig[i]) {
          ins.first->second[j] = 0;
          break;
        }
  }
  return true;
}

// Filter per node: row |= AND over the constraints of the nodes carrying a
// value whose pair count (0 without a pair) + self - the key's minimum is
// within maxSkew (a device-planned constraint: the key check only)
void filter_row(const std::vector<Constraint>& cs, const std::vector<const KeyView*>& kv, const Counts& count,
                uint32_t dmask, int32_t Wp, uint64_t* row) {
  const int32_t nk = static_cast<int32_t>(cs.size());
  std::vector<uint64_t> acc(static_cast<size_t>(Wp), ~0ull), part(static_cast<size_t>(Wp));
  for (int32_t k = 0; k < nk; ++k) {
    const KeyView& v = *kv[k];
    if ((dmask >> k) & 1) {
      for (int32_t i = 0; i < Wp; ++i) acc[i] &= v.has[i];
      continue;
    }
    const std::vector<int64_t>& cnt = count.find(cs[k].key)->second;
    int64_t mn = INT64_MAX;  // TpKeyToCriticalPaths[key][0].MatchNum: the minimum over the key's pairs
    for (int64_t x : cnt)
      if (x >= 0) mn = std::min(mn, x);
    std::fill(part.begin(), part.end(), 0ull);
    for (size_t j = 0; j < v.values.size(); ++j) {
      const int64_t match = cnt[j] < 0 ? 0 : cnt[j];
      if (match + cs[k].self - mn <= cs[k].max_skew)
        for (int32_t i = 0; i < Wp; ++i) part[i] |= v.bits[j * Wp + i];
    }
    for (int32_t i = 0; i < Wp; ++i) acc[i] &= part[i];
  }
  for (int32_t i = 0; i < Wp; ++i) row[i] |= acc[i];
}

void all_nodes(int32_t n_spot, uint64_t* row) {
  for (int32_t n = 0; n < n_spot; ++n) row[n >> 6] |= 1ull << (n & 63);
}

}  // namespace

void spread_row(SpreadIndex& ix, const int32_t* w, const uint64_t* aff_row, uint32_t dmask, uint64_t* row,
                SpreadReuse* keep, int32_t atom) {
  const sr_snapshot* snap = ix.snap;
  const int32_t n_spot = ix.n_spot, Wp = ix.Wp;  // the encoder's row width (KeyView strides)
  const int32_t ns = w[0], nk = w[1];
  std::vector<Constraint> cs(static_cast<size_t>(nk));
  std::vector<const int32_t*> sel(static_cast<size_t>(nk) + 1);  // each constraint's selector words, and the end
  const int32_t* p = w + 2;
  for (int32_t k = 0; k < nk; ++k) {
    sel[k] = p + 3;
    p = parse(p, &cs[k]);
  }
  sel[nk] = p;
  std::vector<const KeyView*> kv(static_cast<size_t>(nk));
  for (int32_t k = 0; k < nk; ++k) kv[k] = &ix.key(cs[k].key);
  Counts count;
  if (!pair_slots(cs, kv, aff_row, Wp, count)) {  // static: nothing for a reuse to follow
    all_nodes(n_spot, row);
    return;
  }
  SpreadReuse::Query q;
  if (keep) {
    q.atom = atom;
    q.words.assign(w, p);
    q.aff.assign(aff_row, aff_row + Wp);
    q.dmask = dmask;
    q.ctr.assign(static_cast<size_t>(nk), -1);
    for (int32_t k = 0; k < nk; ++k) keep->keys.emplace(cs[k].key, *kv[k]);
  }
  // processNode: every selected pod, every constraint, the pair of its node's
  // value ("" when the node lacks the key)
  std::vector<std::pair<int32_t, int32_t>> all;
  std::vector<std::pair<int32_t, int32_t>> node_cnt;  // (node, pods): the lists run in node order
  std::vector<int32_t> sel_words;
  for (int32_t k = 0; k < nk; ++k) {
    const Constraint& ck = cs[k];
    if (ck.nil) continue;
    node_cnt.clear();
    const std::vector<std::pair<int32_t, int32_t>>* list;
    if (ck.n_ml > 0) {
      list = ix.pods_with(ck.ml[0], ck.ml[1]);
    } else {
      if (all.empty())
        for (int32_t n = 0; n < n_spot; ++n)
          for (int32_t e : snap->state[n].pods) all.emplace_back(n, e);
      list = &all;
    }
    std::vector<int64_t>& cnt = count[ck.key];
    if (list)
      for (const auto& ne : *list) {
        const SnapPod& sp = snap->pods[ne.second];
        if (sp.term || sp.ns != ns) continue;  // terminating (unknown: planned on the reference path)
        if (!selects(ck, snap->lkey.data() + sp.lab, snap->lval.data() + sp.lab, static_cast<int32_t>(sp.nlab))) continue;
        const int32_t j = kv[k]->slot[ne.first];
        if (j >= 0 && cnt[j] >= 0) ++cnt[j];
        if (keep) {
          if (!node_cnt.empty() && node_cnt.back().first == ne.first) ++node_cnt.back().second;
          else node_cnt.emplace_back(ne.first, 1);
        }
      }
    if (keep) {
      sel_words.assign(1, ns);
      sel_words.insert(sel_words.end(), sel[k], sel[k + 1]);
      q.ctr[k] = keep->counter(sel_words.data(), sel_words.size(), node_cnt);
    }
  }
  if (keep) keep->queries.push_back(std::move(q));
  std::vector<uint64_t> acc(static_cast<size_t>(Wp), 0);
  filter_row(cs, kv, count, dmask, Wp, acc.data());
  for (int32_t i = 0; i < Wp; ++i) row[i] |= acc[i];
  if (std::getenv("SR_SPREAD_CHECK")) {  // debug: the scan must agree
    std::vector<uint64_t> r2(static_cast<size_t>(Wp), 0);
    spread_row_scan(snap, w, aff_row, dmask, r2.data());
    for (int32_t i = 0; i < Wp; ++i)
      if (r2[i] != acc[i]) {
        std::fprintf(stderr, "spread_row: indexed row differs from the scan at word %d\n", i);
        std::abort();
      }
  }
}

bool spread_reuse_patch(SpreadReuse& R, const sr_snapshot* snap, const std::vector<int32_t>& nodes, uint64_t* A,
                        std::vector<int32_t>& tab, bool* tab_changed, std::vector<int32_t>& atoms,
                        std::vector<int32_t>& words) {
  const int32_t n_spot = R.n_spot, Wp = R.Wp;
  if (static_cast<int32_t>(snap->nodes.size()) != n_spot) return false;
  for (SpreadReuse::Counter& C : R.ctr) C.changed = false;
  bool any = false;
  std::unordered_map<int32_t, int32_t> now;  // counter -> pods on the node
  Constraint ck;
  for (int32_t n : nodes) {
    now.clear();
    for (int32_t e : snap->state[n].pods) {
      const SnapPod& sp = snap->pods[e];
      if (sp.term) continue;
      const int32_t *lk = snap->lkey.data() + sp.lab, *lv = snap->lval.data() + sp.lab;
      const int32_t nl = static_cast<int32_t>(sp.nlab);
      auto try_ctr = [&](int32_t c) {
        const std::vector<int32_t>& w = R.ctr[c].words;
        if (w[0] != sp.ns) return;
        parse_sel(w.data() + 1, &ck);
        if (selects(ck, lk, lv, nl)) ++now[c];
      };
      for (int32_t c : R.unindexed) try_ctr(c);
      for (int32_t i = 0; i < nl; ++i) {
        auto it = R.by_label.find(static_cast<uint64_t>(static_cast<uint32_t>(lk[i])) << 32 | static_cast<uint32_t>(lv[i]));
        if (it != R.by_label.end())
          for (int32_t c : it->second) try_ctr(c);
      }
    }
    std::vector<int32_t>& had = R.node_nz[n];
    for (int32_t c : had) {  // counters that had pods here
      auto it = now.find(c);
      const int32_t x = it == now.end() ? 0 : it->second;
      if (R.ctr[c].get(n) != x) {
        R.ctr[c].set(n, x);
        R.ctr[c].changed = any = true;
      }
    }
    for (const auto& cx : now)  // counters new here
      if (std::find(had.begin(), had.end(), cx.first) == had.end()) {
        R.ctr[cx.first].set(n, cx.second);
        R.ctr[cx.first].changed = any = true;
      }
    had.clear();
    for (const auto& cx : now) had.push_back(cx.first);
  }
  if (!any) return true;
  // rows: recounted per pair from the node counts
  std::vector<uint64_t> row(static_cast<size_t>(Wp));
  std::vector<Constraint> cs;
  std::vector<const KeyView*> kv;
  for (const SpreadReuse::Query& q : R.queries) {
    bool moved = false;
    for (int32_t c : q.ctr) moved = moved || (c >= 0 && R.ctr[c].changed);
    if (!moved) continue;
    const int32_t nk = q.words[1];
    cs.assign(static_cast<size_t>(nk), Constraint{});
    kv.assign(static_cast<size_t>(nk), nullptr);
    const int32_t* p = q.words.data() + 2;
    for (int32_t k = 0; k < nk; ++k) {
      p = parse(p, &cs[k]);
      kv[k] = &R.keys.find(cs[k].key)->second;
    }
    Counts count;
    std::fill(row.begin(), row.end(), 0ull);
    if (!pair_slots(cs, kv, q.aff.data(), Wp, count)) {
      all_nodes(n_spot, row.data());
    } else {
      for (int32_t k = 0; k < nk; ++k) {
        if (q.ctr[k] < 0) continue;
        std::vector<int64_t>& cnt = count[cs[k].key];
        for (const auto& e : R.ctr[q.ctr[k]].nz) {
          const int32_t j = kv[k]->slot[e.first];
          if (j >= 0 && cnt[j] >= 0) cnt[j] += e.second;
        }
      }
      filter_row(cs, kv, count, q.dmask, Wp, row.data());
    }
    uint64_t* a = A + static_cast<size_t>(q.atom) * Wp;
    bool differs = false;
    for (int32_t i = 0; i < Wp; ++i)
      if (a[i] != row[i]) {
        a[i] = row[i];
        words.push_back(i);
        differs = true;
      }
    if (differs) atoms.push_back(q.atom);
  }
  // domain-path tables (analyse_spread's formulas)
  std::vector<int32_t> dense;
  for (const SpreadReuse::Slot& s : R.slots) {
    if (!R.ctr[s.ctr].changed) continue;
    dense.assign(static_cast<size_t>(n_spot), 0);
    for (const auto& e : R.ctr[s.ctr].nz) dense[e.first] = e.second;
    const std::vector<int32_t>& cnt = dense;
    if (s.local) {
      int64_t m0 = INT64_MAX, n0 = 0;
      for (int32_t n = 0; n < n_spot; ++n) {
        if (!((s.pairs[n >> 6] >> (n & 63)) & 1)) continue;
        if (cnt[n] < m0) {
          m0 = cnt[n];
          n0 = 0;
        }
        n0 += cnt[n] == m0 ? 1 : 0;
      }
      if (n0 <= s.n_counted) return false;  // the minimum could move: the reference path's
      for (int32_t n = 0; n < n_spot; ++n) {
        const bool in = (s.pairs[n >> 6] >> (n & 63)) & 1;
        const int32_t v = in ? static_cast<int32_t>(std::max<int64_t>(
                                   INT32_MIN, std::min<int64_t>(INT32_MAX - 1, static_cast<int64_t>(s.skew) - s.self + m0 - cnt[n])))
                             : INT32_MAX;
        int32_t& t = tab[s.off + static_cast<uint32_t>(n)];
        if (t != v) {
          t = v;
          *tab_changed = true;
        }
      }
    } else {
      const std::vector<int32_t>& dom = R.doms[s.dom];
      int64_t bc[kDomMax] = {0};
      for (int32_t n = 0; n < n_spot; ++n) {
        const int32_t d = dom[n] >= 0 ? dom[n] : s.edom;
        if (d >= 0 && ((s.pm >> d) & 1)) bc[d] += cnt[n];
      }
      for (int32_t d = 0; d < kDomMax; ++d) {
        const int32_t v = static_cast<int32_t>(std::min<int64_t>(bc[d], INT32_MAX / 4));
        int32_t& t = tab[s.off + static_cast<uint32_t>(d)];
        if (t != v) {
          t = v;
          *tab_changed = true;
        }
      }
    }
  }
  return true;
}

void spread_row_scan(const sr_snapshot* snap, const int32_t* w, const uint64_t* aff_row, uint32_t dmask,
                     uint64_t* row) {
  const int32_t n_spot = static_cast<int32_t>(snap->nodes.size());
  const int32_t ns = w[0], nk = w[1];
  std::vector<Constraint> cs(static_cast<size_t>(nk));
  const int32_t* p = w + 2;
  for (int32_t k = 0; k < nk; ++k) p = parse(p, &cs[k]);
  // the nodes' values of the constraints' keys (INT32_MIN: absent)
  std::vector<int32_t> val(static_cast<size_t>(nk) * n_spot, INT32_MIN);
  for (int32_t n = 0; n < n_spot; ++n)
    for (const auto& kv : snap->nodes[n].labels)
      for (int32_t k = 0; k < nk; ++k)
        if (kv.first == cs[k].key) val[static_cast<size_t>(k) * n_spot + n] = kv.second;
  auto value = [&](int32_t k, int32_t n) { return val[static_cast<size_t>(k) * n_spot + n]; };
  // PreFilter: the pairs of the nodes passing NodeAffinity and carrying every key
  std::unordered_map<uint64_t, int64_t> count;
  for (int32_t n = 0; n < n_spot; ++n) {
    if (!(aff_row[n >> 6] >> (n & 63) & 1)) continue;
    bool all = true;
    for (int32_t k = 0; k < nk && all; ++k) all = value(k, n) != INT32_MIN;
    if (!all) continue;
    for (int32_t k = 0; k < nk; ++k) count.emplace(pair_key(cs[k].key, value(k, n)), 0);
  }
  if (count.empty()) {  // empty TpPairToMatchNum: Filter passes every node
    for (int32_t n = 0; n < n_spot; ++n) row[n >> 6] |= 1ull << (n & 63);
    return;
  }
  // processNode: every node, every constraint, the pair of the node's value ("" when absent)
  for (int32_t m = 0; m < n_spot; ++m)
    for (int32_t k = 0; k < nk; ++k) {
      const int32_t v = value(k, m) == INT32_MIN ? snap->id_empty : value(k, m);
      auto it = count.find(pair_key(cs[k].key, v));
      if (it == count.end()) continue;
      for (int32_t e : snap->state[m].pods) {
        const SnapPod& sp = snap->pods[e];
        if (sp.term || sp.ns != ns) continue;  // terminating (unknown: planned on the reference path)
        if (selects(cs[k], snap->lkey.data() + sp.lab, snap->lval.data() + sp.lab, static_cast<int32_t>(sp.nlab)))
          it->second++;
      }
    }
  std::unordered_map<int32_t, int64_t> min_of;  // per key: TpKeyToCriticalPaths[key][0].MatchNum
  for (const auto& kv : count) {
    const int32_t key = static_cast<int32_t>(kv.first >> 32);
    auto ins = min_of.emplace(key, kv.second);
    if (!ins.second) ins.first->second = std::min(ins.first->second, kv.second);
  }
  for (int32_t n = 0; n < n_spot; ++n) {
    bool ok = true;
    for (int32_t k = 0; k < nk && ok; ++k) {
      if (value(k, n) == INT32_MIN) {
        ok = false;  // the node lacks the key: UnschedulableAndUnresolvable
        break;
      }
      if ((dmask >> k) & 1) continue;  // planned on the device (domain path): the key check only
      auto it = count.find(pair_key(cs[k].key, value(k, n)));
      const int64_t match = it == count.end() ? 0 : it->second;
      ok = match + cs[k].self - min_of[cs[k].key] <= cs[k].max_skew;
    }
    if (ok) row[n >> 6] |= 1ull << (n & 63);
  }
}

}  // namespace sr
