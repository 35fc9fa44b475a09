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

const int32_t* parse(const int32_t* w, Constraint* c) {
  c->max_skew = *w++;
  c->key = *w++;
  c->self = *w++;
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

void spread_words(const sr_cluster* c, int32_t pod, std::vector<int32_t>& out) {
  const sr_spread* S = c->spread;
  out.clear();
  out.push_back(c->pod_affinity->ns[pod]);
  out.push_back(S->off[pod + 1] - S->off[pod]);
  std::vector<std::pair<int32_t, int32_t>> ml;
  for (int32_t k = S->off[pod]; k < S->off[pod + 1]; ++k) {
    out.push_back(S->max_skew[k]);
    out.push_back(S->topology_key[k]);
    out.push_back(spread_selects(c, k, pod) ? 1 : 0);
    out.push_back(S->selector_nil[k] ? 1 : 0);
    ml.clear();
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
}

void spread_row(SpreadIndex& ix, const int32_t* w, const uint64_t* aff_row, uint32_t dmask, uint64_t* row) {
  const sr_snapshot* snap = ix.snap;
  const int32_t n_spot = ix.n_spot, Wp = ix.Wp;  // the encoder's row width (KeyView strides)
  const int32_t ns = w[0], nk = w[1];
  std::vector<Constraint> cs(static_cast<size_t>(nk));
  const int32_t* p = w + 2;
  for (int32_t k = 0; k < nk; ++k) p = parse(p, &cs[k]);
  std::vector<const SpreadIndex::KeyView*> kv(static_cast<size_t>(nk));
  for (int32_t k = 0; k < nk; ++k) kv[k] = &ix.key(cs[k].key);
  // PreFilter: the nodes passing NodeAffinity and carrying every key define
  // the pairs; none at all -> Filter passes every node
  std::vector<uint64_t> elig(aff_row, aff_row + Wp);
  for (int32_t k = 0; k < nk; ++k)
    for (int32_t i = 0; i < Wp; ++i) elig[i] &= kv[k]->has[i];
  bool any = false;
  for (int32_t i = 0; i < Wp && !any; ++i) any = elig[i] != 0;
  if (!any) {
    for (int32_t n = 0; n < n_spot; ++n) row[n >> 6] |= 1ull << (n & 63);
    return;
  }
  // per constraint, per value of its key: the pair exists, its count (two
  // constraints on one key add into the same pairs: counted by key below)
  std::unordered_map<int32_t, std::vector<int64_t>> count;  // key -> per value (-1: no such pair)
  for (int32_t k = 0; k < nk; ++k) {
    auto ins = count.emplace(cs[k].key, std::vector<int64_t>());
    if (!ins.second) continue;
    const SpreadIndex::KeyView& v = *kv[k];
    ins.first->second.assign(v.values.size(), -1);
    for (size_t j = 0; j < v.values.size(); ++j)
      for (int32_t i = 0; i < Wp; ++i)
        if (v.bits[j * Wp + i] & elig[i]) {
          ins.first->second[j] = 0;
          break;
        }
  }
  // processNode: every selected pod, every constraint, the pair of its node's
  // value ("" when the node lacks the key)
  auto value_slot = [&](const SpreadIndex::KeyView& v, int32_t n) -> int32_t {
    const int32_t x = v.val[n] == INT32_MIN ? snap->id_empty : v.val[n];
    for (size_t j = 0; j < v.values.size(); ++j)
      if (v.values[j] == x) return static_cast<int32_t>(j);
    return -1;
  };
  std::vector<std::pair<int32_t, int32_t>> all;
  for (int32_t k = 0; k < nk; ++k) {
    const Constraint& ck = cs[k];
    if (ck.nil) continue;
    const std::vector<std::pair<int32_t, int32_t>>* list;
    if (ck.n_ml > 0) {
      list = ix.pods_with(ck.ml[0], ck.ml[1]);
      if (!list) continue;
    } else {
      if (all.empty())
        for (int32_t n = 0; n < n_spot; ++n)
          for (int32_t e : snap->state[n].pods) all.emplace_back(n, e);
      list = &all;
    }
    std::vector<int64_t>& cnt = count[ck.key];
    for (const auto& ne : *list) {
      const SnapPod& sp = snap->pods[ne.second];
      if (sp.term || sp.ns != ns) continue;  // terminating (unknown: planned on the reference path)
      if (!selects(ck, snap->lkey.data() + sp.lab, snap->lval.data() + sp.lab, static_cast<int32_t>(sp.nlab))) continue;
      const int32_t j = value_slot(*kv[k], ne.first);
      if (j >= 0 && cnt[j] >= 0) ++cnt[j];
    }
  }
  // Filter per node: row = AND over the constraints of the nodes carrying a
  // value whose pair count (0 without a pair) + self - the key's minimum is
  // within maxSkew (a device-planned constraint: the key check only)
  std::vector<uint64_t> acc(static_cast<size_t>(Wp), ~0ull), part(static_cast<size_t>(Wp));
  for (int32_t k = 0; k < nk; ++k) {
    const SpreadIndex::KeyView& v = *kv[k];
    if ((dmask >> k) & 1) {
      for (int32_t i = 0; i < Wp; ++i) acc[i] &= v.has[i];
      continue;
    }
    const std::vector<int64_t>& cnt = count[cs[k].key];
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
