// Host-only check of the tick-to-tick paths of NewNodeMap and
// GetClusterSnapshot (nodes/nodes.go:63-104, 226-232): on a synthetic config,
// tick after tick of cluster mutations (pods whose requests change, pods that
// move, leave or lose their stamp, priorities, node allocatable / labels /
// names),
// sr_new_node_map_cached must equal sr_new_node_map and a snapshot kept
// current by sr_snapshot_refresh must equal one built by sr_snapshot_create,
// field by field (nodes, states, the pods' copies, fingerprints, totals).
//   make -C k8s-spot-rescheduler_amd tools && k8s-spot-rescheduler_amd/bin/refresh_check <config> [ticks] [mutations per tick] [threshold]
// Prints the medians of both paths for one-pod ticks afterwards (timing only).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../k8s-spot-rescheduler_amd/csrc/host.hpp"
#include "../k8s-spot-rescheduler_amd/csrc/synth/sr_synth.h"

#ifdef SR_NM_PROFILE
namespace sr { extern double nm_phase_ms[10]; }
#endif

namespace {

double ms_since(std::chrono::steady_clock::time_point a) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}

template <class T>
T* mut(const T* p) {
  return const_cast<T*>(p);
}

struct NodeMapOut {
  std::vector<int32_t> spot, od, off, idx;
  std::vector<int64_t> req, fr;
  int32_t ns = 0, nod = 0;
  sr_node_map view(int nn, int np) {
    spot.assign(nn, 0);
    od.assign(nn, 0);
    off.assign(nn + 1, 0);
    idx.assign(np > 0 ? np : 1, 0);
    req.assign(nn, 0);
    fr.assign(nn, 0);
    return sr_node_map{spot.data(), &ns, od.data(), &nod, off.data(), idx.data(), req.data(), fr.data()};
  }
  bool operator==(const NodeMapOut& o) const {
    return ns == o.ns && nod == o.nod && std::equal(spot.begin(), spot.begin() + ns, o.spot.begin()) &&
           std::equal(od.begin(), od.begin() + nod, o.od.begin()) && off == o.off &&
           std::equal(idx.begin(), idx.begin() + off.back(), o.idx.begin()) && req == o.req && fr == o.fr;
  }
};

bool same_ports(const sr::NodeState& a, const sr::NodeState& b) {
  if (a.ports.size() != b.ports.size()) return false;
  for (size_t k = 0; k < a.ports.size(); ++k)
    if (a.ports[k].ip != b.ports[k].ip || a.ports[k].proto != b.ports[k].proto || a.ports[k].port != b.ports[k].port)
      return false;
  return true;
}

// What the planner can read of a snapshot: "" if `a` and `b` hold the same.
const char* snapshot_diff(const sr_snapshot* a, const sr_snapshot* b, size_t* at) {
  *at = 0;
  if (a->nodes.size() != b->nodes.size()) return "node count";
  if (a->node_names != b->node_names || a->node_sfp != b->node_sfp || a->node_dfp != b->node_dfp) return "views";
  if (a->anti_total != b->anti_total || a->opaque_total != b->opaque_total || a->unknown_total != b->unknown_total ||
      a->scalar_unknown_total != b->scalar_unknown_total || a->term_unknown_total != b->term_unknown_total)
    return "totals";
  if (a->id_empty != b->id_empty || a->id_metadata_name != b->id_metadata_name || a->forked != b->forked)
    return "ids";
  for (size_t i = 0; i < a->nodes.size(); ++i) {
    *at = i;
    const sr::SpotNode &x = a->nodes[i], &y = b->nodes[i];
    if (x.name != y.name || x.static_fp != y.static_fp || x.alloc_pods != y.alloc_pods ||
        x.unschedulable != y.unschedulable || std::memcmp(x.alloc, y.alloc, sizeof(x.alloc)) ||
        x.labels != y.labels || x.scalar_alloc != y.scalar_alloc || x.vol_limit != y.vol_limit ||
        x.taints.size() != y.taints.size())
      return "spot node";
    const sr::NodeState &s = a->state[i], &t = b->state[i];
    if (std::memcmp(s.requested, t.requested, sizeof(s.requested)) || s.npods != t.npods || s.anti != t.anti ||
        s.opaque != t.opaque || s.unknown != t.unknown || s.scalar_unknown != t.scalar_unknown ||
        s.term_unknown != t.term_unknown || !same_ports(s, t) || s.scalar_req != t.scalar_req || s.att != t.att ||
        s.pods.size() != t.pods.size())
      return "node state";
    for (size_t k = 0; k < s.pods.size(); ++k) {
      const sr::SnapPod &p = a->pods[s.pods[k]], &q = b->pods[t.pods[k]];
      if (p.ns != q.ns || p.meta != q.meta || p.anti != q.anti || p.opaque != q.opaque || p.term != q.term ||
          a->stamps[s.pods[k]] != b->stamps[t.pods[k]] || p.nlab != q.nlab || p.nterms != q.nterms)
        return "pod copy";
      if (!std::equal(a->lkey.begin() + p.lab, a->lkey.begin() + p.lab + p.nlab, b->lkey.begin() + q.lab) ||
          !std::equal(a->lval.begin() + p.lab, a->lval.begin() + p.lab + p.nlab, b->lval.begin() + q.lab))
        return "pod labels";
      if (p.nterms && !std::equal(a->term_words.begin() + p.terms, a->term_words.begin() + p.terms + p.nterms,
                                  b->term_words.begin() + q.terms))
        return "pod terms";
    }
  }
  return "";
}

struct Rng {
  uint64_t x = 0x2545F4914F6CDD1Dull;
  uint64_t next() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

}  // namespace

int main(int argc, char** argv) {
  sr_synth_params sp{};
  sp.config = argc > 1 ? atoi(argv[1]) : 3;
  sp.pinned_fraction = -1;
  const int ticks = argc > 2 ? atoi(argv[2]) : 100;
  const int per_tick = argc > 3 ? atoi(argv[3]) : 4;
  const int threshold = argc > 4 ? atoi(argv[4]) : 0;
  sr_synth* syn = sr_synth_generate(&sp);
  sr_cluster c;
  sr_synth_view(syn, &c);
  sr_node_label od, spl;
  sr_synth_labels(syn, &od, &spl);
  const int nn = c.nodes.n, np = c.pods.n;
  if (!c.pod_stamp) {
    printf("config %d has no pod stamps\n", sp.config);
    return 1;
  }
  sr_node_map_params prm{od, spl, threshold};
  sr_node_map_cache* cache = nullptr;
  sr_node_map_cache_create(&cache);
  Rng rng;
  uint64_t stamp_seq = 0x5EED0000ull;
  auto new_stamp = [&](int32_t pod) { mut(c.pod_stamp)[pod] = (++stamp_seq * 0x9E3779B97F4A7C15ull) | 1; };
  std::vector<std::pair<int32_t, uint64_t>> zeroed;  // pods whose stamp is 0 for a while
  int kinds[8] = {0};
  auto mutate = [&](int kind) {
    const int32_t pod = static_cast<int32_t>(rng.below(static_cast<uint64_t>(np)));
    kinds[kind]++;
    switch (kind) {
      case 0: {  // requests change (cpu: the node's RequestedCPU and its place in the spot order)
        const int64_t d = static_cast<int64_t>(rng.below(200)) - 100;
        mut(c.pods.cpu_sort_milli)[pod] = std::max<int64_t>(0, c.pods.cpu_sort_milli[pod] + d);
        mut(c.pods.req_milli_cpu)[pod] = std::max<int64_t>(0, c.pods.req_milli_cpu[pod] + d);
        if (c.acc_milli_cpu) mut(c.acc_milli_cpu)[pod] = std::max<int64_t>(0, c.acc_milli_cpu[pod] + d);
        mut(c.pods.req_memory)[pod] += static_cast<int64_t>(rng.below(1 << 20));
        if (c.acc_memory) mut(c.acc_memory)[pod] = c.pods.req_memory[pod];
        new_stamp(pod);
        break;
      }
      case 1:  // the pod moves to another node
        mut(c.pods.node)[pod] = static_cast<int32_t>(rng.below(static_cast<uint64_t>(nn)));
        new_stamp(pod);
        break;
      case 2:  // the pod leaves (unbound)
        mut(c.pods.node)[pod] = -1;
        new_stamp(pod);
        break;
      case 3:  // stamp unknown for a few ticks
        zeroed.emplace_back(pod, c.pod_stamp[pod]);
        mut(c.pod_stamp)[pod] = 0;
        break;
      case 4:  // priority (the spot-node filter with a threshold)
        mut(c.pods.priority)[pod] = static_cast<int32_t>(rng.below(3)) - 1;
        new_stamp(pod);
        break;
      case 5: {  // node allocatable / unschedulable (static part)
        const int32_t node = static_cast<int32_t>(rng.below(static_cast<uint64_t>(nn)));
        mut(c.nodes.alloc_milli_cpu)[node] += 1000;
        mut(c.nodes.unschedulable)[node] ^= static_cast<uint8_t>(rng.below(8) == 0);
        break;
      }
      case 6: {  // a node loses / regains its spot label (joins the spot set or leaves it)
        const int32_t node = static_cast<int32_t>(rng.below(static_cast<uint64_t>(nn)));
        for (int32_t j = c.nodes.label_off[node]; j < c.nodes.label_off[node + 1]; ++j) {
          if (c.nodes.label_key[j] == spl.key) mut(c.nodes.label_key)[j] = c.id_metadata_name;
          else if (c.nodes.label_key[j] == c.id_metadata_name) mut(c.nodes.label_key)[j] = spl.key;
        }
        break;
      }
      case 7: {  // two nodes swap names (a node replaced by another of the same name)
        const int32_t a = static_cast<int32_t>(rng.below(static_cast<uint64_t>(nn)));
        const int32_t b = static_cast<int32_t>(rng.below(static_cast<uint64_t>(nn)));
        std::swap(mut(c.nodes.name)[a], mut(c.nodes.name)[b]);
        break;
      }
      default:
        break;
    }
  };
  NodeMapOut ref, got;
  sr_snapshot* kept = nullptr;
  int bad = 0, states_err = 0;
  long rebuilt_sum = 0, sorted_sum = 0;
  for (int t = 0; t < ticks; ++t) {
    if (t > 0) {
      for (int m = 0; m < per_tick; ++m) mutate(static_cast<int>(rng.below(8)));
      if (t % 5 == 0)
        for (auto z = zeroed.rbegin(); z != zeroed.rend(); ++z)  // known again: the last stamp it had
          if (!c.pod_stamp[z->first]) mut(c.pod_stamp)[z->first] = z->second;
      if (t % 5 == 0) zeroed.clear();
    }
    sr_node_map m1 = ref.view(nn, np), m2 = got.view(nn, np);
    const sr_status s1 = sr_new_node_map(&c, &prm, &m1);
    int32_t sorted = 0;
    const sr_status s2 = sr_new_node_map_cached(cache, &c, &prm, &m2, &sorted);
    if (s1 != s2) {
      printf("tick %d: node map status %d vs %d\n", t, s1, s2);
      return 2;
    }
    if (s1 != SR_OK) {  // a nil priority: both refuse (not produced by these mutations)
      printf("tick %d: node map status %d\n", t, s1);
      return 2;
    }
    sorted_sum += sorted;
    if (!(ref == got) && bad++ < 5) printf("tick %d: cached node map differs\n", t);
    sr_snapshot* fresh = nullptr;
    sr_snapshot_create(&c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), &fresh);
    if (!kept) {
      sr_snapshot_create(&c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), &kept);
    } else {
      if (t % 13 == 5) {  // forked: refused, the snapshot untouched
        sr_snapshot_fork(kept);
        if (sr_snapshot_refresh(kept, &c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), nullptr) !=
            SR_ERR_STATE)
          ++states_err;
        sr_snapshot_revert(kept);
      }
      if (t % 11 == 3 && kept->nodes.size())  // a pod added to the kept snapshot: gone after the refresh
        sr_snapshot_add_pod(kept, &c, static_cast<int32_t>(rng.below(np)),
                            static_cast<int32_t>(rng.below(kept->nodes.size())));
      int32_t rebuilt = 0;
      // mostly linked to the node map cache (sr_snapshot_refresh_cached), now and then the plain refresh
      const sr_status rs = t % 7 == 2 ? sr_snapshot_refresh(kept, &c, ref.spot.data(), ref.ns, ref.off.data(),
                                                             ref.idx.data(), &rebuilt)
                                      : sr_snapshot_refresh_cached(kept, cache, &c, ref.spot.data(), ref.ns,
                                                                    ref.off.data(), ref.idx.data(), &rebuilt);
      if (rs != SR_OK) {
        printf("tick %d: refresh failed\n", t);
        return 2;
      }
      rebuilt_sum += rebuilt;
    }
    size_t at = 0;
    const char* d = snapshot_diff(kept, fresh, &at);
    if (*d && bad++ < 5) printf("tick %d: refreshed snapshot differs (%s at position %zu)\n", t, d, at);
    sr_snapshot_destroy(fresh);
  }
  // an invalid input leaves the snapshot as it was
  {
    const int32_t bad_spot = nn;
    const uint64_t v = kept->version;
    if (sr_snapshot_refresh(kept, &c, &bad_spot, 1, ref.off.data(), ref.idx.data(), nullptr) != SR_ERR_INVALID_ARG ||
        kept->version != v)
      ++states_err;
  }
  printf("refresh check: config %d, %d ticks x %d mutations (kinds %d %d %d %d %d %d %d %d), nodes rebuilt per tick %.1f "
         "of %d, nodes sorted per tick %.1f of %d, mismatches %d, state errors %d\n",
         sp.config, ticks, per_tick, kinds[0], kinds[1], kinds[2], kinds[3], kinds[4], kinds[5], kinds[6], kinds[7],
         ticks > 1 ? static_cast<double>(rebuilt_sum) / (ticks - 1) : 0.0, ref.ns,
         static_cast<double>(sorted_sum) / ticks, nn, bad, states_err);

  // timing: ticks with one pod's requests changed
  std::vector<double> t_map, t_map_c, t_create, t_refresh, t_refresh_c;
  std::vector<double> ph[9], t_pfd;
  sr_pod_drain drain;
  sr_synth_drain(syn, &drain);
  const sr_drain_params dprm{0, 0, 1};
  for (int r = 0; r < 30; ++r) {
    mutate(0);
    sr_node_map m1 = ref.view(nn, np), m2 = got.view(nn, np);
    auto t0 = std::chrono::steady_clock::now();
    sr_new_node_map(&c, &prm, &m1);
    t_map.push_back(ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    sr_new_node_map_cached(cache, &c, &prm, &m2, nullptr);
    t_map_c.push_back(ms_since(t0));
#ifdef SR_NM_PROFILE
    for (int k = 0; k < 5; ++k) ph[k].push_back(sr::nm_phase_ms[k]);
#endif
    sr_snapshot* fresh = nullptr;
    t0 = std::chrono::steady_clock::now();
    sr_snapshot_create(&c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), &fresh);
    t_create.push_back(ms_since(t0));
    t0 = std::chrono::steady_clock::now();
    if (r < 15) {
      sr_snapshot_refresh(kept, &c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), nullptr);
      t_refresh.push_back(ms_since(t0));
    } else {  // linked to this tick's cached node map (the previous refresh was linked too, but the first)
      sr_snapshot_refresh_cached(kept, cache, &c, ref.spot.data(), ref.ns, ref.off.data(), ref.idx.data(), nullptr);
      t_refresh_c.push_back(ms_since(t0));
#ifdef SR_NM_PROFILE
      for (int k = 5; k < 9; ++k) ph[k].push_back(sr::nm_phase_ms[k]);
#endif
    }
    {  // the candidate lists of the tick (podsForDeletion over the on-demand nodes)
      std::vector<int32_t> coff(ref.nod + 1), cpods(std::max(1, ref.off.back())), bp(std::max(1, ref.nod)),
          br(std::max(1, ref.nod));
      t0 = std::chrono::steady_clock::now();
      sr_pods_for_deletion(&c, &drain, &dprm, ref.od.data(), ref.nod, ref.off.data(), ref.idx.data(), coff.data(),
                           cpods.data(), bp.data(), br.data());
      t_pfd.push_back(ms_since(t0));
    }
    sr_snapshot_destroy(fresh);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("one-pod ticks (median ms): new_node_map %.3f cached %.3f | snapshot_create %.3f refresh %.3f cached %.3f | "
         "pods_for_deletion %.3f\n", med(t_map), med(t_map_c), med(t_create), med(t_refresh), med(t_refresh_c),
         med(t_pfd));
#ifdef SR_NM_PROFILE
  printf("cached node map phases (median ms): LIST grouping %.3f kinds+slots %.3f pass1 %.3f pass2 %.3f lists %.3f\n",
         med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]));
  printf("cached refresh phases (median ms): by name %.3f pass1 %.3f pass2 %.3f rebuild+totals %.3f\n", med(ph[5]),
         med(ph[6]), med(ph[7]), med(ph[8]));
#endif
  sr_snapshot_destroy(kept);
  sr_node_map_cache_destroy(cache);
  sr_synth_destroy(syn);
  return bad || states_err ? 2 : 0;
}
