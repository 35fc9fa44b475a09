// Host-only harness: NewNodeMap + snapshot + encode_workload on a synthetic
// config, printing the workload's dimensions and host-side timings (no GPU).
//   make -C k8s-spot-rescheduler_amd tools && k8s-spot-rescheduler_amd/bin/encode_stats 3 [max candidates] [check | reuse [ticks [burst]]]
//   (reuse-perm: pods on spot nodes change requests between ticks, the spot order moves;
//    reuse-scalar: every spot node allocating an extended resource is filled past its allocatable
//    for two ticks in six and freed again, so scalar query rows go empty <-> non-empty while reused)
// Encodes are timed cold (empty encoder cache), warm (the same snapshot
// again) and after one spot node changed (a fresh snapshot with one more pod
// on one node), the steady state of a planner between two ticks.
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "../k8s-spot-rescheduler_amd/csrc/host.hpp"
#include "../k8s-spot-rescheduler_amd/csrc/synth/sr_synth.h"

namespace sr { extern double encode_phase_ms[16]; }

static double ms_since(std::chrono::steady_clock::time_point a) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}

static void phases(const char* tag) {
  const double* p = sr::encode_phase_ms;
  printf("  %-6s phases(ms): views %.3f pass1 %.3f ports %.3f gather %.3f shards %.3f specs-new %.3f keys %.3f "
         "classes %.3f atoms %.3f lb+empty %.3f pods %.3f trows %.3f recs %.3f lists %.3f reuse %.3f\n",
         tag, p[0], p[5], p[1], p[9], p[14], p[7], p[2], p[3], p[4], p[8], p[10], p[12], p[13], p[6], p[11]);
}

int main(int argc, char** argv) {
  sr_synth_params p{};
  p.config = argc > 1 ? atoi(argv[1]) : 3;
  p.pinned_fraction = -1;
  const bool realistic = std::getenv("SR_SYNTH_REALISTIC") != nullptr;
  if (realistic) {  // bench --variant realistic (spotplanner/synth.py REALISTIC)
    p.stateful_fraction = 0.15;
    p.init_fraction = 0.2;
    p.gpu_fraction = 0.3;
  }
  const bool affinity = std::getenv("SR_SYNTH_AFFINITY") != nullptr;
  if (affinity) {  // bench --variant affinity (spotplanner/synth.py AFFINITY)
    p.anti_fraction = 0.10;
    p.spread_fraction = 0.10;
  }
  sr_synth* s = sr_synth_generate(&p);
  sr_cluster c;
  sr_synth_view(s, &c);
  sr_node_label od, sp;
  sr_synth_labels(s, &od, &sp);
  const int nn = c.nodes.n, np = c.pods.n;
  std::vector<int32_t> spot(nn), odn(nn), off(nn + 1), idx(np);
  std::vector<int64_t> req(nn), fr(nn);
  int32_t ns = 0, nod = 0;
  sr_node_map m{spot.data(), &ns, odn.data(), &nod, off.data(), idx.data(), req.data(), fr.data()};
  sr_node_map_params prm{od, sp, 0};
  auto t0 = std::chrono::steady_clock::now();
  if (sr_new_node_map(&c, &prm, &m) != SR_OK) return 1;
  const double ms_map = ms_since(t0);
  sr_snapshot* snap = nullptr;
  t0 = std::chrono::steady_clock::now();
  sr_snapshot_create(&c, spot.data(), ns, off.data(), idx.data(), &snap);
  const double ms_snap = ms_since(t0);
  std::vector<int32_t> coff{0}, cp;
  const int max_cands = argc > 2 ? atoi(argv[2]) : nod;
  if (max_cands < nod) nod = max_cands;
  for (int i = 0; i < nod; ++i) {
    int node = odn[i];
    for (int j = off[node]; j < off[node + 1]; ++j)
      if (!(c.pods.flags[idx[j]] & (SR_POD_MIRROR | SR_POD_DAEMONSET_CONTROLLER))) cp.push_back(idx[j]);
    coff.push_back(cp.size());
  }
  sr_candidates cands{nod, coff.data(), cp.data(), nullptr};
  sr::Workload w;
  sr::EncoderCache cache;
  std::string err;
  printf("config %d: nodes %d pods %d spot %d od %d cand_pods %zu\n", p.config, nn, np, ns, nod, cp.size());
  printf("new_node_map %.2f ms, snapshot %.2f ms\n", ms_map, ms_snap);
  t0 = std::chrono::steady_clock::now();
  if (sr::encode_workload(&cache, snap, &c, &cands, &w, &err) != SR_OK) {
    printf("encode failed: %s\n", err.c_str());
    return 1;
  }
  printf("cold encode %.3f ms (new specs %d, memo hits %d)\n", ms_since(t0), cache.last_new_specs, cache.last_memo_hits);
  phases("cold");
  double best = 1e30;
  for (int r = 0; r < 20; ++r) {
    t0 = std::chrono::steady_clock::now();
    sr::encode_workload(&cache, snap, &c, &cands, &w, &err);
    best = std::min(best, ms_since(t0));
  }
  printf("warm encode (same snapshot) best %.3f ms\n", best);
  phases("warm");
  // one spot node changed: a fresh snapshot (as every tick builds) with one
  // more pod on spot position 7
  best = 1e30;
  int last_state = 0, last_static = 0;
  for (int r = 0; r < 10; ++r) {
    sr_snapshot* s2 = nullptr;
    sr_snapshot_create(&c, spot.data(), ns, off.data(), idx.data(), &s2);
    if (r & 1) sr_snapshot_add_pod(s2, &c, cp.empty() ? 0 : cp[0], std::min(7, ns - 1));
    t0 = std::chrono::steady_clock::now();
    sr::encode_workload(&cache, s2, &c, &cands, &w, &err);
    best = std::min(best, ms_since(t0));
    last_state = cache.last_state_changed;
    last_static = cache.last_static_changed;
    sr_snapshot_destroy(s2);
  }
  printf("one-node-changed encode (fresh snapshot) best %.3f ms (state nodes %d, static rebuilt %d, memo hits %d, "
         "reused %d, pod patches %d)\n", best, last_state, last_static, cache.last_memo_hits, cache.last_reused,
         cache.last_pod_patches);
  phases("1node");
  const bool check_perm = argc > 3 && std::string(argv[3]) == "check-perm";
  if (argc > 3 && (std::string(argv[3]) == "check" || check_perm)) {
    // the state view patched node by node equals the one rebuilt from scratch:
    // consecutive fresh snapshots, each with a few more pods on random spot nodes
    std::vector<std::pair<int32_t, int32_t>> extra;
    uint64_t x = 88172645463325252ull;
    auto rnd = [&](uint64_t n) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x % n; };
    int ticks = 0, patched = 0;
    int moved_ticks = 0;
    for (int r = 0; r < 300 && !cp.empty(); ++r) {
      if (check_perm && r > 0) {  // pods on spot nodes change cpu requests: the spot order moves
        for (int k = 0, nk = 1 + static_cast<int>(rnd(3)); k < nk; ++k) {
          const int32_t node = spot[rnd(static_cast<uint64_t>(ns))];
          if (off[node + 1] == off[node]) continue;
          const int32_t pod = idx[off[node] + static_cast<int32_t>(rnd(static_cast<uint64_t>(off[node + 1] - off[node])))];
          const int64_t d = static_cast<int64_t>(rnd(400)) - 150;
          auto bump = [&](const int64_t* a) { const_cast<int64_t*>(a)[pod] = std::max<int64_t>(0, a[pod] + d); };
          bump(c.pods.cpu_sort_milli);
          bump(c.pods.req_milli_cpu);
          if (c.acc_milli_cpu) bump(c.acc_milli_cpu);
          const_cast<uint64_t*>(c.pod_stamp)[pod] = (x | 1);
        }
        std::vector<int32_t> before(spot.begin(), spot.begin() + ns);
        if (sr_new_node_map(&c, &prm, &m) != SR_OK) return 1;
        moved_ticks += !std::equal(before.begin(), before.end(), spot.begin());
      }
      sr_snapshot* s2 = nullptr;
      sr_snapshot_create(&c, spot.data(), ns, off.data(), idx.data(), &s2);
      if (r % 7 == 6) extra.clear();  // sometimes the extra pods leave again
      const int add = 1 + static_cast<int>(rnd(3));
      for (int a = 0; a < add; ++a)
        extra.emplace_back(cp[rnd(cp.size())], static_cast<int32_t>(rnd(static_cast<uint64_t>(ns))));
      for (auto& e : extra) sr_snapshot_add_pod(s2, &c, e.first, e.second);
      sr::encode_workload(&cache, s2, &c, &cands, &w, &err);
      patched += cache.patched_from != ~0ull;
      sr::EncoderCache fresh;
      sr::Workload w2;
      sr::encode_workload(&fresh, s2, &c, &cands, &w2, &err);
      for (int d = 0; d < 3; ++d)
        if (cache.sorted_free[d] != fresh.sorted_free[d] || cache.node_vals[d] != fresh.node_vals[d]) {
          printf("views differ at tick %d, dimension %d\n", r, d);
          return 2;
        }
      if (cache.node_rec != fresh.node_rec || cache.node_free != fresh.node_free ||
          cache.podcount_row != fresh.podcount_row) {
        printf("node records differ at tick %d\n", r);
        return 2;
      }
      sr_snapshot_destroy(s2);
      ++ticks;
    }
    printf("state views consistent: %d ticks (%d patched node by node, spot order moved %d)\n", ticks, patched,
           moved_ticks);
  }
  const bool perm = argc > 3 && std::string(argv[3]) == "reuse-perm";
  const bool scal = argc > 3 && std::string(argv[3]) == "reuse-scalar";
  if (argc > 3 && (std::string(argv[3]) == "reuse" || perm || scal)) {
    // candidate-side reuse: every tick a fresh snapshot with a few more (or
    // fewer) pods on random spot nodes and the same candidate input; the
    // reused workload must plan like one encoded from scratch: same atoms,
    // programs and requests, per pod the same dead flag, class and threshold
    // per dimension
    std::vector<std::pair<int32_t, int32_t>> extra;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&](uint64_t n) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x % n; };
    const int ticks = argc > 4 ? atoi(argv[4]) : 200;
    const int burst = argc > 5 ? atoi(argv[5]) : 24;  // pods added every fifth tick (many new free values)
    int reused = 0, full = 0, bad = 0;
    long patches = 0;
    double ms_reuse = 0, ms_views = 0;
    int permuted = 0, flips = 0;
    // reuse-scalar: a candidate pod listing one extended resource (no volume
    // limit key) and, per spot node allocating that name, enough copies of it
    // to exceed the allocatable
    std::vector<std::pair<int32_t, int32_t>> fill;
    if (scal && c.pod_scalar_off && c.node_scalar_off) {
      int32_t gp = -1, name = 0;
      int64_t rq = 0;
      for (int32_t q : cp) {
        const int32_t b = c.pod_scalar_off[q], e = c.pod_scalar_off[q + 1];
        bool ok = e > b;
        for (int32_t i = b; i < e && ok; ++i) ok = c.pod_scalar_name[i] >= 0 && c.pod_scalar_acc[i] > 0;
        if (c.volumes) ok = ok && c.volumes->att_off[q] == c.volumes->att_off[q + 1];
        if (ok) { gp = q; name = c.pod_scalar_name[b]; rq = c.pod_scalar_acc[b]; break; }
      }
      for (int32_t k = 0; gp >= 0 && k < ns; ++k)
        for (int32_t i = c.node_scalar_off[spot[k]]; i < c.node_scalar_off[spot[k] + 1]; ++i)
          if (c.node_scalar_name[i] == name)
            for (int64_t u = 0; u <= c.node_scalar_alloc[i] / rq; ++u) fill.emplace_back(gp, k);
      printf("reuse-scalar: pod %d fills %zu slots\n", gp, fill.size());
      if (fill.empty()) return 3;
    }
    // the pods added at random: in reuse-scalar mode only pods without
    // attachable volumes (a candidate's attachable volume on a spot node sends
    // it to the reference path, and such a fallback ends the reuse)
    std::vector<int32_t> pool;
    for (int32_t q : cp) {
      bool ok = true;
      if (scal && c.pod_scalar_off)
        for (int32_t i = c.pod_scalar_off[q]; i < c.pod_scalar_off[q + 1] && ok; ++i) ok = c.pod_scalar_name[i] >= 0;
      if (scal && c.volumes) ok = ok && c.volumes->att_off[q] == c.volumes->att_off[q + 1];
      if (ok) pool.push_back(q);
    }
    for (int r = 0; r < ticks && !pool.empty(); ++r) {
      if (perm && r > 0) {
        // reuse-perm: pods on spot nodes change their cpu request (and stamp):
        // NewNodeMap re-sorts the spot list, the snapshot follows its order
        for (int k = 0, nk = 1 + static_cast<int>(rnd(3)); k < nk; ++k) {
          const int32_t node = spot[rnd(static_cast<uint64_t>(ns))];
          if (off[node + 1] == off[node]) continue;
          const int32_t pod = idx[off[node] + static_cast<int32_t>(rnd(static_cast<uint64_t>(off[node + 1] - off[node])))];
          const int64_t d = static_cast<int64_t>(rnd(400)) - 150;
          auto bump = [&](const int64_t* a) { const_cast<int64_t*>(a)[pod] = std::max<int64_t>(0, a[pod] + d); };
          bump(c.pods.cpu_sort_milli);
          bump(c.pods.req_milli_cpu);
          if (c.acc_milli_cpu) bump(c.acc_milli_cpu);
          const_cast<uint64_t*>(c.pod_stamp)[pod] = (x | 1);
        }
        std::vector<int32_t> before(spot.begin(), spot.begin() + ns);
        if (sr_new_node_map(&c, &prm, &m) != SR_OK) return 1;
        permuted += !std::equal(before.begin(), before.end(), spot.begin());
      }
      sr_snapshot* s2 = nullptr;
      sr_snapshot_create(&c, spot.data(), ns, off.data(), idx.data(), &s2);
      if (r % 9 == 8) extra.clear();
      const int add = r % 5 == 4 ? burst : 1 + static_cast<int>(rnd(3));  // sometimes a burst: many new free values
      for (int a = 0; a < add; ++a)
        extra.emplace_back(pool[rnd(pool.size())], static_cast<int32_t>(rnd(static_cast<uint64_t>(ns))));
      for (auto& e : extra) sr_snapshot_add_pod(s2, &c, e.first, e.second);
      if (scal && r % 6 >= 2 && r % 6 < 4)
        for (auto& e : fill) sr_snapshot_add_pod(s2, &c, e.first, e.second);
      // the realistic variant compares with a full encode by a copy of the
      // encoder as it was before this call: its class and atom numbering
      // depends on the dictionaries' history (scalar and volume queries)
      std::unique_ptr<sr::EncoderCache> twin;
      if (realistic || affinity) twin.reset(new sr::EncoderCache(cache));
      t0 = std::chrono::steady_clock::now();
      if (sr::encode_workload(&cache, s2, &c, &cands, &w, &err) != SR_OK) return 1;
      const double ms = ms_since(t0);
      if (cache.last_reused) {
        ++reused;
        flips += w.class_flip;
        patches += cache.last_pod_patches;
        ms_reuse += ms;
        ms_views += sr::encode_phase_ms[0];
      } else {
        ++full;
      }
      sr::EncoderCache fresh;
      sr::Workload f;
      if (sr::encode_workload(twin ? twin.get() : &fresh, s2, &c, &cands, &f, &err) != SR_OK) return 1;
      auto fail = [&](const char* what, long i) {
        if (bad++ < 5) printf("tick %d (reused %d): %s differs at %ld\n", r, cache.last_reused, what, i);
      };
      if (w.atoms != f.atoms) {
        long a = 0;
        while (a < f.n_atoms && std::equal(f.atoms.begin() + a * f.Wp, f.atoms.begin() + (a + 1) * f.Wp, w.atoms.begin() + a * f.Wp)) ++a;
        fail("atoms", a);
      }
      if (w.sp_tab != f.sp_tab) fail("spread tables", 0);
      if (w.dyn_cand != f.dyn_cand || w.dyn_pod != f.dyn_pod || w.dk_dom != f.dk_dom) fail("domain path", 0);
      if (w.pod_src != f.pod_src || w.cand_off != f.cand_off || w.list != f.list || w.status_host != f.status_host)
        fail("candidate lists", 0);
      const int32_t nb = f.empty_class >= 0 ? f.empty_class : f.n_classes;  // classes before the empty one
      if (w.cls_prog_off.size() < static_cast<size_t>(nb) + 1 ||
          !std::equal(f.cls_prog_off.begin(), f.cls_prog_off.begin() + nb + 1, w.cls_prog_off.begin()) ||
          !std::equal(f.cls_prog.begin(), f.cls_prog.begin() + f.cls_prog_off[nb], w.cls_prog.begin()))
        fail("class programs", 0);
      auto thr = [](const sr::Workload& v, int32_t row) { return row == 0 ? INT64_MIN : v.t_thr[row]; };
      for (size_t q = 0; q < f.pod_src.size(); ++q) {
        const int32_t* a = &w.pod_rows[q * 4];
        const int32_t* b = &f.pod_rows[q * 4];
        const bool da = a[0] == w.empty_class, db = b[0] == f.empty_class;
        if (da != db || (!da && a[0] != b[0])) fail("class", static_cast<long>(q));
        for (int d = 0; d < 3 && !da; ++d)
          if (thr(w, a[1 + d]) != thr(f, b[1 + d]) || w.t_dim[a[1 + d]] != f.t_dim[b[1 + d]]) fail("threshold", static_cast<long>(q));
        for (int k = 0; k < 4; ++k)
          if (w.pod_rec[q * 6 + k] != f.pod_rec[q * 6 + k]) fail("request words", static_cast<long>(q));
        const uint64_t Wp64 = static_cast<uint64_t>(w.Wp);
        if (w.pod_rec[q * 6 + 4] != (static_cast<uint64_t>(a[0]) * Wp64 | static_cast<uint64_t>(w.n_classes + a[1]) * Wp64 << 32) ||
            w.pod_rec[q * 6 + 5] != (static_cast<uint64_t>(w.n_classes + a[2]) * Wp64 |
                                     static_cast<uint64_t>(w.n_classes + a[3]) * Wp64 << 32))
          fail("row words", static_cast<long>(q));
      }
      sr_snapshot_destroy(s2);
    }
    printf("reuse check: %d ticks (%d reused, %d full), %ld pod patches, reuse encode avg %.3f ms (views %.3f), "
           "spot order moved %d, class flips %d, mismatches %d\n", reused + full, reused, full, patches,
           reused ? ms_reuse / reused : 0.0, reused ? ms_views / reused : 0.0, permuted, flips, bad);
    if (bad) return 2;
  }
  printf("Wp %d atoms %d classes %d program ops %zu t_rows %zu\n", w.Wp, w.n_atoms, w.n_classes, w.cls_prog.size(),
         w.t_dim.size());
  int tc[4] = {0, 0, 0, 0};
  for (int d : w.t_dim) tc[d]++;
  printf("t rows: cpu %d mem %d eph %d all %d; max cand pods %d\n", tc[0], tc[1], tc[2], tc[3], w.max_cand_pods);
  sr_snapshot_destroy(snap);
  sr_synth_destroy(s);
  return 0;
}
