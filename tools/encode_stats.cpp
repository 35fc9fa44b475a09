// Host-only harness: NewNodeMap + snapshot + encode_workload on a synthetic
// config, printing the workload's dimensions and host-side timings (no GPU).
//   make -C k8s-spot-rescheduler_amd tools && k8s-spot-rescheduler_amd/build/encode_stats 3
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "../k8s-spot-rescheduler_amd/csrc/host.hpp"
#include "../k8s-spot-rescheduler_amd/csrc/synth/sr_synth.h"

namespace sr { extern double encode_phase_ms[16]; }

int main(int argc, char** argv) {
  sr_synth_params p{};
  p.config = argc > 1 ? atoi(argv[1]) : 3;
  p.pinned_fraction = -1;
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
  auto t1 = std::chrono::steady_clock::now();
  sr_snapshot* snap = nullptr;
  sr_snapshot_create(&c, spot.data(), ns, off.data(), idx.data(), &snap);
  auto t2 = std::chrono::steady_clock::now();
  std::vector<int32_t> coff{0}, cp;
  for (int i = 0; i < nod; ++i) {
    int node = odn[i];
    for (int j = off[node]; j < off[node + 1]; ++j)
      if (!(c.pods.flags[idx[j]] & (SR_POD_MIRROR | SR_POD_DAEMONSET_CONTROLLER))) cp.push_back(idx[j]);
    coff.push_back(cp.size());
  }
  sr_candidates cands{nod, coff.data(), cp.data(), nullptr};
  sr::Workload w;
  std::string err;
  auto t3 = std::chrono::steady_clock::now();
  int reps = 20;
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto a = std::chrono::steady_clock::now();
    sr::encode_workload(snap, &c, &cands, &w, &err);
    best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
  }
  auto t4 = std::chrono::steady_clock::now();
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  printf("config %d: nodes %d pods %d spot %d od %d cand_pods %zu\n", p.config, nn, np, ns, nod, cp.size());
  printf("new_node_map %.2f ms, snapshot %.2f ms, encode %.2f ms (best %.2f)\n", ms(t0, t1), ms(t1, t2), ms(t3, t4) / reps, best);
  printf("phases(ms): dims %.2f fallback+ports+taints %.2f pod-static %.2f classes %.2f nodes+atoms %.2f t-rows+pods %.2f lists %.2f (pod-static: keys %.2f; t-setup %.2f)\n",
         sr::encode_phase_ms[0], sr::encode_phase_ms[1], sr::encode_phase_ms[2], sr::encode_phase_ms[3],
         sr::encode_phase_ms[4], sr::encode_phase_ms[5], sr::encode_phase_ms[6], sr::encode_phase_ms[7], sr::encode_phase_ms[8]);
  printf("fine(ms): pass1 %.2f ports+taints %.2f | atoms-nodes %.2f atoms-reqs %.2f | lb+recs %.2f empty %.2f trows %.2f ranks %.2f recoffs %.2f\n",
         sr::encode_phase_ms[8], sr::encode_phase_ms[1], sr::encode_phase_ms[9], sr::encode_phase_ms[4],
         sr::encode_phase_ms[10], sr::encode_phase_ms[11], sr::encode_phase_ms[12], sr::encode_phase_ms[13], sr::encode_phase_ms[5]);
  printf("keys split: gather+hash %.3f shards %.3f merge %.3f\n", sr::encode_phase_ms[14], sr::encode_phase_ms[15], sr::encode_phase_ms[7]);
  printf("Wp %d atoms %d classes %d program ops %zu t_rows %zu\n", w.Wp, w.n_atoms, w.n_classes, w.cls_prog.size(),
         w.t_dim.size());
  int tc[4] = {0, 0, 0, 0};
  for (int d : w.t_dim) tc[d]++;
  printf("t rows: cpu %d mem %d eph %d all %d; max cand pods %d\n", tc[0], tc[1], tc[2], tc[3], w.max_cand_pods);
  sr_snapshot_destroy(snap);
  sr_synth_destroy(s);
  return 0;
}
