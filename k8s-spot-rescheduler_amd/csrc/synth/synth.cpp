// synth.cpp — deterministic synthetic clusters (bench / test infrastructure).
//
// Spec (after SURVEY.md §8d): splitmix64 seeded with
// 0x5EED0000 + config; nodes in a shuffled on-demand/spot "API list" order;
// every node gets one DaemonSet pod first, then ReplicaSet pods until a
// per-node CPU fill target; pod CPU drawn from {50,100,100,250,500,1000,2000}m
// (tie-heavy on purpose: Go's unstable sort order matters), memory
// log-uniform 64Mi..8Gi.  Config-specific mixes: PreferNoSchedule taints (C2),
// zones / instance types / teams, nodeSelector, required node affinity,
// NoSchedule dedicated taints and tolerations, pods pinned to on-demand nodes
// (C3/C4), host ports + specific host IPs (C5).
#include "sr_synth.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

struct sr_synth {
  std::vector<std::string> strings;
  std::unordered_map<std::string, int32_t> ids;
  // nodes
  std::vector<int32_t> name;
  std::vector<int64_t> alloc_cpu, alloc_mem, alloc_eph, alloc_pods;
  std::vector<uint8_t> unsched;
  std::vector<int32_t> label_off{0}, label_key, label_val;
  std::vector<int32_t> taint_off{0}, taint_key, taint_val, taint_eff;
  // pods
  std::vector<int32_t> pod_node;
  std::vector<int64_t> cpu_sort, req_cpu, req_mem, req_eph;
  std::vector<int32_t> priority;
  std::vector<uint8_t> has_priority;
  std::vector<uint32_t> flags;
  std::vector<int32_t> sel_off{0}, sel_key, sel_val;
  std::vector<uint8_t> aff;
  std::vector<int32_t> term_off{0}, term_expr_off{0}, term_field_off{0};
  std::vector<int32_t> expr_key, expr_op, expr_val_off{0}, expr_vals;
  std::vector<int32_t> field_key, field_op, field_val_off{0}, field_vals;
  std::vector<int32_t> tol_off{0}, tol_key, tol_op, tol_val, tol_eff;
  std::vector<int32_t> port_off{0}, port_proto, port_num, port_ip;
  // drain attributes (sr_pod_drain): ReplicaSet or DaemonSet controllers, running
  std::vector<uint32_t> drain_flags;
  std::vector<uint8_t> phase, restart;
  std::vector<int64_t> deletion_age, grace;
  sr_node_label od{}, spot{};
  std::vector<uint8_t> str_label;  // sr_cluster.str_label over `strings`
  // realistic variant (sr_synth_params.*_fraction)
  bool has_volumes = false, has_scalars = false, has_acc = false;
  std::vector<int64_t> acc_cpu, acc_mem, acc_eph;  // NodeInfo.AddPod accounting (containers only)
  std::vector<int32_t> pod_sc_off{0}, pod_sc_name;
  std::vector<int64_t> pod_sc_req, pod_sc_acc;
  std::vector<int32_t> node_sc_off{0}, node_sc_name;
  std::vector<int64_t> node_sc_alloc;
  std::vector<uint8_t> v_prefilter, v_disk_ro, v_att_noncsi;
  std::vector<int32_t> v_disk_off{0}, v_disk_kind, v_disk_id;
  std::vector<int32_t> v_att_off{0}, v_att_key, v_att_id;
  std::vector<int32_t> v_limit_off{0}, v_limit_key;
  std::vector<int64_t> v_limit;
  std::vector<int32_t> v_zone_off{0}, v_zone_key, v_zone_val_off{0}, v_zone_vals;
  std::vector<int32_t> v_pv_off{0}, v_pv_term_off{0}, v_term_expr_off{0}, v_term_field_off{0};
  std::vector<int32_t> v_expr_key, v_expr_op, v_expr_val_off{0}, v_expr_vals;
  std::vector<int32_t> v_field_key, v_field_op, v_field_val_off{0}, v_field_vals;
  int32_t zone_keys[4] = {-1, -1, -1, -1};
  mutable sr_volumes vview{};  // the sr_volumes of sr_synth_view
  // affinity variant (sr_synth_params.anti_fraction / spread_fraction)
  bool has_affinity = false;
  std::vector<int32_t> a_ns, a_label_off{0}, a_label_key, a_label_val, a_anti_off{0};
  std::vector<int32_t> a_topo, a_ns_off{0}, a_ml_off{0}, a_ml_key, a_ml_val, a_me_off{0};
  std::vector<uint8_t> a_sel_nil;
  std::vector<int32_t> s_off{0}, s_skew, s_topo, s_ml_off{0}, s_ml_key, s_ml_val, s_me_off{0};
  std::vector<uint8_t> s_sel_nil, s_term;
  std::vector<int32_t> a_none{0};  // the empty tables' non-null base
  mutable sr_pod_affinity aview{};
  mutable sr_spread sview{};
  std::vector<uint64_t> stamp;  // sr_cluster.pod_stamp: pods never change after generation

  int32_t id(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    int32_t i = static_cast<int32_t>(strings.size());
    ids.emplace(s, i);
    strings.push_back(s);
    return i;
  }
};

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }
  int below(int n) { return static_cast<int>(next() % static_cast<uint64_t>(n)); }
  bool chance(double p) { return uni() < p; }
};

// apimachinery v0.19.2 util/validation [upstream], as the Go shim calls it:
// ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9] (qualifiedNameFmt)
bool qname_part(const std::string& s) {
  auto alnum = [](char ch) { return (ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z') || (ch >= '0' && ch <= '9'); };
  if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
  for (char ch : s)
    if (!alnum(ch) && ch != '-' && ch != '_' && ch != '.') return false;
  return true;
}
bool dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t a = 0;
  while (a <= s.size()) {  // labels [a-z0-9]([-a-z0-9]*[a-z0-9])? separated by '.'
    size_t b = s.find('.', a);
    if (b == std::string::npos) b = s.size();
    if (b == a) return false;
    auto lc = [](char ch) { return (ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9'); };
    if (!lc(s[a]) || !lc(s[b - 1])) return false;
    for (size_t i = a; i < b; ++i)
      if (!lc(s[i]) && s[i] != '-') return false;
    a = b + 1;
  }
  return true;
}
uint8_t label_flags(const std::string& s) {
  uint8_t f = 0;
  if (s.empty() || (s.size() <= 63 && qname_part(s))) f |= SR_STR_LABEL_VALUE;  // IsValidLabelValue
  const size_t slash = s.find('/');
  std::string name = s;
  bool ok = true;
  if (slash != std::string::npos) {  // IsQualifiedName: [prefix "/"] name
    ok = s.find('/', slash + 1) == std::string::npos && dns1123_subdomain(s.substr(0, slash));
    name = s.substr(slash + 1);
  }
  if (ok && name.size() <= 63 && qname_part(name)) f |= SR_STR_LABEL_KEY;
  return f;
}

constexpr int64_t kMi = 1024ll * 1024;
constexpr int64_t kGi = 1024ll * kMi;

struct Cfg {
  int n_od, n_spot, pods_min, pods_max;
  double od_fill_lo, od_fill_hi, spot_fill_lo, spot_fill_hi;
  bool prefer_taints, topology, constraints, ports;
  double pinned;
  int64_t pods_per_node_x100;  // BASELINE.json's pod count per node x 100 (0: whatever the fill gives);
                               // the fill lands a little below it and small pods top it up exactly
};

Cfg config_defaults(int c) {
  switch (c) {
    case 1: return {10, 10, 9, 9, 0.3, 0.6, 0.4, 0.9, false, false, false, false, 0.0, 0};
    case 2: return {300, 700, 0, 0, 0.45, 0.85, 0.45, 0.85, true, true, false, false, 0.0, 3000};
    case 3: return {1500, 3500, 0, 0, 0.5, 0.98, 0.5, 0.98, false, true, true, false, 0.15, 3000};
    case 4: return {15000, 35000, 0, 0, 0.5, 0.98, 0.5, 0.98, false, true, true, false, 0.15, 3000};
    default: return {300, 700, 0, 0, 0.55, 0.98, 0.55, 0.98, false, true, false, true, 0.0, 0};
  }
}

struct PodSpec {
  int64_t cpu = 0, mem = 0, eph = 0;
  int64_t init_cpu = 0, init_mem = 0;  // an init container (realistic variant)
  int32_t gpu = 0;                     // nvidia.com/gpu request
  int32_t volume = -1;                 // a bound EBS CSI claim: its volume id string
  int32_t zone = -1;                   // ... its PV's zone value
  int32_t prio = 0;
  uint32_t flags = 0;
  int32_t ns = -1, app = -1;  // affinity variant: namespace and app label
  bool anti = false, spread = false;
  std::vector<std::pair<int32_t, int32_t>> sel;
  bool aff = false;
  struct Expr {
    int32_t key, op;
    std::vector<int32_t> vals;
  };
  std::vector<std::vector<Expr>> terms;
  struct Tol {
    int32_t key, op, val, eff;
  };
  std::vector<Tol> tols;
  struct P {
    int32_t proto, port, ip;
  };
  std::vector<P> ports;
};

void push_pod(sr_synth* s, int32_t node, const PodSpec& p) {
  s->pod_node.push_back(node);
  s->cpu_sort.push_back(p.cpu);
  s->req_cpu.push_back(std::max(p.cpu, p.init_cpu));  // computePodResourceRequest: max with the init container
  s->req_mem.push_back(std::max(p.mem, p.init_mem));
  s->req_eph.push_back(p.eph);
  s->acc_cpu.push_back(p.cpu);  // calculateResource: the containers only
  s->acc_mem.push_back(p.mem);
  s->acc_eph.push_back(p.eph);
  if (p.gpu > 0) {
    s->pod_sc_name.push_back(s->id("nvidia.com/gpu"));
    s->pod_sc_req.push_back(p.gpu);
    s->pod_sc_acc.push_back(p.gpu);
  }
  s->pod_sc_off.push_back(static_cast<int32_t>(s->pod_sc_name.size()));
  s->v_prefilter.push_back(0);
  s->v_disk_off.push_back(0);
  if (p.volume >= 0) {  // one bound EBS CSI claim: attachable, zone label, node affinity
    s->v_att_key.push_back(s->id("attachable-volumes-csi-ebs.csi.aws.com"));
    s->v_att_id.push_back(p.volume);
    s->v_att_noncsi.push_back(0);
    s->v_zone_key.push_back(s->id("topology.kubernetes.io/zone"));
    s->v_zone_vals.push_back(p.zone);
    s->v_zone_val_off.push_back(static_cast<int32_t>(s->v_zone_vals.size()));
    s->v_expr_key.push_back(s->id("topology.kubernetes.io/zone"));
    s->v_expr_op.push_back(SR_OP_IN);
    s->v_expr_vals.push_back(p.zone);
    s->v_expr_val_off.push_back(static_cast<int32_t>(s->v_expr_vals.size()));
    s->v_term_expr_off.push_back(static_cast<int32_t>(s->v_expr_key.size()));
    s->v_term_field_off.push_back(static_cast<int32_t>(s->v_field_key.size()));
    s->v_pv_term_off.push_back(static_cast<int32_t>(s->v_term_expr_off.size() - 1));
  }
  s->v_att_off.push_back(static_cast<int32_t>(s->v_att_key.size()));
  s->v_zone_off.push_back(static_cast<int32_t>(s->v_zone_key.size()));
  s->v_pv_off.push_back(static_cast<int32_t>(s->v_pv_term_off.size() - 1));
  s->priority.push_back(p.prio);
  s->has_priority.push_back(1);
  s->flags.push_back(p.flags);
  for (auto& kv : p.sel) {
    s->sel_key.push_back(kv.first);
    s->sel_val.push_back(kv.second);
  }
  s->sel_off.push_back(static_cast<int32_t>(s->sel_key.size()));
  s->aff.push_back(p.aff ? 1 : 0);
  for (auto& t : p.terms) {
    for (auto& e : t) {
      s->expr_key.push_back(e.key);
      s->expr_op.push_back(e.op);
      s->expr_vals.insert(s->expr_vals.end(), e.vals.begin(), e.vals.end());
      s->expr_val_off.push_back(static_cast<int32_t>(s->expr_vals.size()));
    }
    s->term_expr_off.push_back(static_cast<int32_t>(s->expr_key.size()));
    s->term_field_off.push_back(static_cast<int32_t>(s->field_key.size()));
  }
  s->term_off.push_back(static_cast<int32_t>(s->term_expr_off.size() - 1));
  for (auto& t : p.tols) {
    s->tol_key.push_back(t.key);
    s->tol_op.push_back(t.op);
    s->tol_val.push_back(t.val);
    s->tol_eff.push_back(t.eff);
  }
  s->tol_off.push_back(static_cast<int32_t>(s->tol_key.size()));
  for (auto& q : p.ports) {
    s->port_proto.push_back(q.proto);
    s->port_num.push_back(q.port);
    s->port_ip.push_back(q.ip);
  }
  s->port_off.push_back(static_cast<int32_t>(s->port_proto.size()));
  if (s->has_affinity) {  // namespace, app label; the Deployment's anti-affinity term / spread constraint
    s->a_ns.push_back(p.ns);
    s->a_label_key.push_back(s->id("app"));
    s->a_label_val.push_back(p.app);
    s->a_label_off.push_back(static_cast<int32_t>(s->a_label_key.size()));
    if (p.anti) {  // podAntiAffinity required: topologyKey hostname, matchLabels app=<name>
      s->a_topo.push_back(s->id("kubernetes.io/hostname"));
      s->a_ns_off.push_back(static_cast<int32_t>(s->a_ns_off.back()));
      s->a_sel_nil.push_back(0);
      s->a_ml_key.push_back(s->id("app"));
      s->a_ml_val.push_back(p.app);
      s->a_ml_off.push_back(static_cast<int32_t>(s->a_ml_key.size()));
      s->a_me_off.push_back(s->a_me_off.back());
    }
    s->a_anti_off.push_back(static_cast<int32_t>(s->a_topo.size()));
    if (p.spread) {  // topologySpreadConstraints: maxSkew 1, zone, DoNotSchedule, matchLabels app=<name>
      s->s_skew.push_back(1);
      s->s_topo.push_back(s->id("topology.kubernetes.io/zone"));
      s->s_sel_nil.push_back(0);
      s->s_ml_key.push_back(s->id("app"));
      s->s_ml_val.push_back(p.app);
      s->s_ml_off.push_back(static_cast<int32_t>(s->s_ml_key.size()));
      s->s_me_off.push_back(s->s_me_off.back());
    }
    s->s_off.push_back(static_cast<int32_t>(s->s_skew.size()));
    s->s_term.push_back(0);
  }
  s->drain_flags.push_back((p.flags & SR_POD_DAEMONSET_CONTROLLER) ? SR_DRAIN_CTRL_DAEMONSET : SR_DRAIN_CTRL_REPLICASET);
  s->phase.push_back(SR_PHASE_RUNNING);
  s->restart.push_back(SR_RESTART_ALWAYS);
  s->deletion_age.push_back(0);
  s->grace.push_back(-1);
}

}  // namespace

extern "C" {

sr_synth* sr_synth_generate(const sr_synth_params* prm) {
  const int config = prm && prm->config >= 1 && prm->config <= 5 ? prm->config : 1;
  Cfg cfg = config_defaults(config);
  if (prm && prm->n_on_demand > 0) cfg.n_od = prm->n_on_demand;
  if (prm && prm->n_spot > 0) cfg.n_spot = prm->n_spot;
  if (prm && prm->pinned_fraction >= 0) cfg.pinned = prm->pinned_fraction;
  const double f_stateful = prm ? prm->stateful_fraction : 0, f_init = prm ? prm->init_fraction : 0,
               f_gpu = prm ? prm->gpu_fraction : 0;
  Rng rng{prm && prm->seed ? prm->seed : 0x5EED0000ull + static_cast<uint64_t>(config)};
  auto* s = new sr_synth();
  // fixed ids first
  const int32_t E = s->id(""), MN = s->id("metadata.name"), UK = s->id("node.kubernetes.io/unschedulable");
  (void)E;
  (void)MN;
  (void)UK;
  const int32_t ROLE = s->id("kubernetes.io/role"), WORKER = s->id("worker"), SPOTW = s->id("spot-worker");
  const int32_t HOST = s->id("kubernetes.io/hostname");
  const int32_t ZONE = s->id("topology.kubernetes.io/zone");
  const int32_t ITYPE = s->id("node.kubernetes.io/instance-type");
  const int32_t TEAM = s->id("team"), DEDICATED = s->id("dedicated"), GPU = s->id("gpu");
  const int32_t ODT = s->id("on-demand"), SPT = s->id("spot"), TRUE_ = s->id("true");
  int32_t zones[3], teams[4], types[8];
  for (int i = 0; i < 3; ++i) zones[i] = s->id(std::string("zone-") + static_cast<char>('a' + i));
  for (int i = 0; i < 4; ++i) teams[i] = s->id(std::string("team-") + static_cast<char>('a' + i));
  const int type_cores[8] = {4, 8, 16, 32, 64, 8, 16, 32};
  const int type_gib[8] = {16, 32, 64, 128, 256, 16, 32, 256};
  for (int i = 0; i < 8; ++i) types[i] = s->id("type-" + std::to_string(i));
  const int n_types = cfg.topology && cfg.constraints ? 8 : 5;
  s->od = sr_node_label{ROLE, WORKER, 1};
  s->spot = sr_node_label{ROLE, SPOTW, 1};
  s->has_volumes = f_stateful > 0;
  const double f_anti = prm ? prm->anti_fraction : 0, f_spread = prm ? prm->spread_fraction : 0;
  s->has_affinity = f_anti > 0 || f_spread > 0;
  // affinity variant: Deployments of ~5 replicas, their kinds and replicas
  // drawn from their own stream (the rest of the cluster is unchanged)
  Rng arng{(prm && prm->seed ? prm->seed : 0x5EED0000ull + static_cast<uint64_t>(config)) ^ 0xAFF1A17Eull};
  const int64_t n_deploy = std::max<int64_t>(1, (static_cast<int64_t>(cfg.n_od + cfg.n_spot) * 30) / 5);
  int32_t ns_ids[16];
  if (s->has_affinity)
    for (int i = 0; i < 16; ++i) ns_ids[i] = s->id("ns-" + std::to_string(i));
  auto deploy_kind = [&](int64_t d) {  // 0 none, 1 anti-affinity, 2 spread (a hash of d: stable)
    const double u = static_cast<double>((static_cast<uint64_t>(d) * 0x9E3779B97F4A7C15ull) >> 11) *
                     (1.0 / 9007199254740992.0);
    return u < f_anti ? 1 : u < f_anti + f_spread ? 2 : 0;
  };
  std::vector<int64_t> node_anti;  // the anti-affinity Deployments with a replica on the current node
  auto assign_deploy = [&](PodSpec& p) {
    if (!s->has_affinity) return;
    int64_t d = static_cast<int64_t>(arng.next() % static_cast<uint64_t>(n_deploy));
    for (int t = 0; t < 8 && deploy_kind(d) == 1 &&
                    std::find(node_anti.begin(), node_anti.end(), d) != node_anti.end(); ++t)
      d = static_cast<int64_t>(arng.next() % static_cast<uint64_t>(n_deploy));
    int kind = deploy_kind(d);
    if (kind == 1 && std::find(node_anti.begin(), node_anti.end(), d) != node_anti.end()) kind = -1;  // none
    if (kind == 1) node_anti.push_back(d);
    p.ns = ns_ids[d % 16];
    p.app = s->id(kind < 0 ? "solo-" + std::to_string(s->pod_node.size()) : "app-" + std::to_string(d));
    p.anti = kind == 1;
    p.spread = kind == 2;
    if (p.anti) p.flags |= SR_POD_HAS_REQ_ANTI_AFFINITY;
  };
  s->has_scalars = f_gpu > 0;
  s->has_acc = f_init > 0;
  if (s->has_volumes) {
    s->zone_keys[0] = s->id("failure-domain.beta.kubernetes.io/zone");
    s->zone_keys[1] = s->id("failure-domain.beta.kubernetes.io/region");
    s->zone_keys[2] = ZONE;
    s->zone_keys[3] = s->id("topology.kubernetes.io/region");
  }
  int32_t n_volumes = 0;

  const int n_nodes = cfg.n_od + cfg.n_spot;
  std::vector<uint8_t> is_spot(n_nodes, 0);
  for (int i = 0; i < cfg.n_spot; ++i) is_spot[i] = 1;
  for (int i = n_nodes - 1; i > 0; --i) std::swap(is_spot[i], is_spot[rng.below(i + 1)]);  // list order

  const int64_t cpu_choices[7] = {50, 100, 100, 250, 500, 1000, 2000};
  char buf[64];
  std::vector<int64_t> node_used(static_cast<size_t>(n_nodes), 0);
  std::vector<int32_t> node_pods(static_cast<size_t>(n_nodes), 0);
  for (int node = 0; node < n_nodes; ++node) {
    const bool spot = is_spot[node];
    std::snprintf(buf, sizeof(buf), "node-%06d", node);
    const int32_t nm = s->id(buf);
    const int t = rng.below(n_types);
    s->name.push_back(nm);
    s->alloc_cpu.push_back(1000ll * type_cores[t]);
    s->alloc_mem.push_back(type_gib[t] * kGi);
    s->alloc_eph.push_back(100 * kGi);
    s->alloc_pods.push_back(110);
    const bool unsched = cfg.constraints && spot && rng.chance(0.01);
    s->unsched.push_back(unsched ? 1 : 0);
    // labels
    s->label_key.push_back(ROLE);
    s->label_val.push_back(spot ? SPOTW : WORKER);
    s->label_key.push_back(HOST);
    s->label_val.push_back(nm);
    int32_t team = -1, node_zone = -1;
    if (cfg.topology) {
      node_zone = zones[rng.below(3)];
      s->label_key.push_back(ZONE);
      s->label_val.push_back(node_zone);
      s->label_key.push_back(ITYPE);
      s->label_val.push_back(types[t]);
    }
    if (cfg.constraints && rng.chance(0.5)) {
      team = teams[rng.below(4)];
      s->label_key.push_back(TEAM);
      s->label_val.push_back(team);
    }
    s->label_off.push_back(static_cast<int32_t>(s->label_key.size()));
    // taints
    if (cfg.prefer_taints && (!spot || rng.chance(0.10))) {
      s->taint_key.push_back(spot ? SPT : ODT);
      s->taint_val.push_back(TRUE_);
      s->taint_eff.push_back(SR_EFFECT_PREFER_NO_SCHEDULE);
    }
    if (cfg.constraints && spot && rng.chance(0.15)) {
      s->taint_key.push_back(DEDICATED);
      s->taint_val.push_back(team >= 0 ? team : teams[rng.below(4)]);
      s->taint_eff.push_back(SR_EFFECT_NO_SCHEDULE);
    }
    if (unsched) {
      s->taint_key.push_back(UK);
      s->taint_val.push_back(E);
      s->taint_eff.push_back(SR_EFFECT_NO_SCHEDULE);
    }
    s->taint_off.push_back(static_cast<int32_t>(s->taint_key.size()));
    // realistic variant: GPUs on 1 in 8 nodes, the EBS CSI driver's attach limit on every node
    const bool gpu_node = f_gpu > 0 && rng.chance(0.125);
    if (gpu_node) {
      s->node_sc_name.push_back(s->id("nvidia.com/gpu"));
      s->node_sc_alloc.push_back(4);
    }
    s->node_sc_off.push_back(static_cast<int32_t>(s->node_sc_name.size()));
    if (f_stateful > 0) {
      s->v_limit_key.push_back(s->id("attachable-volumes-csi-ebs.csi.aws.com"));
      s->v_limit.push_back(25);
    }
    s->v_limit_off.push_back(static_cast<int32_t>(s->v_limit_key.size()));

    node_anti.clear();
    // DaemonSet pod first in the node's list
    PodSpec ds;
    if (s->has_affinity) {
      ds.ns = s->id("kube-system");
      ds.app = s->id("node-exporter");
    }
    ds.cpu = 100;
    ds.mem = 128 * kMi;
    ds.flags = SR_POD_DAEMONSET_CONTROLLER;
    if (cfg.ports) ds.ports.push_back({SR_PROTO_TCP, 9100, -1});
    push_pod(s, node, ds);
    // ReplicaSet pods up to a CPU fill target
    const double lo = spot ? cfg.spot_fill_lo : cfg.od_fill_lo, hi = spot ? cfg.spot_fill_hi : cfg.od_fill_hi;
    const int64_t target = static_cast<int64_t>((lo + (hi - lo) * rng.uni()) * 1000.0 * type_cores[t]);
    // C1 has a fixed pod count (rescheduler_test-sized); the others fill each
    // node to its CPU target (at most 109 pods: allocatable pods is 110).
    const int want = config == 1 ? cfg.pods_min : 108;
    int64_t used = ds.cpu;
    for (int k = 0; k < want; ++k) {
      PodSpec p;
      p.cpu = cpu_choices[rng.below(7)];
      if (config != 1 && used + p.cpu > target) break;
      used += p.cpu;
      p.mem = static_cast<int64_t>(std::exp(std::log(64.0) + (std::log(8192.0) - std::log(64.0)) * rng.uni())) * kMi;
      if (cfg.constraints && rng.chance(0.10)) p.eph = (1 + rng.below(10)) * kGi;
      if (spot && rng.chance(0.10)) p.prio = -1;
      if (!spot && cfg.constraints) {
        if (rng.chance(cfg.pinned)) {
          p.sel.push_back({ROLE, WORKER});  // pinned to on-demand nodes: never movable to spot
        } else if (rng.chance(0.20)) {
          const int kind = rng.below(4);
          if (kind < 2) p.sel.push_back({ZONE, zones[rng.below(3)]});
          else if (kind == 2) p.sel.push_back({ITYPE, types[rng.below(n_types)]});
          else p.sel.push_back({TEAM, teams[rng.below(4)]});
        }
        if (rng.chance(0.10)) {
          p.aff = true;
          const int nt = 1 + rng.below(3);
          for (int ti = 0; ti < nt; ++ti) {
            std::vector<PodSpec::Expr> term;
            const int ne = 1 + rng.below(2);
            for (int ei = 0; ei < ne; ++ei) {
              switch (rng.below(4)) {
                case 0:
                  term.push_back({ZONE, SR_OP_IN, {zones[rng.below(3)], zones[rng.below(3)]}});
                  break;
                case 1:
                  term.push_back({ITYPE, SR_OP_NOT_IN, {types[rng.below(n_types)]}});
                  break;
                case 2:
                  term.push_back({TEAM, SR_OP_EXISTS, {}});
                  break;
                default:
                  term.push_back({GPU, SR_OP_DOES_NOT_EXIST, {}});
                  break;
              }
            }
            p.terms.push_back(std::move(term));
          }
        }
        if (rng.chance(0.20)) {
          if (rng.chance(0.5))
            p.tols.push_back({DEDICATED, SR_TOL_EQUAL, teams[rng.below(4)], SR_EFFECT_NO_SCHEDULE});
          else
            p.tols.push_back({DEDICATED, SR_TOL_EXISTS, E, SR_EFFECT_EMPTY});
        }
      }
      if (f_init > 0 && rng.chance(f_init)) {  // e.g. a migration / warm-up step heavier than the app
        p.init_cpu = 2 * p.cpu;
        p.init_mem = p.mem + 256 * kMi;
      }
      if (gpu_node && rng.chance(f_gpu)) p.gpu = 1;
      if (f_stateful > 0 && node_zone >= 0 && p.prio >= 0 && rng.chance(f_stateful)) {
        std::snprintf(buf, sizeof(buf), "vol-%08d", n_volumes++);
        p.volume = s->id(buf);
        p.zone = node_zone;
      }
      assign_deploy(p);
      if (cfg.ports && rng.chance(0.30)) {
        static const int32_t kPorts[3] = {80, 443, 8080};
        const int32_t port = kPorts[rng.below(3)];
        int32_t ip = -1;
        if (rng.chance(0.02)) {
          std::snprintf(buf, sizeof(buf), "10.0.%d.%d", rng.below(4), rng.below(250));
          ip = s->id(buf);
        }
        p.ports.push_back({SR_PROTO_TCP, port, ip});
      }
      push_pod(s, node, p);
    }
    node_used[node] = used;
  }
  // Top-up to BASELINE.json's pod count (C2 30k, C3 150k, C4 1.5M for the
  // default node counts): 50m / 64Mi ReplicaSet pods appended round robin to
  // nodes with a free pod slot and 50m of CPU headroom (LIST order: last on
  // their node).
  if (cfg.pods_per_node_x100 > 0) {
    std::fill(node_pods.begin(), node_pods.end(), 0);
    for (int32_t nd : s->pod_node) ++node_pods[nd];
    const int64_t target = cfg.pods_per_node_x100 * n_nodes / 100;
    int64_t total = static_cast<int64_t>(s->pod_node.size());
    for (bool room = true; total < target && room;) {
      room = false;
      for (int node = 0; node < n_nodes && total < target; ++node) {
        if (node_pods[node] >= 110 || node_used[node] + 50 > s->alloc_cpu[node]) continue;
        PodSpec p;
        p.cpu = 50;
        p.mem = 64 * kMi;
        if (s->has_affinity) {
          node_anti.clear();  // (a filler pod never joins an anti-affinity Deployment)
          p.ns = ns_ids[node % 16];
          p.app = s->id("filler-" + std::to_string(node));
        }
        push_pod(s, node, p);
        node_used[node] += 50;
        ++node_pods[node];
        ++total;
        room = true;
      }
    }
  }
  for (const std::string& str : s->strings) s->str_label.push_back(label_flags(str));
  // Stamps (sr_cluster.pod_stamp): the generation is a function of the
  // parameters, so (parameters, pod index) names the pod's content; two
  // clusters of different parameters never share a stamp.
  uint64_t h = 0xCBF29CE484222325ull;
  auto fold = [&](uint64_t x) { h = (h ^ x) * 0x100000001B3ull; };
  if (prm) {  // field by field (the struct has padding)
    auto bits = [](double d) {
      uint64_t u;
      std::memcpy(&u, &d, sizeof(u));
      return u;
    };
    fold(static_cast<uint64_t>(prm->config));
    fold(prm->seed);
    fold(static_cast<uint64_t>(prm->n_on_demand));
    fold(static_cast<uint64_t>(prm->n_spot));
    for (double d : {prm->pinned_fraction, prm->stateful_fraction, prm->init_fraction, prm->gpu_fraction,
                     prm->anti_fraction, prm->spread_fraction})
      fold(bits(d));
  }
  s->stamp.resize(s->pod_node.size());
  for (size_t i = 0; i < s->stamp.size(); ++i) {
    uint64_t x = h ^ (0x9E3779B97F4A7C15ull * (i + 1));
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    s->stamp[i] = x | 1;  // never 0 (unknown)
  }
  return s;
}

void sr_synth_destroy(sr_synth* s) { delete s; }

void sr_synth_view(const sr_synth* s, sr_cluster* c) {
  sr_nodes& n = c->nodes;
  n.n = static_cast<int32_t>(s->name.size());
  n.name = s->name.data();
  n.alloc_milli_cpu = s->alloc_cpu.data();
  n.alloc_memory = s->alloc_mem.data();
  n.alloc_ephemeral = s->alloc_eph.data();
  n.alloc_pods = s->alloc_pods.data();
  n.unschedulable = s->unsched.data();
  n.label_off = s->label_off.data();
  n.label_key = s->label_key.data();
  n.label_val = s->label_val.data();
  n.taint_off = s->taint_off.data();
  n.taint_key = s->taint_key.data();
  n.taint_val = s->taint_val.data();
  n.taint_effect = s->taint_eff.data();
  sr_pods& p = c->pods;
  p.n = static_cast<int32_t>(s->pod_node.size());
  p.node = s->pod_node.data();
  p.cpu_sort_milli = s->cpu_sort.data();
  p.req_milli_cpu = s->req_cpu.data();
  p.req_memory = s->req_mem.data();
  p.req_ephemeral = s->req_eph.data();
  p.priority = s->priority.data();
  p.has_priority = s->has_priority.data();
  p.flags = s->flags.data();
  p.sel_off = s->sel_off.data();
  p.sel_key = s->sel_key.data();
  p.sel_val = s->sel_val.data();
  p.aff_required = s->aff.data();
  p.term_off = s->term_off.data();
  p.term_expr_off = s->term_expr_off.data();
  p.term_field_off = s->term_field_off.data();
  p.expr_key = s->expr_key.data();
  p.expr_op = s->expr_op.data();
  p.expr_val_off = s->expr_val_off.data();
  p.expr_vals = s->expr_vals.data();
  p.field_key = s->field_key.data();
  p.field_op = s->field_op.data();
  p.field_val_off = s->field_val_off.data();
  p.field_vals = s->field_vals.data();
  p.tol_off = s->tol_off.data();
  p.tol_key = s->tol_key.data();
  p.tol_op = s->tol_op.data();
  p.tol_val = s->tol_val.data();
  p.tol_effect = s->tol_eff.data();
  p.port_off = s->port_off.data();
  p.port_proto = s->port_proto.data();
  p.port_num = s->port_num.data();
  p.port_ip = s->port_ip.data();
  c->id_empty = 0;
  c->id_metadata_name = 1;
  c->id_unschedulable_key = 2;
  c->pod_affinity = nullptr;  // the BASELINE configs carry no pod (anti-)affinity
  c->n_strings = static_cast<int32_t>(s->str_label.size());
  c->str_int = nullptr;       // ... nor node-affinity Gt / Lt
  c->str_int_ok = nullptr;
  c->str_label = s->str_label.data();
  c->pod_scalar_off = c->node_scalar_off = nullptr;  // no scalar resources in the BASELINE configs
  c->pod_scalar_name = c->node_scalar_name = nullptr;
  c->pod_scalar_req = c->pod_scalar_acc = c->node_scalar_alloc = nullptr;
  c->acc_milli_cpu = c->acc_memory = c->acc_ephemeral = nullptr;  // AddPod adds the fit request
  c->spread = nullptr;  // no topology spread constraints in the BASELINE configs
  c->volumes = nullptr;  // realistic variant only (sr_synth_params.stateful_fraction)
  c->pod_stamp = s->stamp.data();
  if (s->has_affinity) {
    sr_pod_affinity& a = s->aview;
    a = sr_pod_affinity{};
    a.ns = s->a_ns.data();
    a.label_off = s->a_label_off.data();
    a.label_key = s->a_label_key.data();
    a.label_val = s->a_label_val.data();
    a.anti_off = s->a_anti_off.data();
    a.topology_key = s->a_topo.data();
    a.ns_off = s->a_ns_off.data();
    a.ns_ids = s->a_none.data();
    a.selector_nil = s->a_sel_nil.data();
    a.ml_off = s->a_ml_off.data();
    a.ml_key = s->a_ml_key.data();
    a.ml_val = s->a_ml_val.data();
    a.me_off = s->a_me_off.data();
    a.me_key = a.me_op = a.me_val_off = a.me_vals = s->a_none.data();
    a.aff_off = nullptr;
    c->pod_affinity = &a;
    sr_spread& sp = s->sview;
    sp = sr_spread{};
    sp.off = s->s_off.data();
    sp.max_skew = s->s_skew.data();
    sp.topology_key = s->s_topo.data();
    sp.selector_nil = s->s_sel_nil.data();
    sp.ml_off = s->s_ml_off.data();
    sp.ml_key = s->s_ml_key.data();
    sp.ml_val = s->s_ml_val.data();
    sp.me_off = s->s_me_off.data();
    sp.me_key = sp.me_op = sp.me_val_off = sp.me_vals = s->a_none.data();
    sp.terminating = s->s_term.data();
    c->spread = &sp;
  }
  if (s->has_acc) {
    c->acc_milli_cpu = s->acc_cpu.data();
    c->acc_memory = s->acc_mem.data();
    c->acc_ephemeral = s->acc_eph.data();
  }
  if (s->has_scalars) {
    c->pod_scalar_off = s->pod_sc_off.data();
    c->pod_scalar_name = s->pod_sc_name.data();
    c->pod_scalar_req = s->pod_sc_req.data();
    c->pod_scalar_acc = s->pod_sc_acc.data();
    c->node_scalar_off = s->node_sc_off.data();
    c->node_scalar_name = s->node_sc_name.data();
    c->node_scalar_alloc = s->node_sc_alloc.data();
  }
  if (s->has_volumes) {
    sr_volumes& v = s->vview;
    v = sr_volumes{};
    v.prefilter_fail = s->v_prefilter.data();
    v.disk_off = s->v_disk_off.data();
    v.disk_kind = s->v_disk_kind.data();
    v.disk_id = s->v_disk_id.data();
    v.disk_ro = s->v_disk_ro.data();
    v.att_off = s->v_att_off.data();
    v.att_key = s->v_att_key.data();
    v.att_id = s->v_att_id.data();
    v.att_noncsi = s->v_att_noncsi.data();
    v.limit_off = s->v_limit_off.data();
    v.limit_key = s->v_limit_key.data();
    v.limit = s->v_limit.data();
    v.zone_off = s->v_zone_off.data();
    v.zone_key = s->v_zone_key.data();
    v.zone_val_off = s->v_zone_val_off.data();
    v.zone_vals = s->v_zone_vals.data();
    for (int i = 0; i < 4; ++i) v.zone_keys[i] = s->zone_keys[i];
    v.pv_off = s->v_pv_off.data();
    v.pv_term_off = s->v_pv_term_off.data();
    v.term_expr_off = s->v_term_expr_off.data();
    v.term_field_off = s->v_term_field_off.data();
    v.expr_key = s->v_expr_key.data();
    v.expr_op = s->v_expr_op.data();
    v.expr_val_off = s->v_expr_val_off.data();
    v.expr_vals = s->v_expr_vals.data();
    v.field_key = s->v_field_key.data();
    v.field_op = s->v_field_op.data();
    v.field_val_off = s->v_field_val_off.data();
    v.field_vals = s->v_field_vals.data();
    c->volumes = &v;
  }
}

void sr_synth_drain(const sr_synth* s, sr_pod_drain* d) {
  d->n = static_cast<int32_t>(s->drain_flags.size());
  d->flags = s->drain_flags.data();
  d->phase = s->phase.data();
  d->restart_policy = s->restart.data();
  d->deletion_age_ns = s->deletion_age.data();
  d->grace_seconds = s->grace.data();
}

void sr_synth_labels(const sr_synth* s, sr_node_label* on_demand, sr_node_label* spot) {
  if (on_demand) *on_demand = s->od;
  if (spot) *spot = s->spot;
}

const char* sr_synth_string(const sr_synth* s, int32_t id) {
  if (id < 0 || id >= static_cast<int32_t>(s->strings.size())) return "";
  return s->strings[id].c_str();
}

int32_t sr_synth_num_strings(const sr_synth* s) { return static_cast<int32_t>(s->strings.size()); }

uint8_t sr_synth_label_flags(const char* s) { return label_flags(s ? std::string(s) : std::string()); }

}  // extern "C"
