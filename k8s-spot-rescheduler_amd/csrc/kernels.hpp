// kernels.hpp — device view of the workload and the kernel launchers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sr {

// Pointers into the device arena (layout: DESIGN.md §HBM layout).
struct DevWorkload {
  int32_t n_spot, n_pad, Wp, WR, WT;
  const int64_t* free_cpu;
  const int64_t* free_mem;
  const int64_t* free_eph;
  const int32_t* pods_left;
  const uint64_t* port_bits;
  const uint64_t* req_bits;    // [WR][n_pad]
  const uint64_t* taint_bits;  // [WT][n_pad]
  const uint64_t* cls_sel;     // [classes][WR]
  const uint64_t* cls_tol;     // [classes][WT]
  const uint64_t* cls_port;
  const int32_t* cls_flags;
  const int32_t* cls_term_off;
  const uint64_t* term_mask;   // [terms][WR]
  int32_t n_a, n_b;
  const int32_t* a_class;
  const int32_t* a_zero;
  const int64_t* a_cpu;
  const int64_t* a_eph;
  const int64_t* b_mem;
  const int32_t* b_all;
  int32_t n_pods;
  const int32_t* pod_a;
  const int32_t* pod_b;
  const int32_t* pod_zero;
  const int64_t* pod_cpu;
  const int64_t* pod_mem;
  const int64_t* pod_eph;
  const uint64_t* pod_ports;
  int32_t n_cand;
  const int32_t* cand_off;
  const int32_t* cand_global;
  const int32_t* list_small;
  const int32_t* list_large;
  int32_t n_small, n_large;
  // outputs / scratch
  uint64_t* A;         // [n_a][Wp]
  uint64_t* B;         // [n_b][Wp]
  uint64_t* F;         // [n_pods][Wp] dense feasibility bitmask vs the base snapshot
  int32_t* out_node;   // [n_pods] spot position or -1
  int32_t* out_status; // [n_cand]
  int32_t* d_min;      // [2] {first_ok, first_fallback} (global indices, INT_MAX = none)
  int32_t* result;     // [4 + max pods] {winner, local, npods, first_fallback, mapping...}
};

// K0: A and B rows (also resets d_min: d_min[1] = local first fallback).
hipError_t launch_tables(const DevWorkload& w, int32_t local_first_fallback, hipStream_t s);
// K1: F = A[pod_a] & B[pod_b].
hipError_t launch_feasibility(const DevWorkload& w, hipStream_t s);
// K2: per-candidate first-fit placement; atomicMin of first_ok into d_min[0].
hipError_t launch_placement(const DevWorkload& w, hipStream_t s);
// K3: winner mapping into `result`.
hipError_t launch_winner(const DevWorkload& w, hipStream_t s);

}  // namespace sr
