// mvc_internal.h — device-side state layouts and helpers shared by the
// exact-schedule and parallel-schedule kernels of libmvc_hip.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mvc_philox.h"
#include "mvc_pmath.h"

#define MVC_MAXV 64          // max views handled in LDS-resident scalars
#define MVC_WAVE 64          // CDNA wavefront

// ---------------------------------------------------------------------------
// Exact schedule: one 64-lane workgroup per chain walks the reference's
// sequential customer loop (multiview_gibbs.cpp:157-200).
// State mirrors multiview_state.h:7-33 with two changes that do not alter any
// arithmetic: (1) tables live in stable *slots* plus a slot<->position
// permutation, so the reference's swap-and-pop relabel (multiview_utils.cpp:
// 175-190) is O(1) instead of walking the member list; (2) per view only the
// live dishes (l_vk > 0) are stored, compacted in ascending raw id, which is
// exactly the iteration order of every reference loop over k (dead slots are
// skipped there: utils.cpp:52-53,229-230, hyper.cpp:186,307-308).
// ---------------------------------------------------------------------------
struct ExactChain {
  int32_t TC, KC;              // capacities (table slots, live dishes per view)
  int32_t *z;                  // [n] slot of each customer
  int32_t *n_t;                // [TC] customers per slot
  int32_t *pos_of_slot;        // [TC]
  int32_t *slot_at_pos;        // [TC]
  int32_t *free_slots;         // [TC] stack of unused slots
  int32_t *dish;               // [V*TC] live-dish index of slot, per view
  int32_t *d_id, *d_n, *d_l;   // [V*KC] raw id, n_vk, l_vk
  double *d_S1, *d_S2;         // [V*KC] sum_y, sum_y2
  double *f, *logf;            // [V*KC] per-customer scratch
  double *P;                   // [TC] per-customer table probabilities
  double *mhbuf;               // [n+1] log(m - sigma) table for the EPPF
  double *ldt;                 // [V][n+2] the sweep's log-determinant terms (ref_f_vk)
  int32_t *Kact;               // [V] live dishes
  int32_t *next_id;            // [V] next raw dish id (reference: V.K)
  double *hyper;               // [3V+2] tau, alpha, sigma, alpha_g, sigma_g
  int32_t T, n_free;
  uint64_t draws;              // sequential-stream draws consumed
  int32_t resume_i;            // next customer of the current sweep
  int32_t status;              // MVC_ST_*
  int32_t chain_id;            // global chain id (Philox stream)
  int32_t todo;                // sweeps left in the current launch (mvc_exact_sweep_kernel)
};

#define MVC_ST_RUNNING 0
#define MVC_ST_OVERFLOW 1      // capacity exhausted before customer resume_i
#define MVC_ST_DONE 2          // sweep (incl. hyperparameter MH) finished
#define MVC_ST_ERROR 3

// ---------------------------------------------------------------------------
// Parallel schedule.  Positions are dense 0..T-1; dishes are
// live lists per view.  S1 is stored dim-major per view: S1T[v][d][KC].
// ---------------------------------------------------------------------------
struct ParState {
  int32_t n, V, D, TC, KC;
  int32_t T;                   // tables (host mirror)
  int32_t *z;                  // [n] table position
  int32_t *n_t;                // [TC]
  int32_t *dish;               // [V*TC] live index
  int32_t *d_id, *d_n, *d_l;   // [V*KC]
  double *S1T;                 // [V*D*KC]
  double *S2;                  // [V*KC]
  double *Q;                   // [V*KC] ||S1||^2 (fma chain)
  double *c0, *cb;             // [V*KC] frozen-state coefficients
  double *lmass;               // [TC] log(n_t - sigma_g)
  double *hyper;               // [3V+2]
  int32_t *Kact;               // [V]
  int32_t *next_id;            // [V]
  int32_t *Ltot;               // [V]
};

// ---------------------------------------------------------------------------
// wave helpers (64 lanes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double shfl_xor_d(double x, int m) {
  return __shfl_xor(x, m, 64);
}
__device__ __forceinline__ double shfl_d(double x, int src) {
  return __shfl(x, src, 64);
}
// Cross-lane moves for fp64 values, gfx950 (no LDS traffic):
//   down<h>(x), h = 1,2,4,8 : DPP row_shl:h, lane l receives lane l+h of its
//                             16-lane row (0 past the row end);
//   down16(x) / down32(x)   : v_permlane16_swap / v_permlane32_swap, lane l
//                             receives lane l+16 (even rows) / l+32 (l < 32).
// The reductions below are prefix trees: after the step with offset h only
// lanes l < h hold tree values, which is all the tree64 association needs
// (node l at offset h = lane l + lane l+h, oracle butterfly64()); the root
// is read back with v_readlane.  Callers keep the whole wave converged.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int H>
__device__ __forceinline__ double down_d(double x) {
  static_assert(H == 1 || H == 2 || H == 4 || H == 8, "row shift");
  return dpp_d<0x100 + H>(x);
}
__device__ __forceinline__ double down16_d(double x) {
  const long long b = __double_as_longlong(x);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __longlong_as_double(((long long)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ double down32_d(double x) {
  const long long b = __double_as_longlong(x);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  return __longlong_as_double(((long long)hi[1] << 32) | (unsigned)lo[1]);
}
// broadcast lane 0 of each 16-lane row to the row (DPP row_newbcast:0)
__device__ __forceinline__ double row_bcast0_d(double x) { return dpp_d<0x150>(x); }
// wave-uniform read of lane `l` (l wave-uniform)
__device__ __forceinline__ double readlane_d(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int readlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

__device__ __forceinline__ double dmax(double a, double b) { return b > a ? b : a; }

__device__ __forceinline__ double wave_max(double x) {
  x = dmax(x, down32_d(x));
  x = dmax(x, down16_d(x));
  x = dmax(x, down_d<8>(x));
  x = dmax(x, down_d<4>(x));
  x = dmax(x, down_d<2>(x));
  x = dmax(x, down_d<1>(x));
  return readlane_d(x, 0);
}
// max over each 16-lane row, broadcast to the row
__device__ __forceinline__ double row16_max(double x) {
  x = dmax(x, down_d<8>(x));
  x = dmax(x, down_d<4>(x));
  x = dmax(x, down_d<2>(x));
  x = dmax(x, down_d<1>(x));
  return row_bcast0_d(x);
}
// tree64 over the 64 lanes (slot = lane); returns the root, wave-uniform.
// Same association as butterfly64() in oracle/mvc_oracle.cpp: at offset h
// node l = node l + node l+h.
__device__ __forceinline__ double wave_tree_sum(double x) {
  x = x + down32_d(x);
  x = x + down16_d(x);
  x = x + down_d<8>(x);
  x = x + down_d<4>(x);
  x = x + down_d<2>(x);
  x = x + down_d<1>(x);
  return readlane_d(x, 0);
}
// pw16 of the 16 lanes of each row (pairs (c, c + h), h = 1, 2, 4, 8: the
// oracle's pw16 association), broadcast to the row.
__device__ __forceinline__ double row_pw16(double x) {
  x = x + down_d<1>(x);
  x = x + down_d<2>(x);
  x = x + down_d<4>(x);
  x = x + down_d<8>(x);
  return row_bcast0_d(x);
}
// tree16 over each row's 16 lanes (tree64 of a chunk whose upper 48 slots
// were already folded in by the caller), root broadcast to the row.
__device__ __forceinline__ double row16_tree_sum(double x) {
  x = x + down_d<8>(x);
  x = x + down_d<4>(x);
  x = x + down_d<2>(x);
  x = x + down_d<1>(x);
  return row_bcast0_d(x);
}
// Same tree, keeping the node values of every level for the descent.  In
// the oracle's notation lvl[5] = v32, lvl[4] = v16, ..., lvl[1] = v2,
// lvl[0] = root (returned), lvl[6] = leaves; node l of lvl[k] sits in lane l.
struct Tree64Levels {
  double v32, v16, v8, v4, v2;
};
__device__ __forceinline__ double wave_tree_sum_levels(double x, Tree64Levels &L) {
  x = x + down32_d(x);   L.v32 = x;
  x = x + down16_d(x);   L.v16 = x;
  x = x + down_d<8>(x);  L.v8 = x;
  x = x + down_d<4>(x);  L.v4 = x;
  x = x + down_d<2>(x);  L.v2 = x;
  x = x + down_d<1>(x);
  return readlane_d(x, 0);
}
// Descent (oracle Tree64::select_chunk) on wave-uniform values: node l at
// offset h has children lvl[k+1][l] and lvl[k+1][l+h]; go right unless the
// right child is 0 or r < left.  Returns the slot; r is updated.
__device__ __forceinline__ int wave_tree_select(const Tree64Levels &L, double leaf, double &r) {
  int l = 0;
#define MVC_DESCEND(VAL, H)                                   \
  {                                                           \
    const double a = readlane_d((VAL), l);                    \
    const double b = readlane_d((VAL), l + (H));              \
    if (!(b == 0.0 || r < a)) { r = r - a; l = l + (H); }     \
  }
  MVC_DESCEND(L.v2, 1)
  MVC_DESCEND(L.v4, 2)
  MVC_DESCEND(L.v8, 4)
  MVC_DESCEND(L.v16, 8)
  MVC_DESCEND(L.v32, 16)
  MVC_DESCEND(leaf, 32)
#undef MVC_DESCEND
  return l;
}

#define HIP_CHECK_RET(expr)                                                   \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) return _e;                                          \
  } while (0)
