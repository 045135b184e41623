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
  int32_t *Kact;               // [V] live dishes
  int32_t *next_id;            // [V] next raw dish id (reference: V.K)
  double *hyper;               // [3V+2] tau, alpha, sigma, alpha_g, sigma_g
  int32_t T, n_free;
  uint64_t draws;              // sequential-stream draws consumed
  int32_t resume_i;            // next customer of the current sweep
  int32_t status;              // MVC_ST_*
  int32_t chain_id;            // global chain id (Philox stream)
  int32_t pad;
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
__device__ __forceinline__ double wave_max(double x) {
  for (int m = 32; m >= 1; m >>= 1) {
    const double o = shfl_xor_d(x, m);
    x = o > x ? o : x;
  }
  return x;
}
// tree64 butterfly over the 64 lanes (slot = lane); every lane gets the sum.
// Identical association to butterfly64() in oracle/mvc_oracle.cpp: at offset
// h lane l adds lane l^h, i.e. pairs (l, l+h) for l < h.
__device__ __forceinline__ double wave_tree_sum(double x) {
  for (int m = 32; m >= 1; m >>= 1) x = x + shfl_xor_d(x, m);
  return x;
}
// Same butterfly, keeping the value each lane holds after every step; used
// for the descent.  In the oracle's notation lvl[5] = v32, lvl[4] = v16,
// lvl[3] = v8, lvl[2] = v4, lvl[1] = v2, lvl[0] = v1 (root), lvl[6] = leaves.
struct Tree64Levels {
  double v32, v16, v8, v4, v2, v1;   // value after the step with that offset
};
__device__ __forceinline__ double wave_tree_sum_levels(double x, Tree64Levels &L) {
  x = x + shfl_xor_d(x, 32); L.v32 = x;
  x = x + shfl_xor_d(x, 16); L.v16 = x;
  x = x + shfl_xor_d(x, 8);  L.v8 = x;
  x = x + shfl_xor_d(x, 4);  L.v4 = x;
  x = x + shfl_xor_d(x, 2);  L.v2 = x;
  x = x + shfl_xor_d(x, 1);  L.v1 = x;
  return x;
}
// Descent (oracle Tree64::select_chunk).  lvl[k][l] (2^k entries) equals the
// value lane l holds after the step with offset 2^k, for l < 2^k; leaves are
// the inputs (level 6).  Wave-uniform r; returns the selected slot.
__device__ __forceinline__ int wave_tree_select(const Tree64Levels &L, double leaf, double &r) {
  int l = 0;
  // node at level kk (h = 2^kk) has children lvl[kk+1][l] and lvl[kk+1][l+h]
#define MVC_DESCEND(VAL, H)                                   \
  {                                                           \
    const double a = __shfl((VAL), l, 64);                    \
    const double b = __shfl((VAL), l + (H), 64);              \
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
