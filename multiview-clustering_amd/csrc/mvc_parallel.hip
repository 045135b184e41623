// mvc_parallel.hip — the parallel ("mode P") execution of the reference's
// sequential sweep on gfx950.
//
// Per sweep (one stream; the host reads the repair's outcome once per batch):
//   phase A   : every customer draws its table against the sweep-start state
//               (virtual self-removal), two kernels per batch: an lp producer
//               (MFMA: mvc_par_lpall_kernel / lpview / lpbig; generic:
//               lpgen) writes lp of every (customer, dish) to the lp buffer,
//               the draw kernel (one lane per customer) reduces it in dish /
//               table order and draws with the Philox counter (customer,
//               sweep, chain);
//   repair    : the in-order repair of mvc_repair.h (the decisions after the
//               first mover, re-evaluated against the moved state);
//   compaction: dead tables / dishes dropped (only after a sweep with moves);
//   hyper     : one workgroup: ||S1||^2, the MH updates of
//               multiview_hyper.cpp:233-292 (closed-form EPPF, tree64
//               order), then the next sweep's coefficients.
// Every fp64 expression matches SeqSampler in oracle/mvc_oracle.cpp.
// Compile with -ffp-contract=off.

#include "mvc_internal.h"

namespace {

constexpr double kEps = 1e-6;
constexpr int kStatsChunk = 4096;   // must equal oracle kStatsChunk

struct Coef { double c0, cb; };
__device__ __forceinline__ Coef coef(int n_, double Q, double tau, double L2pt, int D) {
  const double a = tau + (double)n_;
  const double b = tau + (double)(n_ + 1);
  Coef c;
  c.c0 = (double)D * ((-0.5 * L2pt) - 0.5 * mvc_log(b / a)) - (0.5 * Q) / ((tau * a) * b);
  c.cb = 1.0 / (tau * b);
  return c;
}

// Kernel argument bundle (passed by value).
struct Sweep {
  ParState P;
  const double *y;        // [V][n][D]
  const double *Y2;       // [V][n]
  const double *L2pt;     // [V]  log(2 pi tau)
  const double *cnew;     // [V]  D * (-0.5 L2pt)
  const int32_t *Koff;    // [V+1] prefix of Kact
  int32_t *choice;        // [n] position or -1 (birth)
  const int32_t *status;  // [V+4]; status[V+3] = tables with n_t > 0
  const double *yt;       // MFMA A-fragment layout of y (mvc_par_ytile_kernel)
  const double *S1t;      // MFMA B-fragment layout of S1 (mvc_par_s1tile_kernel)
  int32_t SP;             // k-steps per view in yt/S1t (D/4 rounded up to MVC_ZR)
  double *vmax;           // [V][n] the view maximum m_v of each customer (producer -> draw)
  int32_t T, sumK;
  uint64_t seed;
  uint32_t chain, sweep;
  int32_t *fmin;          // non-null: the register draw reduces the first mover into it (mvc_seq_first_kernel's work)
};

}  // namespace

typedef double mvc_d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Phase 1 runs as two kernels per batch of customers:
//   1. an lp producer writes lp[i][Koff[v] + j] (frozen dish j of view v,
//      self-removal applied to the customer's own dish) into the lp buffer,
//      slabs of 16 customers, dish-major:  lpb[(li >> 4) * sumK * 16 +
//      k * 16 + lpb_slot(li & 15)],  li = i - b0;
//        * MFMA producer (D % 4 == 0, D >= 16, K_v <= 64): G = Y S1^T tiles
//          with v_mfma_f64_16x16x4_f64, S1 B-fragments staged through LDS by
//          the block, y A-fragments streamed from the tiled copy yt;
//        * generic producer (any D): one lane per customer, fma_dot loops;
//   2. the draw kernel: one lane per customer, sequential reductions over
//      dishes and tables (the spec of oracle eval_view_seq /
//      resample_customer), no cross-lane traffic.
// ---------------------------------------------------------------------------
#define MVC_Z_KMAX 64
#define MVC_Z_VMAX 8

// Within a slab, customer row rho sits at slot 4 (rho & 3) + (rho >> 2): the
// rows one lane of the MFMA producer holds (grp, grp + 4, grp + 8, grp + 12 of
// a 16 x 16 tile) are then 32 contiguous bytes, stored as two 16-byte
// pieces, and a dish's 16 rows are still one 128-byte line.
__host__ __device__ inline int lpb_slot(int rho) { return 4 * (rho & 3) + (rho >> 2); }
__host__ __device__ inline size_t lpb_index(int li, int k, int sumK) {
  return ((size_t)(li >> 4) * (size_t)sumK + (size_t)k) * 16 + (size_t)lpb_slot(li & 15);
}

// A-fragment layout, k-steps in pairs (one 16 B load per lane covers two):
// yt[((v*ntile + tile)*SP + 2*(s/2))*64 + 2*lane + (s & 1)] = y[v][16 tile +
// (lane & 15)][4 s + (lane >> 4)], zero outside n x D (SP is even).
extern "C" __global__ void mvc_par_ytile_kernel(int n, int V, int D, int SP, const double *y, double *yt) {
  const int ntile = (n + 15) >> 4;
  const size_t total = (size_t)V * ntile * SP * 64;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t q = e >> 7;                       // (view, tile, pair)
    const int r = (int)(e & 127);
    const int ln = r >> 1;
    const int SPP = SP >> 1;
    const int s = 2 * (int)(q % SPP) + (r & 1);
    const size_t vt = q / SPP;
    const int tile = (int)(vt % ntile);
    const int v = (int)(vt / ntile);
    const int row = tile * 16 + (ln & 15), d = 4 * s + (ln >> 4);
    yt[e] = (row < n && d < D) ? y[((size_t)v * n + row) * D + d] : 0.0;
  }
}

// B-fragment layout per view (ncolt_v = ceil(K_v / 16) column tiles):
// S1t[S1o_v + (s * ncolt_v + ct) * 64 + lane] = S1[v][d = 4 s + (lane >> 4)]
// [j = 16 ct + (lane & 15)], zero outside D x K_v; S1o_v = SP*64*sum_{u<v}
// ncolt_u.
extern "C" __global__ void mvc_par_s1tile_kernel(ParState P, const int32_t *Koff, int SP, double *S1t) {
  const int V = P.V, D = P.D, KC = P.KC;
  size_t off[MVC_Z_VMAX + 1];
  off[0] = 0;
  for (int v = 0; v < V; ++v) off[v + 1] = off[v] + (size_t)SP * 64 * ((Koff[v + 1] - Koff[v] + 15) >> 4);
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < off[V]; e += (size_t)gridDim.x * blockDim.x) {
    int v = 0;
    while (e >= off[v + 1]) ++v;
    const int K = Koff[v + 1] - Koff[v];
    const int nct = (K + 15) >> 4;
    const size_t loc = e - off[v];
    const int ln = (int)(loc & 63);
    const size_t q = loc >> 6;
    const int ct = (int)(q % nct), s = (int)(q / nct);
    const int d = 4 * s + (ln >> 4), j = 16 * ct + (ln & 15);
    S1t[e] = (d < D && j < K) ? P.S1T[((size_t)v * D + d) * KC + j] : 0.0;
  }
}

// LDS hand-off between lanes of one wavefront: a wave's LDS instructions
// execute in order, so only the compiler must not reorder across this point
// (a memory fence here would also wait for every outstanding global load,
// i.e. drain the y prefetch).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
// Block barrier for LDS hand-off only: waits for this wave's LDS ops, not
// for its global loads in flight (__syncthreads would emit vmcnt(0)).
__device__ __forceinline__ void block_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef double mvc_d2 __attribute__((ext_vector_type(2)));

// MFMA lp producer, one launch per view.  The view's S1
// B-fragments for every k-step (S1t block, <= 64 KB at D = 128) are staged
// in LDS once per block; waves then run independently over their 16-customer
// tiles, streaming the A-fragments from yt (paired layout: one 16 B load per
// lane covers two k-steps, 1 KB per wave) through a ring of RP registers:
// each k-step pair waits for the oldest load only and issues the load RP
// pairs ahead (across tile boundaries), so HBM latency hides behind 2 RP
// k-steps of every wave on the CU.  The tile's lp goes straight from the
// accumulators to the lp buffer (a fixed number of stores per tile).
#define MVC_ZR 8              // SP (k-steps per view) is padded to a multiple of this
__host__ __device__ inline size_t lpview_shared_bytes(int SP, int NT, int K, int T) {
  return 8 * ((size_t)SP * NT * 64 + 3 * (size_t)K + 8 * 48) + 4 * (2 * (size_t)K + 2 * (size_t)T + 8 * 16) + 64;
}

// k-step pairs of one 16-customer tile: SPPT > 0 fully unrolled (static ring
// slots, so the compiler can count outstanding loads exactly and never drains
// the ring), SPPT == 0 a runtime loop for other D.
template <int NT, int SPPT, int RP>
__device__ __forceinline__ void lpview_tile_mfma(const mvc_d2 *cur, const mvc_d2 *nxt, int SPP, const double *Bl,
                                                 mvc_d2 (&ring)[RP], mvc_d4 (&acc)[4]) {
  if constexpr (SPPT > 0) {
    // B-fragments one k-step pair ahead (LDS latency off the MFMA issue path)
    double bc[2 * NT], bn[2 * NT];
#pragma unroll
    for (int t = 0; t < 2 * NT; ++t) bc[t] = Bl[t * 64];
#pragma unroll
    for (int q = 0; q < SPPT; ++q) {
      const int u = q % RP;
      const mvc_d2 a = ring[u];
      ring[u] = (q + RP < SPPT) ? cur[(q + RP) * 64] : nxt[(q + RP - SPPT) * 64];
      if (q + 1 < SPPT) {
        const double *bk = Bl + (size_t)(2 * (q + 1)) * NT * 64;
#pragma unroll
        for (int t = 0; t < 2 * NT; ++t) bn[t] = bk[t * 64];
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], bc[t], acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], bc[NT + t], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);           // keep each refill RP pairs ahead (no sinking)
#pragma unroll
      for (int t = 0; t < 2 * NT; ++t) bc[t] = bn[t];
    }
  } else {
    for (int s0 = 0; s0 < SPP; s0 += RP) {
#pragma unroll
      for (int u = 0; u < RP; ++u) {
        const int q = s0 + u;
        const mvc_d2 a = ring[u];
        ring[u] = (q + RP < SPP) ? cur[(size_t)(q + RP) * 64] : nxt[(size_t)(q + RP - SPP) * 64];
        const double *bk = Bl + (size_t)(2 * q) * NT * 64;
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], bk[t * 64], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], bk[(NT + t) * 64], acc[t], 0, 0, 0);
      }
    }
  }
}

template <int NT, int SPPT, int RP>
__global__ __launch_bounds__(512) void mvc_par_lpview_kernel(Sweep A, int v, int b0, int nb, double *lpb,
                                                             double *discard) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, BW = blockDim.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n, T = A.T;
  const int SP = A.SP, SPP = SPPT > 0 ? SPPT : (SP >> 1);   // k-steps, k-step pairs per tile
  const int koff = A.Koff[v], K = A.Koff[v + 1] - koff, sumK = A.Koff[V];
  const double tau = P.hyper[v], L2pt = A.L2pt[v];
  double *Bs = (double *)smem;                     // [SP][NT][64]
  double *d_c0 = Bs + (size_t)SP * NT * 64;        // [K]
  double *d_cb = d_c0 + K;
  double *d_Q = d_cb + K;
  double *wsp = d_Q + K;                           // per wave: y2s[16], selfG[16], mrest[16]
  double *y2s = wsp + w * 48;
  double *selfG = y2s + 16;
  double *mrest = selfG + 16;
  int *ip = (int *)(wsp + 8 * 48);
  int *d_n = ip;                                   // [K]
  int *d_l = d_n + K;                              // [K]
  int *t_dish = d_l + K;                           // [T]
  int *t_n = t_dish + T;                           // [T]
  int *zs = t_n + T + w * 16;                      // per wave [16]
  {
    size_t off = 0;
    for (int u = 0; u < v; ++u) off += (size_t)SP * 64 * ((A.Koff[u + 1] - A.Koff[u] + 15) >> 4);
    const mvc_d2 *src = (const mvc_d2 *)(A.S1t + off);
    mvc_d2 *dst = (mvc_d2 *)Bs;
    for (int e = tid; e < SP * NT * 32; e += blockDim.x) dst[e] = src[e];
  }
  for (int j = tid; j < K; j += blockDim.x) {
    d_c0[j] = P.c0[v * KC + j];
    d_cb[j] = P.cb[v * KC + j];
    d_Q[j] = P.Q[v * KC + j];
    d_n[j] = P.d_n[v * KC + j];
    d_l[j] = P.d_l[v * KC + j];
  }
  for (int p = tid; p < T; p += blockDim.x) {
    t_dish[p] = P.dish[v * P.TC + p];
    t_n[p] = P.n_t[p];
  }
  __syncthreads();
  const double cnew = A.cnew[v];

  const int ntile = (nb + 15) >> 4;
  const int ntile_all = (n + 15) >> 4;
  const int tile0 = b0 >> 4;
  const int gw = blockIdx.x * BW + w, NWT = gridDim.x * BW;
  if (gw >= ntile) return;                         // whole wave: no barriers below
  const int nmy = (ntile - gw + NWT - 1) / NWT;    // tiles of this wave
  const mvc_d2 *ybase = (const mvc_d2 *)(A.yt + (size_t)v * ntile_all * SP * 64) + lane;
  auto tptr = [&](int m) -> const mvc_d2 * {       // A-fragments of the wave's m-th tile (clamped)
    return ybase + (size_t)(tile0 + gw + min(m, nmy - 1) * NWT) * SPP * 64;
  };
  double *const dslot = discard + lane;            // stores of padding / out-of-batch lanes
  mvc_d2 ring[RP];
  {
    const mvc_d2 *c0p = tptr(0), *c1p = tptr(1);
#pragma unroll
    for (int u = 0; u < RP; ++u) ring[u] = (u < SPP) ? c0p[u * 64] : c1p[(u - SPP) * 64];
  }
  const double *Bl = Bs + lane;
  for (int m = 0; m < nmy; ++m) {
    const int tile = gw + m * NWT;                 // batch-local tile
    const int li0 = tile * 16;
    // this tile's z and Y2 (row = lane & 15); used in the epilogue
    const int li_row = min(li0 + col, nb - 1);
    const int pz = P.z[b0 + li_row];
    const double y2 = A.Y2[(size_t)v * n + b0 + li_row];
    mvc_d4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
    lpview_tile_mfma<NT, SPPT, RP>(tptr(m), tptr(m + 1), SPP, Bl, ring, acc);
    // ---- epilogue: lp of the tile's 16 customers for this view
    if (grp == 0) { zs[col] = pz; y2s[col] = y2; }
    wave_lds_sync();
    double hy[4], hr[4];
    int j0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double y2r = y2s[grp + 4 * r];
      hy[r] = 0.5 * y2r;
      hr[r] = (-0.5 * y2r) / tau;
      j0[r] = t_dish[zs[grp + 4 * r]];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // G of the own dish -> LDS
      const int jt = j0[r] >> 4;
      double g = acc[0][r];
#pragma unroll
      for (int t = 1; t < NT; ++t)
        if (jt == t) g = acc[t][r];
      if (col == (j0[r] & 15)) selfG[grp + 4 * r] = g;
    }
    // frozen-dish lp for every (row, dish): a fixed number of unconditional
    // stores (invalid lanes go to their discard slot; the own dish is
    // overwritten below by this same wave, in program order)
    // The view maximum of the draw (oracle eval_view_seq: max over included
    // dishes, then the new dish) is formed here: the frozen dishes other than
    // the own one by a 16-lane max per row, the own dish and the new dish by
    // the row's lane below; m_v goes to vmax, so the draw reads each lp row once.
    double mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -MVC_PM_INF;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int j = 16 * t + col;
      const int jc = min(j, K - 1);
      const double c0j = d_c0[jc], cbj = d_cb[jc];
      const bool inc = j < K && d_l[jc] > 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double val = __builtin_fma(acc[t][r] + hy[r], cbj, c0j) + hr[r];
        const int li = li0 + grp + 4 * r;
        double *dst = (j < K && li < nb) ? lpb + lpb_index(li, koff + j, sumK) : dslot;
        *dst = val;
        if (inc && j != j0[r] && val > mx[r]) mx[r] = val;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double mr = row16_max(mx[r]);
      if (col == 0) mrest[grp + 4 * r] = mr;
    }
    wave_lds_sync();
    {   // own dish, one row per lane
      const double G = selfG[col];
      const int jj = t_dish[pz];
      const double Gp = G - y2;
      const double Qp = (d_Q[jj] - 2.0 * G) + y2;
      const Coef cf = coef(d_n[jj] - 1, Qp, tau, L2pt, D);
      const double hself = (-0.5 * y2) / tau;
      const double sv = __builtin_fma(Gp + 0.5 * y2, cf.cb, cf.c0) + hself;
      const bool ok = lane < 16 && li0 + col < nb;
      double *dst = ok ? lpb + lpb_index(li0 + col, koff + jj, sumK) : dslot;
      *dst = sv;
      const int l0p = d_l[jj] - ((t_n[pz] - 1) > 0 ? 0 : 1);
      double m = mrest[col];
      if (l0p > 0 && sv > m) m = sv;
      const double lfn = cnew + hself;
      if (lfn > m) m = lfn;
      double *dm = ok ? A.vmax + (size_t)v * n + b0 + li0 + col : dslot;
      *dm = m;
    }
    wave_lds_sync();
  }
}

// The dish-block producer's tiles with the k-steps unrolled (SPC = D / 4):
// the same MFMA chain and epilogue as the runtime-SP loop of
// mvc_par_lpbig_kernel, so the same bits.
// Two k-steps of A-fragments from one 16-byte load per lane: lane (row, q)
// holds y[row][8p + 2q], y[row][8p + 2q + 1] (x, y below, rows q = 0..3 of
// the wave); k-step 2p needs d = 8p + k on lane (row, k), k-step 2p + 1
// d = 8p + 4 + k.  permlane16_swap(x, y) makes the 16-lane rows (0,1 | 4,5)
// and (2,3 | 6,7), permlane32_swap of those (0,1,2,3) and (4,5,6,7).
__device__ __forceinline__ void lpbig_pair_ksteps(mvc_d2 xy, double &a0, double &a1) {
  const long long bx = __double_as_longlong(xy[0]), by = __double_as_longlong(xy[1]);
  const auto l16 = __builtin_amdgcn_permlane16_swap((unsigned)bx, (unsigned)by, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap((unsigned)(bx >> 32), (unsigned)(by >> 32), false, false);
  const auto l32 = __builtin_amdgcn_permlane32_swap(l16[0], l16[1], false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(h16[0], h16[1], false, false);
  a0 = __longlong_as_double(((long long)h32[0] << 32) | (unsigned)l32[0]);
  a1 = __longlong_as_double(((long long)h32[1] << 32) | (unsigned)l32[1]);
}

// A dish block's view maximum of a customer: vmode 0 writes it (the view's
// first block), 1 maxes it into the earlier blocks' value (launches in block
// order), 2 is an atomic max into a row pre-filled with -inf (every block of
// the view in one launch, mvc_par_lpbig_group_kernel).  Max is exact, so the
// block order does not matter: the same bits every way.  Lanes without a
// customer (!ok) store to their discard slot, but never atomically: those
// slots are shared by every wave of the grid.
__device__ __forceinline__ void lpbig_vmax_put(int vmode, bool ok, double *dm, double m, double mprev) {
  if (vmode == 2) {
    if (ok) __builtin_amdgcn_flat_atomic_fmax_f64(dm, m);
  } else {
    if (vmode == 1) m = dmax(m, mprev);
    *dm = m;
  }
}

// The dish-block producer's tiles with the k-steps unrolled (SPC = D / 4):
// the same MFMA chain and epilogue as the runtime-SP loop of
// mvc_par_lpbig_kernel, so the same bits.  A-fragments are read 16 bytes per
// lane (two k-steps, lpbig_pair_ksteps), RP pair loads ahead.
template <int NTB, int SPC>
__device__ __forceinline__ void lpbig_tiles(const Sweep &A, int v, int jb0, int kb, int vmode, int b0, int nb,
                                            double *lpb, double *dslot, const double *yv, const double *Bs, double *y2s,
                                            double *selfG, double *mrest, const double *b_c0, const double *b_cb,
                                            const double *b_Q, const int *b_l, const int *b_dn, const int *t_dish,
                                            const int *t_n, int *zs, int gw, int NWT, int ntile, double tau,
                                            double L2pt, double cnew) {
#ifndef MVC_BIG_RP
#define MVC_BIG_RP 8
#endif
  constexpr int NP = SPC / 2, RP = (NP % MVC_BIG_RP == 0) ? MVC_BIG_RP : 8;   // k-step pairs per tile, in flight
  static_assert(NP >= RP && NP % RP == 0, "unrolled k-step pairs");
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63, col = lane & 15, grp = lane >> 4;
  const int V = P.V, D = 4 * SPC, n = P.n;
  const int koff = A.Koff[v], sumK = A.Koff[V];
  // this lane's pairs of row (col) of tile t (clamped to the batch: unconditional loads); pair p at [4 p]
  auto rowp = [&](int t) -> const mvc_d2 * {
    const int tt = t < ntile ? t : (ntile - 1);
    return (const mvc_d2 *)(yv + (size_t)(b0 + min(tt * 16 + col, nb - 1)) * D) + grp;
  };
  mvc_d2 ar[RP];
  const mvc_d2 *yr = rowp(gw);
#pragma unroll
  for (int u = 0; u < RP; ++u) ar[u] = yr[4 * u];
  for (int tile = gw; tile < ntile; tile += NWT) {
    const int li0 = tile * 16;
    const int li_row = min(li0 + col, nb - 1);
    const bool ok = lane < 16 && li0 + col < nb;
    // the epilogue's global reads, issued ahead of this tile's MFMAs
    const int pz = P.z[b0 + li_row];
    const double y2 = A.Y2[(size_t)v * n + b0 + li_row];
    double *dm = ok ? A.vmax + (size_t)v * n + b0 + li0 + col : dslot;
    const double mprev = *dm;   // (unconditional load: read only when vmode == 1)
    const mvc_d2 *yn = rowp(tile + NWT);
    mvc_d4 acc[NTB];
#pragma unroll
    for (int t = 0; t < NTB; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
    double bc[NTB];
#pragma unroll
    for (int t = 0; t < NTB; ++t) bc[t] = Bs[t * 64 + lane];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      double a2[2];
      lpbig_pair_ksteps(ar[p % RP], a2[0], a2[1]);
      ar[p % RP] = p + RP < NP ? yr[4 * (p + RP)] : yn[4 * (p + RP - NP)];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int s = 2 * p + h;
        double bn[NTB];
        const double *bk = Bs + (size_t)(s + 1 < SPC ? s + 1 : SPC - 1) * NTB * 64 + lane;
#pragma unroll
        for (int t = 0; t < NTB; ++t) bn[t] = bk[t * 64];
#pragma unroll
        for (int t = 0; t < NTB; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[h], bc[t], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NTB; ++t) bc[t] = bn[t];
      }
      __builtin_amdgcn_sched_barrier(0);   // keep each refill RP pairs ahead (no sinking)
    }
    yr = yn;
    // ---- epilogue (the runtime-SP loop's, with the own dish's Q / d_n from LDS)
    if (grp == 0) { zs[col] = pz; y2s[col] = y2; }
    wave_lds_sync();
    double hy[4], hr[4];
    int j0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double y2r = y2s[grp + 4 * r];
      hy[r] = 0.5 * y2r;
      hr[r] = (-0.5 * y2r) / tau;
      j0[r] = t_dish[zs[grp + 4 * r]];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int jl = j0[r] - jb0;
      double g = acc[0][r];
#pragma unroll
      for (int t = 1; t < NTB; ++t)
        if ((jl >> 4) == t) g = acc[t][r];
      if (jl >= 0 && jl < kb && col == (jl & 15)) selfG[grp + 4 * r] = g;
    }
    double mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -MVC_PM_INF;
#pragma unroll
    for (int t = 0; t < NTB; ++t) {
      const int j = jb0 + 16 * t + col;
      const double c0j = b_c0[16 * t + col], cbj = b_cb[16 * t + col];
      const bool inj = j < jb0 + kb;
      const bool inc = inj && b_l[16 * t + col] > 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double val = __builtin_fma(acc[t][r] + hy[r], cbj, c0j) + hr[r];
        const int li = li0 + grp + 4 * r;
        double *dst = (inj && li < nb) ? lpb + lpb_index(li, koff + j, sumK) : dslot;
        *dst = val;
        if (inc && j != j0[r] && val > mx[r]) mx[r] = val;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double mr = row16_max(mx[r]);
      if (col == 0) mrest[grp + 4 * r] = mr;
    }
    wave_lds_sync();
    {   // own dish (when in this block) and the view maximum, one row per lane
      const int jj = t_dish[pz];
      const int jl = jj - jb0;
      const bool own = jl >= 0 && jl < kb;
      const int jb = own ? jl : 0;
      double m = mrest[col];
      const double hself = (-0.5 * y2) / tau;
      {   // (unconditional: lanes without their own dish here store to the discard slot)
        const double G = selfG[col];
        const double Gp = G - y2;
        const double Qp = (b_Q[jb] - 2.0 * G) + y2;
        const Coef cf = coef(b_dn[jb] - 1, Qp, tau, L2pt, D);
        const double sv = __builtin_fma(Gp + 0.5 * y2, cf.cb, cf.c0) + hself;
        double *dst = (ok && own) ? lpb + lpb_index(li0 + col, koff + jj, sumK) : dslot;
        *dst = sv;
        const int l0p = b_l[jb] - ((t_n[pz] - 1) > 0 ? 0 : 1);
        if (own && l0p > 0 && sv > m) m = sv;
      }
      const double lfn = cnew + hself;
      if (lfn > m) m = lfn;
      lpbig_vmax_put(vmode, ok, dm, m, mprev);
    }
    wave_lds_sync();
  }
}

// MFMA lp producer for one block of up to 16*NTB dishes of view v (dishes
// jb0 .. jb0 + kb), for views with K_v > 64 or when the tiled copy yt was not
// built (BASELINE config 5: N = 10M, D = 256, K = 256 -- y alone is 164 GB).
// Same tile and epilogue as mvc_par_lpview_kernel, with the A-fragments read
// from y itself (row-major: lane = (row, k), k-step s covers d = 4s + k, so
// the fma chain over d stays in ascending order: the same bits) or from yt,
// and the dish block's B-fragments in LDS.  A view with K_v > 16*NTB is one
// launch per dish block (y re-read per block: at D = 256, K = 256 the
// arithmetic intensity stays ~16 flop/B, above the fp64 ridge).  The first
// block writes the view maximum m_v of each customer, later blocks max it in.
//
// SPC > 0 (= A.SP = D / 4, no padded k-steps): the tile is fully unrolled, so
// every slot of the A-fragment ring is a fixed register and the loads are
// unconditional (rows past the batch read the last row; their results go to
// the discard slot), the ring runs on into the next tile (its first RA k-steps
// are issued during this tile's last ones), and the epilogue reads nothing
// from global memory but the tile's z / Y2 / previous view maximum, issued
// at the tile start: no in-order vmcnt drain per k-step chunk or per tile.
template <int NTB, int SPC>
__device__ __forceinline__ void lpbig_run(const Sweep &A, int v, int jb0, int kb, int vmode, int b0, int nb,
                                          double *lpb, double *discard, int gw, int NWT, char *smem) {
  const ParState &P = A.P;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, BW = blockDim.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n, T = A.T;
  const int SP = A.SP;                              // k-steps (padded to MVC_ZR)
  const int koff = A.Koff[v], K = A.Koff[v + 1] - koff, sumK = A.Koff[V];
  const double tau = P.hyper[v], L2pt = A.L2pt[v];
  double *Bs = (double *)smem;                      // [SP][NTB][64]
  double *wsp = Bs + (size_t)SP * NTB * 64;         // per wave: y2s[16], selfG[16], mrest[16]
  double *y2s = wsp + w * 48;
  double *selfG = y2s + 16;
  double *mrest = selfG + 16;
  double *b_c0 = wsp + BW * 48;                     // [16 NTB] the block's dish coefficients
  double *b_cb = b_c0 + 16 * NTB;
  double *b_Q = b_cb + 16 * NTB;                    // [16 NTB] ||S1||^2 of the block's dishes
  int *ip = (int *)(b_Q + 16 * NTB);
  int *b_l = ip;                                    // [16 NTB] table counts l of the block's dishes
  int *b_dn = b_l + 16 * NTB;                       // [16 NTB] member counts of the block's dishes
  int *t_dish = b_dn + 16 * NTB;                    // [T]
  int *t_n = t_dish + T;                            // [T]
  int *zs = t_n + T + w * 16;                       // per wave [16]
  for (int e = tid; e < 16 * NTB; e += blockDim.x) {
    const int jc = min(jb0 + e, K - 1);
    b_c0[e] = P.c0[v * KC + jc];
    b_cb[e] = P.cb[v * KC + jc];
    b_Q[e] = P.Q[v * KC + jc];
    b_l[e] = P.d_l[v * KC + jc];
    b_dn[e] = P.d_n[v * KC + jc];
  }
  {   // B-fragments of the dish block: Bs[(s * NTB + t) * 64 + lane] = S1[d = 4s + grp][j = jb0 + 16t + col]
    const double *S1v = P.S1T + (size_t)v * D * KC;
    for (int e = tid; e < SP * NTB * 64; e += blockDim.x) {
      const int ln = e & 63, st = e >> 6, t = st % NTB, ss = st / NTB;
      const int d = 4 * ss + (ln >> 4), j = jb0 + 16 * t + (ln & 15);
      Bs[e] = (d < D && j < jb0 + kb) ? S1v[(size_t)d * KC + j] : 0.0;
    }
  }
  for (int p = tid; p < T; p += blockDim.x) {
    t_dish[p] = P.dish[v * P.TC + p];
    t_n[p] = P.n_t[p];
  }
  __syncthreads();
  const double cnew = A.cnew[v];
  const int ntile = (nb + 15) >> 4;
  double *const dslot = discard + lane;
  const double *yv = A.y + (size_t)v * n * D;
  if constexpr (SPC > 0) {
    lpbig_tiles<NTB, SPC>(A, v, jb0, kb, vmode, b0, nb, lpb, dslot, yv, Bs, y2s, selfG, mrest, b_c0, b_cb, b_Q, b_l,
                          b_dn, t_dish, t_n, zs, gw, NWT, ntile, tau, L2pt, cnew);
    return;
  }
  for (int tile = gw; tile < ntile; tile += NWT) {
    const int li0 = tile * 16;
    const int li_row = min(li0 + col, nb - 1);
    const int pz = P.z[b0 + li_row];
    const double y2 = A.Y2[(size_t)v * n + b0 + li_row];
    const double *yrow = yv + (size_t)(b0 + li_row) * D;   // this lane's row (col), k = grp
    const bool rok = li0 + col < nb;
    mvc_d4 acc[NTB];
#pragma unroll
    for (int t = 0; t < NTB; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
    // A-fragments: 4 k-steps of loads in flight ahead of the MFMAs
    constexpr int RA = 16;
    double ar[RA];
#pragma unroll
    for (int u = 0; u < RA; ++u) {
      const int d = 4 * u + grp;
      ar[u] = (rok && d < D && u < SP) ? yrow[d] : 0.0;
    }
    // B-fragments one k-step ahead (LDS latency off the MFMA issue path)
    double bc[NTB];
#pragma unroll
    for (int t = 0; t < NTB; ++t) bc[t] = Bs[t * 64 + lane];
    for (int s0 = 0; s0 < SP; s0 += RA) {
#pragma unroll
      for (int u = 0; u < RA; ++u) {
        const int sstep = s0 + u;
        const double a = ar[u];
        const int dn = 4 * (sstep + RA) + grp;
        ar[u] = (rok && dn < D && sstep + RA < SP) ? yrow[dn] : 0.0;
        double bn[NTB];
        const double *bk = Bs + (size_t)min(sstep + 1, SP - 1) * NTB * 64 + lane;
#pragma unroll
        for (int t = 0; t < NTB; ++t) bn[t] = bk[t * 64];
#pragma unroll
        for (int t = 0; t < NTB; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bc[t], acc[t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NTB; ++t) bc[t] = bn[t];
      }
    }
    // ---- epilogue (as mvc_par_lpview_kernel, dishes jb0 + 16 t + col)
    if (grp == 0) { zs[col] = pz; y2s[col] = y2; }
    wave_lds_sync();
    double hy[4], hr[4];
    int j0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double y2r = y2s[grp + 4 * r];
      hy[r] = 0.5 * y2r;
      hr[r] = (-0.5 * y2r) / tau;
      j0[r] = t_dish[zs[grp + 4 * r]];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // G of the own dish (when in this block) -> LDS
      const int jl = j0[r] - jb0;
      double g = acc[0][r];
#pragma unroll
      for (int t = 1; t < NTB; ++t)
        if ((jl >> 4) == t) g = acc[t][r];
      if (jl >= 0 && jl < kb && col == (jl & 15)) selfG[grp + 4 * r] = g;
    }
    double mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -MVC_PM_INF;
#pragma unroll
    for (int t = 0; t < NTB; ++t) {
      const int j = jb0 + 16 * t + col;
      const double c0j = b_c0[16 * t + col], cbj = b_cb[16 * t + col];
      const bool inj = j < jb0 + kb;
      const bool inc = inj && b_l[16 * t + col] > 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double val = __builtin_fma(acc[t][r] + hy[r], cbj, c0j) + hr[r];
        const int li = li0 + grp + 4 * r;
        double *dst = (inj && li < nb) ? lpb + lpb_index(li, koff + j, sumK) : dslot;
        *dst = val;
        if (inc && j != j0[r] && val > mx[r]) mx[r] = val;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double mr = row16_max(mx[r]);
      if (col == 0) mrest[grp + 4 * r] = mr;
    }
    wave_lds_sync();
    {   // own dish (when in this block) and the view maximum, one row per lane
      const int jj = t_dish[pz];
      const bool own = jj >= jb0 && jj < jb0 + kb;
      double m = mrest[col];
      const double hself = (-0.5 * y2) / tau;
      const bool ok = lane < 16 && li0 + col < nb;
      if (own) {
        const double G = selfG[col];
        const double Gp = G - y2;
        const double Qp = (P.Q[v * KC + jj] - 2.0 * G) + y2;
        const Coef cf = coef(P.d_n[v * KC + jj] - 1, Qp, tau, L2pt, D);
        const double sv = __builtin_fma(Gp + 0.5 * y2, cf.cb, cf.c0) + hself;
        double *dst = ok ? lpb + lpb_index(li0 + col, koff + jj, sumK) : dslot;
        *dst = sv;
        const int l0p = P.d_l[v * KC + jj] - ((t_n[pz] - 1) > 0 ? 0 : 1);
        if (l0p > 0 && sv > m) m = sv;
      }
      const double lfn = cnew + hself;
      if (lfn > m) m = lfn;
      double *dm = ok ? A.vmax + (size_t)v * n + b0 + li0 + col : dslot;
      lpbig_vmax_put(vmode, ok, dm, m, vmode == 1 && ok ? *dm : m);
    }
    wave_lds_sync();
  }
}
// one dish block per launch, blocks of a view in order (vmode 0 for the first)
template <int NTB, int SPC>
__global__ __launch_bounds__(512) void mvc_par_lpbig_kernel(Sweep A, int v, int jb0, int kb, int first, int b0, int nb,
                                                            double *lpb, double *discard) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int BW = blockDim.x >> 6, w = threadIdx.x >> 6;
  lpbig_run<NTB, SPC>(A, v, jb0, kb, first ? 0 : 1, b0, nb, lpb, discard, blockIdx.x * BW + w, gridDim.x * BW, smem);
}
// Every dish block of view v in one launch (nblk blocks of 16 NTB dishes, one
// workgroup per CU): the workgroups that share an XCD (b and b + 8, dealt
// round-robin over the 8 XCDs -- for speed only, any placement is correct)
// form groups of nblk, one per dish block, and the members of a group walk the
// same customer tiles in the same order, so each y tile is fetched from HBM
// once and re-read by the group's other dish blocks from the XCD's L2 (or the
// Infinity Cache) instead of once per dish-block launch.  The view maximum is
// an atomic max into the pre-filled row (lpbig_vmax_put, vmode 2).  gridDim.x is
// a multiple of 8; workgroups beyond the last whole group per XCD, and dish
// blocks past K_v, have no work.
template <int NTB, int SPC>
__global__ __launch_bounds__(512) void mvc_par_lpbig_group_kernel(Sweep A, int v, int nblk, int b0, int nb,
                                                                  double *lpb, double *discard) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = gridDim.x >> 3, local = blockIdx.x >> 3, xs = blockIdx.x & 7;
  const int GL = L / nblk, gi = local / nblk, db = local - gi * nblk;
  const int K = A.Koff[v + 1] - A.Koff[v];
  const int jb0 = 16 * NTB * db, kb = min(16 * NTB, K - jb0);
  if (gi >= GL || kb <= 0) return;   // whole workgroup, before any barrier
  const int BW = blockDim.x >> 6, w = threadIdx.x >> 6;
  const int group = xs + 8 * gi, G = 8 * GL;
  lpbig_run<NTB, SPC>(A, v, jb0, kb, 2, b0, nb, lpb, discard, group * BW + w, G * BW, smem);
}
// vmax[v][b0 .. b0 + nb) = -inf before a grouped launch
__global__ void mvc_par_vmax_fill_kernel(double *row, int nb) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) row[i] = -MVC_PM_INF;
}
__host__ inline size_t lpbig_shared_bytes(int SP, int NTB, int T, int waves) {
  return 8 * ((size_t)SP * NTB * 64 + (size_t)waves * 48 + 48 * NTB) + 4 * (32 * NTB + 2 * (size_t)T + (size_t)waves * 16) + 64;
}

// Generic lp producer: one lane per customer (any D).
extern "C" __global__ __launch_bounds__(256) void mvc_par_lpgen_kernel(Sweep A, int b0, int nb, double *lpb) {
  const ParState &P = A.P;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n;
  const int sumK = A.Koff[V];
  for (int li = blockIdx.x * blockDim.x + threadIdx.x; li < nb; li += gridDim.x * blockDim.x) {
    const int i = b0 + li;
    const int p0 = P.z[i];
    for (int v = 0; v < V; ++v) {
      const int K = A.Koff[v + 1] - A.Koff[v], koff = A.Koff[v];
      const int j0 = P.dish[v * P.TC + p0];
      const double tau = P.hyper[v];
      const double Y2i = A.Y2[(size_t)v * n + i];
      const double hy = 0.5 * Y2i, h = (-0.5 * Y2i) / tau;
      const double *yrow = A.y + ((size_t)v * n + i) * D;
      const double *S1v = P.S1T + (size_t)v * D * KC;
      double G0 = 0.0, mx = -MVC_PM_INF;
      for (int j = 0; j < K; ++j) {
        double G = 0.0;
        for (int d = 0; d < D; ++d) G = __builtin_fma(yrow[d], S1v[(size_t)d * KC + j], G);
        if (j == j0) G0 = G;
        const double val = __builtin_fma(G + hy, P.cb[v * KC + j], P.c0[v * KC + j]) + h;
        lpb[lpb_index(li, koff + j, sumK)] = val;
        if (j != j0 && P.d_l[v * KC + j] > 0 && val > mx) mx = val;
      }
      // own dish: reduced statistics (same thread, stored after the loop)
      const double Gp = G0 - Y2i;
      const double Qp = (P.Q[v * KC + j0] - 2.0 * G0) + Y2i;
      const Coef c = coef(P.d_n[v * KC + j0] - 1, Qp, tau, A.L2pt[v], D);
      const double sv = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
      lpb[lpb_index(li, koff + j0, sumK)] = sv;
      // the view maximum of the draw (see mvc_par_lpview_kernel)
      const int l0p = P.d_l[v * KC + j0] - ((P.n_t[p0] - 1) > 0 ? 0 : 1);
      if (l0p > 0 && sv > mx) mx = sv;
      const double lfn = A.cnew[v] + h;
      if (lfn > mx) mx = lfn;
      A.vmax[(size_t)v * n + i] = mx;
    }
  }
}

// Draw kernel: one lane per customer (oracle ParallelSampler::
// resample_customer).  Per view: max and sum of w exp(lp - m) in dish order;
// tables: scores in position order, cumulative weights with a checkpoint
// every BS tables so the pick re-walks one block only.  Every uniform
// per-table / per-dish quantity is staged in LDS first (a gather whose index
// comes from global memory would pay two dependent memory round trips).
// pw16 (oracle pw16): pairwise tree over 16 values, pairs (c, c + h) for
// h = 1, 2, 4, 8; in-lane form of the 16-lane xor butterfly.
__device__ __forceinline__ double pw16(const double (&a)[16]) {
  double b[8], c[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) b[k] = a[2 * k] + a[2 * k + 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) c[k] = b[2 * k] + b[2 * k + 1];
  return (c[0] + c[1]) + (c[2] + c[3]);
}
// pw16 descent (oracle pw16_select): at a node with halves (L, R) go left iff
// R == 0 || r < L, else r -= L.
__device__ __forceinline__ int pw16_select(const double (&a)[16], double r) {
  double b[8], c[4], d[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) b[k] = a[2 * k] + a[2 * k + 1];
#pragma unroll
  for (int k = 0; k < 4; ++k) c[k] = b[2 * k] + b[2 * k + 1];
  d[0] = c[0] + c[1];
  d[1] = c[2] + c[3];
  // selects, not dynamic indexing (private arrays stay in registers)
  auto pick2 = [](const double *x, int n2, int idx, double &L, double &R) {
    L = x[0]; R = x[1];
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (k < n2 && k == idx) { L = x[2 * k]; R = x[2 * k + 1]; }
  };
  int lo = 0;
  double L, R;
  auto step = [&](int h) {
    if (!(R == 0.0 || r < L)) { r = r - L; lo += h; }
  };
  L = d[0]; R = d[1]; step(8);
  pick2(c, 2, lo >> 3, L, R); step(4);
  pick2(b, 4, lo >> 2, L, R); step(2);
  pick2(a, 8, lo >> 1, L, R); step(1);
  return lo;
}

#define MVC_ZD_NCP 16
__host__ __device__ inline size_t zdraw_shared_bytes(int V, int T, int sumK) {
  return 8 * ((size_t)MVC_ZD_NCP * 256 + (size_t)T) + 4 * ((size_t)V * T + (size_t)sumK + (size_t)V + 1) + 64;
}
// kSc: the table scores are computed once (one gather pass) into the
// coalesced scratch sc[p * nb + li] and re-read by the weight and select
// passes; without it they are re-gathered from the lp buffer in each pass.
// The view maximum m_v comes from the producer (vmax), as in the register
// draw, so each lp row is read once by the view pass.
template <bool kSc>
__global__ __launch_bounds__(256) void mvc_par_zdraw_kernel(Sweep A, int b0, int nb, const double *lpb, double *sc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int V = P.V, KC = P.KC, TC = P.TC, n = P.n;
  const int T = A.T;
  const int tid = threadIdx.x;
  double *cp_s = (double *)smem;                   // [MVC_ZD_NCP][256]
  double *s_base = cp_s + MVC_ZD_NCP * 256;        // [T] log mass (or -inf)
  int *s_tix = (int *)(s_base + T);                // [T][V] Koff[v] + dish_v(p)
  int *s_koff = s_tix + (size_t)T * V;             // [V+1]
  int *s_dl = s_koff + V + 1;                      // [sumK] l of each dish
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  if (tid <= V) s_koff[tid] = A.Koff[tid];
  __syncthreads();
  const int sumK = s_koff[V];
  for (int p = tid; p < T; p += blockDim.x) {
    const int np = P.n_t[p];
    s_base[p] = (np >= 1 && (double)np - sg > 0.0) ? P.lmass[p] : -MVC_PM_INF;
    for (int v = 0; v < V; ++v) s_tix[p * V + v] = s_koff[v] + P.dish[v * TC + p];
  }
  for (int k = tid; k < sumK; k += blockDim.x) {
    int v = 0;
    while (v + 1 < V && s_koff[v + 1] <= k) ++v;
    s_dl[k] = P.d_l[v * KC + (k - s_koff[v])];
  }
  __syncthreads();
  const int T_ne = A.status[V + 3];
  const int BS = max(16, ((T + MVC_ZD_NCP - 1) / MVC_ZD_NCP + 15) & ~15);   // multiple of 16
  const int nblk = (T + BS - 1) / BS;
  for (int li = blockIdx.x * blockDim.x + tid; li < nb; li += gridDim.x * blockDim.x) {
    const int i = b0 + li;
    const int p0 = P.z[i];
    const bool alive = (P.n_t[p0] - 1) > 0;
    const double *lpi = lpb + lpb_index(li, 0, sumK);   // dish k at lpi[k * 16]
    double s_new = mvc_log(ag + sg * (double)(T_ne - (alive ? 0 : 1)));
    for (int v = 0; v < V; ++v) {
      const int koff = s_koff[v], K = s_koff[v + 1] - koff;
      const int j0 = s_tix[p0 * V + v] - koff;
      const double alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
      const double lfn = A.cnew[v] + (-0.5 * A.Y2[(size_t)v * n + i]) / P.hyper[v];
      const int l0p = s_dl[koff + j0] - (alive ? 0 : 1);
      const int *dl = s_dl + koff;
      const double *lpv = lpi + (size_t)koff * 16;
      // m_v: the max over the included dishes and the new dish, from the producer
      const double m = A.vmax[(size_t)v * n + i];
      // 16 column partials (dish j -> column j & 15, ascending j), then pw16
      double col[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) col[c] = 0.0;
      for (int j = 0; j < K; j += 16) {
        double x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = lpv[(size_t)min(j + u, K - 1) * 16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int l = (j + u == j0) ? l0p : dl[min(j + u, K - 1)];
          double w = (double)l - sigma;
          if (w < 0.0) w = 0.0;
          const bool in = j + u < K && l > 0;
          const double t = w * mvc_exp(in ? x[u] - m : 0.0);
          if (in) col[u] = col[u] + t;
        }
      }
      double S = pw16(col);
      const int Kact = K - ((l0p == 0) ? 1 : 0);
      double wn = alpha + (double)Kact * sigma;
      if (wn < 0.0) wn = 0.0;
      S = S + wn * mvc_exp(lfn - m);
      const double denom = alpha + (double)(P.Ltot[v] - (alive ? 0 : 1));
      const double lm = (denom <= 0.0) ? lfn : (m + mvc_log(S)) - mvc_log(denom);
      s_new = s_new + lm;
    }
    // own table's base score with the customer removed
    const int np0 = P.n_t[p0] - 1;
    const double m0 = (double)np0 - sg;
    const double base_self = (np0 >= 1 && m0 > 0.0) ? mvc_log(m0) : -MVC_PM_INF;
    // scores of tables p .. p+3 (clamped); view-order sums, 4 V gathers in flight
    auto score4 = [&](int p, double (&sp)[4]) {
      int pc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        pc[u] = min(p + u, T - 1);
        sp[u] = (pc[u] == p0) ? base_self : s_base[pc[u]];
      }
      for (int v = 0; v < V; ++v) {
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = lpi[(size_t)s_tix[pc[u] * V + v] * 16];
#pragma unroll
        for (int u = 0; u < 4; ++u) sp[u] = sp[u] + x[u];
      }
    };
    double M = -MVC_PM_INF;
    double *scl = sc + li;   // kSc: table p's score at scl[p * nb]
    for (int p = 0; p < T; p += 4) {
      double sp[4];
      score4(p, sp);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (p + u < T) {
          if (sp[u] > M) M = sp[u];
          if constexpr (kSc) scl[(size_t)(p + u) * nb] = sp[u];
        }
    }
    if (s_new > M) M = s_new;
    // weights in blocks of 16 positions: block sums pw16, running totals
    // C_b = C_{b-1} + B_b; a checkpoint (C before the segment) every BS tables
    auto block_e = [&](int b, double (&e)[16]) {
#pragma unroll
      for (int q = 0; q < 16; q += 4) {
        double sp[4];
        if constexpr (kSc) {
#pragma unroll
          for (int u = 0; u < 4; ++u) sp[u] = scl[(size_t)min(16 * b + q + u, T - 1) * nb];
        } else {
          score4(16 * b + q, sp);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool in = 16 * b + q + u < T && sp[u] != -MVC_PM_INF;
          const double x = mvc_exp(in ? sp[u] - M : 0.0);
          e[q + u] = in ? x : 0.0;
        }
      }
    };
    const int TB = (T + 15) >> 4, BSB = BS >> 4;   // blocks, blocks per segment
    double tot = 0.0;
    for (int b = 0; b < TB; ++b) {
      if (b % BSB == 0) cp_s[(b / BSB) * 256 + tid] = tot;
      double e[16];
      block_e(b, e);
      tot = tot + pw16(e);
    }
    const double W = mvc_exp(s_new - M) + tot;
    double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
    int pick = -1;
    if (r < tot) {
      int g = 0;
      while (g + 1 < nblk && !(r < cp_s[(g + 1) * 256 + tid])) ++g;
      double c = cp_s[g * 256 + tid];
      for (int b = g * BSB; b < TB; ++b) {
        double e[16];
        block_e(b, e);
        const double cn = c + pw16(e);
        if (r < cn) {
          pick = 16 * b + pw16_select(e, r - c);
          break;
        }
        c = cn;
      }
    }
    A.choice[i] = pick;
  }
}

// Register-resident draw for T <= TM tables and K_v <= 64 dishes (the common
// case): same arithmetic, same order as mvc_par_zdraw_kernel, but each view's
// lp row is loaded once into registers (the max and the sum both read them)
// and the table scores live in registers, so the table phase is ONE gather
// pass (V loads per table) instead of 2.25; the running cumulative weights
// overwrite the scores and the pick is the first p with r < cum_p.  An
// excluded table adds +0.0, which leaves the running sum bit-identical.
// One customer's lp row in the lp buffer: dish k's value at a uniform base
// (lpb + 16 k, scalar registers) plus the customer's 32-bit byte offset, so
// every gather is a saddr load with no per-lane address arithmetic.
typedef int mvc_i4 __attribute__((ext_vector_type(4)));
extern "C" __device__ double mvc_raw_buffer_load_f64(mvc_i4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.f64");
struct LpRow {
  mvc_i4 rsrc;       // buffer resource over the lp buffer (scalar registers)
  int boff;          // this customer's byte offset in its slab (< 2^31: kLpbBudget)
  __device__ __forceinline__ LpRow(const double *lpb, int boff_) : boff(boff_) {
    const uint64_t a = (uint64_t)lpb;
    rsrc = (mvc_i4){(int)(uint32_t)a, (int)(uint32_t)(a >> 32), -1, 0x00020000};   // raw, no range limit
  }
  // k must be wave-uniform (it becomes the SGPR soffset)
  __device__ __forceinline__ double operator()(int k) const { return mvc_raw_buffer_load_f64(rsrc, boff, k * 128, 0); }
  // k per lane
  __device__ __forceinline__ double at(int k) const { return mvc_raw_buffer_load_f64(rsrc, boff + k * 128, 0, 0); }
};

// View reduction of the draw (oracle eval_view_seq): the sum of
// w_j exp(lp_j - m) as 16 column partials (dish j -> column j & 15, ascending
// j) folded by pw16; m (the max over included dishes and the new dish) comes
// from the producer (vmax), so every row is read once.  w_j = max(l_j - sigma,
// 0) for l_j > 0 and -1 (excluded) otherwise: uniform per dish (s_w, staged
// once per block) except the customer's own dish (w0).  KB > 0: row loaded
// into registers at once; KB == 0: streamed in batches of 16.
#ifndef MVC_ZEXP_LAG
#define MVC_ZEXP_LAG 1   // exps in flight per lane in the register draw (register pressure vs ILP)
#endif
template <int KB>
__device__ __forceinline__ double zview_sum(const LpRow &row, int koff, int K, int j0, double w0, const double *sw,
                                            double m, double *stg = nullptr) {
  double col[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) col[c] = 0.0;
  // an excluded dish (w = -1) adds +0; its argument is clamped at 0 (its lp
  // may exceed m, which is over the included dishes, and exp would overflow:
  // 0 * inf); an included dish has lp <= m, so the clamp changes nothing there
  if constexpr (KB > 0) {
    double x[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) x[j] = row(koff + min(j, K - 1));
    if (stg) {                                     // wave-uniform: keep the row in LDS for the table gathers
#pragma unroll
      for (int j = 0; j < KB; ++j)
        if (j < K) stg[j * 64] = x[j];
    }
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      if (j < K) {
        const double w = (j == j0) ? w0 : sw[j];
        double xe = __builtin_fmin(x[j] - m, 0.0);
        asm volatile("" : "+v"(xe) : "v"(col[(j + 16 - MVC_ZEXP_LAG) & 15]));    // MVC_ZEXP_LAG exps in flight (register pressure)
        col[j & 15] = col[j & 15] + __builtin_fmax(w, 0.0) * mvc_exp_le0(xe);   // dead dish (w = -1): + 0, exact
      }
    }
  } else {
    int j = 0;
    for (; j + 16 <= K; j += 16) {
      double x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = row(koff + j + u);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const double w = (j + u == j0) ? w0 : sw[j + u];
        double xe = __builtin_fmin(x[u] - m, 0.0);
        asm volatile("" : "+v"(xe) : "v"(col[(u + 16 - MVC_ZEXP_LAG) & 15]));
        col[u] = col[u] + __builtin_fmax(w, 0.0) * mvc_exp_le0(xe);
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (j + u < K) {
        const double w = (j + u == j0) ? w0 : sw[j + u];
        col[u] = col[u] + __builtin_fmax(w, 0.0) * mvc_exp_le0(__builtin_fmin(row(koff + j + u) - m, 0.0));
      }
    }
  }
  return pw16(col);
}

#define MVC_ZSTAGE 24          // dishes per wave whose lp rows the register draw keeps in LDS (3 blocks/CU)

// The register draw's block-shared tables (LDS).
struct ZregLds {
  const double *base;    // [TM] log mass of each table (or -inf: excluded)
  const double *w;       // [sumK] dish weights max(l - sigma, 0), -1 for l = 0
  const int *tix;        // [TM][V] Koff[v] + dish_v(p)
  const int *koff;       // [V+1]
  const int *lmin;       // [VMAX] 1: every dish of view v has l >= 1
  const int *soff;       // [VMAX] staging offset of view v (dishes), -1: not staged
  const int *dl;         // [sumK] l of each dish
};

// One customer of the register draw (one lane): the view terms (each lp row
// read once; rows of K_v <= 16 in registers, staged rows kept in LDS for the
// gathers), the table scores in view order, weights, block totals and the
// pw16 descent.  Returns the choice (table position, -1 = birth).
template <int TM>
__device__ __forceinline__ int zdraw_reg_one(const Sweep &A, const ZregLds &Z, int i, const LpRow &row, double *s_stage,
                                             int lane) {
  const ParState &P = A.P;
  const int V = P.V, n = P.n;
  const int T = __builtin_amdgcn_readfirstlane(A.T);
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int T_ne = A.status[V + 3];
  // view v's maximum and Y2 are loaded one view ahead (with z and the first
  // view's row), not at the top of each view's iteration
  double m_nx = A.vmax[i], y2_nx = A.Y2[i];
  const int p0 = P.z[i];
  const bool alive = (P.n_t[p0] - 1) > 0;
  double s_new = mvc_log(ag + sg * (double)(T_ne - (alive ? 0 : 1)));
  for (int v = 0; v < V; ++v) {
    const double m = m_nx, y2v = y2_nx;
    {
      const size_t vn = (size_t)min(v + 1, V - 1) * n + i;
      m_nx = A.vmax[vn];
      y2_nx = A.Y2[vn];
    }
    const int koff = __builtin_amdgcn_readfirstlane(Z.koff[v]);
    const int K = __builtin_amdgcn_readfirstlane(Z.koff[v + 1]) - koff;
    const int j0 = Z.tix[p0 * V + v] - koff;
    const double sigma = P.hyper[2 * V + v];
    const double lfn = A.cnew[v] + (-0.5 * y2v) / P.hyper[v];
    const int l0p = Z.dl[koff + j0] - (alive ? 0 : 1);
    double w0 = (double)l0p - sigma;
    if (w0 < 0.0) w0 = 0.0;
    if (!(l0p > 0)) w0 = -1.0;
    const double *sw = Z.w + koff;
    double S;
    const bool allv = __builtin_amdgcn_readfirstlane(Z.lmin[v]) != 0;
    const int so = __builtin_amdgcn_readfirstlane(Z.soff[v]);
    double *stg = so >= 0 ? s_stage + (size_t)so * 64 + lane : nullptr;
    if (!allv) S = zview_sum<0>(row, koff, K, j0, w0, sw, m);           // general: streamed
    else if (K <= 8) S = zview_sum<8>(row, koff, K, j0, w0, sw, m, stg);     // row in registers
    else if (K <= 16) S = zview_sum<16>(row, koff, K, j0, w0, sw, m, stg);
    else S = zview_sum<0>(row, koff, K, j0, w0, sw, m);
    const int Kact = K - ((l0p == 0) ? 1 : 0);
    double wn = P.hyper[V + v] + (double)Kact * sigma;
    if (wn < 0.0) wn = 0.0;
    S = S + wn * mvc_exp_le0(lfn - m);
    const double denom = P.hyper[V + v] + (double)(P.Ltot[v] - (alive ? 0 : 1));
    const double lm = (denom <= 0.0) ? lfn : (m + mvc_log(S)) - mvc_log(denom);
    s_new = s_new + lm;
  }
  const int np0 = P.n_t[p0] - 1;
  const double m0 = (double)np0 - sg;
  const double base_self = (np0 >= 1 && m0 > 0.0) ? mvc_log(m0) : -MVC_PM_INF;
  // table scores in view order, 16 tables' gathers in flight per step
  double sp[TM];
#pragma unroll
  for (int p = 0; p < TM; ++p) {   // p >= T: -inf, so its weight below is exp(-inf) = 0 like a dead table's
    const int pc = min(p, T - 1);
    sp[p] = p < T ? ((pc == p0) ? base_self : Z.base[pc]) : -MVC_PM_INF;
  }
#pragma unroll
  for (int c = 0; c < TM; c += 16) {
    for (int v = 0; v < V; ++v) {
      double x[16];
      const int so = __builtin_amdgcn_readfirstlane(Z.soff[v]);
      if (so >= 0) {                             // staged row: LDS [dish][lane], conflict-free
        const double *st = s_stage + (size_t)(so - Z.koff[v]) * 64 + lane;
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = st[(size_t)__builtin_amdgcn_readfirstlane(Z.tix[min(c + u, T - 1) * V + v]) * 64];
      } else {
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = row(__builtin_amdgcn_readfirstlane(Z.tix[min(c + u, T - 1) * V + v]));
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) sp[c + u] = sp[c + u] + x[u];
    }
  }
  double M = -MVC_PM_INF;
#pragma unroll
  for (int p = 0; p < TM; ++p)
    if (p < T && sp[p] > M) M = sp[p];
  if (s_new > M) M = s_new;
  // weights e_p in place; block sums pw16, running block totals C_b
  double C[TM / 16];
  double tot = 0.0;
#pragma unroll
  for (int b = 0; b < TM / 16; ++b) {
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int p = 16 * b + c;
      // a dead table or p >= T has sp = -inf: exp_le0(-inf) = +0, the spec's 0 weight
      double xe = sp[p] - M;
      asm volatile("" : "+v"(xe) : "v"(sp[(p + TM - MVC_ZEXP_LAG) % TM]));   // MVC_ZEXP_LAG exps in flight, not TM live
      sp[p] = mvc_exp_le0(xe);
    }
    double blk[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) blk[c] = sp[16 * b + c];
    tot = tot + pw16(blk);
    C[b] = tot;
  }
  const double W = mvc_exp_le0(s_new - M) + tot;
  double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
  int pick = -1;
  if (r < tot) {
    int bsel = TM / 16 - 1;
    double prev = 0.0;
#pragma unroll
    for (int b = TM / 16 - 1; b >= 0; --b)
      if (r < C[b]) { bsel = b; prev = b > 0 ? C[b - 1] : 0.0; }
    r = r - prev;
    double blk[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      double x = sp[c];
#pragma unroll
      for (int b = 1; b < TM / 16; ++b)
        if (bsel == b) x = sp[16 * b + c];
      blk[c] = x;
    }
    pick = 16 * bsel + pw16_select(blk, r);
  }
  return pick;
}

template <int TM>
#ifndef MVC_ZDRAW_MINB
#define MVC_ZDRAW_MINB 3      // blocks of 4 waves per CU the register budget must allow
#endif
__global__ __launch_bounds__(256, MVC_ZDRAW_MINB) void mvc_par_zdraw_reg_kernel(Sweep A, int b0, int nb, const double *lpb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int V = P.V, KC = P.KC, TC = P.TC;
  const int T = __builtin_amdgcn_readfirstlane(A.T);
  const int tid = threadIdx.x;
  const int sumK0 = __builtin_amdgcn_readfirstlane(A.Koff[V]);
  double *s_base = (double *)smem;                 // [TM] log mass (or -inf)
  double *s_w = s_base + TM;                       // [sumK] dish weights max(l - sigma, 0) / -1
  double *s_stage = s_w + sumK0;                   // [4 waves][MVC_ZSTAGE][64] staged lp rows
  int *s_tix = (int *)(s_stage + 4 * MVC_ZSTAGE * 64);   // [TM][V] Koff[v] + dish_v(p)
  int *s_koff = s_tix + (size_t)TM * V;            // [V+1]
  int *s_lmin = s_koff + V + 1;                    // [VMAX] 1: every dish of view v has l >= 1
  int *s_soff = s_lmin + MVC_Z_VMAX;               // [VMAX] staging offset of view v (dishes), -1: not staged
  int *s_dl = s_soff + MVC_Z_VMAX;                 // [sumK] l of each dish
  s_stage += (size_t)(threadIdx.x >> 6) * MVC_ZSTAGE * 64;
  const double sg = P.hyper[3 * V + 1];
  if (tid <= V) s_koff[tid] = A.Koff[tid];
  __syncthreads();
  const int sumK = s_koff[V];
  for (int p = tid; p < T; p += blockDim.x) {
    const int np = P.n_t[p];
    s_base[p] = (np >= 1 && (double)np - sg > 0.0) ? P.lmass[p] : -MVC_PM_INF;
    for (int v = 0; v < V; ++v) s_tix[p * V + v] = s_koff[v] + P.dish[v * TC + p];
  }
  if (tid < MVC_Z_VMAX) s_lmin[tid] = 1;
  __syncthreads();
  for (int k = tid; k < sumK; k += blockDim.x) {
    int v = 0;
    while (v + 1 < V && s_koff[v + 1] <= k) ++v;
    const int l = P.d_l[v * KC + (k - s_koff[v])];
    double w = (double)l - P.hyper[2 * V + v];
    if (w < 0.0) w = 0.0;
    s_dl[k] = l;
    s_w[k] = l > 0 ? w : -1.0;
    if (l < 1) s_lmin[v] = 0;                    // benign race: every writer stores 0
  }
  __syncthreads();
  if (tid == 0) {   // views whose rows the draw holds in registers (K <= 16) also go to LDS, budget permitting
    int tot = 0;
    for (int v = 0; v < V; ++v) {
      const int K = s_koff[v + 1] - s_koff[v];
      const bool st = s_lmin[v] != 0 && K <= 16 && tot + K <= MVC_ZSTAGE;
      s_soff[v] = st ? tot : -1;
      tot += st ? K : 0;
    }
  }
  __syncthreads();
  const ZregLds Z{s_base, s_w, s_tix, s_koff, s_lmin, s_soff, s_dl};
  const int li = blockIdx.x * blockDim.x + tid;   // one customer per thread (no loop-invariant hoisting)
  if (li >= nb) return;
  const LpRow row(lpb, (int)(lpb_index(li, 0, sumK) * 8));
  const int pick = zdraw_reg_one<TM>(A, Z, b0 + li, row, s_stage, tid & 63);
  A.choice[b0 + li] = pick;
  if (A.fmin) {   // the wave's first customer whose choice is not its table (a wave's customers are consecutive)
    const uint64_t mv = __ballot(pick != P.z[b0 + li]);
    if (mv && (tid & 63) == (int)__ffsll((long long)mv) - 1) atomicMin(A.fmin, b0 + li);
  }
}
__host__ __device__ inline size_t zdraw_reg_shared_bytes(int V, int TM, int sumK) {
  return 8 * ((size_t)TM + (size_t)sumK + (size_t)4 * MVC_ZSTAGE * 64) +
         4 * ((size_t)V * TM + (size_t)V + 1 + 2 * MVC_Z_VMAX + (size_t)sumK) + 16;
}

// Row draw for T > 64 tables (or K_v > 64 dishes): one 16-lane DPP row per
// customer, four customers per wavefront, a block (16 rows) on one 16-customer
// slab of the lp buffer at a time.  The same arithmetic in the same order as
// mvc_par_zdraw_kernel / the register draw (oracle resample_customer):
//   * view terms: lane c of the row owns column c (dishes j = 16 t + c), its
//     partial is the sequential sum over ascending t, and the row's DPP tree
//     (row_pw16) is the spec's pw16 over the 16 columns;
//   * table scores: lane c owns positions p = 16 k + c (k < NB), each a
//     view-order sum; block k of 16 positions is register k of the row, so
//     B_k = row_pw16(e_k), and the running block totals C_k are formed in
//     block order in every lane;
//   * the pick: the first block with r < C_k, then the pw16 descent over that
//     block's 16 leaves (staged in LDS).
// One lane-per-customer kernel would gather V*T values per customer through
// every lane; here each lane gathers V*T/16 and the row's values share cache
// lines (the slab layout interleaves the 16 customers of a block).
#ifndef MVC_ZROW_MINB
#define MVC_ZROW_MINB 4       // blocks of 4 waves per CU the row draw's register budget must allow
#endif
__device__ __forceinline__ int lane_row_base(int row) { return 16 * (row & 3); }   // first lane of a row in its wave
// One customer's lp row for the row draw: in the lp buffer (buffer loads,
// per-lane dish index) or in the block's LDS copy of its 16-customer slab.
struct LdsRow {
  const double *p;     // the slab in LDS, this customer's column: dish k at p[16 k]
  __device__ __forceinline__ double at(int k) const { return p[16 * k]; }
};

// the row draw's exp: Horner coefficients in VGPRs where the register
// budget allows (the LDS form, two waves per SIMD), else in SGPRs
template <bool kV>
__device__ __forceinline__ double zexp(double x) { return kV ? mvc_exp_le0(x) : mvc_exp_le0_sk(x); }

template <int NB, bool kLds>
__global__ __launch_bounds__(256, (NB >= 32 || kLds) ? 2 : MVC_ZROW_MINB) void mvc_par_zdraw_row_kernel(Sweep A, int b0, int nb,
                                                                                            const double *lpb) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int V = P.V, KC = P.KC, TC = P.TC, n = P.n;
  const int T = __builtin_amdgcn_readfirstlane(A.T);
  const int tid = threadIdx.x, row = tid >> 4, c = tid & 15;
  const int sumK0 = __builtin_amdgcn_readfirstlane(A.Koff[V]);
  double *s_slab = (double *)smem;                 // kLds: [sumK][16] the block's slab of the lp buffer
  double *s_base = s_slab + (kLds ? (size_t)16 * sumK0 : 0);   // [16 NB] log mass (or -inf: excluded / padding)
  double *s_sel = s_base + 16 * NB;                // [16 rows][16] the picked block's leaves
  int *s_tix = (int *)(s_sel + 256);               // [16 NB][V] Koff[v] + dish_v(p) (padding: Koff[v])
  int *s_koff = s_tix + 16 * NB * V;               // [V+1]
  int *s_dl = s_koff + V + 1;                      // [sumK] l of each dish
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  if (tid <= V) s_koff[tid] = A.Koff[tid];
  __syncthreads();
  const int sumK = s_koff[V];
  for (int p = tid; p < 16 * NB; p += blockDim.x) {
    const int np = p < T ? P.n_t[p] : 0;
    s_base[p] = (p < T && np >= 1 && (double)np - sg > 0.0) ? P.lmass[p] : -MVC_PM_INF;
    for (int v = 0; v < V; ++v) s_tix[p * V + v] = s_koff[v] + (p < T ? P.dish[v * TC + p] : 0);
  }
  for (int k = tid; k < sumK; k += blockDim.x) {
    int v = 0;
    while (v + 1 < V && s_koff[v + 1] <= k) ++v;
    s_dl[k] = P.d_l[v * KC + (k - s_koff[v])];
  }
  __syncthreads();
  const int T_ne = A.status[V + 3];
  double *sel = s_sel + row * 16;
  for (int g = blockIdx.x; g * 16 < nb; g += gridDim.x) {
    const int li = g * 16 + row;
    const bool ok = li < nb;
    const int lic = min(li, nb - 1);
    const int i = b0 + lic;
    // this customer's per-view scalars, lane c of the row holding view c,
    // loaded together ahead of the slab (one memory latency per round instead
    // of one per view)
    const int vq = min(c, V - 1);
    const int p0 = P.z[i];
    const double m_lane = A.vmax[(size_t)vq * n + i];
    const double y2_lane = A.Y2[(size_t)vq * n + i];
    if constexpr (kLds) {   // the slab (16 customers x sumK dishes, contiguous) into LDS, 8 loads in flight
      const mvc_d2 *src = (const mvc_d2 *)(lpb + (size_t)g * sumK * 16);
      mvc_d2 *dst = (mvc_d2 *)s_slab;
      const int ne = sumK * 8;
      for (int e0 = 0; e0 < ne; e0 += 8 * 256) {
        mvc_d2 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = src[min(e0 + u * 256 + tid, ne - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (e0 + u * 256 + tid < ne) dst[e0 + u * 256 + tid] = q[u];
      }
      __syncthreads();
    }
    const auto lp = [&] {
      if constexpr (kLds) return LdsRow{s_slab + lpb_slot(row)};
      else return LpRow(lpb, (int)(lpb_index(lic, 0, sumK) * 8));   // dish k of this customer: lp.at(k)
    }();
    const bool alive = (P.n_t[p0] - 1) > 0;
    double Smine = 0.0;                            // lane v of the row keeps view v's column sum
    for (int v = 0; v < V; ++v) {
      const int koff = s_koff[v], K = s_koff[v + 1] - koff;
      const int j0 = s_tix[p0 * V + v] - koff;
      const double sigma = P.hyper[2 * V + v];
      const int l0p = s_dl[koff + j0] - (alive ? 0 : 1);
      const double m = __shfl(m_lane, lane_row_base(row) + v, 64);
      // column c: included dishes j = 16 t + c in ascending t (an excluded
      // dish adds +0: its weight and argument are zeroed); the loads of 8
      // t at a time are issued before their exps
      double col = 0.0;
      for (int t0 = 0; 16 * t0 < K; t0 += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = lp.at(koff + min(16 * (t0 + u) + c, K - 1));
        const int tn = (K - 16 * t0 + 15) >> 4;   // dish blocks of this chunk with any dish (uniform)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (u >= tn) break;                     // (a block past K_v would add +0 in every lane)
          const int j = 16 * (t0 + u) + c;
          const int l = (j == j0) ? l0p : s_dl[koff + min(j, K - 1)];
          double w = (double)l - sigma;                 // w_j = max(l - sigma, 0), included iff l > 0
          if (w < 0.0) w = 0.0;
          const bool in = j < K && l > 0;
          double xe = in ? x[u] - m : 0.0;
          if constexpr (!kLds) asm volatile("" : "+v"(xe) : "v"(col));   // one exp in flight (4 waves per SIMD)
          col = col + (in ? w : 0.0) * zexp<kLds>(xe);
        }
      }
      const double S = row_pw16(col);
      if (c == v) Smine = S;
    }
    // the per-view scalar terms, lane v of the row for view v (one wave
    // instruction stream for all views instead of V), then the view-order sum
    double lm = 0.0;
    {
      const int v = min(c, V - 1);
      const int koff = s_koff[v], K = s_koff[v + 1] - koff;
      const int j0 = s_tix[p0 * V + v] - koff;
      const double alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
      const double lfn = A.cnew[v] + (-0.5 * y2_lane) / P.hyper[v];
      const int l0p = s_dl[koff + j0] - (alive ? 0 : 1);
      const double m = m_lane;
      const int Kact = K - ((l0p == 0) ? 1 : 0);
      double wn = alpha + (double)Kact * sigma;
      if (wn < 0.0) wn = 0.0;
      const double S = Smine + wn * zexp<kLds>(lfn - m);
      const double denom = alpha + (double)(P.Ltot[v] - (alive ? 0 : 1));
      lm = (denom <= 0.0) ? lfn : (m + mvc_log_nb(S)) - mvc_log_nb(denom);
    }
    double s_new = mvc_log_nb(ag + sg * (double)(T_ne - (alive ? 0 : 1)));
    for (int v = 0; v < V; ++v) s_new = s_new + __shfl(lm, lane_row_base(row) + v, 64);
    // table scores of positions 16 k + c, view order
    const int np0 = P.n_t[p0] - 1;
    const double m0 = (double)np0 - sg;
    const double base_self = (np0 >= 1 && m0 > 0.0) ? mvc_log_nb(m0) : -MVC_PM_INF;
    double sp[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int p = 16 * k + c;
      sp[k] = (p == p0) ? base_self : s_base[p];
    }
    for (int v = 0; v < V; ++v) {
      double x[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) x[k] = lp.at(s_tix[(16 * k + c) * V + v]);
#pragma unroll
      for (int k = 0; k < NB; ++k) sp[k] = sp[k] + x[k];
    }
    double M = -MVC_PM_INF;
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (16 * k + c < T && sp[k] > M) M = sp[k];
    M = row16_max(M);
    if (s_new > M) M = s_new;
    // weights in place, block sums, running block totals C_k (block order,
    // formed in every lane of the row; lane k keeps C_k)
    constexpr int NG = (NB + 15) / 16;             // lane c keeps C_k of blocks k = c + 16 g
    double tot = 0.0, Cm[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) Cm[g] = 0.0;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      sp[k] = (16 * k + c < T) ? zexp<kLds>(sp[k] - M) : 0.0;   // excluded: exp(-inf) = +0
      tot = tot + row_pw16(sp[k]);
      if (c == (k & 15)) Cm[k >> 4] = tot;
    }
    const double W = zexp<kLds>(s_new - M) + tot;
    double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
    // the first block k with r < C_k: the lowest such lane of the row, group by group
    int kb = NB - 1;
#pragma unroll
    for (int g = NG - 1; g >= 0; --g) {
      const uint64_t hit = __ballot(16 * g + c < NB && r < Cm[g]);
      const uint64_t mine = (hit >> lane_row_base(row)) & 0xFFFFull;
      if (mine) kb = 16 * g + __builtin_ctzll(mine);
    }
    // C_{kb-1} from its lane (the whole wave takes part in the shuffle)
    const int kp = max(kb - 1, 0);
    double cv = Cm[0];
#pragma unroll
    for (int g = 1; g < NG; ++g)
      if ((kp >> 4) == g) cv = Cm[g];
    const double cprev = __shfl(cv, lane_row_base(row) + (kp & 15), 64);
    const double prev = kb > 0 ? cprev : 0.0;
    double leaf = sp[0];
#pragma unroll
    for (int k = 1; k < NB; ++k)
      if (kb == k) leaf = sp[k];
    sel[c] = leaf;                                  // the block's leaves (LDS)
    wave_lds_sync();
    int pick = -1;
    if (r < tot) {
      double a[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) a[u] = sel[u];
      pick = 16 * kb + pw16_select(a, r - prev);
    }
    if (ok && c == 0) A.choice[i] = pick;
    if constexpr (kLds) __syncthreads();           // the slab is rewritten next round
    else wave_lds_sync();
  }
}
__host__ __device__ inline size_t zdraw_row_shared_bytes(int V, int NB, int sumK, bool lds) {
  return 8 * ((size_t)16 * NB + 256 + (lds ? (size_t)16 * sumK : 0)) +
         4 * ((size_t)16 * NB * V + (size_t)V + 1 + (size_t)sumK) + 16;
}

// ---------------------------------------------------------------------------
// View patterns (compile-time per-view dish-block counts) of the all-views
// producer below: bits 0-3 = V, bits 4 + 2 v .. = NT_v - 1 (dish blocks of 16
// in view v).  Views run in order, unrolled at compile time, so a tile is
// straight-line code (no joins between views with different NT, which cost
// the register allocator ~60 VGPRs).  Instances: the bench's K_v = 64, 32,
// 16, 8 and configs[1]'s 16, 8 shapes, every view count <= 4 with a common
// dish-block count of 1 or 2, and up to two views of 4 blocks.
// ---------------------------------------------------------------------------
#define MVC_FZ_TB 4               // table blocks of 16 (T <= 64)
#define MVC_FZ_PAT(V, n0, n1, n2, n3) ((V) | (((n0) - 1) << 4) | (((n1) - 1) << 6) | (((n2) - 1) << 8) | (((n3) - 1) << 10))
#define MVC_FZ_PATS(X)                                                                                     \
  X(MVC_FZ_PAT(4, 4, 2, 1, 1)) X(MVC_FZ_PAT(3, 4, 2, 1, 1)) X(MVC_FZ_PAT(2, 4, 2, 1, 1))                  \
  X(MVC_FZ_PAT(2, 2, 1, 1, 1)) X(MVC_FZ_PAT(1, 1, 1, 1, 1)) X(MVC_FZ_PAT(2, 1, 1, 1, 1))                  \
  X(MVC_FZ_PAT(3, 1, 1, 1, 1)) X(MVC_FZ_PAT(4, 1, 1, 1, 1)) X(MVC_FZ_PAT(1, 2, 2, 2, 2))                  \
  X(MVC_FZ_PAT(2, 2, 2, 2, 2)) X(MVC_FZ_PAT(3, 2, 2, 2, 2)) X(MVC_FZ_PAT(4, 2, 2, 2, 2))                  \
  X(MVC_FZ_PAT(1, 4, 4, 4, 4)) X(MVC_FZ_PAT(2, 4, 4, 4, 4)) X(MVC_FZ_PAT(3, 2, 1, 1, 1))
__host__ __device__ constexpr int fz_pat_v(uint32_t pat) { return (int)(pat & 15u); }
__host__ __device__ constexpr int fz_pat_nt(uint32_t pat, int v) { return (int)((pat >> (4 + 2 * v)) & 3u) + 1; }


// ---------------------------------------------------------------------------
// All-views lp producer: the per-view producers' work in ONE launch.  Every
// view's S1 B-fragments sit in LDS (one block per CU); each wave takes a
// 16-customer tile through all views in order (view pattern PAT fixed at
// compile time, see MVC_FZ_PATS), so MFMA-heavy views (K_v = 64) and
// stream-heavy ones (K_v <= 16) alternate inside each wave and the two waves
// of a SIMD overlap them; one launch instead of V removes V - 1 prologues and
// tails.  Same outputs and arithmetic as mvc_par_lpview_kernel (lp rows and
// the view maxima vmax).
// ---------------------------------------------------------------------------
struct LpaLds {
  const double *Bs, *c0, *cb, *Q;
  const double *xs, *dens, *cbs;   // per dish: the own-dish coefficient parts (see lpall_self_coef)
  const int *dn, *dl, *tix, *nt, *koff, *boff;
};
// Per-wave LDS of the all-views producer: the tile's y2 and h = (-y2/2)/tau
// per (view, row), the own-dish G and the max over the other included dishes
// per (view, row) [4][16] each, and the rows' tables [16].
constexpr int kLpaWaveD = 4 * 4 * 16;   // doubles
constexpr int kLpaWaveI = 16;           // ints
__host__ __device__ inline size_t lpall_shared_bytes(size_t s1t_doubles, int V, int sumK, int waves) {
  return 16 * 4 + 8 * (s1t_doubles + 6 * (size_t)sumK + (size_t)waves * kLpaWaveD) +
         4 * (2 * (size_t)sumK + (size_t)MVC_FZ_TB * 16 * V + MVC_FZ_TB * 16 + (size_t)waves * kLpaWaveI) + 64;
}

// The own-dish coefficient of coef(n - 1, Q', tau, L2pt, D) split into its
// parts that do not depend on the customer: c0 = X - (0.5 Q') / den with
// X = D ((-0.5 L2pt) - 0.5 log(b / a)), den = (tau a) b, and cb = 1 / (tau b),
// a = tau + (n - 1), b = tau + n (the same operations as coef, so the same
// bits), staged once per block instead of one log and three divisions per
// customer and view.
__device__ __forceinline__ void lpall_self_coef(int dn, double tau, double L2pt, int D, double &X, double &den,
                                                double &cb) {
  const int n_ = dn - 1;
  const double a = tau + (double)n_;
  const double b = tau + (double)(n_ + 1);
  X = (double)D * ((-0.5 * L2pt) - 0.5 * mvc_log(b / a));
  den = (tau * a) * b;
  cb = 1.0 / (tau * b);
}

extern "C" __device__ void mvc_raw_buffer_store_f64(double v, mvc_i4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.f64");
extern "C" __device__ void mvc_raw_buffer_store_v2f64(mvc_d2 v, mvc_i4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v2f64");

// One view of one 16-customer tile: the MFMA block, then the lp of every
// (row, frozen dish) stored (buffer stores: a 32-bit lane offset, invalid
// lanes to their discard slot), the own dish's G and the max over the other
// included dishes per row to LDS; the own dish itself is done for all views
// at once at the end of the tile (lpa_tile_end).
template <int NT, int SPPT, int RP>
__device__ __forceinline__ void lpa_view(const Sweep &A, const LpaLds &L, int v, int li0, int nb, const mvc_d2 *cur,
                                         const mvc_d2 *nxt, mvc_d2 (&ring)[RP], mvc_i4 rsrc, int tile_boff,
                                         int disc_boff, double *wsp, const int *zs) {
  const int lane = threadIdx.x & 63, col = lane & 15, grp = lane >> 4;
  const int V = A.P.V;
  const int koff = L.koff[v], K = L.koff[v + 1] - koff;
  mvc_d4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
  lpview_tile_mfma<NT, SPPT, RP>(cur, nxt, SPPT, L.Bs + L.boff[v] + lane, ring, acc);
  const double *y2t = wsp + v * 16, *ht = wsp + 64 + v * 16;
  double *selfG = wsp + 128 + v * 16, *mrest = wsp + 192 + v * 16;
  double hy[4], hr[4];
  int j0[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    hy[r] = 0.5 * y2t[grp + 4 * r];
    hr[r] = ht[grp + 4 * r];
    j0[r] = L.tix[zs[grp + 4 * r] * V + v] - koff;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {   // G of the own dish -> LDS
    const int jt = j0[r] >> 4;
    double g = acc[0][r];
#pragma unroll
    for (int t = 1; t < NT; ++t)
      if (jt == t) g = acc[t][r];
    if (col == (j0[r] & 15)) selfG[grp + 4 * r] = g;
  }
  // frozen-dish lp for every (row, dish): a fixed number of unconditional
  // stores (the own dish is overwritten at the end of the tile by this same
  // wave, in program order); the max over the other included dishes per row
  double mx[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) mx[r] = -MVC_PM_INF;
  // byte offset of (row grp + 4 r, dish koff + 16 t + col) within the tile:
  // 128 (koff + 16 t + col) + 8 lpb_slot(grp + 4 r) = ... + 32 grp + 8 r, so a
  // lane's four rows are two 16-byte stores.  Rows past the batch end go to
  // their own (unread) slots of the last slab; dishes past K_v to the discard.
  const int lbase = tile_boff + 128 * (koff + col) + 32 * grp;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = 16 * t + col;
    const int kc = koff + min(j, K - 1);
    const double c0j = L.c0[kc], cbj = L.cb[kc];
    const bool inc = j < K && L.dl[kc] > 0;
    double val[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      val[r] = __builtin_fma(acc[t][r] + hy[r], cbj, c0j) + hr[r];
      if (inc && j != j0[r] && val[r] > mx[r]) mx[r] = val[r];
    }
    const int off = j < K ? lbase + 2048 * t : disc_boff;
    mvc_raw_buffer_store_v2f64((mvc_d2){val[0], val[1]}, rsrc, off, 0, 0);
    mvc_raw_buffer_store_v2f64((mvc_d2){val[2], val[3]}, rsrc, j < K ? off + 16 : disc_boff, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double x = mx[r];
    x = dmax(x, down_d<8>(x));
    x = dmax(x, down_d<4>(x));
    x = dmax(x, down_d<2>(x));
    x = dmax(x, down_d<1>(x));
    if (col == 0) mrest[grp + 4 * r] = x;   // lane 0 of the row holds the row's max
  }
}

// The own dish of every (view, row) of the tile, one lane each (lane = row +
// 16 view, V <= 4): its lp with the customer removed (oracle: the self-removed
// coefficients) overwrites the frozen value, and the view maximum m_v (the
// max over the included dishes and the new dish, oracle eval_view_seq) goes
// to vmax, so the draw reads each lp row once.
__device__ __forceinline__ void lpa_tile_end(const Sweep &A, const LpaLds &L, int b0, int li0, int nb, double y2,
                                             double h, double cnew, int pz, mvc_i4 rsrc, int tile_boff, int disc_boff,
                                             const double *wsp, double *dslot) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63, row = lane & 15, v = lane >> 4;
  const int V = P.V, n = P.n;
  const int vv = min(v, V - 1);
  const double G = wsp[128 + vv * 16 + row];
  const int kk = L.tix[pz * V + vv];
  const double Gp = G - y2;
  const double Qp = (L.Q[kk] - 2.0 * G) + y2;
  const double c0 = L.xs[kk] - (0.5 * Qp) / L.dens[kk];
  const double sv = __builtin_fma(Gp + 0.5 * y2, L.cbs[kk], c0) + h;
  const bool ok = v < V && li0 + row < nb;
  mvc_raw_buffer_store_f64(sv, rsrc, ok ? tile_boff + 128 * kk + 8 * lpb_slot(row) : disc_boff, 0, 0);
  const bool alive = (L.nt[pz] - 1) > 0;
  const int l0p = L.dl[kk] - (alive ? 0 : 1);
  double m = wsp[192 + vv * 16 + row];
  if (l0p > 0 && sv > m) m = sv;
  const double lfn = cnew + h;
  if (lfn > m) m = lfn;
  double *dm = ok ? A.vmax + (size_t)vv * n + b0 + li0 + row : dslot;
  *dm = m;
}

template <int SPPT, int RP, uint32_t PAT, int VI>
__device__ __forceinline__ void lpa_views(const Sweep &A, const LpaLds &L, int li0, int nb, const mvc_d2 *ybase,
                                          size_t vstride, size_t tcur, size_t tnext, mvc_d2 (&ring)[RP], mvc_i4 rsrc,
                                          int tile_boff, int disc_boff, double *wsp, const int *zs) {
  if constexpr (VI < fz_pat_v(PAT)) {
    const mvc_d2 *cur = ybase + (size_t)VI * vstride + tcur;
    const mvc_d2 *nxt = (VI + 1 < fz_pat_v(PAT)) ? ybase + (size_t)(VI + 1) * vstride + tcur : ybase + tnext;
    lpa_view<fz_pat_nt(PAT, VI), SPPT, RP>(A, L, VI, li0, nb, cur, nxt, ring, rsrc, tile_boff, disc_boff, wsp, zs);
    lpa_views<SPPT, RP, PAT, VI + 1>(A, L, li0, nb, ybase, vstride, tcur, tnext, ring, rsrc, tile_boff, disc_boff, wsp,
                                     zs);
  }
}

template <int SPPT, int RP, uint32_t PAT>
#ifndef MVC_LPA_WAVES
#define MVC_LPA_WAVES 8       // waves per block (one block per CU) of the all-views producer
#endif
#ifndef MVC_LPA_RP16
#define MVC_LPA_RP16 8        // ring depth (k-step pairs in flight per wave) at D = 128
#endif
__global__ __launch_bounds__(64 * MVC_LPA_WAVES) void mvc_par_lpall_kernel(Sweep A, int b0, int nb, double *lpb,
                                                                          double *discard) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, BW = blockDim.x >> 6;
  constexpr int V = fz_pat_v(PAT);
  const int KC = P.KC, TC = P.TC, n = P.n, D = P.D;
  const int T = __builtin_amdgcn_readfirstlane(A.T);
  constexpr int SP = 2 * SPPT;
  int *s_koff = (int *)smem;                                   // [V+1]
  int *s_boff = s_koff + V + 1;                                // [V+1] (doubles)
  if (tid <= V) {
    s_koff[tid] = A.Koff[tid];
    int acc = 0;
    for (int u = 0; u < tid; ++u) acc += SP * 64 * fz_pat_nt(PAT, u);
    s_boff[tid] = acc;
  }
  __syncthreads();
  const int sumK = s_koff[V];
  const int nB = s_boff[V];
  double *Bs = (double *)(smem + 16 * 4);
  double *f_c0 = Bs + nB, *f_cb = f_c0 + sumK, *f_Q = f_cb + sumK;
  double *f_xs = f_Q + sumK, *f_dens = f_xs + sumK, *f_cbs = f_dens + sumK;
  double *wsp = f_cbs + sumK + (size_t)w * kLpaWaveD;          // per wave: y2, h, selfG, mrest [4][16] each
  int *f_dn = (int *)(f_cbs + sumK + (size_t)BW * kLpaWaveD), *f_dl = f_dn + sumK;
  int *f_tix = f_dl + sumK, *f_nt = f_tix + MVC_FZ_TB * 16 * V;
  int *zs = f_nt + MVC_FZ_TB * 16 + w * kLpaWaveI;
  {
    const mvc_d2 *src = (const mvc_d2 *)A.S1t;
    mvc_d2 *dst = (mvc_d2 *)Bs;
    for (int e = tid; e < nB / 2; e += blockDim.x) dst[e] = src[e];
  }
  for (int k = tid; k < sumK; k += blockDim.x) {
    int v = 0;
    while (v + 1 < V && s_koff[v + 1] <= k) ++v;
    const int j = k - s_koff[v];
    f_c0[k] = P.c0[v * KC + j];
    f_cb[k] = P.cb[v * KC + j];
    f_Q[k] = P.Q[v * KC + j];
    const int dn = P.d_n[v * KC + j];
    f_dn[k] = dn;
    f_dl[k] = P.d_l[v * KC + j];
    lpall_self_coef(dn, P.hyper[v], A.L2pt[v], D, f_xs[k], f_dens[k], f_cbs[k]);
  }
  for (int p = tid; p < MVC_FZ_TB * 16; p += blockDim.x) {
    f_nt[p] = p < T ? P.n_t[p] : 0;
    for (int v = 0; v < V; ++v) f_tix[p * V + v] = s_koff[v] + (p < T ? P.dish[v * TC + p] : 0);
  }
  __syncthreads();
  const LpaLds L{Bs, f_c0, f_cb, f_Q, f_xs, f_dens, f_cbs, f_dn, f_dl, f_tix, f_nt, s_koff, s_boff};

  // customers [b0, b0 + nb) (b0 a multiple of 16): local tiles; yt, z, Y2 and
  // vmax are indexed by customer, the lp buffer by batch position
  const int ntile = (nb + 15) >> 4, tb0 = b0 >> 4;
  const int gw = blockIdx.x * BW + w, NWT = gridDim.x * BW;
  if (gw >= ntile) return;                         // whole wave: no barriers below
  const int nmy = (ntile - gw + NWT - 1) / NWT;
  const size_t vstride = (size_t)((n + 15) >> 4) * SPPT * 64;
  const mvc_d2 *ybase = (const mvc_d2 *)A.yt + lane;
  auto toff = [&](int m) -> size_t { return (size_t)(tb0 + gw + min(m, nmy - 1) * NWT) * SPPT * 64; };
  mvc_d2 ring[RP];
  {
    const mvc_d2 *c0p = ybase + toff(0);
#pragma unroll
    for (int u = 0; u < RP; ++u) ring[u] = c0p[u * 64];
  }
  double *const dslot = discard + lane;
  // the lp buffer through a buffer resource: 32-bit byte offsets (the
  // buffer is < 2^31 bytes, kLpbBudget); the discard slots follow it
  const uint64_t lpa = (uint64_t)lpb;
  const mvc_i4 rsrc = (mvc_i4){(int)(uint32_t)lpa, (int)(uint32_t)(lpa >> 32), -1, 0x00020000};
  const int disc_boff = (int)((uint64_t)(discard - lpb) * 8) + 16 * lane;   // 16-byte stores
  const int row = lane & 15, vl = lane >> 4;      // this lane's (row, view) in the tile start / end passes
  const int vq = min(vl, V - 1);
  const double tau_l = P.hyper[vq], cnew_l = A.cnew[vq];
  // The tile's z and Y2 are loaded one tile ahead: vmcnt retires in order,
  // so a load issued at the tile start would make its first use wait for
  // every y prefetch in flight (the ring) as well.
  auto rowof = [&](int mm) { return min(b0 + (gw + min(mm, nmy - 1) * NWT) * 16 + row, n - 1); };
  int pz_next = P.z[rowof(0)];
  double y2_next = A.Y2[(size_t)vq * n + rowof(0)];
  for (int m = 0; m < nmy; ++m) {
    const int li0 = (gw + m * NWT) * 16;
    const int pz = pz_next;
    const double y2 = y2_next;
    pz_next = P.z[rowof(m + 1)];
    y2_next = A.Y2[(size_t)vq * n + rowof(m + 1)];
    // tile start: y2 and h of (view vl, row) -- one division per lane per
    // tile; unconditional LDS writes (lanes of one row store the same z)
    const double h = (-0.5 * y2) / tau_l;
    wsp[vl * 16 + row] = y2;
    wsp[64 + vl * 16 + row] = h;
    zs[row] = pz;
    wave_lds_sync();
    const int tile_boff = li0 * sumK * 8;           // (li0 >> 4) * sumK * 16 doubles
    lpa_views<SPPT, RP, PAT, 0>(A, L, li0, nb, ybase, vstride, toff(m), toff(m + 1), ring, rsrc, tile_boff, disc_boff,
                                wsp, zs);
    wave_lds_sync();
    lpa_tile_end(A, L, b0, li0, nb, y2, h, cnew_l, pz, rsrc, tile_boff, disc_boff, wsp, dslot);
    wave_lds_sync();
  }
}


#include "mvc_repair.h"

// Y2[v][i] = sum_d y^2, fma chain in d order (oracle ParallelSampler::fma_dot)
extern "C" __global__ void mvc_par_y2_kernel(int n, int V, int D, const double *y, double *Y2) {
  const size_t total = (size_t)n * V;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const double *r = y + e * D;
    double acc = 0.0;
    for (int d = 0; d < D; ++d) acc = __builtin_fma(r[d], r[d], acc);
    Y2[e] = acc;
  }
}

// ---------------------------------------------------------------------------
// Stats rebuild, chunked ordered sums.  Block (chunk c,
// view v): (1) dish of every customer of the chunk into LDS; (2) thread j
// builds the ascending member list of dish j by one broadcast pass over the
// chunk; (3) thread per (dish j, dim d), d fastest, accumulates y over the
// members in ascending order in a register (the spec's sequential sum) with
// 8 loads in flight.  part1[c][Koff[v]+j][d], part2[c][Koff[v]+j].
// ---------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void mvc_par_stats_partial_kernel(
    ParState P, const double *y, const double *Y2, const int32_t *Koff, int stride, uint64_t vmask,
    double *part1, double *part2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int c = blockIdx.x, v = blockIdx.y;
  if (!((vmask >> v) & 1ull)) return;
  const int tid = threadIdx.x;
  const int n = P.n, D = P.D, TC = P.TC;
  const int K = P.Kact[v];
  const int i0 = c * kStatsChunk, cnt = min(n, i0 + kStatsChunk) - i0;
  int *jsub = (int *)smem;               // [kStatsChunk]
  int *list = jsub + kStatsChunk;        // [kStatsChunk]
  int *off = list + kStatsChunk;         // [K + 1]
  for (int q = tid; q < cnt; q += 256) jsub[q] = P.dish[v * TC + P.z[i0 + q]];
  __syncthreads();
  // member counts -> offsets (thread j counts; single pass per dish chunk)
  for (int j0 = 0; j0 < K; j0 += 256) {
    const int j = j0 + tid;
    int m = 0;
    if (j < K)
      for (int q = 0; q < cnt; ++q) m += (jsub[q] == j) ? 1 : 0;
    if (j < K) off[j + 1] = m;
  }
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    for (int j = 0; j < K; ++j) off[j + 1] += off[j];
  }
  __syncthreads();
  for (int j0 = 0; j0 < K; j0 += 256) {
    const int j = j0 + tid;
    if (j < K) {
      int w = off[j];
      for (int q = 0; q < cnt; ++q)
        if (jsub[q] == j) list[w++] = q;
    }
  }
  __syncthreads();
  const size_t base = (size_t)c * stride + Koff[v];
  const double *yv = y + ((size_t)v * n + i0) * D;
  const int items = K * D;
  for (int it = tid; it < items + K; it += 256) {
    if (it < items) {
      const int j = it / D, d = it - (it / D) * D;
      const int m0 = off[j], m1 = off[j + 1];
      double acc = 0.0;
      int m = m0;
      for (; m + 8 <= m1; m += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = yv[(size_t)list[m + u] * D + d];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + x[u];
      }
      for (; m < m1; ++m) acc = acc + yv[(size_t)list[m] * D + d];
      part1[(base + j) * D + d] = acc;
    } else {
      const int j = it - items;
      double acc = 0.0;
      for (int m = off[j]; m < off[j + 1]; ++m) acc = acc + Y2[(size_t)v * n + i0 + list[m]];
      part2[base + j] = acc;
    }
  }
}

// S1T[v][d][j] = sum_c part1[c][..] (ascending c, from 0.0); same for S2.
// stride = dish-row stride of the partial buffers (>= Koff[V]).
extern "C" __global__ void mvc_par_stats_combine_kernel(ParState P, const int32_t *Koff, int stride, int nchunk,
                                                        uint64_t vmask, const double *part1, const double *part2) {
  const int D = P.D, KC = P.KC, V = P.V;
  const size_t tot = (size_t)Koff[V] * (D + 1);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e / (D + 1));
    const int d = (int)(e % (D + 1));
    int v = 0;
    while (v + 1 < V && Koff[v + 1] <= k) ++v;
    if (!((vmask >> v) & 1ull)) continue;
    const int j = k - Koff[v];
    double s = 0.0;
    if (d < D) {
      for (int c = 0; c < nchunk; ++c) s = s + part1[((size_t)c * stride + k) * D + d];
      P.S1T[((size_t)v * D + d) * KC + j] = s;
    } else {
      for (int c = 0; c < nchunk; ++c) s = s + part2[(size_t)c * stride + k];
      P.S2[v * KC + j] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// Hyperparameter MH + next-sweep coefficients, ONE workgroup of 256.
// ---------------------------------------------------------------------------
namespace {

struct BlockCtx {
  double *red;      // LDS [4]
  double *scratch;  // global, >= leaves/64 + ... per level (two halves)
  size_t half;      // scratch half size
};

// tree64 over n <= 64^3 leaves produced by leaf(e), executed by the whole
// block: 64-leaf chunk sums into LDS (level 1), chunk sums of those (level
// 2), then the root.  Same association as oracle Tree64::build (each level's
// node c = butterfly64 of the 64 nodes below it, zero-padded).
template <class F>
__device__ double block_tree64(int64_t n, F leaf) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  __shared__ double s_p1[4096];
  __shared__ double s_p2[64];
  __shared__ double s_root;
  if (n <= 0) return 0.0;
  const int m = (int)((n + 63) / 64);
  for (int c = w; c < m; c += nw) {
    const int64_t e = (int64_t)c * 64 + lane;
    const double x = e < n ? leaf(e) : 0.0;
    const double s = wave_tree_sum(x);
    if (lane == 0) s_p1[c] = s;
  }
  __syncthreads();
  const int m2 = (m + 63) / 64;
  if (m > 1) {
    for (int c = w; c < m2; c += nw) {
      const int e = c * 64 + lane;
      const double s = wave_tree_sum(e < m ? s_p1[e] : 0.0);
      if (lane == 0) s_p2[c] = s;
    }
    __syncthreads();
  }
  if (w == 0) {
    double r;
    if (m == 1) r = s_p1[0];
    else if (m2 == 1) r = s_p2[0];
    else r = wave_tree_sum(lane < m2 ? s_p2[lane] : 0.0);
    if (lane == 0) s_root = r;
  }
  __syncthreads();
  const double r = s_root;
  __syncthreads();
  return r;
}

// Four EPPF evaluations at once on one wave (the MH's speculative form for
// small states, mvc_par_hyper_kernel): row r of the wave (lanes 16 r ..
// 16 r + 15) evaluates the EPPF of a partition of K <= 16
// blocks of sizes size(j) and total tot at (a[r], s[r]), exactly as the
// kernel's eppf does with one wave: its tree64 sums have their leaves in
// lanes 0..K-1 and +0 above (no partial sum is -0), so the row tree
// (offsets 8, 4, 2, 1) is the wave tree's value (whose offsets 32 and 16 add
// +0 there); the three scalar log-gammas on lanes 0 / 1 / 2 of the row.  E[r]
// is the row's value, wave-uniform.  Only the arithmetic part: the callers
// apply eppf's early returns per row.
template <class F>
__device__ __forceinline__ void eppf_rows4(int K, int tot, F size, const double (&a)[4], const double (&s)[4],
                                           double (&E)[4]) {
  const int lane = threadIdx.x & 63, r = lane >> 4, j = lane & 15;
  double ar = a[0], sr = s[0];
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (r == q) { ar = a[q]; sr = s[q]; }
  const double l1 = j < K ? mvc_log_nb(ar + (double)j * sr) : 0.0;
  const double qa = j == 0 ? ar + (double)tot : (j == 1 ? ar + 1.0 : 1.0 - sr);
  const double qg = mvc_lgamma_pos_nb(qa);
  const double P2 = row_bcast_d<0>(qg) - row_bcast_d<1>(qg);
  const double lg1 = row_bcast_d<2>(qg);
  const double l3 = j < K ? mvc_lgamma_pos_nb((double)size(min(j, K - 1)) - sr) - lg1 : 0.0;
  const double P1 = row16_tree_sum(l1), P3 = row16_tree_sum(l3);
  const double e = (P1 - P2) + P3;
#pragma unroll
  for (int q = 0; q < 4; ++q) E[q] = readlane_d(e, 16 * q);
}

struct MHArgs {
  ParState P;
  int32_t *status;        // [V+3]: T, K[V], err, NB  -> we add T_ne at status[V+3]
  int32_t *Koff;          // [V+1] (prefix of Kact, maintained by the host / the repair's compaction)
  double *L2pt, *cnew;    // [V] (output)
  uint64_t seed;
  uint32_t chain, sweep;
  int do_mh;
  const Repair *gate;     // non-null: run only if the sweep's repair is done with no move
  int gate_mode;          // 1: with gate, run iff the repair is done (moves or not; its compaction ran before)
};

}  // namespace

// 8 waves (two per SIMD): waves 0-6 run the per-view MH steps (views w, w + 7,
// ...: one view per wave for the reference's few views); wave 7 runs the
// global pair at the same time when T is small (one-wave tree64 = the block
// tree64's association), else the whole block runs it afterwards.
constexpr int kHypWaves = 8, kHypViewWaves = kHypWaves - 1, kHypThreads = 64 * kHypWaves, kHypGlobalWaveT = 512;
__device__ __forceinline__ void hyper_body(MHArgs &A) {
  ParState &P = A.P;
  const int tid = threadIdx.x;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n;
  __shared__ int s_i[8];
#ifdef MVC_HYP_PROF
  const uint64_t t0 = wall_clock64();
#define HYP_MARK(name) if (tid == 0 && A.sweep == 5) printf("hyp %s %llu\n", name, (unsigned long long)(wall_clock64() - t0))
#else
#define HYP_MARK(name)
#endif
  // gated launch (enqueued before the host has read the repair's outcome):
  // runs only for a finished repair with no move, where nothing (compaction,
  // relabel, capacity growth) has to come between the repair and the MH
  if (A.gate && !(A.gate->done && (A.gate_mode == 1 || A.gate->moves == 0) && A.gate->overflow == 0 &&
                  A.gate->restride == 0))
    return;
  const int T = A.status[0];
  __shared__ int s_koff[MVC_MAXV + 1];
  __shared__ int s_kact[MVC_MAXV];
  __shared__ double s_hyp[3 * MVC_MAXV + 2];   // the sweep's hyperparameters (the MH's updates written through)
  // The view offsets, the hyperparameters and this thread's first table
  // count are loaded together (one memory latency, not one per view).
  if (tid < V) s_kact[tid] = P.Kact[tid];
  for (int k = tid; k < 3 * V + 2; k += kHypThreads) s_hyp[k] = P.hyper[k];
  const int nt_me = P.n_t[max(0, min(tid, T - 1))];
  __syncthreads();
  if (tid == 0) {
    s_koff[0] = 0;
    for (int v = 0; v < V; ++v) s_koff[v + 1] = s_koff[v] + s_kact[v];
  }
  __syncthreads();
  // ---- Q = ||S1||^2 per live dish (fma chain in d order), all views at once;
  //      the strided S1 loads are issued 16 ahead of the chain.  The thread's
  //      first dish keeps Q and its member count for the coefficients below ----
  double q_me = 0.0;
  int dn_me = 0;
  {
    for (int k = tid; k < s_koff[V]; k += kHypThreads) {
      int v = 0;
      while (k >= s_koff[v + 1]) ++v;
      const int j = k - s_koff[v];
      if (k == tid) dn_me = P.d_n[v * KC + j];
      const double *col = P.S1T + (size_t)v * D * KC + j;
      double q = 0.0;
      int d = 0;
      for (; d + 16 <= D; d += 16) {
        double x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = col[(size_t)(d + u) * KC];
#pragma unroll
        for (int u = 0; u < 16; ++u) q = __builtin_fma(x[u], x[u], q);
      }
      for (; d < D; ++d) {
        const double x = col[(size_t)d * KC];
        q = __builtin_fma(x, x, q);
      }
      P.Q[v * KC + j] = q;
      if (k == tid) q_me = q;
    }
  }
  {   // integer sums (order-free): L_v = sum of the view's table counts, tables non-empty
    const int lane = tid & 63, w = tid >> 6;
    for (int v = w; v <= V; v += kHypWaves) {
      const int m = v < V ? s_kact[v] : T;
      int acc = 0;
      for (int j = lane; j < m; j += 64) acc += v < V ? P.d_l[v * KC + j] : (P.n_t[j] > 0 ? 1 : 0);
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) {
        if (v < V) P.Ltot[v] = acc;
        else { s_i[0] = acc; A.status[V + 3] = acc; }
      }
    }
  }
  __syncthreads();
  HYP_MARK("q+sums");
  const double *hyp = s_hyp;
  auto put_hyp = [&](int k, double x) { s_hyp[k] = x; P.hyper[k] = x; };
  if (A.do_mh) {
    // Every MH step draws from its own window of the MH counter (oracle
    // update_hyper): tau of view v at 3v, alpha/sigma of view v at 3V + 6v,
    // the global pair at 9V.  The per-view steps are independent, so wave w
    // runs views w, w + 7, ... with wavefront-level tree64 sums (same
    // association as block_tree64); the global pair then runs on the block.
    auto unif_at = [&](uint32_t k) -> double { return mvc_uniform(A.seed, k, A.sweep, A.chain, MVC_TAG_MH); };
    auto rnorm_at = [&](uint32_t k, double mu, double sd) -> double {
      const double u1 = unif_at(k);
      const double u2 = unif_at(k + 1);
      return mu + sd * mvc_norm_from_uniforms(u1, u2);
    };
    auto prior_alpha = [](double a) -> double {
      if (a <= 0.0) return -MVC_PM_INF;
      return (4.0 - 1.0) * mvc_log(a) - 3.0 * a;
    };
    auto prior_sigma = [](double s) -> double {
      if (s <= 0.0 || s >= 1.0) return -MVC_PM_INF;
      return (1.0 - 1.0) * mvc_log(s) + (5.0 - 1.0) * mvc_log(1.0 - s);
    };
    auto reflect_unit = [](double value) -> double {
      double p = value;
      while (p <= kEps || p >= 1.0 - kEps) {
        if (p <= kEps) p = 2.0 * kEps - p;
        if (p >= 1.0 - kEps) p = 2.0 * (1.0 - kEps) - p;
      }
      return p < kEps ? kEps : (p > 1.0 - kEps ? 1.0 - kEps : p);
    };
    // EPPF of a partition: K blocks of sizes size(j) >= 1, total tot; tree is
    // the wave- or block-level tree64
    auto eppf = [&](int K, int tot, auto size, double a, double s, auto tree) -> double {
      if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
      if (a <= -s) return -MVC_PM_INF;
      // any term a + j s <= 0 ?  (monotone in j for s > 0: check j = 0)
      if (K > 0 && !(a + 0.0 * s > 0.0)) return -MVC_PM_INF;
      const double P1 = tree(K, [&](int64_t j) { return mvc_log_nb(a + (double)j * s); });
      // the three scalar log-gammas on lanes 0 / 1 / 2 of one branch-free
      // evaluation (the same arguments and function, so the same values)
      const int ql = threadIdx.x & 63;
      const double qa = ql == 0 ? a + (double)tot : (ql == 1 ? a + 1.0 : 1.0 - s);
      const double qg = mvc_lgamma_pos_nb(qa);
      const double P2 = readlane_d(qg, 0) - readlane_d(qg, 1);
      const double lg1 = readlane_d(qg, 2);
      const double P3 = tree(K, [&](int64_t j) { return mvc_lgamma_pos_nb((double)size((int)j) - s) - lg1; });
      return (P1 - P2) + P3;
    };
    // ---- per-view steps, one wavefront per view (multiview_hyper.cpp:211-266)
    const bool global_on_wave = T <= kHypGlobalWaveT;
    // The tree64 leaves e of a thread are e = 64 c + (tid & 63) (wave and
    // block trees alike), so each thread loads its leaves' table counts for
    // c < 8 once, not once per EPPF evaluation (4 of them in the pair).
    const int hl = tid & 63;
    int nt_pre[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) nt_pre[c] = P.n_t[max(0, min(64 * c + hl, T - 1))];
    auto nt_at = [&](int p) -> int {
      if (p >= 512) return P.n_t[p];
      int x = nt_pre[0];
#pragma unroll
      for (int c = 1; c < 8; ++c)
        if ((p >> 6) == c) x = nt_pre[c];
      return x;
    };
    auto global_pair = [&](auto tree) {   // (:268-291), counters 9V ..
      auto eppf_global = [&](double a, double s) -> double {
        if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
        if (a <= -s) return -MVC_PM_INF;
        if (T <= 0) return 0.0;
        return eppf(T, n, nt_at, a, s, tree);
      };
      const uint32_t k0 = 9u * (uint32_t)V;
      double ag_old = hyp[3 * V];
      if (ag_old <= 0.0) ag_old = kEps;
      const double la = mvc_log(ag_old > kEps ? ag_old : kEps) + rnorm_at(k0, 0.0, 0.1);
      double ag_prop = mvc_exp(la);
      if (!(ag_prop > kEps)) ag_prop = kEps;
      const double sg0 = hyp[3 * V + 1];
      const double lo = eppf_global(ag_old, sg0) + prior_alpha(ag_old);
      const double ln = eppf_global(ag_prop, sg0) + prior_alpha(ag_prop);
      const double lq = mvc_log(ag_prop) - mvc_log(ag_old);
      double a_g = hyp[3 * V];
      if (mvc_log(unif_at(k0 + 2)) < (ln - lo) + lq) a_g = ag_prop;
      const double sg_old = sg0;
      const double sg_prop = reflect_unit(sg_old + rnorm_at(k0 + 3, 0.0, 0.05));
      const double u2 = unif_at(k0 + 5);
      const double pn = (sg_prop <= kEps || sg_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_prop) + prior_sigma(sg_prop);
      const double po = (sg_old <= kEps || sg_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_old) + prior_sigma(sg_old);
      double s_g = sg_old;
      if (mvc_log(u2) < pn - po) s_g = sg_prop;
      return std::make_pair(a_g, s_g);
    };
    // The speculative form for small states (every dish list and the tables
    // <= 16, V <= 7, every alpha > 0, the reference's own call at steady
    // state): a step's two EPPF evaluations and the sigma step's two, for
    // both outcomes of the alpha step, run at once on the four rows of one
    // wave (eppf_rows4), the tau step's two posteriors on two rows; then the
    // same accept decisions on the same values.  With alpha > 0 the alpha
    // step's "old" value is the current alpha, so the sigma step's EPPFs are
    // two of the four rows whichever way the alpha step went.
    bool fast = V <= kHypViewWaves && T <= 16 && hyp[3 * V] > 0.0;
    for (int v = 0; v < V; ++v) fast = fast && s_kact[v] <= 16 && hyp[V + v] > 0.0;
    if (fast) {
      const int lane = tid & 63, wv = tid >> 6, row = lane >> 4, j = lane & 15;
      if (wv < V) {   // view wv
        const int v = wv;
        const int Kv = s_kact[v], Lv = P.Ltot[v];
        const uint32_t kt = 3u * (uint32_t)v, ka = 3u * (uint32_t)V + 6u * (uint32_t)v;
        const double zt = rnorm_at(kt, 0.0, 0.3), za = rnorm_at(ka, 0.0, 0.1), zs = rnorm_at(ka + 3, 0.0, 0.05);
        // tau (multiview_hyper.cpp:211-231): rows 0 / 1 the posterior at t_old / t_prop
        double tau_v = hyp[v];
        double t_old = tau_v;
        if (t_old <= 0.0) t_old = kEps;
        const double t_prop = mvc_exp(mvc_log(t_old) + zt);
        {
          const double t = row == 0 ? t_old : t_prop;
          const double L = mvc_log((2.0 * MVC_PI) * t);
          const int jj = min(j, max(Kv - 1, 0));
          const int nk = P.d_n[v * KC + jj];
          double leaf = 0.0;
          if (j < Kv && nk != 0) {
            double sse = P.S2[v * KC + jj] - P.Q[v * KC + jj] / (double)nk;
            if (sse < 0.0) sse = 0.0;
            leaf = ((-0.5 * (double)nk) * (double)D) * L - 0.5 * (sse / t);
          }
          const double ll = row16_tree_sum(leaf);
          const double post = ll + ((-3.0 * mvc_log(t)) - 1.0 / t);
          const double l_old = readlane_d(post, 0), l_new = readlane_d(post, 16);
          if (t_prop > 0.0) {
            const double acc = (l_new - l_old) + (mvc_log(t_prop) - mvc_log(t_old));
            if (mvc_log(unif_at(kt + 2)) < acc) tau_v = t_prop;
          }
        }
        // alpha_v, sigma_v (:239-266)
        const double a_orig = hyp[V + v], s_v0 = hyp[2 * V + v];
        const double a_old = a_orig;   // > 0 (the fast form's condition)
        double a_prop = mvc_exp(mvc_log(a_old > kEps ? a_old : kEps) + za);
        if (!(a_prop > kEps)) a_prop = kEps;
        const double s_prop = reflect_unit(s_v0 + zs);
        const double ar[4] = {a_old, a_prop, a_orig, a_prop}, sr[4] = {s_v0, s_v0, s_prop, s_prop};
        double E[4];
        eppf_rows4(Kv, Lv, [&](int jj) { return P.d_l[v * KC + jj]; }, ar, sr, E);
        auto ev = [&](int q) -> double {   // eppf_view's early returns
          if (!(sr[q] > kEps && sr[q] < 1.0 - kEps)) return -MVC_PM_INF;
          if (ar[q] <= -sr[q]) return -MVC_PM_INF;
          if (Lv == 0) return 0.0;
          if (Kv > 0 && !(ar[q] + 0.0 * sr[q] > 0.0)) return -MVC_PM_INF;
          return E[q];
        };
        double a_v = a_orig, s_v = s_v0;
        const double lo = ev(0) + prior_alpha(a_old);
        const double ln = ev(1) + prior_alpha(a_prop);
        const double lq = mvc_log(a_prop) - mvc_log(a_old);
        const bool took = mvc_log(unif_at(ka + 2)) < (ln - lo) + lq;
        if (took) a_v = a_prop;
        const double u2 = unif_at(ka + 5);
        const double pn = (s_prop <= kEps || s_prop >= 1.0 - kEps) ? -MVC_PM_INF : ev(took ? 3 : 2) + prior_sigma(s_prop);
        const double po = (s_v0 <= kEps || s_v0 >= 1.0 - kEps) ? -MVC_PM_INF : ev(took ? 1 : 0) + prior_sigma(s_v0);
        if (mvc_log(u2) < pn - po) s_v = s_prop;
        if (lane == 0) { put_hyp(v, tau_v); put_hyp(V + v, a_v); put_hyp(2 * V + v, s_v); }
      } else if (wv == kHypViewWaves) {   // the global pair (:268-291), counters 9V ..
        const uint32_t k0 = 9u * (uint32_t)V;
        const double za = rnorm_at(k0, 0.0, 0.1), zs = rnorm_at(k0 + 3, 0.0, 0.05);
        const double ag_orig = hyp[3 * V], sg0 = hyp[3 * V + 1];
        const double ag_old = ag_orig;   // > 0
        double ag_prop = mvc_exp(mvc_log(ag_old > kEps ? ag_old : kEps) + za);
        if (!(ag_prop > kEps)) ag_prop = kEps;
        const double sg_prop = reflect_unit(sg0 + zs);
        const double ar[4] = {ag_old, ag_prop, ag_orig, ag_prop}, sr[4] = {sg0, sg0, sg_prop, sg_prop};
        double E[4];
        eppf_rows4(T, n, [&](int p) { return P.n_t[p]; }, ar, sr, E);
        auto eg = [&](int q) -> double {   // eppf_global's and eppf's early returns
          if (!(sr[q] > kEps && sr[q] < 1.0 - kEps)) return -MVC_PM_INF;
          if (ar[q] <= -sr[q]) return -MVC_PM_INF;
          if (T <= 0) return 0.0;
          if (!(ar[q] + 0.0 * sr[q] > 0.0)) return -MVC_PM_INF;
          return E[q];
        };
        const double lo = eg(0) + prior_alpha(ag_old);
        const double ln = eg(1) + prior_alpha(ag_prop);
        const double lq = mvc_log(ag_prop) - mvc_log(ag_old);
        double a_g = ag_orig, s_g = sg0;
        const bool took = mvc_log(unif_at(k0 + 2)) < (ln - lo) + lq;
        if (took) a_g = ag_prop;
        const double u2 = unif_at(k0 + 5);
        const double pn = (sg_prop <= kEps || sg_prop >= 1.0 - kEps) ? -MVC_PM_INF : eg(took ? 3 : 2) + prior_sigma(sg_prop);
        const double po = (sg0 <= kEps || sg0 >= 1.0 - kEps) ? -MVC_PM_INF : eg(took ? 1 : 0) + prior_sigma(sg0);
        if (mvc_log(u2) < pn - po) s_g = sg_prop;
        if (lane == 0) { put_hyp(3 * V, a_g); put_hyp(3 * V + 1, s_g); }
      }
    } else {
      __shared__ double s_wpart[kHypWaves][64];
      __shared__ double s_wpart2[kHypWaves][64];
      const int lane = tid & 63, wv = tid >> 6;
      // tree64 by one wavefront, nn <= 64^3 leaves: 64-leaf chunk sums,
      // reduced 64 at a time into level-2 nodes, then the root (oracle
      // Tree64::build's association)
      auto wtree = [&](int64_t nn, auto leaf) -> double {
        if (nn <= 0) return 0.0;
        const int mch = (int)((nn + 63) / 64);
        const int m2 = (mch + 63) / 64;
        double root = 0.0;
        for (int c2 = 0; c2 < m2; ++c2) {
          const int cn = min(64, mch - c2 * 64);
          double l2 = 0.0;
          for (int cc = 0; cc < cn; ++cc) {
            const int64_t e = ((int64_t)c2 * 64 + cc) * 64 + lane;
            const double x = e < nn ? leaf(e) : 0.0;
            const double cs = wave_tree_sum(x);
            if (mch == 1) l2 = cs;
            else if (lane == 0) s_wpart[wv][cc] = cs;
          }
          if (mch > 1) {
            wave_lds_sync();
            l2 = wave_tree_sum(lane < cn ? s_wpart[wv][lane] : 0.0);
            wave_lds_sync();
          }
          if (m2 == 1) root = l2;
          else if (lane == 0) s_wpart2[wv][c2] = l2;
        }
        if (m2 > 1) {
          wave_lds_sync();
          root = wave_tree_sum(lane < m2 ? s_wpart2[wv][lane] : 0.0);
          wave_lds_sync();
        }
        return root;
      };
      if (wv == kHypViewWaves && global_on_wave) {
        const auto g = global_pair(wtree);
        if (lane == 0) { put_hyp(3 * V, g.first); put_hyp(3 * V + 1, g.second); }
      }
      for (int v = wv; v < V && wv < kHypViewWaves; v += kHypViewWaves) {
        const int Kv = P.Kact[v], Lv = P.Ltot[v];
        // dish `lane` of the view (the wave tree's first chunk) loaded once for
        // the six tree evaluations below; its tau-leaf parts are the same
        // expressions as the leaf's, so the same values
        const int jl = max(0, min(lane, Kv - 1));
        const int dl_pre = P.d_l[v * KC + jl], nk_pre = P.d_n[v * KC + jl];
        double sse_pre = 0.0;
        if (nk_pre != 0) {
          sse_pre = P.S2[v * KC + jl] - P.Q[v * KC + jl] / (double)nk_pre;
          if (sse_pre < 0.0) sse_pre = 0.0;
        }
        const double a_pre = (-0.5 * (double)nk_pre) * (double)D;
        auto eppf_view = [&](double a, double s) -> double {
          if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
          if (a <= -s) return -MVC_PM_INF;
          if (Lv == 0) return 0.0;
          return eppf(Kv, Lv, [&](int j) { return j < 64 ? dl_pre : P.d_l[v * KC + j]; }, a, s, wtree);
        };
        auto post_tau = [&](double t) -> double {
          if (t <= 0.0) return -MVC_PM_INF;
          const double L = mvc_log((2.0 * MVC_PI) * t);
          const double ll = wtree(Kv, [&](int64_t j) {
            if (j < 64) return nk_pre == 0 ? 0.0 : a_pre * L - 0.5 * (sse_pre / t);
            const int nk = P.d_n[v * KC + j];
            if (nk == 0) return 0.0;
            double sse = P.S2[v * KC + j] - P.Q[v * KC + j] / (double)nk;
            if (sse < 0.0) sse = 0.0;
            return ((-0.5 * (double)nk) * (double)D) * L - 0.5 * (sse / t);
          });
          const double prior = (-3.0 * mvc_log(t)) - 1.0 / t;
          return ll + prior;
        };
        // tau (multiview_hyper.cpp:211-231), counters 3v ..
#ifdef MVC_HYP_PROF
        const uint64_t tw0 = wall_clock64();
#endif
        double tau_v = hyp[v];
        {
          const uint32_t k0 = 3u * (uint32_t)v;
          double t_old = tau_v;
          if (t_old <= 0.0) t_old = kEps;
          const double l_old = post_tau(t_old);
          const double t_prop = mvc_exp(mvc_log(t_old) + rnorm_at(k0, 0.0, 0.3));
          if (t_prop > 0.0) {
            const double l_new = post_tau(t_prop);
            const double acc = (l_new - l_old) + (mvc_log(t_prop) - mvc_log(t_old));
            if (mvc_log(unif_at(k0 + 2)) < acc) tau_v = t_prop;
          }
        }
        // alpha_v, sigma_v (:239-266), counters 3V + 6v ..
#ifdef MVC_HYP_PROF
        const uint64_t tw1 = wall_clock64();
        uint64_t tw2 = 0;
#endif
        double a_v = hyp[V + v], s_v = hyp[2 * V + v];
        {
          const uint32_t k0 = 3u * (uint32_t)V + 6u * (uint32_t)v;
          double a_old = a_v;
          if (a_old <= 0.0) a_old = kEps;
          const double la = mvc_log(a_old > kEps ? a_old : kEps) + rnorm_at(k0, 0.0, 0.1);
          double a_prop = mvc_exp(la);
          if (!(a_prop > kEps)) a_prop = kEps;
          const double lo = (a_old <= 0.0) ? -MVC_PM_INF : eppf_view(a_old, s_v) + prior_alpha(a_old);
          const double ln = (a_prop <= 0.0) ? -MVC_PM_INF : eppf_view(a_prop, s_v) + prior_alpha(a_prop);
          const double lq = mvc_log(a_prop) - mvc_log(a_old);
          if (mvc_log(unif_at(k0 + 2)) < (ln - lo) + lq) a_v = a_prop;
#ifdef MVC_HYP_PROF
          tw2 = wall_clock64();
#endif
          const double s_old = s_v;
          const double s_prop = reflect_unit(s_old + rnorm_at(k0 + 3, 0.0, 0.05));
          const double u2 = unif_at(k0 + 5);
          const double pn = (s_prop <= kEps || s_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(a_v, s_prop) + prior_sigma(s_prop);
          const double po = (s_old <= kEps || s_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(a_v, s_old) + prior_sigma(s_old);
          if (mvc_log(u2) < pn - po) s_v = s_prop;
        }
        if (lane == 0) { put_hyp(v, tau_v); put_hyp(V + v, a_v); put_hyp(2 * V + v, s_v); }
#ifdef MVC_HYP_PROF
        if (lane == 0 && A.sweep == 5)
          printf("hyp view %d: start %llu tau %llu alpha %llu sigma %llu\n", v, (unsigned long long)(tw0 - t0),
                 (unsigned long long)(tw1 - t0), (unsigned long long)(tw2 - t0), (unsigned long long)(wall_clock64() - t0));
#endif
      }
    }
    __syncthreads();
    HYP_MARK("views");
    // ---- global pair (:268-291) on the whole block when T is large
    if (!global_on_wave) {
      auto btree = [&](int64_t nn, auto leaf) -> double { return block_tree64(nn, leaf); };
      const auto g = global_pair(btree);
      __syncthreads();
      if (tid == 0) { put_hyp(3 * V, g.first); put_hyp(3 * V + 1, g.second); }
    }
    __syncthreads();
  }
  HYP_MARK("mh");
  // ---- coefficients of the next sweep (frozen state): log(2 pi tau_v) on
  //      thread v, then every dish of every view in one pass ----
  __shared__ double s_L2pt[MVC_MAXV];
  if (tid < V) {
    const double L = mvc_log((2.0 * MVC_PI) * hyp[tid]);
    s_L2pt[tid] = L;
    A.L2pt[tid] = L;
    A.cnew[tid] = (double)D * (-0.5 * L);
  }
  __syncthreads();
  for (int k = tid; k < s_koff[V]; k += kHypThreads) {
    int v = 0;
    while (k >= s_koff[v + 1]) ++v;
    const int j = k - s_koff[v];
    const bool mine = k == tid;   // (the Q loop's first dish of this thread)
    const Coef c = coef(mine ? dn_me : P.d_n[v * KC + j], mine ? q_me : P.Q[v * KC + j], hyp[v], s_L2pt[v], D);
    P.c0[v * KC + j] = c.c0;
    P.cb[v * KC + j] = c.cb;
  }
  const double sg = hyp[3 * V + 1];
  for (int p = tid; p < T; p += kHypThreads) P.lmass[p] = mvc_log((double)(p == tid ? nt_me : P.n_t[p]) - sg);
  HYP_MARK("coef");
#undef HYP_MARK
}
extern "C" __global__ __launch_bounds__(kHypThreads) void mvc_par_hyper_kernel(MHArgs A) { hyper_body(A); }
// The same for several chains (one block per chain): the chain-batched sweep
extern "C" __global__ __launch_bounds__(kHypThreads) void mvc_par_hyper_kernel_b(const MHArgs *As) {
  MHArgs A = As[blockIdx.x];
  hyper_body(A);
}

// Every chain's sample of a chain set in one snapshot (blockIdx.y = chain):
// z [n], the tables' raw dish ids d_id[v][dish[v][p]] for p < T (T from the
// status row), the hyperparameters [3V + 2] and T.
struct SnapArgs {
  const int32_t *z, *dish, *did, *status;
  const double *hyp;
  int32_t TC, KC;
};
extern "C" __global__ void mvc_par_snapshot_all_kernel(const SnapArgs *As, int n, int V, int dcap, int32_t *dz,
                                                       int32_t *ddish, int32_t *dT, double *dhyp) {
  const int c = blockIdx.y;
  const SnapArgs S = As[c];
  const int T = S.status[0];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dz[(size_t)c * n + i] = S.z[i];
  if (blockIdx.x == 0) {
    const int H = 3 * V + 2;
    for (int k = threadIdx.x; k < V * dcap; k += blockDim.x) {
      const int v = k / dcap, p = k - v * dcap;
      ddish[(size_t)c * V * dcap + k] = p < T ? S.did[(size_t)v * S.KC + S.dish[(size_t)v * S.TC + p]] : 0;
    }
    for (int k = threadIdx.x; k < H; k += blockDim.x) dhyp[(size_t)c * H + k] = S.hyp[k];
    if (threadIdx.x == 0) dT[c] = T;
  }
}

// ===========================================================================
// Host side of the parallel schedule.
// ===========================================================================
#include <algorithm>
#include <cstdio>
#include <exception>
#include <memory>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mvc_host.h"

namespace mvc {

namespace {
constexpr int kParTC = 1 << 18;   // table capacity (three-level tree64 of the MH's global EPPF)
constexpr int kParKC = (1 << 18) - 1;   // live dishes per view (+1 new element: three-level tree64)
constexpr size_t kLpbBudget = (size_t)1 << 28;   // phase-1 lp buffer: 2 GiB of doubles per batch
constexpr int kSeqWaves = 1024;    // waves of the repair eval grid (SeqArgs.G)
constexpr int kSeqWmin = 1024;     // repair window after a mover
constexpr int kSeqWmax = 1 << 16;  // cap of the window doubling over mover-free stretches
constexpr int kSeqRunLimit = 64;   // stays in a row after which the run kernel hands over to grid windows
constexpr size_t kSeqLdsBudget = 150 * 1024;   // run kernel: per-wave LDS scratch of all its waves
// the lane-per-customer loop of small chains (mvc_seq_run_kernel<5>): customers,
// dims, tables (its evaluation's registers) and dishes per view it takes on
constexpr int kLaneMaxN = 1024, kLaneMaxD = 16, kLaneMaxV = 8, kLaneTM = 32, kLaneMaxK = 32;   // (V: one view per lane of 8)
constexpr int kWideGridMax = 256;  // grid-wide evaluation: at most this many blocks per customer
constexpr int kWideBatch = 32;     // grid-wide evaluation: customers (lp + fin pairs) per repair round
constexpr int kWideFinLds = 152 * 1024;   // the fin kernel's dynamic LDS (wide_fin_resample: dish list, block totals)

template <class Tp>
Tp *dmalloc(size_t count) {
  void *p = nullptr;
  const size_t bytes = sizeof(Tp) * std::max<size_t>(count, 1);
  MVC_HIP(hipMalloc(&p, bytes));
  if (poison_byte() >= 0) MVC_HIP(hipMemset(p, poison_byte(), bytes));
  return (Tp *)p;
}
}  // namespace

int poison_byte() {
  static const int b = [] {
    const char *e = getenv("MVC_POISON");
    return (e && e[0]) ? (int)(strtol(e, nullptr, 0) & 0xFF) : -1;
  }();
  return b;
}
// MVC_LDS_FILL=<byte>: the repair run kernel fills its LDS with that byte at
// launch (diagnostics: a read of LDS the launch never wrote becomes
// deterministic); -1 when unset
int lds_fill_byte() {
  static const int b = [] {
    const char *e = getenv("MVC_LDS_FILL");
    return (e && e[0]) ? (int)(strtol(e, nullptr, 0) & 0xFF) : -1;
  }();
  return b;
}
// MVC_RUN_CHECK=1: the repair run kernels check every index their commits
// write through and report the first bad one (Repair::dbg) instead of storing
bool run_check() {
  static const bool on = [] {
    const char *e = getenv("MVC_RUN_CHECK");
    return e && e[0] == '1';
  }();
  return on;
}
// MVC_DEBUG_SYNC=1|2 (see ParallelSampler::dbg): the level, 0 when unset
int debug_sync_level() {
  static const int l = [] {
    const char *e = getenv("MVC_DEBUG_SYNC");
    return e ? atoi(e) : 0;
  }();
  return l;
}
bool debug_sync() { return debug_sync_level() >= 1; }

class ParallelSampler : public Sampler {
 public:
  int n, V, D, TC, KC, nchunk;
  double *y = nullptr, *Y2 = nullptr;
  double *yt = nullptr;            // MFMA A-fragment layout of y (z-kernel)
  int SP = 0;                      // k-steps per view in yt / S1t (0: no MFMA path)
  struct Chain {
    ParState P{};
    double *L2pt = nullptr, *cnew = nullptr;
    int32_t *Koff = nullptr, *status = nullptr;
    int32_t *choice = nullptr;
    int32_t *pos_new = nullptr, *jmap = nullptr;   // compaction maps [TC], [V*KC]
    Repair *R = nullptr;                           // repair state (mvc_repair.h), device
    int32_t last[4] = {0, 0, 0, 0};                // repair counters of the last sweep (repair_stats)
    double *S1t = nullptr;         // MFMA B-fragment layout of S1 (K_v <= 64)
    // pinned host sources of the async uploads ([V+1] Koff, then [MAXV] view
    // list): pageable sources would make each copy a blocking staged copy that
    // waits for the stream.  The next write to them happens after the next
    // sweep's status synchronisation, so they outlive the copies.
    int32_t *hpin = nullptr;
    bool s1t_ok = false;
    bool s1t_stale = false;        // S1 changed in a chain-batched lane sweep: S1t rebuilt before the next phase A
    int T = 0;
    std::vector<int32_t> K;
    uint32_t gid = 0;
    std::vector<void *> owned;
  };
  std::vector<Chain> chains;
  double *seq_scr = nullptr;      // repair eval scratch (SeqScratch), kSeqWaves waves
  int64_t seq_stride = 0;
  Repair *rs_host = nullptr;      // pinned copy of a chain's Repair after each batch
  hipEvent_t rs_ev = nullptr;     // recorded after that copy (the host waits on it, not on the stream)
  double *lpb = nullptr;          // phase-1 lp buffer (lpb_index layout)
  double *vmax = nullptr;         // [V][n] view maxima of the draw (producer -> draw)
  double *zsc = nullptr;          // generic draw: table scores [T][batch] (mvc_par_zdraw_kernel<true>)
  size_t zsc_cap = 0;             // doubles
  size_t lpb_cap = 0;             // doubles
  size_t lp_cap = 0;               // doubles per wave
  double *part1 = nullptr, *part2 = nullptr;
  size_t part_cap = 0;             // sumK capacity of partials
  int32_t *st_host = nullptr;   // pinned [2V+4]: the per-sweep status readback
  bool force_generic = false;
  bool force_zdraw_lds = false;   // MVC_PATH zdraw=lds: the LDS-checkpoint draw kernel for every T
  bool force_zdraw_row = false;   // zdraw=row: the row draw for every T <= 512 (default: 64 < T <= 512)
  bool no_zrow_lds = false;       // zdraw=row-global: the row draw reads the lp buffer directly
  static constexpr size_t zsc_max_bytes = (size_t)1 << 30;   // the checkpoint draw's table-score scratch limit
  // within-chain N-sharding (mvc_sampler_set_shard): phase A covers this
  // rank's customers only; exch_cb all-gathers the choices into shard_exch
  int shard_rank = 0, shard_world = 1;
  bool first_in_draw = false;     // this sweep's register draw reduced the first mover into Repair::fmin
  int32_t *shard_exch = nullptr;
  int (*shard_cb)(void *) = nullptr;
  void *shard_user = nullptr;
  bool no_lpall = false;          // MVC_PATH lpall=0: per-view producer launches even where the all-views producer applies
  bool phase_a_only = false;      // sweep_chain stops after phase A (mvc_sampler_phase_a)
  bool phase_a_ran = false;
  int n_cu = 256;
  bool repair_grid_only = false;  // MVC_PATH repair=grid: every mover through a grid window round (no run kernel)
  bool force_big = false;         // big=1: the dish-block producer even where the tiled one applies (tests)
  bool big_runtime_sp = false;    // big_sp=runtime: the dish-block producer's runtime k-step loop only (tests)
  bool big_group = true;          // big_group=0: one launch per dish block (y re-read per block) instead of the XCD-grouped launch
  static constexpr int big_bpc_narrow = 3;   // 4-wave blocks per CU of the dish-block producer's 16 / 32-dish instances
  static constexpr int run_limit = kSeqRunLimit;
  // waves=N: customers the run kernel evaluates per step.  4 by default:
  // one evaluating wave per SIMD (a second wave on a SIMD halves the first
  // customer's issue rate, and with dense movers the first customer decides)
  int run_waves = 4;
  bool use_wide = true;           // wide=0: global-scratch run kernel speculates one customer per wave
  bool wide_grid = true;          // wide=block: the wide evaluation on the run kernel's one block instead of the grid
  double *wide_part = nullptr;    // grid-wide evaluation: per-block partials [kWideGridMax][2V]
  int wide_fin_lds = kWideFinLds; // the fin kernel's LDS evaluation up to this many bytes (wide_fin=0: off)
  bool force_global = false;      // run_lds=0: the run kernel's global-scratch layout (tests)
  bool use_lc = true;             // lc=0: the run kernel's per-wave evaluation without the lane-column form
  bool use_lane = true;           // lc=col: no lane-per-customer loop for small chains (lane columns instead)
  bool lane_now = false;          // this sweep runs the lane-per-customer loop (sweep_pre)
  bool use_vp = true;             // vp=0: the lane-column kernel without value prediction
  // Small chains (n <= small_n_plain, MVC_PATH small_plain=N): the lane-column loop without value
  // prediction and a stay limit of 16. At the reference's own call (N = 200, V = 5) the
  // prediction waves' overlay evaluation costs more per step than the steps it saves
  // (1,578 -> 2,262 sweeps/s, profiles/r5af_*); at N = 1M (the literal) it is worth 1.5x.
  int small_n_plain = 1024;
  static constexpr int small_first_rounds = 4;   // the first batch of repair rounds of a small chain
  bool vp_stats = false;          // vp_stats=1: value prediction's steps and hits per sweep on stderr

  // MVC_DEBUG_SYNC=1: wait for the launch just made and name it in the error;
  // =2: also read the chain state back and check its invariants (z against
  // the table counts, dish indices against the dish lists, the dish table /
  // customer counts), naming the first launch after which one fails
  void dbg(const char *what, const Chain &c, uint32_t s, bool rep = true) {
    if (!debug_sync()) return;
    hipError_t e = hipStreamSynchronize(stream);
    if (e == hipSuccess) e = hipGetLastError();
    const std::string where = std::string(what) + " (chain " + std::to_string(c.gid) + ", sweep " +
                              std::to_string(s) + ", T " + std::to_string(c.T) + ")";
    if (e != hipSuccess) throw Error(MVC_ERR_HIP, "debug sync after " + where + ": " + hipGetErrorString(e));
    if (debug_level() >= 2) {
      const std::string bad = check_state(c, rep);
      if (!bad.empty()) throw Error(MVC_ERR_STATE, "state check after " + where + ": " + bad);
    }
  }
  static int debug_level() { return debug_sync_level(); }
  // Invariants of a chain's state between launches:
  // positions p < T (R->T; table slots are stable within a sweep), dishes
  // j < Klist[v]; every customer in a table, n_t = members, d_l = live tables
  // per dish, d_n = customers per dish.  Empty string when they hold.
  // rep: within a sweep's repair (bounds R->T, R->Klist), else between
  // sweeps (the status row's T and Kact).
  std::string check_state(const Chain &c, bool rep) {
    Repair R;
    MVC_HIP(hipMemcpy(&R, c.R, sizeof(Repair), hipMemcpyDeviceToHost));
    std::vector<int32_t> z(n), nt(TC), dish((size_t)V * TC), dl((size_t)V * KC), dn((size_t)V * KC), st(2 * V + 4),
        kact(V);
    MVC_HIP(hipMemcpy(z.data(), c.P.z, 4 * z.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(nt.data(), c.P.n_t, 4 * nt.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(dish.data(), c.P.dish, 4 * dish.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(dl.data(), c.P.d_l, 4 * dl.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(dn.data(), c.P.d_n, 4 * dn.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(st.data(), c.status, 4 * st.size(), hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(kact.data(), c.P.Kact, 4 * kact.size(), hipMemcpyDeviceToHost));
    const int T = rep ? R.T : st[0];
    std::vector<int> K(V);
    for (int v = 0; v < V; ++v) K[v] = rep ? R.Klist[v] : kact[v];
    auto msg = [](const std::string &a, long long x, long long y, long long w) {
      return a + " " + std::to_string(x) + " " + std::to_string(y) + " " + std::to_string(w);
    };
    if (T < 1 || T > TC) return msg("T out of range (T, TC, -)", T, TC, 0);
    for (int v = 0; v < V; ++v)
      if (K[v] < 1 || K[v] > KC) return msg("K out of range (v, K, KC)", v, K[v], KC);
    std::vector<int64_t> cnt(T, 0);
    for (int i = 0; i < n; ++i) {
      if (z[i] < 0 || z[i] >= T) return msg("z out of range (i, z, T)", i, z[i], T);
      cnt[z[i]]++;
    }
    for (int p = 0; p < T; ++p)
      if (cnt[p] != nt[p]) return msg("n_t != members (p, n_t, members)", p, nt[p], cnt[p]);
    for (int v = 0; v < V; ++v) {
      std::vector<int64_t> l(K[v], 0), m(K[v], 0);
      for (int p = 0; p < T; ++p) {
        if (nt[p] <= 0) continue;
        const int j = dish[(size_t)v * TC + p];
        if (j < 0 || j >= K[v]) return msg("dish out of range (v, p, j)", v, p, j);
        l[j]++;
        m[j] += nt[p];
      }
      for (int j = 0; j < K[v]; ++j) {
        if (l[j] != dl[(size_t)v * KC + j]) return msg("d_l != live tables (v, j, d_l)", v, j, dl[(size_t)v * KC + j]);
        if (m[j] != dn[(size_t)v * KC + j]) return msg("d_n != customers (v, j, d_n)", v, j, dn[(size_t)v * KC + j]);
      }
    }
    if (rep && (R.cur < 0 || R.cur > n)) return msg("repair cursor out of range (cur, n, -)", R.cur, n, 0);
    return "";
  }

  template <class Tp>
  Tp *own(Chain &c, size_t count) {
    Tp *p = dmalloc<Tp>(count);
    c.owned.push_back(p);
    return p;
  }

  ParallelSampler(const mvc_config &cf, const double *const *views) {
    std::vector<double> yh((size_t)cf.n_views * cf.n * cf.dim);
    for (int v = 0; v < cf.n_views; ++v)
      std::memcpy(&yh[(size_t)v * cf.n * cf.dim], views[v], sizeof(double) * (size_t)cf.n * cf.dim);
    init(cf, yh.data(), nullptr);
  }
  // yh: the views, contiguous [V][n][D] on the host.  share: another
  // sampler on the same device and data whose device copies of y, Y2 and the
  // MFMA tiling this one reads instead of making its own (ChainSet).
  ParallelSampler(const mvc_config &cf, const double *yh, const ParallelSampler *share) { init(cf, yh, share); }
  // data already on the device (mvc_sampler_create_synthetic): takes ownership
  ParallelSampler(const mvc_config &cf, DeviceData &&dd) {
    y = dd.y;
    Y2 = dd.Y2;
    dd.y = dd.Y2 = nullptr;
    tau0 = dd.tau0;
    init(cf, nullptr, nullptr, true);
  }

  bool owns_y = true;
  bool owns_stream = true;
  std::vector<double> tau0;        // device data: initial tau_v per view (host data: from the views)
  void init(const mvc_config &cf, const double *yh_in, const ParallelSampler *share, bool dev_data = false) {
    cfg = cf;
    n = cf.n; V = cf.n_views; D = cf.dim;
    // initial capacities (mvc_config.table_cap / dish_cap); a birth beyond
    // them grows every chain (grow_capacity), up to kParTC / kParKC
    TC = std::min(kParTC, std::max(16, cf.table_cap > 0 ? cf.table_cap : 1024));
    KC = std::min(kParKC, std::max(15, cf.dish_cap > 0 ? cf.dish_cap : 1023));
    nchunk = (n + 4095) / 4096;
    if (V > MVC_MAXV) throw Error(MVC_ERR_UNSUPPORTED, "at most 64 views");
    MVC_HIP(hipSetDevice(cf.device));
    {   // the sweep loop waits on the device once per sweep (new T, K): spin
        // instead of yielding so the GPU idles as briefly as possible.  The
        // flag applies to the current device (set just above), and only
        // before that device's context exists; otherwise it is left as is.
      (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
      (void)hipGetLastError();
    }
    if (share && n <= kLaneMaxN) {
      // a chain of a set of small chains (ChainSet) works on the set's first
      // chain's stream: their sweeps are one batched stream of launches
      // (ChainSet::sweep_batched, lane_batch) and a stream costs ~20 ms to
      // create, which a short call of many small chains would pay per chain
      stream = share->stream;
      owns_stream = false;
    } else {
      MVC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }
    timers.stream = stream;
    timers.on = (cf.flags & MVC_FLAG_TIMING) != 0;
    timers.coarse = (cf.flags & MVC_FLAG_TIMING_COARSE) != 0;
    vmax = dmalloc<double>((size_t)V * n);
    if (share) {   // the data arrays of another sampler (constant after its construction)
      owns_y = false;
      y = share->y;
      Y2 = share->Y2;
      yt = share->yt;
      SP = share->SP;
      tau0 = share->tau0;
    } else if (dev_data) {
      // y and Y2 were made on the device (owned from here on)
    } else {
      y = dmalloc<double>((size_t)V * n * D);
      Y2 = dmalloc<double>((size_t)V * n);
      MVC_HIP(hipMemcpyAsync(y, yh_in, sizeof(double) * (size_t)V * n * D, hipMemcpyHostToDevice, stream));
      hipLaunchKernelGGL(mvc_par_y2_kernel, dim3(1024), dim3(256), 0, stream, n, V, D, (const double *)y, Y2);
      MVC_HIP(hipGetLastError());
    }
    // the MFMA tiling yt is a second copy of y: build it only when it fits
    // beside y with room for the lp buffer and the chains' state (at N = 10M,
    // D = 256 the two copies would not fit in 288 GB; the generic producer
    // then runs on y alone)
    size_t yt_bytes = 0;
    if (!share && D % 4 == 0 && D >= 16 && V <= MVC_Z_VMAX) {
      const int sp = ((D / 4 + MVC_ZR - 1) / MVC_ZR) * MVC_ZR;
      yt_bytes = sizeof(double) * (size_t)V * (((size_t)n + 15) / 16) * sp * 64;
      size_t mfree = 0, mtotal = 0;
      MVC_HIP(hipMemGetInfo(&mfree, &mtotal));
      const size_t reserve = sizeof(double) * kLpbBudget + (size_t)cf.n_chains * ((size_t)V * n * 32 + ((size_t)1 << 30));
      if (yt_bytes + reserve > mfree) yt_bytes = 0;
    }
    if (yt_bytes) {
      SP = ((D / 4 + MVC_ZR - 1) / MVC_ZR) * MVC_ZR;
      const size_t ntile = ((size_t)n + 15) / 16;
      yt = dmalloc<double>((size_t)V * ntile * SP * 64);
      hipLaunchKernelGGL(mvc_par_ytile_kernel, dim3(4096), dim3(256), 0, stream, n, V, D, SP, (const double *)y, yt);
      MVC_HIP(hipGetLastError());
    }
    MVC_HIP(hipHostMalloc((void **)&st_host, sizeof(int32_t) * (2 * V + 4), hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&rs_host, sizeof(Repair), hipHostMallocDefault));
    alloc_seq_scratch();
    std::fill(st_host, st_host + 2 * V + 4, 0);
    // execution-path overrides (MVC_PATH, tests and A/B runs)
    force_generic = path_int("generic", 0) == 1;
    if (const char *e = path_opt("zdraw")) {
      force_zdraw_lds = std::strcmp(e, "lds") == 0;
      force_zdraw_row = std::strncmp(e, "row", 3) == 0;
      no_zrow_lds = std::strcmp(e, "row-global") == 0;
    }
    no_lpall = path_int("lpall", 1) == 0;
    {
      hipDeviceProp_t prop;
      MVC_HIP(hipGetDeviceProperties(&prop, cf.device));
      n_cu = std::max(1, prop.multiProcessorCount);
    }
    for (const void *f : {(const void *)mvc_par_zdraw_kernel<true>, (const void *)mvc_par_zdraw_kernel<false>})
      MVC_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    lpview_attr<4, 4>();
    lpview_attr<8, 8>();
    lpview_attr<16, 8>();
    lpview_attr<0, 4>();
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_stats_partial_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    lpall_attr<4, 4>();
    lpall_attr<8, 8>();
    lpall_attr<16, 8>();
    // (instance 2 runs the global-scratch layout only: no dynamic LDS)
    for (const void *f : {(const void *)mvc_seq_run_kernel<0>, (const void *)mvc_seq_run_kernel<3>,
                          (const void *)mvc_seq_run_kernel<4>, (const void *)mvc_seq_run_kernel<5>,
                          (const void *)mvc_seq_run_kernel<6>, (const void *)mvc_seq_run_kernel_b<0>,
                          (const void *)mvc_seq_run_kernel_b<3>, (const void *)mvc_seq_run_kernel_b<4>,
                          (const void *)mvc_seq_run_kernel_b<6>})
      MVC_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSeqLdsBudget));   // + the kernel's static LDS <= 160 KB
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_seq_wide_fin_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kWideFinLds));
    if (path_int("wide_fin", 1) == 0) wide_fin_lds = 0;   // the global-scratch evaluation
    if (const char *e = path_opt("repair")) repair_grid_only = std::strcmp(e, "grid") == 0;
    force_big = path_int("big", 0) == 1;
    for (const void *f : {(const void *)mvc_par_zdraw_row_kernel<4, true>, (const void *)mvc_par_zdraw_row_kernel<8, true>,
                          (const void *)mvc_par_zdraw_row_kernel<16, true>, (const void *)mvc_par_zdraw_row_kernel<32, true>})
      MVC_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
#define MVC_LPBIG_FNS(NTB_)                                                                            \
  (const void *)mvc_par_lpbig_kernel<NTB_, 0>, (const void *)mvc_par_lpbig_kernel<NTB_, 16>,             \
      (const void *)mvc_par_lpbig_kernel<NTB_, 32>, (const void *)mvc_par_lpbig_kernel<NTB_, 64>,      \
      (const void *)mvc_par_lpbig_group_kernel<NTB_, 0>, (const void *)mvc_par_lpbig_group_kernel<NTB_, 16>, \
      (const void *)mvc_par_lpbig_group_kernel<NTB_, 32>, (const void *)mvc_par_lpbig_group_kernel<NTB_, 64>
    for (const void *f : {MVC_LPBIG_FNS(4), MVC_LPBIG_FNS(2), MVC_LPBIG_FNS(1)})
      MVC_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#undef MVC_LPBIG_FNS
    big_runtime_sp = path_opt("big_sp") && std::strcmp(path_opt("big_sp"), "runtime") == 0;
    big_group = path_int("big_group", 1) != 0;
    run_waves = std::max(1, std::min(kSeqRunWaves, path_int("waves", run_waves)));
    if (const char *e = path_opt("lc")) {   // 0: neither lane-column nor lane loop; col: lane columns only
      use_lc = e[0] != '0';
      use_lane = use_lc && e[0] != 'c';
    }
    use_vp = path_int("vp", 1) != 0;
    small_n_plain = path_int("small_plain", small_n_plain);
    vp_stats = path_int("vp_stats", 0) == 1;
    if (const char *e = path_opt("wide")) {
      use_wide = e[0] != '0';
      wide_grid = e[0] != 'b';
    }
    force_global = path_int("run_lds", 1) == 0;
    chains.resize(cf.n_chains);
    for (int c = 0; c < cf.n_chains; ++c) init_chain(chains[c], chain_gid(cf, c), yh_in);
    MVC_HIP(hipStreamSynchronize(stream));
  }

  // ---- asynchronous sample output (Sampler::save_async) ----
  static constexpr int kSaveSlots = 4;
  struct SaveSlot {
    int32_t *dz = nullptr, *ddish = nullptr, *ddid = nullptr;   // device snapshot
    double *dhyp = nullptr;
    int32_t *hz = nullptr, *hdish = nullptr, *hdid = nullptr;   // pinned host copy
    double *hhyp = nullptr;
    hipEvent_t snap = nullptr, done = nullptr;
    bool busy = false;
    int chain = 0, T = 0;
    SampleFn fn;
  };
  SaveSlot saves[kSaveSlots];
  int save_next = 0, save_pending = 0;
  hipStream_t cstream = nullptr;

  void finish_slot(SaveSlot &q) {
    MVC_HIP(hipEventSynchronize(q.done));
    std::vector<int32_t> dish_raw((size_t)V * std::max(q.T, 1));
    for (int v = 0; v < V; ++v)
      for (int p = 0; p < q.T; ++p) dish_raw[(size_t)v * q.T + p] = q.hdid[(size_t)v * KC + q.hdish[(size_t)v * TC + p]];
    q.busy = false;
    --save_pending;
    q.fn(q.chain, q.T, q.hz, dish_raw.data(), q.hhyp);
  }

  bool save_async(int chain, const SampleFn &fn) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    Chain &c = chains[chain];
    if (!cstream) MVC_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    // slots are reused in order, so finishing the oldest keeps samples in order
    SaveSlot &q = saves[save_next];
    if (q.busy) finish_slot(q);
    if (!q.dz) {
      q.dz = dmalloc<int32_t>(n);
      q.ddish = dmalloc<int32_t>((size_t)V * TC);
      q.ddid = dmalloc<int32_t>((size_t)V * KC);
      q.dhyp = dmalloc<double>(3 * V + 2);
      MVC_HIP(hipHostMalloc((void **)&q.hz, sizeof(int32_t) * std::max(n, 1), hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hdish, sizeof(int32_t) * (size_t)V * TC, hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hdid, sizeof(int32_t) * (size_t)V * KC, hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hhyp, sizeof(double) * (3 * V + 2), hipHostMallocDefault));
      MVC_HIP(hipEventCreateWithFlags(&q.snap, hipEventDisableTiming));
      MVC_HIP(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
    }
    MVC_HIP(hipMemcpyAsync(q.dz, c.P.z, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, stream));
    MVC_HIP(hipMemcpyAsync(q.ddish, c.P.dish, sizeof(int32_t) * (size_t)V * TC, hipMemcpyDeviceToDevice, stream));
    MVC_HIP(hipMemcpyAsync(q.ddid, c.P.d_id, sizeof(int32_t) * (size_t)V * KC, hipMemcpyDeviceToDevice, stream));
    MVC_HIP(hipMemcpyAsync(q.dhyp, c.P.hyper, sizeof(double) * (3 * V + 2), hipMemcpyDeviceToDevice, stream));
    MVC_HIP(hipEventRecord(q.snap, stream));
    MVC_HIP(hipStreamWaitEvent(cstream, q.snap, 0));
    MVC_HIP(hipMemcpyAsync(q.hz, q.dz, sizeof(int32_t) * n, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hdish, q.ddish, sizeof(int32_t) * (size_t)V * TC, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hdid, q.ddid, sizeof(int32_t) * (size_t)V * KC, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hhyp, q.dhyp, sizeof(double) * (3 * V + 2), hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipEventRecord(q.done, cstream));
    q.busy = true;
    q.chain = chain;
    q.T = c.T;
    q.fn = fn;
    ++save_pending;
    save_next = (save_next + 1) % kSaveSlots;
    return true;
  }

  void flush_saves() override {
    for (int k = 0; k < kSaveSlots && save_pending > 0; ++k) {
      SaveSlot &q = saves[(save_next + k) % kSaveSlots];   // oldest first
      if (q.busy) finish_slot(q);
    }
  }

  // Buffers replaced while sweeping (capacity growth, scratch resizes) are
  // retired, not freed: hipFree / hipHostFree synchronise the whole device,
  // which would stall every other chain sharing the GPU (ChainSet) behind
  // this chain's growth.  They are freed with the handle, or once they add
  // up to more than 4 GiB.
  std::vector<void *> retired_dev, retired_host;
  size_t retired_bytes = 0;
  void retire(void *p, size_t bytes = 0) {
    if (!p) return;
    retired_dev.push_back(p);
    retired_bytes += bytes;
    if (retired_bytes > ((size_t)4 << 30)) free_retired();
  }
  void retire_host(void *p) {
    if (p) retired_host.push_back(p);
  }
  void free_retired() {
    for (void *p : retired_dev) hipFree(p);
    for (void *p : retired_host) hipHostFree(p);
    retired_dev.clear();
    retired_host.clear();
    retired_bytes = 0;
  }

  ~ParallelSampler() override {
    if (stream) hipStreamSynchronize(stream);
    if (cstream) hipStreamSynchronize(cstream);
    free_retired();
    for (SaveSlot &q : saves) {
      for (void *p : {(void *)q.dz, (void *)q.ddish, (void *)q.ddid, (void *)q.dhyp})
        if (p) hipFree(p);
      for (void *p : {(void *)q.hz, (void *)q.hdish, (void *)q.hdid, (void *)q.hhyp})
        if (p) hipHostFree(p);
      if (q.snap) hipEventDestroy(q.snap);
      if (q.done) hipEventDestroy(q.done);
    }
    if (cstream) hipStreamDestroy(cstream);
    for (auto &c : chains) {
      for (void *p : c.owned) hipFree(p);
      if (c.hpin) hipHostFree(c.hpin);
    }
    if (owns_y)
      for (void *p : {(void *)y, (void *)Y2, (void *)yt})
        if (p) hipFree(p);
    for (void *p : {(void *)seq_scr, (void *)lpb, (void *)part1, (void *)part2, (void *)vmax,
                    (void *)zsc, (void *)wide_part})
      if (p) hipFree(p);
    if (st_host) hipHostFree(st_host);
    if (rs_host) hipHostFree(rs_host);
    if (rs_ev) hipEventDestroy(rs_ev);
    if (stream && owns_stream) hipStreamDestroy(stream);
  }

  // capacity-sized arrays of a chain (TC tables, KC dishes per view)
  void alloc_cap(Chain &c) {
    ParState &P = c.P;
    P.TC = TC; P.KC = KC;
    P.n_t = own<int32_t>(c, TC);
    P.dish = own<int32_t>(c, (size_t)V * TC);
    P.d_id = own<int32_t>(c, (size_t)V * KC);
    P.d_n = own<int32_t>(c, (size_t)V * KC);
    P.d_l = own<int32_t>(c, (size_t)V * KC);
    P.S1T = own<double>(c, (size_t)V * D * KC);
    P.S2 = own<double>(c, (size_t)V * KC);
    P.Q = own<double>(c, (size_t)V * KC);
    P.c0 = own<double>(c, (size_t)V * KC);
    P.cb = own<double>(c, (size_t)V * KC);
    P.lmass = own<double>(c, TC);
    c.pos_new = own<int32_t>(c, TC);
    c.jmap = own<int32_t>(c, (size_t)V * KC);
  }

  void alloc_chain(Chain &c) {
    ParState &P = c.P;
    P.n = n; P.V = V; P.D = D;
    P.z = own<int32_t>(c, n);
    alloc_cap(c);
    P.hyper = own<double>(c, 3 * V + 2);
    P.Kact = own<int32_t>(c, V);
    P.next_id = own<int32_t>(c, V);
    P.Ltot = own<int32_t>(c, V);
    c.L2pt = own<double>(c, V);
    c.cnew = own<double>(c, V);
    c.Koff = own<int32_t>(c, V + 1);
    c.status = own<int32_t>(c, 2 * V + 4);
    c.choice = own<int32_t>(c, n);
    c.R = own<Repair>(c, 1);
    MVC_HIP(hipHostMalloc((void **)&c.hpin, sizeof(int32_t) * (V + 1 + MVC_MAXV), hipHostMallocDefault));
  }

  void init_chain(Chain &c, uint32_t gid, const double *yh) {
    c.gid = gid;
    alloc_chain(c);
    InitState S;
    if (yh) {
      S = draw_initial_state(yh, n, V, D, cfg.seed, gid);
    } else {   // device data: the same draws, tau_v from the device's column sums
      S = draw_initial_draws(n, V, cfg.seed, gid);
      S.tau = tau0;
    }
    // multiview_gibbs.cpp:12-98 in dense-position / live-list form
    std::vector<int32_t> nt(4, 0);
    for (int i = 0; i < n; ++i) nt[S.table[i]]++;
    std::vector<int32_t> dish((size_t)V * TC, 0), did((size_t)V * KC, 0), dn((size_t)V * KC, 0), dl((size_t)V * KC, 0);
    c.K.assign(V, 0);
    std::vector<int32_t> next(V, 2);
    std::vector<double> hyp(3 * V + 2);
    for (int v = 0; v < V; ++v) {
      int l2[2] = {0, 0}, map2[2] = {-1, -1};
      for (int t = 0; t < 4; ++t) l2[S.dish_raw[v * 4 + t]]++;
      for (int k = 0; k < 2; ++k)
        if (l2[k] > 0) { map2[k] = c.K[v]; did[v * KC + c.K[v]] = k; dl[v * KC + c.K[v]] = l2[k]; c.K[v]++; }
      for (int t = 0; t < 4; ++t) {
        const int j = map2[S.dish_raw[v * 4 + t]];
        dish[(size_t)v * TC + t] = j;
        dn[v * KC + j] += nt[t];
      }
      hyp[v] = S.tau[v];
      hyp[V + v] = 1.0;
      hyp[2 * V + v] = 0.5;
    }
    hyp[3 * V] = 1.0;
    hyp[3 * V + 1] = 0.6;
    c.T = 4;
    ParState &P = c.P;
    auto up = [&](void *dst, const void *src, size_t bytes) {
      MVC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    };
    up(P.z, S.table.data(), sizeof(int32_t) * n);
    up(P.n_t, nt.data(), sizeof(int32_t) * 4);
    up(P.dish, dish.data(), sizeof(int32_t) * dish.size());
    up(P.d_id, did.data(), sizeof(int32_t) * did.size());
    up(P.d_n, dn.data(), sizeof(int32_t) * dn.size());
    up(P.d_l, dl.data(), sizeof(int32_t) * dl.size());
    up(P.Kact, c.K.data(), sizeof(int32_t) * V);
    up(P.next_id, next.data(), sizeof(int32_t) * V);
    up(P.hyper, hyp.data(), sizeof(double) * hyp.size());
    std::vector<int32_t> st(2 * V + 4, 0);   // status: T, K[V], -, -, T_ne (set by the hyper kernel)
    st[0] = 4;
    for (int v = 0; v < V; ++v) st[1 + v] = c.K[v];
    up(c.status, st.data(), sizeof(int32_t) * st.size());
    MVC_HIP(hipStreamSynchronize(stream));
    rebuild_stats(c);
    launch_hyper(c, 0, 0);
  }

  int sumK(const Chain &c) const {
    int s = 0;
    for (int k : c.K) s += k;
    return s;
  }

  void upload_koff(Chain &c) {
    int32_t *koff = c.hpin;
    koff[0] = 0;
    for (int v = 0; v < V; ++v) koff[v + 1] = koff[v] + c.K[v];
    MVC_HIP(hipMemcpyAsync(c.Koff, koff, sizeof(int32_t) * (V + 1), hipMemcpyHostToDevice, stream));
  }


  // Full chunked rebuild of the views in vmask.
  void rebuild_views(Chain &c, uint64_t vmask) {
    const int sk = sumK(c);
    if ((size_t)sk > part_cap) {
      retire(part1);
      retire(part2);
      part_cap = (size_t)sk + 64;
      part1 = dmalloc<double>((size_t)nchunk * part_cap * D);
      part2 = dmalloc<double>((size_t)nchunk * part_cap);
    }
    int Kmax = 1;
    for (int k : c.K) Kmax = std::max(Kmax, k);
    const size_t lds = sizeof(int) * (2 * 4096 + (size_t)Kmax + 1);
    hipLaunchKernelGGL(mvc_par_stats_partial_kernel, dim3(nchunk, V), dim3(256), lds, stream, c.P, (const double *)y,
                       (const double *)Y2, (const int32_t *)c.Koff, (int)part_cap, vmask, part1, part2);
    MVC_HIP(hipGetLastError());
    const size_t tot = (size_t)sk * (D + 1);
    hipLaunchKernelGGL(mvc_par_stats_combine_kernel, dim3((unsigned)std::min<size_t>(4096, (tot + 255) / 256)), dim3(256),
                       0, stream, c.P, (const int32_t *)c.Koff, (int)part_cap, nchunk, vmask, (const double *)part1,
                       (const double *)part2);
    MVC_HIP(hipGetLastError());
  }

  void tile_s1(Chain &c) {
    c.s1t_stale = false;
    int Kmax = 1;
    for (int k : c.K) Kmax = std::max(Kmax, k);
    c.s1t_ok = false;
    if (SP > 0 && Kmax <= MVC_Z_KMAX) {
      if (!c.S1t) c.S1t = own<double>(c, (size_t)V * SP * 4 * 64);
      hipLaunchKernelGGL(mvc_par_s1tile_kernel, dim3(256), dim3(256), 0, stream, c.P, (const int32_t *)c.Koff, SP,
                         c.S1t);
      MVC_HIP(hipGetLastError());
      c.s1t_ok = true;
    }
  }

  // initial state / set_state: every view from scratch
  void rebuild_stats(Chain &c) {
    upload_koff(c);
    hipEvent_t ev = nullptr;
    timers.begin("stats", &ev);
    rebuild_views(c, V >= 64 ? ~0ull : ((1ull << V) - 1));
    tile_s1(c);
    timers.end("stats", ev);
  }

  MHArgs mh_args(const Chain &c, int do_mh, uint32_t sweep_ix, const Repair *gate = nullptr, int gate_mode = 0) const {
    MHArgs A;
    A.P = c.P;
    A.status = c.status;
    A.Koff = c.Koff;
    A.L2pt = c.L2pt;
    A.cnew = c.cnew;
    A.seed = cfg.seed;
    A.chain = c.gid;
    A.sweep = sweep_ix;
    A.do_mh = do_mh;
    A.gate = gate;
    A.gate_mode = gate_mode;
    return A;
  }
  void launch_hyper(Chain &c, int do_mh, uint32_t sweep_ix, const Repair *gate = nullptr, int gate_mode = 0) {
    const MHArgs A = mh_args(c, do_mh, sweep_ix, gate, gate_mode);
    hipEvent_t ev = nullptr;
    timers.begin("hyper", &ev);
    hipLaunchKernelGGL(mvc_par_hyper_kernel, dim3(1), dim3(kHypThreads), 0, stream, A);
    MVC_HIP(hipGetLastError());
    if (!gate) dbg("hyper", c, sweep_ix, false);   // (the gated launch runs behind the outcome copy: synced by its caller)
    timers.end("hyper", ev);
  }

  // per-wave global scratch of the repair's grid windows: kSeqWaves waves,
  // fewer when tables / dishes number in the tens of thousands (<= 2 GiB)
  int seq_waves = kSeqWaves;
  void alloc_seq_scratch() {
    retire(seq_scr, sizeof(double) * (size_t)seq_waves * seq_stride);
    seq_stride = seq_scratch_stride(V, TC, KC);
    const int64_t fit = ((int64_t)1 << 28) / seq_stride;
    seq_waves = (int)std::max<int64_t>(kSeqRunWaves, std::min<int64_t>(kSeqWaves, fit / 4 * 4));
    seq_scr = dmalloc<double>((size_t)seq_waves * seq_stride);
  }

  SeqArgs make_seq(Chain &c, uint32_t s) {
    SeqArgs A;
    A.P = c.P;
    A.y = y;
    A.Y2 = Y2;
    A.L2pt = c.L2pt;
    A.cnew = c.cnew;
    A.choice = c.choice;
    A.status = c.status;
    A.Koff = c.Koff;
    A.R = c.R;
    A.scr = seq_scr;
    A.scr_stride = seq_stride;
    // eval grid waves: one per scratch slot, and no more than one per customer
    // (a small chain's windows cover the whole sweep; idle blocks cost dispatch)
    A.G = std::min(seq_waves, std::max(4, (n + 3) / 4 * 4));
    A.Wmin = kSeqWmin;
    A.Wmax = kSeqWmax;
    A.seed = cfg.seed;
    A.chain = c.gid;
    A.sweep = s;
    return A;
  }

  Sweep make_sweep(Chain &c, uint32_t s) {
    Sweep A;
    A.fmin = nullptr;
    A.P = c.P;
    A.y = y;
    A.Y2 = Y2;
    A.L2pt = c.L2pt;
    A.cnew = c.cnew;
    A.Koff = c.Koff;
    A.choice = c.choice;
    A.status = c.status;
    A.yt = yt;
    A.S1t = c.S1t;
    A.SP = SP;
    A.vmax = vmax;
    A.T = c.T;
    A.sumK = sumK(c);
    A.seed = cfg.seed;
    A.chain = c.gid;
    A.sweep = s;
    return A;
  }

  // waves per block of the MFMA producer: 4, two blocks per CU = 2 waves per
  // SIMD.  Measured (scripts/lpv_sweep.py, D = 128, K = 64/32/16/8): more
  // waves per SIMD only contend for the f64 MFMA pipe and the load queue
  // (lp 1.11 ms at 4x2, 1.12 at 4x3 / 4x4, 1.22 at 6x2, 1.36 at 2x4).
  int lpview_waves(int) const { return 4; }
  template <int SPPT, int RP>
  void launch_lpview_nt(int NT, dim3 grid, dim3 block, size_t lds, const Sweep &A, int v, int b0, int nb) {
    double *disc = lpb + lpb_cap;
    switch (NT) {
      case 1: hipLaunchKernelGGL((mvc_par_lpview_kernel<1, SPPT, RP>), grid, block, lds, stream, A, v, b0, nb, lpb, disc); break;
      case 2: hipLaunchKernelGGL((mvc_par_lpview_kernel<2, SPPT, RP>), grid, block, lds, stream, A, v, b0, nb, lpb, disc); break;
      case 3: hipLaunchKernelGGL((mvc_par_lpview_kernel<3, SPPT, RP>), grid, block, lds, stream, A, v, b0, nb, lpb, disc); break;
      default: hipLaunchKernelGGL((mvc_par_lpview_kernel<4, SPPT, RP>), grid, block, lds, stream, A, v, b0, nb, lpb, disc); break;
    }
  }
  // SP (k-steps per tile) is a multiple of 8: pairs per tile SPP = SP / 2
  void launch_lpview(int NT, dim3 grid, dim3 block, size_t lds, const Sweep &A, int v, int b0, int nb) {
    switch (SP / 2) {
      case 4: launch_lpview_nt<4, 4>(NT, grid, block, lds, A, v, b0, nb); break;
      case 8: launch_lpview_nt<8, 8>(NT, grid, block, lds, A, v, b0, nb); break;
      case 16: launch_lpview_nt<16, 8>(NT, grid, block, lds, A, v, b0, nb); break;
      default: launch_lpview_nt<0, 4>(NT, grid, block, lds, A, v, b0, nb); break;
    }
  }
  template <int SPPT, int RP>
  static void lpview_attr() {
    for (const void *f : {(const void *)mvc_par_lpview_kernel<1, SPPT, RP>, (const void *)mvc_par_lpview_kernel<2, SPPT, RP>,
                          (const void *)mvc_par_lpview_kernel<3, SPPT, RP>, (const void *)mvc_par_lpview_kernel<4, SPPT, RP>})
      MVC_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  }

  template <int SPPT, int RP>
  void launch_lpall(uint32_t pat, dim3 grid, dim3 block, size_t lds, const Sweep &A, int b0, int nb) {
    double *disc = lpb + lpb_cap;
    switch (pat) {
#define X(p)                                                                                       \
  case p:                                                                                          \
    hipLaunchKernelGGL((mvc_par_lpall_kernel<SPPT, RP, p>), grid, block, lds, stream, A, b0, nb, lpb, disc); \
    break;
      MVC_FZ_PATS(X)
#undef X
      default: throw Error(MVC_ERR_STATE, "all-views producer: no instance for this view pattern");
    }
  }
  template <int SPPT, int RP>
  static void lpall_attr() {
#define X(p)                                                                                            \
  MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_lpall_kernel<SPPT, RP, p>,                          \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    MVC_FZ_PATS(X)
#undef X
  }
  void sweep_chain(Chain &c, uint32_t s) {
    bool phaseA = false;
    if (sweep_pre(c, s, phaseA)) repair(c, s, phaseA);
  }
  // A sweep up to the repair: phase A (producer + draw) of this rank's
  // customers and, when sharded, the exchange of the choices.  false: the
  // caller stops here (mvc_sampler_phase_a).
  bool sweep_pre(Chain &c, uint32_t s, bool &phaseA_out) {
    // small chains: the run kernel's lane-per-customer loop runs the whole
    // sweep from customer 0 (its first step is phase A)
    lane_now = lane_sweep(c);
    if (!lane_now && c.s1t_stale) {   // after chain-batched lane sweeps (ChainSet::sweep_batched)
      c.s1t_stale = false;
      tile_s1(c);
    }
    Sweep A = make_sweep(c, s);
    const SeqArgs Q0 = make_seq(c, s);
    hipLaunchKernelGGL(mvc_seq_init_kernel, dim3(1), dim3(64), 0, stream, Q0, lane_now ? 1 : 0);
    MVC_HIP(hipGetLastError());
    dbg("seq_init", c, s);
    if (lane_now) {
      zpath = 32 | 256;
      phaseA_out = false;
      return true;
    }
    hipEvent_t e0 = nullptr;
    // phase 1 in customer batches: lp producer (MFMA or generic), then draw
    int Kmax = 0, Kmin = 1 << 30;
    for (int k : c.K) { Kmax = std::max(Kmax, k); Kmin = std::min(Kmin, k); }
    const int sk = sumK(c);
    const bool use_mfma = !force_generic && !force_big && c.s1t_ok && Kmin >= 1 && Kmax <= MVC_Z_KMAX &&
                          lpview_shared_bytes(SP, (Kmax + 15) / 16, Kmax, c.T) <= 160 * 1024;
    // the dish-block MFMA producer (y read directly) where the tiled path does
    // not apply: the widest dish block whose B-fragments fit, 8 waves per block
    // (one block per CU) when they take more than half the LDS, else 4 waves
    // and two blocks per CU -- two waves per SIMD either way
    const int SPb = ((D / 4 + MVC_ZR - 1) / MVC_ZR) * MVC_ZR;
    int big_ntb = 0, big_waves = 4;
    for (int nt : {4, 2, 1}) {
      if (big_ntb) break;
      if (lpbig_shared_bytes(SPb, nt, c.T, 4) <= 80 * 1024) { big_ntb = nt; big_waves = 4; }
      else if (lpbig_shared_bytes(SPb, nt, c.T, 8) <= 150 * 1024) { big_ntb = nt; big_waves = 8; }
    }
    const bool use_big = !use_mfma && !force_generic && D % 4 == 0 && D >= 16 && Kmin >= 1 && big_ntb > 0;
    // batch: multiple of 64 customers, lp buffer <= kLpbBudget doubles
    const size_t per64 = (size_t)std::max(1, sk) * 64;
    size_t nb_max = std::max<size_t>(64, (kLpbBudget / per64) * 64);
    const size_t nb_full = ((size_t)n + 63) / 64 * 64;
    const size_t nbatch_sz = std::min(nb_max, nb_full);
    const size_t need = (nbatch_sz / 64) * per64;
    const bool use_zreg = !force_zdraw_lds && !force_zdraw_row && c.T <= 64 && Kmax <= 64 && sk <= MVC_Z_VMAX * 64 &&
                          zdraw_reg_shared_bytes(V, 64, sk) <= 64 * 1024;
    // the row draw (16 lanes per customer) where the register draw does not
    // apply; lane v of a customer's row holds view v's scalars, so V <= 16
    const int row_nb = c.T <= 64 ? 4 : c.T <= 128 ? 8 : c.T <= 256 ? 16 : 32;
    const bool use_zrow = !use_zreg && !force_zdraw_lds && c.T <= 512 && V <= 16 &&
                          zdraw_row_shared_bytes(V, row_nb, sk, false) <= 64 * 1024;
    // the row draw with its slab in LDS where two blocks fit a CU
    const bool zrow_lds = use_zrow && !no_zrow_lds && zdraw_row_shared_bytes(V, row_nb, sk, true) <= 80 * 1024;
    // phase A on the two-kernel path needs the draw's LDS tables; beyond them
    // the repair's eval kernel evaluates the sweep from customer 0 instead
    const bool phaseA = use_zreg || use_zrow || zdraw_shared_bytes(V, c.T, sk) <= 160 * 1024;
    // the all-views producer: T <= 64, K_v <= 64, every view's S1
    // B-fragments in LDS at once, fully unrolled k-step pairs
    size_t s1t_d = 0;
    for (int v = 0; v < V; ++v) s1t_d += (size_t)SP * 64 * ((c.K[v] + 15) / 16);
    const int spp = SP / 2;
    uint32_t fz_pat = (uint32_t)V;
    for (int v = 0; v < V && v < 4; ++v) fz_pat |= (uint32_t)(std::min(4, (c.K[v] + 15) / 16) - 1) << (4 + 2 * v);
    bool pat_ok = V <= 4 && Kmax <= 64;
    switch (pat_ok ? fz_pat : 0u) {
#define X(p) case p:
      MVC_FZ_PATS(X)
#undef X
      break;
      default: pat_ok = false;
    }
    if (phaseA && need > lpb_cap) {
      retire(lpb, sizeof(double) * (lpb_cap + 128));
      lpb_cap = need;
      lpb = dmalloc<double>(lpb_cap + 128);   // + 128: the producers' per-lane discard slots (16 B per lane)
    }
    bool zpath_lpall = false;
    timers.begin("zresample", &e0);
    // this rank's customers [lo, hi) (the whole chain unless sharded)
    const size_t S = (size_t)shard_len(n, shard_world);
    const size_t lo = std::min((size_t)n, (size_t)shard_rank * S), hi = std::min((size_t)n, lo + S);
    for (size_t b0 = lo; phaseA && b0 < hi; b0 += nbatch_sz) {
      const int nb = (int)std::min(nbatch_sz, hi - b0);
      hipEvent_t el = nullptr, ed = nullptr;
      timers.begin("lp", &el);
      const size_t lpa_lds = lpall_shared_bytes(s1t_d, V, sk, MVC_LPA_WAVES);
      const bool use_lpall = !no_lpall && use_mfma && pat_ok && c.T <= 16 * MVC_FZ_TB &&
                             (spp == 4 || spp == 8 || spp == 16) && lpa_lds <= 160 * 1024;
      if (use_lpall) {
        const int ntile = (nb + 15) / 16;
        const int grid = std::max(1, std::min(n_cu, (ntile + MVC_LPA_WAVES - 1) / MVC_LPA_WAVES));
        switch (spp) {
          case 4: launch_lpall<4, 4>(fz_pat, dim3(grid), dim3(64 * MVC_LPA_WAVES), lpa_lds, A, (int)b0, nb); break;
          case 8: launch_lpall<8, 8>(fz_pat, dim3(grid), dim3(64 * MVC_LPA_WAVES), lpa_lds, A, (int)b0, nb); break;
          default: launch_lpall<16, MVC_LPA_RP16>(fz_pat, dim3(grid), dim3(64 * MVC_LPA_WAVES), lpa_lds, A, (int)b0, nb); break;
        }
        zpath_lpall = true;
      } else if (use_mfma) {
        const int ntile = (nb + 15) / 16;
        for (int v = 0; v < V; ++v) {
          const int NT = (c.K[v] + 15) / 16;
          const size_t lds = lpview_shared_bytes(SP, NT, c.K[v], c.T);
          const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / std::max<size_t>(lds, 1)));
          const int bw = lpview_waves(NT);
          const int grid = std::max(1, std::min(per_cu * n_cu, (ntile + bw - 1) / bw));
          launch_lpview(NT, dim3(grid), dim3(64 * bw), lds, A, v, (int)b0, nb);
          MVC_HIP(hipGetLastError());
        }
      } else if (use_big) {
        // K_v > 64 or no tiled copy: dish blocks of 16 * NTB, A-fragments from y
        const int ntile = (nb + 15) / 16;
        for (int v = 0; v < V; ++v) {
          // a view with few dishes takes the narrowest block that holds them
          // (the MFMAs of the padding columns are not issued); the blocks'
          // lp values and the max-combined view maximum are the same bits
          // whatever the blocking
          int vntb = big_ntb;
          while (vntb > 1 && 16 * (vntb / 2) >= c.K[v]) vntb /= 2;
          int vwaves = big_waves;
          if (vntb != big_ntb) vwaves = lpbig_shared_bytes(SPb, vntb, c.T, 4) <= 80 * 1024 ? 4 : 8;
          const int nblk = (c.K[v] + 16 * vntb - 1) / (16 * vntb);
          if (big_group && nblk >= 2) {
            // every dish block of the view in one launch, XCD-grouped (y read once)
            const size_t lds = lpbig_shared_bytes(SPb, vntb, c.T, vwaves);
            int per_cu = vwaves == 8 ? 1 : (vntb <= 2 ? big_bpc_narrow : 2);
            per_cu = std::max(1, std::min<int>(per_cu, (int)((160 * 1024) / std::max<size_t>(lds, 1))));
            const int grid = per_cu * n_cu;
            if (n_cu % 8 == 0 && grid / 8 >= nblk) {
              hipLaunchKernelGGL(mvc_par_vmax_fill_kernel, dim3(std::min(1024, (nb + 255) / 256)), dim3(256), 0, stream,
                                 A.vmax + (size_t)v * n + b0, nb);
              Sweep Ab = A;
              Ab.SP = SPb;
              const int spc = (4 * SPb == D && !big_runtime_sp && (SPb == 16 || SPb == 32 || SPb == 64)) ? SPb : 0;
#define MVC_LPBIG(NTB_, SPC_)                                                                                        \
  hipLaunchKernelGGL((mvc_par_lpbig_group_kernel<NTB_, SPC_>), dim3(grid), dim3(64 * vwaves), lds, stream, Ab, v, nblk, \
                     (int)b0, nb, lpb, lpb + lpb_cap)
#define MVC_LPBIG_SP(NTB_)         \
  switch (spc) {                   \
    case 16: MVC_LPBIG(NTB_, 16); break; \
    case 32: MVC_LPBIG(NTB_, 32); break; \
    case 64: MVC_LPBIG(NTB_, 64); break; \
    default: MVC_LPBIG(NTB_, 0); break;  \
  }
              switch (vntb) {
                case 4: MVC_LPBIG_SP(4) break;
                case 2: MVC_LPBIG_SP(2) break;
                default: MVC_LPBIG_SP(1) break;
              }
#undef MVC_LPBIG_SP
#undef MVC_LPBIG
              MVC_HIP(hipGetLastError());
              continue;
            }
          }
          for (int jb0 = 0, first = 1; jb0 < c.K[v]; jb0 += 16 * vntb, first = 0) {
            const int kb = std::min(16 * vntb, c.K[v] - jb0);
            const size_t lds = lpbig_shared_bytes(SPb, vntb, c.T, vwaves);
            // blocks per CU: the register budget allows three 4-wave blocks of the
            // narrow instances (<= 168 VGPRs), two of the 64-dish one; LDS permitting
            int per_cu = vwaves == 8 ? 1 : (vntb <= 2 ? big_bpc_narrow : 2);
            per_cu = std::max(1, std::min<int>(per_cu, (int)((160 * 1024) / std::max<size_t>(lds, 1))));
            const int grid = std::max(1, std::min(per_cu * n_cu, (ntile + vwaves - 1) / vwaves));
            Sweep Ab = A;
            Ab.SP = SPb;
            // the unrolled instance where D = 4 SP exactly (no padded k-steps)
            const int spc = (4 * SPb == D && !big_runtime_sp && (SPb == 16 || SPb == 32 || SPb == 64)) ? SPb : 0;
#define MVC_LPBIG(NTB_, SPC_)                                                                                   \
  hipLaunchKernelGGL((mvc_par_lpbig_kernel<NTB_, SPC_>), dim3(grid), dim3(64 * vwaves), lds, stream, Ab, v, jb0, kb, \
                     first, (int)b0, nb, lpb, lpb + lpb_cap)
#define MVC_LPBIG_SP(NTB_)         \
  switch (spc) {                   \
    case 16: MVC_LPBIG(NTB_, 16); break; \
    case 32: MVC_LPBIG(NTB_, 32); break; \
    case 64: MVC_LPBIG(NTB_, 64); break; \
    default: MVC_LPBIG(NTB_, 0); break;  \
  }
            switch (vntb) {
              case 4: MVC_LPBIG_SP(4) break;
              case 2: MVC_LPBIG_SP(2) break;
              default: MVC_LPBIG_SP(1) break;
            }
#undef MVC_LPBIG_SP
#undef MVC_LPBIG
            MVC_HIP(hipGetLastError());
          }
        }
      } else {
        hipLaunchKernelGGL(mvc_par_lpgen_kernel, dim3(std::min(4096, (nb + 255) / 256)), dim3(256), 0, stream, A,
                           (int)b0, nb, lpb);
      }
      MVC_HIP(hipGetLastError());
      dbg("lp producer", c, s, false);
      timers.end("lp", el);
      timers.begin("draw", &ed);
      const dim3 zg((nb + 255) / 256);   // the register kernel takes one customer per thread
      // the register draw finds the first mover itself when it sees every customer (no shard)
      first_in_draw = use_zreg && shard_world == 1;
      A.fmin = first_in_draw ? &c.R->fmin : nullptr;
      if (use_zreg && c.T <= 16)
        hipLaunchKernelGGL(mvc_par_zdraw_reg_kernel<16>, zg, dim3(256), zdraw_reg_shared_bytes(V, 16, sk), stream, A,
                           (int)b0, nb, (const double *)lpb);
      else if (use_zreg && c.T <= 32)
        hipLaunchKernelGGL(mvc_par_zdraw_reg_kernel<32>, zg, dim3(256), zdraw_reg_shared_bytes(V, 32, sk), stream, A,
                           (int)b0, nb, (const double *)lpb);
      else if (use_zreg)
        hipLaunchKernelGGL(mvc_par_zdraw_reg_kernel<64>, zg, dim3(256), zdraw_reg_shared_bytes(V, 64, sk), stream, A,
                           (int)b0, nb, (const double *)lpb);
      else if (use_zrow) {
        // 16 customers (one slab) per block and round
        const dim3 rg(std::max(1, std::min((nb + 15) / 16, (zrow_lds ? 2 : 8) * n_cu)));
        const size_t rl = zdraw_row_shared_bytes(V, row_nb, sk, zrow_lds);
        const double *lc = lpb;
#define MVC_ZROW(NBV)                                                                                      \
  if (zrow_lds) hipLaunchKernelGGL((mvc_par_zdraw_row_kernel<NBV, true>), rg, dim3(256), rl, stream, A, (int)b0, nb, lc); \
  else hipLaunchKernelGGL((mvc_par_zdraw_row_kernel<NBV, false>), rg, dim3(256), rl, stream, A, (int)b0, nb, lc);
        switch (row_nb) {
          case 4: MVC_ZROW(4) break;
          case 8: MVC_ZROW(8) break;
          case 16: MVC_ZROW(16) break;
          default: MVC_ZROW(32) break;
        }
#undef MVC_ZROW
      } else {
        // the table-score scratch (T x nb doubles) when it stays under 1 GiB
        const size_t scn = (size_t)c.T * (size_t)nb;
        const bool use_sc = scn * sizeof(double) <= zsc_max_bytes;
        if (use_sc && scn > zsc_cap) {
          retire(zsc, sizeof(double) * zsc_cap);
          zsc_cap = scn + scn / 2;
          zsc = dmalloc<double>(zsc_cap);
        }
        if (use_sc)
          hipLaunchKernelGGL(mvc_par_zdraw_kernel<true>, dim3(std::min(4096, (nb + 255) / 256)), dim3(256),
                             zdraw_shared_bytes(V, c.T, sk), stream, A, (int)b0, nb, (const double *)lpb, zsc);
        else
          hipLaunchKernelGGL(mvc_par_zdraw_kernel<false>, dim3(std::min(4096, (nb + 255) / 256)), dim3(256),
                             zdraw_shared_bytes(V, c.T, sk), stream, A, (int)b0, nb, (const double *)lpb, zsc);
      }
      MVC_HIP(hipGetLastError());
      dbg("z draw", c, s, false);
      timers.end("draw", ed);
    }
    timers.end("zresample", e0);
    if (phase_a_only) {                            // mvc_sampler_phase_a: the pass alone
      phase_a_ran = phaseA;
      zpath = phaseA ? ((use_mfma ? 2 : 0) | (use_zreg ? 4 : 0) | (zpath_lpall ? 16 : 0) | (use_big ? 64 : 0) |
                        (use_zrow ? 128 : 0)) : 32;
      return false;
    }
    if (phaseA && shard_world > 1) {
      // the other ranks' phase-A choices: this shard into the exchange buffer,
      // the caller's all-gather (synchronous), every shard back.  Each rank
      // then runs the same repair on the same state: no other exchange.
      if (hi > lo)
        MVC_HIP(hipMemcpyAsync(shard_exch + lo, c.choice + lo, (hi - lo) * sizeof(int32_t), hipMemcpyDeviceToDevice,
                               stream));
      MVC_HIP(hipStreamSynchronize(stream));
      // a failed exchange stops the sweep here: nothing has read the buffer
      // and phase A changed no chain state (only choice / lp / vmax)
      if (shard_cb(shard_user) != 0)
        throw Error(MVC_ERR_CALLBACK, "set_shard: the all_gather callback reported failure; the sweep was not run");
      MVC_HIP(hipMemcpyAsync(c.choice, shard_exch, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, stream));
    }
    zpath = phaseA ? ((use_mfma ? 2 : 0) | (use_zreg ? 4 : 0) | (zpath_lpall ? 16 : 0) |
                      (use_big ? 64 : 0) | (use_zrow ? 128 : 0)) : 32;
    phaseA_out = phaseA;
    return true;
  }

  // The small chains' lane-per-customer loop (mvc_seq_run_kernel<5>, L.lc ==
  // 3): the state cache with S1, tables up to kLaneTM (the evaluation's
  // registers), dish lists with room to double, and a ring holding the whole
  // sweep's rows; no per-wave scratch.  L.lc == 0: it does not fit.
  SeqLds lane_layout(int T, const int32_t *Klist) const {
    int kmax = 1;
    for (int v = 0; v < V; ++v) kmax = std::max(kmax, (int)Klist[v]);
    SeqLds L{};
    L.limit = kNoWindows;
    L.ks = (kmax + std::max(16, kmax) + 15) / 32 * 32 + 16;
    L.ts = kLaneTM;
    L.s1 = 1;
    L.cache_dbl = seq_lds_cache(V, D, L.ks, L.ts, true);
    L.stride = 0;
    L.nws = kSeqLcThreads / 64;
    int rn = 2;
    while (rn < n) rn *= 2;
    if (T >= L.ts || 8 * (L.cache_dbl + (int64_t)rn * seq_ring_slot(V, D)) > (int64_t)kSeqLdsBudget) return L;
    L.lds = 1;
    L.tw = 1;
    L.ring = rn;
    L.pfn = 0;
    L.vpo = 0;
    L.lc = 3;
    L.small = (T <= kLaneSmall && kmax <= kLaneSmall) ? 1 : 0;
    return L;
  }
  // the layout of a repair round: the lane loop while this sweep runs it and
  // the state still fits it, else the run kernels' (run_layout)
  SeqLds pick_layout(int T, const int32_t *Klist, bool vp_ok) const {
    if (lane_now) {
      bool ok = T < kLaneTM;
      for (int v = 0; v < V; ++v) ok = ok && Klist[v] <= kLaneMaxK;
      if (ok) {
        const SeqLds L = lane_layout(T, Klist);
        if (L.lc == 3) return L;
      }
    }
    return run_layout(T, Klist, vp_ok);
  }
  bool lane_sweep(const Chain &c) const {
    if (!use_lane || force_global || repair_grid_only || phase_a_only || shard_world > 1) return false;
    if (n > kLaneMaxN || D > kLaneMaxD || V > kLaneMaxV || c.T >= kLaneTM) return false;
    for (int k : c.K)
      if (k > kLaneMaxK) return false;
    return lane_layout(c.T, c.K.data()).lc == 3;
  }

  // LDS layout of the run kernel's per-wave scratch for T tables and dish
  // lists Klist, with room for growth (a birth past it makes the kernel exit
  // with R->restride; the host then relaunches with a new layout).  Falls back
  // to the per-wave global scratch when even a few waves do not fit.
  SeqLds run_layout(int T, const int32_t *Klist, bool vp_ok = true) const {
    int kmax = 1;
    for (int v = 0; v < V; ++v) kmax = std::max(kmax, (int)Klist[v]);
    SeqLds L{};
    // small chains: the run kernel walks the whole sweep (a window round is a
    // launch triple and a host read-back, more than the steps it saves)
    L.limit = n <= small_n_plain ? 16 : run_limit;
    // in order of preference: S1 cached with room to double (a cold sweep's
    // births then rarely restride; in a chain batch a restride ends the round
    // for every chain), S1 cached with room to grow by half, then without S1,
    // then tight margins without S1
    for (int attempt = force_global ? 4 : 0; attempt < 4; ++attempt) {
      const bool s1 = attempt <= 1;
      const int kgrow = attempt == 0 ? std::max(16, kmax) : attempt < 3 ? std::max(8, kmax / 2) : 4;
      const int tgrow = attempt == 0 ? std::max(128, T) : attempt < 3 ? std::max(64, T / 2) : 16;
      // ks = 16 (mod 32): the lane-column evaluation's rows (views) read dish
      // j of [v][ks] arrays at v ks + j, so rows 0 / 1 (and 2 / 3) of a
      // ds_read_b64 lane group then fall on disjoint banks (2 ks dwords = 32
      // mod 64), and of a ds_read_b32 too (ks = 16 mod 32)
      L.ks = (kmax + kgrow + 15) / 32 * 32 + 16;
      L.ts = (T + tgrow + 63) / 64 * 64;   // whole 64-table chunks (the lane-column evaluation's e[] scratch)
      if (attempt == 0 && use_lc && L.ts > 64 * kLcChunks) continue;   // doubling would leave the lane-column form
      L.s1 = s1 ? 1 : 0;
      L.cache_dbl = seq_lds_cache(V, D, L.ks, L.ts, s1);
      L.stride = seq_lds_stride(V, D, L.ks, L.ts);
      const int64_t room = (int64_t)kSeqLdsBudget / 8 - L.cache_dbl;
      const int cap = run_waves;   // customers per step
      L.nws = room > 0 ? (int)std::min<int64_t>(cap, room / L.stride) : 0;
      if (L.nws >= std::min(cap, s1 ? 4 : 2)) {
        L.lds = 1;
        L.tw = 1;
        L.lc = 0;   // the lane-column kernel needs the ring (set below)
        // the staged-row ring in what is left: a power of two >= 2 nws customers
        const int64_t slot = seq_ring_slot(V, D);
        const int64_t left = room - (int64_t)L.nws * L.stride;
        int rn = 0;
        for (int r = 256; r >= 2 * L.nws; r >>= 1)
          if ((int64_t)r * slot <= left) { rn = r; break; }
        L.ring = rn;
        L.pfn = rn ? std::max(1, rn / 2) : 0;
        L.lc = (use_lc && s1 && rn > 0 && L.ts <= 64 * kLcChunks) ? 1 : 0;
        if (L.lc) L.nws = std::min(L.nws, kSeqLcThreads / 64);   // its block has 4 waves
        // value prediction (lc == 2) where its overlay fits: V <= kVpV, every dish list <= 128, and the
        // overlay's S1 columns [kVpE][D] after the ring (which follows the clamped nws scratches)
        L.vpo = L.cache_dbl + (int64_t)L.nws * L.stride + (int64_t)rn * slot;
        if (L.lc && use_vp && vp_ok && n > small_n_plain && V <= kVpV && kmax <= 128 && L.nws >= kSeqLcThreads / 64 &&
            left - (int64_t)rn * slot >= (int64_t)kVpE * D)
          L.lc = 2;
        return L;
      }
    }
    L.lds = 0;   // per-wave global scratch (SeqScratch(A, w)): capacity-sized, never restrides
    L.lc = 0;
    // the whole block on one customer (seq_resample_wide): the dish / table
    // lists are long here, and where the state outgrows the LDS nearly every
    // customer moves (cold-start transients), so speculation buys little
    L.tw = use_wide ? kSeqRunWaves : 1;
    L.s1 = 0;
    L.nws = use_wide ? 1 : run_waves;
    L.stride = 0;
    L.cache_dbl = 0;
    return L;
  }

  // Phase A's choices are exact up to the first customer that does not stay;
  // from there the repair commits movers in customer order (mvc_repair.h,
  // DESIGN.md §4.8), then compaction and the MH.  Each round is the run
  // kernel (dense movers: commit + 8-customer speculation in a device loop)
  // and a grid window (sparse movers).  One host synchronisation per batch of
  // rounds; at steady state a single batch of one round.  A birth beyond the
  // capacity grows every chain and resumes.
  // The in-order repair of one chain, in three parts so
  // that a ChainSet can run the rounds of all its chains as batched launches:
  // repair_start (first mover / first window), the rounds with the outcome
  // read back per batch (repair_outcome), repair_finish (compaction, MH).
  struct RepairRun {
    SeqArgs Q;
    SeqLds L;
    dim3 eg;
    bool vp_ok = true, early_mh = false;
    bool birth_retry = false;   // a capacity growth interrupted a birth: the birth kernel follows the next run kernel
    bool birth_between = false; // the small lane loop: the birth kernel before every round but the batch's first
    int rounds = 1;
    hipEvent_t e1 = nullptr;
  };
  void repair_start(Chain &c, uint32_t s, bool phaseA, RepairRun &rr, bool allow_early_mh = true) {
    timers.begin("repair", &rr.e1);
    rr.Q = make_seq(c, s);
    rr.eg = dim3(rr.Q.G / 4);   // the eval grid: SeqArgs.G waves (re-read after a capacity growth)
    const dim3 eb(256);
    if (phaseA) {
      if (!first_in_draw)
        hipLaunchKernelGGL(mvc_seq_first_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0,
                           stream, n, (const int32_t *)c.choice, (const int32_t *)c.P.z, c.R);
    } else if (!lane_now)
      hipLaunchKernelGGL(mvc_seq_eval_kernel, rr.eg, eb, 0, stream, rr.Q);
    MVC_HIP(hipGetLastError());
    dbg("seq_first / eval", c, s);
    rr.vp_ok = true;   // value prediction until it stops itself in this sweep (R->vpoff)
    rr.L = pick_layout(c.T, c.K.data(), rr.vp_ok);
    // the gated early MH (below) only where no per-phase timers bracket the
    // repair and the MH separately (they would time the MH as repair)
    // (not for small chains: nearly every sweep of theirs moves someone, so the
    // gated launch would be a no-op launch per sweep)
    rr.early_mh = allow_early_mh && (!timers.on || timers.coarse) && n > small_n_plain;
    if (rr.early_mh && !rs_ev) MVC_HIP(hipEventCreateWithFlags(&rs_ev, hipEventDisableTiming));
    // the first batch of rounds: one; small chains four (their repair
    // usually takes 2-5 rounds, and a batch costs a host round trip)
    rr.rounds = (n <= small_n_plain && !lane_now) ? small_first_rounds : 1;
  }
  // The run kernel's dynamic LDS for layout L.
  int64_t run_dyn(const SeqLds &L) const {
    return L.lds ? 8 * (L.cache_dbl + L.stride * L.nws + (int64_t)L.ring * seq_ring_slot(V, D) +
                        (L.lc == 2 ? (int64_t)kVpE * D : 0))
                 : 0;
  }
  // The grid-wide evaluation where the state is on the global layout (L.lds = 0) and
  // the block-wide evaluation applies (L.tw > 1): one customer over many CUs
  bool run_wgrid(const SeqLds &L) const { return !repair_grid_only && wide_grid && L.lds == 0 && L.tw > 1; }
  // rr.rounds repair rounds of one chain on its stream
  void repair_rounds(Chain &c, uint32_t s, RepairRun &rr) {
    const dim3 eb(256);
    SeqLds &L = rr.L;
    const bool wgrid = run_wgrid(L);
    int wblk = 1;
    if (wgrid) {
      if (!wide_part) wide_part = dmalloc<double>((size_t)kWideGridMax * 2 * V);
      // blocks for the dish list (plus the births a round may add): two 64-dish chunks per wave
      int nk = 0;
      for (int k : c.K) nk += k;
      nk += nk / 4 + 64;
      wblk = std::max(1, std::min(kWideGridMax, (nk + 2 * kWideGridThreads - 1) / (2 * kWideGridThreads)));
    }
    for (int r = 0; r < rr.rounds; ++r) {
      if (repair_grid_only)
        hipLaunchKernelGGL(mvc_seq_apply_kernel, dim3(1), dim3(256), 0, stream, rr.Q);
      else if (wgrid) {
        hipLaunchKernelGGL(mvc_seq_wide_begin_kernel, dim3(1), dim3(64), 0, stream, rr.Q);
        for (int b = 0; b < kWideBatch; ++b) {
          hipLaunchKernelGGL(mvc_seq_wide_lp_kernel, dim3(wblk), dim3(kWideGridThreads), 0, stream, rr.Q, wide_part);
          hipLaunchKernelGGL(mvc_seq_wide_fin_kernel, dim3(1), dim3(kSeqRunThreads), wide_fin_lds, stream, rr.Q,
                             (const double *)wide_part, wblk, L.limit, wide_fin_lds);
        }
        MVC_HIP(hipGetLastError());
        dbg("seq_wide (begin + lp/fin pairs)", c, s);
      } else {
        L.dyn = run_dyn(L);
        L.fill = lds_fill_byte();
        L.chk = run_check() ? 1 : 0;
        if (L.lc == 3 && L.small && (rr.birth_retry || (rr.birth_between && r > 0))) {
          // the small lane loop left a birth pending: commit it first (a no-op without one)
          rr.birth_retry = false;
          hipLaunchKernelGGL(mvc_seq_birth_kernel, dim3(1), dim3(kSeqRunThreads), 0, stream, rr.Q);
          MVC_HIP(hipGetLastError());
          dbg("seq_birth", c, s);
        }
        hipLaunchKernelGGL(L.lc ? (L.lc == 3 ? (L.small ? mvc_seq_run_kernel<5> : mvc_seq_run_kernel<6>)
                                             : L.lc == 2 ? mvc_seq_run_kernel<4> : mvc_seq_run_kernel<3>)
                                : L.tw == 1 ? mvc_seq_run_kernel<0> : mvc_seq_run_kernel<2>,
                           dim3(1), dim3(L.lc == 3 && L.small ? kLaneSmallThreads : L.lc ? kSeqLcThreads : kSeqRunThreads),
                           (size_t)L.dyn, stream, rr.Q, L);
      }
      MVC_HIP(hipGetLastError());
      dbg(repair_grid_only ? "seq_apply" : L.lc == 3 ? (L.small ? "seq_run<5>" : "seq_run<6>") : L.lc == 2 ? "seq_run<4>" : L.lc ? "seq_run<3>" : L.tw == 1 ? "seq_run<0>" : "seq_run<2>", c, s);
      if (L.lc && !(L.lc == 3 && L.small) && !repair_grid_only && rr.birth_retry) {   // a birth the loop left pending (births commit in the kernel)
        rr.birth_retry = false;
        hipLaunchKernelGGL(mvc_seq_birth_kernel, dim3(1), dim3(kSeqRunThreads), 0, stream, rr.Q);
        MVC_HIP(hipGetLastError());
        dbg("seq_birth", c, s);
      }
      if (!(L.lc == 3 && !repair_grid_only)) {   // (the lane loop opens no windows)
        hipLaunchKernelGGL(mvc_seq_eval_kernel, rr.eg, eb, 0, stream, rr.Q);
        MVC_HIP(hipGetLastError());
        dbg("seq_eval", c, s);
      }
    }
    MVC_HIP(hipGetLastError());
  }
  // Acts on a batch's outcome rs (read back): 0 run the same rounds again
  // (after a capacity growth / relayout), 1 done, 2 more rounds.
  int repair_outcome(Chain &c, uint32_t s, RepairRun &rr, const Repair &rs) {
    if (rs.dbg[0]) {   // MVC_RUN_CHECK: a run kernel's index check failed
      std::string v;
      for (int k = 1; k < 8; ++k) v += " " + std::to_string(rs.dbg[k]);
      throw Error(MVC_ERR_STATE, "run kernel index check " + std::to_string(rs.dbg[0]) + " failed (chain " +
                                     std::to_string(c.gid) + ", sweep " + std::to_string(s) + ", lc " +
                                     std::to_string(rr.L.lc) + "):" + v);
    }
    if (rs.overflow) {
      rr.birth_retry = true;
      grow_capacity(rs.overflow);
      rr.Q = make_seq(c, s);
      rr.eg = dim3(rr.Q.G / 4);   // the scratch may have fewer slots now
      return 0;
    }
    if (rs.vpoff && rr.vp_ok) {   // predictions missed (or a dish list outgrew them): plain lane columns
      rr.vp_ok = false;
      if (rr.L.lc == 2) rr.L.lc = 1;
    }
    if (rs.restride) {
      rr.L = pick_layout(rs.T, rs.Klist, rr.vp_ok);
      MVC_HIP(hipMemsetAsync(&c.R->restride, 0, sizeof(int32_t), stream));
      return 0;
    }
    if (rs.done) return 1;
    if (rr.L.lc == 3 && rr.L.small && rs.pend && rs.pchoice < 0) rr.birth_retry = true;   // (committed before the next launch)
    rr.rounds = std::min(rr.rounds * 4, 1024);
    return 2;
  }
  void repair_finish(Chain &c, uint32_t s, RepairRun &rr, const Repair &rs, bool sync_status = true) {
    const bool moved = rs.moves > 0;
    if (moved) {
      // small chains: the compaction block relabels z itself (one launch less per sweep)
      const int relabel_in_block = n <= 16384 ? 1 : 0;
      hipLaunchKernelGGL(mvc_seq_compact_kernel, dim3(1), dim3(1024), 0, stream, rr.Q, c.pos_new, c.jmap,
                         relabel_in_block);
      if (!relabel_in_block)
        hipLaunchKernelGGL(mvc_seq_relabel_kernel, dim3(std::max(1, std::min(1024, (n + 255) / 256))), dim3(256), 0,
                           stream, n, c.P.z, (const int32_t *)c.pos_new, (const Repair *)c.R);
      MVC_HIP(hipGetLastError());
      dbg("seq_compact + relabel", c, s, false);
    }
    timers.end("repair", rr.e1);
#ifdef MVC_RUN_PROF
    fprintf(stderr, "runprof moves %d iters %llu | lc: views %.2f tables+weights %.2f draw %.2f | commit %.2f check %.2f spec %.2f decide %.2f (us per iter)\n",
            rs.moves, rs.prof[7], rs.prof[0] * 0.01 / std::max(1ull, rs.prof[7]),
            rs.prof[1] * 0.01 / std::max(1ull, rs.prof[7]), rs.prof[2] * 0.01 / std::max(1ull, rs.prof[7]),
            rs.prof[3] * 0.01 / std::max(1ull, rs.prof[7]), rs.prof[4] * 0.01 / std::max(1ull, rs.prof[7]),
            rs.prof[5] * 0.01 / std::max(1ull, rs.prof[7]), rs.prof[6] * 0.01 / std::max(1ull, rs.prof[7]));
    fprintf(stderr, "runprof decided %llu same-as-phase-A %llu | movers %llu same-as-phase-A %llu\n", rs.prof[8],
            rs.prof[9], rs.prof[10], rs.prof[11]);
    if (rs.prof[18] + rs.prof[19]) {
      const double nd = (double)std::max(1ull, rs.prof[18]), nc = (double)std::max(1ull, rs.prof[19]);
      fprintf(stderr, "wideprof decided %llu commits %llu | combine %.2f lm %.2f tables %.2f weights %.2f draw %.2f (us per decided) "
              "commit %.2f (us per commit)\n", rs.prof[18], rs.prof[19], rs.prof[12] * 0.01 / nd,
              rs.prof[13] * 0.01 / nd, rs.prof[14] * 0.01 / nd, rs.prof[15] * 0.01 / nd,
              rs.prof[16] * 0.01 / nd, rs.prof[17] * 0.01 / nc);
      fprintf(stderr, "wideprof effective shader clock %.0f MHz (%llu clocks over %llu ticks of 100 MHz)\n",
              rs.prof[20] ? 100.0 * (double)rs.prof[21] / (double)rs.prof[20] : 0.0, rs.prof[21],
              rs.prof[20]);
    }
#endif
    if (vp_stats)   // MVC_VP_STATS=1: value prediction's steps and full hits of this sweep, on stderr
      fprintf(stderr, "mvc vp steps %d hits %d off %d\n", rs.vpsteps, rs.vphits, rs.vpoff);
    c.last[0] = rs.moves;
    c.last[1] = rs.births;
    c.last[2] = rs.rounds;
    c.last[3] = rs.newdish;
    if (!(rr.early_mh && !moved)) launch_hyper(c, 1, s);   // else the gated launch above ran it
    if (moved) {   // new T and dish counts for the next sweep's launch shapes
      MVC_HIP(hipMemcpyAsync(st_host, c.status, sizeof(int32_t) * (2 * V + 4), hipMemcpyDeviceToHost, stream));
      if (sync_status) repair_status(c);
      else status_pending = true;
    }
  }
  bool status_pending = false;
  Repair last_rs{};                // the chain-batched sweep's final outcome of this chain
  // the next sweep's launch shapes from the status copied back by repair_finish
  void repair_status(Chain &c) {
    MVC_HIP(hipStreamSynchronize(stream));
    status_pending = false;
    c.T = st_host[0];
    for (int v = 0; v < V; ++v) c.K[v] = st_host[1 + v];
    tile_s1(c);   // S1 changed: the next phase A's MFMA B-fragments
  }
  void repair(Chain &c, uint32_t s, bool phaseA) {
    RepairRun rr;
    repair_start(c, s, phaseA, rr);
#ifndef MVC_RUN_PROF
    if (lane_now && (!timers.on || timers.coarse)) {
      repair_lane_tail(c, s, rr);
      return;
    }
#endif
    for (;;) {
      repair_rounds(c, s, rr);
      MVC_HIP(hipMemcpyAsync(rs_host, c.R, sizeof(Repair), hipMemcpyDeviceToHost, stream));
      if (rr.early_mh) {
        // the MH goes into the stream behind the copy, gated on the device by
        // the repair's outcome (it runs iff the repair is done with no move),
        // so the GPU runs it while the host waits for the copy and decides the
        // next launches; it is a no-op in the other cases, which launch it below
        MVC_HIP(hipEventRecord(rs_ev, stream));
        launch_hyper(c, 1, s, c.R);
        MVC_HIP(hipEventSynchronize(rs_ev));
        dbg("gated hyper", c, s);
      } else {
        MVC_HIP(hipStreamSynchronize(stream));
      }
      if (repair_outcome(c, s, rr, *rs_host) == 1) break;
    }
    repair_finish(c, s, rr, *rs_host);
  }
  // A small chain's lane sweep (one chain swept alone): the sweep's tail --
  // compaction (a no-op on the device unless the repair is done with moves),
  // the status and outcome read-backs, then the MH (gated on the device: it
  // runs iff the repair is done) -- enqueued behind every batch of rounds, so
  // a sweep is one host synchronisation, and the MH runs while the host reads
  // the outcome and prepares the next sweep's launches.  The same kernels on
  // the same state in the same order as repair_finish's.
  void repair_lane_tail(Chain &c, uint32_t s, RepairRun &rr) {
    if (!rs_ev) MVC_HIP(hipEventCreateWithFlags(&rs_ev, hipEventDisableTiming));
    if (rr.L.lc == 3 && rr.L.small) {
      // the small instance ends its launch at a birth (~0.2 per sweep): a
      // birth launch and a second round behind the first, so such a sweep
      // needs no second host round trip (both are no-ops after a sweep
      // without a birth)
      rr.rounds = 2;
      rr.birth_between = true;
    }
    for (;;) {
      repair_rounds(c, s, rr);
      hipLaunchKernelGGL(mvc_seq_compact_kernel, dim3(1), dim3(1024), 0, stream, rr.Q, c.pos_new, c.jmap, 1);
      MVC_HIP(hipMemcpyAsync(st_host, c.status, sizeof(int32_t) * (2 * V + 4), hipMemcpyDeviceToHost, stream));
      MVC_HIP(hipMemcpyAsync(rs_host, c.R, sizeof(Repair), hipMemcpyDeviceToHost, stream));
      MVC_HIP(hipEventRecord(rs_ev, stream));
      launch_hyper(c, 1, s, c.R, 1);
      MVC_HIP(hipEventSynchronize(rs_ev));
      dbg("lane tail (compaction, gated hyper)", c, s);
      if (repair_outcome(c, s, rr, *rs_host) == 1) break;
    }
    const Repair &rs = *rs_host;
    timers.end("repair", rr.e1);
    if (vp_stats) fprintf(stderr, "mvc vp steps %d hits %d off %d\n", rs.vpsteps, rs.vphits, rs.vpoff);
    c.last[0] = rs.moves;
    c.last[1] = rs.births;
    c.last[2] = rs.rounds;
    c.last[3] = rs.newdish;
    if (rs.moves > 0) {   // new T and dish counts for the next sweep's launch shapes (S1t: s1t_stale)
      c.T = st_host[0];
      for (int v = 0; v < V; ++v) c.K[v] = st_host[1 + v];
      c.s1t_stale = true;
    }
  }

  // Double the table (flags & 1) and/or dish (flags & 2) capacity of every
  // chain, keeping the contents (oracle: unbounded, multiview_utils.cpp:
  // 209-216, 251-258).  The repair step that overflowed changed nothing and
  // is redone.
  void grow_capacity(int flags) {
    // the table limit: the MH's three-level tree64 over the table sizes
    // (64^3 = 262,144); MVC_MAX_TABLES lowers it (tests of the limit's error)
    int max_tc = kParTC;
    max_tc = std::max(16, std::min(kParTC, path_int("max_tables", kParTC)));
    const int TC2 = (flags & 1) ? std::min(max_tc, 2 * TC) : TC;
    const int KC2 = (flags & 2) ? std::min(kParKC, 2 * KC + 1) : KC;
    if (TC2 == TC && KC2 == KC)
      throw Error(MVC_ERR_UNSUPPORTED, "parallel mode: a birth needs table " + std::to_string(TC + 1) + " (limit " +
                                           std::to_string(max_tc) + " tables, " + std::to_string(kParKC) +
                                           " dishes per view); the sweep stopped at that customer, so the handle cannot continue");
    flush_saves();
    for (SaveSlot &q : saves) {   // the ring slots are capacity-sized
      for (void *p : {(void *)q.dz, (void *)q.ddish, (void *)q.ddid, (void *)q.dhyp}) retire(p);
      for (void *p : {(void *)q.hz, (void *)q.hdish, (void *)q.hdid, (void *)q.hhyp}) retire_host(p);
      if (q.snap) hipEventDestroy(q.snap);
      if (q.done) hipEventDestroy(q.done);
      q = SaveSlot();
    }
    const int TC1 = TC, KC1 = KC;
    TC = TC2;
    KC = KC2;
    for (Chain &c : chains) {
      const ParState old = c.P;
      std::vector<void *> old_owned;
      std::swap(old_owned, c.owned);
      const int32_t *old_pos = c.pos_new, *old_jmap = c.jmap;
      (void)old_pos; (void)old_jmap;
      alloc_cap(c);
      ParState &P = c.P;
      auto cp2 = [&](void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t rows) {
        MVC_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToDevice, stream));
      };
      cp2(P.n_t, 4 * TC2, old.n_t, 4 * TC1, 4 * TC1, 1);
      cp2(P.dish, 4 * TC2, old.dish, 4 * TC1, 4 * TC1, V);
      cp2(P.lmass, 8 * TC2, old.lmass, 8 * TC1, 8 * TC1, 1);
      cp2(P.d_id, 4 * KC2, old.d_id, 4 * KC1, 4 * KC1, V);
      cp2(P.d_n, 4 * KC2, old.d_n, 4 * KC1, 4 * KC1, V);
      cp2(P.d_l, 4 * KC2, old.d_l, 4 * KC1, 4 * KC1, V);
      cp2(P.S1T, 8 * KC2, old.S1T, 8 * KC1, 8 * KC1, (size_t)V * D);
      cp2(P.S2, 8 * KC2, old.S2, 8 * KC1, 8 * KC1, V);
      cp2(P.Q, 8 * KC2, old.Q, 8 * KC1, 8 * KC1, V);
      cp2(P.c0, 8 * KC2, old.c0, 8 * KC1, 8 * KC1, V);
      cp2(P.cb, 8 * KC2, old.cb, 8 * KC1, 8 * KC1, V);
      MVC_HIP(hipMemsetAsync(&c.R->overflow, 0, sizeof(int32_t), stream));
      MVC_HIP(hipStreamSynchronize(stream));
      // everything not capacity-sized moves over; the old capacity arrays go
      const std::vector<void *> cap_old = {old.n_t, old.dish, old.lmass, old.d_id, old.d_n, old.d_l, old.S1T,
                                           old.S2, old.Q, old.c0, old.cb, (void *)old_pos, (void *)old_jmap};
      for (void *p : old_owned) {
        if (std::find(cap_old.begin(), cap_old.end(), p) != cap_old.end()) retire(p);
        else c.owned.push_back(p);
      }
    }
    alloc_seq_scratch();
  }

  void sweep(int n_sweeps) override {
    for (int it = 0; it < n_sweeps; ++it) {
      hipEvent_t ev = nullptr;
      timers.begin("sweep", &ev);
      for (auto &c : chains) sweep_chain(c, (uint32_t)sweeps_done);
      timers.end("sweep", ev);
      ++sweeps_done;
    }
  }

  void synchronize() override { MVC_HIP(hipStreamSynchronize(stream)); timers.collect(); }

  bool phase_a(int chain, int32_t *out) override {
    if (chains.size() != 1 || chain != 0) return false;
    synchronize();
    Chain &c = chains[0];
    phase_a_only = true;
    try {
      sweep_chain(c, (uint32_t)sweeps_done);
    } catch (...) {
      phase_a_only = false;
      throw;
    }
    phase_a_only = false;
    if (!phase_a_ran) return false;
    MVC_HIP(hipMemcpyAsync(out, c.choice, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    synchronize();
    return true;
  }

  bool set_shard(int rank, int world, int32_t *exch, int (*cb)(void *), void *user) override {
    if (chains.size() > 1) return false;   // one chain per sharded handle (mvc.h)
    if (world < 1 || rank < 0 || rank >= world || (world > 1 && (!exch || !cb)))
      throw Error(MVC_ERR_ARG, "set_shard: rank / world / exchange");
    synchronize();
    shard_rank = rank;
    shard_world = world;
    shard_exch = exch;
    shard_cb = cb;
    shard_user = user;
    return true;
  }
  bool repair_stats(int chain, int32_t *out) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    for (int k = 0; k < 4; ++k) out[k] = chains[chain].last[k];
    return true;
  }

  const int32_t *device_labels(int chain) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    MVC_HIP(hipStreamSynchronize(stream));
    return chains[chain].P.z;
  }

  void copy_rows(int view, const int32_t *idx, int64_t m, double *out) override {
    if (view < 0 || view >= V) throw Error(MVC_ERR_ARG, "copy_rows: view out of range");
    for (int64_t r = 0; r < m; ++r)
      if (idx[r] < 0 || idx[r] >= n) throw Error(MVC_ERR_ARG, "copy_rows: row index out of range");
    MVC_HIP(hipStreamSynchronize(stream));
    gather_rows(y, n, D, view, idx, m, out, stream);
  }

  void get_state(int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of, int32_t dish_cap,
                 double *hyper) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    Chain &c = chains[chain];
    MVC_HIP(hipStreamSynchronize(stream));
    if (n_tables) *n_tables = c.T;
    if (table_of) MVC_HIP(hipMemcpy(table_of, c.P.z, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    if (dish_of) {
      std::vector<int32_t> dish((size_t)V * TC), did((size_t)V * KC);
      MVC_HIP(hipMemcpy(dish.data(), c.P.dish, sizeof(int32_t) * dish.size(), hipMemcpyDeviceToHost));
      MVC_HIP(hipMemcpy(did.data(), c.P.d_id, sizeof(int32_t) * did.size(), hipMemcpyDeviceToHost));
      for (int v = 0; v < V; ++v)
        for (int p = 0; p < std::min(c.T, (int)dish_cap); ++p)
          dish_of[(size_t)v * dish_cap + p] = did[(size_t)v * KC + dish[(size_t)v * TC + p]];
    }
    if (hyper) MVC_HIP(hipMemcpy(hyper, c.P.hyper, sizeof(double) * (3 * V + 2), hipMemcpyDeviceToHost));
  }

  void get_dish_counts(int chain, int32_t *k_out) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    for (int v = 0; v < V; ++v) k_out[v] = chains[chain].K[v];
  }

  void get_stats(int chain, int view, int32_t *K, double *S1, double *S2, int32_t *n_vk, int32_t cap) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    Chain &c = chains[chain];
    MVC_HIP(hipStreamSynchronize(stream));
    const int k = c.K[view];
    if (K) *K = k;
    const int m = std::min<int>(k, cap);
    if (m <= 0) return;
    if (S1) {
      std::vector<double> row((size_t)D * KC);
      MVC_HIP(hipMemcpy(row.data(), c.P.S1T + (size_t)view * D * KC, sizeof(double) * row.size(),
                        hipMemcpyDeviceToHost));
      for (int j = 0; j < m; ++j)
        for (int d = 0; d < D; ++d) S1[(size_t)j * D + d] = row[(size_t)d * KC + j];
    }
    if (S2) MVC_HIP(hipMemcpy(S2, c.P.S2 + (size_t)view * KC, sizeof(double) * m, hipMemcpyDeviceToHost));
    if (n_vk) MVC_HIP(hipMemcpy(n_vk, c.P.d_n + (size_t)view * KC, sizeof(int32_t) * m, hipMemcpyDeviceToHost));
  }

  void set_state(int chain, const int32_t *table_of, int32_t T, const int32_t *dish_of, const double *hyper) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    const UserState U = check_user_state(n, V, table_of, T, dish_of);
    int Kmax = 0;
    for (int v = 0; v < V; ++v) Kmax = std::max(Kmax, (int)U.ids[v].size());
    while (T > TC || Kmax > KC) {
      MVC_HIP(hipStreamSynchronize(stream));
      grow_capacity((T > TC ? 1 : 0) | (Kmax > KC ? 2 : 0));
    }
    Chain &c = chains[chain];
    std::vector<int32_t> dish((size_t)V * TC, 0), did((size_t)V * KC, 0), dn((size_t)V * KC, 0), dl((size_t)V * KC, 0);
    c.K.assign(V, 0);
    for (int v = 0; v < V; ++v) {
      const int K = (int)U.ids[v].size();
      if (K > KC) throw Error(MVC_ERR_UNSUPPORTED, "set_state: too many dishes for the parallel-mode capacity");
      c.K[v] = K;
      for (int j = 0; j < K; ++j) { did[v * KC + j] = U.ids[v][j]; dl[v * KC + j] = U.l[v][j]; }
      for (int p = 0; p < T; ++p) {
        dish[(size_t)v * TC + p] = U.dish[v][p];
        dn[v * KC + U.dish[v][p]] += U.n_t[p];
      }
    }
    MVC_HIP(hipStreamSynchronize(stream));
    ParState &P = c.P;
    auto up = [&](void *dst, const void *src, size_t bytes) {
      MVC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    };
    up(P.z, table_of, sizeof(int32_t) * n);
    up(P.n_t, U.n_t.data(), sizeof(int32_t) * T);
    up(P.dish, dish.data(), sizeof(int32_t) * dish.size());
    up(P.d_id, did.data(), sizeof(int32_t) * did.size());
    up(P.d_n, dn.data(), sizeof(int32_t) * dn.size());
    up(P.d_l, dl.data(), sizeof(int32_t) * dl.size());
    up(P.Kact, c.K.data(), sizeof(int32_t) * V);
    up(P.next_id, U.next_id.data(), sizeof(int32_t) * V);
    up(P.hyper, hyper, sizeof(double) * (3 * V + 2));
    std::vector<int32_t> st(2 * V + 4, 0);
    st[0] = T;
    for (int v = 0; v < V; ++v) st[1 + v] = c.K[v];
    up(c.status, st.data(), sizeof(int32_t) * st.size());
    MVC_HIP(hipStreamSynchronize(stream));
    c.T = T;
    rebuild_stats(c);
    launch_hyper(c, 0, 0);
    MVC_HIP(hipStreamSynchronize(stream));
  }
};

// Several chains on one device, concurrently (BASELINE config 3:
// 8 chains on one MI355X).  Each chain is a one-chain ParallelSampler with
// its own stream, phase-A buffers and repair state, sharing the device copy
// of the data; sweep() drives them from one host thread per chain, so one
// chain's latency-bound repair (one CU) overlaps the others' work.  Chain c
// keeps its global id chain_gid(cfg, c), so every draw is the one the serial
// loop would make: the chains are bitwise the same.
class ChainSet : public Sampler {
 public:
  std::vector<std::unique_ptr<ParallelSampler>> subs;
  ChainSet(const mvc_config &cf, const double *const *views) {
    cfg = cf;
    const int V = cf.n_views, n = cf.n, D = cf.dim;
    std::vector<double> yh((size_t)V * n * D);
    for (int v = 0; v < V; ++v) std::memcpy(&yh[(size_t)v * n * D], views[v], sizeof(double) * (size_t)n * D);
    for (int c = 0; c < cf.n_chains; ++c) {
      mvc_config one = cf;
      one.n_chains = 1;
      one.first_chain = (int32_t)chain_gid(cf, c);
      one.chain_stride = 1;
      subs.emplace_back(new ParallelSampler(one, yh.data(), c == 0 ? nullptr : subs[0].get()));
    }
    stream = subs[0]->stream;
  }
  ChainSet(const mvc_config &cf, DeviceData &&dd) {
    cfg = cf;
    for (int c = 0; c < cf.n_chains; ++c) {
      mvc_config one = cf;
      one.n_chains = 1;
      one.first_chain = (int32_t)chain_gid(cf, c);
      one.chain_stride = 1;
      if (c == 0) subs.emplace_back(new ParallelSampler(one, std::move(dd)));
      else subs.emplace_back(new ParallelSampler(one, nullptr, subs[0].get()));
    }
    stream = subs[0]->stream;
  }
  ~ChainSet() override {
    if (set_cstream) hipStreamSynchronize(set_cstream);
    for (auto &q : set_saves) {
      if (q.snap) hipEventDestroy(q.snap);
      if (q.done) hipEventDestroy(q.done);
      set_slot_free(q);
    }
    if (set_cstream) hipStreamDestroy(set_cstream);
    batch_free();
    while (!subs.empty()) subs.pop_back();   // the data owner (chain 0) last
  }
  template <class F>
  void each(F f) {
    std::vector<std::thread> ts;
    std::vector<std::exception_ptr> errs(subs.size());
    for (size_t c = 0; c < subs.size(); ++c)
      ts.emplace_back([&, c] {
        try {
          MVC_HIP(hipSetDevice(cfg.device));
          f(*subs[c]);
        } catch (...) {
          errs[c] = std::current_exception();
        }
      });
    for (auto &t : ts) t.join();
    for (auto &e : errs)
      if (e) std::rethrow_exception(e);
  }
  ParallelSampler &at(int chain) {
    if (chain < 0 || chain >= (int)subs.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    return *subs[chain];
  }
  void sweep(int n_sweeps) override {
    for (auto &s : subs) {   // timing flags set on the handle apply to every chain
      s->timers.on = timers.on;
      s->timers.coarse = timers.coarse;
    }
    if (batch_on) {
      for (int it = 0; it < n_sweeps; ++it) sweep_batched();
    } else {
      each([&](ParallelSampler &s) { s.sweep(n_sweeps); });
    }
    sweeps_done += n_sweeps;
    zpath = subs[0]->zpath;
  }

  // ---- the chain-batched sweep ----
  // Phase A of every chain on its own stream; then the in-order repair of all
  // chains as batched launches on one stream (the run kernel with one block
  // per chain, the window evaluation with a block range per chain) and one
  // read-back of all chains' outcomes per batch of rounds; then compaction
  // and the MH of every chain on its stream.  The same kernels run on the same
  // state as a chain swept alone, so every chain is the same chain, bit for bit;
  // concurrency no longer needs a hardware queue per chain.
  bool batch_on = [] {
    return path_int("chain_batch", 1) != 0;   // chain_batch=0: one host thread and stream per chain
  }();
  SeqArgs *bA_dev = nullptr, *bA_host = nullptr, *bE_dev = nullptr, *bE_host = nullptr;
  SeqLds *bL_dev = nullptr, *bL_host = nullptr;
  Repair *bR_dev = nullptr, *bR_host = nullptr;
  // the lane sweeps' batched launches: init arguments, compaction, MH, status rows
  SeqArgs *bI_dev = nullptr, *bI_host = nullptr;
  CompactArgs *bC_dev = nullptr, *bC_host = nullptr;
  MHArgs *bM_dev = nullptr, *bM_host = nullptr;
  int32_t *bS_dev = nullptr, *bS_host = nullptr;
  std::vector<hipEvent_t> b_ev;
  hipEvent_t b_join = nullptr;
  bool last_lane_batch = false;   // the last sweep ran every chain's work on the batch stream (lane_batch)
  void batch_alloc() {
    if (bA_dev) return;
    const size_t C = subs.size();
    const size_t SL = 2 * (size_t)cfg.n_views + 4;
    MVC_HIP(hipMalloc(&bI_dev, sizeof(SeqArgs) * C));
    MVC_HIP(hipMalloc(&bC_dev, sizeof(CompactArgs) * C));
    MVC_HIP(hipMalloc(&bM_dev, sizeof(MHArgs) * C));
    MVC_HIP(hipMalloc(&bS_dev, sizeof(int32_t) * C * SL));
    MVC_HIP(hipHostMalloc((void **)&bI_host, sizeof(SeqArgs) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bC_host, sizeof(CompactArgs) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bM_host, sizeof(MHArgs) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bS_host, sizeof(int32_t) * C * SL, hipHostMallocDefault));
    MVC_HIP(hipMalloc(&bA_dev, sizeof(SeqArgs) * C));
    MVC_HIP(hipMalloc(&bE_dev, sizeof(SeqArgs) * C));
    MVC_HIP(hipMalloc(&bL_dev, sizeof(SeqLds) * C));
    MVC_HIP(hipMalloc(&bR_dev, sizeof(Repair) * C));
    MVC_HIP(hipHostMalloc((void **)&bA_host, sizeof(SeqArgs) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bE_host, sizeof(SeqArgs) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bL_host, sizeof(SeqLds) * C, hipHostMallocDefault));
    MVC_HIP(hipHostMalloc((void **)&bR_host, sizeof(Repair) * C, hipHostMallocDefault));
    b_ev.assign(C, nullptr);
    for (auto &e : b_ev) MVC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    MVC_HIP(hipEventCreateWithFlags(&b_join, hipEventDisableTiming));
  }
  void batch_free() {
    if (!bA_dev) return;
    for (void *p : {(void *)bA_dev, (void *)bE_dev, (void *)bL_dev, (void *)bR_dev, (void *)bI_dev, (void *)bC_dev,
                    (void *)bM_dev, (void *)bS_dev})
      hipFree(p);
    for (void *p : {(void *)bA_host, (void *)bE_host, (void *)bL_host, (void *)bR_host, (void *)bI_host,
                    (void *)bC_host, (void *)bM_host, (void *)bS_host})
      hipHostFree(p);
    for (auto &e : b_ev) hipEventDestroy(e);
    hipEventDestroy(b_join);
    bA_dev = nullptr;
  }
  void sweep_batched() {
    MVC_HIP(hipSetDevice(cfg.device));
    batch_alloc();
    const int C = (int)subs.size();
    hipStream_t bs = subs[0]->stream;   // the batch stream
    Timers &tm = subs[0]->timers;       // the handle's "sweep" timer: batch stream, joined by every chain
    hipEvent_t ev_sweep = nullptr;
    tm.begin("sweep", &ev_sweep);
    std::vector<ParallelSampler::RepairRun> rr(C);
    std::vector<char> done(C, 0);
    // Every chain in the small chains' lane loop (and no per-phase timers or
    // debug synchronisation): the whole sweep of every chain on the batch
    // stream, each per-chain launch (the repair's init, compaction, MH,
    // status read-back) one batched launch for all chains -- the same kernels
    // on the same arguments, so the same chains, with ~10 host calls per
    // sweep instead of ~10 per chain.
    bool lane_batch = (!tm.on || tm.coarse) && debug_sync_level() == 0;
    for (int c = 0; c < C && lane_batch; ++c) {
      ParallelSampler &S = *subs[c];
      lane_batch = !S.repair_grid_only && S.lane_sweep(S.chains[0]);
    }
    if (!lane_batch && last_lane_batch) {   // the chains' streams after the batch stream's last sweep and saves
      MVC_HIP(hipEventRecord(b_join, bs));
      for (int c = 1; c < C; ++c) MVC_HIP(hipStreamWaitEvent(subs[c]->stream, b_join, 0));
    }
    if (lane_batch && !last_lane_batch) {   // the batch stream after each chain's last work on its own stream
      for (int c = 1; c < C; ++c) {
        MVC_HIP(hipEventRecord(b_ev[c], subs[c]->stream));
        MVC_HIP(hipStreamWaitEvent(bs, b_ev[c], 0));
      }
    }
    last_lane_batch = lane_batch;
    if (lane_batch) {
      // 1. the repair state of every chain (mvc_seq_init_kernel, run_start: the lane loop starts at customer 0)
      for (int c = 0; c < C; ++c) {
        ParallelSampler &S = *subs[c];
        auto &ch = S.chains[0];
        const uint32_t s = (uint32_t)S.sweeps_done;
        S.lane_now = true;
        S.zpath = 32 | 256;
        S.repair_start(ch, s, false, rr[c], false);   // (host only for a lane sweep)
        bI_host[c] = rr[c].Q;
      }
      MVC_HIP(hipMemcpyAsync(bI_dev, bI_host, sizeof(SeqArgs) * C, hipMemcpyHostToDevice, bs));
      hipLaunchKernelGGL(mvc_seq_init_kernel_b, dim3(C), dim3(64), 0, bs, (const SeqArgs *)bI_dev, 1);
      MVC_HIP(hipGetLastError());
    } else {
    // 1. phase A and the first mover, every chain on its own stream
    for (int c = 0; c < C; ++c) {
      ParallelSampler &S = *subs[c];
      auto &ch = S.chains[0];
      const uint32_t s = (uint32_t)S.sweeps_done;
      bool phaseA = false;
      S.sweep_pre(ch, s, phaseA);
      S.repair_start(ch, s, phaseA, rr[c], false);
      if (c > 0) {
        MVC_HIP(hipEventRecord(b_ev[c], S.stream));
        MVC_HIP(hipStreamWaitEvent(bs, b_ev[c], 0));
      }
    }
    }
    // 2. rounds of every unfinished chain, batched by run-kernel instance
    for (;;) {
      std::vector<int> act;
      for (int c = 0; c < C; ++c)
        if (!done[c]) act.push_back(c);
      if (act.empty()) break;
      int rounds = 1, bpc = 1 << 30;
      for (int c : act) {
        rounds = std::max(rounds, rr[c].rounds);
        bpc = std::min(bpc, std::max(1, rr[c].Q.G / 4));
      }
      // the instances: 4 / 3 lane columns (+ value prediction), 0 one wave per
      // customer, 2 the block-wide evaluation; -1 launched per chain (grid-wide
      // evaluation, grid-only repair)
      std::vector<int> kinds(C, -1);
      for (int c : act) {
        const ParallelSampler &S = *subs[c];
        const SeqLds &L = rr[c].L;
        // (lane loops batched in the general instance <6>: births commit in the kernel)
        kinds[c] = (S.repair_grid_only || S.run_wgrid(L)) ? -1 : L.lc == 3 ? 6 : L.lc == 2 ? 4 : L.lc ? 3 : L.tw == 1 ? 0 : 2;
      }
      int nb = 0;   // batched members, grouped by kind
      std::vector<std::pair<int, int>> groups;   // (kind, first index), each up to the next
      std::vector<size_t> dyn;
      for (int k : {6, 4, 3, 0, 2}) {
        const int first = nb;
        size_t dmax = 0;
        for (int c : act) {
          if (kinds[c] != k) continue;
          ParallelSampler &S = *subs[c];
          SeqLds &L = rr[c].L;
          L.dyn = S.run_dyn(L);
          L.fill = lds_fill_byte();
          L.chk = run_check() ? 1 : 0;
          bA_host[nb] = rr[c].Q;
          bL_host[nb] = L;
          dmax = std::max(dmax, (size_t)L.dyn);
          ++nb;
        }
        if (nb > first) {
          groups.push_back({k, first});
          dyn.push_back(dmax);
        }
      }
      // every active chain's arguments for the outcome gather, the batched
      // chains first: only they take part in the batched window evaluation
      // (its wave stride set to the batched grid's).  A chain launched on its
      // own stream runs its own window evaluation inside repair_rounds; the
      // batched one must not evaluate it concurrently.
      // (the lane loop's chains, kind 6, open no windows: after the others)
      std::vector<int> ord;
      for (int c : act)
        if (kinds[c] >= 0 && kinds[c] != 6) ord.push_back(c);
      const int n_bat = (int)ord.size();
      for (int c : act)
        if (kinds[c] == 6) ord.push_back(c);
      for (int c : act)
        if (kinds[c] < 0) ord.push_back(c);
      for (size_t j = 0; j < ord.size(); ++j) {
        bE_host[j] = rr[ord[j]].Q;
        if ((int)j < n_bat) bE_host[j].G = 4 * bpc;
      }
      if (nb) {
        MVC_HIP(hipMemcpyAsync(bA_dev, bA_host, sizeof(SeqArgs) * nb, hipMemcpyHostToDevice, bs));
        MVC_HIP(hipMemcpyAsync(bL_dev, bL_host, sizeof(SeqLds) * nb, hipMemcpyHostToDevice, bs));
      }
      MVC_HIP(hipMemcpyAsync(bE_dev, bE_host, sizeof(SeqArgs) * act.size(), hipMemcpyHostToDevice, bs));
      // the chains launched one by one run on their own streams after the batch stream's work so far
      bool any_single = false;
      for (int c : act)
        if (kinds[c] < 0) any_single = true;
      if (any_single) MVC_HIP(hipEventRecord(b_join, bs));
      for (int r = 0; r < rounds; ++r) {
        for (size_t g = 0; g < groups.size(); ++g) {
          const int k = groups[g].first, f = groups[g].second;
          const int m = (g + 1 < groups.size() ? groups[g + 1].second : nb) - f;
          const dim3 grid(m);
          const SeqArgs *a = bA_dev + f;
          const SeqLds *l = bL_dev + f;
          switch (k) {
            case 6: hipLaunchKernelGGL(mvc_seq_run_kernel_b<6>, grid, dim3(kSeqLcThreads), dyn[g], bs, a, l); break;
            case 4: hipLaunchKernelGGL(mvc_seq_run_kernel_b<4>, grid, dim3(kSeqLcThreads), dyn[g], bs, a, l); break;
            case 3: hipLaunchKernelGGL(mvc_seq_run_kernel_b<3>, grid, dim3(kSeqLcThreads), dyn[g], bs, a, l); break;
            case 0: hipLaunchKernelGGL(mvc_seq_run_kernel_b<0>, grid, dim3(kSeqRunThreads), dyn[g], bs, a, l); break;
            default: hipLaunchKernelGGL(mvc_seq_run_kernel_b<2>, grid, dim3(kSeqRunThreads), dyn[g], bs, a, l); break;
          }
          MVC_HIP(hipGetLastError());
        }
        if (n_bat) {
          hipLaunchKernelGGL(mvc_seq_eval_kernel_b, dim3((unsigned)(n_bat * bpc)), dim3(256), 0, bs,
                             (const SeqArgs *)bE_dev, bpc);
          MVC_HIP(hipGetLastError());
        }
      }
      for (int c : act) {   // the others, one by one on their streams
        if (kinds[c] >= 0) continue;
        ParallelSampler &S = *subs[c];
        MVC_HIP(hipStreamWaitEvent(S.stream, b_join, 0));
        const int keep = rr[c].rounds;
        rr[c].rounds = rounds;
        S.repair_rounds(S.chains[0], (uint32_t)S.sweeps_done, rr[c]);
        rr[c].rounds = keep;
        MVC_HIP(hipEventRecord(b_ev[c], S.stream));
        MVC_HIP(hipStreamWaitEvent(bs, b_ev[c], 0));
      }
      const int SL = 2 * cfg.n_views + 4;
      const unsigned na = (unsigned)act.size();
      if (lane_batch) {
        // the sweep's tail of the chains still active, gated on the device per
        // chain: compaction (a no-op unless its repair is done with moves),
        // the status rows, and behind the read-back's event the MH, which runs
        // iff the repair is done -- one host synchronisation per batch of rounds
        for (unsigned j = 0; j < na; ++j) {
          ParallelSampler &S = *subs[ord[j]];
          auto &ch = S.chains[0];
          bC_host[j] = CompactArgs{rr[ord[j]].Q, ch.pos_new, ch.jmap, 1};   // (n <= 1,024: the block relabels z)
          bM_host[j] = S.mh_args(ch, 1, (uint32_t)S.sweeps_done, ch.R, 1);
        }
        MVC_HIP(hipMemcpyAsync(bC_dev, bC_host, sizeof(CompactArgs) * na, hipMemcpyHostToDevice, bs));
        hipLaunchKernelGGL(mvc_seq_compact_kernel_b, dim3(na), dim3(1024), 0, bs, (const CompactArgs *)bC_dev);
        hipLaunchKernelGGL(mvc_seq_gather_status_kernel, dim3(na), dim3(64), 0, bs, (const CompactArgs *)bC_dev, SL,
                           bS_dev);
      }
      // every chain's outcome in one copy
      hipLaunchKernelGGL(mvc_seq_gather_repair_kernel, dim3(na), dim3(64), 0, bs, (const SeqArgs *)bE_dev, bR_dev);
      MVC_HIP(hipGetLastError());
      MVC_HIP(hipMemcpyAsync(bR_host, bR_dev, sizeof(Repair) * na, hipMemcpyDeviceToHost, bs));
      if (lane_batch) {
        MVC_HIP(hipMemcpyAsync(bS_host, bS_dev, sizeof(int32_t) * na * SL, hipMemcpyDeviceToHost, bs));
        MVC_HIP(hipMemcpyAsync(bM_dev, bM_host, sizeof(MHArgs) * na, hipMemcpyHostToDevice, bs));
        MVC_HIP(hipEventRecord(b_join, bs));
        hipLaunchKernelGGL(mvc_par_hyper_kernel_b, dim3(na), dim3(kHypThreads), 0, bs, (const MHArgs *)bM_dev);
        MVC_HIP(hipGetLastError());
        MVC_HIP(hipEventSynchronize(b_join));
      } else {
        MVC_HIP(hipStreamSynchronize(bs));
      }
      for (size_t j = 0; j < ord.size(); ++j) {
        const int c = ord[j];
        ParallelSampler &S = *subs[c];
        rr[c].rounds = rounds;
        const int res = S.repair_outcome(S.chains[0], (uint32_t)S.sweeps_done, rr[c], bR_host[j]);
        if (res == 1) {
          done[c] = 1;
          S.last_rs = bR_host[j];
          if (lane_batch) {   // the outcome, and the next sweep's shapes from the status row
            auto &ch = S.chains[0];
            const Repair &rs = bR_host[j];
            ch.last[0] = rs.moves;
            ch.last[1] = rs.births;
            ch.last[2] = rs.rounds;
            ch.last[3] = rs.newdish;
            if (rs.moves > 0) {
              const int32_t *st = bS_host + j * SL;
              ch.T = st[0];
              for (int v = 0; v < cfg.n_views; ++v) ch.K[v] = st[1 + v];
              ch.s1t_stale = true;   // (S1t, only read by a phase A, is re-tiled when the chain leaves the lane loop)
            }
          }
        } else if (res == 0) {
          MVC_HIP(hipStreamSynchronize(S.stream));   // (a relayout's reset on the chain's stream)
        }
      }
    }
    if (lane_batch) {
      // 3. (the compaction and the MH ran behind each chain's last batch of rounds)
      for (int c = 0; c < C; ++c) subs[c]->sweeps_done += 1;
    } else {
    // 3. compaction and the MH of every chain, on its stream after the batch
    MVC_HIP(hipEventRecord(b_join, bs));
    for (int c = 0; c < C; ++c) {
      ParallelSampler &S = *subs[c];
      if (c > 0) MVC_HIP(hipStreamWaitEvent(S.stream, b_join, 0));
      S.repair_finish(S.chains[0], (uint32_t)S.sweeps_done, rr[c], S.last_rs, false);
    }
    for (int c = 0; c < C; ++c) {
      ParallelSampler &S = *subs[c];
      if (S.status_pending) S.repair_status(S.chains[0]);
      S.sweeps_done += 1;
    }
    }
    if (tm.on && ev_sweep) {
      for (int c = 1; c < C; ++c) {
        MVC_HIP(hipEventRecord(b_ev[c], subs[c]->stream));
        MVC_HIP(hipStreamWaitEvent(bs, b_ev[c], 0));
      }
    }
    tm.end("sweep", ev_sweep);
  }
  void synchronize() override {
    for (auto &s : subs) s->synchronize();
  }
  void get_state(int chain, int32_t *t, int32_t *T, int32_t *d, int32_t cap, double *h) override {
    at(chain).get_state(0, t, T, d, cap, h);
  }
  void get_dish_counts(int chain, int32_t *k) override { at(chain).get_dish_counts(0, k); }
  void get_stats(int chain, int view, int32_t *K, double *S1, double *S2, int32_t *n_vk, int32_t cap) override {
    at(chain).get_stats(0, view, K, S1, S2, n_vk, cap);
  }
  void set_state(int chain, const int32_t *t, int32_t T, const int32_t *d, const double *h) override {
    at(chain).set_state(0, t, T, d, h);
  }
  bool save_async(int chain, const SampleFn &fn) override {
    flush_set_saves();   // (older samples of save_all_async first)
    return at(chain).save_async(0, [fn, chain](int, int T, const int32_t *t, const int32_t *d, const double *h) {
      fn(chain, T, t, d, h);
    });
  }
  void flush_saves() override {
    flush_set_saves();
    for (auto &s : subs) s->flush_saves();
  }

  // ---- every chain's sample in one snapshot (after a lane_batch sweep) ----
  // One snapshot kernel for all chains on the batch stream, one read-back on
  // a copy stream; the samples reach fn chain by chain, in order, when the
  // slot is reused or at flush_saves (as the exact schedule's save_all_async).
  // After other sweeps the chains' own save_async runs (false here).
  struct SetSlot {
    SnapArgs *args_dev = nullptr, *args_host = nullptr;
    int32_t *dz = nullptr, *ddish = nullptr, *dT = nullptr, *hz = nullptr, *hdish = nullptr, *hT = nullptr;
    double *dhyp = nullptr, *hhyp = nullptr;
    int dcap = 0;
    hipEvent_t snap = nullptr, done = nullptr;
    bool busy = false;
    SampleFn fn;
  };
  static constexpr int kSetSlots = 4;
  SetSlot set_saves[kSetSlots];
  int set_next = 0;
  hipStream_t set_cstream = nullptr;
  void set_slot_free(SetSlot &q) {
    for (void *p : {(void *)q.args_dev, (void *)q.dz, (void *)q.ddish, (void *)q.dT, (void *)q.dhyp}) hipFree(p);
    for (void *p : {(void *)q.args_host, (void *)q.hz, (void *)q.hdish, (void *)q.hT, (void *)q.hhyp}) hipHostFree(p);
    q = SetSlot();
  }
  void set_slot_finish(SetSlot &q) {
    MVC_HIP(hipEventSynchronize(q.done));
    const int C = (int)subs.size(), V = cfg.n_views, n = cfg.n, H = 3 * V + 2;
    std::vector<int32_t> d;
    for (int c = 0; c < C; ++c) {
      const int T = q.hT[c];
      d.assign((size_t)V * std::max(T, 1), 0);
      for (int v = 0; v < V; ++v)
        std::copy(q.hdish + ((size_t)c * V + v) * q.dcap, q.hdish + ((size_t)c * V + v) * q.dcap + T,
                  d.begin() + (size_t)v * T);
      q.fn(c, T, q.hz + (size_t)c * n, d.data(), q.hhyp + (size_t)c * H);
    }
    q.busy = false;
  }
  void flush_set_saves() {
    for (int k = 0; k < kSetSlots; ++k) {
      SetSlot &q = set_saves[(set_next + k) % kSetSlots];   // oldest first
      if (q.busy) set_slot_finish(q);
    }
  }
  bool save_all_async(const SampleFn &fn) override {
    if (!last_lane_batch) return false;
    for (auto &s : subs) s->flush_saves();   // (older samples of the chains' own save_async first)
    MVC_HIP(hipSetDevice(cfg.device));
    if (!set_cstream) MVC_HIP(hipStreamCreateWithFlags(&set_cstream, hipStreamNonBlocking));
    SetSlot &q = set_saves[set_next];
    if (q.busy) set_slot_finish(q);
    const int C = (int)subs.size(), V = cfg.n_views, n = cfg.n, H = 3 * V + 2;
    int dcap = 1;
    for (auto &sp : subs) dcap = std::max(dcap, sp->chains[0].T);
    if (q.dcap < dcap) {
      if (q.dz) set_slot_free(q);
      dcap = std::max(dcap, 2 * q.dcap);   // (room to grow)
      MVC_HIP(hipMalloc(&q.args_dev, sizeof(SnapArgs) * C));
      MVC_HIP(hipMalloc(&q.dz, sizeof(int32_t) * (size_t)C * std::max(n, 1)));
      MVC_HIP(hipMalloc(&q.ddish, sizeof(int32_t) * (size_t)C * V * dcap));
      MVC_HIP(hipMalloc(&q.dT, sizeof(int32_t) * C));
      MVC_HIP(hipMalloc(&q.dhyp, sizeof(double) * (size_t)C * H));
      MVC_HIP(hipHostMalloc((void **)&q.args_host, sizeof(SnapArgs) * C, hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hz, sizeof(int32_t) * (size_t)C * std::max(n, 1), hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hdish, sizeof(int32_t) * (size_t)C * V * dcap, hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hT, sizeof(int32_t) * C, hipHostMallocDefault));
      MVC_HIP(hipHostMalloc((void **)&q.hhyp, sizeof(double) * (size_t)C * H, hipHostMallocDefault));
      q.dcap = dcap;
    }
    if (!q.snap) {
      MVC_HIP(hipEventCreateWithFlags(&q.snap, hipEventDisableTiming));
      MVC_HIP(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
    }
    for (int c = 0; c < C; ++c) {
      const ParallelSampler &S = *subs[c];
      const auto &ch = S.chains[0];
      q.args_host[c] = SnapArgs{ch.P.z, ch.P.dish, ch.P.d_id, ch.status, ch.P.hyper, (int32_t)ch.P.TC, (int32_t)ch.P.KC};
    }
    // (the slot's pinned arguments are rewritten only after set_slot_finish: this copy has run)
    MVC_HIP(hipMemcpyAsync(q.args_dev, q.args_host, sizeof(SnapArgs) * C, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(mvc_par_snapshot_all_kernel, dim3(std::min(64, (n + 255) / 256 + 1), C), dim3(256), 0, stream,
                       (const SnapArgs *)q.args_dev, n, V, q.dcap, q.dz, q.ddish, q.dT, q.dhyp);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipEventRecord(q.snap, stream));
    MVC_HIP(hipStreamWaitEvent(set_cstream, q.snap, 0));
    MVC_HIP(hipMemcpyAsync(q.hz, q.dz, sizeof(int32_t) * (size_t)C * n, hipMemcpyDeviceToHost, set_cstream));
    MVC_HIP(hipMemcpyAsync(q.hdish, q.ddish, sizeof(int32_t) * (size_t)C * V * q.dcap, hipMemcpyDeviceToHost, set_cstream));
    MVC_HIP(hipMemcpyAsync(q.hT, q.dT, sizeof(int32_t) * C, hipMemcpyDeviceToHost, set_cstream));
    MVC_HIP(hipMemcpyAsync(q.hhyp, q.dhyp, sizeof(double) * (size_t)C * H, hipMemcpyDeviceToHost, set_cstream));
    MVC_HIP(hipEventRecord(q.done, set_cstream));
    q.busy = true;
    q.fn = fn;
    set_next = (set_next + 1) % kSetSlots;
    return true;
  }
  const int32_t *device_labels(int chain) override { return at(chain).device_labels(0); }
  void copy_rows(int view, const int32_t *idx, int64_t m, double *out) override { subs[0]->copy_rows(view, idx, m, out); }
  bool repair_stats(int chain, int32_t *out) override { return at(chain).repair_stats(0, out); }
  // timing: chain 0's timers (every chain runs the same kernels)
  void set_timing(bool on, bool coarse) override {
    timers.on = on;
    timers.coarse = coarse;
    for (auto &s : subs) s->set_timing(on, coarse);
  }
  void reset_timers() override {
    for (auto &s : subs) s->reset_timers();
  }
  bool kernel_time(const char *name, double *ms, int64_t *launches) override {
    return subs[0]->kernel_time(name, ms, launches);
  }
};

Sampler *make_parallel_sampler_device(const mvc_config &cfg, DeviceData &&dd) {
  if (cfg.n_chains > 1 && path_int("chain_threads", 1) != 0) return new ChainSet(cfg, std::move(dd));
  return new ParallelSampler(cfg, std::move(dd));
}

Sampler *make_parallel_sampler(const mvc_config &cfg, const double *const *views) {
  // chain_threads=0 (MVC_PATH): one handle runs its chains one after another
  if (cfg.n_chains > 1 && path_int("chain_threads", 1) != 0) return new ChainSet(cfg, views);
  return new ParallelSampler(cfg, views);
}

}  // namespace mvc
