// mvc_parallel.hip — the parallel ("mode P") sweep on gfx950.
//
// Per sweep:
//   zresample : every customer draws its table against the state frozen at
//               sweep start (virtual self-removal), one wavefront per
//               customer, log-space probabilities, tree64 sums, Philox
//               counters (chain, sweep, customer).
//   births    : customers that chose a new table draw one dish per view.
//   commit    : survivors + births -> dense positions, live-dish lists,
//               counts (integer atomics: order independent).
//   stats     : S1/S2 rebuilt in a fixed chunked order (bit-reproducible).
//   hyper     : one workgroup: ||S1||^2, the MH updates of
//               multiview_hyper.cpp:233-292 (EPPF sums via lgamma + size
//               histograms, tree64 order), then next sweep's coefficients.
// Every fp64 expression matches ParallelSampler in oracle/mvc_oracle.cpp.
// Compile with -ffp-contract=off.
#include <hipcub/hipcub.hpp>

#include "mvc_internal.h"

namespace {

constexpr double kEps = 1e-6;
constexpr int kStatsChunk = 4096;   // must equal oracle kStatsChunk
constexpr int kMaxChunks = 64;      // two-level tree64: <= 4096 elements

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
  double *scratch;        // per wave: [sumK]
  int32_t *choice;        // [n] position or -1 (birth)
  const int32_t *blist;   // [NB] birth customers, ascending
  // birth resolution (phase 2) state
  int32_t *p2meta;        // [V+2]: T2, K2[V], error
  int32_t *p2_c;          // [TC] customers of phase-2 table t
  int32_t *p2_tup;        // [TC*V] extended dish index (frozen j or K_v + q)
  int32_t *n2, *l2;       // [V*KC]
  double *S1_2T;          // [(v*D + d)*KC + q]
  double *lp2;            // [V*KC] lp of phase-2 dishes for the current birth
  int32_t *btab;          // [NB] phase-2 table of each birth
  const int32_t *nbirth;  // [1]
  const int32_t *status;  // [V+4]; status[V+3] = tables with n_t > 0
  const double *yt;       // MFMA A-fragment layout of y (mvc_par_ytile_kernel)
  const double *S1t;      // MFMA B-fragment layout of S1 (mvc_par_s1tile_kernel)
  int32_t SP;             // k-steps per view in yt/S1t (D/4 rounded up to MVC_Z_KS)
  int32_t T, sumK;
  uint64_t seed;
  uint32_t chain, sweep;
};

// Per-view mixture of the new-table marginal for customer i.
// Writes lp of every live dish into lp[0..K); returns lmarg; outputs the max
// m, the tree sum S and (lane c) the level-0 chunk partial of chunk c.
struct ViewOut { double lmarg, m, S, part; int nc; double lf_new, w_new; };

__device__ __forceinline__ ViewOut view_eval(const Sweep &A, int i, int v, int p0, bool alive, double *lp,
                                            bool with_p2 = false) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n;
  const int K = P.Kact[v];
  const int K2 = with_p2 ? A.p2meta[1 + v] : 0;
  const int j0 = P.dish[v * P.TC + p0];
  const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
  const double Y2i = A.Y2[(size_t)v * n + i];
  const double hy = 0.5 * Y2i;
  const double h = (-0.5 * Y2i) / tau;
  const double *yrow = A.y + ((size_t)v * n + i) * D;
  const double *S1v = P.S1T + (size_t)v * D * KC;
  const int l0 = P.d_l[v * KC + j0];
  const int l0p = alive ? l0 : l0 - 1;
  double mx = -MVC_PM_INF;
  for (int base = 0; base < K; base += 64) {
    const int j = base + lane;
    if (j < K) {
      double G = 0.0;
      for (int d = 0; d < D; ++d) G = __builtin_fma(yrow[d], S1v[(size_t)d * KC + j], G);
      double val;
      int l;
      if (j == j0) {
        l = l0p;
        const double Gp = G - Y2i;
        const double Qp = (P.Q[v * KC + j] - 2.0 * G) + Y2i;
        const Coef c = coef(P.d_n[v * KC + j] - 1, Qp, tau, A.L2pt[v], D);
        val = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
      } else {
        l = P.d_l[v * KC + j];
        val = __builtin_fma(G + hy, P.cb[v * KC + j], P.c0[v * KC + j]) + h;
      }
      lp[j] = val;
      if (l > 0 && val > mx) mx = val;
    }
  }
  int L2sum = 0;
  if (with_p2) {
    const double *S2v = A.S1_2T + (size_t)v * D * KC;
    for (int base = 0; base < K2; base += 64) {
      const int q = base + lane;
      if (q < K2) {
        double G = 0.0, Q = 0.0;
        for (int d = 0; d < D; ++d) G = __builtin_fma(yrow[d], S2v[(size_t)d * KC + q], G);
        for (int d = 0; d < D; ++d) {
          const double sq = S2v[(size_t)d * KC + q];
          Q = __builtin_fma(sq, sq, Q);
        }
        const Coef c = coef(A.n2[v * KC + q], Q, tau, A.L2pt[v], D);
        const double val = __builtin_fma(G + hy, c.cb, c.c0) + h;
        A.lp2[v * KC + q] = val;
        if (val > mx) mx = val;
      }
    }
    for (int q = 0; q < K2; ++q) L2sum += A.l2[v * KC + q];
  }
  ViewOut o;
  o.lf_new = A.cnew[v] + h;
  const int Kact_i = K - ((l0p == 0) ? 1 : 0) + K2;
  double wn = alpha + (double)Kact_i * sigma;
  if (wn < 0.0) wn = 0.0;
  o.w_new = wn;
  mx = wave_max(mx);
  if (o.lf_new > mx) mx = o.lf_new;
  o.m = mx;
  const int NE = K + K2;
  o.nc = (NE + 1 + 63) >> 6;
  double part = 0.0;
  for (int c = 0; c < o.nc; ++c) {
    const int e = c * 64 + lane;
    double leaf = 0.0;
    if (e < K) {
      const int l = (e == j0) ? l0p : P.d_l[v * KC + e];
      if (l > 0) {
        double w = (double)l - sigma;
        if (w < 0.0) w = 0.0;
        leaf = w * mvc_exp(lp[e] - mx);
      }
    } else if (e < NE) {
      double w = (double)A.l2[v * KC + (e - K)] - sigma;
      if (w < 0.0) w = 0.0;
      leaf = w * mvc_exp(A.lp2[v * KC + (e - K)] - mx);
    } else if (e == NE) {
      leaf = wn * mvc_exp(o.lf_new - mx);
    }
    const double cs = wave_tree_sum(leaf);
    if (lane == c) part = cs;
  }
  o.part = part;
  o.S = (o.nc == 1) ? __shfl(part, 0, 64) : wave_tree_sum(lane < o.nc ? part : 0.0);
  const double denom = alpha + (double)((P.Ltot[v] - (alive ? 0 : 1)) + L2sum);
  o.lmarg = (denom <= 0.0) ? o.lf_new : (mx + mvc_log(o.S)) - mvc_log(denom);
  return o;
}

__device__ __forceinline__ int view_select(const Sweep &A, int v, int p0, bool alive, const double *lp,
                                           const ViewOut &o, double r, bool with_p2) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, KC = P.KC;
  const int K = P.Kact[v];
  const int K2 = with_p2 ? A.p2meta[1 + v] : 0;
  const int NE = K + K2;
  const int j0 = P.dish[v * P.TC + p0];
  const double sigma = P.hyper[2 * V + v];
  const int l0p = alive ? P.d_l[v * KC + j0] : P.d_l[v * KC + j0] - 1;
  int c = 0;
  if (o.nc > 1) {
    Tree64Levels L;
    const double pv = lane < o.nc ? o.part : 0.0;
    wave_tree_sum_levels(pv, L);
    c = wave_tree_select(L, pv, r);
  }
  const int e = c * 64 + lane;
  double leaf = 0.0;
  if (e < K) {
    const int l = (e == j0) ? l0p : P.d_l[v * KC + e];
    if (l > 0) {
      double w = (double)l - sigma;
      if (w < 0.0) w = 0.0;
      leaf = w * mvc_exp(lp[e] - o.m);
    }
  } else if (e < NE) {
    double w = (double)A.l2[v * KC + (e - K)] - sigma;
    if (w < 0.0) w = 0.0;
    leaf = w * mvc_exp(A.lp2[v * KC + (e - K)] - o.m);
  } else if (e == NE) {
    leaf = o.w_new * mvc_exp(o.lf_new - o.m);
  }
  Tree64Levels L2;
  wave_tree_sum_levels(leaf, L2);
  const int l = wave_tree_select(L2, leaf, r);
  return c * 64 + l;
}

// table score s_p (or -inf if excluded) for customer with own table p0;
// lp of view v dish j is lp[(Koff[v] + j) * stride]
__device__ __forceinline__ double table_score(const Sweep &A, int p, int p0, double sg, const double *lp,
                                             int stride) {
  const ParState &P = A.P;
  const int np = P.n_t[p] - (p == p0 ? 1 : 0);
  if (np < 1) return -MVC_PM_INF;
  const double mass = (double)np - sg;
  if (mass <= 0.0) return -MVC_PM_INF;
  double sp = (p == p0) ? mvc_log(mass) : P.lmass[p];
  for (int v = 0; v < P.V; ++v) sp = sp + lp[(size_t)(A.Koff[v] + P.dish[v * P.TC + p]) * stride];
  return sp;
}

// Table draw of one customer (wave-uniform), DESIGN.md §4.3: lane = table
// slot, tree64 over the table leaves, birth iff r >= B.  Returns the
// position or -1.
__device__ __forceinline__ int choose_table(const Sweep &A, int i, int p0, double s_new, const double *lp,
                                            int stride) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int T = A.T;
  const double sg = P.hyper[3 * P.V + 1];
  double M = s_new;
  for (int base = 0; base < T; base += 64) {
    const int p = base + lane;
    if (p < T) {
      const double sp = table_score(A, p, p0, sg, lp, stride);
      if (sp > M) M = sp;
    }
  }
  M = wave_max(M);
  const int nc = (T + 63) >> 6;
  double part = 0.0;
  for (int c = 0; c < nc; ++c) {
    const int p = c * 64 + lane;
    double leaf = 0.0;
    if (p < T) {
      const double sp = table_score(A, p, p0, sg, lp, stride);
      if (sp != -MVC_PM_INF) leaf = mvc_exp(sp - M);
    }
    const double cs = wave_tree_sum(leaf);
    if (lane == c) part = cs;
  }
  double B;
  if (nc == 0) B = 0.0;
  else if (nc == 1) B = __shfl(part, 0, 64);
  else B = wave_tree_sum(lane < nc ? part : 0.0);
  const double e_new = mvc_exp(s_new - M);
  const double W = e_new + B;
  double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
  if (!(r < B)) return -1;
  int c = 0;
  if (nc > 1) {
    Tree64Levels L;
    const double pv = lane < nc ? part : 0.0;
    wave_tree_sum_levels(pv, L);
    c = wave_tree_select(L, pv, r);
  }
  const int p = c * 64 + lane;
  double leaf = 0.0;
  if (p < T) {
    const double sp = table_score(A, p, p0, sg, lp, stride);
    if (sp != -MVC_PM_INF) leaf = mvc_exp(sp - M);
  }
  Tree64Levels L2;
  wave_tree_sum_levels(leaf, L2);
  return c * 64 + wave_tree_select(L2, leaf, r);
}

__device__ __forceinline__ double grp16_max(double x) {
  for (int m = 8; m >= 1; m >>= 1) {
    const double o = __shfl_xor(x, m, 64);
    x = o > x ? o : x;
  }
  return x;
}

}  // namespace

// ---------------------------------------------------------------------------
// zresample, generic path (any D): one wavefront per customer, grid-stride.
// ---------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void mvc_par_zresample_kernel(Sweep A) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  double *lpall = A.scratch + (size_t)wid * A.sumK;
  const int V = P.V;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int T_ne = A.status[V + 3];
  for (int i = wid; i < P.n; i += nw) {
    const int p0 = P.z[i];
    const bool alive = (P.n_t[p0] - 1) > 0;
    double s_new = mvc_log(ag + sg * (double)(T_ne - (alive ? 0 : 1)));
    for (int v = 0; v < V; ++v) {
      const ViewOut o = view_eval(A, i, v, p0, alive, lpall + A.Koff[v]);
      s_new = s_new + o.lmarg;
    }
    const int pick = choose_table(A, i, p0, s_new, lpall, 1);
    if (lane == 0) A.choice[i] = pick;
  }
}

// ---------------------------------------------------------------------------
// zresample, MFMA path (D % 4 == 0, D >= 16, every K_v <= 255, T <= 256).
// One wavefront per tile of 16 customers; 4 wavefronts per block.
//   * table descriptors (log mass, size, per-view lp row index) and dish
//     descriptors (c0, cb, Q, n, l) of the frozen state are staged in LDS once
//     per block;
//   * G = Y_tile * S1^T with v_mfma_f64_16x16x4_f64 (a k-ordered fma chain,
//     bitwise equal to the spec's fma_dot);
//   * the per-view mixture is evaluated in the MFMA C layout (lane = 16 *
//     row-group + dish column, 4 customers per lane): the tree64 butterfly
//     over dish slot e = 16 t + col is in-register for offsets 32 and 16 and
//     xor-8/4/2/1 shuffles inside each 16-lane group;
//   * lp of every (customer, dish) goes to per-wave LDS; the table draw then
//     runs per customer with lane = table slot, keeping scores and the tree
//     levels in registers (one pass, no recomputation).
// Bitwise identical to the generic path (tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
typedef double mvc_d4 __attribute__((ext_vector_type(4)));

#define MVC_MFMA_TMAX 256

struct MfmaLds {          // carve of the dynamic LDS
  double *t_lmass;        // [T]
  int *t_n;               // [T]
  int *t_idx;             // [V*T]  Koff[v] + dish[v][p]
  double *d_c0, *d_cb, *d_Q;   // [sumK]
  int *d_n, *d_l;         // [sumK]
  double *lpw, *lmw;      // per wave
};

__device__ __forceinline__ size_t mfma_shared_bytes(int T, int V, int sumK) {
  return (size_t)T * 8 + (size_t)T * 4 + (size_t)V * T * 4 + (size_t)sumK * (3 * 8 + 2 * 4) + 64;
}

extern "C" __global__ __launch_bounds__(256) void mvc_par_zresample_mfma_kernel(Sweep A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const ParState &P = A.P;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC, n = P.n;
  const int T = A.T;
  const int sumK = A.Koff[V];
  // ---- carve: doubles first (8-byte aligned), ints after
  MfmaLds L;
  {
    double *dp = (double *)smem;
    L.t_lmass = dp; dp += T;
    L.d_c0 = dp; dp += sumK;
    L.d_cb = dp; dp += sumK;
    L.d_Q = dp; dp += sumK;
    int *ip = (int *)dp;
    L.t_n = ip; ip += T;
    L.t_idx = ip; ip += V * T;
    L.d_n = ip; ip += sumK;
    L.d_l = ip; ip += sumK;
    char *cp = (char *)(((uintptr_t)ip + 15) & ~(uintptr_t)15);
    L.lpw = (double *)cp + (size_t)w * ((size_t)sumK * 16 + (size_t)V * 16);
    L.lmw = L.lpw + (size_t)sumK * 16;
  }
  for (int p = tid; p < T; p += 256) {
    L.t_lmass[p] = P.lmass[p];
    L.t_n[p] = P.n_t[p];
    for (int v = 0; v < V; ++v) L.t_idx[v * T + p] = A.Koff[v] + P.dish[v * TC + p];
  }
  for (int k = tid; k < sumK; k += 256) {
    int v = 0;
    while (v + 1 < V && A.Koff[v + 1] <= k) ++v;
    const int j = k - A.Koff[v];
    L.d_c0[k] = P.c0[v * KC + j];
    L.d_cb[k] = P.cb[v * KC + j];
    L.d_Q[k] = P.Q[v * KC + j];
    L.d_n[k] = P.d_n[v * KC + j];
    L.d_l[k] = P.d_l[v * KC + j];
  }
  __syncthreads();
  double *lpw = L.lpw, *lmw = L.lmw;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int T_ne = A.status[V + 3];
  const int ntile = (n + 15) >> 4;
  for (int tile = blockIdx.x * 4 + w; tile < ntile; tile += gridDim.x * 4) {
    const int i0 = tile * 16;
    int p0r[4];
    bool alr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + grp + 4 * r;
      p0r[r] = i < n ? P.z[i] : 0;
      alr[r] = i < n ? (L.t_n[p0r[r]] - 1) > 0 : true;
    }
    for (int v = 0; v < V; ++v) {
      const int K = P.Kact[v];
      const int koff = A.Koff[v];
      const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
      const double L2pt = A.L2pt[v];
      const double cnew = A.cnew[v];
      double Y2r[4], mx[4];
      int j0[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + grp + 4 * r;
        Y2r[r] = i < n ? A.Y2[(size_t)v * n + i] : 0.0;
        j0[r] = L.t_idx[v * T + p0r[r]] - koff;
        mx[r] = -MVC_PM_INF;
      }
      const double *S1v = P.S1T + (size_t)v * D * KC;
      const int arow = i0 + col;
      const bool rowok = arow < n;
      const double *yrow = A.y + ((size_t)v * n + (rowok ? arow : 0)) * D;
      const int ng = (K + 63) >> 6;
      for (int g = 0; g < ng; ++g) {
        mvc_d4 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
        const int nt = min(4, (K - g * 64 + 15) >> 4);
        int d = 0;
        for (; d + 8 <= D; d += 8) {            // 2 k-steps per iteration
          double a0 = rowok ? yrow[d + grp] : 0.0;
          double a1 = rowok ? yrow[d + 4 + grp] : 0.0;
          double b0[4], b1[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int j = g * 64 + t * 16 + col;
            const bool ok = t < nt && j < K;
            b0[t] = ok ? S1v[(size_t)(d + grp) * KC + j] : 0.0;
            b1[t] = ok ? S1v[(size_t)(d + 4 + grp) * KC + j] : 0.0;
          }
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < nt) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0[t], acc[t], 0, 0, 0);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (t < nt) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1[t], acc[t], 0, 0, 0);
        }
        for (; d < D; d += 4) {
          const double a = rowok ? yrow[d + grp] : 0.0;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (t >= nt) continue;
            const int j = g * 64 + t * 16 + col;
            const double b = j < K ? S1v[(size_t)(d + grp) * KC + j] : 0.0;
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
          }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = g * 64 + t * 16 + col;
          if (t < nt && j < K) {
            const int k = koff + j;
            const int lj = L.d_l[k];
            const double c0j = L.d_c0[k], cbj = L.d_cb[k];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const double G = acc[t][r];
              const double hy = 0.5 * Y2r[r];
              const double h = (-0.5 * Y2r[r]) / tau;
              double val;
              int l = lj;
              if (j == j0[r]) {
                if (!alr[r]) l -= 1;
                const double Gp = G - Y2r[r];
                const double Qp = (L.d_Q[k] - 2.0 * G) + Y2r[r];
                const Coef c = coef(L.d_n[k] - 1, Qp, tau, L2pt, D);
                val = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
              } else {
                val = __builtin_fma(G + hy, cbj, c0j) + h;
              }
              lpw[(size_t)k * 16 + grp + 4 * r] = val;
              if (l > 0 && val > mx[r]) mx[r] = val;
            }
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int nc = (K + 1 + 63) >> 6;
#pragma unroll 1
      for (int r = 0; r < 4; ++r) {
        const int row = grp + 4 * r;
        const double h = (-0.5 * Y2r[r]) / tau;
        const double lfn = cnew + h;
        const int l0 = L.d_l[koff + j0[r]];
        const int l0p = alr[r] ? l0 : l0 - 1;
        double m = grp16_max(mx[r]);
        if (lfn > m) m = lfn;
        const int Kact_i = K - ((l0p == 0) ? 1 : 0);
        double wn = alpha + (double)Kact_i * sigma;
        if (wn < 0.0) wn = 0.0;
        double part[4] = {0.0, 0.0, 0.0, 0.0};
        for (int g = 0; g < nc; ++g) {
          double x[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = g * 64 + t * 16 + col;
            double leaf = 0.0;
            if (e < K) {
              const int l = (e == j0[r]) ? l0p : L.d_l[koff + e];
              if (l > 0) {
                double ww = (double)l - sigma;
                if (ww < 0.0) ww = 0.0;
                leaf = ww * mvc_exp(lpw[(size_t)(koff + e) * 16 + row] - m);
              }
            } else if (e == K) {
              leaf = wn * mvc_exp(lfn - m);
            }
            x[t] = leaf;
          }
          double s0 = (x[0] + x[2]) + (x[1] + x[3]);   // offsets 32, 16
          s0 = s0 + __shfl_xor(s0, 8, 64);             // offsets 8, 4, 2, 1
          s0 = s0 + __shfl_xor(s0, 4, 64);
          s0 = s0 + __shfl_xor(s0, 2, 64);
          s0 = s0 + __shfl_xor(s0, 1, 64);
          if (g == 0) part[0] = s0;
          else if (g == 1) part[1] = s0;
          else if (g == 2) part[2] = s0;
          else part[3] = s0;
        }
        const double S = (nc == 1) ? part[0] : (part[0] + part[2]) + (part[1] + part[3]);
        const double denom = alpha + (double)(P.Ltot[v] - (alr[r] ? 0 : 1));
        const double lm = (denom <= 0.0) ? lfn : (m + mvc_log(S)) - mvc_log(denom);
        if (col == 0) lmw[v * 16 + row] = lm;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // ---- table draw per customer: lane = table slot, one pass (T <= 256)
    const int nct = (T + 63) >> 6;
    for (int c = 0; c < 16; ++c) {
      const int i = i0 + c;
      if (i >= n) break;
      const int p0 = P.z[i];
      const bool alive = (L.t_n[p0] - 1) > 0;
      double s_new = mvc_log(ag + sg * (double)(T_ne - (alive ? 0 : 1)));
      for (int v = 0; v < V; ++v) s_new = s_new + lmw[v * 16 + c];
      double sc[4];
      double M = s_new;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = q * 64 + lane;
        double sp = -MVC_PM_INF;
        if (q < nct && p < T) {
          const int np = L.t_n[p] - (p == p0 ? 1 : 0);
          const double mass = (double)np - sg;
          if (np >= 1 && mass > 0.0) {
            sp = (p == p0) ? mvc_log(mass) : L.t_lmass[p];
            for (int v = 0; v < V; ++v) sp = sp + lpw[(size_t)L.t_idx[v * T + p] * 16 + c];
          }
        }
        sc[q] = sp;
        if (sp > M) M = sp;
      }
      M = wave_max(M);
      double leafq[4], part = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        leafq[q] = (q < nct && sc[q] != -MVC_PM_INF) ? mvc_exp(sc[q] - M) : 0.0;
        if (q < nct) {
          const double cs = wave_tree_sum(leafq[q]);
          if (lane == q) part = cs;
        }
      }
      double B;
      if (nct == 0) B = 0.0;
      else if (nct == 1) B = __shfl(part, 0, 64);
      else B = wave_tree_sum(lane < nct ? part : 0.0);
      const double W = mvc_exp(s_new - M) + B;
      double rr = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
      int pick = -1;
      if (rr < B) {
        int cq = 0;
        if (nct > 1) {
          Tree64Levels Lv;
          const double pv = lane < nct ? part : 0.0;
          wave_tree_sum_levels(pv, Lv);
          cq = wave_tree_select(Lv, pv, rr);
        }
        const double leaf = cq == 0 ? leafq[0] : (cq == 1 ? leafq[1] : (cq == 2 ? leafq[2] : leafq[3]));
        Tree64Levels L2;
        wave_tree_sum_levels(leaf, L2);
        pick = cq * 64 + wave_tree_select(L2, leaf, rr);
      }
      if (lane == 0) A.choice[i] = pick;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// zresample, block-lockstep MFMA path.  Conditions: D % 4 ==
// 0, D >= 16, every K_v <= 64, T <= 128, V <= 8.
//
// A block of MVC_Z_NW wavefronts walks MVC_Z_NW tiles of 16 customers at a
// time, all waves in step over (view, k-chunk).  Per chunk of MVC_Z_KS
// k-steps (4 dims each):
//   * the S1 B-fragments of the chunk (S1t, <= 16 KB) are staged into a
//     double-buffered LDS slot shared by the block -- loaded from L2 one
//     chunk ahead, so every wave reads B from LDS;
//   * each wave's A-fragments (yt: one 512-byte coalesced row of 64 lanes per
//     k-step) are prefetched one chunk ahead into registers, so the HBM
//     stream of y has a chunk of MFMA work to hide behind;
//   * G += A * B with v_mfma_f64_16x16x4_f64 (k-ordered fma chain = the
//     spec's fma_dot), accumulators in registers across the view's chunks.
// After a view's last chunk the wave evaluates the view's mixture in the MFMA
// C layout (lane = 16 * row-group + dish column, rows grp + 4r), the self-dish
// coefficients once per row, and adds the view's lp of each table's dish into
// per-lane table scores (lane = table slot).  After the last view the table
// draw runs per customer on those scores (DPP trees, readlane descent).
// Bitwise identical to the generic path (tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
#define MVC_Z_NW 8            // wavefronts per block
#define MVC_Z_KS 8            // k-steps per staged chunk
#define MVC_Z_LS 80           // lp row stride (doubles): odd multiple of 16
#define MVC_Z_TMAX 128
#define MVC_Z_KMAX 64
#define MVC_Z_VMAX 8
#define MVC_Z_BUFD (MVC_Z_KS * 4 * 64)   // doubles per S1 chunk buffer

__host__ __device__ inline size_t z_shared_bytes(int T, int V, int sumK) {
  return 8 * ((size_t)2 * T + 3 * (size_t)sumK + 2 * MVC_Z_BUFD +
              (size_t)MVC_Z_NW * (16 * MVC_Z_LS + 4 * 16 + 16 * MVC_Z_VMAX)) +
         4 * ((size_t)T + (size_t)V * T + 2 * (size_t)sumK + 2 * (size_t)V + (size_t)MVC_Z_NW * 16) + 64;
}

// A-fragment layout: yt[((v*ntile + tile)*SP + s)*64 + lane] = y[v][16 tile +
// (lane & 15)][4 s + (lane >> 4)], zero outside n x D.
extern "C" __global__ void mvc_par_ytile_kernel(int n, int V, int D, int SP, const double *y, double *yt) {
  const int ntile = (n + 15) >> 4;
  const size_t total = (size_t)V * ntile * SP * 64;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int ln = (int)(e & 63);
    const size_t q = e >> 6;
    const int s = (int)(q % SP);
    const size_t vt = q / SP;
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

template <int NT>
__device__ __forceinline__ void z_mfma_chunk(const double (&a)[MVC_Z_KS], const double *__restrict__ buf,
                                             mvc_d4 (&acc)[4]) {
#pragma unroll
  for (int s = 0; s < MVC_Z_KS; ++s) {
    double b[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) b[t] = buf[(s * NT + t) * 64];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[t], acc[t], 0, 0, 0);
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

typedef double mvc_d2 __attribute__((ext_vector_type(2)));
struct ZStage {
  mvc_d2 st[2];          // this thread's share of the next S1 chunk
  double an[MVC_Z_KS];    // next chunk's A fragments
  int pz;                 // z of row (lane & 15) of the next tile
  double y2[2];           // Y2[grp + 4q][row] of the next tile
};
struct ZGeom { int per_it, nCC, ntile, SP, n, V, nblk, blk, w, tid, lane, col, grp; };

// issue the global loads of flat chunk X (tile iteration, view, k-chunk)
__device__ __forceinline__ void z_issue(const Sweep &A, const ZGeom &g, const int *s_nct, const int *s_S1o, int X,
                                        ZStage &o) {
  const int it = X / g.per_it;
  const int rem = X - it * g.per_it;
  const int v = rem / g.nCC, cc = rem - v * g.nCC;
  const int tile = min((it * g.nblk + g.blk) * MVC_Z_NW + g.w, g.ntile - 1);
  const int nct = s_nct[v];
  const mvc_d2 *src = (const mvc_d2 *)(A.S1t + ((size_t)s_S1o[v] + (size_t)cc * MVC_Z_KS * nct) * 64);
  const int units = MVC_Z_KS * nct * 32;
  // unconditional loads (clamped to the chunk) keep the stage in registers
  o.st[0] = src[min(g.tid, units - 1)];
  o.st[1] = src[min(g.tid + MVC_Z_NW * 64, units - 1)];
  const double *ap = A.yt + (((size_t)v * g.ntile + tile) * g.SP + (size_t)cc * MVC_Z_KS) * 64 + g.lane;
#pragma unroll
  for (int s = 0; s < MVC_Z_KS; ++s) o.an[s] = ap[s * 64];
  if (rem == 0) {   // first chunk of a tile: its customers' z and Y2
    const int i = min(tile * 16 + g.col, g.n - 1);
    o.pz = A.P.z[i];
    o.y2[0] = (g.grp < g.V) ? A.Y2[(size_t)g.grp * g.n + i] : 0.0;
    o.y2[1] = (g.grp + 4 < g.V) ? A.Y2[(size_t)(g.grp + 4) * g.n + i] : 0.0;
  }
}
// write the staged S1 chunk X into its LDS buffer; block barrier
__device__ __forceinline__ void z_commit(const ZGeom &g, const int *s_nct, double *sbuf, int X, const ZStage &o) {
  const int it = X / g.per_it;
  const int rem = X - it * g.per_it;
  const int v = rem / g.nCC;
  const int units = MVC_Z_KS * s_nct[v] * 32;
  mvc_d2 *dst = (mvc_d2 *)(sbuf + (X & 1) * MVC_Z_BUFD);
  if (g.tid < units) dst[g.tid] = o.st[0];
  if (g.tid + MVC_Z_NW * 64 < units) dst[g.tid + MVC_Z_NW * 64] = o.st[1];
  __syncthreads();
}

template <int QT>
__device__ __forceinline__ void z_kernel_body(const Sweep &A, char *smem) {
  const ParState &P = A.P;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int V = P.V, D = P.D, TC = P.TC, KC = P.KC, n = P.n;
  const int T = A.T;
  const int SP = A.SP;
  const int sumK = A.Koff[V];
  const int ntile = (n + 15) >> 4;
  // ---- LDS carve (doubles first)
  double *dp = (double *)smem;
  double *sbuf = dp; dp += 2 * MVC_Z_BUFD;   // first: 16-byte aligned (double2)
  double *t_b0 = dp; dp += T;            // base score of table p (p != p0)
  double *t_b1 = dp; dp += T;            // base score of table p when p == p0
  double *d_c0 = dp; dp += sumK;
  double *d_cb = dp; dp += sumK;
  double *d_Q = dp; dp += sumK;
  double *wbase = dp + (size_t)w * (16 * MVC_Z_LS + 4 * 16 + 16 * MVC_Z_VMAX);
  dp += (size_t)MVC_Z_NW * (16 * MVC_Z_LS + 4 * 16 + 16 * MVC_Z_VMAX);
  double *lpv = wbase;                   // [16][LS] lp of the current view
  double *selfG = lpv + 16 * MVC_Z_LS;   // [16]
  double *selfv = selfG + 16;            // [16]
  double *rowS = selfv + 16;             // [16]
  double *rowM = rowS + 16;              // [16]
  double *y2s = rowM + 16;               // [VMAX][16] Y2 of the tile's rows
  int *ip = (int *)dp;
  int *t_n = ip; ip += T;
  int *t_dish = ip; ip += V * T;
  int *d_n = ip; ip += sumK;
  int *d_l = ip; ip += sumK;
  int *s_nct = ip; ip += V;
  int *s_S1o = ip; ip += V;              // in units of 64 doubles
  int *zs = ip + w * 16;                 // [16] z of the tile's rows

  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  for (int p = tid; p < T; p += blockDim.x) {
    const int np = P.n_t[p];
    t_n[p] = np;
    t_b0[p] = (np >= 1 && (double)np - sg > 0.0) ? P.lmass[p] : -MVC_PM_INF;
    const double m1 = (double)(np - 1) - sg;
    t_b1[p] = (np - 1 >= 1 && m1 > 0.0) ? mvc_log(m1) : -MVC_PM_INF;
    for (int v = 0; v < V; ++v) t_dish[v * T + p] = P.dish[v * TC + p];
  }
  for (int k = tid; k < sumK; k += blockDim.x) {
    int v = 0;
    while (v + 1 < V && A.Koff[v + 1] <= k) ++v;
    const int j = k - A.Koff[v];
    d_c0[k] = P.c0[v * KC + j];
    d_cb[k] = P.cb[v * KC + j];
    d_Q[k] = P.Q[v * KC + j];
    d_n[k] = P.d_n[v * KC + j];
    d_l[k] = P.d_l[v * KC + j];
  }
  if (tid == 0) {
    int o = 0;
    for (int v = 0; v < V; ++v) {
      const int nct = (A.Koff[v + 1] - A.Koff[v] + 15) >> 4;
      s_nct[v] = nct;
      s_S1o[v] = o;
      o += SP * nct;
    }
  }
  __syncthreads();

  const int T_ne = A.status[V + 3];
  const double snewA = mvc_log(ag + sg * (double)T_ne);
  const double snewD = mvc_log(ag + sg * (double)(T_ne - 1));
  const int nCC = SP / MVC_Z_KS;
  const int per_it = V * nCC;
  const int stride_t = gridDim.x * MVC_Z_NW;
  const int nIt = (ntile - (int)blockIdx.x * MVC_Z_NW + stride_t - 1) / stride_t;
  const int nX = nIt > 0 ? nIt * per_it : 0;
  if (nX == 0) return;

  // ---- pipeline registers
  double a[MVC_Z_KS];
  ZStage stg;
  stg.pz = 0;
  stg.y2[0] = stg.y2[1] = 0.0;
  const ZGeom geo{per_it, nCC, ntile, SP, n, V, (int)gridDim.x, (int)blockIdx.x, w, tid, lane, col, grp};
  // ---- per-tile state
  int i0 = 0, i_row = 0, p0_row = 0;     // row = lane & 15
  bool alive_row = false, tile_active = false;
  double u_row = 0.0, snew_acc = 0.0;
  double sc[16][QT];
  // ---- per-view state
  mvc_d4 acc[4];

  z_issue(A, geo, s_nct, s_S1o, 0, stg);
  z_commit(geo, s_nct, sbuf, 0, stg);
#pragma unroll
  for (int s = 0; s < MVC_Z_KS; ++s) a[s] = stg.an[s];

  for (int X = 0; X < nX; ++X) {
    const int it = X / per_it;
    const int rem = X - it * per_it;
    const int v = rem / nCC, cc = rem - v * nCC;
    const int K = A.Koff[v + 1] - A.Koff[v];
    const int koff = A.Koff[v];
    const int NT = s_nct[v];
    if (rem == 0) {
      // ---- tile setup (z, Y2 arrived with the chunk-0 prefetch)
      const int tile = (it * (int)gridDim.x + (int)blockIdx.x) * MVC_Z_NW + w;
      tile_active = tile < ntile;
      i0 = min(tile, ntile - 1) * 16;
      i_row = i0 + col;
      if (grp == 0) zs[col] = stg.pz;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (grp + 4 * q < V) y2s[(grp + 4 * q) * 16 + col] = stg.y2[q];
      wave_lds_sync();
      p0_row = stg.pz;
      alive_row = (t_n[p0_row] - 1) > 0;
      u_row = mvc_uniform(A.seed, (uint32_t)i_row, A.sweep, A.chain, MVC_TAG_Z);
      snew_acc = alive_row ? snewA : snewD;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int p0c = zs[c];
#pragma unroll
        for (int q = 0; q < QT; ++q) {
          const int p = q * 64 + lane;
          sc[c][q] = p < T ? (p == p0c ? t_b1[p] : t_b0[p]) : -MVC_PM_INF;
        }
      }
    }
    if (cc == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = (mvc_d4){0.0, 0.0, 0.0, 0.0};
    }
    if (X + 1 < nX) z_issue(A, geo, s_nct, s_S1o, X + 1, stg);
    const double *bufl = sbuf + (X & 1) * MVC_Z_BUFD + lane;
    switch (NT) {
      case 1: z_mfma_chunk<1>(a, bufl, acc); break;
      case 2: z_mfma_chunk<2>(a, bufl, acc); break;
      case 3: z_mfma_chunk<3>(a, bufl, acc); break;
      default: z_mfma_chunk<4>(a, bufl, acc); break;
    }
    if (cc == nCC - 1) {
      // ================= view epilogue =================
      const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
      const double L2pt = A.L2pt[v], cnew = A.cnew[v];
      double hy[4], hr[4];
      int j0[4];
      bool alr[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double y2r = y2s[v * 16 + grp + 4 * r];
        hy[r] = 0.5 * y2r;
        hr[r] = (-0.5 * y2r) / tau;
        const int p0 = zs[grp + 4 * r];
        j0[r] = t_dish[v * T + p0];
        alr[r] = (t_n[p0] - 1) > 0;
      }
      // self dish: G of (row, j0) to LDS (coefficients once per row below)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jt = j0[r] >> 4;
        double g = acc[0][r];
        if (jt == 1) g = acc[1][r];
        if (jt == 2) g = acc[2][r];
        if (jt == 3) g = acc[3][r];
        if (col == (j0[r] & 15)) selfG[grp + 4 * r] = g;
      }
      // acc -> lp in place (frozen-dish coefficients)
      int lj[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = 16 * t + col;
        const int k = koff + min(j, K - 1);
        const double c0j = d_c0[k], cbj = d_cb[k];
        lj[t] = j < K ? d_l[k] : 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] = __builtin_fma(acc[t][r] + hy[r], cbj, c0j) + hr[r];
      }
      wave_lds_sync();
      {
        const double G = selfG[col];
        const double y2 = y2s[v * 16 + col];
        const int k0 = koff + t_dish[v * T + p0_row];
        const double Gp = G - y2;
        const double Qp = (d_Q[k0] - 2.0 * G) + y2;
        const Coef cf = coef(d_n[k0] - 1, Qp, tau, L2pt, D);
        const double sv = __builtin_fma(Gp + 0.5 * y2, cf.cb, cf.c0) + (-0.5 * y2) / tau;
        if (lane < 16) selfv[col] = sv;
      }
      wave_lds_sync();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = grp + 4 * r;
        const double svr = selfv[row];
        const int l0 = d_l[koff + j0[r]];
        const int l0p = alr[r] ? l0 : l0 - 1;
        double mx = -MVC_PM_INF;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = 16 * t + col;
          const bool self = (j == j0[r]);
          if (self) acc[t][r] = svr;
          const int l = self ? l0p : lj[t];
          if (j < K && l > 0) mx = dmax(mx, acc[t][r]);
        }
        double m = row16_max(mx);
        const double lfn = cnew + hr[r];
        if (lfn > m) m = lfn;
        const int Kact_i = K - ((l0p == 0) ? 1 : 0);
        double wn = alpha + (double)Kact_i * sigma;
        if (wn < 0.0) wn = 0.0;
        const double xnew = wn * mvc_exp(lfn - m);
        double x[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = 16 * t + col;
          const int l = (j == j0[r]) ? l0p : lj[t];
          const bool ok = j < K && l > 0;
          double ww = (double)l - sigma;
          if (ww < 0.0) ww = 0.0;
          const double ex = mvc_exp(ok ? acc[t][r] - m : 0.0);
          x[t] = ok ? ww * ex : (j == K ? xnew : 0.0);
        }
        const double S0 = row16_tree_sum((x[0] + x[2]) + (x[1] + x[3]));
        const double S = (K == 64) ? S0 + xnew : S0;
        if (col == 0) { rowS[row] = S; rowM[row] = m; }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = 16 * t + col;
          if (j < K) lpv[row * MVC_Z_LS + j] = acc[t][r];
        }
      }
      wave_lds_sync();
      {   // lane-parallel per-row marginal (row = lane & 15)
        const double S = rowS[col], m = rowM[col];
        const double y2 = y2s[v * 16 + col];
        const double lfn = cnew + (-0.5 * y2) / tau;
        const double denom = alpha + (double)(P.Ltot[v] - (alive_row ? 0 : 1));
        const double lm = (denom <= 0.0) ? lfn : (m + mvc_log(S)) - mvc_log(denom);
        snew_acc = snew_acc + lm;
      }
      // table scores: lane = table slot
#pragma unroll
      for (int q = 0; q < QT; ++q) {
        const int p = q * 64 + lane;
        const int dj = p < T ? t_dish[v * T + p] : 0;
#pragma unroll
        for (int c = 0; c < 16; ++c) sc[c][q] = sc[c][q] + lpv[c * MVC_Z_LS + dj];
      }
      if (v == V - 1) {
        // ================= table draw =================
        const int nct = (T + 63) >> 6;
        wave_lds_sync();   // rowS/rowM of the marginal step are consumed
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const double snc = readlane_d(snew_acc, c);
          double M = -MVC_PM_INF;
#pragma unroll
          for (int q = 0; q < QT; ++q) M = dmax(M, sc[c][q]);
          M = wave_max(M);
          if (!(M > snc)) M = snc;
          double B = 0.0;
#pragma unroll
          for (int q = 0; q < QT; ++q) {
            const double lf = sc[c][q] != -MVC_PM_INF ? mvc_exp(sc[c][q] - M) : 0.0;
            sc[c][q] = lf;
            if (q < nct) {
              const double cs = wave_tree_sum(lf);
              B = (q == 0) ? cs : B + cs;
            }
          }
          if (lane == 0) { rowM[c] = M; rowS[c] = B; }
        }
        wave_lds_sync();
        const double Mc = rowM[col], Bc = rowS[col];
        const double W = mvc_exp(snew_acc - Mc) + Bc;
        const double rr_row = u_row * W;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          double rr = readlane_d(rr_row, c);
          const double Bu = readlane_d(Bc, c);
          int pick = -1;
          if (rr < Bu) {
            int cq = 0;
            if (QT > 1 && nct > 1) {
              // two-chunk partial tree: node values p0 = part[0], p1 = part[1]
              const double p0s = wave_tree_sum(sc[c][0]);
              const double p1s = wave_tree_sum(sc[c][QT - 1]);
              if (!(p1s == 0.0 || rr < p0s)) { rr = rr - p0s; cq = 1; }
            }
            Tree64Levels Lv;
            const double leaf = (cq == 0) ? sc[c][0] : sc[c][QT - 1];
            wave_tree_sum_levels(leaf, Lv);
            pick = cq * 64 + wave_tree_select(Lv, leaf, rr);
          }
          if (lane == 0 && tile_active && i0 + c < n) A.choice[i0 + c] = pick;
        }
      }
    }
    if (X + 1 < nX) {
      z_commit(geo, s_nct, sbuf, X + 1, stg);
#pragma unroll
      for (int s = 0; s < MVC_Z_KS; ++s) a[s] = stg.an[s];
    }
  }
}

extern "C" __global__ __launch_bounds__(MVC_Z_NW * 64) void mvc_par_zresample_z1_kernel(Sweep A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  z_kernel_body<1>(A, smem);
}
extern "C" __global__ __launch_bounds__(MVC_Z_NW * 64) void mvc_par_zresample_z2_kernel(Sweep A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  z_kernel_body<2>(A, smem);
}

// Phase 2: births resolved sequentially in ascending
// customer order by ONE wavefront.  Each birth joins a table born earlier in
// this sweep or opens one (dish per view from frozen + phase-2 + new dishes).
extern "C" __global__ __launch_bounds__(64) void mvc_par_births_kernel(Sweep A) {
  const ParState &P = A.P;
  const int lane = threadIdx.x;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC;
  double *lpall = A.scratch;
  const int NB = *A.nbirth;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int T_ne = A.status[V + 3];
  if (lane == 0) {
    A.p2meta[0] = 0;
    for (int v = 0; v < V; ++v) A.p2meta[1 + v] = 0;
    A.p2meta[V + 1] = 0;
  }
  __syncthreads();
  for (int b = 0; b < NB; ++b) {
    const int i = A.blist[b];
    const int p0 = P.z[i];
    const bool alive = (P.n_t[p0] - 1) > 0;
    const int T2 = A.p2meta[0];
    // capacity: one more table and one more dish per view
    int bad = (A.T + T2 + 1 > TC) ? 1 : 0;
    for (int v = 0; v < V; ++v) bad |= (P.Kact[v] + A.p2meta[1 + v] + 1 > KC) ? 1 : 0;
    if (bad) {
      if (lane == 0) A.p2meta[V + 1] = 1;
      return;
    }
    double s_new = mvc_log(ag + sg * (double)((T_ne - (alive ? 0 : 1)) + T2));
    for (int v = 0; v < V; ++v) {
      const ViewOut o = view_eval(A, i, v, p0, alive, lpall + A.Koff[v], true);
      s_new = s_new + o.lmarg;
    }
    __syncthreads();
    auto lpx = [&](int v, int ex) -> double {
      const int K = P.Kact[v];
      return ex < K ? lpall[A.Koff[v] + ex] : A.lp2[v * KC + (ex - K)];
    };
    auto score = [&](int t) -> double {
      double st = mvc_log((double)A.p2_c[t] - sg);
      for (int v = 0; v < V; ++v) st = st + lpx(v, A.p2_tup[t * V + v]);
      return st;
    };
    double M = s_new;
    for (int base = 0; base < T2; base += 64) {
      const int t = base + lane;
      if (t < T2) { const double st = score(t); if (st > M) M = st; }
    }
    M = wave_max(M);
    const int nc = (T2 + 63) >> 6;
    double part = 0.0;
    for (int c = 0; c < nc; ++c) {
      const int t = c * 64 + lane;
      const double leaf = t < T2 ? mvc_exp(score(t) - M) : 0.0;
      const double cs = wave_tree_sum(leaf);
      if (lane == c) part = cs;
    }
    double B;
    if (nc == 0) B = 0.0;
    else if (nc == 1) B = __shfl(part, 0, 64);
    else B = wave_tree_sum(lane < nc ? part : 0.0);
    const double W = mvc_exp(s_new - M) + B;
    double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z2) * W;
    int t_pick;
    if (r < B) {
      int c = 0;
      if (nc > 1) {
        Tree64Levels L;
        const double pv = lane < nc ? part : 0.0;
        wave_tree_sum_levels(pv, L);
        c = wave_tree_select(L, pv, r);
      }
      const int t = c * 64 + lane;
      const double leaf = t < T2 ? mvc_exp(score(t) - M) : 0.0;
      Tree64Levels L2;
      wave_tree_sum_levels(leaf, L2);
      t_pick = c * 64 + wave_tree_select(L2, leaf, r);
      __syncthreads();
      if (lane == 0) A.p2_c[t_pick] += 1;
      for (int v = 0; v < V; ++v) {
        const int K = P.Kact[v];
        const int ex = A.p2_tup[t_pick * V + v];
        if (ex >= K) {
          const int q = ex - K;
          if (lane == 0) A.n2[v * KC + q] += 1;
          const double *yrow = A.y + ((size_t)v * P.n + i) * D;
          for (int d = lane; d < D; d += 64) {
            double *cell = A.S1_2T + ((size_t)v * D + d) * KC + q;
            *cell = *cell + yrow[d];
          }
        }
      }
    } else {
      t_pick = T2;
      for (int v = 0; v < V; ++v) {
        const int K = P.Kact[v];
        const int K2 = A.p2meta[1 + v];
        int ex;
        // recompute this view's mixture (identical arithmetic) for the draw
        const ViewOut o = view_eval(A, i, v, p0, alive, lpall + A.Koff[v], true);
        if (!(o.S > 0.0)) {
          ex = K + K2;
        } else {
          const double rv = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_DISH + 1u + (uint32_t)v) * o.S;
          ex = view_select(A, v, p0, alive, lpall + A.Koff[v], o, rv, true);
        }
        __syncthreads();
        const double *yrow = A.y + ((size_t)v * P.n + i) * D;
        if (ex == K + K2) {     // brand-new phase-2 dish
          if (lane == 0) { A.n2[v * KC + K2] = 0; A.l2[v * KC + K2] = 0; A.p2meta[1 + v] = K2 + 1; }
          for (int d = lane; d < D; d += 64) A.S1_2T[((size_t)v * D + d) * KC + K2] = 0.0;
          __syncthreads();
        }
        if (ex >= K) {
          const int q = ex - K;
          if (lane == 0) { A.l2[v * KC + q] += 1; A.n2[v * KC + q] += 1; }
          for (int d = lane; d < D; d += 64) {
            double *cell = A.S1_2T + ((size_t)v * D + d) * KC + q;
            *cell = *cell + yrow[d];
          }
        }
        if (lane == 0) A.p2_tup[T2 * V + v] = ex;
        __syncthreads();
      }
      if (lane == 0) { A.p2_c[T2] = 1; A.p2meta[0] = T2 + 1; }
    }
    if (lane == 0) A.btab[b] = t_pick;
    __syncthreads();
  }
}

// commit step 1: table counts and birth flags
// (per-block LDS histogram, then one global add per touched table: integer
// counts, so the result is independent of the order)
extern "C" __global__ __launch_bounds__(256) void mvc_par_count_kernel(int n, int T, const int32_t *choice,
                                                                      int32_t *cnt, int32_t *flag) {
  __shared__ int h[4096];
  for (int p = threadIdx.x; p < T; p += blockDim.x) h[p] = 0;
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = choice[i];
    flag[i] = c < 0 ? 1 : 0;
    if (c >= 0) atomicAdd(&h[c], 1);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < T; p += blockDim.x)
    if (h[p]) atomicAdd(&cnt[p], h[p]);
}

// commit step 2 (one workgroup of 256): new tables, dish lists, counts.
// status[0] = T_new, status[1..V] = K_new, status[V+1] = error flag,
// status[V+2] = tables opened by the birth resolution.
extern "C" __global__ __launch_bounds__(256) void mvc_par_commit_kernel(
    ParState P, int T, const int32_t *cnt, const int32_t *p2meta, const int32_t *p2_c, const int32_t *p2_tup,
    int32_t *pos_new, int32_t *tmp_dish /*[V*TC]*/, int32_t *tmp_nt /*[TC]*/, int32_t *lcnt /*[V*KC]*/,
    int32_t *jmap /*[V*KC]*/, int32_t *status) {
  __shared__ int s_scan[256];
  const int tid = threadIdx.x;
  const int V = P.V, TC = P.TC, KC = P.KC;
  const int T2 = p2meta[0];
  auto block_scan = [&](int x, int &total) {   // exclusive scan of x over the block
    s_scan[tid] = x;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const int t = tid >= off ? s_scan[tid - off] : 0;
      __syncthreads();
      s_scan[tid] += t;
      __syncthreads();
    }
    const int incl = s_scan[tid];
    total = s_scan[255];
    __syncthreads();
    return incl - x;
  };
  if (p2meta[V + 1] != 0) {
    if (tid == 0) status[V + 1] = 1;
    return;
  }
  // survivors in ascending position
  int run = 0;
  for (int base = 0; base < T; base += 256) {
    const int p = base + tid;
    const int alive = (p < T && cnt[p] > 0) ? 1 : 0;
    int tot;
    const int ex = block_scan(alive, tot);
    if (p < T) pos_new[p] = alive ? run + ex : -1;
    run += tot;
  }
  const int Tsurv = run;
  const int Tn = Tsurv + T2;
  if (tid == 0) { status[0] = Tn; status[V + 1] = 0; status[V + 2] = T2; }
  if (Tn > TC) { if (tid == 0) status[V + 1] = 1; return; }
  __syncthreads();
  for (int v = 0; v < V; ++v) {
    const int Kold = P.Kact[v];
    const int nnew = p2meta[1 + v];
    for (int t = tid; t < T2; t += 256) tmp_dish[v * TC + Tsurv + t] = p2_tup[t * V + v];
    for (int p = tid; p < T; p += 256)
      if (pos_new[p] >= 0) tmp_dish[v * TC + pos_new[p]] = P.dish[v * TC + p];
    for (int j = tid; j < Kold + nnew; j += 256) lcnt[v * KC + j] = 0;
    __syncthreads();
    for (int p = tid; p < Tn; p += 256) atomicAdd(&lcnt[v * KC + tmp_dish[v * TC + p]], 1);
    __syncthreads();
    // compact surviving dishes (ascending extended index == ascending raw id)
    const int Kext = Kold + nnew;
    int kr = 0;
    for (int base = 0; base < Kext; base += 256) {
      const int j = base + tid;
      const int live = (j < Kext && lcnt[v * KC + j] > 0) ? 1 : 0;
      int tot;
      const int ex = block_scan(live, tot);
      if (j < Kext) jmap[v * KC + j] = live ? kr + ex : -1;
      kr += tot;
    }
    __syncthreads();
    // in-place left compaction, one 256-chunk at a time (writes never reach
    // entries of a later chunk)
    const int next = P.next_id[v];
    for (int base = 0; base < Kext; base += 256) {
      const int j = base + tid;
      int id = 0, l = 0, keep = 0;
      if (j < Kext) {
        keep = jmap[v * KC + j] >= 0;
        id = j < Kold ? P.d_id[v * KC + j] : next + (j - Kold);
        l = lcnt[v * KC + j];
      }
      __syncthreads();
      if (keep) {
        const int jn = jmap[v * KC + j];
        P.d_id[v * KC + jn] = id;
        P.d_l[v * KC + jn] = l;
        P.d_n[v * KC + jn] = 0;
      }
      __syncthreads();
    }
    if (tid == 0) {
      P.next_id[v] = next + nnew;
      P.Kact[v] = kr;
      status[1 + v] = kr;
    }
    __syncthreads();
    for (int p = tid; p < Tn; p += 256) P.dish[v * TC + p] = jmap[v * KC + tmp_dish[v * TC + p]];
    __syncthreads();
  }
  // table counts, n_vk
  for (int p = tid; p < T; p += 256)
    if (pos_new[p] >= 0) tmp_nt[pos_new[p]] = cnt[p];
  for (int t = tid; t < T2; t += 256) tmp_nt[Tsurv + t] = p2_c[t];
  __syncthreads();
  for (int p = tid; p < Tn; p += 256) {
    const int c = tmp_nt[p];
    P.n_t[p] = c;
    for (int v = 0; v < V; ++v) atomicAdd(&P.d_n[v * KC + P.dish[v * TC + p]], c);
  }
}

// commit step 3: relabel customers (births -> Tsurv + their phase-2 table)
extern "C" __global__ void mvc_par_relabel_kernel(int n, int V, const int32_t *choice, const int32_t *pos_new,
                                                  const int32_t *brank, const int32_t *btab, const int32_t *status,
                                                  int32_t *z) {
  const int32_t Tn = status[0];
  const int32_t T2 = status[V + 2];
  const int32_t Tsurv = Tn - T2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = choice[i];
    z[i] = c >= 0 ? pos_new[c] : Tsurv + btab[brank[i]];
  }
}

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
    ParState P, const double *y, const double *Y2, const int32_t *Koff, int stride, int unused,
    double *part1, double *part2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  (void)unused;
  const int c = blockIdx.x, v = blockIdx.y;
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
                                                        const double *part1, const double *part2) {
  const int D = P.D, KC = P.KC, V = P.V;
  const size_t tot = (size_t)Koff[V] * (D + 1);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < tot; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e / (D + 1));
    const int d = (int)(e % (D + 1));
    int v = 0;
    while (v + 1 < V && Koff[v + 1] <= k) ++v;
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

// tree64 over n leaves produced by leaf(e), executed by the whole block.
// Level partials ping-pong between the two halves of ctx.scratch.
template <class F>
__device__ double block_tree64(const BlockCtx &ctx, int64_t n, F leaf) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ double s_root;
  if (n <= 0) return 0.0;
  double *src = nullptr;
  double *dst = ctx.scratch;
  int64_t m = (n + 63) / 64;
  for (int64_t c = w; c < m; c += 4) {
    const int64_t e = c * 64 + lane;
    const double x = e < n ? leaf(e) : 0.0;
    const double s = wave_tree_sum(x);
    if (lane == 0) dst[c] = s;
  }
  __syncthreads();
  while (m > 1) {
    src = dst;
    dst = (src == ctx.scratch) ? ctx.scratch + ctx.half : ctx.scratch;
    const int64_t m2 = (m + 63) / 64;
    for (int64_t c = w; c < m2; c += 4) {
      const int64_t e = c * 64 + lane;
      const double x = e < m ? src[e] : 0.0;
      const double s = wave_tree_sum(x);
      if (lane == 0) dst[c] = s;
    }
    __syncthreads();
    m = m2;
  }
  if (tid == 0) s_root = dst[0];
  __syncthreads();
  const double r = s_root;
  __syncthreads();
  return r;
}

// In-place exclusive SUFFIX scan of a[0..len) by the whole block:
// a[m] <- sum_{s > m} a[s].  Integer, so any order gives the same result.
__device__ void block_suffix_exclusive(int32_t *a, int len) {
  __shared__ int sc[256];
  __shared__ int carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int top = len - 1; top >= 0; top -= 256) {
    const int m = top - tid;              // descending within the chunk
    const int x = m >= 0 ? a[m] : 0;
    sc[tid] = x;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      const int t = tid >= off ? sc[tid - off] : 0;
      __syncthreads();
      sc[tid] += t;
      __syncthreads();
    }
    const int incl = sc[tid];
    const int c0 = carry;
    __syncthreads();
    if (m >= 0) a[m] = c0 + incl - x;
    if (tid == 255) carry = c0 + incl;
    __syncthreads();
  }
}

struct MHArgs {
  ParState P;
  int32_t *status;        // [V+3]: T, K[V], err, NB  -> we add T_ne at status[V+3]
  int32_t *Koff;          // [V+1] (output)
  double *L2pt, *cnew;    // [V] (output)
  int32_t *histT;         // [n+2] scratch: c_m for tables
  int32_t *histL;         // [V*(TC+2)] scratch: c_m for dishes
  double *scratch;        // tree levels
  size_t half;
  uint64_t seed;
  uint32_t chain, sweep;
  int do_mh;
};

}  // namespace

extern "C" __global__ __launch_bounds__(256) void mvc_par_hyper_kernel(MHArgs A) {
  ParState &P = A.P;
  const int tid = threadIdx.x;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC, n = P.n;
  __shared__ double s_red[8];
  __shared__ double s_b[4];
  __shared__ int s_i[8];
  BlockCtx ctx{s_red, A.scratch, A.half};
  const int T = A.status[0];
  // ---- Q = ||S1||^2 per live dish, Ltot, Koff ----
  for (int v = 0; v < V; ++v) {
    const int K = P.Kact[v];
    for (int j = tid; j < K; j += 256) {
      double q = 0.0;
      for (int d = 0; d < D; ++d) {
        const double s = P.S1T[((size_t)v * D + d) * KC + j];
        q = __builtin_fma(s, s, q);
      }
      P.Q[v * KC + j] = q;
    }
  }
  if (tid == 0) {
    for (int v = 0; v < V; ++v) {
      int lt = 0;
      for (int j = 0; j < P.Kact[v]; ++j) lt += P.d_l[v * KC + j];
      P.Ltot[v] = lt;
    }
    int tne = 0, maxn = 0;
    for (int p = 0; p < T; ++p) { if (P.n_t[p] > 0) ++tne; maxn = max(maxn, P.n_t[p]); }
    s_i[0] = tne;
    s_i[1] = maxn;
    A.status[V + 3] = tne;
  }
  __syncthreads();
  const int maxn = s_i[1];
  double *hyp = P.hyper;
  if (A.do_mh) {
    // c_m = #{tables with n_t > m}, m = 0..maxn
    for (int m = tid; m <= maxn + 1; m += 256) A.histT[m] = 0;
    __syncthreads();
    for (int p = tid; p < T; p += 256) atomicAdd(&A.histT[P.n_t[p]], 1);
    __syncthreads();
    block_suffix_exclusive(A.histT, maxn + 1);   // c_m = sum_{s > m} hist[s]
    for (int v = 0; v < V; ++v) {
      int *hl = A.histL + (size_t)v * (TC + 2);
      for (int m = tid; m < TC + 2; m += 256) hl[m] = 0;
    }
    __syncthreads();
    int maxl_loc = 0;
    for (int v = 0; v < V; ++v) {
      int *hl = A.histL + (size_t)v * (TC + 2);
      for (int j = tid; j < P.Kact[v]; j += 256) atomicAdd(&hl[P.d_l[v * KC + j]], 1);
    }
    __syncthreads();
    for (int v = 0; v < V; ++v) {
      int *hl = A.histL + (size_t)v * (TC + 2);
      int mx = 0;
      for (int j = tid; j < P.Kact[v]; j += 256) mx = max(mx, P.d_l[v * KC + j]);
      for (int m = 32; m >= 1; m >>= 1) mx = max(mx, __shfl_xor(mx, m, 64));
      if ((tid & 63) == 0) s_i[2 + (tid >> 6)] = mx;
      __syncthreads();
      mx = max(max(s_i[2], s_i[3]), max(s_i[4], s_i[5]));
      __syncthreads();
      block_suffix_exclusive(hl, mx + 1);
      if (tid == 0) hl[TC + 1] = mx;   // stash max l
      __syncthreads();
    }
    (void)maxl_loc;

    uint32_t kdraw = 0;
    auto unif = [&]() -> double {   // block-uniform
      if (tid == 0) s_b[0] = mvc_uniform(A.seed, kdraw, A.sweep, A.chain, MVC_TAG_MH);
      __syncthreads();
      const double u = s_b[0];
      __syncthreads();
      ++kdraw;
      return u;
    };
    auto rnorm = [&](double mu, double sd) -> double {
      const double u1 = unif();
      const double u2 = unif();
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
    // EPPF of a partition: K blocks, total tot, counts c_m (exclusive suffix),
    // max block size mx.
    auto eppf = [&](int K, int tot, const int *cm, int mx, double a, double s) -> double {
      if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
      if (a <= -s) return -MVC_PM_INF;
      // any term a + j s <= 0 ?  (monotone in j for s > 0: check j = 0)
      if (K > 0 && !(a + 0.0 * s > 0.0)) return -MVC_PM_INF;
      const double P1 = block_tree64(ctx, K, [&](int64_t j) { return mvc_log(a + (double)j * s); });
      const double P2 = mvc_lgamma_pos(a + (double)tot) - mvc_lgamma_pos(a + 1.0);
      const double P3 = block_tree64(ctx, mx > 1 ? mx - 1 : 0,
                                     [&](int64_t e) { const int m = (int)e + 1; return (double)cm[m] * mvc_log((double)m - s); });
      return (P1 - P2) + P3;
    };
    auto eppf_view = [&](int v, double a, double s) -> double {
      if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
      if (a <= -s) return -MVC_PM_INF;
      if (P.Ltot[v] == 0) return 0.0;
      const int *hl = A.histL + (size_t)v * (TC + 2);
      return eppf(P.Kact[v], P.Ltot[v], hl, hl[TC + 1], a, s);
    };
    auto eppf_global = [&](double a, double s) -> double {
      if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
      if (a <= -s) return -MVC_PM_INF;
      if (T <= 0) return 0.0;
      return eppf(T, n, A.histT, maxn, a, s);
    };
    auto post_tau = [&](int v, double t) -> double {
      if (t <= 0.0) return -MVC_PM_INF;
      const double L = mvc_log((2.0 * MVC_PI) * t);
      const double ll = block_tree64(ctx, P.Kact[v], [&](int64_t j) {
        const int nk = P.d_n[v * KC + j];
        if (nk == 0) return 0.0;
        double sse = P.S2[v * KC + j] - P.Q[v * KC + j] / (double)nk;
        if (sse < 0.0) sse = 0.0;
        return ((-0.5 * (double)nk) * (double)D) * L - 0.5 * (sse / t);
      });
      const double prior = (-3.0 * mvc_log(t)) - 1.0 / t;
      return ll + prior;
    };
    // ---- multiview_hyper.cpp:211-231 ----
    for (int v = 0; v < V; ++v) {
      double t_old = hyp[v];
      if (t_old <= 0.0) t_old = kEps;
      const double l_old = post_tau(v, t_old);
      const double t_prop = mvc_exp(mvc_log(t_old) + rnorm(0.0, 0.3));
      if (t_prop <= 0.0) continue;
      const double l_new = post_tau(v, t_prop);
      const double acc = (l_new - l_old) + (mvc_log(t_prop) - mvc_log(t_old));
      const double u = unif();
      if (mvc_log(u) < acc) { if (tid == 0) hyp[v] = t_prop; }
      __syncthreads();
    }
    // ---- :239-266 ----
    for (int v = 0; v < V; ++v) {
      double a_old = hyp[V + v];
      if (a_old <= 0.0) a_old = kEps;
      const double la = mvc_log(a_old > kEps ? a_old : kEps) + rnorm(0.0, 0.1);
      double a_prop = mvc_exp(la);
      if (!(a_prop > kEps)) a_prop = kEps;
      const double sv = hyp[2 * V + v];
      const double lo = (a_old <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_old, sv) + prior_alpha(a_old);
      const double ln = (a_prop <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_prop, sv) + prior_alpha(a_prop);
      const double lq = mvc_log(a_prop) - mvc_log(a_old);
      const double u = unif();
      if (mvc_log(u) < (ln - lo) + lq) { if (tid == 0) hyp[V + v] = a_prop; }
      __syncthreads();
      const double s_old = hyp[2 * V + v];
      const double s_prop = reflect_unit(s_old + rnorm(0.0, 0.05));
      const double u2 = unif();
      const double av = hyp[V + v];
      const double pn = (s_prop <= kEps || s_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(v, av, s_prop) + prior_sigma(s_prop);
      const double po = (s_old <= kEps || s_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(v, av, s_old) + prior_sigma(s_old);
      if (mvc_log(u2) < pn - po) { if (tid == 0) hyp[2 * V + v] = s_prop; }
      __syncthreads();
    }
    // ---- :268-291 ----
    {
      double ag_old = hyp[3 * V];
      if (ag_old <= 0.0) ag_old = kEps;
      const double la = mvc_log(ag_old > kEps ? ag_old : kEps) + rnorm(0.0, 0.1);
      double ag_prop = mvc_exp(la);
      if (!(ag_prop > kEps)) ag_prop = kEps;
      const double sg0 = hyp[3 * V + 1];
      const double lo = eppf_global(ag_old, sg0) + prior_alpha(ag_old);
      const double ln = eppf_global(ag_prop, sg0) + prior_alpha(ag_prop);
      const double lq = mvc_log(ag_prop) - mvc_log(ag_old);
      const double u = unif();
      if (mvc_log(u) < (ln - lo) + lq) { if (tid == 0) hyp[3 * V] = ag_prop; }
      __syncthreads();
      const double sg_old = hyp[3 * V + 1];
      const double sg_prop = reflect_unit(sg_old + rnorm(0.0, 0.05));
      const double u2 = unif();
      const double a_g = hyp[3 * V];
      const double pn = (sg_prop <= kEps || sg_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_prop) + prior_sigma(sg_prop);
      const double po = (sg_old <= kEps || sg_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_old) + prior_sigma(sg_old);
      if (mvc_log(u2) < pn - po) { if (tid == 0) hyp[3 * V + 1] = sg_prop; }
      __syncthreads();
    }
  }
  // ---- coefficients of the next sweep (frozen state) ----
  for (int v = 0; v < V; ++v) {
    const double tau = hyp[v];
    const double L = mvc_log((2.0 * MVC_PI) * tau);
    if (tid == 0) { A.L2pt[v] = L; A.cnew[v] = (double)D * (-0.5 * L); }
    for (int j = tid; j < P.Kact[v]; j += 256) {
      const Coef c = coef(P.d_n[v * KC + j], P.Q[v * KC + j], tau, L, D);
      P.c0[v * KC + j] = c.c0;
      P.cb[v * KC + j] = c.cb;
    }
  }
  const double sg = hyp[3 * V + 1];
  for (int p = tid; p < T; p += 256) P.lmass[p] = mvc_log((double)P.n_t[p] - sg);
}

// ===========================================================================
// Host side of the parallel schedule.
// ===========================================================================
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mvc_host.h"

namespace mvc {

namespace {
constexpr int kParTC = 4096;   // table capacity (two-level tree64)
constexpr int kParKC = 4095;   // live dishes per view (+1 new element <= 4096)
constexpr int kZGrid = 2048;   // zresample / birth grid (4 waves per block)

template <class Tp>
Tp *dmalloc(size_t count) {
  void *p = nullptr;
  MVC_HIP(hipMalloc(&p, sizeof(Tp) * std::max<size_t>(count, 1)));
  return (Tp *)p;
}
}  // namespace

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
    int32_t *choice = nullptr, *flags = nullptr, *brank = nullptr, *blist = nullptr, *nbirth = nullptr;
    int32_t *cnt = nullptr, *pos_new = nullptr, *tmp_dish = nullptr, *tmp_nt = nullptr;
    int32_t *p2meta = nullptr, *p2_c = nullptr, *p2_tup = nullptr, *n2 = nullptr, *l2 = nullptr, *btab = nullptr;
    double *S1_2T = nullptr, *lp2 = nullptr;
    int32_t *lcnt = nullptr, *jmap = nullptr, *histT = nullptr, *histL = nullptr;
    double *mh_scratch = nullptr;
    size_t mh_half = 0;
    double *S1t = nullptr;         // MFMA B-fragment layout of S1 (K_v <= 64)
    bool s1t_ok = false;
    int T = 0;
    std::vector<int32_t> K;
    uint32_t gid = 0;
    std::vector<void *> owned;
  };
  std::vector<Chain> chains;
  double *lp_scratch = nullptr;
  size_t lp_cap = 0;               // doubles per wave
  double *part1 = nullptr, *part2 = nullptr;
  size_t part_cap = 0;             // sumK capacity of partials
  void *cub_tmp = nullptr;
  size_t cub_bytes = 0;
  std::vector<int32_t> st_host;
  bool force_generic = false;
  bool force_mfma1 = false;
  int n_cu = 256;
  bool last_path_mfma = false;

  template <class Tp>
  Tp *own(Chain &c, size_t count) {
    Tp *p = dmalloc<Tp>(count);
    c.owned.push_back(p);
    return p;
  }

  ParallelSampler(const mvc_config &cf, const double *const *views) {
    cfg = cf;
    n = cf.n; V = cf.n_views; D = cf.dim;
    TC = kParTC; KC = kParKC;
    nchunk = (n + 4095) / 4096;
    if (V > MVC_MAXV) throw Error(MVC_ERR_UNSUPPORTED, "at most 64 views");
    MVC_HIP(hipSetDevice(cf.device));
    MVC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    timers.stream = stream;
    timers.on = (cf.flags & MVC_FLAG_TIMING) != 0;
    std::vector<double> yh((size_t)V * n * D);
    for (int v = 0; v < V; ++v) std::memcpy(&yh[(size_t)v * n * D], views[v], sizeof(double) * (size_t)n * D);
    y = dmalloc<double>(yh.size());
    Y2 = dmalloc<double>((size_t)V * n);
    MVC_HIP(hipMemcpyAsync(y, yh.data(), sizeof(double) * yh.size(), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(mvc_par_y2_kernel, dim3(1024), dim3(256), 0, stream, n, V, D, (const double *)y, Y2);
    MVC_HIP(hipGetLastError());
    if (D % 4 == 0 && D >= 16 && V <= MVC_Z_VMAX) {
      SP = ((D / 4 + MVC_Z_KS - 1) / MVC_Z_KS) * MVC_Z_KS;
      const size_t ntile = ((size_t)n + 15) / 16;
      yt = dmalloc<double>((size_t)V * ntile * SP * 64);
      hipLaunchKernelGGL(mvc_par_ytile_kernel, dim3(4096), dim3(256), 0, stream, n, V, D, SP, (const double *)y, yt);
      MVC_HIP(hipGetLastError());
    }
    // hipcub temp storage (scan + select over n)
    size_t b1 = 0, b2 = 0;
    MVC_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b1, (int32_t *)nullptr, (int32_t *)nullptr, n, stream));
    hipcub::CountingInputIterator<int32_t> it(0);
    MVC_HIP(hipcub::DeviceSelect::Flagged(nullptr, b2, it, (int32_t *)nullptr, (int32_t *)nullptr,
                                          (int32_t *)nullptr, n, stream));
    cub_bytes = std::max(b1, b2);
    MVC_HIP(hipMalloc(&cub_tmp, cub_bytes));
    st_host.assign(V + 4, 0);
    const char *fg = getenv("MVC_FORCE_GENERIC");
    force_generic = fg && fg[0] == '1';
    const char *f1 = getenv("MVC_FORCE_MFMA1");
    force_mfma1 = f1 && f1[0] == '1';
    {
      hipDeviceProp_t prop;
      MVC_HIP(hipGetDeviceProperties(&prop, cf.device));
      n_cu = std::max(1, prop.multiProcessorCount);
    }
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_zresample_mfma_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_zresample_z1_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_zresample_z2_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    MVC_HIP(hipFuncSetAttribute((const void *)mvc_par_stats_partial_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    chains.resize(cf.n_chains);
    for (int c = 0; c < cf.n_chains; ++c) init_chain(chains[c], (uint32_t)(cf.first_chain + c), yh.data());
    MVC_HIP(hipStreamSynchronize(stream));
  }

  ~ParallelSampler() override {
    if (stream) hipStreamSynchronize(stream);
    for (auto &c : chains)
      for (void *p : c.owned) hipFree(p);
    for (void *p : {(void *)y, (void *)Y2, (void *)yt, (void *)lp_scratch, (void *)part1, (void *)part2, cub_tmp})
      if (p) hipFree(p);
    if (stream) hipStreamDestroy(stream);
  }

  void alloc_chain(Chain &c) {
    ParState &P = c.P;
    P.n = n; P.V = V; P.D = D; P.TC = TC; P.KC = KC;
    P.z = own<int32_t>(c, n);
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
    P.hyper = own<double>(c, 3 * V + 2);
    P.Kact = own<int32_t>(c, V);
    P.next_id = own<int32_t>(c, V);
    P.Ltot = own<int32_t>(c, V);
    c.L2pt = own<double>(c, V);
    c.cnew = own<double>(c, V);
    c.Koff = own<int32_t>(c, V + 1);
    c.status = own<int32_t>(c, V + 4);
    c.choice = own<int32_t>(c, n);
    c.flags = own<int32_t>(c, n);
    c.brank = own<int32_t>(c, n);
    c.blist = own<int32_t>(c, n);
    c.nbirth = own<int32_t>(c, 1);
    c.p2meta = own<int32_t>(c, V + 2);
    c.p2_c = own<int32_t>(c, TC);
    c.p2_tup = own<int32_t>(c, (size_t)TC * V);
    c.n2 = own<int32_t>(c, (size_t)V * KC);
    c.l2 = own<int32_t>(c, (size_t)V * KC);
    c.S1_2T = own<double>(c, (size_t)V * D * KC);
    c.lp2 = own<double>(c, (size_t)V * KC);
    c.btab = own<int32_t>(c, n);
    c.cnt = own<int32_t>(c, TC);
    c.pos_new = own<int32_t>(c, TC);
    c.tmp_dish = own<int32_t>(c, (size_t)V * TC);
    c.tmp_nt = own<int32_t>(c, TC);
    c.lcnt = own<int32_t>(c, (size_t)V * KC);
    c.jmap = own<int32_t>(c, (size_t)V * KC);
    c.histT = own<int32_t>(c, (size_t)n + 2);
    c.histL = own<int32_t>(c, (size_t)V * (TC + 2));
    c.mh_half = (size_t)n / 64 + 128;
    c.mh_scratch = own<double>(c, 2 * c.mh_half);
  }

  void init_chain(Chain &c, uint32_t gid, const double *yh) {
    c.gid = gid;
    alloc_chain(c);
    const InitState S = draw_initial_state(yh, n, V, D, cfg.seed, gid);
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
    std::vector<int32_t> st(V + 4, 0);
    st[0] = 4;
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
    std::vector<int32_t> ko(V + 1, 0);
    for (int v = 0; v < V; ++v) ko[v + 1] = ko[v] + c.K[v];
    MVC_HIP(hipMemcpyAsync(c.Koff, ko.data(), sizeof(int32_t) * ko.size(), hipMemcpyHostToDevice, stream));
    // the copy source must outlive the async copy
    MVC_HIP(hipStreamSynchronize(stream));
  }

  void rebuild_stats(Chain &c) {
    upload_koff(c);
    const int sk = sumK(c);
    if ((size_t)sk > part_cap) {
      if (part1) hipFree(part1);
      if (part2) hipFree(part2);
      part_cap = (size_t)sk + 64;
      part1 = dmalloc<double>((size_t)nchunk * part_cap * D);
      part2 = dmalloc<double>((size_t)nchunk * part_cap);
    }
    int Kmax = 1;
    for (int k : c.K) Kmax = std::max(Kmax, k);
    const size_t lds = sizeof(int) * (2 * 4096 + (size_t)Kmax + 1);
    const int dg = 0;
    hipEvent_t ev = nullptr;
    timers.begin("stats", &ev);
    hipLaunchKernelGGL(mvc_par_stats_partial_kernel, dim3(nchunk, V), dim3(256), lds, stream, c.P, (const double *)y,
                       (const double *)Y2, (const int32_t *)c.Koff, (int)part_cap, dg, part1, part2);
    MVC_HIP(hipGetLastError());
    const size_t tot = (size_t)sk * (D + 1);
    hipLaunchKernelGGL(mvc_par_stats_combine_kernel, dim3((unsigned)std::min<size_t>(4096, (tot + 255) / 256)), dim3(256),
                       0, stream, c.P, (const int32_t *)c.Koff, (int)part_cap, nchunk, (const double *)part1,
                       (const double *)part2);
    MVC_HIP(hipGetLastError());
    c.s1t_ok = false;
    if (SP > 0 && Kmax <= MVC_Z_KMAX) {
      if (!c.S1t) c.S1t = own<double>(c, (size_t)V * SP * 4 * 64);
      hipLaunchKernelGGL(mvc_par_s1tile_kernel, dim3(256), dim3(256), 0, stream, c.P, (const int32_t *)c.Koff, SP,
                         c.S1t);
      MVC_HIP(hipGetLastError());
      c.s1t_ok = true;
    }
    timers.end("stats", ev);
  }

  void launch_hyper(Chain &c, int do_mh, uint32_t sweep_ix) {
    MHArgs A;
    A.P = c.P;
    A.status = c.status;
    A.Koff = c.Koff;
    A.L2pt = c.L2pt;
    A.cnew = c.cnew;
    A.histT = c.histT;
    A.histL = c.histL;
    A.scratch = c.mh_scratch;
    A.half = c.mh_half;
    A.seed = cfg.seed;
    A.chain = c.gid;
    A.sweep = sweep_ix;
    A.do_mh = do_mh;
    hipEvent_t ev = nullptr;
    timers.begin("hyper", &ev);
    hipLaunchKernelGGL(mvc_par_hyper_kernel, dim3(1), dim3(256), 0, stream, A);
    MVC_HIP(hipGetLastError());
    timers.end("hyper", ev);
  }

  void ensure_lp(size_t per_wave) {
    if (per_wave <= lp_cap) return;
    if (lp_scratch) hipFree(lp_scratch);
    lp_cap = per_wave + 64;
    lp_scratch = dmalloc<double>((size_t)kZGrid * 4 * lp_cap);
  }

  Sweep make_sweep(Chain &c, uint32_t s) {
    Sweep A;
    A.P = c.P;
    A.y = y;
    A.Y2 = Y2;
    A.L2pt = c.L2pt;
    A.cnew = c.cnew;
    A.Koff = c.Koff;
    A.scratch = lp_scratch;
    A.choice = c.choice;
    A.blist = c.blist;
    A.p2meta = c.p2meta;
    A.p2_c = c.p2_c;
    A.p2_tup = c.p2_tup;
    A.n2 = c.n2;
    A.l2 = c.l2;
    A.S1_2T = c.S1_2T;
    A.lp2 = c.lp2;
    A.btab = c.btab;
    A.nbirth = c.nbirth;
    A.status = c.status;
    A.yt = yt;
    A.S1t = c.S1t;
    A.SP = SP;
    A.T = c.T;
    A.sumK = (int32_t)lp_cap;
    A.seed = cfg.seed;
    A.chain = c.gid;
    A.sweep = s;
    return A;
  }

  void sweep_chain(Chain &c, uint32_t s) {
    ensure_lp((size_t)sumK(c));
    upload_koff(c);
    Sweep A = make_sweep(c, s);
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    // MFMA path when the view width allows it
    int Kmax = 0, Kmin = 1 << 30;
    for (int k : c.K) { Kmax = std::max(Kmax, k); Kmin = std::min(Kmin, k); }
    const int sk = sumK(c);
    const size_t mfma_lds = ((size_t)c.T * 8 + (size_t)c.T * 4 + (size_t)V * c.T * 4 + (size_t)sk * 32 + 64) +
                            4 * ((size_t)sk * 16 + (size_t)V * 16) * sizeof(double);
    const bool use_mfma = !force_generic && D % 4 == 0 && D >= 16 && Kmax <= 255 && c.T <= MVC_MFMA_TMAX &&
                          mfma_lds <= 160 * 1024;
    const size_t z_lds = z_shared_bytes(c.T, V, sk);
    const bool use_z = !force_generic && !force_mfma1 && c.s1t_ok && Kmin >= 1 && Kmax <= MVC_Z_KMAX && c.T <= MVC_Z_TMAX &&
                       z_lds <= 160 * 1024;
    timers.begin("zresample", &e0);
    if (use_z) {
      // one block of MVC_Z_NW waves per CU
      const int ntile = (n + 15) / 16;
      const int grid = std::max(1, std::min(n_cu, (ntile + MVC_Z_NW - 1) / MVC_Z_NW));
      if (c.T <= 64)
        hipLaunchKernelGGL(mvc_par_zresample_z1_kernel, dim3(grid), dim3(MVC_Z_NW * 64), z_lds, stream, A);
      else
        hipLaunchKernelGGL(mvc_par_zresample_z2_kernel, dim3(grid), dim3(MVC_Z_NW * 64), z_lds, stream, A);
    } else if (use_mfma) {
      const int ntile = (n + 15) / 16;
      hipLaunchKernelGGL(mvc_par_zresample_mfma_kernel, dim3(std::min(2048, (ntile + 3) / 4)), dim3(256), mfma_lds,
                         stream, A);
    } else {
      hipLaunchKernelGGL(mvc_par_zresample_kernel, dim3(std::min(kZGrid, (n + 3) / 4)), dim3(256), 0, stream, A);
    }
    MVC_HIP(hipGetLastError());
    timers.end("zresample", e0);
    last_path_mfma = use_mfma || use_z;
    zpath = use_z ? 2 : (use_mfma ? 1 : 0);
    timers.begin("commit", &e1);
    MVC_HIP(hipMemsetAsync(c.cnt, 0, sizeof(int32_t) * TC, stream));
    hipLaunchKernelGGL(mvc_par_count_kernel, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, stream, n, c.T,
                       (const int32_t *)c.choice, c.cnt, c.flags);
    MVC_HIP(hipGetLastError());
    size_t bytes = cub_bytes;
    MVC_HIP(hipcub::DeviceScan::ExclusiveSum(cub_tmp, bytes, c.flags, c.brank, n, stream));
    bytes = cub_bytes;
    hipcub::CountingInputIterator<int32_t> it(0);
    MVC_HIP(hipcub::DeviceSelect::Flagged(cub_tmp, bytes, it, c.flags, c.blist, c.nbirth, n, stream));
    timers.end("commit", e1);
    hipEvent_t eb = nullptr;
    timers.begin("births", &eb);
    hipLaunchKernelGGL(mvc_par_births_kernel, dim3(1), dim3(64), 0, stream, A);
    MVC_HIP(hipGetLastError());
    timers.end("births", eb);
    timers.begin("commit", &e1);
    hipLaunchKernelGGL(mvc_par_commit_kernel, dim3(1), dim3(256), 0, stream, c.P, c.T, (const int32_t *)c.cnt,
                       (const int32_t *)c.p2meta, (const int32_t *)c.p2_c, (const int32_t *)c.p2_tup, c.pos_new,
                       c.tmp_dish, c.tmp_nt, c.lcnt, c.jmap, c.status);
    MVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(mvc_par_relabel_kernel, dim3(std::min(4096, (n + 255) / 256)), dim3(256), 0, stream, n, V,
                       (const int32_t *)c.choice, (const int32_t *)c.pos_new, (const int32_t *)c.brank,
                       (const int32_t *)c.btab, (const int32_t *)c.status, c.P.z);
    MVC_HIP(hipGetLastError());
    timers.end("commit", e1);
    // the one host synchronisation of a sweep: new T and dish counts
    MVC_HIP(hipMemcpyAsync(st_host.data(), c.status, sizeof(int32_t) * (V + 4), hipMemcpyDeviceToHost, stream));
    MVC_HIP(hipStreamSynchronize(stream));
    if (st_host[V + 1] != 0)
      throw Error(MVC_ERR_UNSUPPORTED, "parallel mode: table (4096) or dish (4095 per view) capacity exceeded");
    c.T = st_host[0];
    for (int v = 0; v < V; ++v) c.K[v] = st_host[1 + v];
    rebuild_stats(c);
    launch_hyper(c, 1, s);
    (void)e2;
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

  void set_state(int chain, const int32_t *table_of, int32_t T, const int32_t *dish_of, const double *hyper) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    const UserState U = check_user_state(n, V, table_of, T, dish_of);
    if (T > TC) throw Error(MVC_ERR_UNSUPPORTED, "set_state: more tables than the parallel-mode capacity (4096)");
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
    std::vector<int32_t> st(V + 4, 0);
    st[0] = T;
    up(c.status, st.data(), sizeof(int32_t) * st.size());
    MVC_HIP(hipStreamSynchronize(stream));
    c.T = T;
    rebuild_stats(c);
    launch_hyper(c, 0, 0);
    MVC_HIP(hipStreamSynchronize(stream));
  }
};

Sampler *make_parallel_sampler(const mvc_config &cfg, const double *const *views) {
  return new ParallelSampler(cfg, views);
}

}  // namespace mvc
