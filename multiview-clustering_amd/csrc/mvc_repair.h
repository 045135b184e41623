// mvc_repair.h — the in-order repair that makes the data-parallel pass an
// exact execution of the SEQUENTIAL schedule.  Included by
// mvc_parallel.hip (it uses that file's Coef / coef() and the wave helpers
// of mvc_internal.h).
//
// The reference sweeps customers in index order and customer i+1 sees
// customer i's move (multiview_gibbs.cpp:157-200).  A sweep here is:
//   1. phase A: every customer's conditional against the sweep-start state
//      (the MFMA producer + draw kernels); its choice is exact up to and
//      including the FIRST customer f whose choice is not "stay";
//   2. repair rounds, each two launches:
//        apply  (one block): commit customer cur = f (move; a birth draws its
//               dishes against the current state, opens the table and any new
//               dish), then open the next window [cur, cur + W);
//        eval   (G waves):   the exact conditional of every window customer
//               against the current state (one wavefront per customer, the
//               oracle's arithmetic), atomicMin of the first mover;
//      until every customer is final.  Customers between two movers stay, so
//      the state they were evaluated against is the one the sequential
//      schedule has at their turn;
//   3. compaction of dead tables / dishes (gated: only after a move), then
//      the hyperparameter MH.
// At steady state phase A finds no mover and step 2 is a single no-op round.
// Every decision equals oracle SeqSampler's, bit for bit.
#pragma once

struct Repair {
  int32_t cur;        // customers < cur are final
  int32_t pend;       // 1: choice[cur] was evaluated against the current state (commit it)
  int32_t win0, win1; // window evaluated by the last eval launch (win1 > win0: results pending)
  int32_t fmin;       // first mover found in the pending window (n: none)
  int32_t W;          // size of the next window
  int32_t done;       // every customer final
  int32_t overflow;   // 1: a birth needs a table slot beyond TC; 2: a dish slot beyond KC
  int32_t T;          // table positions (births append; dead tables keep their slot)
  int32_t T_ne;       // tables with n_t > 0
  int32_t mode;       // kSeqScan: windows on the grid (mvc_seq_eval_kernel); kSeqRun: the one-block run kernel
  int32_t pchoice;    // choice of customer cur when pend (its exact conditional draw)
  int32_t streak;     // consecutive stays seen by the run kernel since its last mover
  int32_t restride;   // 1: the run kernel's LDS layout is too small for T / the dish lists (host relaunches)
  int32_t moves, births, newdish, rounds;
  int32_t lastm, gapq;  // the last mover, and the moving average (x16) of the gaps between movers
  int32_t vpoff;        // 1: value prediction stopped for this sweep (predictions miss, or a dish list > 128)
  int32_t vpsteps, vphits;   // vp steps, and those whose predictions all held
  int32_t dbg[8];       // MVC_RUN_CHECK: the first index check that failed in a run kernel (code, values), 0: none
  int32_t Klist[MVC_MAXV];
  unsigned long long prof[22];  // MVC_RUN_PROF builds: run-kernel phase ticks (100 MHz), steps, decided customers, phase-A hits;
                                // [12..19] the grid-wide fin kernel's (combine, lm, table scores, weights, draw, commit, decided, commits),
                                // [20] / [21] its wall ticks / shader clocks from decision start to exit (the effective clock)
};

constexpr int32_t kSeqScan = 0, kSeqRun = 1;

// MVC_RUN_PROF builds (scripts/build_variant.sh NAME -DMVC_RUN_PROF): thread 0
// of the run kernel accumulates wall-clock ticks (100 MHz) per phase in LDS
// (no global read-modify-write inside the timed phases) and adds them to
// R->prof when the kernel exits; the host prints them per sweep.  Tuning aid only.
#ifdef MVC_RUN_PROF
__shared__ unsigned long long mvc_prof_lds[12];
#define RUN_T0() uint64_t _rt = wall_clock64()
#define RUN_MARK(k) do { const uint64_t _n = wall_clock64(); \
    if (threadIdx.x == 0) mvc_prof_lds[k] += _n - _rt; _rt = _n; } while (0)
#else
#define RUN_T0() do {} while (0)
#define RUN_MARK(k) do {} while (0)
#endif
// run kernel block: 8 waves (256 VGPRs each: the per-customer evaluation
// spills at the 128 VGPRs of a 16-wave block)
constexpr int kSeqRunThreads = 512, kSeqRunWaves = kSeqRunThreads / 64;
// the lane-column run kernel: 4 waves, one per SIMD (its evaluation is issue-
// bound; a second wave per SIMD would halve the first customer's rate)
constexpr int kSeqLcThreads = 256;
// the small chains' lane loop (mvc_seq_run_kernel<5>): 8 waves, two per SIMD,
// 64 customers per step (its registers allow it; the general lane kernel <6>
// and the lane-column kernels keep 4 waves)
constexpr int kLaneSmallThreads = 512;

// LDS layout of the run kernel's per-wave scratch (host-chosen at launch):
// lp [V][ks] | e [ts + 16] | B, C [ts/16 + 2]; nws waves speculate.
// lds = 0: the per-wave global scratch (SeqArgs.scr) instead.
// LDS of the run kernel: the state cache (SCache: n_t [ts], dish [V][ts],
// d_l, d_n [V][ks], Klist, Ltot [V], T, T_ne; c0, cb, Q, xm, ym, cbm [V][ks];
// lmass [ts]; S1T [V][D][ks] when s1) and the per-wave scratch (SeqScratch).
struct SeqLds {
  int32_t lds, nws, ks, ts;
  int32_t limit;        // stays in a row after which the run kernel hands over to the grid windows
  int32_t s1;           // S1 cached in LDS
  int64_t cache_dbl;    // doubles of the state cache (the per-wave scratch follows)
  int64_t stride;       // doubles per wave
  int32_t ring;         // customers in the staged-row ring (power of 2, after the per-wave scratch; 0: none)
  int32_t pfn;          // customers prefetched into the ring per step
  int32_t tw;           // waves per customer (1: seq_resample; kSeqRunWaves: seq_resample_wide); nws customers per step
  int32_t lc;           // 1: the lane-column evaluation (seq_resample_lc; LDS layout with S1 cached, ts <= 512); 2: + value prediction
  int64_t vpo;          // lc == 2: offset (doubles) of the overlay's S1 columns [kVpE][D] in the dynamic LDS
  int64_t dyn;          // bytes of dynamic LDS of the launch
  int32_t small;        // lc == 3: every dish list and the tables <= kLaneSmall (mvc_seq_run_kernel<5>)
  int32_t fill;         // MVC_LDS_FILL diagnostics: >= 0 fills the block's LDS with this byte at launch
  int32_t chk;          // MVC_RUN_CHECK diagnostics: check every index a commit writes through (R->dbg)
};

// MVC_RUN_CHECK: the first failed index check of the run kernel's block
// (code, then up to 7 values); a failed check skips the write it guards and
// the loop stops at its next barrier, so a bad index is reported instead of
// becoming a wild store.
__shared__ int mvc_run_bad[8];
__device__ __forceinline__ bool run_chk(bool ok, int code, int a = 0, int b = 0, int c = 0, int d = 0, int e = 0,
                                        int f = 0) {
  if (ok) return true;
  if (atomicCAS(&mvc_run_bad[0], 0, code) == 0) {
    mvc_run_bad[1] = a; mvc_run_bad[2] = b; mvc_run_bad[3] = c;
    mvc_run_bad[4] = d; mvc_run_bad[5] = e; mvc_run_bad[6] = f;
  }
  return false;
}
// ring slot: y rows [V][D], Y2 [V], z (as a double)
__host__ __device__ inline int64_t seq_ring_slot(int V, int D) { return (int64_t)V * D + V + 1; }

// lp row stride of the LDS scratch: the lane-column evaluation stores dish j
// of a row at j + j / 32 (lc_lpx), so the table gathers of dishes j and j + 32
// (the same bank of ds_read_b64 otherwise) fall on different banks
__host__ __device__ inline int seq_lps(int ks) { return ks + (ks >> 5) + 1; }
__host__ __device__ inline int64_t seq_lds_stride(int V, int D, int ks, int ts) {
  // lp [V][seq_lps] | aux [V][ks] | e | B, C | mv | koff | ys [V][D] + Y2 [V] + lm_v [V] + member maxima [4]
  return (int64_t)V * seq_lps(ks) + (int64_t)V * ks + ts + 16 + ts / 16 + 2 + V + V + 2 + (int64_t)V * D + V + V + 4;
}
__host__ __device__ inline int64_t seq_lds_cache(int V, int D, int ks, int ts, bool s1) {
  const int64_t ints = (int64_t)ts + (int64_t)V * ts + 2 * (int64_t)V * ks + 2 * V + 2;
  return (ints + 1) / 2 + 7 * (int64_t)V * ks + ts + (s1 ? (int64_t)V * D * ks : 0);
}

struct SeqArgs {
  ParState P;
  const double *y;        // [V][n][D]
  const double *Y2;       // [V][n]
  const double *L2pt;     // [V]
  const double *cnew;     // [V]
  int32_t *choice;        // [n]
  int32_t *status;        // [2V+4]
  int32_t *Koff;          // [V+1] prefix of the dish counts (rewritten by the compaction)
  Repair *R;
  double *scr;            // per wave: SeqScratch layout, stride scr_stride doubles
  int64_t scr_stride;
  int32_t G;              // waves of the eval grid
  int32_t Wmin, Wmax;     // window size after a mover / cap of the doubling
  uint64_t seed;
  uint32_t chain, sweep;
};

namespace {

// per-wave scratch: lp [V][ks] | aux [V][ks] (dish terms) | table scores /
// weights [ts + 16] | block sums [ts/16 + 2] | per-view max [V] | view
// offsets [V + 1] | (run kernel) y rows [V][D] + Y2 [V] | (global) the
// dish-draw tree levels
struct SeqScratch {
  double *lp, *aux, *e, *B, *mv, *tree;
  int32_t *koff;
  double *ys;   // run kernel: the customer's y rows [V][D] and Y2 [V]
  int lps;      // lp / aux stride per view
  __device__ void carve(double *base, int V, int ks, int ts, int lp_stride) {
    lps = lp_stride;
    lp = base;
    aux = lp + (size_t)V * lp_stride;
    e = aux + (size_t)V * ks;
    B = e + ts + 16;
    mv = B + ts / 16 + 2;
    koff = (int32_t *)(mv + V);   // [V + 1] view offsets, then [V] K_act
    ys = mv + V + V + 2;
  }
  double *wide;   // global scratch: the wide evaluation's shared values (seq_wide_len)
  __device__ SeqScratch(const SeqArgs &A, int wave) {
    carve(A.scr + (int64_t)wave * A.scr_stride, A.P.V, A.P.KC, A.P.TC, A.P.KC);
    tree = ys;   // the global scratch has no staged rows
    ys = nullptr;
    wide = A.scr + (int64_t)(wave + 1) * A.scr_stride - (17 * A.P.V + 16);
  }
  // run kernel, LDS (no dish-draw tree)
  __device__ SeqScratch(double *base, int V, int ks, int ts) {
    carve(base, V, ks, ts, seq_lps(ks));
    tree = nullptr;
    wide = nullptr;
  }
};
__host__ __device__ inline int64_t seq_scratch_head(int V, int ks, int ts) {
  return 2 * (int64_t)V * ks + ts + 16 + ts / 16 + 2 + V + V + 2;
}
__host__ inline int64_t seq_scratch_stride(int V, int TC, int KC) {
  // tree levels: K+1 leaves, then ceil(./64) ... (< (K+1)/63 + 3 more)
  const int64_t leaves = (int64_t)KC + 1;
  const int64_t tree = leaves + leaves / 63 + 8;
  // + the wide evaluation's lm_v [V], member maxima [8], per-member view maxima / counts [8][V] x 2
  return seq_scratch_head(V, KC, TC) + tree + 64 + 17 * (int64_t)V + 16;
}

// oracle pw16: pairs (c, c + h) for h = 1, 2, 4, 8
__device__ __forceinline__ double pw16_seq(const double *x) {
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = x[c];
#pragma unroll
  for (int h = 1; h < 16; h <<= 1)
#pragma unroll
    for (int c = 0; c < 16; c += 2 * h) a[c] = a[c] + a[c + h];
  return a[0];
}
// oracle pw16_select: the pw16 levels in registers (static indices only, so
// nothing goes to scratch), descent left iff R == 0 || r < L.
__device__ __forceinline__ int pw16_select_seq(const double *x, double r) {
  double l0[16], l1[8], l2[4], l3[2];
#pragma unroll
  for (int c = 0; c < 16; ++c) l0[c] = x[c];
#pragma unroll
  for (int c = 0; c < 8; ++c) l1[c] = l0[2 * c] + l0[2 * c + 1];
#pragma unroll
  for (int c = 0; c < 4; ++c) l2[c] = l1[2 * c] + l1[2 * c + 1];
#pragma unroll
  for (int c = 0; c < 2; ++c) l3[c] = l2[2 * c] + l2[2 * c + 1];
  int idx = 0;   // node index at the current level
  auto step = [&](double L, double R) {
    idx *= 2;
    if (!(R == 0.0 || r < L)) {
      r = r - L;
      idx += 1;
    }
  };
  step(l3[0], l3[1]);
  {
    double L = l2[0], R = l2[1];
#pragma unroll
    for (int q = 1; q < 2; ++q) if (q == idx) { L = l2[2 * q]; R = l2[2 * q + 1]; }
    step(L, R);
  }
  {
    double L = l1[0], R = l1[1];
#pragma unroll
    for (int q = 1; q < 4; ++q) if (q == idx) { L = l1[2 * q]; R = l1[2 * q + 1]; }
    step(L, R);
  }
  {
    double L = l0[0], R = l0[1];
#pragma unroll
    for (int q = 1; q < 8; ++q) if (q == idx) { L = l0[2 * q]; R = l0[2 * q + 1]; }
    step(L, R);
  }
  return idx;
}

// pw16_select across a wave: lane base + l (l < 16, base a multiple of 16)
// holds element l; r wave-uniform.  Levels by DPP row shifts (node c at
// offset h = x[c] + x[c + h], the pw16 association), descent left iff R == 0
// || r < L.
__device__ __forceinline__ int pw16_select_wave(double x, double r, int base = 0) {
  const double l1 = x + down_d<1>(x);
  const double l2 = l1 + down_d<2>(l1);
  const double l3 = l2 + down_d<4>(l2);
  int lo = 0;
#define MVC_PW16_DESCEND(VAL, H)                              \
  {                                                           \
    const double a = readlane_d((VAL), base + lo);            \
    const double b = readlane_d((VAL), base + lo + (H));      \
    if (!(b == 0.0 || r < a)) { r = r - a; lo = lo + (H); }   \
  }
  MVC_PW16_DESCEND(l3, 8)
  MVC_PW16_DESCEND(l2, 4)
  MVC_PW16_DESCEND(l1, 2)
  MVC_PW16_DESCEND(x, 1)
#undef MVC_PW16_DESCEND
  return lo;
}

__device__ __forceinline__ int wave_count(bool p) { return __popcll(__ballot(p)); }

// acc + sum_d a[d] b[d * bs], one fma chain in ascending d (the oracle's
// fma_dot order).  The loads of each 8-wide batch are issued before its
// fmas, so a chain of D fmas waits on D/8 memory latencies, not D.
__device__ __forceinline__ double fma_dot_strided(const double *a, const double *b, size_t bs, int D, double acc) {
  int d = 0;
  for (; d + 8 <= D; d += 8) {
    double xa[8], xb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xa[u] = a[d + u];
      xb[u] = b[(size_t)(d + u) * bs];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_fma(xa[u], xb[u], acc);
  }
  for (; d < D; ++d) acc = __builtin_fma(a[d], b[(size_t)d * bs], acc);
  return acc;
}
__device__ __forceinline__ double fma_sq_strided(const double *b, size_t bs, int D) {
  double acc = 0.0;
  int d = 0;
  for (; d + 16 <= D; d += 16) {
    double xb[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) xb[u] = b[(size_t)(d + u) * bs];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = __builtin_fma(xb[u], xb[u], acc);
  }
  for (; d < D; ++d) acc = __builtin_fma(b[(size_t)d * bs], b[(size_t)d * bs], acc);
  return acc;
}

// Where the per-customer evaluation reads the mutable chain state: the global
// arrays (grid kernels), or the run kernel's LDS cache of them (same values;
// the commit writes both).  Dish arrays are [v * ks + j], tables [v * ts + p],
// S1 [(v * D + d) * s1s + j].
struct SView {
  const int32_t *n_t, *dish;
  const int32_t *d_l, *d_n;
  const double *c0, *cb, *Q;
  const double *xm, *ym, *cbm;   // self-removal coefficient parts (nullptr: computed per use)
  const double *lmass;           // [ts] log(n_t - sigma_g)
  const double *S1T;
  const int32_t *Klist, *Ltot, *T, *T_ne;
  int ts, ks, s1s;
};
__device__ __forceinline__ SView global_view(const SeqArgs &A) {
  const ParState &P = A.P;
  SView G;
  G.n_t = P.n_t; G.dish = P.dish;
  G.d_l = P.d_l; G.d_n = P.d_n;
  G.c0 = P.c0; G.cb = P.cb; G.Q = P.Q;
  G.xm = G.ym = G.cbm = nullptr;
  G.lmass = P.lmass;
  G.S1T = P.S1T;
  G.Klist = A.R->Klist; G.Ltot = P.Ltot; G.T = &A.R->T; G.T_ne = &A.R->T_ne;
  G.ts = P.TC; G.ks = P.KC; G.s1s = P.KC;
  return G;
}

// The customer's data: y rows [V][D] and Y2 [V], either in global memory or
// staged in the wave's LDS scratch (run kernel).
struct Cust {
  const double *y;    // y[v * ystride + d]
  size_t ystride;
  const double *Y2;   // Y2[v * y2stride]
  size_t y2stride;
};
__device__ __forceinline__ Cust global_cust(const SeqArgs &A, int i) {
  Cust c;
  c.y = A.y + (size_t)i * A.P.D;
  c.ystride = (size_t)A.P.n * A.P.D;
  c.Y2 = A.Y2 + i;
  c.y2stride = (size_t)A.P.n;
  return c;
}

// lp of every listed dish of view v for customer i (the customer's own dish
// j0 with itself removed) into lp[0..K); oracle
// eval_view_seq / eval_view.  Returns the number of included dishes (l' > 0)
// and their max in *mx.
__device__ int seq_view_lp(const SeqArgs &A, const SView &W, const Cust &C, int v, bool alive, int j0, double *lp,
                           double *mx_out) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int D = P.D, ks = W.ks;
  const int K = W.Klist[v];
  const double tau = P.hyper[v];
  const double Y2i = C.Y2[(size_t)v * C.y2stride];
  const double hy = 0.5 * Y2i;
  const double h = (-0.5 * Y2i) / tau;
  const double *yrow = C.y + (size_t)v * C.ystride;
  const double *S1v = W.S1T + (size_t)v * D * W.s1s;
  const int l0 = W.d_l[v * ks + j0];
  const int l0p = alive ? l0 : l0 - 1;
  double mx = -MVC_PM_INF;
  int nl = 0;
  for (int base = 0; base < K; base += 64) {
    const int j = base + lane;
    bool inc = false;
    if (j < K) {
      const double G = fma_dot_strided(yrow, S1v + j, (size_t)W.s1s, D, 0.0);
      double val;
      int l;
      if (j == j0) {
        l = l0p;
        const double Gp = G - Y2i;
        const double Qp = (W.Q[v * ks + j] - 2.0 * G) + Y2i;
        const Coef c = coef(W.d_n[v * ks + j] - 1, Qp, tau, A.L2pt[v], D);
        val = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
      } else {
        l = W.d_l[v * ks + j];
        val = __builtin_fma(G + hy, W.cb[v * ks + j], W.c0[v * ks + j]) + h;
      }
      lp[j] = val;
      inc = l > 0;
      if (inc && val > mx) mx = val;
    }
    nl += wave_count(inc);
  }
  *mx_out = wave_max(mx);
  return nl;
}

__device__ __forceinline__ int row16_isum(int x) {
  x += __shfl_xor(x, 1, 64);
  x += __shfl_xor(x, 2, 64);
  x += __shfl_xor(x, 4, 64);
  x += __shfl_xor(x, 8, 64);
  return x;
}

// Exact conditional draw of customer i against the current state (oracle
// ParallelSampler::resample_customer + eval_view_seq): a table position, or
// -1 = birth.  p0 = z[i] (the customer's table before this sweep's
// decision).  One wavefront, shaped for latency (the repair's serial chain):
// every view's dishes in one lane-parallel pass (lp, then the weighted
// terms), the per-view column sums / pw16 / marginal of four views at once
// on the four 16-lane rows, table weights with their block sums by row DPP,
// running block totals through readlanes.  Same operations in the same
// order per quantity as the oracle, so the same bits.
__device__ int seq_resample(const SeqArgs &A, const SView &W, const Cust &C, int i, int p0, const SeqScratch &S) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63, row = lane >> 4, col = lane & 15;
  const int V = P.V, D = P.D, ts = W.ts, ks = W.ks, lps = S.lps;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int np0 = W.n_t[p0] - 1;
  const bool alive = np0 > 0;
  const int Tne_i = *W.T_ne - (alive ? 0 : 1);
  const double mass0 = (double)np0 - sg;
  const double lmass0 = (np0 >= 1 && mass0 > 0.0) ? mvc_log(mass0) : 0.0;   // the own table, customer removed
  RUN_T0();
  if (lane == 0) {   // offsets of the views in the concatenated dish list
    int acc = 0;
    for (int v = 0; v < V; ++v) {
      S.koff[v] = acc;
      acc += W.Klist[v];
    }
    S.koff[V] = acc;
  }
  __threadfence_block();
  const int NK = S.koff[V];
  // pass 1: lp of every listed dish (the own dish j0 with the customer removed)
  for (int g0 = 0; g0 < NK; g0 += 64) {
    const int g = g0 + lane;
    if (g < NK) {
      int v = 0;
      while (g >= S.koff[v + 1]) ++v;
      const int j = g - S.koff[v];
      const double tau = P.hyper[v];
      const double Y2i = C.Y2[(size_t)v * C.y2stride];
      const double hy = 0.5 * Y2i;
      const double h = (-0.5 * Y2i) / tau;
      const double G = fma_dot_strided(C.y + (size_t)v * C.ystride, W.S1T + (size_t)v * D * W.s1s + j, (size_t)W.s1s, D, 0.0);
      double val;
      if (j == W.dish[v * ts + p0]) {
        const double Gp = G - Y2i;
        const double Qp = (W.Q[v * ks + j] - 2.0 * G) + Y2i;
        double c0, cb;
        if (W.xm) {
          c0 = W.xm[v * ks + j] - (0.5 * Qp) / W.ym[v * ks + j];
          cb = W.cbm[v * ks + j];
        } else {
          const Coef c = coef(W.d_n[v * ks + j] - 1, Qp, tau, A.L2pt[v], D);
          c0 = c.c0;
          cb = c.cb;
        }
        val = __builtin_fma(Gp + hy, cb, c0) + h;
      } else {
        val = __builtin_fma(G + hy, W.cb[v * ks + j], W.c0[v * ks + j]) + h;
      }
      S.lp[v * lps + j] = val;
    }
  }
  __threadfence_block();
  // per view (four views at once, view vg + row): max over the included
  // dishes (l' > 0) and the new dish, and K_act
  double lfn_r = 0.0, m_r = 0.0;   // of this row's view, per group (recomputed below)
  for (int vg = 0; vg < V; vg += 4) {
    const int v = vg + row;
    double mx = -MVC_PM_INF;
    int cnt = 0;
    if (v < V) {
      const int K = W.Klist[v];
      const int j0 = W.dish[v * ts + p0];
      for (int j = col; j < K; j += 16) {
        const int l = W.d_l[v * ks + j] - ((j == j0 && !alive) ? 1 : 0);
        if (l > 0) {
          ++cnt;
          const double x = S.lp[v * lps + j];
          if (x > mx) mx = x;
        }
      }
    }
    mx = row16_max(mx);
    cnt = row16_isum(cnt);
    if (v < V && col == 0) {
      const double Y2i = C.Y2[(size_t)v * C.y2stride];
      const double lfn = A.cnew[v] + (-0.5 * Y2i) / P.hyper[v];
      S.mv[v] = lfn > mx ? lfn : mx;
      S.koff[V + 1 + v] = cnt;   // K_act (koff has room: [V + 1] offsets then [V] counts)
    }
  }
  __threadfence_block();
  // pass 2: the weighted terms w_j exp(lp_j - m_v) of every included dish, 0 otherwise
  for (int g0 = 0; g0 < NK; g0 += 64) {
    const int g = g0 + lane;
    if (g < NK) {
      int v = 0;
      while (g >= S.koff[v + 1]) ++v;
      const int j = g - S.koff[v];
      const int l = W.d_l[v * ks + j] - ((j == W.dish[v * ts + p0] && !alive) ? 1 : 0);
      double t = 0.0;
      if (l > 0) {
        double w = (double)l - P.hyper[2 * V + v];
        if (w < 0.0) w = 0.0;
        t = w * mvc_exp(S.lp[v * lps + j] - S.mv[v]);
      }
      S.aux[v * lps + j] = t;
    }
  }
  __threadfence_block();
  // per view (four at once): column partials j mod 16 in ascending j, pw16,
  // the new dish, lm_v; s_new in view order
  double s_new = mvc_log(ag + sg * (double)Tne_i);
  for (int vg = 0; vg < V; vg += 4) {
    const int v = vg + row;
    double lm = 0.0;
    double cs = 0.0;
    if (v < V) {
      const int K = W.Klist[v];
      for (int j = col; j < K; j += 16) cs = cs + S.aux[v * lps + j];
    }
    double Sv = row_pw16(cs);
    if (v < V) {
      const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
      const double Y2i = C.Y2[(size_t)v * C.y2stride];
      const double lfn = A.cnew[v] + (-0.5 * Y2i) / tau;
      const double m = S.mv[v];
      double wn = alpha + (double)S.koff[V + 1 + v] * sigma;
      if (wn < 0.0) wn = 0.0;
      Sv = Sv + wn * mvc_exp(lfn - m);
      const double denom = alpha + (double)(W.Ltot[v] - (alive ? 0 : 1));
      lm = (denom <= 0.0) ? lfn : (m + mvc_log(Sv)) - mvc_log(denom);
    }
    for (int r = 0; r < 4 && vg + r < V; ++r) s_new = s_new + readlane_d(lm, 16 * r);
  }
  (void)lfn_r; (void)m_r;
  RUN_MARK(0);
  // table scores: log(n_p' - sigma_g) + sum_v lp_{v, dish_v(p)} (view order)
  const int T = *W.T;
  const int TB = (T + 15) / 16;
  double M = -MVC_PM_INF;
  // four 64-table chunks per step: their count / log-mass / dish loads are
  // issued together, then the lp gathers (hundreds of tables in the early
  // sweeps of a cold start: the loads, not the adds, are the latency)
  constexpr int kU = 4;
  for (int q0 = 0; q0 < TB * 16; q0 += 64 * kU) {
    int np[kU];
    double lm[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = q0 + 64 * u + lane;
      np[u] = p < T ? W.n_t[p] - (p == p0 ? 1 : 0) : 0;
      lm[u] = p < T ? ((p == p0) ? lmass0 : W.lmass[p]) : 0.0;
    }
    double sp[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = q0 + 64 * u + lane;
      const double mass = (double)np[u] - sg;
      sp[u] = (p < T && np[u] >= 1 && mass > 0.0) ? lm[u] : -MVC_PM_INF;
    }
    for (int v = 0; v < V; ++v) {
      int dj[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = q0 + 64 * u + lane;
        dj[u] = (sp[u] != -MVC_PM_INF) ? W.dish[v * ts + p] : 0;
      }
      double lv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) lv[u] = S.lp[v * lps + dj[u]];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (sp[u] != -MVC_PM_INF) sp[u] = sp[u] + lv[u];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int p = q0 + 64 * u + lane;
      if (p < TB * 16) S.e[p] = sp[u];
      if (sp[u] > M) M = sp[u];
    }
  }
  M = wave_max(M);
  if (s_new > M) M = s_new;
  __threadfence_block();
  RUN_MARK(1);
  // weights exp(sp - M) (0 for excluded / padding), block sums by row pw16
  for (int q0 = 0; q0 < TB * 16; q0 += 64) {
    const int p = q0 + lane;
    double wgt = 0.0;
    if (p < TB * 16) {
      const double x = S.e[p];
      wgt = x != -MVC_PM_INF ? mvc_exp(x - M) : 0.0;
      S.e[p] = wgt;
    }
    const double Bv = row_pw16(wgt);
    const int b = (q0 >> 4) + row;
    if (col == 0 && b < TB) S.B[b] = Bv;
  }
  __threadfence_block();
  RUN_MARK(2);
  // running block totals C_b (in block order) through readlanes of the block sums
  double tot = 0.0;
  for (int b0 = 0; b0 < TB; b0 += 64) {
    const double Bl = (b0 + lane < TB) ? S.B[b0 + lane] : 0.0;
    const int nb = min(64, TB - b0);
    for (int k = 0; k < nb; ++k) tot = tot + readlane_d(Bl, k);
  }
  const double Wt = mvc_exp(s_new - M) + tot;
  double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * Wt;
  int pick = -1;
  if (r < tot) {
    double c = 0.0, cprev = 0.0;
    int bsel = TB - 1;
    bool found = false;
    for (int b0 = 0; b0 < TB && !found; b0 += 64) {
      const double Bl = (b0 + lane < TB) ? S.B[b0 + lane] : 0.0;
      const int nb = min(64, TB - b0);
      for (int k = 0; k < nb; ++k) {
        const double c2 = c + readlane_d(Bl, k);
        if (r < c2) {
          bsel = b0 + k;
          cprev = c;
          found = true;
          break;
        }
        c = c2;
      }
    }
    r = r - cprev;
    const double x = lane < 16 ? S.e[bsel * 16 + lane] : 0.0;
    pick = bsel * 16 + pw16_select_wave(x, r);
  }
  RUN_MARK(3);
  return pick;
}

// seq_resample by the whole block for ONE customer (run kernel, global-scratch
// layout: T or the dish lists too large for the LDS cache, e.g. the Reuters
// transient with T ~ 18k tables and thousands of dishes per view).  Member r
// of the tw waves takes every tw-th 64-dish chunk of the concatenated dish
// list (two dishes per lane in flight) for the lp and the terms, a stride of
// the per-view max / count scans, and every tw-th 64-table chunk; member 0
// does the order-sensitive sums (column partials, running block totals) and
// the draw.  Same operations in the same order per quantity as seq_resample,
// so the same bits.  Block-wide (seven __syncthreads); S is the team's
// scratch (wave 0's), S.wide its shared values.  Returns the pick on member 0.
// rest_only: pass 1 (the lp rows) and the per-member max / count already ran
// elsewhere (the grid-wide evaluation, mvc_seq_wide_lp_kernel): S.lp holds the
// rows and member row 0 of pmx / pcnt the combined max / count per view.
__device__ int seq_resample_wide(const SeqArgs &A, const SView &W, const Cust &C, int i, int p0, const SeqScratch &S,
                                 int r, int tw, bool act, bool rest_only = false) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63, row = lane >> 4, col = lane & 15;
  const int V = P.V, D = P.D, ts = W.ts, ks = W.ks, lps = S.lps;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  double *lmv = S.wide, *mxr = lmv + V, *pmx = mxr + 8, *pcnt = pmx + 8 * V;
  int32_t *kact = S.koff + V + 1;
  int np0 = 0, Tne_i = 0, NK = 0;
  bool alive = false;
  double lmass0 = 0.0;
  RUN_T0();
  if (act) {
    np0 = W.n_t[p0] - 1;
    alive = np0 > 0;
    Tne_i = *W.T_ne - (alive ? 0 : 1);
    const double mass0 = (double)np0 - sg;
    lmass0 = (np0 >= 1 && mass0 > 0.0) ? mvc_log(mass0) : 0.0;
    for (int v = 0; v < V; ++v) NK += W.Klist[v];
  }
  auto locate = [&](int g, int &v, int &j) {
    v = 0;
    int off = 0;
    while (v + 1 < V && g >= off + W.Klist[v]) { off += W.Klist[v]; ++v; }
    j = g - off;
  };
  auto lp_val = [&](int v, int j, double G) -> double {
    const double tau = P.hyper[v];
    const double Y2i = C.Y2[(size_t)v * C.y2stride];
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau;
    if (j == W.dish[v * ts + p0]) {
      const double Gp = G - Y2i;
      const double Qp = (W.Q[v * ks + j] - 2.0 * G) + Y2i;
      const Coef c = coef(W.d_n[v * ks + j] - 1, Qp, tau, A.L2pt[v], D);
      return __builtin_fma(Gp + hy, c.cb, c.c0) + h;
    }
    return __builtin_fma(G + hy, W.cb[v * ks + j], W.c0[v * ks + j]) + h;
  };
  // the customer's y rows in LDS (V D <= 2048): pass 1's y operands become
  // LDS reads, so its global loads are S1 only (16 per dish in flight)
  constexpr int kWideY = 2048;
  __shared__ double s_yw[kWideY];
  const bool ylds = V * D <= kWideY;
  if (ylds && !rest_only) {
    if (act)
      for (int e = threadIdx.x; e < V * D; e += blockDim.x) {
        const int v = e / D, d = e - v * D;
        s_yw[e] = C.y[(size_t)v * C.ystride + d];
      }
    __syncthreads();
  }
  // pass 1: lp, two dishes per lane (chunks c and c + tw), two fma chains in ascending d
  if (act && ylds && !rest_only) {
    for (int c = r; 64 * c < NK; c += 2 * tw) {
      const int ga = 64 * c + lane, gb = 64 * (c + tw) + lane;
      const bool va = ga < NK, vb = gb < NK;
      int v_a = 0, j_a = 0, v_b = 0, j_b = 0;
      if (va) locate(ga, v_a, j_a);
      if (vb) locate(gb, v_b, j_b);
      const int oa = v_a * D, ob = v_b * D;
      const double *sa = W.S1T + (size_t)v_a * D * W.s1s + j_a, *sb = W.S1T + (size_t)v_b * D * W.s1s + j_b;
      const size_t bs = (size_t)W.s1s;
      double acc_a = 0.0, acc_b = 0.0;
      int d = 0;
      for (; d + 16 <= D; d += 16) {
        double za[16], zb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          za[u] = sa[(size_t)(d + u) * bs];
          zb[u] = sb[(size_t)(d + u) * bs];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc_a = __builtin_fma(s_yw[oa + d + u], za[u], acc_a);
          acc_b = __builtin_fma(s_yw[ob + d + u], zb[u], acc_b);
        }
      }
      for (; d < D; ++d) {
        acc_a = __builtin_fma(s_yw[oa + d], sa[(size_t)d * bs], acc_a);
        acc_b = __builtin_fma(s_yw[ob + d], sb[(size_t)d * bs], acc_b);
      }
      if (va) S.lp[v_a * lps + j_a] = lp_val(v_a, j_a, acc_a);
      if (vb) S.lp[v_b * lps + j_b] = lp_val(v_b, j_b, acc_b);
    }
  }
  if (act && !ylds && !rest_only) {
    for (int c = r; 64 * c < NK; c += 2 * tw) {
      const int ga = 64 * c + lane, gb = 64 * (c + tw) + lane;
      const bool va = ga < NK, vb = gb < NK;
      int v_a = 0, j_a = 0, v_b = 0, j_b = 0;
      if (va) locate(ga, v_a, j_a);
      if (vb) locate(gb, v_b, j_b);
      const double *ya = C.y + (size_t)v_a * C.ystride, *yb = C.y + (size_t)v_b * C.ystride;
      const double *sa = W.S1T + (size_t)v_a * D * W.s1s + j_a, *sb = W.S1T + (size_t)v_b * D * W.s1s + j_b;
      const size_t bs = (size_t)W.s1s;
      double acc_a = 0.0, acc_b = 0.0;
      int d = 0;
      for (; d + 8 <= D; d += 8) {
        double xa[8], za[8], xb[8], zb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          xa[u] = ya[d + u];
          za[u] = sa[(size_t)(d + u) * bs];
          xb[u] = yb[d + u];
          zb[u] = sb[(size_t)(d + u) * bs];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc_a = __builtin_fma(xa[u], za[u], acc_a);
          acc_b = __builtin_fma(xb[u], zb[u], acc_b);
        }
      }
      for (; d < D; ++d) {
        acc_a = __builtin_fma(ya[d], sa[(size_t)d * bs], acc_a);
        acc_b = __builtin_fma(yb[d], sb[(size_t)d * bs], acc_b);
      }
      if (va) S.lp[v_a * lps + j_a] = lp_val(v_a, j_a, acc_a);
      if (vb) S.lp[v_b * lps + j_b] = lp_val(v_b, j_b, acc_b);
    }
  }
  __syncthreads();
  // per-member max / count of the included dishes, four views at once (rows)
  if (act && !rest_only) {
    for (int vg = 0; vg < V; vg += 4) {
      const int v = vg + row;
      double mx = -MVC_PM_INF;
      int cnt = 0;
      if (v < V) {
        const int K = W.Klist[v];
        const int j0 = W.dish[v * ts + p0];
        for (int j = col + 16 * r; j < K; j += 16 * tw) {
          const int l = W.d_l[v * ks + j] - ((j == j0 && !alive) ? 1 : 0);
          if (l > 0) {
            ++cnt;
            const double x = S.lp[v * lps + j];
            if (x > mx) mx = x;
          }
        }
      }
      mx = row16_max(mx);
      cnt = row16_isum(cnt);
      if (v < V && col == 0) {
        pmx[r * V + v] = mx;
        pcnt[r * V + v] = (double)cnt;
      }
    }
  }
  __syncthreads();
  if (act && r == 0) {   // combine the members (max and count: order-free), the new dish
    for (int v = lane; v < V; v += 64) {
      double mx = -MVC_PM_INF;
      int cnt = 0;
      for (int q = 0; q < (rest_only ? 1 : tw); ++q) {
        const double x = pmx[q * V + v];
        if (x > mx) mx = x;
        cnt += (int)pcnt[q * V + v];
      }
      const double Y2i = C.Y2[(size_t)v * C.y2stride];
      const double lfn = A.cnew[v] + (-0.5 * Y2i) / P.hyper[v];
      S.mv[v] = lfn > mx ? lfn : mx;
      kact[v] = cnt;
    }
  }
  __syncthreads();
  // pass 2: the weighted terms of the member's chunks
  if (act) {
    for (int c = r; 64 * c < NK; c += tw) {
      const int g = 64 * c + lane;
      if (g < NK) {
        int v, j;
        locate(g, v, j);
        const int l = W.d_l[v * ks + j] - ((j == W.dish[v * ts + p0] && !alive) ? 1 : 0);
        double t = 0.0;
        if (l > 0) {
          double wgt = (double)l - P.hyper[2 * V + v];
          if (wgt < 0.0) wgt = 0.0;
          t = wgt * mvc_exp(S.lp[v * lps + j] - S.mv[v]);
        }
        S.aux[v * lps + j] = t;
      }
    }
  }
  __syncthreads();
  // member 0: column partials in ascending j, pw16, the new dish, lm_v
  if (act && r == 0) {
    for (int vg = 0; vg < V; vg += 4) {
      const int v = vg + row;
      double cs = 0.0;
      if (v < V) {
        const int K = W.Klist[v];
        // this lane's column j = col, col + 16, ... in ascending j: batches of
        // 16 values, the next batch's loads in flight while one is summed
        const double *ax = S.aux + (size_t)v * lps + col;
        const int cnt = K > col ? (K - col + 15) >> 4 : 0;
        double xa[16], xb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xa[u] = u < cnt ? ax[16 * u] : 0.0;
        for (int e0 = 0; e0 < cnt; e0 += 16) {
#pragma unroll
          for (int u = 0; u < 16; ++u) xb[u] = e0 + 16 + u < cnt ? ax[16 * (e0 + 16 + u)] : 0.0;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (e0 + u < cnt) cs = cs + xa[u];
#pragma unroll
          for (int u = 0; u < 16; ++u) xa[u] = xb[u];
        }
      }
      double Sv = row_pw16(cs);
      if (v < V && col == 0) {
        const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
        const double Y2i = C.Y2[(size_t)v * C.y2stride];
        const double lfn = A.cnew[v] + (-0.5 * Y2i) / tau;
        const double m = S.mv[v];
        double wn = alpha + (double)kact[v] * sigma;
        if (wn < 0.0) wn = 0.0;
        Sv = Sv + wn * mvc_exp(lfn - m);
        const double denom = alpha + (double)(W.Ltot[v] - (alive ? 0 : 1));
        lmv[v] = (denom <= 0.0) ? lfn : (m + mvc_log(Sv)) - mvc_log(denom);
      }
    }
  }
  __syncthreads();
  RUN_MARK(0);
  // s_new in view order (every member); scores of the member's 64-table chunks
  double s_new = 0.0, M = -MVC_PM_INF;
  const int T = act ? *W.T : 0;
  const int TB = (T + 15) / 16;
  if (act) {
    s_new = mvc_log(ag + sg * (double)Tne_i);
    for (int v = 0; v < V; ++v) s_new = s_new + lmv[v];
    constexpr int kU = 8;   // 8 chunks per step: the loads are the latency
    const int nch = TB * 16;
    for (int c0 = r; c0 * 64 < nch; c0 += tw * kU) {
      int np[kU];
      double lm[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        np[u] = p < T ? W.n_t[p] - (p == p0 ? 1 : 0) : 0;
        lm[u] = p < T ? ((p == p0) ? lmass0 : W.lmass[p]) : 0.0;
      }
      double sp[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        const double mass = (double)np[u] - sg;
        sp[u] = (p < T && np[u] >= 1 && mass > 0.0) ? lm[u] : -MVC_PM_INF;
      }
      for (int v = 0; v < V; ++v) {
        int dj[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int p = (c0 + u * tw) * 64 + lane;
          dj[u] = (sp[u] != -MVC_PM_INF) ? W.dish[v * ts + p] : 0;
        }
        double lv[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) lv[u] = S.lp[v * lps + dj[u]];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (sp[u] != -MVC_PM_INF) sp[u] = sp[u] + lv[u];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        if (p < nch) S.e[p] = sp[u];
        if (sp[u] > M) M = sp[u];
      }
    }
    M = wave_max(M);
    if (lane == 0) mxr[r] = M;
  }
  __syncthreads();
  RUN_MARK(1);
  if (act) {
    for (int k = 0; k < tw; ++k) M = mxr[k] > M ? mxr[k] : M;
    if (s_new > M) M = s_new;
    for (int c0 = r; c0 * 64 < TB * 16; c0 += tw) {
      const int p = c0 * 64 + lane;
      double wgt = 0.0;
      if (p < TB * 16) {
        const double x = S.e[p];
        wgt = x != -MVC_PM_INF ? mvc_exp(x - M) : 0.0;
        S.e[p] = wgt;
      }
      const double Bv = row_pw16(wgt);
      const int b = c0 * 4 + row;
      if (col == 0 && b < TB) S.B[b] = Bv;
    }
  }
  __syncthreads();
  RUN_MARK(2);
  int pick = -1;
  if (act && r == 0) {
    // running block totals in block order; lane q keeps the total before
    // 64-block chunk q (TB <= 4096), so the draw walks one chunk only
    double tot = 0.0, cst = 0.0;
    const int nch = (TB + 63) >> 6;
    auto ldB = [&](int q) -> double { return (q < nch && 64 * q + lane < TB) ? S.B[64 * q + lane] : 0.0; };
    double B1 = ldB(0), B2 = ldB(1), B3 = ldB(2), B4 = ldB(3);   // four chunks in flight
    for (int q = 0; q < nch; ++q) {
      const double Bl = B1;
      B1 = B2;
      B2 = B3;
      B3 = B4;
      B4 = ldB(q + 4);
      if (lane == q) cst = tot;
      const int nb = min(64, TB - 64 * q);
      for (int k = 0; k < nb; ++k) tot = tot + readlane_d(Bl, k);
    }
    const double Wt = mvc_exp(s_new - M) + tot;
    double u = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * Wt;
    if (u < tot) {
      double c = 0.0, cprev = 0.0;
      int bsel = TB - 1;
      bool found = false;
      int bstart = 0;
      if (nch <= 64) {   // the first chunk whose end total exceeds u (totals are nondecreasing)
        const double nxt = __shfl_down(cst, 1, 64);
        const double cend = (lane + 1 < nch) ? nxt : tot;
        const uint64_t hit = __ballot(lane < nch && u < cend);
        const int q = hit ? (int)__ffsll((long long)hit) - 1 : 0;
        bstart = 64 * q;
        c = readlane_d(cst, q);
      }
      for (int b0 = bstart; b0 < TB && !found; b0 += 64) {
        const double Bl = (b0 + lane < TB) ? S.B[b0 + lane] : 0.0;
        const int nb = min(64, TB - b0);
        for (int k = 0; k < nb; ++k) {
          const double c2 = c + readlane_d(Bl, k);
          if (u < c2) {
            bsel = b0 + k;
            cprev = c;
            found = true;
            break;
          }
          c = c2;
        }
      }
      u = u - cprev;
      const double x = lane < 16 ? S.e[bsel * 16 + lane] : 0.0;
      pick = bsel * 16 + pw16_select_wave(x, u);
    }
  }
  RUN_MARK(3);
  return pick;
}

// tree64 over x[0..m) (oracle Tree64::build): level arrays stored one after
// the other from `lv` (level k starts at the sum of the lower levels' counts);
// returns the root.  nlev receives the number of levels (leaves included).
__device__ double seq_tree_build(double *lv, int m, int &nlev) {
  const int lane = threadIdx.x & 63;
  int o = 0, cnt = m;
  nlev = 1;
  double root = 0.0;
  do {
    const int nc = (cnt + 63) / 64;
    const int o2 = o + cnt;
    for (int c = 0; c < nc; ++c) {
      const int e = c * 64 + lane;
      const double x = e < cnt ? lv[o + e] : 0.0;
      const double s = wave_tree_sum(x);
      if (lane == 0) lv[o2 + c] = s;
      root = s;
    }
    __threadfence_block();
    o = o2;
    cnt = nc;
    ++nlev;
  } while (cnt > 1);
  return root;
}
// oracle Tree64::select
__device__ int seq_tree_select(const double *lv, int m, int nlev, double r) {
  const int lane = threadIdx.x & 63;
  int idx = 0;
  for (int k = nlev - 2; k >= 0; --k) {
    int cnt = m, off = 0;
    for (int q = 0; q < k; ++q) {
      off += cnt;
      cnt = (cnt + 63) / 64;
    }
    const int base = idx * 64;
    const int c = min(64, cnt - base);
    const double x = lane < c ? lv[off + base + lane] : 0.0;
    Tree64Levels L;
    wave_tree_sum_levels(x, L);
    const int l = wave_tree_select(L, x, r);
    idx = base + l;
  }
  return idx;
}

// Exact integer sum over each 16-lane row, every lane of the row gets it
// (xor butterfly by DPP: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror; after the first two steps the 4-groups are uniform, so the
// mirrors deliver the sibling 4- and 8-groups).
__device__ __forceinline__ int row16_isum_dpp(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, true);
  return x;
}
// lane k of each 16-lane row broadcast to the row (DPP row_newbcast:k)
template <int k>
__device__ __forceinline__ double row_bcast_d(double x) { return dpp_d<0x150 + k>(x); }

// Value prediction (vp, the lane-column kernel's second instance): the repair
// draws customer i with the same uniform as phase A, so its decision nearly
// always equals its phase-A choice (98 % at the literal and at configs[1]
// steady state).  A vp step evaluates customers i .. i+3 at once, customer
// i + w against the state with the PREDICTED decisions (phase-A choices) of
// i .. i+w-1 applied.  That state is the current one plus an overlay of what
// the predicted moves touch (their tables' counts and log masses, T_ne, L_v,
// and per view the left / joined dishes' counts, coefficients and S1 columns),
// built at the start of the step with the commit's own arithmetic.  The step
// then decides customers up to the first whose decision differs from its
// prediction: every one of them was evaluated against the state the
// sequential schedule has at its turn.
constexpr int kVpMoves = 4, kVpV = 8, kVpE = kVpMoves * kVpV * 2;
struct VpOv {
  int nm;                                      // predicted customers in the overlay (i .. i+nm-1)
  int mv[kVpMoves], p0[kVpMoves], c[kVpMoves]; // mv: customer i+m is a predicted move p0 -> c
  int dies[kVpMoves], born[kVpMoves];          // its table p0 dies, its table c is born (with the earlier moves applied)
  int pz[kVpMoves], pcs[kVpMoves];             // the step's customers' tables and predictions
  int ntp0[kVpMoves], ntc[kVpMoves], tne[kVpMoves];   // after move m
  int ltot[kVpMoves * kVpV];                   // L_v after move m
  int chg[kVpMoves * kVpV];                    // move m changes the dish of view v (S1 deltas)
  int j[kVpE], dn[kVpE], dl[kVpE];             // dish entry e = (m kVpV + v) 2 + (0 left | 1 joined), values after m
  int s1x[kVpE];                               // 1: the entry's S1 column differs from the state's (in the LDS area vpo)
  double lmp0[kVpMoves], lmc[kVpMoves];
  double Q[kVpE], c0[kVpE], cb[kVpE], xm[kVpE], ym[kVpE], cbm[kVpE];
};
__shared__ VpOv mvc_vp_ov;
// one wave's view of the overlay: the moves m < nw apply
struct VpCtx {
  int nw;                          // moves of the overlay this wave's customer sees
  int tne;                         // T_ne with them applied
  const double *s1;                // the overlay's S1 columns [kVpE][D] (LDS)
};
// the overlay entry of dish j of view v (the latest move m < nw touching it), or -1
template <bool kVp>
__device__ __forceinline__ int vp_de(const VpCtx &X, int v, int j) {
  int e = -1;
  if constexpr (kVp) {
#pragma unroll
    for (int m = 0; m < kVpMoves; ++m)
      if (m < X.nw) {
        const int e0 = (m * kVpV + v) * 2;
        if (mvc_vp_ov.j[e0] == j) e = e0;
        if (mvc_vp_ov.j[e0 + 1] == j) e = e0 + 1;
      }
  }
  return e;
}
// n_t and log mass of table p with the moves m < nw applied
template <bool kVp>
__device__ __forceinline__ void vp_table(const VpCtx &X, int p, int &nt, double &lm) {
  if constexpr (kVp) {
#pragma unroll
    for (int m = 0; m < kVpMoves; ++m)
      if (m < X.nw && mvc_vp_ov.mv[m]) {
        if (p == mvc_vp_ov.p0[m]) {
          nt = mvc_vp_ov.ntp0[m];
          lm = mvc_vp_ov.lmp0[m];
        }
        if (p == mvc_vp_ov.c[m]) {
          nt = mvc_vp_ov.ntc[m];
          lm = mvc_vp_ov.lmc[m];
        }
      }
  }
}
// L_v with the moves m < nw applied
template <bool kVp>
__device__ __forceinline__ int vp_ltot(const VpCtx &X, int v, int base) {
  int L = base;
  if constexpr (kVp) {
#pragma unroll
    for (int m = 0; m < kVpMoves; ++m)
      if (m < X.nw && mvc_vp_ov.mv[m]) L = mvc_vp_ov.ltot[m * kVpV + v];
  }
  return L;
}

// Where the lane-column evaluation keeps dish j of a view's lp row in the
// LDS scratch (seq_lps): one pad double per 32 dishes.
__device__ __forceinline__ int lc_lpx(int j) { return j + (j >> 5); }

// The own dish's value with the customer removed from its
// dot product G = y . S1[:, j0].
template <bool kVp = false>
__device__ __forceinline__ double lc_self(const SView &W, int vv, int ks, int j0, double G, double Y2i, double hy,
                                          double h, int eown = -1) {
  double Q = W.Q[vv * ks + j0], xm = W.xm[vv * ks + j0], ym = W.ym[vv * ks + j0], cbm = W.cbm[vv * ks + j0];
  if (kVp && eown >= 0) {
    Q = mvc_vp_ov.Q[eown];
    xm = mvc_vp_ov.xm[eown];
    ym = mvc_vp_ov.ym[eown];
    cbm = mvc_vp_ov.cbm[eown];
  }
  const double Gp = G - Y2i;
  const double Qp = (Q - 2.0 * G) + Y2i;
  const double c0 = xm - (0.5 * Qp) / ym;
  return __builtin_fma(Gp + hy, cbm, c0) + h;
}
// One view's terms for the lane-column evaluation, NU dishes per lane
// (j = col + 16 u, K <= 16 NU): the NU dot products run as interleaved fma
// chains, each in ascending d (the own dish's chain is the one its self-
// removed value starts from: the same operations as a separate chain), every
// LDS load of a step issued before its first use; the lp values and counts
// stay in registers for the column partial.  Lanes past K load a clamped
// column and contribute nothing (w = 0, exp(-inf) = 0: cs + 0 = cs).
template <int NU, bool kVp = false>
__device__ __forceinline__ void lc_view_terms(const SView &W, const double *yv, const double *S1v, int s1s, int D,
                                              int vv, int ks, int col, int K, int j0, int l0p, double hy, double h,
                                              double Y2i, double lfn, double sigma, const int *dl, double *lpv,
                                              double &mx, int &cnt, double &cs, const VpCtx &X) {
  int jc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) jc[u] = min(col + 16 * u, ks - 1);
  // vp: the dishes of this view the overlay's moves m < nw touch, loaded once
  // (vp_de's lookup against registers instead of LDS reads per dish; -2
  // matches no dish)
  int oj[2 * kVpMoves];
#pragma unroll
  for (int q = 0; q < 2 * kVpMoves; ++q) oj[q] = (kVp && q / 2 < X.nw) ? mvc_vp_ov.j[((q / 2) * kVpV + vv) * 2 + (q & 1)] : -2;
  auto de = [&](int j) {
    int e = -1;
#pragma unroll
    for (int q = 0; q < 2 * kVpMoves; ++q)
      if (oj[q] == j) e = ((q / 2) * kVpV + vv) * 2 + (q & 1);
    return e;
  };
  // vp: a dish whose S1 column an earlier predicted move changed is read from
  // the overlay's copy of that column (stride 1) instead of the state's
  const double *colp[NU];
  int cst[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    colp[u] = S1v + jc[u];
    cst[u] = s1s;
    if constexpr (kVp) {
      const int e = de(col + 16 * u);
      if (e >= 0 && mvc_vp_ov.s1x[e]) {
        colp[u] = X.s1 + (size_t)e * D;
        cst[u] = 1;
      }
    }
  }
  double G[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) G[u] = 0.0;
  // d in blocks of DB, every load of a block issued before its fmas
  constexpr int DB = NU <= 2 ? 16 : 4;
  int d = 0;
  for (; d + DB <= D; d += DB) {
    double yd[DB], sd[DB][NU];
#pragma unroll
    for (int k = 0; k < DB; ++k) {
      yd[k] = yv[d + k];
#pragma unroll
      for (int u = 0; u < NU; ++u) sd[k][u] = kVp ? colp[u][(d + k) * cst[u]] : S1v[(d + k) * s1s + jc[u]];
    }
#pragma unroll
    for (int k = 0; k < DB; ++k)
#pragma unroll
      for (int u = 0; u < NU; ++u) G[u] = __builtin_fma(yd[k], sd[k][u], G[u]);
  }
  for (; d < D; ++d) {
    const double yd = yv[d];
#pragma unroll
    for (int u = 0; u < NU; ++u) G[u] = __builtin_fma(yd, kVp ? colp[u][d * cst[u]] : S1v[d * s1s + jc[u]], G[u]);
  }
  double Gown = 0.0;
#pragma unroll
  for (int u = 0; u < NU; ++u)
    if (col + 16 * u == j0) Gown = G[u];
  const double self = lc_self<kVp>(W, vv, ks, j0, Gown, Y2i, hy, h, kVp ? de(j0) : -1);
  double lp[NU];
  int lj[NU];
  mx = -MVC_PM_INF;
  cnt = 0;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int j = col + 16 * u;
    const bool valid = j < K, own = j == j0;
    double cbj = W.cb[vv * ks + jc[u]], c0j = W.c0[vv * ks + jc[u]];
    int dlj = dl[jc[u]];
    if constexpr (kVp) {
      const int e = de(j);
      if (e >= 0) {
        cbj = mvc_vp_ov.cb[e];
        c0j = mvc_vp_ov.c0[e];
        dlj = mvc_vp_ov.dl[e];
      }
    }
    const double fr = __builtin_fma(G[u] + hy, cbj, c0j) + h;
    lp[u] = own ? self : fr;
    lj[u] = valid ? (own ? l0p : dlj) : 0;
    if (valid) lpv[lc_lpx(j)] = lp[u];
    if (lj[u] > 0) {
      ++cnt;
      if (lp[u] > mx) mx = lp[u];
    }
  }
  mx = row16_max(mx);
  cnt = row16_isum_dpp(cnt);
  const double m = lfn > mx ? lfn : mx;
  cs = 0.0;
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    double w = (double)lj[u] - sigma;
    if (w < 0.0) w = 0.0;
    cs = cs + w * mvc_exp_le0(lj[u] > 0 ? lp[u] - m : -MVC_PM_INF);
  }
}
// 8-lane rows (every K_v <= 8, V <= 8): one view per 8 lanes, so every view
// of a customer in one pass instead of a pass per 4 views.  The values are
// the 16-lane evaluation's: lanes 8..15 of a 16-lane row hold no dish there,
// so their column partials are +0 and their maxima -inf and counts 0; the
// row's pw16 is then the pw8 of columns 0..7 plus +0 (a non-negative sum:
// the same value), its maximum and count those of the 8 lanes.
__device__ __forceinline__ double row8_max_all(double x) {   // xor butterfly: every lane of the 8-group
  x = dmax(x, dpp_d<0xB1>(x));    // quad_perm [1,0,3,2]
  x = dmax(x, dpp_d<0x4E>(x));    // quad_perm [2,3,0,1]
  x = dmax(x, dpp_d<0x141>(x));   // row_half_mirror: the sibling quad
  return x;
}
__device__ __forceinline__ int row8_isum_dpp(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, true);
  return x;
}
// pw8 of the 8-group's column partials (pairs (c, c + h), h = 1, 2, 4), valid
// in the group's first lane
__device__ __forceinline__ double row8_pw_head(double x) {
  x = x + down_d<1>(x);
  x = x + down_d<2>(x);
  x = x + down_d<4>(x);
  return x;
}
// lc_view_terms<1> on an 8-lane row (col = lane & 7, dish j = col)
__device__ __forceinline__ void lc_view_terms8(const SView &W, const double *yv, const double *S1v, int s1s, int D, int vv,
                                               int ks, int col, int K, int j0, int l0p, double hy, double h, double Y2i,
                                               double lfn, double sigma, const int *dl, double *lpv, double &mx, int &cnt,
                                               double &cs) {
  const int jc = min(col, ks - 1);
  double G = 0.0;
  constexpr int DB = 16;
  int d = 0;
  for (; d + DB <= D; d += DB) {
    double yd[DB], sd[DB];
#pragma unroll
    for (int k = 0; k < DB; ++k) {
      yd[k] = yv[d + k];
      sd[k] = S1v[(d + k) * s1s + jc];
    }
#pragma unroll
    for (int k = 0; k < DB; ++k) G = __builtin_fma(yd[k], sd[k], G);
  }
  for (; d < D; ++d) G = __builtin_fma(yv[d], S1v[d * s1s + jc], G);
  const bool valid = col < K, own = col == j0;
  const double self = lc_self<false>(W, vv, ks, j0, own ? G : 0.0, Y2i, hy, h, -1);
  const double fr = __builtin_fma(G + hy, W.cb[vv * ks + jc], W.c0[vv * ks + jc]) + h;
  const double lp = own ? self : fr;
  const int lj = valid ? (own ? l0p : dl[jc]) : 0;
  if (valid) lpv[lc_lpx(col)] = lp;
  mx = row8_max_all((lj > 0 && lp > -MVC_PM_INF) ? lp : -MVC_PM_INF);   // (lc_view_terms: if (lp > mx) mx = lp)
  cnt = row8_isum_dpp(lj > 0 ? 1 : 0);
  const double m = lfn > mx ? lfn : mx;
  double w = (double)lj - sigma;
  if (w < 0.0) w = 0.0;
  cs = 0.0 + w * mvc_exp_le0(lj > 0 ? lp - m : -MVC_PM_INF);
}

// The same for any K (more than 8 dishes per lane): one dish at a time.
__device__ __forceinline__ void lc_view_terms_loop(const SView &W, const double *yv, const double *S1v, int s1s, int D,
                                                int vv, int ks, int col, int K, int j0, int l0p, double hy, double h,
                                                double Y2i, double lfn, double sigma, const int *dl, double *lpv,
                                                double &mx, int &cnt, double &cs) {
  double Gs = 0.0;
  for (int d = 0; d < D; ++d) Gs = __builtin_fma(yv[d], S1v[d * s1s + j0], Gs);
  const double self = lc_self(W, vv, ks, j0, Gs, Y2i, hy, h);
  mx = -MVC_PM_INF;
  cnt = 0;
  for (int j = col; j < K; j += 16) {
    double G = 0.0;
    for (int d = 0; d < D; ++d) G = __builtin_fma(yv[d], S1v[d * s1s + j], G);
    const double fr = __builtin_fma(G + hy, W.cb[vv * ks + j], W.c0[vv * ks + j]) + h;
    const bool own = j == j0;
    const double val = own ? self : fr;
    const int l = own ? l0p : dl[j];
    lpv[lc_lpx(j)] = val;
    if (l > 0) {
      ++cnt;
      if (val > mx) mx = val;
    }
  }
  mx = row16_max(mx);
  cnt = row16_isum_dpp(cnt);
  const double m = lfn > mx ? lfn : mx;
  cs = 0.0;
  for (int j = col; j < K; j += 16) {
    const int l = (j == j0) ? l0p : dl[j];
    double w = (double)l - sigma;
    if (w < 0.0) w = 0.0;
    cs = cs + w * mvc_exp_le0(l > 0 ? lpv[lc_lpx(j)] - m : -MVC_PM_INF);
  }
}

// The table part of the lane-column evaluation: scores log(n_p' - sigma_g) +
// sum_v lp_{v, dish_v(p)} (view order; -inf when excluded) of QB 64-table
// chunks per step, every view's dish index loaded before the gathers (4 views
// at a time); their max M (with s_new); weights exp(score - M) to the wave's
// scratch e[]; block sums pw16 per row and running block totals C_b kept in
// lane b.  kOne: one step covers every table (nch <= QB), so the scores stay
// in registers between the two passes.  Same operations and order for every QB.
template <int QB, bool kOne, bool kVp = false, int VC = 4>   // VC: views whose dish indices are loaded per round
__device__ __forceinline__ void lc_scores_weights(const SView &W, const SeqScratch &S, int V, int ts, int lps, int p0,
                                                  int T, double sg, double lmass0, double s_new, double &M,
                                                  double &tot, double &Cb, const VpCtx &X) {
  const int lane = threadIdx.x & 63;
  const int TB = (T + 15) >> 4, nch = (T + 63) >> 6;
  double xk[QB];
  M = -MVC_PM_INF;
  for (int q0 = 0; q0 < nch; q0 += QB) {
    double x[QB];
    bool inc[QB];
    int pp[QB];
#pragma unroll
    for (int h2 = 0; h2 < QB; ++h2) {
      const int p = 64 * (q0 + h2) + lane;
      pp[h2] = p;
      int ntp = p < T ? W.n_t[p] : 0;
      double lmp = p < T ? W.lmass[p] : 0.0;
      vp_table<kVp>(X, p, ntp, lmp);
      const int np = p < T ? ntp - (p == p0 ? 1 : 0) : 0;
      const double mass = (double)np - sg;
      inc[h2] = p < T && np >= 1 && mass > 0.0;
      x[h2] = inc[h2] ? (p == p0 ? lmass0 : lmp) : -MVC_PM_INF;
    }
    for (int v0 = 0; v0 < V; v0 += VC) {
      int dj[QB][VC];
#pragma unroll
      for (int h2 = 0; h2 < QB; ++h2)
#pragma unroll
        for (int u = 0; u < VC; ++u)
          dj[h2][u] = (inc[h2] && v0 + u < V) ? W.dish[(v0 + u) * ts + pp[h2]] : 0;
      double lv[QB][VC];
#pragma unroll
      for (int h2 = 0; h2 < QB; ++h2)
#pragma unroll
        for (int u = 0; u < VC; ++u) lv[h2][u] = S.lp[min(v0 + u, V - 1) * lps + lc_lpx(dj[h2][u])];
#pragma unroll
      for (int h2 = 0; h2 < QB; ++h2)
#pragma unroll
        for (int u = 0; u < VC; ++u)
          if (inc[h2] && v0 + u < V) x[h2] = x[h2] + lv[h2][u];   // view order
    }
#pragma unroll
    for (int h2 = 0; h2 < QB; ++h2) {
      if (q0 + h2 < nch) {
        if (kOne)
          xk[h2] = x[h2];
        else
          S.e[pp[h2]] = x[h2];
        if (x[h2] > M) M = x[h2];
      }
    }
  }
  M = wave_max(M);
  if (s_new > M) M = s_new;
  tot = 0.0;
  Cb = 0.0;
  for (int q0 = 0; q0 < nch; q0 += QB) {
    double e[QB];
#pragma unroll
    for (int h2 = 0; h2 < QB; ++h2) e[h2] = kOne ? xk[h2] : S.e[64 * min(q0 + h2, nch - 1) + lane];
#pragma unroll
    for (int h2 = 0; h2 < QB; ++h2) e[h2] = mvc_exp_le0(e[h2] - M);
#pragma unroll
    for (int h2 = 0; h2 < QB; ++h2) {
      const int q = q0 + h2;
      if (q < nch) {
        S.e[64 * q + lane] = e[h2];
        const double B = row_pw16(e[h2]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = 4 * q + r;
          if (b < TB) {
            tot = tot + readlane_d(B, 16 * r);
            if (lane == b) Cb = tot;
          }
        }
      }
    }
  }
}

// seq_resample shaped for latency on the run kernel's LDS state ("lane
// columns"): the same decision, bit for bit, with every reduction either
// in-lane or a 16-lane row tree.  Lane (row r, column c) owns view v = g + r
// of view group g (views g .. g + 3) and that view's dishes j = c, c + 16,
// c + 32, ... in ascending order, so the spec's column partial col_c (the
// sequential sum over j = c mod 16) is this lane's running
// sum and pw16 over the columns is the row's DPP tree; the view maximum and
// K_act are row reductions.  The per-view logs (log S_v, log of the
// denominator) of four views, the new-table log and the own table's log mass
// share one log evaluation (one lane each).  Tables: lane p of 64-table
// chunks (T <= 64 kLcChunks), the lp rows gathered from the wave's LDS
// scratch, block sums by row pw16, running block totals in lane b (b < 64)
// so the draw finds its block with one ballot.  hyp / cnewv: the sweep's
// hyperparameters and new-dish constants, staged in LDS at kernel launch.
constexpr int kLcChunks = 8;   // tables <= 512 (block totals in lanes b < 64 need TB <= 64)
template <bool kVp = false>
__device__ __forceinline__ int seq_resample_lc(const SeqArgs &A, const SView &W, const Cust &C, int i, int p0, const SeqScratch &S,
                               const double *hyp, const double *cnewv, const VpCtx &X = VpCtx{}) {
  const int lane = threadIdx.x & 63, row = lane >> 4, col = lane & 15;
  const int V = A.P.V, D = A.P.D, ts = W.ts, ks = W.ks, lps = S.lps, s1s = W.s1s;
  const double ag = hyp[3 * V], sg = hyp[3 * V + 1];
  int nt0 = W.n_t[p0];
  double lm_unused = 0.0;
  vp_table<kVp>(X, p0, nt0, lm_unused);
  const int np0 = nt0 - 1;
  const bool alive = np0 > 0;
  const int Tne_i = (kVp ? X.tne : *W.T_ne) - (alive ? 0 : 1);
  const double mass0 = (double)np0 - sg;
  double s_new = 0.0, lmass0 = 0.0;
  const double u_i = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z);   // independent of the rest
  RUN_T0();
  int kmx = 0;
  for (int v = 0; v < V; ++v) kmx = max(kmx, W.Klist[v]);
  if (!kVp && V <= 8 && kmx <= 8) {   // every view in one pass on 8-lane rows (the same values)
    const int r8 = lane >> 3, c8 = lane & 7;
    const int v = r8;
    const bool vok = v < V;
    const int vv = vok ? v : V - 1;
    const int K = vok ? W.Klist[vv] : 0;
    const double tau = hyp[vv], alpha = hyp[V + vv], sigma = hyp[2 * V + vv];
    const double Y2i = C.Y2[vv * (int)C.y2stride];
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau;
    const double lfn = cnewv[vv] + h;
    const int j0 = W.dish[vv * ts + p0];
    const int *dl = W.d_l + vv * ks;
    const int l0p = dl[j0] - (alive ? 0 : 1);
    double mx, cs;
    int cnt;
    lc_view_terms8(W, C.y + vv * (int)C.ystride, W.S1T + vv * D * s1s, s1s, D, vv, ks, c8, K, j0, l0p, hy, h, Y2i, lfn,
                   sigma, dl, S.lp + vv * lps, mx, cnt, cs);
    const double m = lfn > mx ? lfn : mx;
    double Sv = row8_pw_head(cs);
    double wn = alpha + (double)cnt * sigma;
    if (wn < 0.0) wn = 0.0;
    Sv = Sv + wn * mvc_exp_le0(lfn - m);
    const double denom = alpha + (double)(W.Ltot[vv] - (alive ? 0 : 1));
    double arg = c8 == 0 ? Sv : (c8 == 1 ? denom : 1.0);
    if (r8 == 0 && c8 == 2) arg = ag + sg * (double)Tne_i;
    if (r8 == 0 && c8 == 3) arg = mass0;
    const double Lg = mvc_log(arg);
    const double logden = down_d<1>(Lg);   // column 1's log, in column 0
    const double lm = (denom <= 0.0) ? lfn : (m + Lg) - logden;   // valid in column 0
    s_new = readlane_d(Lg, 2);
    lmass0 = readlane_d(Lg, 3);
    for (int r = 0; r < V; ++r) s_new = s_new + readlane_d(lm, 8 * r);   // view order
  } else
  for (int g = 0; g < V; g += 4) {
    const int v = g + row;
    const bool vok = v < V;
    const int vv = vok ? v : V - 1;   // rows past the last view mirror it (their results are not used)
    const int K = vok ? W.Klist[vv] : 0;
    const double tau = hyp[vv], alpha = hyp[V + vv], sigma = hyp[2 * V + vv];
    const double Y2i = C.Y2[vv * (int)C.y2stride];
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau;
    const double lfn = cnewv[vv] + h;
    const int j0 = W.dish[vv * ts + p0];
    const double *yv = C.y + vv * (int)C.ystride;
    const double *S1v = W.S1T + vv * D * s1s;
    const int *dl = W.d_l + vv * ks;
    double *lpv = S.lp + vv * lps;
    int dl0 = dl[j0];
    if constexpr (kVp) {
      const int e = vp_de<kVp>(X, vv, j0);
      if (e >= 0) dl0 = mvc_vp_ov.dl[e];
    }
    const int l0p = dl0 - (alive ? 0 : 1);
    // lp of this lane's dishes (to the scratch for the table gathers), their
    // max over the included ones (l' > 0), K_act, and the column partial
    // w_j exp(lp_j - m) in ascending j (excluded dishes add +0)
    double mx, cs;
    int cnt;
    const int nu = (max(max(readlane_i(K, 0), readlane_i(K, 16)), max(readlane_i(K, 32), readlane_i(K, 48))) + 15) >> 4;
    if (nu <= 1)
      lc_view_terms<1, kVp>(W, yv, S1v, s1s, D, vv, ks, col, K, j0, l0p, hy, h, Y2i, lfn, sigma, dl, lpv, mx, cnt, cs, X);
    else if (nu <= 2)
      lc_view_terms<2, kVp>(W, yv, S1v, s1s, D, vv, ks, col, K, j0, l0p, hy, h, Y2i, lfn, sigma, dl, lpv, mx, cnt, cs, X);
    else if (nu <= 4)
      lc_view_terms<4, kVp>(W, yv, S1v, s1s, D, vv, ks, col, K, j0, l0p, hy, h, Y2i, lfn, sigma, dl, lpv, mx, cnt, cs, X);
    else if (kVp || nu <= 8)   // (the vp kernel runs only while every K_v <= 128)
      lc_view_terms<8, kVp>(W, yv, S1v, s1s, D, vv, ks, col, K, j0, l0p, hy, h, Y2i, lfn, sigma, dl, lpv, mx, cnt, cs, X);
    else
      lc_view_terms_loop(W, yv, S1v, s1s, D, vv, ks, col, K, j0, l0p, hy, h, Y2i, lfn, sigma, dl, lpv, mx, cnt, cs);
    const double m = lfn > mx ? lfn : mx;
    double Sv = row_pw16(cs);
    double wn = alpha + (double)cnt * sigma;
    if (wn < 0.0) wn = 0.0;
    Sv = Sv + wn * mvc_exp_le0(lfn - m);
    const double denom = alpha + (double)(vp_ltot<kVp>(X, vv, W.Ltot[vv]) - (alive ? 0 : 1));
    // one log for the group: column 0 log S_v, column 1 log(denominator);
    // group 0, row 0 also the new-table mass (column 2) and the own table's
    // mass without the customer (column 3)
    double arg = col == 0 ? Sv : (col == 1 ? denom : 1.0);
    if (g == 0 && row == 0 && col == 2) arg = ag + sg * (double)Tne_i;
    if (g == 0 && row == 0 && col == 3) arg = mass0;
    const double Lg = mvc_log(arg);
    const double logS = row_bcast_d<0>(Lg), logden = row_bcast_d<1>(Lg);
    const double lm = (denom <= 0.0) ? lfn : (m + logS) - logden;
    if (g == 0) {
      s_new = readlane_d(Lg, 2);
      lmass0 = readlane_d(Lg, 3);
    }
    for (int r = 0; r < 4 && g + r < V; ++r) s_new = s_new + readlane_d(lm, 16 * r);   // view order
  }
  RUN_MARK(0);
  // table scores log(n_p' - sigma_g) + sum_v lp_{v, dish_v(p)} (view order),
  // -inf when excluded; to the wave's scratch e[]
  const int T = *W.T, TB = (T + 15) >> 4, nch = (T + 63) >> 6;
  double M, tot, Cb;
  if (nch <= 1)   // T <= 64: one chunk, every view's dish indices in one round when V <= 8
    lc_scores_weights<1, true, kVp, 8>(W, S, V, ts, lps, p0, T, sg, lmass0, s_new, M, tot, Cb, X);
  else if (nch <= 2)
    lc_scores_weights<2, true, kVp>(W, S, V, ts, lps, p0, T, sg, lmass0, s_new, M, tot, Cb, X);
  else if (nch <= 4)
    lc_scores_weights<4, true, kVp>(W, S, V, ts, lps, p0, T, sg, lmass0, s_new, M, tot, Cb, X);
  else
    lc_scores_weights<4, false, kVp>(W, S, V, ts, lps, p0, T, sg, lmass0, s_new, M, tot, Cb, X);
  RUN_MARK(1);
  const double Wt = mvc_exp_le0(s_new - M) + tot;
  double r = u_i * Wt;
  if (!(r < tot)) {
    RUN_MARK(2);
    return -1;
  }
  const uint64_t hit = __ballot(lane < TB && r < Cb);
  const int bsel = (int)__ffsll((long long)hit) - 1;
  r = r - (bsel > 0 ? readlane_d(Cb, bsel - 1) : 0.0);
  const double x = S.e[16 * (bsel & ~3) + lane];   // the block's row of its 64-table chunk
  const int pick = 16 * bsel + pw16_select_wave(x, r, 16 * (bsel & 3));
  RUN_MARK(2);
  return pick;
}

// Dish of a birth in view v (oracle SeqSampler::draw_dish): leaves w_j
// exp(lp_j - m) of the included dishes, the new dish last; tree64; r = u S.
// lp: [K] scratch, tree: the tree64 levels' scratch.  Returns a list index;
// Klist[v] = a new dish.
// lpre (optional): the customer's lp row of view v against the current
// state with its max (incl. the new dish) mpre and count kpre, as the wide
// evaluation left them (seq_resample_wide: the same values seq_view_lp gives).
__device__ int seq_dish_draw(const SeqArgs &A, const SView &W, const Cust &C, int i, int v, bool alive, int j0,
                             double *lpw, double *tree, const double *lpre = nullptr, double mpre = 0.0,
                             int kpre = 0) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, ks = W.ks;
  const int K = W.Klist[v];
  const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
  const double Y2i = C.Y2[(size_t)v * C.y2stride];
  const double lfn = A.cnew[v] + (-0.5 * Y2i) / tau;
  double m;
  int Kact;
  const double *lp;
  if (lpre) {
    lp = lpre;
    m = mpre;
    Kact = kpre;
  } else {
    Kact = seq_view_lp(A, W, C, v, alive, j0, lpw, &m);
    __threadfence_block();
    lp = lpw;
  }
  if (lfn > m) m = lfn;
  double wn = alpha + (double)Kact * sigma;
  if (wn < 0.0) wn = 0.0;
  const int l0p = alive ? W.d_l[v * ks + j0] : W.d_l[v * ks + j0] - 1;
  for (int e = lane; e <= K; e += 64) {
    double leaf = 0.0;
    if (e < K) {
      const int l = (e == j0) ? l0p : W.d_l[v * ks + e];
      if (l > 0) {
        double w = (double)l - sigma;
        if (w < 0.0) w = 0.0;
        leaf = w * mvc_exp(lp[e] - m);
      }
    } else {
      leaf = wn * mvc_exp(lfn - m);
    }
    tree[e] = leaf;
  }
  __threadfence_block();
  int nlev;
  const double tot = seq_tree_build(tree, K + 1, nlev);
  if (!(tot > 0.0)) return K;
  const double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_DISH + 1u + (uint32_t)v) * tot;
  return seq_tree_select(tree, K + 1, nlev, r);
}

// seq_tree_build / seq_tree_select with the leaf level read through leaf(e)
// (e < m) instead of stored: the levels above it go to `up` one after the
// other.  The same sums in the same association, so the same root and pick.
template <class F>
__device__ double seq_tree_build_f(F leaf, int m, double *up, int &nlev) {
  const int lane = threadIdx.x & 63;
  int cnt = (m + 63) / 64;
  double root = 0.0;
  for (int c = 0; c < cnt; ++c) {
    const int e = c * 64 + lane;
    const double s = wave_tree_sum(e < m ? leaf(e) : 0.0);
    if (lane == 0) up[c] = s;
    root = s;
  }
  __threadfence_block();
  nlev = 2;
  int o = 0;
  while (cnt > 1) {
    const int nc = (cnt + 63) / 64;
    const int o2 = o + cnt;
    for (int c = 0; c < nc; ++c) {
      const int e = c * 64 + lane;
      const double s = wave_tree_sum(e < cnt ? up[o + e] : 0.0);
      if (lane == 0) up[o2 + c] = s;
      root = s;
    }
    __threadfence_block();
    o = o2;
    cnt = nc;
    ++nlev;
  }
  return root;
}
template <class F>
__device__ int seq_tree_select_f(F leaf, const double *up, int m, int nlev, double r) {
  const int lane = threadIdx.x & 63;
  int idx = 0;
  for (int k = nlev - 2; k >= 0; --k) {
    int cnt = m, off = 0;
    for (int q = 0; q < k; ++q) {
      off += cnt;
      cnt = (cnt + 63) / 64;
    }
    const int base = idx * 64;
    const int c = min(64, cnt - base);
    const double x = lane < c ? (k == 0 ? leaf(base + lane) : up[off - m + base + lane]) : 0.0;
    Tree64Levels L;
    wave_tree_sum_levels(x, L);
    const int l = wave_tree_select(L, x, r);
    idx = base + l;
  }
  return idx;
}

// The fin kernel's evaluation left in LDS (wide_fin_resample): every view's
// weighted dish terms w_j exp(lp_j - m_v) -- exactly seq_dish_draw's leaves
// for the same customer and state -- and the new dish's leaf; `up` holds V
// tree scratches of upstride doubles.  L == nullptr: none.
struct FinLeaves {
  const double *L;
  const int *koff;
  const double *newleaf;
  double *up;
  int upstride;
};
// seq_dish_draw from those leaves (no lp row, no exps): the same tree64, the same draw.
__device__ int seq_dish_draw_leaves(const SeqArgs &A, const SView &W, int i, int v, const FinLeaves &fl) {
  const int K = W.Klist[v];
  const double *lv = fl.L + fl.koff[v];
  const double nl = fl.newleaf[v];
  auto leaf = [&](int e) { return e < K ? lv[e] : nl; };
  double *up = fl.up + (size_t)v * fl.upstride;
  int nlev;
  const double tot = seq_tree_build_f(leaf, K + 1, up, nlev);
  if (!(tot > 0.0)) return K;
  const double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_DISH + 1u + (uint32_t)v) * tot;
  return seq_tree_select_f(leaf, up, K + 1, nlev, r);
}

}  // namespace

// Before phase A: the whole sweep is one pending window [0, n).
// run_start: the sweep starts in the run kernel at customer 0 (the small
// chains' lane-per-customer loop, whose first step is phase A) instead of a
// window over the whole sweep.
__device__ __forceinline__ void seq_init_body(const SeqArgs &A, int run_start) {
  if (threadIdx.x != 0) return;
  Repair *R = A.R;
  const int V = A.P.V, n = A.P.n;
  R->cur = 0;
  R->pend = 0;
  R->win0 = 0;
  R->win1 = run_start ? 0 : n;
  R->fmin = n;
  R->W = A.Wmin;
  R->lastm = 0;
  R->gapq = 0;
  R->vpoff = 0;
  R->vpsteps = 0;
  R->vphits = 0;
  R->done = 0;
  R->overflow = 0;
  R->mode = run_start ? kSeqRun : kSeqScan;
  R->pchoice = 0;
  R->streak = 0;
  R->restride = 0;
  R->T = A.status[0];
  R->T_ne = A.status[V + 3];
  R->moves = R->births = R->newdish = R->rounds = 0;
  for (int k = 0; k < 22; ++k) R->prof[k] = 0;
  for (int k = 0; k < 8; ++k) R->dbg[k] = 0;
  for (int v = 0; v < V; ++v) R->Klist[v] = A.P.Kact[v];
}
extern "C" __global__ void mvc_seq_init_kernel(SeqArgs A, int run_start) { seq_init_body(A, run_start); }
// The same for several chains (one block per chain): the chain-batched sweep
extern "C" __global__ void mvc_seq_init_kernel_b(const SeqArgs *As, int run_start) {
  seq_init_body(As[blockIdx.x], run_start);
}

// After phase A: the first customer whose choice is not its own table.
extern "C" __global__ __launch_bounds__(256) void mvc_seq_first_kernel(int n, const int32_t *choice, const int32_t *z,
                                                                      Repair *R) {
  int best = n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (choice[i] != z[i]) { best = i; break; }
  // the first hit of each thread is its minimum (ascending grid stride)
  const uint64_t m = __ballot(best < n);
  if (m) {
    int b = best;
    for (int o = 32; o >= 1; o >>= 1) b = min(b, __shfl_xor(b, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMin(&R->fmin, b);
  }
}

namespace {

// The run kernel's LDS copies of the mutable state (layout: SeqLds); every
// write of the commit goes to the global arrays and, when present, here.
struct SCache {
  int32_t *n_t, *dish, *d_l, *d_n, *Klist, *Ltot, *T, *T_ne;
  double *c0, *cb, *Q, *xm, *ym, *cbm, *lmass;
  double *S2;                  // [V][ks]: the commit's S2 read-modify-writes stay in LDS (stores to HBM only)
  double *S1T;   // nullptr: S1 is read from global memory
  const double *hyp, *L2pt;    // the sweep's hyperparameters [3V+2] and log(2 pi tau) [V], staged at launch
  const double *cnew;          // [V] D (-1/2 log(2 pi tau)), staged at launch
  int ts, ks;
};
__device__ __forceinline__ SView cache_view(const SCache &c, const SeqArgs &A) {
  SView W;
  W.n_t = c.n_t; W.dish = c.dish; W.d_l = c.d_l; W.d_n = c.d_n;
  W.c0 = c.c0; W.cb = c.cb; W.Q = c.Q;
  W.xm = c.xm; W.ym = c.ym; W.cbm = c.cbm; W.lmass = c.lmass;
  W.S1T = c.S1T ? c.S1T : A.P.S1T;
  W.s1s = c.S1T ? c.ks : A.P.KC;
  W.Klist = c.Klist; W.Ltot = c.Ltot; W.T = c.T; W.T_ne = c.T_ne;
  W.ts = c.ts; W.ks = c.ks;
  return W;
}

// The run kernel's dynamic LDS (the state cache, per-wave scratch, ring) and
// its per-sweep constants (hyper [3V+2] | cnew [V] | L2pt [V]).  Every
// pointer into them is derived here from the symbols themselves, never
// loaded from memory, so the compiler keeps LDS accesses as ds_* (a pointer
// that went through a struct in memory would be a flat access, which also
// waits on every outstanding global store).
extern __shared__ double mvc_seq_lds[];
__shared__ double mvc_seq_const[5 * MVC_MAXV + 2];
__device__ __forceinline__ SCache lds_cache(int V, int D, int ts, int ks, int s1) {
  SCache cc{};
  int32_t *ip = (int32_t *)mvc_seq_lds;
  cc.ts = ts;
  cc.ks = ks;
  cc.n_t = ip; ip += ts;
  cc.dish = ip; ip += V * ts;
  cc.d_l = ip; ip += V * ks;
  cc.d_n = ip; ip += V * ks;
  cc.Klist = ip; ip += V;
  cc.Ltot = ip; ip += V;
  cc.T = ip++;
  cc.T_ne = ip++;
  double *dp = mvc_seq_lds + (ip - (int32_t *)mvc_seq_lds + 1) / 2;
  cc.c0 = dp; dp += V * ks;
  cc.cb = dp; dp += V * ks;
  cc.Q = dp; dp += V * ks;
  cc.xm = dp; dp += V * ks;
  cc.ym = dp; dp += V * ks;
  cc.cbm = dp; dp += V * ks;
  cc.lmass = dp; dp += ts;
  cc.S2 = dp; dp += V * ks;
  cc.S1T = s1 ? dp : nullptr;
  cc.hyp = mvc_seq_const;
  cc.cnew = mvc_seq_const + 3 * MVC_MAXV + 2;
  cc.L2pt = mvc_seq_const + 4 * MVC_MAXV + 2;
  return cc;
}

// The parts of coef(n - 1, Qp) that do not depend on the customer (the own
// dish's self-removed coefficient, §4.2): c0 = xm - (0.5 Qp) / ym, cb = cbm.
__device__ __forceinline__ void self_coef_parts(int n_, double tau, double L2pt, int D, double &xm, double &ym,
                                                double &cbm) {
  const double a = tau + (double)(n_ - 1);
  const double b = tau + (double)n_;
  xm = (double)D * ((-0.5 * L2pt) - 0.5 * mvc_log(b / a));
  ym = (tau * a) * b;
  cbm = 1.0 / (tau * b);
}

// Block barrier.  lds_only: the waves hand each other only LDS data (the run
// kernel with its whole state cached in LDS, S1 included): wait for this
// wave's LDS operations, not for its global stores -- __syncthreads' release
// fence waits for every outstanding store (vmcnt), i.e. an L2 round trip per
// barrier after the commits' write-through stores.
__device__ __forceinline__ void seq_bar(bool lds_only) {
  if (lds_only) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else __syncthreads();
}

// Commit customer i's exact choice c (a table position, or -1 = birth) to the
// state (oracle SeqSampler::sweep_once body + move); p0 = z[i].  The state is
// read through W (global or the LDS cache cc) and written to the global
// arrays and cc.  Block-cooperative: every thread of the block calls it.  A
// birth draws its dishes against the current state first (wave w < nwd:
// views w, w + nwd, ...; lp scratch lpw, tree64 scratch treew); if the new table or a
// new dish does not fit the capacity the state is left unchanged,
// R->overflow is set and false is returned (the host grows the capacity and
// the commit is redone, bit for bit: its draws are counter-addressed).
// cnt: the moves / births / new-dish counters (R->moves... or the run
// kernel's LDS copies).
__device__ bool seq_commit(SeqArgs &A, const SView &W, const SCache *cc, const Cust &Ci, int i, int p0, int c,
                           double *lpw, double *treew, int32_t *cnt, int nwd, const SeqScratch *pre = nullptr,
                           bool lds_only = false, FinLeaves fl = FinLeaves{}) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC;
  const int ks = W.ks, ts = W.ts;
  __shared__ int s_ovf, s_c, s_dies, s_born;
  __shared__ int s_tup[MVC_MAXV], s_j0[MVC_MAXV], s_j1[MVC_MAXV];
  // constants from LDS when the run kernel staged them (a global load here
  // would wait for every store the commits have issued: vmcnt is in order)
  const double *hyp = (cc && cc->hyp) ? cc->hyp : P.hyper;
  const double *l2pt = (cc && cc->L2pt) ? cc->L2pt : A.L2pt;
  if (c < 0) {
    // a birth: dishes drawn against the current state, then the table
    const bool alive = (W.n_t[p0] - 1) > 0;
    for (int v = w; v < V && w < nwd; v += nwd) {   // waves w < nwd own a scratch (lpw, treew)
      const int t = fl.L  ? seq_dish_draw_leaves(A, W, i, v, fl)
                    : pre ? seq_dish_draw(A, W, Ci, i, v, alive, W.dish[v * ts + p0], lpw, treew,
                                          pre->lp + (size_t)v * pre->lps, pre->mv[v], pre->koff[V + 1 + v])
                          : seq_dish_draw(A, W, Ci, i, v, alive, W.dish[v * ts + p0], lpw, treew);
      if (lane == 0) s_tup[v] = t;
    }
    __syncthreads();
    if (tid == 0) {
      const int T = *W.T;
      int ovf = (T + 1 > TC) ? 1 : 0;
      for (int v = 0; v < V; ++v)
        if (s_tup[v] == W.Klist[v] && W.Klist[v] + 1 > KC) ovf |= 2;
      if (ovf) R->overflow = ovf;
      s_ovf = ovf;
    }
    __syncthreads();
    if (s_ovf) return false;   // nothing changed
    for (int v = 0; v < V; ++v) {
      const int j = W.Klist[v];
      if (s_tup[v] != j) continue;   // uniform (shared + state reads after the barrier)
      for (int d = tid; d < D; d += blockDim.x) {
        P.S1T[((size_t)v * D + d) * KC + j] = 0.0;
        if (cc && cc->S1T) cc->S1T[((size_t)v * D + d) * ks + j] = 0.0;
      }
    }
    __syncthreads();
    if (tid == 0) {
      for (int v = 0; v < V; ++v) {
        const int j = W.Klist[v];
        if (s_tup[v] == j) {
          P.d_id[v * KC + j] = P.next_id[v]++;
          P.d_n[v * KC + j] = 0;
          P.d_l[v * KC + j] = 0;
          P.S2[v * KC + j] = 0.0;
          P.Q[v * KC + j] = 0.0;
          if (cc) cc->S2[v * ks + j] = 0.0;
          R->Klist[v] = j + 1;
          if (cc) {
            cc->d_n[v * ks + j] = 0;
            cc->d_l[v * ks + j] = 0;
            cc->Q[v * ks + j] = 0.0;
            cc->Klist[v] = j + 1;
          }
          cnt[2] += 1;
        }
      }
      const int p1 = *W.T;
      R->T = p1 + 1;
      P.n_t[p1] = 0;
      for (int v = 0; v < V; ++v) P.dish[v * TC + p1] = s_tup[v];
      if (cc) {
        *cc->T = p1 + 1;
        cc->n_t[p1] = 0;
        for (int v = 0; v < V; ++v) cc->dish[v * ts + p1] = s_tup[v];
      }
      cnt[1] += 1;
      s_c = p1;
    }
    __syncthreads();
    c = s_c;
  }
  // move i: p0 -> c (oracle SeqSampler::move)
  if (tid == 0) {
    const int nt0 = W.n_t[p0] - 1, ntc = W.n_t[c];
    s_dies = nt0 == 0;
    s_born = ntc == 0;
    P.n_t[p0] = nt0;
    P.n_t[c] = ntc + 1;
    const double sg = hyp[3 * V + 1];
    const double lm0 = mvc_log((double)nt0 - sg), lmc = mvc_log((double)(ntc + 1) - sg);
    P.lmass[p0] = lm0;
    P.lmass[c] = lmc;
    if (cc) {
      cc->n_t[p0] = nt0;
      cc->n_t[c] = ntc + 1;
      cc->lmass[p0] = lm0;
      cc->lmass[c] = lmc;
    }
    for (int v = 0; v < V; ++v) {
      s_j0[v] = W.dish[v * ts + p0];
      s_j1[v] = W.dish[v * ts + c];
    }
    int Tne = *W.T_ne;
    if (s_dies) --Tne;
    if (s_born) ++Tne;
    R->T_ne = Tne;
    if (cc) *cc->T_ne = Tne;
    P.z[i] = c;
  }
  seq_bar(lds_only);
  if (tid < V && (s_dies || s_born)) {   // table counts of the two tables' dishes
    const int v = tid;
    int L = W.Ltot[v];
    if (s_dies) {
      const int j = s_j0[v];
      const int l = W.d_l[v * ks + j] - 1;
      P.d_l[v * KC + j] = l;
      if (cc) cc->d_l[v * ks + j] = l;
      --L;
    }
    if (s_born) {
      const int j = s_j1[v];
      const int l = W.d_l[v * ks + j] + 1;   // after the decrement above when j == s_j0[v]
      P.d_l[v * KC + j] = l;
      if (cc) cc->d_l[v * ks + j] = l;
      ++L;
    }
    P.Ltot[v] = L;
    if (cc) cc->Ltot[v] = L;
  }
  for (int e = tid; e < V * D; e += blockDim.x) {
    const int v = e / D, d = e - v * D;
    const int j0 = s_j0[v], j1 = s_j1[v];
    if (j0 == j1) continue;
    const double yd = Ci.y[(size_t)v * Ci.ystride + d];
    const double *src = W.S1T + ((size_t)v * D + d) * W.s1s;
    const double a0 = src[j0] - yd, a1 = src[j1] + yd;
    double *col = P.S1T + ((size_t)v * D + d) * KC;
    col[j0] = a0;
    col[j1] = a1;
    if (cc && cc->S1T) {
      double *cl = cc->S1T + ((size_t)v * D + d) * ks;
      cl[j0] = a0;
      cl[j1] = a1;
    }
  }
  if (tid < V) {
    const int v = tid, j0 = s_j0[v], j1 = s_j1[v];
    if (j0 != j1) {
      const double y2 = Ci.Y2[(size_t)v * Ci.y2stride];
      const double a0 = (cc ? cc->S2[v * ks + j0] : P.S2[v * KC + j0]) - y2;
      const double a1 = (cc ? cc->S2[v * ks + j1] : P.S2[v * KC + j1]) + y2;
      P.S2[v * KC + j0] = a0;
      P.S2[v * KC + j1] = a1;
      if (cc) {
        cc->S2[v * ks + j0] = a0;
        cc->S2[v * ks + j1] = a1;
      }
      const int n0 = W.d_n[v * ks + j0] - 1, n1 = W.d_n[v * ks + j1] + 1;
      P.d_n[v * KC + j0] = n0;
      P.d_n[v * KC + j1] = n1;
      if (cc) {
        cc->d_n[v * ks + j0] = n0;
        cc->d_n[v * ks + j1] = n1;
      }
    }
  }
  seq_bar(lds_only);
  if (tid < 2 * V) {   // Q and the coefficients of the two dishes (oracle refresh_dish)
    const int v = tid >> 1, j = (tid & 1) ? s_j1[v] : s_j0[v];
    if (s_j0[v] != s_j1[v]) {
      const double q = fma_sq_strided(W.S1T + (size_t)v * D * W.s1s + j, (size_t)W.s1s, D);
      const Coef cf = coef(W.d_n[v * ks + j], q, hyp[v], l2pt[v], D);
      P.Q[v * KC + j] = q;
      P.c0[v * KC + j] = cf.c0;
      P.cb[v * KC + j] = cf.cb;
      if (cc) {
        cc->Q[v * ks + j] = q;
        cc->c0[v * ks + j] = cf.c0;
        cc->cb[v * ks + j] = cf.cb;
        self_coef_parts(W.d_n[v * ks + j], hyp[v], l2pt[v], D, cc->xm[v * ks + j], cc->ym[v * ks + j],
                        cc->cbm[v * ks + j]);
      }
    }
  }
  if (tid == 0) cnt[0] += 1;
  seq_bar(lds_only);
  return true;
}

// seq_commit of a birth with every call inside it inlined (flatten): the
// lane-column run kernels commit their births themselves, and an outlined
// call there would pass the kernel's arguments through scratch memory.
__device__ __attribute__((flatten, always_inline)) inline bool seq_commit_birth_inline(SeqArgs &A, int i, double *lpw,
                                                                                        double *treew, int nwd) {
  return seq_commit(A, global_view(A), nullptr, global_cust(A, i), i, A.P.z[i], -1, lpw, treew, &A.R->moves, nwd);
}

// A store to global memory as a global_store (not flat: a flat store also
// counts on lgkmcnt, so every LDS-only barrier after it would wait for HBM).
template <class T>
__device__ __forceinline__ void gst(T *p, T v) {
  *(__attribute__((address_space(1))) T *)p = v;
}

// A move p0 -> c (c >= 0) for the run kernel with its whole state in LDS
// (S1 included): the updates of seq_commit (oracle SeqSampler::move) in the
// same operations and order per quantity, split over the block's waves by
// what they write, so no wave reads what another writes in the same commit:
//   wave 0: the two tables (n_t, log mass, T_ne, z, the move count);
//   wave 1: table counts of the dishes (d_l, L_v) and S2;
//   waves 2 / 3: the dish left / joined in every view that changed dish: S1,
//           then Q and the coefficients, then d_n, each from its own writes
//           (in order within a wave; the two dishes differ).
// nt0 / ntc: n_t[p0] and n_t[c] before the move, read by the evaluating wave
// when it drew c (the tables' counts are wave 0's to write).  No block
// barrier inside: the caller's next barrier publishes the LDS writes; global
// arrays are written through (store only) for the kernels after this one.
__device__ __forceinline__ void seq_commit_move_split(SeqArgs &A, const SCache &cc, const Cust &Ci, int i, int p0, int c, int nt0,
                                      int ntc, int32_t *cnt, bool chk = false) {
  ParState &P = A.P;
  Repair *R = A.R;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int V = P.V, D = P.D, KC = P.KC, ks = cc.ks, ts = cc.ts;
  if (chk) {   // MVC_RUN_CHECK: the move's tables and every view's two dishes
    bool ok = run_chk(p0 >= 0 && p0 < *cc.T && c >= 0 && c < *cc.T && i >= 0 && i < P.n, 6, i, p0, c, *cc.T);
    for (int v = 0; v < V && ok; ++v) {
      const int j0 = cc.dish[v * ts + p0], j1 = cc.dish[v * ts + c];
      ok = run_chk(j0 >= 0 && j0 < cc.Klist[v] && j1 >= 0 && j1 < cc.Klist[v], 7, i, v, j0, j1, cc.Klist[v]);
    }
    if (!ok) return;
  }
  const double *hyp = cc.hyp, *l2pt = cc.L2pt;
  const bool dies = nt0 == 1, born = ntc == 0;
  if (w == 0) {
    const double sg = hyp[3 * V + 1];
    const double lmv = mvc_log((double)(lane == 0 ? nt0 - 1 : ntc + 1) - sg);   // lanes 0, 1
    if (lane == 0) {
      const int Tne = *cc.T_ne - (dies ? 1 : 0) + (born ? 1 : 0);
      cc.n_t[p0] = nt0 - 1;
      cc.n_t[c] = ntc + 1;
      cc.lmass[p0] = lmv;
      *cc.T_ne = Tne;
      cnt[0] += 1;
      gst(&P.n_t[p0], nt0 - 1);
      gst(&P.n_t[c], ntc + 1);
      gst(&P.lmass[p0], lmv);
      gst(&R->T_ne, Tne);
      gst(&P.z[i], c);
    }
    if (lane == 1) {
      cc.lmass[c] = lmv;
      gst(&P.lmass[c], lmv);
    }
  } else if (w == 1) {
    for (int v = lane; v < V; v += 64) {
      const int j0 = cc.dish[v * ts + p0], j1 = cc.dish[v * ts + c];
      if (dies || born) {
        int L = cc.Ltot[v];
        if (dies) {
          const int l = cc.d_l[v * ks + j0] - 1;
          cc.d_l[v * ks + j0] = l;
          gst(&P.d_l[v * KC + j0], l);
          --L;
        }
        if (born) {
          const int l = cc.d_l[v * ks + j1] + 1;   // after the decrement above when j1 == j0
          cc.d_l[v * ks + j1] = l;
          gst(&P.d_l[v * KC + j1], l);
          ++L;
        }
        cc.Ltot[v] = L;
        gst(&P.Ltot[v], L);
      }
      if (j0 != j1) {
        const double y2 = Ci.Y2[(size_t)v * Ci.y2stride];
        const double a0 = cc.S2[v * ks + j0] - y2, a1 = cc.S2[v * ks + j1] + y2;
        cc.S2[v * ks + j0] = a0;
        cc.S2[v * ks + j1] = a1;
        gst(&P.S2[v * KC + j0], a0);
        gst(&P.S2[v * KC + j1], a1);
      }
    }
  } else if (w < 4) {   // (waves past 3, in the 8-wave lane kernel, take no part)
    // wave 2: the dish the customer leaves (j0), wave 3: the one it joins (j1),
    // in every view where they differ: S1 (lanes over d), then Q and the
    // coefficients (lanes < V: coef; V <= lane < 2V: the self-removed parts),
    // then d_n (oracle refresh_dish; the two waves touch different dishes)
    const bool join = w == 3;
    for (int e = lane; e < V * D; e += 64) {
      const int v = e / D, d = e - v * D;
      const int j0 = cc.dish[v * ts + p0], j1 = cc.dish[v * ts + c];
      if (j0 == j1) continue;
      const int j = join ? j1 : j0;
      const double yd = Ci.y[(size_t)v * Ci.ystride + d];
      double *cl = cc.S1T + ((size_t)v * D + d) * ks;
      const double a = join ? cl[j] + yd : cl[j] - yd;
      cl[j] = a;
      gst(&P.S1T[((size_t)v * D + d) * KC + j], a);
    }
    for (int k0 = 0; k0 < 2 * V; k0 += 64) {
      // coef(n', Q) (lanes k < V) and self_coef_parts(n') (V <= k < 2V) share
      // their operations: D (-L2pt / 2 - log(b / a) / 2), (tau a) b and
      // 1 / (tau b) with (a, b) = (tau + n', tau + n' + 1), resp. (tau + n' - 1,
      // tau + n'); one instruction stream for both kinds of lane
      const int k = k0 + lane;
      const bool act = k < 2 * V, part = k >= V;
      const int v = act ? (part ? k - V : k) : 0;
      const int j0 = cc.dish[v * ts + p0], j1 = cc.dish[v * ts + c];
      const int j = join ? j1 : j0;
      const bool go = act && j0 != j1;
      const int nj = cc.d_n[v * ks + j] + (join ? 1 : -1);
      const double q = fma_sq_strided(cc.S1T + (size_t)v * D * ks + j, (size_t)ks, D);
      const double tau = hyp[v];
      const double a = tau + (double)(part ? nj - 1 : nj);
      const double b = tau + (double)(part ? nj : nj + 1);
      const double X = (double)D * ((-0.5 * l2pt[v]) - 0.5 * mvc_log_nb(b / a));
      const double Y = (tau * a) * b;
      const double Z = 1.0 / (tau * b);
      const double c0 = X - (0.5 * q) / Y;
      if (go && !part) {
        cc.Q[v * ks + j] = q;
        cc.c0[v * ks + j] = c0;
        cc.cb[v * ks + j] = Z;
        gst(&P.Q[v * KC + j], q);
        gst(&P.c0[v * KC + j], c0);
        gst(&P.cb[v * KC + j], Z);
      }
      if (go && part) {
        cc.xm[v * ks + j] = X;
        cc.ym[v * ks + j] = Y;
        cc.cbm[v * ks + j] = Z;
      }
    }
    // d_n last: the loop above read the counts before the move
    for (int v = lane; v < V; v += 64) {
      const int j0 = cc.dish[v * ts + p0], j1 = cc.dish[v * ts + c];
      if (j0 == j1) continue;
      const int j = join ? j1 : j0;
      const int nj = cc.d_n[v * ks + j] + (join ? 1 : -1);
      cc.d_n[v * ks + j] = nj;
      gst(&P.d_n[v * KC + j], nj);
    }
  }
}

// The run kernel's stay limit adapts to how sparse the movers are: after
// L.limit stays in a row it hands over to grid windows, but where the gaps
// between movers average more than kSparseGap customers a window (one
// customer per wavefront over the grid, ~the latency of one evaluation) finds
// the next mover sooner than run steps of a few customers each, so the limit
// drops to kSparseLimit (measured: configs[3] after its cold transient, gaps
// ~160: 1.36 s per sweep at 64, 0.40 at 8; configs[1], gaps ~5: 0.35 s at 64,
// 0.45 at 8).  Only the schedule of the work changes, not any decision.
constexpr int kSparseGap = 32, kSparseLimit = 8;
__device__ __forceinline__ void note_mover(int32_t &lastm, int32_t &gapq, int f) {
  const int gap = min(f - lastm, 1 << 20);
  gapq = (3 * gapq + 16 * gap) >> 2;
  lastm = f;
}
constexpr int kNoWindows = 1 << 29;   // a limit this large: the run kernel never hands over to windows
__device__ __forceinline__ int stay_limit(int limit, int gapq) {
  return (limit < kNoWindows && gapq > 16 * kSparseGap) ? min(limit, kSparseLimit) : limit;
}

// Resolve the grid window evaluated by the last mvc_seq_eval_kernel (thread 0).
__device__ __forceinline__ void seq_resolve_window(const SeqArgs &A, Repair *R) {
  const int n = A.P.n;
  if (R->done || R->overflow || !(R->win1 > R->win0)) return;
  const int f = R->fmin;
  if (f < R->win1) {   // the first mover of the window: its choice is exact
    R->cur = f;
    R->pend = 1;
    R->pchoice = A.choice[f];
    R->W = A.Wmin;
    note_mover(R->lastm, R->gapq, f);
  } else {             // a mover-free window: every customer in it is final
    R->cur = R->win1;
    R->W = min(2 * R->W, A.Wmax);
  }
  R->win0 = R->win1 = 0;
  R->fmin = n;
}

}  // namespace

// Grid-window repair step (one block of 256 = 4 waves): resolve the last
// window, commit its first mover, open the next window.
extern "C" __global__ __launch_bounds__(256) void mvc_seq_apply_kernel(SeqArgs A) {
  Repair *R = A.R;
  const int tid = threadIdx.x;
  const int n = A.P.n;
  __shared__ int s_go, s_i, s_c;
  if (tid == 0) {
    const int go = !(R->done || R->overflow);
    seq_resolve_window(A, R);
    if (go) R->rounds += 1;
    s_go = go && R->pend;
    if (s_go) {
      s_i = R->cur;
      s_c = R->pchoice;
    }
  }
  __syncthreads();
  if (s_go) {
    const SeqScratch S(A, tid >> 6);
    if (!seq_commit(A, global_view(A), nullptr, global_cust(A, s_i), s_i, A.P.z[s_i], s_c, S.lp, S.tree, &R->moves,
                    blockDim.x >> 6))
      return;   // overflow: the host grows and relaunches this step
    if (tid == 0) {
      R->cur = s_i + 1;
      R->pend = 0;
    }
  }
  if (tid == 0 && !(R->done || R->overflow)) {
    if (R->cur >= n) {
      R->done = 1;
    } else if (!R->pend) {
      R->win0 = R->cur;
      R->win1 = min(n, R->cur + R->W);
      R->fmin = n;
    }
  }
}

// The birth left pending by the lane-column run kernel (its loop stops at a
// birth): the block-cooperative commit on the global state (dish draws on the
// 8 waves), then the next run launch resumes at the following customer and
// re-stages its LDS cache.  A no-op unless a birth is pending.
extern "C" __global__ __launch_bounds__(kSeqRunThreads) void mvc_seq_birth_kernel(SeqArgs A) {
  Repair *R = A.R;
  const int tid = threadIdx.x;
  __shared__ int s_go, s_i;
  if (tid == 0) {
    s_go = !(R->done || R->overflow || R->restride) && R->pend && R->pchoice < 0;
    s_i = R->cur;
  }
  __syncthreads();
  if (!s_go) return;
  const SeqScratch S(A, tid >> 6);
  if (!seq_commit(A, global_view(A), nullptr, global_cust(A, s_i), s_i, A.P.z[s_i], -1, S.lp, S.tree, &R->moves,
                  blockDim.x >> 6))
    return;   // overflow: the host grows and relaunches this step
  if (tid == 0) {
    R->cur = s_i + 1;
    R->pend = 0;
    R->streak = 0;
    // the birth was the sweep's last customer: every customer is final (a
    // run kernel must not start its loop at cur == n)
    if (R->cur >= A.P.n) R->done = 1;
  }
}

// ---------------------------------------------------------------------------
// Grid-wide evaluation: where the state outgrows the run
// kernel's LDS (the Reuters transient: T ~ 18k tables, thousands of dishes per
// view) nearly every customer moves and one customer's evaluation is long
// (sum K_v D dot products against S1 columns in HBM, T V table gathers), so a
// customer is spread over the whole grid: a round is
//   mvc_seq_wide_begin_kernel   resolve the last grid window (as the run kernel);
//   B x { mvc_seq_wide_lp_kernel   the lp rows of customer cur over every block
//                                  (pass 1 of seq_resample_wide), per-block max /
//                                  count of the included dishes per view;
//         mvc_seq_wide_fin_kernel  one block: the rest of seq_resample_wide from
//                                  the combined partials (the order-sensitive sums
//                                  on wave 0), then the decision and its commit
//                                  (births draw their dishes from the same rows) };
//   mvc_seq_eval_kernel         the grid window when the stays run long.
// Every quantity has the operations and order of seq_resample_wide, so the
// decisions are the oracle's bit for bit; only the partition of the
// order-free max / count over the dishes differs.
// ---------------------------------------------------------------------------
constexpr int kWideGridThreads = 256;
extern "C" __global__ void mvc_seq_wide_begin_kernel(SeqArgs A) {
  if (threadIdx.x != 0) return;
  Repair *R = A.R;
  const int n = A.P.n;
  const int go = !(R->done || R->overflow || R->restride);
  if (go && R->win1 > R->win0) {
    seq_resolve_window(A, R);
    if (R->pend) {
      R->mode = kSeqRun;
      R->streak = 0;
    }
  }
  if (!go) return;
  R->rounds += 1;
  if (!(R->mode == kSeqRun || R->pend)) {   // scan mode: the next grid window
    if (R->cur >= n) {
      R->done = 1;
    } else {
      R->win0 = R->cur;
      R->win1 = min(n, R->cur + R->W);
      R->fmin = n;
    }
  } else if (R->cur >= n && !R->pend) {
    R->done = 1;
  }
}

// part: [gridDim.x][2 V] per-block max (or -inf) and count (as a double)
extern "C" __global__ __launch_bounds__(kWideGridThreads) void mvc_seq_wide_lp_kernel(SeqArgs A, double *part) {
  const Repair *R = A.R;
  const ParState &P = A.P;
  if (R->done || R->overflow || R->restride || R->mode != kSeqRun || R->pend || R->cur >= P.n) return;   // block-uniform
  const int i = R->cur;
  const int V = P.V, D = P.D;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = kWideGridThreads / 64;
  const int gr = blockIdx.x * NW + w, gtw = gridDim.x * NW;
  const SView W = global_view(A);
  const SeqScratch S(A, 0);
  const Cust C = global_cust(A, i);
  const int p0 = P.z[i];
  const bool alive = (W.n_t[p0] - 1) > 0;
  const int ts = W.ts, ks = W.ks, lps = S.lps;
  __shared__ double s_mx[NW][MVC_MAXV];
  __shared__ int s_cnt[NW][MVC_MAXV];
  constexpr int kWideY = 2048;
  __shared__ double s_yw[kWideY];
  const bool ylds = V * D <= kWideY;
  for (int v = lane; v < V; v += 64) {
    s_mx[w][v] = -MVC_PM_INF;
    s_cnt[w][v] = 0;
  }
  if (ylds)
    for (int e = tid; e < V * D; e += blockDim.x) {
      const int v = e / D, d = e - v * D;
      s_yw[e] = C.y[(size_t)v * C.ystride + d];
    }
  __syncthreads();
  int NK = 0;
  for (int v = 0; v < V; ++v) NK += W.Klist[v];
  auto locate = [&](int g, int &v, int &j) {
    v = 0;
    int off = 0;
    while (v + 1 < V && g >= off + W.Klist[v]) { off += W.Klist[v]; ++v; }
    j = g - off;
  };
  // lp of dish j of view v from its dot product G (seq_resample_wide's lp_val)
  auto lp_val = [&](int v, int j, double G) -> double {
    const double tau = P.hyper[v];
    const double Y2i = C.Y2[(size_t)v * C.y2stride];
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau;
    if (j == W.dish[v * ts + p0]) {
      const double Gp = G - Y2i;
      const double Qp = (W.Q[v * ks + j] - 2.0 * G) + Y2i;
      const Coef c = coef(W.d_n[v * ks + j] - 1, Qp, tau, A.L2pt[v], D);
      return __builtin_fma(Gp + hy, c.cb, c.c0) + h;
    }
    return __builtin_fma(G + hy, W.cb[v * ks + j], W.c0[v * ks + j]) + h;
  };
  // the chunk's views (its dishes are consecutive in the concatenated list): a
  // segmented max / count of the included dishes into this wave's row
  auto fold = [&](int g, bool valid, int v, int j, double x) {
    const int gl = min(64 * (g / 64) + 63, NK - 1);
    int vf, jf, vl, jl;
    locate(64 * (g / 64), vf, jf);
    locate(gl, vl, jl);
    bool inc = false;
    if (valid) {
      const int l = W.d_l[v * ks + j] - ((j == W.dish[v * ts + p0] && !alive) ? 1 : 0);
      inc = l > 0;
    }
    for (int vv = vf; vv <= vl; ++vv) {
      const bool in = inc && v == vv;
      const double m = wave_max(in ? x : -MVC_PM_INF);
      const int c = wave_count(in);
      if (lane == 0) {
        if (m > s_mx[w][vv]) s_mx[w][vv] = m;
        s_cnt[w][vv] += c;
      }
    }
  };
  // pass 1 of seq_resample_wide: two dishes per lane (chunks c and c + gtw),
  // two fma chains in ascending d
  for (int c = gr; 64 * c < NK; c += 2 * gtw) {
    const int ga = 64 * c + lane, gb = 64 * (c + gtw) + lane;
    const bool va = ga < NK, vb = gb < NK;
    int v_a = 0, j_a = 0, v_b = 0, j_b = 0;
    if (va) locate(ga, v_a, j_a);
    if (vb) locate(gb, v_b, j_b);
    const double *sa = W.S1T + (size_t)v_a * D * W.s1s + j_a, *sb = W.S1T + (size_t)v_b * D * W.s1s + j_b;
    const size_t bs = (size_t)W.s1s;
    double acc_a = 0.0, acc_b = 0.0;
    if (ylds) {
      const int oa = v_a * D, ob = v_b * D;
      int d = 0;
      for (; d + 16 <= D; d += 16) {
        double za[16], zb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          za[u] = sa[(size_t)(d + u) * bs];
          zb[u] = sb[(size_t)(d + u) * bs];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc_a = __builtin_fma(s_yw[oa + d + u], za[u], acc_a);
          acc_b = __builtin_fma(s_yw[ob + d + u], zb[u], acc_b);
        }
      }
      for (; d < D; ++d) {
        acc_a = __builtin_fma(s_yw[oa + d], sa[(size_t)d * bs], acc_a);
        acc_b = __builtin_fma(s_yw[ob + d], sb[(size_t)d * bs], acc_b);
      }
    } else {
      const double *ya = C.y + (size_t)v_a * C.ystride, *yb = C.y + (size_t)v_b * C.ystride;
      for (int d = 0; d < D; ++d) {
        acc_a = __builtin_fma(ya[d], sa[(size_t)d * bs], acc_a);
        acc_b = __builtin_fma(yb[d], sb[(size_t)d * bs], acc_b);
      }
    }
    const double xa = va ? lp_val(v_a, j_a, acc_a) : 0.0, xb = vb ? lp_val(v_b, j_b, acc_b) : 0.0;
    if (va) S.lp[v_a * lps + j_a] = xa;
    if (vb) S.lp[v_b * lps + j_b] = xb;
    fold(64 * c, va, v_a, j_a, xa);
    if (64 * (c + gtw) < NK) fold(64 * (c + gtw), vb, v_b, j_b, xb);
  }
  __syncthreads();
  for (int v = tid; v < V; v += blockDim.x) {   // the block's partials (max and count: order-free)
    double m = -MVC_PM_INF;
    int cnt = 0;
    for (int q = 0; q < NW; ++q) {
      if (s_mx[q][v] > m) m = s_mx[q][v];
      cnt += s_cnt[q][v];
    }
    part[(size_t)blockIdx.x * 2 * V + v] = m;
    part[(size_t)blockIdx.x * 2 * V + V + v] = (double)cnt;
  }
}

// The fin kernel's part of seq_resample_wide (rest_only: the grid wrote the lp
// rows to S.lp and the combined per-view max / count to member row 0) with its
// block-local arrays in the dynamic LDS L (max(NK, TB) doubles, the caller
// checks the fit): the lp rows copied in once, the table scores gathered from
// there, the weighted terms written over the rows, the column sums and the
// running block totals read back from LDS.  In seq_resample_wide those were
// global round trips inside wave 0's order-sensitive loops (Reuters, 16k
// tables and 15k dishes: ~165 us per customer, `profiles/r4m_*`).  The table
// scores are formed before the view terms (they do not depend on them; M and
// s_new are taken after both), and every quantity keeps seq_resample_wide's
// operations and order, so the pick is the same bit for bit.  Block-wide.
// Also writes S.mv and the K_act row of S.koff, which a birth's dish draws
// read.  Returns the pick on member 0 (r == 0), -1 elsewhere.
// doubles of one view's tree levels above the leaves (K + 1 leaves)
__host__ __device__ inline int fin_tree_up(int K) { return (K + 1) / 63 + 8; }
// wide_fin_resample's LDS: the dish terms, the block totals, V tree scratches
__host__ __device__ inline int64_t fin_lds_doubles(int NK, int TB, int V, int kmax) {
  return (int64_t)NK + TB + (int64_t)V * fin_tree_up(kmax);
}
__device__ int wide_fin_resample(const SeqArgs &A, const SView &W, const Cust &C, int i, int p0, const SeqScratch &S,
                                 int r, int tw, double *L, FinLeaves &fl) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63, row = lane >> 4, col = lane & 15;
  const int V = P.V, ts = W.ts, ks = W.ks, lps = S.lps;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  int32_t *kact = S.koff + V + 1;
  __shared__ int f_koff[MVC_MAXV + 1], f_j0[MVC_MAXV];
  __shared__ double f_mv[MVC_MAXV], f_lmv[MVC_MAXV], f_nl[MVC_MAXV], f_mxr[kSeqRunWaves];
  RUN_T0();
  const int np0 = W.n_t[p0] - 1;
  const bool alive = np0 > 0;
  const int Tne_i = *W.T_ne - (alive ? 0 : 1);
  const double mass0 = (double)np0 - sg;
  const double lmass0 = (np0 >= 1 && mass0 > 0.0) ? mvc_log(mass0) : 0.0;
  const int T = *W.T;
  const int TB = (T + 15) / 16;
  if (threadIdx.x == 0) {
    int o = 0;
    for (int v = 0; v < V; ++v) { f_koff[v] = o; o += W.Klist[v]; }
    f_koff[V] = o;
  }
  for (int v = threadIdx.x; v < V; v += blockDim.x) f_j0[v] = W.dish[v * ts + p0];
  if (r == 0) {   // the combined max and count (member row 0), the new dish
    for (int v = lane; v < V; v += 64) {
      double mx = -MVC_PM_INF;
      int cnt = 0;
      {
        const double x = S.wide[V + 8 + v];
        if (x > mx) mx = x;
        cnt += (int)S.wide[V + 8 + 8 * V + v];
      }
      const double Y2i = C.Y2[(size_t)v * C.y2stride];
      const double lfn = A.cnew[v] + (-0.5 * Y2i) / P.hyper[v];
      const double m = lfn > mx ? lfn : mx;
      S.mv[v] = m;
      f_mv[v] = m;
      kact[v] = cnt;
    }
  }
  __syncthreads();
  const int NK = f_koff[V];
  auto view_of = [&](int g) {
    int v = 0;
    while (v + 1 < V && g >= f_koff[v + 1]) ++v;
    return v;
  };
  {   // the lp rows, concatenated by view: 8 loads per thread in flight
    constexpr int kC = 8;
    const int bd = blockDim.x;
    for (int g0 = threadIdx.x; g0 < NK; g0 += kC * bd) {
      double x[kC];
#pragma unroll
      for (int u = 0; u < kC; ++u) {
        const int g = min(g0 + u * bd, NK - 1);
        const int v = view_of(g);
        x[u] = S.lp[(size_t)v * lps + (g - f_koff[v])];
      }
#pragma unroll
      for (int u = 0; u < kC; ++u)
        if (g0 + u * bd < NK) L[g0 + u * bd] = x[u];
    }
  }
  __syncthreads();
  // table scores in view order (every load of a step issued at once), member maxima
  double M = -MVC_PM_INF;
  {
    constexpr int kU = 8;
    const int nch = TB * 16;
    constexpr int kVR = 4;   // views whose dish indices are loaded with the step's other loads
    for (int c0 = r; c0 * 64 < nch; c0 += tw * kU) {
      int np[kU], dj[kU][kVR];
      double lm[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        const int pc = min(p, T - 1);
        np[u] = p < T ? W.n_t[pc] - (p == p0 ? 1 : 0) : 0;
        lm[u] = p < T ? ((p == p0) ? lmass0 : W.lmass[pc]) : 0.0;
#pragma unroll
        for (int v = 0; v < kVR; ++v) dj[u][v] = W.dish[min(v, V - 1) * ts + pc];
      }
      double sp[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        const double mass = (double)np[u] - sg;
        sp[u] = (p < T && np[u] >= 1 && mass > 0.0) ? lm[u] : -MVC_PM_INF;
      }
#pragma unroll
      for (int v = 0; v < kVR; ++v) {
        if (v < V) {
#pragma unroll
          for (int u = 0; u < kU; ++u)
            if (sp[u] != -MVC_PM_INF) sp[u] = sp[u] + L[f_koff[v] + dj[u][v]];
        }
      }
      for (int v = kVR; v < V; ++v) {   // views past kVR: their dish index loaded here
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int p = (c0 + u * tw) * 64 + lane;
          const int d = W.dish[v * ts + min(p, T - 1)];
          if (sp[u] != -MVC_PM_INF) sp[u] = sp[u] + L[f_koff[v] + d];
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int p = (c0 + u * tw) * 64 + lane;
        if (p < nch) S.e[p] = sp[u];
        if (sp[u] > M) M = sp[u];
      }
    }
    M = wave_max(M);
    if (lane == 0) f_mxr[r] = M;
  }
  __syncthreads();
  RUN_MARK(1);
  // pass 2: the weighted terms, over the rows in LDS (the table counts of 8
  // chunks loaded at once)
  for (int c0 = r; 64 * c0 < NK; c0 += 8 * tw) {
    int lq[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = min(64 * (c0 + u * tw) + lane, NK - 1);
      const int v = view_of(g), j = g - f_koff[v];
      lq[u] = W.d_l[v * ks + j] - ((j == f_j0[v] && !alive) ? 1 : 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int g = 64 * (c0 + u * tw) + lane;
      if (g < NK) {
        const int v = view_of(g);
        const int l = lq[u];
        double t = 0.0;
        if (l > 0) {
          double wgt = (double)l - P.hyper[2 * V + v];
          if (wgt < 0.0) wgt = 0.0;
          t = wgt * mvc_exp(L[g] - f_mv[v]);
        }
        L[g] = t;
      }
    }
  }
  __syncthreads();
  // member 0: column partials in ascending j, pw16, the new dish, lm_v
  if (r == 0) {
    for (int vg = 0; vg < V; vg += 4) {
      const int v = vg + row;
      double cs = 0.0;
      if (v < V) {
        const int K = W.Klist[v];
        const double *ax = L + f_koff[v] + col;
        const int cnt = K > col ? (K - col + 15) >> 4 : 0;
        double xa[16];
        for (int e0 = 0; e0 < cnt; e0 += 16) {
#pragma unroll
          for (int u = 0; u < 16; ++u) xa[u] = e0 + u < cnt ? ax[16 * (e0 + u)] : 0.0;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (e0 + u < cnt) cs = cs + xa[u];
        }
      }
      double Sv = row_pw16(cs);
      if (v < V && col == 0) {
        const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
        const double Y2i = C.Y2[(size_t)v * C.y2stride];
        const double lfn = A.cnew[v] + (-0.5 * Y2i) / tau;
        const double m = f_mv[v];
        double wn = alpha + (double)kact[v] * sigma;
        if (wn < 0.0) wn = 0.0;
        const double nl = wn * mvc_exp(lfn - m);   // also the new dish's leaf of a birth's dish draw
        f_nl[v] = nl;
        Sv = Sv + nl;
        const double denom = alpha + (double)(W.Ltot[v] - (alive ? 0 : 1));
        f_lmv[v] = (denom <= 0.0) ? lfn : (m + mvc_log(Sv)) - mvc_log(denom);
      }
    }
  }
  __syncthreads();
  RUN_MARK(0);
  // s_new in view order (every member); weights, block sums B_b into L after the terms
  double *Lb = L + NK;
  double s_new = mvc_log(ag + sg * (double)Tne_i);
  for (int v = 0; v < V; ++v) s_new = s_new + f_lmv[v];
  for (int k = 0; k < tw; ++k) M = f_mxr[k] > M ? f_mxr[k] : M;
  if (s_new > M) M = s_new;
  for (int c0 = r; c0 * 64 < TB * 16; c0 += tw) {
    const int p = c0 * 64 + lane;
    double wgt = 0.0;
    if (p < TB * 16) {
      const double x = S.e[p];
      wgt = x != -MVC_PM_INF ? mvc_exp(x - M) : 0.0;
      S.e[p] = wgt;
    }
    const double Bv = row_pw16(wgt);
    const int b = c0 * 4 + row;
    if (col == 0 && b < TB) Lb[b] = Bv;
  }
  __syncthreads();
  RUN_MARK(2);
  int pick = -1;
  if (r == 0) {   // running block totals in block order on lane 0 from LDS (8 reads in flight), the draw
    __shared__ double f_tot;
    __shared__ int f_bsel;
    __shared__ double f_cprev;
    const double u0 = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z);
    if (lane == 0) {
      double tot = 0.0;
      int b = 0;
      for (; b + 8 <= TB; b += 8) {
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = Lb[b + q];
#pragma unroll
        for (int q = 0; q < 8; ++q) tot = tot + x[q];
      }
      for (; b < TB; ++b) tot = tot + Lb[b];
      const double Wt = mvc_exp(s_new - M) + tot;
      const double u = u0 * Wt;
      int bsel = -1;
      double cprev = 0.0;
      if (u < tot) {   // the first block whose running total exceeds u (the same sums again)
        double c = 0.0;
        bsel = TB - 1;
        b = 0;
        bool found = false;
        for (; b + 8 <= TB && !found; b += 8) {
          double x[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) x[q] = Lb[b + q];
          int hit = 8;
          double cp = c;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const double c2 = c + x[q];
            if (hit == 8 && u < c2) { hit = q; cp = c; }
            c = c2;
          }
          if (hit < 8) { bsel = b + hit; cprev = cp; found = true; }
        }
        for (; b < TB && !found; ++b) {
          const double c2 = c + Lb[b];
          if (u < c2) { bsel = b; cprev = c; found = true; }
          c = c2;
        }
      }
      f_tot = u;
      f_bsel = bsel;
      f_cprev = cprev;
    }
    wave_lds_sync();
    const int bsel = f_bsel;
    if (bsel >= 0) {
      const double u = f_tot - f_cprev;
      const double x = lane < 16 ? S.e[bsel * 16 + lane] : 0.0;
      pick = bsel * 16 + pw16_select_wave(x, u);
    } else {
      pick = -1;
    }
  }
  RUN_MARK(3);
  int kmax = 0;
  for (int v = 0; v < V; ++v) kmax = max(kmax, W.Klist[v]);
  fl.L = L;
  fl.koff = f_koff;
  fl.newleaf = f_nl;
  fl.up = Lb + TB;
  fl.upstride = fin_tree_up(kmax);
  return pick;
}

// One block of kSeqRunThreads: a pending mover from a resolved window is
// committed; otherwise customer cur is decided from the lp rows and partials
// of mvc_seq_wide_lp_kernel (nblk blocks) and committed when it moves.  After
// `limit` stays in a row (stay_limit) it hands over to the grid windows.
extern "C" __global__ __launch_bounds__(kSeqRunThreads) void mvc_seq_wide_fin_kernel(SeqArgs A, const double *part,
                                                                                     int nblk, int limit, int lds_cap) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x, w = tid >> 6, nw = blockDim.x >> 6;
  const int n = P.n, V = P.V;
  __shared__ int s_go, s_i, s_pend, s_pc, s_c;
  if (tid == 0) {
    s_go = !(R->done || R->overflow || R->restride) && R->mode == kSeqRun && R->cur < n;
    s_i = R->cur;
    s_pend = R->pend;
    s_pc = R->pchoice;
  }
  __syncthreads();
  if (!s_go) return;
  const int i = s_i;
  const int p0 = P.z[i];
  const SeqScratch Sw(A, w);
#ifdef MVC_RUN_PROF
  if (tid < 12) mvc_prof_lds[tid] = 0;
  __syncthreads();
  uint64_t f0 = wall_clock64();
  const uint64_t w_start = f0, c_start = clock64();
  auto fin_flush = [&](int decided, int committed) {   // thread 0: this launch's phases into R->prof[12..]
    if (tid == 0) {
      R->prof[20] += wall_clock64() - w_start;
      R->prof[21] += clock64() - c_start;
      R->prof[17] += committed ? wall_clock64() - f0 : 0;
      for (int k = 0; k < 4; ++k) R->prof[13 + k] += mvc_prof_lds[k];
      R->prof[18] += decided;
      R->prof[19] += committed;
    }
  };
#define FIN_MARK(k) do { const uint64_t _n = wall_clock64(); if (tid == 0) R->prof[k] += _n - f0; f0 = _n; } while (0)
#else
  auto fin_flush = [](int, int) {};
#define FIN_MARK(k) do {} while (0)
#endif
  if (s_pend) {   // a window's first mover (its lp rows are not in the scratch: computed by the commit)
    if (!seq_commit(A, global_view(A), nullptr, global_cust(A, i), i, p0, s_pc, Sw.lp, Sw.tree, &R->moves, nw))
      return;   // overflow: the host grows and the next round redoes this commit
    fin_flush(0, 1);
    if (tid == 0) {
      R->cur = i + 1;
      R->pend = 0;
      R->streak = 0;
      if (R->cur >= n) R->done = 1;
    }
    return;
  }
  const SeqScratch S0(A, 0);
  {   // the per-block partials combined into member row 0 of the wide scratch
    double *pmx = S0.wide + V + 8, *pcnt = pmx + 8 * V;
    for (int v = tid; v < V; v += blockDim.x) {
      double m = -MVC_PM_INF, c = 0.0;
      for (int b = 0; b < nblk; ++b) {
        const double x = part[(size_t)b * 2 * V + v];
        if (x > m) m = x;
        c += part[(size_t)b * 2 * V + V + v];   // integers below 2^53: exact in any order
      }
      pmx[v] = m;
      pcnt[v] = c;
    }
  }
  __syncthreads();
  FIN_MARK(12);
  int c;
  FinLeaves fl{};
  bool use_fl = false;
  {   // the LDS-resident evaluation when the dish terms, block totals and dish-draw trees fit
    const SView W0 = global_view(A);
    int nk = 0, kmax = 0;
    for (int v = 0; v < V; ++v) {
      nk += W0.Klist[v];
      kmax = max(kmax, W0.Klist[v]);
    }
    const int tb = (*W0.T + 15) / 16;
    if (fin_lds_doubles(nk, tb, V, kmax) * 8 <= (int64_t)lds_cap) {
      c = wide_fin_resample(A, W0, global_cust(A, i), i, p0, S0, w, nw, mvc_seq_lds, fl);
      use_fl = true;
    } else {
      c = seq_resample_wide(A, W0, global_cust(A, i), i, p0, S0, w, nw, true, true);
    }
  }
  if (tid == 0) s_c = c;   // member 0's pick
  __syncthreads();
#ifdef MVC_RUN_PROF
  f0 = wall_clock64();
#endif
  const int ch = s_c;
  if (ch == p0) {   // stays
    fin_flush(1, 0);
    if (tid == 0) {
      R->cur = i + 1;
      R->streak += 1;
      if (R->streak >= stay_limit(limit, R->gapq)) {
        R->mode = kSeqScan;
        if (R->cur < n) {
          R->win0 = R->cur;
          R->win1 = min(n, R->cur + R->W);
          R->fmin = n;
        }
      }
      if (R->cur >= n) R->done = 1;
    }
    return;
  }
  // a move or a birth: committed on the global state, dish draws from the rows above
  if (!seq_commit(A, global_view(A), nullptr, global_cust(A, i), i, p0, ch, Sw.lp, Sw.tree, &R->moves, nw, &S0, false,
                  use_fl ? fl : FinLeaves{})) {
    if (tid == 0) {   // overflow: left pending (the next round commits it after the growth)
      R->pend = 1;
      R->pchoice = ch;
    }
    return;
  }
  fin_flush(1, 1);
#undef FIN_MARK
  if (tid == 0) {
    note_mover(R->lastm, R->gapq, i);
    R->cur = i + 1;
    R->streak = 0;
    if (R->cur >= n) R->done = 1;
  }
}

// The run kernel's repair cursor (LDS, owned by thread 0 while the kernel
// runs; read from R at entry and written back at exit).
struct RunCursor {
  int go, stop, cur, pend, pc, pp0, mode, streak, done, i;
  int fill;                       // ring: customers [.., fill) are requested (slot = customer % ring)
  int landed;                     // ring: customers [.., landed) are in LDS (every request before them waited for)
  int lpc;                        // wide evaluation: the customer whose lp rows wave 0's scratch holds (-1: none)
  int32_t cnt[3];                 // moves, births, new dishes
  int32_t lastm, gapq;            // Repair::lastm / gapq
  int ch[kSeqRunWaves], p0[kSeqRunWaves];
  int chb[2][kSeqLcThreads / 64], p0b[2][kSeqLcThreads / 64];   // the lane-column loop's, by step parity
  int ntb[2][kSeqLcThreads / 64][2];   // ... and n_t of the mover's two tables before its move
};

namespace {

// The staged-row ring of the run kernel: slot k holds customer c with
// c % ring == k (y rows [V][D], Y2 [V], z).
struct Ring {
  double *base;
  int n, slot;
  __device__ double *at(int c) const { return base + (int64_t)(c & (n - 1)) * slot; }
  __device__ Cust cust(int c, int V, int D) const {
    Cust C;
    C.y = at(c);
    C.ystride = (size_t)D;
    C.Y2 = at(c) + (size_t)V * D;
    C.y2stride = 1;
    return C;
  }
};
// Asynchronous fill of the ring with customers [c0, c1) (c1 - c0 <= ring,
// within one pass of the ring): direct global -> LDS dword loads
// (global_load_lds_dword: no registers, completion on vmcnt), the dword
// range of the slots split over the waves, 64 dwords per instruction.  The
// caller waits (s_waitcnt + barrier) before anyone reads the slots.  Slot
// dwords: y rows [V][D] (2 per double), Y2 [V], then z (int) twice.
// nwc: the block's waves when known at compile time (blockDim.x is a load
// from the dispatch packet, and that load waits for every outstanding store).
template <int nwc = 0>
__device__ __forceinline__ void ring_fill_async(const SeqArgs &A, const Ring &G, int c0, int c1) {
  const int V = A.P.V, D = A.P.D, n = A.P.n;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = nwc ? nwc : (int)(blockDim.x >> 6);
  const int sdw = 2 * G.slot;
  int c = c0;
  while (c < c1) {   // contiguous runs of slots (split at the ring's end)
    const int k0 = c & (G.n - 1);
    const int run = min(c1 - c, G.n - k0);
    const int cnt = run * sdw;
    char *dst0 = (char *)(G.base + (int64_t)k0 * G.slot);
    for (int q = w; q * 64 < cnt; q += nw) {
      const int k = q * 64 + lane;
      if (k < cnt) {
        const int cc = c + k / sdw, dw = k - (k / sdw) * sdw, e = dw >> 1, half = dw & 1;
        const int32_t *src;
        if (e < V * D) {
          const int v = e / D, d = e - v * D;
          src = (const int32_t *)(A.y + ((size_t)v * n + cc) * D + d) + half;
        } else if (e < V * D + V) {
          src = (const int32_t *)(A.Y2 + (size_t)(e - V * D) * n + cc) + half;
        } else {   // z, then the phase-A choice (value prediction's guess)
          src = half ? A.choice + cc : A.P.z + cc;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(dst0 + (int64_t)q * 256), 4, 0, 0);
      }
    }
    c += run;
  }
}
__device__ __forceinline__ int ring_z(const Ring &G, int c, int V, int D) {
  return ((const int32_t *)(G.at(c) + (size_t)V * D + V))[0];
}
__device__ __forceinline__ int ring_pred(const Ring &G, int c, int V, int D) {
  return ((const int32_t *)(G.at(c) + (size_t)V * D + V))[1];
}

// The run kernel's loop, for state read through the LDS cache (kLds) or the
// global arrays.  Returns why it stopped early: kRunOvf | kRunRestride (flags
// by value, so nothing of the kernel lives in scratch memory).
constexpr int kRunOvf = 1, kRunRestride = 2, kRunVpOff = 4;
template <bool kLds, bool kWide>
__device__ int seq_run_loop(SeqArgs &A, const SeqLds &L, const SView &Wv, const SCache *ccp, const SeqScratch &S,
                            const Ring &G, double *tree, RunCursor &U) {
  const ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, n = P.n;
  const bool ring = kLds && G.n > 0;
  const bool lsync = kLds && ccp && ccp->S1T;   // every state read is an LDS read: LDS-only barriers
  for (;;) {
    // invariant here: U.mode == kSeqRun || U.pend, not done
    RUN_T0();
    if (U.pend) {
      const bool staged = ring && U.cur < U.landed && U.cur >= U.fill - G.n;
      const Cust Ci = staged ? G.cust(U.cur, V, D) : global_cust(A, U.cur);
      // dish draws of a birth: wave w < nwd, each with its own lp scratch
      // wide evaluation of this very customer against this state: its lp rows are reused by the dish draws
      const SeqScratch S0(A, 0);
      const bool reuse = kWide && !kLds && U.lpc == U.cur;
      if (!seq_commit(A, Wv, ccp, Ci, U.cur, U.pp0, U.pc, S.lp, tree, U.cnt,
                             kLds ? L.nws : (int)(blockDim.x >> 6), reuse ? &S0 : nullptr, lsync)) {
        // overflow: the host grows and relaunches
        return kRunOvf;
      }
      RUN_MARK(3);
      if (tid == 0) {
        U.cur = U.cur + 1;
        U.pend = 0;
        U.streak = 0;
      }
    }
    if (tid == 0) {
      U.stop = 0;
      if (U.cur >= n) {
        U.done = 1;
        U.stop = 1;
      } else if (kLds) {   // the LDS layout must hold the current lists plus one birth
        int bad = *Wv.T >= L.ts ? 1 : 0;
        for (int v = 0; v < V; ++v) bad |= Wv.Klist[v] >= L.ks ? 1 : 0;
        if (bad) U.stop = 2;
      }
      U.i = U.cur;
    }
    seq_bar(lsync);
    RUN_MARK(4);
    if (U.stop) return U.stop == 2 ? kRunRestride : 0;
    const int i0 = U.i;
    const int need = min(n, i0 + L.nws);
    int fill_next = 0, landed_next = 0;
    if (ring) {
      // The rows arrive in batches, requested half a ring ahead, so a step
      // waits for memory only when its customers are beyond what has landed
      // (once per batch; by then the batch was requested tens of steps ago).
      // Every wait is s_waitcnt(0): vmcnt also counts the commits' stores.
      fill_next = max(U.fill, i0);
      landed_next = U.landed;
      if (need > U.landed) {
        if (fill_next < need) {
          ring_fill_async(A, G, fill_next, need);
          fill_next = need;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        landed_next = fill_next;
      }
      if (fill_next - i0 <= G.n / 2 && fill_next < n) {   // keep the next batch in flight
        const int f1 = min(n, i0 + G.n);
        ring_fill_async(A, G, fill_next, f1);
        fill_next = f1;
      }
    }
    if constexpr (kWide && !kLds) {   // global scratch: the whole block on one customer
      const int i = i0;
      const bool act = i < n;
      const int p0 = act ? P.z[i] : 0;
      const int c = seq_resample_wide(A, Wv, global_cust(A, act ? i : 0), i, p0, SeqScratch(A, 0), w, L.tw, act);
      if (act && w == 0 && lane == 0) {
        U.ch[0] = c;
        U.p0[0] = p0;
      }
    }
    const int i = i0 + w;
    if (!kWide && w < L.nws && i < n) {
      int p0;
      Cust C;
      if (ring) {
        C = G.cust(i, V, D);
        p0 = ring_z(G, i, V, D);
      } else if (kLds) {   // stage the customer's rows in LDS: one memory latency for the whole evaluation
        p0 = P.z[i];   // customers after cur keep their sweep-start table until committed
        for (int e = lane; e < V * D; e += 64) {
          const int v = e / D, d = e - v * D;
          S.ys[e] = A.y[((size_t)v * n + i) * D + d];
        }
        if (lane < V) S.ys[V * D + lane] = A.Y2[(size_t)lane * n + i];
        __threadfence_block();
        C.y = S.ys;
        C.ystride = (size_t)D;
        C.Y2 = S.ys + (size_t)V * D;
        C.y2stride = 1;
      } else {
        p0 = P.z[i];
        C = global_cust(A, i);
      }
      const int c = seq_resample(A, Wv, C, i, p0, S);
      if (lane == 0) {
        U.ch[w] = c;
        U.p0[w] = p0;
      }
    }
    seq_bar(lsync);
    RUN_MARK(5);
    if (tid == 0) {
      if (ring) {
        U.fill = fill_next;
        U.landed = landed_next;
      }
      int f = -1;
      const int m = min(L.nws, n - U.i);
      for (int k = 0; k < m; ++k)
        if (U.ch[k] != U.p0[k]) { f = k; break; }
      if (f >= 0) {
        U.cur = U.i + f;
        U.pend = 1;
        U.pc = U.ch[f];
        U.pp0 = U.p0[f];
        U.lpc = (kWide && !kLds) ? U.cur : -1;
        note_mover(U.lastm, U.gapq, U.cur);
      } else {
        U.cur = U.i + m;
        U.streak += m;
        if (U.streak >= stay_limit(L.limit, U.gapq)) U.mode = kSeqScan;
        if (U.cur >= n) U.done = 1;
      }
      U.go = !U.done && (U.mode == kSeqRun || U.pend);
    }
    seq_bar(lsync);
    RUN_MARK(6);
#ifdef MVC_RUN_PROF
    if (tid == 0) mvc_prof_lds[7] += 1;
#endif
    if (!U.go) return 0;
  }
}

// seq_run_loop for the lane-column evaluation (L.lc: the whole state in LDS,
// S1 included, the staged-row ring), compiled as its own kernel instance so
// nothing of the other evaluation shapes sits in its registers.
//   * moves are committed by wave 0 alone (seq_commit_move_wave); a birth
//     ends the loop with the birth pending, and mvc_seq_birth_kernel commits
//     it on the global state before the next launch (births are rare here,
//     and the general commit inlined would raise the loop's register pressure);
//   * the cursor lives in registers, the same in every wave: each wave
//     derives it from the same LDS values after the same barriers, so a step
//     is {commit; barrier; evaluate; barrier} with no single-thread decision
//     section; the speculated choices are double-buffered by step parity (a
//     step without a commit has only one barrier, so a fast wave may write
//     the next step's choices while a slow one still reads this step's);
//   * every barrier waits for LDS operations only.
__device__ __forceinline__ int seq_run_loop_lc(SeqArgs &A, const SeqLds &L, const Ring &G, RunCursor &U) {
  int flags = 0;
  const ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, n = P.n;
  const SCache cc = lds_cache(V, D, L.ts, L.ks, 1);   // L.lc implies S1 in LDS
  SView Wv = cache_view(cc, A);
  Wv.S1T = cc.S1T;                                      // no select against the global copy: LDS for sure
  Wv.s1s = cc.ks;
  const SeqScratch S(mvc_seq_lds + L.cache_dbl + (int64_t)w * L.stride, V, L.ks, L.ts);
  int cur = U.cur, pend = U.pend, pc = U.pc, pp0 = U.pp0, mode = U.mode, streak = U.streak, done = U.done;
  int fill = U.fill, landed = U.landed, par = 0;
  int pnt0 = 0, pntc = 0;   // n_t of the pending mover's two tables before its move
  int lastm = U.lastm, gapq = U.gapq;
  if (pend && pc >= 0) {    // a mover carried over from the previous launch
    pnt0 = cc.n_t[pp0];
    pntc = cc.n_t[pc];
  }
  if (pend && pc >= 0) {   // a mover carried over from the previous launch (a resolved window): stage its row
    ring_fill_async<kSeqLcThreads / 64>(A, G, cur, cur + 1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    fill = landed = cur + 1;
  }
  {   // the LDS layout must hold the current lists plus one birth.  Checked once:
      // this loop commits moves only (a birth ends it), which add no table and
      // no dish, so T and the dish lists stay as they are until it returns
    bool bad = *cc.T >= L.ts;
    for (int v = 0; v < V; ++v) bad = bad || cc.Klist[v] >= L.ks;
    if (bad) flags |= kRunRestride;
  }
  for (;;) {
    RUN_T0();
    if (flags & kRunRestride) break;
    if (pend) {
      if (pc < 0) break;   // a birth: left pending for mvc_seq_birth_kernel (inlined here, the
                           // general commit costs the loop 184 B of scratch and flat accesses)
      // the mover was evaluated in the previous step (or staged above), so its
      // row is in the ring (landed, not yet reused: requests stop a ring ahead of it)
      seq_commit_move_split(A, cc, G.cust(cur, V, D), cur, pp0, pc, pnt0, pntc, U.cnt, L.chk);
      cur = cur + 1;
      pend = 0;
      streak = 0;
      RUN_MARK(3);
      if (cur >= n) {
        done = 1;
        break;
      }
      seq_bar(true);   // the commit, visible to every wave
      if (L.chk && mvc_run_bad[0]) break;
    }
    RUN_MARK(4);
    const int i0 = cur;
    const int need = min(n, i0 + L.nws);
    // rows in batches half a ring ahead; a step waits only beyond what has
    // landed (slots being refilled belong to customers before cur: final)
    if (need > landed) {
      if (fill < need) {
        ring_fill_async<kSeqLcThreads / 64>(A, G, max(fill, i0), need);
        fill = need;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      landed = fill;
    }
    if (fill - i0 <= G.n / 2 && fill < n) {
      const int f1 = min(n, i0 + G.n);
      ring_fill_async<kSeqLcThreads / 64>(A, G, max(fill, i0), f1);
      fill = f1;
    }
    const int i = i0 + w;
    if (w < L.nws && i < n) {
      const int p0 = ring_z(G, i, V, D);
      const int c = seq_resample_lc(A, Wv, G.cust(i, V, D), i, p0, S, cc.hyp, cc.cnew);
      if (lane == 0) {
        U.chb[par][w] = c;
        U.p0b[par][w] = p0;
        if (c != p0 && c >= 0) {
          U.ntb[par][w][0] = cc.n_t[p0];
          U.ntb[par][w][1] = cc.n_t[c];
        }
      }
    }
    seq_bar(true);
    RUN_MARK(5);
    // every wave: the first customer whose choice is not its table (the step's
    // choices read together, then the first mismatch below m by selects)
    const int m = min(L.nws, n - i0);
    constexpr int kW = kSeqLcThreads / 64;
    int chs[kW], p0s[kW];
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      chs[k] = U.chb[par][k];
      p0s[k] = U.p0b[par][k];
    }
    int f = -1;
#pragma unroll
    for (int k = kW - 1; k >= 0; --k)
      if (k < m && chs[k] != p0s[k]) f = k;
    if (f >= 0) {
      cur = i0 + f;
      pend = 1;
      pc = U.chb[par][f];
      pp0 = U.p0b[par][f];
      if (pc >= 0) {
        pnt0 = U.ntb[par][f][0];
        pntc = U.ntb[par][f][1];
      }
      note_mover(lastm, gapq, cur);
    } else {
      cur = i0 + m;
      streak += m;
      if (streak >= stay_limit(L.limit, gapq)) mode = kSeqScan;
      if (cur >= n) done = 1;
    }
#ifdef MVC_RUN_PROF
    if (tid == 0) {   // how often the sequential decision equals the phase-A choice (A.choice)
      const int nd = f >= 0 ? f + 1 : m;
      for (int k = 0; k < nd; ++k) {
        const int ck = U.chb[par][k];
        mvc_prof_lds[8] += 1;
        if (A.choice[i0 + k] == ck) mvc_prof_lds[9] += 1;
        if (k == f) {
          mvc_prof_lds[10] += 1;
          if (A.choice[i0 + k] == ck) mvc_prof_lds[11] += 1;
        }
      }
    }
#endif
    par ^= 1;
    RUN_MARK(6);
#ifdef MVC_RUN_PROF
    if (tid == 0) mvc_prof_lds[7] += 1;
#endif
    if (done || !(mode == kSeqRun || pend)) break;
  }
  __builtin_amdgcn_s_waitcnt(0);   // no row request outlives the wave
  __syncthreads();                 // every wave out of the loop before thread 0 writes the cursor back
  if (tid == 0) {
    U.cur = cur;
    U.pend = pend;
    U.pc = pc;
    U.pp0 = pp0;
    U.mode = mode;
    U.streak = streak;
    U.done = done;
    U.fill = fill;
    U.landed = landed;
    U.lastm = lastm;
    U.gapq = gapq;
  }
  return flags;
}

// ---- value prediction: the overlay, its commit, the loop ----

// The step's predicted moves (uniform, every thread the same): customer
// i0 + m moves p0 -> c when its phase-A choice c >= 0 differs from its table
// p0; dies / born from the table counts with the earlier predicted moves applied.
struct VpMoves {
  int mv[kVpMoves], p0[kVpMoves], c[kVpMoves], dies[kVpMoves], born[kVpMoves];
};
// a[i] for a runtime i without indexing a register array (which would go to scratch)
template <class T>
__device__ __forceinline__ T vsel(const T (&a)[kVpMoves], int i) {
  T r = a[0];
#pragma unroll
  for (int k = 1; k < kVpMoves; ++k)
    if (i == k) r = a[k];
  return r;
}
__device__ __forceinline__ VpMoves vp_moves(const SCache &cc, int nm, const int (&pz)[kVpMoves],
                                            const int (&pcs)[kVpMoves]) {
  VpMoves M;
#pragma unroll
  for (int m = 0; m < kVpMoves; ++m) {
    M.mv[m] = m < nm && pcs[m] >= 0 && pcs[m] != pz[m];
    M.p0[m] = pz[m];
    M.c[m] = pcs[m];
    M.dies[m] = M.born[m] = 0;
    if (M.mv[m]) {
      int a = cc.n_t[M.p0[m]], b = cc.n_t[M.c[m]];
#pragma unroll
      for (int m2 = 0; m2 < m; ++m2)
        if (M.mv[m2]) {
          a += (M.p0[m] == M.c[m2] ? 1 : 0) - (M.p0[m] == M.p0[m2] ? 1 : 0);
          b += (M.c[m] == M.c[m2] ? 1 : 0) - (M.c[m] == M.p0[m2] ? 1 : 0);
        }
      M.dies[m] = a == 1;
      M.born[m] = b == 0;
    }
  }
  return M;
}

// The step's predicted moves into the overlay header (thread 0; a barrier
// before vp_build): per-lane indexing by move reads them from LDS (indexing a
// register array by a per-lane value would put it in scratch).
__device__ __forceinline__ void vp_publish(const VpMoves &M, const int (&pz)[kVpMoves], const int (&pcs)[kVpMoves]) {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int m = 0; m < kVpMoves; ++m) {
      mvc_vp_ov.pz[m] = pz[m];
      mvc_vp_ov.pcs[m] = pcs[m];
      mvc_vp_ov.mv[m] = M.mv[m];
      mvc_vp_ov.p0[m] = M.p0[m];
      mvc_vp_ov.c[m] = M.c[m];
      mvc_vp_ov.dies[m] = M.dies[m];
      mvc_vp_ov.born[m] = M.born[m];
    }
  }
}

// Build the overlay (mvc_vp_ov) of the predicted moves of customers
// i0 .. i0 + nm - 1 on the current LDS state: every value with the
// arithmetic its commit would use (seq_commit_move_split), for the state
// after moves 0 .. m.  yr[m]: customer i0 + m's staged row.  Block-wide; the
// caller's barrier publishes it.
__device__ __forceinline__ void vp_build(const SeqArgs &A, const SCache &cc, const VpMoves &M, int nm,
                                         const double *const (&yr)[kVpMoves], double *ovs1) {
  const int tid = threadIdx.x;
  const int V = A.P.V, D = A.P.D, ks = cc.ks, ts = cc.ts;
  const double *hyp = cc.hyp, *l2pt = cc.L2pt;
  const double sg = hyp[3 * V + 1];
  if (tid < 2 * kVpMoves) {   // the two tables of move m
    const int m = tid >> 1, which = tid & 1;
    if (mvc_vp_ov.mv[m]) {
      const int p = which ? mvc_vp_ov.c[m] : mvc_vp_ov.p0[m];
      int n_ = cc.n_t[p];
#pragma unroll
      for (int m2 = 0; m2 < kVpMoves; ++m2)
        if (m2 <= m && M.mv[m2]) n_ += (p == M.c[m2] ? 1 : 0) - (p == M.p0[m2] ? 1 : 0);
      const double lm = mvc_log((double)n_ - sg);
      if (which) {
        mvc_vp_ov.ntc[m] = n_;
        mvc_vp_ov.lmc[m] = lm;
      } else {
        mvc_vp_ov.ntp0[m] = n_;
        mvc_vp_ov.lmp0[m] = lm;
      }
    }
    if (which == 0) {
      int tne = *cc.T_ne;
#pragma unroll
      for (int m2 = 0; m2 < kVpMoves; ++m2)
        if (m2 <= m && M.mv[m2]) tne += (M.born[m2] ? 1 : 0) - (M.dies[m2] ? 1 : 0);
      mvc_vp_ov.tne[m] = tne;
    }
  } else if (tid >= 64 && tid < 64 + kVpMoves * kVpV) {   // L_v after move m (the commit's order of updates)
    const int t = tid - 64, m = t / kVpV, v = t - m * kVpV;
    if (v < V) {
      int L = cc.Ltot[v];
#pragma unroll
      for (int m2 = 0; m2 < kVpMoves; ++m2)
        if (m2 <= m && M.mv[m2] && (M.dies[m2] || M.born[m2])) {
          if (M.dies[m2]) --L;
          if (M.born[m2]) ++L;
        }
      mvc_vp_ov.ltot[m * kVpV + v] = L;
    }
  } else if (tid >= 128 && tid < 128 + 2 * kVpE) {   // dish entries (m, v, left | joined) x (coef | self parts)
    const int t = tid - 128, part = t & 1, e = t >> 1, which = e & 1, mvv = e >> 1;
    const int m = mvv / kVpV, v = mvv - m * kVpV;
    const bool act = mvc_vp_ov.mv[m] && v < V;
    const int vs = act ? v : 0;
    const int pm0 = mvc_vp_ov.p0[m], pmc = mvc_vp_ov.c[m];
    const int j0 = cc.dish[vs * ts + pm0], j1 = cc.dish[vs * ts + (act ? pmc : pm0)];
    const int j = which ? j1 : j0;
    // the moves 0 .. m that change this dish's statistics (dish of view v changed, j left or joined)
    int n_ = cc.d_n[vs * ks + j], dl = cc.d_l[vs * ks + j];
    bool touched = false;
    int jl[kVpMoves], jj[kVpMoves], ch[kVpMoves];
#pragma unroll
    for (int m2 = 0; m2 < kVpMoves; ++m2) {
      jl[m2] = cc.dish[vs * ts + M.p0[m2]];
      jj[m2] = M.mv[m2] ? cc.dish[vs * ts + M.c[m2]] : jl[m2];
      ch[m2] = m2 <= m && M.mv[m2] && jl[m2] != jj[m2];
      if (ch[m2]) {
        if (j == jl[m2]) { --n_; touched = true; }
        if (j == jj[m2]) { ++n_; touched = true; }
      }
      if (m2 <= m && M.mv[m2]) {
        if (M.dies[m2] && j == jl[m2]) --dl;
        if (M.born[m2] && j == jj[m2]) ++dl;
      }
    }
    double Q = cc.Q[vs * ks + j], c0 = cc.c0[vs * ks + j], cb = cc.cb[vs * ks + j];
    double xm = cc.xm[vs * ks + j], ym = cc.ym[vs * ks + j], cbm = cc.cbm[vs * ks + j];
    const int eo = (m * kVpV + v) * 2 + which;
    if (act && touched) {   // the commit's refresh of this dish, after moves 0 .. m
      double q = 0.0;
      for (int d = 0; d < D; ++d) {
        double x = cc.S1T[((size_t)vs * D + d) * ks + j];
#pragma unroll
        for (int m2 = 0; m2 < kVpMoves; ++m2)
          if (ch[m2]) {
            if (j == jl[m2]) x = x - yr[m2][vs * D + d];
            if (j == jj[m2]) x = x + yr[m2][vs * D + d];
          }
        q = __builtin_fma(x, x, q);
        if (part == 0) ovs1[(size_t)eo * D + d] = x;
      }
      const double tau = hyp[vs];
      const double a = tau + (double)(part ? n_ - 1 : n_);
      const double b = tau + (double)(part ? n_ : n_ + 1);
      const double Xc = (double)D * ((-0.5 * l2pt[vs]) - 0.5 * mvc_log_nb(b / a));
      const double Yc = (tau * a) * b;
      const double Zc = 1.0 / (tau * b);
      if (part) {
        xm = Xc;
        ym = Yc;
        cbm = Zc;
      } else {
        Q = q;
        c0 = Xc - (0.5 * q) / Yc;
        cb = Zc;
      }
    }
    if (part == 0) {
      mvc_vp_ov.j[eo] = act ? j : -1;
      mvc_vp_ov.s1x[eo] = act && touched;
      mvc_vp_ov.dn[eo] = n_;
      mvc_vp_ov.dl[eo] = dl;
      mvc_vp_ov.Q[eo] = Q;
      mvc_vp_ov.c0[eo] = c0;
      mvc_vp_ov.cb[eo] = cb;
      if (which == 0) mvc_vp_ov.chg[m * kVpV + v] = act && j0 != j1;
    } else {
      mvc_vp_ov.xm[eo] = xm;
      mvc_vp_ov.ym[eo] = ym;
      mvc_vp_ov.cbm[eo] = cbm;
    }
  }
}

// Commit the predicted moves of customers i0 .. i0 + nc - 1 (they held): the
// overlay's values after the last of them into the LDS state and HBM (S1 from
// the overlay's columns: each column the overlay built for a dish with the
// moves before and at its entry applied in move order, the values the moves'
// sequential updates give), S2 updated in move order (one thread per view).
// Block-wide: S1 on every wave, S2 on wave 1, the dish entries on wave 2, the
// tables on wave 3.
__device__ __forceinline__ bool vp_entry_final(int e, int nc, int V, int j) {
  const int mvv = e >> 1, m = mvv / kVpV, v = mvv - m * kVpV;
  if (!(m < nc && v < V && j >= 0)) return false;
  bool fin = !((e & 1) == 0 && mvc_vp_ov.j[e + 1] == j);   // j0 == j1: the joined entry writes
#pragma unroll
  for (int m2 = 0; m2 < kVpMoves; ++m2)
    if (m2 > m && m2 < nc) {
      const int e2 = (m2 * kVpV + v) * 2;
      if (mvc_vp_ov.j[e2] == j || mvc_vp_ov.j[e2 + 1] == j) fin = false;
    }
  return fin;
}
__device__ __forceinline__ void vp_commit(SeqArgs &A, const SCache &cc, const VpMoves &M, int i0, int nc,
                                          const double *const (&yr)[kVpMoves], const double *ovs1, int32_t *cnt,
                                          bool chk) {
  ParState &P = A.P;
  Repair *R = A.R;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int V = P.V, D = P.D, KC = P.KC, ks = cc.ks, ts = cc.ts;
  int last = -1, nmv = 0;
#pragma unroll
  for (int m = 0; m < kVpMoves; ++m)
    if (m < nc && M.mv[m]) {
      last = m;
      ++nmv;
    }
  if (last < 0) return;
  // S1: the final column of every dish a committed move changed, from the
  // overlay entry of the last committed move touching it (threads over (entry, d))
  for (int k = tid; k < kVpE * D; k += nt) {
    const int e = k / D, d = k - e * D;
    const int j = mvc_vp_ov.j[e];
    if (!mvc_vp_ov.s1x[e] || !vp_entry_final(e, nc, V, j)) continue;
    const int v = (e >> 1) % kVpV;
    if (chk && !run_chk(j < cc.Klist[v], 1, i0, e, v, j, cc.Klist[v])) continue;
    const double x = ovs1[(size_t)e * D + d];
    cc.S1T[((size_t)v * D + d) * ks + j] = x;
    gst(&P.S1T[((size_t)v * D + d) * KC + j], x);
  }
  if (tid >= 64 && tid < 64 + V) {
    const int v = tid - 64;
#pragma unroll
    for (int m = 0; m < kVpMoves; ++m)
      if (m < nc && M.mv[m]) {
        const int j0 = cc.dish[v * ts + M.p0[m]], j1 = cc.dish[v * ts + M.c[m]];
        if (chk && !run_chk(j0 >= 0 && j0 < cc.Klist[v] && j1 >= 0 && j1 < cc.Klist[v], 2, i0, m, v, j0, j1,
                            cc.Klist[v]))
          continue;
        if (j0 != j1) {
          const double y2 = yr[m][V * D + v];
          const double a0 = cc.S2[v * ks + j0] - y2, a1 = cc.S2[v * ks + j1] + y2;
          cc.S2[v * ks + j0] = a0;
          cc.S2[v * ks + j1] = a1;
          gst(&P.S2[v * KC + j0], a0);
          gst(&P.S2[v * KC + j1], a1);
        }
      }
    cc.Ltot[v] = mvc_vp_ov.ltot[last * kVpV + v];
    gst(&P.Ltot[v], mvc_vp_ov.ltot[last * kVpV + v]);
  }
  // dish entries whose dish no later committed move touches: their final values
  if (tid >= 128 && tid < 128 + kVpE) {
    const int e = tid - 128, mvv = e >> 1, m = mvv / kVpV, v = mvv - m * kVpV;
    const int j = mvc_vp_ov.j[e];
    if (m < nc && v < V && j >= 0) {
      bool fin = vp_entry_final(e, nc, V, j);
      if (chk && !run_chk(j < cc.Klist[v], 3, i0, e, v, j, cc.Klist[v])) fin = false;
      if (fin) {
        cc.d_n[v * ks + j] = mvc_vp_ov.dn[e];
        cc.d_l[v * ks + j] = mvc_vp_ov.dl[e];
        cc.Q[v * ks + j] = mvc_vp_ov.Q[e];
        cc.c0[v * ks + j] = mvc_vp_ov.c0[e];
        cc.cb[v * ks + j] = mvc_vp_ov.cb[e];
        cc.xm[v * ks + j] = mvc_vp_ov.xm[e];
        cc.ym[v * ks + j] = mvc_vp_ov.ym[e];
        cc.cbm[v * ks + j] = mvc_vp_ov.cbm[e];
        gst(&P.d_n[v * KC + j], mvc_vp_ov.dn[e]);
        gst(&P.d_l[v * KC + j], mvc_vp_ov.dl[e]);
        gst(&P.Q[v * KC + j], mvc_vp_ov.Q[e]);
        gst(&P.c0[v * KC + j], mvc_vp_ov.c0[e]);
        gst(&P.cb[v * KC + j], mvc_vp_ov.cb[e]);
      }
    }
  }
  // the tables (last touch), T_ne, z and the move count (wave 3)
  if (tid >= 192 && tid < 192 + 2 * kVpMoves) {
    const int m = (tid - 192) >> 1, which = tid & 1;
    if (m < nc && mvc_vp_ov.mv[m]) {
      const int p = which ? mvc_vp_ov.c[m] : mvc_vp_ov.p0[m];
      bool fin = true;
#pragma unroll
      for (int m2 = 0; m2 < kVpMoves; ++m2)
        if (m2 > m && m2 < nc && M.mv[m2] && (M.p0[m2] == p || M.c[m2] == p)) fin = false;
      if (chk && !run_chk(p >= 0 && p < *cc.T && i0 + m < A.P.n, 4, i0, m, which, p, *cc.T)) fin = false;
      if (fin) {
        const int n_ = which ? mvc_vp_ov.ntc[m] : mvc_vp_ov.ntp0[m];
        const double lm = which ? mvc_vp_ov.lmc[m] : mvc_vp_ov.lmp0[m];
        cc.n_t[p] = n_;
        cc.lmass[p] = lm;
        gst(&P.n_t[p], n_);
        gst(&P.lmass[p], lm);
      }
      if (which == 0) gst(&P.z[i0 + m], mvc_vp_ov.c[m]);
    }
    if (tid == 192) {
      *cc.T_ne = mvc_vp_ov.tne[last];
      gst(&R->T_ne, mvc_vp_ov.tne[last]);
      cnt[0] += nmv;
    }
  }
}

// The value-prediction loop (L.vp; the lane-column state, V <= kVpV, every
// dish list <= 128): a step builds the overlay of customers i .. i+3's
// predicted moves, evaluates the four customers at once (customer i + w
// against the overlay of the moves before it), keeps the decisions up to and
// including the first that differs from its prediction, commits the held
// predictions from the overlay and a differing move the ordinary way.  Births
// end the loop (mvc_seq_birth_kernel); so does a low hit rate (R->vpoff: the
// lane-column loop takes the rest of the sweep).
__device__ __forceinline__ int seq_run_loop_vp(SeqArgs &A, const SeqLds &L, const Ring &G, RunCursor &U) {
  int flags = 0;
  const ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, n = P.n;
  const SCache cc = lds_cache(V, D, L.ts, L.ks, 1);
  SView Wv = cache_view(cc, A);
  Wv.S1T = cc.S1T;
  Wv.s1s = cc.ks;
  const SeqScratch S(mvc_seq_lds + L.cache_dbl + (int64_t)w * L.stride, V, L.ks, L.ts);
  int cur = U.cur, pend = U.pend, pc = U.pc, pp0 = U.pp0, mode = U.mode, streak = U.streak, done = U.done;
  int fill = U.fill, landed = U.landed, par = 0;
  int lastm = U.lastm, gapq = U.gapq;
  int steps = 0, hits = 0;
  // a move to commit the ordinary way at the top of the next step (customer rci: rp0 -> rc)
  int rci = -1, rp0 = 0, rc = 0;
  bool skip = false;
  if (A.R->vpoff) {   // stopped earlier in this sweep (later rounds of the batch): nothing to do
    flags |= kRunVpOff;
    skip = true;
  } else if (pend && pc < 0) {   // a birth: mvc_seq_birth_kernel
    skip = true;
  } else if (pend) {   // a mover carried over from the previous launch
    ring_fill_async<kSeqLcThreads / 64>(A, G, cur, cur + 1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    fill = landed = cur + 1;
    rci = cur;
    rp0 = pp0;
    rc = pc;
    cur = cur + 1;
    pend = 0;
    streak = 0;
    if (cur >= n) done = 1;
  }
  while (!skip) {
    RUN_T0();
    if (rci >= 0) {   // (its row is in the ring: landed, and requests stop a ring ahead)
      const int nt0 = cc.n_t[rp0], ntc = cc.n_t[rc];
      seq_bar(true);
      seq_commit_move_split(A, cc, G.cust(rci, V, D), rci, rp0, rc, nt0, ntc, U.cnt, L.chk);
      rci = -1;
      seq_bar(true);
      if (L.chk && mvc_run_bad[0]) break;
    }
    if (cur >= n) done = 1;   // (a run launched at cur == n: nothing left to decide)
    if (done || mode != kSeqRun) break;
    {   // the LDS layout must hold the lists plus one birth; the vp evaluation needs K_v <= 128
      bool bad = *cc.T >= L.ts, big = false;
      for (int v = 0; v < V; ++v) {
        bad = bad || cc.Klist[v] >= L.ks;
        big = big || cc.Klist[v] > 128;
      }
      if (bad) {
        flags |= kRunRestride;
        break;
      }
      if (big || (steps >= 128 && 2 * hits < steps)) {
        flags |= kRunVpOff;
        break;
      }
    }
    const int i0 = cur;
    const int need = min(n, i0 + kSeqLcThreads / 64);
    if (L.chk)
      run_chk(i0 >= 0 && i0 < n && fill >= 0 && fill <= n && landed <= fill && (fill < need || need - max(fill, i0) <= G.n),
              10, i0, fill, landed, need, G.n);
    if (need > landed) {
      if (fill < need) {
        ring_fill_async<kSeqLcThreads / 64>(A, G, max(fill, i0), need);
        fill = need;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      landed = fill;
    }
    if (fill - i0 <= G.n / 2 && fill < n) {
      const int f1 = min(n, i0 + G.n);
      ring_fill_async<kSeqLcThreads / 64>(A, G, max(fill, i0), f1);
      fill = f1;
    }
    // the predictions; a predicted birth ends the step's depth (its new table is unknown)
    const int nav = min(kVpMoves, n - i0);
    int pz[kVpMoves], pcs[kVpMoves];
    const double *yr[kVpMoves];
    int depth = nav;
#pragma unroll
    for (int k = 0; k < kVpMoves; ++k) {
      const int ik = min(i0 + k, n - 1);
      pz[k] = ring_z(G, ik, V, D);
      pcs[k] = ring_pred(G, ik, V, D);
      yr[k] = G.at(ik);
      if (k < depth && pcs[k] < 0) depth = k + 1;
      if (L.chk && k < nav)
        run_chk(pz[k] >= 0 && pz[k] < *cc.T && pcs[k] >= -1 && pcs[k] < *cc.T, 8, i0, k, pz[k], pcs[k], *cc.T);
    }
    const VpMoves M = vp_moves(cc, depth, pz, pcs);
    vp_publish(M, pz, pcs);
    seq_bar(true);
    double *const ovs1 = mvc_seq_lds + L.vpo;
    vp_build(A, cc, M, depth, yr, ovs1);
    seq_bar(true);
    RUN_MARK(4);
    if (w < depth) {
      VpCtx X;
      X.nw = w;
      X.tne = *cc.T_ne;
      X.s1 = ovs1;
#pragma unroll
      for (int m = 0; m < kVpMoves; ++m)
        if (m < w && M.mv[m]) X.tne = mvc_vp_ov.tne[m];
      const int c = seq_resample_lc<true>(A, Wv, G.cust(i0 + w, V, D), i0 + w,
                                          mvc_vp_ov.pz[w], S, cc.hyp, cc.cnew, X);
      if (lane == 0) U.chb[par][w] = c;
      if (L.chk && lane == 0) run_chk(c >= -1 && c < *cc.T, 9, i0, w, c, *cc.T);
    }
    seq_bar(true);
    RUN_MARK(5);
    // keep the decisions up to the first that differs from its prediction
    int a = depth;
#pragma unroll
    for (int k = kVpMoves - 1; k >= 0; --k)
      if (k < depth && U.chb[par][k] != pcs[k]) a = k;
    ++steps;
    if (a == depth) ++hits;
    // a held predicted birth is the step's last customer (depth was cut there;
    // depth >= 1 here: cur < n)
    const bool pbirth = a == depth && depth > 0 && mvc_vp_ov.pcs[depth - 1] < 0;
    const int nc = pbirth ? depth - 1 : a;   // customers whose held predictions commit from the overlay
    vp_commit(A, cc, M, i0, nc, yr, ovs1, U.cnt, L.chk);
    int mlast = -1;   // the last mover decided in this step
#pragma unroll
    for (int k = 0; k < kVpMoves; ++k)
      if (k < nc && M.mv[k]) mlast = i0 + k;
    int decided = nc;
    bool stop = false;
    const int kx = pbirth ? depth - 1 : a;   // the customer after the held predictions, if any
    if (kx < depth) {
      const int ck = U.chb[par][kx], zk = mvc_vp_ov.pz[kx];
      decided = kx + 1;
      if (ck != zk) {
        mlast = i0 + kx;
        if (ck < 0) {   // a birth: pending for mvc_seq_birth_kernel
          cur = i0 + kx;
          pend = 1;
          pc = -1;
          pp0 = zk;
          stop = true;
        } else {        // an unpredicted move: the ordinary commit (next step's top), on the state with the held ones
          rci = i0 + kx;
          rp0 = zk;
          rc = ck;
        }
      }
    }
    if (stop) {
      if (mlast >= 0) note_mover(lastm, gapq, mlast);
      break;
    }
    cur = i0 + decided;
    if (mlast >= 0) {
      note_mover(lastm, gapq, mlast);
      streak = cur - 1 - mlast;
    } else {
      streak += decided;
    }
    if (streak >= stay_limit(L.limit, gapq)) mode = kSeqScan;
    if (cur >= n) done = 1;
    par ^= 1;
    seq_bar(true);
    if (L.chk && mvc_run_bad[0]) break;
    RUN_MARK(6);
#ifdef MVC_RUN_PROF
    if (tid == 0) mvc_prof_lds[7] += 1;
#endif
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) {
    U.cur = cur;
    U.pend = pend;
    U.pc = pc;
    U.pp0 = pp0;
    U.mode = mode;
    U.streak = streak;
    U.done = done;
    U.fill = fill;
    U.landed = landed;
    U.lastm = lastm;
    U.gapq = gapq;
    A.R->vpsteps += steps;
    A.R->vphits += hits;
  }
  return flags;
}

// ---- small chains: eight lanes per customer (L.lc == 3) ----
//
// The logs an evaluation shares with every other customer of the step,
// computed once per wave, one per lane, into the wave's LDS row (the same
// expressions, so the same values): k = v < V log(alpha_v + L_v), k = V + v
// log(alpha_v + L_v - 1) (the own table dies), k = 2V / 2V + 1 log(ag + sg
// T_ne) / log(ag + sg (T_ne - 1)), k = 2V + 2 + p log((n_p - 1) - sg) (the
// own table without the customer).  Needs 2V + 2 + T <= 64 (V <= 8, T < 32).
constexpr int kLanePre = 64;   // 2V + 2 + T <= 64 (V <= 8, T < 32)
__shared__ double mvc_lane_pre[kLaneSmallThreads / 64][kLanePre];
struct LanePre {
  const double *pre;   // this wave's row
  __device__ __forceinline__ double at(int k) const { return pre[k]; }
};
// The values, one per lane and half (k = 64 h + lane), computed by the
// evaluation itself (interleaved with its own work), then published into the
// wave's row (lane_pre_publish) before the first read.
struct LanePreVals {
  double x;
};
__device__ __forceinline__ LanePreVals lane_pre_vals(const SView &W, int V, const double *hyp) {
  const int lane = threadIdx.x & 63;
  const double ag = hyp[3 * V], sg = hyp[3 * V + 1];
  const int T = *W.T, T_ne = *W.T_ne;
  LanePreVals P;
  const int k = lane;
  double arg = 1.0;
  if (k < 2 * V) {
    const int v = k < V ? k : k - V;
    arg = hyp[V + v] + (double)(W.Ltot[v] - (k < V ? 0 : 1));
  } else if (k < 2 * V + 2) {
    arg = ag + sg * (double)(T_ne - (k == 2 * V ? 0 : 1));
  } else if (k < 2 * V + 2 + T) {
    arg = (double)(W.n_t[k - 2 * V - 2] - 1) - sg;
  }
  P.x = mvc_log(arg);
  return P;
}
__device__ __forceinline__ LanePre lane_pre_publish(const LanePreVals &P) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double *row = mvc_lane_pre[w];
  row[lane] = P.x;
  wave_lds_sync();
  return LanePre{row};
}

// Lane u of every 8-lane group broadcast to its group (u < 8 compile-time
// after unrolling): DPP row_newbcast of lane u / 8 + u of the 16-lane row.
__device__ __forceinline__ double group8_bcast(double x, int u) {
  const bool hi = (threadIdx.x & 8) != 0;
  switch (u) {
    case 0: return hi ? row_bcast_d<8>(x) : row_bcast_d<0>(x);
    case 1: return hi ? row_bcast_d<9>(x) : row_bcast_d<1>(x);
    case 2: return hi ? row_bcast_d<10>(x) : row_bcast_d<2>(x);
    case 3: return hi ? row_bcast_d<11>(x) : row_bcast_d<3>(x);
    case 4: return hi ? row_bcast_d<12>(x) : row_bcast_d<4>(x);
    case 5: return hi ? row_bcast_d<13>(x) : row_bcast_d<5>(x);
    case 6: return hi ? row_bcast_d<14>(x) : row_bcast_d<6>(x);
    default: return hi ? row_bcast_d<15>(x) : row_bcast_d<7>(x);
  }
}

// seq_resample for one customer on an 8-lane group of a wave, lane v of the
// group owning view v (V <= 8), against the run kernel's LDS state: the same
// decision, bit for bit, as the wave-shaped forms above,
// because every reduction of the spec is either sequential per column or a
// fixed tree that one lane walks itself, or a sum in view order taken over
// the group's lanes in that order:
//   * lane v, view v: the lp of every listed dish (the own dish j0
//     self-removed, lc_self), the max over the included ones and the new
//     dish, K_act; the column partials col_c = sum over j = c mod 16 in
//     ascending j of w_j exp(lp_j - m) (excluded dishes add +0, as a lane
//     column does), pw16 of the columns (pw16_seq: row_pw16's association),
//     the new dish, lm_v; and lp of the dish of every table p < T;
//   * every lane of the group: s_new and the table scores as sums in view
//     order of the lanes' values (broadcast from lane v of the group), the
//     weights exp(sp - M), block sums pw16 per 16 tables, running block
//     totals in block order, the draw: the first block with r < C_b, then
//     pw16_select inside it.  The group's lanes agree; lane 0's is used.
// Every lane of the wave calls it (customers past n with a clamped index):
// the broadcasts read other lanes.
// KB: dishes per view handled as straight-line code (every K_v <= KB: the
// lp values, counts and exps of all of them issued together, the ones past
// K_v masked to the same +0 a skipped dish adds), 0: the general loop over
// blocks of 16.  TR: table registers (T <= TR); positions past TR are the
// compile-time +0 of the last block's padding.
template <int KB, int TR>
__device__ __forceinline__ int seq_resample_lane8(const SeqArgs &A, const SView &W, const Cust &C, int i, int p0,
                                                  const double *hyp, const double *cnewv) {
  static_assert(TR <= 64 && (TR % 16 == 0 || TR < 16), "TR: whole blocks of 16, or part of one");
  static_assert(KB == 0 || KB <= 16, "KB: the straight-line dishes");
  constexpr int NBk = (TR + 15) / 16;
  constexpr int TM = 16 * NBk;
  RUN_T0();
  const int v = threadIdx.x & 7;
  const int V = A.P.V, D = A.P.D, ts = W.ts, ks = W.ks, s1s = W.s1s;
  const bool vok = v < V;
  const int vv = vok ? v : V - 1;
  const double sg = hyp[3 * V + 1];
  const int np0 = W.n_t[p0] - 1;
  const bool alive = np0 > 0;
  const int T = *W.T;
  const double u_i = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z);   // independent of the rest
  const LanePreVals PV = lane_pre_vals(W, V, hyp);                                     // (interleaved with the views)
  // ---- lane v: view v's terms and the lp of every table's dish
  const int K = W.Klist[vv];
  const double tau = hyp[vv], alpha = hyp[V + vv], sigma = hyp[2 * V + vv];
  const double Y2i = C.Y2[vv * (int)C.y2stride];
  const double hy = 0.5 * Y2i;
  const double h = (-0.5 * Y2i) / tau;
  const double lfn = cnewv[vv] + h;
  const int j0 = W.dish[vv * ts + p0];
  const int *dl = W.d_l + vv * ks;
  const int l0p = dl[j0] - (alive ? 0 : 1);
  const double *yv = C.y + vv * (int)C.ystride;
  const double *S1v = W.S1T + (size_t)vv * D * s1s;
  const double *cbv = W.cb + vv * ks, *c0v = W.c0 + vv * ks;
  auto dot = [&](int j) {   // G = y . S1[:, j], one fma chain in ascending d
    if (D == 1) return __builtin_fma(yv[0], S1v[j], 0.0);
    double G = 0.0;
    for (int d = 0; d < D; ++d) G = __builtin_fma(yv[d], S1v[d * s1s + j], G);
    return G;
  };
  const double self = lc_self(W, vv, ks, j0, dot(j0), Y2i, hy, h);
  auto lpj = [&](int j) { return j == j0 ? self : __builtin_fma(dot(j) + hy, cbv[j], c0v[j]) + h; };
  double col[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) col[c] = 0.0;
  double mx = -MVC_PM_INF;
  int cnt = 0;
  double m;
  if constexpr (KB > 0) {
    // every dish of the view at once: lp, max over the included ones, K_act,
    // then the column terms (a dish past K_v: l = 0, its term w exp(-inf) =
    // 0 * 0 = +0, the value col[c] keeps when the general loop skips it)
    double x[KB];
    int l[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int jc = min(u, K - 1);
      x[u] = lpj(jc);
      l[u] = u < K ? (u == j0 ? l0p : dl[jc]) : 0;
    }
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (l[u] > 0) {
        ++cnt;
        if (x[u] > mx) mx = x[u];
      }
    m = lfn > mx ? lfn : mx;
    static_assert(KB % 2 == 0, "dishes in pairs");
#pragma unroll
    for (int u = 0; u < KB; u += 2) {   // two exps interleaved (mvc_exp_le0_x2: the same values)
      double w0 = (double)l[u] - sigma, w1 = (double)l[u + 1] - sigma;
      if (w0 < 0.0) w0 = 0.0;
      if (w1 < 0.0) w1 = 0.0;
      double e0, e1;
      mvc_exp_le0_x2(l[u] > 0 ? x[u] - m : -MVC_PM_INF, l[u + 1] > 0 ? x[u + 1] - m : -MVC_PM_INF, e0, e1);
      col[u] = col[u] + w0 * e0;
      col[u + 1] = col[u + 1] + w1 * e1;
    }
  } else {
    // pass 1: max over the included dishes, K_act; the first 16 lp kept
    double lr[16];
    for (int t0 = 0; t0 < K; t0 += 16) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int j = t0 + c;
        if (j < K) {
          const double x = lpj(j);
          if (t0 == 0) lr[c] = x;
          const int l = j == j0 ? l0p : dl[j];
          if (l > 0) {
            ++cnt;
            if (x > mx) mx = x;
          }
        }
      }
    }
    m = lfn > mx ? lfn : mx;
    // pass 2: column partials in ascending j
    for (int t0 = 0; t0 < K; t0 += 16) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int j = t0 + c;
        if (j < K) {
          const double x = t0 == 0 ? lr[c] : lpj(j);
          const int l = j == j0 ? l0p : dl[j];
          double w = (double)l - sigma;
          if (w < 0.0) w = 0.0;
          col[c] = col[c] + w * mvc_exp_le0(l > 0 ? x - m : -MVC_PM_INF);
        }
      }
    }
  }
  double Sv = pw16_seq(col);
  {
    double wn = alpha + (double)cnt * sigma;
    if (wn < 0.0) wn = 0.0;
    Sv = Sv + wn * mvc_exp_le0(lfn - m);
  }
  const double logS = mvc_log(Sv);
  RUN_MARK(2);
  if constexpr (TR <= 8) {
    // ---- every table in its own lane (T <= 8): lane q of the group forms
    // table q's score from the views' lp of its dish, in view order, with
    // view u's per-customer values (the self-removed value of the own dish,
    // hy, h, the own dish) broadcast from lane u -- the same lpj expression on
    // the same inputs as lane u's, so the same values; then one exp per lane,
    // and the block's 16 leaves (tables 8..15 the padding's +0) broadcast for
    // the spec's pw16 sum and descent
    const int q = v;
    const LanePre LP = lane_pre_publish(PV);
    double lm;
    {
      const double denom = alpha + (double)(W.Ltot[vv] - (alive ? 0 : 1));
      const double logden = LP.at(alive ? vv : V + vv);
      lm = (denom <= 0.0) ? lfn : (m + logS) - logden;
    }
    double s_new = LP.at(alive ? 2 * V : 2 * V + 1);   // log(ag + sg T_ne')
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < V) s_new = s_new + group8_bcast(lm, u);
    const double lmass0 = LP.at(2 * V + 2 + p0);   // log((n_p0 - 1) - sg)
    const int qc = min(q, T - 1);
    double sc = -MVC_PM_INF;
    bool incq = false;   // table q included in the draw (n_q' >= 1, n_q' - sigma_g > 0)
    if (q < T) {
      const int np = W.n_t[q] - (q == p0 ? 1 : 0);
      const double mass = (double)np - sg;
      if (np >= 1 && mass > 0.0) {
        sc = (q == p0) ? lmass0 : W.lmass[q];
        incq = true;
      }
    }
    const double j0d = (double)j0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (u < V) {
        const double self_u = group8_bcast(self, u), hy_u = group8_bcast(hy, u), h_u = group8_bcast(h, u);
        const int j0_u = (int)group8_bcast(j0d, u);
        const int j = W.dish[u * ts + qc];
        double x;
        if (j == j0_u) {
          x = self_u;
        } else {
          const double *yu = C.y + u * (int)C.ystride;
          const double *S1u = W.S1T + (size_t)u * D * s1s;
          double G;
          if (D == 1) {
            G = __builtin_fma(yu[0], S1u[j], 0.0);
          } else {
            G = 0.0;
            for (int d = 0; d < D; ++d) G = __builtin_fma(yu[d], S1u[d * s1s + j], G);
          }
          x = __builtin_fma(G + hy_u, W.cb[u * ks + j], W.c0[u * ks + j]) + h_u;
        }
        if (incq) sc = sc + x;
      }
    }
    RUN_MARK(4);
    double M = row8_max_all(q < T ? sc : -MVC_PM_INF);
    if (s_new > M) M = s_new;
    const double eq = q < T ? mvc_exp_le0(sc - M) : 0.0;   // excluded: exp(-inf) = +0
    double x16[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) x16[k] = group8_bcast(eq, k);
#pragma unroll
    for (int k = 8; k < 16; ++k) x16[k] = 0.0;
    const double tot = 0.0 + pw16_seq(x16);
    const double Wt = mvc_exp_le0(s_new - M) + tot;
    const double r = u_i * Wt;
    if (!(r < tot)) {
      RUN_MARK(5);
      return -1;   // the new table
    }
    const int pick = pw16_select_seq(x16, r);
    RUN_MARK(5);
    return pick;
  }
  double lt[TR];   // lp of table p's dish in this lane's view
#pragma unroll
  for (int p = 0; p < TR; ++p) lt[p] = lpj(W.dish[vv * ts + min(p, T - 1)]);
  const LanePre LP = lane_pre_publish(PV);
  double lm;
  {
    const double denom = alpha + (double)(W.Ltot[vv] - (alive ? 0 : 1));
    const double logden = LP.at(alive ? vv : V + vv);
    lm = (denom <= 0.0) ? lfn : (m + logS) - logden;
  }
  // ---- the group: sums in view order over its lanes (DPP broadcasts from lane u of the group)
  double s_new = LP.at(alive ? 2 * V : 2 * V + 1);   // log(ag + sg T_ne')
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (u < V) s_new = s_new + group8_bcast(lm, u);
  const double lmass0 = LP.at(2 * V + 2 + p0);   // log((n_p0 - 1) - sg)
  double sp[TM];
  uint64_t inc = 0;   // tables included in the draw (n_p' >= 1, n_p' - sigma_g > 0)
#pragma unroll
  for (int p = 0; p < TM; ++p) {
    sp[p] = -MVC_PM_INF;
    if (p < TR && p < T) {
      const int np = W.n_t[p] - (p == p0 ? 1 : 0);
      const double mass = (double)np - sg;
      if (np >= 1 && mass > 0.0) {
        sp[p] = (p == p0) ? lmass0 : W.lmass[p];
        inc |= 1ull << p;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (u < V) {
#pragma unroll
      for (int p = 0; p < TR; ++p) {
        if (TR <= 4 || p < T) {
          const double x = group8_bcast(lt[p], u);
          if ((inc >> p) & 1ull) sp[p] = sp[p] + x;
        }
      }
    }
  }
  RUN_MARK(4);
  double M = -MVC_PM_INF;
#pragma unroll
  for (int p = 0; p < TR; ++p)
    if (p < T && sp[p] > M) M = sp[p];
  if (s_new > M) M = s_new;
  // weights in place (excluded tables and padding: +0), block sums, running block totals C_b
  double tot = 0.0, Cb[NBk];
#pragma unroll
  for (int b = 0; b < NBk; ++b) {
    Cb[b] = 0.0;
    if (16 * b < T) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int p = 16 * b + q;
        sp[p] = (p < TR && p < T) ? mvc_exp_le0(sp[p] - M) : 0.0;   // excluded: exp(-inf) = +0
      }
      tot = tot + pw16_seq(sp + 16 * b);
      Cb[b] = tot;
    }
  }
  const double Wt = mvc_exp_le0(s_new - M) + tot;
  double r = u_i * Wt;
  if (!(r < tot)) {
    RUN_MARK(5);
    return -1;   // the new table
  }
  int bsel = NBk - 1;
#pragma unroll
  for (int b = NBk - 1; b >= 0; --b)
    if (16 * b < T && r < Cb[b]) bsel = b;
  double cprev = 0.0;
#pragma unroll
  for (int b = 1; b < NBk; ++b)
    if (b == bsel) cprev = Cb[b - 1];
  r = r - (bsel > 0 ? cprev : 0.0);
  double x16[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    x16[q] = sp[q];
#pragma unroll
    for (int b = 1; b < NBk; ++b)
      if (b == bsel) x16[q] = sp[16 * b + q];
  }
  const int pick = 16 * bsel + pw16_select_seq(x16, r);
  RUN_MARK(5);
  return pick;
}

// The run kernel's loop for small chains (L.lc == 3): the whole sweep staged
// in the ring (ring >= n), every 8-lane group of the block one customer of
// the next 32, so a step evaluates 32 customers against the current state
// (the first steps are phase A: no separate producer / draw / window
// launches).  The first customer whose choice is not its table is the mover;
// the ones before it are final.  Step = {commit; barrier; evaluate; barrier;
// decide}, the cursor in registers (every wave derives it from the same LDS
// values), the per-wave candidates double-buffered by step parity.  Moves are
// committed by the four waves (seq_commit_move_split); a birth ends the loop
// and seq_run_body commits it on the global state, then resumes here.
// customers per step: 8 lanes each, every lane of the block
template <bool kSmall>
constexpr int lane_cust() { return (kSmall ? kLaneSmallThreads : kSeqLcThreads) / 8; }
// kSmall (mvc_seq_run_kernel<5>, L.small): every dish list and the tables <= 8,
// one straight-line evaluation instance and no birth commit in the kernel
// (a birth ends the launch; mvc_seq_birth_kernel commits it), so the loop's
// registers are the small evaluation's (a larger state exits with restride).
constexpr int kLaneSmall = 8;
template <bool kSmall>
__device__ __forceinline__ int seq_run_loop_lane(SeqArgs &A, const SeqLds &L, const Ring &G, RunCursor &U) {
  constexpr int kW = (kSmall ? kLaneSmallThreads : kSeqLcThreads) / 64;
  constexpr int kLaneCust = lane_cust<kSmall>();
  int flags = 0;
  const ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, n = P.n;
  const SCache cc = lds_cache(V, D, L.ts, L.ks, 1);
  SView Wv = cache_view(cc, A);
  Wv.S1T = cc.S1T;
  Wv.s1s = cc.ks;
  __shared__ int s_mv[2][kW][5];   // per wave: first mover (offset in the step, -1: none), its choice, table, n_t of both
  int cur = U.cur, pend = U.pend, pc = U.pc, pp0 = U.pp0, done = U.done, par = 0;
  int pnt0 = 0, pntc = 0;
  if (pend && pc >= 0) {
    pnt0 = cc.n_t[pp0];
    pntc = cc.n_t[pc];
  }
  if (cur < n) {   // every remaining customer's row (ring >= n: one pass)
    ring_fill_async<kW>(A, G, cur, n);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  {   // the layout holds the lists plus one birth (moves add no table and no dish)
    bool bad = *cc.T >= L.ts || (kSmall && *cc.T > kLaneSmall);
    for (int v = 0; v < V; ++v) bad = bad || cc.Klist[v] >= L.ks || (kSmall && cc.Klist[v] > kLaneSmall);
    if (bad) flags |= kRunRestride;
  }
  for (;;) {
    RUN_T0();
    if (flags & kRunRestride) break;
    if (cur >= n) {
      done = 1;
      break;
    }
    if (pend) {
      if (pc < 0) break;   // a birth: committed by seq_run_body
      seq_commit_move_split(A, cc, G.cust(cur, V, D), cur, pp0, pc, pnt0, pntc, U.cnt, L.chk);
      cur = cur + 1;
      pend = 0;
      if (cur >= n) {
        done = 1;
        break;
      }
      seq_bar(true);
      if (L.chk && mvc_run_bad[0]) break;
    }
    RUN_MARK(3);
    const int q = tid >> 3;            // this group's customer in the step
    const int i = cur + q;
    const int ic = min(i, n - 1);      // (past n: a clamped customer, result unused)
    const int p0 = ring_z(G, ic, V, D);
    RUN_MARK(0);
    const int T = *cc.T;
    int c;
    if constexpr (kSmall) {   // the reference's own call at steady state
      c = seq_resample_lane8<kLaneSmall, kLaneSmall>(A, Wv, G.cust(ic, V, D), ic, p0, cc.hyp, cc.cnew);
    } else {
      int kmx = 0;
      for (int v = 0; v < V; ++v) kmx = max(kmx, cc.Klist[v]);
      if (T <= kLaneSmall && kmx <= kLaneSmall)
        c = seq_resample_lane8<kLaneSmall, kLaneSmall>(A, Wv, G.cust(ic, V, D), ic, p0, cc.hyp, cc.cnew);
      else if (T <= 16)
        c = seq_resample_lane8<0, 16>(A, Wv, G.cust(ic, V, D), ic, p0, cc.hyp, cc.cnew);
      else
        c = seq_resample_lane8<0, 32>(A, Wv, G.cust(ic, V, D), ic, p0, cc.hyp, cc.cnew);
    }
    RUN_MARK(1);
    const bool mv = (lane & 7) == 0 && i < n && c != p0;
    const uint64_t hit = __ballot(mv);
    const int first = hit ? (int)__builtin_ctzll(hit) : 0;
    if (lane == first) {
      int *sm = s_mv[par][w];
      sm[0] = hit ? q : -1;
      sm[1] = c;
      sm[2] = p0;
      if (mv && c >= 0) {
        sm[3] = cc.n_t[p0];
        sm[4] = cc.n_t[c];
      }
    }
    seq_bar(true);
    int f = -1, fw = 0;
#pragma unroll
    for (int k = kW - 1; k >= 0; --k)
      if (s_mv[par][k][0] >= 0) {
        f = s_mv[par][k][0];
        fw = k;
      }
    if (f >= 0) {
      cur = cur + f;
      pend = 1;
      pc = s_mv[par][fw][1];
      pp0 = s_mv[par][fw][2];
      if (pc >= 0) {
        pnt0 = s_mv[par][fw][3];
        pntc = s_mv[par][fw][4];
      }
    } else {
      cur = cur + kLaneCust;
    }
    par ^= 1;
    RUN_MARK(6);
#ifdef MVC_RUN_PROF
    if (tid == 0) mvc_prof_lds[7] += 1;
#endif
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) {
    U.cur = cur;
    U.pend = pend;
    U.pc = pc;
    U.pp0 = pp0;
    U.done = done;
    U.fill = U.landed = n;
  }
  return flags;
}

}  // namespace

// The run kernel (one block of kSeqRunThreads = 8 waves): the
// repair where movers are dense.  It commits the pending mover, then its nws
// waves evaluate the next nws customers against the current state in
// parallel; the first of them that does not stay is the next mover, the
// ones before it are final.  A loop on the device: no launch and no
// grid-wide synchronisation per mover.  The state the evaluations read is an
// LDS copy (SCache, filled at launch, written through by the commits), so a
// customer costs one memory latency (its y rows) plus LDS work.  After
// L.limit stays in a row the movers are sparse: the kernel opens a grid
// window (mvc_seq_eval_kernel) and exits; the next launch resolves it.
// One instance per evaluation shape, compiled separately so each keeps its
// own register allocation.
// kMode 0: one wave per customer; 2: wide (L.tw > 1, global layout); 3: lane columns (L.lc == 1);
// 4: + value prediction (L.lc == 2); 5 / 6: eight lanes per customer, small chains (L.lc == 3;
// 5: small states, L.small)
template <int kMode>
__device__ __forceinline__ void seq_run_body(SeqArgs &A, const SeqLds &L) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x, w = tid >> 6, nt = blockDim.x;
  const int V = P.V, D = P.D, n = P.n, KC = P.KC, TC = P.TC;
  __shared__ RunCursor U;
  if (L.fill >= 0) {   // diagnostics: every LDS byte the launch may read, set to a known pattern first
    const uint32_t pat = 0x01010101u * (uint32_t)L.fill;
    uint32_t *dl = (uint32_t *)mvc_seq_lds;
    for (int64_t k = tid; k < L.dyn / 4; k += nt) dl[k] = pat;
    for (int k = tid; k < (int)(sizeof(mvc_seq_const) / 4); k += nt) ((uint32_t *)mvc_seq_const)[k] = pat;
    for (int k = tid; k < (int)(sizeof(RunCursor) / 4); k += nt) ((uint32_t *)&U)[k] = pat;
    if constexpr (kMode == 4)
      for (int k = tid; k < (int)(sizeof(VpOv) / 4); k += nt) ((uint32_t *)&mvc_vp_ov)[k] = pat;
    __syncthreads();
  }
#ifdef MVC_RUN_PROF
  if (tid < 12) mvc_prof_lds[tid] = 0;
#endif
  if (tid < 8) mvc_run_bad[tid] = 0;   // (MVC_RUN_CHECK; published by the barrier below)
  // The lane-column loops stop at a birth (its dish draws want the block's
  // waves and the global state); the birth is committed here on the global
  // state and the loop resumes at the next customer with its LDS cache
  // re-staged, so a sweep with births is one launch, not one per birth (the
  // mvc_seq_birth_kernel the host launches after this kernel is then a no-op).
  for (;;) {
    if (tid == 0) {
      const int go = !(R->done || R->overflow || R->restride);
      if (go && R->win1 > R->win0) {
        seq_resolve_window(A, R);
        if (R->pend) {
          R->mode = kSeqRun;
          R->streak = 0;
        }
      }
      if (go) R->rounds += 1;
      U.go = go;
      U.cur = R->cur;
      U.pend = R->pend;
      U.pc = R->pchoice;
      U.pp0 = U.pend ? P.z[U.cur] : 0;
      U.mode = R->mode;
      U.streak = R->streak;
      U.done = R->done;
      U.fill = U.cur;   // nothing staged yet
      U.landed = U.cur;
      U.lpc = -1;
      U.cnt[0] = R->moves;
      U.cnt[1] = R->births;
      U.cnt[2] = R->newdish;
      U.lastm = R->lastm;
      U.gapq = R->gapq;
    }
    __syncthreads();
    if (!U.go || !(U.mode == kSeqRun || U.pend)) {
      if (tid == 0 && U.go && !(R->win1 > R->win0)) {   // scan mode: open the next grid window
        if (R->cur >= n && !R->pend) {
          R->done = 1;
        } else {
          R->win0 = R->cur;
          R->win1 = min(n, R->cur + R->W);
          R->fmin = n;
        }
      }
      return;
    }
    int flags = 0;   // kRunOvf | kRunRestride | kRunVpOff
    double *tree = SeqScratch(A, w).tree;   // global per-wave scratch: the dish draws' tree64 levels
    if (L.lds) {   // the state cache, from the global state at launch
      const int ts = L.ts, ks = L.ks;
      const SCache cc = lds_cache(V, D, ts, ks, L.s1);
      // the sweep's hyperparameters and per-view constants (the evaluation and
      // the commits read them from LDS; the MH changes them only after the repair)
      for (int k = tid; k < 3 * V + 2; k += nt) mvc_seq_const[k] = P.hyper[k];
      for (int k = tid; k < V; k += nt) {
        mvc_seq_const[3 * MVC_MAXV + 2 + k] = A.cnew[k];
        mvc_seq_const[4 * MVC_MAXV + 2 + k] = A.L2pt[k];
      }
      const int T = R->T;
      for (int k = tid; k < T; k += nt) {
        cc.n_t[k] = P.n_t[k];
        cc.lmass[k] = P.lmass[k];
      }
      for (int k = tid; k < V * T; k += nt) {
        const int v = k / T, p = k - v * T;
        cc.dish[v * ts + p] = P.dish[v * TC + p];
      }
      for (int k = tid; k < V * ks; k += nt) {
        const int v = k / ks, j = k - v * ks;
        if (j < R->Klist[v]) {
          cc.d_l[k] = P.d_l[v * KC + j];
          cc.d_n[k] = P.d_n[v * KC + j];
          cc.c0[k] = P.c0[v * KC + j];
          cc.cb[k] = P.cb[v * KC + j];
          cc.Q[k] = P.Q[v * KC + j];
          cc.S2[k] = P.S2[v * KC + j];
          self_coef_parts(cc.d_n[k], P.hyper[v], A.L2pt[v], D, cc.xm[k], cc.ym[k], cc.cbm[k]);
        }
      }
      if (L.s1) {
        for (int k = tid; k < V * D * ks; k += nt) {
          const int row = k / ks, j = k - row * ks;
          if (j < R->Klist[row / D]) cc.S1T[k] = P.S1T[(size_t)row * KC + j];
        }
      }
      if (tid < V) {
        cc.Klist[tid] = R->Klist[tid];
        cc.Ltot[tid] = P.Ltot[tid];
      }
      if (tid == 0) {
        *cc.T = R->T;
        *cc.T_ne = R->T_ne;
      }
      __syncthreads();
      Ring G;
      G.n = L.ring;
      G.slot = (int)seq_ring_slot(V, D);
      G.base = mvc_seq_lds + L.cache_dbl + (int64_t)L.nws * L.stride;
      if constexpr (kMode == 3)
        flags = seq_run_loop_lc(A, L, G, U);
      else if constexpr (kMode == 4)
        flags = seq_run_loop_vp(A, L, G, U);
      else if constexpr (kMode == 5)
        flags = seq_run_loop_lane<true>(A, L, G, U);
      else if constexpr (kMode == 6)
        flags = seq_run_loop_lane<false>(A, L, G, U);
      else
        flags = seq_run_loop<true, false>(A, L, cache_view(cc, A), &cc,
                                          SeqScratch(mvc_seq_lds + L.cache_dbl + (int64_t)w * L.stride, V, L.ks, L.ts),
                                          G, tree, U);
      __builtin_amdgcn_s_waitcnt(0);   // no row request outlives the wave
    } else if constexpr (kMode < 3) {   // (the lane-column kernels always have the LDS layout)
      Ring G{nullptr, 0, 0};
      flags = seq_run_loop<false, kMode == 2>(A, L, global_view(A), nullptr, SeqScratch(A, w), G, tree, U);
    }
    if (tid == 0) {   // write the cursor back; open a grid window when handing over
  #ifdef MVC_RUN_PROF
      for (int k = 0; k < 12; ++k) R->prof[k] += mvc_prof_lds[k];
  #endif
      R->cur = U.cur;
      R->pend = U.pend;
      R->pchoice = U.pc;
      R->mode = U.mode;
      R->streak = U.streak;
      R->moves = U.cnt[0];
      R->births = U.cnt[1];
      R->newdish = U.cnt[2];
      R->lastm = U.lastm;
      R->gapq = U.gapq;
      if (L.chk && mvc_run_bad[0])
        for (int k = 0; k < 8; ++k) R->dbg[k] = mvc_run_bad[k];
      if (flags & kRunRestride) R->restride = 1;
      if (flags & kRunVpOff) R->vpoff = 1;
      if (U.done && !U.pend) {
        R->done = 1;
      } else if (!(flags & (kRunOvf | kRunRestride)) && U.mode == kSeqScan && !U.pend) {
        R->win0 = U.cur;
        R->win1 = min(n, U.cur + R->W);
        R->fmin = n;
      }
    }
    if constexpr (kMode >= 3 && kMode != 5) {   // (the small lane loop leaves births to mvc_seq_birth_kernel)
      __shared__ int s_birth, s_bi;
      __syncthreads();
      if (tid == 0) {
        s_birth = !(R->done || R->overflow || R->restride) && R->pend && R->pchoice < 0;
        s_bi = R->cur;
      }
      __syncthreads();
      if (!s_birth) return;
      const SeqScratch Sb(A, w);
      if (!seq_commit_birth_inline(A, s_bi, Sb.lp, Sb.tree, nt >> 6)) return;   // overflow: the host grows and relaunches this step
      if (tid == 0) {
        R->cur = s_bi + 1;
        R->pend = 0;
        R->streak = 0;
        if (R->cur >= n) R->done = 1;   // every customer is final (see mvc_seq_birth_kernel)
      }
      __syncthreads();
    } else {
      return;
    }
  }
}

template <int kMode>
__global__ __launch_bounds__(kMode == 5 ? kLaneSmallThreads : kMode >= 3 ? kSeqLcThreads : kSeqRunThreads) void mvc_seq_run_kernel(
    SeqArgs A, SeqLds L) {
  seq_run_body<kMode>(A, L);
}
// The same for several chains at once (one block per chain, its arguments
// and LDS layout from device arrays): the chain-batched repair of a handle's
// chains, one launch per round instead of one stream and launch per chain.
template <int kMode>
__global__ __launch_bounds__(kMode >= 3 ? kSeqLcThreads : kSeqRunThreads) void mvc_seq_run_kernel_b(const SeqArgs *As,
                                                                                                 const SeqLds *Ls) {
  SeqArgs A = As[blockIdx.x];
  const SeqLds L = Ls[blockIdx.x];
  seq_run_body<kMode>(A, L);
}

// The exact conditional of every customer of the pending window against the
// current state, one wavefront per customer; the first mover by atomicMin.
__device__ __forceinline__ void seq_eval_body(const SeqArgs &A, int gw) {
  Repair *R = A.R;
  const int lane = threadIdx.x & 63;
  if (R->done || R->overflow || R->restride) return;
  const int w0 = R->win0, w1 = R->win1;
  if (w1 <= w0) return;
  const SeqScratch S(A, gw);
  const SView W = global_view(A);
  for (int i = w0 + gw; i < w1; i += A.G) {
    const int f = readlane_i(__hip_atomic_load(&R->fmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0);
    if (i > f) break;   // a mover before i: i is re-evaluated after it
    const int p0 = A.P.z[i];
    const int c = seq_resample(A, W, global_cust(A, i), i, p0, S);
    if (lane == 0) {
      A.choice[i] = c;
      if (c != p0) atomicMin(&R->fmin, i);
    }
  }
}
extern "C" __global__ __launch_bounds__(256) void mvc_seq_eval_kernel(SeqArgs A) {
  seq_eval_body(A, blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}
// Every batched chain's repair state into one array (one read-back per batch).
extern "C" __global__ void mvc_seq_gather_repair_kernel(const SeqArgs *As, Repair *out) {
  const uint32_t *src = (const uint32_t *)As[blockIdx.x].R;
  uint32_t *dst = (uint32_t *)(out + blockIdx.x);
  for (int k = threadIdx.x; k < (int)(sizeof(Repair) / 4); k += blockDim.x) dst[k] = src[k];
}
// Batched: bpc blocks per chain, chain = blockIdx.x / bpc.
extern "C" __global__ __launch_bounds__(256) void mvc_seq_eval_kernel_b(const SeqArgs *As, int bpc) {
  const SeqArgs A = As[blockIdx.x / bpc];
  seq_eval_body(A, (blockIdx.x % bpc) * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

// After the last repair step of a sweep that moved someone: drop dead tables
// (order kept) and dead dishes (l = 0, order kept) in place (oracle
// SeqSampler::compact).  pos_new [TC], jmap [V*KC].
// relabel != 0 (small n): the block also relabels z (mvc_seq_relabel_kernel's
// work, without its launch).
__device__ __forceinline__ void seq_compact_body(SeqArgs &A, int32_t *pos_new, int32_t *jmap, int relabel) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC;
  __shared__ int s_T, s_K[MVC_MAXV];
  if (!(R->done && R->moves > 0)) return;
  const int T = R->T;
  const uint64_t below = (1ull << lane) - 1;   // lanes before this one
  // In-place compactions in chunks of 64 entries per wave: each chunk's
  // entries are read into registers before any of its writes, and an entry
  // only moves down (its new position <= its old one), so no write of a
  // chunk reaches an entry not yet read.  The surviving order is kept.
  // 1. wave 0: the surviving tables' new positions; waves 1..: the dish
  //    lists of the views (order kept), their rows moved down
  if (w == 0) {
    int base = 0;
    for (int p0 = 0; p0 < T; p0 += 64) {
      const int p = p0 + lane;
      const bool alive = p < T && P.n_t[p] > 0;
      const uint64_t m = __ballot(alive);
      if (p < T) pos_new[p] = alive ? base + __builtin_popcountll(m & below) : -1;
      base += __builtin_popcountll(m);
    }
    if (lane == 0) s_T = base;
  } else {
    for (int v = w - 1; v < V; v += nw - 1) {
      const int K = R->Klist[v];
      int base = 0;
      for (int j0 = 0; j0 < K; j0 += 64) {
        const int j = j0 + lane, e = v * KC + j;
        const bool in = j < K;
        const int dl = in ? P.d_l[e] : 0;
        const bool alive = in && dl > 0;
        const int id = alive ? P.d_id[e] : 0, dn = alive ? P.d_n[e] : 0;
        const double s2 = alive ? P.S2[e] : 0.0;
        const uint64_t m = __ballot(alive);
        const int o = base + __builtin_popcountll(m & below);
        __builtin_amdgcn_s_waitcnt(0);   // the chunk read before it is written
        if (in) jmap[e] = alive ? o : -1;
        if (alive) {
          const int eo = v * KC + o;
          P.d_id[eo] = id;
          P.d_n[eo] = dn;
          P.d_l[eo] = dl;
          P.S2[eo] = s2;
        }
        base += __builtin_popcountll(m);
      }
      if (lane == 0) s_K[v] = base;
    }
  }
  __syncthreads();
  // 2. the S1 columns of the surviving dishes, one wave per (view, d) row
  for (int row = w; row < V * D; row += nw) {
    const int v = row / D, K = R->Klist[v];
    double *col = P.S1T + (size_t)row * KC;
    const int32_t *jm = jmap + v * KC;
    for (int j0 = 0; j0 < K; j0 += 64) {
      const int j = j0 + lane;
      const int t = j < K ? jm[j] : -1;
      const double x = t >= 0 ? col[j] : 0.0;
      __builtin_amdgcn_s_waitcnt(0);
      if (t >= 0) col[t] = x;
    }
  }
  // 3. the surviving tables' dishes (view v) and counts (task V)
  for (int task = w; task <= V; task += nw) {
    for (int p0 = 0; p0 < T; p0 += 64) {
      const int p = p0 + lane;
      const int q = p < T ? pos_new[p] : -1;
      int x = 0;
      if (q >= 0) x = task < V ? jmap[task * KC + P.dish[task * TC + p]] : P.n_t[p];
      __builtin_amdgcn_s_waitcnt(0);
      if (q >= 0) {
        if (task < V) P.dish[task * TC + q] = x;
        else P.n_t[q] = x;
      }
    }
  }
  if (relabel)   // pos_new is complete (step 1, before the barrier above)
    for (int i = tid; i < P.n; i += blockDim.x) P.z[i] = pos_new[P.z[i]];
  __syncthreads();
  if (tid == 0) {
    A.status[0] = s_T;
    for (int v = 0; v < V; ++v) {
      A.status[1 + v] = s_K[v];
      P.Kact[v] = s_K[v];
    }
    A.status[V + 3] = s_T;
    int acc = 0;
    A.Koff[0] = 0;
    for (int v = 0; v < V; ++v) {
      acc += s_K[v];
      A.Koff[v + 1] = acc;
    }
  }
}
extern "C" __global__ __launch_bounds__(1024) void mvc_seq_compact_kernel(SeqArgs A, int32_t *pos_new, int32_t *jmap,
                                                                          int relabel) {
  seq_compact_body(A, pos_new, jmap, relabel);
}
// The same for several chains (one block per chain; a chain that did not
// move returns at once): the chain-batched sweep
struct CompactArgs {
  SeqArgs Q;
  int32_t *pos_new, *jmap;
  int32_t relabel;
};
extern "C" __global__ __launch_bounds__(1024) void mvc_seq_compact_kernel_b(const CompactArgs *As) {
  SeqArgs A = As[blockIdx.x].Q;
  seq_compact_body(A, As[blockIdx.x].pos_new, As[blockIdx.x].jmap, As[blockIdx.x].relabel);
}
// Every chain's status row [2V + 4] into out[chain][2V + 4] (one read-back)
extern "C" __global__ void mvc_seq_gather_status_kernel(const CompactArgs *As, int len, int32_t *out) {
  const int32_t *src = As[blockIdx.x].Q.status;
  for (int k = threadIdx.x; k < len; k += blockDim.x) out[(size_t)blockIdx.x * len + k] = src[k];
}

extern "C" __global__ void mvc_seq_relabel_kernel(int n, int32_t *z, const int32_t *pos_new, const Repair *R) {
  if (!(R->done && R->moves > 0)) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) z[i] = pos_new[z[i]];
}
