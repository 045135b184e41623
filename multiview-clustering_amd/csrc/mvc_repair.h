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
  int32_t moves, births, newdish, rounds;
  int32_t Klist[MVC_MAXV];   // dish list length per view (dishes that died this sweep stay, l = 0)
};

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

// per-wave scratch: lp [V][KC] | table scores / weights [TC] | block sums
// [TC/16+1] | running totals [TC/16+1] | dish-draw tree levels
struct SeqScratch {
  double *lp, *e, *B, *C, *tree;
  __device__ SeqScratch(const SeqArgs &A, int wave) {
    double *base = A.scr + (int64_t)wave * A.scr_stride;
    lp = base;
    e = lp + (size_t)A.P.V * A.P.KC;
    B = e + A.P.TC + 16;
    C = B + A.P.TC / 16 + 2;
    tree = C + A.P.TC / 16 + 2;
  }
};
__host__ inline int64_t seq_scratch_stride(int V, int TC, int KC) {
  // tree levels: K+1 leaves, then ceil(./64) ... (< (K+1)/63 + 3 more)
  const int64_t leaves = (int64_t)KC + 1;
  const int64_t tree = leaves + leaves / 63 + 8;
  return (int64_t)V * KC + TC + 16 + 2 * (TC / 16 + 2) + tree + 64;
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
// oracle pw16_select
__device__ __forceinline__ int pw16_select_seq(const double *x, double r) {
  double lv[5][16];
#pragma unroll
  for (int c = 0; c < 16; ++c) lv[0][c] = x[c];
#pragma unroll
  for (int k = 0, h = 1; k < 4; ++k, h <<= 1)
#pragma unroll
    for (int c = 0; c < 16; c += 2 * h) lv[k + 1][c] = lv[k][c] + lv[k][c + h];
  int lo = 0;
  for (int k = 3, h = 8; k >= 0; --k, h >>= 1) {
    const double L = lv[k][lo], R = lv[k][lo + h];
    if (!(R == 0.0 || r < L)) {
      r = r - L;
      lo += h;
    }
  }
  return lo;
}

__device__ __forceinline__ int wave_count(bool p) { return __popcll(__ballot(p)); }

// lp of every listed dish of view v for customer i (the customer's own dish
// j0 with itself removed) into lp[0..K); oracle
// eval_view_seq / eval_view.  Returns the number of included dishes (l' > 0)
// and their max in *mx.
__device__ int seq_view_lp(const SeqArgs &A, int i, int v, bool alive, int j0, double *lp, double *mx_out) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, D = P.D, KC = P.KC, n = P.n;
  const int K = A.R->Klist[v];
  const double tau = P.hyper[v], sigma = P.hyper[2 * V + v];
  (void)sigma;
  const double Y2i = A.Y2[(size_t)v * n + i];
  const double hy = 0.5 * Y2i;
  const double h = (-0.5 * Y2i) / tau;
  const double *yrow = A.y + ((size_t)v * n + i) * D;
  const double *S1v = P.S1T + (size_t)v * D * KC;
  const int l0 = P.d_l[v * KC + j0];
  const int l0p = alive ? l0 : l0 - 1;
  double mx = -MVC_PM_INF;
  int nl = 0;
  for (int base = 0; base < K; base += 64) {
    const int j = base + lane;
    bool inc = false;
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
      inc = l > 0;
      if (inc && val > mx) mx = val;
    }
    nl += wave_count(inc);
  }
  *mx_out = wave_max(mx);
  return nl;
}

// lm_v of oracle eval_view_seq (column partials j mod 16 in ascending j,
// pw16 over the columns, then the new dish); lp[] from seq_view_lp.
__device__ double seq_view_marg(const SeqArgs &A, int i, int v, bool alive, int j0, double *lp) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, KC = P.KC, n = P.n;
  const int K = A.R->Klist[v];
  const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
  double m;
  const int Kact = seq_view_lp(A, i, v, alive, j0, lp, &m);
  __threadfence_block();
  const double Y2i = A.Y2[(size_t)v * n + i];
  const double h = (-0.5 * Y2i) / tau;
  const double lfn = A.cnew[v] + h;
  if (lfn > m) m = lfn;
  const int l0p = alive ? P.d_l[v * KC + j0] : P.d_l[v * KC + j0] - 1;
  double col = 0.0;
  if (lane < 16) {
    for (int j = lane; j < K; j += 16) {
      const int l = (j == j0) ? l0p : P.d_l[v * KC + j];
      if (l > 0) {
        double w = (double)l - sigma;
        if (w < 0.0) w = 0.0;
        col = col + w * mvc_exp(lp[j] - m);
      }
    }
  }
  double cols[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) cols[c] = readlane_d(col, c);
  double S = pw16_seq(cols);
  double wn = alpha + (double)Kact * sigma;
  if (wn < 0.0) wn = 0.0;
  S = S + wn * mvc_exp(lfn - m);
  const double denom = alpha + (double)(P.Ltot[v] - (alive ? 0 : 1));
  if (denom <= 0.0) return lfn;
  return (m + mvc_log(S)) - mvc_log(denom);
}

// Exact conditional draw of customer i against the current state (oracle
// ParallelSampler::resample_customer): a table position, or -1 = birth.
__device__ int seq_resample(const SeqArgs &A, int i, const SeqScratch &S) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, KC = P.KC, TC = P.TC;
  const int p0 = P.z[i];
  const bool alive = (P.n_t[p0] - 1) > 0;
  const double ag = P.hyper[3 * V], sg = P.hyper[3 * V + 1];
  const int Tne_i = A.R->T_ne - (alive ? 0 : 1);
  double s_new = mvc_log(ag + sg * (double)Tne_i);
  for (int v = 0; v < V; ++v)
    s_new = s_new + seq_view_marg(A, i, v, alive, P.dish[v * TC + p0], S.lp + (size_t)v * KC);
  __threadfence_block();
  const int T = A.R->T;
  const int TB = (T + 15) / 16;
  double M = -MVC_PM_INF;
  for (int p = lane; p < TB * 16; p += 64) {
    double sp = -MVC_PM_INF;
    if (p < T) {
      const int np = P.n_t[p] - (p == p0 ? 1 : 0);
      const double mass = (double)np - sg;
      if (np >= 1 && mass > 0.0) {
        sp = mvc_log(mass);
        for (int v = 0; v < V; ++v) sp = sp + S.lp[(size_t)v * KC + P.dish[v * TC + p]];
      }
    }
    S.e[p] = sp;
    if (sp > M) M = sp;
  }
  M = wave_max(M);
  if (s_new > M) M = s_new;
  __threadfence_block();
  for (int p = lane; p < TB * 16; p += 64) {
    const double x = S.e[p];
    S.e[p] = x != -MVC_PM_INF ? mvc_exp(x - M) : 0.0;
  }
  __threadfence_block();
  for (int b = lane; b < TB; b += 64) S.B[b] = pw16_seq(S.e + (size_t)b * 16);
  __threadfence_block();
  int pick = 0;
  if (lane == 0) {
    double tot = 0.0;
    for (int b = 0; b < TB; ++b) {
      tot = tot + S.B[b];
      S.C[b] = tot;
    }
    const double W = mvc_exp(s_new - M) + tot;
    double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_Z) * W;
    if (!(r < tot)) {
      pick = -1;
    } else {
      int b = 0;
      while (!(r < S.C[b])) ++b;
      r = r - (b > 0 ? S.C[b - 1] : 0.0);
      pick = b * 16 + pw16_select_seq(S.e + (size_t)b * 16, r);
    }
  }
  return readlane_i(pick, 0);
}

// tree64 over x[0..m) (oracle Tree64::build): level arrays stored one after
// the other from `lv`; returns the root.  nlev receives the number of levels
// (leaves included), off[] their offsets.
__device__ double seq_tree_build(double *lv, int m, int *off, int &nlev) {
  const int lane = threadIdx.x & 63;
  int o = 0, cnt = m;
  nlev = 0;
  off[nlev++] = 0;
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
    off[nlev++] = o;
  } while (cnt > 1);
  return root;
}
// oracle Tree64::select
__device__ int seq_tree_select(const double *lv, int m, const int *off, int nlev, double r) {
  const int lane = threadIdx.x & 63;
  int idx = 0;
  for (int k = nlev - 2; k >= 0; --k) {
    int cnt = m;
    for (int q = 0; q < k; ++q) cnt = (cnt + 63) / 64;
    const int base = idx * 64;
    const int c = min(64, cnt - base);
    const double x = lane < c ? lv[off[k] + base + lane] : 0.0;
    Tree64Levels L;
    wave_tree_sum_levels(x, L);
    const int l = wave_tree_select(L, x, r);
    idx = base + l;
  }
  return idx;
}

// Dish of a birth in view v (oracle SeqSampler::draw_dish): leaves w_j
// exp(lp_j - m) of the included dishes, the new dish last; tree64; r = u S.
// Returns a list index; Klist[v] = a new dish.
__device__ int seq_dish_draw(const SeqArgs &A, int i, int v, bool alive, int j0, const SeqScratch &S) {
  const ParState &P = A.P;
  const int lane = threadIdx.x & 63;
  const int V = P.V, KC = P.KC, n = P.n;
  const int K = A.R->Klist[v];
  const double tau = P.hyper[v], alpha = P.hyper[V + v], sigma = P.hyper[2 * V + v];
  double *lp = S.lp + (size_t)v * KC;
  double m;
  const int Kact = seq_view_lp(A, i, v, alive, j0, lp, &m);
  __threadfence_block();
  const double Y2i = A.Y2[(size_t)v * n + i];
  const double lfn = A.cnew[v] + (-0.5 * Y2i) / tau;
  if (lfn > m) m = lfn;
  double wn = alpha + (double)Kact * sigma;
  if (wn < 0.0) wn = 0.0;
  const int l0p = alive ? P.d_l[v * KC + j0] : P.d_l[v * KC + j0] - 1;
  for (int e = lane; e <= K; e += 64) {
    double leaf = 0.0;
    if (e < K) {
      const int l = (e == j0) ? l0p : P.d_l[v * KC + e];
      if (l > 0) {
        double w = (double)l - sigma;
        if (w < 0.0) w = 0.0;
        leaf = w * mvc_exp(lp[e] - m);
      }
    } else {
      leaf = wn * mvc_exp(lfn - m);
    }
    S.tree[e] = leaf;
  }
  __threadfence_block();
  int off[8], nlev;
  const double tot = seq_tree_build(S.tree, K + 1, off, nlev);
  if (!(tot > 0.0)) return K;
  const double r = mvc_uniform(A.seed, (uint32_t)i, A.sweep, A.chain, MVC_TAG_DISH + 1u + (uint32_t)v) * tot;
  return seq_tree_select(S.tree, K + 1, off, nlev, r);
}

}  // namespace

// Before phase A: the whole sweep is one pending window [0, n).
extern "C" __global__ void mvc_seq_init_kernel(SeqArgs A) {
  if (threadIdx.x != 0) return;
  Repair *R = A.R;
  const int V = A.P.V, n = A.P.n;
  R->cur = 0;
  R->pend = 0;
  R->win0 = 0;
  R->win1 = n;
  R->fmin = n;
  R->W = A.Wmin;
  R->done = 0;
  R->overflow = 0;
  R->T = A.status[0];
  R->T_ne = A.status[V + 3];
  R->moves = R->births = R->newdish = R->rounds = 0;
  for (int v = 0; v < V; ++v) R->Klist[v] = A.P.Kact[v];
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

// One repair step (one block of 256 = 4 waves).
extern "C" __global__ __launch_bounds__(256) void mvc_seq_apply_kernel(SeqArgs A) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC, n = P.n;
  __shared__ int s_go, s_ovf, s_i, s_p0, s_c, s_dies, s_born;
  __shared__ int s_tup[MVC_MAXV], s_j0[MVC_MAXV], s_j1[MVC_MAXV];
  if (tid == 0) {
    const int go = !(R->done || R->overflow);
    if (go && R->win1 > R->win0) {
      const int f = R->fmin;
      if (f < R->win1) {
        R->cur = f;
        R->pend = 1;
        R->W = A.Wmin;
      } else {
        R->cur = R->win1;
        R->W = min(2 * R->W, A.Wmax);
      }
      R->win0 = R->win1 = 0;
      R->fmin = n;
    }
    if (go) R->rounds += 1;
    s_go = go && R->pend;
    s_ovf = 0;
    if (s_go) {
      s_i = R->cur;
      s_p0 = P.z[s_i];
      s_c = A.choice[s_i];
    }
  }
  __syncthreads();
  if (s_go) {
    const int i = s_i, p0 = s_p0;
    int c = s_c;
    if (c < 0) {
      // a birth: dishes drawn against the current state, then the table
      const bool alive = (P.n_t[p0] - 1) > 0;
      const SeqScratch S(A, w);
      for (int v = w; v < V; v += 4) {
        const int t = seq_dish_draw(A, i, v, alive, P.dish[v * TC + p0], S);
        if (lane == 0) s_tup[v] = t;
      }
      __syncthreads();
      if (tid == 0) {
        int ovf = (R->T + 1 > TC) ? 1 : 0;
        for (int v = 0; v < V; ++v)
          if (s_tup[v] == R->Klist[v] && R->Klist[v] + 1 > KC) ovf |= 2;
        if (ovf) R->overflow = ovf;
        s_ovf = ovf;
      }
      __syncthreads();
      if (s_ovf) return;   // nothing changed: the host grows and relaunches this step
      for (int v = 0; v < V; ++v) {
        if (s_tup[v] != R->Klist[v]) continue;   // uniform (shared + global reads after the barrier)
        const int j = R->Klist[v];
        for (int d = tid; d < D; d += blockDim.x) P.S1T[((size_t)v * D + d) * KC + j] = 0.0;
      }
      __syncthreads();
      if (tid == 0) {
        for (int v = 0; v < V; ++v) {
          if (s_tup[v] == R->Klist[v]) {
            const int j = R->Klist[v];
            P.d_id[v * KC + j] = P.next_id[v]++;
            P.d_n[v * KC + j] = 0;
            P.d_l[v * KC + j] = 0;
            P.S2[v * KC + j] = 0.0;
            P.Q[v * KC + j] = 0.0;
            R->Klist[v] = j + 1;
            R->newdish += 1;
          }
        }
        const int p1 = R->T;
        R->T = p1 + 1;
        P.n_t[p1] = 0;
        for (int v = 0; v < V; ++v) P.dish[v * TC + p1] = s_tup[v];
        R->births += 1;
        s_c = p1;
      }
      __syncthreads();
      c = s_c;
    }
    // move i: p0 -> c (oracle SeqSampler::move)
    if (tid == 0) {
      P.n_t[p0] -= 1;
      s_dies = P.n_t[p0] == 0;
      s_born = P.n_t[c] == 0;
      if (s_dies) {
        R->T_ne -= 1;
        for (int v = 0; v < V; ++v) { P.d_l[v * KC + P.dish[v * TC + p0]] -= 1; P.Ltot[v] -= 1; }
      }
      if (s_born) {
        R->T_ne += 1;
        for (int v = 0; v < V; ++v) { P.d_l[v * KC + P.dish[v * TC + c]] += 1; P.Ltot[v] += 1; }
      }
      P.n_t[c] += 1;
      for (int v = 0; v < V; ++v) {
        s_j0[v] = P.dish[v * TC + p0];
        s_j1[v] = P.dish[v * TC + c];
      }
      P.z[i] = c;
    }
    __syncthreads();
    for (int e = tid; e < V * D; e += blockDim.x) {
      const int v = e / D, d = e - v * D;
      const int j0 = s_j0[v], j1 = s_j1[v];
      if (j0 == j1) continue;
      const double yd = A.y[((size_t)v * n + i) * D + d];
      double *col = P.S1T + ((size_t)v * D + d) * KC;
      col[j0] = col[j0] - yd;
      col[j1] = col[j1] + yd;
    }
    if (tid < V) {
      const int v = tid, j0 = s_j0[v], j1 = s_j1[v];
      if (j0 != j1) {
        const double y2 = A.Y2[(size_t)v * n + i];
        P.S2[v * KC + j0] = P.S2[v * KC + j0] - y2;
        P.S2[v * KC + j1] = P.S2[v * KC + j1] + y2;
        P.d_n[v * KC + j0] -= 1;
        P.d_n[v * KC + j1] += 1;
      }
    }
    __syncthreads();
    if (tid < 2 * V) {   // Q and the coefficients of the two dishes (oracle refresh_dish)
      const int v = tid >> 1, j = (tid & 1) ? s_j1[v] : s_j0[v];
      if (s_j0[v] != s_j1[v]) {
        const double *col = P.S1T + (size_t)v * D * KC + j;
        double q = 0.0;
        for (int d = 0; d < D; ++d) q = __builtin_fma(col[(size_t)d * KC], col[(size_t)d * KC], q);
        P.Q[v * KC + j] = q;
        const Coef cf = coef(P.d_n[v * KC + j], q, P.hyper[v], A.L2pt[v], D);
        P.c0[v * KC + j] = cf.c0;
        P.cb[v * KC + j] = cf.cb;
      }
    }
    if (tid == 0) {
      R->cur = i + 1;
      R->pend = 0;
      R->moves += 1;
    }
    __syncthreads();
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

// The exact conditional of every customer of the pending window against the
// current state, one wavefront per customer; the first mover by atomicMin.
extern "C" __global__ __launch_bounds__(256) void mvc_seq_eval_kernel(SeqArgs A) {
  Repair *R = A.R;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (R->done || R->overflow) return;
  const int w0 = R->win0, w1 = R->win1;
  if (w1 <= w0) return;
  const SeqScratch S(A, gw);
  for (int i = w0 + gw; i < w1; i += A.G) {
    const int f = readlane_i(__hip_atomic_load(&R->fmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), 0);
    if (i > f) break;   // a mover before i: i is re-evaluated after it
    const int c = seq_resample(A, i, S);
    if (lane == 0) {
      A.choice[i] = c;
      if (c != A.P.z[i]) atomicMin(&R->fmin, i);
    }
  }
}

// After the last repair step of a sweep that moved someone: drop dead tables
// (order kept) and dead dishes (l = 0, order kept) in place (oracle
// SeqSampler::compact).  pos_new [TC], jmap [V*KC].
extern "C" __global__ __launch_bounds__(1024) void mvc_seq_compact_kernel(SeqArgs A, int32_t *pos_new, int32_t *jmap) {
  Repair *R = A.R;
  ParState &P = A.P;
  const int tid = threadIdx.x;
  const int V = P.V, D = P.D, KC = P.KC, TC = P.TC;
  __shared__ int s_T, s_K[MVC_MAXV];
  if (!(R->done && R->moves > 0)) return;
  const int T = R->T;
  if (tid == 0) {
    int Tn = 0;
    for (int p = 0; p < T; ++p) pos_new[p] = P.n_t[p] > 0 ? Tn++ : -1;
    s_T = Tn;
  } else if (tid <= V) {
    const int v = tid - 1, K = R->Klist[v];
    int Kn = 0;
    for (int j = 0; j < K; ++j) {
      const int e = v * KC + j;
      if (P.d_l[e] > 0) {
        jmap[e] = Kn;
        const int o = v * KC + Kn;
        P.d_id[o] = P.d_id[e];
        P.d_n[o] = P.d_n[e];
        P.d_l[o] = P.d_l[e];
        P.S2[o] = P.S2[e];
        ++Kn;
      } else {
        jmap[e] = -1;
      }
    }
    s_K[v] = Kn;
  }
  __syncthreads();
  for (int row = tid; row < V * D; row += blockDim.x) {
    const int v = row / D, K = R->Klist[v];
    double *col = P.S1T + (size_t)row * KC;
    const int32_t *jm = jmap + v * KC;
    for (int j = 0; j < K; ++j)
      if (jm[j] >= 0) col[jm[j]] = col[j];
  }
  if (tid < V) {
    const int v = tid;
    for (int p = 0; p < T; ++p)
      if (pos_new[p] >= 0) P.dish[v * TC + pos_new[p]] = jmap[v * KC + P.dish[v * TC + p]];
  } else if (tid == V) {
    for (int p = 0; p < T; ++p)
      if (pos_new[p] >= 0) P.n_t[pos_new[p]] = P.n_t[p];
  }
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

extern "C" __global__ void mvc_seq_relabel_kernel(int n, int32_t *z, const int32_t *pos_new, const Repair *R) {
  if (!(R->done && R->moves > 0)) return;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) z[i] = pos_new[z[i]];
}
