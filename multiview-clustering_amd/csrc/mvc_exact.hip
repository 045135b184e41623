// mvc_exact.hip — the reference's sequential Gibbs schedule on gfx950.
//
// One 64-lane workgroup (one wavefront) owns one chain and walks the
// customer loop of multiview_gibbs.cpp:157-200 in order; lanes parallelise
// each step over tables (positions), live dishes and views.  Every fp64
// operation is the reference's, in the reference's order, with the portable
// exp/log of include/mvc_pmath.h, so the chain is bit-identical to the
// PortableMath ExactSampler of oracle/mvc_oracle.cpp for the same Philox seed.
//
// Many chains run side by side (grid = chains); this is where the GPU's
// throughput comes from: the schedule itself is a dependent chain of n
// small steps.
//
// Compile with -ffp-contract=off (Makefile).
#include "mvc_internal.h"

namespace {

// Byte offsets of a chain's arrays in its allocation (carve), 16-byte
// granules.
struct ExactLayout {
  size_t z, n_t, pos, slot, fre, dish, d_id, d_n, d_l, S1, S2, f, logf, P, mh, ldt, Kact, next_id, hyper, total;
};
__host__ __device__ inline ExactLayout exact_layout(int n, int V, int TC, int KC) {
  ExactLayout L{};
  size_t o = 0;
  auto take = [&](size_t x) { const size_t r = o; o += (x + 15) & ~(size_t)15; return r; };
  L.z = take(4 * (size_t)n);
  L.n_t = take(4 * (size_t)TC);
  L.pos = take(4 * (size_t)TC);
  L.slot = take(4 * (size_t)TC);
  L.fre = take(4 * (size_t)TC);
  L.dish = take(4 * (size_t)V * TC);
  L.d_id = take(4 * (size_t)V * KC);
  L.d_n = take(4 * (size_t)V * KC);
  L.d_l = take(4 * (size_t)V * KC);
  L.S1 = take(8 * (size_t)V * KC);
  L.S2 = take(8 * (size_t)V * KC);
  L.f = take(8 * (size_t)V * KC);
  L.logf = take(8 * (size_t)V * KC);
  L.P = take(8 * (size_t)TC);
  L.mh = take(8 * (size_t)(n + 1));
  L.ldt = take(8 * (size_t)V * (n + 2));
  L.Kact = take(4 * (size_t)V);
  L.next_id = take(4 * (size_t)V);
  L.hyper = take(8 * (size_t)(3 * V + 2));
  L.total = o;
  return L;
}
// the chain's pointers over its allocation `base` in layout L
__host__ __device__ inline void exact_point(ExactChain &C, char *base, const ExactLayout &L) {
  C.z = (int32_t *)(base + L.z);
  C.n_t = (int32_t *)(base + L.n_t);
  C.pos_of_slot = (int32_t *)(base + L.pos);
  C.slot_at_pos = (int32_t *)(base + L.slot);
  C.free_slots = (int32_t *)(base + L.fre);
  C.dish = (int32_t *)(base + L.dish);
  C.d_id = (int32_t *)(base + L.d_id);
  C.d_n = (int32_t *)(base + L.d_n);
  C.d_l = (int32_t *)(base + L.d_l);
  C.d_S1 = (double *)(base + L.S1);
  C.d_S2 = (double *)(base + L.S2);
  C.f = (double *)(base + L.f);
  C.logf = (double *)(base + L.logf);
  C.P = (double *)(base + L.P);
  C.mhbuf = (double *)(base + L.mh);
  C.ldt = (double *)(base + L.ldt);
  C.Kact = (int32_t *)(base + L.Kact);
  C.next_id = (int32_t *)(base + L.next_id);
  C.hyper = (double *)(base + L.hyper);
}

// multiview_utils.cpp:307-338 compute_f_vk, literal expression order.  The
// two log-determinant terms, -0.5 m log(2 pi tau) - 0.5 log(tau (tau + m)),
// depend on the view and the count m only and are the same until the MH moves
// tau, so they come from the sweep's table ref_log_det (ld[m], m = 0 .. n + 1).
__device__ __forceinline__ double ref_log_det(int m, double tau, double l2pt) {
  return -0.5 * m * l2pt - 0.5 * mvc_log(tau * (tau + m));
}
__device__ __forceinline__ double ref_f_vk(int nk, double S1, double S2, double tau, double yvi, const double *ld) {
  const double term1_old = -0.5 * S2 / tau;
  const double term2_old = 0.5 * (S1 * S1) / (tau * (tau + nk));
  const double log_det_old = ld[nk];
  const int n_new = nk + 1;
  const double S1_new = S1 + yvi;
  const double S2_new = S2 + yvi * yvi;
  const double term1_new = -0.5 * S2_new / tau;
  const double term2_new = 0.5 * (S1_new * S1_new) / (tau * (tau + n_new));
  const double log_det_new = ld[n_new];
  const double lp = (log_det_new + term1_new + term2_new) - (log_det_old + term1_old + term2_old);
  return mvc_exp(lp);
}

// multiview_utils.cpp:340-350 compute_f_vk_new (l2pt as in ref_f_vk)
__device__ __forceinline__ double ref_f_new(double tau, double yvi, double l2pt) {
  const double log_norm = -0.5 * l2pt;
  const double log_exp = -0.5 * (yvi * yvi) / tau;
  return mvc_exp(log_norm + log_exp);
}

constexpr double kEps = 1e-6;   // multiview_hyper.cpp:13

// the wave's per-view values, sized for at most MV views (kernel instance
// MV = 8 for the reference's few views: 1.5 KB instead of 6 KB of LDS per
// chain, i.e. more chains resident per CU)
template <int MV>
struct Shared {
  int Kact[MV];
  int next_id[MV];
  int Koff[MV + 1];
  int died[MV];
  int draw_ix[MV];
  double hyp[3 * MV + 2];
  double ys[MV];
  double fnew[MV];
  double l2pt[MV];   // mvc_log(2 pi tau_v) of the current sweep
  double marg[MV];   // log of the view's new-table marginal
  double tw[MV];
  double buf[MVC_WAVE];
  double dv[4];
  int iv[8];
  long long prof[8];   // MVC_EXACT_PROF: shader clocks per phase (ExactSave.prof)
};

// ---------------------------------------------------------------------------
// Sequential left-to-right sums and inverse-CDF searches in the reference's
// order (so the same bits), with the terms loaded 8 at a time: a batch's
// loads are in flight together instead of one dependent round trip per term.
// ---------------------------------------------------------------------------
template <class F>
__device__ __forceinline__ double seq_sum8(double s, int n, F term) {
  int j = 0;
  for (; j + 8 <= n; j += 8) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = term(j + q);
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q];
  }
  for (; j < n; ++j) s += term(j);
  return s;
}
// the first j whose running sum exceeds u, -1 if none
template <class F>
__device__ __forceinline__ int seq_find8(double u, int n, F term) {
  double cum = 0.0;
  int j = 0;
  for (; j + 8 <= n; j += 8) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = term(j + q);
    int hit = 8;   // the batch's first crossing by selects: one branch per batch
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      cum += x[q];
      hit = (hit == 8 && u < cum) ? q : hit;
    }
    if (hit < 8) return j + hit;
  }
  for (; j < n; ++j) {
    cum += term(j);
    if (u < cum) return j;
  }
  return -1;
}

// ---------------------------------------------------------------------------
// hyperparameter MH (multiview_hyper.cpp:211-292), executed by the wave.
// Sums are accumulated in the reference's order by lane 0; lanes only
// produce the addends.
// ---------------------------------------------------------------------------
template <class Sh>
struct MH {
  ExactChain &C;
  Sh &sh;
  int V, n, lane;
  uint64_t seed;

  __device__ double unif() {   // lane 0 only
    return mvc_seq_uniform(seed, (uint32_t)C.chain_id, C.draws++);
  }
  __device__ double rnorm(double mu, double sd) {  // lane 0 only
    const double u1 = unif();
    const double u2 = unif();
    return mu + sd * mvc_norm_from_uniforms(u1, u2);
  }
  __device__ double bcast(double x) {
    if (lane == 0) sh.dv[0] = x;
    __syncthreads();
    const double r = sh.dv[0];
    __syncthreads();
    return r;
  }
  static __device__ double prior_alpha(double a) {
    if (a <= 0.0) return -MVC_PM_INF;
    return (4.0 - 1.0) * mvc_log(a) - 3.0 * a;
  }
  static __device__ double prior_sigma(double s) {
    if (s <= 0.0 || s >= 1.0) return -MVC_PM_INF;
    return (1.0 - 1.0) * mvc_log(s) + (5.0 - 1.0) * mvc_log(1.0 - s);
  }
  // hyper.cpp:176-209 (all lanes call; result valid on all lanes)
  __device__ double post_tau(int v, double tau) {
    if (tau <= 0.0) return -MVC_PM_INF;
    const int K = sh.Kact[v];
    const int KC = C.KC;
    double ll = 0.0;
    for (int base = 0; base < K; base += MVC_WAVE) {
      const int j = base + lane;
      double term = 0.0;
      if (j < K) {
        const int nk = C.d_n[v * KC + j];
        if (nk != 0) {
          const double sy = C.d_S1[v * KC + j], sy2 = C.d_S2[v * KC + j];
          double sse = sy2 - (sy * sy) / (double)nk;
          if (sse < 0.0) sse = 0.0;
          term = -0.5 * nk * mvc_log(2.0 * MVC_PI * tau) - 0.5 * (sse / tau);
        }
      }
      sh.buf[lane] = term;
      __syncthreads();
      if (lane == 0) {
        const int cnt = min(MVC_WAVE, K - base);
        for (int q = 0; q < cnt; ++q)
          if (C.d_n[v * KC + base + q] != 0) ll += sh.buf[q];
      }
      __syncthreads();
    }
    ll = bcast(ll);
    const double prior = 2.0 * mvc_log(1.0) - 0.0 - (2.0 + 1.0) * mvc_log(tau) - 1.0 / tau;
    return ll + prior;
  }
  // hyper.cpp:295-342 log_EPPF over live dishes of view v
  __device__ double eppf_view(int v, double alpha, double sigma) {
    if (!(sigma > kEps && sigma < 1.0 - kEps)) return -MVC_PM_INF;
    if (alpha <= -sigma) return -MVC_PM_INF;
    const int K = sh.Kact[v];
    const int KC = C.KC;
    int total = 0;
    for (int j = 0; j < K; ++j) total += C.d_l[v * KC + j];   // uniform loop
    if (total == 0) return 0.0;
    double lp = 0.0;
    int bad = 0;
    // sum_j log(alpha + j*sigma), j < K_active
    for (int base = 0; base < K; base += MVC_WAVE) {
      const int j = base + lane;
      double t = 0.0;
      if (j < K) { const double term = alpha + j * sigma; if (term <= 0.0) bad = 1; t = mvc_log(term); }
      sh.buf[lane] = t;
      __syncthreads();
      if (lane == 0) { const int c = min(MVC_WAVE, K - base); for (int q = 0; q < c; ++q) lp += sh.buf[q]; }
      __syncthreads();
    }
    // - sum_{i=1}^{total-1} log(alpha + i)
    for (int base = 1; base < total; base += MVC_WAVE) {
      const int i = base + lane;
      double t = 0.0;
      if (i < total) { const double term = alpha + i; if (term <= 0.0) bad = 1; t = mvc_log(term); }
      sh.buf[lane] = t;
      __syncthreads();
      if (lane == 0) { const int c = min(MVC_WAVE, total - base); for (int q = 0; q < c; ++q) lp -= sh.buf[q]; }
      __syncthreads();
    }
    // + sum_k sum_{m=1}^{l_k-1} log(m - sigma), k ascending
    int maxl = 0;
    for (int j = 0; j < K; ++j) maxl = max(maxl, C.d_l[v * KC + j]);
    for (int m = 1 + lane; m < maxl; m += MVC_WAVE) {
      const double term = (double)m - sigma;
      if (term <= 0.0) bad = 1;
      C.mhbuf[m] = mvc_log(term);
    }
    __syncthreads();
    if (lane == 0)   // the same additions in the same order, 8 loads in flight
      for (int j = 0; j < K; ++j) lp = seq_sum8(lp, C.d_l[v * KC + j] - 1, [&](int m) { return C.mhbuf[1 + m]; });
    __syncthreads();
    bad = __any(bad);
    lp = bcast(lp);
    return bad ? -MVC_PM_INF : lp;
  }
  // hyper.cpp:53-83 log_global_EPPF
  __device__ double eppf_global(double alpha, double sigma) {
    if (!(sigma > kEps && sigma < 1.0 - kEps)) return -MVC_PM_INF;
    if (alpha <= -sigma) return -MVC_PM_INF;
    const int T = C.T;
    if (T <= 0) return 0.0;
    double lp = 0.0;
    int bad = 0;
    for (int base = 0; base < T; base += MVC_WAVE) {
      const int j = base + lane;
      double t = 0.0;
      if (j < T) { const double term = alpha + j * sigma; if (term <= 0.0) bad = 1; t = mvc_log(term); }
      sh.buf[lane] = t;
      __syncthreads();
      if (lane == 0) { const int c = min(MVC_WAVE, T - base); for (int q = 0; q < c; ++q) lp += sh.buf[q]; }
      __syncthreads();
    }
    for (int base = 1; base < n; base += MVC_WAVE) {
      const int i = base + lane;
      double t = 0.0;
      if (i < n) { const double term = alpha + i; if (term <= 0.0) bad = 1; t = mvc_log(term); }
      sh.buf[lane] = t;
      __syncthreads();
      if (lane == 0) { const int c = min(MVC_WAVE, n - base); for (int q = 0; q < c; ++q) lp -= sh.buf[q]; }
      __syncthreads();
    }
    int maxc = 0;
    for (int p = lane; p < T; p += MVC_WAVE) maxc = max(maxc, C.n_t[C.slot_at_pos[p]]);
    for (int m = 32; m >= 1; m >>= 1) maxc = max(maxc, __shfl_xor(maxc, m, 64));
    for (int m = 1 + lane; m < maxc; m += MVC_WAVE) {
      const double term = (double)m - sigma;
      if (term <= 0.0) bad = 1;
      C.mhbuf[m] = mvc_log(term);
    }
    __syncthreads();
    if (lane == 0)
      for (int p = 0; p < T; ++p)   // n_t in position order (hyper.cpp:74)
        lp = seq_sum8(lp, C.n_t[C.slot_at_pos[p]] - 1, [&](int m) { return C.mhbuf[1 + m]; });
    __syncthreads();
    bad = __any(bad);
    lp = bcast(lp);
    return bad ? -MVC_PM_INF : lp;
  }
  static __device__ double reflect_unit(double value) {   // hyper.cpp:110-122
    double p = value;
    while (p <= kEps || p >= 1.0 - kEps) {
      if (p <= kEps) p = 2.0 * kEps - p;
      if (p >= 1.0 - kEps) p = 2.0 * (1.0 - kEps) - p;
    }
    return p < kEps ? kEps : (p > 1.0 - kEps ? 1.0 - kEps : p);
  }
  __device__ double propose_alpha(double a_old) {   // hyper.cpp:100-108, lane 0
    double la = mvc_log(a_old > kEps ? a_old : kEps);
    la += rnorm(0.0, 0.1);
    const double c = mvc_exp(la);
    return (c > kEps) ? c : kEps;
  }
  // hyper.cpp:233-292 update_hyperparameters
  __device__ void run() {
    double *tau = sh.hyp, *alpha = sh.hyp + V, *sigma = sh.hyp + 2 * V;
    double &ag = sh.hyp[3 * V], &sg = sh.hyp[3 * V + 1];
    for (int v = 0; v < V; ++v) {                                    // :211-231
      double t_old = tau[v];
      if (t_old <= 0.0) t_old = kEps;
      const double l_old = post_tau(v, t_old);
      double t_prop = 0.0;
      if (lane == 0) t_prop = mvc_exp(mvc_log(t_old) + rnorm(0.0, 0.3));
      t_prop = bcast(t_prop);
      if (t_prop <= 0.0) continue;
      const double l_new = post_tau(v, t_prop);
      const double lq = mvc_log(t_prop) - mvc_log(t_old);
      const double acc = (l_new - l_old) + lq;
      if (lane == 0 && mvc_log(unif()) < acc) tau[v] = t_prop;
      __syncthreads();
    }
    for (int v = 0; v < V; ++v) {
      double a_old = alpha[v];
      if (a_old <= 0.0) a_old = kEps;
      double a_prop = 0.0;
      if (lane == 0) a_prop = propose_alpha(a_old);
      a_prop = bcast(a_prop);
      const double lo = (a_old <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_old, sigma[v]) + prior_alpha(a_old);
      const double ln = (a_prop <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_prop, sigma[v]) + prior_alpha(a_prop);
      const double lq = mvc_log(a_prop) - mvc_log(a_old);
      if (lane == 0 && mvc_log(unif()) < (ln - lo) + lq) alpha[v] = a_prop;
      __syncthreads();
      const double s_old = sigma[v];
      double s_prop = 0.0, u = 0.0;
      if (lane == 0) { s_prop = reflect_unit(s_old + rnorm(0.0, 0.05)); u = unif(); }
      s_prop = bcast(s_prop);
      const double av = alpha[v];
      const double pn = (s_prop <= kEps || s_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(v, av, s_prop) + prior_sigma(s_prop);
      const double po = (s_old <= kEps || s_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_view(v, av, s_old) + prior_sigma(s_old);
      if (lane == 0 && mvc_log(u) < pn - po) sigma[v] = s_prop;
      __syncthreads();
    }
    double ag_old = ag;
    if (ag_old <= 0.0) ag_old = kEps;
    double ag_prop = 0.0;
    if (lane == 0) ag_prop = propose_alpha(ag_old);
    ag_prop = bcast(ag_prop);
    const double sg0 = sg;
    const double lo = eppf_global(ag_old, sg0) + prior_alpha(ag_old);
    const double ln = eppf_global(ag_prop, sg0) + prior_alpha(ag_prop);
    const double lq = mvc_log(ag_prop) - mvc_log(ag_old);
    if (lane == 0 && mvc_log(unif()) < (ln - lo) + lq) ag = ag_prop;
    __syncthreads();
    const double sg_old = sg;
    double sg_prop = 0.0, u = 0.0;
    if (lane == 0) { sg_prop = reflect_unit(sg_old + rnorm(0.0, 0.05)); u = unif(); }
    sg_prop = bcast(sg_prop);
    const double a_g = ag;
    const double pn = (sg_prop <= kEps || sg_prop >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_prop) + prior_sigma(sg_prop);
    const double po = (sg_old <= kEps || sg_old >= 1.0 - kEps) ? -MVC_PM_INF : eppf_global(a_g, sg_old) + prior_sigma(sg_old);
    if (lane == 0 && mvc_log(u) < pn - po) sg = sg_prop;
    __syncthreads();
  }
};

}  // namespace

// In-kernel sample output (mvc_run with the exact schedule): the kernel
// writes each saved sweep's state (save_state, utils.cpp:291-303) into the
// chain's slot of a device buffer as it finishes the sweep, so a launch can run
// many sweeps even when every sweep is saved.  Chain c's sample s lives at
// slot c * nslot + s; s = (g - first) / thin for global sweep g.
struct ExactSave {
  int32_t *z;          // [C][nslot][n] table_of (nullptr: no saving)
  int32_t *dish;       // [C][nslot][V][dcap] raw dish ids, positions < T
  int32_t *T;          // [C][nslot]
  double *hyp;         // [C][nslot][3V+2]
  int32_t dcap, nslot, ktot, thin;
  int64_t sweep_base, burn, first;   // global index of the launch's first sweep, burn-in, first saved sweep
  long long *prof;     // MVC_EXACT_PROF=1: [C][8] shader clocks per phase of the customer step (else nullptr)
};
// table_of[i] = position of i's table; dish_of[v][p] = raw dish id (the
// snapshot kernels' layout), by one wavefront
__device__ __forceinline__ void exact_snapshot_wave(const ExactChain &C, int n, int V, int T, const double *hyp, int lane,
                                                    int32_t *tz, int32_t *dd, int dcap) {
  (void)hyp;
  for (int i = lane; i < n; i += MVC_WAVE) tz[i] = C.pos_of_slot[C.z[i]];
  for (int v = 0; v < V; ++v)
    for (int p = lane; p < T && p < dcap; p += MVC_WAVE)
      dd[v * dcap + p] = C.d_id[v * C.KC + C.dish[v * C.TC + C.slot_at_pos[p]]];
}

// ---------------------------------------------------------------------------
// One sweep (or the rest of one) for every chain: grid = chains, block = 64.
// The chain's capacity-sized arrays (n_t .. P, and z when it fits) are one
// contiguous range of its allocation (carve); when the range fits in the
// lds_bytes of dynamic LDS it is copied in at the start, the kernel works on
// the copy (every dependent access an LDS round trip instead of an L2 one)
// and it is written back at the end.  Same operations, same order: the bits
// do not depend on where the arrays live.
// ---------------------------------------------------------------------------
// kMode (per launch, from the largest chain): 2 = every array n_t .. P and z
// in LDS, 1 = z in global memory, 0 = all in global memory.  The pointers are
// rebuilt from the LDS symbol (or from y, for global ones) inside the
// instance, so the compiler emits ds_* (or global_*) instructions instead of
// flat ones that wait on both counters.
template <class T>
__device__ __forceinline__ T *ex_global(const double *base, T *p) {
  return (T *)((const char *)base + ((const char *)p - (const char *)base));
}

// The customer step's barriers.  The workgroup is one wavefront, so a barrier
// only has to order memory: with the chain's arrays in LDS (kMode >= 1; z, if
// global, is read at step i and written at its commit only) an LDS-only fence
// suffices, which leaves global loads (the next customer's y, the log-det
// table) in flight across it; kMode 0 keeps __syncthreads.
template <int kMode>
__device__ __forceinline__ void ex_sync() {
  if constexpr (kMode >= 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  } else {
    __syncthreads();
  }
}

template <int kMode, int MV>
__global__ __launch_bounds__(64) void mvc_exact_sweep_kernel(
    const double *__restrict__ y, int n, int V, ExactChain *chains, uint64_t seed, ExactSave SV) {
  __shared__ Shared<MV> sh;
  extern __shared__ __attribute__((aligned(16))) char ex_lds[];
  ExactChain &Cg = chains[blockIdx.x];
  ExactChain C = Cg;               // pointers + scalars in registers
  const int lane = threadIdx.x;
  if (C.status == MVC_ST_ERROR || C.todo <= 0) return;
  const int TC = C.TC, KC = C.KC;
  char *gbeg = nullptr;
  size_t nbytes = 0;
  C.mhbuf = ex_global(y, C.mhbuf);
  C.ldt = ex_global(y, C.ldt);
  if constexpr (kMode == 0) {
    C.z = ex_global(y, C.z); C.n_t = ex_global(y, C.n_t); C.pos_of_slot = ex_global(y, C.pos_of_slot);
    C.slot_at_pos = ex_global(y, C.slot_at_pos); C.free_slots = ex_global(y, C.free_slots);
    C.dish = ex_global(y, C.dish); C.d_id = ex_global(y, C.d_id); C.d_n = ex_global(y, C.d_n);
    C.d_l = ex_global(y, C.d_l); C.d_S1 = ex_global(y, C.d_S1); C.d_S2 = ex_global(y, C.d_S2);
    C.f = ex_global(y, C.f); C.logf = ex_global(y, C.logf); C.P = ex_global(y, C.P);
  } else {
    gbeg = kMode == 2 ? (char *)C.z : (char *)C.n_t;
    nbytes = (size_t)((char *)C.mhbuf - gbeg);
    const uint4 *src = (const uint4 *)gbeg;   // 16-byte granules (carve)
    uint4 *dst = (uint4 *)ex_lds;
    for (size_t e = lane; e < nbytes / 16; e += MVC_WAVE) dst[e] = src[e];
    auto re = [&](auto *&ptr) { ptr = (std::remove_reference_t<decltype(ptr)>)(ex_lds + ((char *)ptr - gbeg)); };
    if constexpr (kMode == 2) re(C.z);
    else C.z = ex_global(y, C.z);
    re(C.n_t); re(C.pos_of_slot); re(C.slot_at_pos); re(C.free_slots); re(C.dish);
    re(C.d_id); re(C.d_n); re(C.d_l); re(C.d_S1); re(C.d_S2); re(C.f); re(C.logf); re(C.P);
  }

  for (int v = lane; v < V; v += MVC_WAVE) {
    sh.Kact[v] = C.Kact[v];
    sh.next_id[v] = C.next_id[v];
  }
  for (int q = lane; q < 3 * V + 2; q += MVC_WAVE) sh.hyp[q] = C.hyper[q];
  if (lane < 8) sh.prof[lane] = 0;
  __syncthreads();
  // phase clocks (diagnostic, off unless SV.prof): 0 remove, 1 f_vk, 2 marginals +
  // table probabilities, 3 normaliser, 4 normalise + find, 5 join a table,
  // 6 open a table, 7 MH + sample output
  const bool prof = SV.prof != nullptr;
  long long tp = prof ? clock64() : 0;
  auto tick = [&](int k) {
    if (prof) {
      const long long t = clock64();
      if (lane == 0) sh.prof[k] += t - tp;
      tp = t;
    }
  };

  int T = C.T;
  int n_free = C.n_free;
  const double *tau = sh.hyp, *alpha = sh.hyp + V, *sigma = sh.hyp + 2 * V;
  int status = MVC_ST_RUNNING;
  int i = C.resume_i;
  int todo = C.todo;

  for (; todo > 0; --todo, i = 0) {   // the launch's sweeps, each from customer resume_i / 0
    const double ag = sh.hyp[3 * V], sg = sh.hyp[3 * V + 1];   // the MH of the previous sweep may have moved them
    if (lane < V) sh.l2pt[lane] = mvc_log(2.0 * MVC_PI * tau[lane]);
    __syncthreads();
    for (int v = 0; v < V; ++v)   // the sweep's log-determinant table (ref_f_vk)
      for (int m = lane; m < n + 2; m += MVC_WAVE) C.ldt[(size_t)v * (n + 2) + m] = ref_log_det(m, tau[v], sh.l2pt[v]);
    __syncthreads();
    double ynx = lane < V ? y[(size_t)lane * n + i] : 0.0;
    bool koff_dirty = true;   // uniform: Koff must be rebuilt (sweep start, a dish died or was opened)
    for (; i < n; ++i) {
      // -------- capacity guard (every step may add 1 table and 1 dish/view)
      int need = (T + 1 > TC || n_free < 1) ? 1 : 0;
      for (int v = 0; v < V; ++v) need |= (sh.Kact[v] + 1 > KC) ? 1 : 0;
      if (need) { status = MVC_ST_OVERFLOW; break; }
      // the table draw's uniform (gibbs.cpp:185): its counter is the step's
      // first draw, so it is formed here, beside the step's LDS waits
      const double u_tab = mvc_seq_uniform(seed, (uint32_t)C.chain_id, C.draws);

      if (lane < V) sh.ys[lane] = ynx;
      if (lane < V && i + 1 < n) ynx = y[(size_t)lane * n + i + 1];   // the next customer's y, in flight during this step
      // ---------------- remove_customer(i)   utils.cpp:138-192
      const int s = C.z[i];
      ex_sync<kMode>();
      if (lane < V) {
        const int k = C.dish[lane * TC + s];
        const double yv = sh.ys[lane];
        C.d_n[lane * KC + k] -= 1;
        C.d_S1[lane * KC + k] -= yv;
        C.d_S2[lane * KC + k] -= yv * yv;
      }
      int nt_s = C.n_t[s] - 1;
      ex_sync<kMode>();
      if (lane == 0) C.n_t[s] = nt_s;
      if (nt_s == 0) {
        // table dies: l_vk-- (:170-173), swap-and-pop (:175-190)
        if (lane < V) {
          const int k = C.dish[lane * TC + s];
          int dead = -1;
          if (k >= 0) {
            const int l = C.d_l[lane * KC + k];
            if (l > 0) {
              C.d_l[lane * KC + k] = l - 1;
              if (l - 1 == 0) dead = k;
            }
          }
          sh.died[lane] = dead;
        }
        const int pos = C.pos_of_slot[s];
        const int last = T - 1;
        ex_sync<kMode>();
        if (lane == 0) {
          if (pos != last) {
            const int sl = C.slot_at_pos[last];
            C.slot_at_pos[pos] = sl;
            C.pos_of_slot[sl] = pos;
          }
          C.free_slots[n_free] = s;
        }
        T -= 1;
        n_free += 1;
        ex_sync<kMode>();
        // compact the live dish list of every view whose dish died
        for (int v = 0; v < V; ++v) {
          const int k = sh.died[v];
          if (k < 0) continue;
          const int K = sh.Kact[v];
          // shift entries k+1..K-1 down by one (read all, barrier, write)
          for (int base = k + 1; base < K; base += MVC_WAVE) {
            const int j = base + lane;
            int id = 0, nn = 0, ll = 0;
            double s1 = 0.0, s2 = 0.0;
            if (j < K) {
              id = C.d_id[v * KC + j]; nn = C.d_n[v * KC + j]; ll = C.d_l[v * KC + j];
              s1 = C.d_S1[v * KC + j]; s2 = C.d_S2[v * KC + j];
            }
            ex_sync<kMode>();
            if (j < K) {
              C.d_id[v * KC + j - 1] = id; C.d_n[v * KC + j - 1] = nn; C.d_l[v * KC + j - 1] = ll;
              C.d_S1[v * KC + j - 1] = s1; C.d_S2[v * KC + j - 1] = s2;
            }
            ex_sync<kMode>();
          }
          for (int p = lane; p < T; p += MVC_WAVE) {
            const int sl = C.slot_at_pos[p];
            const int dk = C.dish[v * TC + sl];
            if (dk > k) C.dish[v * TC + sl] = dk - 1;
          }
          ex_sync<kMode>();
          if (lane == 0) sh.Kact[v] = K - 1;
          koff_dirty = true;
          ex_sync<kMode>();
        }
      }

      tick(0);
      // ---------------- f_vk and log f_vk for every live dish (utils.cpp:83-108)
      if (koff_dirty) {   // the views' offsets in the dish list, after a dish count changed
        if (lane == 0) {
          int acc = 0;
          for (int v = 0; v < V; ++v) { sh.Koff[v] = acc; acc += sh.Kact[v]; }
          sh.Koff[V] = acc;
        }
        ex_sync<kMode>();
        koff_dirty = false;
      }
      const int Ktot = sh.Koff[V];
      for (int e = lane; e < Ktot; e += MVC_WAVE) {
        int v = 0;   // the view of entry e: how many view offsets 1 .. V-1 lie at or below it
        for (int k = 1; k < V; ++k) v += (e >= sh.Koff[k]) ? 1 : 0;
        const int j = e - sh.Koff[v];
        const double f = ref_f_vk(C.d_n[v * KC + j], C.d_S1[v * KC + j], C.d_S2[v * KC + j], tau[v], sh.ys[v],
                                  C.ldt + (size_t)v * (n + 2));
        C.f[v * KC + j] = f;
        C.logf[v * KC + j] = mvc_log(f);
      }
      if (lane < V) sh.fnew[lane] = ref_f_new(tau[lane], sh.ys[lane], sh.l2pt[lane]);
      ex_sync<kMode>();
      tick(1);

      // ---------------- marginal of a new table per view (utils.cpp:40-69)
      if (lane < V) {
        const int v = lane;
        const int K = sh.Kact[v];
        const double total = seq_sum8(0.0, K, [&](int j) { return (double)C.d_l[v * KC + j]; });
        const double denom = alpha[v] + total;
        double m;
        if (denom <= 0.0) {
          m = sh.fnew[v];
        } else {
          double acc = seq_sum8(0.0, K, [&](int j) {
            double w = (C.d_l[v * KC + j] - sigma[v]);
            if (w < 0.0) w = 0.0;
            return w * C.f[v * KC + j];
          });
          double wn = (alpha[v] + K * sigma[v]);
          if (wn < 0.0) wn = 0.0;
          acc += wn * sh.fnew[v];
          m = acc / denom;
        }
        sh.marg[v] = mvc_log(m);   // the normaliser's log term, one view per lane
      }

      // ---------------- table probabilities (utils.cpp:83-116)
      int tne = 0;
      for (int p = lane; p < T; p += MVC_WAVE) {
        const int sl = C.slot_at_pos[p];
        const int nt = C.n_t[sl];
        double pr = 0.0;
        if (nt != 0) {
          ++tne;
          double lpt = 0.0;
          for (int v0 = 0; v0 < V; v0 += 8) {   // 8 views' dish indices, then their log f, in flight together
            int kq[8];
            double g[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) kq[q] = (v0 + q < V) ? C.dish[(v0 + q) * TC + sl] : 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) g[q] = (v0 + q < V) ? C.logf[(v0 + q) * KC + kq[q]] : 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (v0 + q < V) lpt += g[q];
          }
          const double mass = nt - sg;
          pr = (mass <= 0.0) ? 0.0 : mass * mvc_exp(lpt);
        }
        C.P[p] = pr;
      }
      for (int m = 32; m >= 1; m >>= 1) tne += __shfl_xor(tne, m, 64);
      ex_sync<kMode>();
      tick(2);

      // ---------------- normaliser, draw (gibbs.cpp:169-191)
      if (lane == 0) {
        double lnew = 0.0;
        for (int v = 0; v < V; ++v) lnew += sh.marg[v];      // utils.cpp:118-122 (logs taken per view above)
        const double mass_new = ag + sg * tne;                          // :124-135
        const double p_new = (mass_new <= 0.0) ? 0.0 : mass_new * mvc_exp(lnew);
        sh.dv[1] = seq_sum8(p_new, T, [&](int p) { return C.P[p]; });
      }
      ex_sync<kMode>();
      tick(3);
      const double sum_p = sh.dv[1];
      int t_star;
      if (sum_p <= 0.0) {
        t_star = -2;                       // gibbs.cpp:172-176 -> table at position 0
      } else {
        for (int p = lane; p < T; p += MVC_WAVE) C.P[p] = C.P[p] / sum_p;
        ex_sync<kMode>();
        if (lane == 0) {
          const double u = u_tab;
          sh.iv[0] = seq_find8(u, T, [&](int p) { return C.P[p]; });
        }
        C.draws += 1;
        ex_sync<kMode>();
        t_star = sh.iv[0];
      }
      tick(4);

      if (t_star != -1) {
        // add_customer_to_existing_table (utils.cpp:194-207)
        const int sl = C.slot_at_pos[t_star < 0 ? 0 : t_star];
        ex_sync<kMode>();
        if (lane == 0) { C.z[i] = sl; C.n_t[sl] = C.n_t[sl] + 1; }
        if (lane < V) {
          const int k = C.dish[lane * TC + sl];
          const double yv = sh.ys[lane];
          C.d_n[lane * KC + k] += 1;
          C.d_S1[lane * KC + k] += yv;
          C.d_S2[lane * KC + k] += yv * yv;
        }
        ex_sync<kMode>();
        tick(5);
      } else {
        // create_empty_table + add_customer_to_new_table (utils.cpp:209-222)
        koff_dirty = true;   // a view may open a dish
        n_free -= 1;
        const int sl = C.free_slots[n_free];
        const int pos = T;
        ex_sync<kMode>();
        if (lane == 0) {
          C.slot_at_pos[pos] = sl;
          C.pos_of_slot[sl] = pos;
          C.n_t[sl] = 1;
          C.z[i] = sl;
        }
        T += 1;
        // assign_dishes_new_table (utils.cpp:278-289): per view weights
        if (lane < V) {
          const int v = lane;
          const int K = sh.Kact[v];
          double total = seq_sum8(0.0, K, [&](int j) {
            double w = (C.d_l[v * KC + j] - sigma[v]) * C.f[v * KC + j];
            if (w < 0) w = 0;
            return w;
          });
          double wn = (alpha[v] + sigma[v] * K) * sh.fnew[v];
          if (wn < 0) wn = 0;
          total += wn;
          sh.tw[v] = total;
        }
        ex_sync<kMode>();
        if (lane == 0) {                       // draws are consumed in view order
          uint64_t d = C.draws;
          for (int v = 0; v < V; ++v) sh.draw_ix[v] = (sh.tw[v] <= 0) ? -1 : (int)(d++ - C.draws);
          sh.iv[1] = (int)(d - C.draws);
        }
        ex_sync<kMode>();
        if (lane < V) {
          const int v = lane;
          const int K = sh.Kact[v];
          int kk = -1;
          const double total = sh.tw[v];
          if (total > 0) {
            const double u = 0.0 + (total - 0.0) * mvc_seq_uniform(seed, (uint32_t)C.chain_id, C.draws + (uint64_t)sh.draw_ix[v]);
            kk = seq_find8(u, K, [&](int j) {
              double w = (C.d_l[v * KC + j] - sigma[v]) * C.f[v * KC + j];
              if (w < 0) w = 0;
              return w;
            });
          }
          if (kk < 0) {                        // fresh dish slot (utils.cpp:250-258,268-275)
            kk = K;
            C.d_id[v * KC + kk] = sh.next_id[v];
            C.d_n[v * KC + kk] = 0;
            C.d_l[v * KC + kk] = 0;
            C.d_S1[v * KC + kk] = 0.0;
            C.d_S2[v * KC + kk] = 0.0;
            sh.next_id[v] += 1;
            sh.Kact[v] = K + 1;
          }
          const double yv = sh.ys[v];
          C.dish[v * TC + sl] = kk;
          C.d_l[v * KC + kk] += 1;
          C.d_n[v * KC + kk] += 1;
          C.d_S1[v * KC + kk] += yv;
          C.d_S2[v * KC + kk] += yv * yv;
        }
        C.draws += (uint64_t)sh.iv[1];
        ex_sync<kMode>();
        tick(6);
      }
    }

    if (status != MVC_ST_RUNNING) break;
    // end of sweep: hyperparameters (gibbs.cpp:202)
    C.T = T;
    MH<Shared<MV>> mh{C, sh, V, n, lane, seed};
    mh.run();
    // the MH draws on lane 0 only: every lane continues from lane 0's counter
    // (the next sweep's dish draws run on lanes 0 .. V-1)
    C.draws = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(C.draws >> 32)) << 32) |
              (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)C.draws);
    if (SV.z) {   // a saved sweep (gibbs.cpp:205-206): save_state into this chain's sample slot
      const int64_t g = SV.sweep_base + (SV.ktot - todo);
      if (g >= SV.burn && (g - SV.burn) % SV.thin == 0) {
        const size_t slot = (size_t)blockIdx.x * SV.nslot + (size_t)((g - SV.first) / SV.thin);
        __syncthreads();
        exact_snapshot_wave(C, n, V, T, sh.hyp, lane, SV.z + slot * n, SV.dish + slot * V * SV.dcap, SV.dcap);
        if (lane == 0) SV.T[slot] = T;
        for (int q = lane; q < 3 * V + 2; q += MVC_WAVE) SV.hyp[slot * (3 * V + 2) + q] = sh.hyp[q];
      }
    }
    tick(7);
  }
  if (status == MVC_ST_RUNNING) status = MVC_ST_DONE;
  __syncthreads();
  if (prof && lane < 8) SV.prof[(size_t)blockIdx.x * 8 + lane] += sh.prof[lane];
  for (int v = lane; v < V; v += MVC_WAVE) {
    C.Kact[v] = sh.Kact[v];
    C.next_id[v] = sh.next_id[v];
  }
  for (int q = lane; q < 3 * V + 2; q += MVC_WAVE) C.hyper[q] = sh.hyp[q];
  if (lane == 0) {
    Cg.T = T;
    Cg.n_free = n_free;
    Cg.draws = C.draws;
    Cg.resume_i = i;
    Cg.status = status;
    Cg.todo = todo;
  }
  if constexpr (kMode != 0) {      // the LDS copy back to the chain's allocation
    __syncthreads();
    const uint4 *src = (const uint4 *)ex_lds;
    uint4 *dst = (uint4 *)gbeg;
    for (size_t e = lane; e < nbytes / 16; e += MVC_WAVE) dst[e] = src[e];
  }
}

// Snapshot of one chain in reference output form (utils.cpp:291-303):
// table_of[i] = position of i's table; dish_of[v][p] = raw dish id.
extern "C" __global__ void mvc_exact_snapshot_kernel(int n, int V, const ExactChain *chains, int chain,
                                                     int32_t *table_of, int32_t *dish_of, int dish_cap) {
  const ExactChain &C = chains[chain];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  for (int i = tid; i < n; i += stride) table_of[i] = C.pos_of_slot[C.z[i]];
  const int T = C.T;
  for (int e = tid; e < V * T; e += stride) {
    const int v = e / T, p = e % T;
    if (p < dish_cap) dish_of[v * dish_cap + p] = C.d_id[v * C.KC + C.dish[v * C.TC + C.slot_at_pos[p]]];
  }
}

// Snapshot of every chain at once (mvc_run's saved samples): chain c =
// blockIdx.y writes table_of[c][n], dish_of[c][V][dcap] (positions < T), T[c]
// and hyper[c][3V+2] into one save slot, read back asynchronously.
extern "C" __global__ void mvc_exact_snapshot_all_kernel(int n, int V, const ExactChain *chains, int dcap,
                                                         int32_t *table_of, int32_t *dish_of, int32_t *T_out,
                                                         double *hyper) {
  const int c = blockIdx.y;
  const ExactChain &C = chains[c];
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  int32_t *tz = table_of + (size_t)c * n;
  for (int i = tid; i < n; i += stride) tz[i] = C.pos_of_slot[C.z[i]];
  const int T = C.T;
  int32_t *dd = dish_of + (size_t)c * V * dcap;
  for (int e = tid; e < V * T; e += stride) {
    const int v = e / T, p = e % T;
    if (p < dcap) dd[v * dcap + p] = C.d_id[v * C.KC + C.dish[v * C.TC + C.slot_at_pos[p]]];
  }
  if (tid == 0) T_out[c] = T;
  for (int e = tid; e < 3 * V + 2; e += stride) hyper[(size_t)c * (3 * V + 2) + e] = C.hyper[e];
}

// ===========================================================================
// Host side of the exact schedule.
// ===========================================================================
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>

#include "mvc_host.h"

namespace mvc {

namespace {

// Device allocation of one chain at capacities (TC, KC); host mirror of the
// struct keeps the device pointers.
struct ExactAlloc {
  ExactChain h{};          // host copy of the device struct
  void *block = nullptr;   // single device allocation
};

size_t exact_bytes(int n, int V, int TC, int KC) { return exact_layout(n, V, TC, KC).total; }

void carve(ExactAlloc &A, int n, int V, int TC, int KC) {
  ExactChain &C = A.h;
  C.TC = TC;
  C.KC = KC;
  exact_point(C, (char *)A.block, exact_layout(n, V, TC, KC));
}

// Host-side image of a chain's state (used for init and capacity growth).
struct ExactImage {
  int TC, KC, T, n_free;
  std::vector<int32_t> z, n_t, pos_of_slot, slot_at_pos, free_slots, dish;
  std::vector<int32_t> d_id, d_n, d_l, Kact, next_id;
  std::vector<double> d_S1, d_S2, hyper;
};

void upload(ExactAlloc &A, const ExactImage &I, int n, int V, hipStream_t st) {
  ExactChain &C = A.h;
  auto cp = [&](void *dst, const void *src, size_t bytes) {
    MVC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
  };
  cp(C.z, I.z.data(), sizeof(int32_t) * n);
  cp(C.n_t, I.n_t.data(), sizeof(int32_t) * I.TC);
  cp(C.pos_of_slot, I.pos_of_slot.data(), sizeof(int32_t) * I.TC);
  cp(C.slot_at_pos, I.slot_at_pos.data(), sizeof(int32_t) * I.TC);
  cp(C.free_slots, I.free_slots.data(), sizeof(int32_t) * I.TC);
  cp(C.dish, I.dish.data(), sizeof(int32_t) * (size_t)V * I.TC);
  cp(C.d_id, I.d_id.data(), sizeof(int32_t) * (size_t)V * I.KC);
  cp(C.d_n, I.d_n.data(), sizeof(int32_t) * (size_t)V * I.KC);
  cp(C.d_l, I.d_l.data(), sizeof(int32_t) * (size_t)V * I.KC);
  cp(C.d_S1, I.d_S1.data(), sizeof(double) * (size_t)V * I.KC);
  cp(C.d_S2, I.d_S2.data(), sizeof(double) * (size_t)V * I.KC);
  cp(C.Kact, I.Kact.data(), sizeof(int32_t) * V);
  cp(C.next_id, I.next_id.data(), sizeof(int32_t) * V);
  cp(C.hyper, I.hyper.data(), sizeof(double) * (3 * V + 2));
  C.T = I.T;
  C.n_free = I.n_free;
}

void download(const ExactAlloc &A, ExactImage &I, int n, int V, hipStream_t st) {
  const ExactChain &C = A.h;
  I.TC = C.TC; I.KC = C.KC; I.T = C.T; I.n_free = C.n_free;
  auto rs = [&](std::vector<int32_t> &v, size_t k, const void *src) {
    v.resize(k);
    MVC_HIP(hipMemcpyAsync(v.data(), src, sizeof(int32_t) * k, hipMemcpyDeviceToHost, st));
  };
  auto rd = [&](std::vector<double> &v, size_t k, const void *src) {
    v.resize(k);
    MVC_HIP(hipMemcpyAsync(v.data(), src, sizeof(double) * k, hipMemcpyDeviceToHost, st));
  };
  rs(I.z, n, C.z);
  rs(I.n_t, C.TC, C.n_t);
  rs(I.pos_of_slot, C.TC, C.pos_of_slot);
  rs(I.slot_at_pos, C.TC, C.slot_at_pos);
  rs(I.free_slots, C.TC, C.free_slots);
  rs(I.dish, (size_t)V * C.TC, C.dish);
  rs(I.d_id, (size_t)V * C.KC, C.d_id);
  rs(I.d_n, (size_t)V * C.KC, C.d_n);
  rs(I.d_l, (size_t)V * C.KC, C.d_l);
  rd(I.d_S1, (size_t)V * C.KC, C.d_S1);
  rd(I.d_S2, (size_t)V * C.KC, C.d_S2);
  rs(I.Kact, V, C.Kact);
  rs(I.next_id, V, C.next_id);
  rd(I.hyper, 3 * V + 2, C.hyper);
  MVC_HIP(hipStreamSynchronize(st));
}

// Re-stride an image to larger capacities.  Free slots are appended so that
// the slots TC_old..TC_new-1 become available (LIFO order preserved below).
void grow(ExactImage &I, int V, int TC2, int KC2) {
  if (TC2 > I.TC) {
    std::vector<int32_t> dish2((size_t)V * TC2, 0);
    for (int v = 0; v < V; ++v)
      std::copy(I.dish.begin() + (size_t)v * I.TC, I.dish.begin() + (size_t)(v + 1) * I.TC,
                dish2.begin() + (size_t)v * TC2);
    I.dish.swap(dish2);
    I.n_t.resize(TC2, 0);
    I.pos_of_slot.resize(TC2, -1);
    I.slot_at_pos.resize(TC2, -1);
    // free stack: new slots go below the existing free ones so the existing
    // LIFO order (which decides which slot a new table takes) is irrelevant
    // to results anyway -- slots are internal names.
    std::vector<int32_t> fs;
    for (int s = TC2 - 1; s >= I.TC; --s) fs.push_back(s);
    for (int k = 0; k < I.n_free; ++k) fs.push_back(I.free_slots[k]);
    I.free_slots = fs;
    I.free_slots.resize(TC2, -1);
    I.n_free += TC2 - I.TC;
    I.TC = TC2;
  }
  if (KC2 > I.KC) {
    auto re = [&](auto &vec) {
      using Tv = typename std::decay<decltype(vec)>::type::value_type;
      std::vector<Tv> out((size_t)V * KC2, Tv(0));
      for (int v = 0; v < V; ++v)
        std::copy(vec.begin() + (size_t)v * I.KC, vec.begin() + (size_t)(v + 1) * I.KC,
                  out.begin() + (size_t)v * KC2);
      vec.swap(out);
    };
    re(I.d_id); re(I.d_n); re(I.d_l); re(I.d_S1); re(I.d_S2);
    I.KC = KC2;
  }
}

}  // namespace

class ExactSampler : public Sampler {
 public:
  int n, V;
  double *y_dev = nullptr;
  std::vector<ExactAlloc> chains;
  ExactChain *chains_dev = nullptr;

  ExactSampler(const mvc_config &c, const double *const *views) {
    cfg = c;
    n = c.n;
    V = c.n_views;
    if (c.dim != 1) throw Error(MVC_ERR_UNSUPPORTED, "exact mode requires dim == 1 (the reference's scalar views)");
    if (V > MVC_MAXV) throw Error(MVC_ERR_UNSUPPORTED, "exact mode supports at most 64 views");
    MVC_HIP(hipSetDevice(c.device));
    MVC_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    timers.stream = stream;
    timers.on = (c.flags & MVC_FLAG_TIMING) != 0;
    timers.coarse = (c.flags & MVC_FLAG_TIMING_COARSE) != 0;
    std::vector<double> y((size_t)V * n);
    for (int v = 0; v < V; ++v) std::memcpy(&y[(size_t)v * n], views[v], sizeof(double) * n);
    MVC_HIP(hipMalloc(&y_dev, sizeof(double) * y.size()));
    MVC_HIP(hipMemcpyAsync(y_dev, y.data(), sizeof(double) * y.size(), hipMemcpyHostToDevice, stream));
    // Default capacities 71 and 39 (7 mod 32), not 64 and 32: the per-view rows
    // [V][TC] and [V][KC] are read with one lane per view at the same index
    // (v * KC + j) and with one lane per dish across views, and a row stride
    // that is a multiple of 32 dwords puts every view on the same LDS bank.
    // For n <= 512 the table capacity starts at its bound n + 1 (T <= n), so
    // the cold transient (T ~ n at New_Simulation's sweeps 3-10) needs no
    // overflow relaunch and per-chain regrowth.
    const int TC = std::max(c.table_cap > 0 ? c.table_cap : (n + 1 <= 512 ? std::max(n + 1, 71) : 71), 8);
    const int KC = std::max(c.dish_cap > 0 ? c.dish_cap : 39, 4);
    chains.resize(c.n_chains);
    for (int ch = 0; ch < c.n_chains; ++ch) {
      const uint32_t gid = chain_gid(c, ch);
      InitState S = draw_initial_state(y.data(), n, V, 1, c.seed, gid);
      ExactImage I = image_from_init(S, y.data(), TC, KC);
      ExactAlloc &A = chains[ch];
      MVC_HIP(hipMalloc(&A.block, exact_bytes(n, V, TC, KC)));
      carve(A, n, V, TC, KC);
      upload(A, I, n, V, stream);
      MVC_HIP(hipStreamSynchronize(stream));   // I is a temporary
      A.h.draws = S.draws;
      A.h.resume_i = 0;
      A.h.status = MVC_ST_RUNNING;
      A.h.chain_id = (int32_t)gid;
    }
    MVC_HIP(hipMalloc(&chains_dev, sizeof(ExactChain) * chains.size()));
    push_structs();
    if (const char *e = getenv("MVC_EXACT_PROF"); e && e[0] == '1') {
      MVC_HIP(hipMalloc(&prof_dev, sizeof(long long) * 8 * chains.size()));
      MVC_HIP(hipMemsetAsync(prof_dev, 0, sizeof(long long) * 8 * chains.size(), stream));
    }
    MVC_HIP(hipStreamSynchronize(stream));
  }

  // MVC_EXACT_PROF=1: the kernel's shader clocks per phase, summed over the
  // handle's launches; printed per customer step (mean over chains) at close
  long long *prof_dev = nullptr;
  void report_prof() {
    if (!prof_dev) return;
    const size_t C = chains.size();
    std::vector<long long> h(8 * C);
    if (hipMemcpy(h.data(), prof_dev, sizeof(long long) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    double tot[8] = {0};
    for (size_t c = 0; c < C; ++c)
      for (int k = 0; k < 8; ++k) tot[k] += (double)h[c * 8 + k];
    const double steps = (double)C * (double)sweeps_done * n;
    static const char *names[8] = {"remove", "f_vk", "marg+tables", "normaliser", "normalise+find", "join", "open",
                                   "mh+save"};
    std::fprintf(stderr, "{\"exact_prof_clocks_per_customer\": {");
    double all = 0;
    for (int k = 0; k < 8; ++k) {
      std::fprintf(stderr, "%s\"%s\": %.1f", k ? ", " : "", names[k], tot[k] / steps);
      all += tot[k];
    }
    std::fprintf(stderr, ", \"total\": %.1f, \"chains\": %zu, \"sweeps\": %lld}}\n", all / steps, C,
                 (long long)sweeps_done);
  }

  // save slots of save_all_async (every chain's sample in one snapshot)
  struct SaveSlot {
    int32_t *dz = nullptr, *ddish = nullptr, *dT = nullptr;
    double *dhyp = nullptr;
    int32_t *hz = nullptr, *hdish = nullptr, *hT = nullptr;
    double *hhyp = nullptr;
    int dcap = 0;
    hipEvent_t snap = nullptr, done = nullptr;
    bool busy = false;
    SampleFn fn;
  };
  static constexpr int kSaveSlots = 4;
  SaveSlot saves[kSaveSlots];
  int save_next = 0;
  hipStream_t cstream = nullptr;

  void free_slot(SaveSlot &q) {
    hipFree(q.dz); hipFree(q.ddish); hipFree(q.dT); hipFree(q.dhyp);
    hipHostFree(q.hz); hipHostFree(q.hdish); hipHostFree(q.hT); hipHostFree(q.hhyp);
    q.dz = q.ddish = q.dT = nullptr; q.dhyp = nullptr;
    q.hz = q.hdish = q.hT = nullptr; q.hhyp = nullptr;
    q.dcap = 0;
  }
  void finish_slot(SaveSlot &q) {
    MVC_HIP(hipEventSynchronize(q.done));
    const int C = (int)chains.size(), H = 3 * V + 2;
    std::vector<int32_t> d;
    for (int c = 0; c < C; ++c) {
      const int T = q.hT[c];
      d.assign((size_t)V * T, 0);
      for (int v = 0; v < V; ++v)
        std::copy(q.hdish + ((size_t)c * V + v) * q.dcap, q.hdish + ((size_t)c * V + v) * q.dcap + T,
                  d.begin() + (size_t)v * T);
      q.fn(c, T, q.hz + (size_t)c * n, d.data(), q.hhyp + (size_t)c * H);
    }
    q.busy = false;
  }
  // One snapshot kernel for all chains into a device slot, read back on a
  // second stream; the samples reach fn (chain by chain, in order) when the
  // slot is reused or at flush_saves.  Replaces two get_state calls per chain
  // and sample, each of which synchronised the device.
  bool save_all_async(const SampleFn &fn) override {
    if (!cstream) MVC_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    SaveSlot &q = saves[save_next];
    if (q.busy) finish_slot(q);
    const int C = (int)chains.size(), H = 3 * V + 2;
    int dcap = 1;
    for (auto &A : chains) dcap = std::max(dcap, A.h.TC);
    if (q.dcap < dcap) {
      if (q.dz) free_slot(q);
      MVC_HIP(hipMalloc(&q.dz, sizeof(int32_t) * (size_t)C * std::max(n, 1)));
      MVC_HIP(hipMalloc(&q.ddish, sizeof(int32_t) * (size_t)C * V * dcap));
      MVC_HIP(hipMalloc(&q.dT, sizeof(int32_t) * C));
      MVC_HIP(hipMalloc(&q.dhyp, sizeof(double) * (size_t)C * H));
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
    hipLaunchKernelGGL(mvc_exact_snapshot_all_kernel, dim3(std::min(64, (n + 255) / 256 + 1), C), dim3(256), 0, stream,
                       n, V, (const ExactChain *)chains_dev, q.dcap, q.dz, q.ddish, q.dT, q.dhyp);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipEventRecord(q.snap, stream));
    MVC_HIP(hipStreamWaitEvent(cstream, q.snap, 0));
    MVC_HIP(hipMemcpyAsync(q.hz, q.dz, sizeof(int32_t) * (size_t)C * n, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hdish, q.ddish, sizeof(int32_t) * (size_t)C * V * q.dcap, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hT, q.dT, sizeof(int32_t) * C, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipMemcpyAsync(q.hhyp, q.dhyp, sizeof(double) * (size_t)C * H, hipMemcpyDeviceToHost, cstream));
    MVC_HIP(hipEventRecord(q.done, cstream));
    q.busy = true;
    q.fn = fn;
    save_next = (save_next + 1) % kSaveSlots;
    return true;
  }
  void flush_saves() override {
    for (int k = 0; k < kSaveSlots; ++k) {
      SaveSlot &q = saves[(save_next + k) % kSaveSlots];   // oldest first
      if (q.busy) finish_slot(q);
    }
  }

  ~ExactSampler() override {
    if (stream) hipStreamSynchronize(stream);
    report_prof();
    if (prof_dev) hipFree(prof_dev);
    if (cstream) hipStreamSynchronize(cstream);
    for (auto &q : saves) {
      free_slot(q);
      if (q.snap) hipEventDestroy(q.snap);
      if (q.done) hipEventDestroy(q.done);
    }
    if (cstream) hipStreamDestroy(cstream);
    for (auto &A : chains) if (A.block) hipFree(A.block);
    if (chains_dev) hipFree(chains_dev);
    if (y_dev) hipFree(y_dev);
    if (stream) hipStreamDestroy(stream);
  }

  ExactImage image_from_init(const InitState &S, const double *y, int TC, int KC) {
    // multiview_gibbs.cpp:12-103 in slot/live-list form
    ExactImage I;
    I.TC = TC; I.KC = KC; I.T = 4;
    I.z = S.table;
    I.n_t.assign(TC, 0);
    for (int i = 0; i < n; ++i) I.n_t[S.table[i]]++;
    I.pos_of_slot.assign(TC, -1);
    I.slot_at_pos.assign(TC, -1);
    for (int p = 0; p < 4; ++p) { I.pos_of_slot[p] = p; I.slot_at_pos[p] = p; }
    I.n_free = TC - 4;
    I.free_slots.assign(TC, -1);
    for (int k = 0; k < I.n_free; ++k) I.free_slots[k] = TC - 1 - k;   // pop gives slot 4 first
    I.dish.assign((size_t)V * TC, 0);
    I.d_id.assign((size_t)V * KC, 0); I.d_n.assign((size_t)V * KC, 0); I.d_l.assign((size_t)V * KC, 0);
    I.d_S1.assign((size_t)V * KC, 0.0); I.d_S2.assign((size_t)V * KC, 0.0);
    I.Kact.assign(V, 0);
    I.next_id.assign(V, 2);
    I.hyper.assign(3 * V + 2, 0.0);
    for (int v = 0; v < V; ++v) {
      int l2[2] = {0, 0}, n2[2] = {0, 0};
      double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
      for (int t = 0; t < 4; ++t) l2[S.dish_raw[v * 4 + t]]++;
      for (int i = 0; i < n; ++i) {          // :64-73, ascending i
        const int k = S.dish_raw[v * 4 + S.table[i]];
        const double val = y[(size_t)v * n + i];
        n2[k]++;
        s1[k] += val;
        s2[k] += val * val;
      }
      int map2[2] = {-1, -1};
      for (int k = 0; k < 2; ++k)
        if (l2[k] > 0) {
          const int j = I.Kact[v]++;
          map2[k] = j;
          I.d_id[v * KC + j] = k; I.d_n[v * KC + j] = n2[k]; I.d_l[v * KC + j] = l2[k];
          I.d_S1[v * KC + j] = s1[k]; I.d_S2[v * KC + j] = s2[k];
        }
      for (int t = 0; t < 4; ++t) I.dish[(size_t)v * TC + t] = map2[S.dish_raw[v * 4 + t]];
      I.hyper[v] = S.tau[v];
      I.hyper[V + v] = 1.0;
      I.hyper[2 * V + v] = 0.5;
    }
    I.hyper[3 * V] = 1.0;
    I.hyper[3 * V + 1] = 0.6;
    return I;
  }

  // dynamic LDS of the sweep kernel: the largest chain's array range that fits
  // kExactLds (with z when every chain's does), 0 when none fits
  static constexpr size_t kExactLds = 48 * 1024;
  int lds_bytes(int *mode = nullptr) const {
    size_t full = 0, part = 0;
    for (auto &A : chains) {
      full = std::max(full, (size_t)((char *)A.h.mhbuf - (char *)A.h.z));
      part = std::max(part, (size_t)((char *)A.h.mhbuf - (char *)A.h.n_t));
    }
    int m = full <= kExactLds ? 2 : (part <= kExactLds ? 1 : 0);
    if (const char *e = path_opt("exact_lds"); e && e[0] >= '0' && e[0] <= '2') m = std::min(m, e[0] - '0');   // tests (MVC_PATH)
    if (mode) *mode = m;
    return (int)(m == 2 ? full : (m == 1 ? part : 0));
  }

  void push_structs() {
    std::vector<ExactChain> hs(chains.size());
    for (size_t k = 0; k < chains.size(); ++k) hs[k] = chains[k].h;
    MVC_HIP(hipMemcpyAsync(chains_dev, hs.data(), sizeof(ExactChain) * hs.size(), hipMemcpyHostToDevice, stream));
    MVC_HIP(hipStreamSynchronize(stream));
  }
  void pull_structs() {
    std::vector<ExactChain> hs(chains.size());
    MVC_HIP(hipMemcpyAsync(hs.data(), chains_dev, sizeof(ExactChain) * hs.size(), hipMemcpyDeviceToHost, stream));
    MVC_HIP(hipStreamSynchronize(stream));
    for (size_t k = 0; k < chains.size(); ++k) {
      ExactChain &C = chains[k].h;
      C.T = hs[k].T; C.n_free = hs[k].n_free; C.draws = hs[k].draws;
      C.resume_i = hs[k].resume_i; C.status = hs[k].status; C.todo = hs[k].todo;
    }
  }

  void grow_chain(ExactAlloc &A) {
    ExactImage I;
    download(A, I, n, V, stream);
    int TC2 = I.TC, KC2 = I.KC;
    // doubling, capped at n + 1: T <= n and K_v <= T, so a step's T + 1 and
    // K_v + 1 never exceed it (a smaller footprint keeps more chains per CU)
    if (I.n_free < 1) TC2 = std::max(I.TC + 1, std::min(I.TC * 2, n + 1));
    for (int v = 0; v < V; ++v) if (I.Kact[v] + 1 > I.KC) KC2 = std::max(I.KC + 1, std::min(I.KC * 2, n + 1));
    grow(I, V, TC2, KC2);
    ExactAlloc B;
    B.h = A.h;
    MVC_HIP(hipMalloc(&B.block, exact_bytes(n, V, TC2, KC2)));
    carve(B, n, V, TC2, KC2);
    upload(B, I, n, V, stream);
    MVC_HIP(hipStreamSynchronize(stream));
    MVC_HIP(hipFree(A.block));
    B.h.status = MVC_ST_RUNNING;
    A = B;
  }

  // sweeps per kernel launch: each chain runs its sweeps on its own, so a
  // launch lasts about the longest chain's sum of sweeps rather than the sum
  // of the longest sweeps, and the per-sweep launch + read-back is amortised
  static constexpr int kSweepsPerLaunch = 64;
  // k sweeps from every chain's current state in launches (capacity growth
  // relaunches from where a chain stopped); SV: the in-kernel sample output
  // the kernel instance of the storage mode (mvc_exact_sweep_kernel) and view bound
  template <int M>
  void launch_mode(int lb, const ExactSave &SV) {
    const dim3 g((unsigned)chains.size()), b(64);
    if (V <= 8)
      hipLaunchKernelGGL((mvc_exact_sweep_kernel<M, 8>), g, b, lb, stream, (const double *)y_dev, n, V, chains_dev,
                         cfg.seed, SV);
    else
      hipLaunchKernelGGL((mvc_exact_sweep_kernel<M, MVC_MAXV>), g, b, lb, stream, (const double *)y_dev, n, V,
                         chains_dev, cfg.seed, SV);
  }
  void launch_sweep(int mode, int lb, const ExactSave &SV) {
    if (mode == 2) launch_mode<2>(lb, SV);
    else if (mode == 1) launch_mode<1>(lb, SV);
    else launch_mode<0>(lb, SV);
  }
  void run_launch(int k, ExactSave SV) {
    SV.prof = prof_dev;
    for (auto &A : chains) { A.h.status = MVC_ST_RUNNING; A.h.resume_i = 0; A.h.todo = k; }
    push_structs();
    hipEvent_t ev0 = nullptr;
    timers.begin("sweep", &ev0);
    for (int round = 0;; ++round) {
      hipEvent_t ev = nullptr;
      timers.begin("exact_sweep", &ev);
      int mode = 0;
      const int lb = lds_bytes(&mode);
      launch_sweep(mode, lb, SV);
      MVC_HIP(hipGetLastError());
      timers.end("exact_sweep", ev);
      pull_structs();
      bool again = false;
      for (auto &A : chains) {
        if (A.h.status == MVC_ST_OVERFLOW) { grow_chain(A); again = true; }
        else if (A.h.status != MVC_ST_DONE) throw Error(MVC_ERR_STATE, "exact sweep kernel left a chain unfinished");
      }
      if (!again) break;
      push_structs();
      if (round > 64 + 64 * k) throw Error(MVC_ERR_STATE, "capacity growth did not converge");
    }
    timers.end("sweep", ev0);
    sweeps_done += k;
  }
  void sweep(int n_sweeps) override {
    for (int left = n_sweeps; left > 0;) {
      const int k = std::min(left, kSweepsPerLaunch);
      run_launch(k, ExactSave{});
      left -= k;
    }
  }

  // mvc_run's loop (gibbs.cpp:150-206) with every saved sweep written by the
  // kernel itself (ExactSave): launches of up to kSweepsPerLaunch sweeps
  // whatever the thinning, the samples of a launch read back in one copy.
  // The device buffer holds one launch's samples of every chain (at most
  // kSaveBudget bytes; fewer sweeps per launch when that is short).
  static constexpr size_t kSaveBudget = (size_t)4 << 30;
  bool run_saving(int n_iter, int burn_in, int thin, bool quiet, const SampleFn &fn) override {
    const int C = (int)chains.size(), H = 3 * V + 2, dcap = std::max(n, 1);
    const size_t per_sample = sizeof(int32_t) * ((size_t)n + (size_t)V * dcap + 1) + sizeof(double) * H;
    // the sample buffers of one launch: at most kSaveBudget and a quarter of
    // the device's free memory (the run_part fallback saves without them)
    size_t budget = kSaveBudget, free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) budget = std::min(budget, free_b / 4);
    const int64_t fit = (int64_t)(budget / std::max<size_t>(1, per_sample * C));
    if (fit < 1 || thin < 1) return false;
    const int klim = (int)std::min<int64_t>(kSweepsPerLaunch, fit * thin);
    int32_t *dz = nullptr, *dd = nullptr, *dT = nullptr;
    double *dh = nullptr;
    std::vector<int32_t> hT;
    // pinned host buffers for the samples (grown as needed): z, dish (Tmax
    // wide), hyper; pageable memory where pinned memory is refused
    int32_t *hz = nullptr, *hd = nullptr;
    double *hh = nullptr;
    size_t hz_cap = 0, hd_cap = 0, hh_cap = 0;
    std::vector<void *> pageable;
    auto host_free = [&](void *q) {
      auto it = std::find(pageable.begin(), pageable.end(), q);
      if (it != pageable.end()) { std::free(q); pageable.erase(it); }
      else hipHostFree(q);
    };
    auto pinned = [&](auto *&ptr, size_t &cap, size_t count) {
      using Tp = std::remove_reference_t<decltype(*ptr)>;
      if (count <= cap) return;
      if (ptr) host_free(ptr);
      ptr = nullptr;
      if (hipHostMalloc((void **)&ptr, sizeof(Tp) * count, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        ptr = (Tp *)std::malloc(sizeof(Tp) * count);
        if (!ptr) throw Error(MVC_ERR_HIP, "out of host memory for the samples");
        pageable.push_back(ptr);
      }
      cap = count;
    };
    auto release = [&]() {
      for (void *q : {(void *)dz, (void *)dd, (void *)dT, (void *)dh}) if (q) hipFree(q);
      for (void *q : {(void *)hz, (void *)hd, (void *)hh}) if (q) host_free(q);
    };
    // the device buffers for the most samples one launch can hold, before the
    // first launch: if they do not fit, nothing has run yet and the caller's
    // sweep + save_all_async path takes over
    int nslot = 0;
    {
      if (n_iter > std::max(burn_in, 0)) {
        nslot = std::min(klim, (klim + thin - 1) / thin + 1);
        const bool ok = hipMalloc(&dz, sizeof(int32_t) * (size_t)C * nslot * std::max(n, 1)) == hipSuccess &&
                        hipMalloc(&dd, sizeof(int32_t) * (size_t)C * nslot * V * dcap) == hipSuccess &&
                        hipMalloc(&dT, sizeof(int32_t) * (size_t)C * nslot) == hipSuccess &&
                        hipMalloc(&dh, sizeof(double) * (size_t)C * nslot * H) == hipSuccess;
        if (!ok) {
          (void)hipGetLastError();
          release();
          return false;
        }
      }
    }
    try {
      for (int it0 = 0; it0 < n_iter;) {
        const int k = std::min(klim, n_iter - it0);
        // the saved sweeps of [it0, it0 + k): global index = sweeps_done + offset
        const int64_t g0 = sweeps_done;
        auto saved = [&](int it) { return it >= burn_in && (it - burn_in) % thin == 0; };
        int first = -1, m = 0;
        for (int it = it0; it < it0 + k; ++it)
          if (saved(it)) { if (first < 0) first = it; ++m; }
        ExactSave SV{};
        if (m > 0) {
          if (m > nslot) {
            for (void *p : {(void *)dz, (void *)dd, (void *)dT, (void *)dh}) if (p) hipFree(p);
            dz = dd = dT = nullptr; dh = nullptr;
            nslot = m;
            MVC_HIP(hipMalloc(&dz, sizeof(int32_t) * (size_t)C * nslot * std::max(n, 1)));
            MVC_HIP(hipMalloc(&dd, sizeof(int32_t) * (size_t)C * nslot * V * dcap));
            MVC_HIP(hipMalloc(&dT, sizeof(int32_t) * (size_t)C * nslot));
            MVC_HIP(hipMalloc(&dh, sizeof(double) * (size_t)C * nslot * H));
          }
          SV.z = dz; SV.dish = dd; SV.T = dT; SV.hyp = dh;
          SV.dcap = dcap; SV.nslot = nslot; SV.ktot = k; SV.thin = thin;
          // sweep it of the call is global sweep g0 + (it - it0)
          SV.sweep_base = g0;
          SV.burn = g0 + (burn_in - it0);
          SV.first = g0 + (first - it0);
        }
        run_launch(k, SV);
        if (!quiet)
          for (int it = it0; it < it0 + k; ++it)
            if ((it + 1) % 100 == 0) std::fprintf(stderr, "Iteration %d / %d\n", it + 1, n_iter);   // gibbs.cpp:152-155
        if (m > 0) {   // samples in order, chain by chain (the callback's per-chain order)
          const size_t ns = (size_t)C * nslot;
          hT.resize(ns);
          MVC_HIP(hipMemcpyAsync(hT.data(), dT, sizeof(int32_t) * ns, hipMemcpyDeviceToHost, stream));
          MVC_HIP(hipStreamSynchronize(stream));
          int Tmax = 1;   // only the first Tmax dish entries of each [dcap] row are copied
          for (int c = 0; c < C; ++c)
            for (int sm = 0; sm < m; ++sm) Tmax = std::max(Tmax, hT[(size_t)c * nslot + sm]);
          pinned(hz, hz_cap, ns * n);
          pinned(hd, hd_cap, ns * V * Tmax);
          pinned(hh, hh_cap, ns * H);
          MVC_HIP(hipMemcpyAsync(hz, dz, sizeof(int32_t) * ns * n, hipMemcpyDeviceToHost, stream));
          MVC_HIP(hipMemcpy2DAsync(hd, sizeof(int32_t) * Tmax, dd, sizeof(int32_t) * dcap, sizeof(int32_t) * Tmax,
                                   ns * V, hipMemcpyDeviceToHost, stream));
          MVC_HIP(hipMemcpyAsync(hh, dh, sizeof(double) * ns * H, hipMemcpyDeviceToHost, stream));
          MVC_HIP(hipStreamSynchronize(stream));
          // each chain's samples in order; the chains split over host threads
          // (fn writes per chain: thousands of chains x the launch's samples)
          auto emit = [&](int c0, int c1) {
            std::vector<int32_t> dt;
            for (int c = c0; c < c1; ++c)
              for (int sm = 0; sm < m; ++sm) {
                const size_t slot = (size_t)c * nslot + sm;
                const int T = hT[slot];
                dt.resize((size_t)V * T);
                for (int v = 0; v < V; ++v)
                  std::copy(hd + (slot * V + v) * Tmax, hd + (slot * V + v) * Tmax + T, dt.begin() + (size_t)v * T);
                fn(c, T, hz + slot * n, dt.data(), hh + slot * H);
              }
          };
          const int nth = C >= 256 ? std::min(8, std::max(1, (int)std::thread::hardware_concurrency())) : 1;
          if (nth <= 1) {
            emit(0, C);
          } else {
            // an exception on a worker (fn grows vectors) is carried back to
            // this thread and rethrown after every thread has joined, so the
            // C ABI returns a status instead of std::terminate
            std::vector<std::exception_ptr> err(nth);
            auto part = [&](int t) {
              try { emit((int)((int64_t)C * t / nth), (int)((int64_t)C * (t + 1) / nth)); }
              catch (...) { err[t] = std::current_exception(); }
            };
            std::vector<std::thread> th;
            for (int t = 1; t < nth; ++t) {
              try { th.emplace_back(part, t); }
              catch (...) { part(t); }       // no thread: run the range here
            }
            part(0);
            for (auto &x : th) x.join();
            for (auto &e : err) if (e) std::rethrow_exception(e);
          }
        }
        it0 += k;
      }
    } catch (...) {
      release();
      throw;
    }
    release();
    return true;
  }

  void synchronize() override { MVC_HIP(hipStreamSynchronize(stream)); timers.collect(); }

  void get_state(int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of, int32_t dish_cap,
                 double *hyper) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    pull_structs();
    const ExactChain &C = chains[chain].h;
    const int T = C.T;
    if (n_tables) *n_tables = T;
    int32_t *t_dev = nullptr, *d_dev = nullptr;
    const int cap = std::max(T, 1);
    MVC_HIP(hipMalloc(&t_dev, sizeof(int32_t) * n));
    MVC_HIP(hipMalloc(&d_dev, sizeof(int32_t) * (size_t)V * cap));
    hipLaunchKernelGGL(mvc_exact_snapshot_kernel, dim3(std::min(1024, (n + 255) / 256 + 1)), dim3(256), 0, stream,
                       n, V, (const ExactChain *)chains_dev, chain, t_dev, d_dev, cap);
    MVC_HIP(hipGetLastError());
    std::vector<int32_t> dd((size_t)V * cap);
    if (table_of) MVC_HIP(hipMemcpyAsync(table_of, t_dev, sizeof(int32_t) * n, hipMemcpyDeviceToHost, stream));
    MVC_HIP(hipMemcpyAsync(dd.data(), d_dev, sizeof(int32_t) * dd.size(), hipMemcpyDeviceToHost, stream));
    std::vector<double> hy(3 * V + 2);
    MVC_HIP(hipMemcpyAsync(hy.data(), C.hyper, sizeof(double) * hy.size(), hipMemcpyDeviceToHost, stream));
    MVC_HIP(hipStreamSynchronize(stream));
    hipFree(t_dev);
    hipFree(d_dev);
    if (dish_of)
      for (int v = 0; v < V; ++v)
        for (int p = 0; p < std::min(T, (int)dish_cap); ++p) dish_of[(size_t)v * dish_cap + p] = dd[(size_t)v * cap + p];
    if (hyper) std::copy(hy.begin(), hy.end(), hyper);
  }

  void set_state(int chain, const int32_t *table_of, int32_t T, const int32_t *dish_of, const double *hyper) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    const UserState U = check_user_state(n, V, table_of, T, dish_of);
    std::vector<double> yh((size_t)V * n);
    MVC_HIP(hipMemcpy(yh.data(), y_dev, sizeof(double) * yh.size(), hipMemcpyDeviceToHost));
    int TC = chains[chain].h.TC, KC = chains[chain].h.KC;
    while (TC < T + 1) TC *= 2;
    for (int v = 0; v < V; ++v)
      while (KC < (int)U.ids[v].size() + 1) KC *= 2;
    ExactImage I;
    I.TC = TC; I.KC = KC; I.T = T;
    I.z.assign(table_of, table_of + n);           // slot p == position p
    I.n_t.assign(TC, 0);
    for (int p = 0; p < T; ++p) I.n_t[p] = U.n_t[p];
    I.pos_of_slot.assign(TC, -1);
    I.slot_at_pos.assign(TC, -1);
    for (int p = 0; p < T; ++p) { I.pos_of_slot[p] = p; I.slot_at_pos[p] = p; }
    I.n_free = TC - T;
    I.free_slots.assign(TC, -1);
    for (int k = 0; k < I.n_free; ++k) I.free_slots[k] = TC - 1 - k;
    I.dish.assign((size_t)V * TC, 0);
    I.d_id.assign((size_t)V * KC, 0); I.d_n.assign((size_t)V * KC, 0); I.d_l.assign((size_t)V * KC, 0);
    I.d_S1.assign((size_t)V * KC, 0.0); I.d_S2.assign((size_t)V * KC, 0.0);
    I.Kact.assign(V, 0);
    I.next_id = U.next_id;
    I.hyper.assign(hyper, hyper + 3 * V + 2);
    for (int v = 0; v < V; ++v) {
      const int K = (int)U.ids[v].size();
      I.Kact[v] = K;
      for (int j = 0; j < K; ++j) { I.d_id[v * KC + j] = U.ids[v][j]; I.d_l[v * KC + j] = U.l[v][j]; }
      for (int p = 0; p < T; ++p) I.dish[(size_t)v * TC + p] = U.dish[v][p];
      for (int i = 0; i < n; ++i) {        // sufficient statistics, ascending i
        const int j = U.dish[v][table_of[i]];
        const double val = yh[(size_t)v * n + i];
        I.d_n[v * KC + j]++;
        I.d_S1[v * KC + j] += val;
        I.d_S2[v * KC + j] += val * val;
      }
    }
    ExactAlloc &A = chains[chain];
    ExactAlloc B;
    B.h = A.h;
    MVC_HIP(hipMalloc(&B.block, exact_bytes(n, V, TC, KC)));
    carve(B, n, V, TC, KC);
    upload(B, I, n, V, stream);
    MVC_HIP(hipStreamSynchronize(stream));
    MVC_HIP(hipFree(A.block));
    B.h.draws = 0;
    B.h.resume_i = 0;
    B.h.status = MVC_ST_RUNNING;
    A = B;
    push_structs();
  }

  void get_dish_counts(int chain, int32_t *k_out) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    MVC_HIP(hipMemcpyAsync(k_out, chains[chain].h.Kact, sizeof(int32_t) * V, hipMemcpyDeviceToHost, stream));
    MVC_HIP(hipStreamSynchronize(stream));
  }

  void get_stats(int chain, int view, int32_t *K, double *S1, double *S2, int32_t *n_vk, int32_t cap) override {
    if (chain < 0 || chain >= (int)chains.size()) throw Error(MVC_ERR_ARG, "chain out of range");
    const ExactChain &h = chains[chain].h;
    MVC_HIP(hipStreamSynchronize(stream));
    int32_t k = 0;
    MVC_HIP(hipMemcpy(&k, h.Kact + view, sizeof(int32_t), hipMemcpyDeviceToHost));
    if (K) *K = k;
    const int c = std::min<int>(k, cap);
    const size_t off = (size_t)view * h.KC;
    if (S1 && c) MVC_HIP(hipMemcpy(S1, h.d_S1 + off, sizeof(double) * c, hipMemcpyDeviceToHost));
    if (S2 && c) MVC_HIP(hipMemcpy(S2, h.d_S2 + off, sizeof(double) * c, hipMemcpyDeviceToHost));
    if (n_vk && c) MVC_HIP(hipMemcpy(n_vk, h.d_n + off, sizeof(int32_t) * c, hipMemcpyDeviceToHost));
  }
};

Sampler *make_exact_sampler(const mvc_config &cfg, const double *const *views) {
  return new ExactSampler(cfg, views);
}

}  // namespace mvc
