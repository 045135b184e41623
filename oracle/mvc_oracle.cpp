// mvc_oracle.cpp — CPU ORACLE for the MI355X multiview Gibbs sampler.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load this library.  The product
// (multiview-clustering_amd/, libmvc_hip.so) never links or calls it.
//
// PARITY STATUS: "parity unpinned" against the reference binary.  The
// reference (/root/reference/Multiview/*.cpp) includes <Rcpp.h> and calls R's
// RNG; R/Rcpp/Rmath are absent from this image and writing stand-in headers
// is not allowed, so the reference cannot be compiled here, and the
// reference's own tests (tests/dummy_test.cpp:3-5, CHECK(1 == 1)) hold no
// golden vectors.  This file is a line-by-line *restatement* of the
// reference algorithm (citations below); it is pinned by (a) published
// Philox4x32-10 known-answer vectors, (b) accuracy checks of its math against
// glibc / scipy, and (c) invariant checks in tests/.
//
// Three samplers:
//   * ExactSampler   — the reference schedule (multiview_gibbs.cpp:134-212),
//     D = 1, sequential RNG stream.  Template parameter selects the math:
//     LibmMath (std::exp/std::log exactly like the reference) or PortableMath
//     (include/mvc_pmath.h, bit-identical to the GPU).
//   * SeqSampler (mode 1, "parallel" in the C ABI) — the SAME sequential
//     schedule (customer i+1 sees customer i's move) with the GPU-shaped
//     per-customer conditional of DESIGN.md §4.2-4.3, any D, counter-
//     addressed Philox draws.  libmvc_hip.so executes this chain with a
//     data-parallel speculative pass plus an in-order repair (DESIGN.md
//     §4.8); the GPU is checked against it bit for bit.
//   * ParallelSampler::run (mode 3, JACOBI) — round 1's schedule: every
//     customer resampled against the state frozen at sweep start.  It does
//     not leave the posterior invariant (tests/test_posterior.py shows the
//     bias) and is kept only as that documented negative result; its
//     per-customer conditional (resample_customer, eval_view_seq) is the one
//     SeqSampler evaluates.
//
// Build: oracle/Makefile  (g++ -O2 -ffp-contract=off, no fast-math).
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <algorithm>
#include <vector>
#include <string>
#include <stdexcept>

#include "mvc_philox.h"
#include "mvc_pmath.h"

namespace {

constexpr double kEps = 1e-6;            // multiview_hyper.cpp:13
constexpr int kStatsChunk = 4096;        // parallel-mode stats rebuild chunk

struct LibmMath {
  static double exp(double x) { return std::exp(x); }
  static double log(double x) { return std::log(x); }
};
struct PortableMath {
  static double exp(double x) { return mvc_exp(x); }
  static double log(double x) { return mvc_log(x); }
};

// ---------------------------------------------------------------------------
// The R-shaped RNG stream (stand-in for R's unif_rand / norm_rand).
// R::runif(a,b) = a + (b-a)*unif_rand()          (R nmath/runif.c)
// R::rnorm(m,s) = m + s*norm_rand(), INVERSION   (R nmath/rnorm.c, snorm.c)
// ---------------------------------------------------------------------------
struct SeqRng {
  uint64_t seed;
  uint32_t chain;
  uint64_t draws;
  double unif_rand() { return mvc_seq_uniform(seed, chain, draws++); }
  double runif(double a, double b) {
    if (a == b) return a;
    return a + (b - a) * unif_rand();
  }
  double norm_rand() {
    const double u1 = unif_rand();
    const double u2 = unif_rand();
    return mvc_norm_from_uniforms(u1, u2);
  }
  double rnorm(double mu, double sd) {
    if (sd == 0.0) return mu;
    return mu + sd * norm_rand();
  }
};

// Output common to both samplers (mirrors the Rcpp::List of
// multiview_gibbs.cpp:121-130).
struct Result {
  int n = 0, V = 0, S = 0;
  std::vector<int> table_of;               // S x n
  std::vector<int> sample_T;               // S
  std::vector<int64_t> dish_off;           // S+1 offsets into dish_of
  std::vector<int> dish_of;                // per sample: V x T_s (view-major)
  std::vector<double> alpha_v, sigma_v, tau_v;  // S x V
  std::vector<double> alpha_g, sigma_g;    // S
  std::vector<int> trace_T;                // per sweep: T after the sweep
  std::vector<uint64_t> trace_draws;       // per sweep: sequential draws used so far
  std::vector<int64_t> trace_moves, trace_births, trace_newdish;  // SeqSampler, per sweep
  // ExactSampler, per sweep: the reference's linear-space underflow
  // (multiview_utils.cpp:107,114,124-135; multiview_gibbs.cpp:169-176):
  // customers whose sum_p <= 0 took the table-0 fallback; tables with
  // n_t - sigma_g > 0 whose probability underflowed to 0 (summed over
  // customers); customers with at least one such table; customers whose
  // new-table probability underflowed with a positive mass
  std::vector<int64_t> trace_fallback, trace_uf_tables, trace_uf_customers, trace_uf_new;
  // final sufficient statistics (parallel sampler): per view, live dishes in
  // ascending raw id; S1 [K][D], S2 [K], n_vk [K]
  std::vector<std::vector<double>> fS1, fS2;
  std::vector<std::vector<int>> fnk;
  int D = 1;
  std::string error;
};

// ===========================================================================
// ExactSampler: restatement of the reference schedule.
// State layout follows multiview_state.h:7-33 (process globals -> members).
// ===========================================================================
template <class Math>
struct ExactSampler {
  struct View {                               // multiview_state.h:7-18
    int K = 0;
    std::vector<int> n_vk, l_vk;
    std::vector<double> sum_y, sum_y2;
    double alpha_v = 1.0, sigma_v = 0.5, tau_v = 1.0;
  };
  int n = 0, d = 0;
  std::vector<std::vector<double>> y;         // y[v][i]
  double alpha_global = 1.0, sigma_global = 0.5;
  int T = 0;
  std::vector<int> table_of, n_t;
  std::vector<std::vector<int>> members;      // customers_at_table
  std::vector<std::vector<int>> dish_of;      // dish_of[v][t] (raw slot id)
  std::vector<View> views;
  SeqRng rng;

  // ---- multiview_gibbs.cpp:12-103 initialize_state_from_data ----
  void initialize() {
    const int tables0 = 4, dishes0 = 2;
    T = tables0;
    table_of.assign(n, 0);
    n_t.assign(T, 0);
    members.assign(T, {});
    for (int i = 0; i < n; ++i) {                                     // :25-33
      int t = (int)std::floor(rng.runif(0.0, (double)T));
      if (t < 0) t = 0;
      if (t >= T) t = T - 1;
      table_of[i] = t;
      members[t].push_back(i);
      n_t[t]++;
    }
    dish_of.assign(d, std::vector<int>(T, 0));
    views.assign(d, View());
    for (int v = 0; v < d; ++v) {
      View &W = views[v];
      W.K = dishes0;
      W.n_vk.assign(W.K, 0);
      W.l_vk.assign(W.K, 0);
      W.sum_y.assign(W.K, 0.0);
      W.sum_y2.assign(W.K, 0.0);
      for (int t = 0; t < T; ++t) {                                   // :55-62
        int k = (int)std::floor(rng.runif(0.0, (double)W.K));
        if (k < 0) k = 0;
        if (k >= W.K) k = W.K - 1;
        dish_of[v][t] = k;
        W.l_vk[k]++;
      }
      for (int i = 0; i < n; ++i) {                                   // :64-73
        const int k = dish_of[v][table_of[i]];
        const double val = y[v][i];
        W.n_vk[k]++;
        W.sum_y[k] += val;
        W.sum_y2[k] += val * val;
      }
      W.alpha_v = 1.0;                                                // :75-76
      W.sigma_v = 0.5;
      double s1 = 0.0;                                                // :78-94
      for (int i = 0; i < n; ++i) s1 += y[v][i];
      const double mean = s1 / std::max(1, n);
      double var = 0.0;
      if (n > 1) {
        for (int i = 0; i < n; ++i) {
          const double diff = y[v][i] - mean;
          var += diff * diff;
        }
        var /= (n - 1);
      } else {
        var = 1.0;
      }
      if (var <= 0.0) var = 1.0;
      W.tau_v = var * 0.25 * 0.01;
    }
    alpha_global = 1;                                                 // :97-98
    sigma_global = 0.6;
  }

  // Warm start (mvc_sampler_set_state): tables at positions, raw dish ids,
  // sufficient statistics as ascending-i sums (the init order :64-73).
  void load_state(const int *tab, int T_, const int *dish_raw, const double *hyper) {
    T = T_;
    table_of.assign(tab, tab + n);
    n_t.assign(T, 0);
    members.assign(T, {});
    for (int i = 0; i < n; ++i) { n_t[table_of[i]]++; members[table_of[i]].push_back(i); }
    dish_of.assign(d, std::vector<int>(T));
    views.assign(d, View());
    for (int v = 0; v < d; ++v) {
      View &W = views[v];
      int mx = 0;
      for (int t = 0; t < T; ++t) { dish_of[v][t] = dish_raw[(size_t)v * T + t]; mx = std::max(mx, dish_of[v][t]); }
      W.K = mx + 1;
      W.n_vk.assign(W.K, 0); W.l_vk.assign(W.K, 0);
      W.sum_y.assign(W.K, 0.0); W.sum_y2.assign(W.K, 0.0);
      for (int t = 0; t < T; ++t) W.l_vk[dish_of[v][t]]++;
      for (int i = 0; i < n; ++i) {
        const int k = dish_of[v][table_of[i]];
        const double val = y[v][i];
        W.n_vk[k]++;
        W.sum_y[k] += val;
        W.sum_y2[k] += val * val;
      }
      W.tau_v = hyper[v];
      W.alpha_v = hyper[d + v];
      W.sigma_v = hyper[2 * d + v];
    }
    alpha_global = hyper[3 * d];
    sigma_global = hyper[3 * d + 1];
  }

  // ---- multiview_utils.cpp:307-338 compute_f_vk ----
  double f_vk(int v, int k, int i) const {
    const View &W = views[v];
    const double yvi = y[v][i];
    const double tau = W.tau_v;
    const int nk = W.n_vk[k];
    const double S1 = W.sum_y[k];
    const double S2 = W.sum_y2[k];
    const double term1_old = -0.5 * S2 / tau;
    const double term2_old = 0.5 * (S1 * S1) / (tau * (tau + nk));
    const double log_det_old = -0.5 * nk * Math::log(2.0 * MVC_PI * tau)
                               - 0.5 * Math::log(tau * (tau + nk));
    const int n_new = nk + 1;
    const double S1_new = S1 + yvi;
    const double S2_new = S2 + yvi * yvi;
    const double term1_new = -0.5 * S2_new / tau;
    const double term2_new = 0.5 * (S1_new * S1_new) / (tau * (tau + n_new));
    const double log_det_new = -0.5 * n_new * Math::log(2.0 * MVC_PI * tau)
                               - 0.5 * Math::log(tau * (tau + n_new));
    const double lp = (log_det_new + term1_new + term2_new) -
                      (log_det_old + term1_old + term2_old);
    return Math::exp(lp);
  }

  // ---- multiview_utils.cpp:340-350 compute_f_vk_new ----
  double f_new(int v, int i) const {
    const double yvi = y[v][i];
    const double tau = views[v].tau_v;
    const double log_norm = -0.5 * Math::log(2.0 * MVC_PI * tau);
    const double log_exp = -0.5 * (yvi * yvi) / tau;
    return Math::exp(log_norm + log_exp);
  }

  // ---- multiview_utils.cpp:40-69 compute_marginal_likelihood_new_table ----
  double marg_new_table(int v, int i) const {
    const View &W = views[v];
    double total = 0.0;
    for (int c : W.l_vk) total += c;
    const double denom = W.alpha_v + total;
    if (denom <= 0.0) return f_new(v, i);
    double acc = 0.0;
    int K_active = 0;
    for (int k = 0; k < W.K; ++k) {
      if (W.l_vk[k] > 0) {
        K_active++;
        double w = (W.l_vk[k] - W.sigma_v);
        if (w < 0.0) w = 0.0;
        acc += w * f_vk(v, k, i);
      }
    }
    double w_new = (W.alpha_v + K_active * W.sigma_v);
    if (w_new < 0.0) w_new = 0.0;
    acc += w_new * f_new(v, i);
    return acc / denom;
  }

  // ---- multiview_utils.cpp:71-136 compute_table_probs_with_cache ----
  // The per-customer cache (reference: unordered_map per view, cleared per
  // customer, :77-79) only memoises f_vk; here a stamped vector per view.
  std::vector<std::vector<double>> cache_val;
  std::vector<std::vector<int64_t>> cache_stamp;
  int64_t stamp = 0;
  double cached_f(int v, int k, int i) {
    if ((int)cache_val[v].size() < views[v].K) {
      cache_val[v].resize(views[v].K);
      cache_stamp[v].resize(views[v].K, -1);
    }
    if (cache_stamp[v][k] != stamp) {
      cache_val[v][k] = f_vk(v, k, i);
      cache_stamp[v][k] = stamp;
    }
    return cache_val[v][k];
  }
  int64_t uf_tables = 0, uf_customers = 0, uf_new = 0, fallback = 0;   // underflow counters (Result traces)
  void table_probs(int i, std::vector<double> &p, double &p_new) {
    ++stamp;
    int64_t uf_here = 0;
    if ((int)cache_val.size() != d) { cache_val.assign(d, {}); cache_stamp.assign(d, {}); }
    for (int t = 0; t < T; ++t) {
      if (n_t[t] == 0) { p[t] = 0.0; continue; }
      double lpt = 0.0;
      for (int v = 0; v < d; ++v) lpt += Math::log(cached_f(v, dish_of[v][t], i));
      const double mass = n_t[t] - sigma_global;
      p[t] = (mass <= 0.0) ? 0.0 : mass * Math::exp(lpt);
      if (mass > 0.0 && p[t] == 0.0) ++uf_here;
    }
    uf_tables += uf_here;
    uf_customers += uf_here > 0 ? 1 : 0;
    double lnew = 0.0;
    for (int v = 0; v < d; ++v) lnew += Math::log(marg_new_table(v, i));
    int T_ne = 0;
    for (int t = 0; t < T; ++t)
      if (n_t[t] > 0) ++T_ne;
    const double mass_new = alpha_global + sigma_global * T_ne;
    p_new = (mass_new <= 0.0) ? 0.0 : mass_new * Math::exp(lnew);
    if (mass_new > 0.0 && p_new == 0.0) ++uf_new;
  }

  // ---- multiview_utils.cpp:138-192 remove_customer ----
  void remove_customer(int i) {
    const int t = table_of[i];
    if (t < 0 || t >= T) throw std::runtime_error("remove_customer: invalid table");
    auto &lst = members[t];
    auto it = std::find(lst.begin(), lst.end(), i);
    if (it == lst.end()) throw std::runtime_error("customer not at table");
    std::swap(*it, lst.back());
    lst.pop_back();
    n_t[t]--;
    for (int v = 0; v < d; ++v) {
      const int k = dish_of[v][t];
      View &W = views[v];
      W.n_vk[k]--;
      W.sum_y[k] -= y[v][i];
      W.sum_y2[k] -= y[v][i] * y[v][i];
    }
    table_of[i] = -1;
    if (n_t[t] == 0) {
      for (int v = 0; v < d; ++v) {
        const int k = dish_of[v][t];
        if (k >= 0 && views[v].l_vk[k] > 0) views[v].l_vk[k]--;
      }
      const int last = T - 1;
      if (t != last) {                    // swap-and-pop relabel :175-185
        members[t] = std::move(members[last]);
        n_t[t] = n_t[last];
        for (int v = 0; v < d; ++v) dish_of[v][t] = dish_of[v][last];
        for (int j : members[t]) table_of[j] = t;
      }
      members.pop_back();
      n_t.pop_back();
      for (int v = 0; v < d; ++v) dish_of[v].pop_back();
      T--;
    }
  }

  // ---- multiview_utils.cpp:194-222 ----
  void add_existing(int i, int t) {
    table_of[i] = t;
    members[t].push_back(i);
    n_t[t]++;
    for (int v = 0; v < d; ++v) {
      const int k = dish_of[v][t];
      View &W = views[v];
      W.n_vk[k]++;
      W.sum_y[k] += y[v][i];
      W.sum_y2[k] += y[v][i] * y[v][i];
    }
  }
  int create_empty_table() {
    const int t = T;
    T++;
    n_t.push_back(0);
    members.emplace_back();
    for (int v = 0; v < d; ++v) dish_of[v].push_back(-1);
    return t;
  }
  void add_new_table(int i, int t) {
    table_of[i] = t;
    members[t].push_back(i);
    n_t[t] = 1;
  }

  // ---- multiview_utils.cpp:224-276 sample_dish_for_new_table ----
  int fresh_dish(View &W) {
    const int k = W.K;
    W.K++;
    W.n_vk.push_back(0);
    W.l_vk.push_back(0);
    W.sum_y.push_back(0.0);
    W.sum_y2.push_back(0.0);
    return k;
  }
  int sample_dish(int v, int i) {
    View &W = views[v];
    std::vector<double> w;
    std::vector<int> cand;
    for (int k = 0; k < W.K; ++k) {
      if (W.l_vk[k] > 0) {
        double x = (W.l_vk[k] - W.sigma_v) * f_vk(v, k, i);
        if (x < 0) x = 0;
        w.push_back(x);
        cand.push_back(k);
      }
    }
    const int K_active = (int)cand.size();
    double x_new = (W.alpha_v + W.sigma_v * K_active) * f_new(v, i);
    if (x_new < 0) x_new = 0;
    w.push_back(x_new);
    double total = 0;
    for (double x : w) total += x;
    if (total <= 0) return fresh_dish(W);
    const double u = rng.runif(0.0, total);
    double cum = 0;
    for (size_t j = 0; j < cand.size(); ++j) {
      cum += w[j];
      if (u < cum) return cand[j];
    }
    return fresh_dish(W);
  }
  // ---- multiview_utils.cpp:278-289 ----
  void assign_dishes(int i, int t) {
    for (int v = 0; v < d; ++v) {
      const int k = sample_dish(v, i);
      dish_of[v][t] = k;
      View &W = views[v];
      W.l_vk[k]++;
      W.n_vk[k]++;
      W.sum_y[k] += y[v][i];
      W.sum_y2[k] += y[v][i] * y[v][i];
    }
  }

  // ---- multiview_hyper.cpp ----
  static double prior_alpha(double a) {                               // :344-351
    if (a <= 0.0) return -INFINITY;
    return (4.0 - 1.0) * Math::log(a) - 3.0 * a;
  }
  static double prior_sigma(double s) {                               // :353-360
    if (s <= 0.0 || s >= 1.0) return -INFINITY;
    return (1.0 - 1.0) * Math::log(s) + (5.0 - 1.0) * Math::log(1.0 - s);
  }
  double log_eppf_view(int v, double alpha, double sigma) const {     // :295-342
    if (v < 0 || v >= d) return -INFINITY;
    if (!(sigma > kEps && sigma < 1.0 - kEps)) return -INFINITY;
    if (alpha <= -sigma) return -INFINITY;
    const View &W = views[v];
    std::vector<int> sizes;
    int total = 0;
    for (int c : W.l_vk)
      if (c > 0) { sizes.push_back(c); total += c; }
    if (total == 0) return 0.0;
    double lp = 0.0;
    const int K_active = (int)sizes.size();
    for (int j = 0; j < K_active; ++j) {
      const double term = alpha + j * sigma;
      if (term <= 0.0) return -INFINITY;
      lp += Math::log(term);
    }
    for (int i = 1; i < total; ++i) {
      const double term = alpha + i;
      if (term <= 0.0) return -INFINITY;
      lp -= Math::log(term);
    }
    for (int lk : sizes)
      for (int m = 1; m < lk; ++m) {
        const double term = (double)m - sigma;
        if (term <= 0.0) return -INFINITY;
        lp += Math::log(term);
      }
    return lp;
  }
  double log_eppf_global(double alpha, double sigma) const {          // :53-83
    if (!(sigma > kEps && sigma < 1.0 - kEps)) return -INFINITY;
    if (alpha <= -sigma) return -INFINITY;
    if (T <= 0 || n_t.empty()) return 0.0;
    double lp = 0.0;
    for (int j = 0; j < T; ++j) {
      const double term = alpha + j * sigma;
      if (term <= 0.0) return -INFINITY;
      lp += Math::log(term);
    }
    for (int i = 1; i < n; ++i) {
      const double term = alpha + i;
      if (term <= 0.0) return -INFINITY;
      lp -= Math::log(term);
    }
    for (int c : n_t)
      for (int m = 1; m < c; ++m) {
        const double term = (double)m - sigma;
        if (term <= 0.0) return -INFINITY;
        lp += Math::log(term);
      }
    return lp;
  }
  double post_alpha_view(int v, double a) const {                     // :34-41
    if (a <= 0.0) return -INFINITY;
    return log_eppf_view(v, a, views[v].sigma_v) + prior_alpha(a);
  }
  double post_sigma_view(int v, double s) const {                     // :43-51
    if (s <= kEps || s >= 1.0 - kEps) return -INFINITY;
    return log_eppf_view(v, views[v].alpha_v, s) + prior_sigma(s);
  }
  double post_alpha_global(double a) const {                          // :86-90
    return log_eppf_global(a, sigma_global) + prior_alpha(a);
  }
  double post_sigma_global(double s) const {                          // :92-98
    if (s <= kEps || s >= 1.0 - kEps) return -INFINITY;
    return log_eppf_global(alpha_global, s) + prior_sigma(s);
  }
  double propose_alpha(double a_old) {                                // :100-108
    double la = Math::log(std::max(a_old, kEps));
    la += rng.rnorm(0.0, 0.1);
    const double c = Math::exp(la);
    return (c > kEps) ? c : kEps;
  }
  static double reflect_unit(double value) {                          // :110-122
    double p = value;
    while (p <= kEps || p >= 1.0 - kEps) {
      if (p <= kEps) p = 2.0 * kEps - p;
      if (p >= 1.0 - kEps) p = 2.0 * (1.0 - kEps) - p;
    }
    return std::clamp(p, kEps, 1.0 - kEps);
  }
  double propose_sigma(double s_old) {                                // :124-128
    return reflect_unit(s_old + rng.rnorm(0.0, 0.05));
  }
  double post_tau(int v, double tau) const {                          // :176-209
    const View &W = views[v];
    if (tau <= 0.0) return -INFINITY;
    double ll = 0.0;
    for (int k = 0; k < W.K; ++k) {
      const int nk = W.n_vk[k];
      if (nk == 0) continue;
      double sse = W.sum_y2[k] - (W.sum_y[k] * W.sum_y[k]) / (double)nk;
      if (sse < 0.0) sse = 0.0;
      ll += -0.5 * nk * Math::log(2.0 * MVC_PI * tau) - 0.5 * (sse / tau);
    }
    const double a_tau = 2.0, b_tau = 1.0;
    // lgamma(2) == 0 exactly (glibc and the definition)
    const double prior = a_tau * Math::log(b_tau) - 0.0 - (a_tau + 1.0) * Math::log(tau)
                         - b_tau / tau;
    return ll + prior;
  }
  void update_tau() {                                                 // :211-231
    for (int v = 0; v < d; ++v) {
      View &W = views[v];
      double t_old = W.tau_v;
      if (t_old <= 0.0) t_old = kEps;
      const double l_old = post_tau(v, t_old);
      const double t_prop = Math::exp(Math::log(t_old) + rng.rnorm(0.0, 0.3)); // :166-174
      if (t_prop <= 0.0) continue;
      const double l_new = post_tau(v, t_prop);
      const double lq = Math::log(t_prop) - Math::log(t_old);
      const double acc = (l_new - l_old) + lq;
      if (Math::log(rng.unif_rand()) < acc) W.tau_v = t_prop;
    }
  }
  void update_hyper() {                                               // :233-292
    update_tau();
    for (int v = 0; v < d; ++v) {
      View &W = views[v];
      double a_old = W.alpha_v;
      if (a_old <= 0.0) a_old = kEps;
      const double a_prop = propose_alpha(a_old);
      const double lo = post_alpha_view(v, a_old);
      const double ln = post_alpha_view(v, a_prop);
      const double lq = Math::log(a_prop) - Math::log(a_old);
      if (Math::log(rng.unif_rand()) < (ln - lo) + lq) W.alpha_v = a_prop;
      const double s_old = W.sigma_v;
      const double s_prop = propose_sigma(s_old);
      const double u = rng.unif_rand();
      if (Math::log(u) < post_sigma_view(v, s_prop) - post_sigma_view(v, s_old)) W.sigma_v = s_prop;
    }
    double ag_old = alpha_global;
    if (ag_old <= 0.0) ag_old = kEps;
    const double ag_prop = propose_alpha(ag_old);
    const double lo = post_alpha_global(ag_old);
    const double ln = post_alpha_global(ag_prop);
    const double lq = Math::log(ag_prop) - Math::log(ag_old);
    if (Math::log(rng.unif_rand()) < (ln - lo) + lq) alpha_global = ag_prop;
    const double sg_old = sigma_global;
    const double sg_prop = propose_sigma(sg_old);
    const double u = rng.unif_rand();
    if (Math::log(u) < post_sigma_global(sg_prop) - post_sigma_global(sg_old)) sigma_global = sg_prop;
  }

  void save(Result &R) const {                                        // utils.cpp:291-303
    R.table_of.insert(R.table_of.end(), table_of.begin(), table_of.end());
    R.sample_T.push_back(T);
    for (int v = 0; v < d; ++v) R.dish_of.insert(R.dish_of.end(), dish_of[v].begin(), dish_of[v].end());
    R.dish_off.push_back((int64_t)R.dish_of.size());
    for (int v = 0; v < d; ++v) {
      R.alpha_v.push_back(views[v].alpha_v);
      R.sigma_v.push_back(views[v].sigma_v);
      R.tau_v.push_back(views[v].tau_v);
    }
    R.alpha_g.push_back(alpha_global);
    R.sigma_g.push_back(sigma_global);
    R.S++;
  }

  // ---- multiview_gibbs.cpp:134-212 gibbs_sampler ----
  void run(int M, int burn_in, int thin, Result &R) {
    R.dish_off.push_back(0);
    std::vector<double> p;
    for (int iter = 0; iter < M; ++iter) {
      for (int i = 0; i < n; ++i) {
        remove_customer(i);
        p.assign(T, 0.0);
        double p_new = 0.0;
        table_probs(i, p, p_new);
        double sum_p = p_new;
        for (int t = 0; t < T; ++t) sum_p += p[t];
        if (sum_p <= 0.0) { ++fallback; add_existing(i, 0); continue; }
        for (int t = 0; t < T; ++t) p[t] /= sum_p;
        p_new /= sum_p;
        const double u = rng.unif_rand();
        double cum = 0.0;
        int t_star = -1;
        for (int t = 0; t < T; ++t) {
          cum += p[t];
          if (u < cum) { t_star = t; break; }
        }
        if (t_star == -1) {
          const int t_new = create_empty_table();
          add_new_table(i, t_new);
          assign_dishes(i, t_new);
        } else {
          add_existing(i, t_star);
        }
      }
      update_hyper();
      R.trace_T.push_back(T);
      R.trace_draws.push_back(rng.draws);
      R.trace_fallback.push_back(fallback);
      R.trace_uf_tables.push_back(uf_tables);
      R.trace_uf_customers.push_back(uf_customers);
      R.trace_uf_new.push_back(uf_new);
      fallback = uf_tables = uf_customers = uf_new = 0;
      if (iter >= burn_in && ((iter - burn_in) % thin == 0)) save(R);
    }
  }
};

// ===========================================================================
// tree64: the fixed reduction order of the parallel mode.
// 64-slot butterfly (pairs l, l+h for h = 32..1, zero padded) per chunk of
// 64 consecutive elements, applied recursively to the chunk partials.
// ===========================================================================
static double butterfly64(const double *x, size_t n) {
  double s[64];
  for (size_t l = 0; l < 64; ++l) s[l] = l < n ? x[l] : 0.0;
  for (int h = 32; h >= 1; h >>= 1)
    for (int l = 0; l < h; ++l) s[l] = s[l] + s[l + h];
  return s[0];
}

struct Tree64 {
  std::vector<std::vector<double>> lv;   // lv[0] = leaves, lv[k+1] = chunk sums of lv[k]
  double build(const std::vector<double> &x) {
    lv.clear();
    if (x.empty()) return 0.0;
    lv.push_back(x);
    do {
      const std::vector<double> &cur = lv.back();
      const size_t m = (cur.size() + 63) / 64;
      std::vector<double> nxt(m);
      for (size_t c = 0; c < m; ++c) {
        const size_t base = c * 64;
        nxt[c] = butterfly64(cur.data() + base, std::min<size_t>(64, cur.size() - base));
      }
      lv.push_back(std::move(nxt));
    } while (lv.back().size() > 1);
    return lv.back()[0];
  }
  // Descent inside one 64-slot chunk; r relative to the chunk sum.
  static int select_chunk(const double *x, size_t n, double &r) {
    double lvl[7][64];
    for (size_t l = 0; l < 64; ++l) lvl[6][l] = l < n ? x[l] : 0.0;
    int k = 6;
    for (int h = 32; h >= 1; h >>= 1, --k)
      for (int l = 0; l < h; ++l) lvl[k - 1][l] = lvl[k][l] + lvl[k][l + h];
    // node (level index k, position l) with h = 2^k, children at level k+1: l and l+h
    int l = 0;
    for (int kk = 0, h = 1; kk < 6; ++kk, h <<= 1) {
      const double a = lvl[kk + 1][l];
      const double b = lvl[kk + 1][l + h];
      if (b == 0.0 || r < a) {
        // left
      } else {
        r = r - a;
        l = l + h;
      }
    }
    return l;
  }
  // Select a leaf for target r (0 <= r < total).  Requires build() first.
  size_t select(double r) const {
    size_t idx = 0;   // chunk index at the current level
    for (int k = (int)lv.size() - 2; k >= 0; --k) {
      const std::vector<double> &cur = lv[k];
      const size_t base = idx * 64;
      const size_t cnt = std::min<size_t>(64, cur.size() - base);
      const int l = select_chunk(cur.data() + base, cnt, r);
      idx = base + (size_t)l;
    }
    return idx;
  }
};

// pw16: pairwise tree over 16 slots, pairs (c, c + h) for h = 1, 2, 4, 8 (the
// wavefront's xor butterfly across one 16-lane DPP row)
static double pw16(const double *x) {
  double a[16];
  for (int c = 0; c < 16; ++c) a[c] = x[c];
  for (int h = 1; h < 16; h <<= 1)
    for (int c = 0; c < 16; c += 2 * h) a[c] = a[c] + a[c + h];
  return a[0];
}

// Descent through the pw16 tree: at a node with halves (L, R) go left iff
// R == 0 || r < L, else r -= L.  The half sums are the tree's own partials.
static int pw16_select(const double *x, double r) {
  double lv[5][16];
  for (int c = 0; c < 16; ++c) lv[0][c] = x[c];
  for (int k = 0, h = 1; k < 4; ++k, h <<= 1)
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

static double tree64_sum(const std::vector<double> &x) {
  Tree64 t;
  return t.build(x);
}

// ===========================================================================
// ParallelSampler: the parallel-z schedule ("mode P").
// ===========================================================================
struct ParallelSampler {
  int n = 0, V = 0, D = 0;
  const double *y = nullptr;                 // [V][n][D]
  std::vector<double> Y2;                    // [V][n]  fma-chain sum_d y^2
  uint64_t seed = 0;
  uint32_t chain = 0;
  // hyper
  std::vector<double> tau, alpha, sigma;
  double ag = 1.0, sg = 0.6;
  // tables (positions)
  int T = 0;
  std::vector<int> z, n_t;                   // z[i] = position
  std::vector<std::vector<int>> dish;        // dish[v][p] = live index
  // dishes per view (live list, ascending raw id)
  std::vector<std::vector<int>> ids, nk, lk;
  std::vector<std::vector<double>> S1;       // [v][j*D + d]
  std::vector<std::vector<double>> S2;       // [v][j]
  std::vector<int> next_id;
  SeqRng init_rng;

  double yv(int v, int i, int d) const { return y[((size_t)v * n + i) * D + d]; }

  static double fma_dot(const double *a, const double *b, int D) {
    double acc = 0.0;
    for (int d = 0; d < D; ++d) acc = __builtin_fma(a[d], b[d], acc);
    return acc;
  }

  // chunked ordered rebuild of n, S1, S2 from z/dish
  void rebuild_stats() {
    for (int v = 0; v < V; ++v) rebuild_view(v);
  }

  // chunked ordered rebuild of one view
  void rebuild_view(int v) {
    {
      const int K = (int)ids[v].size();
      nk[v].assign(K, 0);
      S1[v].assign((size_t)K * D, 0.0);
      S2[v].assign(K, 0.0);
      std::vector<double> part1((size_t)K * D), part2(K);
      for (int c0 = 0; c0 < n; c0 += kStatsChunk) {
        const int c1 = std::min(n, c0 + kStatsChunk);
        std::fill(part1.begin(), part1.end(), 0.0);
        std::fill(part2.begin(), part2.end(), 0.0);
        for (int i = c0; i < c1; ++i) {
          const int j = dish[v][z[i]];
          for (int d = 0; d < D; ++d) part1[(size_t)j * D + d] = part1[(size_t)j * D + d] + yv(v, i, d);
          part2[j] = part2[j] + Y2[(size_t)v * n + i];
        }
        for (size_t e = 0; e < part1.size(); ++e) S1[v][e] = S1[v][e] + part1[e];
        for (int j = 0; j < K; ++j) S2[v][j] = S2[v][j] + part2[j];
      }
      for (int i = 0; i < n; ++i) nk[v][dish[v][z[i]]]++;
    }
  }

  void initialize() {
    Y2.assign((size_t)V * n, 0.0);
    for (int v = 0; v < V; ++v)
      for (int i = 0; i < n; ++i) {
        const double *r = y + ((size_t)v * n + i) * D;
        Y2[(size_t)v * n + i] = fma_dot(r, r, D);
      }
    // same draws as multiview_gibbs.cpp:12-62 on the sequential stream
    T = 4;
    z.assign(n, 0);
    n_t.assign(T, 0);
    for (int i = 0; i < n; ++i) {
      int t = (int)std::floor(init_rng.runif(0.0, (double)T));
      if (t < 0) t = 0;
      if (t >= T) t = T - 1;
      z[i] = t;
      n_t[t]++;
    }
    dish.assign(V, std::vector<int>(T, 0));
    ids.assign(V, {}); nk.assign(V, {}); lk.assign(V, {});
    S1.assign(V, {}); S2.assign(V, {});
    next_id.assign(V, 2);
    tau.assign(V, 1.0); alpha.assign(V, 1.0); sigma.assign(V, 0.5);
    for (int v = 0; v < V; ++v) {
      int raw[4];
      int l2[2] = {0, 0};
      for (int t = 0; t < T; ++t) {
        int k = (int)std::floor(init_rng.runif(0.0, 2.0));
        if (k < 0) k = 0;
        if (k >= 2) k = 1;
        raw[t] = k;
        l2[k]++;
      }
      // live list = raw ids with l > 0, ascending
      int map2[2] = {-1, -1};
      for (int k = 0; k < 2; ++k)
        if (l2[k] > 0) { map2[k] = (int)ids[v].size(); ids[v].push_back(k); lk[v].push_back(l2[k]); }
      for (int t = 0; t < T; ++t) dish[v][t] = map2[raw[t]];
      // tau: multiview_gibbs.cpp:78-94, averaged over the D dims
      double vsum = 0.0;
      for (int d = 0; d < D; ++d) {
        double s1 = 0.0;
        for (int i = 0; i < n; ++i) s1 += yv(v, i, d);
        const double mean = s1 / std::max(1, n);
        double var = 0.0;
        if (n > 1) {
          for (int i = 0; i < n; ++i) { const double df = yv(v, i, d) - mean; var += df * df; }
          var /= (n - 1);
        } else {
          var = 1.0;
        }
        if (var <= 0.0) var = 1.0;
        vsum += var;
      }
      const double var = vsum / (double)D;
      tau[v] = var * 0.25 * 0.01;
    }
    ag = 1.0;
    sg = 0.6;
    rebuild_stats();
  }

  void load_state(const int *tab, int T_, const int *dish_raw, const double *hyper) {
    Y2.assign((size_t)V * n, 0.0);
    for (int v = 0; v < V; ++v)
      for (int i = 0; i < n; ++i) {
        const double *r = y + ((size_t)v * n + i) * D;
        Y2[(size_t)v * n + i] = fma_dot(r, r, D);
      }
    load_partition(tab, T_, dish_raw, hyper);
    rebuild_stats();
  }

  // the partition and hyperparameters of load_state (no statistics)
  void load_partition(const int *tab, int T_, const int *dish_raw, const double *hyper) {
    T = T_;
    z.assign(tab, tab + n);
    n_t.assign(T, 0);
    for (int i = 0; i < n; ++i) n_t[z[i]]++;
    dish.assign(V, std::vector<int>(T));
    ids.assign(V, {}); nk.assign(V, {}); lk.assign(V, {});
    S1.assign(V, {}); S2.assign(V, {});
    next_id.assign(V, 0);
    tau.assign(V, 0.0); alpha.assign(V, 0.0); sigma.assign(V, 0.0);
    for (int v = 0; v < V; ++v) {
      std::vector<int> raw(dish_raw + (size_t)v * T, dish_raw + (size_t)(v + 1) * T);
      std::vector<int> srt = raw;
      std::sort(srt.begin(), srt.end());
      srt.erase(std::unique(srt.begin(), srt.end()), srt.end());
      ids[v] = srt;
      lk[v].assign(srt.size(), 0);
      for (int p = 0; p < T; ++p) {
        const int j = (int)(std::lower_bound(srt.begin(), srt.end(), raw[p]) - srt.begin());
        dish[v][p] = j;
        lk[v][j]++;
      }
      next_id[v] = srt.back() + 1;
      tau[v] = hyper[v];
      alpha[v] = hyper[V + v];
      sigma[v] = hyper[2 * V + v];
    }
    ag = hyper[3 * V];
    sg = hyper[3 * V + 1];
  }

  struct Coef { double c0, cb; };
  Coef coef(int n_, double Q, double tau_v, double L2pt) const {
    const double a = tau_v + (double)n_;
    const double b = tau_v + (double)(n_ + 1);
    Coef c;
    c.c0 = (double)D * ((-0.5 * L2pt) - 0.5 * mvc_log(b / a)) - (0.5 * Q) / ((tau_v * a) * b);
    c.cb = 1.0 / (tau_v * b);
    return c;
  }

  // per-view per-customer element list of the marginal mixture
  struct ViewEval {
    std::vector<double> lv;     // element log values, size K+1 (last = new dish)
    std::vector<double> w;      // weights
    std::vector<char> inc;      // included
    double m = 0.0;             // max over included
    std::vector<double> leaves; // inc ? w*exp(lv-m) : 0
    double S = 0.0;             // tree64(leaves)
    double lmarg = 0.0;
  };

  // shared per-sweep constants
  std::vector<std::vector<double>> Qd;        // [v][j]
  std::vector<std::vector<Coef>> cf;          // [v][j]
  std::vector<double> L2pt, cnew;             // [v]
  std::vector<int> Ltot;                      // [v]
  int T_ne = 0;

  void sweep_constants() {
    Qd.assign(V, {}); cf.assign(V, {});
    L2pt.assign(V, 0.0); cnew.assign(V, 0.0); Ltot.assign(V, 0);
    for (int v = 0; v < V; ++v) {
      const int K = (int)ids[v].size();
      L2pt[v] = mvc_log((2.0 * MVC_PI) * tau[v]);
      cnew[v] = (double)D * (-0.5 * L2pt[v]);
      Qd[v].resize(K);
      cf[v].resize(K);
      int lt = 0;
      for (int j = 0; j < K; ++j) {
        const double *s = &S1[v][(size_t)j * D];
        Qd[v][j] = fma_dot(s, s, D);
        cf[v][j] = coef(nk[v][j], Qd[v][j], tau[v], L2pt[v]);
        lt += lk[v][j];
      }
      Ltot[v] = lt;
    }
    T_ne = 0;
    for (int p = 0; p < T; ++p)
      if (n_t[p] > 0) ++T_ne;
  }

  // Dishes created earlier in the same sweep by the birth resolution
  // (DESIGN.md §4.5): per view counts and sums, extended index K_v + q.
  struct Phase2 {
    int T2 = 0;
    std::vector<int> c;                       // [t] customers
    std::vector<std::vector<int>> tup;        // [t][v] extended dish index
    std::vector<std::vector<int>> n2, l2;     // [v][q]
    std::vector<std::vector<double>> S1_2;    // [v][q*D + d]
  };

  void eval_view(int i, int v, bool alive, int j0, ViewEval &E, const Phase2 *P2 = nullptr) const {
    const int K = (int)ids[v].size();
    const int K2 = P2 ? (int)P2->n2[v].size() : 0;
    const int NE = K + K2;
    const double Y2i = Y2[(size_t)v * n + i];
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau[v];
    const double *yi = y + ((size_t)v * n + i) * D;
    E.lv.assign(NE + 1, 0.0); E.w.assign(NE + 1, 0.0); E.inc.assign(NE + 1, 0);
    int Kact = K;
    for (int j = 0; j < K; ++j) {
      const double G = fma_dot(yi, &S1[v][(size_t)j * D], D);
      int l = lk[v][j];
      double lp;
      if (j == j0) {
        if (!alive) l -= 1;
        const double Gp = G - Y2i;
        const double Qp = (Qd[v][j] - 2.0 * G) + Y2i;
        const Coef c = coef(nk[v][j] - 1, Qp, tau[v], L2pt[v]);
        lp = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
      } else {
        lp = __builtin_fma(G + hy, cf[v][j].cb, cf[v][j].c0) + h;
      }
      E.lv[j] = lp;
      if (l > 0) {
        E.inc[j] = 1;
        double w = (double)l - sigma[v];
        if (w < 0.0) w = 0.0;
        E.w[j] = w;
      } else {
        Kact -= 1;
      }
    }
    int L2sum = 0;
    for (int q = 0; q < K2; ++q) {
      const double *s2 = &P2->S1_2[v][(size_t)q * D];
      const double G = fma_dot(yi, s2, D);
      const double Q = fma_dot(s2, s2, D);
      const Coef c = coef(P2->n2[v][q], Q, tau[v], L2pt[v]);
      E.lv[K + q] = __builtin_fma(G + hy, c.cb, c.c0) + h;
      E.inc[K + q] = 1;
      double w = (double)P2->l2[v][q] - sigma[v];
      if (w < 0.0) w = 0.0;
      E.w[K + q] = w;
      L2sum += P2->l2[v][q];
    }
    E.lv[NE] = cnew[v] + h;
    double wn = alpha[v] + (double)(Kact + K2) * sigma[v];
    if (wn < 0.0) wn = 0.0;
    E.w[NE] = wn;
    E.inc[NE] = 1;
    double m = -MVC_PM_INF;
    for (int e = 0; e <= NE; ++e)
      if (E.inc[e] && E.lv[e] > m) m = E.lv[e];
    E.m = m;
    E.leaves.assign(NE + 1, 0.0);
    for (int e = 0; e <= NE; ++e)
      if (E.inc[e]) E.leaves[e] = E.w[e] * mvc_exp(E.lv[e] - m);
    E.S = tree64_sum(E.leaves);
    const double denom = alpha[v] + (double)((Ltot[v] - (alive ? 0 : 1)) + L2sum);
    if (denom <= 0.0)
      E.lmarg = E.lv[NE];
    else
      E.lmarg = (m + mvc_log(E.S)) - mvc_log(denom);
  }

  // Phase 1 per-view marginal: sequential reductions in
  // dish order, so one GPU lane can own one customer.  lp of every dish goes
  // to lp_out[0..K); returns lm_v.
  double eval_view_seq(int i, int v, bool alive, int j0, double *lp_out) const {
    return eval_view_seq_r(y + ((size_t)v * n + i) * D, Y2[(size_t)v * n + i], v, alive, j0, lp_out);
  }
  // the same for a customer whose view-v row is yi with sum of squares Y2i
  double eval_view_seq_r(const double *yi, double Y2i, int v, bool alive, int j0, double *lp_out) const {
    const int K = (int)ids[v].size();
    const double hy = 0.5 * Y2i;
    const double h = (-0.5 * Y2i) / tau[v];
    int l0p = 0;
    for (int j = 0; j < K; ++j) {
      const double G = fma_dot(yi, &S1[v][(size_t)j * D], D);
      if (j == j0) {
        l0p = lk[v][j] - (alive ? 0 : 1);
        const double Gp = G - Y2i;
        const double Qp = (Qd[v][j] - 2.0 * G) + Y2i;
        const Coef c = coef(nk[v][j] - 1, Qp, tau[v], L2pt[v]);
        lp_out[j] = __builtin_fma(Gp + hy, c.cb, c.c0) + h;
      } else {
        lp_out[j] = __builtin_fma(G + hy, cf[v][j].cb, cf[v][j].c0) + h;
      }
    }
    const double lfn = cnew[v] + h;
    // max over included dishes (l' > 0) in dish order, then the new dish
    double m = -MVC_PM_INF;
    for (int j = 0; j < K; ++j) {
      const int l = (j == j0) ? l0p : lk[v][j];
      if (l > 0 && lp_out[j] > m) m = lp_out[j];
    }
    if (lfn > m) m = lfn;
    // sum of w * exp(lp - m): column partials (dish j -> column j mod 16,
    // sequential in ascending j), then the pairwise tree over the 16 columns
    // (pw16), then the new dish
    double col[16] = {0.0};
    for (int j = 0; j < K; ++j) {
      const int l = (j == j0) ? l0p : lk[v][j];
      if (l > 0) {
        double w = (double)l - sigma[v];
        if (w < 0.0) w = 0.0;
        col[j & 15] = col[j & 15] + w * mvc_exp(lp_out[j] - m);
      }
    }
    double S = pw16(col);
    // K_act: dishes with l' > 0 (mid-sweep the sequential schedule keeps
    // dishes that died this sweep in the list with l = 0)
    int Kact = 0;
    for (int j = 0; j < K; ++j)
      if (((j == j0) ? l0p : lk[v][j]) > 0) ++Kact;
    double wn = alpha[v] + (double)Kact * sigma[v];
    if (wn < 0.0) wn = 0.0;
    S = S + wn * mvc_exp(lfn - m);
    const double denom = alpha[v] + (double)(Ltot[v] - (alive ? 0 : 1));
    if (denom <= 0.0) return lfn;
    return (m + mvc_log(S)) - mvc_log(denom);
  }

  // Phase 1: table against the frozen state; -1 = birth.
  // Table weights e_p = exp(sp_p - M) (0 for excluded tables and for the
  // padding p >= T) in blocks of 16 positions; block sums B_b = pw16, running
  // block totals C_b = C_{b-1} + B_b (C_{-1} = 0); Tot = C_last,
  // W = exp(s_new - M) + Tot, r = u W.  r >= Tot is a birth; otherwise the
  // first block with r < C_b is entered with r - C_{b-1} and the leaf is the
  // pw16 descent (pw16_select) inside it.
  int resample_customer(int i, int s) const {
    std::vector<const double *> rows(V);
    std::vector<double> y2(V);
    for (int v = 0; v < V; ++v) {
      rows[v] = y + ((size_t)v * n + i) * D;
      y2[v] = Y2[(size_t)v * n + i];
    }
    return resample_rows(i, s, rows.data(), y2.data());
  }
  // resample_customer for customer i with view rows rows[v] (D doubles) and
  // their sums of squares y2[v] (checks at sizes where y is not on the host)
  int resample_rows(int i, int s, const double *const *rows, const double *y2) const {
    const int p0 = z[i];
    const bool alive = (n_t[p0] - 1) > 0;
    std::vector<std::vector<double>> lp(V);
    const int Tne_i = T_ne - (alive ? 0 : 1);
    double s_new = mvc_log(ag + sg * (double)Tne_i);
    for (int v = 0; v < V; ++v) {
      lp[v].resize(ids[v].size());
      s_new = s_new + eval_view_seq_r(rows[v], y2[v], v, alive, dish[v][p0], lp[v].data());
    }
    const int TB = (T + 15) / 16;
    std::vector<double> sc((size_t)TB * 16, -MVC_PM_INF);
    double M = -MVC_PM_INF;
    for (int p = 0; p < T; ++p) {
      const int np = n_t[p] - (p == p0 ? 1 : 0);
      const double mass = (double)np - sg;
      if (np < 1 || !(mass > 0.0)) continue;
      double sp = mvc_log(mass);
      for (int v = 0; v < V; ++v) sp = sp + lp[v][dish[v][p]];
      sc[p] = sp;
      if (sp > M) M = sp;
    }
    if (s_new > M) M = s_new;
    std::vector<double> e((size_t)TB * 16), C(TB);
    double tot = 0.0;
    for (int b = 0; b < TB; ++b) {
      for (int c = 0; c < 16; ++c) {
        const double x = sc[(size_t)b * 16 + c];
        e[(size_t)b * 16 + c] = x != -MVC_PM_INF ? mvc_exp(x - M) : 0.0;
      }
      tot = tot + pw16(&e[(size_t)b * 16]);
      C[b] = tot;
    }
    const double W = mvc_exp(s_new - M) + tot;
    double r = mvc_uniform(seed, (uint32_t)i, (uint32_t)s, chain, MVC_TAG_Z) * W;
    if (!(r < tot)) return -1;
    int b = 0;
    while (!(r < C[b])) ++b;
    r = r - (b > 0 ? C[b - 1] : 0.0);
    return b * 16 + pw16_select(&e[(size_t)b * 16], r);
  }

  // Phase 2: births in ascending customer order either join
  // a table born earlier in this sweep or open a new one with one dish per
  // view drawn from the mixture over frozen, phase-2 and brand-new dishes.
  // Returns for every birth (ascending) its phase-2 table.
  std::vector<int> resolve_births(const std::vector<int> &births, int s, Phase2 &P2) const {
    P2 = Phase2();
    P2.n2.assign(V, {}); P2.l2.assign(V, {}); P2.S1_2.assign(V, {});
    std::vector<int> btab(births.size());
    std::vector<ViewEval> E(V);
    for (size_t b = 0; b < births.size(); ++b) {
      const int i = births[b];
      const int p0 = z[i];
      const bool alive = (n_t[p0] - 1) > 0;
      for (int v = 0; v < V; ++v) eval_view(i, v, alive, dish[v][p0], E[v], &P2);
      double M = -MVC_PM_INF;
      std::vector<double> sc(P2.T2);
      for (int t = 0; t < P2.T2; ++t) {
        double st = mvc_log((double)P2.c[t] - sg);
        for (int v = 0; v < V; ++v) st = st + E[v].lv[P2.tup[t][v]];
        sc[t] = st;
        if (st > M) M = st;
      }
      const int Tne_i = T_ne - (alive ? 0 : 1);
      double s_new = mvc_log(ag + sg * (double)(Tne_i + P2.T2));
      for (int v = 0; v < V; ++v) s_new = s_new + E[v].lmarg;
      if (s_new > M) M = s_new;
      std::vector<double> e(P2.T2);
      for (int t = 0; t < P2.T2; ++t) e[t] = mvc_exp(sc[t] - M);
      Tree64 tb;
      const double B = tb.build(e);
      const double W = mvc_exp(s_new - M) + B;
      const double r = mvc_uniform(seed, (uint32_t)i, (uint32_t)s, chain, MVC_TAG_Z2) * W;
      int t;
      if (r < B) {
        t = (int)tb.select(r);
        P2.c[t] += 1;
        for (int v = 0; v < V; ++v) {
          const int K = (int)ids[v].size();
          const int ex = P2.tup[t][v];
          if (ex >= K) {
            const int q = ex - K;
            P2.n2[v][q] += 1;
            for (int d = 0; d < D; ++d)
              P2.S1_2[v][(size_t)q * D + d] = P2.S1_2[v][(size_t)q * D + d] + yv(v, i, d);
          }
        }
      } else {
        std::vector<int> tup(V);
        for (int v = 0; v < V; ++v) {
          const int K = (int)ids[v].size();
          const int K2 = (int)P2.n2[v].size();
          int ex;
          if (!(E[v].S > 0.0)) {
            ex = K + K2;
          } else {
            Tree64 td;
            td.build(E[v].leaves);
            const double rv = mvc_uniform(seed, (uint32_t)i, (uint32_t)s, chain, MVC_TAG_DISH + 1u + (uint32_t)v) * E[v].S;
            ex = (int)td.select(rv);
          }
          if (ex == K + K2) {
            P2.n2[v].push_back(0);
            P2.l2[v].push_back(0);
            P2.S1_2[v].resize((size_t)(K2 + 1) * D, 0.0);
          }
          if (ex >= K) {
            const int q = ex - K;
            P2.l2[v][q] += 1;
            P2.n2[v][q] += 1;
            for (int d = 0; d < D; ++d)
              P2.S1_2[v][(size_t)q * D + d] = P2.S1_2[v][(size_t)q * D + d] + yv(v, i, d);
          }
          tup[v] = ex;
        }
        t = P2.T2++;
        P2.c.push_back(1);
        P2.tup.push_back(tup);
      }
      btab[b] = t;
    }
    return btab;
  }

  void commit(const std::vector<int> &choice, const std::vector<int> &births, const std::vector<int> &btab,
              const Phase2 &P2) {
    std::vector<int> cnt(T, 0);
    for (int i = 0; i < n; ++i)
      if (choice[i] >= 0) cnt[choice[i]]++;
    std::vector<int> Kold(V), nnew(V);
    for (int v = 0; v < V; ++v) {
      Kold[v] = (int)ids[v].size();
      nnew[v] = (int)P2.n2[v].size();
    }
    // surviving tables: old in ascending position, then phase-2 tables
    std::vector<int> pos_new(T, -1);
    int Tn = 0;
    for (int p = 0; p < T; ++p)
      if (cnt[p] > 0) pos_new[p] = Tn++;
    const int Tsurv = Tn;
    Tn += P2.T2;
    std::vector<int> nt_new(Tn);
    std::vector<std::vector<int>> dext(V, std::vector<int>(Tn));
    for (int p = 0; p < T; ++p)
      if (pos_new[p] >= 0) {
        nt_new[pos_new[p]] = cnt[p];
        for (int v = 0; v < V; ++v) dext[v][pos_new[p]] = dish[v][p];
      }
    for (int t = 0; t < P2.T2; ++t) {
      nt_new[Tsurv + t] = P2.c[t];
      for (int v = 0; v < V; ++v) dext[v][Tsurv + t] = P2.tup[t][v];
    }
    std::vector<int> z_new(n);
    {
      size_t b = 0;
      for (int i = 0; i < n; ++i) z_new[i] = choice[i] >= 0 ? pos_new[choice[i]] : Tsurv + btab[b++];
    }
    (void)births;
    const std::vector<int> z_old = z;
    const std::vector<std::vector<int>> dish_old = dish;
    std::vector<std::vector<int>> jmaps(V);
    for (int v = 0; v < V; ++v) {
      const int Kext = Kold[v] + nnew[v];
      std::vector<int> l(Kext, 0);
      for (int p = 0; p < Tn; ++p) l[dext[v][p]]++;
      std::vector<int> jmap(Kext, -1);
      std::vector<int> ids_new, l_new;
      for (int j = 0; j < Kext; ++j)
        if (l[j] > 0) {
          jmap[j] = (int)ids_new.size();
          ids_new.push_back(j < Kold[v] ? ids[v][j] : next_id[v] + (j - Kold[v]));
          l_new.push_back(l[j]);
        }
      next_id[v] += nnew[v];
      for (int p = 0; p < Tn; ++p) dext[v][p] = jmap[dext[v][p]];
      ids[v] = ids_new;
      lk[v] = l_new;
      jmaps[v] = jmap;
    }
    T = Tn;
    n_t = nt_new;
    dish = dext;
    z = z_new;
    update_stats(z_old, dish_old, jmaps, Kold);
  }

  // Sufficient statistics after a commit.  Per view: the
  // dishes that survive keep their sums (re-indexed by the compaction map),
  // new dishes start at 0; then every customer whose dish changed moves its
  // y from the old dish (if that dish survived) to the new one, in ascending
  // customer order -- the reference's incremental remove/add updates
  // (multiview_utils.cpp:155-157, 199-206).  If more than n/8 customers of
  // the view changed dish, the view is rebuilt from scratch instead.
  void update_stats(const std::vector<int> &z_old, const std::vector<std::vector<int>> &dish_old,
                    const std::vector<std::vector<int>> &jmaps, const std::vector<int> &Kold) {
    for (int v = 0; v < V; ++v) {
      const int K = (int)ids[v].size();
      const std::vector<int> &jmap = jmaps[v];
      std::vector<int> dold(n), dnew(n);
      int moved = 0;
      for (int i = 0; i < n; ++i) {
        dold[i] = jmap[dish_old[v][z_old[i]]];
        dnew[i] = dish[v][z[i]];
        if (dold[i] != dnew[i]) ++moved;
      }
#ifdef MVC_ORACLE_FORCE_REBUILD
      if (true) {
#else
      if ((int64_t)8 * moved > (int64_t)n) {
#endif
        rebuild_view(v);
        continue;
      }
      std::vector<double> s1((size_t)K * D, 0.0), s2(K, 0.0);
      for (int j = 0; j < Kold[v]; ++j)
        if (jmap[j] >= 0) {
          for (int d = 0; d < D; ++d) s1[(size_t)jmap[j] * D + d] = S1[v][(size_t)j * D + d];
          s2[jmap[j]] = S2[v][j];
        }
      for (int i = 0; i < n; ++i) {
        if (dold[i] == dnew[i]) continue;
        if (dold[i] >= 0) {
          for (int d = 0; d < D; ++d) s1[(size_t)dold[i] * D + d] = s1[(size_t)dold[i] * D + d] - yv(v, i, d);
          s2[dold[i]] = s2[dold[i]] - Y2[(size_t)v * n + i];
        }
        for (int d = 0; d < D; ++d) s1[(size_t)dnew[i] * D + d] = s1[(size_t)dnew[i] * D + d] + yv(v, i, d);
        s2[dnew[i]] = s2[dnew[i]] + Y2[(size_t)v * n + i];
      }
      S1[v] = s1;
      S2[v] = s2;
      nk[v].assign(K, 0);
      for (int i = 0; i < n; ++i) nk[v][dnew[i]]++;
    }
  }

  // ---- parallel-mode hyperparameter MH ----
  struct MHRng {
    uint64_t seed; uint32_t chain; uint32_t sweep; uint32_t k;
    double unif() { return mvc_uniform(seed, k++, sweep, chain, MVC_TAG_MH); }
    double rnorm(double mu, double sd) {
      const double u1 = unif();
      const double u2 = unif();
      return mu + sd * mvc_norm_from_uniforms(u1, u2);
    }
  };
  static double prior_alpha(double a) {
    if (a <= 0.0) return -MVC_PM_INF;
    return (4.0 - 1.0) * mvc_log(a) - 3.0 * a;
  }
  static double prior_sigma(double s) {
    if (s <= 0.0 || s >= 1.0) return -MVC_PM_INF;
    return (1.0 - 1.0) * mvc_log(s) + (5.0 - 1.0) * mvc_log(1.0 - s);
  }
  // EPPF of a partition with block sizes `sz` (in order), total `tot`
  static double eppf(const std::vector<int> &sz, int tot, double a, double s) {
    if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
    if (a <= -s) return -MVC_PM_INF;
    const int K = (int)sz.size();
    std::vector<double> t1(K);
    for (int j = 0; j < K; ++j) {
      const double term = a + (double)j * s;
      if (term <= 0.0) return -MVC_PM_INF;
      t1[j] = mvc_log(term);
    }
    const double P1 = tree64_sum(t1);
    const double P2 = mvc_lgamma_pos(a + (double)tot) - mvc_lgamma_pos(a + 1.0);
    // sum_j sum_{m=1}^{sz_j - 1} log(m - s) (multiview_hyper.cpp:325-336) as
    // sum_j [lgamma(sz_j - s) - lgamma(1 - s)], block order, tree64
    const double lg1 = mvc_lgamma_pos(1.0 - s);
    std::vector<double> t3(K);
    for (int j = 0; j < K; ++j) t3[j] = mvc_lgamma_pos((double)sz[j] - s) - lg1;
    const double P3 = tree64_sum(t3);
    return (P1 - P2) + P3;
  }
  double eppf_view(int v, double a, double s) const {
    if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
    if (a <= -s) return -MVC_PM_INF;
    int tot = 0;
    for (int c : lk[v]) tot += c;
    if (tot == 0) return 0.0;
    return eppf(lk[v], tot, a, s);
  }
  double eppf_global(double a, double s) const {
    if (!(s > kEps && s < 1.0 - kEps)) return -MVC_PM_INF;
    if (a <= -s) return -MVC_PM_INF;
    if (T <= 0) return 0.0;
    return eppf(n_t, n, a, s);
  }
  double post_tau(int v, double t) const {
    if (t <= 0.0) return -MVC_PM_INF;
    const int K = (int)ids[v].size();
    const double L = mvc_log((2.0 * MVC_PI) * t);
    std::vector<double> terms(K, 0.0);
    for (int j = 0; j < K; ++j) {
      if (nk[v][j] == 0) continue;
      const double *s = &S1[v][(size_t)j * D];
      const double Q = fma_dot(s, s, D);
      double sse = S2[v][j] - Q / (double)nk[v][j];
      if (sse < 0.0) sse = 0.0;
      terms[j] = ((-0.5 * (double)nk[v][j]) * (double)D) * L - 0.5 * (sse / t);
    }
    const double ll = tree64_sum(terms);
    const double prior = (-3.0 * mvc_log(t)) - 1.0 / t;
    return ll + prior;
  }
  static double reflect_unit(double value) {
    double p = value;
    while (p <= kEps || p >= 1.0 - kEps) {
      if (p <= kEps) p = 2.0 * kEps - p;
      if (p >= 1.0 - kEps) p = 2.0 * (1.0 - kEps) - p;
    }
    return std::clamp(p, kEps, 1.0 - kEps);
  }
  // Each MH step draws from its own fixed window of the MH counter (tau of
  // view v: 3v..3v+2; alpha/sigma of view v: 3V+6v..+5; global: 9V..9V+5),
  // so the per-view steps are independent and run on separate GPU wavefronts
  // (DESIGN.md §4.7).  The step order within a window is the reference's
  // (multiview_hyper.cpp:233-292).
  void update_hyper(int s) {
    for (int v = 0; v < V; ++v) {
      MHRng R{seed, chain, (uint32_t)s, (uint32_t)(3 * v)};
      double t_old = tau[v];
      if (t_old <= 0.0) t_old = kEps;
      const double l_old = post_tau(v, t_old);
      const double t_prop = mvc_exp(mvc_log(t_old) + R.rnorm(0.0, 0.3));
      if (t_prop <= 0.0) continue;
      const double l_new = post_tau(v, t_prop);
      const double acc = (l_new - l_old) + (mvc_log(t_prop) - mvc_log(t_old));
      if (mvc_log(R.unif()) < acc) tau[v] = t_prop;
    }
    for (int v = 0; v < V; ++v) {
      MHRng R{seed, chain, (uint32_t)s, (uint32_t)(3 * V + 6 * v)};
      double a_old = alpha[v];
      if (a_old <= 0.0) a_old = kEps;
      double la = mvc_log(std::max(a_old, kEps)) + R.rnorm(0.0, 0.1);
      double a_prop = mvc_exp(la);
      if (!(a_prop > kEps)) a_prop = kEps;
      const double lo = (a_old <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_old, sigma[v]) + prior_alpha(a_old);
      const double ln = (a_prop <= 0.0) ? -MVC_PM_INF : eppf_view(v, a_prop, sigma[v]) + prior_alpha(a_prop);
      const double lq = mvc_log(a_prop) - mvc_log(a_old);
      if (mvc_log(R.unif()) < (ln - lo) + lq) alpha[v] = a_prop;
      const double s_old = sigma[v];
      const double s_prop = reflect_unit(s_old + R.rnorm(0.0, 0.05));
      const double u = R.unif();
      auto ps = [&](double sv) {
        if (sv <= kEps || sv >= 1.0 - kEps) return -MVC_PM_INF;
        return eppf_view(v, alpha[v], sv) + prior_sigma(sv);
      };
      if (mvc_log(u) < ps(s_prop) - ps(s_old)) sigma[v] = s_prop;
    }
    MHRng R{seed, chain, (uint32_t)s, (uint32_t)(9 * V)};
    double ag_old = ag;
    if (ag_old <= 0.0) ag_old = kEps;
    double la = mvc_log(std::max(ag_old, kEps)) + R.rnorm(0.0, 0.1);
    double ag_prop = mvc_exp(la);
    if (!(ag_prop > kEps)) ag_prop = kEps;
    const double lo = eppf_global(ag_old, sg) + prior_alpha(ag_old);
    const double ln = eppf_global(ag_prop, sg) + prior_alpha(ag_prop);
    const double lq = mvc_log(ag_prop) - mvc_log(ag_old);
    if (mvc_log(R.unif()) < (ln - lo) + lq) ag = ag_prop;
    const double sg_old = sg;
    const double sg_prop = reflect_unit(sg_old + R.rnorm(0.0, 0.05));
    const double u = R.unif();
    auto pg = [&](double sv) {
      if (sv <= kEps || sv >= 1.0 - kEps) return -MVC_PM_INF;
      return eppf_global(ag, sv) + prior_sigma(sv);
    };
    if (mvc_log(u) < pg(sg_prop) - pg(sg_old)) sg = sg_prop;
  }

  void save(Result &R) const {
    R.table_of.insert(R.table_of.end(), z.begin(), z.end());
    R.sample_T.push_back(T);
    for (int v = 0; v < V; ++v)
      for (int p = 0; p < T; ++p) R.dish_of.push_back(ids[v][dish[v][p]]);
    R.dish_off.push_back((int64_t)R.dish_of.size());
    for (int v = 0; v < V; ++v) {
      R.alpha_v.push_back(alpha[v]);
      R.sigma_v.push_back(sigma[v]);
      R.tau_v.push_back(tau[v]);
    }
    R.alpha_g.push_back(ag);
    R.sigma_g.push_back(sg);
    R.S++;
  }

  void run(int M, int burn_in, int thin, Result &R) {
    R.dish_off.push_back(0);
    std::vector<int> choice(n), births;
    Phase2 P2;
    for (int s = 0; s < M; ++s) {
      sweep_constants();
      births.clear();
      for (int i = 0; i < n; ++i) {
        choice[i] = resample_customer(i, s);
        if (choice[i] < 0) births.push_back(i);
      }
      const std::vector<int> btab = resolve_births(births, s, P2);
      commit(choice, births, btab, P2);
      update_hyper(s);
      R.trace_T.push_back(T);
      R.trace_draws.push_back(init_rng.draws);
      if (s >= burn_in && ((s - burn_in) % thin == 0)) save(R);
    }
  }
};

// ===========================================================================
// SeqSampler: the sequential schedule of the reference (multiview_gibbs.cpp:
// 157-200: customer i+1 sees customer i's move) with the GPU-shaped
// per-customer conditional of DESIGN.md §4.2-4.3.  This is the specification
// of the parallel-execution ("speculative") schedule that libmvc_hip.so runs:
// the GPU evaluates every customer against the sweep-start state in one
// data-parallel pass and then repairs, in customer order, exactly the
// decisions that earlier moves could have changed.  The
// Markov kernel is the reference's systematic-scan collapsed Gibbs sweep.
//
// Differences from the reference that do not change the kernel:
//  * a customer's own removal is virtual (self-dish coefficients, §4.2):
//    staying is a bitwise no-op on the sums; stats change only on a move;
//  * table positions are stable within a sweep (a table that empties keeps
//    its slot with weight 0; multiview_utils.cpp:175-190 swaps the last table
//    in instead), a birth appends a position, dead tables are compacted
//    (order kept) after the sweep — the inverse CDF scans a fixed order;
//  * dead dish slots (l = 0) are dropped at the end of the sweep (the
//    reference keeps them forever, multiview_utils.cpp:251-258; they carry
//    no weight), raw ids keep growing;
//  * uniforms are counter-addressed: table draw Philox(i, sweep, chain,
//    TAG_Z), dish draw of a birth Philox(i, sweep, chain, TAG_DISH+1+v).
// ===========================================================================
struct SeqSampler : ParallelSampler {
  int64_t moves = 0, births = 0, newdish = 0;

  void refresh_dish(int v, int j) {
    const double *s = &S1[v][(size_t)j * D];
    Qd[v][j] = fma_dot(s, s, D);
    cf[v][j] = coef(nk[v][j], Qd[v][j], tau[v], L2pt[v]);
  }

  // new dish slot in view v (raw id next_id[v]); returns its list index
  int open_dish(int v) {
    ids[v].push_back(next_id[v]++);
    nk[v].push_back(0);
    lk[v].push_back(0);
    S1[v].resize(S1[v].size() + D, 0.0);
    S2[v].push_back(0.0);
    Qd[v].push_back(0.0);
    cf[v].push_back(coef(0, 0.0, tau[v], L2pt[v]));
    ++newdish;
    return (int)ids[v].size() - 1;
  }

  // dish of a birth in view v: tree64 over the leaves w_j exp(lp_j - m) of
  // the included dishes (ascending list index) and the new dish (last);
  // r = u S; returns a list index, ids[v].size() = a new dish.
  int draw_dish(int i, int v, bool alive, int j0, int s) const {
    ViewEval E;
    eval_view(i, v, alive, j0, E);
    const int K = (int)ids[v].size();
    if (!(E.S > 0.0)) return K;
    Tree64 td;
    td.build(E.leaves);
    const double rv = mvc_uniform(seed, (uint32_t)i, (uint32_t)s, chain, MVC_TAG_DISH + 1u + (uint32_t)v) * E.S;
    return (int)td.select(rv);
  }

  void move(int i, int p0, int p1) {
    n_t[p0]--;
    if (n_t[p0] == 0) {
      T_ne--;
      for (int v = 0; v < V; ++v) { lk[v][dish[v][p0]]--; Ltot[v]--; }
    }
    if (n_t[p1] == 0) {
      T_ne++;
      for (int v = 0; v < V; ++v) { lk[v][dish[v][p1]]++; Ltot[v]++; }
    }
    n_t[p1]++;
    for (int v = 0; v < V; ++v) {
      const int j0 = dish[v][p0], j1 = dish[v][p1];
      if (j0 == j1) continue;
      const double *yi = y + ((size_t)v * n + i) * D;
      double *a = &S1[v][(size_t)j0 * D];
      double *b = &S1[v][(size_t)j1 * D];
      for (int d = 0; d < D; ++d) a[d] = a[d] - yi[d];
      for (int d = 0; d < D; ++d) b[d] = b[d] + yi[d];
      S2[v][j0] = S2[v][j0] - Y2[(size_t)v * n + i];
      S2[v][j1] = S2[v][j1] + Y2[(size_t)v * n + i];
      nk[v][j0]--;
      nk[v][j1]++;
      refresh_dish(v, j0);
      refresh_dish(v, j1);
    }
    z[i] = p1;
  }

  // drop empty tables (order kept) and dead dishes (l = 0; order kept)
  void compact() {
    std::vector<int> pos_new(T, -1);
    int Tn = 0;
    for (int p = 0; p < T; ++p)
      if (n_t[p] > 0) pos_new[p] = Tn++;
    std::vector<int> nt2(Tn);
    std::vector<std::vector<int>> dish2(V, std::vector<int>(Tn));
    for (int p = 0; p < T; ++p)
      if (pos_new[p] >= 0) {
        nt2[pos_new[p]] = n_t[p];
        for (int v = 0; v < V; ++v) dish2[v][pos_new[p]] = dish[v][p];
      }
    for (int i = 0; i < n; ++i) z[i] = pos_new[z[i]];
    for (int v = 0; v < V; ++v) {
      const int K = (int)ids[v].size();
      std::vector<int> jmap(K, -1), ids2, nk2, lk2;
      std::vector<double> s1, s2;
      for (int j = 0; j < K; ++j) {
        if (lk[v][j] <= 0) continue;
        jmap[j] = (int)ids2.size();
        ids2.push_back(ids[v][j]);
        nk2.push_back(nk[v][j]);
        lk2.push_back(lk[v][j]);
        s1.insert(s1.end(), S1[v].begin() + (size_t)j * D, S1[v].begin() + (size_t)(j + 1) * D);
        s2.push_back(S2[v][j]);
      }
      for (int p = 0; p < Tn; ++p) dish2[v][p] = jmap[dish2[v][p]];
      ids[v] = ids2; nk[v] = nk2; lk[v] = lk2; S1[v] = s1; S2[v] = s2;
    }
    T = Tn;
    n_t = nt2;
    dish = dish2;
  }

  void sweep_once(int s) {
    sweep_constants();
    for (int i = 0; i < n; ++i) {
      const int p0 = z[i];
      const int c = resample_customer(i, s);
      if (c == p0) continue;
      ++moves;
      if (c >= 0) {
        move(i, p0, c);
        continue;
      }
      ++births;
      const bool alive = (n_t[p0] - 1) > 0;
      std::vector<int> tup(V);
      for (int v = 0; v < V; ++v) tup[v] = draw_dish(i, v, alive, dish[v][p0], s);
      for (int v = 0; v < V; ++v)
        if (tup[v] == (int)ids[v].size()) tup[v] = open_dish(v);
      const int p1 = T++;
      n_t.push_back(0);
      for (int v = 0; v < V; ++v) dish[v].push_back(tup[v]);
      move(i, p0, p1);
    }
    compact();
  }

  void run(int M, int burn_in, int thin, Result &R) {
    R.dish_off.push_back(0);
    for (int s = 0; s < M; ++s) {
      moves = births = newdish = 0;
      sweep_once(s);
      update_hyper(s);
      R.trace_T.push_back(T);
      R.trace_draws.push_back(init_rng.draws);
      R.trace_moves.push_back(moves);
      R.trace_births.push_back(births);
      R.trace_newdish.push_back(newdish);
      if (s >= burn_in && ((s - burn_in) % thin == 0)) save(R);
    }
  }
};

}  // namespace

// ===========================================================================
// C ABI for tests (ctypes)
// ===========================================================================
extern "C" {

// mode: 0 = exact (reference schedule, D must be 1), 1 = parallel
// math: 0 = glibc libm (reference), 1 = portable (GPU spec); parallel mode
//       always uses portable math.
void *mvo_run(const double *y, int n, int V, int D, int M, int burn_in, int thin,
              uint64_t seed, int chain, int mode, int math) {
  Result *R = new Result();
  R->n = n;
  R->V = V;
  try {
    if (n < 2 || V < 1 || D < 1 || M < 0 || burn_in < 0 || thin < 1)
      throw std::runtime_error("invalid arguments");
    if (mode == 0) {
      if (D != 1) throw std::runtime_error("exact mode requires D == 1");
      auto go = [&](auto &S) {
        S.n = n;
        S.d = V;
        S.y.assign(V, std::vector<double>(n));
        for (int v = 0; v < V; ++v)
          for (int i = 0; i < n; ++i) S.y[v][i] = y[(size_t)v * n + i];
        S.rng = SeqRng{seed, (uint32_t)chain, 0};
        S.initialize();
        S.run(M, burn_in, thin, *R);
      };
      if (math == 0) { ExactSampler<LibmMath> S; go(S); }
      else { ExactSampler<PortableMath> S; go(S); }
    } else if (mode == 1) {
      SeqSampler P;
      P.n = n; P.V = V; P.D = D; P.y = y;
      P.seed = seed; P.chain = (uint32_t)chain;
      P.init_rng = SeqRng{seed, (uint32_t)chain, 0};
      P.initialize();
      P.run(M, burn_in, thin, *R);
      R->fS1 = P.S1; R->fS2 = P.S2; R->fnk = P.nk; R->D = D;
    } else {
      ParallelSampler P;
      P.n = n; P.V = V; P.D = D; P.y = y;
      P.seed = seed; P.chain = (uint32_t)chain;
      P.init_rng = SeqRng{seed, (uint32_t)chain, 0};
      P.initialize();
      P.run(M, burn_in, thin, *R);
      R->fS1 = P.S1; R->fS2 = P.S2; R->fnk = P.nk; R->D = D;
    }
  } catch (const std::exception &e) {
    R->error = e.what();
  }
  return R;
}

// Same as mvo_run, but the chain starts from a given state instead of the
// reference initialisation (mirrors mvc_sampler_set_state: RNG draw 0).
void *mvo_run_from(const double *y, int n, int V, int D, int M, int burn_in, int thin, uint64_t seed, int chain,
                   int mode, int math, const int *table_of, int T, const int *dish_of, const double *hyper) {
  Result *R = new Result();
  R->n = n;
  R->V = V;
  try {
    if (mode == 0) {
      if (D != 1) throw std::runtime_error("exact mode requires D == 1");
      auto go = [&](auto &S) {
        S.n = n;
        S.d = V;
        S.y.assign(V, std::vector<double>(n));
        for (int v = 0; v < V; ++v)
          for (int i = 0; i < n; ++i) S.y[v][i] = y[(size_t)v * n + i];
        S.rng = SeqRng{seed, (uint32_t)chain, 0};
        S.load_state(table_of, T, dish_of, hyper);
        S.run(M, burn_in, thin, *R);
      };
      if (math == 0) { ExactSampler<LibmMath> S; go(S); }
      else { ExactSampler<PortableMath> S; go(S); }
    } else if (mode == 1) {
      SeqSampler P;
      P.n = n; P.V = V; P.D = D; P.y = y;
      P.seed = seed; P.chain = (uint32_t)chain;
      P.init_rng = SeqRng{seed, (uint32_t)chain, 0};
      P.load_state(table_of, T, dish_of, hyper);
      P.run(M, burn_in, thin, *R);
      R->fS1 = P.S1; R->fS2 = P.S2; R->fnk = P.nk; R->D = D;
    } else {
      ParallelSampler P;
      P.n = n; P.V = V; P.D = D; P.y = y;
      P.seed = seed; P.chain = (uint32_t)chain;
      P.init_rng = SeqRng{seed, (uint32_t)chain, 0};
      P.load_state(table_of, T, dish_of, hyper);
      P.run(M, burn_in, thin, *R);
      R->fS1 = P.S1; R->fS2 = P.S2; R->fnk = P.nk; R->D = D;
    }
  } catch (const std::exception &e) {
    R->error = e.what();
  }
  return R;
}

// Phase-A table draw (ParallelSampler::resample_customer against the
// sweep-start state) of customers idx[0..m) in sweep `sweep`, given the state
// as a partition (table_of[n], dish_raw[V][T], hyper[3V+2]) and the per-view
// statistics in ascending raw-id order (S1 [K_v][D], S2 [K_v], nk [K_v],
// concatenated over views), and only the sampled customers' rows
// rows[m][V][D]: checks the device's full-size conditional where y itself
// does not fit on the host (BASELINE configs[4]).  Returns 0, or -1 with the
// message in err.
int mvo_phase_a(int n, int V, int D, const int *table_of, int T, const int *dish_raw, const double *hyper,
                const int *K, const double *S1, const double *S2, const int *nk, uint64_t seed, int chain, int sweep,
                int m, const int *idx, const double *rows, int *out, char *err, int errlen) {
  try {
    ParallelSampler P;
    P.n = n; P.V = V; P.D = D; P.y = nullptr;
    P.seed = seed; P.chain = (uint32_t)chain;
    P.load_partition(table_of, T, dish_raw, hyper);
    P.nk.assign(V, {}); P.S1.assign(V, {}); P.S2.assign(V, {});
    size_t o1 = 0, o2 = 0;
    for (int v = 0; v < V; ++v) {
      if (K[v] != (int)P.ids[v].size()) throw std::runtime_error("K_v does not match the partition's dishes");
      P.nk[v].assign(nk + o2, nk + o2 + K[v]);
      P.S2[v].assign(S2 + o2, S2 + o2 + K[v]);
      P.S1[v].assign(S1 + o1, S1 + o1 + (size_t)K[v] * D);
      o1 += (size_t)K[v] * D;
      o2 += K[v];
    }
    P.sweep_constants();
    std::vector<const double *> rp(V);
    std::vector<double> y2(V);
    for (int k = 0; k < m; ++k) {
      for (int v = 0; v < V; ++v) {
        rp[v] = rows + ((size_t)k * V + v) * D;
        y2[v] = ParallelSampler::fma_dot(rp[v], rp[v], D);
      }
      out[k] = P.resample_rows(idx[k], sweep, rp.data(), y2.data());
    }
    return 0;
  } catch (const std::exception &e) {
    if (err && errlen > 0) snprintf(err, errlen, "%s", e.what());
    return -1;
  }
}

int mvo_stats_K(void *h, int v) {
  Result *R = (Result *)h;
  return v < (int)R->fnk.size() ? (int)R->fnk[v].size() : 0;
}
void mvo_copy_stats(void *h, int v, double *S1, double *S2, int *nk) {
  Result *R = (Result *)h;
  const size_t K = R->fnk[v].size();
  memcpy(S1, R->fS1[v].data(), sizeof(double) * K * R->D);
  memcpy(S2, R->fS2[v].data(), sizeof(double) * K);
  memcpy(nk, R->fnk[v].data(), sizeof(int) * K);
}

const char *mvo_error(void *h) {
  Result *R = (Result *)h;
  return R->error.empty() ? nullptr : R->error.c_str();
}
int mvo_num_saved(void *h) { return ((Result *)h)->S; }
int mvo_num_sweeps(void *h) { return (int)((Result *)h)->trace_T.size(); }
int mvo_sample_T(void *h, int s) { return ((Result *)h)->sample_T[s]; }
void mvo_copy_table_of(void *h, int s, int *out) {
  Result *R = (Result *)h;
  memcpy(out, R->table_of.data() + (size_t)s * R->n, sizeof(int) * R->n);
}
void mvo_copy_dish_of(void *h, int s, int *out) {
  Result *R = (Result *)h;
  const int64_t a = R->dish_off[s], b = R->dish_off[s + 1];
  memcpy(out, R->dish_of.data() + a, sizeof(int) * (size_t)(b - a));
}
void mvo_copy_hyper(void *h, double *alpha_v, double *sigma_v, double *tau_v,
                    double *alpha_g, double *sigma_g) {
  Result *R = (Result *)h;
  memcpy(alpha_v, R->alpha_v.data(), sizeof(double) * R->alpha_v.size());
  memcpy(sigma_v, R->sigma_v.data(), sizeof(double) * R->sigma_v.size());
  memcpy(tau_v, R->tau_v.data(), sizeof(double) * R->tau_v.size());
  memcpy(alpha_g, R->alpha_g.data(), sizeof(double) * R->alpha_g.size());
  memcpy(sigma_g, R->sigma_g.data(), sizeof(double) * R->sigma_g.size());
}
void mvo_copy_trace(void *h, int *T, uint64_t *draws) {
  Result *R = (Result *)h;
  memcpy(T, R->trace_T.data(), sizeof(int) * R->trace_T.size());
  memcpy(draws, R->trace_draws.data(), sizeof(uint64_t) * R->trace_draws.size());
}
void mvo_copy_trace_moves(void *h, int64_t *moves, int64_t *births, int64_t *newdish) {
  Result *R = (Result *)h;
  const size_t m = R->trace_moves.size();
  for (size_t s = 0; s < R->trace_T.size(); ++s) {
    moves[s] = s < m ? R->trace_moves[s] : -1;
    births[s] = s < m ? R->trace_births[s] : -1;
    newdish[s] = s < m ? R->trace_newdish[s] : -1;
  }
}
// ExactSampler's per-sweep underflow counters (zeros for the other samplers)
void mvo_copy_trace_underflow(void *h, int64_t *fallback, int64_t *uf_tables, int64_t *uf_customers,
                              int64_t *uf_new) {
  Result *R = (Result *)h;
  const size_t S = R->trace_T.size();
  for (size_t s = 0; s < S; ++s) {
    const bool have = s < R->trace_fallback.size();
    fallback[s] = have ? R->trace_fallback[s] : 0;
    uf_tables[s] = have ? R->trace_uf_tables[s] : 0;
    uf_customers[s] = have ? R->trace_uf_customers[s] : 0;
    uf_new[s] = have ? R->trace_uf_new[s] : 0;
  }
}

void mvo_free(void *h) { delete (Result *)h; }

// ---- spec primitives, exposed so tests can check the GPU against them ----
void mvo_pm_exp(const double *x, double *o, int64_t n) { for (int64_t i = 0; i < n; ++i) o[i] = mvc_exp(x[i]); }
void mvo_pm_log(const double *x, double *o, int64_t n) { for (int64_t i = 0; i < n; ++i) o[i] = mvc_log(x[i]); }
void mvo_pm_lgamma(const double *x, double *o, int64_t n) { for (int64_t i = 0; i < n; ++i) o[i] = mvc_lgamma_pos(x[i]); }
void mvo_pm_qnorm(const double *x, double *o, int64_t n) { for (int64_t i = 0; i < n; ++i) o[i] = mvc_qnorm(x[i]); }
void mvo_philox(const uint32_t *ctr, uint32_t k0, uint32_t k1, uint32_t *out) {
  mvc_u32x4 c{ctr[0], ctr[1], ctr[2], ctr[3]};
  const mvc_u32x4 r = mvc_philox4x32_10(c, k0, k1);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}
void mvo_seq_uniforms(uint64_t seed, uint32_t chain, uint64_t start, double *o, int64_t n) {
  for (int64_t i = 0; i < n; ++i) o[i] = mvc_seq_uniform(seed, chain, start + (uint64_t)i);
}
double mvo_tree64_sum(const double *x, int64_t n) {
  return tree64_sum(std::vector<double>(x, x + n));
}
int64_t mvo_tree64_select(const double *x, int64_t n, double r) {
  Tree64 t;
  t.build(std::vector<double>(x, x + n));
  return (int64_t)t.select(r);
}

}  // extern "C"
