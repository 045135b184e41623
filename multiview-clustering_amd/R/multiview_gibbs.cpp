// multiview_gibbs.cpp — drop-in replacement for the reference's R entry point.
//
// Same exported signature and result list as
//   /root/reference/Multiview/multiview_gibbs.cpp:105-131
//   // [[Rcpp::export]] Rcpp::List run_gibbs_cpp(const Rcpp::List& data_views,
//                                                int M, int burn_in, int thin)
// so New_Simulation.R (sourceCpp("multiview_gibbs.cpp") at :10, the call at
// :128-133, get_final_clusters at :135-149, the trace plots at :199-315) runs
// unchanged.  The sampling itself happens on the GPU in libmvc_hip.so; this
// file only converts R objects and calls the C ABI (include/mvc.h), which it
// loads with dlopen so sourceCpp needs no extra link flags.
//
//   MVC_HIP_LIB   path of libmvc_hip.so (default: "libmvc_hip.so" via the
//                 dynamic loader's search path)
//   MVC_MODE      "parallel" (default: the reference's sequential schedule as a
//                 data-parallel pass + in-order repair, any D; the faster of the
//                 two on New_Simulation.R's own call) or "exact"
//                 (the reference's arithmetic literally, one wavefront per
//                 chain; scalar views only, as the reference)
//   MVC_CHAINS    independent chains (default 1).  With more than one, the
//                 result list is chain 0's (so the script runs unchanged) plus
//                 `chains` (every chain's list) and `pooled` (posterior means
//                 and Gelman-Rubin R-hat of the hyperparameters)
//   MVC_DEVICES   GPUs the chains are spread over (default 1; chain c on device
//                 MVC_DEVICE + c % MVC_DEVICES, one host thread per device)
//   MVC_DEVICE    first HIP device ordinal (default 0)
//
// The Philox key is drawn from R's RNG (two unif_rand() calls), so set.seed()
// in the script still determines the run; the stream itself is Philox, not
// R's Mersenne Twister.
#include <Rcpp.h>
#include <dlfcn.h>

#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

struct mvc_config {   // layout of include/mvc.h (ABI version 2)
  int32_t n, n_views, dim, n_iter, burn_in, thin;
  uint64_t seed;
  int32_t n_chains, first_chain, device, mode, table_cap, dish_cap, flags;
  int32_t n_devices, chain_stride;
};
struct mvc_result;

struct Api {
  void (*config_init)(mvc_config *);
  int (*abi_version)();
  int (*run)(const mvc_config *, const double *const *, mvc_result **, char *, size_t);
  int (*num_saved)(const mvc_result *);
  int (*num_tables)(const mvc_result *, int, int);
  const int32_t *(*table_of)(const mvc_result *, int, int);
  const int32_t *(*dish_of)(const mvc_result *, int, int);
  const double *(*trace)(const mvc_result *, int, int);
  int (*summary)(const mvc_result *, double *, double *);
  void (*result_free)(mvc_result *);
};

int env_int(const char *name, int dflt) {
  const char *e = std::getenv(name);
  if (!e || !*e) return dflt;
  char *end = nullptr;
  const long v = std::strtol(e, &end, 10);
  return (end && *end == '\0') ? (int)v : dflt;
}

template <class F>
void bind(void *h, const char *name, F &f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) Rcpp::stop(std::string("libmvc_hip.so: missing symbol ") + name);
}

const Api &api() {
  static Api a;
  static bool ready = false;
  if (ready) return a;
  const char *path = std::getenv("MVC_HIP_LIB");
  // (no hardware-queue request: the chains of one call share a stream for
  // their repair, so HIP's default queues serve them)
  void *h = dlopen(path ? path : "libmvc_hip.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) Rcpp::stop(std::string("cannot load libmvc_hip.so: ") + dlerror());
  bind(h, "mvc_config_init", a.config_init);
  bind(h, "mvc_abi_version", a.abi_version);
  bind(h, "mvc_run", a.run);
  bind(h, "mvc_result_num_saved", a.num_saved);
  bind(h, "mvc_result_num_tables", a.num_tables);
  bind(h, "mvc_result_table_of", a.table_of);
  bind(h, "mvc_result_dish_of", a.dish_of);
  bind(h, "mvc_result_trace", a.trace);
  bind(h, "mvc_result_summary", a.summary);
  bind(h, "mvc_result_free", a.result_free);
  if (a.abi_version() != 2) Rcpp::stop("libmvc_hip.so: unsupported ABI version");
  ready = true;
  return a;
}

}  // namespace

// [[Rcpp::export]]
Rcpp::List run_gibbs_cpp(const Rcpp::List &data_views, int M, int burn_in, int thin) {
  const Api &A = api();
  const int V = data_views.size();
  if (V < 1) Rcpp::stop("data_views must hold at least one view");
  // n from view 0 (reference multiview_gibbs.cpp:110); a numeric vector is a
  // D = 1 view, an n x D matrix (column-major in R) is transposed to [n][D].
  int n = 0, D = 0;
  std::vector<std::vector<double>> rows(V);
  for (int v = 0; v < V; ++v) {
    SEXP x = data_views[v];
    Rcpp::NumericVector vec(x);
    int nv, dv;
    if (Rf_isMatrix(x)) {
      Rcpp::NumericMatrix m(x);
      nv = m.nrow();
      dv = m.ncol();
      rows[v].resize((size_t)nv * dv);
      for (int i = 0; i < nv; ++i)
        for (int d = 0; d < dv; ++d) rows[v][(size_t)i * dv + d] = m(i, d);
    } else {
      nv = vec.size();
      dv = 1;
      rows[v].assign(vec.begin(), vec.end());
    }
    if (v == 0) { n = nv; D = dv; }
    if (nv != n || dv != D) Rcpp::stop("all views must have the same number of observations and columns");
  }
  std::vector<const double *> ptrs(V);
  for (int v = 0; v < V; ++v) ptrs[v] = rows[v].data();

  mvc_config cfg;
  A.config_init(&cfg);
  cfg.n = n;
  cfg.n_views = V;
  cfg.dim = D;
  cfg.n_iter = M;
  cfg.burn_in = burn_in;
  cfg.thin = thin;
  const uint64_t hi = (uint64_t)(R::unif_rand() * 4294967296.0);   // Philox key from R's RNG
  const uint64_t lo = (uint64_t)(R::unif_rand() * 4294967296.0);
  cfg.seed = (hi << 32) | lo;
  const char *mode = std::getenv("MVC_MODE");
  const std::string m = mode ? mode : "parallel";
  if (m != "exact" && m != "parallel") Rcpp::stop("MVC_MODE must be \"exact\" or \"parallel\"");
  if (m == "exact" && D > 1)
    Rcpp::stop("MVC_MODE=exact needs scalar views (the reference's D = 1); unset it or use parallel for n x D matrices");
  cfg.mode = m == "parallel" ? 1 : 0;
  cfg.device = env_int("MVC_DEVICE", 0);
  cfg.n_chains = env_int("MVC_CHAINS", 1);
  cfg.n_devices = env_int("MVC_DEVICES", 1);
  if (cfg.n_chains < 1 || cfg.n_devices < 1) Rcpp::stop("MVC_CHAINS and MVC_DEVICES must be positive integers");

  mvc_result *res = nullptr;
  char err[1024] = {0};
  if (A.run(&cfg, ptrs.data(), &res, err, sizeof(err)) != 0) Rcpp::stop(std::string("mvc_run: ") + err);

  const int S = A.num_saved(res);
  // one chain's list, named as multiview_gibbs.cpp:121-130
  auto chain_list = [&](int c) {
    Rcpp::List table_of(S), dish_of(S);
    for (int s = 0; s < S; ++s) {
      const int T = A.num_tables(res, c, s);
      const int32_t *t = A.table_of(res, c, s);
      table_of[s] = Rcpp::IntegerVector(t, t + n);
      const int32_t *d = A.dish_of(res, c, s);
      Rcpp::List per_view(V);
      for (int v = 0; v < V; ++v) per_view[v] = Rcpp::IntegerVector(d + (size_t)v * T, d + (size_t)(v + 1) * T);
      dish_of[s] = per_view;
    }
    auto per_view_trace = [&](int which) {
      const double *p = A.trace(res, c, which);
      Rcpp::List out(V);
      for (int v = 0; v < V; ++v) out[v] = Rcpp::NumericVector(p + (size_t)v * S, p + (size_t)(v + 1) * S);
      return out;
    };
    const double *ag = A.trace(res, c, 3);
    const double *sg = A.trace(res, c, 4);
    return Rcpp::List::create(
        Rcpp::Named("table_of") = table_of, Rcpp::Named("dish_of") = dish_of,
        Rcpp::Named("loglik") = Rcpp::NumericVector(0),
        Rcpp::Named("alpha_v") = per_view_trace(0), Rcpp::Named("sigma_v") = per_view_trace(1),
        Rcpp::Named("tau_v") = per_view_trace(2),
        Rcpp::Named("alpha_global") = Rcpp::NumericVector(ag, ag + S),
        Rcpp::Named("sigma_global") = Rcpp::NumericVector(sg, sg + S));
  };
  Rcpp::List out = chain_list(0);
  if (cfg.n_chains > 1) {
    Rcpp::List chains(cfg.n_chains);
    for (int c = 0; c < cfg.n_chains; ++c) chains[c] = chain_list(c);
    std::vector<double> mean(3 * V + 2), rhat(3 * V + 2);
    A.summary(res, mean.data(), rhat.data());
    const Rcpp::List c0 = out;
    out = Rcpp::List::create(
        Rcpp::Named("table_of") = c0[0], Rcpp::Named("dish_of") = c0[1], Rcpp::Named("loglik") = c0[2],
        Rcpp::Named("alpha_v") = c0[3], Rcpp::Named("sigma_v") = c0[4], Rcpp::Named("tau_v") = c0[5],
        Rcpp::Named("alpha_global") = c0[6], Rcpp::Named("sigma_global") = c0[7],
        Rcpp::Named("chains") = chains,
        Rcpp::Named("pooled") = Rcpp::List::create(
            Rcpp::Named("mean") = Rcpp::NumericVector(mean.begin(), mean.end()),
            Rcpp::Named("rhat") = Rcpp::NumericVector(rhat.begin(), rhat.end())));
  }
  A.result_free(res);
  return out;
}
