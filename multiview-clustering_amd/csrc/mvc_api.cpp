// mvc_api.cpp — C ABI of libmvc_hip.so (declared in include/mvc.h).
//
// Thin dispatch: validates arguments, owns result memory, converts C++
// exceptions into status codes (nothing throws across the ABI).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "mvc.h"
#include "mvc_host.h"

namespace mvc {

const char *path_opt(const char *key) {
  // MVC_PATH is re-read on every call (tests change it between handles), and
  // the value returned lives in a thread-local copy until the next call
  thread_local std::string val;
  const char *e = std::getenv("MVC_PATH");
  if (!e) return nullptr;
  const std::string s(e), k(key);
  size_t pos = 0;
  while (pos <= s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    const std::string item = s.substr(pos, end - pos);
    const size_t eq = item.find('=');
    if (eq != std::string::npos && item.substr(0, eq) == k) {
      val = item.substr(eq + 1);
      return val.c_str();
    }
    pos = end + 1;
  }
  return nullptr;
}
int path_int(const char *key, int dflt) {
  const char *v = path_opt(key);
  return (v && v[0]) ? std::atoi(v) : dflt;
}


InitState draw_initial_draws(int n, int V, uint64_t seed, uint32_t chain) {
  // multiview_gibbs.cpp:12-62: T0 = 4 tables drawn for i ascending, then per
  // view K0 = 2 dishes for t ascending, all from R::runif(0, K).
  InitState S;
  uint64_t k = 0;
  auto runif = [&](double a, double b) {
    if (a == b) return a;
    return a + (b - a) * mvc_seq_uniform(seed, chain, k++);
  };
  S.table.resize(n);
  for (int i = 0; i < n; ++i) {
    int t = (int)std::floor(runif(0.0, 4.0));
    if (t < 0) t = 0;
    if (t >= 4) t = 3;
    S.table[i] = t;
  }
  S.dish_raw.resize((size_t)V * 4);
  for (int v = 0; v < V; ++v)
    for (int t = 0; t < 4; ++t) {
      int kk = (int)std::floor(runif(0.0, 2.0));
      if (kk < 0) kk = 0;
      if (kk >= 2) kk = 1;
      S.dish_raw[v * 4 + t] = kk;
    }
  S.draws = k;
  return S;
}

InitState draw_initial_state(const double *y, int n, int V, int D, uint64_t seed, uint32_t chain) {
  InitState S = draw_initial_draws(n, V, seed, chain);
  // tau_v = Var_{n-1}(y_v) * 0.25 * 0.01  (multiview_gibbs.cpp:78-94);
  // for dim > 1 the mean of the per-dimension variances.
  S.tau.resize(V);
  for (int v = 0; v < V; ++v) {
    double vsum = 0.0;
    for (int d = 0; d < D; ++d) {
      double s1 = 0.0;
      for (int i = 0; i < n; ++i) s1 += y[((size_t)v * n + i) * D + d];
      const double mean = s1 / std::max(1, n);
      double var = 0.0;
      if (n > 1) {
        for (int i = 0; i < n; ++i) {
          const double df = y[((size_t)v * n + i) * D + d] - mean;
          var += df * df;
        }
        var /= (n - 1);
      } else {
        var = 1.0;
      }
      if (var <= 0.0) var = 1.0;
      vsum += var;
    }
    const double var = vsum / (double)D;
    S.tau[v] = var * 0.25 * 0.01;
  }
  return S;
}

UserState check_user_state(int n, int V, const int32_t *table_of, int32_t T, const int32_t *dish_of) {
  if (!table_of || !dish_of) throw Error(MVC_ERR_ARG, "set_state: NULL table_of / dish_of");
  if (T < 1) throw Error(MVC_ERR_ARG, "set_state: n_tables must be >= 1");
  UserState U;
  U.T = T;
  U.n_t.assign(T, 0);
  for (int i = 0; i < n; ++i) {
    if (table_of[i] < 0 || table_of[i] >= T) throw Error(MVC_ERR_ARG, "set_state: table_of out of range");
    U.n_t[table_of[i]]++;
  }
  for (int p = 0; p < T; ++p)
    if (U.n_t[p] == 0) throw Error(MVC_ERR_ARG, "set_state: every table must hold at least one customer");
  U.ids.resize(V); U.l.resize(V); U.dish.resize(V); U.next_id.resize(V);
  for (int v = 0; v < V; ++v) {
    std::vector<int32_t> raw(dish_of + (size_t)v * T, dish_of + (size_t)(v + 1) * T);
    for (int32_t r : raw)
      if (r < 0) throw Error(MVC_ERR_ARG, "set_state: negative dish id");
    std::vector<int32_t> srt = raw;
    std::sort(srt.begin(), srt.end());
    srt.erase(std::unique(srt.begin(), srt.end()), srt.end());
    U.ids[v] = srt;
    U.l[v].assign(srt.size(), 0);
    U.dish[v].resize(T);
    for (int p = 0; p < T; ++p) {
      const int j = (int)(std::lower_bound(srt.begin(), srt.end(), raw[p]) - srt.begin());
      U.dish[v][p] = j;
      U.l[v][j]++;
    }
    U.next_id[v] = srt.back() + 1;
  }
  return U;
}

hipEvent_t Timers::get() {
  hipEvent_t e;
  if (!pool.empty()) {
    e = pool.back();
    pool.pop_back();
  } else {
    MVC_HIP(hipEventCreate(&e));
  }
  return e;
}
bool Timers::wanted(const char *name) const {
  if (!on) return false;
  if (!coarse) return true;
  const std::string s(name);
  return s == "zresample" || s == "sweep" || s == "exact_sweep";
}
void Timers::begin(const char *name, hipEvent_t *ev) {
  *ev = nullptr;
  if (!wanted(name)) return;
  *ev = get();
  MVC_HIP(hipEventRecord(*ev, stream));
}
void Timers::end(const char *name, hipEvent_t a) {
  if (!on || !a) return;
  hipEvent_t b = get();
  MVC_HIP(hipEventRecord(b, stream));
  pending.push_back({a, b, name});
  if (pending.size() > 4096) {
    MVC_HIP(hipStreamSynchronize(stream));
    collect();
  }
}
void Timers::collect() {
  for (auto &r : pending) {
    MVC_HIP(hipEventSynchronize(r.b));
    float ms = 0.f;
    MVC_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    auto &e = acc[r.name];
    e.first += ms;
    e.second += 1;
    pool.push_back(r.a);
    pool.push_back(r.b);
  }
  pending.clear();
}
void Timers::reset() {
  if (stream) hipStreamSynchronize(stream);
  collect();
  acc.clear();
}
Timers::~Timers() {
  for (auto &r : pending) {
    hipEventDestroy(r.a);
    hipEventDestroy(r.b);
  }
  for (hipEvent_t e : pool) hipEventDestroy(e);
}

}  // namespace mvc

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
namespace {
thread_local std::string g_last_error;
const double K_dummy = 0.0;   // stands in for host views that a call does not take

int fail(int code, const std::string &msg, char *err, size_t errlen) {
  g_last_error = msg;
  if (err && errlen) {
    std::snprintf(err, errlen, "%s", msg.c_str());
  }
  return code;
}

template <class F>
int guarded(char *err, size_t errlen, F &&f) {
  (void)hipGetLastError();   // never report a stale error of an earlier call
  try {
    f();
    g_last_error.clear();
    return MVC_OK;
  } catch (const mvc::Error &e) {
    return fail(e.code, e.what(), err, errlen);
  } catch (const std::bad_alloc &) {
    return fail(MVC_ERR_HIP, "host allocation failed", err, errlen);
  } catch (const std::exception &e) {
    return fail(MVC_ERR_STATE, e.what(), err, errlen);
  }
}

// MVC_DEVICE_MAP=a,b,...: logical device d of mvc_run's n_devices split runs
// on physical device map[d % len] instead of device + d.  A test aid: with
// "0,0" the per-device threads, chain striding and result interleave of
// n_devices = 2 run on one GPU (two handles on one device).  Empty or unset:
// no map.
std::vector<int> device_map() {
  std::vector<int> map;
  const char *e = std::getenv("MVC_DEVICE_MAP");
  if (!e) return map;
  const std::string s(e);
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string tok = s.substr(i, j - i);
    if (!tok.empty()) {
      char *end = nullptr;
      const long d = std::strtol(tok.c_str(), &end, 10);
      if (!end || *end != '\0') throw mvc::Error(MVC_ERR_ARG, "MVC_DEVICE_MAP: not a list of device ordinals");
      map.push_back((int)d);
    }
    i = j + 1;
  }
  return map;
}

void validate(const mvc_config *c, const double *const *views) {
  using mvc::Error;
  if (!c) throw Error(MVC_ERR_ARG, "config is NULL");
  if (c->n < 2) throw Error(MVC_ERR_ARG, "n must be >= 2 (the reference divides by n-1)");
  if (c->n_views < 1) throw Error(MVC_ERR_ARG, "n_views must be >= 1");
  if (c->dim < 1) throw Error(MVC_ERR_ARG, "dim must be >= 1");
  if (c->n_iter < 0 || c->burn_in < 0) throw Error(MVC_ERR_ARG, "n_iter and burn_in must be >= 0");
  if (c->thin < 1) throw Error(MVC_ERR_ARG, "thin must be >= 1");
  if (c->n_chains < 1) throw Error(MVC_ERR_ARG, "n_chains must be >= 1");
  if (c->mode != MVC_MODE_EXACT && c->mode != MVC_MODE_PARALLEL) throw Error(MVC_ERR_ARG, "unknown mode");
  if (c->n_devices < 0) throw Error(MVC_ERR_ARG, "n_devices must be >= 0");
  if (c->chain_stride < 0) throw Error(MVC_ERR_ARG, "chain_stride must be >= 0");
  if (!views) throw Error(MVC_ERR_ARG, "views is NULL");
  for (int v = 0; v < c->n_views; ++v)
    if (!views[v]) throw Error(MVC_ERR_ARG, "views[v] is NULL");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) throw Error(MVC_ERR_HIP, "no HIP device visible");
  if (c->device < 0 || c->device >= ndev) throw Error(MVC_ERR_ARG, "device ordinal out of range");
  const std::vector<int> map = device_map();
  if (!map.empty()) {
    for (int d : map)
      if (d < 0 || d >= ndev) throw Error(MVC_ERR_ARG, "MVC_DEVICE_MAP names a device that is not visible");
  } else if (c->n_devices > 1 && c->device + std::min(c->n_devices, c->n_chains) > ndev) {
    throw Error(MVC_ERR_ARG, "n_devices: devices device .. device + n_devices - 1 are not all visible");
  }
}

}  // namespace

namespace {

// One device's share of mvc_run: its chains in one handle, sweeps and the
// saved samples (multiview_gibbs.cpp:150-210 incl. save_state at :205-206).
// Samples are stored contiguously per chain (thousands of chains x hundreds of
// samples would otherwise be millions of small allocations): table_of[c] is
// S x n, dish_of[c] the samples' [V][T_s] blocks one after the other, doff[c]
// their S + 1 offsets.
struct RunPart {
  int S = 0;
  std::vector<std::vector<int32_t>> table_of, dish_of;   // [chain] flat
  std::vector<std::vector<size_t>> doff;                 // [chain][s]
  std::vector<std::vector<int>> T;
  std::vector<std::vector<std::vector<double>>> traces;  // [chain][which]
};

void run_part(const mvc_config &cf, const double *const *views, RunPart &R) {
  std::unique_ptr<mvc::Sampler> S(cf.mode == MVC_MODE_EXACT ? mvc::make_exact_sampler(cf, views)
                                                           : mvc::make_parallel_sampler(cf, views));
  const int C = cf.n_chains, V = cf.n_views, n = cf.n;
  const int H = 3 * V + 2;
  auto saved = [&](int it) { return it >= cf.burn_in && ((it - cf.burn_in) % cf.thin == 0); };   // gibbs.cpp:205
  int64_t S_exp = 0;
  for (int it = 0; it < cf.n_iter; ++it) S_exp += saved(it) ? 1 : 0;
  R.table_of.resize(C);
  R.dish_of.resize(C);
  R.doff.assign(C, std::vector<size_t>(1, 0));
  R.T.resize(C);
  R.traces.assign(C, std::vector<std::vector<double>>(5));
  std::vector<std::vector<double>> hv(C);   // [chain] S x (3V + 2) hyper vectors
  for (int c = 0; c < C; ++c) {
    R.table_of[c].reserve((size_t)S_exp * n);
    R.doff[c].reserve((size_t)S_exp + 1);
    R.T[c].reserve((size_t)S_exp);
    hv[c].reserve((size_t)S_exp * H);
  }
  std::vector<double> hyper(H);
  const bool quiet = (cf.flags & MVC_FLAG_QUIET) != 0;
  const mvc::Sampler::SampleFn save_fn = [&](int c, int T, const int32_t *t, const int32_t *d, const double *h) {
    R.table_of[c].insert(R.table_of[c].end(), t, t + n);
    R.dish_of[c].insert(R.dish_of[c].end(), d, d + (size_t)V * T);
    R.doff[c].push_back(R.dish_of[c].size());
    R.T[c].push_back(T);
    hv[c].insert(hv[c].end(), h, h + H);
  };
  if (S->run_saving(cf.n_iter, cf.burn_in, cf.thin, quiet, save_fn)) {   // samples written on the device (exact)
    for (int it = 0; it < cf.n_iter; ++it) R.S += saved(it) ? 1 : 0;
  } else {
  for (int iter0 = 0, iter = 0; iter0 < cf.n_iter; iter0 = iter + 1) {
    // the sweeps up to the next saved one in one call (the exact schedule
    // then runs them without a launch and read-back per sweep)
    iter = iter0;
    while (iter + 1 < cf.n_iter && !saved(iter)) ++iter;
    for (int it = iter0; it <= iter; ++it)
      if (!quiet && (it + 1) % 100 == 0)                           // gibbs.cpp:152-155
        std::fprintf(stderr, "Iteration %d / %d\n", it + 1, cf.n_iter);
    S->sweep(iter - iter0 + 1);
    if (saved(iter)) {
      if (S->save_all_async(save_fn)) {                   // all chains in one snapshot (exact schedule)
        R.S++;
        continue;
      }
      for (int c = 0; c < C; ++c) {
        if (S->save_async(c, save_fn)) continue;        // device snapshot + async D2H (f3)
        std::vector<int32_t> t(n);
        int32_t T = 0;
        // first query T, then fetch dish_of with an exact capacity
        S->get_state(c, t.data(), &T, nullptr, 0, hyper.data());
        std::vector<int32_t> d((size_t)V * std::max(T, 1));
        S->get_state(c, nullptr, &T, d.data(), std::max(T, 1), nullptr);
        save_fn(c, T, t.data(), d.data(), hyper.data());
      }
      R.S++;
    }
  }
  }
  S->flush_saves();
  S->synchronize();
  const int Sn = R.S;
  for (int c = 0; c < C; ++c) {
    auto &tr = R.traces[c];
    tr[MVC_TRACE_ALPHA_V].resize((size_t)V * Sn);
    tr[MVC_TRACE_SIGMA_V].resize((size_t)V * Sn);
    tr[MVC_TRACE_TAU_V].resize((size_t)V * Sn);
    tr[MVC_TRACE_ALPHA_GLOBAL].resize(Sn);
    tr[MVC_TRACE_SIGMA_GLOBAL].resize(Sn);
    for (int s = 0; s < Sn; ++s) {
      const double *h = hv[c].data() + (size_t)s * H;
      for (int v = 0; v < V; ++v) {
        tr[MVC_TRACE_TAU_V][(size_t)v * Sn + s] = h[v];
        tr[MVC_TRACE_ALPHA_V][(size_t)v * Sn + s] = h[V + v];
        tr[MVC_TRACE_SIGMA_V][(size_t)v * Sn + s] = h[2 * V + v];
      }
      tr[MVC_TRACE_ALPHA_GLOBAL][s] = h[3 * V];
      tr[MVC_TRACE_SIGMA_GLOBAL][s] = h[3 * V + 1];
    }
  }
}

}  // namespace

struct mvc_result {
  int S = 0, C = 0, n = 0, V = 0;
  // [chain] flat, as RunPart: table_of S x n, dish_of the [V][T_s] blocks at doff[chain][s]
  std::vector<std::vector<int32_t>> table_of, dish_of;
  std::vector<std::vector<size_t>> doff;
  std::vector<std::vector<int>> T;
  // [chain][which] traces
  std::vector<std::vector<std::vector<double>>> traces;
};

struct mvc_sampler {
  std::unique_ptr<mvc::Sampler> impl;
};

extern "C" {

void mvc_config_init(mvc_config *c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->dim = 1;
  c->thin = 1;
  c->n_chains = 1;
  c->mode = MVC_MODE_EXACT;
}

int mvc_abi_version(void) { return MVC_ABI_VERSION; }
const char *mvc_last_error(void) { return g_last_error.c_str(); }

int mvc_sampler_create(const mvc_config *cfg, const double *const *views, mvc_sampler **out, char *err,
                       size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!out) throw mvc::Error(MVC_ERR_ARG, "out is NULL");
    *out = nullptr;
    validate(cfg, views);
    auto *h = new mvc_sampler();
    try {
      h->impl.reset(cfg->mode == MVC_MODE_EXACT ? mvc::make_exact_sampler(*cfg, views)
                                                : mvc::make_parallel_sampler(*cfg, views));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int mvc_sampler_create_synthetic(const mvc_config *cfg, int32_t K, uint64_t data_seed, double sd, double mu_sd,
                                 int32_t *z_out, mvc_sampler **out, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!out) throw mvc::Error(MVC_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (!cfg) throw mvc::Error(MVC_ERR_ARG, "config is NULL");
    if (cfg->mode != MVC_MODE_PARALLEL)
      throw mvc::Error(MVC_ERR_UNSUPPORTED, "synthetic device data: parallel schedule only");
    // validate() checks the views' pointers: hand it V dummies (never read)
    std::vector<const double *> dummy(std::max(1, cfg->n_views), &K_dummy);
    validate(cfg, dummy.data());
    mvc::DeviceData dd = mvc::synth_device_data(cfg->device, cfg->n, cfg->n_views, cfg->dim, K, data_seed, sd, mu_sd,
                                                z_out);
    auto *h = new mvc_sampler();
    try {
      h->impl.reset(mvc::make_parallel_sampler_device(*cfg, std::move(dd)));
    } catch (...) {
      if (dd.y) hipFree(dd.y);
      if (dd.Y2) hipFree(dd.Y2);
      delete h;
      throw;
    }
    *out = h;
  });
}

int mvc_sampler_copy_rows(mvc_sampler *s, int32_t view, const int32_t *idx, int64_t m, double *out, char *err,
                          size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl || (m > 0 && (!idx || !out))) throw mvc::Error(MVC_ERR_ARG, "NULL argument");
    if (m < 0) throw mvc::Error(MVC_ERR_ARG, "m < 0");
    if (m == 0) return;
    s->impl->copy_rows(view, idx, m, out);
  });
}

int mvc_sampler_sweep(mvc_sampler *s, int n_sweeps, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl) throw mvc::Error(MVC_ERR_ARG, "sampler is NULL");
    if (n_sweeps < 0) throw mvc::Error(MVC_ERR_ARG, "n_sweeps < 0");
    s->impl->sweep(n_sweeps);
  });
}

int mvc_sampler_synchronize(mvc_sampler *s, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl) throw mvc::Error(MVC_ERR_ARG, "sampler is NULL");
    s->impl->synchronize();
  });
}

int mvc_sampler_sweeps_done(const mvc_sampler *s) { return (s && s->impl) ? s->impl->sweeps_done : -1; }

int mvc_sampler_get_state(mvc_sampler *s, int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of,
                          int32_t dish_of_cap, double *hyper, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl) throw mvc::Error(MVC_ERR_ARG, "sampler is NULL");
    s->impl->get_state(chain, table_of, n_tables, dish_of, dish_of_cap, hyper);
  });
}

int mvc_sampler_set_state(mvc_sampler *s, int chain, const int32_t *table_of, int32_t n_tables,
                          const int32_t *dish_of, const double *hyper, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl || !hyper) throw mvc::Error(MVC_ERR_ARG, "NULL argument");
    s->impl->set_state(chain, table_of, n_tables, dish_of, hyper);
  });
}

int mvc_ari(int device, const int32_t *a, const int32_t *b, int64_t n, double *ari, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!a || !b || !ari) throw mvc::Error(MVC_ERR_ARG, "NULL argument");
    if (n < 1) throw mvc::Error(MVC_ERR_ARG, "n must be >= 1");
    MVC_HIP(hipSetDevice(device));
    int32_t *d = nullptr;
    MVC_HIP(hipMalloc(&d, sizeof(int32_t) * 2 * (size_t)n));
    try {
      MVC_HIP(hipMemcpy(d, a, sizeof(int32_t) * n, hipMemcpyHostToDevice));
      MVC_HIP(hipMemcpy(d + n, b, sizeof(int32_t) * n, hipMemcpyHostToDevice));
      *ari = mvc::ari_device(d, d + n, n, nullptr);
    } catch (...) {
      hipFree(d);
      throw;
    }
    hipFree(d);
  });
}

int mvc_sampler_ari(mvc_sampler *s, int chain, const int32_t *truth, double *ari, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl || !truth || !ari) throw mvc::Error(MVC_ERR_ARG, "NULL argument");
    mvc::Sampler &S = *s->impl;
    const int64_t n = S.cfg.n;
    MVC_HIP(hipSetDevice(S.cfg.device));
    int32_t *d = nullptr;
    MVC_HIP(hipMalloc(&d, sizeof(int32_t) * 2 * (size_t)n));
    try {
      MVC_HIP(hipMemcpyAsync(d + n, truth, sizeof(int32_t) * n, hipMemcpyHostToDevice, S.stream));
      const int32_t *z = S.device_labels(chain);
      if (!z) {   // labels on the host (exact schedule): one upload
        std::vector<int32_t> h((size_t)n);
        int32_t T = 0;
        S.get_state(chain, h.data(), &T, nullptr, 0, nullptr);
        MVC_HIP(hipMemcpyAsync(d, h.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, S.stream));
        MVC_HIP(hipStreamSynchronize(S.stream));
        z = d;
      }
      *ari = mvc::ari_device(z, d + n, n, S.stream);
    } catch (...) {
      hipFree(d);
      throw;
    }
    hipFree(d);
  });
}

int mvc_sampler_get_dish_counts(mvc_sampler *s, int chain, int32_t *k_out, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl || !k_out) throw mvc::Error(MVC_ERR_ARG, "NULL argument");
    s->impl->get_dish_counts(chain, k_out);
  });
}

int mvc_sampler_get_stats(mvc_sampler *s, int chain, int view, int32_t *n_dishes, double *S1, double *S2,
                          int32_t *n_vk, int32_t dish_cap, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!s || !s->impl) throw mvc::Error(MVC_ERR_ARG, "sampler is NULL");
    if (view < 0 || view >= s->impl->cfg.n_views) throw mvc::Error(MVC_ERR_ARG, "view out of range");
    if (dish_cap < 0) throw mvc::Error(MVC_ERR_ARG, "dish_cap < 0");
    s->impl->get_stats(chain, view, n_dishes, S1, S2, n_vk, dish_cap);
  });
}

int mvc_sampler_kernel_time(mvc_sampler *s, const char *kernel, double *total_ms, int64_t *launches) {
  if (!s || !s->impl || !kernel) return MVC_ERR_ARG;
  try {
    s->impl->kernel_time(kernel, total_ms, launches);
  } catch (...) {
    return MVC_ERR_HIP;
  }
  return MVC_OK;
}

void mvc_sampler_reset_timers(mvc_sampler *s) {
  if (s && s->impl) {
    try {
      s->impl->reset_timers();
    } catch (...) {
    }
  }
}

int mvc_sampler_set_timing(mvc_sampler *s, int32_t flags) {
  if (!s || !s->impl) return MVC_ERR_ARG;
  try {
    s->impl->set_timing((flags & MVC_FLAG_TIMING) != 0, (flags & MVC_FLAG_TIMING_COARSE) != 0);
  } catch (...) {
    return MVC_ERR_HIP;
  }
  return MVC_OK;
}

int mvc_sampler_zpath(mvc_sampler *s) { return (s && s->impl) ? s->impl->zpath : -1; }

int mvc_sampler_phase_a(mvc_sampler *s, int chain, int32_t *choice) {
  if (!s || !s->impl || !choice) return MVC_ERR_ARG;
  try {
    return s->impl->phase_a(chain, choice) ? MVC_OK : MVC_ERR_UNSUPPORTED;
  } catch (const mvc::Error &e) {
    return e.code;
  }
}

int mvc_sampler_repair_stats(mvc_sampler *s, int chain, int32_t *out) {
  if (!s || !s->impl || !out) return MVC_ERR_ARG;
  try {
    return s->impl->repair_stats(chain, out) ? MVC_OK : MVC_ERR_UNSUPPORTED;
  } catch (const mvc::Error &e) {
    return e.code;
  }
}

int mvc_sampler_set_shard(mvc_sampler *s, int32_t rank, int32_t world, int32_t *exchange,
                          int (*all_gather)(void *), void *user) {
  if (!s || !s->impl) return MVC_ERR_ARG;
  try {
    return s->impl->set_shard(rank, world, exchange, all_gather, user) ? MVC_OK : MVC_ERR_UNSUPPORTED;
  } catch (const mvc::Error &e) {
    return e.code;
  }
}

int64_t mvc_shard_len(int64_t n, int32_t world) { return mvc::shard_len(n, world); }

void *mvc_sampler_stream(mvc_sampler *s) { return (s && s->impl) ? (void *)s->impl->stream : nullptr; }

void mvc_sampler_destroy(mvc_sampler *s) { delete s; }

int mvc_run(const mvc_config *cfg, const double *const *views, mvc_result **out, char *err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!out) throw mvc::Error(MVC_ERR_ARG, "out is NULL");
    *out = nullptr;
    validate(cfg, views);
    const int C = cfg->n_chains, V = cfg->n_views;
    // chain c on device `device + c % nd`, one host thread per device; a
    // device's chains form one handle with chain ids first_chain + (d + k nd)
    // * stride, k = 0, 1, ... (the id keys every Philox counter, so a chain
    // is the same wherever it runs)
    const int nd = std::max(1, std::min(cfg->n_devices, C));
    const std::vector<int> dmap = nd > 1 ? device_map() : std::vector<int>();
    std::vector<RunPart> parts(nd);
    std::vector<std::exception_ptr> errs(nd);
    auto one = [&](int d) {
      try {
        mvc_config sc = *cfg;
        sc.device = dmap.empty() ? cfg->device + d : dmap[d % dmap.size()];
        sc.n_devices = 1;
        sc.first_chain = (int32_t)mvc::chain_gid(*cfg, d);
        sc.chain_stride = (cfg->chain_stride > 0 ? cfg->chain_stride : 1) * nd;
        sc.n_chains = (C - d + nd - 1) / nd;
        if (d > 0) sc.flags |= MVC_FLAG_QUIET;   // one progress line per iteration
        run_part(sc, views, parts[d]);
      } catch (...) {
        errs[d] = std::current_exception();
      }
    };
    if (nd == 1) {
      one(0);
    } else {
      std::vector<std::thread> ts;
      for (int d = 0; d < nd; ++d) ts.emplace_back(one, d);
      for (auto &t : ts) t.join();
    }
    for (auto &e : errs)
      if (e) std::rethrow_exception(e);
    auto R = std::make_unique<mvc_result>();
    R->C = C;
    R->n = cfg->n;
    R->V = V;
    R->S = parts[0].S;
    for (int c = 0; c < C; ++c) {
      RunPart &P = parts[c % nd];
      const int k = c / nd;
      R->table_of.push_back(std::move(P.table_of[k]));
      R->dish_of.push_back(std::move(P.dish_of[k]));
      R->doff.push_back(std::move(P.doff[k]));
      R->T.push_back(std::move(P.T[k]));
      R->traces.push_back(std::move(P.traces[k]));
    }
    *out = R.release();
  });
}

int mvc_result_summary(const mvc_result *r, double *mean, double *rhat) {
  if (!r) return MVC_ERR_ARG;
  const int V = r->V, S = r->S, C = r->C, W = 3 * V + 2;
  // hyper order tau, alpha, sigma (per view), alpha_g, sigma_g
  auto draw = [&](int c, int s, int k) -> double {
    const auto &tr = r->traces[c];
    if (k < V) return tr[MVC_TRACE_TAU_V][(size_t)k * S + s];
    if (k < 2 * V) return tr[MVC_TRACE_ALPHA_V][(size_t)(k - V) * S + s];
    if (k < 3 * V) return tr[MVC_TRACE_SIGMA_V][(size_t)(k - 2 * V) * S + s];
    return tr[k == 3 * V ? MVC_TRACE_ALPHA_GLOBAL : MVC_TRACE_SIGMA_GLOBAL][s];
  };
  const double nan = std::nan("");
  for (int k = 0; k < W; ++k) {
    double tot = 0.0;
    std::vector<double> cm(C, 0.0), cv(C, 0.0);
    for (int c = 0; c < C; ++c) {
      double a = 0.0;
      for (int s = 0; s < S; ++s) a += draw(c, s, k);
      cm[c] = S > 0 ? a / S : nan;
      tot += a;
      if (S > 1) {
        double q = 0.0;
        for (int s = 0; s < S; ++s) q += (draw(c, s, k) - cm[c]) * (draw(c, s, k) - cm[c]);
        cv[c] = q / (S - 1);
      }
    }
    if (mean) mean[k] = (S > 0 && C > 0) ? tot / ((double)S * C) : nan;
    if (rhat) {
      // Gelman-Rubin: B = n/(m-1) sum (mean_j - grand)^2, W = mean of the
      // within-chain variances, var+ = (n-1)/n W + B/n, R = sqrt(var+/W)
      if (C < 2 || S < 2) {
        rhat[k] = nan;
        continue;
      }
      double grand = 0.0, Wv = 0.0, B = 0.0;
      for (int c = 0; c < C; ++c) { grand += cm[c]; Wv += cv[c]; }
      grand /= C;
      Wv /= C;
      for (int c = 0; c < C; ++c) B += (cm[c] - grand) * (cm[c] - grand);
      B *= (double)S / (C - 1);
      const double vplus = (S - 1.0) / S * Wv + B / S;
      rhat[k] = Wv > 0.0 ? std::sqrt(vplus / Wv) : nan;
    }
  }
  return MVC_OK;
}

int mvc_result_num_saved(const mvc_result *r) { return r ? r->S : -1; }
int mvc_result_num_chains(const mvc_result *r) { return r ? r->C : -1; }
int mvc_result_num_tables(const mvc_result *r, int chain, int s) {
  if (!r || chain < 0 || chain >= r->C || s < 0 || s >= r->S) return -1;
  return r->T[chain][s];
}
const int32_t *mvc_result_table_of(const mvc_result *r, int chain, int s) {
  if (!r || chain < 0 || chain >= r->C || s < 0 || s >= r->S) return nullptr;
  return r->table_of[chain].data() + (size_t)s * r->n;
}
const int32_t *mvc_result_dish_of(const mvc_result *r, int chain, int s) {
  if (!r || chain < 0 || chain >= r->C || s < 0 || s >= r->S) return nullptr;
  return r->dish_of[chain].data() + r->doff[chain][s];
}
int mvc_result_copy_chain(const mvc_result *r, int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of) {
  if (!r || chain < 0 || chain >= r->C) return MVC_ERR_ARG;
  if (table_of) std::copy(r->table_of[chain].begin(), r->table_of[chain].end(), table_of);
  if (n_tables) std::copy(r->T[chain].begin(), r->T[chain].end(), n_tables);
  if (dish_of) std::copy(r->dish_of[chain].begin(), r->dish_of[chain].end(), dish_of);
  return MVC_OK;
}
const double *mvc_result_trace(const mvc_result *r, int chain, int which) {
  if (!r || chain < 0 || chain >= r->C || which < 0 || which > 4) return nullptr;
  return r->traces[chain][which].data();
}
void mvc_result_free(mvc_result *r) { delete r; }

}  // extern "C"
