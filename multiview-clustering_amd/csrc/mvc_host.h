// mvc_host.h — host-side sampler classes behind the C ABI (include/mvc.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mvc.h"
#include "mvc_internal.h"

namespace mvc {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define MVC_STR2(x) #x
#define MVC_STR(x) MVC_STR2(x)
#define MVC_HIP(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess)                                                                              \
      throw ::mvc::Error(MVC_ERR_HIP, std::string(#expr) + " [" + ::mvc::base_name(__FILE__) +          \
                                          ":" MVC_STR(__LINE__) "]: " + hipGetErrorString(_e));        \
  } while (0)
inline const char *base_name(const char *p) {
  const char *b = p;
  for (; *p; ++p)
    if (*p == '/') b = p + 1;
  return b;
}

// Diagnostics switches, read once from the environment:
//   MVC_POISON=<byte>  every device allocation of the samplers is filled with
//                      that byte (uninitialised reads become deterministic);
//   MVC_DEBUG_SYNC=1   the parallel sampler synchronises its stream after each
//                      launch and names the kernel in the error (a fault is
//                      attributed to the launch that caused it).
int poison_byte();      // -1: off
int lds_fill_byte();    // MVC_LDS_FILL, -1: off
bool run_check();       // MVC_RUN_CHECK
bool debug_sync();

// MVC_PATH: the execution-path overrides of the tests and A/B runs, one
// variable of comma-separated key=value items (e.g. "lc=0,waves=3"), read
// when a sampler is created.  Every key selects a path that is bitwise the
// default's and is pinned by a test (DESIGN.md §9 lists them).  path_opt
// returns the value of key, or nullptr when it is not set.
const char *path_opt(const char *key);
int path_int(const char *key, int dflt);   // the value as an int, dflt when unset

// Initial state draws of multiview_gibbs.cpp:12-62 on the sequential Philox
// stream (shared by both schedules), plus tau_v of :78-94.
struct InitState {
  std::vector<int32_t> table;            // [n] position 0..3
  std::vector<int32_t> dish_raw;         // [V*4] raw dish id (0/1) of each initial table
  std::vector<double> tau;               // [V]
  uint64_t draws = 0;                    // sequential draws consumed
};
InitState draw_initial_state(const double *y /*[V][n][D]*/, int n, int V, int D, uint64_t seed,
                             uint32_t chain);
// The table / dish draws of draw_initial_state only (tau left empty).
InitState draw_initial_draws(int n, int V, uint64_t seed, uint32_t chain);

// Views already on the device (synthetic data generated there): the sampler
// takes ownership of y and Y2.
struct DeviceData {
  double *y = nullptr;              // [V][n][D]
  double *Y2 = nullptr;             // [V][n], fma chain in ascending d
  std::vector<double> tau0;         // [V] initial tau_v (multiview_gibbs.cpp:78-94)
};
// mvc_synth.hip: the SURVEY §8d synthetic recipe on the device; z_host[n]
// (optional) receives the generating labels.
DeviceData synth_device_data(int device, int n, int V, int D, int K, uint64_t seed, double sd, double mu_sd,
                             int32_t *z_host);
// Rows idx[0..m) of view `view` of a device y [V][n][D] to the host.
void gather_rows(const double *y, int n, int D, int view, const int32_t *idx_host, int64_t m, double *out_host,
                 hipStream_t st);

// Per-kernel HIP-event timers (MVC_FLAG_TIMING).
struct Timers {
  bool on = false;
  bool coarse = false;                 // MVC_FLAG_TIMING_COARSE: the whole-pass timers only
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> pool;        // recycled events (no create/destroy per record)
  hipEvent_t get();
  bool wanted(const char *name) const;
  struct Rec { hipEvent_t a, b; std::string name; };
  std::vector<Rec> pending;
  std::map<std::string, std::pair<double, int64_t>> acc;
  void begin(const char *name, hipEvent_t *ev);
  void end(const char *name, hipEvent_t a);
  void collect();
  void reset();
  ~Timers();
};

class Sampler {
 public:
  virtual ~Sampler() {}
  virtual void sweep(int n_sweeps) = 0;
  virtual void synchronize() = 0;
  virtual void get_state(int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of,
                         int32_t dish_cap, double *hyper) = 0;
  virtual void get_dish_counts(int chain, int32_t *k_out) = 0;
  virtual void get_stats(int chain, int view, int32_t *K, double *S1, double *S2, int32_t *n_vk,
                         int32_t dish_cap) = 0;
  virtual void set_state(int chain, const int32_t *table_of, int32_t T, const int32_t *dish_of,
                         const double *hyper) = 0;
  // Asynchronous sample output: the chain state is
  // snapshotted on the device (a D2D copy into a ring slot, ordered after the
  // sweep on the sampler's stream) and copied to pinned host memory on a
  // second stream, so saving a sample does not stall the sweeps.  fn is called
  // on the host thread, in sample order, once the copy has landed (from a
  // later save_async or from flush_saves).  dish_of is [V][T] raw dish ids.
  using SampleFn = std::function<void(int chain, int T, const int32_t *table_of, const int32_t *dish_of,
                                      const double *hyper)>;
  virtual bool save_async(int chain, const SampleFn &fn) { (void)chain; (void)fn; return false; }
  virtual void flush_saves() {}
  // Every chain's sample at once (one snapshot, read back asynchronously;
  // fn(chain, ...) runs for chains 0..C-1 in order); false where unsupported.
  virtual bool save_all_async(const SampleFn &fn) { (void)fn; return false; }
  // mvc_run's whole loop (gibbs.cpp:150-206) with the saved sweeps written on
  // the device as the sweeps run (fn per chain and sample, each chain's
  // samples in order; calls for DIFFERENT chains may run concurrently on host
  // threads); false where unsupported (the caller then sweeps and saves itself).
  virtual bool run_saving(int n_iter, int burn_in, int thin, bool quiet, const SampleFn &fn) {
    (void)n_iter; (void)burn_in; (void)thin; (void)quiet; (void)fn;
    return false;
  }
  // Device pointer to the chain's table labels [n] (valid until the next
  // sweep; the stream is synchronised), or nullptr when they live on the host.
  virtual const int32_t *device_labels(int chain) { (void)chain; return nullptr; }
  // Rows idx[0..m) of view `view` of the sampler's data (m x dim doubles).
  virtual void copy_rows(int view, const int32_t *idx, int64_t m, double *out) {
    (void)view; (void)idx; (void)m; (void)out;
    throw Error(MVC_ERR_UNSUPPORTED, "copy_rows: not available for this schedule");
  }
  // Repair counters of the chain's last parallel sweep:
  // out[0] customers that moved, out[1] births, out[2] repair rounds,
  // out[3] dishes opened.  False for the exact schedule.
  virtual bool repair_stats(int chain, int32_t *out) { (void)chain; (void)out; return false; }
  // Phase A alone (mvc_sampler_phase_a): the data-parallel pass of the next
  // sweep against the current state, choices into out[n]; no state changes.
  // False where unsupported (the exact schedule, several chains per handle).
  virtual bool phase_a(int chain, int32_t *out) { (void)chain; (void)out; return false; }
  // Within-chain N-sharding (mvc_sampler_set_shard): false where unsupported
  // (the exact schedule, several chains per handle).
  virtual bool set_shard(int rank, int world, int32_t *exch, int (*cb)(void *), void *user) {
    (void)rank; (void)world; (void)exch; (void)cb; (void)user;
    return false;
  }
  // HIP-event timing (mvc_sampler_set_timing / reset_timers / kernel_time)
  virtual void set_timing(bool on, bool coarse) {
    synchronize();
    timers.on = on;
    timers.coarse = coarse;
  }
  virtual void reset_timers() { timers.reset(); }
  virtual bool kernel_time(const char *name, double *ms, int64_t *launches) {
    synchronize();
    auto it = timers.acc.find(name);
    if (ms) *ms = it == timers.acc.end() ? 0.0 : it->second.first;
    if (launches) *launches = it == timers.acc.end() ? 0 : it->second.second;
    return true;
  }
  mvc_config cfg;
  int sweeps_done = 0;
  int zpath = -1;                        // mvc_sampler_zpath
  hipStream_t stream = nullptr;
  Timers timers;
};

// Adjusted Rand index (mvc_ari.hip): exact pair counts on the device, combined
// in mcclust::arandi's operation order (New_Simulation.R:189).
double ari_device(const int32_t *da, const int32_t *db, int64_t n, hipStream_t stream);
double ari_from_pairs(uint64_t a, uint64_t sa, uint64_t sb, int64_t n);

// Global id of a handle's local chain c (mvc_config.chain_stride): the id
// keys every Philox counter of the chain.
inline uint32_t chain_gid(const mvc_config &c, int local) {
  return (uint32_t)(c.first_chain + local * (c.chain_stride > 0 ? c.chain_stride : 1));
}

// Customers per shard of within-chain N-sharding: ceil(n / world) rounded up
// to 64 (the phase-A batches' alignment); shard r is [r S, min(n, (r+1) S)).
inline int64_t shard_len(int64_t n, int world) {
  const int64_t w = world < 1 ? 1 : world;
  return ((n + w - 1) / w + 63) / 64 * 64;
}

// Validated host view of a user-supplied state (warm start / resume).
struct UserState {
  int T = 0;
  std::vector<int32_t> n_t;                  // [T]
  std::vector<std::vector<int32_t>> ids;     // [v] live raw ids, ascending
  std::vector<std::vector<int32_t>> l;       // [v] tables per live dish
  std::vector<std::vector<int32_t>> dish;    // [v][T] live index
  std::vector<int32_t> next_id;              // [v] max id + 1
};
UserState check_user_state(int n, int V, const int32_t *table_of, int32_t T, const int32_t *dish_of);

Sampler *make_exact_sampler(const mvc_config &cfg, const double *const *views);
Sampler *make_parallel_sampler(const mvc_config &cfg, const double *const *views);
Sampler *make_parallel_sampler_device(const mvc_config &cfg, DeviceData &&dd);

}  // namespace mvc
