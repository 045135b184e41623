/*
 * mvc.h — C ABI of libmvc_hip.so, the MI355X-native Gibbs sampler for the
 * two-level Pitman–Yor multiview clustering model of JunR3/Multiview-Clustering.
 *
 * Plain C: no torch or HIP types cross this boundary.  Every entry point
 * returns an int status (MVC_OK == 0) and never throws; on failure the
 * message is copied into err[0..errlen) and also kept per thread
 * (mvc_last_error()).
 *
 * Reference interfaces replaced:
 *   mvc_run()              <- Rcpp::List run_gibbs_cpp(const Rcpp::List& data_views,
 *                              int M, int burn_in, int thin)
 *                              /root/reference/Multiview/multiview_gibbs.cpp:105-131
 *                              (decl. multiview_gibbs.h:8-9).  data_views = V numeric
 *                              vectors of length n -> views[v] (n*dim doubles each).
 *   mvc_result_*()         <- the named Rcpp::List built at multiview_gibbs.cpp:121-130
 *                              (table_of, dish_of, loglik, alpha_v, sigma_v, tau_v,
 *                              alpha_global, sigma_global).
 *   mvc_sampler_sweep()    <- void gibbs_sampler(int M, int burn_in, int thin)
 *                              multiview_gibbs.cpp:134-212 (one call = n_sweeps
 *                              iterations of the loop at :150).
 *   mvc_sampler_create()   <- static void initialize_state_from_data()
 *                              multiview_gibbs.cpp:12-103 + the globals of
 *                              multiview_state.cpp:4-27 (now per-handle state).
 *   mvc_sampler_get_state()<- void save_state() multiview_utils.cpp:291-303.
 *   seed                   <- R's RNG under set.seed() (multiview_utils.cpp:305-306,
 *                              multiview_gibbs.cpp:26,56; multiview_rng.h is dead code).
 *                              Replaced by counter-based Philox4x32-10 (mvc_philox.h).
 *
 * Integration stubs for R (Rcpp + dlopen) and Python (ctypes): INTEGRATION.md.
 */
#ifndef MVC_H
#define MVC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVC_ABI_VERSION 2

/* status codes */
#define MVC_OK 0
#define MVC_ERR_ARG 1        /* invalid argument (sizes, mode, NULL)            */
#define MVC_ERR_HIP 2        /* HIP runtime error (no device, OOM, launch)       */
#define MVC_ERR_STATE 3      /* sampler state invariant violated (bug)          */
#define MVC_ERR_UNSUPPORTED 4
#define MVC_ERR_CALLBACK 5   /* a caller-supplied callback reported failure       */

/* schedules */
#define MVC_MODE_EXACT 0     /* reference schedule, bit-exact vs. the CPU oracle  */
#define MVC_MODE_PARALLEL 1  /* the same sequential schedule, executed data-parallel
                                (speculative pass + in-order repair) */

typedef struct mvc_config {
  int32_t n;            /* customers (observations)                              */
  int32_t n_views;      /* V = length(data_views)                                */
  int32_t dim;          /* D per view (1 in the reference)                        */
  int32_t n_iter;       /* M                                                      */
  int32_t burn_in;      /* burn_in                                                */
  int32_t thin;         /* thin (>= 1)                                            */
  uint64_t seed;        /* Philox key                                             */
  int32_t n_chains;     /* independent chains on this device                      */
  int32_t first_chain;  /* global id of chain 0 (multi-GPU sharding)              */
  int32_t device;       /* HIP device ordinal                                     */
  int32_t mode;         /* MVC_MODE_EXACT | MVC_MODE_PARALLEL                     */
  int32_t table_cap;    /* initial table capacity per chain (0 = auto)            */
  int32_t dish_cap;     /* initial dish capacity per view per chain (0 = auto)    */
  int32_t flags;        /* MVC_FLAG_*                                             */
  /* ABI 2 */
  int32_t n_devices;    /* mvc_run: chains spread over devices device ..          */
                        /* device + n_devices - 1, chain c on device + c % n_devices */
                        /* (one host thread per device); 0 or 1: `device` only    */
  int32_t chain_stride; /* global id of local chain c = first_chain + c * stride  */
                        /* (0 = 1); the id keys every Philox counter              */
} mvc_config;

#define MVC_FLAG_TIMING 1   /* record per-kernel HIP-event times (mvc_sampler_kernel_time) */
#define MVC_FLAG_QUIET  2   /* no progress lines on stderr                                 */
#define MVC_FLAG_TIMING_COARSE 4   /* with MVC_FLAG_TIMING: only "zresample", "sweep" and
                                      "exact_sweep" (two events per timer; the per-phase
                                      events cost ~5 us of idle GPU each per sweep)       */

void mvc_config_init(mvc_config *cfg);   /* fills defaults: thin=1, n_chains=1, ... */
int mvc_abi_version(void);
const char *mvc_last_error(void);

/* ------------------------------------------------------------------------ */
/* One-shot drop-in: the whole run_gibbs_cpp() call.                          */
/* views[v] -> host array of n*dim doubles ([n][dim] row-major).              */
/* ------------------------------------------------------------------------ */
typedef struct mvc_result mvc_result;

int mvc_run(const mvc_config *cfg, const double *const *views, mvc_result **out,
            char *err, size_t errlen);

int mvc_result_num_saved(const mvc_result *r);                 /* S */
int mvc_result_num_chains(const mvc_result *r);
int mvc_result_num_tables(const mvc_result *r, int chain, int s);               /* T_s */
const int32_t *mvc_result_table_of(const mvc_result *r, int chain, int s);      /* n     */
const int32_t *mvc_result_dish_of(const mvc_result *r, int chain, int s);       /* V*T_s, view-major */
/* hyperparameter traces: which = MVC_TRACE_*; *_v traces are V*S (view-major) */
#define MVC_TRACE_ALPHA_V 0
#define MVC_TRACE_SIGMA_V 1
#define MVC_TRACE_TAU_V 2
#define MVC_TRACE_ALPHA_GLOBAL 3
#define MVC_TRACE_SIGMA_GLOBAL 4
const double *mvc_result_trace(const mvc_result *r, int chain, int which);
/* Every saved sample of one chain in one call (bulk form of the three
 * accessors above): table_of[S][n], n_tables[S], dish_of = the samples'
 * view-major [V][T_s] blocks one after the other (V * sum_s T_s entries).
 * Any pointer may be NULL (e.g. n_tables alone first, to size dish_of). */
int mvc_result_copy_chain(const mvc_result *r, int chain, int32_t *table_of, int32_t *n_tables, int32_t *dish_of);
/* Posterior summary over every chain's saved samples (no reference
 * counterpart: the reference runs one chain).  mean[3V+2] and rhat[3V+2] in
 * the hyper order tau[V], alpha[V], sigma[V], alpha_g, sigma_g: pooled means
 * and the Gelman-Rubin potential scale reduction (NaN with fewer than two
 * chains or two saved samples).  Either pointer may be NULL. */
int mvc_result_summary(const mvc_result *r, double *mean, double *rhat);
void mvc_result_free(mvc_result *r);

/* ------------------------------------------------------------------------ */
/* Handle API: data uploaded once, sweeps enqueued on the handle's stream.    */
/* ------------------------------------------------------------------------ */
typedef struct mvc_sampler mvc_sampler;

int mvc_sampler_create(const mvc_config *cfg, const double *const *views, mvc_sampler **out,
                       char *err, size_t errlen);
/* Run n_sweeps further iterations (sweep index continues across calls). */
int mvc_sampler_sweep(mvc_sampler *s, int n_sweeps, char *err, size_t errlen);
int mvc_sampler_synchronize(mvc_sampler *s, char *err, size_t errlen);
int mvc_sampler_sweeps_done(const mvc_sampler *s);
/* Copy one chain's current state: table_of[n] (table positions), *n_tables,
 * dish_of[V * dish_of_cap] (view-major, raw dish ids, first *n_tables per view
 * are valid), hyper[3V+2] = tau[V], alpha[V], sigma[V], alpha_g, sigma_g.
 * Any output pointer may be NULL. */
int mvc_sampler_get_state(mvc_sampler *s, int chain, int32_t *table_of, int32_t *n_tables,
                          int32_t *dish_of, int32_t dish_of_cap, double *hyper,
                          char *err, size_t errlen);
/* Warm start / resume: replace one chain's state.  table_of[n] = table
 * position in [0, n_tables) (every table non-empty), dish_of[V*n_tables]
 * (view-major) = raw dish id of each table, hyper[3V+2] as in get_state.
 * The chain's RNG stream restarts at draw 0; the sweep counter is kept. */
int mvc_sampler_set_state(mvc_sampler *s, int chain, const int32_t *table_of, int32_t n_tables,
                          const int32_t *dish_of, const double *hyper, char *err, size_t errlen);
/* Number of live dishes per view (k_out[V]). */
int mvc_sampler_get_dish_counts(mvc_sampler *s, int chain, int32_t *k_out, char *err, size_t errlen);
/* Sufficient statistics of one view (live dishes, ascending raw dish id):
 * *n_dishes = K; S1[K*dim] (row-major [k][d] sums of y), S2[K] (sums of
 * |y|^2), n_vk[K] (customers per dish).  Replaces reading ViewState's
 * sum_y / sum_y2 / n_vk (multiview_state.h:7-18).  Outputs may be NULL;
 * at most dish_cap dishes are copied. */
int mvc_sampler_get_stats(mvc_sampler *s, int chain, int view, int32_t *n_dishes, double *S1, double *S2,
                          int32_t *n_vk, int32_t dish_cap, char *err, size_t errlen);
/* HIP-event kernel timing (needs MVC_FLAG_TIMING): kernel = "zresample",
 * "repair", "stats", "hyper", "exact_sweep", or "sweep" (whole sweep). */
int mvc_sampler_kernel_time(mvc_sampler *s, const char *kernel, double *total_ms,
                            int64_t *launches);
void mvc_sampler_reset_timers(mvc_sampler *s);
/* Adjusted Rand index of the chain's current table labels against truth[n]
 * (host array, any int32 labels), computed on the device from exact pair
 * counts in mcclust::arandi's operation order (the ARI of
 * New_Simulation.R:189).  MVC_ERR_UNSUPPORTED when range(labels) x
 * range(truth) > 2^26 contingency cells. */
int mvc_sampler_ari(mvc_sampler *s, int chain, const int32_t *truth, double *ari, char *err, size_t errlen);
/* Switch timing at run time: flags = 0 (off), MVC_FLAG_TIMING (every
 * phase) or MVC_FLAG_TIMING | MVC_FLAG_TIMING_COARSE (whole passes only).
 * Synchronises the handle's stream; accumulated times are kept. */
int mvc_sampler_set_timing(mvc_sampler *s, int32_t flags);
/* z-resample kernels used by the last parallel sweep: bits 0-1 the lp
 * producer (0 generic, one lane per customer; 2 per-view MFMA tiles), bit 2
 * set when the register-resident draw kernel ran (T <= 64, K_v <= 64), bit 4
 * the all-views MFMA producer, bit 5 phase A left to the repair, bit 6 the
 * dish-block MFMA producer, bit 7 the row draw (16 lanes per customer,
 * T <= 512); -1 for the exact schedule or before the first sweep.  (No reference
 * counterpart: diagnostics of this implementation.) */
int mvc_sampler_zpath(mvc_sampler *s);
/* Counters of the chain's last parallel sweep: out[0]
 * customers that changed table, out[1] births, out[2] in-order repair rounds,
 * out[3] dishes opened.  MVC_ERR_UNSUPPORTED for the exact schedule.  (No
 * reference counterpart: diagnostics of this implementation.) */
int mvc_sampler_repair_stats(mvc_sampler *s, int chain, int32_t *out);
/* Phase A alone: the data-parallel pass of the next parallel sweep (every
 * customer evaluated against the current state with that sweep's uniforms,
 * DESIGN.md §4.8) into choice[n] (table position, -1 = a new table); the
 * chain's state and sweep count are unchanged.  MVC_ERR_UNSUPPORTED for the
 * exact schedule and for handles with several chains.  (No reference
 * counterpart: a diagnostic that lets tests check the pass directly.) */
int mvc_sampler_phase_a(mvc_sampler *s, int chain, int32_t *choice);
/* Within-chain N-sharding (one chain split over `world` processes, one GPU
 * each, every rank holding the whole data and state).  Phase A of each sweep
 * (the data-parallel evaluation against the sweep-start state) covers only
 * this rank's customers, shard `rank` = [rank S, min(n, (rank+1) S)) with
 * S = mvc_shard_len(n, world).  The handle copies its shard's choices into
 * `exchange` (device memory, world * S int32), synchronises its stream and
 * calls all_gather(user), which must return 0 once every rank's shard is in
 * `exchange` (e.g. an RCCL all-gather in place).  A nonzero return fails the
 * sweep with MVC_ERR_CALLBACK before anything reads the exchange buffer: the
 * chain state is left as it was before the sweep.  Otherwise every rank runs the
 * same in-order repair, compaction and MH on the same state, so the ranks
 * stay identical to each other and to the unsharded chain, bit for bit.
 * world = 1 turns sharding off.  One chain per handle; MVC_ERR_UNSUPPORTED
 * for the exact schedule or several chains.  (No reference counterpart: the
 * reference runs one chain in one process.) */
int mvc_sampler_set_shard(mvc_sampler *s, int32_t rank, int32_t world, int32_t *exchange,
                          int (*all_gather)(void *), void *user);
int64_t mvc_shard_len(int64_t n, int32_t world);
/* Synthetic data generated on the device, no host copy of y (SURVEY.md §8d
 * recipe): z_i ~ U{0..K-1}, per-view cluster c_v = z mod K_v with K_v =
 * max(1, K >> v), means mu_v[c] ~ N(0, mu_sd^2 I_D), y_v[i] = mu_v[c_v(i)] +
 * sd N(0, I_D), drawn from Philox keyed by data_seed (mvc_synth.hip; a
 * different stream from the Python package's numpy generator).  Creates a
 * parallel-mode handle on it (cfg->n, n_views, dim as usual; views are not
 * passed); z_out[n] (host, may be NULL) receives the generating labels.
 * tau_v's initial value comes from device column sums (one pass, not the
 * host's two-pass loop bit for bit).  MVC_ERR_UNSUPPORTED for the exact
 * schedule.  (No reference counterpart: the data source of BASELINE
 * configs[4], N = 10M x 8 views x 256 dims = 164 GB, which fits the HBM but
 * not the host.) */
int mvc_sampler_create_synthetic(const mvc_config *cfg, int32_t K, uint64_t data_seed, double sd, double mu_sd,
                                 int32_t *z_out, mvc_sampler **out, char *err, size_t errlen);
/* Rows idx[0..m) of view `view` of the handle's data, m x dim doubles, to
 * the host (checks against the CPU restatement at sizes the host cannot
 * hold whole).  Parallel schedule only. */
int mvc_sampler_copy_rows(mvc_sampler *s, int32_t view, const int32_t *idx, int64_t m, double *out, char *err,
                          size_t errlen);
/* Opaque HIP stream the handle launches on (hipStream_t as void*). */
void *mvc_sampler_stream(mvc_sampler *s);
void mvc_sampler_destroy(mvc_sampler *s);

/* ------------------------------------------------------------------------ */
/* Spec primitives on the device (parity tests of RNG / math / reductions).   */
/* x, out are HOST arrays; computed on the device.                             */
/* op: 0 exp, 1 log, 2 lgamma, 3 qnorm, 4 sqrt, 5 exp (SGPR-coefficient form),  */
/*     6 log (branch-free form): 5 and 6 are bitwise equal to 0 and 1;         */
/*     7 exp for x <= 709.78, not NaN (equal to 0 there)                        */
/* ------------------------------------------------------------------------ */
/* Adjusted Rand index of two host label arrays a[n], b[n] on the device
 * (same computation as mvc_sampler_ari). */
int mvc_ari(int device, const int32_t *a, const int32_t *b, int64_t n, double *ari, char *err, size_t errlen);
int mvc_device_math(int device, int op, const double *x, double *out, int64_t n,
                    char *err, size_t errlen);
int mvc_device_seq_uniforms(int device, uint64_t seed, uint32_t chain, uint64_t start,
                            double *out, int64_t n, char *err, size_t errlen);
/* tree64 sum and select of the parallel mode, one wave per row:
 * x[rows][n] -> sums[rows], sel[rows] for targets r[rows] (r<sum). */
int mvc_device_tree64(int device, const double *x, int64_t rows, int64_t n, const double *r,
                      double *sums, int64_t *sel, char *err, size_t errlen);
/* G = Y * S1^T with the fma-chain order of DESIGN.md §4.1 on the MFMA path
 * (Y[n][D], S1[K][D], G[n][K]); used to pin the f64 MFMA accumulation order. */
int mvc_device_gemm_check(int device, const double *Y, const double *S1, int64_t n, int64_t K,
                          int64_t D, double *G, char *err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* MVC_H */
