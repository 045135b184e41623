/*
 * mvc_abi_example.c — drives libmvc_hip.so through the C ABI only (dlopen +
 * dlsym, the same path the Rcpp drop-in multiview-clustering_amd/R/
 * multiview_gibbs.cpp takes), without Python or HIP headers.
 *
 *   gcc -O2 -Iinclude -o mvc_abi_example examples/mvc_abi_example.c -ldl
 *   ./mvc_abi_example LIB IN OUT
 *
 * IN  (binary): int32 n, V, D, M, burn_in, thin, mode; uint64 seed; then
 *     V * n * D float64 (view-major, [n][D] per view).
 * OUT (binary): int32 S, T_last; table_of of the last saved iteration
 *     (n int32); dish_of (V * T_last int32); alpha_global, sigma_global
 *     traces (S float64 each).
 * Exit status 0 on success; the library's error message on stderr otherwise.
 */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

#include "mvc.h"

typedef void (*config_init_f)(mvc_config *);
typedef int (*run_f)(const mvc_config *, const double *const *, mvc_result **, char *, size_t);
typedef int (*num_saved_f)(const mvc_result *);
typedef int (*num_tables_f)(const mvc_result *, int, int);
typedef const int32_t *(*ints_f)(const mvc_result *, int, int);
typedef const double *(*trace_f)(const mvc_result *, int, int);
typedef void (*free_f)(mvc_result *);

#define BIND(h, T, name)                                      \
  T name##_p = (T)dlsym(h, #name);                            \
  if (!name##_p) {                                            \
    fprintf(stderr, "missing %s\n", #name);                   \
    return 2;                                                 \
  }

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s libmvc_hip.so in.bin out.bin\n", argv[0]);
    return 2;
  }
  void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
  BIND(h, config_init_f, mvc_config_init)
  BIND(h, run_f, mvc_run)
  BIND(h, num_saved_f, mvc_result_num_saved)
  BIND(h, num_tables_f, mvc_result_num_tables)
  BIND(h, ints_f, mvc_result_table_of)
  BIND(h, ints_f, mvc_result_dish_of)
  BIND(h, trace_f, mvc_result_trace)
  BIND(h, free_f, mvc_result_free)

  FILE *f = fopen(argv[2], "rb");
  if (!f) { perror("in"); return 2; }
  int32_t hdr[7];
  uint64_t seed;
  if (fread(hdr, sizeof(int32_t), 7, f) != 7 || fread(&seed, sizeof(seed), 1, f) != 1) return 2;
  const int n = hdr[0], V = hdr[1], D = hdr[2];
  double *y = (double *)malloc(sizeof(double) * (size_t)V * n * D);
  if (fread(y, sizeof(double), (size_t)V * n * D, f) != (size_t)V * n * D) return 2;
  fclose(f);
  const double **views = (const double **)malloc(sizeof(double *) * V);
  for (int v = 0; v < V; ++v) views[v] = y + (size_t)v * n * D;

  mvc_config cfg;
  mvc_config_init_p(&cfg);
  cfg.n = n; cfg.n_views = V; cfg.dim = D;
  cfg.n_iter = hdr[3]; cfg.burn_in = hdr[4]; cfg.thin = hdr[5]; cfg.mode = hdr[6];
  cfg.seed = seed;
  cfg.flags = MVC_FLAG_QUIET;
  mvc_result *res = NULL;
  char err[1024] = {0};
  if (mvc_run_p(&cfg, views, &res, err, sizeof(err)) != MVC_OK) {
    fprintf(stderr, "mvc_run: %s\n", err);
    return 1;
  }
  const int S = mvc_result_num_saved_p(res);
  const int T = S ? mvc_result_num_tables_p(res, 0, S - 1) : 0;
  FILE *o = fopen(argv[3], "wb");
  if (!o) { perror("out"); return 2; }
  int32_t oh[2] = {S, T};
  fwrite(oh, sizeof(int32_t), 2, o);
  if (S) {
    fwrite(mvc_result_table_of_p(res, 0, S - 1), sizeof(int32_t), (size_t)n, o);
    fwrite(mvc_result_dish_of_p(res, 0, S - 1), sizeof(int32_t), (size_t)V * T, o);
    fwrite(mvc_result_trace_p(res, 0, MVC_TRACE_ALPHA_GLOBAL), sizeof(double), (size_t)S, o);
    fwrite(mvc_result_trace_p(res, 0, MVC_TRACE_SIGMA_GLOBAL), sizeof(double), (size_t)S, o);
  }
  fclose(o);
  mvc_result_free_p(res);
  free(views);
  free(y);
  printf("mvc_abi_example: S=%d T=%d\n", S, T);
  return 0;
}
