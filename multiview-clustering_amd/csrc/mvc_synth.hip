// mvc_synth.hip — synthetic multiview data generated on the device (SURVEY.md
// §8d recipe), for workloads whose y does not fit host memory: BASELINE
// configs[4] is N = 10M, V = 8, D = 256 -> 164 GB of fp64, beyond the GPU
// box's 270 GiB host cap once the generator's own buffers are counted, but
// well inside the MI355X's 288 GB of HBM.  (No reference counterpart: the
// reference's data come from New_Simulation.R:47-60 in R.)
//
//   z_i      = floor(K u_i),            u_i = Philox{i, 0, 0, TAG_SYN_Z}
//   c_v(i)   = z_i mod K_v,             K_v = max(1, K >> v)
//   mu_v[c]  = mu_sd N(Philox{v K + c, d, 0, TAG_SYN_MU})
//   y_v[i,d] = mu_v[c_v(i)][d] + sd N(Philox{i, d, v, TAG_SYN_Y})
// N(...) is R's inversion normal from the block's two uniforms
// (mvc_norm_from_uniforms(u(x, y), u(z, w))).  Y2[v][i] = sum_d y^2 (fma
// chain in ascending d: the spec of mvc_par_y2_kernel) is formed in the
// same pass, and so are the per-(view, dim) column sums and sums of squares
// that initialise tau_v (multiview_gibbs.cpp:78-94) on the host.
#include <algorithm>
#include <cmath>
#include <vector>

#include "mvc_host.h"

#define MVC_TAG_SYN_Z 0x4D56535Au   /* 'MVSZ' */
#define MVC_TAG_SYN_MU 0x4D56534Du  /* 'MVSM' */
#define MVC_TAG_SYN_Y 0x4D565359u   /* 'MVSY' */

namespace {

__host__ __device__ inline double syn_normal(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t tag) {
  mvc_u32x4 c;
  c.x = c0; c.y = c1; c.z = c2; c.w = tag;
  const mvc_u32x4 r = mvc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return mvc_norm_from_uniforms(mvc_u01_from_bits(r.x, r.y), mvc_u01_from_bits(r.z, r.w));
}

__host__ __device__ inline int32_t syn_label(uint64_t seed, int64_t i, int K) {
  mvc_u32x4 c;
  c.x = (uint32_t)i; c.y = (uint32_t)(i >> 32); c.z = 0; c.w = MVC_TAG_SYN_Z;
  const mvc_u32x4 r = mvc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const int z = (int)(mvc_u01_from_bits(r.x, r.y) * (double)K);
  return z < K ? z : K - 1;
}

}  // namespace

extern "C" __global__ void mvc_synth_mu_kernel(int V, int K, int D, double mu_sd, uint64_t seed, double *mu) {
  const int64_t total = (int64_t)V * K * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(e % D);
    const int64_t vc = e / D;   // v K + c
    mu[e] = mu_sd * syn_normal(seed, (uint32_t)vc, (uint32_t)d, 0u, MVC_TAG_SYN_MU);
  }
}

// One thread per (view, customer) row, d ascending: the row's values, its Y2
// fma chain, and per-d wave sums of y and y^2.  Each wave accumulates into
// its own LDS slot in row order, and the block combines the slots in wave
// order at the end, so the column sums (and the tau_v they seed) are the
// same bits on every run.  Dimensions go in tiles of kSynDT (the LDS slots
// hold one tile); a row's Y2 chain is carried from tile to tile through Y2
// itself, so it stays the one fma chain in ascending d.
constexpr int kSynThreads = 256, kSynWaves = kSynThreads / 64, kSynDT = 1024;
extern "C" __global__ __launch_bounds__(kSynThreads) void mvc_synth_y_kernel(int n, int D, int K, double sd,
                                                                             uint64_t seed, const double *mu,
                                                                             double *y, double *Y2, int32_t *z,
                                                                             double *colpart) {
  extern __shared__ double s_col[];   // [kSynWaves][2 DT]: each wave's sum y, sum y^2 per d of the tile
  const int v = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Kv = max(1, K >> v);
  const int64_t nblk = gridDim.x;
  for (int d0 = 0; d0 < D; d0 += kSynDT) {
    const int DT = min(kSynDT, D - d0);
    double *my = s_col + (size_t)w * 2 * DT;
    for (int d = tid; d < kSynWaves * 2 * DT; d += blockDim.x) s_col[d] = 0.0;
    __syncthreads();
    for (int64_t r0 = (int64_t)blockIdx.x * kSynThreads; r0 < n; r0 += nblk * kSynThreads) {
      const int64_t i = r0 + tid;
      const bool ok = i < n;
      const int32_t zi = syn_label(seed, ok ? i : 0, K);
      if (ok && v == 0 && z && d0 == 0) z[i] = zi;
      const double *m = mu + ((size_t)v * K + (size_t)(zi % Kv)) * D;
      double *row = y + ((size_t)v * n + (size_t)(ok ? i : 0)) * D;
      double acc = (ok && d0 > 0) ? Y2[(size_t)v * n + i] : 0.0;
      for (int dd = 0; dd < DT; ++dd) {
        const int d = d0 + dd;
        const double x = ok ? m[d] + sd * syn_normal(seed, (uint32_t)i, (uint32_t)d, (uint32_t)v, MVC_TAG_SYN_Y) : 0.0;
        if (ok) row[d] = x;
        acc = __builtin_fma(x, x, acc);
        const double s1 = wave_tree_sum(x), s2 = wave_tree_sum(x * x);
        if (lane == 0) {   // this wave's slot only: a fixed order of additions
          my[dd] += s1;
          my[DT + dd] += s2;
        }
      }
      if (ok) Y2[(size_t)v * n + i] = acc;
    }
    __syncthreads();
    double *out = colpart + ((size_t)v * gridDim.x + blockIdx.x) * 2 * D;
    for (int q = tid; q < 2 * DT; q += blockDim.x) {
      double acc = s_col[q];
      for (int u = 1; u < kSynWaves; ++u) acc += s_col[(size_t)u * 2 * DT + q];
      out[(q < DT ? 0 : D) + d0 + (q < DT ? q : q - DT)] = acc;
    }
    __syncthreads();
  }
}

extern "C" __global__ void mvc_gather_rows_kernel(int n, int D, const double *y, int view, const int32_t *idx,
                                                  int64_t m, double *out) {
  const int64_t total = m * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    const int d = (int)(e - r * D);
    out[e] = y[((size_t)view * n + (size_t)idx[r]) * D + d];
  }
}

namespace mvc {

DeviceData synth_device_data(int device, int n, int V, int D, int K, uint64_t seed, double sd, double mu_sd,
                             int32_t *z_host) {
  if (K < 1) throw Error(MVC_ERR_ARG, "synthetic data: K must be >= 1");
  if (!(sd >= 0.0) || !(mu_sd >= 0.0)) throw Error(MVC_ERR_ARG, "synthetic data: sd and mu_sd must be >= 0");
  if (V > 31) throw Error(MVC_ERR_UNSUPPORTED, "synthetic data: at most 31 views (K_v = K >> v)");
  MVC_HIP(hipSetDevice(device));
  DeviceData DD;
  hipStream_t st = nullptr;
  MVC_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  double *mu = nullptr, *colpart = nullptr;
  int32_t *zd = nullptr;
  const int grid = 2048;
  try {
    MVC_HIP(hipMalloc(&DD.y, sizeof(double) * (size_t)V * n * D));
    MVC_HIP(hipMalloc(&DD.Y2, sizeof(double) * (size_t)V * n));
    MVC_HIP(hipMalloc(&mu, sizeof(double) * (size_t)V * K * D));
    MVC_HIP(hipMalloc(&colpart, sizeof(double) * (size_t)V * grid * 2 * D));
    if (z_host) MVC_HIP(hipMalloc(&zd, sizeof(int32_t) * (size_t)n));
    hipLaunchKernelGGL(mvc_synth_mu_kernel, dim3(256), dim3(256), 0, st, V, K, D, mu_sd, seed, mu);
    MVC_HIP(hipGetLastError());
    hipLaunchKernelGGL(mvc_synth_y_kernel, dim3(grid, V), dim3(kSynThreads), sizeof(double) * kSynWaves * 2 * std::min(D, kSynDT), st, n, D, K, sd,
                       seed, (const double *)mu, DD.y, DD.Y2, zd, colpart);
    MVC_HIP(hipGetLastError());
    std::vector<double> cp((size_t)V * grid * 2 * D);
    MVC_HIP(hipMemcpyAsync(cp.data(), colpart, sizeof(double) * cp.size(), hipMemcpyDeviceToHost, st));
    if (z_host) MVC_HIP(hipMemcpyAsync(z_host, zd, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, st));
    MVC_HIP(hipStreamSynchronize(st));
    // tau_v = 0.0025 x the mean over d of the variance (n - 1 denominator) of
    // column d (multiview_gibbs.cpp:78-94 with the D-dim extension of
    // draw_initial_state), from one-pass sums: the host path's two-pass loop
    // is not bit-reproduced for device data (documented in DESIGN.md §10)
    DD.tau0.assign(V, 0.0);
    for (int v = 0; v < V; ++v) {
      long double vsum = 0.0L;
      for (int d = 0; d < D; ++d) {
        long double s1 = 0.0L, s2 = 0.0L;
        for (int b = 0; b < grid; ++b) {
          s1 += cp[((size_t)v * grid + b) * 2 * D + d];
          s2 += cp[((size_t)v * grid + b) * 2 * D + D + d];
        }
        long double var = n > 1 ? (s2 - s1 * s1 / n) / (n - 1) : 1.0L;
        if (!(var > 0.0L)) var = 1.0L;
        vsum += var;
      }
      DD.tau0[v] = (double)(vsum / D) * 0.25 * 0.01;
    }
  } catch (...) {
    for (void *p : {(void *)mu, (void *)colpart, (void *)zd, (void *)DD.y, (void *)DD.Y2})
      if (p) hipFree(p);
    hipStreamDestroy(st);
    throw;
  }
  for (void *p : {(void *)mu, (void *)colpart, (void *)zd}) if (p) hipFree(p);
  hipStreamDestroy(st);
  return DD;
}

void gather_rows(const double *y, int n, int D, int view, const int32_t *idx_host, int64_t m, double *out_host,
                 hipStream_t st) {
  int32_t *idx = nullptr;
  double *buf = nullptr;
  try {
    MVC_HIP(hipMalloc(&idx, sizeof(int32_t) * std::max<int64_t>(m, 1)));
    MVC_HIP(hipMalloc(&buf, sizeof(double) * std::max<int64_t>(m * D, 1)));
    MVC_HIP(hipMemcpyAsync(idx, idx_host, sizeof(int32_t) * m, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(mvc_gather_rows_kernel, dim3(1024), dim3(256), 0, st, n, D, y, view, (const int32_t *)idx, m, buf);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipMemcpyAsync(out_host, buf, sizeof(double) * m * D, hipMemcpyDeviceToHost, st));
    MVC_HIP(hipStreamSynchronize(st));
  } catch (...) {
    if (idx) hipFree(idx);
    if (buf) hipFree(buf);
    throw;
  }
  hipFree(idx);
  hipFree(buf);
}

}  // namespace mvc
