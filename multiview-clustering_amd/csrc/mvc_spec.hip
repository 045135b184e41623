// mvc_spec.hip — device evaluation of the spec primitives (portable math,
// Philox stream, tree64, fp64 MFMA accumulation order) so the parity tests
// can compare the GPU against the CPU oracle bit for bit.
#include <algorithm>
#include <vector>

#include "mvc_host.h"
#include "mvc_internal.h"

typedef double mvc_d4 __attribute__((ext_vector_type(4)));

extern "C" __global__ void mvc_spec_math_kernel(int op, const double *x, double *o, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double a = x[i];
    double r;
    switch (op) {
      case 0: r = mvc_exp(a); break;
      case 1: r = mvc_log(a); break;
      case 2: r = mvc_lgamma_pos(a); break;
      case 3: r = mvc_qnorm(a); break;
      case 5: r = mvc_exp_sk(a); break;            // the fused kernel's variants
      case 6: r = mvc_log_nb(a); break;
      case 7: r = mvc_exp_le0(a); break;           // the draw's a - max form
      case 8: r = mvc_lgamma_pos_nb(a); break;     // the MH kernel's EPPF form
      default: r = __builtin_sqrt(a); break;
    }
    o[i] = r;
  }
}

extern "C" __global__ void mvc_spec_uniform_kernel(uint64_t seed, uint32_t chain, uint64_t start, double *o, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = mvc_seq_uniform(seed, chain, start + (uint64_t)i);
}

// one wave per row, rows of n <= 4096 elements (two-level tree64)
extern "C" __global__ void mvc_spec_tree_kernel(const double *x, int64_t rows, int64_t n, const double *rr, double *sums,
                                                int64_t *sel) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (row >= rows) return;
  const double *xr = x + row * n;
  const int nc = (int)((n + 63) >> 6);
  double part = 0.0;
  for (int c = 0; c < nc; ++c) {
    const int64_t e = (int64_t)c * 64 + lane;
    const double leaf = e < n ? xr[e] : 0.0;
    const double cs = wave_tree_sum(leaf);
    if (lane == c) part = cs;
  }
  const double S = (nc == 1) ? __shfl(part, 0, 64) : wave_tree_sum(lane < nc ? part : 0.0);
  double r = rr[row];
  int c = 0;
  if (nc > 1) {
    Tree64Levels L;
    const double pv = lane < nc ? part : 0.0;
    wave_tree_sum_levels(pv, L);
    c = wave_tree_select(L, pv, r);
  }
  const int64_t e = (int64_t)c * 64 + lane;
  const double leaf = e < n ? xr[e] : 0.0;
  Tree64Levels L2;
  wave_tree_sum_levels(leaf, L2);
  const int l = wave_tree_select(L2, leaf, r);
  if (lane == 0) {
    sums[row] = S;
    sel[row] = (int64_t)c * 64 + l;
  }
}

// G = Y S1^T via v_mfma_f64_16x16x4_f64; one wave per 16x16 output tile.
// Y[n][D], S1[K][D] row-major, n%16 == K%16 == D%4 == 0 (host pads).
extern "C" __global__ void mvc_spec_gemm_kernel(const double *Y, const double *S1, int n, int K, int D, double *G) {
  const int lane = threadIdx.x & 63;
  const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int tn = K / 16;
  if (tile >= (n / 16) * tn) return;
  const int i0 = (tile / tn) * 16, j0 = (tile % tn) * 16;
  mvc_d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k = 0; k < D; k += 4) {
    const double a = Y[(size_t)(i0 + (lane & 15)) * D + k + (lane >> 4)];
    const double b = S1[(size_t)(j0 + (lane & 15)) * D + k + (lane >> 4)];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) G[(size_t)(i0 + (lane >> 4) + 4 * r) * K + j0 + (lane & 15)] = acc[r];
}

namespace {
thread_local std::string g_spec_err;
int spec_fail(const std::exception &e, char *err, size_t errlen) {
  if (err && errlen) snprintf(err, errlen, "%s", e.what());
  return MVC_ERR_HIP;
}
template <class Tp>
struct DBuf {
  Tp *p = nullptr;
  explicit DBuf(size_t n) { MVC_HIP(hipMalloc(&p, sizeof(Tp) * std::max<size_t>(n, 1))); }
  ~DBuf() { if (p) hipFree(p); }
};
}  // namespace

extern "C" int mvc_device_math(int device, int op, const double *x, double *out, int64_t n, char *err, size_t errlen) {
  try {
    MVC_HIP(hipSetDevice(device));
    DBuf<double> dx(n), dox(n);
    MVC_HIP(hipMemcpy(dx.p, x, sizeof(double) * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mvc_spec_math_kernel, dim3(1024), dim3(256), 0, 0, op, (const double *)dx.p, dox.p, n);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipMemcpy(out, dox.p, sizeof(double) * n, hipMemcpyDeviceToHost));
    return MVC_OK;
  } catch (const std::exception &e) {
    return spec_fail(e, err, errlen);
  }
}

extern "C" int mvc_device_seq_uniforms(int device, uint64_t seed, uint32_t chain, uint64_t start, double *out, int64_t n,
                                       char *err, size_t errlen) {
  try {
    MVC_HIP(hipSetDevice(device));
    DBuf<double> d(n);
    hipLaunchKernelGGL(mvc_spec_uniform_kernel, dim3(1024), dim3(256), 0, 0, seed, chain, start, d.p, n);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipMemcpy(out, d.p, sizeof(double) * n, hipMemcpyDeviceToHost));
    return MVC_OK;
  } catch (const std::exception &e) {
    return spec_fail(e, err, errlen);
  }
}

extern "C" int mvc_device_tree64(int device, const double *x, int64_t rows, int64_t n, const double *r, double *sums,
                                 int64_t *sel, char *err, size_t errlen) {
  try {
    if (n < 1 || n > 4096) throw mvc::Error(MVC_ERR_ARG, "tree64 test supports 1..4096 elements per row");
    MVC_HIP(hipSetDevice(device));
    DBuf<double> dx(rows * n), dr(rows), ds(rows);
    DBuf<int64_t> dsel(rows);
    MVC_HIP(hipMemcpy(dx.p, x, sizeof(double) * rows * n, hipMemcpyHostToDevice));
    MVC_HIP(hipMemcpy(dr.p, r, sizeof(double) * rows, hipMemcpyHostToDevice));
    const unsigned blocks = (unsigned)((rows * 64 + 255) / 256);
    hipLaunchKernelGGL(mvc_spec_tree_kernel, dim3(blocks), dim3(256), 0, 0, (const double *)dx.p, rows, n,
                       (const double *)dr.p, ds.p, dsel.p);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipMemcpy(sums, ds.p, sizeof(double) * rows, hipMemcpyDeviceToHost));
    MVC_HIP(hipMemcpy(sel, dsel.p, sizeof(int64_t) * rows, hipMemcpyDeviceToHost));
    return MVC_OK;
  } catch (const mvc::Error &e) {
    if (err && errlen) snprintf(err, errlen, "%s", e.what());
    return e.code;
  } catch (const std::exception &e) {
    return spec_fail(e, err, errlen);
  }
}

extern "C" int mvc_device_gemm_check(int device, const double *Y, const double *S1, int64_t n, int64_t K, int64_t D,
                                     double *G, char *err, size_t errlen) {
  try {
    if (n % 16 || K % 16 || D % 4) throw mvc::Error(MVC_ERR_ARG, "gemm check needs n%16==K%16==D%4==0");
    MVC_HIP(hipSetDevice(device));
    DBuf<double> dy(n * D), ds(K * D), dg(n * K);
    MVC_HIP(hipMemcpy(dy.p, Y, sizeof(double) * n * D, hipMemcpyHostToDevice));
    MVC_HIP(hipMemcpy(ds.p, S1, sizeof(double) * K * D, hipMemcpyHostToDevice));
    const int64_t tiles = (n / 16) * (K / 16);
    hipLaunchKernelGGL(mvc_spec_gemm_kernel, dim3((unsigned)((tiles * 64 + 255) / 256)), dim3(256), 0, 0,
                       (const double *)dy.p, (const double *)ds.p, (int)n, (int)K, (int)D, dg.p);
    MVC_HIP(hipGetLastError());
    MVC_HIP(hipMemcpy(G, dg.p, sizeof(double) * n * K, hipMemcpyDeviceToHost));
    return MVC_OK;
  } catch (const mvc::Error &e) {
    if (err && errlen) snprintf(err, errlen, "%s", e.what());
    return e.code;
  } catch (const std::exception &e) {
    return spec_fail(e, err, errlen);
  }
}
