// stream_probe.hip — read-bandwidth probe for the lp producer's access
// pattern (diagnostic only, not part of the library).
//   A: per-wave 16 KB tiles (tile = gw + m * NWT), 1 KB per wave-load, ring
//      of RP loads in flight, 16 B per lane (the lpview A-fragment stream)
//   B: plain grid-stride 16 B/lane coalesced read of the same buffer
//   C: pattern A plus MFMA-free fake epilogue stores (4 per tile)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2 __attribute__((ext_vector_type(2)));

template <int RP, int SPPT, int STORE>
__global__ __launch_bounds__(512) void probeA(const d2 *y, int ntile, double *out, double *lp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, BW = blockDim.x >> 6;
  const int gw = blockIdx.x * BW + w, NWT = gridDim.x * BW;
  if (gw >= ntile) return;
  const int nmy = (ntile - gw + NWT - 1) / NWT;
  auto tptr = [&](int m) { return y + (size_t)(gw + min(m, nmy - 1) * NWT) * SPPT * 64 + lane; };
  d2 ring[RP];
#pragma unroll
  for (int u = 0; u < RP; ++u) ring[u] = tptr(0)[u * 64];
  double acc = 0.0;
  for (int m = 0; m < nmy; ++m) {
    const d2 *cur = tptr(m), *nxt = tptr(m + 1);
#pragma unroll
    for (int q = 0; q < SPPT; ++q) {
      const int u = q % RP;
      const d2 a = ring[u];
      ring[u] = (q + RP < SPPT) ? cur[(q + RP) * 64] : nxt[(q + RP - SPPT) * 64];
      acc += a[0] + a[1];
      __builtin_amdgcn_sched_barrier(0);
    }
    const int tile = gw + m * NWT;
    if (STORE == 1) {          // lpview today: 16 lines x 32 B per instruction
#pragma unroll
      for (int r = 0; r < 4; ++r) lp[((size_t)tile * 8 + (lane & 15)) * 16 + (lane >> 4) + 4 * r] = acc;
    } else if (STORE == 2) {   // 4 x 512 B contiguous (dwordx2 per lane)
#pragma unroll
      for (int r = 0; r < 4; ++r) lp[(size_t)tile * 128 + r * 64 + lane] = acc;
    } else if (STORE == 3) {   // 2 x 1 KB contiguous (dwordx4 per lane)
      d2 *l2 = (d2 *)lp;
#pragma unroll
      for (int r = 0; r < 2; ++r) l2[(size_t)tile * 64 + r * 64 + lane] = (d2){acc, acc};
    }
  }
  if (acc == 12345.678) out[0] = acc;
}

typedef double d4 __attribute__((ext_vector_type(4)));
// pattern A + NT MFMA tiles per k-step (B from registers), no epilogue
template <int NT>
__global__ __launch_bounds__(384) void probeM(const d2 *y, int ntile, double *out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, BW = blockDim.x >> 6;
  const int gw = blockIdx.x * BW + w, NWT = gridDim.x * BW;
  if (gw >= ntile) return;
  const int nmy = (ntile - gw + NWT - 1) / NWT;
  constexpr int RP = 8, SPPT = 16;
  auto tptr = [&](int m) { return y + (size_t)(gw + min(m, nmy - 1) * NWT) * SPPT * 64 + lane; };
  d2 ring[RP];
#pragma unroll
  for (int u = 0; u < RP; ++u) ring[u] = tptr(0)[u * 64];
  d4 acc[NT];
  const double b = 1.0 + lane * 1e-3;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = (d4){0, 0, 0, 0};
  for (int m = 0; m < nmy; ++m) {
    const d2 *cur = tptr(m), *nxt = tptr(m + 1);
#pragma unroll
    for (int q = 0; q < SPPT; ++q) {
      const int u = q % RP;
      const d2 a = ring[u];
      ring[u] = (q + RP < SPPT) ? cur[(q + RP) * 64] : nxt[(q + RP - SPPT) * 64];
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], b, acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], b, acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  double s = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  if (s == 12345.678) out[0] = s;
}
// MFMA throughput only: independent chains, no memory
template <int NT>
__global__ __launch_bounds__(256) void probeF(int iters, double *out) {
  d4 acc[NT];
  const double a = 1.0 + threadIdx.x * 1e-6, b = 0.999;
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = (d4){0, 0, 0, 0};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  if (s == 12345.678) out[0] = s;
}

__global__ void probeB(const d2 *y, size_t n2, double *out) {
  double acc = 0.0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const d2 a = y[i];
    acc += a[0] + a[1];
  }
  if (acc == 12345.678) out[0] = acc;
}

int main() {
  const int ntile = 62500, SPPT = 16;
  const size_t n2 = (size_t)ntile * SPPT * 64;      // d2 elements: 1.024 GB
  d2 *y; double *out, *lp;
  hipMalloc(&y, n2 * 16); hipMalloc(&out, 8); hipMalloc(&lp, (size_t)ntile * 8 * 16 * 8);
  hipMemset(y, 0, n2 * 16);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](const char *name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.1f us  %6.2f TB/s\n", name, ms * 100.0, n2 * 16 / (ms / 10 * 1e-3) / 1e12);
  };
  for (int bpc : {1, 2}) {
    char nm[64];
    snprintf(nm, 64, "A rp8 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<8, 16, 0>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
    snprintf(nm, 64, "A rp4 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<4, 16, 0>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
    snprintf(nm, 64, "A rp16 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<16, 16, 0>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
    snprintf(nm, 64, "C1 rp8 scattered 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<8, 16, 1>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
    snprintf(nm, 64, "C2 rp8 4x512B 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<8, 16, 2>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
    snprintf(nm, 64, "C3 rp8 2x1KB 512t x %d/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((probeA<8, 16, 3>), dim3(256 * bpc), dim3(512), 0, 0, y, ntile, out, lp); });
  }
  for (int wpb : {4, 6, 8}) {
    char nm[64];
    snprintf(nm, 64, "M NT=1 %dw x 2/CU", wpb);
    timeit(nm, [&] { hipLaunchKernelGGL((probeM<1>), dim3(512), dim3(64 * wpb), 0, 0, y, ntile, out); });
    snprintf(nm, 64, "M NT=2 %dw x 2/CU", wpb);
    timeit(nm, [&] { hipLaunchKernelGGL((probeM<2>), dim3(512), dim3(64 * wpb), 0, 0, y, ntile, out); });
    snprintf(nm, 64, "M NT=4 %dw x 2/CU", wpb);
    timeit(nm, [&] { hipLaunchKernelGGL((probeM<4>), dim3(512), dim3(64 * wpb), 0, 0, y, ntile, out); });
  }
  {
    const int iters = 4096;
    hipEvent_t f0, f1; hipEventCreate(&f0); hipEventCreate(&f1);
    for (int nt : {1, 2, 4}) {
      auto L = [&] {
        if (nt == 1) hipLaunchKernelGGL((probeF<1>), dim3(256 * 4), dim3(256), 0, 0, iters, out);
        if (nt == 2) hipLaunchKernelGGL((probeF<2>), dim3(256 * 4), dim3(256), 0, 0, iters, out);
        if (nt == 4) hipLaunchKernelGGL((probeF<4>), dim3(256 * 4), dim3(256), 0, 0, iters, out);
      };
      L(); hipDeviceSynchronize();
      hipEventRecord(f0); L(); hipEventRecord(f1); hipEventSynchronize(f1);
      float ms; hipEventElapsedTime(&ms, f0, f1);
      const double flops = 256.0 * 4 * 4 * (double)iters * nt * 2048;   // waves * mfma * 16*16*4*2
      printf("F mfma_f64_16x16x4 chains=%d      %8.1f us  %6.2f TFLOP/s\n", nt, ms * 1e3, flops / (ms * 1e-3) / 1e12);
    }
  }
  timeit("B grid-stride 256t x 8192", [&] { hipLaunchKernelGGL(probeB, dim3(8192), dim3(256), 0, 0, y, n2, out); });
  timeit("B grid-stride 256t x 2048", [&] { hipLaunchKernelGGL(probeB, dim3(2048), dim3(256), 0, 0, y, n2, out); });
  return 0;
}
