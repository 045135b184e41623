// mvc_ari.hip — adjusted Rand index of two labelings on the device (SURVEY
// §8f f4: the caller's ARI, New_Simulation.R:5,189, mcclust::arandi).
//
// Three passes over HBM-resident labels, all integer work (order-free, so the
// result does not depend on the launch shape):
//   1. label ranges (wave min/max, one atomic per wave);
//   2. contingency counts n_ij and the margins (per-block LDS histograms when
//      the table fits in LDS, else global atomics);
//   3. the three pair sums  a = sum C(n_ij,2), sa = sum C(row,2),
//      sb = sum C(col,2)  in uint64.
// The host combines the exact integers in mcclust::arandi's operation order
// (adjust = TRUE):  correc = sa * sb / C(n,2);
//                   (a - correc) / (0.5 sa + 0.5 sb - correc).
// R's choose(k, 2) of a count is the exact integer as a double for k < 2^26
// (nmath choose.c: n * ((n - 1) / 2), then rounded to an integer), and sums
// of exact integers below 2^53 are exact in any order, so the fp64 result
// equals arandi's bit for bit; a 1 x 1 table gives 0 / 0 = NaN, as in R.
#include <algorithm>
#include <climits>
#include <vector>

#include "mvc_host.h"
#include "mvc_internal.h"

namespace {

constexpr int kAriThreads = 256;
constexpr int64_t kAriMaxCells = (int64_t)1 << 26;   // contingency cells (256 MiB of uint32)
constexpr int kAriLdsCells = 8192;                  // per-block LDS histogram (32 KiB)

__device__ __forceinline__ int wave_min_i(int x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ int wave_max_i(int x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
  return x;
}

// rng[0..3] = min a, max a, min b, max b
__global__ __launch_bounds__(kAriThreads) void mvc_ari_range_kernel(const int32_t *a, const int32_t *b, int64_t n,
                                                                     int32_t *rng) {
  int lo_a = INT_MAX, hi_a = INT_MIN, lo_b = INT_MAX, hi_b = INT_MIN;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = a[i], y = b[i];
    lo_a = min(lo_a, x); hi_a = max(hi_a, x);
    lo_b = min(lo_b, y); hi_b = max(hi_b, y);
  }
  lo_a = wave_min_i(lo_a); hi_a = wave_max_i(hi_a);
  lo_b = wave_min_i(lo_b); hi_b = wave_max_i(hi_b);
  if ((threadIdx.x & 63) == 0) {
    atomicMin(rng + 0, lo_a); atomicMax(rng + 1, hi_a);
    atomicMin(rng + 2, lo_b); atomicMax(rng + 3, hi_b);
  }
}

// cont[ra * rb] (row-major, row = a label), rows[ra], cols[rb]
__global__ __launch_bounds__(kAriThreads) void mvc_ari_count_kernel(const int32_t *a, const int32_t *b, int64_t n,
                                                                     const int32_t *rng, uint32_t *cont,
                                                                     uint32_t *rows, uint32_t *cols) {
  extern __shared__ uint32_t s_h[];
  const int lo_a = rng[0], lo_b = rng[2];
  const int ra = rng[1] - lo_a + 1, rb = rng[3] - lo_b + 1;
  const int64_t cells = (int64_t)ra * rb;
  const bool lds = cells + ra + rb <= kAriLdsCells;   // uniform over the grid
  if (lds) {
    for (int k = threadIdx.x; k < cells + ra + rb; k += blockDim.x) s_h[k] = 0;
    __syncthreads();
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = a[i] - lo_a, c = b[i] - lo_b;
    if (lds) {
      atomicAdd(s_h + (int64_t)r * rb + c, 1u);
      atomicAdd(s_h + cells + r, 1u);
      atomicAdd(s_h + cells + ra + c, 1u);
    } else {
      atomicAdd(cont + (int64_t)r * rb + c, 1u);
      atomicAdd(rows + r, 1u);
      atomicAdd(cols + c, 1u);
    }
  }
  if (lds) {
    __syncthreads();
    for (int k = threadIdx.x; k < cells + ra + rb; k += blockDim.x) {
      const uint32_t v = s_h[k];
      if (!v) continue;
      if (k < cells) atomicAdd(cont + k, v);
      else if (k < cells + ra) atomicAdd(rows + (k - cells), v);
      else atomicAdd(cols + (k - cells - ra), v);
    }
  }
}

__device__ __forceinline__ unsigned long long pairs(uint32_t c) {
  return (unsigned long long)c * (c - (c > 0 ? 1u : 0u)) / 2ull;
}

// sums[0] = sum C(n_ij, 2), sums[1] = sum C(row, 2), sums[2] = sum C(col, 2)
__global__ __launch_bounds__(kAriThreads) void mvc_ari_pairs_kernel(const int32_t *rng, const uint32_t *cont,
                                                                     const uint32_t *rows, const uint32_t *cols,
                                                                     unsigned long long *sums) {
  const int ra = rng[1] - rng[0] + 1, rb = rng[3] - rng[2] + 1;
  const int64_t cells = (int64_t)ra * rb;
  unsigned long long s0 = 0, s1 = 0, s2 = 0;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < cells + ra + rb;
       k += (int64_t)gridDim.x * blockDim.x) {
    if (k < cells) s0 += pairs(cont[k]);
    else if (k < cells + ra) s1 += pairs(rows[k - cells]);
    else s2 += pairs(cols[k - cells - ra]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (s0) atomicAdd(sums + 0, s0);
    if (s1) atomicAdd(sums + 1, s1);
    if (s2) atomicAdd(sums + 2, s2);
  }
}

template <class Tp>
struct DMem {
  Tp *p = nullptr;
  explicit DMem(size_t n) { MVC_HIP(hipMalloc(&p, sizeof(Tp) * std::max<size_t>(n, 1))); }
  ~DMem() { if (p) hipFree(p); }
};

}  // namespace

namespace mvc {

// mcclust::arandi (adjust = TRUE) on exact pair counts, in R's left-to-right
// operation order:
//   correc <- sum(choose(tab.1,2)) * sum(choose(tab.2,2)) / choose(n,2)
//   (sum(choose(tab.12,2)) - correc) /
//       (0.5*sum(choose(tab.1,2)) + 0.5*sum(choose(tab.2,2)) - correc)
// A 1 x 1 table (or n < 2) gives NaN there (0/0); IEEE does the same here.
double ari_from_pairs(uint64_t a_, uint64_t sa_, uint64_t sb_, int64_t n) {
  const double a = (double)a_, sa = (double)sa_, sb = (double)sb_;
  const double nn = (double)((uint64_t)n * (uint64_t)(n - 1) / 2);
  const double correc = (sa * sb) / nn;
  return (a - correc) / ((0.5 * sa + 0.5 * sb) - correc);
}

// ARI of two device label arrays on `stream` (synchronises it).
double ari_device(const int32_t *da, const int32_t *db, int64_t n, hipStream_t stream) {
  if (n < 1) throw Error(MVC_ERR_ARG, "ari: n must be >= 1");
  DMem<int32_t> rng(4);
  const int32_t init[4] = {INT_MAX, INT_MIN, INT_MAX, INT_MIN};
  MVC_HIP(hipMemcpyAsync(rng.p, init, sizeof(init), hipMemcpyHostToDevice, stream));
  const unsigned grid = (unsigned)std::min<int64_t>(2048, (n + kAriThreads - 1) / kAriThreads);
  hipLaunchKernelGGL(mvc_ari_range_kernel, dim3(grid), dim3(kAriThreads), 0, stream, da, db, n, rng.p);
  MVC_HIP(hipGetLastError());
  int32_t h[4];
  MVC_HIP(hipMemcpyAsync(h, rng.p, sizeof(h), hipMemcpyDeviceToHost, stream));
  MVC_HIP(hipStreamSynchronize(stream));
  const int64_t ra = (int64_t)h[1] - h[0] + 1, rb = (int64_t)h[3] - h[2] + 1;
  if (ra * rb > kAriMaxCells)
    throw Error(MVC_ERR_UNSUPPORTED, "ari: label ranges too wide for the contingency table (range_a * range_b > 2^26)");
  const int64_t cells = ra * rb;
  DMem<uint32_t> cnt(cells + ra + rb);
  DMem<unsigned long long> sums(3);
  MVC_HIP(hipMemsetAsync(cnt.p, 0, sizeof(uint32_t) * (cells + ra + rb), stream));
  MVC_HIP(hipMemsetAsync(sums.p, 0, sizeof(unsigned long long) * 3, stream));
  const bool lds = cells + ra + rb <= kAriLdsCells;
  hipLaunchKernelGGL(mvc_ari_count_kernel, dim3(grid), dim3(kAriThreads), lds ? sizeof(uint32_t) * kAriLdsCells : 0,
                     stream, da, db, n, (const int32_t *)rng.p, cnt.p, cnt.p + cells, cnt.p + cells + ra);
  MVC_HIP(hipGetLastError());
  const unsigned pgrid = (unsigned)std::min<int64_t>(1024, (cells + ra + rb + kAriThreads - 1) / kAriThreads);
  hipLaunchKernelGGL(mvc_ari_pairs_kernel, dim3(pgrid), dim3(kAriThreads), 0, stream, (const int32_t *)rng.p,
                     (const uint32_t *)cnt.p, (const uint32_t *)(cnt.p + cells), (const uint32_t *)(cnt.p + cells + ra),
                     sums.p);
  MVC_HIP(hipGetLastError());
  unsigned long long s[3];
  MVC_HIP(hipMemcpyAsync(s, sums.p, sizeof(s), hipMemcpyDeviceToHost, stream));
  MVC_HIP(hipStreamSynchronize(stream));
  return ari_from_pairs(s[0], s[1], s[2], n);
}

}  // namespace mvc
