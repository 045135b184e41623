/*
 * mvc_pmath.h — "portable math": fp64 exp / log / lgamma / normal-quantile
 * built only from IEEE-754 correctly rounded operations (+ - * / fma sqrt)
 * and integer bit manipulation, so the SAME source gives bit-identical
 * results on the gfx950 device (hipcc) and on the x86-64 host (gcc).
 *
 * Both sides MUST be compiled with -ffp-contract=off and without fast-math:
 * every fused multiply-add below is written explicitly with __builtin_fma.
 *
 * Why: the reference chain (multiview_gibbs.cpp:157-200) is chaotic in the
 * last ulp; bit-exact GPU == CPU parity needs one exp/log implementation on
 * both sides instead of glibc libm vs. the device libm.  The oracle can also
 * run with glibc libm (the reference's own std::exp/std::log) and the
 * agreement rate between the two math modes is reported by the tests.
 *
 * Algorithms:
 *   exp   : k = rint(x/ln2); r = x - k ln2 (two-constant Cody-Waite via fma);
 *           Taylor series of e^r to r^14 (Horner/fma); scale by 2^k.
 *   log   : x = 2^e m, m in [sqrt2/2, sqrt2); f = m-1, s = f/(2+f);
 *           log(1+f) = f - hfsq + s (hfsq + R(s^2)),  R(z) = sum 2 z^n/(2n+1)
 *           (the classic fdlibm decomposition, Taylor coefficients).
 *   lgamma: upward recurrence to x >= 12, then Stirling series (B_2k terms).
 *   qnorm : Wichura's AS241 (PPND16) exactly as R's qnorm5 for
 *           lower_tail=1, log_p=0 (R's norm_rand INVERSION method).
 * Accuracy vs. glibc is measured in tests/test_rng_math.py.
 */
#ifndef MVC_PMATH_H
#define MVC_PMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define MVC_PM static __host__ __device__ __forceinline__
#else
#define MVC_PM static inline
#endif

MVC_PM uint64_t mvc_d2u(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
MVC_PM double mvc_u2d(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }

#define MVC_PM_INF  (mvc_u2d(0x7FF0000000000000ull))
#define MVC_PM_NAN  (mvc_u2d(0x7FF8000000000000ull))

#define MVC_LN2_HI 0.6931471805598903          /* 0x3fe62e42fefa3800, 42 bits */
#define MVC_LN2_LO 5.497923018708371e-14       /* ln2 - LN2_HI */
#define MVC_INVLN2 1.4426950408889634
#define MVC_HALF_LOG_2PI 0.9189385332046728
#define MVC_PI 3.14159265358979323846          /* M_PI as used by the reference */

#if defined(__HIPCC__)
/* The exp's Horner steps from 1/14! down to 1/2! as ONE inline-asm block of
 * three-operand v_fma_f64 (coefficients in VGPRs or SGPRs): the same
 * instructions on the same values as the host's __builtin_fma chain, without
 * the compiler's v_mov_b64 + v_fmac_f64 pairs and without the s_nop it puts
 * after every separate asm statement.  Consecutive dependent v_fma_f64 need
 * no wait states on gfx950 (the compiler emits them back to back itself). */
#if !defined(MVC_PM_NO_ASM_FMA)
#define MVC_HORNER12(p, r, K0, K)                                                                   \
  asm("v_fma_f64 %0, %2, %1, %3\n\tv_fma_f64 %0, %0, %1, %4\n\tv_fma_f64 %0, %0, %1, %5\n\t"         \
      "v_fma_f64 %0, %0, %1, %6\n\tv_fma_f64 %0, %0, %1, %7\n\tv_fma_f64 %0, %0, %1, %8\n\t"          \
      "v_fma_f64 %0, %0, %1, %9\n\tv_fma_f64 %0, %0, %1, %10\n\tv_fma_f64 %0, %0, %1, %11\n\t"        \
      "v_fma_f64 %0, %0, %1, %12\n\tv_fma_f64 %0, %0, %1, %13"                                     \
      : "=&v"(p)                                                                                   \
      : "v"(r), K0(1.1470745597729725e-11), K(1.6059043836821613e-10), K(2.08767569878681e-09),     \
        K(2.505210838544172e-08), K(2.755731922398589e-07), K(2.7557319223985893e-06),             \
        K(2.48015873015873e-05), K(0.0001984126984126984), K(0.001388888888888889),                \
        K(0.008333333333333333), K(0.041666666666666664), K(0.16666666666666666))
/* The same steps for two independent arguments interleaved in one block
 * (each value's instructions and operands unchanged, so the same bits): two
 * exps' dependent chains overlap where one wave per SIMD has nothing else to
 * issue. */
#define MVC_HORNER12X2(p, q, r, s, K0, K)                                                            \
  asm("v_fma_f64 %0, %4, %2, %5\n\tv_fma_f64 %1, %4, %3, %5\n\t"                                       \
      "v_fma_f64 %0, %0, %2, %6\n\tv_fma_f64 %1, %1, %3, %6\n\t"                                       \
      "v_fma_f64 %0, %0, %2, %7\n\tv_fma_f64 %1, %1, %3, %7\n\t"                                       \
      "v_fma_f64 %0, %0, %2, %8\n\tv_fma_f64 %1, %1, %3, %8\n\t"                                       \
      "v_fma_f64 %0, %0, %2, %9\n\tv_fma_f64 %1, %1, %3, %9\n\t"                                       \
      "v_fma_f64 %0, %0, %2, %10\n\tv_fma_f64 %1, %1, %3, %10\n\t"                                     \
      "v_fma_f64 %0, %0, %2, %11\n\tv_fma_f64 %1, %1, %3, %11\n\t"                                     \
      "v_fma_f64 %0, %0, %2, %12\n\tv_fma_f64 %1, %1, %3, %12\n\t"                                     \
      "v_fma_f64 %0, %0, %2, %13\n\tv_fma_f64 %1, %1, %3, %13\n\t"                                     \
      "v_fma_f64 %0, %0, %2, %14\n\tv_fma_f64 %1, %1, %3, %14\n\t"                                     \
      "v_fma_f64 %0, %0, %2, %15\n\tv_fma_f64 %1, %1, %3, %15"                                         \
      : "=&v"(p), "=&v"(q)                                                                         \
      : "v"(r), "v"(s), K0(1.1470745597729725e-11), K(1.6059043836821613e-10),                     \
        K(2.08767569878681e-09), K(2.505210838544172e-08), K(2.755731922398589e-07),               \
        K(2.7557319223985893e-06), K(2.48015873015873e-05), K(0.0001984126984126984),              \
        K(0.001388888888888889), K(0.008333333333333333), K(0.041666666666666664),                 \
        K(0.16666666666666666))
#else
#define MVC_HORNER12X2(p, q, r, s, K0, K) \
  do {                                    \
    MVC_HORNER12(p, r, K0, K);            \
    MVC_HORNER12(q, s, K0, K);            \
  } while (0)
#define MVC_HORNER12(p, r, K0, K)                                                                   \
  do {                                                                                              \
    p = __builtin_fma(1.1470745597729725e-11, r, 1.6059043836821613e-10);                           \
    p = __builtin_fma(p, r, 2.08767569878681e-09);                                                  \
    p = __builtin_fma(p, r, 2.505210838544172e-08); p = __builtin_fma(p, r, 2.755731922398589e-07); \
    p = __builtin_fma(p, r, 2.7557319223985893e-06); p = __builtin_fma(p, r, 2.48015873015873e-05); \
    p = __builtin_fma(p, r, 0.0001984126984126984); p = __builtin_fma(p, r, 0.001388888888888889);  \
    p = __builtin_fma(p, r, 0.008333333333333333); p = __builtin_fma(p, r, 0.041666666666666664);   \
    p = __builtin_fma(p, r, 0.16666666666666666);                                                   \
  } while (0)
#endif
#endif

MVC_PM double mvc_exp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  /* Device: the same value without branches (divergence-free; 64 unrolled
   * calls in the draw kernel would otherwise spill exec masks).  The three
   * scalings below all equal the correctly rounded e * 2^k, which is what
   * v_ldexp_f64 computes; the range checks become selects. */
  {
    const double shifter = 6755399441055744.0;
    double kd = x * MVC_INVLN2;
    kd = kd + shifter;
    kd = kd - shifter;
    kd = __builtin_fmin(__builtin_fmax(kd, -1100.0), 1100.0);
    const int k = (int)kd;
    double r = __builtin_fma(-kd, MVC_LN2_HI, x);
    r = __builtin_fma(-kd, MVC_LN2_LO, r);
    /* the Horner steps to 1/2!: one asm block (MVC_HORNER12) */
    double p;
    MVC_HORNER12(p, r, "v", "v");
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    const double e = __builtin_fma(p, r, 1.0);
    double res = __builtin_amdgcn_ldexp(e, k);
    res = (x > 709.782712893384) ? MVC_PM_INF : res;
    res = (x < -745.1332191019412) ? 0.0 : res;
    return (x == x) ? res : x + x;
  }
#endif
  if (!(x == x)) return x + x;
  if (x > 709.782712893384) return MVC_PM_INF;
  if (x < -745.1332191019412) return 0.0;
  const double shifter = 6755399441055744.0; /* 1.5 * 2^52 */
  double kd = x * MVC_INVLN2;
  kd = kd + shifter;
  kd = kd - shifter;                       /* round-to-nearest-even integer */
  const int k = (int)kd;
  double r = __builtin_fma(-kd, MVC_LN2_HI, x);
  r = __builtin_fma(-kd, MVC_LN2_LO, r);
  double p = 1.1470745597729725e-11;       /* 1/14! */
  p = __builtin_fma(p, r, 1.6059043836821613e-10);
  p = __builtin_fma(p, r, 2.08767569878681e-09);
  p = __builtin_fma(p, r, 2.505210838544172e-08);
  p = __builtin_fma(p, r, 2.755731922398589e-07);
  p = __builtin_fma(p, r, 2.7557319223985893e-06);
  p = __builtin_fma(p, r, 2.48015873015873e-05);
  p = __builtin_fma(p, r, 0.0001984126984126984);
  p = __builtin_fma(p, r, 0.001388888888888889);
  p = __builtin_fma(p, r, 0.008333333333333333);
  p = __builtin_fma(p, r, 0.041666666666666664);
  p = __builtin_fma(p, r, 0.16666666666666666);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double e = __builtin_fma(p, r, 1.0);
  if (k >= -1021 && k <= 1023) return e * mvc_u2d((uint64_t)(k + 1023) << 52);
  if (k > 1023) return (e * mvc_u2d((uint64_t)(k - 1 + 1023) << 52)) * 2.0;
  /* subnormal result: exact scale into the normal range, one rounding after */
  return (e * mvc_u2d((uint64_t)(k + 54 + 1023) << 52)) * 5.551115123125783e-17; /* 2^-54 */
}

#if defined(__HIPCC__)
/* mvc_exp with the Horner coefficients as SGPR operands: the same
 * instructions on the same values (bitwise equal to mvc_exp); for kernels
 * whose VGPR budget cannot hold 22 registers of hoisted constants. */
static __device__ __forceinline__ double mvc_exp_sk(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  /* Device: the same value without branches (divergence-free; 64 unrolled
   * calls in the draw kernel would otherwise spill exec masks).  The three
   * scalings below all equal the correctly rounded e * 2^k, which is what
   * v_ldexp_f64 computes; the range checks become selects. */
  {
    const double shifter = 6755399441055744.0;
    double kd = x * MVC_INVLN2;
    kd = kd + shifter;
    kd = kd - shifter;
    kd = __builtin_fmin(__builtin_fmax(kd, -1100.0), 1100.0);
    const int k = (int)kd;
    double r = __builtin_fma(-kd, MVC_LN2_HI, x);
    r = __builtin_fma(-kd, MVC_LN2_LO, r);
    /* the Horner steps to 1/2!: one asm block (MVC_HORNER12) */
    double p;
    MVC_HORNER12(p, r, "v", "s");   /* one SGPR operand per VOP3 */
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    const double e = __builtin_fma(p, r, 1.0);
    double res = __builtin_amdgcn_ldexp(e, k);
    res = (x > 709.782712893384) ? MVC_PM_INF : res;
    res = (x < -745.1332191019412) ? 0.0 : res;
    return (x == x) ? res : x + x;
  }
#else
  return mvc_exp(x);
#endif
}

/* mvc_exp for arguments x <= 709.78 that are not NaN (the draw's a - max
 * forms): the overflow and NaN selects are dropped, nothing else changes, so
 * it is bitwise equal to mvc_exp on that domain (the underflow select stays:
 * the clamped reduction is garbage below -745).  6 of ~28 instructions. */
static __device__ __forceinline__ double mvc_exp_le0(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double shifter = 6755399441055744.0;
  double kd = x * MVC_INVLN2;
  kd = kd + shifter;
  kd = kd - shifter;
  kd = __builtin_fmin(__builtin_fmax(kd, -1100.0), 1100.0);
  const int k = (int)kd;
  double r = __builtin_fma(-kd, MVC_LN2_HI, x);
  r = __builtin_fma(-kd, MVC_LN2_LO, r);
  double p;
  MVC_HORNER12(p, r, "v", "v");
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double e = __builtin_fma(p, r, 1.0);
  const double res = __builtin_amdgcn_ldexp(e, k);
  return (x < -745.1332191019412) ? 0.0 : res;
#else
  return mvc_exp(x);
#endif
}
/* Two mvc_exp_le0 at once (MVC_HORNER12X2): the same value for each. */
static __device__ __forceinline__ void mvc_exp_le0_x2(double x0, double x1, double &e0, double &e1) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double shifter = 6755399441055744.0;
  double kd0 = x0 * MVC_INVLN2, kd1 = x1 * MVC_INVLN2;
  kd0 = kd0 + shifter;
  kd1 = kd1 + shifter;
  kd0 = kd0 - shifter;
  kd1 = kd1 - shifter;
  kd0 = __builtin_fmin(__builtin_fmax(kd0, -1100.0), 1100.0);
  kd1 = __builtin_fmin(__builtin_fmax(kd1, -1100.0), 1100.0);
  const int k0 = (int)kd0, k1 = (int)kd1;
  double r0 = __builtin_fma(-kd0, MVC_LN2_HI, x0), r1 = __builtin_fma(-kd1, MVC_LN2_HI, x1);
  r0 = __builtin_fma(-kd0, MVC_LN2_LO, r0);
  r1 = __builtin_fma(-kd1, MVC_LN2_LO, r1);
  double p0, p1;
  MVC_HORNER12X2(p0, p1, r0, r1, "v", "v");
  p0 = __builtin_fma(p0, r0, 0.5);
  p1 = __builtin_fma(p1, r1, 0.5);
  p0 = __builtin_fma(p0, r0, 1.0);
  p1 = __builtin_fma(p1, r1, 1.0);
  const double a0 = __builtin_fma(p0, r0, 1.0), a1 = __builtin_fma(p1, r1, 1.0);
  const double res0 = __builtin_amdgcn_ldexp(a0, k0), res1 = __builtin_amdgcn_ldexp(a1, k1);
  e0 = (x0 < -745.1332191019412) ? 0.0 : res0;
  e1 = (x1 < -745.1332191019412) ? 0.0 : res1;
#else
  e0 = mvc_exp(x0);
  e1 = mvc_exp(x1);
#endif
}
/* mvc_exp_le0 with the Horner coefficients as SGPR operands (bitwise equal):
 * for kernels whose VGPR budget sets their occupancy. */
static __device__ __forceinline__ double mvc_exp_le0_sk(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double shifter = 6755399441055744.0;
  double kd = x * MVC_INVLN2;
  kd = kd + shifter;
  kd = kd - shifter;
  kd = __builtin_fmin(__builtin_fmax(kd, -1100.0), 1100.0);
  const int k = (int)kd;
  double r = __builtin_fma(-kd, MVC_LN2_HI, x);
  r = __builtin_fma(-kd, MVC_LN2_LO, r);
  double p;
  MVC_HORNER12(p, r, "v", "s");
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  const double e = __builtin_fma(p, r, 1.0);
  const double res = __builtin_amdgcn_ldexp(e, k);
  return (x < -745.1332191019412) ? 0.0 : res;
#else
  return mvc_exp(x);
#endif
}
#endif

MVC_PM double mvc_log(double x) {
  if (!(x == x)) return x + x;
  if (x < 0.0) return MVC_PM_NAN;
  if (x == 0.0) return -MVC_PM_INF;
  uint64_t u = mvc_d2u(x);
  if (u == 0x7FF0000000000000ull) return x;
  int e = 0;
  if (u < 0x0010000000000000ull) {          /* subnormal */
    x = x * 18014398509481984.0;            /* 2^54 */
    u = mvc_d2u(x);
    e = -54;
  }
  e += (int)(u >> 52) - 1023;
  uint64_t mant = u & 0x000FFFFFFFFFFFFFull;
  uint64_t ebits = 0x3FF0000000000000ull;
  if (mant > 0x6A09E667F3BCDull) {          /* m > sqrt(2): use m/2 */
    ebits = 0x3FE0000000000000ull;
    e += 1;
  }
  const double m = mvc_u2d(mant | ebits);
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double R = 0.08;                          /* 2/25 */
  R = __builtin_fma(R, z, 0.08695652173913043);
  R = __builtin_fma(R, z, 0.09523809523809523);
  R = __builtin_fma(R, z, 0.10526315789473684);
  R = __builtin_fma(R, z, 0.11764705882352941);
  R = __builtin_fma(R, z, 0.13333333333333333);
  R = __builtin_fma(R, z, 0.15384615384615385);
  R = __builtin_fma(R, z, 0.18181818181818182);
  R = __builtin_fma(R, z, 0.2222222222222222);
  R = __builtin_fma(R, z, 0.2857142857142857);
  R = __builtin_fma(R, z, 0.4);
  R = __builtin_fma(R, z, 0.6666666666666666);
  R = R * z;
  const double hfsq = 0.5 * f * f;
  if (e == 0) return f - (hfsq - s * (hfsq + R));
  const double dk = (double)e;
  return dk * MVC_LN2_HI - ((hfsq - (s * (hfsq + R) + dk * MVC_LN2_LO)) - f);
}

#if defined(__HIPCC__)
/* mvc_log without branches (device): every path of mvc_log computed with the
 * same operations, the result picked by selects, so it is bitwise equal to
 * mvc_log for every input and keeps a wavefront converged. */
static __device__ __forceinline__ double mvc_log_nb(double x) {
  const uint64_t u0 = mvc_d2u(x);
  const bool sub = u0 < 0x0010000000000000ull;           /* +0 and subnormals (x >= 0) */
  const double xs = sub ? x * 18014398509481984.0 : x;   /* 2^54 */
  const uint64_t u = mvc_d2u(xs);
  int e = (sub ? -54 : 0) + (int)((u >> 52) & 0x7FF) - 1023;
  const uint64_t mant = u & 0x000FFFFFFFFFFFFFull;
  const bool big = mant > 0x6A09E667F3BCDull;
  const uint64_t ebits = big ? 0x3FE0000000000000ull : 0x3FF0000000000000ull;
  e += big ? 1 : 0;
  const double m = mvc_u2d(mant | ebits);
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  double R = 0.08;
  R = __builtin_fma(R, z, 0.08695652173913043);
  R = __builtin_fma(R, z, 0.09523809523809523);
  R = __builtin_fma(R, z, 0.10526315789473684);
  R = __builtin_fma(R, z, 0.11764705882352941);
  R = __builtin_fma(R, z, 0.13333333333333333);
  R = __builtin_fma(R, z, 0.15384615384615385);
  R = __builtin_fma(R, z, 0.18181818181818182);
  R = __builtin_fma(R, z, 0.2222222222222222);
  R = __builtin_fma(R, z, 0.2857142857142857);
  R = __builtin_fma(R, z, 0.4);
  R = __builtin_fma(R, z, 0.6666666666666666);
  R = R * z;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)e;
  double res = (e == 0) ? f - (hfsq - s * (hfsq + R))
                        : dk * MVC_LN2_HI - ((hfsq - (s * (hfsq + R) + dk * MVC_LN2_LO)) - f);
  res = (u0 == 0x7FF0000000000000ull) ? x : res;
  res = (x == 0.0) ? -MVC_PM_INF : res;
  res = (x < 0.0) ? MVC_PM_NAN : res;
  return (x == x) ? res : x + x;
}
#endif

/* log Gamma(x) for x > 0 (used only by the parallel-mode EPPF). */
MVC_PM double mvc_lgamma_pos(double x) {
  if (!(x > 0.0)) return MVC_PM_NAN;
  if (x == MVC_PM_INF) return x;
  double prod = 1.0;
  double xx = x;
  while (xx < 12.0) { prod = prod * xx; xx = xx + 1.0; }
  const double ix = 1.0 / xx;
  const double ix2 = ix * ix;
  double ser = -0.029550653594771242;
  ser = __builtin_fma(ser, ix2, 0.00641025641025641);
  ser = __builtin_fma(ser, ix2, -0.0019175269175269176);
  ser = __builtin_fma(ser, ix2, 0.0008417508417508417);
  ser = __builtin_fma(ser, ix2, -0.0005952380952380953);
  ser = __builtin_fma(ser, ix2, 0.0007936507936507937);
  ser = __builtin_fma(ser, ix2, -0.002777777777777778);
  ser = __builtin_fma(ser, ix2, 0.08333333333333333);
  ser = ser * ix;
  double lg = (xx - 0.5) * mvc_log(xx) - xx;
  lg = lg + MVC_HALF_LOG_2PI;
  lg = lg + ser;
  return lg - mvc_log(prod);
}

#if defined(__HIPCC__)
/* mvc_lgamma_pos without branches (device): the recurrence's at most 12 steps
 * unrolled, a step once xx >= 12 leaving prod and xx unchanged (select), and
 * mvc_log_nb for the logs: the same operations on the same values as
 * mvc_lgamma_pos, so bitwise equal for every input, with the wavefront
 * converged when its lanes' arguments differ. */
static __device__ __forceinline__ double mvc_lgamma_pos_nb(double x) {
  double prod = 1.0;
  double xx = x;
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    const bool go = xx < 12.0;
    prod = go ? prod * xx : prod;
    xx = go ? xx + 1.0 : xx;
  }
  const double ix = 1.0 / xx;
  const double ix2 = ix * ix;
  double ser = -0.029550653594771242;
  ser = __builtin_fma(ser, ix2, 0.00641025641025641);
  ser = __builtin_fma(ser, ix2, -0.0019175269175269176);
  ser = __builtin_fma(ser, ix2, 0.0008417508417508417);
  ser = __builtin_fma(ser, ix2, -0.0005952380952380953);
  ser = __builtin_fma(ser, ix2, 0.0007936507936507937);
  ser = __builtin_fma(ser, ix2, -0.002777777777777778);
  ser = __builtin_fma(ser, ix2, 0.08333333333333333);
  ser = ser * ix;
  double lg = (xx - 0.5) * mvc_log_nb(xx) - xx;
  lg = lg + MVC_HALF_LOG_2PI;
  lg = lg + ser;
  double r = lg - mvc_log_nb(prod);
  r = (x == MVC_PM_INF) ? x : r;
  return (x > 0.0) ? r : MVC_PM_NAN;
}
#endif

/* R's qnorm5(p, 0, 1, lower_tail=TRUE, log_p=FALSE): Wichura AS241. */
MVC_PM double mvc_qnorm(double p) {
  if (!(p > 0.0 && p < 1.0)) {
    if (p == 0.0) return -MVC_PM_INF;
    if (p == 1.0) return MVC_PM_INF;
    return MVC_PM_NAN;
  }
  const double q = p - 0.5;
  double r, val;
  const double aq = q < 0.0 ? -q : q;
  if (aq <= 0.425) {
    r = 0.180625 - q * q;
    val = q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r +
                    67265.770927008700853) * r + 45921.953931549871457) * r +
                  13731.693765509461125) * r + 1971.5909503065514427) * r +
                133.14166789178437745) * r + 3.387132872796366608) /
          (((((((r * 5226.495278852545925 + 28729.085735721942674) * r +
                39307.89580009271061) * r + 21213.794301586595867) * r +
              5394.1960214247511077) * r + 687.1870074920579083) * r +
            42.313330701600911252) * r + 1.0);
    return val;
  }
  if (q > 0.0)
    r = 0.5 - p + 0.5;                       /* R_DT_CIv(p) */
  else
    r = p;
  r = __builtin_sqrt(-mvc_log(r));
  if (r <= 5.0) {
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r +
                .24178072517745061177) * r + 1.27045825245236838258) * r +
              3.64784832476320460504) * r + 5.7694972214606914055) * r +
            4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r +
                .0151986665636164571966) * r + .14810397642748007459) * r +
              .68976733498510000455) * r + 1.6763848301838038494) * r +
            2.05319162663775882187) * r + 1.0);
  } else {
    r += -5.0;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r +
                .0012426609473880784386) * r + .026532189526576123093) * r +
              .296560571828504891230) * r + 1.7848265399172913358) * r +
            5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r +
                1.8463183175100546818e-5) * r + 7.868691311456132591e-4) * r +
              .0148753612908506148525) * r + .13692988092273580531) * r +
            .59983220655588793769) * r + 1.0);
  }
  if (q < 0.0) val = -val;
  return val;
}

/* R's norm_rand(), INVERSION kind: two uniforms -> one N(0,1) variate. */
MVC_PM double mvc_norm_from_uniforms(double u1, double u2) {
  const double BIG = 134217728.0; /* 2^27 */
  const double u = (double)(int)(BIG * u1) + u2;
  return mvc_qnorm(u / BIG);
}

#endif /* MVC_PMATH_H */
