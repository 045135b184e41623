/*
 * mvc_philox.h — counter-based Philox4x32-10 RNG shared by the HIP sampler
 * and the CPU oracle (one spec, compiled by hipcc for gfx950 and by gcc).
 *
 * Replaces the reference's RNG layer:
 *   - /root/reference/Multiview/multiview_rng.h:9-24 (dead std::mt19937 code)
 *   - R::runif / R::rnorm calls at multiview_utils.cpp:261,305-306 and
 *     multiview_gibbs.cpp:26,56 (R's Mersenne-Twister + INVERSION normals).
 *
 * Philox4x32-10 is the published Random123 generator (Salmon et al., SC'11):
 * multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key bumps 0x9E3779B9 / 0xBB67AE85,
 * 10 rounds. Known-answer vectors are checked in tests/test_rng_math.py.
 *
 * Streams (all keyed by the 64-bit user seed):
 *   MVC_TAG_SEQ  : sequential stream (exact mode and initialisation), counter
 *                  {draw_lo, draw_hi, chain, TAG}; one Philox block per
 *                  uniform.  This stands in for R's unif_rand() stream.
 *   MVC_TAG_Z    : parallel-mode table draw of customer i in sweep s,
 *                  counter {i, s, chain, TAG}.
 *   MVC_TAG_Z2   : parallel-mode birth resolution (join a table born
 *                  earlier in the sweep or open one), counter {i, s, chain, TAG}.
 *   MVC_TAG_DISH : parallel-mode birth dish draw, counter {i, s, chain,
 *                  TAG + 1 + v}.
 *   MVC_TAG_MH   : parallel-mode hyperparameter stream, counter
 *                  {draw, s, chain, TAG}.
 */
#ifndef MVC_PHILOX_H
#define MVC_PHILOX_H

#include <stdint.h>

#if defined(__HIPCC__)
#define MVC_HD static __host__ __device__ __forceinline__
#else
#define MVC_HD static inline
#endif

#define MVC_TAG_SEQ  0x4D564345u /* 'MVCE' */
#define MVC_TAG_Z    0x4D565A30u /* 'MVZ0' */
#define MVC_TAG_Z2   0x4D565A32u /* 'MVZ2' birth resolution */
#define MVC_TAG_DISH 0x4D564400u /* 'MVD\0' + 1 + view */
#define MVC_TAG_MH   0x4D564D48u /* 'MVMH' */

typedef struct mvc_u32x4 { uint32_t x, y, z, w; } mvc_u32x4;

MVC_HD mvc_u32x4 mvc_philox4x32_10(mvc_u32x4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c.z;
    mvc_u32x4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

/* 52 random bits -> double in the OPEN interval (0,1):
 * u = (b + 0.5) * 2^-52, every step exact. Never 0, never 1. */
MVC_HD double mvc_u01_from_bits(uint32_t lo, uint32_t hi) {
  const uint64_t b = (((uint64_t)hi << 32) | (uint64_t)lo) >> 12;
  return ((double)b + 0.5) * 2.220446049250313080847e-16; /* 2^-52 */
}

MVC_HD double mvc_uniform(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t tag) {
  mvc_u32x4 c;
  c.x = c0; c.y = c1; c.z = c2; c.w = tag;
  const mvc_u32x4 r = mvc_philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return mvc_u01_from_bits(r.x, r.y);
}

/* Draw number `idx` of chain `chain`'s sequential stream. */
MVC_HD double mvc_seq_uniform(uint64_t seed, uint32_t chain, uint64_t idx) {
  return mvc_uniform(seed, (uint32_t)idx, (uint32_t)(idx >> 32), chain, MVC_TAG_SEQ);
}

#endif /* MVC_PHILOX_H */
