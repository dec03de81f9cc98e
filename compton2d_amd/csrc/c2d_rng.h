/*
 * c2d_rng.h — per-lane counter-based RNG keyed by packet lineage.
 *
 * Replaces the reference's lagged-Fibonacci zone streams (src/rand.f:9-316:
 * seed_zone, initialize_rand, fibran, RNFSTR/RNFARR) whose draws depend on
 * the depth-first order in which one worker tracks every packet of a zone.
 * Here every packet owns a Philox4x32-10 stream (key = 64-bit lineage key,
 * counter = draws consumed), and children derive their keys from the
 * parent's key at the point of the split, so a packet history is the same
 * whatever lane, wave, generation or GPU tracks it.
 *
 * Lineage rules (shared by the HIP kernels and the oracle's lineage mode):
 *   step key      S  = derive(seed, TAG_STEP, ncycle, 0)
 *   volume source    = derive(S, TAG_VOL,   n, cell)          n = packet index in zone
 *   surface source   = derive(S, TAG_SURF+side, n, surface)   side 0..3 = i,o,u,l
 *   census source    = key stored in the census record
 *   probe copy p     = derive(K_src, TAG_PROBE, p, 0)         (imctrk2d.f:125 split1 loop)
 *   recombined       = derive(K_src, TAG_RECOMB, 0, 0)        (imctrk2d.f:690-704)
 *   scatter copy ii  = derive(K_par, TAG_SCAT2, ii, ctr_par)  (imctrk2d.f:611 split2 loop)
 *   split3 copy ii2  = derive(K_chd, TAG_SCAT3, ii2, ctr_chd) (imctrk2d.f:633 split3 loop)
 *   census key       = derive(K_pkt, TAG_CENSUS, ctr_pkt, 0)  (imctrk2d.f:571 new seed)
 */
#ifndef C2D_RNG_H
#define C2D_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define C2D_RHD __host__ __device__ __forceinline__
#else
#define C2D_RHD static inline
#endif

#define C2D_TAG_STEP    0x01u
#define C2D_TAG_VOL     0x02u
#define C2D_TAG_SURF    0x03u   /* + side (0..3) */
#define C2D_TAG_PROBE   0x07u
#define C2D_TAG_RECOMB  0x08u
#define C2D_TAG_SCAT2   0x09u
#define C2D_TAG_SCAT3   0x0Au
#define C2D_TAG_CENSUS  0x0Bu

#define C2D_DRAW_C3     0x5EEDD1CEu
#define C2D_DERIVE_C3   0x9E3779B9u

C2D_RHD uint32_t c2d_mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

/* Philox4x32-10 (Salmon et al., SC'11). */
C2D_RHD void c2d_philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = c2d_mulhi32(M0, c[0]), lo0 = M0 * c[0];
    uint32_t hi1 = c2d_mulhi32(M1, c[2]), lo1 = M1 * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += W0; k1 += W1;
  }
}

/* Uniform in (0,1): 53 random bits, never 0 or 1 (all operations exact). */
C2D_RHD double c2d_u01_bits(uint32_t a, uint32_t b) {
  uint64_t x = (((uint64_t)a << 32) | (uint64_t)b) >> 11;
  return ((double)x + 0.5) * 1.1102230246251565404e-16;   /* 2^-53 */
}

/* Draw number n of stream `key`. */
C2D_RHD double c2d_draw(uint64_t key, uint32_t n) {
  uint32_t c[4] = {n, 0u, 0u, C2D_DRAW_C3};
  c2d_philox(c, (uint32_t)key, (uint32_t)(key >> 32));
  return c2d_u01_bits(c[0], c[1]);
}

C2D_RHD uint64_t c2d_derive(uint64_t key, uint32_t tag, uint32_t a, uint32_t b) {
  uint32_t c[4] = {a, b, tag, C2D_DERIVE_C3};
  c2d_philox(c, (uint32_t)key, (uint32_t)(key >> 32));
  return ((uint64_t)c[1] << 32) | (uint64_t)c[0];
}

C2D_RHD uint64_t c2d_step_key(uint64_t seed, int32_t ncycle) {
  return c2d_derive(seed, C2D_TAG_STEP, (uint32_t)ncycle, 0u);
}

#endif /* C2D_RNG_H */
