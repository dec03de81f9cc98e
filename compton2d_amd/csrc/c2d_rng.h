/*
 * c2d_rng.h — per-lane counter-based RNG keyed by packet lineage.
 *
 * Replaces the reference's lagged-Fibonacci zone streams (src/rand.f:9-316:
 * seed_zone, initialize_rand, fibran, RNFSTR/RNFARR) whose draws depend on
 * the depth-first order in which one worker tracks every packet of a zone.
 * Here every packet owns a counter-based stream (key = 64-bit lineage key,
 * counter = draws consumed): draw n of stream (key, sub) is the SplitMix64
 * output (Steele, Lea & Flood, OOPSLA 2014; passes BigCrush) for the state
 * key + gamma * ((sub << 32 | n) + 1), one 64-bit output per draw.  Children derive
 * their keys from the parent's key at the point of the split with
 * Philox4x32-10 (Salmon et al., SC'11), so a packet history is the same
 * whatever lane, wave, generation or GPU tracks it.
 *
 * A stream is (key, sub): sub = 0 for a packet's own stream, and the split1
 * copies of a source (which only differ in their random numbers) use
 * sub-streams of the source key instead of derived keys, so starting a
 * copy costs no key derivation.
 *
 * Lineage rules (shared by the HIP kernels and the oracle's lineage mode):
 *   step key      S  = derive(seed, TAG_STEP, ncycle, 0)
 *   volume source    = derive(S, TAG_VOL,   n, cell)          n = packet index in zone
 *   surface source   = derive(S, TAG_SURF+side, n, surface)   side 0..3 = i,o,u,l
 *   census source    = key stored in the census record
 *   probe copy p     = (K_src, sub 1+p)                       (imctrk2d.f:125 split1 loop)
 *   probe bundle g0  = (K_src, sub C2D_SUB_BUNDLE | g0)       probes g0.. tracked together:
 *                      their collision decisions and the colliders' absorption points
 *                      (DESIGN.md §2c);
 *   bundle points g0 = (K_src, sub C2D_SUB_ABSPT | g0)        the survivors' absorption points:
 *                      two 32-bit uniforms per 64-bit output (c2d_abspt), fresh
 *                      outputs for every shared step;
 *                      a collider's record carries (K_src, sub 1+p, bundle ctr)
 *   recombined       = (K_src, sub C2D_SUB_RECOMB)            (imctrk2d.f:690-704)
 *   scatter copy ii  = derive(K_par, TAG_SCAT2, ii, ctr_par; sub_par)  (imctrk2d.f:611)
 *   split3 copy ii2  = derive(K_chd, TAG_SCAT3, ii2, ctr_chd)          (imctrk2d.f:633)
 *   its resample k   = (K_split3, sub k), counter 0 at each attempt    (imctrk2d.f:634-648,
 *                      `goto 215`); the copy flies on from its first success's stream
 *   census key       = census_key(K_pkt, ctr_pkt, sub_pkt)             (imctrk2d.f:571)
 *   compb2d's first rejection loop (compb_2d.f:59-93): iteration j draws
 *                      counters c0 + 5j .. c0 + 5j + 4 of the packet's stream (c0:
 *                      the counter at the call), the rest of compb2d follows
 *                      c0 + 5 (j_accepted + 1)
 * Draw n of (key, sub) = u53(mix64(key + gamma * ((sub << 32 | n) + 1)));
 * derive(key, tag, a, b; sub) = Philox_key({a, b, tag | sub << 8, C_DERIVE}).
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
#ifndef C2D_PHILOX_MAD
#define C2D_PHILOX_MAD 0
#endif
#ifndef C2D_PHILOX_ROUNDS
#define C2D_PHILOX_ROUNDS 10
#endif
#pragma unroll
  for (int r = 0; r < C2D_PHILOX_ROUNDS; ++r) {
#if C2D_PHILOX_MAD
    /* one 32x32->64 product per multiplier (a single v_mad_u64_u32 on CDNA
     * instead of separate mul_hi / mul_lo) */
    const uint64_t p0 = (uint64_t)M0 * (uint64_t)c[0];
    const uint64_t p1 = (uint64_t)M1 * (uint64_t)c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
#else
    uint32_t hi0 = c2d_mulhi32(M0, c[0]), lo0 = M0 * c[0];
    uint32_t hi1 = c2d_mulhi32(M1, c[2]), lo1 = M1 * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
#endif
    k0 += W0; k1 += W1;
  }
}

/* Uniform in (0,1): 53 random bits, never 0 or 1 (all operations exact). */
C2D_RHD double c2d_u01_bits(uint32_t a, uint32_t b) {
  uint64_t x = (((uint64_t)a << 32) | (uint64_t)b) >> 11;
  return ((double)x + 0.5) * 1.1102230246251565404e-16;   /* 2^-53 */
}

#define C2D_SUB_RECOMB  0xFFFFFFu   /* 24-bit sub-stream ids: probes use 1 .. split1 */
#define C2D_SUB_BUNDLE  0x800000u   /* | g0: the stream of the probe bundle starting at g0 */
#define C2D_SUB_ABSPT   0xC00000u   /* | g0: that bundle's absorption-point stream          */

/* Uniform in (0,1) from 32 random bits, never 0 or 1 (exact). */
C2D_RHD double c2d_u01_32(uint32_t a) {
  return ((double)a + 0.5) * 2.3283064365386962890625e-10;   /* 2^-32 */
}

/* SplitMix64's output function. */
C2D_RHD uint64_t c2d_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* 64-bit output n of stream (key, sub): output (sub << 32 | n) of the
 * SplitMix64 sequence seeded with the key (state key + (i + 1) * gamma), so
 * the streams of one key are disjoint 2^32-long segments of it. */
C2D_RHD uint64_t c2d_stream64(uint64_t key, uint32_t sub, uint32_t n) {
  return c2d_mix64(key + 0x9E3779B97F4A7C15ull * ((((uint64_t)sub << 32) | (uint64_t)n) + 1ull));
}

/* Draw number n of stream (key, sub): 53 random bits, in (0,1). */
C2D_RHD double c2d_draw_s(uint64_t key, uint32_t sub, uint32_t n) {
  const uint64_t x = c2d_stream64(key, sub, n);
  return c2d_u01_bits((uint32_t)(x >> 32), (uint32_t)x);
}

C2D_RHD double c2d_draw(uint64_t key, uint32_t n) { return c2d_draw_s(key, 0u, n); }

/* Absorption-point stream of a probe bundle: output n as two 32-bit uniforms
 * (c2d_u01_32 of the high and the low half). */
C2D_RHD uint64_t c2d_abspt(uint64_t key, uint32_t sub, uint32_t n) {
  return c2d_stream64(key, sub, n);
}

/* Lineage key of a census packet for the next step (replaces the per-packet
 * fibran reseed, imctrk2d.f:571): a SplitMix64 hash of the packet's key and
 * its stream position (sub, ctr), one per census write. */
C2D_RHD uint64_t c2d_census_key(uint64_t key, uint32_t ctr, uint32_t sub) {
  const uint64_t pos = ((uint64_t)sub << 32) | (uint64_t)ctr;
  return c2d_mix64(key ^ c2d_mix64(pos + 0x9E3779B97F4A7C15ull * (uint64_t)C2D_TAG_CENSUS));
}

C2D_RHD uint64_t c2d_derive_s(uint64_t key, uint32_t tag, uint32_t a, uint32_t b, uint32_t sub) {
  uint32_t c[4] = {a, b, tag | (sub << 8), C2D_DERIVE_C3};
  c2d_philox(c, (uint32_t)key, (uint32_t)(key >> 32));
  return ((uint64_t)c[1] << 32) | (uint64_t)c[0];
}

C2D_RHD uint64_t c2d_derive(uint64_t key, uint32_t tag, uint32_t a, uint32_t b) {
  return c2d_derive_s(key, tag, a, b, 0u);
}

C2D_RHD uint64_t c2d_step_key(uint64_t seed, int32_t ncycle) {
  return c2d_derive(seed, C2D_TAG_STEP, (uint32_t)ncycle, 0u);
}

#endif /* C2D_RNG_H */
