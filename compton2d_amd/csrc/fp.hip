/*
 * fp.hip — Fokker-Planck electron update on gfx950.
 *
 * c2d_fp_kernel: the reference's FP_calc (src/update2d.f:337-1739) for one
 * zone per 64-lane wavefront (one workgroup = one wave).  The zone's
 * 200-bin state (f_old, f_new, Chang-Cooper coefficients, rates) and its
 * 400-bin photon field live in LDS for all implicit sub-steps (thousands
 * per MC step in optically thin zones).  Work is split by what parity
 * allows:
 *   - element-wise stages (rates dg_sy with its exp, the Chang-Cooper
 *     smw/bigW/bigC coefficients with their 3 exps per bin, injection
 *     profiles, the n_field x F_IC contraction, power-law fit terms) run
 *     one energy bin per lane;
 *   - reductions and recurrences whose order fixes the result bit for bit
 *     (the reference's sequential sums, the Thomas solve tridag
 *     :2476-2518, the temperature search :1440-1468) are evaluated by every
 *     lane in the reference order from LDS (broadcast reads), so no
 *     cross-lane exchange is needed;
 *   - McDonald's series (src/volume2d.f:598-626), thousands of terms per
 *     call inside the temperature search, evaluates K2 and K3 together, 64
 *     terms per pass: the argument-independent parts of each term come from
 *     a table (see mcdonald23_w), exp(z*ts) is lane-parallel, and the terms
 *     are accumulated in order through readlane up to the reference's
 *     stopping term.
 * Arithmetic is c2d_math.h with -ffp-contract=off, so results equal the
 * det-math build of the oracle (oracle/c2d_fp_oracle.c) bit for bit.
 * Branches of FP_calc that never reach an output (Coulomb/Moeller rates
 * and their rate-file cache, dg_br, loop 300's dg_A/disp_A) are not
 * computed; see the oracle's header for the argument.
 *
 * c2d_tridag_kernel: the batched Thomas solve alone (one zone per lane),
 * exported as c2d_fp_tridag for unit parity against tridag.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_wave.hpp"

namespace c2d {

constexpr int TRI_BLOCK = 64;
constexpr int TRI_MAXN = 256;

__global__ void __launch_bounds__(TRI_BLOCK) c2d_tridag_kernel(const double* __restrict__ a,
                                                               const double* __restrict__ b,
                                                               const double* __restrict__ c,
                                                               const double* __restrict__ r,
                                                               double* __restrict__ x, int ncell,
                                                               int nt) {
  const int cell = blockIdx.x * TRI_BLOCK + threadIdx.x;
  if (cell >= ncell) return;
  const size_t o = (size_t)cell * nt;
  double gam[TRI_MAXN];
  double f[TRI_MAXN];
  const double b1 = b[o];
  if (fabs(b1) <= 1.0e-100) {   /* 'Error: b(1) = 0.' -> return, x unchanged */
    return;
  }
  double bet = b1;
  f[0] = r[o] / bet;
  for (int i = 1; i < nt; i++) {
    gam[i] = c[o + i - 1] / bet;
    bet = b[o + i] - a[o + i] * gam[i];
    if (fabs(bet) <= 1.0e-100) {
      for (int n = 0; n < nt; n++) x[o + n] = 0.0;
      return;
    }
    f[i] = (r[o + i] - a[o + i] * f[i - 1]) / bet;
  }
  for (int i = nt - 2; i >= 0; i--) {
    f[i] = f[i] - gam[i + 1] * f[i + 1];
    if (f[i + 1] < 0.0) f[i + 1] = 0.0;
  }
  for (int i = 0; i < nt; i++) x[o + i] = f[i];
}

namespace {

using namespace wave;
constexpr int NT = C2D_NUM_NT;
constexpr int NPH = C2D_NPHFIELD;
constexpr double PI_REF = 3.1415926536;       /* general.pa:24 */
constexpr double C_LIGHT = 2.9979245620e10;   /* general.pa:25 */
constexpr double LNL = 20.0;                  /* update2d.f:143 */
constexpr int MAX_FP_STEPS = 1000000;         /* update2d.f:585-599 */

/* ---- McDonald K2/K3 across the zone's workgroup ------------------------
 * The zone's FP_calc runs on wave 0.  Its temperature search spends most of
 * the kernel in McDonald's series (thousands of terms per gamma_bar at the
 * Theta of a heated zone), whose terms are independent and whose stopping
 * term depends on the term alone, while the sums must be added in order.
 * Waves 1..MCD_PROD compute the terms, 2*64 per wave per pass, into a
 * double-buffered LDS block (with their stop ballots); wave 0 adds them in
 * order while the next pass is computed.  One s_barrier per pass; every wave
 * derives "both series stopped" from the same ballots, so all leave the loop
 * after the same barrier.  Sums, stopping terms and results are those of the
 * single-wave mcdonald23_w bit for bit (same terms, same order). */
/* The launch picks the waves per zone (blockDim.x / 64, 1..FP_WAVES_MAX;
 * c2d_launch_fp): more where few zones leave SIMDs idle, one (the
 * single-wave series, c2d_wave.hpp) where the zones alone fill the chip. */
constexpr int FP_WAVES_MAX = 8;
/* The kernel is instantiated for WMAX = 1 (one wave per zone, launch bounds
 * 64: the codegen of a single-wave solve, measured 2.3x faster than the same
 * code compiled for 512-thread workgroups) and WMAX = FP_WAVES_MAX. */
constexpr int MCD_PROD_MAX = FP_WAVES_MAX - 1;
constexpr int MCD_BLK = 2 * FPB;                       /* terms per producer per pass */
constexpr int MCD_PASS_MAX = MCD_PROD_MAX * MCD_BLK;
constexpr int MCD_BATCH = 16;                          /* divides MCD_BLK */
enum { MCD_CMD_EXIT = 0, MCD_CMD_SERIES = 1, MCD_CMD_BATCH = 2 };

/* Temperature-search candidates evaluated together (one per lane of every
 * wave of the zone): the search of update2d.f:1440-1468 walks the chain
 * Theta*1.005^k (or /1.005^k) and stops at the first gamma_bar crossing
 * gbar; when it walks far (a zone heating by orders of magnitude within an
 * MC step: C3 takes ~800 steps per zone), evaluating the next NB chain
 * members at once replaces NB sequential McDonald pairs by one pass in
 * which each lane sums ITS candidate's series in order.  gamma_bar is a pure
 * function of Theta and the chain is formed by the same repeated
 * multiplication, so every value used equals the sequential one bit for bit;
 * members past the crossing are simply not used (or reused by the next
 * sub-step's search, which continues the same chain). */
constexpr int NB_MAX = FP_WAVES_MAX * FPB;
#ifndef C2D_FP_NSINGLE
#define C2D_FP_NSINGLE 3
#endif
constexpr int FP_NSINGLE = C2D_FP_NSINGLE;   /* search steps before batching */
#ifndef C2D_FP_PREFETCH
#define C2D_FP_PREFETCH 1
#endif

/* the producer waves' LDS (only multi-wave kernels reference it) */
struct McdCoop {
  alignas(16) double term[2][MCD_PASS_MAX][2];         /* [buffer][n][K2 term, K3 term] */
  unsigned long long mask[2][MCD_PROD_MAX][4];         /* stop2 a/b, stop3 a/b ballots  */
  double z;                                            /* SERIES: argument; BATCH: start */
  int cmd, dir;                                        /* BATCH: +1 (x1.005) / -1 (/1.005) */
};
/* a batch's chain members and their gamma_bar, sized per kernel instance so
 * the single-wave kernel keeps its LDS small (occupancy: 1024 zones must fit) */
template <int N>
struct McdBatch {
  double bc[N], bg[N];
};

/* exp(gammln(2.5)), exp(gammln(3.5)) of McDonald's normalisation, computed
 * once per launch (c2d_fp_kernel) instead of per series */
__shared__ double s_eg[2];

/* gamma_bar (volume2d.f:572-594) of this lane's Theta, McDonald's series
 * summed sequentially by the lane (volume2d.f:598-626): n is wave-uniform, so
 * the abscissa table reads are scalar loads; two terms per iteration give the
 * exp/divide chains some overlap; each series stops at its own term. */
__device__ double gamma_bar_lane(double Theta, const double* __restrict__ tab, long long& guard) {
  double g;
  if (Theta < F32(0.2)) {
    g = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) +
         F32(3.384) * (Theta * Theta * Theta)) /
            (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
        Theta;
  } else {
    const double z = 1.0 / Theta;
    const double dt = 1.001, d = dt - 1.0, s = 5.0e-1 * (1.0 + dt);
    double sum2 = 0.0, sum3 = 0.0, t = 1.0;
    bool run2 = true, run3 = true;
    int n = 0;
#if C2D_FP_PREFETCH
    /* the next iteration's abscissa rows are loaded before this one's terms */
    double4 ra = *(const double4*)tab, rb = *(const double4*)(tab + 4);
#endif
    for (; n + 2 <= C2D_FP_MCD_N; n += 2) {
      if (!__ballot(run2 || run3)) break;
#if C2D_FP_PREFETCH
      const double ta = ra.x, tsa = ra.y, p2a = ra.z, p3a = ra.w;
      const double tb = rb.x, tsb = rb.y, p2b = rb.z, p3b = rb.w;
      if (n + 4 <= C2D_FP_MCD_N) {
        ra = *(const double4*)(tab + (size_t)(n + 2) * 4);
        rb = *(const double4*)(tab + (size_t)(n + 3) * 4);
      }
#else
      const double* e = tab + (size_t)n * 4;
      const double ta = e[0], tsa = e[1], p2a = e[2], p3a = e[3];
      const double tb = e[4], tsb = e[5], p2b = e[6], p3b = e[7];
#endif
      const double ya = z * tsa, yb = z * tsb;
      double sd2a = 0.0, sd3a = 0.0, sd2b = 0.0, sd3b = 0.0;
      if (ya < 2.25e2) {
        const double ey = c2d_exp_bf(ya);
        sd2a = p2a / ey;
        sd3a = p3a / ey;
      }
      if (yb < 2.25e2) {
        const double ey = c2d_exp_bf(yb);
        sd2b = p2b / ey;
        sd3b = p3b / ey;
      }
      const double tna = ta * dt, tnb = tb * dt;
      if (run2) {
        sum2 = sum2 + d * ta * sd2a;
        if (!(tna < 2.0 || sd2a > 1.0e-8)) run2 = false;
        else {
          sum2 = sum2 + d * tb * sd2b;
          if (!(tnb < 2.0 || sd2b > 1.0e-8)) run2 = false;
        }
      }
      if (run3) {
        sum3 = sum3 + d * ta * sd3a;
        if (!(tna < 2.0 || sd3a > 1.0e-8)) run3 = false;
        else {
          sum3 = sum3 + d * tb * sd3b;
          if (!(tnb < 2.0 || sd3b > 1.0e-8)) run3 = false;
        }
      }
      t = tnb;
    }
    guard += n;
    /* beyond the table: the abscissae by the reference's own chain */
    while (run2 || run3) {
      const double ts = t * s;
      const double p2 = c2d_pow(ts * ts - 1.0, 1.5), p3 = c2d_pow(ts * ts - 1.0, 2.5);
      const double y = z * ts;
      double sd2 = 0.0, sd3 = 0.0;
      if (y < 2.25e2) {
        const double ey = c2d_exp_bf(y);
        sd2 = p2 / ey;
        sd3 = p3 / ey;
      }
      const double tn = t * dt;
      if (run2) {
        sum2 = sum2 + d * t * sd2;
        if (!(tn < 2.0 || sd2 > 1.0e-8)) run2 = false;
      }
      if (run3) {
        sum3 = sum3 + d * t * sd3;
        if (!(tn < 2.0 || sd3 > 1.0e-8)) run3 = false;
      }
      t = tn;
      if (++guard > GUARD_MAX) break;
    }
    double K2, K3;
    mcdonald23_finish_c(z, sum2, sum3, s_eg[0], s_eg[1], K2, K3);
    g = K3 / K2 - Theta;
  }
  if (g < 1.0) g = 1.0;
  return g;
}

/* gamma_bar memo shared by every zone of the launch and by later steps
 * (FpParams.gb_*, allocated with the McDonald table).  gamma_bar is a pure
 * function of Theta, and the temperature searches of zones that start from
 * the same Theta (C3: every zone from the 1000 keV tea clamp, update2d.f:
 * 266-276) walk the same chain Theta*1.005^k bit for bit, so one zone's
 * McDonald pairs serve all of them, step after step.  Open addressing on the
 * bits of Theta; a slot's key is claimed once by CAS (0 -> key) and its
 * value written once, by the claimer, so a reader that finds the key and a
 * non-zero value (gamma_bar >= 1) has the exact value; anything else (stale
 * line, value not yet written, table full) is a miss and the caller computes
 * -- results are bit-identical either way. */
constexpr int GB_PROBES = 8;
struct GbMemo {
  unsigned long long* key;
  double* val;
  uint32_t mask;
};
__device__ __forceinline__ uint32_t gb_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k;
}
__device__ __forceinline__ bool gb_lookup(const GbMemo& M, double th, double& g) {
  if (!M.key) return false;
  const unsigned long long k = c2d_bits(th);
  uint32_t h = gb_hash(k) & M.mask;
  for (int i = 0; i < GB_PROBES; i++) {
    const unsigned long long kk = __hip_atomic_load(M.key + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kk == k) {
      const double v = __hip_atomic_load(M.val + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v != 0.0) { g = v; return true; }
      return false;
    }
    if (kk == 0ull) return false;
    h = (h + 1u) & M.mask;
  }
  return false;
}
__device__ __forceinline__ void gb_insert(const GbMemo& M, double th, double g) {
  if (!M.key) return;
  const unsigned long long k = c2d_bits(th);
  uint32_t h = gb_hash(k) & M.mask;
  for (int i = 0; i < GB_PROBES; i++) {
    const unsigned long long prev = atomicCAS(M.key + h, 0ull, k);
    if (prev == 0ull) {
      __hip_atomic_store(M.val + h, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (prev == k) return;
    h = (h + 1u) & M.mask;
  }
}

/* chain member idx+1 from th0 (the search's own repeated x or / 1.005),
 * then its gamma_bar, into the batch arrays */
template <int N>
__device__ __forceinline__ void batch_member(McdBatch<N>& C, double th0, int dir, int idx,
                                             const double* __restrict__ tab, long long& guard,
                                             const GbMemo& M) {
  double c = th0;
  for (int i = 0; i <= idx; i++) c = (dir > 0) ? c * F32(1.005) : c / F32(1.005);
  double g;
  if (!gb_lookup(M, c, g)) {
    g = gamma_bar_lane(c, tab, guard);
    gb_insert(M, c, g);
  }
  C.bc[idx] = c;
  C.bg[idx] = g;
}

/* waves of this zone's workgroup (uniform) */
template <int WMAX>
__device__ __forceinline__ int fp_nwaves() {
  return WMAX == 1 ? 1 : (int)(blockDim.x / FPB);
}

/* run flags after pass p's ballots (identical on every wave) */
__device__ __forceinline__ void mcd_pass_runs(const McdCoop& C, int p, int nprod, bool& run2,
                                              bool& run3) {
  const unsigned long long(*m)[4] = C.mask[p & 1];
  for (int w = 0; w < nprod; w++) {
    if (m[w][0] | m[w][1]) run2 = false;
    if (m[w][2] | m[w][3]) run3 = false;
  }
}

/* producer waves: serve series requests until wave 0 posts MCD_CMD_EXIT */
__device__ __forceinline__ void mcd_producer(McdCoop& C, McdBatch<NB_MAX>& B,
                                             const double* __restrict__ tab, int wave, int lane,
                                             const GbMemo& M) {
  for (;;) {
    __syncthreads();                                   /* request posted by wave 0 */
    if (C.cmd == MCD_CMD_EXIT) return;
    if (C.cmd == MCD_CMD_BATCH) {
      long long g = 0;
      batch_member(B, C.z, C.dir, wave * FPB + lane, tab, g, M);
      __syncthreads();                                 /* batch complete */
      continue;
    }
    const double z = C.z;
    const int nprod = fp_nwaves<FP_WAVES_MAX>() - 1, pass = nprod * MCD_BLK;
    const int npass = C2D_FP_MCD_N / pass;
    bool run2 = true, run3 = true;
    for (int p = 0; p < npass; p++) {
      const int n0 = p * pass + (wave - 1) * MCD_BLK;
      const McdTerm a = mcd_term_tab(z, n0 + lane, tab);
      const McdTerm b = mcd_term_tab(z, n0 + FPB + lane, tab);
      double(*t)[2] = C.term[p & 1] + (wave - 1) * MCD_BLK;
      t[lane][0] = a.term2;
      t[lane][1] = a.term3;
      t[FPB + lane][0] = b.term2;
      t[FPB + lane][1] = b.term3;
      const unsigned long long s2a = __ballot(a.stop2), s2b = __ballot(b.stop2);
      const unsigned long long s3a = __ballot(a.stop3), s3b = __ballot(b.stop3);
      if (lane == 0) {
        unsigned long long* m = C.mask[p & 1][wave - 1];
        m[0] = s2a; m[1] = s2b; m[2] = s3a; m[3] = s3b;
      }
      __syncthreads();                                 /* pass p complete */
      mcd_pass_runs(C, p, nprod, run2, run3);
      if (!run2 && !run3) break;
    }
  }
}

/* wave 0: K2, K3 of McDonald(2, z), McDonald(3, z) with the producers */
template <int WMAX>
__device__ __forceinline__ void mcdonald23_coop(McdCoop& C, double z, int lane, const double* __restrict__ tab,
                                double& K2, double& K3, long long& guard, double* scr) {
  if (lane == 0) {
    C.z = z;
    C.cmd = MCD_CMD_SERIES;
  }
  __syncthreads();                                     /* post the request */
  const int nprod = fp_nwaves<WMAX>() - 1, pass = nprod * MCD_BLK, npass = C2D_FP_MCD_N / pass;
  double sum2 = 0.0, sum3 = 0.0;
  bool run2 = true, run3 = true;
  int p = 0;
  for (; p < npass; p++) {
    __syncthreads();                                   /* pass p complete */
    const double(*t)[2] = C.term[p & 1];
    const unsigned long long(*m)[4] = C.mask[p & 1];
    bool clean = run2 && run3;
    for (int w = 0; w < nprod; w++) clean = clean && !(m[w][0] | m[w][1] | m[w][2] | m[w][3]);
    if (clean) {
      /* operands of MCD_BATCH terms are loaded before their adds, so the
       * chain waits for the adds alone, not one LDS latency per term */
      for (int q0 = 0; q0 < pass; q0 += MCD_BATCH) {
        double2 v[MCD_BATCH];
#pragma unroll
        for (int i = 0; i < MCD_BATCH; i++) v[i] = *(const double2*)t[q0 + i];
#pragma unroll
        for (int i = 0; i < MCD_BATCH; i++) {
          sum2 = sum2 + v[i].x;
          sum3 = sum3 + v[i].y;
        }
      }
      guard += pass;
    } else {
      for (int h = 0; h < 2 * nprod; h++) {            /* 64-term blocks in n order */
        const int w = h >> 1, half = h & 1;
        const unsigned long long m2 = m[w][half], m3 = m[w][2 + half];
        const int n2 = mcd_take(run2, m2), n3 = mcd_take(run3, m3);
        const double(*tb)[2] = t + h * FPB;
        for (int q = 0; q < n2; q++) sum2 = sum2 + tb[q][0];
        for (int q = 0; q < n3; q++) sum3 = sum3 + tb[q][1];
        if (m2) run2 = false;
        if (m3) run3 = false;
        guard += n2 > n3 ? n2 : n3;
      }
    }
    if (!run2 && !run3) break;
  }
  if (run2 || run3) {                                  /* beyond the coop passes: alone */
    const int n0 = npass * pass;
    mcdonald23_from(z, lane, tab, n0, tab[(size_t)n0 * 4], sum2, sum3, run2, run3, guard, scr);
  }
  mcdonald23_finish_c(z, sum2, sum3, s_eg[0], s_eg[1], K2, K3);
}

/* wave 0: evaluate chain members 1..NB from th0 on every wave of the zone */
template <int WMAX, int N>
__device__ __forceinline__ void search_batch(McdCoop& C, McdBatch<N>& B, double th0, int dir, int lane,
                                             const double* __restrict__ tab, long long& guard,
                                             const GbMemo& M) {
  if (fp_nwaves<WMAX>() > 1) {
    if (lane == 0) {
      C.z = th0;
      C.dir = dir;
      C.cmd = MCD_CMD_BATCH;
    }
    __syncthreads();                                   /* post the request */
  }
  batch_member(B, th0, dir, lane, tab, guard, M);
  __syncthreads();                                     /* batch complete */
}

/* gamma_bar (volume2d.f:572-594) with the cooperative series */
template <int WMAX>
__device__ __forceinline__ double gamma_bar_coop(McdCoop& C, double Theta, int lane, const double* tab,
                                 long long& guard, double* scr) {
  double g;
  if (Theta < F32(0.2)) {
    g = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) +
         F32(3.384) * (Theta * Theta * Theta)) /
            (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
        Theta;
  } else {
    double K2, K3;
    if (fp_nwaves<WMAX>() > 1)
      mcdonald23_coop<WMAX>(C, 1.0 / Theta, lane, tab, K2, K3, guard, scr);
    else {
      const double z = 1.0 / Theta;
      double sum2 = 0.0, sum3 = 0.0;
      mcdonald23_from(z, lane, tab, 0, 1.0, sum2, sum3, true, true, guard, scr);
      mcdonald23_finish_c(z, sum2, sum3, s_eg[0], s_eg[1], K2, K3);
    }
    g = K3 / K2 - Theta;
  }
  if (g < 1.0) g = 1.0;
  return g;
}

}  // namespace

/* hand-offs of wave 0's 200-bin arrays (only wave 0 touches them) */
template <int WMAX>
__device__ __forceinline__ void fp_sync() {
  if (WMAX == 1)
    __syncthreads();
  else
    wave_sync();
}

/* The zone's LDS, at namespace scope so that every access is a ds_* op with
 * a known address space (pointers to it passed into a function compile to
 * flat accesses: 2.5x slower on this kernel). */
__shared__ double s_gnt[NT + 2], s_gam[NT + 2], s_fold[NT + 2], s_fnew[NT + 2];
__shared__ double s_dgic[NT + 2], s_dgdt[NT + 2], s_disp[NT + 2];
__shared__ double s_a[NT + 2], s_b[NT + 2], s_c[NT + 2];
__shared__ double s_mcd[4 * FPB];   /* McDonald term exchange (c2d_wave.hpp) */
__shared__ double s_smw[NT + 2], s_bigW[NT + 2], s_bigC[NT + 2], s_em[NT + 2], s_inj[NT + 2];
__shared__ double s_Pnt[NT + 2], s_nf[NPH];
__shared__ double s_seq[2 * FPB];  /* in-order sums: wave 0's staged values (seq_sum_lds) */
__shared__ McdCoop s_coop;
__shared__ McdBatch<FPB> s_batch1;
__shared__ McdBatch<NB_MAX> s_batch8;
template <int WMAX>
__device__ __forceinline__ auto& batch_lds() {
  if constexpr (WMAX == 1)
    return s_batch1;
  else
    return s_batch8;
}

/* FP_calc of one zone on one wave (the kernel's wave 0).  Only this wave
 * touches the 200-bin arrays, so their hand-offs are wave barriers; the
 * workgroup barriers belong to the McDonald cooperation alone. */
template <int WMAX>
__device__ __forceinline__ void fp_zone_body(const FpParams& P, const int lane) {
  const int cell = blockIdx.x;
  const int j = cell / P.nr + 1, k = cell % P.nr + 1;
  const Geo* G = P.geo;
  const double* zin = P.zin + (size_t)cell * FZ_N;
  double* zo = P.zout + (size_t)cell * FO_N;
  long long guard = 0;

  const double volume = zin[FZ_VOL], tea = zin[FZ_TEA], tna = zin[FZ_TNA];
  const double B = zin[FZ_B], Eloss_sy = zin[FZ_ELSY], f_pair = zin[FZ_FPAIR];
  const double ecens = P.ecens ? P.ecens[cell] : zin[FZ_ECENS];
  const double zmax = G->z[P.nz], rmax = G->r[P.nr];

  const double t_esc = P.r_esc * zmax / C_LIGHT;   /* :460-461 */
  const double t_acc = P.r_acc * zmax / C_LIGHT;
  double Te_new = tea;
  double n_p = zin[FZ_NE];
  double ne = n_p * (1. + f_pair);
  double n_positron = n_p * f_pair;
  double n_lept = ne + n_positron;
  if (n_lept < 1.0e-11) {                           /* :478 */
    if (lane == 0) {
      zo[FO_TE] = Te_new;
      for (int q = 0; q < C2D_FP_NDIAG; q++) zo[FO_DIAG + q] = 0.0;
      zo[FO_DIAG + C2D_FP_SKIPPED] = 1.0;
    }
    return;
  }
  for (int i = lane; i < NT; i += FPB) {
    s_gnt[i + 1] = P.gnt[i];
    s_gam[i + 1] = P.gnt[i] + 1.0;
    s_fold[i + 1] = P.f_in[(size_t)cell * NT + i];
    s_Pnt[i + 1] = P.P_in[(size_t)cell * NT + i];
  }
  for (int i = lane; i < NPH; i += FPB) s_nf[i] = P.nf[(size_t)cell * NPH + i];
  fp_sync<WMAX>();

  /* E_el, normalisation (:482-509) */
  double E_el = 0.0, E_pos = 0.0;
  E_el = seq_sum_lds(E_el, 2, NT, lane, s_seq,
                 [&](int i) { return (s_gnt[i] - s_gnt[i - 1]) * s_gam[i] * s_fold[i]; });
  E_el = E_el * ne * 8.176e-7 * volume;
  double e_old = 0.0 + E_el + E_pos + zin[FZ_ECOLD];
  double e_new = 0.0 + ecens;
  double sum_p = seq_sum_lds(0., 1, NT - 1, lane, s_seq,
                         [&](int i) { return (s_gnt[i + 1] - s_gnt[i]) * s_fold[i]; });
  fp_sync<WMAX>();
  for (int i = lane + 1; i <= NT; i += FPB) s_fold[i] = s_fold[i] / sum_p;
  fp_sync<WMAX>();
  if (lane == 0) s_fold[NT] = 0.0;

  /* flare (:532-562) */
  const double rmid = 5.0e-1 * (G->r[k] + G->r[k - 1]);   /* r[0] = rmin */
  const double zmid = 5.0e-1 * (G->z[j] + G->z[j - 1]);   /* z[0] = zmin */
  double tl_flare = 0.0;
  if (P.cf_sentinel == 1) {
    const double ar = (rmid - P.r_flare) / P.sigma_r;
    const double az = (zmid - P.z_flare) / P.sigma_z;
    const double at = (P.time - P.t_flare) / P.sigma_t;
    const double y = 5.0e-1 * (ar * ar + az * az + at * at);
    tl_flare = (y < 1.0e2) ? P.flare_amp / c2d_exp_bf(y) : 0.0;
  }
  const double tlev = zin[FZ_TURB] + tl_flare;
  const double Tp_flare = tna * (1.0 + tl_flare);
  const double Th_p = Tp_flare / 9.382e5;
  double Th_e = tea / 5.11e2;
  const double f_th = 1.5 * volume * n_lept;
  /* dg_ic(i) = -sum_ph n_field(ph) F_IC(i,ph) / volume (:568-574), bin per lane */
  for (int i = lane + 1; i <= NT - 1; i += FPB) {
    double s = 0.0;
    const double* ft = P.FT + (i - 1);
    for (int ph = 0; ph < NPH; ph++) s = s - s_nf[ph] * ft[(size_t)ph * NT] / volume;
    s_dgic[i] = s;
  }
  if (lane == 0) s_dgic[NT] = 0.0;   /* hazard H10 */
  const double dz = G->z[j] - G->z[j - 1];          /* :628-632 */
  fp_sync<WMAX>();

  double hr = 0.0, hr_st = 0.0, sum_E = 0.0, t_fp = 0.0;
  int fp_steps = 0;
  /* gamma_bar is a pure function and label 200 evaluates it at the Th_e the
   * previous sub-step's temperature search ended on, whose value that search
   * computed last: reuse it (one McDonald pair per sub-step saved, exact) */
  double g_av_next = 0.0, hr_th_c_next = 0.0;
  /* The temperature search steps Theta by x1.005 or /1.005 from the last
   * sub-step's value, so successive sub-steps keep re-evaluating the same few
   * arguments (T oscillating across the crossing). gamma_bar is a pure
   * function of Theta: a 4-entry memo keyed on the exact bits returns the
   * value it would recompute (bit-identical), skipping its McDonald pair. */
  const GbMemo memo{P.gb_key, P.gb_val, P.gb_mask};
  double memo_th[4] = {-1.0, -1.0, -1.0, -1.0}, memo_g[4] = {0.0, 0.0, 0.0, 0.0};
  int memo_next = 0;
  auto gamma_bar_m = [&](double th) -> double {
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (memo_th[q] == th) return memo_g[q];
    double g;
    double gm = 0.0;
    const bool hit = gb_lookup(memo, th, gm);
    if (__builtin_amdgcn_readfirstlane((int)hit)) {
      g = c2d_from_bits(((unsigned long long)__builtin_amdgcn_readfirstlane((int)(c2d_bits(gm) >> 32)) << 32) |
                        (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c2d_bits(gm)));
    } else {
      g = gamma_bar_coop<WMAX>(s_coop, th, lane, P.mcd, guard, s_mcd);
      if (lane == 0) gb_insert(memo, th, g);
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (q == memo_next) { memo_th[q] = th; memo_g[q] = g; }
    memo_next = (memo_next + 1) & 3;
    return g;
  };
  /* gamma_bar of the search's next chain member: from the last batch while
   * the walk follows its chain, by a new batch once this search has taken
   * FP_NSINGLE steps (it is walking far), else singly (memo / cooperative
   * series).  bdir = 0: no usable batch. */
  int bdir = 0, bpos = 0, bn = 0;
  auto search_eval = [&](double prev, double next, int dir, int k) -> double {
    auto& B = batch_lds<WMAX>();
    if (bdir == dir && bpos < bn && B.bc[bpos] == next) return B.bg[bpos++];
    if (k >= FP_NSINGLE && next >= F32(0.2)) {
      search_batch<WMAX>(s_coop, B, prev, dir, lane, P.mcd, guard, memo);
      bdir = dir;
      bpos = 1;
      bn = fp_nwaves<WMAX>() * FPB;
      return B.bg[0];
    }
    bdir = 0;
    return gamma_bar_m(next);
  };
#ifdef C2D_FP_PROF
  long long pf_gb = 0, pf_tri = 0, pf_loop0 = clock64(), pf_t0, pf_calls = 0;
#define PF_BEGIN() pf_t0 = clock64()
#define PF_END(acc) acc += clock64() - pf_t0
#else
#define PF_BEGIN()
#define PF_END(acc)
#endif
  for (;;) {
    /* label 200 (:577) */
    double g_av = (fp_steps == 0) ? gamma_bar_m(Th_e) : g_av_next;
    /* hr_th_c = hr_th_c - x_i, i.e. + (-x_i) bit for bit */
    /* after the first sub-step this sum was formed beside the previous
     * sub-step's gbar (same f_old, n_lept and order: the same value) */
    const double hr_th_c = (fp_steps == 0)
        ? seq_sum_lds(0.0, 1, NT - 1, lane, s_seq, [&](int i) {
            return -(8.176e-7 * s_dgic[i] * s_fold[i] * (s_gnt[i + 1] - s_gnt[i]) * volume * n_lept);
          })
        : hr_th_c_next;
    if (fp_steps > MAX_FP_STEPS) {
      if (lane == 0) atomicOr(P.err, FPERR_STEPS);
      return;
    }
    const double gamma_R = 2.1e-3 * __builtin_sqrt(n_lept) / (B * __builtin_sqrt(g_av));
    const double sT = Th_e + Th_p;
    const double h_T = F32(.79788) * (2. * (sT * sT) + 2.0 * sT + 1.0) /
                       (c2d_pow(sT, 1.5) * (1.0 + 1.875 * Th_e + .8203 * (Th_e * Th_e)));
    const double hr_th_Coul = f_th * 1.7386e-26 * n_p * LNL * h_T * (Tp_flare - Te_new);
    const double yR = gamma_R / g_av;
    const double hr_th_sy = (yR < 100.0) ? -Eloss_sy / (P.dt * c2d_exp_bf(yR)) : 0.0;
    double hr_th_A = tlev * hr_th_Coul;
    if (hr_th_A < 1.0e-20) hr_th_A = 1.0e-20;
    const double hr_th_total = hr_th_sy + hr_th_c + hr_th_A;
    const double dT_total = 6.25e8 * P.dt * hr_th_total / f_th;
    double f_t_implicit = P.df_implicit * Te_new / fabs(dT_total);
    if (f_t_implicit > P.df_T) f_t_implicit = P.df_T;
    const double f_sy = 1.058e-15 * (B * B) / 8.176e-7;
    const double g_thr = 1.0 + 4.0 * Th_e;
    /* dgdt, disp (:880-889, :1035-1049): bin per lane */
    for (int i = lane + 1; i <= NT; i += FPB) {
      const double gi = s_gam[i];
      const double y = gamma_R / gi;
      const double dg_sy = (y < 100.0) ? -(f_sy * (gi * gi - 1.0) / c2d_exp_bf(y)) : -1.0e-50;
      const double dg_A = gi / t_acc;
      s_disp[i] = gi * gi / t_acc / 2.0;
      s_dgdt[i] = dg_sy + s_dgic[i] + dg_A;
    }
    double hr_nt_A = 0.0, hr_st_A = 0.0;
    for (int c0 = 1; c0 <= NT - 1; c0 += FPB) {        /* loop 350 sums, in order */
      const int i = c0 + lane;
      double v = 0.0;
      bool st = false;
      if (i <= NT - 1) {
        const double gi = s_gam[i];
        v = gi / t_acc * s_fold[i] * (s_gam[i + 1] - gi);
        st = gi > g_thr;
      }
      const unsigned long long stm = __ballot(st);
      s_seq[lane] = v;
      wave_sync();
      const int mn = (NT - c0) < FPB ? (NT - c0) : FPB;
#pragma unroll 8
      for (int m = 0; m < mn; m++) {
        const double x = s_seq[m];
        hr_nt_A = hr_nt_A + x;
        if ((stm >> m) & 1ull) hr_st_A = hr_st_A + x;
      }
      wave_sync();
    }
    hr_st_A = hr_st_A * 8.176e-7 * n_lept * volume;
    hr_nt_A = hr_nt_A * 8.176e-7 * n_lept * volume;
    const double heat_total = hr_th_Coul + hr_nt_A;
    e_old = e_old + heat_total * f_t_implicit * P.dt;
    if (fp_steps == 0) {
      hr = hr + heat_total;
      hr_st = hr_st + hr_st_A;
    }
    double d_t = f_t_implicit * P.dt;                  /* :1142-1146 */
    if (d_t > (P.dt - t_fp)) d_t = 1.00001 * (P.dt - t_fp);
    if (P.pair_sw == 1) {
      /* pairs on with no positrons (H6: n_pos = dn_pp = 0, f_pair = 0): the
       * pa_calc rates vanish, so loop 460 (:1187-1217) adds 0/ne and clips
       * f_old below 1e-50; trid_p solves for npos = 0 (:1400), unused here */
      fp_sync<WMAX>();
      for (int i = lane + 1; i <= NT - 1; i += FPB) {
        double v = s_fold[i] + 0.0 / ne;
        if (v < 1.0e-50) v = 0.0;
        s_fold[i] = v;
      }
      fp_sync<WMAX>();
    }
    n_positron = 0.0;                                  /* :1164-1167 / :1218 */
    ne = n_p + n_positron;
    /* injection (:1226-1306) */
    double n_inject = 0.0;
    bool inj_any = false;
    double inj_rho = 0.0, inj_sum = 0.0;
    if (P.pick_sw == 1) {
      for (int i = lane + 1; i <= NT - 1; i += FPB) {
        const double x = s_gam[i] - P.inj_gg;
        s_inj[i] = 1.0e2 * c2d_exp_bf(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                   (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
      }
      fp_sync<WMAX>();
      inj_sum = seq_sum_lds(0.0, 1, NT - 1, lane, s_seq,
                        [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
      inj_rho = P.pick_rate * d_t;
      inj_any = true;
    }
    if (inj_any) {
      fp_sync<WMAX>();
      for (int i = lane + 1; i <= NT - 1; i += FPB) {
        const double v = inj_rho * s_inj[i] / inj_sum;
        s_inj[i] = v;
        s_fold[i] = s_fold[i] + v / ne;
      }
      fp_sync<WMAX>();
      n_inject = seq_sum_lds(n_inject, 1, NT - 1, lane, s_seq,
                         [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
    }
    if (P.inj_switch != 0) {
      const double tt = P.time + t_fp - P.inj_t;
      if (tt > dz / P.inj_v * (double)(j - 1) && tt < dz / P.inj_v * (double)j && k <= P.nr) {
        fp_sync<WMAX>();
        for (int i = lane + 1; i <= NT - 1; i += FPB) {
          const double gi = s_gam[i];
          double v;
          if (P.inj_dis == 1) {
            const double x = gi - P.inj_gg;
            v = 1.0e2 * c2d_exp_bf(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
          } else {
            const double inj_g2var =
                P.inj_g2 * c2d_pow(10.0, (P.time + t_fp - P.inj_t) * P.inj_v / zmax);
            if (gi > P.inj_g1) {
              const double inj_y = (P.g2var_switch == 1) ? gi / inj_g2var : gi / P.inj_g2;
              v = (inj_y < 1.0e2) ? 1.0e2 / (c2d_pow(gi, P.inj_p) * c2d_exp_bf(inj_y)) : 0.0;
            } else {
              v = 0.0;
            }
          }
          s_inj[i] = v;
        }
        fp_sync<WMAX>();
        double isum = 0.0, inj_E = 0.0;
        seq_sum2_lds(isum, inj_E, 1, NT - 1, lane, s_seq,
                 [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); },
                 [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]) * s_gam[i]; });
        inj_E = inj_E / isum;
        const double inj_rate = P.inj_L / 8.186e-7 / inj_E / (PI_REF * (rmax * rmax) * dz);
        const double rho = inj_rate * d_t;
        fp_sync<WMAX>();
        for (int i = lane + 1; i <= NT - 1; i += FPB) {
          const double v = rho * s_inj[i] / isum;
          s_inj[i] = v;
          s_fold[i] = s_fold[i] + v / ne;
        }
        fp_sync<WMAX>();
        n_inject = seq_sum_lds(n_inject, 1, NT - 1, lane, s_seq,
                           [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
      }
    }
    ne = ne + n_inject;
    n_p = n_p + n_inject;
    n_lept = n_lept + n_inject;
    ne = ne * t_esc / (t_esc + d_t);                  /* escape (:1309-1313) */
    n_p = n_p * t_esc / (t_esc + d_t);
    n_lept = n_lept * t_esc / (t_esc + d_t);
    fp_sync<WMAX>();
    /* Chang-Cooper coefficients (:1363-1390): smw, bigW, bigC and the
     * exp(-smw) factor for i = 1..NT-1, then a, b, c for i = 2..NT-1 */
    for (int i = lane + 1; i <= NT - 1; i += FPB) {
      double bigB, Dg;
      if (i == 1) {
        bigB = -(s_dgdt[1] + s_dgdt[2]);
        Dg = s_gnt[2] - s_gnt[1];
      } else {
        bigB = -(s_dgdt[i] + s_dgdt[i + 1]) / 2.0;
        Dg = s_gnt[i + 1] - s_gnt[i];
      }
      const double bigC = (s_disp[i] + s_disp[i + 1]) / 2.0;
      const double smw = Dg * bigB / bigC;
      s_smw[i] = smw;
      s_bigW[i] = smw / (c2d_exp_bf(smw) - 1.0);
      s_em[i] = bigC * smw / (1.0 - c2d_exp_bf(-smw));   /* bigC*smw/(1-exp(-smw)) */
      s_bigC[i] = bigC;
    }
    fp_sync<WMAX>();
    for (int i = lane + 2; i <= NT - 1; i += FPB) {
      const double D_gminus = s_gnt[i] - s_gnt[i - 1];
      const double D_gplus = s_gnt[i + 1] - s_gnt[i];
      const double Delta_g = __builtin_sqrt(s_gnt[i] / s_gnt[i - 1]) * D_gminus;
      s_c[i] = -d_t * (s_em[i] / Delta_g / D_gplus);
      s_b[i] = 1.0 + d_t / Delta_g * (s_bigC[i] * s_bigW[i] / D_gplus + s_em[i - 1] / D_gminus) +
               d_t / t_esc;
      s_a[i] = -d_t / Delta_g * s_bigC[i - 1] * s_bigW[i - 1] / D_gminus;
    }
    if (lane == 0) {
      s_a[1] = 0.0; s_b[1] = 1.0; s_c[1] = 0.0;
      s_a[NT] = 0.0; s_b[NT] = 1.0; s_c[NT] = 0.0;
    }
    fp_sync<WMAX>();
    PF_BEGIN();
    /* tridag (:2476-2518): the recurrences run in the reference order on
     * wave-uniform values read by every lane from LDS (broadcast loads that
     * issue ahead of the chain).  The bet/gam recurrence and the u
     * recurrence are independent but for bet_i, so their divisions overlap;
     * no branch per element: a vanishing bet is flagged and the solution
     * zeroed after the sweep, as the reference's early return leaves it.
     * Lane m keeps element c0 + m of each 64-bin chunk; gam is kept in s_smw. */
    {
      double bet = s_b[1];
      double u = s_fold[1] / bet;
      bool zero = false;
      if (lane == 0) s_fnew[1] = u;
      for (int c0 = 2; c0 <= NT; c0 += FPB) {
        double gmine = 0.0, umine = 0.0;
        const int mn = (NT - c0 + 1) < FPB ? (NT - c0 + 1) : FPB;
#pragma unroll 4
        for (int m = 0; m < mn; m++) {
          const int i = c0 + m;
          const double am = s_a[i], bm = s_b[i], cm = s_c[i - 1], rm = s_fold[i];
          const double gam = cm / bet;
          bet = bm - am * gam;
          zero = zero || (fabs(bet) <= 1.0e-100);
          u = (rm - am * u) / bet;
          gmine = (lane == m) ? gam : gmine;
          umine = (lane == m) ? u : umine;
        }
        const int i = c0 + lane;
        if (i <= NT) {
          s_smw[i] = gmine;
          s_fnew[i] = umine;
        }
      }
      fp_sync<WMAX>();
      if (zero) {
        for (int i = lane + 1; i <= NT; i += FPB) s_fnew[i] = 0.0;
      } else {
        /* back substitution on the unclipped values, then the reference's
         * clipping of u(2..num_nt) (each u(i+1) is clipped after u(i) used it) */
        double up = s_fnew[NT];
        for (int c1 = NT - 1; c1 >= 1; c1 -= FPB) {
          double mine = 0.0;
          const int mn = c1 < FPB ? c1 : FPB;
#pragma unroll 8
          for (int m = 0; m < mn; m++) {
            const int i = c1 - m;
            up = s_fnew[i] - s_smw[i + 1] * up;
            mine = (lane == m) ? up : mine;
          }
          const int i = c1 - lane;
          if (i >= 1) s_fnew[i] = mine;
        }
        fp_sync<WMAX>();
        for (int i = lane + 2; i <= NT; i += FPB)
          if (s_fnew[i] < 0.0) s_fnew[i] = 0.0;
      }
      fp_sync<WMAX>();
    }
    PF_END(pf_tri);
    if (lane == 0) {
      s_fnew[NT] = 0.0;
      s_fnew[1] = 0.0;
    }
    fp_sync<WMAX>();
    sum_p = 0.;
    double sE = 0.;
    for (int c0 = 1; c0 <= NT - 1; c0 += FPB) {       /* :1415-1419 */
      const int i = c0 + lane;
      double av = 0.0, bv = 0.0;
      if (i <= NT - 1) {
        const double fi = s_fnew[i], dg = s_gnt[i + 1] - s_gnt[i];
        av = dg * fi;
        bv = dg * s_gam[i] * fi;
      }
      s_seq[lane] = av;
      s_seq[FPB + lane] = bv;
      wave_sync();
      double mine = 0.0;
      const int mn = (NT - c0) < FPB ? (NT - c0) : FPB;
#pragma unroll 8
      for (int m = 0; m < mn; m++) {
        sum_p = sum_p + s_seq[m];
        sE = sE + s_seq[FPB + m];
        mine = (lane == m) ? sum_p : mine;
      }
      wave_sync();
      if (i <= NT - 1) s_Pnt[i] = mine;
    }
    sum_E = sE / sum_p;
    t_fp = t_fp + d_t;
    fp_steps = fp_steps + 1;
    fp_sync<WMAX>();
    for (int i = lane + 1; i <= NT; i += FPB) {
      const double v = s_fnew[i] / sum_p;
      s_fnew[i] = v;
      s_fold[i] = v;
    }
    fp_sync<WMAX>();
    /* new temperature (:1440-1468) */
    /* gbar, and the next sub-step's hr_th_c over the same bins (s_fold = s_fnew
     * now; n_lept and volume do not change before label 200): two in-order
     * chains in one pass */
    double gbar = 0.0;
    hr_th_c_next = 0.0;
    seq_sum2_lds(gbar, hr_th_c_next, 1, NT - 1, lane, s_seq,
                 [&](int i) { return s_gam[i] * s_fnew[i] * (s_gnt[i + 1] - s_gnt[i]); },
                 [&](int i) {
                   return -(8.176e-7 * s_dgic[i] * s_fold[i] * (s_gnt[i + 1] - s_gnt[i]) * volume * n_lept);
                 });
    double The_new = Th_e;
    PF_BEGIN();
    if (gbar > g_av) {
      int k = 0;
      while (gbar > g_av) {
        const double prev = The_new;
        The_new = The_new * F32(1.005);
#ifdef C2D_FP_PROF
        pf_calls++;
#endif
        g_av = search_eval(prev, The_new, +1, k++);
        if (guard > GUARD_MAX) break;
      }
    } else {
      int k = 0;
      while (gbar < g_av) {
        const double prev = The_new;
        The_new = The_new / F32(1.005);
#ifdef C2D_FP_PROF
        pf_calls++;
#endif
        g_av = search_eval(prev, The_new, -1, k++);
        if (The_new < 1.0e-2) break;
        if (guard > GUARD_MAX) break;
      }
    }
    PF_END(pf_gb);
    if (guard > GUARD_MAX) {
      if (lane == 0) atomicOr(P.err, FPERR_GUARD);
      return;
    }
    Te_new = 5.11e2 * The_new;
    Th_e = The_new;
    g_av_next = g_av;                                  /* = gamma_bar(Th_e) */
    if (!(t_fp < P.dt)) break;                         /* :1473 */
  }

  /* outputs (:1481-1500) */
  E_el = 0.0;
  E_pos = 0.0;
  E_el = seq_sum_lds(E_el, 2, NT, lane, s_seq,
                 [&](int i) { return s_fnew[i] * s_gam[i] * (s_gnt[i] - s_gnt[i - 1]); });
  E_el = E_el * ne * 8.176e-7 * volume;
  e_new = e_new + E_el + E_pos;
  for (int i = lane; i < NT; i += FPB) {
    P.f_out[(size_t)cell * NT + i] = s_fnew[i + 1];
    P.P_out[(size_t)cell * NT + i] = s_Pnt[i + 1] / sum_p;
  }
  /* nonthermal parameters (:1654-1736) */
  int i;
  for (i = 5; i <= NT - 5; i++)
    if (s_fnew[i] > 1.0e-10) break;
  const double gmin = s_gam[i];
  const int i_nt = i;
  for (i = NT - 5; i >= 5; i--)
    if (s_fnew[i] > 1.0e-15) break;
  const double gmax = s_gam[i];
  const auto dfn = [&](int q) { return (s_gam[q + 1] - s_gam[q]) * s_fnew[q]; };
  const double sum_th = seq_sum_lds(0.0, 1, i_nt - 1, lane, s_seq, dfn);
  const double sum_nt = seq_sum_lds(0.0, i_nt, NT - 1, lane, s_seq, dfn);
  double amxwl = sum_th / (sum_nt + sum_th);
  double p_nth = zin[FZ_PNTH];
  if (amxwl > 9.999e-1) {
    amxwl = 1.0;
  } else {
    p_nth = F32(0.1);
    double sum_g = 1.0e50, sumg_old;
    /* first bin with gamma/gmax >= 100 ends the fit sum (:1707-1717) */
    int i_end = NT - 1;
    for (i = i_nt; i <= NT - 2; i++)
      if (!(s_gam[i] / gmax < 100.0)) {
        i_end = i;
        break;
      }
    for (;;) {
      sumg_old = sum_g;
      sum_g = 0.0;
      double sum_gg = 0.0;
      const double p_1 = 1.0 - p_nth;
      double N_nt;
      if (fabs(p_1) > 1.0e-4)
        N_nt = (1. - amxwl) * p_1 / (c2d_pow(gmax, p_1) - c2d_pow(gmin, p_1));
      else
        N_nt = (1.0 - amxwl) / c2d_log(gmax / gmin);
      for (int c0 = i_nt; c0 < i_end; c0 += FPB) {
        const int q = c0 + lane;
        double v1 = 0.0, v2 = 0.0;
        if (q < i_end) {
          const double f_pl = N_nt / (c2d_pow(s_gam[q], p_nth) * c2d_exp_bf(s_gam[q] / gmax));
          v1 = f_pl * s_gam[q] * (s_gnt[q + 1] - s_gnt[q]);
          v2 = f_pl * (s_gnt[q + 1] - s_gnt[q]);
        }
        s_seq[lane] = v1;
        s_seq[FPB + lane] = v2;
        wave_sync();
        const int mn = (i_end - c0) < FPB ? (i_end - c0) : FPB;
#pragma unroll 8
        for (int m = 0; m < mn; m++) {
          sum_g = sum_g + s_seq[m];
          sum_gg = sum_gg + s_seq[FPB + m];
        }
        wave_sync();
      }
      sum_g = sum_g / sum_gg;
      sum_g = fabs(sum_g - sum_E);
      if (sum_g < sumg_old && p_nth < 10.) {
        p_nth = p_nth + 0.5e-1;
        continue;
      }
      break;
    }
  }
  if (lane == 0) {
    zo[FO_TE] = Te_new;
    zo[FO_NE] = n_p;
    zo[FO_GMIN] = gmin;
    zo[FO_GMAX] = gmax;
    zo[FO_AMXWL] = amxwl;
    zo[FO_PNTH] = p_nth;
    zo[FO_DIAG + C2D_FP_E_OLD] = e_old;
    zo[FO_DIAG + C2D_FP_E_NEW] = e_new;
    zo[FO_DIAG + C2D_FP_HR] = hr;
    zo[FO_DIAG + C2D_FP_HR_ST] = hr_st;
    zo[FO_DIAG + C2D_FP_DELTA_T] = fabs(Te_new - tea) / Te_new;
    zo[FO_DIAG + C2D_FP_STEPS] = (double)fp_steps;
    zo[FO_DIAG + C2D_FP_SKIPPED] = 0.0;
    zo[FO_DIAG + 7] = 0.0;
#ifdef C2D_FP_PROF
    zo[FO_DIAG + 0] = (double)pf_gb;
    zo[FO_DIAG + 1] = (double)pf_tri;
    zo[FO_DIAG + 2] = (double)(clock64() - pf_loop0);
    zo[FO_DIAG + 3] = (double)pf_calls;
#endif
  }
}

/* One zone per workgroup of FP_WAVES waves.  Wave 0 runs FP_calc (its
 * 200-bin state in LDS, one bin per lane); waves 1.. compute McDonald terms
 * for it (mcd_producer).  Line numbers: src/update2d.f. */
template <int WMAX>
__global__ void __launch_bounds__(WMAX * FPB) c2d_fp_kernel(const FpParams P) {
  /* wave-uniform by construction (readfirstlane): a scalar branch, so no
   * wave ever steps through the other role's barriers with EXEC = 0 */
  if (threadIdx.x == 0) {
    s_eg[0] = c2d_exp_bf(gammln(5.0e-1 + 2.0));
    s_eg[1] = c2d_exp_bf(gammln(5.0e-1 + 3.0));
  }
  __syncthreads();
  if (WMAX > 1) {
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x) / FPB;
    if (wave != 0) {
      mcd_producer(s_coop, s_batch8, P.mcd, wave, threadIdx.x % FPB, GbMemo{P.gb_key, P.gb_val, P.gb_mask});
      return;
    }
  }
  const int lane = threadIdx.x;
  fp_zone_body<WMAX>(P, lane);
  /* release the producers */
  if (fp_nwaves<WMAX>() > 1) {
    if (lane == 0) s_coop.cmd = MCD_CMD_EXIT;
    __syncthreads();
  }
}

}  // namespace c2d

extern "C" int c2d_launch_tridag(const double* a, const double* b, const double* c,
                                 const double* r, double* x, int ncell, int nt,
                                 hipStream_t stream) {
  if (nt > c2d::TRI_MAXN) return (int)hipErrorInvalidValue;
  const int grid = (ncell + c2d::TRI_BLOCK - 1) / c2d::TRI_BLOCK;
  hipLaunchKernelGGL(c2d::c2d_tridag_kernel, dim3(grid), dim3(c2d::TRI_BLOCK), 0, stream, a, b, c,
                     r, x, ncell, nt);
  return (int)hipGetLastError();
}

/* waves per zone: up to FP_WAVES_MAX while zone x waves stays near one wave
 * per SIMD (C3: 270 zones -> 4 waves, 25 ms vs 29 ms with 8), down to 1
 * (the single-wave series) once they fill the chip (1024 SIMDs on MI355X);
 * C2D_FP_WAVES overrides (A/B runs) */
extern "C" int c2d_fp_waves(int ncell, int n_simd) {
  if (const char* e = getenv("C2D_FP_WAVES")) {
    const int w = atoi(e);
    if (w >= 1 && w <= c2d::FP_WAVES_MAX) return w;
  }
  int w = c2d::FP_WAVES_MAX;
  while (w > 1 && (long long)ncell * w > 9LL * n_simd / 8) w /= 2;
  return w;
}

extern "C" int c2d_launch_fp(const c2d::FpParams* P, int ncell, int waves, hipStream_t stream) {
  if (ncell <= 0) return 0;
  if (waves < 1 || waves > c2d::FP_WAVES_MAX) return (int)hipErrorInvalidValue;
  if (waves == 1)
    hipLaunchKernelGGL(c2d::c2d_fp_kernel<1>, dim3(ncell), dim3(c2d::wave::FPB), 0, stream, *P);
  else
    hipLaunchKernelGGL(c2d::c2d_fp_kernel<c2d::FP_WAVES_MAX>, dim3(ncell), dim3(waves * c2d::wave::FPB),
                       0, stream, *P);
  return (int)hipGetLastError();
}
