/*
 * fp_fast.hip — the Fokker-Planck electron update (FP_calc,
 * src/update2d.f:337-1739) as a block-parallel kernel: C2D_FP_FAST.
 *
 * fp.hip's c2d_fp_kernel reproduces FP_calc bit for bit, so every sum,
 * the Thomas solve (tridag, update2d.f:2476-2518) and McDonald's series
 * (volume2d.f:598-626) run in the reference's order: one in-order latency
 * chain per zone per implicit sub-step.  Off the tea clamp a zone takes
 * thousands of sub-steps and the update is that chain's length.
 * This kernel keeps the same arithmetic per bin and per series term and
 * changes only the ORDER of the additions and the tridiagonal algorithm, so
 * its results differ from the exact kernel's by rounding (the stated
 * tolerance, DESIGN §4b and tests/test_gpu_fp.py):
 *   - one zone per workgroup of BS threads (BS/64 waves); thread t owns
 *     energy bin t+1 for every element-wise stage;
 *   - the reference's sequential sums are block reductions (wave butterfly,
 *     then the waves' partials in wave order: every thread gets the same
 *     bits, so all scalar control flow stays uniform across the block);
 *   - the cumulative Pnt is a block inclusive scan;
 *   - the 200-row Chang-Cooper system is solved by parallel cyclic reduction
 *     (8 levels, one row per thread, double-buffered in LDS, one barrier per
 *     level) instead of the Thomas recurrence;
 *   - McDonald's K2/K3 terms are evaluated BS at a time; each series' first
 *     stopping term is found by a block minimum, so the terms added are
 *     exactly the reference's (same stopping index); their sum is a tree.
 *     exp(-y) multiplies instead of exp(y) dividing (one exp, no divide);
 *   - gamma_bar keeps the exact kernel's memos (4 entries per zone, and a
 *     table shared by all zones and steps -- a separate one, since the
 *     values differ from the exact kernel's in the last bits).
 * The temperature search walks the same lattice Theta*1.005^k and stops at
 * the same crossing unless gbar and gamma_bar agree to within rounding.
 * Line numbers: src/update2d.f unless stated.
 */
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_wave.hpp"

namespace c2d {
namespace {

using namespace wave;
constexpr int NT = C2D_NUM_NT;
constexpr int NPH = C2D_NPHFIELD;
constexpr double PI_REF = 3.1415926536;       /* general.pa:24 */
constexpr double C_LIGHT = 2.9979245620e10;   /* general.pa:25 */
constexpr double LNL = 20.0;                  /* update2d.f:143 */
constexpr int MAX_FP_STEPS = 1000000;         /* update2d.f:585-599 */
constexpr int WMAXF = 8;                      /* waves per zone at most (BS = 512) */

/* zone state in LDS (namespace scope: ds_* accesses) */
__shared__ double f_gnt[NT + 2], f_gam[NT + 2], f_fold[NT + 2], f_fnew[NT + 2];
__shared__ double f_dgic[NT + 2], f_dgdt[NT + 2], f_disp[NT + 2];
__shared__ double f_bigW[NT + 2], f_bigC[NT + 2], f_em[NT + 2], f_Pnt[NT + 2], f_nf[NPH];
__shared__ double f_pcr[2][4][256];          /* PCR rows a, b, c, d (double-buffered) */
__shared__ double f_red[2][2][WMAXF];        /* block reductions: [slot][value][wave] */
__shared__ int f_ired[2][2][WMAXF];          /* block integer min/max                 */
__shared__ double f_eg[3];                   /* exp(gammln(2.5)), exp(gammln(3.5)), their ratio */
constexpr int ZMEMO = 64;                    /* the zone's gamma_bar memo (direct-mapped) */
__shared__ double f_mth[ZMEMO], f_mgv[ZMEMO];

/* one block of BS threads; `slot` alternates so each reduction needs one barrier */
template <int BS>
struct Blk {
  static constexpr int W = BS / FPB;
  int tid, lane, wave;
  int slot = 0, islot = 0;

  /* DPP move of a double within 16-lane rows (both halves, same control) */
  template <int CTRL>
  __device__ __forceinline__ static double dpp(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
  }
  /* the wave's sum: within each 16-lane row by DPP (xor 1, xor 2, rotate 4,
   * rotate 8), then the four rows' sums (lanes 0, 16, 32, 48) read as
   * uniform values and added in row order, so every lane holds the same bits */
  __device__ __forceinline__ static double wsum(double v) {
    v = v + dpp<0xB1>(v);          /* quad_perm [1,0,3,2] */
    v = v + dpp<0x4E>(v);          /* quad_perm [2,3,0,1] */
    v = v + dpp<0x124>(v);         /* row_ror:4           */
    v = v + dpp<0x128>(v);         /* row_ror:8           */
    double r = rl(v, 0);
    r = r + rl(v, 16);
    r = r + rl(v, 32);
    r = r + rl(v, 48);
    return r;
  }
  /* two sums at once; identical bits in every thread */
  __device__ __forceinline__ void sum2(double& a, double& b) {
    a = wsum(a);
    b = wsum(b);
    if (lane == 0) {
      f_red[slot][0][wave] = a;
      f_red[slot][1][wave] = b;
    }
    __syncthreads();
    double x = 0.0, y = 0.0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      x = x + f_red[slot][0][w];
      y = y + f_red[slot][1][w];
    }
    a = x;
    b = y;
    slot ^= 1;
  }
  __device__ __forceinline__ double sum(double a) {
    double b = 0.0;
    sum2(a, b);
    return a;
  }
  /* block minimum and maximum of two ints (same in every thread) */
  __device__ __forceinline__ void minmax(int& mn, int& mx) {
#pragma unroll
    for (int o = FPB / 2; o > 0; o >>= 1) {
      const int a = __shfl_xor(mn, o, FPB), b = __shfl_xor(mx, o, FPB);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    if (lane == 0) {
      f_ired[islot][0][wave] = mn;
      f_ired[islot][1][wave] = mx;
    }
    __syncthreads();
    mn = INT_MAX;
    mx = INT_MIN;
#pragma unroll
    for (int w = 0; w < W; w++) {
      mn = f_ired[islot][0][w] < mn ? f_ired[islot][0][w] : mn;
      mx = f_ired[islot][1][w] > mx ? f_ired[islot][1][w] : mx;
    }
    islot ^= 1;
  }
  /* first set flag of each of two series over a pass of T*BS terms (term
   * k*BS + tid is flag [k] of thread tid): a wave's first by ballot, then the
   * waves' minimum through LDS; INT_MAX if none is set */
  __device__ __forceinline__ static int first_lane(unsigned long long m) {
    return m ? __ffsll((long long)m) - 1 : INT_MAX;
  }
  template <int T>
  __device__ __forceinline__ void firsts(const bool (&fa)[T], const bool (&fb)[T], int& f2, int& f3) {
    int w2 = INT_MAX, w3 = INT_MAX;
#pragma unroll
    for (int k = T - 1; k >= 0; k--) {           /* the lowest k with a flag wins */
      const int la = first_lane(__ballot(fa[k])), lb = first_lane(__ballot(fb[k]));
      if (la != INT_MAX) w2 = k * BS + wave * FPB + la;
      if (lb != INT_MAX) w3 = k * BS + wave * FPB + lb;
    }
    if (lane == 0) {
      f_ired[islot][0][wave] = w2;
      f_ired[islot][1][wave] = w3;
    }
    __syncthreads();
    f2 = INT_MAX;
    f3 = INT_MAX;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const int x = f_ired[islot][0][w], y = f_ired[islot][1][w];
      f2 = x < f2 ? x : f2;
      f3 = y < f3 ? y : f3;
    }
    islot ^= 1;
  }
  /* block minima of two ints */
  __device__ __forceinline__ void min2(int& a, int& b) {
#pragma unroll
    for (int o = FPB / 2; o > 0; o >>= 1) {
      const int x = __shfl_xor(a, o, FPB), y = __shfl_xor(b, o, FPB);
      a = x < a ? x : a;
      b = y < b ? y : b;
    }
    if (lane == 0) {
      f_ired[islot][0][wave] = a;
      f_ired[islot][1][wave] = b;
    }
    __syncthreads();
    a = INT_MAX;
    b = INT_MAX;
#pragma unroll
    for (int w = 0; w < W; w++) {
      a = f_ired[islot][0][w] < a ? f_ired[islot][0][w] : a;
      b = f_ired[islot][1][w] < b ? f_ired[islot][1][w] : b;
    }
    islot ^= 1;
  }
  /* scan() of v together with the block sum of w, behind the same barrier */
  __device__ __forceinline__ double scan_sum(double v, double& total, double& w) {
    v = v + dpp<0x111>(v);
    v = v + dpp<0x112>(v);
    v = v + dpp<0x114>(v);
    v = v + dpp<0x118>(v);
    const double r0 = rl(v, 15), r1 = rl(v, 31), r2 = rl(v, 47);
    const int row = lane >> 4;
    if (row == 1) v = v + r0;
    if (row == 2) v = v + (r0 + r1);
    if (row == 3) v = v + ((r0 + r1) + r2);
    w = wsum(w);
    if (lane == FPB - 1) f_red[slot][0][wave] = v;
    if (lane == 0) f_red[slot][1][wave] = w;
    __syncthreads();
    double before = 0.0, all = 0.0, ws = 0.0;
#pragma unroll
    for (int q = 0; q < W; q++) {
      const double x = f_red[slot][0][q];
      if (q < wave) before = before + x;
      all = all + x;
      ws = ws + f_red[slot][1][q];
    }
    slot ^= 1;
    total = all;
    w = ws;
    return before + v;
  }
  /* inclusive prefix sum of v over the threads in tid order, and the total */
  __device__ __forceinline__ double scan(double v, double& total) {
    /* within 16-lane rows by DPP row shifts (lanes shifted in from outside
     * the row read 0), then the preceding rows' totals */
    v = v + dpp<0x111>(v);         /* row_shr:1 */
    v = v + dpp<0x112>(v);         /* row_shr:2 */
    v = v + dpp<0x114>(v);         /* row_shr:4 */
    v = v + dpp<0x118>(v);         /* row_shr:8 */
    const double r0 = rl(v, 15), r1 = rl(v, 31), r2 = rl(v, 47);
    const int row = lane >> 4;
    if (row == 1) v = v + r0;
    if (row == 2) v = v + (r0 + r1);
    if (row == 3) v = v + ((r0 + r1) + r2);
    if (lane == FPB - 1) f_red[slot][0][wave] = v;
    __syncthreads();
    double before = 0.0, all = 0.0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const double x = f_red[slot][0][w];
      if (w < wave) before = before + x;
      all = all + x;
    }
    slot ^= 1;
    total = all;
    return before + v;
  }
};

/* gamma_bar memo shared by every zone and step (the fast kernel's own
 * table: see fp.hip GbMemo for the protocol) */
constexpr int GB_PROBES = 8;
__device__ __forceinline__ uint32_t gb_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k;
}
__device__ __forceinline__ bool gb_lookup(const FpParams& P, double th, double& g) {
  if (!P.gb_key) return false;
  const unsigned long long k = c2d_bits(th);
  uint32_t h = gb_hash(k) & P.gb_mask;
  for (int i = 0; i < GB_PROBES; i++) {
    const unsigned long long kk = __hip_atomic_load(P.gb_key + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kk == k) {
      const double v = __hip_atomic_load(P.gb_val + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v != 0.0) { g = v; return true; }
      return false;
    }
    if (kk == 0ull) return false;
    h = (h + 1u) & P.gb_mask;
  }
  return false;
}
__device__ __forceinline__ void gb_insert(const FpParams& P, double th, double g) {
  if (!P.gb_key) return;
  const unsigned long long k = c2d_bits(th);
  uint32_t h = gb_hash(k) & P.gb_mask;
  for (int i = 0; i < GB_PROBES; i++) {
    const unsigned long long prev = atomicCAS(P.gb_key + h, 0ull, k);
    if (prev == 0ull) {
      __hip_atomic_store(P.gb_val + h, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (prev == k) return;
    h = (h + 1u) & P.gb_mask;
  }
}

/* McDonald K2, K3 (volume2d.f:598-626) by the whole block: terms n0 + tid of
 * each pass, the first stopping term of each series by a block minimum (so
 * exactly the reference's terms enter), per-thread partial sums, one tree
 * sum at the end.  Beyond the abscissa table wave 0 finishes the series with
 * c2d_wave's replayed chain (never reached on the reference's decks). */
#ifdef C2D_FP_PROF
__shared__ long long f_pf[4];   /* McDonald passes, cycles in the pass loop, in the finish */
#endif
/* exp(x) for -745 < x <= 0 (McDonald's terms, y < 225): x = k ln2 + r with
 * |r| <= ln2/2, e^r by its Taylor polynomial to degree 13 (truncation
 * < 5e-18) in FMAs, 2^k by v_ldexp -- ~17 dependent operations where
 * fdlibm's form (c2d_exp_bf) has a division in its chain; within 2 ulp */
__device__ __forceinline__ double exp_nonpos(double x) {
  const double kd = __builtin_rint(x * 1.4426950408889634);
  double r = __builtin_fma(-kd, 6.93147180369123816490e-01, x);
  r = __builtin_fma(-kd, 1.90821492927058770002e-10, r);
  double p = 1.6059043836821613e-10;                 /* 1/13! */
  p = __builtin_fma(p, r, 2.0876756987868100e-09);  /* 1/12! */
  p = __builtin_fma(p, r, 2.5052108385441720e-08);  /* 1/11! */
  p = __builtin_fma(p, r, 2.7557319223985893e-07);  /* 1/10! */
  p = __builtin_fma(p, r, 2.7557319223985888e-06);  /* 1/9!  */
  p = __builtin_fma(p, r, 2.4801587301587302e-05);  /* 1/8!  */
  p = __builtin_fma(p, r, 1.9841269841269841e-04);  /* 1/7!  */
  p = __builtin_fma(p, r, 1.3888888888888889e-03);  /* 1/6!  */
  p = __builtin_fma(p, r, 8.3333333333333332e-03);  /* 1/5!  */
  p = __builtin_fma(p, r, 4.1666666666666664e-02);  /* 1/4!  */
  p = __builtin_fma(p, r, 1.6666666666666666e-01);  /* 1/3!  */
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p, (int)kd);
}

/* 2^(j/64), j = 0..63, correctly rounded (decimal arithmetic at 50 digits) */
__constant__ double c_exp2_64[64] = {
    1, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.1023825833078409, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.2021567314527031, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.2553807570246911, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.3396675240533029,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.5590044002378369, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.6457554781539649, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.7186192981224779, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.9784560263879509,
};
__shared__ double f_e64[64];

/* exp(x), -745 < x <= 0, table-driven: x = (64 m + j) ln2/64 + r with
 * |r| <= ln2/128, e^x = 2^m 2^(j/64) e^r, e^r by its Taylor polynomial to
 * degree 5 (truncation < 4e-17); the N chains interleaved as below */
template <int N>
__device__ __forceinline__ void exp_nonpos_tab(const double (&x)[N], double (&e)[N]) {
  double kd[N], r[N], p[N];
  int ki[N];
#pragma unroll
  for (int j = 0; j < N; j++) {
    kd[j] = __builtin_rint(x[j] * 92.332482616893658);            /* 64 / ln2 */
    r[j] = __builtin_fma(-kd[j], 6.93147180369123816490e-01 / 64.0, x[j]);
    r[j] = __builtin_fma(-kd[j], 1.90821492927058770002e-10 / 64.0, r[j]);
    ki[j] = (int)kd[j];
    p[j] = 1.0 / 120.0;
  }
  constexpr double C[5] = {1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
#pragma unroll
  for (int i = 0; i < 5; i++) {
#pragma unroll
    for (int j = 0; j < N; j++) p[j] = __builtin_fma(p[j], r[j], C[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < N; j++) e[j] = __builtin_ldexp(p[j] * f_e64[ki[j] & 63], ki[j] >> 6);
}

/* one abscissa row through a global (not flat) pointer */
__device__ __forceinline__ double4 gld4(const double* p) {
  const C2D_GLOBAL double* q = (const C2D_GLOBAL double*)p;
  return make_double4(q[0], q[1], q[2], q[3]);
}

/* the abscissa row of term n: the table's, or past it (never reached on the
 * reference's decks: the table covers Theta up to ~1e5) the chain continued
 * from the table's last t by a power of dt instead of the reference's
 * repeated product: the same values to rounding */
__device__ __forceinline__ double4 mcd_row(const double* __restrict__ tab, int n) {
  if (n < C2D_FP_MCD_N) return gld4((tab + (size_t)n * 4));
  const double dt = 1.001, sm = 5.0e-1 * (1.0 + dt);
  const double t = tab[(size_t)(C2D_FP_MCD_N - 1) * 4] * c2d_exp_bf((double)(n - C2D_FP_MCD_N + 1) * c2d_log(dt));
  const double ts = t * sm;
  const double q = ts * ts - 1.0, rq = __builtin_sqrt(q);
  return make_double4(t, ts, q * rq, q * q * rq);
}

/* McDonald terms per thread per pass (C2D_FPF_TPT: 2 or 4) */
#ifndef C2D_FPF_TPT
#define C2D_FPF_TPT 4
#endif
constexpr int TPT = C2D_FPF_TPT;

/* one pass of TPT*BS terms (row x[k]: term n0 + k*BS + tid) */
template <int BS>
__device__ __forceinline__ void mcd_pass(Blk<BS>& B, double z, const double4 (&x)[TPT], double& s2, double& s3,
                                         bool& run2, bool& run3) {
  const double dt = 1.001, d = dt - 1.0;
  double v2[TPT], v3[TPT];
  bool st2[TPT], st3[TPT];
  /* branch-free, so the TPT exp chains interleave: exp of the argument
   * clamped to the reference's cut, the term zeroed beyond it */
  double em[TPT], ny[TPT];
#pragma unroll
  for (int k = 0; k < TPT; k++) {
    const double y = z * x[k].y;
    ny[k] = -(y < 2.25e2 ? y : 2.25e2);
  }
  exp_nonpos_tab<TPT>(ny, em);
#pragma unroll
  for (int k = 0; k < TPT; k++)
    if (!(ny[k] > -2.25e2)) em[k] = 0.0;              /* y >= 225: the reference's zero term */
#pragma unroll
  for (int k = 0; k < TPT; k++) {
    v2[k] = x[k].z * em[k];
    v3[k] = x[k].w * em[k];
    const double tn = x[k].x * dt;
    st2[k] = !(tn < 2.0 || v2[k] > 1.0e-8);
    st3[k] = !(tn < 2.0 || v3[k] > 1.0e-8);
  }
  int f2, f3;
#ifdef C2D_FP_PROF_MCD
  const long long pa = clock64();
#endif
  B.template firsts<TPT>(st2, st3, f2, f3);
#ifdef C2D_FP_PROF_MCD
  if (B.tid == 0) f_pf[3] += clock64() - pa;        /* the stopping test incl. its barrier */
#endif
  /* terms up to and including each series' first stopping term */
#pragma unroll
  for (int k = 0; k < TPT; k++) {
    const int n = k * BS + B.tid;
    if (run2 && n <= f2) s2 = s2 + d * x[k].x * v2[k];
    if (run3 && n <= f3) s3 = s3 + d * x[k].x * v3[k];
  }
  if (f2 != INT_MAX) run2 = false;
  if (f3 != INT_MAX) run3 = false;
}

/* McDonald K2, K3 (volume2d.f:598-626) by the whole block: TPT*BS terms per
 * pass (TPT per thread, the next pass's abscissa rows loaded ahead), each
 * series' first stopping term by ballot + a block minimum (so exactly the
 * reference's terms enter), per-thread partial sums, one tree sum at the end. */
template <int BS>
__device__ void mcdonald23_fast(Blk<BS>& B, double z, const double* __restrict__ tab, double& K2, double& K3,
                                long long& guard) {
  constexpr int PASS = TPT * BS;
  static_assert(C2D_FP_MCD_N % PASS == 0, "table passes");
  double s2 = 0.0, s3 = 0.0;
  bool run2 = true, run3 = true;
#ifdef C2D_FP_PROF
  const long long pt0 = clock64();
#endif
  int n0 = 0;
  const double* row = tab + (size_t)B.tid * 4;
  double4 e[TPT];
#pragma unroll
  for (int k = 0; k < TPT; k++) e[k] = gld4((row + (size_t)k * BS * 4));
  for (; n0 < C2D_FP_MCD_N; n0 += PASS) {
#ifdef C2D_FP_PROF
    if (B.tid == 0) f_pf[0]++;
#endif
    double4 x[TPT];
#pragma unroll
    for (int k = 0; k < TPT; k++) x[k] = e[k];
    /* next pass's rows, ahead: global (not flat) loads, so the LDS waits
     * of the pass (lgkmcnt) do not wait for them too */
    if (n0 + PASS < C2D_FP_MCD_N) {
#pragma unroll
      for (int k = 0; k < TPT; k++) e[k] = gld4((row + (size_t)(n0 + PASS + k * BS) * 4));
    }
    mcd_pass<BS>(B, z, x, s2, s3, run2, run3);
    guard += PASS;
    if (!run2 && !run3) break;
  }
  /* past the table (never reached on the reference's decks) */
  for (; (run2 || run3) && guard <= GUARD_MAX; n0 += PASS) {
    double4 x[TPT];
#pragma unroll
    for (int k = 0; k < TPT; k++) x[k] = mcd_row(tab, n0 + k * BS + B.tid);
    mcd_pass<BS>(B, z, x, s2, s3, run2, run3);
    guard += PASS;
  }
#ifdef C2D_FP_PROF
  const long long pt1 = clock64();
#endif
  B.sum2(s2, s3);
  mcdonald23_finish_c(z, s2, s3, f_eg[0], f_eg[1], K2, K3);
#ifdef C2D_FP_PROF
  if (B.tid == 0) {
    f_pf[1] += pt1 - pt0;
    f_pf[2] += clock64() - pt1;
  }
#endif
}

/* 1/x: v_rcp_f64 and two Newton steps (fast mode: < 1 ulp) */
__device__ __forceinline__ double rcp_nr(double x) {
  double q = __builtin_amdgcn_rcp(x);
  q = __builtin_fma(__builtin_fma(-x, q, 1.0), q, q);
  return __builtin_fma(__builtin_fma(-x, q, 1.0), q, q);
}
/* ... with 1/0 = inf as IEEE division has it (the Newton steps turn the
 * estimate's inf into NaN) */
__device__ __forceinline__ double rcp_nr_safe(double x) {
  const double q = rcp_nr(x);
  return x == 0.0 ? __builtin_amdgcn_rcp(x) : q;
}

/* McDonald moment table (C2D_FPF_MTAB).  Both series are sums over one fixed
 * abscissa lattice, S(z) = sum_{n <= f(z)} w_n exp(-z ts_n), so around a grid
 * point z0 (y_n = z0 ts_n, eta = z/z0 - 1)
 *   S(z) = sum_k (-eta)^k N_k(z0),   N_k = sum_{n <= f(z0)} w_n e^{-y_n} y_n^k / k!
 * as long as the stopping index is the same; the terms between f(z0) and
 * f(z) (f moves by ~0.5 term per grid step) are added or removed one by one,
 * each found by the reference's own stopping test at z.  With 1024 points per
 * octave |eta| <= 3.4e-4, and the terms that carry the sums have y < ~30: 7
 * moments leave (eta y)^7/7! < 1e-17 of a term.  The abscissa rows around
 * f(z0) ride in the entry, so a pair is one load of an entry (336 B), two
 * Horner chains and four exps per series, instead of ~8000 terms; the sum
 * differs from the term-by-term one by rounding (the moments are compensated
 * sums in n order; 1.1e-15, tests/test_gpu_fp.py).  Entries whose series
 * would run past the abscissa table are marked f = -1: the series instead. */
constexpr int MT_K = C2D_FPF_MT_K, MT_W = C2D_FPF_MT_W, MT_N = C2D_FPF_MT_N;
constexpr int MT_ROWS = 4 + 2 * MT_K;           /* the rows of series 2, then 3 */

/* the reference's term of one series at z and its stopping test
 * (volume2d.f:608-620), as mcd_pass computes them, for one abscissa row */
__device__ __forceinline__ double mt_term(double z, double t, double ts, double p, bool& stop) {
  const double y = z * ts;
  double ny[1] = {-(y < 2.25e2 ? y : 2.25e2)}, em[1];
  exp_nonpos_tab<1>(ny, em);
  if (!(ny[0] > -2.25e2)) em[0] = 0.0;
  const double v = p * em[0];
  stop = !(t * 1.001 < 2.0 || v > 1.0e-8);
  return (1.001 - 1.0) * t * v;
}
template <int SER>
__device__ __forceinline__ double mt_term_tab(const double* __restrict__ tab, double z, int n, bool& stop) {
  const double4 x = gld4(tab + (size_t)n * 4);
  return mt_term(z, x.x, x.y, SER == 2 ? x.z : x.w, stop);
}

/* s: the series at z from the moments at z0 (stopping index f0); tm[], st[]:
 * the terms and stopping tests at z of the rows f0-1 .. f0+2.  Moves the
 * stopping index to z's.  False: more than 4 terms apart, or past the table */
template <int SER>
__device__ __forceinline__ bool mt_fix(const double* __restrict__ tab, double z, int f0, const double (&tm)[4],
                                       const bool (&st)[4], double& s) {
  if (st[1]) {                                /* f(z) <= f0 */
    if (!st[0]) return true;                  /* f(z) = f0 */
    double sub = tm[1], t1 = tm[0];           /* drop f0; f0-1 stops too: look further down */
    int f = f0 - 1;
    for (int it = 0;; it++) {
      if (f == 0) break;
      bool sp;
      const double tp = mt_term_tab<SER>(tab, z, f - 1, sp);
      if (!sp) break;
      if (it == 3) return false;
      sub = sub + t1;
      t1 = tp;
      f--;
    }
    s = s - sub;
    return true;
  }
  s = s + tm[2];                              /* f(z) > f0 */
  if (st[2]) return true;
  s = s + tm[3];
  if (st[3]) return true;
  for (int n = f0 + 3, it = 0;; n++, it++) {
    if (n >= C2D_FP_MCD_N || it == 2) return false;
    bool sn;
    s = s + mt_term_tab<SER>(tab, z, n, sn);
    if (sn) return true;
  }
}

/* both sums at z from the table (every thread alike: same bits, uniform) */
__device__ __forceinline__ bool mcd_mtab(const double* __restrict__ mom, const double* __restrict__ tab, double z,
                                         double& S2, double& S3, long long* tmr = nullptr) {
  if (!mom || !(z >= 0x1p-17 && z <= 0x1p3)) return false;
  const float l2 = __builtin_amdgcn_logf((float)z);           /* log2 z, ~1e-7 */
  int j = (int)__builtin_rintf((l2 - (float)C2D_FPF_MT_LO) * (float)C2D_FPF_MT_Q);
  j = j < 0 ? 0 : (j > MT_N - 1 ? MT_N - 1 : j);
  const double* e = mom + (size_t)j * MT_W;
  /* the whole entry at once: every address is known before any value */
  const C2D_GLOBAL double* eg = (const C2D_GLOBAL double*)e;
  double w[MT_W];
#pragma unroll
  for (int q = 0; q < MT_W; q++) w[q] = eg[q];
  const int f2 = (int)w[2], f3 = (int)w[3];
  if (f2 < 1 || f3 < 1) return false;
  /* the eight rows' terms at z (both series side by side: one exp chain of
   * eight interleaved), and the two Horner chains beside them */
  double ny[8], em[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const double y = z * w[MT_ROWS + 3 * q + 1];
    ny[q] = -(y < 2.25e2 ? y : 2.25e2);
  }
  exp_nonpos_tab<8>(ny, em);
  const double ne = -__builtin_fma(z, w[1], -1.0);            /* -eta */
  double s2 = w[4 + MT_K - 1], s3 = w[4 + 2 * MT_K - 1];
#pragma unroll
  for (int k = MT_K - 2; k >= 0; k--) {
    s2 = __builtin_fma(s2, ne, w[4 + k]);
    s3 = __builtin_fma(s3, ne, w[4 + MT_K + k]);
  }
  double tm2[4], tm3[4];
  bool st2[4], st3[4];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (!(ny[q] > -2.25e2)) em[q] = 0.0;
    const double t = w[MT_ROWS + 3 * q], v = w[MT_ROWS + 3 * q + 2] * em[q];
    const bool st = !(t * 1.001 < 2.0 || v > 1.0e-8);
    const double tm = (1.001 - 1.0) * t * v;
    if (q < 4) { tm2[q] = tm; st2[q] = st; } else { tm3[q - 4] = tm; st3[q - 4] = st; }
  }
  if (tmr) tmr[0] = clock64() + (long long)(s2 + s3 + tm2[0] + tm3[0] == 1.2345 ? 1 : 0);
  if (!mt_fix<2>(tab, z, f2, tm2, st2, s2) || !mt_fix<3>(tab, z, f3, tm3, st3, s3)) return false;
  if (tmr) tmr[1] = tmr[2] = clock64() + (long long)(s2 + s3 == 1.2345 ? 1 : 0);
  S2 = s2;
  S3 = s3;
  return true;
}

/* C2D_FPF_MT_PF: the table entries of the next search's first candidates
 * (Theta 1.005^{+-1}) fetched into the caches at the top of the sub-step,
 * by 12 lanes of wave 0 through global -> LDS loads into a scratch row (no
 * registers held, nothing waits for them): the search then finds them in L2 */
#ifndef C2D_FPF_MT_PF
#define C2D_FPF_MT_PF 1
#endif
__shared__ uint32_t f_mtpf[64];
typedef const __attribute__((address_space(1))) void* fpf_gptr_t;
typedef __attribute__((address_space(3))) void* fpf_lptr_t;
__device__ __forceinline__ void mt_prefetch(const double* __restrict__ mom, double th, int lane) {
  if (!mom || lane >= 12) return;
  const double t = lane < 6 ? th * F32(1.005) : th / F32(1.005);     /* the search's own lattice */
  const double z = rcp_nr(t);
  if (!(z >= 0x1p-17 && z <= 0x1p3)) return;
  int j = (int)__builtin_rintf((__builtin_amdgcn_logf((float)z) - (float)C2D_FPF_MT_LO) * (float)C2D_FPF_MT_Q);
  j = j < 0 ? 0 : (j > MT_N - 1 ? MT_N - 1 : j);
  /* an entry spans 336 B: one dword every 64 B touches each of its cache lines */
  const uint32_t* a = reinterpret_cast<const uint32_t*>(mom + (size_t)j * MT_W) + (lane % 6) * 16;
  __builtin_amdgcn_global_load_lds((fpf_gptr_t)a, (fpf_lptr_t)&f_mtpf[0], 4, 0, 0);
}

/* Neumaier's compensated sum */
__device__ __forceinline__ void nsum(double& s, double& c, double w) {
  const double t = s + w;
  c = c + ((fabs(s) >= fabs(w)) ? (s - t) + w : (w - t) + s);
  s = t;
}

/* the table: one entry per thread, the series in n order at z0 */
__global__ void __launch_bounds__(64) c2d_fp_mom_kernel(const double* __restrict__ tab, double* __restrict__ mom) {
  f_e64[threadIdx.x] = c_exp2_64[threadIdx.x];
  __syncthreads();
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= MT_N) return;
  const double z0 = c2d_exp_bf(((double)j / C2D_FPF_MT_Q + C2D_FPF_MT_LO) * 6.93147180559945309417e-01);
  double a2[MT_K], c2[MT_K], a3[MT_K], c3[MT_K];
#pragma unroll
  for (int k = 0; k < MT_K; k++) a2[k] = c2[k] = a3[k] = c3[k] = 0.0;
  bool run2 = true, run3 = true;
  int f2 = -1, f3 = -1;
  for (int n = 0; n < C2D_FP_MCD_N && (run2 || run3); n++) {
    const double4 x = gld4(tab + (size_t)n * 4);
    const double y = z0 * x.y;
    double ny[1] = {-(y < 2.25e2 ? y : 2.25e2)}, em[1];
    exp_nonpos_tab<1>(ny, em);
    if (!(ny[0] > -2.25e2)) em[0] = 0.0;
    const double v2 = x.z * em[0], v3 = x.w * em[0];
    const double tn = x.x * 1.001, dtt = (1.001 - 1.0) * x.x;
    if (run2) {
      double w = dtt * v2;
#pragma unroll
      for (int k = 0; k < MT_K; k++) {
        nsum(a2[k], c2[k], w);
        w = w * y / (double)(k + 1);
      }
      if (!(tn < 2.0 || v2 > 1.0e-8)) {
        run2 = false;
        f2 = n;
      }
    }
    if (run3) {
      double w = dtt * v3;
#pragma unroll
      for (int k = 0; k < MT_K; k++) {
        nsum(a3[k], c3[k], w);
        w = w * y / (double)(k + 1);
      }
      if (!(tn < 2.0 || v3 > 1.0e-8)) {
        run3 = false;
        f3 = n;
      }
    }
  }
  /* usable: stopped at least one row into the table and 3 rows before its end */
  const bool ok2 = f2 >= 1 && f2 < C2D_FP_MCD_N - 3, ok3 = f3 >= 1 && f3 < C2D_FP_MCD_N - 3;
  double* e = mom + (size_t)j * MT_W;
  e[0] = z0;
  e[1] = 1.0 / z0;
  e[2] = ok2 ? (double)f2 : -1.0;
  e[3] = ok3 ? (double)f3 : -1.0;
#pragma unroll
  for (int k = 0; k < MT_K; k++) {
    e[4 + k] = a2[k] + c2[k];
    e[4 + MT_K + k] = a3[k] + c3[k];
  }
  for (int q = 0; q < 4; q++) {
    const int n2 = ok2 ? f2 - 1 + q : 0, n3 = ok3 ? f3 - 1 + q : 0;
    e[MT_ROWS + 3 * q] = tab[(size_t)n2 * 4];
    e[MT_ROWS + 3 * q + 1] = tab[(size_t)n2 * 4 + 1];
    e[MT_ROWS + 3 * q + 2] = tab[(size_t)n2 * 4 + 2];
    e[MT_ROWS + 12 + 3 * q] = tab[(size_t)n3 * 4];
    e[MT_ROWS + 12 + 3 * q + 1] = tab[(size_t)n3 * 4 + 1];
    e[MT_ROWS + 12 + 3 * q + 2] = tab[(size_t)n3 * 4 + 3];
  }
}

template <int BS>
__device__ double gamma_bar_fast(Blk<BS>& B, double Theta, const double* tab, const double* mom, long long& guard) {
  double g;
  if (Theta < F32(0.2)) {
    g = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) + F32(3.384) * (Theta * Theta * Theta)) /
            (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
        Theta;
  } else {
    double K2, K3, S2, S3;
    const double z = rcp_nr(Theta);
    if (mcd_mtab(mom, tab, z, S2, S3)) {
      /* K3/K2 = (z/2) (S3/S2) exp(gammln(2.5))/exp(gammln(3.5)) (volume2d.f:623-624):
       * the normalisations' powers of z/2 cancel but one */
      g = (5.0e-1 * z) * (S3 * rcp_nr(S2)) * f_eg[2] - Theta;
    } else {
      mcdonald23_fast<BS>(B, z, tab, K2, K3, guard);
      g = K3 / K2 - Theta;
    }
  }
  if (g < 1.0) g = 1.0;
  return g;
}

/* PCR on rows 1..NT (row i in thread i-1): a x_{i-1} + b x_i + c x_{i+1} = d.
 * Rows outside 1..NT act as the identity (a = c = d = 0, b = 1). */
template <int BS>
__device__ double pcr_solve(Blk<BS>& B, double a, double b, double c, double dd) {
  const int i = B.tid + 1;
  const bool own = i <= NT;
  int buf = 0;
  for (int s = 1; s < NT; s <<= 1) {
    if (own) {
      f_pcr[buf][0][i] = a;
      f_pcr[buf][1][i] = b;
      f_pcr[buf][2][i] = c;
      f_pcr[buf][3][i] = dd;
    }
    __syncthreads();
    if (own) {
      double am = 0.0, bm = 1.0, cm = 0.0, dm = 0.0, ap = 0.0, bp = 1.0, cp = 0.0, dp = 0.0;
      if (i - s >= 1) {
        am = f_pcr[buf][0][i - s]; bm = f_pcr[buf][1][i - s];
        cm = f_pcr[buf][2][i - s]; dm = f_pcr[buf][3][i - s];
      }
      if (i + s <= NT) {
        ap = f_pcr[buf][0][i + s]; bp = f_pcr[buf][1][i + s];
        cp = f_pcr[buf][2][i + s]; dp = f_pcr[buf][3][i + s];
      }
      /* a / bm and c / bp through reciprocals: v_rcp_f64 and two Newton
       * steps each, the two chains side by side (fast mode: < 1 ulp) */
      double q1 = __builtin_amdgcn_rcp(bm), q2 = __builtin_amdgcn_rcp(bp);
      q1 = __builtin_fma(__builtin_fma(-bm, q1, 1.0), q1, q1);
      q2 = __builtin_fma(__builtin_fma(-bp, q2, 1.0), q2, q2);
      q1 = __builtin_fma(__builtin_fma(-bm, q1, 1.0), q1, q1);
      q2 = __builtin_fma(__builtin_fma(-bp, q2, 1.0), q2, q2);
      const double k1 = a * q1, k2 = c * q2;
      const double na = -am * k1, nc = -cp * k2;
      const double nb = b - cm * k1 - ap * k2;
      const double nd = dd - dm * k1 - dp * k2;
      a = na; b = nb; c = nc; dd = nd;
    }
    buf ^= 1;
  }
  return own ? dd / b : 0.0;
}

/* The same system, rows 1..NT (row i in thread i-1, rows past NT identity
 * rows), by partitions: wave w holds rows 64w+1..64w+64 and reduces its own
 * block by cyclic reduction across its lanes (through wave-private LDS rows,
 * no barrier; lane shuffles measured slower, r04s)
 * for three right-hand sides at once, d and the two spikes that couple the
 * block to the last unknown L of the previous partition and the first
 * unknown F of the next (x = y - v L_{w-1} - w F_{w+1}); the partitions' edge
 * rows form a chain over the W-1 interfaces that every thread then solves
 * for itself, behind one barrier (8 barriers for pcr_solve). */
__shared__ double f_if[WMAXF][6];
__shared__ double2 f_sac[WMAXF][FPB], f_sdv[WMAXF][FPB];   /* (a, c), (d, v) per lane */
__shared__ double f_sw[WMAXF][FPB];
template <int BS>
__device__ double spike_solve(Blk<BS>& B, double a, double b, double c, double d) {
  constexpr int W = BS / FPB;
  const int lane = B.lane, wave = B.wave;
  double v = (lane == 0) ? a : 0.0;           /* left spike  */
  double w = (lane == FPB - 1) ? c : 0.0;     /* right spike */
  if (lane == 0) a = 0.0;
  if (lane == FPB - 1) c = 0.0;
  /* unit diagonal: row r reads x_r + a x_{r-s} + c x_{r+s} = (d, v, w) */
  double r = rcp_nr(b);
  a = a * r; c = c * r; d = d * r; v = v * r; w = w * r;
#pragma unroll 1
  for (int s = 1; s < FPB; s <<= 1) {
    const int lm = lane - s, lp = lane + s;
    /* through the wave's own LDS rows: the wave's lanes store and then load
     * in program order, so no barrier (a wavefront fence keeps the order) */
    f_sac[wave][lane] = make_double2(a, c);
    f_sdv[wave][lane] = make_double2(d, v);
    f_sw[wave][lane] = w;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int qm = lm < 0 ? 0 : lm, qp = lp >= FPB ? FPB - 1 : lp;
    const double2 acm = f_sac[wave][qm], dvm = f_sdv[wave][qm];
    const double2 acp = f_sac[wave][qp], dvp = f_sdv[wave][qp];
    double am = acm.x, cm = acm.y, dm = dvm.x, vm = dvm.y, wm = f_sw[wave][qm];
    double ap = acp.x, cp = acp.y, dp = dvp.x, vp = dvp.y, wp = f_sw[wave][qp];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lm < 0) am = cm = dm = vm = wm = 0.0;      /* outside the block: a = 0 there */
    if (lp >= FPB) ap = cp = dp = vp = wp = 0.0;
    r = rcp_nr(1.0 - a * cm - c * ap);
    const double na = -(a * am), nc = -(c * cp);
    d = (d - a * dm - c * dp) * r;
    v = (v - a * vm - c * vp) * r;
    w = (w - a * wm - c * wp) * r;
    a = na * r;
    c = nc * r;
  }
  if (lane == 0) {
    f_if[wave][0] = d; f_if[wave][1] = v; f_if[wave][2] = w;
  }
  if (lane == FPB - 1) {
    f_if[wave][3] = d; f_if[wave][4] = v; f_if[wave][5] = w;
  }
  __syncthreads();
  /* interfaces p = 1..W-1 carry (L_{p-1}, F_p):
   *   L_{p-1} = A_p + Bp_p F_p,  F_p = G_p + H_p F_{p+1},  F_W = 0 */
  double A[W], Bp[W], G[W], H[W], F[W + 1], L[W];
  A[1] = f_if[0][3];
  Bp[1] = -f_if[0][5];
#pragma unroll
  for (int p = 1; p < W; p++) {
    const double yf = f_if[p][0], vf = f_if[p][1], wf = f_if[p][2];
    const double q = rcp_nr(1.0 + vf * Bp[p]);
    G[p] = (yf - vf * A[p]) * q;
    H[p] = -(wf * q);
    if (p + 1 < W) {
      const double yl = f_if[p][3], vl = f_if[p][4], wl = f_if[p][5];
      A[p + 1] = yl - vl * (A[p] + Bp[p] * G[p]);
      Bp[p + 1] = -(vl * Bp[p] * H[p] + wl);
    }
  }
  F[W] = 0.0;
#pragma unroll
  for (int p = W - 1; p >= 1; p--) {
    F[p] = G[p] + H[p] * F[p + 1];
    L[p - 1] = A[p] + Bp[p] * F[p];
  }
  double xl = 0.0, xr = 0.0;
#pragma unroll
  for (int p = 0; p < W; p++) {
    if (p + 1 == wave) xl = L[p];
    if (p == wave + 1) xr = F[p];
  }
  return (B.tid < NT) ? d - v * xl - w * xr : 0.0;
}

/* FP_calc of one zone (blockIdx.x) by the whole block */
template <int BS>
__device__ __forceinline__ void fp_zone_fast(const FpParams& P, Blk<BS>& B, const int cell) {
  const int tid = B.tid;
  const int j = cell / P.nr + 1, k = cell % P.nr + 1;
  const Geo* G = P.geo;
  const double* zin = P.zin + (size_t)cell * FZ_N;
  double* zo = P.zout + (size_t)cell * FO_N;
  long long guard = 0;
  const int i = tid + 1;                   /* this thread's energy bin */
  const bool own = i <= NT;

  const double volume = zin[FZ_VOL], tea = zin[FZ_TEA], tna = zin[FZ_TNA];
  const double Bf = zin[FZ_B], Eloss_sy = zin[FZ_ELSY], f_pair = zin[FZ_FPAIR];
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
    if (tid == 0) {
      zo[FO_TE] = Te_new;
      for (int q = 0; q < C2D_FP_NDIAG; q++) zo[FO_DIAG + q] = 0.0;
      zo[FO_DIAG + C2D_FP_SKIPPED] = 1.0;
    }
    return;
  }
  if (own) {
    f_gnt[i] = P.gnt[i - 1];
    f_gam[i] = P.gnt[i - 1] + 1.0;
    f_fold[i] = P.f_in[(size_t)cell * NT + i - 1];
    f_Pnt[i] = P.P_in[(size_t)cell * NT + i - 1];
  }
  for (int q = tid; q < NPH; q += BS) f_nf[q] = P.nf[(size_t)cell * NPH + q];
  __syncthreads();
  /* this thread's bin widths (used by most sums) */
  const double dgp = (i <= NT - 1) ? f_gnt[i + 1] - f_gnt[i] : 0.0;    /* gnt(i+1)-gnt(i) */
  const double dgm = (i >= 2 && own) ? f_gnt[i] - f_gnt[i - 1] : 0.0;  /* gnt(i)-gnt(i-1) */
  const double gi = own ? f_gam[i] : 0.0;

  /* E_el, normalisation (:482-509) */
  double E_el = B.sum((i >= 2 && own) ? dgm * gi * f_fold[i] : 0.0);
  double E_pos = 0.0;
  E_el = E_el * ne * 8.176e-7 * volume;
  double e_old = 0.0 + E_el + E_pos + zin[FZ_ECOLD];
  double e_new = 0.0 + ecens;
  double sum_p = B.sum((i <= NT - 1) ? dgp * f_fold[i] : 0.0);
  if (own) f_fold[i] = (i == NT) ? 0.0 : f_fold[i] / sum_p;

  /* flare (:532-562) */
  const double rmid = 5.0e-1 * (G->r[k] + G->r[k - 1]);
  const double zmid = 5.0e-1 * (G->z[j] + G->z[j - 1]);
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
  const double r_fth = rcp_nr_safe(f_th), r_dt = rcp_nr_safe(P.dt), r_tesc = rcp_nr_safe(t_esc);
  /* dg_ic(i) = -sum_ph n_field(ph) F_IC(i,ph) / volume (:568-574) */
  if (i <= NT - 1) {
    double s = 0.0;
    const double* ft = P.FT + (i - 1);
    for (int ph = 0; ph < NPH; ph++) s = s - f_nf[ph] * ft[(size_t)ph * NT] / volume;
    f_dgic[i] = s;
  }
  if (i == NT) f_dgic[NT] = 0.0;     /* hazard H10 */
  const double dz = G->z[j] - G->z[j - 1];          /* :628-632 */
  __syncthreads();

  double hr = 0.0, hr_st = 0.0, sum_E = 0.0, t_fp = 0.0;
  int fp_steps = 0;
  double g_av_next = 0.0, hr_th_c_next = 0.0;
#ifdef C2D_FP_PROF
  /* section timers (tools/fp_prof.py): zone_diag 0 = gamma_bar incl. memo,
   * 1 = PCR solve, 2 = whole sub-step loop, 3 = McDonald pairs computed */
  long long pf_gb = 0, pf_tri = 0, pf_loop0 = clock64(), pf_t0 = 0, pf_mcd = 0;
  long long pf_sa = 0, pf_sb = 0, pf_sc = 0, pf_s0 = 0;   /* C2D_FP_PROF_SEC sections */
  long long pm_calls = 0, pm_lds = 0, pm_glob = 0;         /* C2D_FP_PROF_MEMO counts */
#define PF_BEGIN() pf_t0 = clock64()
#define PF_END(acc) acc += clock64() - pf_t0
#else
#define PF_BEGIN()
#define PF_END(acc)
#endif
#ifdef C2D_FP_PROF_SEC
#define PS_BEGIN() pf_s0 = clock64()
#define PS_END(acc) acc += clock64() - pf_s0
#else
#define PS_BEGIN()
#define PS_END(acc)
#endif
  /* gamma_bar is a pure function of Theta, and a zone's search revisits the
   * lattice values around its temperature sub-step after sub-step: a
   * 64-entry direct-mapped memo in LDS keyed on Theta's bits answers those.
   * glob: also consult and fill the table shared by all zones, which pays
   * where zones walk the same chain (C3: every zone from the tea clamp, many
   * lattice steps per search): used for a zone's first value and from a
   * search's third step on; a zone tracking its own temperature stays off it */
  for (int q = tid; q < ZMEMO; q += BS) f_mth[q] = -1.0;
  __syncthreads();
  auto gamma_bar_m = [&](double th, bool glob) -> double {
    const uint64_t hb = c2d_bits(th);
    const int slot = (int)((hb ^ (hb >> 17) ^ (hb >> 31)) & (ZMEMO - 1));
#ifdef C2D_FP_PROF_MEMO
    pm_calls++;
    if (f_mth[slot] == th) pm_lds++;
#endif
    if (f_mth[slot] == th) return f_mgv[slot];
    double g = 0.0;
    glob = glob && (!P.mom || P.mt_glob);
    if (glob) {
      /* read by thread 0 and broadcast, so every thread takes the same branch */
      if (tid == 0) {
        double gm = 0.0;
        f_red[B.slot][0][0] = gb_lookup(P, th, gm) ? gm : 0.0;
      }
      __syncthreads();
      g = f_red[B.slot][0][0];
      B.slot ^= 1;
#ifdef C2D_FP_PROF_MEMO
      if (g != 0.0) pm_glob++;
#endif
    }
    if (g == 0.0) {
      g = gamma_bar_fast<BS>(B, th, P.mcd, P.mom, guard);
#ifdef C2D_FP_PROF
      if (th >= F32(0.2)) pf_mcd++;
#endif
      if (glob && tid == 0) gb_insert(P, th, g);
    }
    /* the slot is rewritten only once every thread has looked it up, and
     * read again only once the rewrite is visible to all: the memo stays
     * uniform across the block, so every thread takes the same branches */
    __syncthreads();
    if (tid == 0) {
      f_mth[slot] = th;
      f_mgv[slot] = g;
    }
    __syncthreads();
    return g;
  };
  const double vn = 8.176e-7;
  /* what does not change between sub-steps, once: the acceleration
   * dispersion disp and its Chang-Cooper midpoint bigC, the grid factor
   * Delta_g of the tridiagonal coefficients, and the pick-up injection
   * profile with its normalisation (the reference recomputes them every
   * sub-step from the same operands: the same values) */
  double Delta_g_i = 1.0, inj_prof = 0.0;
  /* and, as products and reciprocals (fast mode: a few ulp from the
   * reference's quotients): the synchrotron, acceleration and loop-350
   * factors of dgdt and hr_nt_A, 1/gamma */
  const double f_sy = 1.058e-15 * (Bf * Bf) / 8.176e-7;
  const double sy_i = own ? f_sy * (gi * gi - 1.0) : 0.0;
  const double rg_i = own ? 1.0 / gi : 0.0;
  const double base_i = own ? f_dgic[i] + gi / t_acc : 0.0;
  const double kH_i = (i <= NT - 1) ? gi / t_acc * (f_gam[i + 1] - gi) : 0.0;
  if (own) {
    f_disp[i] = gi * gi / t_acc / 2.0;
    if (P.pick_sw == 1 && i <= NT - 1) {
      const double x = gi - P.inj_gg;
      inj_prof = 1.0e2 * c2d_exp_bf(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                 (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
    }
  }
  __syncthreads();
  const double bigC_i = (i <= NT - 1) ? (f_disp[i] + f_disp[i + 1]) / 2.0 : 0.0;
  if (i <= NT - 1) f_bigC[i] = bigC_i;
  if (i >= 2 && i <= NT - 1) Delta_g_i = __builtin_sqrt(f_gnt[i] / f_gnt[i - 1]) * dgm;
  const double inj_sum0 = B.sum(inj_prof * dgp);     /* also publishes bigC */
  const double r_inj0 = rcp_nr(inj_sum0);
  /* Chang-Cooper and tridiagonal factors: smw = bigB kS; with kP = 1/(Delta_g
   * D_gplus), kM = 1/(Delta_g D_gminus): tc = -d_t em_i kP, ta = -d_t bigW_{i-1}
   * bigC_{i-1} kM, tb = 1 + d_t (bigW_i bigC_i kP + em_{i-1} kM) + d_t/t_esc */
  double kS = 0.0, kP = 0.0, kM = 0.0, kC = 0.0, kA = 0.0;
  if (i <= NT - 1) kS = ((i == 1) ? f_gnt[2] - f_gnt[1] : dgp) / bigC_i;
  if (i >= 2 && i <= NT - 1) {
    kP = 1.0 / (Delta_g_i * dgp);
    kM = 1.0 / (Delta_g_i * dgm);
    kC = bigC_i * kP;
    kA = f_bigC[i - 1] * kM;
  }
  for (;;) {
    /* label 200 (:577) */
#if C2D_FPF_MT_PF
    if (B.wave == 0 && Th_e >= F32(0.2)) mt_prefetch(P.mom, Th_e, B.lane);
#endif
    PF_BEGIN();
    const double g_av0 = (fp_steps == 0) ? gamma_bar_m(Th_e, true) : g_av_next;
    PF_END(pf_gb);
    double g_av = g_av0;
    PS_BEGIN();
    const double hr_th_c = (fp_steps == 0)
        ? B.sum((i <= NT - 1) ? -(vn * f_dgic[i] * f_fold[i] * dgp * volume * n_lept) : 0.0)
        : hr_th_c_next;
    if (fp_steps > MAX_FP_STEPS) {
      if (tid == 0) atomicOr(P.err, FPERR_STEPS);
      return;
    }
    /* this chain runs once per sub-step on every thread, ahead of everything
     * else: its quotients through rcp_nr and exp(-y) through exp_nonpos
     * (fast mode: a few ulp from the reference's IEEE operations) */
    const double gamma_R = 2.1e-3 * __builtin_sqrt(n_lept) * rcp_nr_safe(Bf * __builtin_sqrt(g_av));
    const double sT = Th_e + Th_p;
    const double h_T = F32(.79788) * (2. * (sT * sT) + 2.0 * sT + 1.0) *
                       rcp_nr(sT * __builtin_sqrt(sT) * (1.0 + 1.875 * Th_e + .8203 * (Th_e * Th_e)));
    const double hr_th_Coul = f_th * 1.7386e-26 * n_p * LNL * h_T * (Tp_flare - Te_new);
    const double yR = gamma_R * rcp_nr(g_av);
    const double hr_th_sy = (yR < 100.0) ? -Eloss_sy * exp_nonpos(-yR) * r_dt : 0.0;
    double hr_th_A = tlev * hr_th_Coul;
    if (hr_th_A < 1.0e-20) hr_th_A = 1.0e-20;
    const double hr_th_total = hr_th_sy + hr_th_c + hr_th_A;
    const double dT_total = 6.25e8 * P.dt * hr_th_total * r_fth;
    double f_t_implicit = P.df_implicit * Te_new * rcp_nr_safe(fabs(dT_total));
    if (f_t_implicit > P.df_T) f_t_implicit = P.df_T;
    if (P.probe) {   /* cost probe: the sub-steps this first one implies (:1142, :1473) */
      if (tid == 0) {
        zo[FO_DIAG + C2D_FP_STEPS] = 1.0 / f_t_implicit;
        zo[FO_DIAG + C2D_FP_SKIPPED] = 0.0;
      }
      return;
    }
    const double g_thr = 1.0 + 4.0 * Th_e;
    /* dgdt, disp (:880-889, :1035-1049) */
    if (own) {
      const double y = gamma_R * rg_i;
      const double dg_sy = (y < 100.0) ? -(sy_i * exp_nonpos(-y)) : -1.0e-50;
      f_dgdt[i] = dg_sy + base_i;
    }
    /* loop 350 sums */
    double hr_nt_A = 0.0, hr_st_A = 0.0;
    if (i <= NT - 1) {
      const double v = kH_i * f_fold[i];
      hr_nt_A = v;
      hr_st_A = gi > g_thr ? v : 0.0;
    }
    B.sum2(hr_nt_A, hr_st_A);                          /* also publishes dgdt */
    PS_END(pf_sa);
    PS_BEGIN();
    hr_st_A = hr_st_A * vn * n_lept * volume;
    hr_nt_A = hr_nt_A * vn * n_lept * volume;
    const double heat_total = hr_th_Coul + hr_nt_A;
    e_old = e_old + heat_total * f_t_implicit * P.dt;
    if (fp_steps == 0) {
      hr = hr + heat_total;
      hr_st = hr_st + hr_st_A;
    }
    double d_t = f_t_implicit * P.dt;                  /* :1142-1146 */
    if (d_t > (P.dt - t_fp)) d_t = 1.00001 * (P.dt - t_fp);
    if (P.pair_sw == 1 && i <= NT - 1) {               /* H6: inert positrons, loop 460 clip */
      double v = f_fold[i] + 0.0 / ne;
      if (v < 1.0e-50) v = 0.0;
      f_fold[i] = v;
    }
    n_positron = 0.0;                                  /* :1164-1167 / :1218 */
    ne = n_p + n_positron;
    /* injection (:1226-1306) */
    double n_inject = 0.0;
    if (P.pick_sw == 1) {
      /* sum_i (inj_rho prof_i / inj_sum) dg_i is inj_rho to rounding: the
       * fast mode takes it so, without the second block sum */
      const double inj_rho = P.pick_rate * d_t;
      if (i <= NT - 1) f_fold[i] = f_fold[i] + inj_rho * inj_prof * (r_inj0 * rcp_nr(ne));
      n_inject = n_inject + inj_rho;
    }
    if (P.inj_switch != 0) {
      const double tt = P.time + t_fp - P.inj_t;
      if (tt > dz / P.inj_v * (double)(j - 1) && tt < dz / P.inj_v * (double)j && k <= P.nr) {
        double v = 0.0;
        if (i <= NT - 1) {
          if (P.inj_dis == 1) {
            const double x = gi - P.inj_gg;
            v = 1.0e2 * c2d_exp_bf(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
          } else {
            const double inj_g2var = P.inj_g2 * c2d_pow(10.0, (P.time + t_fp - P.inj_t) * P.inj_v / zmax);
            if (gi > P.inj_g1) {
              const double inj_y = (P.g2var_switch == 1) ? gi / inj_g2var : gi / P.inj_g2;
              v = (inj_y < 1.0e2) ? 1.0e2 / (c2d_pow(gi, P.inj_p) * c2d_exp_bf(inj_y)) : 0.0;
            }
          }
        }
        double isum = v * dgp, inj_E = v * dgp * gi;
        B.sum2(isum, inj_E);
        inj_E = inj_E / isum;
        const double inj_rate = P.inj_L / 8.186e-7 / inj_E / (PI_REF * (rmax * rmax) * dz);
        const double rho = inj_rate * d_t;
        double nv = 0.0;
        if (i <= NT - 1) {
          const double w = rho * v / isum;
          f_fold[i] = f_fold[i] + w / ne;
          nv = w * dgp;
        }
        n_inject = n_inject + B.sum(nv);
      }
    }
    ne = ne + n_inject;
    n_p = n_p + n_inject;
    n_lept = n_lept + n_inject;
    const double f_esc = t_esc * rcp_nr(t_esc + d_t);  /* escape (:1309-1313) */
    ne = ne * f_esc;
    n_p = n_p * f_esc;
    n_lept = n_lept * f_esc;
    const double dte = d_t * r_tesc;
    /* Chang-Cooper coefficients (:1363-1390) */
    if (i <= NT - 1) {
      const double bigB = (i == 1) ? -(f_dgdt[1] + f_dgdt[2]) : -(f_dgdt[i] + f_dgdt[i + 1]) * 0.5;
      const double smw = bigB * kS;
      /* IEEE divisions kept: exp(smw) - 1 rounds to 0 for |smw| below an ulp, where
       * x / 0 = inf as in the reference but rcp_nr(0) is NaN */
      f_bigW[i] = smw / (c2d_exp_bf(smw) - 1.0);
      f_em[i] = bigC_i * smw / (1.0 - c2d_exp_bf(-smw));
    }
    __syncthreads();
    double ta = 0.0, tb = 1.0, tc = 0.0;
    if (i >= 2 && i <= NT - 1) {
      tc = -(d_t * (f_em[i] * kP));
      tb = 1.0 + d_t * (f_bigW[i] * kC + f_em[i - 1] * kM) + dte;
      ta = -(d_t * (f_bigW[i - 1] * kA));
    }
    PS_END(pf_sb);
    /* tridag (:2476-2518) by cyclic reduction; clip u(2..num_nt) (:2512) */
    PF_BEGIN();
    /* C2D_FPF_SPIKE=0: plain PCR with a barrier per level (measured equal, r04s) */
#ifndef C2D_FPF_SPIKE
#define C2D_FPF_SPIKE 1
#endif
#if C2D_FPF_SPIKE
    double u = spike_solve<BS>(B, ta, tb, tc, own ? f_fold[i] : 0.0);
#else
    double u = pcr_solve<BS>(B, ta, tb, tc, own ? f_fold[i] : 0.0);
#endif
    PF_END(pf_tri);
    PS_BEGIN();
    if (i >= 2 && u < 0.0) u = 0.0;
    if (i == NT || i == 1) u = 0.0;
    /* Pnt prefix, sum_p, sum_E (:1415-1419) */
    double tot = 0.0, sE = (i <= NT - 1) ? dgp * gi * u : 0.0;
    const double pv = (i <= NT - 1) ? dgp * u : 0.0;
    const double pref = B.scan_sum(pv, tot, sE);      /* one barrier for both */
    sum_p = tot;
    if (i <= NT - 1) f_Pnt[i] = pref;
    const double r_sum = rcp_nr(sum_p);
    sum_E = sE * r_sum;
    t_fp = t_fp + d_t;
    fp_steps = fp_steps + 1;
    const double fn = own ? u * r_sum : 0.0;
    if (own) {
      f_fnew[i] = fn;
      f_fold[i] = fn;
    }
    /* gbar and the next sub-step's hr_th_c (:1440, label 200) */
    double gbar = (i <= NT - 1) ? gi * fn * dgp : 0.0;
    hr_th_c_next = (i <= NT - 1) ? -(vn * f_dgic[i] * fn * dgp * volume * n_lept) : 0.0;
    B.sum2(gbar, hr_th_c_next);
    PS_END(pf_sc);
    /* new temperature (:1440-1468) */
    double The_new = Th_e;
    PF_BEGIN();
    /* one loop for both directions: gamma_bar's code is inlined once here */
    const bool up = gbar > g_av;
    while (up ? gbar > g_av : gbar < g_av) {
      The_new = up ? The_new * F32(1.005) : The_new / F32(1.005);
      g_av = gamma_bar_m(The_new, true);
      if (!up && The_new < 1.0e-2) break;
      if (guard > GUARD_MAX) break;
    }
    PF_END(pf_gb);
    if (guard > GUARD_MAX) {
      if (tid == 0) atomicOr(P.err, FPERR_GUARD);
      return;
    }
    Te_new = 5.11e2 * The_new;
    Th_e = The_new;
    g_av_next = g_av;
    if (!(t_fp < P.dt)) break;                         /* :1473 */
  }
  __syncthreads();

  /* outputs (:1481-1500) */
  const double fo = own ? f_fnew[i] : 0.0;
  E_el = B.sum((i >= 2 && own) ? fo * gi * dgm : 0.0);
  E_pos = 0.0;
  E_el = E_el * ne * 8.176e-7 * volume;
  e_new = e_new + E_el + E_pos;
  if (own) {
    P.f_out[(size_t)cell * NT + i - 1] = fo;
    P.P_out[(size_t)cell * NT + i - 1] = f_Pnt[i] / sum_p;
  }
  /* nonthermal parameters (:1654-1736) */
  int lo = (own && i >= 5 && i <= NT - 5 && fo > 1.0e-10) ? i : INT_MAX;
  int hi = (own && i >= 5 && i <= NT - 5 && fo > 1.0e-15) ? i : INT_MIN;
  B.minmax(lo, hi);
  const int i_nt = lo == INT_MAX ? NT - 4 : lo;
  const int i_mx = hi == INT_MIN ? 4 : hi;
  const double gmin = f_gam[i_nt];
  const double gmax = f_gam[i_mx];
  const double dfn = (i <= NT - 1) ? (f_gam[i + 1] - gi) * fo : 0.0;
  double sum_th = (i <= i_nt - 1) ? dfn : 0.0, sum_nt = (i >= i_nt && i <= NT - 1) ? dfn : 0.0;
  B.sum2(sum_th, sum_nt);
  double amxwl = sum_th / (sum_nt + sum_th);
  double p_nth = zin[FZ_PNTH];
  if (amxwl > 9.999e-1) {
    amxwl = 1.0;
  } else {
    p_nth = F32(0.1);
    double sum_g = 1.0e50, sumg_old;
    /* first bin with gamma/gmax >= 100 ends the fit sum (:1707-1717) */
    int e0 = (i >= i_nt && i <= NT - 2 && !(gi / gmax < 100.0)) ? i : INT_MAX, e1 = INT_MIN;
    B.minmax(e0, e1);
    const int i_end = e0 == INT_MAX ? NT - 1 : e0;
    for (;;) {
      sumg_old = sum_g;
      const double p_1 = 1.0 - p_nth;
      double N_nt;
      if (fabs(p_1) > 1.0e-4)
        N_nt = (1. - amxwl) * p_1 / (c2d_pow(gmax, p_1) - c2d_pow(gmin, p_1));
      else
        N_nt = (1.0 - amxwl) / c2d_log(gmax / gmin);
      double v1 = 0.0, v2 = 0.0;
      if (i >= i_nt && i < i_end) {
        const double f_pl = N_nt / (c2d_pow(gi, p_nth) * c2d_exp_bf(gi / gmax));
        v1 = f_pl * gi * dgp;
        v2 = f_pl * dgp;
      }
      B.sum2(v1, v2);
      sum_g = v1 / v2;
      sum_g = fabs(sum_g - sum_E);
      if (sum_g < sumg_old && p_nth < 10.) {
        p_nth = p_nth + 0.5e-1;
        continue;
      }
      break;
    }
  }
  if (tid == 0) {
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
    zo[FO_DIAG + 3] = (double)pf_mcd;
    zo[FO_DIAG + 4] = (double)f_pf[0];
    zo[FO_DIAG + 6] = (double)f_pf[1];
    zo[FO_DIAG + 7] = (double)f_pf[2];
#endif
#ifdef C2D_FP_PROF_MCD
    zo[FO_DIAG + 7] = (double)f_pf[3];
#endif
#ifdef C2D_FP_PROF_MEMO
    zo[FO_DIAG + 4] = (double)pm_calls;
    zo[FO_DIAG + 6] = (double)pm_lds;
    zo[FO_DIAG + 7] = (double)pm_glob;
#endif
#ifdef C2D_FP_PROF_SEC
    zo[FO_DIAG + 4] = (double)pf_sa;
    zo[FO_DIAG + 6] = (double)pf_sb;
    zo[FO_DIAG + 7] = (double)pf_sc;
#endif
  }
}

__shared__ int f_zone;
/* workgroups per CU the register budget is sized for (C2D_FPF_MINB 2: <= 256
 * VGPRs, so two zones share a CU) */
#ifndef C2D_FPF_MINB
#define C2D_FPF_MINB 1
#endif
template <int BS>
__global__ void __launch_bounds__(BS, C2D_FPF_MINB) c2d_fp_fast_kernel(const FpParams* __restrict__ Pp) {
  const FpParams& P = *Pp;
  Blk<BS> B;
  B.tid = threadIdx.x;
  B.lane = B.tid & (FPB - 1);
  B.wave = B.tid / FPB;
  if (B.tid == 0) {
    f_eg[0] = c2d_exp_bf(gammln(5.0e-1 + 2.0));
    for (int j = 0; j < 64; j++) f_e64[j] = c_exp2_64[j];
    f_eg[1] = c2d_exp_bf(gammln(5.0e-1 + 3.0));
    f_eg[2] = f_eg[0] / f_eg[1];
  }
  /* one zone after another from the queue: a zone's time is its sub-step
   * count x one latency chain, and the costliest zones come first, each on a
   * CU of its own; the cheap ones fill in behind the first to finish */
  for (;;) {
    if (B.tid == 0) {
#ifdef C2D_FP_PROF
      f_pf[0] = f_pf[1] = f_pf[2] = f_pf[3] = 0;
#endif
      f_zone = atomicAdd(P.zq, 1);
    }
    __syncthreads();
    const int q = f_zone;
    __syncthreads();                       /* f_zone is rewritten next round */
    if (q >= P.ncell) break;
    fp_zone_fast<BS>(P, B, P.zorder ? P.zorder[q] : q);
    __syncthreads();
  }
}

}  // namespace
}  // namespace c2d

/* threads per zone (one workgroup per zone; C2D_FPF_BS, 256 or 512): 4 waves,
 * one per SIMD of the zone's CU, or 8, two per SIMD, so one wave's
 * dependent f64 chains (McDonald's exp) issue under the other's */
#ifndef C2D_FPF_BS
#define C2D_FPF_BS 256
#endif
extern "C" int c2d_fp_fast_block(int, int) { return C2D_FPF_BS; }

/* dP: the parameters in device memory (uploaded by the caller on `stream`) */
extern "C" int c2d_launch_fp_fast(const c2d::FpParams* dP, int ncell, int block, int grid, hipStream_t stream) {
  if (ncell <= 0) return 0;
  if (block != C2D_FPF_BS || grid <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(c2d::c2d_fp_fast_kernel<C2D_FPF_BS>, dim3(grid < ncell ? grid : ncell), dim3(C2D_FPF_BS), 0,
                     stream, dP);
  return (int)hipGetLastError();
}

/* the McDonald moment table for the fast kernel (C2D_FPF_MT_N x C2D_FPF_MT_W
 * doubles at `mom`), from the abscissa table `mcd`; once per context */
extern "C" int c2d_fp_mom_build(const double* mcd, double* mom, hipStream_t stream) {
  hipLaunchKernelGGL(c2d::c2d_fp_mom_kernel, dim3((C2D_FPF_MT_N + 63) / 64), dim3(64), 0, stream, mcd, mom);
  return (int)hipGetLastError();
}

namespace c2d {
namespace {
/* selftest: K2, K3 at z from the table and from the series (one block per z),
 * with the shader cycles each took */
__global__ void __launch_bounds__(256) c2d_fp_mtab_test_kernel(const double* __restrict__ tab,
                                                               const double* __restrict__ mom,
                                                               const double* __restrict__ zs, double* out) {
  Blk<256> B;
  B.tid = threadIdx.x;
  B.lane = B.tid & (FPB - 1);
  B.wave = B.tid / FPB;
  if (B.tid < 64) f_e64[B.tid] = c_exp2_64[B.tid];
  if (B.tid == 0) {
    f_eg[0] = c2d_exp_bf(gammln(5.0e-1 + 2.0));
    f_eg[1] = c2d_exp_bf(gammln(5.0e-1 + 3.0));
    f_eg[2] = f_eg[0] / f_eg[1];
  }
  __syncthreads();
  const double z = zs[blockIdx.x];
  double S2 = 0.0, S3 = 0.0, K2t = 0.0, K3t = 0.0, K2s, K3s;
  long long guard = 0;
  /* timed: what gamma_bar_fast does with the table (from z) */
  long long tmr[3] = {0, 0, 0};
  const long long t0 = clock64();
  const bool ok = mcd_mtab(mom, tab, z, S2, S3, tmr);
  const double gq = ok ? (5.0e-1 * z) * (S3 * rcp_nr(S2)) * f_eg[2] - rcp_nr(z) : 0.0;
  const long long t1 = clock64();
  if (ok) mcdonald23_finish_c(z, S2, S3, f_eg[0], f_eg[1], K2t, K3t);
  __syncthreads();
  const long long t2 = clock64();
  mcdonald23_fast<256>(B, z, tab, K2s, K3s, guard);
  const long long t3 = clock64();
  if (B.tid == 0) {
    double* o = out + (size_t)blockIdx.x * 8;
    o[0] = K2t; o[1] = K3t; o[2] = K2s; o[3] = K3s; o[4] = ok ? 1.0 : 0.0;
    o[5] = (double)(t1 - t0); o[6] = (double)(t3 - t2); o[7] = gq;
#ifdef C2D_MTAB_TIMERS
    o[0] = (double)(tmr[0] - t0); o[1] = (double)(tmr[1] - tmr[0]); o[2] = (double)(tmr[2] - tmr[1]);
    o[3] = (double)(t1 - tmr[2]);
#endif
  }
}
}  // namespace
}  // namespace c2d

extern "C" int c2d_fp_mtab_test(const double* mcd, const double* mom, const double* z, double* out, int n,
                                hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(c2d::c2d_fp_mtab_test_kernel, dim3((unsigned)n), dim3(256), 0, stream, mcd, mom, z, out);
  return (int)hipGetLastError();
}
