/*
 * c2d_wave.hpp — wavefront-level helpers shared by the FP kernel (fp.hip)
 * and the emission/absorption kernel (vem.hip): in-order sums across a
 * wave through readlane (the reference's serial rounding without LDS on the
 * dependency chain) and McDonald's K2/K3 series 64 terms per pass.
 * Call from whole, converged 64-lane waves.
 */
#ifndef C2D_WAVE_HPP
#define C2D_WAVE_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "c2d_device.hpp"
#include "c2d_math.h"

namespace c2d {
namespace wave {

constexpr int FPB = 64;                        /* lanes of a wavefront */
constexpr long long GUARD_MAX = 1ll << 34;     /* never reached by valid input */
#ifndef F32
#define F32(x) ((double)(float)(x))
#endif

__device__ __forceinline__ double rl(double v, int m) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), m);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), m);
  return __hiloint2double(hi, lo);
}

/* acc = acc + f(i) for i = lo..hi, in this order: f is evaluated lane-parallel
 * (bin i = c0 + lane of each 64-bin chunk), the additions run in sequence on
 * wave-uniform values fetched with readlane, so the rounding is that of the
 * reference's serial loop while no LDS load sits on the dependency chain. */
template <class F>
__device__ __forceinline__ double seq_sum(double acc, int lo, int hi, int lane, F f) {
  for (int c0 = lo; c0 <= hi; c0 += FPB) {
    const int i = c0 + lane;
    const double v = (i <= hi) ? f(i) : 0.0;
    const int mn = (hi - c0 + 1) < FPB ? (hi - c0 + 1) : FPB;
    for (int m = 0; m < mn; m++) acc = acc + rl(v, m);
  }
  return acc;
}
/* two independent serial sums over the same bins, interleaved */
template <class F, class G>
__device__ __forceinline__ void seq_sum2(double& a1, double& a2, int lo, int hi, int lane, F f,
                                         G g) {
  for (int c0 = lo; c0 <= hi; c0 += FPB) {
    const int i = c0 + lane;
    const double v1 = (i <= hi) ? f(i) : 0.0;
    const double v2 = (i <= hi) ? g(i) : 0.0;
    const int mn = (hi - c0 + 1) < FPB ? (hi - c0 + 1) : FPB;
    for (int m = 0; m < mn; m++) {
      a1 = a1 + rl(v1, m);
      a2 = a2 + rl(v2, m);
    }
  }
}

/* The same in-order sums with the lane-parallel values staged through `scr`
 * (LDS, FPB doubles per value owned by this wave): every lane reads them back
 * with broadcast loads that issue ahead of the add chain, so the chain runs
 * at the adds' latency instead of a readlane's SGPR hazards (mcdonald23_from
 * below measured ~15 against ~108 cycles per term). */
__device__ __forceinline__ void wave_sync();
template <class F>
__device__ __forceinline__ double seq_sum_lds(double acc, int lo, int hi, int lane, double* scr, F f) {
  for (int c0 = lo; c0 <= hi; c0 += FPB) {
    const int i = c0 + lane;
    scr[lane] = (i <= hi) ? f(i) : 0.0;
    wave_sync();
    const int mn = (hi - c0 + 1) < FPB ? (hi - c0 + 1) : FPB;
    if (mn == FPB) {
#pragma unroll 16
      for (int m = 0; m < FPB; m++) acc = acc + scr[m];
    } else {
      for (int m = 0; m < mn; m++) acc = acc + scr[m];
    }
    wave_sync();
  }
  return acc;
}
/* two interleaved in-order sums; scr holds 2*FPB doubles */
template <class F, class G>
__device__ __forceinline__ void seq_sum2_lds(double& a1, double& a2, int lo, int hi, int lane, double* scr,
                                             F f, G g) {
  for (int c0 = lo; c0 <= hi; c0 += FPB) {
    const int i = c0 + lane;
    scr[lane] = (i <= hi) ? f(i) : 0.0;
    scr[FPB + lane] = (i <= hi) ? g(i) : 0.0;
    wave_sync();
    const int mn = (hi - c0 + 1) < FPB ? (hi - c0 + 1) : FPB;
    if (mn == FPB) {
#pragma unroll 16
      for (int m = 0; m < FPB; m++) {
        a1 = a1 + scr[m];
        a2 = a2 + scr[FPB + m];
      }
    } else {
      for (int m = 0; m < mn; m++) {
        a1 = a1 + scr[m];
        a2 = a2 + scr[FPB + m];
      }
    }
    wave_sync();
  }
}

/* gammln (volume2d.f:647-668) */
__device__ inline double gammln(double xx) {
  const double cof[6] = {76.18009172947146, -86.50532032941677, 24.01409824083091,
                         -1.231739572450155, .1208650973866179e-2, -.5395239384953e-5};
  const double stp = 2.5066282746310005;
  double x = xx, y = x, tmp = x + 5.5;
  tmp = (x + 0.5) * c2d_log(tmp) - tmp;
  double ser = 1.000000000190015;
#pragma unroll
  for (int j = 0; j < 6; j++) {
    y = y + 1.0;
    ser = ser + cof[j] / y;
  }
  return tmp + c2d_log(stp * ser / x);
}

/* McDonald (volume2d.f:598-626) for nu = 2 and 3 together, 64 series terms per
 * pass (wave-uniform call).  Both series run over the same abscissae
 * t_n = 1.001^n (by repeated multiplication), ts_n = t_n*s, and
 * (ts_n^2 - 1)^a: those depend on n only, so the first C2D_FP_MCD_N of them
 * come from a table built once on the host with the same c2d_math code
 * (c2d_fp_set_config); only exp(z*ts) depends on the argument.  Beyond the
 * table the abscissa chain is replayed per lane from the last value.  Terms
 * are added in the reference's order up to each series' own stopping term,
 * so K2 and K3 equal two sequential McDonald calls bit for bit.  The terms of
 * a pass go through `scr` (LDS, 4*FPB doubles owned by this wave): every lane
 * reads them back with broadcast loads that issue ahead of the add chain, so
 * the chain runs at the adds' latency (a readlane chain serialises on its
 * SGPR hazards: ~108 cycles per term against ~15). */
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* One term of each series at n = n0 + lane from the abscissa table. */
struct McdTerm {
  double term2, term3, tn;
  bool stop2, stop3;
};
__device__ __forceinline__ McdTerm mcd_term_tab(double z, int n, const double* __restrict__ tab) {
  const double dt = 1.001, d = dt - 1.0;
  const double* e = tab + (size_t)n * 4;
  const double t = e[0], ts = e[1], p2 = e[2], p3 = e[3];
  const double y = z * ts;
  double sd2 = 0.0, sd3 = 0.0;
  if (y < 2.25e2) {
    const double ey = c2d_exp_bf(y);
    sd2 = p2 / ey;
    sd3 = p3 / ey;
  }
  McdTerm r;
  r.term2 = d * t * sd2;
  r.term3 = d * t * sd3;
  r.tn = t * dt;
  r.stop2 = !(r.tn < 2.0 || sd2 > 1.0e-8);
  r.stop3 = !(r.tn < 2.0 || sd3 > 1.0e-8);
  return r;
}

/* Number of terms of a 64-term block that enter a running series: up to and
 * including its first stopping term (0 once the series has stopped). */
__device__ __forceinline__ int mcd_take(bool run, unsigned long long st) {
  return run ? (st ? __ffsll((long long)st) : FPB) : 0;
}

/* `scr` holds 4*FPB doubles (LDS, owned by this wave).  While both 64-term
 * blocks of a pass lie inside the abscissa table, each lane evaluates two
 * terms (n and n+64): their exp/divide chains are independent, so one
 * exposes its latency while the other issues (one wave per SIMD hides
 * nothing else).  The sums still run in n order over exactly the terms the
 * reference adds, so the result is unchanged bit for bit. */
/* The series from term n0 on (t0 = t_n0 by the reference's chain), adding
 * to sum2/sum3 while run2/run3; returns with both series stopped. */
__device__ inline void mcdonald23_from(double z, int lane, const double* __restrict__ tab, int n0,
                                       double t0, double& sum2, double& sum3, bool run2, bool run3,
                                       long long& guard, double* scr) {
  const double dt = 1.001, s = 5.0e-1 * (1.0 + dt);
  while (run2 || run3) {
    if (n0 + 2 * FPB <= C2D_FP_MCD_N) {
      const McdTerm a = mcd_term_tab(z, n0 + lane, tab);
      const McdTerm b = mcd_term_tab(z, n0 + FPB + lane, tab);
      const unsigned long long sa2 = __ballot(a.stop2), sa3 = __ballot(a.stop3);
      const unsigned long long sb2 = __ballot(b.stop2), sb3 = __ballot(b.stop3);
      const int na2 = mcd_take(run2, sa2), na3 = mcd_take(run3, sa3);
      const int nb2 = mcd_take(run2 && !sa2, sb2), nb3 = mcd_take(run3 && !sa3, sb3);
      scr[lane] = a.term2;
      scr[FPB + lane] = b.term2;
      scr[2 * FPB + lane] = a.term3;
      scr[3 * FPB + lane] = b.term3;
      wave_sync();
      const int n2 = na2 + nb2, n3 = na3 + nb3;
      if (n2 == 2 * FPB && n3 == 2 * FPB) {
#pragma unroll 16
        for (int m = 0; m < 2 * FPB; m++) {
          sum2 = sum2 + scr[m];
          sum3 = sum3 + scr[2 * FPB + m];
        }
      } else {
        for (int m = 0; m < n2; m++) sum2 = sum2 + scr[m];
        for (int m = 0; m < n3; m++) sum3 = sum3 + scr[2 * FPB + m];
      }
      wave_sync();
      if (sa2 || sb2) run2 = false;
      if (sa3 || sb3) run3 = false;
      guard += n2 > n3 ? n2 : n3;
      if (guard > GUARD_MAX) break;
      t0 = rl(b.tn, FPB - 1);
      n0 += 2 * FPB;
      continue;
    }
    /* single 64-term pass (tail of the table, then abscissae replayed per lane) */
    const double d = dt - 1.0;
    const int n = n0 + lane;
    double t, ts, p2, p3;
    if (n0 + FPB <= C2D_FP_MCD_N) {
      const double* e = tab + (size_t)n * 4;
      t = e[0]; ts = e[1]; p2 = e[2]; p3 = e[3];
    } else {
      t = t0;
      for (int m = 0; m < lane; m++) t = t * dt;
      ts = t * s;
      p2 = c2d_pow(ts * ts - 1.0, 1.5);
      p3 = c2d_pow(ts * ts - 1.0, 2.5);
    }
    const double y = z * ts;
    double sd2 = 0.0, sd3 = 0.0;
    if (y < 2.25e2) {
      const double ey = c2d_exp_bf(y);
      sd2 = p2 / ey;
      sd3 = p3 / ey;
    }
    const double term2 = d * t * sd2, term3 = d * t * sd3;
    const double tn = t * dt;
    const unsigned long long st2 = __ballot(!(tn < 2.0 || sd2 > 1.0e-8));
    const unsigned long long st3 = __ballot(!(tn < 2.0 || sd3 > 1.0e-8));
    const int n2 = mcd_take(run2, st2);
    const int n3 = mcd_take(run3, st3);
    const int nm = n2 > n3 ? n2 : n3;
    scr[lane] = term2;
    scr[FPB + lane] = term3;
    wave_sync();
    if (n2 == FPB && n3 == FPB) {
#pragma unroll 16
      for (int m = 0; m < FPB; m++) {
        sum2 = sum2 + scr[m];
        sum3 = sum3 + scr[FPB + m];
      }
    } else {
      for (int m = 0; m < n2; m++) sum2 = sum2 + scr[m];
      for (int m = 0; m < n3; m++) sum3 = sum3 + scr[FPB + m];
    }
    wave_sync();
    if (st2) run2 = false;
    if (st3) run3 = false;
    guard += nm;
    if (guard > GUARD_MAX) break;
    t0 = rl(tn, FPB - 1);
    n0 += FPB;
  }
}

/* McDonald's normalisation (volume2d.f:623-624) of the two sums */
__device__ __forceinline__ void mcdonald23_finish(double z, double sum2, double sum3, double& K2,
                                                  double& K3) {
  K2 = __builtin_sqrt(3.14159265) * c2d_pow(5.0e-1 * z, 2.0) * sum2 / c2d_exp_bf(gammln(5.0e-1 + 2.0));
  K3 = __builtin_sqrt(3.14159265) * c2d_pow(5.0e-1 * z, 3.0) * sum3 / c2d_exp_bf(gammln(5.0e-1 + 3.0));
}
/* ... with the argument-free factors exp(gammln(2.5)), exp(gammln(3.5))
 * given (the same values, computed once per launch) and c2d_pow's log of
 * 0.5 z shared by both powers (c2d_pow(x, y) = c2d_exp_bf(y * c2d_log(x))) */
__device__ __forceinline__ void mcdonald23_finish_c(double z, double sum2, double sum3, double eg2,
                                                    double eg3, double& K2, double& K3) {
  const double lz = c2d_log(5.0e-1 * z);
  K2 = __builtin_sqrt(3.14159265) * c2d_exp_bf(2.0 * lz) * sum2 / eg2;
  K3 = __builtin_sqrt(3.14159265) * c2d_exp_bf(3.0 * lz) * sum3 / eg3;
}

__device__ inline void mcdonald23_w(double z, int lane, const double* __restrict__ tab, double& K2,
                                    double& K3, long long& guard, double* scr) {
  double sum2 = 0.0, sum3 = 0.0;
  mcdonald23_from(z, lane, tab, 0, 1.0, sum2, sum3, true, true, guard, scr);
  mcdonald23_finish(z, sum2, sum3, K2, K3);
}

/* gamma_bar (volume2d.f:572-594) */
__device__ inline double gamma_bar_w(double Theta, int lane, const double* tab, long long& guard,
                                     double* scr) {
  double g;
  if (Theta < F32(0.2)) {
    g = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) +
         F32(3.384) * (Theta * Theta * Theta)) /
            (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
        Theta;
  } else {
    double K2, K3;
    mcdonald23_w(1.0 / Theta, lane, tab, K2, K3, guard, scr);
    g = K3 / K2 - Theta;
  }
  if (g < 1.0) g = 1.0;
  return g;
}


}  // namespace wave
}  // namespace c2d

#endif
