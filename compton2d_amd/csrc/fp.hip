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

}  // namespace

/* One zone per workgroup (= one wave).  Line numbers: src/update2d.f. */
__global__ void __launch_bounds__(FPB) c2d_fp_kernel(const FpParams P) {
  __shared__ double s_gnt[NT + 2], s_gam[NT + 2], s_fold[NT + 2], s_fnew[NT + 2];
  __shared__ double s_dgic[NT + 2], s_dgdt[NT + 2], s_disp[NT + 2];
  __shared__ double s_a[NT + 2], s_b[NT + 2], s_c[NT + 2];
  __shared__ double s_mcd[4 * FPB];   /* McDonald term exchange (c2d_wave.hpp) */
  __shared__ double s_smw[NT + 2], s_bigW[NT + 2], s_bigC[NT + 2], s_em[NT + 2], s_inj[NT + 2];
  __shared__ double s_Pnt[NT + 2], s_nf[NPH];

  const int cell = blockIdx.x;
  const int lane = threadIdx.x;
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
  __syncthreads();

  /* E_el, normalisation (:482-509) */
  double E_el = 0.0, E_pos = 0.0;
  E_el = seq_sum(E_el, 2, NT, lane,
                 [&](int i) { return (s_gnt[i] - s_gnt[i - 1]) * s_gam[i] * s_fold[i]; });
  E_el = E_el * ne * 8.176e-7 * volume;
  double e_old = 0.0 + E_el + E_pos + zin[FZ_ECOLD];
  double e_new = 0.0 + ecens;
  double sum_p = seq_sum(0., 1, NT - 1, lane,
                         [&](int i) { return (s_gnt[i + 1] - s_gnt[i]) * s_fold[i]; });
  __syncthreads();
  for (int i = lane + 1; i <= NT; i += FPB) s_fold[i] = s_fold[i] / sum_p;
  __syncthreads();
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
    tl_flare = (y < 1.0e2) ? P.flare_amp / c2d_exp(y) : 0.0;
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
  __syncthreads();

  double hr = 0.0, hr_st = 0.0, sum_E = 0.0, t_fp = 0.0;
  int fp_steps = 0;
  /* gamma_bar is a pure function and label 200 evaluates it at the Th_e the
   * previous sub-step's temperature search ended on, whose value that search
   * computed last: reuse it (one McDonald pair per sub-step saved, exact) */
  double g_av_next = 0.0;
  /* The temperature search steps Theta by x1.005 or /1.005 from the last
   * sub-step's value, so successive sub-steps keep re-evaluating the same few
   * arguments (T oscillating across the crossing). gamma_bar is a pure
   * function of Theta: a 4-entry memo keyed on the exact bits returns the
   * value it would recompute (bit-identical), skipping its McDonald pair. */
  double memo_th[4] = {-1.0, -1.0, -1.0, -1.0}, memo_g[4] = {0.0, 0.0, 0.0, 0.0};
  int memo_next = 0;
  auto gamma_bar_m = [&](double th) -> double {
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (memo_th[q] == th) return memo_g[q];
    const double g = gamma_bar_w(th, lane, P.mcd, guard, s_mcd);
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (q == memo_next) { memo_th[q] = th; memo_g[q] = g; }
    memo_next = (memo_next + 1) & 3;
    return g;
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
    const double hr_th_c = seq_sum(0.0, 1, NT - 1, lane, [&](int i) {
      return -(8.176e-7 * s_dgic[i] * s_fold[i] * (s_gnt[i + 1] - s_gnt[i]) * volume * n_lept);
    });
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
    const double hr_th_sy = (yR < 100.0) ? -Eloss_sy / (P.dt * c2d_exp(yR)) : 0.0;
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
      const double dg_sy = (y < 100.0) ? -(f_sy * (gi * gi - 1.0) / c2d_exp(y)) : -1.0e-50;
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
      const int mn = (NT - c0) < FPB ? (NT - c0) : FPB;
      for (int m = 0; m < mn; m++) {
        const double x = rl(v, m);
        hr_nt_A = hr_nt_A + x;
        if ((stm >> m) & 1ull) hr_st_A = hr_st_A + x;
      }
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
      __syncthreads();
      for (int i = lane + 1; i <= NT - 1; i += FPB) {
        double v = s_fold[i] + 0.0 / ne;
        if (v < 1.0e-50) v = 0.0;
        s_fold[i] = v;
      }
      __syncthreads();
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
        s_inj[i] = 1.0e2 * c2d_exp(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                   (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
      }
      __syncthreads();
      inj_sum = seq_sum(0.0, 1, NT - 1, lane,
                        [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
      inj_rho = P.pick_rate * d_t;
      inj_any = true;
    }
    if (inj_any) {
      __syncthreads();
      for (int i = lane + 1; i <= NT - 1; i += FPB) {
        const double v = inj_rho * s_inj[i] / inj_sum;
        s_inj[i] = v;
        s_fold[i] = s_fold[i] + v / ne;
      }
      __syncthreads();
      n_inject = seq_sum(n_inject, 1, NT - 1, lane,
                         [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
    }
    if (P.inj_switch != 0) {
      const double tt = P.time + t_fp - P.inj_t;
      if (tt > dz / P.inj_v * (double)(j - 1) && tt < dz / P.inj_v * (double)j && k <= P.nr) {
        __syncthreads();
        for (int i = lane + 1; i <= NT - 1; i += FPB) {
          const double gi = s_gam[i];
          double v;
          if (P.inj_dis == 1) {
            const double x = gi - P.inj_gg;
            v = 1.0e2 * c2d_exp(-((x * x) / 2.0 / (P.inj_sigma * P.inj_sigma))) /
                (P.inj_sigma * __builtin_sqrt(2.0 * PI_REF));
          } else {
            const double inj_g2var =
                P.inj_g2 * c2d_pow(10.0, (P.time + t_fp - P.inj_t) * P.inj_v / zmax);
            if (gi > P.inj_g1) {
              const double inj_y = (P.g2var_switch == 1) ? gi / inj_g2var : gi / P.inj_g2;
              v = (inj_y < 1.0e2) ? 1.0e2 / (c2d_pow(gi, P.inj_p) * c2d_exp(inj_y)) : 0.0;
            } else {
              v = 0.0;
            }
          }
          s_inj[i] = v;
        }
        __syncthreads();
        double isum = 0.0, inj_E = 0.0;
        seq_sum2(isum, inj_E, 1, NT - 1, lane,
                 [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); },
                 [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]) * s_gam[i]; });
        inj_E = inj_E / isum;
        const double inj_rate = P.inj_L / 8.186e-7 / inj_E / (PI_REF * (rmax * rmax) * dz);
        const double rho = inj_rate * d_t;
        __syncthreads();
        for (int i = lane + 1; i <= NT - 1; i += FPB) {
          const double v = rho * s_inj[i] / isum;
          s_inj[i] = v;
          s_fold[i] = s_fold[i] + v / ne;
        }
        __syncthreads();
        n_inject = seq_sum(n_inject, 1, NT - 1, lane,
                           [&](int i) { return s_inj[i] * (s_gnt[i + 1] - s_gnt[i]); });
      }
    }
    ne = ne + n_inject;
    n_p = n_p + n_inject;
    n_lept = n_lept + n_inject;
    ne = ne * t_esc / (t_esc + d_t);                  /* escape (:1309-1313) */
    n_p = n_p * t_esc / (t_esc + d_t);
    n_lept = n_lept * t_esc / (t_esc + d_t);
    __syncthreads();
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
      s_bigW[i] = smw / (c2d_exp(smw) - 1.0);
      s_em[i] = bigC * smw / (1.0 - c2d_exp(-smw));   /* bigC*smw/(1-exp(-smw)) */
      s_bigC[i] = bigC;
    }
    __syncthreads();
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
    __syncthreads();
    PF_BEGIN();
    /* tridag (:2476-2518): the recurrences run in the reference order on
     * wave-uniform values (readlane) with each 64-bin chunk's operands staged
     * in registers; gam is kept in s_smw */
    {
      double bet = s_b[1];
      double u = s_fold[1] / bet;
      bool zero = false;
      if (lane == 0) s_fnew[1] = u;
      for (int c0 = 2; c0 <= NT && !zero; c0 += FPB) {
        const int i = c0 + lane;
        const bool in = i <= NT;
        const double av = in ? s_a[i] : 0.0, bv = in ? s_b[i] : 0.0;
        const double cv = in ? s_c[i - 1] : 0.0, rv = in ? s_fold[i] : 0.0;
        double gmine = 0.0, umine = 0.0;
        const int mn = (NT - c0 + 1) < FPB ? (NT - c0 + 1) : FPB;
        for (int m = 0; m < mn; m++) {
          const double am = rl(av, m);
          const double gam = rl(cv, m) / bet;
          bet = rl(bv, m) - am * gam;
          if (fabs(bet) <= 1.0e-100) {
            zero = true;
            break;
          }
          u = (rl(rv, m) - am * u) / bet;
          if (lane == m) {
            gmine = gam;
            umine = u;
          }
        }
        if (!zero && in) {
          s_smw[i] = gmine;
          s_fnew[i] = umine;
        }
      }
      __syncthreads();
      if (zero) {
        for (int i = lane + 1; i <= NT; i += FPB) s_fnew[i] = 0.0;
      } else {
        /* back substitution on the unclipped values, then the reference's
         * clipping of u(2..num_nt) (each u(i+1) is clipped after u(i) used it) */
        double up = s_fnew[NT];
        for (int c1 = NT - 1; c1 >= 1; c1 -= FPB) {
          const int i = c1 - lane;
          const bool in = i >= 1;
          const double fv = in ? s_fnew[i] : 0.0, gv = in ? s_smw[i + 1] : 0.0;
          double mine = 0.0;
          const int mn = c1 < FPB ? c1 : FPB;
          for (int m = 0; m < mn; m++) {
            up = rl(fv, m) - rl(gv, m) * up;
            if (lane == m) mine = up;
          }
          if (in) s_fnew[i] = mine;
        }
        __syncthreads();
        for (int i = lane + 2; i <= NT; i += FPB)
          if (s_fnew[i] < 0.0) s_fnew[i] = 0.0;
      }
      __syncthreads();
    }
    PF_END(pf_tri);
    if (lane == 0) {
      s_fnew[NT] = 0.0;
      s_fnew[1] = 0.0;
    }
    __syncthreads();
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
      double mine = 0.0;
      const int mn = (NT - c0) < FPB ? (NT - c0) : FPB;
      for (int m = 0; m < mn; m++) {
        sum_p = sum_p + rl(av, m);
        sE = sE + rl(bv, m);
        if (lane == m) mine = sum_p;
      }
      if (i <= NT - 1) s_Pnt[i] = mine;
    }
    sum_E = sE / sum_p;
    t_fp = t_fp + d_t;
    fp_steps = fp_steps + 1;
    __syncthreads();
    for (int i = lane + 1; i <= NT; i += FPB) {
      const double v = s_fnew[i] / sum_p;
      s_fnew[i] = v;
      s_fold[i] = v;
    }
    __syncthreads();
    /* new temperature (:1440-1468) */
    const double gbar = seq_sum(0.0, 1, NT - 1, lane, [&](int i) {
      return s_gam[i] * s_fnew[i] * (s_gnt[i + 1] - s_gnt[i]);
    });
    double The_new = Th_e;
    PF_BEGIN();
    if (gbar > g_av) {
      while (gbar > g_av) {
        The_new = The_new * F32(1.005);
#ifdef C2D_FP_PROF
        pf_calls++;
#endif
        g_av = gamma_bar_m(The_new);
        if (guard > GUARD_MAX) break;
      }
    } else {
      while (gbar < g_av) {
        The_new = The_new / F32(1.005);
#ifdef C2D_FP_PROF
        pf_calls++;
#endif
        g_av = gamma_bar_m(The_new);
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
  E_el = seq_sum(E_el, 2, NT, lane,
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
  const double sum_th = seq_sum(0.0, 1, i_nt - 1, lane, dfn);
  const double sum_nt = seq_sum(0.0, i_nt, NT - 1, lane, dfn);
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
          const double f_pl = N_nt / (c2d_pow(s_gam[q], p_nth) * c2d_exp(s_gam[q] / gmax));
          v1 = f_pl * s_gam[q] * (s_gnt[q + 1] - s_gnt[q]);
          v2 = f_pl * (s_gnt[q + 1] - s_gnt[q]);
        }
        const int mn = (i_end - c0) < FPB ? (i_end - c0) : FPB;
        for (int m = 0; m < mn; m++) {
          sum_g = sum_g + rl(v1, m);
          sum_gg = sum_gg + rl(v2, m);
        }
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

extern "C" int c2d_launch_fp(const c2d::FpParams* P, int ncell, hipStream_t stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(c2d::c2d_fp_kernel, dim3(ncell), dim3(64), 0, stream, *P);
  return (int)hipGetLastError();
}
