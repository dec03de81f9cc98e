/*
 * oracle/c2d_fp_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Fokker-Planck electron update
 * (bbw7561135/Compton2d, src/ snapshot): the parity checker for the GPU
 * solver (compton2d_amd/csrc/fp.hip).  Only tests/ and the bench's CPU
 * baseline load it; the product path never does.
 *
 *   update (master part)            src/update2d.f:138-277
 *   photon_fill (dT_max only)       src/update2d.f:1792-1913
 *   FP_calc                         src/update2d.f:337-1739
 *   tridag                          src/update2d.f:2476-2518
 *   gamma_bar, McDonald, GammaF, gammln   src/volume2d.f:572-668
 *
 * FP_calc also computes quantities that never reach its outputs: the
 * Coulomb/Moeller rates dg_cp, dg_ce, disp_cp, disp_ce with the te_mo
 * iteration and the rate-file cache that exist only for them
 * (:674-1022, hazard H7), dg_br, the Landau-damped dg_A/disp_A of loop 300
 * (overwritten unconditionally at :1036-1037), fcorr_turb and fcorr_coul.
 * The solve sees dgdt = dg_sy + dg_ic + dg_A and disp = disp_A only
 * (:1048-1049), and the energy bookkeeping sees hr_th_Coul and hr_nt_A
 * (:1034, :1079), so those branches are not restated: every output is
 * unchanged.
 *
 * Hazard H10: dg_ic(num_nt) is never assigned (loop :568-574 stops at
 * num_nt-1) yet dgdt(num_nt) enters b_i(num_nt-1) through smw(num_nt-1)
 * (:1375-1386).  It is taken as 0, here and on the GPU.
 * pair_switch = 1 is restated for the MPI reference's inert pairs (H6:
 * n_pos, dn_pp and f_pair stay 0): pa_calc's rates are then -0/0, trid_p
 * solves for npos = 0, and the only trace on the electrons is loop 460's
 * f_old clip below 1e-50 (:1187-1217).  f_pair != 0 is rejected.
 *
 * Built twice with c2d_oracle.c: glibc libm (liboracle_ref: parity with the
 * Fortran FP_calc) and c2d_math.h (liboracle_det: parity with the GPU).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/compton2d.h"

#ifdef C2O_DETMATH
#include "../compton2d_amd/csrc/c2d_math.h"
#define LOG c2d_log
#define EXP c2d_exp
#define POW c2d_pow
#else
#include <math.h>
#define LOG log
#define EXP exp
#define POW pow
#endif
#define SQRT __builtin_sqrt
#define FABS __builtin_fabs
#define F32(x) ((double)(float)(x))

#define NT C2D_NUM_NT
#define NPH C2D_NPHFIELD

static const double PI_REF = 3.1415926536;     /* general.pa:24 */
static const double C_LIGHT = 2.9979245620e10; /* general.pa:25 */
static const double LNL = 20.0;                /* update2d.f:143 / :285 */
static const double TEMP_MIN = 5.0, TEMP_MAX = 1.0e3;   /* update2d.f:17-18 */
#define GUARD_MAX ((int64_t)1 << 34)   /* safety cap, never reached by valid input */

/* gammln (volume2d.f:647-668, Numerical Recipes) */
static double gammln(double xx) {
  static const double cof[6] = {76.18009172947146, -86.50532032941677, 24.01409824083091,
                                -1.231739572450155, .1208650973866179e-2, -.5395239384953e-5};
  const double stp = 2.5066282746310005;
  double x = xx, y = x, tmp = x + 5.5;
  tmp = (x + 0.5) * LOG(tmp) - tmp;
  double ser = 1.000000000190015;
  for (int j = 0; j < 6; j++) {
    y = y + 1.0;
    ser = ser + cof[j] / y;
  }
  return tmp + LOG(stp * ser / x);
}

/* McDonald (volume2d.f:598-626): modified Bessel function K_nu(z) */
static double mcdonald(double nu, double z, int64_t* guard) {
  double sum = 0.0, t = 1.0, sd;
  const double dt = 1.001, d = dt - 1.0, s = 5.0e-1 * (1.0 + dt), a = nu - 5.0e-1;
  do {
    const double ts = t * s;
    const double y = z * ts;
    if (y < 2.25e2)
      sd = POW(ts * ts - 1.0, a) / EXP(y);
    else
      sd = 0.0;
    sum = sum + d * t * sd;
    t = t * dt;
    if (++*guard > GUARD_MAX) return 0.0;
  } while (t < 2.0 || sd > 1.0e-8);
  return SQRT(3.14159265) * POW(5.0e-1 * z, nu) * sum / EXP(gammln(5.0e-1 + nu));
}

/* gamma_bar (volume2d.f:572-594): mean Lorentz factor of a Maxwellian */
static double gamma_bar_g(double Theta, int64_t* guard) {
  double g;
  if (Theta < F32(0.2)) {
    g = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) +
         F32(3.384) * (Theta * Theta * Theta)) /
            (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
        Theta;
  } else {
    const double K2 = mcdonald(2.0, 1.0 / Theta, guard);
    const double K3 = mcdonald(3.0, 1.0 / Theta, guard);
    g = K3 / K2 - Theta;
  }
  if (g < 1.0) g = 1.0;
  return g;
}

double c2o_mcdonald(double nu, double z) {
  int64_t guard = 0;
  return mcdonald(nu, z, &guard);
}

double c2o_gamma_bar(double Theta) {
  int64_t guard = 0;
  return gamma_bar_g(Theta, &guard);
}

/* tridag (update2d.f:2476-2518); 1-based arrays, n = num_nt */
static void tridag(const double* a, const double* b, const double* c, const double* r, double* u) {
  double gam[NT + 2];
  if (FABS(b[1]) <= 1.0e-100) return;
  double bet = b[1];
  u[1] = r[1] / bet;
  for (int i = 2; i <= NT; i++) {
    gam[i] = c[i - 1] / bet;
    bet = b[i] - a[i] * gam[i];
    if (FABS(bet) <= 1.0e-100) {
      for (int n = 1; n <= NT; n++) u[n] = 0.0;
      return;
    }
    u[i] = (r[i] - a[i] * u[i - 1]) / bet;
  }
  for (int i = NT - 1; i >= 1; i--) {
    u[i] = u[i] - gam[i + 1] * u[i + 1];
    if (u[i + 1] < 0.0) u[i + 1] = 0.0;
  }
}

/* one zone's FP_calc state (1-based arrays like the reference) */
typedef struct fp_zone {
  int j, k;
  double vol, tea, tna, n_e, B, Eloss_sy, ecens, ec_old, turb_lev, f_pair;
  double f_nt[NT + 2], Pnt[NT + 2];
  const double* n_field;                    /* [NPH], 0-based */
  double Te_new, gmin, gmax, amxwl, p_nth;  /* p_nth in/out */
  double diag[C2D_FP_NDIAG];
} fp_zone;

#define MAX_FP_STEPS 1000000   /* update2d.f:585-599 stops the run */

/* FP_calc (update2d.f:337-1739) for pair_switch = 0.  Returns 0, or -1
 * where the reference stops (fp_steps > 1e6) or a guard trips. */
static int fp_calc(const c2d_config* g, const c2d_fp_config* fc, double time, double dt,
                   const double* FIC /* [i<NT][NPH] */, fp_zone* Z) {
  const int nz = g->nz, nr = g->nr, j = Z->j, k = Z->k;
  const double zmax = g->z[nz - 1], rmax = g->r[nr - 1];
  double gnt[NT + 2], gamma[NT + 2];
  double f_old[NT + 2], f_new[NT + 2], a_i[NT + 2], b_i[NT + 2], c_i[NT + 2];
  double dg_ic[NT + 2], dg_sy[NT + 2], dgdt[NT + 2], disp[NT + 2];
  double bigC[NT + 2], bigW[NT + 2], smw[NT + 2], inject_ne[NT + 2];
  int64_t guard = 0;
  memset(f_new, 0, sizeof f_new);
  for (int i = 1; i <= NT; i++) gnt[i] = g->gnt[i - 1];
  memset(Z->diag, 0, sizeof Z->diag);

  const double t_esc = fc->r_esc * zmax / C_LIGHT;   /* :460-461 */
  const double t_acc = fc->r_acc * zmax / C_LIGHT;
  double t_fp = 0.0;
  int fp_steps = 0;
  Z->Te_new = Z->tea;
  const double volume = Z->vol;
  double E_el = 0.0, E_pos = 0.0;
  double n_p = Z->n_e;
  double ne = n_p * (1. + Z->f_pair);
  double n_positron = n_p * Z->f_pair;
  double n_lept = ne + n_positron;
  if (n_lept < 1.0e-11) {                            /* :478 */
    Z->diag[C2D_FP_SKIPPED] = 1.0;
    return 0;
  }
  for (int i = 1; i <= NT; i++) {                    /* :482-492 */
    gamma[i] = gnt[i] + 1.0;
    if (i > 1) {
      const double Delta_g = gnt[i] - gnt[i - 1];
      E_el = E_el + Delta_g * gamma[i] * Z->f_nt[i];
    }
  }
  E_el = E_el * ne * 8.176e-7 * volume;
  double e_old = 0.0 + E_el + E_pos + Z->ec_old;   /* :497-498 */
  double e_new = 0.0 + Z->ecens;
  double sum_p = 0.;
  for (int i = 1; i <= NT - 1; i++) sum_p = sum_p + (gnt[i + 1] - gnt[i]) * Z->f_nt[i];
  for (int i = 1; i <= NT; i++) {                    /* :504-509 */
    Z->f_nt[i] = Z->f_nt[i] / sum_p;
    f_old[i] = Z->f_nt[i];
  }
  f_old[NT] = 0.0;

  /* flare (:532-562) */
  const double rmid = (k > 1) ? 5.0e-1 * (g->r[k - 1] + g->r[k - 2]) : 5.0e-1 * (g->r[k - 1] + g->rmin);
  const double zmid = (j > 1) ? 5.0e-1 * (g->z[j - 1] + g->z[j - 2]) : 5.0e-1 * (g->z[j - 1] + g->zmin);
  double tl_flare = 0.0;
  if (fc->cf_sentinel == 1) {
    const double ar = (rmid - fc->r_flare) / fc->sigma_r;
    const double az = (zmid - fc->z_flare) / fc->sigma_z;
    const double at = (time - fc->t_flare) / fc->sigma_t;
    const double y = 5.0e-1 * (ar * ar + az * az + at * at);
    tl_flare = (y < 1.0e2) ? fc->flare_amp / EXP(y) : 0.0;
  }
  const double tlev = Z->turb_lev + tl_flare;
  const double Tp_flare = Z->tna * (1.0 + tl_flare);
  const double Th_p = Tp_flare / 9.382e5;
  double Th_e = Z->tea / 5.11e2;
  const double f_th = 1.5 * volume * n_lept;
  /* Compton cooling from the photon field (:568-574) */
  for (int i = 1; i <= NT - 1; i++) {
    double s = 0.0;
    for (int ph = 1; ph <= NPH; ph++)
      s = s - Z->n_field[ph - 1] * FIC[(size_t)(i - 1) * NPH + (ph - 1)] / volume;
    dg_ic[i] = s;
  }
  dg_ic[NT] = 0.0;   /* H10 */
  const double dz = (j == 1) ? g->z[0] - g->zmin : g->z[j - 1] - g->z[j - 2];   /* :628-632 */

  double hr = 0.0, hr_st = 0.0, sum_E = 0.0;
  for (;;) {
    /* label 200 (:577) */
    double g_av = gamma_bar_g(Th_e, &guard);
    double hr_th_c = 0.0;
    for (int i = 1; i <= NT - 1; i++)
      hr_th_c = hr_th_c - 8.176e-7 * dg_ic[i] * f_old[i] * (gnt[i + 1] - gnt[i]) * volume * n_lept;
    if (fp_steps > MAX_FP_STEPS) return -1;
    const double gamma_R = 2.1e-3 * SQRT(n_lept) / (Z->B * SQRT(g_av));
    const double sT = Th_e + Th_p;
    const double h_T = F32(.79788) * (2. * (sT * sT) + 2.0 * sT + 1.0) /
                       (POW(sT, 1.5) * (1.0 + 1.875 * Th_e + .8203 * (Th_e * Th_e)));
    const double hr_th_Coul = f_th * 1.7386e-26 * n_p * LNL * h_T * (Tp_flare - Z->Te_new);
    double y = gamma_R / g_av;
    const double hr_th_sy = (y < 100.0) ? -Z->Eloss_sy / (dt * EXP(y)) : 0.0;
    double hr_th_A = tlev * hr_th_Coul;
    if (hr_th_A < 1.0e-20) hr_th_A = 1.0e-20;
    const double hr_th_total = hr_th_sy + hr_th_c + hr_th_A;   /* :656 */
    const double dT_total = 6.25e8 * dt * hr_th_total / f_th;
    double f_t_implicit = fc->df_implicit * Z->Te_new / FABS(dT_total);
    if (f_t_implicit > fc->df_T) f_t_implicit = fc->df_T;
    /* rates that reach the solve (:862, :877, :880-889, :1035-1069) */
    const double f_sy = 1.058e-15 * (Z->B * Z->B) / 8.176e-7;
    const double g_thr = 1.0 + 4.0 * Th_e;
    for (int i = 1; i <= NT; i++) {
      y = gamma_R / gamma[i];
      if (y < 100.0)
        dg_sy[i] = -(f_sy * (gamma[i] * gamma[i] - 1.0) / EXP(y));
      else
        dg_sy[i] = -1.0e-50;
    }
    double hr_nt_A = 0.0, hr_st_A = 0.0;
    for (int i = 1; i <= NT; i++) {
      const double dg_A = gamma[i] / t_acc;
      const double disp_A = gamma[i] * gamma[i] / t_acc / 2.0;
      disp[i] = disp_A;
      dgdt[i] = dg_sy[i] + dg_ic[i] + dg_A;
      if (i < NT) {
        hr_nt_A = hr_nt_A + dg_A * f_old[i] * (gamma[i + 1] - gamma[i]);
        if (gamma[i] > g_thr) hr_st_A = hr_st_A + dg_A * f_old[i] * (gamma[i + 1] - gamma[i]);
      }
    }
    hr_st_A = hr_st_A * 8.176e-7 * n_lept * volume;
    hr_nt_A = hr_nt_A * 8.176e-7 * n_lept * volume;
    const double heat_total = hr_th_Coul + hr_nt_A;   /* hr_nt_Coul = hr_th_Coul (:1034) */
    e_old = e_old + heat_total * f_t_implicit * dt;   /* :1105 */
    if (fp_steps == 0) {
      hr = hr + heat_total;
      hr_st = hr_st + hr_st_A;
    }
    double d_t = f_t_implicit * dt;                     /* :1142-1146 */
    if (d_t > (dt - t_fp)) d_t = 1.00001 * (dt - t_fp);
    if (fc->pair_switch == 1) {
      /* pairs on, no positrons (H6): loop 460 (:1187-1217) with dn_pp = 0 and
       * pa_calc's dne_pa = -ne*f*pa_el = -0 adds 0/ne and clips f_old */
      for (int i = 1; i <= NT - 1; i++) {
        f_old[i] = f_old[i] + 0.0 / ne;
        if (f_old[i] < 1.0e-50) f_old[i] = 0.0;
      }
    }
    /* no positrons either way (:1164-1167, :1218-1221) */
    n_positron = 0.0;
    ne = n_p + n_positron;
    /* injection (:1226-1306) */
    double n_inject = 0.0;
    if (fc->pick_sw == 1) {
      double inj_sum = 0.0;
      for (int i = 1; i <= NT - 1; i++) {
        const double x = gamma[i] - fc->inj_gg;
        inject_ne[i] = 1.0e2 * EXP(-((x * x) / 2.0 / (fc->inj_sigma * fc->inj_sigma))) /
                       (fc->inj_sigma * SQRT(2.0 * PI_REF));
        inj_sum = inj_sum + inject_ne[i] * (gnt[i + 1] - gnt[i]);
      }
      const double inj_rho = fc->pick_rate * d_t;
      for (int i = 1; i <= NT - 1; i++) {
        inject_ne[i] = inj_rho * inject_ne[i] / inj_sum;
        f_old[i] = f_old[i] + inject_ne[i] / ne;
        n_inject = n_inject + inject_ne[i] * (gnt[i + 1] - gnt[i]);
      }
    }
    if (fc->inj_switch != 0) {
      const double tt = time + t_fp - fc->inj_t;
      if (tt > dz / fc->inj_v * (double)(j - 1) && tt < dz / fc->inj_v * (double)j && k <= nr) {
        double inj_sum = 0.0, inj_E = 0.0;
        for (int i = 1; i <= NT - 1; i++) {
          if (fc->inj_dis == 1) {
            const double x = gamma[i] - fc->inj_gg;
            inject_ne[i] = 1.0e2 * EXP(-((x * x) / 2.0 / (fc->inj_sigma * fc->inj_sigma))) /
                           (fc->inj_sigma * SQRT(2.0 * PI_REF));
          } else {
            const double inj_g2var =
                fc->inj_g2 * POW(10.0, (time + t_fp - fc->inj_t) * fc->inj_v / zmax);
            if (gamma[i] > fc->inj_g1) {
              const double inj_y =
                  (fc->g2var_switch == 1) ? gamma[i] / inj_g2var : gamma[i] / fc->inj_g2;
              inject_ne[i] = (inj_y < 1.0e2) ? 1.0e2 / (POW(gamma[i], fc->inj_p) * EXP(inj_y)) : 0.0;
            } else {
              inject_ne[i] = 0.0;
            }
          }
          inj_sum = inj_sum + inject_ne[i] * (gnt[i + 1] - gnt[i]);
          inj_E = inj_E + inject_ne[i] * (gnt[i + 1] - gnt[i]) * gamma[i];
        }
        inj_E = inj_E / inj_sum;
        const double inj_rate = fc->inj_L / 8.186e-7 / inj_E / (PI_REF * (rmax * rmax) * dz);
        const double inj_rho = inj_rate * d_t;
        for (int i = 1; i <= NT - 1; i++) {
          inject_ne[i] = inj_rho * inject_ne[i] / inj_sum;
          f_old[i] = f_old[i] + inject_ne[i] / ne;
          n_inject = n_inject + inject_ne[i] * (gnt[i + 1] - gnt[i]);
        }
      }
    }
    ne = ne + n_inject;
    n_p = n_p + n_inject;
    n_lept = n_lept + n_inject;
    /* escape (:1309-1313) */
    ne = ne * t_esc / (t_esc + d_t);
    n_p = n_p * t_esc / (t_esc + d_t);
    n_lept = n_lept * t_esc / (t_esc + d_t);
    /* Chang-Cooper coefficients (:1319-1390) */
    a_i[1] = 0.0; b_i[1] = 1.0; c_i[1] = 0.0;
    a_i[NT] = 0.0; b_i[NT] = 1.0; c_i[NT] = 0.0;
    for (int i = 2; i <= NT - 1; i++) {
      const double D_gminus = gnt[i] - gnt[i - 1];
      const double D_gplus = gnt[i + 1] - gnt[i];
      const double Delta_g = SQRT(gnt[i] / gnt[i - 1]) * D_gminus;
      if (i == 2) {
        const double bigB1 = -(dgdt[1] + dgdt[2]);
        bigC[1] = (disp[1] + disp[2]) / 2.0;
        smw[1] = D_gminus * bigB1 / bigC[1];
        bigW[1] = smw[1] / (EXP(smw[1]) - 1.0);
      }
      const double bigB = -(dgdt[i] + dgdt[i + 1]) / 2.0;
      bigC[i] = (disp[i] + disp[i + 1]) / 2.0;
      smw[i] = D_gplus * bigB / bigC[i];
      bigW[i] = smw[i] / (EXP(smw[i]) - 1.0);
      c_i[i] = -d_t * (bigC[i] * smw[i] / (1.0 - EXP(-smw[i])) / Delta_g / D_gplus);
      b_i[i] = 1.0 +
               d_t / Delta_g *
                   (bigC[i] * bigW[i] / D_gplus +
                    bigC[i - 1] * smw[i - 1] / (1.0 - EXP(-smw[i - 1])) / D_gminus) +
               d_t / t_esc;
      a_i[i] = -d_t / Delta_g * bigC[i - 1] * bigW[i - 1] / D_gminus;
    }
    tridag(a_i, b_i, c_i, f_old, f_new);
    f_new[NT] = 0.0;
    f_new[1] = 0.0;
    sum_p = 0.;
    double sE = 0.;
    for (int i = 1; i <= NT - 1; i++) {             /* :1415-1419 */
      sum_p = sum_p + (gnt[i + 1] - gnt[i]) * f_new[i];
      sE = sE + (gnt[i + 1] - gnt[i]) * gamma[i] * f_new[i];
      Z->Pnt[i] = sum_p;
    }
    sum_E = sE / sum_p;
    t_fp = t_fp + d_t;
    fp_steps = fp_steps + 1;
    for (int i = 1; i <= NT; i++) {
      f_new[i] = f_new[i] / sum_p;
      f_old[i] = f_new[i];
    }
    /* new temperature (:1440-1468) */
    double gbar = 0.0;
    for (int i = 1; i <= NT - 1; i++) gbar = gbar + gamma[i] * f_new[i] * (gnt[i + 1] - gnt[i]);
    double The_new = Th_e;
    if (gbar > g_av) {
      while (gbar > g_av) {
        The_new = The_new * F32(1.005);
        g_av = gamma_bar_g(The_new, &guard);
        if (guard > GUARD_MAX) return -1;
      }
    } else {
      while (gbar < g_av) {
        The_new = The_new / F32(1.005);
        g_av = gamma_bar_g(The_new, &guard);
        if (The_new < 1.0e-2) break;
        if (guard > GUARD_MAX) return -1;
      }
    }
    Z->Te_new = 5.11e2 * The_new;
    Th_e = The_new;
    if (!(t_fp < dt)) break;                          /* :1473 */
  }
  /* normalised outputs (:1481-1500) */
  E_el = 0.0;
  E_pos = 0.0;
  for (int i = 1; i <= NT; i++) {
    Z->f_nt[i] = f_new[i];
    Z->Pnt[i] = Z->Pnt[i] / sum_p;
    if (i > 1) E_el = E_el + Z->f_nt[i] * gamma[i] * (gnt[i] - gnt[i - 1]);
  }
  E_el = E_el * ne * 8.176e-7 * volume;
  e_new = e_new + E_el + E_pos;
  Z->n_e = n_p;
  /* nonthermal parameters (:1654-1736) */
  int i;
  for (i = 5; i <= NT - 5; i++)
    if (f_new[i] > 1.0e-10) break;
  Z->gmin = gamma[i];
  const int i_nt = i;
  for (i = NT - 5; i >= 5; i--)
    if (f_new[i] > 1.0e-15) break;
  Z->gmax = gamma[i];
  double sum_nt = 0.0, sum_th = 0.0;
  for (i = 1; i <= NT - 1; i++) {
    if (i < i_nt)
      sum_th = sum_th + (gamma[i + 1] - gamma[i]) * f_new[i];
    else
      sum_nt = sum_nt + (gamma[i + 1] - gamma[i]) * f_new[i];
  }
  Z->amxwl = sum_th / (sum_nt + sum_th);
  if (Z->amxwl > 9.999e-1) {
    Z->amxwl = 1.0;
  } else {
    double p_nth = F32(0.1);
    double sum_g = 1.0e50, sumg_old;
    for (;;) {
      sumg_old = sum_g;
      sum_g = 0.0;
      double sum_gg = 0.0;
      const double p_1 = 1.0 - p_nth;
      double N_nt;
      if (FABS(p_1) > 1.0e-4)
        N_nt = (1. - Z->amxwl) * p_1 / (POW(Z->gmax, p_1) - POW(Z->gmin, p_1));
      else
        N_nt = (1.0 - Z->amxwl) / LOG(Z->gmax / Z->gmin);
      for (i = i_nt; i <= NT - 2; i++) {
        const double yy = gamma[i] / Z->gmax;
        if (!(yy < 100.0)) break;
        const double f_pl = N_nt / (POW(gamma[i], p_nth) * EXP(yy));
        sum_g = sum_g + f_pl * gamma[i] * (gnt[i + 1] - gnt[i]);
        sum_gg = sum_gg + f_pl * (gnt[i + 1] - gnt[i]);
      }
      sum_g = sum_g / sum_gg;
      sum_g = FABS(sum_g - sum_E);
      if (sum_g < sumg_old && p_nth < 10.) {
        p_nth = p_nth + 0.5e-1;
        continue;
      }
      break;
    }
    Z->p_nth = p_nth;
  }
  Z->diag[C2D_FP_E_OLD] = e_old;
  Z->diag[C2D_FP_E_NEW] = e_new;
  Z->diag[C2D_FP_HR] = hr;
  Z->diag[C2D_FP_HR_ST] = hr_st;
  Z->diag[C2D_FP_DELTA_T] = FABS(Z->Te_new - Z->tea) / Z->Te_new;
  Z->diag[C2D_FP_STEPS] = (double)fp_steps;
  return 0;
}

static double A2(const c2d_array2* a, int j, int k, double dflt) {
  return a->data ? a->data[j * a->s_j + k * a->s_k] : dflt;
}
static double* M2(const c2d_marray2* a, int j, int k) {
  return a->data ? &a->data[j * a->s_j + k * a->s_k] : NULL;
}

static int fp_step_sel(const c2d_config* g, const c2d_fp_config* fc, const c2d_fp_step_in* in,
                       c2d_fp_step_out* out, const int32_t* sel, int nsel);

/* `update` (update2d.f:138-277) over all zones, serially in zone order. */
int c2o_fp_step(const c2d_config* g, const c2d_fp_config* fc, const c2d_fp_step_in* in,
                c2d_fp_step_out* out) {
  return fp_step_sel(g, fc, in, out, NULL, 0);
}

/* The same for the listed zones only (cell = j*nr + k, ascending): tests
 * check a sample of a large grid's zones (FP_calc's zones are independent);
 * the E_add_up sums then cover those zones only. */
int c2o_fp_step_zones(const c2d_config* g, const c2d_fp_config* fc, const c2d_fp_step_in* in,
                      c2d_fp_step_out* out, const int32_t* cells, int ncells) {
  if (!cells || ncells < 0) return C2D_E_ARG;
  return fp_step_sel(g, fc, in, out, cells, ncells);
}

static int fp_step_sel(const c2d_config* g, const c2d_fp_config* fc, const c2d_fp_step_in* in,
                       c2d_fp_step_out* out, const int32_t* sel, int nsel) {
  if (!g || !fc || !in || !out) return C2D_E_ARG;
  if (fc->pair_switch != 0 && fc->pair_switch != 1) return C2D_E_ARG;
  if (fc->inj_switch != 0 && fc->inj_dis != 1 && fc->inj_dis != 2) return C2D_E_ARG;
  if (!fc->F_IC || !in->n_field.data || !in->ecens.data || !out->f_nt.data || !out->Pnt.data)
    return C2D_E_ARG;
  const int nz = g->nz, nr = g->nr;
  if (fc->pair_switch == 1)
    for (int j = 0; j < nz; j++)
      for (int k = 0; k < nr; k++)
        if (A2(&in->f_pair, j, k, 0.0) != 0.0) return C2D_E_ARG;
  double* FIC = (double*)malloc(sizeof(double) * NT * NPH);
  if (!FIC) return C2D_E_NOMEM;
  for (int i = 0; i < NT; i++)
    for (int ph = 0; ph < NPH; ph++)
      FIC[(size_t)i * NPH + ph] = fc->F_IC[i * fc->F_IC_s_i + ph * fc->F_IC_s_ph];
  double dT_max = (in->ncycle <= 1) ? fc->df_T : 0.0;   /* photon_fill :1912 */
  double E_old = 0.0, E_new = 0.0, hr = 0.0, hr_st = 0.0;
  double nf[NPH];
  int rc = 0;
  int isel = 0;
  for (int j = 0; j < nz && rc == 0; j++)
    for (int k = 0; k < nr && rc == 0; k++) {
      if (sel) {
        if (isel >= nsel || sel[isel] != j * nr + k) continue;
        isel++;
      }
      fp_zone Z;
      memset(&Z, 0, sizeof Z);
      Z.j = j + 1;
      Z.k = k + 1;
      Z.vol = A2(&in->vol, j, k, 0.0);
      Z.tea = A2(&in->tea, j, k, 0.0);
      Z.tna = A2(&in->tna, j, k, 0.0);
      Z.n_e = A2(&in->n_e, j, k, 0.0);
      Z.B = A2(&in->B_field, j, k, 0.0);
      Z.Eloss_sy = A2(&in->Eloss_sy, j, k, 0.0);
      Z.ecens = A2(&in->ecens, j, k, 0.0);
      Z.ec_old = A2(&in->ec_old, j, k, 0.0);
      Z.turb_lev = A2(&in->turb_lev, j, k, 0.0);
      Z.f_pair = A2(&in->f_pair, j, k, 0.0);
      for (int i = 0; i < NT; i++) {
        Z.f_nt[i + 1] = out->f_nt.data[i * out->f_nt.s_i + j * out->f_nt.s_j + k * out->f_nt.s_k];
        Z.Pnt[i + 1] = out->Pnt.data[i * out->Pnt.s_i + j * out->Pnt.s_j + k * out->Pnt.s_k];
      }
      for (int ph = 0; ph < NPH; ph++)
        nf[ph] = in->n_field.data[ph * in->n_field.s_i + j * in->n_field.s_j + k * in->n_field.s_k];
      Z.n_field = nf;
      double* pp = M2(&out->p_nth, j, k);
      double* pgmin = M2(&out->gmin, j, k);
      double* pgmax = M2(&out->gmax, j, k);
      double* pamx = M2(&out->amxwl, j, k);
      Z.p_nth = pp ? *pp : 0.0;
      Z.gmin = pgmin ? *pgmin : 0.0;
      Z.gmax = pgmax ? *pgmax : 0.0;
      Z.amxwl = pamx ? *pamx : 0.0;
      if (fp_calc(g, fc, in->time, in->dt, FIC, &Z) != 0) {
        rc = C2D_E_FP;
        break;
      }
      double* p;
      if ((p = M2(&out->Te_new, j, k))) *p = Z.Te_new;
      if (Z.diag[C2D_FP_SKIPPED] == 0.0) {
        for (int i = 0; i < NT; i++) {
          out->f_nt.data[i * out->f_nt.s_i + j * out->f_nt.s_j + k * out->f_nt.s_k] = Z.f_nt[i + 1];
          out->Pnt.data[i * out->Pnt.s_i + j * out->Pnt.s_j + k * out->Pnt.s_k] = Z.Pnt[i + 1];
        }
        if ((p = M2(&out->n_e, j, k))) *p = Z.n_e;
        if (pgmin) *pgmin = Z.gmin;
        if (pgmax) *pgmax = Z.gmax;
        if (pamx) *pamx = Z.amxwl;
        if (pp) *pp = Z.p_nth;
        E_old = E_old + Z.diag[C2D_FP_E_OLD];
        E_new = E_new + Z.diag[C2D_FP_E_NEW];
        hr = hr + Z.diag[C2D_FP_HR];
        hr_st = hr_st + Z.diag[C2D_FP_HR_ST];
        if (Z.diag[C2D_FP_DELTA_T] > dT_max) dT_max = Z.diag[C2D_FP_DELTA_T];
      }
      /* tea update (update2d.f:266-276) */
      if ((p = M2(&out->tea, j, k)) && Z.tna > 1.) {
        double t = Z.Te_new;
        t = (TEMP_MAX < t) ? TEMP_MAX : t;
        t = (TEMP_MIN > t) ? TEMP_MIN : t;
        *p = t;
      }
      if (out->zone_diag)
        memcpy(out->zone_diag + (size_t)(j * nr + k) * C2D_FP_NDIAG, Z.diag, sizeof Z.diag);
    }
  free(FIC);
  out->E_tot_old = E_old;
  out->E_tot_new = E_new;
  out->hr_total = hr;
  out->hr_st_total = hr_st;
  out->dT_max = dT_max;
  return rc;
}
