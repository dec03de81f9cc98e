/*
 * oracle/c2d_vem_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-step emission/absorption tables
 * (bbw7561135/Compton2d, src/ snapshot): the parity checker for the GPU
 * kernel (compton2d_amd/csrc/vem.hip).  Only tests/ and the bench's CPU
 * baseline load it; the product path never does.
 *
 *   volume_em                       src/volume2d.f:10-394
 *   expk13, expk43                  src/volume2d.f:672-752
 *   gamma_bar, McDonald, gammln     src/volume2d.f:572-668 (c2d_fp_oracle.c)
 *   imcgen2d's per-cell loop        src/imcgen2d.f:209-333 (B from ep_switch,
 *                                   l_min, Eloss_sy, Eloss_cy/Eloss_th scaling)
 *
 * Only what reaches volume_em's outputs is restated: kappa_tot = kappa_sy
 * (:347), the cumulative distributions eps_tot / eps_th (:392-403) and the
 * sums Eloss_cy / Eloss_th (:352-368).  The bremsstrahlung and cyclotron
 * opacities, the power-law synchrotron fit (F_sync_fit_flag = 0) and the
 * pair-annihilation term (pair_switch = 0, hazard H6) do not, and are not.
 *
 * Expression order, the REAL literals of the Fortran (F32) and integer
 * powers (x**2 = x*x, x**3 = (x*x)*x) follow the reference; pinned bit for
 * bit to the reference itself (oracle/ref/c2d_vemdrv.f) by
 * tests/test_vem_oracle.py on the committed fixture tests/golden/vem.npz.
 */
#include <stdint.h>
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
#define F32(x) ((double)(float)(x))

#define NT C2D_NUM_NT
#define NV C2D_N_VOL

static const double PI_REF = 3.1415926536;     /* general.pa:24 */
static const double C_LIGHT = 2.9979245620e10; /* general.pa:25 */

double c2o_gamma_bar(double Theta);             /* c2d_fp_oracle.c */
double c2o_mcdonald(double nu, double z);       /* c2d_fp_oracle.c */

/* expk13 (volume2d.f:672-712): exp(t) K_{1/3}(t) */
static double expk13(double t) {
  const double c1 = F32(0.35502805), c2 = F32(0.25881940);   /* DATA with REAL literals */
  if (t <= 1.0) {
    double z3 = 1.5 * t;
    const double zs = POW(z3, 0.3333333333333333);
    const double z = zs * zs;
    z3 = z3 * z3;
    const double f1 = 1.0 + z3 / 6.0 * (1.0 + z3 / 30.0 * (1.0 + z3 / 56.0));
    const double f2 = z * (1.0 + z3 / 12.0 * (1.0 + z3 / 42.0 * (1.0 + z3 / 90.0)));
    return EXP(t) * PI_REF * 1.7320508 / zs * (c1 * f1 - c2 * f2);
  }
  const double z = 1.0 / (72.0 * t);
  const double poly = 1.0 - 5.0 * z * (1.0 - 38.5 * z);
  return SQRT(0.5 * PI_REF / t) * poly / (1.0 + 1.0 / (1.0 + 58.0 * t * t));
}

/* expk43 (volume2d.f:718-745): exp(t) K_{4/3}(t) */
static double expk43(double t) {
  if (t <= 1.0) {
    const double poly = 1.0 + t * (0.9757317 - 7.6790616e-2 * t);
    return 0.44648975 * POW(2.0 / t, 1.333333333) * poly;
  }
  const double z = 1.0 / (72.0 * t);
  const double poly = 1.0 + 55.0 * z * (1.0 - 8.5 * z);
  return SQRT(0.5 * PI_REF / t) * poly * (1.0 + 1.0 / (1.0 + 50.0 * t * t));
}

/* The photon grid volume_em (re)writes into E_ph (:98, :106-107). */
void c2o_vem_grid(double* E_ph) {
  const double dE = EXP(LOG(1.0e20) / (double)NV);
  double E = 1.0e-10 / dE;
  for (int i = 0; i < NV; i++) {
    E = E * dE;
    E_ph[i] = E;
  }
}

/* volume_em for one cell; f_nt[NT], gnt[NT]; outputs kappa[NV], eps_tot[NV],
 * eps_th[NV] and the raw sums *Eloss_cy, *Eloss_th (volume2d.f:10-394). */
void c2o_volume_em(const double* gnt, const double* f_nt, double T_keV, double ne_local, double B,
                   double l_min, double* kappa, double* eps_tot, double* eps_th, double* Eloss_cy,
                   double* Eloss_th) {
  const double sigmaT = 6.6524616e-25, ee = 4.803e-10, em = 9.109e-28;
  const int n_harmonics = 5;
  double gamma0[NT], gamp[NT], P[NV], P_th[NV];
  const double nu_b = ee * B / (2 * PI_REF * em * C_LIGHT);
  const double Ub = (B * B) / (8.0 * PI_REF);
  const double face = POW(3.0, 1.5) * sigmaT * C_LIGHT * Ub / (PI_REF * nu_b);
  for (int i = 0; i < NT; i++) {
    gamma0[i] = gnt[i] + 1.0;
    gamp[i] = gamma0[i] * SQRT(gamma0[i] * gamma0[i] - 1.0);
  }
  const double dE = EXP(LOG(1.0e20) / (double)NV);
  const double Theta = T_keV / 5.11e2;
  const double kappa_C = 6.65e-25 * ne_local;
  double K2;
  if (Theta < 2.0e-1)
    K2 = 1.2533 * SQRT(Theta) *
         (1. + 1.875 * Theta + 8.2031e-1 * (Theta * Theta) - 2.03e-1 * (Theta * Theta * Theta)) /
         EXP(Theta);
  else
    K2 = c2o_mcdonald(2.0, 1. / Theta);
  const double nu_c = 2.8e6 * B;
  const double nu_min = (double)n_harmonics * nu_c;
  const double nu_p = 9.0e3 * SQRT(ne_local);
  double P_sum = 0., sum_th = 0., ecy = 0., eth = 0.;
  double E = 1.0e-10 / dE;
  const double g_av = c2o_gamma_bar(Theta);
  const double gamma_R = 2.1e-3 * SQRT(ne_local) / (B * SQRT(g_av));
  double y = gamma_R / g_av;
  const double f_rz = (y < 1.0e2) ? EXP(-y) : 0.;
  const double thr = (1.0 / l_min > 1.0e1 * kappa_C) ? 1.0 / l_min : 1.0e1 * kappa_C;
  for (int i = 0; i < NV; i++) {
    E = E * dE;
    const double nu = 2.41487e17 * E;
    /* non-thermal synchrotron (:160-246), F_sync_fit_flag = 0 branch */
    double j_sy = 0., kappa_sy = 0.;
    if (!(nu <= nu_p)) {
      double sum = 0., sum_k = 0.;
      for (int i2 = 0; i2 < NT - 1; i2++) {
        const double facg = 3.0 * (gamma0[i2] * gamma0[i2]) * nu_b;
        const double tt = nu / facg;
        double es;
        if (tt < 1.0e4) {
          const double eq43 = expk43(tt), eq13 = expk13(tt);
          const double ff = tt * tt * (eq43 * eq13 - F32(0.6) * tt * (eq43 - eq13) * (eq43 + eq13));
          es = face * ff * EXP(-2.0 * tt);
        } else {
          es = 0.0;
        }
        const double sd = f_nt[i2] * es;
        const double sd_k = gamp[i2] * es;
        sum = sum + (gnt[i2 + 1] - gnt[i2]) * sd;
        sum_k = sum_k + (f_nt[i2] / gamp[i2] - f_nt[i2 + 1] / gamp[i2 + 1]) * sd_k;
      }
      j_sy = sum * ne_local / (4.0 * PI_REF);
      kappa_sy = sum_k * ne_local / (8.0 * PI_REF * em * (nu * nu));
      if (kappa_sy < 0.) kappa_sy = -1.0 * kappa_sy;
    }
    /* thermal cyclotron emissivity (:252-321); its opacity is not an output */
    double j_cy = 0.;
    if (!(nu <= nu_p)) {
      double f_m = 1.0;
      for (int m = 1; m <= n_harmonics; m++) {
        const double mm = (double)m;
        f_m = f_m / (4. * mm);
        const double nu_m = mm * nu_c;
        const double E_m = 4.14e-18 * nu_m;
        const double D_m = 7.07e-1 * Theta * E_m;
        const double q = (E - E_m) / D_m;
        const double x = q * q;
        if (x < 50.) {
          const double f_cy = f_rz * EXP(-x) * ne_local * (B * B) * POW(Theta, mm - 1.5) *
                              (mm + 1.0) * f_m * POW(mm, 2.0 * mm + 1.0);
          j_cy = j_cy + 8.46e-14 * f_cy * (E * E) / (E_m * E_m * E_m);
        }
      }
      if (nu > nu_min) {
        const double v = nu / (nu_c * (Theta * Theta));
        y = 4.5 * v;
        if (y < 1.0e6)
          j_cy = j_cy + 4.652e-12 * ne_local * nu / (K2 * POW(v, 1.6666667e-1) * EXP(POW(y, 3.33333e-1)));
      }
    }
    kappa[i] = kappa_sy;                                   /* :347 */
    if (kappa_sy < thr) {
      P_sum = P_sum + j_sy * E * (dE - 1.0);
      ecy = ecy + j_cy * E * (dE - 1.0);
    } else {
      const double x = E / T_keV;
      const double tau_tot = kappa_sy * l_min;
      double j_th = (x < 1.0e2) ? 1.47e-47 * (nu * nu * nu) / (EXP(x) - 1.0) : 1.0e-50;
      if (tau_tot < 5.0e1) j_th = j_th * (1.0 - EXP(-tau_tot));
      sum_th = sum_th + j_th * E * (dE - 1.0);
      eth = eth + j_th * E * (dE - 1.0);
    }
    P[i] = P_sum;
    P_th[i] = sum_th;
  }
  for (int i = 0; i < NV; i++) {
    eps_tot[i] = (P_sum > 1.0e-50) ? P[i] / P_sum : 0.;
    eps_th[i] = (sum_th > 1.0e-50) ? P_th[i] / sum_th : 0.;
  }
  *Eloss_cy = ecy;
  *Eloss_th = eth;
}

/* ------------------------------------------------------------------ */
/* imcgen2d's per-cell loop (imcgen2d.f:209-333) over the c2d_vem_* ABI  */
/* ------------------------------------------------------------------ */
static double A2(const c2d_array2* a, int j, int k) { return a->data[j * a->s_j + k * a->s_k]; }
static double* M2(const c2d_marray2* a, int j, int k) {
  return a->data ? a->data + j * a->s_j + k * a->s_k : 0;
}

int c2o_vem_step(const c2d_config* g, const c2d_vem_in* in, c2d_vem_out* out) {
  if (!g || !in || !out) return C2D_E_ARG;
  double E_ph[NV];
  c2o_vem_grid(E_ph);
  if (out->E_ph) memcpy(out->E_ph, E_ph, sizeof E_ph);
  double fnt[NT], kap[NV], et[NV], eh[NV];
  for (int j = 0; j < g->nz; j++)
    for (int k = 0; k < g->nr; k++) {
      const int ep = in->ep_switch.data ? in->ep_switch.data[j * in->ep_switch.s_j + k * in->ep_switch.s_k] : 0;
      const double tea = A2(&in->tea, j, k), ne = A2(&in->n_e, j, k);
      double B = A2(&in->B_field, j, k);
      if (ep == 1 || ep == 2) {                               /* :217-236 */
        const double Th = (ep == 1) ? 1.957e-3 * tea : 1.066e-6 * A2(&in->tna, j, k);
        double uB;
        if (Th < 1.0e-2)
          uB = 1.5 * Th + 7.5 * (Th * Th);
        else
          uB = c2o_mcdonald(3.0, 1.0 / Th) / c2o_mcdonald(2.0, 1.0 / Th) - Th - 1.0;
        if (ep == 1)
          uB = uB * ne * 8.176e-7 * (1. + 2.0 * A2(&in->f_pair, j, k));
        else
          uB = uB * ne * 1.5e-3;
        B = SQRT(2.513e1 * uB);
      }
      double l_min;                                           /* :238-246 */
      const double dz = (j == 0) ? g->z[0] : g->z[j] - g->z[j - 1];
      const double drr = (k == 0) ? g->r[0] - g->rmin : g->r[k] - g->r[k - 1];
      l_min = (dz < drr) ? dz : drr;
      for (int i = 0; i < NT; i++) fnt[i] = in->f_nt.data[i * in->f_nt.s_i + j * in->f_nt.s_j + k * in->f_nt.s_k];
      double ecy, eth;
      c2o_volume_em(g->gnt, fnt, tea, ne, B, l_min, kap, et, eh, &ecy, &eth);
      double s1 = 0.0;                                        /* :169-172 */
      for (int i = 0; i < NT - 1; i++)
        s1 = s1 + ((g->gnt[i] + 1.0) * (g->gnt[i] + 1.0) - 1.0) * fnt[i] * (g->gnt[i + 1] - g->gnt[i]);
      const double vol = A2(&in->vol, j, k), zs = A2(&in->zsurf, j, k);
      const double esy = 1.058e-15 * ne * in->dt * (B * B) * s1 * vol;
      for (int i = 0; i < NV; i++) {
        const int64_t o3 = i;
        if (out->kappa_tot.data)
          out->kappa_tot.data[o3 * out->kappa_tot.s_i + j * out->kappa_tot.s_j + k * out->kappa_tot.s_k] = kap[i];
        if (out->eps_tot.data)
          out->eps_tot.data[o3 * out->eps_tot.s_i + j * out->eps_tot.s_j + k * out->eps_tot.s_k] = et[i];
        if (out->eps_th.data)
          out->eps_th.data[o3 * out->eps_th.s_i + j * out->eps_th.s_j + k * out->eps_th.s_k] = eh[i];
      }
      double* p;
      if ((p = M2(&out->B_field, j, k))) *p = B;
      if ((p = M2(&out->Eloss_sy, j, k))) *p = esy;
      if ((p = M2(&out->Eloss_cy, j, k))) *p = in->dt * vol * ecy;
      if ((p = M2(&out->Eloss_th, j, k))) *p = in->dt * zs * eth;
      if ((p = M2(&out->Eloss_tot, j, k))) *p = esy;       /* :330 */
    }
  return C2D_OK;
}
