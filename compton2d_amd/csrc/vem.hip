/*
 * vem.hip — per-step emission / absorption tables on gfx950 (SURVEY.md
 * §8(f)#2): imcgen2d's per-cell loop (src/imcgen2d.f:209-333) with
 * volume_em (src/volume2d.f:10-394), one workgroup per cell.
 *
 *   wave 0      cell scalars: B from ep_switch and volume_em's K2 / gamma_bar
 *               from McDonald's series (c2d_wave.hpp, 64 terms per pass),
 *               Eloss_sy's 199-term sum, in the reference's order;
 *   all lanes   one photon energy each (400 of VEM_BLOCK): the 199-term
 *               synchrotron sums j_sy / kappa_sy with expk13/expk43 (in bin
 *               order, as the reference's loop), the cyclotron emissivity,
 *               the absorbed/thin branch and its contribution;
 *   wave 0      the running sums P(i), P_th(i), Eloss_cy, Eloss_th over the
 *               400 energies in order (readlane chain), then every lane
 *               normalises its eps_tot(i), eps_th(i).
 *
 * Cell inputs and the electron spectrum sit in LDS.  Only what reaches
 * volume_em's outputs is computed (see oracle/c2d_vem_oracle.c).  c2d_math.h
 * with -ffp-contract=off: bit-identical to the det build of the oracle.
 * Compute-bound: per cell 400 x 199 terms of two Bessel fits and an exp.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_wave.hpp"

namespace c2d {
namespace {

using namespace wave;
constexpr int VEM_BLOCK = 448;                 /* 7 waves >= 400 energies */
constexpr int NT = C2D_NUM_NT;
constexpr int NV = C2D_N_VOL;
constexpr double PI_REF = 3.1415926536;        /* general.pa:24 */
constexpr double C_LIGHT = 2.9979245620e10;    /* general.pa:25 */

/* expk13 (volume2d.f:672-712) */
__device__ __forceinline__ double expk13(double t) {
  const double c1 = F32(0.35502805), c2 = F32(0.25881940);
  if (t <= 1.0) {
    double z3 = 1.5 * t;
    const double zs = c2d_pow(z3, 0.3333333333333333);
    const double z = zs * zs;
    z3 = z3 * z3;
    const double f1 = 1.0 + z3 / 6.0 * (1.0 + z3 / 30.0 * (1.0 + z3 / 56.0));
    const double f2 = z * (1.0 + z3 / 12.0 * (1.0 + z3 / 42.0 * (1.0 + z3 / 90.0)));
    return c2d_exp_bf(t) * PI_REF * 1.7320508 / zs * (c1 * f1 - c2 * f2);
  }
  const double z = 1.0 / (72.0 * t);
  const double poly = 1.0 - 5.0 * z * (1.0 - 38.5 * z);
  return __builtin_sqrt(0.5 * PI_REF / t) * poly / (1.0 + 1.0 / (1.0 + 58.0 * t * t));
}

/* expk43 (volume2d.f:718-745) */
__device__ __forceinline__ double expk43(double t) {
  if (t <= 1.0) {
    const double poly = 1.0 + t * (0.9757317 - 7.6790616e-2 * t);
    return 0.44648975 * c2d_pow(2.0 / t, 1.333333333) * poly;
  }
  const double z = 1.0 / (72.0 * t);
  const double poly = 1.0 + 55.0 * z * (1.0 - 8.5 * z);
  return __builtin_sqrt(0.5 * PI_REF / t) * poly * (1.0 + 1.0 / (1.0 + 50.0 * t * t));
}

}  // namespace

__global__ void __launch_bounds__(VEM_BLOCK) c2d_vem_kernel(const VemParams P) {
  __shared__ double s_gnt[NT], s_f[NT], s_q[NT], s_gamp[NT], s_facg[NT], s_dg[NT];
  __shared__ double s_cP[NV], s_cC[NV], s_cT[NV], s_P[NV], s_Pth[NV];
  __shared__ double s_sc[8];   /* B, K2, f_rz, P_sum, sum_th, Eloss_cy, Eloss_th, Eloss_sy */
  __shared__ double s_mcd[4 * FPB];   /* McDonald term exchange (wave 0) */
  const int cell = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const double* zin = P.zin + (int64_t)cell * VZ_N;
  const double tea = zin[VZ_TEA], ne = zin[VZ_NE];
  for (int i = tid; i < NT; i += VEM_BLOCK) {
    s_gnt[i] = P.gnt[i];
    s_f[i] = P.f_nt[(int64_t)cell * NT + i];
  }
  __syncthreads();
  /* ---- wave 0: cell scalars ---- */
  if (wv == 0) {
    long long guard = 0;
    double B = zin[VZ_B];
    const int ep = (int)zin[VZ_EP];
    if (ep == 1 || ep == 2) {                           /* imcgen2d.f:217-236 */
      const double Th = (ep == 1) ? 1.957e-3 * tea : 1.066e-6 * zin[VZ_TNA];
      double uB;
      if (Th < 1.0e-2) {
        uB = 1.5 * Th + 7.5 * (Th * Th);
      } else {
        double K2b, K3b;
        mcdonald23_w(1.0 / Th, lane, P.mcd, K2b, K3b, guard, s_mcd);
        uB = K3b / K2b - Th - 1.0;
      }
      if (ep == 1)
        uB = uB * ne * 8.176e-7 * (1. + 2.0 * zin[VZ_FPAIR]);
      else
        uB = uB * ne * 1.5e-3;
      B = __builtin_sqrt(2.513e1 * uB);
    }
    const double Theta = tea / 5.11e2;
    double K2 = 0.0, K2m = 0.0, K3m = 0.0;
    const bool big = !(Theta < F32(0.2)) || !(Theta < 2.0e-1);
    if (big) mcdonald23_w(1. / Theta, lane, P.mcd, K2m, K3m, guard, s_mcd);
    if (Theta < 2.0e-1)                                 /* volume2d.f:56-65 */
      K2 = 1.2533 * __builtin_sqrt(Theta) *
           (1. + 1.875 * Theta + 8.2031e-1 * (Theta * Theta) - 2.03e-1 * (Theta * Theta * Theta)) /
           c2d_exp_bf(Theta);
    else
      K2 = K2m;
    double g_av;                                        /* gamma_bar (volume2d.f:572-594) */
    if (Theta < F32(0.2)) {
      g_av = (1. + F32(4.375) * Theta + F32(7.383) * (Theta * Theta) +
              F32(3.384) * (Theta * Theta * Theta)) /
                 (1. + F32(1.875) * Theta + F32(.8203) * (Theta * Theta)) -
             Theta;
    } else {
      g_av = K3m / K2m - Theta;
    }
    if (g_av < 1.0) g_av = 1.0;
    const double gamma_R = 2.1e-3 * __builtin_sqrt(ne) / (B * __builtin_sqrt(g_av));
    const double y = gamma_R / g_av;
    const double f_rz = (y < 1.0e2) ? c2d_exp_bf(-y) : 0.;
    /* Eloss_sy's sum (imcgen2d.f:169-172), in order */
    const double s1 = seq_sum(0.0, 0, NT - 2, lane, [&](int i) {
      const double g1 = s_gnt[i] + 1.0;
      return (g1 * g1 - 1.0) * s_f[i] * (s_gnt[i + 1] - s_gnt[i]);
    });
    if (lane == 0) {
      s_sc[0] = B; s_sc[1] = K2; s_sc[2] = f_rz; s_sc[7] = s1;
    }
  }
  __syncthreads();
  const double B = s_sc[0], K2 = s_sc[1], f_rz = s_sc[2];
  const double em = 9.109e-28, ee = 4.803e-10, sigmaT = 6.6524616e-25;
  const double nu_b = ee * B / (2 * PI_REF * em * C_LIGHT);
  for (int i = tid; i < NT; i += VEM_BLOCK) {
    const double g0 = s_gnt[i] + 1.0;
    const double gp = g0 * __builtin_sqrt(g0 * g0 - 1.0);
    s_gamp[i] = gp;
    s_q[i] = s_f[i] / gp;
    s_facg[i] = 3.0 * (g0 * g0) * nu_b;
    s_dg[i] = (i < NT - 1) ? s_gnt[i + 1] - s_gnt[i] : 0.0;
  }
  __syncthreads();
  /* ---- one energy per lane ---- */
  if (tid < NV) {
    const int i = tid;
    const double Ub = (B * B) / (8.0 * PI_REF);
    const double face = P.pow3_15 * sigmaT * C_LIGHT * Ub / (PI_REF * nu_b);
    const double dE = P.dE, E = P.E_ph[i];
    const double Theta = tea / 5.11e2;
    const double kappa_C = 6.65e-25 * ne;
    const double nu_c = 2.8e6 * B, nu_min = 5.0 * nu_c, nu_p = 9.0e3 * __builtin_sqrt(ne);
    const double nu = 2.41487e17 * E;
    double j_sy = 0., kappa_sy = 0., j_cy = 0.;
    if (!(nu <= nu_p)) {
      double sum = 0., sum_k = 0.;
      for (int i2 = 0; i2 < NT - 1; i2++) {             /* volume2d.f:205-238 */
        const double tt = nu / s_facg[i2];
        double es = 0.0;
        if (tt < 1.0e4) {
          const double eq43 = expk43(tt), eq13 = expk13(tt);
          const double ff = tt * tt * (eq43 * eq13 - F32(0.6) * tt * (eq43 - eq13) * (eq43 + eq13));
          es = face * ff * c2d_exp_bf(-2.0 * tt);
        }
        const double sd = s_f[i2] * es;
        const double sd_k = s_gamp[i2] * es;
        sum = sum + s_dg[i2] * sd;
        sum_k = sum_k + (s_q[i2] - s_q[i2 + 1]) * sd_k;
      }
      j_sy = sum * ne / (4.0 * PI_REF);
      kappa_sy = sum_k * ne / (8.0 * PI_REF * em * (nu * nu));
      if (kappa_sy < 0.) kappa_sy = -1.0 * kappa_sy;
      double f_m = 1.0;                                  /* cyclotron, :252-300 */
      for (int m = 1; m <= 5; m++) {
        const double mm = (double)m;
        f_m = f_m / (4. * mm);
        const double nu_m = mm * nu_c;
        const double E_m = 4.14e-18 * nu_m;
        const double D_m = 7.07e-1 * Theta * E_m;
        const double q = (E - E_m) / D_m;
        const double x = q * q;
        if (x < 50.) {
          const double f_cy = f_rz * c2d_exp_bf(-x) * ne * (B * B) * c2d_pow(Theta, mm - 1.5) *
                              (mm + 1.0) * f_m * c2d_pow(mm, 2.0 * mm + 1.0);
          j_cy = j_cy + 8.46e-14 * f_cy * (E * E) / (E_m * E_m * E_m);
        }
      }
      if (nu > nu_min) {                                 /* :305-310 */
        const double v = nu / (nu_c * (Theta * Theta));
        const double y = 4.5 * v;
        if (y < 1.0e6)
          j_cy = j_cy + 4.652e-12 * ne * nu /
                            (K2 * c2d_pow(v, 1.6666667e-1) * c2d_exp_bf(c2d_pow(y, 3.33333e-1)));
      }
    }
    P.kappa[(int64_t)cell * NV + i] = kappa_sy;           /* :347 */
    const double lm = zin[VZ_LMIN];
    const double thr = (1.0 / lm > 1.0e1 * kappa_C) ? 1.0 / lm : 1.0e1 * kappa_C;
    double cP = 0.0, cC = 0.0, cT = 0.0;
    if (kappa_sy < thr) {
      cP = j_sy * E * (dE - 1.0);
      cC = j_cy * E * (dE - 1.0);
    } else {
      const double x = E / tea;
      const double tau_tot = kappa_sy * lm;
      double j_th = (x < 1.0e2) ? 1.47e-47 * (nu * nu * nu) / (c2d_exp_bf(x) - 1.0) : 1.0e-50;
      if (tau_tot < 5.0e1) j_th = j_th * (1.0 - c2d_exp_bf(-tau_tot));
      cT = j_th * E * (dE - 1.0);
    }
    s_cP[i] = cP; s_cC[i] = cC; s_cT[i] = cT;
  }
  __syncthreads();
  /* ---- wave 0: the reference's running sums over the energies, in order.
   * Adding the 0 of the branch not taken leaves each sum bit-identical. ---- */
  if (wv == 0) {
    double aP = 0.0, aT = 0.0, aC = 0.0;
    for (int c0 = 0; c0 < NV; c0 += FPB) {
      const int i = c0 + lane;
      const double vP = (i < NV) ? s_cP[i] : 0.0, vT = (i < NV) ? s_cT[i] : 0.0;
      const double vC = (i < NV) ? s_cC[i] : 0.0;
      const int mn = (NV - c0) < FPB ? (NV - c0) : FPB;
      double mP = 0.0, mT = 0.0;
      for (int m = 0; m < mn; m++) {
        aP = aP + rl(vP, m);
        aT = aT + rl(vT, m);
        aC = aC + rl(vC, m);
        if (lane == m) { mP = aP; mT = aT; }
      }
      if (i < NV) { s_P[i] = mP; s_Pth[i] = mT; }
    }
    if (lane == 0) {
      s_sc[3] = aP; s_sc[4] = aT; s_sc[5] = aC;
    }
  }
  __syncthreads();
  if (tid < NV) {
    const double P_sum = s_sc[3], sum_th = s_sc[4];
    P.eps_tot[(int64_t)cell * NV + tid] = (P_sum > 1.0e-50) ? s_P[tid] / P_sum : 0.;
    P.eps_th[(int64_t)cell * NV + tid] = (sum_th > 1.0e-50) ? s_Pth[tid] / sum_th : 0.;
  }
  if (tid == 0) {
    const double vol = zin[VZ_VOL], zs = zin[VZ_ZSURF], dt = P.dt;
    double* o = P.zout + (int64_t)cell * VO_N;
    const double esy = 1.058e-15 * ne * dt * (B * B) * s_sc[7] * vol;   /* :173-174 */
    o[VO_B] = B;
    o[VO_ESY] = esy;
    o[VO_ECY] = dt * vol * s_sc[5];                     /* :320 */
    o[VO_ETH] = dt * zs * s_sc[4];                      /* :324 */
    o[VO_ETOT] = esy;                                   /* :330 */
  }
}

}  // namespace c2d

extern "C" int c2d_launch_vem(const c2d::VemParams* P, int ncell, hipStream_t stream) {
  if (ncell <= 0) return 0;
  hipLaunchKernelGGL(c2d::c2d_vem_kernel, dim3(ncell), dim3(c2d::VEM_BLOCK), 0, stream, *P);
  return (int)hipGetLastError();
}
