/*
 * oracle/c2d_obs_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the per-event loops of the reference's post-processing
 * tools (bbw7561135/Compton2d, postprocessing/): the parity checker for the
 * GPU observer-frame binning (compton2d_amd/csrc/observe.hip).  Only tests/
 * and the bench's CPU baseline load it; the product path never does.
 *
 *   SED mode         postprocessing/pspt.c:245-294  (boost, light-travel time,
 *                    closed mu window, first energy bin, first time bin)
 *   light-curve mode postprocessing/plcm.c:382-456  (time - t_offset >= 0,
 *                    first time bin, first half-open mu bin, every energy band)
 *
 * Events are accumulated in input order, so the sums are the tools' own
 * sequential sums.  Built against glibc libm (liboracle_ref: the tools'
 * cos) and against c2d_math.h (liboracle_det: the GPU's cos).  Pinned to
 * the tools themselves, compiled from their sources into oracle/_ref/, by
 * tests/test_observer.py on the committed fixture tests/golden/obs.npz.
 */
#include <math.h>
#include <stdint.h>

#include "../include/compton2d.h"

#ifdef C2O_DETMATH
#include "../compton2d_amd/csrc/c2d_math.h"
#define O_COS(x) c2d_cos(x)
#else
#define O_COS(x) cos(x)
#endif

int c2o_obs_bin(const c2d_obs_bins* b, const double* ev, int64_t n, double* F, double* F2,
                double* cnt) {
  if (!b || (b->mode != C2D_OBS_SED && b->mode != C2D_OBS_LC)) return C2D_E_ARG;
  const double G = b->gam_bulk;
  const int ne = b->n_e, nm = b->n_mu, nt = b->n_t;
  for (int64_t e = 0; e < n; e++) {
    const double* v = ev + e * C2D_EVENT_WORDS;
    double t_bound = v[0], E = v[1], ew = v[2], r = v[3], z = v[4], mu = v[5], phi = v[6];
    mu = -mu;
    const double betta = sqrt(1. - 1. / (G * G));
    const double doppler = G * (1. + mu * betta);
    t_bound = (t_bound - betta * z * 3.33333333e-11) / doppler;
    E = E * doppler;
    ew = ew * doppler;
    mu = (mu + betta) / (1. + mu * betta);
    const double cdt = z * mu / G + sqrt(1. - mu * mu) * (b->rmax - r * O_COS(phi));
    double time = t_bound + 3.33333333e-11 * cdt;
    int k, m, l;
    if (b->mode == C2D_OBS_SED) {
      if (mu < b->mu0[0] || mu > b->mu1[0]) continue;
      for (k = 0; k < ne; k++)
        if (E >= b->E0[k] && E < b->E1[k]) break;
      for (m = 0; m < nt; m++)
        if (time >= b->t0[m] && time < b->t1[m]) break;
      if (k < ne && m < nt) {
        const int64_t h = (int64_t)m * ne + k;
        F[h] += ew;
        F2[h] += ew * ew;
        cnt[h] += 1.0;
      }
    } else {
      time -= b->t_offset;
      if (time < 0.) continue;
      for (k = 0; k < nt; k++)
        if (time >= b->t0[k] && time < b->t1[k]) break;
      for (m = 0; m < nm; m++)
        if (mu >= b->mu0[m] && mu < b->mu1[m]) break;
      for (l = 0; l < ne; l++)
        if (E >= b->E0[l] && E < b->E1[l] && k < nt && m < nm) {
          const int64_t h = ((int64_t)k * nm + m) * ne + l;
          F[h] += ew;
          F2[h] += ew * ew;
          cnt[h] += 1.0;
        }
    }
  }
  return C2D_OK;
}
