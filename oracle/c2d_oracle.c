/*
 * oracle/c2d_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hot path (bbw7561135/Compton2d,
 * src/ snapshot) used as the parity checker for the HIP engine.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it; the product path (compton2d_amd/) never does.
 *
 * Scope restated here (file:line of the reference followed):
 *   imctrk2d       src/imctrk2d.f:8-708    recursive tracker, split1/2/3
 *   compb2d        src/compb_2d.f:1-318    Klein-Nishina scatter
 *   nth2d          src/nontherm2d.f:159-183 electron sampler
 *   comtot/intg_v/dilog  src/comtot2d.f:1-433 (icoms=6 path :219-247)
 *   imcleak/get_bin      src/imcleak2d.f:2-405 (cr_sent=0 branches)
 *   vol_calc       src/imcvol2d_para.f:90-414
 *   z_surf_calc/r_surf_calc/file_sample  src/imcsurf2d_para.f:228-534,694-788
 *   planck         src/planck2d.f:1-141
 *   field_calc     src/imcfield2d.f:57-144
 *   seed_zone, RNFSTR, RNFARR, fibran, ran1, initialize_*rand  src/rand.f:9-359
 *
 * RNG modes:
 *   C2O_RNG_FIB      the reference's lagged-Fibonacci zone streams with its
 *                    exact reseeding points (rand_switch=1).  With the
 *                    glibc-math build this reproduces the Fortran reference
 *                    bit for bit (pinned in tests/test_oracle_reference.py).
 *   C2O_RNG_RAN1     Numerical-Recipes ran1 (rand_switch=2), one global stream.
 *   C2O_RNG_LINEAGE  the per-packet Philox lineage streams of c2d_rng.h, i.e.
 *                    the same random numbers the HIP kernels draw.  With the
 *                    deterministic-math build (C2O_DETMATH) this reproduces
 *                    the GPU histories bit for bit.
 *
 * Parity pinning: fib mode is checked against outputs of the reference
 * itself, built from /root/reference/src by oracle/ref/build_ref.sh, through
 * the golden fixtures in tests/golden/ (see tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/compton2d.h"
#include "../compton2d_amd/csrc/c2d_rng.h"

#ifdef C2O_DETMATH
#include "../compton2d_amd/csrc/c2d_math.h"
#define LOG c2d_log
#define EXP c2d_exp
#define COS c2d_cos
#define ACOS c2d_acos
#define POW c2d_pow
#else
#include <math.h>
#define LOG log
#define EXP exp
#define COS cos
#define ACOS acos
#define POW pow
#endif
#define SQRT __builtin_sqrt

/* general.pa:23-25; physical constants as the reference spells them */
#define PI_REF 3.1415926536
#define C_LIGHT 2.9979245620e10
#define RAD_CP 3.333564097e-11
#define EMASSKEV 5.11e2
#define SIGTHOM 6.6516e-25
/* Fortran REAL (single precision) literals promoted to double */
#define F32(x) ((double)(float)(x))

#define C2O_RNG_FIB 1
#define C2O_RNG_RAN1 2
#define C2O_RNG_LINEAGE 3

#define RANDMAX 10000
#define KK 100
#define LL 37
#define KKK (KK + KK - 1)

/* ------------------------------------------------------------------ */
/* RNG state                                                           */
/* ------------------------------------------------------------------ */
typedef struct fibstate {
  double ranx[KK + 1];            /* COMMON /RSTATE/ RANX(KK), 1-based  */
  double randlist[RANDMAX + 1];   /* COMMON /rlist/, 1-based            */
  int randcounter;                /* COMMON /rcount/                    */
  /* ran1 SAVE state (rand.f:331-335) */
  int32_t idum, iy, iv[33];
} fibstate;

typedef struct rng {
  int mode;
  uint64_t key;
  uint32_t ctr;
  fibstate* fs;
  uint32_t sub;     /* lineage sub-stream (c2d_rng.h) */
} rng_t;

/* RNFARR (rand.f:230-255) */
static void rnfarr(fibstate* s, double* aa /*1-based*/, int n) {
  int j;
  double y;
  for (j = 1; j <= KK; j++) aa[j] = s->ranx[j];
  for (j = KK + 1; j <= n; j++) {
    y = aa[j - KK] + aa[j - LL];
    aa[j] = y - (double)(int32_t)y;
  }
  for (j = 1; j <= LL; j++) {
    y = aa[n + j - KK] + aa[n + j - LL];
    s->ranx[j] = y - (double)(int32_t)y;
  }
  for (j = LL + 1; j <= KK; j++) {
    y = aa[n + j - KK] + s->ranx[j - LL];
    s->ranx[j] = y - (double)(int32_t)y;
  }
}

/* RNFSTR (rand.f:260-316) */
static void rnfstr(fibstate* st, int32_t seed) {
  const int32_t MM = 1 << 30;
  const double ULP = 1.0 / 4503599627370496.0; /* 2^-52 */
  double u[KKK + 2];
  int32_t sseed, s, t, j;
  double ss, v;
  if (seed < 0)
    sseed = MM - 1 - ((-1 - seed) % MM);
  else
    sseed = seed % MM;
  ss = 2.0 * ULP * (double)(sseed + 2);
  for (j = 1; j <= KK; j++) {
    u[j] = ss;
    ss = ss + ss;
    if (ss >= 1.0) ss = ss - 1.0 + 2.0 * ULP;
  }
  u[2] = u[2] + ULP;
  s = sseed;
  t = 70 - 1;
  for (;;) {
    for (j = KK; j >= 2; j--) {
      u[j + j - 1] = u[j];
      u[j + j - 2] = 0.0;
    }
    for (j = KKK; j >= KK + 1; j--) {
      v = u[j - (KK - LL)] + u[j];
      u[j - (KK - LL)] = v - (double)(int32_t)v;
      v = u[j - KK] + u[j];
      u[j - KK] = v - (double)(int32_t)v;
    }
    if (s % 2 == 1) {
      for (j = KK; j >= 1; j--) u[j + 1] = u[j];
      u[1] = u[KK + 1];
      v = u[LL + 1] + u[KK + 1];
      u[LL + 1] = v - (double)(int32_t)v;
    }
    if (s != 0)
      s = s / 2;
    else
      t = t - 1;
    if (!(t > 0)) break;
  }
  for (j = 1; j <= LL; j++) st->ranx[j + KK - LL] = u[j];
  for (j = LL + 1; j <= KK; j++) st->ranx[j - LL] = u[j];
  for (j = 1; j <= 10; j++) rnfarr(st, u, KKK);
}

/* initialize_rand / _zrand / _rrand (rand.f:99-186) */
static void initialize_rand(fibstate* s, int32_t seed) {
  rnfstr(s, seed);
  rnfarr(s, s->randlist, RANDMAX);
  s->randcounter = 1;
}

/* ran1 (rand.f:322-359): REAL (single) arithmetic in the output stage */
static double ran1(fibstate* s, int32_t* idum) {
  const int32_t IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836, NTAB = 32;
  const int32_t NDIV = 1 + (IM - 1) / NTAB;
  const float AM = 1.0f / (float)IM, RNMX = 1.0f - 1.2e-7f;
  int32_t j, k;
  if (*idum <= 0 || s->iy == 0) {
    *idum = (-*idum > 1) ? -*idum : 1;
    for (j = NTAB + 8; j >= 1; j--) {
      k = *idum / IQ;
      *idum = IA * (*idum - k * IQ) - IR * k;
      if (*idum < 0) *idum += IM;
      if (j <= NTAB) s->iv[j] = *idum;
    }
    s->iy = s->iv[1];
  }
  k = *idum / IQ;
  *idum = IA * (*idum - k * IQ) - IR * k;
  if (*idum < 0) *idum += IM;
  j = 1 + s->iy / NDIV;
  s->iy = s->iv[j];
  s->iv[j] = *idum;
  float a = AM * (float)s->iy;
  float m = a < RNMX ? a : RNMX;
  return (double)(int32_t)(m * 1.e7f) / 1.0e7;
}

/* fibran (rand.f:195-223) */
static int32_t g_ran1_seed;   /* rseed in COMMON /random/ for rand_switch=2 */
static double fibran(fibstate* s) {
  if (s->randcounter >= RANDMAX) {
    rnfarr(s, s->randlist, RANDMAX);
    s->randcounter = 1;
  } else {
    s->randcounter = s->randcounter + 1;
  }
  return s->randlist[s->randcounter];
}

static double U(rng_t* g) {
  if (g->mode == C2O_RNG_LINEAGE) return c2d_draw_s(g->key, g->sub, g->ctr++);
  if (g->mode == C2O_RNG_RAN1) return ran1(g->fs, &g_ran1_seed);
  return fibran(g->fs);
}

static rng_t rng_child(const rng_t* g, uint32_t tag, uint32_t a, uint32_t b) {
  rng_t c = *g;
  if (g->mode == C2O_RNG_LINEAGE) {
    c.key = c2d_derive_s(g->key, tag, a, b, g->sub);
    c.ctr = 0;
    c.sub = 0;
  }
  return c;
}

/* split1 copies: sub-streams of the source stream (c2d_rng.h) */
static rng_t rng_sub(const rng_t* g, uint32_t sub) {
  rng_t c = *g;
  if (g->mode == C2O_RNG_LINEAGE) {
    c.ctr = 0;
    c.sub = sub;
  }
  return c;
}

/* seed_zone (rand.f:9-89): integer lagged Fibonacci initialiser */
static void seed_zone(int32_t* SEED, int nz, int nr, int32_t* seeds, int32_t* zseeds,
                      int32_t* rseeds) {
  enum { SKK = 19937, SLL = 7083, STT = 70, SKKK = SKK + SKK - 1 };
  const int32_t MM = 1 << 30;
  static int32_t X[SKKK + 2];
  int32_t sseed, ss, t, j, k, i;
  if (*SEED < 0)
    sseed = MM - 1 - ((-1 - *SEED) % MM);
  else
    sseed = *SEED % MM;
  ss = sseed - (sseed % 2) + 2;
  for (j = 1; j <= SKK; j++) {
    X[j] = ss;
    ss = ss + ss;
    if (ss >= MM) ss = ss - MM + 2;
  }
  X[2] = X[2] + 1;
  ss = sseed;
  t = STT - 1;
  for (;;) {
    for (j = SKK; j >= 2; j--) {
      X[j + j - 1] = X[j];
      X[j + j - 2] = 0;
    }
    for (j = SKKK; j >= SKK + 1; j--) {
      X[j - (SKK - SLL)] = X[j - (SKK - SLL)] - X[j];
      if (X[j - (SKK - SLL)] < 0) X[j - (SKK - SLL)] += MM;
      X[j - SKK] = X[j - SKK] - X[j];
      if (X[j - SKK] < 0) X[j - SKK] += MM;
    }
    if (ss % 2 == 1) {
      for (j = SKK; j >= 1; j--) X[j + 1] = X[j];
      X[1] = X[SKK + 1];
      X[SLL + 1] = X[SLL + 1] - X[SKK + 1];
      if (X[SLL + 1] < 0) X[SLL + 1] += MM;
    }
    if (ss != 0)
      ss = ss / 2;
    else
      t = t - 1;
    if (!(t > 0)) break;
  }
  i = 0;
  for (j = 1; j <= nz; j++)
    for (k = 1; k <= nr; k++) {
      i = i + 1;
      seeds[(j - 1) * nr + (k - 1)] = X[i];
    }
  for (j = 1; j <= nz; j++) {
    i = i + 1;
    zseeds[j - 1] = X[i];
  }
  /* hazard H2: `x(i) = i+1` with i never incremented (rand.f:77-80) */
  for (k = 1; k <= nr; k++) {
    X[i] = i + 1;
    rseeds[k - 1] = X[i];
  }
  *SEED = seeds[0];
}

/* ------------------------------------------------------------------ */
/* context                                                             */
/* ------------------------------------------------------------------ */
typedef struct pkt {
  double xnu, wmu, phi, rpre, zpre, dcen, ew;
  int jph, kph, jgpsp, jgplc, jgpmu;
} pkt_t;

typedef struct cens_rec {
  double d[6];        /* rpre zpre wmu phi ew xnu */
  int32_t i[5];       /* jgpsp jgplc jgpmu jph kph */
  uint64_t key;       /* lineage key, or fibran seed int(fibran()*1e5) */
} cens_rec;

typedef struct c2o_ctx {
  int nz, nr, ncell;
  double rmin, zmin;
  double z[C2D_MAXZONE + 1], r[C2D_MAXZONE + 1];   /* 1-based */
  double E_ph[C2D_N_VOL + 2], E_field[C2D_NPHFIELD + 2], gnt[C2D_NUM_NT + 2];
  int nphtotal, nph_lc, nmu;
  double hu[C2D_NPHOMAX + 2], Elcmin[C2D_NPHLCMAX + 1], Elcmax[C2D_NPHLCMAX + 1];
  double mu[C2D_NMUMAX + 1];
  int split1, split2, split3, spl3_trg;
  int probe_bundles;            /* lineage mode: split1 probes as bundles (C2O_PROBE_BUNDLES=0: per copy) */
  int spec_switch, cr_sent, pair_switch, kappa_lag, rand_switch;
  int trk2012;                  /* c2d_config.trk_variant == C2D_TRK_2012_11 */
  int rng_mode, h4_stale;
  /* MPI-worker emulation (c2o_set_dt_lag): the workers receive dt only in
   * z_surf_bcast (src/surf_mpi.f:68), after their census and volume jobs,
   * so those see the previous step's dt -- 0 in the first step */
  int dt_lag;
  double dt_prev;
  /* MPI-worker emulation (c2o_set_grid_lag, hazard H12): the workers learn
   * nphtotal, nph_lc, hu and Elcmin/Elcmax only in their first z_surf_bcast
   * (src/surf_mpi.f:24-27,76-81; reader runs on the master alone,
   * src/compton2d.f:23-31), after the first step's census and volume jobs:
   * every spectral / light-curve bin those jobs compute is 0 */
  int grid_lag, grid_seen, grid_missing;
  int rank, world;              /* lineage-sharded sources (global index % world == rank) */
  uint64_t seed;
  double t_bound_last;
  fibstate fs;
  int32_t rseed;
  int32_t seeds[C2D_MAXZONE * C2D_MAXZONE], zseeds[C2D_MAXZONE], rseeds[C2D_MAXZONE];
  /* per-cell tables, cell-major */
  double *kappa, *kappa_prev, *kappa_use, *eps_tot, *eps_th, *f_nt, *Pnt;
  double *n_e, *Eloss_th, *Eloss_tot, *zsurf, *ewsv;
  int32_t* nsv;
  int have_prev_kappa;
  /* comtot cache for one imctrk2d(-1) call (imctrk2d.f:102-103,170-178) */
  double* comac_ar;
  int64_t* comac_stamp;
  int64_t comac_call;
  /* step */
  int ncycle;
  double time, dt;
  const c2d_step_in* in;
  uint64_t step_key;
  /* tallies */
  c2d_tally_layout L;
  double* T;
  /* census */
  cens_rec *cin, *cout;
  int64_t nin, nout, ccap;
  /* events */
  double* ev;
  int64_t nev, evcap;
  int err;
} c2o_ctx;

#define CELL(c, j, k) (((j) - 1) * (c)->nr + ((k) - 1))
#define TALLY(c, off) ((c)->T[(c)->L.off])

/* ------------------------------------------------------------------ */
/* comtot (comtot2d.f:1-334, icoms=6 :219-247), intg_v, dilog           */
/* ------------------------------------------------------------------ */
static double dilog(double x) {
  static const double C[21] = {0,
      0.42996693560813697, 0.40975987533077105, -0.01858843665014592,
      0.00145751084062268, -0.00014304184442340, 0.1588415541880e-4,
      -0.190784959387e-5, 0.024195180854e-5, -0.003193341274e-5,
      0.000434545063e-5, -0.000060578480e-5, 0.000008612098e-5,
      -0.000001244332e-5, 0.000000182256e-5, -0.000000027007e-5,
      0.000000004042e-5, -0.000000000610e-5, 0.000000000093e-5,
      -0.000000000014e-5, 0.000000000002e-5};
  const double HF = 0.5, PI2 = PI_REF * PI_REF, PI3 = PI2 / 3, PI6 = PI2 / 6,
               PI12 = PI2 / 12;
  double T, H, Y, S, A, ALFA, B1, B2, B0 = 0.0;
  int i;
  if (x == 1) {
    H = PI6;
  } else if (x == -1) {
    H = -PI12;
  } else {
    T = -x;
    if (T <= -2) {
      Y = -1 / (1 + T);
      S = 1;
      B1 = LOG(-T);
      B2 = LOG(1 + 1 / T);
      A = -PI3 + HF * (B1 * B1 - B2 * B2);
    } else if (T < -1) {
      Y = -1 - T;
      S = -1;
      A = LOG(-T);
      A = -PI6 + A * (A + LOG(1 + 1 / T));
    } else if (T <= -0.5) {
      Y = -(1 + T) / T;
      S = 1;
      A = LOG(-T);
      A = -PI6 + A * (-HF * A + LOG(1 + T));
    } else if (T < 0) {
      Y = -T / (1 + T);
      S = -1;
      B1 = LOG(1 + T);
      A = HF * B1 * B1;
    } else if (T <= 1) {
      Y = T;
      S = 1;
      A = 0;
    } else {
      Y = 1 / T;
      S = -1;
      B1 = LOG(T);
      A = PI6 + HF * B1 * B1;
    }
    H = Y + Y - 1;
    ALFA = H + H;
    B1 = 0;
    B2 = 0;
    for (i = 20; i >= 1; i--) {
      B0 = C[i] + ALFA * B1 - B2;
      B2 = B1;
      B1 = B0;
    }
    H = -(S * (B0 - H * B2) + A);
  }
  return H;
}

static double intg_v(double x) {
  double i1 = -x / 2.0 + 0.5 / (1.0 + x);
  double i2 = 4.0 * dilog(-x);
  double i3 = (9.0 + x + 8.0 / x) * LOG(1.0 + x);
  return i1 + i2 + i3;
}

static double comtot_cell(const c2o_ctx* c, int cell, double xnuc) {
  const double* fnt = c->f_nt + (int64_t)cell * C2D_NUM_NT;  /* fnt[i-1] = f_nt(j,k,i) */
  double cosig = 0.0, x = xnuc / EMASSKEV;
  for (int i = 1; i <= C2D_NUM_NT - 1; i++) {
    double gamma0 = c->gnt[i] + 1.0;
    double betta = SQRT(1.0 - 1.0 / (gamma0 * gamma0));
    double sigma_E;
    if (x * gamma0 * (1 + betta) < 1.0e-2)
      sigma_E = SIGTHOM * (1.0 - 2.0 * x * gamma0);
    else
      sigma_E = 9.375e-2 * SIGTHOM / (gamma0 * gamma0) / betta / (x * x) *
                (intg_v(2 * gamma0 * (1 + betta) * x) - intg_v(2 * gamma0 * (1 - betta) * x));
    cosig = cosig + sigma_E * fnt[i - 1] * (c->gnt[i + 1] - c->gnt[i]);
  }
  if (cosig < 1.0e-40) return 1.0e-40;
  return c->n_e[cell] * cosig;
}

/* ------------------------------------------------------------------ */
/* binning helpers                                                     */
/* ------------------------------------------------------------------ */
/* jgpsp by bisection over hu (compb_2d.f:249-274 etc.).  hubot/hutop factors
 * differ per caller (REAL vs DOUBLE literals); `top_value` is what the caller
 * assigns when xnu >= hutop (vol_calc uses nphtotal, all others 0). */
static int bin_sp(const c2o_ctx* c, double xnu, double fbot, double ftop, int top_value) {
  /* H12: nphtotal = 0 on the worker, so jtop = 1 and hutop = 0.999999*hu(1)
   * with hu not yet broadcast: every xnu takes the top branch, jgpsp = 0 */
  if (c->grid_missing) return 0;
  int jbot = 1, jtop = c->nphtotal + 1, jmid;
  double hubot = fbot * c->hu[1];
  double hutop = ftop * c->hu[jtop];
  if (xnu >= hutop) return top_value;
  if (xnu <= hubot) return 0;
  for (;;) {
    jmid = (jbot + jtop) / 2;
    if (jmid == jbot) break;
    if (xnu == c->hu[jmid]) break;
    if (xnu < c->hu[jmid])
      jtop = jmid;
    else
      jbot = jmid;
  }
  return jmid;
}

static int bin_lc(const c2o_ctx* c, double xnu) {
  if (c->grid_missing) return 0;            /* H12: nph_lc = 0 on the worker */
  for (int m = 1; m <= c->nph_lc; m++)
    if (xnu > c->Elcmin[m] && xnu <= c->Elcmax[m]) return m;
  return 0;
}

static int bin_mu(const c2o_ctx* c, double wmu) {
  for (int n = 1; n <= c->nmu; n++)
    if (wmu <= c->mu[n]) return n;
  return c->nmu;
}

static double clampd(double v, double lim) {
  if (v > lim) v = lim;
  if (v < -lim) v = -lim;
  return v;
}

/* ------------------------------------------------------------------ */
/* nth2d (nontherm2d.f:159-183) and compb2d (compb_2d.f:1-318)          */
/* ------------------------------------------------------------------ */
static int nth2d(c2o_ctx* c, int cell, rng_t* g, double* gamm, double* betb) {
  const double* P = c->Pnt + (int64_t)cell * C2D_NUM_NT;   /* P[i-1] = Pnt(j,k,i) */
  double rnum = U(g);
  rnum = (double)(int32_t)(rnum * 1.0e6) / 1.0e6 + 1.0e-6 * U(g);
  int i;
  for (i = 2; i <= C2D_NUM_NT; i++)
    if (P[i - 1] > rnum) break;
  *gamm = SQRT(c->gnt[i] * c->gnt[i - 1]) + 1.0;
  *betb = SQRT(1.0 - 1.0 / ((*gamm) * (*gamm)));
  TALLY(c, nelectron + i) += 1.0;
  return i;
}

static int compb2d(c2o_ctx* c, pkt_t* p, rng_t* g) {
  const double fuzz = 1.0e-10, lim = 9.9999999e-1;
  int cell = CELL(c, p->jph, p->kph);
  double znu = p->xnu / EMASSKEV;
  double gamm, betb, omeg, tl, tr, znue, znue3, betz, gamz, xxx, xknot;
  double sz, games, phat, znues, wa, wb, swa, cazes, omege, omeges, omegs, znus, gams;
  double cazs, wmus, xnus, cosdphi, dphi, phis;
  int i_gam;
  TALLY(c, counters + C2D_CNT_COMPB) += 1.0;
  /* lineage mode: iteration j of label 100 draws from counters ctr0 + 5j ..
   * ctr0 + 5j + 4 (a znue < 1e-10 skip leaves the fifth unused), so that the
   * GPU can run iterations of one packet wave-parallel (transport.hip kn_iter) */
  const uint32_t ctr0 = g->ctr;
  uint32_t jit = 0;
  for (;; jit++) {                                      /* label 100 */
    if (g->mode == C2O_RNG_LINEAGE) g->ctr = ctr0 + 5u * jit;
    i_gam = nth2d(c, cell, g, &gamm, &betb);
    omeg = 2.0 * U(g) - 1.0;
    omeg = clampd(omeg, lim);
    tl = U(g);
    tr = 0.5 * (1.0 - betb * omeg);
    if (tl > tr) omeg = -omeg;
    omeg = clampd(omeg, lim);
    znue = (1.0 - betb * omeg) * znu * gamm;
    if (znue < 1.0e-10) continue;
    if (znue <= 1.0e-2) {
      xknot = 1.0 - znue * (2.0 - znue * (5.2 - znue * (13.3 - 1.144e3 * znue / 3.5e1)));
    } else {
      znue3 = znue * znue * znue;
      betz = 1.0 + 2.0 * znue;
      gamz = znue * (znue - 2.0) - 2.0;
      xxx = 4.0 * znue + 2.0 * znue3 * (1.0 + znue) / (betz * betz) + gamz * LOG(betz);
      xknot = 3.75e-1 * xxx / znue3;
    }
    if (U(g) > xknot) continue;
    break;
  }
  if (g->mode == C2O_RNG_LINEAGE) g->ctr = ctr0 + 5u * (jit + 1u);
  betz = 1.0 + 2.0 * znue;
  for (;;) {                                            /* labels 200/202 */
    sz = (1.0 + 2.0 * znue * U(g)) / betz;
    games = 1.0 + (1.0 - 1.0 / sz) / znue;
    if ((1.0 - games * games) < 0.0) continue;
    tr = games * games - 1.0 + sz + 1.0 / sz;
    phat = betz + 1.0 / betz;
    if (U(g) * phat > tr) continue;
    break;
  }
  znues = znue * sz;
  for (;;) {                                            /* label 210 */
    wa = U(g);
    wb = 2.0 * U(g) - 1.0;
    swa = wa * wa + wb * wb;
    if (swa >= 1.0 || swa <= 1.0e-20) continue;
    break;
  }
  cazes = (wa * wa - wb * wb) / swa;
  omege = (omeg - betb) / (1.0 - betb * omeg);
  omege = clampd(omege, lim);
  omeges = games * omege + cazes * SQRT((1.0 - omege * omege + fuzz) * (1.0 - games * games));
  omeges = clampd(omeges, lim);
  omegs = (omeges + betb) / (1.0 + omeges * betb);
  omegs = clampd(omegs, lim);
  (void)omegs;
  znus = (1.0 + betb * omeges) * gamm * znues;
  gams = 1.0 - (znue - znues) / (znu * znus);
  gams = clampd(gams, lim);
  for (;;) {                                            /* label 220 */
    wa = U(g);
    wb = 2.0 * U(g) - 1.0;
    swa = wa * wa + wb * wb;
    if (swa >= 1.0 || swa <= 1.0e-20) continue;
    break;
  }
  cazs = (wa * wa - wb * wb) / swa;
  cazs = clampd(cazs, lim);
  wmus = p->wmu * gams + cazs * SQRT((1.0 - gams * gams) * (1.0 - p->wmu * p->wmu + fuzz));
  wmus = clampd(wmus, lim);
  xnus = znus * EMASSKEV;
  cosdphi = (gams - p->wmu * wmus) / SQRT((1.0 - p->wmu * p->wmu) * (1.0 - wmus * wmus));
  cosdphi = clampd(cosdphi, lim);
  dphi = ACOS(cosdphi);
  phis = p->phi + dphi;
  p->jgpsp = bin_sp(c, xnus, 1.000001, 0.999999, 0);
  p->jgplc = bin_lc(c, xnus);
  p->jgpmu = bin_mu(c, wmus);
  p->ew = p->ew * xnus / p->xnu;
  p->xnu = xnus;
  p->wmu = wmus;
  p->phi = phis;
  return i_gam;
}

/* ------------------------------------------------------------------ */
/* imcleak (imcleak2d.f:2-320), cr_sent = 0                             */
/* ------------------------------------------------------------------ */
static void push_event(c2o_ctx* c, double t_bound, const pkt_t* p) {
  if (c->nev >= c->evcap) {
    c->evcap = c->evcap ? c->evcap * 2 : 4096;
    c->ev = (double*)realloc(c->ev, sizeof(double) * C2D_EVENT_WORDS * c->evcap);
  }
  double* e = c->ev + C2D_EVENT_WORDS * c->nev++;
  e[0] = t_bound; e[1] = p->xnu; e[2] = p->ew; e[3] = p->rpre;
  e[4] = p->zpre; e[5] = p->wmu; e[6] = p->phi;
  TALLY(c, counters + C2D_CNT_EVENTS) += 1.0;
}

static void escape_tally(c2o_ctx* c, const pkt_t* p) {
  if (p->jgplc > 0)
    c->T[c->L.edout + (p->jgpmu - 1) * C2D_NPHLCMAX + (p->jgplc - 1)] += p->ew / c->dt;
  if (p->jgpsp > 0 && c->spec_switch == 0)
    c->T[c->L.fout + (p->jgpmu - 1) * C2D_NPHOMAX + (p->jgpsp - 1)] += p->ew;
}

static int imcleak(c2o_ctx* c, pkt_t* p) {
  const c2d_step_in* in = c->in;
  if (p->kph == 0) {
    if (c->rmin > 1.0e-10) {
      c->T[c->L.erlki + p->jph - 1] += p->ew;
      TALLY(c, counters + C2D_CNT_ESCAPES) += 1.0;
      return 1;
    }
    p->phi = 1.0e-6;
    p->kph = 1;
    return 0;
  }
  TALLY(c, counters + C2D_CNT_ESCAPES) += 1.0;
  if (p->jph <= 0) {                                   /* lower z surface */
    if (in->tbbl && in->tbbl[p->kph - 1] > 0.0) {
      c->T[c->L.Ed_in + p->kph - 1] += p->ew;
      c->T[c->L.erlkl + p->kph - 1] += p->ew;
    }
    if (c->ncycle > 0) {
      /* hazard H4: the reference writes a stale COMMON t_bound here */
      double tb = c->h4_stale ? c->t_bound_last : c->time + c->dt - RAD_CP * p->dcen;
      push_event(c, tb, p);
      escape_tally(c, p);
    }
    return 1;
  }
  if (p->jph != c->nz + 1) {                           /* outer r surface */
    c->T[c->L.erlko + p->jph - 1] += p->ew;
    double tb = c->time + c->dt - RAD_CP * p->dcen;
    c->t_bound_last = tb;
    if (c->ncycle > 0) {
      push_event(c, tb, p);
      escape_tally(c, p);
    }
    return 1;
  }
  /* upper z surface (label 500) */
  c->T[c->L.erlku + p->kph - 1] += p->ew;
  double tb = c->time + c->dt - RAD_CP * p->dcen;
  c->t_bound_last = tb;
  if (c->ncycle > 0 && p->wmu < F32(0.98)) {
    push_event(c, tb, p);
    escape_tally(c, p);
  }
  return 1;
}

/* ------------------------------------------------------------------ */
/* imctrk2d (imctrk2d.f:8-708)                                          */
/* ------------------------------------------------------------------ */
static void imctrk2d(c2o_ctx* c, pkt_t* p, int scat_flag, rng_t* g);

static void census_write(c2o_ctx* c, pkt_t* p, rng_t* g) {
  int cell = CELL(c, p->jph, p->kph);
  c->T[c->L.npcen + cell] += 1.0;
  c->T[c->L.ecens + cell] += p->ew;
  int i;
  for (i = 1; i <= C2D_NPHFIELD - 1; i++)
    if (p->xnu < c->E_field[i + 1]) break;
  double Egg_min = (c->E_field[1] * c->E_field[1]) / c->E_field[2];
  if (p->xnu > Egg_min)
    c->T[c->L.n_field + (int64_t)cell * C2D_NPHFIELD + (i - 1)] += 6.25e8 * p->ew / p->xnu;
  if (c->nout >= c->ccap) {
    c->err = C2D_E_CENSUS_OVERFLOW;
    return;
  }
  cens_rec* q = &c->cout[c->nout++];
  q->d[0] = p->rpre; q->d[1] = p->zpre; q->d[2] = p->wmu;
  q->d[3] = p->phi; q->d[4] = p->ew; q->d[5] = p->xnu;
  q->i[0] = p->jgpsp; q->i[1] = p->jgplc; q->i[2] = p->jgpmu;
  q->i[3] = p->jph; q->i[4] = p->kph;
  if (g->mode == C2O_RNG_LINEAGE)
    q->key = c2d_census_key(g->key, g->ctr, g->sub);
  else
    q->key = (uint64_t)(int64_t)(int32_t)(U(g) * 1.0e5);
  TALLY(c, counters + C2D_CNT_CENSUS) += 1.0;
}

static void collision(c2o_ctx* c, pkt_t* p, int scat_flag, rng_t* g) {
  const double twopi = 2.0 * PI_REF;
  pkt_t csv = *p;
  double ewcsv = csv.ew / c->split2;
  double thr_mul = (double)c->split2 * (double)c->split1 * (double)c->spl3_trg;
  (void)scat_flag;
  TALLY(c, counters + C2D_CNT_COLLIDE) += 1.0;
  uint32_t ctr_par = g->ctr;
  for (int ii = 0; ii < c->split2; ii++) {
    *p = csv;
    p->ew = ewcsv;
    rng_t gc = rng_child(g, C2D_TAG_SCAT2, (uint32_t)ii, ctr_par);
    double ewold = p->ew;
    int i_gam = compb2d(c, p, &gc);
    if (p->ew > ewold * c->split2 * c->split1 * c->spl3_trg) {
      (void)thr_mul;
      ewold = ewcsv / c->split3;
      uint32_t ctr_chd = gc.ctr;
      for (int ii2 = 0; ii2 < c->split3; ii2++) {
        rng_t g3 = rng_child(&gc, C2D_TAG_SCAT3, (uint32_t)ii2, ctr_chd);
        rng_t* g3p = (gc.mode == C2O_RNG_LINEAGE) ? &g3 : &gc;
        /* lineage mode: resample k draws from sub-stream k of the copy's key
         * (c2d_rng.h), so the attempts are independent of one another and the
         * GPU evaluates them in parallel (transport.hip scatter kernels);
         * the packet flies on from the first success's stream */
        uint32_t attempt = 0;
        do {
          *p = csv;
          p->ew = ewcsv / c->split3;
          if (gc.mode == C2O_RNG_LINEAGE) {
            g3.sub = attempt;
            g3.ctr = 0;
          }
          attempt++;
          i_gam = compb2d(c, p, g3p);
        } while (p->ew <= ewold * c->split2 * c->split1 * c->spl3_trg);
        int cell = CELL(c, p->jph, p->kph);
        c->T[c->L.edep + cell] = c->T[c->L.edep + cell] + p->ew - ewold;
        c->T[c->L.E_IC + i_gam] = c->T[c->L.E_IC + i_gam] + p->ew - ewold;
        if (p->phi > twopi) p->phi = p->phi - twopi;
        imctrk2d(c, p, 1, g3p);
      }
    } else {
      int cell = CELL(c, p->jph, p->kph);
      c->T[c->L.edep + cell] = c->T[c->L.edep + cell] + p->ew - ewold;
      c->T[c->L.E_IC + i_gam] = c->T[c->L.E_IC + i_gam] + p->ew - ewold;
      if (p->phi > twopi) p->phi = p->phi - twopi;
      imctrk2d(c, p, 1, &gc);
    }
  }
}

/* one packet copy: label 100 ... 900 of imctrk2d.f; returns 1 if it scattered */
static int flight_loop(c2o_ctx* c, pkt_t* p, int s, rng_t* g, double wtmin) {
  /* src/imctrk2d.f clamps |wmu| to 0.99999999 at label 110 and |Eta| to
   * 0.99999999 / 0.999999999; src_20121113 clamps both to 1 (:162-167, :481-484) */
  const int v12 = c->trk2012;
  const double lim8 = v12 ? 1.0 : 9.9999999e-1, lim9 = v12 ? 1.0 : 0.999999999;
  double colmfp = 0.0;
  int at100 = 1;
  for (;;) {
    double sigabs = 1.0e-40, mb_ran;                   /* label 100 */
    if (at100) {
      if (s == 0) {
        mb_ran = 1.0e-10;
      } else {
        mb_ran = U(g);
        if (c->rand_switch == 2) mb_ran = (double)(int32_t)(mb_ran * 1.0e6) / 1.0e6 + 1.0e-6 * U(g);
      }
      if (!(mb_ran > 0.0)) continue;
      colmfp = -LOG(mb_ran);
    }
    /* after a cell boundary src re-enters at label 100 (a fresh colmfp,
     * imctrk2d.f:518-525), src_20121113 at label 110 (:526-533) */
    at100 = !v12;
    if (p->ew < 1.0e-40) return 0;                     /* label 110 */
    p->wmu = clampd(p->wmu, lim8);
    int cell = CELL(c, p->jph, p->kph);
    double comac;
    if (s == -1) {
      if (c->comac_stamp[cell] == c->comac_call) {
        comac = c->comac_ar[cell];
      } else {
        comac = comtot_cell(c, cell, p->xnu);
        c->comac_ar[cell] = comac;
        c->comac_stamp[cell] = c->comac_call;
      }
    } else if (s == 1) {
      comac = comtot_cell(c, cell, p->xnu);
    } else {
      comac = 0.0;
    }
    double sigsc = comac;                              /* velfact = pair_enhance = 1 */
    double xqsqleft = (p->kph == 1) ? c->rmin * c->rmin : c->r[p->kph - 1] * c->r[p->kph - 1];
    double dcol;
    if (s != 0)
      dcol = colmfp / sigsc;
    else
      dcol = 100 * (c->r[c->nr] > c->z[c->nz] ? c->r[c->nr] : c->z[c->nz]);
    double trld;
    int ikind;
    if (p->dcen <= dcol) { trld = p->dcen; ikind = 2; }
    else { trld = dcol; ikind = 3; }
    TALLY(c, counters + C2D_CNT_STEPS) += 1.0;
    /* geometry (imctrk2d.f:228-379) */
    double Eta = COS(p->phi);
    int eta_switch = (p->phi <= PI_REF && p->phi >= 1.0e-10) ? 1 : -1;
    if (!v12) Eta = clampd(Eta, lim8);                 /* commented out in src_20121113:248-249 */
    double rpre = p->rpre, zpre = p->zpre, wmu = p->wmu;
    double disp = Eta * rpre;
    double psq = rpre * rpre * (1.0 - Eta * Eta);
    int kbnd, inout, knew, jnew;
    double rbnd, Zbnd, Rr, f;
    if (Eta < 0.0 && psq < xqsqleft) {
      kbnd = p->kph - 1;
      inout = -1;
      rbnd = (p->kph > 1) ? c->r[p->kph - 1] : c->rmin;
    } else {
      kbnd = p->kph;
      inout = 1;
      rbnd = c->r[p->kph];
    }
    double dpbsq = rbnd * rbnd - psq;
    if (dpbsq < 1.0e-6) dpbsq = 1.0e-6;
    double disbr = (double)inout * SQRT(dpbsq) - disp;
    double trldb = disbr / SQRT(1.0 - wmu * wmu);
    f = disbr;
    double Zr = zpre + wmu * trldb;
    double zlow = (p->jph == 1) ? c->zmin : c->z[p->jph - 1];
    if (Zr > c->z[p->jph]) {
      Zbnd = c->z[p->jph];
      knew = p->kph;
      jnew = p->jph + 1;
      f = (Zbnd - zpre) * SQRT(1.0 - wmu * wmu) / wmu;
      Rr = SQRT(rpre * rpre + f * f + 2.0 * rpre * f * Eta);
      rbnd = Rr;
      trldb = SQRT(f * f + (Zbnd - zpre) * (Zbnd - zpre));
    } else if (Zr < zlow) {
      Zbnd = zlow;
      knew = p->kph;
      jnew = p->jph - 1;
      f = (zlow - zpre) * SQRT(1.0 - wmu * wmu) / wmu;
      Rr = SQRT(rpre * rpre + f * f + 2.0 * rpre * f * Eta);
      rbnd = Rr;
      trldb = SQRT(f * f + (Zbnd - zpre) * (Zbnd - zpre));
    } else {
      knew = p->kph + inout;
      jnew = p->jph;
      Rr = (kbnd > 0) ? c->r[kbnd] : c->rmin;
      rbnd = Rr;
      Zbnd = Zr;
    }
    double rnew, znew;
    if (trldb < trld) {
      ikind = 1;
      trld = trldb;
      rnew = rbnd;
      znew = Zbnd;
    } else {
      jnew = p->jph;
      knew = p->kph;
      f = trld * SQRT(1.0 - wmu * wmu);
      rnew = SQRT(f * f + rpre * rpre + 2.0 * f * rpre * Eta);
      znew = zpre + trld * wmu;
    }
    /* absorption (imctrk2d.f:382-462) */
    int i;
    for (i = 1; i <= C2D_N_VOL - 1; i++)
      if (p->xnu < c->E_ph[i + 1]) break;
    sigabs = sigabs + 1.0 * c->kappa_use[(int64_t)cell * C2D_N_VOL + (i - 1)];
    if (sigabs < 1.0e-40) sigabs = 1.0e-40;
    double xabs = sigabs * trld;
    double ewnew = (xabs < 100.0) ? p->ew * EXP(-xabs) : 0.0;
    /* pair_switch=1 branches (imctrk2d.f:386-407,429-431) are treated as
     * gamma-gamma opacity 0 (hazard H6: k_gg/E_gg never reach the workers). */
    double deleabs = p->ew - ewnew;
    if (deleabs < 1.0e-50) deleabs = 1.0e-50;
    double wmustar;
    if (xabs <= 0.00001) {
      wmustar = wmu;
    } else {
      double mr, sstar;
      for (;;) {
        mr = U(g);
        if (mr < p->ew / deleabs) {
          sstar = -LOG(1.0 - mr * deleabs / p->ew) / sigabs;
          break;
        }
      }
      double denom = SQRT(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
      wmustar = (wmu * rpre + sstar) / denom;
    }
    double delpr = deleabs * wmustar * C_LIGHT;
    if (s != 0) {
      c->T[c->L.edep + cell] = c->T[c->L.edep + cell] + deleabs;
      c->T[c->L.prdep + cell] = c->T[c->L.prdep + cell] + delpr;
    }
    if (ewnew <= wtmin) {
      TALLY(c, counters + C2D_CNT_KILLED) += 1.0;
      return 0;
    }
    p->ew = ewnew;
    p->dcen = p->dcen - trld;
    if (v12)
      Eta = (f + Eta * rpre) / rnew;                   /* src_20121113/imctrk2d.f:478 */
    else
      Eta = (trld + Eta * rpre) / rnew;                /* hazard H1: trld, not f */
    Eta = clampd(Eta, lim9);
    p->phi = ACOS(Eta);
    if (eta_switch == -1) p->phi = 2.0 * PI_REF - p->phi;
    p->rpre = rnew;
    p->zpre = znew;
    if (ikind == 1) {
      colmfp = colmfp - sigsc * trld;                  /* imctrk2d.f:497 / src_20121113:505 */
      if (jnew == c->nz + 1 || jnew == 0 || knew == c->nr + 1 || knew == 0) {
        p->jph = jnew;
        p->kph = knew;
        if (s == -1) return 0;
        if (imcleak(c, p) == 1) {
          if (s == 1) TALLY(c, counters + C2D_CNT_ESC_SCAT) += 1.0;
          return 0;
        }
        continue;
      }
      p->kph = knew;
      p->jph = jnew;
      continue;
    } else if (ikind == 2 && s != -1) {
      census_write(c, p, g);
      return 0;
    } else if (ikind == 3) {
      collision(c, p, s, g);
      return 1;
    }
    return 0;
  }
}

/* Lineage mode: the split1 probe copies of a source (imctrk2d(-1),
 * imctrk2d.f:106-123) as probe bundles, the way the GPU's bundle kernel
 * tracks them.  The probes of a source differ only in their
 * random numbers, so they fly one shared path until a probe collides.  Their
 * collision processes are independent with the same rate sigsc, so the first
 * collision among n of them is exponential with rate n*sigsc; the collider is
 * uniform among them; by memorylessness the others continue unchanged.  A
 * bundle of G = min(split1 - g0, C2O_BUNDLE_MAX) probes draws from one stream
 * (source key, C2D_SUB_BUNDLE | g0):
 *   at the start              tau = -log(u)/n   (optical depth, per probe, to the
 *                                                next collision among the n)
 *   per collision             u -> the collider (k-th of the n alive, k = int(u*n)),
 *                             u -> its absorption point (xabs > 1e-5 only),
 *                             u -> tau of the n-1 others from the collision point
 *   per step, survivors       each one's absorption point (xabs > 1e-5), in probe
 *                             order, from the point stream (key, C2D_SUB_ABSPT | g0):
 *                             two 32-bit uniforms per output, fresh outputs per step
 * Per copy, the geometry, absorption, deposits, collision records and
 * counters are the per-copy tracker's (flight_loop with s = -1); only the
 * random numbers that decide the collisions are drawn per bundle instead of
 * per copy and step.  Returns the probes that scattered. */
#define C2O_BUNDLE_MAX 32
static int probe_bundle(c2o_ctx* c, const pkt_t* src, double s_ew, double wtmin, int g0, int G,
                        const rng_t* g) {
  const int v12 = c->trk2012;
  const double lim8 = v12 ? 1.0 : 9.9999999e-1, lim9 = v12 ? 1.0 : 0.999999999;
  rng_t gb = rng_sub(g, C2D_SUB_BUNDLE | (uint32_t)g0);
  uint32_t actr = 0;                                 /* point-stream outputs */
  pkt_t p = *src;
  p.ew = s_ew;
  uint32_t alive = G >= 32 ? 0xffffffffu : ((1u << G) - 1u);
  int n = G, nscat = 0;
  double tau = -LOG(U(&gb)) / (double)n;
  for (;;) {
    if (p.ew < 1.0e-40) return nscat;                  /* label 110, every probe */
    p.wmu = clampd(p.wmu, lim8);
    int cell = CELL(c, p.jph, p.kph);
    double comac;
    if (c->comac_stamp[cell] == c->comac_call) {
      comac = c->comac_ar[cell];
    } else {
      comac = comtot_cell(c, cell, p.xnu);
      c->comac_ar[cell] = comac;
      c->comac_stamp[cell] = c->comac_call;
    }
    const double sigsc = comac;
    TALLY(c, counters + C2D_CNT_STEPS) += (double)n;
    /* geometry (imctrk2d.f:228-379), shared */
    double xqsqleft = (p.kph == 1) ? c->rmin * c->rmin : c->r[p.kph - 1] * c->r[p.kph - 1];
    double Eta = COS(p.phi);
    int eta_switch = (p.phi <= PI_REF && p.phi >= 1.0e-10) ? 1 : -1;
    if (!v12) Eta = clampd(Eta, lim8);
    const double rpre = p.rpre, zpre = p.zpre, wmu = p.wmu;
    double disp = Eta * rpre;
    double psq = rpre * rpre * (1.0 - Eta * Eta);
    int kbnd, inout, knew, jnew;
    double rbnd, Zbnd, f;
    if (Eta < 0.0 && psq < xqsqleft) {
      kbnd = p.kph - 1;
      inout = -1;
      rbnd = (p.kph > 1) ? c->r[p.kph - 1] : c->rmin;
    } else {
      kbnd = p.kph;
      inout = 1;
      rbnd = c->r[p.kph];
    }
    double dpbsq = rbnd * rbnd - psq;
    if (dpbsq < 1.0e-6) dpbsq = 1.0e-6;
    double disbr = (double)inout * SQRT(dpbsq) - disp;
    double trldb = disbr / SQRT(1.0 - wmu * wmu);
    f = disbr;
    double Zr = zpre + wmu * trldb;
    double zlow = (p.jph == 1) ? c->zmin : c->z[p.jph - 1];
    if (Zr > c->z[p.jph] || Zr < zlow) {
      Zbnd = (Zr > c->z[p.jph]) ? c->z[p.jph] : zlow;
      knew = p.kph;
      jnew = (Zr > c->z[p.jph]) ? p.jph + 1 : p.jph - 1;
      f = (Zbnd - zpre) * SQRT(1.0 - wmu * wmu) / wmu;
      rbnd = SQRT(rpre * rpre + f * f + 2.0 * rpre * f * Eta);
      trldb = SQRT(f * f + (Zbnd - zpre) * (Zbnd - zpre));
    } else {
      knew = p.kph + inout;
      jnew = p.jph;
      rbnd = (kbnd > 0) ? c->r[kbnd] : c->rmin;
      Zbnd = Zr;
    }
    /* a copy that does not collide: boundary (ikind 1) or census (ikind 2) */
    const int bnd = trldb < p.dcen;
    const double trld = bnd ? trldb : p.dcen;
    int ie;
    for (ie = 1; ie <= C2D_N_VOL - 1; ie++)
      if (p.xnu < c->E_ph[ie + 1]) break;
    double sigabs = 1.0e-40 + 1.0 * c->kappa_use[(int64_t)cell * C2D_N_VOL + (ie - 1)];
    if (sigabs < 1.0e-40) sigabs = 1.0e-40;
    /* collisions inside the step (ikind 3: dcol < dcen and not trldb < dcol) */
    double dpos = 0.0;
    while (n > 0) {
      const double dcol = dpos + tau / sigsc;
      if (!(dcol < p.dcen && !(trldb < dcol))) break;
      int k = (int)(U(&gb) * (double)n);
      if (k > n - 1) k = n - 1;
      int i = 0;
      for (uint32_t m = alive;; m &= m - 1u) {
        if (k-- == 0) { i = __builtin_ctz(m); break; }
      }
      alive &= ~(1u << i);
      n--;
      /* the collider's partial step to dcol (flight_loop, ikind = 3) */
      pkt_t q = p;
      const double trc = dcol;
      const double fc = trc * SQRT(1.0 - wmu * wmu);
      const double rnew = SQRT(fc * fc + rpre * rpre + 2.0 * fc * rpre * Eta);
      const double znew = zpre + trc * wmu;
      const double xabs = sigabs * trc;
      const double ewnew = (xabs < 100.0) ? p.ew * EXP(-xabs) : 0.0;
      double deleabs = p.ew - ewnew;
      if (deleabs < 1.0e-50) deleabs = 1.0e-50;
      double wmustar = wmu;
      if (xabs > 0.00001) {
        const double mr = U(&gb);                      /* mr < 1 <= ew/deleabs */
        const double sstar = -LOG(1.0 - mr * deleabs / p.ew) / sigabs;
        const double denom = SQRT(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
        wmustar = (wmu * rpre + sstar) / denom;
      }
      c->T[c->L.edep + cell] = c->T[c->L.edep + cell] + deleabs;
      c->T[c->L.prdep + cell] = c->T[c->L.prdep + cell] + deleabs * wmustar * C_LIGHT;
      if (ewnew <= wtmin) {
        TALLY(c, counters + C2D_CNT_KILLED) += 1.0;
      } else {
        q.ew = ewnew;
        q.dcen = p.dcen - trc;
        double Eta2 = clampd(((v12 ? fc : trc) + Eta * rpre) / rnew, lim9);   /* H1 unless 2012-11 */
        q.phi = ACOS(Eta2);
        if (eta_switch == -1) q.phi = 2.0 * PI_REF - q.phi;
        q.rpre = rnew;
        q.zpre = znew;
        rng_t gp = rng_sub(g, 1u + (uint32_t)(g0 + i));
        gp.ctr = gb.ctr;                                /* collision record: (key, probe sub, ctr) */
        collision(c, &q, -1, &gp);
        nscat++;
      }
      dpos = dcol;
      if (n > 0) tau = -LOG(U(&gb)) / (double)n;
    }
    if (n == 0) return nscat;
    tau = tau - sigsc * (trld - dpos);
    /* the n probes that fly the whole step (imctrk2d.f:382-462) */
    const double xabs = sigabs * trld;
    const double ewnew = (xabs < 100.0) ? p.ew * EXP(-xabs) : 0.0;
    double deleabs = p.ew - ewnew;
    if (deleabs < 1.0e-50) deleabs = 1.0e-50;
    /* the survivors' absorption points: the bundle's point stream (source
     * key, C2D_SUB_ABSPT | g0), two 32-bit uniforms per output (high half
     * first), fresh outputs per shared step (c2d_rng.h c2d_abspt) */
    const double q = deleabs / p.ew;
    uint64_t wo = 0;
    int t = 0;
    for (uint32_t m = alive; m; m &= m - 1u, t++) {
      double wmustar = wmu;
      if (xabs > 0.00001) {
        if ((t & 1) == 0) wo = c2d_abspt(gb.key, C2D_SUB_ABSPT | (uint32_t)g0, actr++);
        const double mr = c2d_u01_32((t & 1) == 0 ? (uint32_t)(wo >> 32) : (uint32_t)wo);
        const double sstar = -LOG(1.0 - mr * q) / sigabs;
        const double denom = SQRT(rpre * rpre + 2.0 * wmu * rpre * sstar + sstar * sstar);
        wmustar = (wmu * rpre + sstar) / denom;
      }
      c->T[c->L.edep + cell] = c->T[c->L.edep + cell] + deleabs;
      c->T[c->L.prdep + cell] = c->T[c->L.prdep + cell] + deleabs * wmustar * C_LIGHT;
    }
    if (ewnew <= wtmin) {
      TALLY(c, counters + C2D_CNT_KILLED) += (double)n;
      return nscat;
    }
    p.ew = ewnew;
    /* the shared move */
    double rnew, znew;
    if (bnd) {
      rnew = rbnd;
      znew = Zbnd;
    } else {
      jnew = p.jph;
      knew = p.kph;
      f = trld * SQRT(1.0 - wmu * wmu);
      rnew = SQRT(f * f + rpre * rpre + 2.0 * f * rpre * Eta);
      znew = zpre + trld * wmu;
    }
    p.dcen = p.dcen - trld;
    Eta = ((v12 ? f : trld) + Eta * rpre) / rnew;      /* hazard H1 unless 2012-11 */
    Eta = clampd(Eta, lim9);
    p.phi = ACOS(Eta);
    if (eta_switch == -1) p.phi = 2.0 * PI_REF - p.phi;
    p.rpre = rnew;
    p.zpre = znew;
    if (!bnd) return nscat;                            /* census: probes end */
    if (jnew == c->nz + 1 || jnew == 0 || knew == c->nr + 1 || knew == 0) return nscat;
    p.jph = jnew;
    p.kph = knew;
  }
}

static void imctrk2d(c2o_ctx* c, pkt_t* p, int scat_flag, rng_t* g) {
  double wtmin = 1.0e-10 * p->ew;
  int nscat = 0;
  pkt_t sv = *p;
  if (scat_flag == -1) {
    sv.ew = p->ew / c->split1;
    c->comac_call++;
  }
  if (scat_flag == -1 && g->mode == C2O_RNG_LINEAGE && c->probe_bundles) {
    for (int g0 = 0; g0 < c->split1; g0 += C2O_BUNDLE_MAX) {
      const int G = (c->split1 - g0 < C2O_BUNDLE_MAX) ? c->split1 - g0 : C2O_BUNDLE_MAX;
      nscat += probe_bundle(c, &sv, sv.ew, wtmin, g0, G, g);
    }
    if (c->split1 - nscat > 0) {
      *p = sv;
      p->ew = (double)(c->split1 - nscat) * sv.ew;
      rng_t gr = rng_sub(g, C2D_SUB_RECOMB);
      imctrk2d(c, p, 0, &gr);
    }
    return;
  }
  int niter = (scat_flag == -1) ? c->split1 : 1;
  for (int it = 0; it < niter; it++) {
    *p = sv;
    if (scat_flag == -1) {
      rng_t gp = rng_sub(g, 1u + (uint32_t)it);
      rng_t* gpp = (g->mode == C2O_RNG_LINEAGE) ? &gp : g;
      nscat += flight_loop(c, p, -1, gpp, wtmin);
    } else {
      nscat += flight_loop(c, p, scat_flag, g, wtmin);
    }
  }
  if (c->split1 - nscat > 0 && scat_flag == -1) {
    *p = sv;
    p->ew = (double)(c->split1 - nscat) * sv.ew;
    rng_t gr = rng_sub(g, C2D_SUB_RECOMB);
    imctrk2d(c, p, 0, (g->mode == C2O_RNG_LINEAGE) ? &gr : g);
  }
}

/* ------------------------------------------------------------------ */
/* sources                                                             */
/* ------------------------------------------------------------------ */
/* planck (planck2d.f:1-141) */
static void planck(c2o_ctx* c, pkt_t* p, double tpl, rng_t* g) {
  double u4, ap0, ap1 = 1.0, ap2 = 1.0, ap3 = 1.0, rn1;
  do {
    u4 = U(g);
    u4 = u4 * U(g);
    u4 = u4 * U(g);
    u4 = u4 * U(g);
  } while (u4 <= 1.0e-200);
  ap0 = -LOG(u4);
  rn1 = 1.08232 * U(g);
  while (!(rn1 <= ap1)) {
    ap2 = ap2 + 1.0;
    ap3 = 1.0 / ap2;
    ap1 = ap1 + (ap3 * ap3) * (ap3 * ap3);
  }
  p->xnu = ap0 * ap3 * tpl;
  p->jgpsp = bin_sp(c, p->xnu, F32(1.000001), F32(0.999999), 0);
  p->jgplc = bin_lc(c, p->xnu);
  p->jgpmu = bin_mu(c, p->wmu);
}

/* file_sample (imcsurf2d_para.f:694-788) */
static void file_sample(c2o_ctx* c, pkt_t* p, const c2d_spectrum* sp, rng_t* g) {
  double x1 = U(g);
  int i;
  for (i = 1; i <= sp->nfile - 1; i++)
    if (sp->P_file[i - 1] > x1) break;
  if (i > sp->nfile - 1) i = sp->nfile - 1;   /* P_file(nfile-1) = 1 > x1 in the reference */
  double x2 = U(g);
  double Ei = sp->E_file[i - 1], a1 = sp->a1[i - 1], Ii = sp->I_file[i - 1], Fi = sp->F_file[i - 1];
  p->xnu = Ei * POW(a1 * Ii * x2 / (Fi * Ei) + 1.0, 1.0 / a1);
  p->jgpsp = bin_sp(c, p->xnu, 1.000001, 0.999999, 0);
  p->jgplc = bin_lc(c, p->xnu);
  p->jgpmu = bin_mu(c, p->wmu);
}

static const c2d_spectrum* spec_for(c2o_ctx* c, const int32_t* idx, int n) {
  if (!idx || idx[n] < 0 || idx[n] >= c->in->n_spectra) {
    c->err = C2D_E_ARG;
    return NULL;
  }
  return &c->in->spectra[idx[n]];
}

/* one volume packet of vol_calc (imcvol2d_para.f:157-392) */
static void vol_packet(c2o_ctx* c, int jv, int kv, rng_t* g, double f_thermal, double f_inn,
                       double f_outer, double f_upper) {
  pkt_t P, *p = &P;
  int cell = CELL(c, jv, kv);
  const double* eth = c->eps_th + (int64_t)cell * C2D_N_VOL;
  const double* etot = c->eps_tot + (int64_t)cell * C2D_N_VOL;
  double rnum, rnum0, x1, x2, psi;
  int i;
  double rlow = (kv == 1) ? c->rmin : c->r[kv - 1];
  p->jph = jv;
  p->kph = kv;
  p->ew = c->ewsv[cell];
  p->dcen = C_LIGHT * c->dt * U(g);
  rnum = U(g);
  if (rnum < f_thermal) {
    i = 0;
    rnum = U(g);
    do { i = i + 1; } while (eth[i - 1] < rnum && i < C2D_N_VOL);
    if (i < C2D_N_VOL)
      p->xnu = c->E_ph[i] + U(g) * (c->E_ph[i + 1] - c->E_ph[i]);
    else
      p->xnu = c->E_ph[i];
    rnum0 = U(g);
    if (rnum0 < f_inn) {
      p->wmu = clampd(2.0 * U(g) - 1.0, 9.9999999e-1);
      x1 = U(g);
      x2 = U(g);
      if (x1 < 0.5) {
        p->phi = 1.1e1 / 7.0 + (1.1e1 / 7.0) * x2;
        if (p->phi < 1.57079638) p->phi = 1.57079638;
      } else {
        p->phi = -1.1e1 / 7.0 - (1.1e1 / 7.0) * x2;
        if (p->phi > -1.57079638) p->phi = -1.57079638;
      }
      p->rpre = (kv == 1) ? F32(1.00001) * c->rmin : F32(1.00001) * c->r[kv - 1];
      p->zpre = (jv == 1) ? c->z[1] * U(g) : c->z[jv - 1] + U(g) * (c->z[jv] - c->z[jv - 1]);
    } else if (rnum0 < f_outer) {
      p->wmu = clampd(2.0 * U(g) - 1.0, 9.9999999e-1);
      p->rpre = F32(0.999999) * c->r[kv];
      p->zpre = (jv == 1) ? c->z[1] * U(g) : c->z[jv - 1] + U(g) * (c->z[jv] - c->z[jv - 1]);
      p->phi = -1.1e1 / 7.0 + 2.2e1 / 7.0 * U(g);
      if (p->phi < -1.5707963) p->phi = -1.57079063;
      if (p->phi > 1.5707963) p->phi = 1.5707963;
    } else if (rnum0 < f_upper) {
      p->wmu = U(g);
      if (p->wmu > 9.9999999e-1) p->wmu = 9.9999999e-1;
      if (p->wmu < 0.0) p->wmu = 0.0;
      p->phi = 4.4e1 / 7.0 * U(g);
      if (p->phi > 2.0 * PI_REF) p->phi = 2.0 * PI_REF;
      psi = U(g);
      p->zpre = F32(0.999999) * c->z[jv];
      p->rpre = SQRT(rlow * rlow + psi * (c->r[kv] * c->r[kv] - rlow * rlow));
    } else {
      p->wmu = -U(g);
      p->phi = 4.4e1 / 7.0 * U(g);
      if (p->wmu > 0.0) p->wmu = 0.0;
      if (p->wmu < -9.9999999e-1) p->wmu = -9.9999999e-1;
      if (p->phi > 2.0 * PI_REF) p->phi = 2.0 * PI_REF;
      if (jv == 1) {
        p->zpre = F32(1.000001) * c->zmin;
        if (p->zpre <= c->zmin) p->zpre = c->zmin + 1.0e-6;
      } else {
        p->zpre = F32(1.000001) * c->z[jv - 1];
        if (p->zpre <= c->z[jv - 1]) p->zpre = c->z[jv - 1] + 1.0e-6;
      }
      psi = U(g);
      p->rpre = SQRT(rlow * rlow + psi * (c->r[kv] * c->r[kv] - rlow * rlow));
    }
  } else {
    i = 0;
    rnum = U(g);
    do { i = i + 1; } while (etot[i - 1] < rnum && i < C2D_N_VOL);
    if (i < C2D_N_VOL)
      p->xnu = c->E_ph[i] + U(g) * (c->E_ph[i + 1] - c->E_ph[i]);
    else
      p->xnu = c->E_ph[i];
    p->wmu = 2.0 * U(g) - 1.0;
    p->phi = 4.4e1 / 7.0 * U(g);
    p->wmu = clampd(p->wmu, 9.9999999e-1);
    if (p->phi > 2.0 * PI_REF) p->phi = 2.0 * PI_REF;
    p->zpre = (jv == 1) ? c->z[1] * U(g) : c->z[jv - 1] + U(g) * (c->z[jv] - c->z[jv - 1]);
    psi = U(g);
    p->rpre = SQRT(rlow * rlow + psi * (c->r[kv] * c->r[kv] - rlow * rlow));
  }
  p->jgpsp = bin_sp(c, p->xnu, F32(1.000001), F32(0.999999), c->nphtotal);
  p->jgplc = bin_lc(c, p->xnu);
  p->jgpmu = bin_mu(c, p->wmu);
  TALLY(c, counters + C2D_CNT_SOURCES) += 1.0;
  imctrk2d(c, p, -1, g);
}

static void vol_zone_fractions(const c2o_ctx* c, int jv, int kv, double* f_thermal,
                               double* f_inn, double* f_outer, double* f_upper) {
  int cell = CELL(c, jv, kv);
  double delz = (jv == 1) ? c->z[1] : c->z[jv] - c->z[jv - 1];
  double zs = c->zsurf[cell];
  double rlow = (kv == 1) ? c->rmin : c->r[kv - 1];
  double fi = (4.4e1 / 7.0 * rlow * delz) / zs;
  double fo = (4.4e1 / 7.0 * c->r[kv] * delz) / zs;
  double fu = (2.2e1 / 7.0 * (c->r[kv] * c->r[kv] - rlow * rlow)) / zs;
  *f_thermal = c->Eloss_th[cell] / c->Eloss_tot[cell];
  *f_inn = fi;
  *f_outer = fi + fo;
  *f_upper = *f_outer + fu;
}

/* z_surf_calc (imcsurf2d_para.f:228-346): inner (i) and outer (o) surfaces */
static void zsurf_packet(c2o_ctx* c, int js, int outer, rng_t* g) {
  const c2d_step_in* in = c->in;
  pkt_t P, *p = &P;
  const double lim10 = 0.9999999999;
  p->jph = js;
  if (!outer) {
    p->wmu = clampd(2.0 * U(g) - 1.0, lim10);
    p->phi = -1.1e1 / 7.0 + 2.2e1 / 7.0 * U(g);
    if (p->phi < -1.5707963) p->phi = -1.57079063;
    if (p->phi > 1.5707963) p->phi = 1.5707963;
    p->rpre = c->rmin;
    p->zpre = (js == 1) ? c->z[1] * U(g) : c->z[js - 1] + U(g) * (c->z[js] - c->z[js - 1]);
    p->ew = in->ewsurfi[js - 1];
    p->dcen = U(g) * C_LIGHT * c->dt;
    if (in->tbbi[js - 1] > 0.0) {
      planck(c, p, in->tbbi[js - 1], g);
    } else {
      const c2d_spectrum* sp = spec_for(c, in->spec_i, js - 1);
      if (!sp) return;
      file_sample(c, p, sp, g);
    }
    p->kph = 1;
  } else {
    double x1, x2;
    p->wmu = clampd(2.0 * U(g) - 1.0, lim10);
    p->rpre = c->r[c->nr];
    p->zpre = (js == 1) ? c->z[1] * U(g) : c->z[js - 1] + U(g) * (c->z[js] - c->z[js - 1]);
    x1 = U(g);
    x2 = U(g);
    if (x1 < 0.5) {
      p->phi = 1.1e1 / 7.0 + (1.1e1 / 7.0) * x2;
      if (p->phi < 1.57079638) p->phi = 1.57079638;
    } else {
      p->phi = -1.1e1 / 7.0 - (1.1e1 / 7.0) * x2;
      if (p->phi > -1.57079638) p->phi = -1.57079638;
    }
    p->ew = in->ewsurfo[js - 1];
    p->dcen = U(g) * C_LIGHT * c->dt;
    if (in->tbbo[js - 1] > 0.0) {
      planck(c, p, in->tbbo[js - 1], g);
    } else {
      const c2d_spectrum* sp = spec_for(c, in->spec_o, js - 1);
      if (!sp) return;
      file_sample(c, p, sp, g);
    }
    p->kph = c->nr;
  }
  TALLY(c, counters + C2D_CNT_SOURCES) += 1.0;
  imctrk2d(c, p, -1, g);
}

/* r_surf_calc (imcsurf2d_para.f:353-534): upper (u) and lower (l) surfaces */
static void rsurf_packet(c2o_ctx* c, int ks, int lower, rng_t* g) {
  const c2d_step_in* in = c->in;
  pkt_t P, *p = &P;
  const double lim10 = 0.9999999999;
  double rlow = (ks == 1) ? c->rmin : c->r[ks - 1];
  double psi;
  p->kph = ks;
  if (!lower) {
    p->wmu = clampd(-U(g), lim10);
    p->phi = 2.0 * PI_REF * U(g);
    psi = U(g);
    p->zpre = c->z[c->nz];
    p->rpre = SQRT(rlow * rlow + psi * (c->r[ks] * c->r[ks] - rlow * rlow));
    p->ew = in->ewsurfu[ks - 1];
    p->dcen = U(g) * C_LIGHT * c->dt;
    if (in->tbbu[ks - 1] > 0.0) {
      planck(c, p, in->tbbu[ks - 1], g);
    } else {
      const c2d_spectrum* sp = spec_for(c, in->spec_u, ks - 1);
      if (!sp) return;
      file_sample(c, p, sp, g);
    }
    p->jph = c->nz;
  } else {
    p->wmu = 9.9999999e-1;
    p->phi = 2.0 * PI_REF * U(g);
    psi = U(g);
    p->zpre = c->zmin;
    p->rpre = SQRT(rlow * rlow + psi * (c->r[ks] * c->r[ks] - rlow * rlow));
    p->ew = in->ewsurfl[ks - 1];
    if (in->tbbl[ks - 1] > 0.0) {
      planck(c, p, in->tbbl[ks - 1], g);
    } else {
      const c2d_spectrum* sp = spec_for(c, in->spec_l, ks - 1);
      if (!sp) return;
      file_sample(c, p, sp, g);
    }
    p->dcen = U(g) * C_LIGHT * c->dt;
    p->jph = 1;
  }
  TALLY(c, counters + C2D_CNT_SOURCES) += 1.0;
  imctrk2d(c, p, -1, g);
}

/* ------------------------------------------------------------------ */
/* public API (ctypes)                                                 */
/* ------------------------------------------------------------------ */
c2o_ctx* c2o_create(const c2d_config* cfg, int rng_mode, int rand_switch, int32_t rseed,
                    int h4_stale) {
  if (cfg->nz < 1 || cfg->nr < 1 || cfg->nz > C2D_MAXZONE || cfg->nr > C2D_MAXZONE) return NULL;
  if (cfg->nphtotal > C2D_NPHOMAX || cfg->nph_lc > C2D_NPHLCMAX || cfg->nmu > C2D_NMUMAX ||
      cfg->nmu < 1 || cfg->cr_sent != 0)
    return NULL;
  c2o_ctx* c = (c2o_ctx*)calloc(1, sizeof(c2o_ctx));
  c->nz = cfg->nz;
  c->nr = cfg->nr;
  c->ncell = cfg->nz * cfg->nr;
  c->rmin = cfg->rmin;
  c->zmin = cfg->zmin;
  for (int j = 1; j <= c->nz; j++) c->z[j] = cfg->z[j - 1];
  for (int k = 1; k <= c->nr; k++) c->r[k] = cfg->r[k - 1];
  for (int i = 1; i <= C2D_N_VOL; i++) c->E_ph[i] = cfg->E_ph[i - 1];
  for (int i = 1; i <= C2D_NPHFIELD; i++) c->E_field[i] = cfg->E_field[i - 1];
  for (int i = 1; i <= C2D_NUM_NT; i++) c->gnt[i] = cfg->gnt[i - 1];
  c->nphtotal = cfg->nphtotal;
  for (int i = 1; i <= c->nphtotal + 1; i++) c->hu[i] = cfg->hu[i - 1];
  c->nph_lc = cfg->nph_lc;
  for (int m = 1; m <= c->nph_lc; m++) {
    c->Elcmin[m] = cfg->Elcmin[m - 1];
    c->Elcmax[m] = cfg->Elcmax[m - 1];
  }
  c->nmu = cfg->nmu;
  for (int n = 1; n <= c->nmu; n++) c->mu[n] = cfg->mu[n - 1];
  c->split1 = cfg->split1;
  {
    /* test knob: C2O_PROBE_BUNDLES=0 tracks the lineage-mode probes one copy
     * at a time with per-copy colmfp draws, (key, 1 + probe) streams -- the
     * statistical reference for the bundles (tests/test_bundle_statistics.py) */
    const char* e = getenv("C2O_PROBE_BUNDLES");
    c->probe_bundles = !(e && e[0] == '0');
  }
  c->split2 = cfg->split2;
  c->split3 = cfg->split3;
  c->spl3_trg = cfg->spl3_trg;
  c->spec_switch = cfg->spec_switch;
  c->cr_sent = cfg->cr_sent;
  c->pair_switch = cfg->pair_switch;
  c->kappa_lag = cfg->kappa_lag;
  c->trk2012 = cfg->trk_variant == C2D_TRK_2012_11;
  c->rng_mode = rng_mode;
  c->rand_switch = rand_switch;
  c->rseed = rseed;
  g_ran1_seed = rseed;
  c->h4_stale = h4_stale;
  c->seed = cfg->seed;
  c->rank = cfg->world > 1 ? cfg->rank : 0;
  c->world = cfg->world > 1 ? cfg->world : 1;
  int64_t nc = c->ncell;
  c->kappa = (double*)calloc(nc * C2D_N_VOL, sizeof(double));
  c->kappa_prev = (double*)calloc(nc * C2D_N_VOL, sizeof(double));
  c->eps_tot = (double*)calloc(nc * C2D_N_VOL, sizeof(double));
  c->eps_th = (double*)calloc(nc * C2D_N_VOL, sizeof(double));
  c->f_nt = (double*)calloc(nc * C2D_NUM_NT, sizeof(double));
  c->Pnt = (double*)calloc(nc * C2D_NUM_NT, sizeof(double));
  c->n_e = (double*)calloc(nc, sizeof(double));
  c->Eloss_th = (double*)calloc(nc, sizeof(double));
  c->Eloss_tot = (double*)calloc(nc, sizeof(double));
  c->zsurf = (double*)calloc(nc, sizeof(double));
  c->ewsv = (double*)calloc(nc, sizeof(double));
  c->nsv = (int32_t*)calloc(nc, sizeof(int32_t));
  c->comac_ar = (double*)calloc(nc, sizeof(double));
  c->comac_stamp = (int64_t*)calloc(nc, sizeof(int64_t));
  c->comac_call = 0;
  for (int64_t i = 0; i < nc; i++) c->comac_stamp[i] = -1;
  c2d_tally_layout_for(c->nz, c->nr, c->nmu, &c->L);
  c->T = (double*)calloc(c->L.total, sizeof(double));
  c->ccap = cfg->census_capacity > 0 ? cfg->census_capacity : 1 << 20;
  c->cin = (cens_rec*)calloc(c->ccap, sizeof(cens_rec));
  c->cout = (cens_rec*)calloc(c->ccap, sizeof(cens_rec));
  return c;
}

void c2o_destroy(c2o_ctx* c) {
  if (!c) return;
  free(c->kappa); free(c->kappa_prev); free(c->eps_tot); free(c->eps_th);
  free(c->f_nt); free(c->Pnt); free(c->n_e); free(c->Eloss_th); free(c->Eloss_tot);
  free(c->zsurf); free(c->ewsv); free(c->nsv); free(c->comac_ar); free(c->comac_stamp);
  free(c->T); free(c->cin); free(c->cout); free(c->ev);
  free(c);
}

static void gather3(const c2o_ctx* c, const c2d_array3* a, int n, double* out) {
  for (int j = 0; j < c->nz; j++)
    for (int k = 0; k < c->nr; k++)
      for (int i = 0; i < n; i++)
        out[((int64_t)(j * c->nr + k)) * n + i] =
            a->data ? a->data[i * a->s_i + j * a->s_j + k * a->s_k] : 0.0;
}
static void gather2(const c2o_ctx* c, const c2d_array2* a, double* out) {
  for (int j = 0; j < c->nz; j++)
    for (int k = 0; k < c->nr; k++)
      out[j * c->nr + k] = a->data ? a->data[j * a->s_j + k * a->s_k] : 0.0;
}

int c2o_step(c2o_ctx* c, const c2d_step_in* in) {
  c->in = in;
  c->err = 0;
  c->ncycle = in->ncycle;
  c->time = in->time;
  c->dt = in->dt;
  const double dt_now = in->dt;
  if (c->dt_lag) c->dt = c->dt_prev;
  c->grid_missing = c->grid_lag && !c->grid_seen;
  memset(c->T, 0, sizeof(double) * c->L.total);
  c->nev = 0;
  gather3(c, &in->kappa_tot, C2D_N_VOL, c->kappa);
  gather3(c, &in->eps_tot, C2D_N_VOL, c->eps_tot);
  gather3(c, &in->eps_th, C2D_N_VOL, c->eps_th);
  gather3(c, &in->f_nt, C2D_NUM_NT, c->f_nt);
  gather3(c, &in->Pnt, C2D_NUM_NT, c->Pnt);
  gather2(c, &in->n_e, c->n_e);
  gather2(c, &in->Eloss_th, c->Eloss_th);
  gather2(c, &in->Eloss_tot, c->Eloss_tot);
  gather2(c, &in->zsurf, c->zsurf);
  gather2(c, &in->ewsv, c->ewsv);
  for (int j = 0; j < c->nz; j++)
    for (int k = 0; k < c->nr; k++)
      c->nsv[j * c->nr + k] = in->nsv.data ? in->nsv.data[j * in->nsv.s_j + k * in->nsv.s_k] : 0;

  fibstate* fs = &c->fs;
  rng_t g0 = {c->rng_mode, 0, 0, fs};
  if (c->rng_mode == C2O_RNG_FIB) seed_zone(&c->rseed, c->nz, c->nr, c->seeds, c->zseeds, c->rseeds);
  c->step_key = c2d_step_key(c->seed, c->ncycle);

  /* census + volume transport use the previous step's kappa (hazard H3) */
  c->kappa_use = c->kappa_lag ? c->kappa_prev : c->kappa;

  /* census (field_calc, imcfield2d.f:57-144) */
  cens_rec* tmp = c->cin; c->cin = c->cout; c->cout = tmp;
  c->nin = c->nout;
  c->nout = 0;
  for (int64_t n = 0; n < c->nin; n++) {
    cens_rec* q = &c->cin[n];
    pkt_t P;
    P.rpre = q->d[0]; P.zpre = q->d[1]; P.wmu = q->d[2]; P.phi = q->d[3];
    P.ew = q->d[4]; P.xnu = q->d[5];
    P.jgpsp = q->i[0]; P.jgplc = q->i[1]; P.jgpmu = q->i[2]; P.jph = q->i[3]; P.kph = q->i[4];
    rng_t g = g0;
    if (c->rng_mode == C2O_RNG_FIB) {
      /* seeds(jph,kph) = ibufin(lwai+6) (imcfield2d.f:115) only touches the
       * worker's copy; volume jobs get the master's seeds (vol_mpi.f:107). */
      initialize_rand(fs, (int32_t)(int64_t)q->key);
    } else if (c->rng_mode == C2O_RNG_LINEAGE) {
      g.key = q->key;
      g.ctr = 0;
    }
    P.dcen = C_LIGHT * c->dt;
    P.wmu = clampd(P.wmu, c->trk2012 ? 1.0 : 0.99999999);   /* imcfield2d.f:119-120 (2012-11: 119-124) */
    TALLY(c, counters + C2D_CNT_SOURCES) += 1.0;
    imctrk2d(c, &P, -1, &g);
    if (c->err) return c->err;
  }
  /* volume (vol_calc) */
  int64_t vol_global = 0, surf_global = 0;
  int32_t seeds_job[C2D_MAXZONE * C2D_MAXZONE];
  memcpy(seeds_job, c->seeds, sizeof(int32_t) * c->ncell);
  for (int jv = 1; jv <= c->nz; jv++)
    for (int kv = 1; kv <= c->nr; kv++) {
      int cell = CELL(c, jv, kv);
      if (c->rng_mode == C2O_RNG_FIB) initialize_rand(fs, seeds_job[cell]);
      int more = c->nsv[cell];
      if (more <= 0) continue;
      double f_th, f_inn, f_out, f_up;
      vol_zone_fractions(c, jv, kv, &f_th, &f_inn, &f_out, &f_up);
      for (int n = 0; n < more; n++) {
        int64_t gidx = vol_global++;
        rng_t g = g0;
        if (c->rng_mode == C2O_RNG_LINEAGE) {
          if (gidx % c->world != c->rank) continue;
          g.key = c2d_derive(c->step_key, C2D_TAG_VOL, (uint32_t)n, (uint32_t)cell);
          g.ctr = 0;
        }
        vol_packet(c, jv, kv, &g, f_th, f_inn, f_out, f_up);
        if (c->err) return c->err;
      }
    }
  /* surfaces use the current kappa_tot, dt and grids (broadcast in z_surf_bcast) */
  c->kappa_use = c->kappa;
  c->dt = dt_now;
  c->grid_missing = 0;
  c->grid_seen = 1;
  for (int js = 1; js <= c->nz; js++) {
    if (c->rng_mode == C2O_RNG_FIB) initialize_rand(fs, c->zseeds[js - 1]);
    for (int side = 0; side < 2; side++) {
      const int32_t* ns = side ? in->nsurfo : in->nsurfi;
      int cnt = ns ? ns[js - 1] : 0;
      for (int n = 0; n < cnt; n++) {
        int64_t gidx = surf_global++;
        rng_t g = g0;
        if (c->rng_mode == C2O_RNG_LINEAGE) {
          if (gidx % c->world != c->rank) continue;
          g.key = c2d_derive(c->step_key, C2D_TAG_SURF + side, (uint32_t)n, (uint32_t)(js - 1));
          g.ctr = 0;
        }
        zsurf_packet(c, js, side, &g);
        if (c->err) return c->err;
      }
    }
  }
  for (int ks = 1; ks <= c->nr; ks++) {
    if (c->rng_mode == C2O_RNG_FIB) initialize_rand(fs, c->rseeds[ks - 1]);
    for (int side = 0; side < 2; side++) {
      const int32_t* ns = side ? in->nsurfl : in->nsurfu;
      int cnt = ns ? ns[ks - 1] : 0;
      for (int n = 0; n < cnt; n++) {
        int64_t gidx = surf_global++;
        rng_t g = g0;
        if (c->rng_mode == C2O_RNG_LINEAGE) {
          if (gidx % c->world != c->rank) continue;
          g.key = c2d_derive(c->step_key, C2D_TAG_SURF + 2 + side, (uint32_t)n, (uint32_t)(ks - 1));
          g.ctr = 0;
        }
        rsurf_packet(c, ks, side, &g);
        if (c->err) return c->err;
      }
    }
  }
  memcpy(c->kappa_prev, c->kappa, sizeof(double) * (int64_t)c->ncell * C2D_N_VOL);
  c->dt_prev = dt_now;
  return c->err;
}

/* hazard H11 (MPI workers' stale dt, see c2o_ctx.dt_lag): off by default */
void c2o_set_dt_lag(c2o_ctx* c, int on) { c->dt_lag = on; }
/* hazard H12 (MPI workers' grids before the first z_surf_bcast, see
 * c2o_ctx.grid_lag): off by default */
void c2o_set_grid_lag(c2o_ctx* c, int on) { c->grid_lag = on; }

const double* c2o_tallies(c2o_ctx* c, int64_t* n) {
  *n = c->L.total;
  return c->T;
}

int64_t c2o_event_count(c2o_ctx* c) { return c->nev; }
int64_t c2o_events(c2o_ctx* c, double* out, int64_t cap) {
  int64_t n = c->nev < cap ? c->nev : cap;
  memcpy(out, c->ev, sizeof(double) * C2D_EVENT_WORDS * n);
  return n;
}

int64_t c2o_census_count(c2o_ctx* c) { return c->nout; }
int64_t c2o_census_export(c2o_ctx* c, double* d6, int32_t* i5, uint64_t* keys, int64_t cap) {
  int64_t n = c->nout < cap ? c->nout : cap;
  for (int64_t m = 0; m < n; m++) {
    memcpy(d6 + 6 * m, c->cout[m].d, 6 * sizeof(double));
    memcpy(i5 + 5 * m, c->cout[m].i, 5 * sizeof(int32_t));
    keys[m] = c->cout[m].key;
  }
  return n;
}
int c2o_census_import(c2o_ctx* c, const double* d6, const int32_t* i5, const uint64_t* keys,
                      int64_t n) {
  if (n > c->ccap) return C2D_E_CENSUS_OVERFLOW;
  for (int64_t m = 0; m < n; m++) {
    memcpy(c->cout[m].d, d6 + 6 * m, 6 * sizeof(double));
    memcpy(c->cout[m].i, i5 + 5 * m, 5 * sizeof(int32_t));
    c->cout[m].key = keys[m];
  }
  c->nout = n;
  return 0;
}

int32_t c2o_rseed(c2o_ctx* c) { return c->rseed; }

/* ---- unit-level entry points used by the golden tests ---- */
static fibstate g_unit_fs;

void c2o_unit_fib_init(int32_t seed) { initialize_rand(&g_unit_fs, seed); }
void c2o_unit_fib_draw(int64_t n, double* out) {
  for (int64_t i = 0; i < n; i++) out[i] = fibran(&g_unit_fs);
}
void c2o_unit_seed_zone(int32_t* seed, int nz, int nr, int32_t* seeds, int32_t* zseeds,
                        int32_t* rseeds) {
  seed_zone(seed, nz, nr, seeds, zseeds, rseeds);
}
void c2o_unit_ran1(int32_t* idum, int64_t n, double* out) {
  static fibstate s;
  for (int64_t i = 0; i < n; i++) out[i] = ran1(&s, idum);
}
double c2o_unit_dilog(double x) { return dilog(x); }
double c2o_unit_intg_v(double x) { return intg_v(x); }
/* comtot for zone (j,k) 1-based with the tables of the last c2o_step, or
 * with tables loaded by c2o_unit_set_tables */
double c2o_unit_comtot(c2o_ctx* c, int j, int k, double xnu) {
  return comtot_cell(c, CELL(c, j, k), xnu);
}
void c2o_unit_set_tables(c2o_ctx* c, const c2d_step_in* in) {
  gather3(c, &in->f_nt, C2D_NUM_NT, c->f_nt);
  gather3(c, &in->Pnt, C2D_NUM_NT, c->Pnt);
  gather2(c, &in->n_e, c->n_e);
}
/* compb2d on packet state st[7] = xnu,wmu,phi,rpre,zpre,dcen,ew; ist[5] =
 * jph,kph,jgpsp,jgplc,jgpmu; draws from the unit fib stream (mode FIB) or
 * from lineage stream (key, *ctr) (mode LINEAGE). Returns i_gam. */
int c2o_unit_compb2d(c2o_ctx* c, double* st, int32_t* ist, int mode, uint64_t key,
                     uint32_t* ctr) {
  pkt_t P = {st[0], st[1], st[2], st[3], st[4], st[5], st[6], ist[0], ist[1], ist[2], ist[3], ist[4]};
  rng_t g = {mode, key, ctr ? *ctr : 0, &g_unit_fs};
  int ig = compb2d(c, &P, &g);
  st[0] = P.xnu; st[1] = P.wmu; st[2] = P.phi; st[3] = P.rpre; st[4] = P.zpre;
  st[5] = P.dcen; st[6] = P.ew;
  ist[2] = P.jgpsp; ist[3] = P.jgplc; ist[4] = P.jgpmu;
  if (ctr) *ctr = g.ctr;
  return ig;
}
double c2o_unit_planck(c2o_ctx* c, double tpl, double wmu, int32_t* bins) {
  pkt_t P;
  memset(&P, 0, sizeof P);
  P.wmu = wmu;
  rng_t g = {C2O_RNG_FIB, 0, 0, &g_unit_fs};
  planck(c, &P, tpl, &g);
  bins[0] = P.jgpsp; bins[1] = P.jgplc; bins[2] = P.jgpmu;
  return P.xnu;
}
double c2o_unit_philox_draw(uint64_t key, uint32_t n) { return c2d_draw(key, n); }
double c2o_unit_philox_draw_s(uint64_t key, uint32_t sub, uint32_t n) { return c2d_draw_s(key, sub, n); }
uint64_t c2o_unit_derive_s(uint64_t key, uint32_t tag, uint32_t a, uint32_t b, uint32_t sub) {
  return c2d_derive_s(key, tag, a, b, sub);
}
uint64_t c2o_unit_derive(uint64_t key, uint32_t tag, uint32_t a, uint32_t b) {
  return c2d_derive(key, tag, a, b);
}
int c2o_is_detmath(void) {
#ifdef C2O_DETMATH
  return 1;
#else
  return 0;
#endif
}

/* elementary functions of this build (c2d_math.h in the det flavor, glibc
 * otherwise): fn 0 log, 1 exp, 2 cos, 3 acos, 4 pow(x, 1/3) */
void c2o_unit_math(int fn, const double* x, double* y, int64_t n) {
  for (int64_t i = 0; i < n; i++) {
    switch (fn) {
      case 0: y[i] = LOG(x[i]); break;
      case 1: y[i] = EXP(x[i]); break;
      case 2: y[i] = COS(x[i]); break;
      case 3: y[i] = ACOS(x[i]); break;
#ifdef C2O_DETMATH
      case 5: y[i] = c2d_log_pos(x[i]); break;   /* the GPU's branch-free log */
      case 6: y[i] = c2d_exp_bf(x[i]); break;    /* the GPU's branch-free exp */
#else
      case 5: y[i] = LOG(x[i]); break;
      case 6: y[i] = EXP(x[i]); break;
#endif
      default: y[i] = POW(x[i], 1.0 / 3.0); break;
    }
  }
}
