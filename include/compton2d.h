/*
 * compton2d.h — C-ABI of the MI355X-native Compton2d IMC engine.
 *
 * Drop-in boundary for the reference's per-step transport entry points
 * (all argument-less Fortran subroutines that talk through COMMON blocks):
 *
 *   reference entry point                         replaced by
 *   -------------------------------------------   --------------------------------------
 *   src/imcfield2d.f:5   imcfield2d (census)       c2d_transport_step  (census phase)
 *   src/imcvol2d_para.f:1 imcvol2d (volume src)    c2d_transport_step  (volume phase)
 *   src/imcsurf2d_para.f:1 imcsurf2d (surface src) c2d_transport_step  (surface phase)
 *   src/imcredist.f:5    imcredist (census bal.)   not needed: census stays on its GPU
 *   src/xec2d.f:325/371  xec_add/graphics_collect  c2d_tally_device_ptr + one all-reduce
 *   src/update2d.f:1929  cens_add_up (REDUCE)      c2d_tally_device_ptr + one all-reduce
 *   src/imcleak2d.f:171  event-file writes         c2d_events
 *   src/census2d.f:1-76  write_cens/read_cens      c2d_census_export / c2d_census_import
 *   src/update2d.f:7     update (FP_calc, tridag,  c2d_fp_set_config + c2d_fp_step
 *     E_add_up, FP_send_job/recv_result)
 *
 * Every array argument is (pointer, strides) so Fortran COMMON arrays with
 * their fixed leading extents (general.pa: n_vol=400, jmax=kmax=99,
 * num_nt=200) are passed without copies; the library gathers only the
 * [1:nz,1:nr] sub-block.  Indices below are 0-based: element (i,j,k) of a
 * c2d_array3 lives at data[i*s_i + j*s_j + k*s_k] with j=0..nz-1 (z zone),
 * k=0..nr-1 (r zone).  For kappa_tot(n_vol,jmax,kmax) pass s_i=1,
 * s_j=n_vol, s_k=n_vol*jmax; for f_nt(jmax,kmax,num_nt) pass s_j=1,
 * s_k=jmax, s_i=jmax*kmax.
 *
 * Errors: every call returns 0 or a negative C2D_E_* code; the message is
 * in c2d_last_error().  Nothing calls exit() (the reference `stop`s at
 * src/imctrk2d.f:573-577, src/imcfield2d.f:84-87).
 * Threading: all calls on one context from one host thread; calls are
 * synchronous on return unless documented otherwise.
 */
#ifndef COMPTON2D_H
#define COMPTON2D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Compile-time extents of the reference (src/general.pa:7-30). */
#define C2D_N_VOL     400   /* photon energy grid of kappa_tot/eps_tot (n_vol)  */
#define C2D_NUM_NT    200   /* electron Lorentz-factor grid (num_nt)            */
#define C2D_NPHFIELD  400   /* internal photon-field grid n_field (nphfield)    */
#define C2D_NPHOMAX   128   /* spectrum bins (nphomax)                          */
#define C2D_NPHLCMAX  10    /* light-curve bands (nphlcmax)                     */
#define C2D_NMUMAX    32    /* angular bins (nmumax)                            */
#define C2D_NFMAX     500   /* external seed spectrum table (nfmax)             */
#define C2D_MAXZONE   99    /* jmax = kmax                                      */

/* Error codes. */
#define C2D_OK                  0
#define C2D_E_ARG              -1   /* bad argument / unsupported option          */
#define C2D_E_HIP              -2   /* HIP runtime error                          */
#define C2D_E_CENSUS_OVERFLOW  -3   /* replaces `stop 'too many photons'`         */
#define C2D_E_EVENT_OVERFLOW   -4   /* escape-event buffer full                   */
#define C2D_E_QUEUE_OVERFLOW   -5   /* scatter-secondary queue full               */
#define C2D_E_NOMEM            -6
#define C2D_E_STATE            -7   /* call order violated                        */
#define C2D_E_FP               -8   /* FP sub-step limit (reference `stop`,
                                       src/update2d.f:585-599), a solver guard,
                                       or NaN/Inf in n_field, ecens or the
                                       updated electron state                     */
#define C2D_E_RCCL             -9   /* RCCL (communicator / all-reduce) error     */
#define C2D_E_IO              -10   /* a file could not be written                */
#define C2D_E_NONFINITE       -11   /* NaN/Inf in a table, a tally or an emission
                                       output (the reference would carry it on:
                                       NaN counts, a collapsed run)               */

/* comtot (src/comtot2d.f:1-334, icoms=6) evaluation mode. */
#define C2D_COMTOT_EXACT  0   /* 199-term electron-spectrum sum per call (reference)   */
#define C2D_COMTOT_TABLE  1   /* per-cell cubic table in log(xnu), rebuilt every step  */

/* c2d_config.trk_variant: which snapshot of the reference's tracker
 * (SURVEY.md §8 hazard H1).  C2D_TRK_SRC (default) is src/imctrk2d.f, bug
 * for bug: the azimuth update uses the 3-D path, Eta = (trld + Eta*rpre)/rnew
 * (:472), a fresh colmfp after every cell boundary (`go to 100`, :518-525),
 * the clamps |wmu| <= 0.99999999 and |Eta| <= 0.999999999 (:161-162,
 * :243-244, :474-476; imcfield2d.f:119-120).  C2D_TRK_2012_11 is
 * src_20121113/imctrk2d.f: Eta = (f + Eta*rpre)/rnew with f the path's
 * projection on the r-plane (:477-479), colmfp kept across boundaries
 * (`go to 110` with colmfp -= sigsc*trld, :505, :526-533; sigabs reset
 * after 110, :159), no idead = 4 re-entry (:521-524), and |wmu|, |Eta|
 * clamped to 1 (:162-167, :481-484; imcfield2d.f:119-124). */
#define C2D_TRK_SRC       0
#define C2D_TRK_2012_11   1

typedef struct c2d_array3 { const double* data; int64_t s_i, s_j, s_k; } c2d_array3;
typedef struct c2d_array2 { const double* data; int64_t s_j, s_k; } c2d_array2;
typedef struct c2d_iarray2 { const int32_t* data; int64_t s_j, s_k; } c2d_iarray2;

/* Seed spectrum for a surface with tbb <= 0: the normalised table that
 * file_sp (src/imcsurf2d_para.f:544-685, host-side) leaves in COMMON /insp/
 * and file_sample (:694-788) draws from. */
typedef struct c2d_spectrum {
  int32_t nfile;
  const double* E_file;   /* [nfile]   */
  const double* a1;       /* [nfile-1] */
  const double* I_file;   /* [nfile-1] */
  const double* F_file;   /* [nfile]   */
  const double* P_file;   /* [nfile-1] cumulative, normalised */
} c2d_spectrum;

/* Run-constant set-up (src/setup2d.f:47-222, src/reader.f). */
typedef struct c2d_config {
  int32_t nz, nr;                 /* zones (reference nz, nr <= 99)           */
  double  rmin, zmin;             /* inner radius, lower z (zmin = 0 in ref)  */
  const double* z;                /* [nz] upper z boundary of zone j          */
  const double* r;                /* [nr] outer r boundary of zone k          */
  const double* E_ph;             /* [C2D_N_VOL] energy grid of kappa/eps     */
  const double* E_field;          /* [C2D_NPHFIELD] grid of n_field           */
  const double* gnt;              /* [C2D_NUM_NT] gamma-1 grid                */
  int32_t nphtotal;               /* spectrum bins; hu has nphtotal+1 edges   */
  const double* hu;
  int32_t nph_lc;                 /* light-curve bands                        */
  const double* Elcmin;
  const double* Elcmax;
  int32_t nmu;                    /* angular bins                             */
  const double* mu;               /* [nmu] upper bin edges                    */
  int32_t split1, split2, split3, spl3_trg;  /* variance reduction (COMMON /split/) */
  int32_t spec_switch;            /* 0: escaping spectrum into fout            */
  int32_t cr_sent;                /* Compton reflection; only 0 supported      */
  int32_t pair_switch;            /* gamma-gamma; inert in the MPI reference (H6) */
  int32_t kappa_lag;              /* 1: census+volume use previous step's kappa_tot (H3) */
  int32_t comtot_mode;            /* C2D_COMTOT_EXACT | C2D_COMTOT_TABLE       */
  int32_t device;                 /* HIP device ordinal                        */
  uint64_t seed;                  /* lineage RNG seed (replaces rseed)        */
  int32_t rank, world;            /* source sharding: this context tracks sources with
                                     (global source index % world) == rank       */
  int64_t census_capacity;        /* packets (per context)                     */
  int64_t event_capacity;         /* escape events per step, >= C2D_EV_SHARDS (32): the
                                     buffer is 32 equal shards, workgroup b appends to
                                     shard b % 32, and a full shard is an overflow     */
  int64_t queue_capacity;         /* scatter records per generation            */
  int32_t census_inplace;         /* 0: census double-buffered (in + out, 128 B per
                                     record, the reference's dbufin/dbufout); 1: one
                                     chunked SoA (64 B per record + 1/16 slack: a
                                     step refills the 1024-record chunks its census
                                     sources have finished with)     */
  int32_t trk_variant;            /* C2D_TRK_SRC (0, default) | C2D_TRK_2012_11    */
} c2d_config;

/* Per-step inputs (what imcgen2d/volume_em/file_sp leave in COMMON). */
typedef struct c2d_step_in {
  int32_t ncycle;                 /* step counter (events only for ncycle > 0) */
  double  time, dt;               /* time, dt(1)                              */
  c2d_array3 kappa_tot;           /* (i<400, j, k) absorption [1/cm]          */
  c2d_array3 eps_tot;             /* (i<400, j, k) volume emission CDF        */
  c2d_array3 eps_th;              /* (i<400, j, k) thermal-surface CDF        */
  c2d_array3 f_nt;                /* (i<200, j, k) electron spectrum          */
  c2d_array3 Pnt;                 /* (i<200, j, k) electron CDF               */
  c2d_array2 n_e;                 /* electron density                         */
  c2d_array2 Eloss_th, Eloss_tot; /* thermal / total emitted energy           */
  c2d_array2 zsurf;               /* zone surface area                        */
  c2d_array2 ewsv;                /* volume packet weight                     */
  c2d_iarray2 nsv;                /* volume packets per zone                  */
  const int32_t* nsurfi; const int32_t* nsurfo;  /* [nz] inner/outer z-surface packets */
  const double*  ewsurfi; const double*  ewsurfo; /* [nz] weights                       */
  const int32_t* nsurfu; const int32_t* nsurfl;  /* [nr] upper/lower r-surface packets */
  const double*  ewsurfu; const double*  ewsurfl; /* [nr]                                */
  const double*  tbbi; const double* tbbo;        /* [nz] boundary temps at time index ti */
  const double*  tbbu; const double* tbbl;        /* [nr]                                 */
  const int32_t* spec_i; const int32_t* spec_o;   /* [nz] spectrum index for tbb<=0       */
  const int32_t* spec_u; const int32_t* spec_l;   /* [nr]                                  */
  int32_t n_spectra;
  const c2d_spectrum* spectra;
  int32_t device_tables;          /* C2D_DEV_* flags: tables already on the device  */
} c2d_step_in;

/* c2d_step_in.device_tables: take tables from the device instead of the
 * host views (which may then be NULL), so a coupled MC step
 *   c2d_volume_em -> c2d_set_step -> c2d_run_step -> c2d_fp_step
 * moves only zone scalars through the host (imcgen2d -> transport -> update,
 * src/xec2d.f:67-87, with no table re-gathering per step). */
#define C2D_DEV_EMISSION   1   /* kappa_tot, eps_tot, eps_th = last c2d_volume_em  */
#define C2D_DEV_ELECTRONS  2   /* f_nt, Pnt = the context's electron state (last
                                  c2d_set_step upload, updated in place by a
                                  c2d_fp_step called with NULL f_nt/Pnt views)    */

/* Fused per-step tally buffer (f64).  One all-reduce over this buffer
 * replaces xec_add, graphics_collect, cens_add_up and E_add_up's scalar
 * MPI_REDUCE loops.  Offsets are in doubles. */
typedef struct c2d_tally_layout {
  int64_t edep, prdep, ecens, npcen;  /* [ncell] each, cell = j*nr + k        */
  int64_t n_field;                    /* [ncell][C2D_NPHFIELD]                */
  int64_t E_IC, nelectron;            /* [C2D_NUM_NT+2] (reference index i)   */
  int64_t fout;                       /* [nmu][C2D_NPHOMAX]: fout(mu,jgpsp)   */
  int64_t edout;                      /* [nmu][C2D_NPHLCMAX]                  */
  int64_t erlki, erlko;               /* [nz]                                 */
  int64_t erlku, erlkl, Ed_in;        /* [nr]                                 */
  int64_t counters;                   /* [C2D_NCOUNTERS]                      */
  int64_t total;
} c2d_tally_layout;

/* counters[] entries (exact integers stored as f64). */
#define C2D_CNT_STEPS      0   /* packet-steps: passes through imctrk2d.f:228-485 */
#define C2D_CNT_ESCAPES    1   /* packets leaving the system (imcleak)           */
#define C2D_CNT_CENSUS     2   /* packets written to census                       */
#define C2D_CNT_COLLIDE    3   /* Compton collisions (ikind=3)                    */
#define C2D_CNT_KILLED     4   /* weight kills (ewnew <= wtmin)                   */
#define C2D_CNT_SOURCES    5   /* source packets started (census+volume+surface)  */
#define C2D_CNT_COMPB      6   /* compb2d calls                                    */
#define C2D_CNT_EVENTS     7   /* event-file records written                      */
#define C2D_CNT_GENS       8   /* scatter generations launched                    */
#define C2D_CNT_ABORTED    9   /* packets stopped by a safety cap (must stay 0)   */
#define C2D_CNT_ESC_SCAT  11   /* escapes of scattered packets (imctrk2d(1) copies) */
#define C2D_NCOUNTERS      16

static inline void c2d_tally_layout_for(int32_t nz, int32_t nr, int32_t nmu,
                                        c2d_tally_layout* L) {
  int64_t nc = (int64_t)nz * nr, o = 0;
  L->edep = o; o += nc;
  L->prdep = o; o += nc;
  L->ecens = o; o += nc;
  L->npcen = o; o += nc;
  L->n_field = o; o += nc * C2D_NPHFIELD;
  L->E_IC = o; o += C2D_NUM_NT + 2;
  L->nelectron = o; o += C2D_NUM_NT + 2;
  L->fout = o; o += (int64_t)nmu * C2D_NPHOMAX;
  L->edout = o; o += (int64_t)nmu * C2D_NPHLCMAX;
  L->erlki = o; o += nz;
  L->erlko = o; o += nz;
  L->erlku = o; o += nr;
  L->erlkl = o; o += nr;
  L->Ed_in = o; o += nr;
  L->counters = o; o += C2D_NCOUNTERS;
  L->total = o;
}

/* Escape event = one line of p###_evb.dat (src/imcleak2d.f:171,181):
 * t_bound, xnu [keV], ew [erg], rpre, zpre [cm], wmu, phi. */
#define C2D_EVENT_WORDS 7

/* Census record (src/imctrk2d.f:558-572; census2d.f 6e14.7 / 6i5):
 * d6 = rpre, zpre, wmu, phi, ew, xnu; i5 = jgpsp, jgplc, jgpmu, jph, kph
 * (1-based as in the reference); key = lineage RNG key (replaces the
 * per-packet fibran seed, hazard H5). */

typedef struct c2d_ctx c2d_ctx;

/* Fokker-Planck per-zone solve (src/update2d.f:337-1739, tridag :2476-2518). */
typedef struct c2d_fp_in {
  int32_t ncell;                  /* zones solved in this call                  */
  const double* a;                /* [ncell][nt] sub-diagonal                   */
  const double* b;                /* [ncell][nt] diagonal                       */
  const double* c;                /* [ncell][nt] super-diagonal                 */
  const double* r;                /* [ncell][nt] right-hand side                */
  int32_t nt;                     /* unknowns per zone (num_nt-1 = 199 in ref)  */
} c2d_fp_in;

/* ------------------------------------------------------------------------
 * Fokker-Planck electron update of one MC step (src/update2d.f:7-327
 * `update` + :337-1739 `FP_calc` for every zone, tridag :2476-2518).
 * Mutable (pointer, strides) views bind the caller's COMMON arrays, which
 * are updated in place exactly where the reference's FP_recv_result /
 * update write them (src/fp_mpi.f:972-1003, src/update2d.f:266-276).
 * ---------------------------------------------------------------------- */
typedef struct c2d_marray3 { double* data; int64_t s_i, s_j, s_k; } c2d_marray3;
typedef struct c2d_marray2 { double* data; int64_t s_j, s_k; } c2d_marray2;

/* Run constants of FP_calc (src/reader.f:512-559, broadcast once by
 * setup_bcast src/fp_mpi.f:12-324; df_implicit/df_T general.pa:27-28;
 * F_IC from IC_loss src/icloss2d.f:1-64, broadcast by FP_bcast
 * src/fp_mpi.f:596). */
typedef struct c2d_fp_config {
  int32_t pair_switch;            /* 0/1; 1 = inert positrons (H6), f_pair = 0  */
  double  df_implicit, df_T;      /* 1e-2, 0.25 in the reference               */
  double  r_esc, r_acc;           /* escape / acceleration time [z(nz)/c]      */
  int32_t cf_sentinel;            /* coronal flare on/off                      */
  double  r_flare, z_flare, t_flare, sigma_r, sigma_z, sigma_t, flare_amp;
  int32_t inj_switch, inj_dis, g2var_switch, pick_sw;
  double  inj_g1, inj_g2, inj_p, inj_t, inj_L, pick_rate, inj_gg, inj_sigma;
  double  inj_v;                  /* sqrt(1-1/g_bulk**2)*c_light (reader.f:559) */
  const double* F_IC;             /* F_IC(i<num_nt, i_ph<nphfield)             */
  int64_t F_IC_s_i, F_IC_s_ph;    /* Fortran F_IC(200,400): s_i=1, s_ph=200    */
} c2d_fp_config;

/* Per-step inputs of `update` (what FP_send_job packs, src/fp_mpi.f:632-686). */
typedef struct c2d_fp_step_in {
  int32_t ncycle;                 /* photon_fill (ncycle <= 1) sets dT_max=df_T */
  double time, dt;                /* time, dt(1)                               */
  c2d_array2 tea, tna, n_e, B_field, Eloss_sy, ec_old, turb_lev, vol;
  c2d_array2 f_pair;              /* NULL data = 0                             */
  c2d_array2 ecens;               /* NULL data: the context's tally buffer     */
  c2d_array3 n_field;             /* (i_ph, j, k); NULL data: tally buffer     */
} c2d_fp_step_in;

/* Per-zone diagnostics (optional output, [ncell][C2D_FP_NDIAG]). */
#define C2D_FP_E_OLD    0   /* zone's share of E_tot_old                       */
#define C2D_FP_E_NEW    1   /* zone's share of E_tot_new                       */
#define C2D_FP_HR       2   /* zone's share of hr_total                        */
#define C2D_FP_HR_ST    3   /* zone's share of hr_st_total                     */
#define C2D_FP_DELTA_T  4   /* |Te_new - tea| / Te_new                         */
#define C2D_FP_STEPS    5   /* implicit FP sub-steps taken                     */
#define C2D_FP_SKIPPED  6   /* 1: n_lept < 1e-11, zone left untouched          */
#define C2D_FP_NDIAG    8

/* In/out state.  f_nt, Pnt, n_e, gmin, gmax, amxwl, p_nth and tea are read
 * and updated in place; Te_new is written.  Views with NULL data are
 * skipped (tea: the update2d.f:266-276 clamp is then left to the caller).
 * f_nt and Pnt both NULL: the context's device electron state is read and
 * updated in place (C2D_DEV_ELECTRONS) and nothing 200-bin crosses the host. */
typedef struct c2d_fp_step_out {
  c2d_marray3 f_nt, Pnt;          /* (i<num_nt, j, k)                          */
  c2d_marray2 Te_new, tea, n_e, gmin, gmax, amxwl, p_nth;
  double* zone_diag;              /* optional [ncell][C2D_FP_NDIAG], cell=j*nr+k */
  double  E_tot_old, E_tot_new, hr_total, hr_st_total, dT_max;  /* E_add_up */
} c2d_fp_step_out;

/* ------------------------------------------------------------------------
 * Per-step emission / absorption tables (replaces the per-cell loop of
 * imcgen2d, src/imcgen2d.f:209-333, with volume_em, src/volume2d.f:10-394):
 * B from ep_switch, l_min, volume_em (kappa_tot = kappa_sy, eps_tot, eps_th,
 * Eloss_cy, Eloss_th), Eloss_sy from f_nt, and the dt*vol / dt*zsurf scaling.
 * Pair annihilation is inert (volume2d.f:322 skips it for f_pair < 1e-10; with
 * pair_switch = 1 a larger f_pair is C2D_E_ARG, hazard H6).
 * ---------------------------------------------------------------------- */
typedef struct c2d_vem_in {
  double dt;                                         /* dt(1)                     */
  c2d_array2 tea, tna, n_e, B_field, f_pair, zsurf, vol;
  c2d_iarray2 ep_switch;                             /* null data: all 0          */
  c2d_array3 f_nt;                                   /* (e-bin, j, k) like Pnt;
                                                        null data: the context's
                                                        device electron state   */
} c2d_vem_in;

typedef struct c2d_vem_out {                         /* any data may be NULL      */
  c2d_marray3 kappa_tot, eps_tot, eps_th;            /* (energy, j, k)            */
  c2d_marray2 B_field, Eloss_sy, Eloss_cy, Eloss_th, Eloss_tot;
  double* E_ph;                                      /* [C2D_N_VOL] photon grid   */
} c2d_vem_out;

/* ------------------------------------------------------------------------
 * Observer-frame binning of escape events on the device (replaces running
 * postprocessing/pspt.c:245-322 and plcm.c:382-456 over p###_evb.dat).
 * Bin edges are explicit arrays so each tool's own edge arithmetic is kept
 * (pspt: t0[n] = t0[0] + n*dt; plcm: t1[k] = t0[k+1] = t0[k] + dt).
 * ---------------------------------------------------------------------- */
#define C2D_OBS_SED 0   /* pspt.c: one closed mu window [mu0,mu1], first energy bin  */
#define C2D_OBS_LC  1   /* plcm.c: time - t_offset >= 0, half-open mu bins, every
                           energy band containing E                                 */
#define C2D_OBS_MAX_T   1024
#define C2D_OBS_MAX_MU  32
#define C2D_OBS_MAX_E   256

typedef struct c2d_obs_bins {
  int32_t mode;                   /* C2D_OBS_SED | C2D_OBS_LC                  */
  double  gam_bulk, rmax;         /* bulk Lorentz factor, r_max [cm]           */
  double  t_offset;               /* LC only                                   */
  int32_t n_t;  const double* t0; const double* t1;    /* observer time bins [s] */
  int32_t n_mu; const double* mu0; const double* mu1;  /* observer-frame cos   */
  int32_t n_e;  const double* E0; const double* E1;    /* observer energy [keV] */
} c2d_obs_bins;

const char* c2d_version(void);
int  c2d_init(const c2d_config* cfg, c2d_ctx** out);
void c2d_finalize(c2d_ctx* ctx);
const char* c2d_last_error(c2d_ctx* ctx);

/* One MC time step: census + volume + surface transport, all scatter
 * generations, tallies into the fused device buffer.  Synchronous.
 * Equivalent to c2d_set_step followed by c2d_run_step. */
int  c2d_transport_step(c2d_ctx* ctx, const c2d_step_in* in);

/* Upload the per-step tables (what imcgen2d/volume_em/file_sp produce) and
 * the clock; rebuilds the comtot table in C2D_COMTOT_TABLE mode. */
int  c2d_set_step(c2d_ctx* ctx, const c2d_step_in* in);
/* Advance the clock only (tables unchanged, e.g. T_const=1 runs). */
int  c2d_set_clock(c2d_ctx* ctx, int32_t ncycle, double time, double dt);
/* Transport with the tables of the last c2d_set_step.
 * On failure the double-buffered census (census_inplace = 0) is left as it
 * was.  The chunked census (census_inplace = 1) is rewritten in place once
 * generation 0 runs, so a failure after that LOSES it: c2d_census_count
 * then reports 0, and the census export/pack/append calls and the next
 * c2d_run_step return C2D_E_STATE until c2d_census_import or
 * c2d_census_truncate starts a new census. */
int  c2d_run_step(c2d_ctx* ctx);
/* Use caller-owned device memory (>= layout.total doubles on the context's
 * device) as the fused tally buffer, e.g. a torch tensor that is then
 * all-reduced over RCCL in place.  NULL restores the internal buffer. */
int  c2d_set_tally_buffer(c2d_ctx* ctx, double* device_ptr);

int  c2d_tally_layout_get(c2d_ctx* ctx, c2d_tally_layout* out);
/* Device pointer of the fused tally buffer (layout above), valid until the
 * next step; callers may all-reduce it in place (RCCL) before reading. */
double* c2d_tally_device_ptr(c2d_ctx* ctx);
/* Copy the fused tally buffer to host memory (total doubles). */
int  c2d_tally_download(c2d_ctx* ctx, double* host, int64_t n);
/* Copy tally words [offset, offset + n) of the fused buffer to host memory
 * (e.g. one tally and the counters, instead of the whole buffer per step). */
int  c2d_tally_download_range(c2d_ctx* ctx, double* host, int64_t offset, int64_t n);

/* Escape events of the last step: copies min(cap, n) records. */
int  c2d_events(c2d_ctx* ctx, double* buf, int64_t cap, int64_t* n);

/* Census held on the device for the next step. */
int  c2d_census_count(c2d_ctx* ctx, int64_t* n);
int  c2d_census_export(c2d_ctx* ctx, double* d6, int32_t* i5, uint64_t* keys,
                       int64_t cap, int64_t* n);
int  c2d_census_import(c2d_ctx* ctx, const double* d6, const int32_t* i5,
                       const uint64_t* keys, int64_t n);
/* Census records in device memory, for moving census between GPUs without
 * the host (imcredist, src/imcredist.f:5-133, as RCCL send/recv or
 * hipMemcpyPeer of packed records): C2D_CENSUS_REC_WORDS 64-bit words per
 * record = rpre, zpre, wmu, phi, ew, xnu (f64 bits), jk | bins << 32, key. */
#define C2D_CENSUS_REC_WORDS 8
/* pack records [first, first+n) into d_rec (device memory of this context's GPU) */
int  c2d_census_pack(c2d_ctx* ctx, int64_t first, int64_t n, uint64_t* d_rec);
/* append n packed records (device memory) to the census */
int  c2d_census_append(c2d_ctx* ctx, const uint64_t* d_rec, int64_t n);
/* keep the first n records (drop the tail, e.g. after packing it for a send) */
int  c2d_census_truncate(c2d_ctx* ctx, int64_t n);

/* Records first, first+stride, ... (at most cap of them) of the census:
 * checkpoints in chunks, or a strided sample of a large census. */
int  c2d_census_export_range(c2d_ctx* ctx, int64_t first, int64_t stride, double* d6,
                             int32_t* i5, uint64_t* keys, int64_t cap, int64_t* n);

/* Batched tridiagonal (Thomas with the reference's clipping) solve: one
 * zone per wavefront.  x is [ncell][nt] on the host. */
int  c2d_fp_tridag(c2d_ctx* ctx, const c2d_fp_in* in, double* x);

/* Fokker-Planck run constants (once per run; replaces setup_bcast and the
 * F_IC part of FP_bcast). */
int  c2d_fp_set_config(c2d_ctx* ctx, const c2d_fp_config* cfg);
/* One `update` (src/update2d.f:7-327) over all nz*nr zones: FP_calc for
 * every zone on the GPU (one wavefront per zone, state in LDS), the
 * E_add_up sums (zone order), the dT_max reduction and the tea update.
 * Replaces FP_send_job / FP_calc / FP_send_result / E_add_up /
 * FP_end_bcast.  Synchronous. */
int  c2d_fp_step(c2d_ctx* ctx, const c2d_fp_step_in* in, c2d_fp_step_out* out);
/* FP_calc arithmetic of the following c2d_fp_step calls:
 *   C2D_FP_EXACT (default): every sum, tridag's Thomas recurrence and
 *     McDonald's series in the reference's order -- bit for bit the det-math
 *     oracle (one in-order latency chain per zone);
 *   C2D_FP_FAST: the same per-bin and per-term arithmetic, the sums as block
 *     reductions/scans, tridag by parallel cyclic reduction, McDonald's terms
 *     summed as a tree (the same terms: the reference's stopping index) --
 *     equal to the exact mode within rounding (DESIGN.md §4b states the
 *     tolerance: f_nt 1e-10 relative, Te_new on the same 1.005 lattice);
 *   C2D_FP_AUTO: per update, C2D_FP_EXACT when every zone's tea sits on the
 *     reference's clamp (tea <= temp_min = 5 or >= temp_max = 1000 keV, the
 *     last update's Te_new clamped, src/update2d.f:266-276; skipped zones
 *     aside) and the last update's slowest zone took <= C2D_FP_AUTO_STEPS
 *     implicit sub-steps (src/update2d.f:1473; no last update: not asked):
 *     the exact kernel's in-order chain is then short (C3: 5 sub-steps,
 *     1.1 ms against the fast kernel's 3.4 ms); C2D_FP_FAST otherwise (off
 *     the clamp: ~29 ms against ~380 ms).  c2d_last_fp_mode reports it.
 * A fast update with no measured zone order yet (the context's first update;
 * either kernel's sub-step counts order the next) takes the zones costliest
 * first by an a-priori estimate: a probe launch evaluates every zone's first
 * implicit sub-step and orders the zones by 1/f_t_implicit (the sub-steps it
 * implies, src/update2d.f:662-665). */
#define C2D_FP_EXACT 0
#define C2D_FP_FAST  1
#define C2D_FP_AUTO  2
#define C2D_FP_AUTO_STEPS 64
int  c2d_fp_set_mode(c2d_ctx* ctx, int32_t mode);
/* The arithmetic the last c2d_fp_step used (C2D_FP_EXACT or C2D_FP_FAST:
 * C2D_FP_AUTO's choice); -1 before the first update. */
int  c2d_last_fp_mode(c2d_ctx* ctx, int32_t* mode);

/* Device timing of the last step's dominant kernel (transport generation 0):
 * milliseconds and launches, measured with HIP events on the library's
 * own stream. */
int  c2d_last_kernel_ms(c2d_ctx* ctx, double* gen0_ms, double* all_ms, int32_t* launches);
/* Diagnostic: section counters of the last step's transport launches
 * (wave-level shader cycles and event counts, tools/tr_prof.py).  All zero
 * unless the library was built with -DC2D_TR_PROF (FAST_FLAGS / EXACT). */
#define C2D_TR_PROF_WORDS 32
int  c2d_transport_prof(c2d_ctx* ctx, uint64_t* out, int32_t n);
/* Start an observer-frame histogram (zeroed on the device): sums of ew, of
 * ew^2 and counts per [n_t][n_mu][n_e] bin. */
int  c2d_obs_begin(c2d_ctx* ctx, const c2d_obs_bins* bins);
/* Bin escape events into it: events == NULL bins the last transport step's
 * device event buffer (c2d_events layout); otherwise n host events of 7 f64
 * (t_bound, xnu, ew, rpre, zpre, wmu, phi). */
int  c2d_obs_accumulate(c2d_ctx* ctx, const double* events, int64_t n);
/* Same for n events already in device memory on the context's GPU (e.g. a
 * gathered event buffer or a torch tensor); no copy. */
int  c2d_obs_accumulate_device(c2d_ctx* ctx, const double* d_events, int64_t n);
/* Download the raw sums ([n_t][n_mu][n_e] each; any pointer may be NULL)
 * and the device time of the binning launches so far (ms). */
int  c2d_obs_result(c2d_ctx* ctx, double* F, double* F2, double* count, double* kernel_ms);
/* The SED tool's binning from its own input dialogue: `deck` is pspt's stdin
 * (one answer a line, an empty line keeps pspt's default, "" or NULL = all
 * defaults; e.g. postprocessing/mrk421_sed.input), parsed and turned into
 * edges with pspt's arithmetic (postprocessing/pspt.c:105-205), then
 * c2d_obs_begin.  Replaces writing p###_evb.dat and running pspt on it. */
int  c2d_obs_begin_pspt(c2d_ctx* ctx, const char* deck);
/* Write pspt's output file (pspt.c:323-353, byte for byte its format) from
 * the histogram so far: `path` (NULL/"" = the deck's output file name),
 * `factor` as pspt's "#factor" line.  world_sum != 0: the histograms of every
 * rank of the context's communicator are summed first (RCCL; every rank
 * calls, rank 0 writes). */
int  c2d_obs_write_pspt(c2d_ctx* ctx, const char* path, int32_t factor, int32_t world_sum);

/* Copy the context's device electron state (C2D_DEV_ELECTRONS) into the
 * caller's f_nt / Pnt views (either may have NULL data), e.g. before
 * write_record (src/write_record.f) in a device-resident run. */
int  c2d_electron_state(c2d_ctx* ctx, c2d_marray3 f_nt, c2d_marray3 Pnt);

/* Device time of the last c2d_fp_step's FP kernel (HIP events, ms). */
int  c2d_last_fp_ms(c2d_ctx* ctx, double* ms);

/* imcgen2d's per-cell emission/absorption loop (volume_em for every cell)
 * on the GPU, one workgroup per cell; results written to the host arrays of
 * `out` that are non-NULL and kept on the device for a following
 * c2d_set_step with C2D_DEV_EMISSION.  Synchronous. */
int  c2d_volume_em(c2d_ctx* ctx, const c2d_vem_in* in, c2d_vem_out* out);
/* Device time of the last c2d_volume_em kernel (HIP events, ms). */
int  c2d_last_vem_ms(c2d_ctx* ctx, double* ms);
/* Packet-steps executed by that generation-0 launch (roofline numerator). */
int  c2d_last_gen0_steps(c2d_ctx* ctx, int64_t* steps);
/* Lane path-steps of the last step: passes of a GPU lane through the
 * geometry block (imctrk2d.f:228-379), of the generation-0 launch and of all
 * launches.  The per-copy tracker makes one per packet-step; a probe bundle
 * one per shared step of all the copies on its path, so
 * packet-steps / path-steps is the work sharing factor.  Either pointer may
 * be NULL. */
int  c2d_last_path_steps(c2d_ctx* ctx, int64_t* gen0_paths, int64_t* all_paths);
/* How the last step closed its census (the dbufout/ibufout of
 * imctrk2d.f:558-572 + imcfield2d.f:96-97): double-buffered, the rounds of
 * the compaction that closed the dead chunk tails and the records it moved;
 * chunked (census_inplace), the batches that packed the partly filled chunks
 * and their records.  physical = the census slots the context holds.  Any
 * pointer may be NULL. */
int  c2d_last_compaction(c2d_ctx* ctx, int32_t* rounds, int64_t* moved, int64_t* physical);
/* Chunked census (census_inplace = 1): the chunks the census occupies, the
 * chunks the last step's bundle kernel freed and refilled within the step,
 * the census chunks it could not count down (these wait for the next step),
 * and the chunks the context holds (1024 records each).  Double-buffered:
 * zeros.  Any pointer may be NULL. */
int  c2d_last_census_chunks(c2d_ctx* ctx, int64_t* chunks, int64_t* recycled, int64_t* unrecycled,
                            int64_t* physical);

/* ------------------------------------------------------------------------
 * Multi-GPU tally reduction over RCCL (xGMI), for hosts that drive one
 * context per GPU themselves (the kept Fortran driver, one MPI rank per GPU).
 * Replaces the per-step scalar MPI_REDUCE loops of xec_add /
 * graphics_collect (src/xec2d.f:325-399) and cens_add_up / E_add_up
 * (src/update2d.f:1929-2078) with ONE in-place all-reduce of the fused tally
 * buffer (c2d_tally_layout) per step.
 *   rank 0: c2d_comm_unique_id(id); the host broadcasts the C2D_COMM_ID_BYTES
 *   bytes (e.g. MPI_Bcast); every rank: c2d_comm_init(ctx, id, rank, world);
 *   per step after c2d_run_step: c2d_allreduce_tallies(ctx).
 * ---------------------------------------------------------------------- */
#define C2D_COMM_ID_BYTES 128
int  c2d_comm_unique_id(void* id, int64_t cap);
int  c2d_comm_init(c2d_ctx* ctx, const void* id, int32_t rank, int32_t world);
/* ncclAllReduce(sum, f64) in place on the context's tally buffer, on the
 * context's stream; synchronous.  Without c2d_comm_init: C2D_E_STATE. */
int  c2d_allreduce_tallies(c2d_ctx* ctx);
/* GPUs visible to this process (hipGetDeviceCount), so an MPI host can map
 * its ranks to devices (c2d_config.device); 0 and C2D_E_HIP without one. */
int  c2d_device_count(int32_t* n);

/* Diagnostics: evaluate the transport kernels' elementary functions on the
 * device (fn 0 log, 1 exp, 2 cos, 3 acos, 4 cbrt-by-pow, 5 sqrt, 6 x/3,
 * 7 Philox draw with key=x, counter=index) for bit-parity checks. */
int  c2d_selftest_math(int device, int fn, const double* x, double* y, int64_t n);
/* Diagnostics: the r-boundary distance of the flight step (src/imctrk2d.f:
 * 251-277: psq, dpbsq, disbr = inout*sqrt(dpbsq) - Eta*rpre, trldb =
 * disbr/sqrt(1 - wmu^2)) for n rays in[4n] = (rpre, Eta, wmu, rbnd; rbnd < 0:
 * the inner boundary |rbnd|, inout = -1) with
 * the fast build's square root / reciprocal sequences after `nr` Newton
 * steps (nr 1: the fast build, 2: its former default) and with IEEE sqrt
 * and division (nr 0: the exact build); out[2n] = (disbr, trldb). */
int  c2d_selftest_geom(int device, int nr, const double* in, double* out, int64_t n);
/* Diagnostics: the fast FP kernel's McDonald pair (volume2d.f:598-626) at n
 * arguments z from its moment table and from its term-by-term series;
 * out[8n] = (K2, K3 from the table, K2, K3 from the series, 1 if the table
 * answered, shader cycles of the table's gamma_bar and of the series,
 * gamma_bar = K3/K2 - 1/z as the fast kernel forms it from the table). */
int  c2d_selftest_mcd_fast(int device, const double* z, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* COMPTON2D_H */
