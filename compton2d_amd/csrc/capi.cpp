/*
 * capi.cpp — C-ABI implementation (include/compton2d.h) over the gfx950
 * transport kernels.  Host-side work is limited to gathering the
 * [1:nz,1:nr] sub-blocks of the caller's (strided, COMMON-layout) tables,
 * tiny per-step prefix sums, and the generation loop.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/compton2d.h"
#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_rng.h"
#include "pspt_host.h"

using namespace c2d;

extern "C" int c2d_launch_transport_exact(const KParams* P, const GenArgs* A, int grid, size_t lds,
                                          int trk, hipStream_t s);
extern "C" int c2d_launch_transport_fast(const KParams* P, const GenArgs* A, int grid, size_t lds,
                                         int trk, hipStream_t s);
extern "C" int c2d_launch_source_exact(const KParams* P, int grid, hipStream_t s);
extern "C" int c2d_launch_source_fast(const KParams* P, int grid, hipStream_t s);
extern "C" int c2d_launch_scatter_exact(const KParams* P, const GenArgs* A, int grid, int hard_grid, hipStream_t s);
extern "C" int c2d_launch_scatter_fast(const KParams* P, const GenArgs* A, int grid, int hard_grid, hipStream_t s);
extern "C" int c2d_transport_occupancy_exact(int* blocks_per_cu, size_t lds, int trk);
extern "C" int c2d_transport_occupancy_fast(int* blocks_per_cu, size_t lds, int trk);
extern "C" int c2d_aux_occupancy_exact(int which, int* blocks_per_cu);
extern "C" int c2d_aux_occupancy_fast(int which, int* blocks_per_cu);
extern "C" int c2d_launch_bundle_exact(const KParams* P, const GenArgs* A, int grid, size_t lds,
                                       int trk, hipStream_t s);
extern "C" int c2d_launch_bundle_fast(const KParams* P, const GenArgs* A, int grid, size_t lds,
                                      int trk, hipStream_t s);
extern "C" int c2d_bundle_occupancy_exact(int* blocks_per_cu, size_t lds, int trk);
extern "C" int c2d_bundle_occupancy_fast(int* blocks_per_cu, size_t lds, int trk);
extern "C" int c2d_launch_comtab_sigma(const double* gnt, double* S, hipStream_t s);
extern "C" int c2d_launch_comtab_gemm(const double* f_nt, const double* gnt, const double* S,
                                      double* tab, int ncell, hipStream_t s);
extern "C" int c2d_launch_fp(const FpParams* P, int ncell, int waves, hipStream_t s);
extern "C" int c2d_launch_fp_fast(const FpParams* dP, int ncell, int block, int grid, hipStream_t s);
extern "C" int c2d_fp_fast_block(int ncell, int n_simd);
extern "C" int c2d_fp_mom_build(const double* mcd, double* mom, hipStream_t stream);
extern "C" int c2d_fp_waves(int ncell, int n_simd);
extern "C" int c2d_launch_vem(const VemParams* P, int ncell, hipStream_t s);
extern "C" int c2d_launch_obs_segs(const ObsDev* O, const double* const* ev, const int64_t* n, int nseg,
                                   int grid, hipStream_t stream);
extern "C" int c2d_launch_obs(const ObsDev* O, const double* ev, int64_t n, int grid,
                              hipStream_t s);
extern "C" size_t c2d_obs_lds_bytes(int n_t, int n_mu, int n_e, int lds_rows);
extern "C" int c2d_obs_block(void);
extern "C" int c2d_launch_tridag(const double* a, const double* b, const double* c,
                                 const double* r, double* x, int ncell, int nt, hipStream_t s);

namespace {

/* CTL_EVSH: the C2D_EV_SHARDS event counters, one per 128-B line */
enum { CTL_WORK = 0, CTL_NCOUT = 1, CTL_POOLH = 2, CTL_N2 = 3, CTL_N3 = 4, CTL_NPK = 5,
       CTL_NOUT = 6, CTL_POOLN = 7, CTL_CNT = 8, CTL_RELN = CTL_CNT + C2D_NCOUNTERS, CTL_RELH, CTL_NHARD,
       CTL_EVSH = 32, CTL_PROF = CTL_EVSH + C2D_EV_SHARDS * C2D_EV_SHARD_STRIDE,
       CTL_WSH = CTL_PROF + C2D_TR_PROF_WORDS,
       CTL_WORDS = CTL_WSH + C2D_WORK_SHARDS * C2D_EV_SHARD_STRIDE };

static_assert(CTL_NHARD < CTL_EVSH, "control words overlap the event counters");

/* the packet store (c2d_device.hpp PktSoA) */
struct DevPk {
  double* d[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  uint32_t* jk = nullptr;
  uint32_t* bins = nullptr;
  uint32_t* ctr = nullptr;
  uint32_t* sub = nullptr;
  uint64_t* key = nullptr;
  int64_t* hard = nullptr;    /* the scatter kernel's hard list (GenArgs.hard) */
  int64_t cap = 0;
  PktSoA soa() const {
    PktSoA s;
    s.rpre = d[0]; s.zpre = d[1]; s.wmu = d[2]; s.phi = d[3]; s.ew = d[4]; s.xnu = d[5];
    s.dcen = d[6]; s.jk = jk; s.bins = bins; s.ctr = ctr; s.sub = sub; s.key = key;
    return s;
  }
  void release() {
    for (double*& p : d) { if (p) (void)hipFree(p); p = nullptr; }
    if (jk) (void)hipFree(jk);
    if (bins) (void)hipFree(bins);
    if (ctr) (void)hipFree(ctr);
    if (sub) (void)hipFree(sub);
    if (key) (void)hipFree(key);
    if (hard) (void)hipFree(hard);
    jk = bins = ctr = sub = nullptr;
    key = nullptr;
    hard = nullptr;
    cap = 0;
  }
};

struct DevCensus {
  c2d_d2* d[3] = {nullptr, nullptr, nullptr};   /* rz, wp, ex (CensusSoA) */
  c2d_u4* tg = nullptr;
  CensusSoA soa() const {
    CensusSoA s;
    s.rz = d[0]; s.wp = d[1]; s.ex = d[2]; s.tg = tg;
    return s;
  }
};

}  // namespace

struct c2d_ctx {
  Geo geo_h;                  /* host copy of the grids (census import's bin lookups) */
  c2d_config cfg;
  int nz = 0, nr = 0, ncell = 0, nmu = 0, nslot = 0;
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev_g0a = nullptr, ev_g0t = nullptr, ev_g0b = nullptr, ev_end = nullptr;
  int n_cu = 0, max_grid = 0, lds_cells = 0;
  size_t lds_max = 64 * 1024;   /* LDS bytes a workgroup may allocate */
  size_t lds_bytes = 0;
  /* generation 0 as probe bundles (c2d_bundle_kernel): its LDS and grid */
  int bundle = 1, bundle_grid = 0;
  int src_grid = 0, sc_grid = 0;   /* CUs x resident blocks of the source / scatter kernels */
  size_t bundle_lds = 0;
  /* census SoA(s) of cens_phys records each.  Double-buffered:
   * census_capacity + one append chunk per wave slot; the compaction's work
   * lists (cscan_cap slots each).  Chunked (census_inplace, c2d_device.hpp
   * C2D_CCHUNK): nchunks chunks, the census's chunk list (clist[ccur],
   * n_clist chunks, all full but the last) and the next step's. */
  int64_t cens_phys = 0;
  uint32_t cens_chunk = 64;
  int64_t n_ws = 0;              /* wave slots: the largest grid's waves (cstate entries) */
  int64_t* cstate = nullptr;     /* [n_ws][2] partly filled chunk per wave slot            */
  int chunked = 0;
  int64_t nchunks = 0;
  int32_t* clist[2] = {nullptr, nullptr};
  int ccur = 0;
  int64_t n_clist = 0;
  bool g0_launched = false;      /* this step's generation 0 has rewritten the chunked census */
  bool census_lost = false;      /* a failed in-place step overwrote the census (c2d_run_step) */
  int32_t* pool = nullptr;       /* [nchunks] free chunks at the step's start */
  int32_t* out_list = nullptr;   /* [nchunks] chunks the step took            */
  int32_t* relist = nullptr;     /* [nchunks] chunks freed and handed on      */
  uint8_t* cflag = nullptr;      /* [nchunks] in-use / partly-filled marks    */
  int32_t* part_id = nullptr;    /* [n_ws] partly filled chunks ...            */
  int64_t* part_off = nullptr;   /* [n_ws + 1] ... and their records' prefix   */
  uint64_t* tmp_rec = nullptr;   /* packed records (moves, exports)           */
  int64_t tmp_cap = 0;
  int64_t last_creuse = 0, last_clost = 0;
  int64_t* cscan = nullptr;      /* [2][cscan_cap]: dead slots below W, live slots at/above W */
  int64_t cscan_cap = 0;
  uint32_t* ctile_cnt = nullptr;           /* [tiles][2] holes, sources per tile       */
  unsigned long long* ctile_off = nullptr; /* [tiles][2] + totals: exclusive prefixes  */
  uint8_t* ctile_flag = nullptr;           /* [tiles] the tile holds a chunk tail        */
  int64_t ctile_cap = 0;
  int last_compact_rounds = 0;
  int64_t last_compact_moved = 0;
  c2d_tally_layout L;
  /* device buffers */
  Geo* geo = nullptr;
  double *gnt = nullptr, *kappa_cur = nullptr, *kappa_prev = nullptr, *eps_tot = nullptr,
         *eps_th = nullptr, *f_nt = nullptr, *Pnt = nullptr, *n_e = nullptr, *vfrac = nullptr,
         *ewsv = nullptr, *surf_ew = nullptr, *surf_tbb = nullptr, *tbbl = nullptr;
  int64_t *vol_prefix = nullptr, *surf_prefix = nullptr;
  int32_t* surf_spec = nullptr;
  SpecDev* spectra = nullptr;
  std::vector<double*> spec_bufs;
  int n_spectra = 0;
  double* comtab = nullptr;
  double* comS = nullptr;
  DevCensus cens[2];         /* census_inplace: cens[0] only; else in / out buffers */
  int cur = 0;               /* the buffer holding the census */
  int64_t n_census = 0;      /* live records: cens[cur][0, n_census) */
  double* ev = nullptr;
  int64_t n_ev = 0;
  int64_t ev_cnt[C2D_EV_SHARDS] = {};   /* events in each shard of the buffer (last step) */
  /* the context's own escapes binned on a second stream (c2d_obs_accumulate
   * with no events): it overlaps the next step's FP / tables / sources, and
   * the next generation-0 launch, which rewrites the event buffer, waits
   * for it (obs_settle reads its time when the host needs the result) */
  hipStream_t obs_stream = nullptr;
  hipEvent_t ev_obs_src = nullptr, ev_obs_a = nullptr, ev_obs_b = nullptr;
  bool obs_inflight = false;
  int64_t ev_cap_sh = 0;                /* per-shard capacity                             */
  ScatRec *q2[2] = {nullptr, nullptr}, *q3[2] = {nullptr, nullptr};
  DevPk pk;
  double* T = nullptr;
  double* T_own = nullptr;
  double* nf_rep = nullptr;     /* C2D_NF_REPL x ncell x nphfield */
  unsigned long long* ctl = nullptr;
  int32_t* derr = nullptr;
  KParams* dP = nullptr;
  /* host state of the current step */
  KParams P;
  bool have_step = false;
  bool have_electrons = false;  /* f_nt/Pnt hold an electron state (C2D_DEV_ELECTRONS) */
  bool have_vem = false;        /* vem_* hold the last c2d_volume_em tables (C2D_DEV_EMISSION) */
  int32_t* mono_flag = nullptr;
  /* RCCL communicator of the tally all-reduce (c2d_comm_init) */
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_world = 1;
  int64_t n_vol_global = 0, n_surf_global = 0;
  int eps_linear = 0;
  uint16_t* cdf_guide = nullptr;   /* [2][ncell][C2D_CDF_GUIDE + 1] (c2d_cdf_guide) */
  bool cdf_guide_on = false;
  std::vector<double> h_stage;
  double last_g0_ms = 0.0, last_all_ms = 0.0;
  float last_src_ms = 0.f;
  unsigned long long last_prof[C2D_TR_PROF_WORDS] = {};  /* transport section counters */
  int64_t last_g0_steps = 0;
  double egg_min = 0.0;          /* E_field(1)^2 / E_field(2) (census n_field threshold) */
  int64_t last_g0_paths = 0, last_all_paths = 0;   /* lane path-steps (C2D_CNT_PATHS_INT) */
  int last_launches = 0;
  /* Fokker-Planck */
  bool fp_ready = false;
  c2d_fp_config fpc;
  double *fp_FT = nullptr, *fp_mcd = nullptr, *fp_zin = nullptr, *fp_fin = nullptr, *fp_Pin = nullptr,
         *fp_nf = nullptr, *fp_fout = nullptr, *fp_Pout = nullptr, *fp_zout = nullptr;
  int32_t* fp_err = nullptr;
  unsigned long long* fp_gb_key = nullptr;   /* gamma_bar memo (fp.hip GbMemo) */
  double* fp_gb_val = nullptr;
  int32_t fp_mode = C2D_FP_EXACT;             /* c2d_fp_set_mode */
  unsigned long long* fpf_gb_key = nullptr;  /* the fast kernel's own gamma_bar memo */
  double* fpf_gb_val = nullptr;
  FpParams* fp_dP = nullptr;                 /* FpParams in device memory (fast kernel) */
  int32_t* fpf_zq = nullptr;                 /* fast kernel: zone queue head + order [1 + ncell] */
  double* fpf_mom = nullptr;                 /* fast kernel: McDonald moment table              */
  std::vector<int32_t> fpf_order;            /* zones by the last update's sub-steps, costliest first */
  bool fpf_ordered = false;                  /* fpf_order holds a measured order */
  /* C2D_FP_AUTO: the next update's choice, from the last update */
  bool fp_auto_known = false, fp_auto_exact = false;
  int32_t last_fp_mode = -1;
  float last_fp_ms = 0.f;
  int last_fp_waves = 0;
  /* emission / absorption tables (c2d_volume_em) */
  double *vem_zin = nullptr, *vem_fnt = nullptr, *vem_eph = nullptr, *vem_kap = nullptr,
         *vem_et = nullptr, *vem_eh = nullptr, *vem_zout = nullptr;
  float last_vem_ms = 0.f;
  /* observer-frame binning */
  bool obs_ready = false;
  ObsDev obs;
  double *obs_edges = nullptr, *obs_hist = nullptr, *obs_ev = nullptr;
  double* pspt_red = nullptr;                 /* world_sum reduction buffer, 2 x n_t x n_e */
  c2d_pspt_deck pspt;                         /* c2d_obs_begin_pspt's deck */
  bool pspt_on = false;
  int64_t obs_ev_cap = 0;
  int obs_wg_per_cu = 1;
  double obs_ms = 0.0;
};

static int fail(c2d_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, x)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail((c), C2D_E_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #x,              \
                  hipGetErrorString(e_));                                              \
  } while (0)

template <class T>
static hipError_t dalloc(T** p, size_t n) {
  if (n == 0) n = 1;
  return hipMalloc((void**)p, n * sizeof(T));
}

extern "C" const char* c2d_version(void) { return "compton2d_amd 0.1.0 (gfx950)"; }

extern "C" const char* c2d_last_error(c2d_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

/* Geo bucket tables of grid_lookup (c2d_device.hpp): bucket b holds the
 * bin (smallest i in [1, n] with x < E[i+1], the bisection's answer) of the
 * smallest double whose top 16 bits are k0 + b. */
static int grid_bin_host(const double* E, int n, double x) {
  int lo = 1, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (x < E[mid + 1]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
static void build_lookup(const double* E, int n, int16_t* start, int32_t* k0) {
  uint64_t u;
  std::memcpy(&u, &E[1], sizeof u);
  *k0 = (int32_t)(u >> 48);
  for (int b = 0; b < C2D_IDX_BUCKETS; b++) {
    const uint64_t k = (uint64_t)(*k0 + b);
    double x = 0.0;
    if (k < 0x7ff0) {
      const uint64_t v = k << 48;
      std::memcpy(&x, &v, sizeof x);
      start[b] = (int16_t)grid_bin_host(E, n, x);
    } else {
      start[b] = (int16_t)(b > 0 ? start[b - 1] : 1);
    }
  }
}

extern "C" int c2d_init(const c2d_config* cfg, c2d_ctx** out) {
  if (!cfg || !out) return C2D_E_ARG;
  *out = nullptr;
  if (cfg->nz < 1 || cfg->nr < 1 || cfg->nz > C2D_MAXZONE || cfg->nr > C2D_MAXZONE)
    return C2D_E_ARG;
  if (cfg->nphtotal < 1 || cfg->nphtotal > C2D_NPHOMAX || cfg->nph_lc < 0 ||
      cfg->nph_lc > C2D_NPHLCMAX || cfg->nmu < 1 || cfg->nmu > C2D_NMUMAX)
    return C2D_E_ARG;
  if (cfg->cr_sent != 0) return C2D_E_ARG;   /* Compton reflection not supported */
  if (cfg->trk_variant != C2D_TRK_SRC && cfg->trk_variant != C2D_TRK_2012_11) return C2D_E_ARG;
  if (cfg->split1 < 1 || cfg->split2 < 1 || cfg->split3 < 1 || cfg->world < 1 ||
      cfg->rank < 0 || cfg->rank >= cfg->world)
    return C2D_E_ARG;
  /* the event buffer is C2D_EV_SHARDS equal shards; each must hold events */
  if (cfg->event_capacity < C2D_EV_SHARDS) return C2D_E_ARG;
  c2d_ctx* c = new c2d_ctx();
  c->cfg = *cfg;
  c->nz = cfg->nz;
  c->nr = cfg->nr;
  c->ncell = cfg->nz * cfg->nr;
  c->nmu = cfg->nmu;
  c->nslot = 2 * cfg->nz + 2 * cfg->nr;
  c2d_tally_layout_for(c->nz, c->nr, c->nmu, &c->L);
  *out = c;

  HIPCHK(c, hipSetDevice(cfg->device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIPCHK(c, hipStreamCreateWithFlags(&c->obs_stream, hipStreamNonBlocking));
  HIPCHK(c, hipEventCreateWithFlags(&c->ev_obs_src, hipEventDisableTiming));
  HIPCHK(c, hipEventCreate(&c->ev_obs_a));
  HIPCHK(c, hipEventCreate(&c->ev_obs_b));
  HIPCHK(c, hipEventCreate(&c->ev_g0a));
  HIPCHK(c, hipEventCreate(&c->ev_g0b));
  HIPCHK(c, hipEventCreate(&c->ev_g0t));
  HIPCHK(c, hipEventCreate(&c->ev_end));
  hipDeviceProp_t prop;
  HIPCHK(c, hipGetDeviceProperties(&prop, cfg->device));
  c->n_cu = prop.multiProcessorCount;
  c->lds_max = std::max<size_t>(prop.sharedMemPerBlock, 64 * 1024);

  /* grids (1-based like the reference COMMON) */
  Geo g;
  memset(&g, 0, sizeof g);
  g.z[0] = cfg->zmin;
  g.r[0] = cfg->rmin;
  for (int j = 0; j < c->nz; j++) g.z[j + 1] = cfg->z[j];
  for (int k = 0; k < c->nr; k++) g.r[k + 1] = cfg->r[k];
  for (int i = 0; i < C2D_N_VOL; i++) g.E_ph[i + 1] = cfg->E_ph[i];
  for (int i = 0; i < C2D_NPHFIELD; i++) g.E_field[i + 1] = cfg->E_field[i];
  c->egg_min = (g.E_field[1] * g.E_field[1]) / g.E_field[2];   /* imctrk2d.f Egg_min */
  build_lookup(g.E_ph, C2D_N_VOL, g.eph_start, &g.eph_k0);
  build_lookup(g.E_field, C2D_NPHFIELD, g.efl_start, &g.efl_k0);
  for (int i = 0; i <= cfg->nphtotal; i++) g.hu[i + 1] = cfg->hu[i];
  for (int m = 0; m < cfg->nph_lc; m++) {
    g.Elcmin[m + 1] = cfg->Elcmin[m];
    g.Elcmax[m + 1] = cfg->Elcmax[m];
  }
  for (int n = 0; n < cfg->nmu; n++) g.mu[n + 1] = cfg->mu[n];
  HIPCHK(c, dalloc(&c->geo, 1));
  HIPCHK(c, hipMemcpy(c->geo, &g, sizeof g, hipMemcpyHostToDevice));
  c->geo_h = g;
  HIPCHK(c, dalloc(&c->gnt, C2D_NUM_NT));
  HIPCHK(c, hipMemcpy(c->gnt, cfg->gnt, sizeof(double) * C2D_NUM_NT, hipMemcpyHostToDevice));

  const size_t nc = (size_t)c->ncell;
  HIPCHK(c, dalloc(&c->kappa_cur, nc * C2D_N_VOL));
  HIPCHK(c, dalloc(&c->kappa_prev, nc * C2D_N_VOL));
  HIPCHK(c, hipMemset(c->kappa_prev, 0, nc * C2D_N_VOL * sizeof(double)));
  HIPCHK(c, dalloc(&c->eps_tot, nc * C2D_N_VOL));
  HIPCHK(c, dalloc(&c->eps_th, nc * C2D_N_VOL));
  HIPCHK(c, dalloc(&c->f_nt, nc * C2D_NUM_NT));
  HIPCHK(c, dalloc(&c->Pnt, nc * C2D_NUM_NT));
  HIPCHK(c, dalloc(&c->n_e, nc));
  HIPCHK(c, dalloc(&c->ewsv, nc));
  HIPCHK(c, dalloc(&c->vfrac, nc * 4));
  HIPCHK(c, dalloc(&c->vol_prefix, nc + 1));
  HIPCHK(c, dalloc(&c->surf_prefix, (size_t)c->nslot + 1));
  HIPCHK(c, dalloc(&c->surf_ew, (size_t)c->nslot));
  HIPCHK(c, dalloc(&c->surf_tbb, (size_t)c->nslot));
  HIPCHK(c, dalloc(&c->surf_spec, (size_t)c->nslot));
  HIPCHK(c, dalloc(&c->tbbl, (size_t)c->nr));
  if (cfg->comtot_mode == C2D_COMTOT_TABLE) {
    HIPCHK(c, dalloc(&c->comtab, nc * C2D_COMTAB_N));
    HIPCHK(c, dalloc(&c->comS, (size_t)C2D_COMTAB_N * C2D_NUM_NT));
    int rc = c2d_launch_comtab_sigma(c->gnt, c->comS, c->stream);
    if (rc) return fail(c, C2D_E_HIP, "comtab_sigma launch: %d", rc);
  }
  HIPCHK(c, dalloc(&c->ev, (size_t)std::max<int64_t>(cfg->event_capacity, 1) * C2D_EVENT_WORDS));
  const int64_t qcap = std::max<int64_t>(cfg->queue_capacity, 1);
  for (int b = 0; b < 2; b++) {
    HIPCHK(c, dalloc(&c->q2[b], qcap));
    HIPCHK(c, dalloc(&c->q3[b], qcap));
  }
  HIPCHK(c, dalloc(&c->T_own, (size_t)c->L.total));
  HIPCHK(c, hipMemset(c->T_own, 0, sizeof(double) * c->L.total));
  HIPCHK(c, dalloc(&c->nf_rep, (size_t)C2D_NF_REPL * c->ncell * C2D_NPHFIELD));
  c->T = c->T_own;
  HIPCHK(c, dalloc(&c->ctl, CTL_WORDS));
  HIPCHK(c, dalloc(&c->derr, 1));
  HIPCHK(c, dalloc(&c->dP, 1));

  /* LDS plan: Geo image + (cell tallies if they fit) + escape tallies */
  const size_t esc = (size_t)c->nmu * (C2D_NPHOMAX + C2D_NPHLCMAX) + 2 * c->nz + 2 * c->nr;
  c->lds_cells = (4 * nc * sizeof(double) <= 48 * 1024) ? 1 : 0;
  c->lds_bytes = sizeof(double) * (GEO_DOUBLES + (c->lds_cells ? 4 * nc : 0) + esc);
  /* persistent grid = CUs x resident blocks per CU (VGPR- or LDS-limited,
   * from the runtime's occupancy calculator for this kernel and LDS size) */
  int blocks_per_cu = 0;
  int orc = cfg->comtot_mode == C2D_COMTOT_TABLE
                ? c2d_transport_occupancy_fast(&blocks_per_cu, c->lds_bytes, cfg->trk_variant)
                : c2d_transport_occupancy_exact(&blocks_per_cu, c->lds_bytes, cfg->trk_variant);
  if (orc) return fail(c, C2D_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)orc));
  c->max_grid = c->n_cu * std::max(1, blocks_per_cu);
  {
    auto occ = cfg->comtot_mode == C2D_COMTOT_TABLE ? c2d_bundle_occupancy_fast
                                                    : c2d_bundle_occupancy_exact;
    int b0 = 0;
    orc = occ(&b0, c->lds_bytes, cfg->trk_variant);
    if (orc) return fail(c, C2D_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)orc));
    c->bundle_lds = c->lds_bytes;
    c->bundle_grid = c->n_cu * std::max(1, b0);
  }
  {
    auto aocc = cfg->comtot_mode == C2D_COMTOT_TABLE ? c2d_aux_occupancy_fast : c2d_aux_occupancy_exact;
    int bs = 0, bc = 0;
    orc = aocc(0, &bs);
    if (!orc) orc = aocc(1, &bc);
    if (orc) return fail(c, C2D_E_HIP, "occupancy query: %s", hipGetErrorString((hipError_t)orc));
    c->src_grid = c->n_cu * std::max(1, bs);
    c->sc_grid = c->n_cu * std::max(1, bc);
  }
  {
    /* the census.  A wave slot keeps one partly filled append chunk over
     * the step's launches (cstate), so a step leaves at most n_ws of them. */
    const int64_t ccap = std::max<int64_t>(cfg->census_capacity, 1);
    c->n_ws = (int64_t)std::max(c->bundle_grid, c->max_grid) * (C2D_TR_BLOCK / 64);
    HIPCHK(c, dalloc(&c->cstate, 2 * (size_t)c->n_ws));
    HIPCHK(c, hipMemset(c->cstate, 0xff, 2 * sizeof(int64_t) * c->n_ws));
    c->chunked = cfg->census_inplace ? 1 : 0;
    if (c->chunked) {
      /* chunked: the chunks of the census, the wave slots' partly filled
       * ones, and 1/16 of the capacity for chunks whose sources are still
       * in flight when the waves need new ones (c2d_device.hpp) */
      c->cens_chunk = C2D_CCHUNK;
      /* additive slack: per wave slot one partly filled chunk, the 2-3 chunks
       * whose sources are in flight and the free stack's turnover; test knob
       * C2D_CHUNK_SLACK replaces it by a fixed number of chunks, so a test
       * can pin that the usable capacity is census_capacity with only the
       * chunks its waves need beside the capacity/16 term */
      int64_t slack = 4 * c->n_ws + 64;
      if (const char* e = getenv("C2D_CHUNK_SLACK")) slack = std::max<long long>(0, atoll(e));
      c->nchunks = (ccap + C2D_CCHUNK - 1) / C2D_CCHUNK + (ccap / 16 + C2D_CCHUNK - 1) / C2D_CCHUNK + slack;
      c->cens_phys = c->nchunks * C2D_CCHUNK;
      for (int b = 0; b < 2; b++) HIPCHK(c, dalloc(&c->clist[b], (size_t)c->nchunks));
      HIPCHK(c, dalloc(&c->pool, (size_t)c->nchunks));
      HIPCHK(c, dalloc(&c->out_list, (size_t)c->nchunks));
      HIPCHK(c, dalloc(&c->relist, (size_t)c->nchunks));
      HIPCHK(c, dalloc(&c->cflag, (size_t)c->nchunks));
      HIPCHK(c, dalloc(&c->part_id, (size_t)c->n_ws));
      HIPCHK(c, dalloc(&c->part_off, (size_t)c->n_ws + 1));
    } else {
      /* double-buffered: append chunks <= 1024 slots, >= 64 (one reservation
       * covers a wave's census lanes), their tails at most 1/8 of the
       * capacity; the physical size adds room for every tail, so a census
       * whose compacted size fits the capacity does not overflow */
      int64_t ch = 1024;
      while (ch > 64 && ch * c->n_ws * 8 > ccap) ch >>= 1;
      c->cens_chunk = (uint32_t)ch;
      c->cens_phys = ccap + c->n_ws * ch + 64;
      c->cscan_cap = std::min<int64_t>(int64_t(1) << 27, std::max<int64_t>(int64_t(1) << 16, ccap / 16));
      /* test knob: a short work list forces many compaction rounds */
      if (const char* e = getenv("C2D_COMPACT_LIST")) c->cscan_cap = std::max<long long>(1, atoll(e));
      HIPCHK(c, dalloc(&c->cscan, 2 * (size_t)c->cscan_cap));
    }
    for (int b = 0; b < (c->chunked ? 1 : 2); b++) {
      for (int f = 0; f < 3; f++) HIPCHK(c, dalloc(&c->cens[b].d[f], (size_t)c->cens_phys));
      HIPCHK(c, dalloc(&c->cens[b].tg, (size_t)c->cens_phys));
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return C2D_OK;
}

extern "C" void c2d_finalize(c2d_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->obs_stream) (void)hipStreamSynchronize(c->obs_stream);   /* it reads the event buffer */
  if (c->mono_flag) (void)hipFree(c->mono_flag);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  void* ptrs[] = {c->geo, c->gnt, c->kappa_cur, c->kappa_prev, c->eps_tot, c->eps_th, c->f_nt,
                  c->Pnt, c->n_e, c->vfrac, c->ewsv, c->surf_ew, c->surf_tbb, c->tbbl,
                  c->vol_prefix, c->surf_prefix, c->surf_spec, c->spectra, c->comtab, c->comS,
                  c->ev, c->q2[0], c->q2[1], c->q3[0], c->q3[1], c->T_own, c->nf_rep, c->ctl, c->derr, c->dP,
                  c->cscan, c->ctile_cnt, c->ctile_off, c->ctile_flag, c->cstate, c->clist[0], c->clist[1],
                  c->pool, c->out_list, c->relist, c->cflag, c->part_id, c->part_off, c->tmp_rec};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int b = 0; b < 2; b++) {
    for (int f = 0; f < 3; f++)
      if (c->cens[b].d[f]) (void)hipFree(c->cens[b].d[f]);
    if (c->cens[b].tg) (void)hipFree(c->cens[b].tg);
  }
  for (double* p : c->spec_bufs) (void)hipFree(p);
  void* optrs[] = {c->obs_edges, c->obs_hist, c->obs_ev, c->pspt_red, c->cdf_guide};
  for (void* p : optrs)
    if (p) (void)hipFree(p);
  void* vptrs[] = {c->vem_zin, c->vem_fnt, c->vem_eph, c->vem_kap, c->vem_et, c->vem_eh, c->vem_zout};
  for (void* q : vptrs)
    if (q) (void)hipFree(q);
  void* fptrs[] = {c->fp_FT, c->fp_mcd, c->fp_zin, c->fp_fin, c->fp_Pin, c->fp_nf, c->fp_fout, c->fp_Pout,
                   c->fp_zout, c->fp_err, c->fp_gb_key, c->fp_gb_val, c->fpf_gb_key, c->fpf_gb_val,
                   c->fp_dP, c->fpf_zq, c->fpf_mom};
  for (void* p : fptrs)
    if (p) (void)hipFree(p);
  c->pk.release();
  if (c->ev_g0a) (void)hipEventDestroy(c->ev_g0a);
  if (c->ev_g0b) (void)hipEventDestroy(c->ev_g0b);
  if (c->ev_g0t) (void)hipEventDestroy(c->ev_g0t);
  if (c->ev_end) (void)hipEventDestroy(c->ev_end);
  if (c->obs_stream) (void)hipStreamSynchronize(c->obs_stream);
  if (c->ev_obs_src) (void)hipEventDestroy(c->ev_obs_src);
  if (c->ev_obs_a) (void)hipEventDestroy(c->ev_obs_a);
  if (c->ev_obs_b) (void)hipEventDestroy(c->ev_obs_b);
  if (c->obs_stream) (void)hipStreamDestroy(c->obs_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

/* gather (i, j, k) of a strided table into dense [cell][n] */
static void gather3(const c2d_ctx* c, const c2d_array3& a, int n, double* out) {
  for (int j = 0; j < c->nz; j++)
    for (int k = 0; k < c->nr; k++) {
      double* o = out + (size_t)(j * c->nr + k) * n;
      if (!a.data) {
        std::fill(o, o + n, 0.0);
        continue;
      }
      const double* base = a.data + j * a.s_j + k * a.s_k;
      if (a.s_i == 1)
        memcpy(o, base, sizeof(double) * n);
      else
        for (int i = 0; i < n; i++) o[i] = base[i * a.s_i];
    }
}
static double at2(const c2d_array2& a, int j, int k) {
  return a.data ? a.data[j * a.s_j + k * a.s_k] : 0.0;
}

extern "C" int c2d_set_clock(c2d_ctx* c, int32_t ncycle, double time, double dt) {
  if (!c) return C2D_E_ARG;
  c->P.ncycle = ncycle;
  c->P.time = time;
  c->P.dt = dt;
  c->P.cdt = 2.9979245620e10 * dt;                 /* dcen = c_light*dt(1), imcfield2d.f:117 */
  c->P.cens_wlim = c->cfg.trk_variant == C2D_TRK_2012_11 ? 1.0 : 0.99999999;
  c->P.step_key = c2d_step_key(c->cfg.seed, ncycle);
  return C2D_OK;
}

/* flag = 1 if some row of a [rows][n] table is not non-decreasing (or NaN):
 * the emission CDFs are then searched linearly, as the reference does */
__global__ void __launch_bounds__(256) c2d_check_monotone(const double* __restrict__ a, int rows, int n,
                                                          int32_t* __restrict__ flag) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < (int64_t)rows * n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(t % n);
    if (i > 0 && !(a[t] >= a[t - 1])) atomicOr(flag, 1);
  }
}

/* flag |= bit if some a[i], i < n, is NaN or +-Inf.  The fail-loud guard on
 * tables, tallies and the electron state: the reference carries a NaN on
 * (NaN counts cast to int, a run that tracks nothing), the library stops. */
__global__ void __launch_bounds__(256) c2d_check_finite(const double* __restrict__ a, int64_t n, int32_t bit,
                                                        int32_t* __restrict__ flag) {
  bool bad = false;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    bad |= !(fabs(a[t]) <= DBL_MAX);
  if (bad) atomicOr(flag, bit);
}

static void check_finite(c2d_ctx* c, const double* a, int64_t n, int32_t bit, int32_t* flag, hipStream_t st) {
  if (n <= 0) return;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 4));
  hipLaunchKernelGGL(c2d_check_finite, dim3(grid), dim3(256), 0, st, a, n, bit, flag);
}

static bool all_finite(const double* a, size_t n) {
  for (size_t i = 0; i < n; i++)
    if (!std::isfinite(a[i])) return false;
  return true;
}

/* guide rows of the emission CDFs (KParams.cdf_guide): row (t, cell), entry q
 * = the smallest i in [1, n] with cdf(i) >= q / C2D_CDF_GUIDE, n if none --
 * cdf_index's own predicate, so its search restricted to [guide[q],
 * guide[q+1]] returns the same index as over [1, n] */
__global__ void __launch_bounds__(256) c2d_cdf_guide(const double* __restrict__ eps_tot,
                                                     const double* __restrict__ eps_th, int ncell, int n,
                                                     uint16_t* __restrict__ guide) {
  const int64_t rows = 2 * (int64_t)ncell, per = C2D_CDF_GUIDE + 1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < rows * per;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t / per;
    const int q = (int)(t % per);
    const double* cdf = (row < ncell ? eps_tot : eps_th) + (row % ncell) * (int64_t)n;
    const double thr = (double)q * (1.0 / C2D_CDF_GUIDE);
    int lo = 1, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid - 1] < thr) lo = mid + 1;
      else hi = mid;
    }
    guide[t] = (uint16_t)lo;
  }
}

extern "C" int c2d_set_step(c2d_ctx* c, const c2d_step_in* in) {
  if (!c || !in) return C2D_E_ARG;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  /* a failed c2d_set_step leaves no step to run (tables may be half replaced) */
  c->have_step = false;
  const int nz = c->nz, nr = c->nr, nc = c->ncell;
  const size_t nvol = (size_t)nc * C2D_N_VOL, nnt = (size_t)nc * C2D_NUM_NT;
  const int dev = in->device_tables;
  if (dev & ~(C2D_DEV_EMISSION | C2D_DEV_ELECTRONS))
    return fail(c, C2D_E_ARG, "c2d_set_step: unknown device_tables flags 0x%x", dev);
  if ((dev & C2D_DEV_EMISSION) && !c->have_vem)
    return fail(c, C2D_E_STATE, "C2D_DEV_EMISSION needs a preceding c2d_volume_em");
  if ((dev & C2D_DEV_ELECTRONS) && !c->have_electrons)
    return fail(c, C2D_E_STATE, "C2D_DEV_ELECTRONS needs an electron state on the device");
  if (dev & C2D_DEV_EMISSION) {
    const hipStream_t st = c->stream;
    HIPCHK(c, hipMemcpyAsync(c->kappa_cur, c->vem_kap, nvol * sizeof(double), hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->eps_tot, c->vem_et, nvol * sizeof(double), hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->eps_th, c->vem_eh, nvol * sizeof(double), hipMemcpyDeviceToDevice, st));
    if (!c->mono_flag) HIPCHK(c, dalloc(&c->mono_flag, 1));
    HIPCHK(c, hipMemsetAsync(c->mono_flag, 0, sizeof(int32_t), st));
    const int grid = (int)std::min<int64_t>(((int64_t)nvol + 255) / 256, (int64_t)c->n_cu * 4);
    hipLaunchKernelGGL(c2d_check_monotone, dim3(grid), dim3(256), 0, st, c->eps_tot, nc, C2D_N_VOL,
                       c->mono_flag);
    hipLaunchKernelGGL(c2d_check_monotone, dim3(grid), dim3(256), 0, st, c->eps_th, nc, C2D_N_VOL,
                       c->mono_flag);
    check_finite(c, c->kappa_cur, (int64_t)nvol, 2, c->mono_flag, st);
    check_finite(c, c->eps_tot, (int64_t)nvol, 2, c->mono_flag, st);
    check_finite(c, c->eps_th, (int64_t)nvol, 2, c->mono_flag, st);
    HIPCHK(c, hipGetLastError());
    int32_t nonmono = 0;
    HIPCHK(c, hipMemcpyAsync(&nonmono, c->mono_flag, sizeof nonmono, hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (nonmono & 2)
      return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in the device emission/absorption tables "
                  "(kappa_tot, eps_tot or eps_th of the last c2d_volume_em)");
    c->eps_linear = nonmono & 1;
  } else {
    std::vector<double>& h = c->h_stage;
    h.resize(nvol);
    gather3(c, in->kappa_tot, C2D_N_VOL, h.data());
    if (!all_finite(h.data(), nvol)) return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in kappa_tot");
    HIPCHK(c, hipMemcpy(c->kappa_cur, h.data(), nvol * sizeof(double), hipMemcpyHostToDevice));
    gather3(c, in->eps_tot, C2D_N_VOL, h.data());
    if (!all_finite(h.data(), nvol)) return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in eps_tot");
    int nonmono = 0;
    for (int cc = 0; cc < nc && !nonmono; cc++)
      for (int i = 1; i < C2D_N_VOL; i++)
        if (!(h[(size_t)cc * C2D_N_VOL + i] >= h[(size_t)cc * C2D_N_VOL + i - 1])) { nonmono = 1; break; }
    HIPCHK(c, hipMemcpy(c->eps_tot, h.data(), nvol * sizeof(double), hipMemcpyHostToDevice));
    gather3(c, in->eps_th, C2D_N_VOL, h.data());
    if (!all_finite(h.data(), nvol)) return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in eps_th");
    for (int cc = 0; cc < nc && !nonmono; cc++)
      for (int i = 1; i < C2D_N_VOL; i++)
        if (!(h[(size_t)cc * C2D_N_VOL + i] >= h[(size_t)cc * C2D_N_VOL + i - 1])) { nonmono = 1; break; }
    HIPCHK(c, hipMemcpy(c->eps_th, h.data(), nvol * sizeof(double), hipMemcpyHostToDevice));
    c->eps_linear = nonmono;
  }
  if (!(dev & C2D_DEV_ELECTRONS)) {
    std::vector<double> hn(nnt);
    gather3(c, in->f_nt, C2D_NUM_NT, hn.data());
    if (!all_finite(hn.data(), nnt)) return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in f_nt");
    HIPCHK(c, hipMemcpy(c->f_nt, hn.data(), nnt * sizeof(double), hipMemcpyHostToDevice));
    gather3(c, in->Pnt, C2D_NUM_NT, hn.data());
    if (!all_finite(hn.data(), nnt)) return fail(c, C2D_E_NONFINITE, "c2d_set_step: NaN/Inf in Pnt");
    HIPCHK(c, hipMemcpy(c->Pnt, hn.data(), nnt * sizeof(double), hipMemcpyHostToDevice));
    c->have_electrons = true;
  }

  /* zone scalars, volume fractions (imcvol2d_para.f:119-149), volume prefix */
  std::vector<double> ne(nc), ew(nc), vf(4 * (size_t)nc);
  std::vector<int64_t> vp(nc + 1);
  vp[0] = 0;
  for (int j = 0; j < nz; j++)
    for (int k = 0; k < nr; k++) {
      const int cell = j * nr + k;
      ne[cell] = at2(in->n_e, j, k);
      ew[cell] = at2(in->ewsv, j, k);
      const int jv = j + 1, kv = k + 1;
      const double zj = c->cfg.z[j], zjm = (jv == 1) ? 0.0 : c->cfg.z[j - 1];
      const double delz = (jv == 1) ? c->cfg.z[0] : zj - zjm;
      const double zs = at2(in->zsurf, j, k);
      const double rlow = (kv == 1) ? c->cfg.rmin : c->cfg.r[k - 1];
      const double rk = c->cfg.r[k];
      const double fi = (4.4e1 / 7.0 * rlow * delz) / zs;
      const double fo = (4.4e1 / 7.0 * rk * delz) / zs;
      const double fu = (2.2e1 / 7.0 * (rk * rk - rlow * rlow)) / zs;
      vf[4 * cell + 0] = at2(in->Eloss_th, j, k) / at2(in->Eloss_tot, j, k);
      vf[4 * cell + 1] = fi;
      vf[4 * cell + 2] = fi + fo;
      vf[4 * cell + 3] = (fi + fo) + fu;
      const int32_t nsv = in->nsv.data ? in->nsv.data[j * in->nsv.s_j + k * in->nsv.s_k] : 0;
      /* a negative count is a NaN budget cast to an integer (imcgen2d.f:448-517
       * on a non-finite Eloss_tot): the reference's `do i=1,nsv` would skip the
       * zone silently and the run would track nothing */
      if (nsv < 0)
        return fail(c, C2D_E_ARG, "c2d_set_step: nsv(%d,%d) = %d < 0 (a non-finite volume budget?)",
                    j + 1, k + 1, (int)nsv);
      if (!std::isfinite(ne[cell]))
        return fail(c, C2D_E_NONFINITE, "c2d_set_step: n_e(%d,%d) is not finite", j + 1, k + 1);
      if (nsv > 0 && !(std::isfinite(ew[cell]) && std::isfinite(vf[4 * cell]) && std::isfinite(vf[4 * cell + 3])))
        return fail(c, C2D_E_NONFINITE, "c2d_set_step: zone (%d,%d) emits %d packets with a non-finite "
                    "weight ewsv or Eloss_th/Eloss_tot", j + 1, k + 1, (int)nsv);
      vp[cell + 1] = vp[cell] + nsv;
    }
  c->n_vol_global = vp[nc];
  HIPCHK(c, hipMemcpy(c->n_e, ne.data(), nc * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->ewsv, ew.data(), nc * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->vfrac, vf.data(), vf.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->vol_prefix, vp.data(), vp.size() * sizeof(int64_t), hipMemcpyHostToDevice));

  /* surface slots: (inner js, outer js) for js=1..nz, then (upper ks, lower ks) */
  const int ns = c->nslot;
  std::vector<int64_t> sp(ns + 1);
  std::vector<double> sew(ns), stb(ns);
  std::vector<int32_t> ssp(ns);
  sp[0] = 0;
  for (int s = 0; s < ns; s++) {
    int32_t cnt = 0, spec = -1;
    double w = 0.0, tb = 0.0;
    if (s < 2 * nz) {
      const int j = s / 2, side = s & 1;
      const int32_t* n = side ? in->nsurfo : in->nsurfi;
      const double* e = side ? in->ewsurfo : in->ewsurfi;
      const double* t = side ? in->tbbo : in->tbbi;
      const int32_t* sx = side ? in->spec_o : in->spec_i;
      cnt = n ? n[j] : 0;
      w = e ? e[j] : 0.0;
      tb = t ? t[j] : 0.0;
      spec = sx ? sx[j] : -1;
    } else {
      const int k = (s - 2 * nz) / 2, side = (s - 2 * nz) & 1;
      const int32_t* n = side ? in->nsurfl : in->nsurfu;
      const double* e = side ? in->ewsurfl : in->ewsurfu;
      const double* t = side ? in->tbbl : in->tbbu;
      const int32_t* sx = side ? in->spec_l : in->spec_u;
      cnt = n ? n[k] : 0;
      w = e ? e[k] : 0.0;
      tb = t ? t[k] : 0.0;
      spec = sx ? sx[k] : -1;
    }
    if (cnt > 0 && !(tb > 0.0) && (spec < 0 || spec >= in->n_spectra))
      return fail(c, C2D_E_ARG, "surface slot %d emits %d packets but has no spectrum", s, cnt);
    if (cnt < 0) return fail(c, C2D_E_ARG, "surface slot %d: packet count %d < 0", s, (int)cnt);
    if (cnt > 0 && !(std::isfinite(w) && std::isfinite(tb)))
      return fail(c, C2D_E_NONFINITE, "surface slot %d emits %d packets with a non-finite weight or "
                  "temperature", s, (int)cnt);
    sp[s + 1] = sp[s] + cnt;
    sew[s] = w;
    stb[s] = tb;
    ssp[s] = spec;
  }
  c->n_surf_global = sp[ns];
  HIPCHK(c, hipMemcpy(c->surf_prefix, sp.data(), sp.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->surf_ew, sew.data(), ns * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->surf_tbb, stb.data(), ns * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->surf_spec, ssp.data(), ns * sizeof(int32_t), hipMemcpyHostToDevice));
  std::vector<double> tl(nr, 0.0);
  for (int k = 0; k < nr; k++) tl[k] = in->tbbl ? in->tbbl[k] : 0.0;
  HIPCHK(c, hipMemcpy(c->tbbl, tl.data(), nr * sizeof(double), hipMemcpyHostToDevice));

  /* seed spectra (file_sp output) */
  for (double* p : c->spec_bufs) (void)hipFree(p);
  c->spec_bufs.clear();
  if (c->spectra) (void)hipFree(c->spectra);
  c->spectra = nullptr;
  c->n_spectra = in->n_spectra;
  if (in->n_spectra > 0) {
    std::vector<SpecDev> hs(in->n_spectra);
    for (int m = 0; m < in->n_spectra; m++) {
      const c2d_spectrum& s = in->spectra[m];
      if (s.nfile < 2 || s.nfile > C2D_NFMAX) return fail(c, C2D_E_ARG, "spectrum %d: nfile %d", m, s.nfile);
      const double* src[5] = {s.E_file, s.a1, s.I_file, s.F_file, s.P_file};
      const int len[5] = {s.nfile, s.nfile - 1, s.nfile - 1, s.nfile, s.nfile - 1};
      double* dst[5];
      for (int f = 0; f < 5; f++)   /* hazard H9: disk/blackbody.in's NaN column */
        if (!src[f] || !all_finite(src[f], (size_t)len[f]))
          return fail(c, C2D_E_NONFINITE, "spectrum %d: missing or NaN/Inf table column %d (hazard H9)", m, f);
      for (int f = 0; f < 5; f++) {
        HIPCHK(c, dalloc(&dst[f], (size_t)len[f]));
        HIPCHK(c, hipMemcpy(dst[f], src[f], len[f] * sizeof(double), hipMemcpyHostToDevice));
        c->spec_bufs.push_back(dst[f]);
      }
      hs[m].nfile = s.nfile;
      hs[m].E_file = dst[0]; hs[m].a1 = dst[1]; hs[m].I_file = dst[2]; hs[m].F_file = dst[3];
      hs[m].P_file = dst[4];
    }
    HIPCHK(c, dalloc(&c->spectra, (size_t)in->n_spectra));
    HIPCHK(c, hipMemcpy(c->spectra, hs.data(), hs.size() * sizeof(SpecDev), hipMemcpyHostToDevice));
  }

  /* the CDFs' guide rows (used while they are monotone; C2D_CDF_GUIDE_OFF=1: A/B) */
  {
    const char* go = getenv("C2D_CDF_GUIDE_OFF");
    c->cdf_guide_on = !(go && go[0] == '1');
    if (c->cdf_guide_on) {
      if (!c->cdf_guide) HIPCHK(c, dalloc(&c->cdf_guide, (size_t)2 * nc * (C2D_CDF_GUIDE + 1)));
      const int64_t nt = (int64_t)2 * nc * (C2D_CDF_GUIDE + 1);
      const int grid = (int)std::min<int64_t>((nt + 255) / 256, (int64_t)c->n_cu * 4);
      hipLaunchKernelGGL(c2d_cdf_guide, dim3(grid), dim3(256), 0, c->stream, c->eps_tot, c->eps_th, nc, C2D_N_VOL,
                         c->cdf_guide);
      HIPCHK(c, hipGetLastError());
    }
  }
  if (c->cfg.comtot_mode == C2D_COMTOT_TABLE) {
    int rc = c2d_launch_comtab_gemm(c->f_nt, c->gnt, c->comS, c->comtab, nc, c->stream);
    if (rc) return fail(c, C2D_E_HIP, "comtab_gemm launch: %d", rc);
  }
  c2d_set_clock(c, in->ncycle, in->time, in->dt);
  c->have_step = true;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return C2D_OK;
}

/* n_field[i] += sum of the C2D_NF_REPL census replicas (replica order: fixed) */
__global__ void __launch_bounds__(256) c2d_nf_reduce(const double* __restrict__ rep, int64_t n,
                                                     double* __restrict__ nf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int r = 0; r < C2D_NF_REPL; r++) s += rep[r * n + i];
    if (s != 0.0) nf[i] += s;
  }
}

/* In-place census compaction: W live records of the R slots [0, R); every
 * dead slot below W takes a live record from [W, R).  Tiles of CT_TILE
 * slots: c2d_census_count counts a tile's holes (dead, below W) and sources
 * (live, at or above W), c2d_census_scan forms the exclusive prefix of both
 * over the tiles (one workgroup), c2d_census_emit writes the k-th hole's and
 * the k-th source's slot into the two work lists (slot order: the moves are
 * monotone, and no counter is contended), c2d_census_fill moves pair k.  A
 * round moves at most `cap` pairs; rounds repeat while holes remain. */
#ifndef C2D_CT_TILE
#define C2D_CT_TILE 16384
#endif
constexpr int CT_TILE = C2D_CT_TILE, CT_BLOCK = 256;

__device__ __forceinline__ void census_class(const c2d_u4* tg, int64_t i, int64_t R, int64_t W,
                                             bool& hole, bool& src) {
  hole = src = false;
  if (i < R) {
    const bool dead = (cens_bins(tg, i) & C2D_CENS_DEAD) != 0u;
    hole = dead && i < W;
    src = !dead && i >= W;
  }
}

__global__ void __launch_bounds__(CT_BLOCK) c2d_census_count(const c2d_u4* __restrict__ tg, int64_t R,
                                                             int64_t W, const uint8_t* __restrict__ flag,
                                                             uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sh[2][CT_BLOCK / 64];
  const int64_t t = blockIdx.x;
  const int64_t base = t * CT_TILE;
  /* the only dead slots are the chunk tails (c2d_chunk_tails): a tile below
   * W without one holds neither holes nor sources */
  if (base + CT_TILE <= W && !flag[t]) {
    if (threadIdx.x < 2) cnt[2 * t + threadIdx.x] = 0u;
    return;
  }
  uint32_t nh = 0, ns = 0;
  for (int j = 0; j < CT_TILE / CT_BLOCK; j++) {
    bool h, s;
    census_class(tg, base + j * CT_BLOCK + threadIdx.x, R, W, h, s);
    nh += (uint32_t)__popcll(__ballot(h));
    ns += (uint32_t)__popcll(__ballot(s));
  }
  if (__lane_id() == 0) { sh[0][threadIdx.x >> 6] = nh; sh[1][threadIdx.x >> 6] = ns; }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t v = 0;
    for (int w = 0; w < CT_BLOCK / 64; w++) v += sh[threadIdx.x][w];
    cnt[2 * t + threadIdx.x] = v;
  }
}

/* exclusive prefix over ntiles (holes, sources) pairs, in place, one
 * workgroup of 1024 threads; totals at off[2 * ntiles], off[2 * ntiles + 1] */
__global__ void __launch_bounds__(1024) c2d_census_scan(uint32_t* __restrict__ cnt, int64_t ntiles,
                                                        unsigned long long* __restrict__ off) {
  __shared__ unsigned long long sh[2][1024];
  const int64_t per = (ntiles + 1023) / 1024;
  const int64_t lo = threadIdx.x * per, hi = lo + per < ntiles ? lo + per : ntiles;
  unsigned long long a = 0, b = 0;
  for (int64_t t = lo; t < hi; t++) { a += cnt[2 * t]; b += cnt[2 * t + 1]; }
  sh[0][threadIdx.x] = a;
  sh[1][threadIdx.x] = b;
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned long long run = 0;
    for (int i = 0; i < 1024; i++) {
      const unsigned long long v = sh[threadIdx.x][i];
      sh[threadIdx.x][i] = run;
      run += v;
    }
    off[2 * ntiles + threadIdx.x] = run;
  }
  __syncthreads();
  a = sh[0][threadIdx.x];
  b = sh[1][threadIdx.x];
  for (int64_t t = lo; t < hi; t++) {
    const unsigned long long ca = cnt[2 * t], cb = cnt[2 * t + 1];
    off[2 * t] = a;
    off[2 * t + 1] = b;
    a += ca;
    b += cb;
  }
}

__global__ void __launch_bounds__(CT_BLOCK) c2d_census_emit(const c2d_u4* __restrict__ tg, int64_t R,
                                                            int64_t W, const unsigned long long* __restrict__ off,
                                                            int64_t cap, int64_t* __restrict__ holes,
                                                            int64_t* __restrict__ srcs) {
  __shared__ uint32_t sh[2][CT_BLOCK / 64];
  const int64_t t = blockIdx.x;
  const int64_t base = t * CT_TILE;
  const int w = threadIdx.x >> 6;
  const uint32_t lane = __lane_id();
  const unsigned long long below = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  unsigned long long rh = off[2 * t], rs = off[2 * t + 1];
  if (off[2 * t + 2] == rh && off[2 * t + 3] == rs) return;   /* no hole, no source */
  for (int j = 0; j < CT_TILE / CT_BLOCK; j++) {
    const int64_t i = base + j * CT_BLOCK + threadIdx.x;
    bool h, s;
    census_class(tg, i, R, W, h, s);
    const unsigned long long mh = __ballot(h), ms = __ballot(s);
    if (lane == 0) { sh[0][w] = (uint32_t)__popcll(mh); sh[1][w] = (uint32_t)__popcll(ms); }
    __syncthreads();
    unsigned long long ph = rh, ps = rs;
    for (int v = 0; v < CT_BLOCK / 64; v++) {
      if (v < w) { ph += sh[0][v]; ps += sh[1][v]; }
      rh += sh[0][v];
      rs += sh[1][v];
    }
    __syncthreads();
    if (h) {
      const unsigned long long k = ph + __popcll(mh & below);
      if ((int64_t)k < cap) holes[k] = i;
    }
    if (s) {
      const unsigned long long k = ps + __popcll(ms & below);
      if ((int64_t)k < cap) srcs[k] = i;
    }
  }
}

__global__ void __launch_bounds__(256) c2d_census_fill(CensusSoA c, const int64_t* __restrict__ holes,
                                                       const int64_t* __restrict__ srcs, int64_t m) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < m;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = holes[t], s = srcs[t];
    const c2d_d2 rz = cld2(c.rz + s), wp = cld2(c.wp + s), ex = cld2(c.ex + s);
    const c2d_u4 tg = cld4(c.tg + s);
    cst2(c.rz + d, rz.x, rz.y);
    cst2(c.wp + d, wp.x, wp.y);
    cst2(c.ex + d, ex.x, ex.y);
    cst4(c.tg + d, tg.x, tg.y, c2d_tg_key(tg));
    cens_set_bins(c.tg, s, C2D_CENS_DEAD);   /* moved: the next round must not list it again */
  }
}

/* ---- census records: packed 8-word form (C2D_CENSUS_REC_WORDS), bit-exact ---- */
__device__ __forceinline__ void rec_pack(const CensusSoA& cs, int64_t s, uint64_t* r) {
  const c2d_d2 rz = cld2(cs.rz + s), wp = cld2(cs.wp + s), ex = cld2(cs.ex + s);
  const c2d_u4 tg = cld4(cs.tg + s);
  r[0] = __double_as_longlong(rz.x);
  r[1] = __double_as_longlong(rz.y);
  r[2] = __double_as_longlong(wp.x);
  r[3] = __double_as_longlong(wp.y);
  r[4] = __double_as_longlong(ex.x);
  r[5] = __double_as_longlong(ex.y);
  r[6] = (uint64_t)tg.x | ((uint64_t)tg.y << 32);
  r[7] = c2d_tg_key(tg);
}
__device__ __forceinline__ void rec_unpack(const CensusSoA& cs, int64_t d, const uint64_t* r) {
  cst2(cs.rz + d, __longlong_as_double(r[0]), __longlong_as_double(r[1]));
  cst2(cs.wp + d, __longlong_as_double(r[2]), __longlong_as_double(r[3]));
  cst2(cs.ex + d, __longlong_as_double(r[4]), __longlong_as_double(r[5]));
  cst4(cs.tg + d, (uint32_t)(r[6] & 0xffffffffull), (uint32_t)(r[6] >> 32), r[7]);
}
/* census record i -> its slot (chunked: through the chunk list) */
__device__ __forceinline__ int64_t cens_slot(const int32_t* clist, int64_t i) {
  return clist ? ((int64_t)clist[i >> C2D_CCHUNK_LOG] << C2D_CCHUNK_LOG) + (i & (C2D_CCHUNK - 1)) : i;
}

/* ---- chunked census (c2d_device.hpp C2D_CCHUNK) ---- */
/* mark the chunks of a list */
__global__ void __launch_bounds__(256) c2d_chunk_mark(const int32_t* __restrict__ list, int64_t n,
                                                      uint8_t* __restrict__ flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[list[i]] = 1;
}

/* append the ids i < n with flag[i] == 0 (pool), or the entries of list with
 * flag[list[j]] == 0 (list != null), to out; one atomic per wave */
__global__ void __launch_bounds__(256) c2d_chunk_select(const int32_t* __restrict__ list, int64_t n,
                                                        const uint8_t* __restrict__ flag,
                                                        int32_t* __restrict__ out,
                                                        unsigned long long* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x; b < n; b += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = b + threadIdx.x;
    int32_t id = 0;
    bool keep = false;
    if (i < n) {
      id = list ? list[i] : (int32_t)i;
      keep = flag[id] == 0;
    }
    const unsigned long long m = __ballot(keep);
    if (m == 0ull) continue;
    const int leader = __ffsll((long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (keep) out[base + __popcll(m & ((1ull << lane) - 1ull))] = id;
  }
}

/* double-buffered census after the step: the unused tail of each wave
 * slot's last chunk (one workgroup per slot) is marked dead and counted */
__global__ void __launch_bounds__(256) c2d_chunk_tails(const int64_t* __restrict__ cstate, uint32_t chunk,
                                                       int64_t cap, c2d_u4* __restrict__ tg,
                                                       unsigned long long* __restrict__ dead) {
  const int64_t base = cstate[2 * blockIdx.x], used = cstate[2 * blockIdx.x + 1];
  if (base < 0 || used <= 0 || used >= (int64_t)chunk || base >= cap) return;
  const int64_t t1 = base + chunk < cap ? base + chunk : cap;
  for (int64_t s = base + used + threadIdx.x; s < t1; s += blockDim.x) cens_set_bins(tg, s, C2D_CENS_DEAD);
  if (threadIdx.x == 0 && t1 > base + used) atomicAdd(dead, (unsigned long long)(t1 - base - used));
}

/* flag the compaction tiles (CT_TILE slots) that hold a chunk tail */
__global__ void __launch_bounds__(256) c2d_tail_tiles(const int64_t* __restrict__ cstate, int64_t n_ws,
                                                      uint32_t chunk, int64_t cap, uint8_t* __restrict__ flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_ws;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t base = cstate[2 * i], used = cstate[2 * i + 1];
    if (base < 0 || used <= 0 || used >= (int64_t)chunk || base >= cap) continue;
    const int64_t t1 = base + chunk < cap ? base + chunk : cap;
    for (int64_t t = (base + used) / CT_TILE; t <= (t1 - 1) / CT_TILE; t++) flag[t] = 1;
  }
}

/* chunked census after the step: the wave slots' partly filled chunks, in
 * slot order: ids, exclusive prefix of their records (part_off[np] = total),
 * flags; out = {np, total}.  One workgroup of 1024. */
__global__ void __launch_bounds__(1024) c2d_chunk_partials(const int64_t* __restrict__ cstate, int64_t n_ws,
                                                           uint32_t chunk, int64_t cap,
                                                           int32_t* __restrict__ part_id,
                                                           int64_t* __restrict__ part_off,
                                                           uint8_t* __restrict__ flag,
                                                           unsigned long long* __restrict__ out) {
  __shared__ int64_t sc[1024], su[1024];
  __shared__ int64_t np_s, tot_s;
  const int t = threadIdx.x;
  if (t == 0) { np_s = 0; tot_s = 0; }
  __syncthreads();
  for (int64_t b0 = 0; b0 < n_ws; b0 += 1024) {
    const int64_t i = b0 + t;
    int64_t base = -1, used = 0;
    if (i < n_ws) {
      base = cstate[2 * i];
      used = cstate[2 * i + 1];
    }
    const bool part = base >= 0 && used > 0 && used < (int64_t)chunk && base < cap;
    sc[t] = part ? 1 : 0;
    su[t] = part ? used : 0;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {     /* inclusive scan */
      const int64_t a = t >= off ? sc[t - off] : 0, u = t >= off ? su[t - off] : 0;
      __syncthreads();
      sc[t] += a;
      su[t] += u;
      __syncthreads();
    }
    if (part) {
      const int64_t k = np_s + sc[t] - 1;
      part_id[k] = (int32_t)(base >> C2D_CCHUNK_LOG);
      part_off[k] = tot_s + su[t] - used;
      flag[base >> C2D_CCHUNK_LOG] = 1;
    }
    __syncthreads();
    if (t == 1023) { np_s += sc[t]; tot_s += su[t]; }
    __syncthreads();
  }
  if (t == 0) {
    part_off[np_s] = tot_s;
    out[0] = (unsigned long long)np_s;
    out[1] = (unsigned long long)tot_s;
  }
}

/* packing the partly filled chunks, in two phases per batch [r0, r1) of
 * their records (record r goes to slot r of the chunks part_id[0, ...):
 * never after its source, so a batch reads nothing an earlier one wrote) */
__global__ void __launch_bounds__(256) c2d_chunk_gather(CensusSoA cs, const int32_t* __restrict__ part_id,
                                                        const int64_t* __restrict__ part_off, int64_t r0,
                                                        int64_t r1, uint64_t* __restrict__ tmp) {
  const int64_t j = blockIdx.x;
  const int64_t off = part_off[j], fill = part_off[j + 1] - off;
  for (int64_t s = threadIdx.x; s < fill; s += blockDim.x) {
    const int64_t r = off + s;
    if (r < r0 || r >= r1) continue;
    rec_pack(cs, ((int64_t)part_id[j] << C2D_CCHUNK_LOG) + s, tmp + (r - r0) * C2D_CENSUS_REC_WORDS);
  }
}
__global__ void __launch_bounds__(256) c2d_chunk_scatter(CensusSoA cs, const int32_t* __restrict__ part_id,
                                                         int64_t r0, int64_t r1,
                                                         const uint64_t* __restrict__ tmp) {
  for (int64_t r = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < r1;
       r += (int64_t)gridDim.x * blockDim.x)
    rec_unpack(cs, ((int64_t)part_id[r >> C2D_CCHUNK_LOG] << C2D_CCHUNK_LOG) + (r & (C2D_CCHUNK - 1)),
               tmp + (r - r0) * C2D_CENSUS_REC_WORDS);
}

static int ensure_tmp(c2d_ctx* c, int64_t want) {
  want = std::max<int64_t>(want, 1 << 16);
  if (c->tmp_cap >= want) return C2D_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->tmp_rec) (void)hipFree(c->tmp_rec);
  c->tmp_rec = nullptr;
  c->tmp_cap = 0;
  HIPCHK(c, dalloc(&c->tmp_rec, (size_t)want * C2D_CENSUS_REC_WORDS));
  c->tmp_cap = want;
  return C2D_OK;
}

/* the free chunks (not in the census's list) into the pool; returns their
 * number (the pool counter at ctl[CTL_POOLN]) */
static int chunk_pool_build(c2d_ctx* c, int64_t* n_free) {
  HIPCHK(c, hipMemsetAsync(c->cflag, 0, (size_t)c->nchunks, c->stream));
  HIPCHK(c, hipMemsetAsync(c->ctl + CTL_POOLN, 0, sizeof(unsigned long long), c->stream));
  const int gm = (int)std::max<int64_t>(1, std::min<int64_t>((c->n_clist + 255) / 256, (int64_t)c->n_cu * 8));
  if (c->n_clist > 0)
    hipLaunchKernelGGL(c2d_chunk_mark, dim3(gm), dim3(256), 0, c->stream, c->clist[c->ccur], c->n_clist,
                       c->cflag);
  const int gp = (int)std::max<int64_t>(1, std::min<int64_t>((c->nchunks + 255) / 256, (int64_t)c->n_cu * 8));
  hipLaunchKernelGGL(c2d_chunk_select, dim3(gp), dim3(256), 0, c->stream, (const int32_t*)nullptr,
                     c->nchunks, c->cflag, c->pool, c->ctl + CTL_POOLN);
  HIPCHK(c, hipGetLastError());
  if (n_free) {
    unsigned long long n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, c->ctl + CTL_POOLN, sizeof n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *n_free = (int64_t)n;
  }
  return C2D_OK;
}

/* after the last generation (chunked): pack the partly filled chunks, and
 * the chunks taken (those emptied by the packing aside) become the census's
 * list, the packed ones last.  *n_records = the census's records. */
static int census_chunks_close(c2d_ctx* c, int64_t* n_records) {
  HIPCHK(c, hipMemsetAsync(c->cflag, 0, (size_t)c->nchunks, c->stream));
  hipLaunchKernelGGL(c2d_chunk_partials, dim3(1), dim3(1024), 0, c->stream, c->cstate, c->n_ws,
                     (uint32_t)C2D_CCHUNK, c->cens_phys, c->part_id, c->part_off, c->cflag,
                     c->ctl + CTL_NCOUT);      /* {np, total} into the (unused) NCOUT, POOLH words */
  HIPCHK(c, hipGetLastError());
  unsigned long long pr[2], n_out = 0;
  HIPCHK(c, hipMemcpyAsync(pr, c->ctl + CTL_NCOUT, sizeof pr, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&n_out, c->ctl + CTL_NOUT, sizeof n_out, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int64_t np = (int64_t)pr[0], tot = (int64_t)pr[1];
  if (np > c->n_ws || (int64_t)n_out > c->nchunks || np > (int64_t)n_out)
    return fail(c, C2D_E_STATE, "census chunks: %lld partly filled of %llu taken", (long long)np, n_out);
  const CensusSoA cs = c->cens[0].soa();
  c->last_compact_rounds = 0;
  c->last_compact_moved = 0;
  if (np > 1) {
    int rc = ensure_tmp(c, std::min<int64_t>(tot, int64_t(1) << 22));
    if (rc) return rc;
    int64_t B = c->tmp_cap;
    /* test knob: short batches force many two-phase rounds */
    if (const char* e = getenv("C2D_CHUNK_BATCH")) B = std::max<int64_t>(1, std::min<int64_t>(B, atoll(e)));
    for (int64_t r0 = 0; r0 < tot; r0 += B) {
      const int64_t r1 = std::min(tot, r0 + B);
      hipLaunchKernelGGL(c2d_chunk_gather, dim3((unsigned)np), dim3(256), 0, c->stream, cs, c->part_id,
                         c->part_off, r0, r1, c->tmp_rec);
      const int g = (int)std::min<int64_t>((r1 - r0 + 255) / 256, (int64_t)c->n_cu * 8);
      hipLaunchKernelGGL(c2d_chunk_scatter, dim3(g), dim3(256), 0, c->stream, cs, c->part_id, r0, r1,
                         c->tmp_rec);
      HIPCHK(c, hipGetLastError());
      c->last_compact_rounds++;
    }
    c->last_compact_moved = tot;
  }
  /* the full chunks taken, then the packed ones */
  const int nxt = 1 - c->ccur;
  const int64_t kp = (tot + C2D_CCHUNK - 1) / C2D_CCHUNK;
  HIPCHK(c, hipMemsetAsync(c->ctl + CTL_NOUT, 0, sizeof(unsigned long long), c->stream));
  if (n_out > 0) {
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(((int64_t)n_out + 255) / 256, (int64_t)c->n_cu * 8));
    hipLaunchKernelGGL(c2d_chunk_select, dim3(g), dim3(256), 0, c->stream, c->out_list, (int64_t)n_out,
                       c->cflag, c->clist[nxt], c->ctl + CTL_NOUT);
    HIPCHK(c, hipGetLastError());
  }
  unsigned long long n_full = 0;
  HIPCHK(c, hipMemcpyAsync(&n_full, c->ctl + CTL_NOUT, sizeof n_full, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((int64_t)n_full != (int64_t)n_out - np)
    return fail(c, C2D_E_STATE, "census chunks: %llu full of %llu taken, %lld partly filled", n_full, n_out,
                (long long)np);
  if (kp > 0)
    HIPCHK(c, hipMemcpyAsync(c->clist[nxt] + n_full, c->part_id, sizeof(int32_t) * kp,
                             hipMemcpyDeviceToDevice, c->stream));
  c->ccur = nxt;
  c->n_clist = (int64_t)n_full + kp;
  *n_records = (int64_t)n_full * C2D_CCHUNK + tot;
  return C2D_OK;
}

static int census_compact(c2d_ctx* c, const DevCensus& cb, int64_t R, int64_t W) {
  c->last_compact_rounds = 0;
  c->last_compact_moved = 0;
  if (W >= R) return C2D_OK;               /* no dead slot */
  const int64_t ntiles = (R + CT_TILE - 1) / CT_TILE;
  if (ntiles > c->ctile_cap) {
    if (c->ctile_cnt) (void)hipFree(c->ctile_cnt);
    if (c->ctile_off) (void)hipFree(c->ctile_off);
    if (c->ctile_flag) (void)hipFree(c->ctile_flag);
    c->ctile_cnt = nullptr;
    c->ctile_off = nullptr;
    c->ctile_flag = nullptr;
    HIPCHK(c, dalloc(&c->ctile_cnt, 2 * (size_t)ntiles));
    HIPCHK(c, dalloc(&c->ctile_off, 2 * (size_t)ntiles + 2));
    HIPCHK(c, dalloc(&c->ctile_flag, (size_t)ntiles));
    c->ctile_cap = ntiles;
  }
  /* tiles that hold a chunk tail (the only dead slots, below or above W) */
  HIPCHK(c, hipMemsetAsync(c->ctile_flag, 0, (size_t)ntiles, c->stream));
  if (c->n_ws > 0) {
    const int tg = (int)std::min<int64_t>((c->n_ws + 255) / 256, (int64_t)c->n_cu * 4);
    hipLaunchKernelGGL(c2d_tail_tiles, dim3(tg), dim3(256), 0, c->stream, c->cstate, c->n_ws,
                       c->cens_chunk, c->cens_phys, c->ctile_flag);
    HIPCHK(c, hipGetLastError());
  }
  const CensusSoA cs = cb.soa();
  int64_t* holes = c->cscan;
  int64_t* srcs = c->cscan + c->cscan_cap;
  for (int round = 0;; round++) {
    hipLaunchKernelGGL(c2d_census_count, dim3((unsigned)ntiles), dim3(CT_BLOCK), 0, c->stream,
                       cb.tg, R, W, c->ctile_flag, c->ctile_cnt);
    hipLaunchKernelGGL(c2d_census_scan, dim3(1), dim3(1024), 0, c->stream, c->ctile_cnt, ntiles,
                       c->ctile_off);
    hipLaunchKernelGGL(c2d_census_emit, dim3((unsigned)ntiles), dim3(CT_BLOCK), 0, c->stream,
                       cb.tg, R, W, c->ctile_off, c->cscan_cap, holes, srcs);
    HIPCHK(c, hipGetLastError());
    unsigned long long nn[2];
    HIPCHK(c, hipMemcpyAsync(nn, c->ctile_off + 2 * ntiles, sizeof nn, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nn[0] != nn[1])
      return fail(c, C2D_E_STATE, "census compaction: %llu dead slots below %lld, %llu live above",
                  nn[0], (long long)W, nn[1]);
    if (nn[0] == 0) break;
    const int64_t m = std::min<int64_t>((int64_t)nn[0], c->cscan_cap);
    const int fg = (int)std::min<int64_t>((m + 255) / 256, (int64_t)c->n_cu * 16);
    hipLaunchKernelGGL(c2d_census_fill, dim3(fg), dim3(256), 0, c->stream, cs, holes, srcs, m);
    HIPCHK(c, hipGetLastError());
    c->last_compact_rounds = round + 1;
    c->last_compact_moved += m;
    if ((int64_t)nn[0] <= c->cscan_cap) break;
  }
  return C2D_OK;
}

static int run_step_body(c2d_ctx* c);

/* A failed step leaves the double-buffered census as it was (the step wrote
 * the other buffer).  The chunked census is rewritten in place from the
 * generation-0 launch on, so a failure after that launch loses it: the
 * context then holds no census and every census read, and the next step,
 * fail with C2D_E_STATE until c2d_census_import or c2d_census_truncate
 * (ADVICE r03). */
extern "C" int c2d_run_step(c2d_ctx* c) {
  if (!c) return C2D_E_ARG;
  if (c->census_lost)
    return fail(c, C2D_E_STATE, "the census was lost by a failed in-place step: c2d_census_import or "
                "c2d_census_truncate first");
  c->g0_launched = false;
  const int rc = run_step_body(c);
  if (rc && c->chunked && c->g0_launched) {
    c->n_census = 0;
    c->n_clist = 0;
    c->census_lost = true;
  }
  return rc;
}

static int census_lost(c2d_ctx* c, const char* who) {
  return fail(c, C2D_E_STATE, "%s: the census was lost by a failed in-place step", who);
}

static int run_step_body(c2d_ctx* c) {
  if (!c->have_step) return fail(c, C2D_E_STATE, "c2d_set_step must precede c2d_run_step");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const c2d_config& cfg = c->cfg;
  KParams& P = c->P;
  P.nz = c->nz; P.nr = c->nr; P.ncell = c->ncell; P.nphtotal = cfg.nphtotal;
  P.nph_lc = cfg.nph_lc; P.nmu = cfg.nmu;
  P.split1 = cfg.split1; P.split2 = cfg.split2; P.split3 = cfg.split3; P.spl3_trg = cfg.spl3_trg;
  P.spec_switch = cfg.spec_switch; P.rank = cfg.rank; P.world = cfg.world;
  P.eps_linear = c->eps_linear;
  P.cdf_guide = (c->cdf_guide_on && !c->eps_linear) ? c->cdf_guide : nullptr;
  P.rmin = cfg.rmin; P.zmin = cfg.zmin;
  P.geo = c->geo; P.gnt = c->gnt;
  P.kappa_cv = cfg.kappa_lag ? c->kappa_prev : c->kappa_cur;
  P.kappa_s = c->kappa_cur;
  P.eps_tot = c->eps_tot; P.eps_th = c->eps_th; P.f_nt = c->f_nt; P.Pnt = c->Pnt;
  P.n_e = c->n_e; P.vfrac = c->vfrac; P.ewsv = c->ewsv;
  P.vol_prefix = c->vol_prefix; P.surf_prefix = c->surf_prefix; P.surf_ew = c->surf_ew;
  P.surf_tbb = c->surf_tbb; P.surf_spec = c->surf_spec; P.tbbl = c->tbbl;
  P.spectra = c->spectra; P.n_spectra = c->n_spectra; P.nslot = c->nslot;
  P.comtab = c->comtab;
  P.comtab_du_inv = (double)(C2D_COMTAB_N - 1) / (C2D_COMTAB_U1 - C2D_COMTAB_U0);
  P.egg_min = c->egg_min;
  /* last step's census records are this step's first items.  Chunked
   * (census_inplace) they are read through the chunk list and the step's
   * census writes fill free chunks of the same SoA; double-buffered the step
   * writes the other buffer from 0. */
  const int out_buf = c->chunked ? 0 : 1 - c->cur;
  P.cin = c->cens[c->cur].soa();
  P.cout = c->cens[out_buf].soa();
  P.n_cin = c->n_census;
  P.cap_cout = c->cens_phys;
  P.cens_chunk = c->cens_chunk;
  P.n_cout = c->ctl + CTL_NCOUT;
  P.clist = c->chunked ? c->clist[c->ccur] : nullptr;
  P.pool = c->pool;
  P.pool_n = c->ctl + CTL_POOLN;
  P.pool_head = c->ctl + CTL_POOLH;
  P.out_list = c->out_list;
  P.n_out = c->ctl + CTL_NOUT;
  P.relist = c->relist;
  P.n_relist = c->ctl + CTL_RELN;
  P.relist_head = c->ctl + CTL_RELH;
  P.cstate = c->cstate;
  P.ev = c->ev; P.cap_ev = cfg.event_capacity;
  P.n_ev_sh = c->ctl + CTL_EVSH;
  c->ev_cap_sh = std::max<int64_t>(cfg.event_capacity / C2D_EV_SHARDS, 0);
  P.cap_ev_sh = c->ev_cap_sh;
  P.cap_q = cfg.queue_capacity;
  P.T = c->T;
  P.nf_rep = c->nf_rep;
  P.off.edep = c->L.edep; P.off.prdep = c->L.prdep; P.off.ecens = c->L.ecens;
  P.off.npcen = c->L.npcen; P.off.n_field = c->L.n_field; P.off.E_IC = c->L.E_IC;
  P.off.nelectron = c->L.nelectron; P.off.fout = c->L.fout; P.off.edout = c->L.edout;
  P.off.erlki = c->L.erlki; P.off.erlko = c->L.erlko; P.off.erlku = c->L.erlku;
  P.off.erlkl = c->L.erlkl; P.off.Ed_in = c->L.Ed_in; P.off.counters = c->L.counters;
  P.cnt = c->ctl + CTL_CNT;
  P.err = c->derr;
  P.lds_cells = c->lds_cells;
  P.prof = c->ctl + CTL_PROF;
  P.n_vol_global = c->n_vol_global;
  P.n_surf_global = c->n_surf_global;
  /* this rank's share of the global source index space (lineage-sharded) */
  auto share = [&](int64_t n) -> int64_t {
    return n > cfg.rank ? (n - cfg.rank + cfg.world - 1) / cfg.world : 0;
  };
  P.n_cens_items = c->n_census;
  P.n_vol_items = share(c->n_vol_global);
  P.n_surf_items = share(c->n_surf_global);
  const int64_t n_src = P.n_vol_items + P.n_surf_items;
  /* double-buffered census with room behind the previous census: the source
   * kernel writes the volume sources there in census format, and generation
   * 0 reads them as census items (the next-source prefetch covers them; no
   * packet-store round trip).  C2D_VOL_CENSUS=0: the packet store. */
  P.vol_cens_base = -1;
  {
    const char* e = getenv("C2D_VOL_CENSUS");
    if (!c->chunked && !(e && e[0] == '0') && P.n_vol_items > 0 &&
        c->n_census + P.n_vol_items <= c->cens_phys) {
      P.vol_cens_base = c->n_census;
      P.n_cens_items = c->n_census + P.n_vol_items;
    }
  }
  const int64_t n_pk_src = n_src - (P.vol_cens_base >= 0 ? P.n_vol_items : 0);
  {
    /* packet store: all of this step's sources, and secondaries in chunks */
    const int64_t want = std::max<int64_t>(
        n_pk_src, std::min<int64_t>(int64_t(1) << 22,
                                 std::max<int64_t>(65536, cfg.queue_capacity *
                                                              std::max(cfg.split2, cfg.split3))));
    if (c->pk.cap < want) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      c->pk.release();
      for (int f = 0; f < 7; f++) HIPCHK(c, dalloc(&c->pk.d[f], want));
      HIPCHK(c, dalloc(&c->pk.jk, want));
      HIPCHK(c, dalloc(&c->pk.bins, want));
      HIPCHK(c, dalloc(&c->pk.ctr, want));
      HIPCHK(c, dalloc(&c->pk.sub, want));
      HIPCHK(c, dalloc(&c->pk.key, want));
      HIPCHK(c, dalloc(&c->pk.hard, want));
      c->pk.cap = want;
    }
  }
  P.pk = c->pk.soa();
  P.cap_pk = c->pk.cap;

  HIPCHK(c, hipMemsetAsync(c->T, 0, sizeof(double) * c->L.total, c->stream));
  HIPCHK(c, hipMemsetAsync(c->nf_rep, 0, sizeof(double) * C2D_NF_REPL * c->ncell * C2D_NPHFIELD,
                           c->stream));
  HIPCHK(c, hipMemsetAsync(c->ctl, 0, sizeof(unsigned long long) * CTL_WORDS, c->stream));
  HIPCHK(c, hipMemsetAsync(c->cstate, 0xff, 2 * sizeof(int64_t) * c->n_ws, c->stream));  /* no chunk */
  if (c->chunked) {
    HIPCHK(c, hipMemsetAsync(c->relist, 0xff, sizeof(int32_t) * c->nchunks, c->stream));
    int rc = chunk_pool_build(c, nullptr);
    if (rc) return rc;
  }
  HIPCHK(c, hipMemsetAsync(c->derr, 0, sizeof(int32_t), c->stream));

  const bool fast = cfg.comtot_mode == C2D_COMTOT_TABLE;
  auto launch_tr = fast ? c2d_launch_transport_fast : c2d_launch_transport_exact;
  auto launch_src = fast ? c2d_launch_source_fast : c2d_launch_source_exact;
  auto launch_sc = fast ? c2d_launch_scatter_fast : c2d_launch_scatter_exact;
  /* grid-stride kernels: one round of resident blocks at most */
  auto aux_grid = [&](int64_t n, int gmax) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(gmax, (n + 255) / 256));
  };
  auto tr_grid = [&](int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(c->max_grid, (n + C2D_TR_BLOCK - 1) / C2D_TR_BLOCK));
  };
  HIPCHK(c, hipMemcpyAsync(c->dP, &P, sizeof(KParams), hipMemcpyHostToDevice, c->stream));
  int gen = 0, qin = 0, launches = 0;
  int64_t n2 = 0, n3 = 0;
  unsigned long long nq[CTL_CNT + C2D_CNT_PATHS_INT + 1 - CTL_N2];
  /* ---- generation 0: census + sampled sources ---- */
  {
    /* the last step's events may still be binned on obs_stream: they are
     * rewritten from here on (the tables, FP and budgets ran beside it) */
    if (c->obs_inflight) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_obs_b, 0));
    HIPCHK(c, hipEventRecord(c->ev_g0a, c->stream));
    if (n_src > 0) {
      int rc = launch_src(c->dP, aux_grid(n_src, c->src_grid), c->stream);
      if (rc) return fail(c, C2D_E_HIP, "source launch: %s", hipGetErrorString((hipError_t)rc));
      launches++;
    }
    GenArgs A = {};
    A.gen = 0;
    A.n_items = P.n_cens_items + n_pk_src;
    A.q2_out = c->q2[1]; A.q3_out = c->q3[1];
    A.n2_out = c->ctl + CTL_N2; A.n3_out = c->ctl + CTL_N3;
    A.n_pk = c->ctl + CTL_NPK;
    A.work_counter = c->ctl + CTL_WORK;
    A.work_sh = c->ctl + CTL_WSH;
    HIPCHK(c, hipEventRecord(c->ev_g0t, c->stream));
    if (A.n_items > 0) {
      auto launch_b = fast ? c2d_launch_bundle_fast : c2d_launch_bundle_exact;
      int64_t gmax = c->bundle_grid;
      /* test knob: a few workgroups, so every wave runs many work chunks and
       * crosses chunk boundaries within one refill */
      if (const char* e = getenv("C2D_BUNDLE_GRID")) gmax = std::max<int64_t>(1, std::min<int64_t>(gmax, atoll(e)));
      const int grid = (int)std::max<int64_t>(
          1, std::min<int64_t>(gmax, (A.n_items + C2D_TR_BLOCK - 1) / C2D_TR_BLOCK));
      c->g0_launched = true;
      int rc = launch_b(c->dP, &A, grid, c->bundle_lds, cfg.trk_variant, c->stream);
      if (rc) return fail(c, C2D_E_HIP, "bundle launch (gen 0): %s", hipGetErrorString((hipError_t)rc));
      launches++;
    }
    HIPCHK(c, hipEventRecord(c->ev_g0b, c->stream));
    HIPCHK(c, hipMemcpyAsync(nq, c->ctl + CTL_N2, sizeof nq, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->last_g0_steps = (int64_t)nq[CTL_CNT - CTL_N2];
    c->last_g0_paths = (int64_t)nq[CTL_CNT + C2D_CNT_PATHS_INT - CTL_N2];
    gen = 1;
  }
  /* ---- generations >= 1: scatter sampling, then transport of the secondaries ---- */
  for (;;) {
    if ((int64_t)nq[0] > cfg.queue_capacity || (int64_t)nq[1] > cfg.queue_capacity)
      return fail(c, C2D_E_QUEUE_OVERFLOW, "scatter queue overflow in generation %d (%llu, %llu > %lld)",
                  gen - 1, nq[0], nq[1], (long long)cfg.queue_capacity);
    n2 = (int64_t)nq[0];
    n3 = (int64_t)nq[1];
    if (n2 + n3 == 0) break;
    qin = 1 - qin;              /* this generation's input = last generation's output */
    HIPCHK(c, hipMemsetAsync(c->ctl + CTL_N2, 0, 2 * sizeof(unsigned long long), c->stream));
    const int64_t total = n2 * cfg.split2 + n3 * cfg.split3;
    /* secondaries per launch pair: the packet store.  Test knob
     * C2D_PK_CHUNK: fewer, so a small case runs the chunked loop */
    int64_t pk_chunk = c->pk.cap;
    if (const char* e = getenv("C2D_PK_CHUNK")) pk_chunk = std::max<int64_t>(1, std::min<int64_t>(pk_chunk, atoll(e)));
    /* test knobs: 0 sends every compb2d first loop to the wave's cooperative
     * resolution, and every split3 copy to the hard kernel */
    int32_t kn_cap = C2D_KN_CAP_DEFAULT, sc_k1 = C2D_SC_K1_DEFAULT;
    if (const char* e = getenv("C2D_KN_CAP_ITERS")) kn_cap = (int32_t)std::max(0, std::min(4096, atoi(e)));
    if (const char* e = getenv("C2D_SC_K1_ATTEMPTS")) sc_k1 = (int32_t)std::max(0, std::min(4096, atoi(e)));
    for (int64_t b = 0; b < total; b += pk_chunk) {
      const int64_t e = std::min<int64_t>(total, b + pk_chunk);
      HIPCHK(c, hipMemsetAsync(c->ctl + CTL_NPK, 0, sizeof(unsigned long long), c->stream));
      HIPCHK(c, hipMemsetAsync(c->ctl + CTL_WORK, 0, sizeof(unsigned long long), c->stream));
      HIPCHK(c, hipMemsetAsync(c->ctl + CTL_NHARD, 0, sizeof(unsigned long long), c->stream));
      GenArgs A = {};
      A.gen = gen;
      A.q2_in = c->q2[qin]; A.q3_in = c->q3[qin];
      A.q2_out = c->q2[1 - qin]; A.q3_out = c->q3[1 - qin];
      A.n2_out = c->ctl + CTL_N2; A.n3_out = c->ctl + CTL_N3;
      A.n_pk = c->ctl + CTL_NPK;
      A.work_counter = c->ctl + CTL_WORK;
      A.n_hard = c->ctl + CTL_NHARD;
      A.hard = c->pk.hard;
      A.item_begin = b; A.item_end = e;
      A.n2_in = n2; A.n3_in = n3;
      A.kn_cap = kn_cap; A.sc_k1 = sc_k1;
      int rc = launch_sc(c->dP, &A, aux_grid(e - b, c->sc_grid), 2 * c->n_cu, c->stream);
      if (rc) return fail(c, C2D_E_HIP, "scatter launch (gen %d): %s", gen, hipGetErrorString((hipError_t)rc));
      rc = launch_tr(c->dP, &A, tr_grid(e - b), c->lds_bytes, cfg.trk_variant, c->stream);
      if (rc) return fail(c, C2D_E_HIP, "transport launch (gen %d): %s", gen, hipGetErrorString((hipError_t)rc));
      launches += 2;
    }
    HIPCHK(c, hipMemcpyAsync(nq, c->ctl + CTL_N2, sizeof nq, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    gen++;
  }
  /* close the census: chunked, pack the partly filled chunks into the next
   * chunk list; double-buffered, mark the unused chunk tails dead and close
   * the dead slots below the live count */
  int64_t cens_live = 0;
  {
    if (!c->chunked && c->n_ws > 0) {
      hipLaunchKernelGGL(c2d_chunk_tails, dim3((unsigned)c->n_ws), dim3(256), 0, c->stream, c->cstate,
                         c->cens_chunk, c->cens_phys, c->cens[out_buf].tg,
                         c->ctl + CTL_CNT + C2D_CNT_DEAD_INT);
      HIPCHK(c, hipGetLastError());
    }
    unsigned long long cw[3];
    int32_t herr0 = 0;
    HIPCHK(c, hipMemcpyAsync(cw, c->ctl + CTL_NCOUT, sizeof cw[0], hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cw + 1, c->ctl + CTL_CNT + C2D_CNT_DEAD_INT, sizeof cw[1],
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cw + 2, c->ctl + CTL_CNT + C2D_CNT_CENSUS, sizeof cw[2],
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&herr0, c->derr, sizeof herr0, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    /* a record slot beyond the physical census: the census is incomplete */
    if (herr0 & ERR_CENSUS) {
      if (c->chunked)
        return fail(c, C2D_E_CENSUS_OVERFLOW, "census overflow: no free census chunk left (%lld chunks "
                    "of %d for capacity %lld)", (long long)c->nchunks, C2D_CCHUNK, (long long)cfg.census_capacity);
      return fail(c, C2D_E_CENSUS_OVERFLOW, "census overflow: more than %lld records before "
                  "compaction (capacity %lld)", (long long)c->cens_phys, (long long)cfg.census_capacity);
    }
    if (c->chunked) {
      int rc = census_chunks_close(c, &cens_live);
      if (rc) return rc;
      if (cens_live != (int64_t)cw[2])
        return fail(c, C2D_E_STATE, "census chunks hold %lld records, %llu written", (long long)cens_live, cw[2]);
      if (cens_live > cfg.census_capacity)
        return fail(c, C2D_E_CENSUS_OVERFLOW, "too many photons: census %lld > capacity %lld",
                    (long long)cens_live, (long long)cfg.census_capacity);
    } else {
      /* reservations past the physical end are chunk tails (never written) */
      const int64_t R = std::min<int64_t>((int64_t)cw[0], c->cens_phys);
      const int64_t D = (int64_t)cw[1];
      cens_live = R - D;
      if (cens_live < 0 || D > R)
        return fail(c, C2D_E_STATE, "census compaction: %lld dead of %lld slots", (long long)D, (long long)R);
      if (cens_live > cfg.census_capacity)
        return fail(c, C2D_E_CENSUS_OVERFLOW, "too many photons: census %lld > capacity %lld",
                    (long long)cens_live, (long long)cfg.census_capacity);
      int rc = census_compact(c, c->cens[out_buf], R, cens_live);
      if (rc) return rc;
    }
  }
  {
    const int64_t n = (int64_t)c->ncell * C2D_NPHFIELD;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 16);
    hipLaunchKernelGGL(c2d_nf_reduce, dim3(grid), dim3(256), 0, c->stream, c->nf_rep, n,
                       c->T + c->L.n_field);
    HIPCHK(c, hipGetLastError());
    launches++;
  }
  HIPCHK(c, hipEventRecord(c->ev_end, c->stream));
  /* fail loudly on a NaN/Inf tally (a non-finite table or weight upstream) */
  check_finite(c, c->T, c->L.total, ERR_NONFINITE, c->derr, c->stream);
  HIPCHK(c, hipGetLastError());
  unsigned long long ctl[CTL_WORDS];
  int32_t herr = 0;
  HIPCHK(c, hipMemcpyAsync(ctl, c->ctl, sizeof ctl, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&herr, c->derr, sizeof herr, hipMemcpyDeviceToHost, c->stream));
  /* census + volume kappa of the next step = this step's (H3) */
  HIPCHK(c, hipMemcpyAsync(c->kappa_prev, c->kappa_cur, sizeof(double) * c->ncell * C2D_N_VOL,
                           hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms0 = 0.f, msall = 0.f;
  if (launches > 0) {
    (void)hipEventElapsedTime(&ms0, c->ev_g0t, c->ev_g0b);
    (void)hipEventElapsedTime(&c->last_src_ms, c->ev_g0a, c->ev_g0t);
    (void)hipEventElapsedTime(&msall, c->ev_g0a, c->ev_end);
  }
  c->last_g0_ms = ms0;
  for (int i = 0; i < C2D_TR_PROF_WORDS; i++) c->last_prof[i] = ctl[CTL_PROF + i];
  c->last_all_ms = msall;
  c->last_launches = launches;
  /* counters into the fused buffer (exact integers as f64) */
  double hc[C2D_NCOUNTERS];
  for (int i = 0; i < C2D_NCOUNTERS; i++) hc[i] = (double)ctl[CTL_CNT + i];
  c->last_all_paths = (int64_t)ctl[CTL_CNT + C2D_CNT_PATHS_INT];
  hc[C2D_CNT_PATHS_INT] = 0.0;              /* internal: not tally counters */
  hc[C2D_CNT_DEAD_INT] = 0.0;
  c->last_creuse = (int64_t)ctl[CTL_CNT + C2D_CNT_CREUSE_INT];
  c->last_clost = (int64_t)ctl[CTL_CNT + C2D_CNT_CLOST_INT];
  hc[C2D_CNT_CREUSE_INT] = 0.0;
  hc[C2D_CNT_CLOST_INT] = 0.0;
  hc[C2D_CNT_GENS] = (double)gen;
  HIPCHK(c, hipMemcpyAsync(c->T + c->L.counters, hc, sizeof hc, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->n_ev = 0;
  unsigned long long ev_reserved = 0;
  for (int sh = 0; sh < C2D_EV_SHARDS; sh++) {
    const unsigned long long m = ctl[CTL_EVSH + sh * C2D_EV_SHARD_STRIDE];
    ev_reserved += m;
    c->ev_cnt[sh] = std::min<int64_t>((int64_t)m, c->ev_cap_sh);
    c->n_ev += c->ev_cnt[sh];
  }
  c->n_census = cens_live;
  c->cur = out_buf;
  c->g0_launched = false;        /* the new census is complete: later failures keep it */
  if (herr & ERR_EVENT) {
    unsigned long long fill = 0;
    for (int sh = 0; sh < C2D_EV_SHARDS; sh++)
      fill = std::max(fill, ctl[CTL_EVSH + sh * C2D_EV_SHARD_STRIDE]);
    return fail(c, C2D_E_EVENT_OVERFLOW,
                "event buffer overflow: %llu events, capacity %lld = %d shards of %lld (the "
                "fullest shard took %llu: size event_capacity >= %d x that)", ev_reserved,
                (long long)cfg.event_capacity, C2D_EV_SHARDS, (long long)c->ev_cap_sh, fill,
                C2D_EV_SHARDS);
  }
  if (herr & ERR_QUEUE) return fail(c, C2D_E_QUEUE_OVERFLOW, "scatter queue overflow");
  if (herr & ERR_SPEC) return fail(c, C2D_E_ARG, "surface packet without a seed spectrum");
  if (herr & ERR_NONFINITE)
    return fail(c, C2D_E_NONFINITE, "NaN/Inf in the step's tallies (edep, n_field, ecens, ...)");
  return C2D_OK;
}

extern "C" int c2d_transport_step(c2d_ctx* c, const c2d_step_in* in) {
  int rc = c2d_set_step(c, in);
  if (rc) return rc;
  return c2d_run_step(c);
}

extern "C" int c2d_tally_layout_get(c2d_ctx* c, c2d_tally_layout* out) {
  if (!c || !out) return C2D_E_ARG;
  *out = c->L;
  return C2D_OK;
}

extern "C" double* c2d_tally_device_ptr(c2d_ctx* c) { return c ? c->T : nullptr; }

extern "C" int c2d_set_tally_buffer(c2d_ctx* c, double* device_ptr) {
  if (!c) return C2D_E_ARG;
  c->T = device_ptr ? device_ptr : c->T_own;
  return C2D_OK;
}

extern "C" int c2d_tally_download(c2d_ctx* c, double* host, int64_t n) {
  if (!c || !host || n < c->L.total) return C2D_E_ARG;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, hipMemcpy(host, c->T, sizeof(double) * c->L.total, hipMemcpyDeviceToHost));
  return C2D_OK;
}

extern "C" int c2d_tally_download_range(c2d_ctx* c, double* host, int64_t offset, int64_t n) {
  if (!c || (!host && n > 0) || offset < 0 || n < 0 || offset + n > c->L.total) return C2D_E_ARG;
  if (n == 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  /* synchronous like c2d_tally_download: ordered after the library's stream
   * and a caller's all-reduce on the null stream alike */
  HIPCHK(c, hipMemcpy(host, c->T + offset, sizeof(double) * n, hipMemcpyDeviceToHost));
  return C2D_OK;
}

extern "C" int c2d_events(c2d_ctx* c, double* buf, int64_t cap, int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  *n = c->n_ev;
  if (!buf) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  int64_t done = 0;   /* the shards' filled prefixes, in shard order */
  for (int sh = 0; sh < C2D_EV_SHARDS && done < cap; sh++) {
    const int64_t m = std::min(cap - done, c->ev_cnt[sh]);
    if (m > 0)
      HIPCHK(c, hipMemcpy(buf + done * C2D_EVENT_WORDS,
                          c->ev + (size_t)sh * c->ev_cap_sh * C2D_EVENT_WORDS,
                          sizeof(double) * C2D_EVENT_WORDS * m, hipMemcpyDeviceToHost));
    done += m;
  }
  return C2D_OK;
}

/* Fast contexts keep the census azimuth encoded (CensusSoA): phi column =
 * cos(phi), C2D_CENS_ESW in bins = the quadrant switch.  The host sees the
 * reference's phi: decoded with the kernel's own c2d_acos, encoded with its
 * c2d_cos (the value the kernel's set_phi would compute).  The kernel clamps
 * the cosine it stores to 0.999999999 (imctrk2d.f:472-477), so cos(phi) ==
 * 1.0 with the switch set only comes from an import of phi < 1e-10 (or of
 * phi within 1e-10 of 2*pi, which the kernel treats identically): it
 * decodes to 0.0, so an import of phi = 0 exports 0. */
static constexpr double C2D_PI_REF = 3.1415926536;   /* general.pa:24 */
static inline bool cens_encoded(const c2d_ctx* c) { return c->cfg.comtot_mode == C2D_COMTOT_TABLE; }
static inline double cens_phi_decode(double eta, uint32_t bins) {
  if (eta == 1.0 && (bins & C2D_CENS_ESW)) return 0.0;
  const double ph = c2d_acos(eta);
  return (bins & C2D_CENS_ESW) ? 2.0 * C2D_PI_REF - ph : ph;
}

extern "C" int c2d_census_count(c2d_ctx* c, int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  *n = c->n_census;
  return C2D_OK;
}

/* census records first, first + stride, ... -> packed records (the chunk
 * list maps them to slots in the chunked census) */
__global__ void __launch_bounds__(256) c2d_census_pack_kernel(CensusSoA cs, const int32_t* __restrict__ clist,
                                                              int64_t first, int64_t stride, int64_t n,
                                                              uint64_t* __restrict__ rec) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    rec_pack(cs, cens_slot(clist, first + i * stride), rec + i * C2D_CENSUS_REC_WORDS);
}

/* packed records -> census records first, first + 1, ... */
__global__ void __launch_bounds__(256) c2d_census_unpack_kernel(CensusSoA cs, const int32_t* __restrict__ clist,
                                                                int64_t first, int64_t n,
                                                                const uint64_t* __restrict__ rec) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    rec_unpack(cs, cens_slot(clist, first + i), rec + i * C2D_CENSUS_REC_WORDS);
}

/* flag = 1 if a packed record's jk word lacks its E_ph bin (ie = 0) or its
 * cell lies off the grid: the kernels read kappa at ie - 1 without a lookup */
__global__ void __launch_bounds__(256) c2d_census_check_kernel(const uint64_t* __restrict__ rec, int64_t n,
                                                               int nz, int nr, int32_t* __restrict__ flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t jk = (uint32_t)(rec[i * C2D_CENSUS_REC_WORDS + 6] & 0xffffffffull);
    const int ie = c2d_cens_ie(jk), j = c2d_cens_j(jk), k = c2d_cens_k(jk);
    if (ie < 1 || ie > C2D_N_VOL || j < 1 || j > nz || k < 1 || k > nr) atomicOr(flag, 1);
  }
}

static const int32_t* cens_list(const c2d_ctx* c) { return c->chunked ? c->clist[c->ccur] : nullptr; }

/* m census records first, first + stride, ... to the host, as the
 * reference's record (d6: rpre zpre wmu phi ew xnu; i5: jgpsp jgplc jgpmu
 * jph kph; keys), in batches through the packed form */
static int census_download(c2d_ctx* c, int64_t first, int64_t stride, int64_t m, double* d6, int32_t* i5,
                           uint64_t* keys) {
  int rc = ensure_tmp(c, std::min<int64_t>(m, int64_t(1) << 20));
  if (rc) return rc;
  const int64_t B = std::min<int64_t>(c->tmp_cap, int64_t(1) << 20);
  std::vector<uint64_t> h((size_t)std::min(m, B) * C2D_CENSUS_REC_WORDS);
  const bool enc = cens_encoded(c);
  const CensusSoA cs = c->cens[c->cur].soa();
  for (int64_t b0 = 0; b0 < m; b0 += B) {
    const int64_t nb = std::min(B, m - b0);
    const int g = (int)std::min<int64_t>((nb + 255) / 256, (int64_t)c->n_cu * 8);
    hipLaunchKernelGGL(c2d_census_pack_kernel, dim3(g), dim3(256), 0, c->stream, cs, cens_list(c),
                       first + b0 * stride, stride, nb, c->tmp_rec);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h.data(), c->tmp_rec, sizeof(uint64_t) * C2D_CENSUS_REC_WORDS * nb,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int64_t t = 0; t < nb; t++) {
      const uint64_t* r = h.data() + t * C2D_CENSUS_REC_WORDS;
      const int64_t o = b0 + t;
      const uint32_t jk = (uint32_t)(r[6] & 0xffffffffull), bins = (uint32_t)(r[6] >> 32);
      if (d6)
        for (int f = 0; f < 6; f++) {
          double v;
          memcpy(&v, r + f, sizeof v);
          d6[6 * o + f] = (f == 3 && enc) ? cens_phi_decode(v, bins) : v;
        }
      if (i5) {
        i5[5 * o + 0] = (int32_t)(bins & 0xff);
        i5[5 * o + 1] = (int32_t)((bins >> 8) & 0xff);
        i5[5 * o + 2] = (int32_t)((bins >> 16) & 0xff);
        i5[5 * o + 3] = (int32_t)c2d_cens_j(jk);
        i5[5 * o + 4] = (int32_t)c2d_cens_k(jk);
      }
      if (keys) keys[o] = r[7];
    }
  }
  return C2D_OK;
}

extern "C" int c2d_census_export_range(c2d_ctx* c, int64_t first, int64_t stride, double* d6,
                                       int32_t* i5, uint64_t* keys, int64_t cap, int64_t* n) {
  if (!c || !n || first < 0 || stride < 1) return C2D_E_ARG;
  if (c->census_lost) return census_lost(c, "c2d_census_export_range");
  const int64_t avail = first < c->n_census ? (c->n_census - first + stride - 1) / stride : 0;
  *n = avail;
  const int64_t m = std::min(cap, avail);
  if (m <= 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  return census_download(c, first, stride, m, d6, i5, keys);
}

extern "C" int c2d_census_export(c2d_ctx* c, double* d6, int32_t* i5, uint64_t* keys, int64_t cap,
                                 int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  if (c->census_lost) return census_lost(c, "c2d_census_export");
  *n = c->n_census;
  const int64_t m = std::min(cap, c->n_census);
  if (m <= 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  return census_download(c, 0, 1, m, d6, i5, keys);
}

extern "C" int c2d_census_import(c2d_ctx* c, const double* d6, const int32_t* i5,
                                 const uint64_t* keys, int64_t n) {
  if (!c || n < 0 || (n > 0 && (!d6 || !i5 || !keys))) return C2D_E_ARG;
  if (n > c->cfg.census_capacity)
    return fail(c, C2D_E_CENSUS_OVERFLOW, "census import %lld > capacity", (long long)n);
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  /* records [0, n) of the SoA (chunked: the list's chunks 0, 1, ...), in
   * batches so the host staging stays bounded */
  const DevCensus& d = c->cens[c->cur];
  const bool enc = cens_encoded(c);
  const int64_t B = std::min<int64_t>(n, int64_t(1) << 20);
  std::vector<c2d_d2> col((size_t)B);
  std::vector<c2d_u4> tg((size_t)B);
  for (int64_t i0 = 0; i0 < n; i0 += B) {
    const int64_t nb = std::min(B, n - i0);
    for (int f = 0; f < 3; f++) {
      for (int64_t t = 0; t < nb; t++) {
        const double* r = d6 + 6 * (i0 + t);
        col[t].x = r[2 * f];
        col[t].y = (f == 1 && enc) ? c2d_cos(r[3]) : r[2 * f + 1];
      }
      HIPCHK(c, hipMemcpy(d.d[f] + i0, col.data(), nb * sizeof(c2d_d2), hipMemcpyHostToDevice));
    }
    for (int64_t t = 0; t < nb; t++) {
      const int64_t i = i0 + t;
      const int32_t* q = i5 + 5 * i;
      if (q[3] < 1 || q[3] > c->nz || q[4] < 1 || q[4] > c->nr || q[0] < 0 || q[0] > 255 ||
          q[1] < 0 || q[1] > 255 || q[2] < 0 || q[2] > 255)
        return fail(c, C2D_E_ARG, "census record %lld out of range", (long long)i);
      uint32_t bins = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
      if (enc) {
        const double ph = d6[6 * i + 3];
        if (!(ph <= C2D_PI_REF && ph >= 1.0e-10)) bins |= C2D_CENS_ESW;
      }
      /* the E_ph / E_field bins of xnu the record carries (c2d_cens_jk), with
       * the kernels' semantics (grid_lookup = the bisection, build_lookup) */
      const double xnu = d6[6 * i + 5];
      const int ie = grid_bin_host(c->geo_h.E_ph, C2D_N_VOL, xnu);
      const int efl = xnu > c->egg_min ? grid_bin_host(c->geo_h.E_field, C2D_NPHFIELD, xnu) : 0;
      tg[t].x = c2d_cens_jk(q[3], q[4], ie, efl);
      tg[t].y = bins;
      tg[t].z = (uint32_t)keys[i];
      tg[t].w = (uint32_t)(keys[i] >> 32);
    }
    HIPCHK(c, hipMemcpy(d.tg + i0, tg.data(), nb * sizeof(c2d_u4), hipMemcpyHostToDevice));
  }
  if (c->chunked) {
    const int64_t k = (n + C2D_CCHUNK - 1) / C2D_CCHUNK;
    std::vector<int32_t> ids(k);
    for (int64_t i = 0; i < k; i++) ids[i] = (int32_t)i;
    if (k) HIPCHK(c, hipMemcpy(c->clist[c->ccur], ids.data(), k * sizeof(int32_t), hipMemcpyHostToDevice));
    c->n_clist = k;
  }
  c->n_census = n;
  c->census_lost = false;
  return C2D_OK;
}

extern "C" int c2d_census_pack(c2d_ctx* c, int64_t first, int64_t n, uint64_t* d_rec) {
  if (!c || first < 0 || n < 0 || (n > 0 && !d_rec)) return C2D_E_ARG;
  if (c->census_lost) return census_lost(c, "c2d_census_pack");
  if (first + n > c->n_census)
    return fail(c, C2D_E_ARG, "c2d_census_pack: records [%lld, %lld) beyond the census (%lld)",
                (long long)first, (long long)(first + n), (long long)c->n_census);
  if (n == 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const int grid = (int)std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 8);
  hipLaunchKernelGGL(c2d_census_pack_kernel, dim3(grid), dim3(256), 0, c->stream,
                     c->cens[c->cur].soa(), cens_list(c), first, (int64_t)1, n, d_rec);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return C2D_OK;
}

extern "C" int c2d_census_append(c2d_ctx* c, const uint64_t* d_rec, int64_t n) {
  if (!c || n < 0 || (n > 0 && !d_rec)) return C2D_E_ARG;
  if (c->census_lost) return census_lost(c, "c2d_census_append");
  if (c->n_census + n > c->cfg.census_capacity)
    return fail(c, C2D_E_CENSUS_OVERFLOW, "c2d_census_append: %lld + %lld > capacity %lld",
                (long long)c->n_census, (long long)n, (long long)c->cfg.census_capacity);
  if (n == 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  {   /* every record carries its cell and E_ph bin (c2d_cens_jk) */
    const int grid = (int)std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 8);
    int32_t bad = 0;
    HIPCHK(c, hipMemsetAsync(c->derr, 0, sizeof(int32_t), c->stream));
    hipLaunchKernelGGL(c2d_census_check_kernel, dim3(grid), dim3(256), 0, c->stream, d_rec, n, c->nz, c->nr,
                       c->derr);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(&bad, c->derr, sizeof bad, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (bad) return fail(c, C2D_E_ARG, "c2d_census_append: a record without its cell or E_ph bin (c2d_census_pack "
                         "format, include/compton2d.h)");
  }
  if (c->chunked) {
    /* the list's last chunk fills up first, then free chunks join the list */
    const int64_t k = (c->n_census + n + C2D_CCHUNK - 1) / C2D_CCHUNK - c->n_clist;
    if (k > 0) {
      int64_t n_free = 0;
      int rc = chunk_pool_build(c, &n_free);
      if (rc) return rc;
      if (n_free < k)
        return fail(c, C2D_E_CENSUS_OVERFLOW, "c2d_census_append: %lld free census chunks, %lld needed",
                    (long long)n_free, (long long)k);
      HIPCHK(c, hipMemcpyAsync(c->clist[c->ccur] + c->n_clist, c->pool, sizeof(int32_t) * k,
                               hipMemcpyDeviceToDevice, c->stream));
      c->n_clist += k;
    }
  }
  const int grid = (int)std::min<int64_t>((n + 255) / 256, (int64_t)c->n_cu * 8);
  hipLaunchKernelGGL(c2d_census_unpack_kernel, dim3(grid), dim3(256), 0, c->stream,
                     c->cens[c->cur].soa(), cens_list(c), c->n_census, n, d_rec);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->n_census += n;
  return C2D_OK;
}

extern "C" int c2d_census_truncate(c2d_ctx* c, int64_t n) {
  if (!c || n < 0 || n > c->n_census) return C2D_E_ARG;
  c->census_lost = false;
  c->n_census = n;
  if (c->chunked) c->n_clist = (n + C2D_CCHUNK - 1) / C2D_CCHUNK;
  return C2D_OK;
}

extern "C" int c2d_fp_tridag(c2d_ctx* c, const c2d_fp_in* in, double* x) {
  if (!c || !in || !x || in->ncell < 0 || in->nt < 1) return C2D_E_ARG;
  if (in->ncell == 0) return C2D_OK;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const size_t n = (size_t)in->ncell * in->nt;
  double *a, *b, *cc, *r, *xd;
  HIPCHK(c, dalloc(&a, n));
  HIPCHK(c, dalloc(&b, n));
  HIPCHK(c, dalloc(&cc, n));
  HIPCHK(c, dalloc(&r, n));
  HIPCHK(c, dalloc(&xd, n));
  HIPCHK(c, hipMemcpy(a, in->a, n * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(b, in->b, n * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(cc, in->c, n * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(r, in->r, n * sizeof(double), hipMemcpyHostToDevice));
  /* |b(1)| <= 1e-100 leaves the previous solution untouched (update2d.f:2490-2493) */
  HIPCHK(c, hipMemcpy(xd, x, n * sizeof(double), hipMemcpyHostToDevice));
  int rc = c2d_launch_tridag(a, b, cc, r, xd, in->ncell, in->nt, c->stream);
  if (rc) return fail(c, C2D_E_HIP, "tridag launch: %d", rc);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(x, xd, n * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(a); (void)hipFree(b); (void)hipFree(cc); (void)hipFree(r); (void)hipFree(xd);
  return C2D_OK;
}

extern "C" int c2d_last_gen0_steps(c2d_ctx* c, int64_t* steps) {
  if (!c || !steps) return C2D_E_ARG;
  *steps = c->last_g0_steps;
  return C2D_OK;
}

extern "C" int c2d_last_path_steps(c2d_ctx* c, int64_t* gen0_paths, int64_t* all_paths) {
  if (!c) return C2D_E_ARG;
  if (gen0_paths) *gen0_paths = c->last_g0_paths;
  if (all_paths) *all_paths = c->last_all_paths;
  return C2D_OK;
}

extern "C" int c2d_last_compaction(c2d_ctx* c, int32_t* rounds, int64_t* moved, int64_t* physical) {
  if (!c) return C2D_E_ARG;
  if (rounds) *rounds = c->last_compact_rounds;
  if (moved) *moved = c->last_compact_moved;
  if (physical) *physical = c->cens_phys;
  return C2D_OK;
}

extern "C" int c2d_last_census_chunks(c2d_ctx* c, int64_t* chunks, int64_t* recycled, int64_t* unrecycled,
                                      int64_t* physical) {
  if (!c) return C2D_E_ARG;
  if (chunks) *chunks = c->chunked ? c->n_clist : 0;
  if (recycled) *recycled = c->last_creuse;
  if (unrecycled) *unrecycled = c->last_clost;
  if (physical) *physical = c->chunked ? c->nchunks : 0;
  return C2D_OK;
}

extern "C" int c2d_transport_prof(c2d_ctx* c, uint64_t* out, int32_t n) {
  if (!c || !out || n < 0) return C2D_E_ARG;
  for (int i = 0; i < n && i < C2D_TR_PROF_WORDS; i++) out[i] = c->last_prof[i];
  return C2D_OK;
}

extern "C" int c2d_last_kernel_ms(c2d_ctx* c, double* gen0_ms, double* all_ms, int32_t* launches) {
  if (!c) return C2D_E_ARG;
  if (gen0_ms) *gen0_ms = c->last_g0_ms;
  if (all_ms) *all_ms = c->last_all_ms;
  if (launches) *launches = c->last_launches;
  return C2D_OK;
}

/* ------------------------------------------------------------------ */
/* Fokker-Planck (src/update2d.f:7-327, FP_calc :337-1739)             */
/* ------------------------------------------------------------------ */
/* McDonald series abscissae (volume2d.f:604-620) for the wave-level K2/K3
 * (c2d_wave.hpp): t_n by repeated multiplication exactly as the reference
 * loop forms it, with the argument-independent factors of each term (same
 * c2d_math code and rounding as the kernels).  Built once per context. */
#define C2D_FP_MEMO_SLOTS (1u << 16)
/* the fast kernel's table: every zone off the clamp inserts its own chain
 * values, so it is sized so that probes stay short (16 MB) */
#define C2D_FPF_MEMO_SLOTS (1u << 20)
/* *dst = a zeroed device buffer of n T's, published only once zeroed */
template <typename T>
static int alloc_zeroed(c2d_ctx* c, T** dst, size_t n) {
  if (*dst) return C2D_OK;
  T* p = nullptr;
  HIPCHK(c, dalloc(&p, n));
  const hipError_t e = hipMemset(p, 0, sizeof(T) * n);
  if (e != hipSuccess) {
    (void)hipFree(p);
    HIPCHK(c, e);
  }
  *dst = p;
  return C2D_OK;
}

static int ensure_mcd(c2d_ctx* c) {
  /* every buffer has its own guard, so a failed allocation is retried by the
   * next call instead of being reported as done with null pointers */
  if (!c->fp_mcd) {
    std::vector<double> mt((size_t)C2D_FP_MCD_N * 4);
    const double dtm = 1.001, sm = 5.0e-1 * (1.0 + dtm);
    double t = 1.0;
    for (int n = 0; n < C2D_FP_MCD_N; n++) {
      const double ts = t * sm;
      mt[(size_t)n * 4 + 0] = t;
      mt[(size_t)n * 4 + 1] = ts;
      mt[(size_t)n * 4 + 2] = c2d_pow(ts * ts - 1.0, 1.5);
      mt[(size_t)n * 4 + 3] = c2d_pow(ts * ts - 1.0, 2.5);
      t = t * dtm;
    }
    double* m = nullptr;
    HIPCHK(c, dalloc(&m, mt.size()));
    const hipError_t e = hipMemcpy(m, mt.data(), mt.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(m);
      HIPCHK(c, e);
    }
    c->fp_mcd = m;
  }
  /* the gamma_bar memo lives as long as the context (gamma_bar is a pure
   * function of Theta); C2D_FP_MEMO=0 disables it (A/B) */
  const char* e = getenv("C2D_FP_MEMO");
  if (!(e && e[0] == '0')) {
    /* zeroed before they are published: a buffer whose memset failed is
     * freed, so the next call retries it instead of reading garbage keys */
    if (int rc = alloc_zeroed(c, &c->fp_gb_key, C2D_FP_MEMO_SLOTS)) return rc;
    if (int rc = alloc_zeroed(c, &c->fp_gb_val, C2D_FP_MEMO_SLOTS)) return rc;
    if (int rc = alloc_zeroed(c, &c->fpf_gb_key, C2D_FPF_MEMO_SLOTS)) return rc;
    if (int rc = alloc_zeroed(c, &c->fpf_gb_val, C2D_FPF_MEMO_SLOTS)) return rc;
  }
  if (!c->fp_dP) HIPCHK(c, dalloc(&c->fp_dP, 1));
  if (!c->fpf_zq) HIPCHK(c, dalloc(&c->fpf_zq, (size_t)c->ncell + 1));
  /* the fast kernel's McDonald moment table (fp_fast.hip mcd_mtab): 6.9 MB,
   * built on the device once (~1 ms); C2D_FPF_MTAB=0 leaves it out (A/B) */
  const char* mt = getenv("C2D_FPF_MTAB");
  if (!(mt && mt[0] == '0') && !c->fpf_mom) {
    double* m = nullptr;
    HIPCHK(c, dalloc(&m, (size_t)C2D_FPF_MT_N * C2D_FPF_MT_W));
    const int rb = c2d_fp_mom_build(c->fp_mcd, m, c->stream);
    const hipError_t e = rb ? (hipError_t)rb : hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      (void)hipFree(m);
      HIPCHK(c, e);
    }
    c->fpf_mom = m;
  }
  if ((int)c->fpf_order.size() != c->ncell) {
    c->fpf_order.resize(c->ncell);
    for (int q = 0; q < c->ncell; q++) c->fpf_order[q] = q;
  }
  return C2D_OK;
}

extern "C" int c2d_fp_set_config(c2d_ctx* c, const c2d_fp_config* fc) {
  if (!c || !fc || !fc->F_IC) return C2D_E_ARG;
  if (fc->pair_switch != 0 && fc->pair_switch != 1)
    return fail(c, C2D_E_ARG, "pair_switch must be 0 or 1 (got %d)", fc->pair_switch);
  if (fc->inj_switch != 0 && fc->inj_dis != 1 && fc->inj_dis != 2)
    return fail(c, C2D_E_ARG, "inj_dis must be 1 or 2 when inj_switch is on (got %d)", fc->inj_dis);
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const size_t nc = (size_t)c->ncell;
  if (!c->fp_FT) {
    HIPCHK(c, dalloc(&c->fp_FT, (size_t)C2D_NPHFIELD * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->fp_zin, nc * FZ_N));
    HIPCHK(c, dalloc(&c->fp_fin, nc * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->fp_Pin, nc * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->fp_nf, nc * C2D_NPHFIELD));
    HIPCHK(c, dalloc(&c->fp_fout, nc * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->fp_Pout, nc * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->fp_zout, nc * FO_N));
    HIPCHK(c, dalloc(&c->fp_err, 1));
  }
  if (int rc = ensure_mcd(c)) return rc;
  /* F_IC(i, ph) -> FT[ph][i]: lanes (bins i) read consecutive addresses */
  std::vector<double> ft((size_t)C2D_NPHFIELD * C2D_NUM_NT);
  for (int ph = 0; ph < C2D_NPHFIELD; ph++)
    for (int i = 0; i < C2D_NUM_NT; i++)
      ft[(size_t)ph * C2D_NUM_NT + i] = fc->F_IC[i * fc->F_IC_s_i + ph * fc->F_IC_s_ph];
  HIPCHK(c, hipMemcpy(c->fp_FT, ft.data(), ft.size() * sizeof(double), hipMemcpyHostToDevice));
  c->fpc = *fc;
  c->fpc.F_IC = nullptr;
  c->fp_ready = true;
  return C2D_OK;
}

extern "C" int c2d_fp_set_mode(c2d_ctx* c, int32_t mode) {
  if (!c) return C2D_E_ARG;
  if (mode != C2D_FP_EXACT && mode != C2D_FP_FAST && mode != C2D_FP_AUTO)
    return fail(c, C2D_E_ARG, "c2d_fp_set_mode: mode %d is not C2D_FP_EXACT, C2D_FP_FAST or C2D_FP_AUTO", mode);
  c->fp_mode = mode;
  return C2D_OK;
}

extern "C" int c2d_last_fp_mode(c2d_ctx* c, int32_t* mode) {
  if (!c || !mode) return C2D_E_ARG;
  *mode = c->last_fp_mode;
  return C2D_OK;
}

/* the reference's tea clamp (src/update2d.f:266-276): temp_min, temp_max */
static bool on_tea_clamp(double te) { return te >= 1.0e3 || te <= 5.0; }

extern "C" int c2d_fp_step(c2d_ctx* c, const c2d_fp_step_in* in, c2d_fp_step_out* out) {
  if (!c || !in || !out) return C2D_E_ARG;
  if (!c->fp_ready) return fail(c, C2D_E_STATE, "c2d_fp_set_config must precede c2d_fp_step");
  const bool el_dev = !out->f_nt.data && !out->Pnt.data;   /* C2D_DEV_ELECTRONS */
  if (!el_dev && (!out->f_nt.data || !out->Pnt.data))
    return fail(c, C2D_E_ARG, "c2d_fp_step: pass both f_nt and Pnt views, or neither (device state)");
  if (el_dev && !c->have_electrons)
    return fail(c, C2D_E_STATE, "c2d_fp_step: no electron state on the device (c2d_set_step first)");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const int nz = c->nz, nr = c->nr, nc = c->ncell;
  const bool nf_dev = in->n_field.data == nullptr, ecens_dev = in->ecens.data == nullptr;
  auto a2 = [](const c2d_array2& a, int j, int k, double d) {
    return a.data ? a.data[j * a.s_j + k * a.s_k] : d;
  };
  auto m2 = [](const c2d_marray2& a, int j, int k) -> double* {
    return a.data ? &a.data[j * a.s_j + k * a.s_k] : nullptr;
  };
  const size_t nnt = el_dev ? 0 : (size_t)nc * C2D_NUM_NT;
  std::vector<double> zin((size_t)nc * FZ_N, 0.0), fin(nnt), pin(nnt),
      nf(nf_dev ? 0 : (size_t)nc * C2D_NPHFIELD);
  for (int j = 0; j < nz; j++)
    for (int k = 0; k < nr; k++) {
      const int cell = j * nr + k;
      double* z = &zin[(size_t)cell * FZ_N];
      z[FZ_VOL] = a2(in->vol, j, k, 0.0);
      z[FZ_TEA] = a2(in->tea, j, k, 0.0);
      z[FZ_TNA] = a2(in->tna, j, k, 0.0);
      z[FZ_NE] = a2(in->n_e, j, k, 0.0);
      z[FZ_B] = a2(in->B_field, j, k, 0.0);
      z[FZ_ELSY] = a2(in->Eloss_sy, j, k, 0.0);
      z[FZ_ECENS] = a2(in->ecens, j, k, 0.0);
      z[FZ_ECOLD] = a2(in->ec_old, j, k, 0.0);
      z[FZ_TURB] = a2(in->turb_lev, j, k, 0.0);
      z[FZ_FPAIR] = a2(in->f_pair, j, k, 0.0);
      if (c->fpc.pair_switch == 1 && z[FZ_FPAIR] != 0.0)
        return fail(c, C2D_E_ARG,
                    "pair_switch=1 needs f_pair = 0 (positrons are inert, H6); zone (%d,%d) has %g",
                    j + 1, k + 1, z[FZ_FPAIR]);
      const double* pp = m2(out->p_nth, j, k);
      z[FZ_PNTH] = pp ? *pp : 0.0;
      for (int i = 0; i < C2D_NUM_NT && !el_dev; i++) {
        fin[(size_t)cell * C2D_NUM_NT + i] =
            out->f_nt.data[i * out->f_nt.s_i + j * out->f_nt.s_j + k * out->f_nt.s_k];
        pin[(size_t)cell * C2D_NUM_NT + i] =
            out->Pnt.data[i * out->Pnt.s_i + j * out->Pnt.s_j + k * out->Pnt.s_k];
      }
      if (!nf_dev)
        for (int ph = 0; ph < C2D_NPHFIELD; ph++)
          nf[(size_t)cell * C2D_NPHFIELD + ph] =
              in->n_field.data[ph * in->n_field.s_i + j * in->n_field.s_j + k * in->n_field.s_k];
    }
  /* C2D_FP_AUTO: exact while the last update left every zone on the tea
   * clamp within a few sub-steps, fast otherwise (include/compton2d.h) */
  int32_t fm = c->fp_mode;
  if (fm == C2D_FP_AUTO) {
    /* the zones' tea as this update starts (the last update's Te_new,
     * clamped) and the last update's slowest zone */
    bool exact = !c->fp_auto_known || c->fp_auto_exact;
    for (int cell = 0; cell < nc; cell++) {
      const double* z = &zin[(size_t)cell * FZ_N];
      if (z[FZ_NE] * (1.0 + z[FZ_FPAIR]) < 1.0e-11) continue;   /* skipped (update2d.f:478) */
      exact = exact && on_tea_clamp(z[FZ_TEA]);
    }
    fm = exact ? C2D_FP_EXACT : C2D_FP_FAST;
  }
  /* NaN/Inf in what FP_calc reads is C2D_E_FP (the reference would carry it
   * into f_nt, tea and the next step's tables) */
  if (!all_finite(zin.data(), zin.size()) || !all_finite(fin.data(), fin.size()) ||
      !all_finite(pin.data(), pin.size()) || !all_finite(nf.data(), nf.size()))
    return fail(c, C2D_E_FP, "c2d_fp_step: NaN/Inf in the zone inputs, f_nt/Pnt or n_field");
  const hipStream_t st = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->fp_zin, zin.data(), zin.size() * sizeof(double), hipMemcpyHostToDevice, st));
  if (!el_dev) {
    HIPCHK(c, hipMemcpyAsync(c->fp_fin, fin.data(), fin.size() * sizeof(double), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->fp_Pin, pin.data(), pin.size() * sizeof(double), hipMemcpyHostToDevice, st));
  }
  if (!nf_dev)
    HIPCHK(c, hipMemcpyAsync(c->fp_nf, nf.data(), nf.size() * sizeof(double), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemsetAsync(c->fp_err, 0, sizeof(int32_t), st));
  FpParams P;
  memset(&P, 0, sizeof P);
  const c2d_fp_config& f = c->fpc;
  P.nz = nz; P.nr = nr; P.pick_sw = f.pick_sw; P.inj_switch = f.inj_switch; P.inj_dis = f.inj_dis;
  P.g2var_switch = f.g2var_switch; P.cf_sentinel = f.cf_sentinel; P.pair_sw = f.pair_switch;
  P.time = in->time; P.dt = in->dt; P.df_implicit = f.df_implicit; P.df_T = f.df_T;
  P.r_esc = f.r_esc; P.r_acc = f.r_acc; P.r_flare = f.r_flare; P.z_flare = f.z_flare;
  P.t_flare = f.t_flare; P.sigma_r = f.sigma_r; P.sigma_z = f.sigma_z; P.sigma_t = f.sigma_t;
  P.flare_amp = f.flare_amp; P.inj_g1 = f.inj_g1; P.inj_g2 = f.inj_g2; P.inj_p = f.inj_p;
  P.inj_t = f.inj_t; P.inj_L = f.inj_L; P.pick_rate = f.pick_rate; P.inj_gg = f.inj_gg;
  P.inj_sigma = f.inj_sigma; P.inj_v = f.inj_v;
  P.geo = c->geo; P.gnt = c->gnt; P.FT = c->fp_FT; P.mcd = c->fp_mcd; P.zin = c->fp_zin;
  /* device electron state: the kernel writes the staging rows (seeded with
   * the current state, so skipped zones carry it), which replace the state
   * only once the step has succeeded: after C2D_E_FP the device electrons
   * are those before the call, as the caller's arrays are in host mode */
  const size_t nt_bytes = (size_t)nc * C2D_NUM_NT * sizeof(double);
  if (el_dev) {
    HIPCHK(c, hipMemcpyAsync(c->fp_fout, c->f_nt, nt_bytes, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->fp_Pout, c->Pnt, nt_bytes, hipMemcpyDeviceToDevice, st));
  }
  P.f_in = el_dev ? c->f_nt : c->fp_fin;
  P.P_in = el_dev ? c->Pnt : c->fp_Pin;
  P.nf = nf_dev ? c->T + c->L.n_field : c->fp_nf;    /* tally layout: [cell][nphfield] */
  P.ecens = ecens_dev ? c->T + c->L.ecens : nullptr;
  P.f_out = c->fp_fout;
  P.P_out = c->fp_Pout;
  P.zout = c->fp_zout; P.err = c->fp_err;
  P.gb_key = c->fp_gb_key; P.gb_val = c->fp_gb_val; P.gb_mask = C2D_FP_MEMO_SLOTS - 1u;
  if (fm == C2D_FP_FAST) {
    if (!c->fp_dP || !c->fpf_zq || !c->fp_mcd)
      return fail(c, C2D_E_STATE, "c2d_fp_step: the fast kernel's buffers are not allocated");
    P.gb_key = c->fpf_gb_key; P.gb_val = c->fpf_gb_val; P.gb_mask = C2D_FPF_MEMO_SLOTS - 1u;
    /* zones from a queue, costliest first (by the last update's sub-step
     * counts), on one workgroup per CU (C2D_FPF_GRID: another grid size,
     * 0 = one workgroup per zone) */
    P.zq = c->fpf_zq;
    P.zorder = c->fpf_zq + 1;
    /* McDonald pairs from the moment table; C2D_FPF_MTAB=2 keeps consulting
     * the shared gamma_bar memo as well */
    const char* mt = getenv("C2D_FPF_MTAB");
    P.mom = (mt && mt[0] == '0') ? nullptr : c->fpf_mom;
    P.mt_glob = (mt && mt[0] == '2') ? 1 : 0;
    P.ncell = (int32_t)nc;
    HIPCHK(c, hipMemcpyAsync(c->fpf_zq + 1, c->fpf_order.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemsetAsync(c->fpf_zq, 0, sizeof(int32_t), st));
    /* C2D_FPF_MEMO_RESET=1: every update starts from an empty gamma_bar memo
     * (measurement: the cost of temperatures the memo has not seen) */
    const char* mr = getenv("C2D_FPF_MEMO_RESET");
    if (mr && mr[0] == '1' && c->fpf_gb_key) {
      HIPCHK(c, hipMemsetAsync(c->fpf_gb_key, 0, sizeof(unsigned long long) * C2D_FPF_MEMO_SLOTS, st));
      HIPCHK(c, hipMemsetAsync(c->fpf_gb_val, 0, sizeof(double) * C2D_FPF_MEMO_SLOTS, st));
    }
    HIPCHK(c, hipMemcpyAsync(c->fp_dP, &P, sizeof P, hipMemcpyHostToDevice, st));
  }
  /* the device-resident inputs: this step's n_field/ecens tallies, f_nt/Pnt */
  if (nf_dev) check_finite(c, P.nf, (int64_t)nc * C2D_NPHFIELD, FPERR_NF_IN, c->fp_err, st);
  if (ecens_dev) check_finite(c, P.ecens, nc, FPERR_NF_IN, c->fp_err, st);
  if (el_dev) {
    check_finite(c, c->f_nt, (int64_t)nc * C2D_NUM_NT, FPERR_NF_IN, c->fp_err, st);
    check_finite(c, c->Pnt, (int64_t)nc * C2D_NUM_NT, FPERR_NF_IN, c->fp_err, st);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev_g0a, st));
  int rc;
  if (fm == C2D_FP_FAST) {
    const int bs = c2d_fp_fast_block(nc, 4 * c->n_cu);
    /* before any order is known: every zone at once (one workgroup each) */
    const char* ge = getenv("C2D_FPF_GRID");
    int grid = ge ? atoi(ge) : (c->fpf_ordered ? c->n_cu : 0);
    if (grid <= 0) grid = (int)nc;
    c->last_fp_waves = bs / 64;
    /* no measured zone order yet: a cost probe first (every zone's first
     * implicit sub-step, one workgroup each), then the queue costliest first
     * by the 1/f_t_implicit it implies (C2D_FPF_PROBE=0: index order) */
    const char* pe = getenv("C2D_FPF_PROBE");
    rc = 0;
    if (!c->fpf_ordered && !ge && !(pe && pe[0] == '0')) {
      FpParams Pp = P;
      Pp.probe = 1;
      Pp.zorder = nullptr;
      HIPCHK(c, hipMemcpyAsync(c->fp_dP, &Pp, sizeof Pp, hipMemcpyHostToDevice, st));
      HIPCHK(c, hipMemsetAsync(c->fpf_zq, 0, sizeof(int32_t), st));
      rc = c2d_launch_fp_fast(c->fp_dP, nc, bs, nc, st);
      if (!rc) {
        std::vector<double> est((size_t)nc * FO_N);
        HIPCHK(c, hipMemcpyAsync(est.data(), c->fp_zout, est.size() * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(c, hipStreamSynchronize(st));
        std::vector<int32_t>& o = c->fpf_order;
        for (int q = 0; q < nc; q++) o[q] = q;
        auto cost = [&](int32_t z) {
          const double v = est[(size_t)z * FO_N + FO_DIAG + C2D_FP_STEPS];
          return (v == v) ? v : 0.0;
        };
        std::stable_sort(o.begin(), o.end(), [&](int32_t a, int32_t b) { return cost(a) > cost(b); });
        HIPCHK(c, hipMemcpyAsync(c->fpf_zq + 1, o.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, st));
        HIPCHK(c, hipMemsetAsync(c->fpf_zq, 0, sizeof(int32_t), st));
        HIPCHK(c, hipMemcpyAsync(c->fp_dP, &P, sizeof P, hipMemcpyHostToDevice, st));
        HIPCHK(c, hipStreamSynchronize(st));    /* the host vectors above go out of scope */
        grid = c->n_cu;
      }
    }
    if (!rc) rc = c2d_launch_fp_fast(c->fp_dP, nc, bs, grid, st);
  } else {
    c->last_fp_waves = c2d_fp_waves(nc, 4 * c->n_cu);
    rc = c2d_launch_fp(&P, nc, c->last_fp_waves, st);
  }
  if (rc) return fail(c, C2D_E_HIP, "fp launch: %s", hipGetErrorString((hipError_t)rc));
  HIPCHK(c, hipEventRecord(c->ev_g0b, st));
  if (el_dev) {   /* staging rows (seeded with the state: skipped zones too) */
    check_finite(c, c->fp_fout, (int64_t)nc * C2D_NUM_NT, FPERR_NF_OUT, c->fp_err, st);
    check_finite(c, c->fp_Pout, (int64_t)nc * C2D_NUM_NT, FPERR_NF_OUT, c->fp_err, st);
    HIPCHK(c, hipGetLastError());
  }
  std::vector<double> zout((size_t)nc * FO_N), fout(nnt), pout(nnt);
  std::vector<double> ecd(ecens_dev ? nc : 0);
  int32_t herr = 0;
  HIPCHK(c, hipMemcpyAsync(zout.data(), c->fp_zout, zout.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  if (!el_dev) {
    HIPCHK(c, hipMemcpyAsync(fout.data(), c->fp_fout, fout.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpyAsync(pout.data(), c->fp_Pout, pout.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  }
  HIPCHK(c, hipMemcpyAsync(&herr, c->fp_err, sizeof herr, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  (void)hipEventElapsedTime(&c->last_fp_ms, c->ev_g0a, c->ev_g0b);
  if (herr & FPERR_STEPS)
    return fail(c, C2D_E_FP, "FP sub-step limit exceeded (reference stops, update2d.f:585-599)");
  if (herr & FPERR_GUARD) return fail(c, C2D_E_FP, "FP temperature/McDonald iteration guard tripped");
  if (herr & FPERR_NF_IN)
    return fail(c, C2D_E_FP, "c2d_fp_step: NaN/Inf in the device n_field/ecens tallies or electron state");
  if (herr & FPERR_NF_OUT) return fail(c, C2D_E_FP, "c2d_fp_step: the update produced NaN/Inf in f_nt/Pnt");
  for (int cell = 0; cell < nc; cell++) {   /* skipped zones write Te only */
    const double* zo = &zout[(size_t)cell * FO_N];
    bool ok = std::isfinite(zo[FO_TE]);
    if (zo[FO_DIAG + C2D_FP_SKIPPED] == 0.0) {
      ok = ok && all_finite(zo, FO_PNTH + 1) && all_finite(zo + FO_DIAG, C2D_FP_NDIAG);
      if (!el_dev)
        ok = ok && all_finite(&fout[(size_t)cell * C2D_NUM_NT], C2D_NUM_NT) &&
             all_finite(&pout[(size_t)cell * C2D_NUM_NT], C2D_NUM_NT);
    }
    if (!ok) return fail(c, C2D_E_FP, "c2d_fp_step: the update of zone %d produced NaN/Inf", cell);
  }
  {   /* next fast update's queue order: most sub-steps first (either kernel counts them) */
    std::vector<int32_t>& o = c->fpf_order;
    std::stable_sort(o.begin(), o.end(), [&](int32_t a, int32_t b) {
      return zout[(size_t)a * FO_N + FO_DIAG + C2D_FP_STEPS] > zout[(size_t)b * FO_N + FO_DIAG + C2D_FP_STEPS];
    });
    c->fpf_ordered = true;
  }
  {   /* C2D_FP_AUTO: the slowest zone's sub-steps, for the next choice */
    double max_steps = 0.0;
    for (int cell = 0; cell < nc; cell++) {
      const double* zo = &zout[(size_t)cell * FO_N];
      if (zo[FO_DIAG + C2D_FP_SKIPPED] == 0.0) max_steps = std::max(max_steps, zo[FO_DIAG + C2D_FP_STEPS]);
    }
    c->fp_auto_known = true;
    c->fp_auto_exact = max_steps <= (double)C2D_FP_AUTO_STEPS;
    c->last_fp_mode = fm;
  }
  if (el_dev) {
    HIPCHK(c, hipMemcpyAsync(c->f_nt, c->fp_fout, nt_bytes, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(c->Pnt, c->fp_Pout, nt_bytes, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipStreamSynchronize(st));
  }
  /* scatter back in zone order; E_add_up sums, dT_max, tea (update2d.f:266-276) */
  double E_old = 0.0, E_new = 0.0, hr = 0.0, hr_st = 0.0;
  double dT_max = (in->ncycle <= 1) ? f.df_T : 0.0;   /* photon_fill, update2d.f:1912 */
  for (int j = 0; j < nz; j++)
    for (int k = 0; k < nr; k++) {
      const int cell = j * nr + k;
      const double* zo = &zout[(size_t)cell * FO_N];
      const double* dg = zo + FO_DIAG;
      double* p;
      if ((p = m2(out->Te_new, j, k))) *p = zo[FO_TE];
      if (dg[C2D_FP_SKIPPED] == 0.0) {
        for (int i = 0; i < C2D_NUM_NT && !el_dev; i++) {
          out->f_nt.data[i * out->f_nt.s_i + j * out->f_nt.s_j + k * out->f_nt.s_k] =
              fout[(size_t)cell * C2D_NUM_NT + i];
          out->Pnt.data[i * out->Pnt.s_i + j * out->Pnt.s_j + k * out->Pnt.s_k] =
              pout[(size_t)cell * C2D_NUM_NT + i];
        }
        if ((p = m2(out->n_e, j, k))) *p = zo[FO_NE];
        if ((p = m2(out->gmin, j, k))) *p = zo[FO_GMIN];
        if ((p = m2(out->gmax, j, k))) *p = zo[FO_GMAX];
        if ((p = m2(out->amxwl, j, k))) *p = zo[FO_AMXWL];
        if ((p = m2(out->p_nth, j, k))) *p = zo[FO_PNTH];
        E_old = E_old + dg[C2D_FP_E_OLD];
        E_new = E_new + dg[C2D_FP_E_NEW];
        hr = hr + dg[C2D_FP_HR];
        hr_st = hr_st + dg[C2D_FP_HR_ST];
        if (dg[C2D_FP_DELTA_T] > dT_max) dT_max = dg[C2D_FP_DELTA_T];
      }
      if ((p = m2(out->tea, j, k)) && a2(in->tna, j, k, 0.0) > 1.) {
        double t = zo[FO_TE];
        t = (1.0e3 < t) ? 1.0e3 : t;
        t = (5.0 > t) ? 5.0 : t;
        *p = t;
      }
      if (out->zone_diag)
        memcpy(out->zone_diag + (size_t)cell * C2D_FP_NDIAG, dg, sizeof(double) * C2D_FP_NDIAG);
    }
  out->E_tot_old = E_old;
  out->E_tot_new = E_new;
  out->hr_total = hr;
  out->hr_st_total = hr_st;
  out->dT_max = dT_max;
  return C2D_OK;
}

extern "C" int c2d_electron_state(c2d_ctx* c, c2d_marray3 f_nt, c2d_marray3 Pnt) {
  if (!c) return C2D_E_ARG;
  if (!c->have_electrons) return fail(c, C2D_E_STATE, "c2d_electron_state: no electron state yet");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const size_t nnt = (size_t)c->ncell * C2D_NUM_NT;
  std::vector<double> h(nnt);
  const c2d_marray3* views[2] = {&f_nt, &Pnt};
  const double* src[2] = {c->f_nt, c->Pnt};
  for (int v = 0; v < 2; v++) {
    const c2d_marray3& m = *views[v];
    if (!m.data) continue;
    HIPCHK(c, hipMemcpy(h.data(), src[v], nnt * sizeof(double), hipMemcpyDeviceToHost));
    for (int j = 0; j < c->nz; j++)
      for (int k = 0; k < c->nr; k++)
        for (int i = 0; i < C2D_NUM_NT; i++)
          m.data[i * m.s_i + j * m.s_j + k * m.s_k] = h[((size_t)j * c->nr + k) * C2D_NUM_NT + i];
  }
  return C2D_OK;
}

extern "C" int c2d_last_fp_ms(c2d_ctx* c, double* ms) {
  if (!c || !ms) return C2D_E_ARG;
  *ms = c->last_fp_ms;
  return C2D_OK;
}

/* ------------------------------------------------------------------ */
/* emission / absorption tables (imcgen2d.f:209-333, volume_em)         */
/* ------------------------------------------------------------------ */
extern "C" int c2d_volume_em(c2d_ctx* c, const c2d_vem_in* in, c2d_vem_out* out) {
  if (!c || !in || !out) return C2D_E_ARG;
  if (!in->tea.data || !in->tna.data || !in->n_e.data || !in->B_field.data || !in->f_pair.data ||
      !in->zsurf.data || !in->vol.data)
    return fail(c, C2D_E_ARG, "c2d_volume_em: missing input array");
  const bool el_dev = !in->f_nt.data;
  if (el_dev && !c->have_electrons)
    return fail(c, C2D_E_STATE, "c2d_volume_em: f_nt NULL but no electron state on the device");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const int nz = c->nz, nr = c->nr;
  const size_t nc = (size_t)c->ncell;
  if (!c->vem_zin) {
    HIPCHK(c, dalloc(&c->vem_zin, nc * VZ_N));
    HIPCHK(c, dalloc(&c->vem_fnt, nc * C2D_NUM_NT));
    HIPCHK(c, dalloc(&c->vem_eph, (size_t)C2D_N_VOL));
    HIPCHK(c, dalloc(&c->vem_kap, nc * C2D_N_VOL));
    HIPCHK(c, dalloc(&c->vem_et, nc * C2D_N_VOL));
    HIPCHK(c, dalloc(&c->vem_eh, nc * C2D_N_VOL));
    HIPCHK(c, dalloc(&c->vem_zout, nc * VO_N));
  }
  if (int rc = ensure_mcd(c)) return rc;
  /* the photon grid volume_em writes into E_ph (volume2d.f:98,106-107) */
  const double dE = c2d_exp(c2d_log(1.0e20) / (double)C2D_N_VOL);
  std::vector<double> eph(C2D_N_VOL);
  double E = 1.0e-10 / dE;
  for (int i = 0; i < C2D_N_VOL; i++) {
    E = E * dE;
    eph[i] = E;
  }
  std::vector<double> zin(nc * VZ_N, 0.0), fnt(nc * C2D_NUM_NT);
  for (int j = 0; j < nz; j++)
    for (int k = 0; k < nr; k++) {
      const size_t cell = (size_t)j * nr + k;
      double* z = &zin[cell * VZ_N];
      z[VZ_TEA] = at2(in->tea, j, k);
      z[VZ_TNA] = at2(in->tna, j, k);
      z[VZ_NE] = at2(in->n_e, j, k);
      z[VZ_B] = at2(in->B_field, j, k);
      z[VZ_FPAIR] = at2(in->f_pair, j, k);
      if (c->cfg.pair_switch == 1 && !(z[VZ_FPAIR] < 1.0e-10))  /* volume2d.f:322 */
        return fail(c, C2D_E_ARG,
                    "volume_em: pair annihilation (pair_switch=1, f_pair=%g in zone (%d,%d)) needs "
                    "a positron population; positrons are inert here (H6)", z[VZ_FPAIR], j + 1, k + 1);
      z[VZ_ZSURF] = at2(in->zsurf, j, k);
      z[VZ_VOL] = at2(in->vol, j, k);
      z[VZ_EP] = in->ep_switch.data ? (double)in->ep_switch.data[j * in->ep_switch.s_j + k * in->ep_switch.s_k] : 0.0;
      /* l_min (imcgen2d.f:238-246) */
      const double dz = (j == 0) ? c->cfg.z[0] : c->cfg.z[j] - c->cfg.z[j - 1];
      const double drr = (k == 0) ? c->cfg.r[0] - c->cfg.rmin : c->cfg.r[k] - c->cfg.r[k - 1];
      z[VZ_LMIN] = (dz < drr) ? dz : drr;
      for (int i = 0; i < C2D_NUM_NT && !el_dev; i++)
        fnt[cell * C2D_NUM_NT + i] = in->f_nt.data[i * in->f_nt.s_i + j * in->f_nt.s_j + k * in->f_nt.s_k];
    }
  if (!all_finite(zin.data(), zin.size()) || !all_finite(fnt.data(), el_dev ? 0 : fnt.size()))
    return fail(c, C2D_E_NONFINITE, "c2d_volume_em: NaN/Inf in the zone inputs or f_nt");
  c->have_vem = false;
  const hipStream_t st = c->stream;
  HIPCHK(c, hipMemcpyAsync(c->vem_zin, zin.data(), zin.size() * sizeof(double), hipMemcpyHostToDevice, st));
  if (!el_dev)
    HIPCHK(c, hipMemcpyAsync(c->vem_fnt, fnt.data(), fnt.size() * sizeof(double), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->vem_eph, eph.data(), eph.size() * sizeof(double), hipMemcpyHostToDevice, st));
  VemParams P;
  P.zin = c->vem_zin; P.f_nt = el_dev ? c->f_nt : c->vem_fnt; P.gnt = c->gnt; P.E_ph = c->vem_eph; P.mcd = c->fp_mcd;
  P.dE = dE; P.pow3_15 = c2d_pow(3.0, 1.5); P.dt = in->dt;
  P.kappa = c->vem_kap; P.eps_tot = c->vem_et; P.eps_th = c->vem_eh; P.zout = c->vem_zout;
  HIPCHK(c, hipEventRecord(c->ev_g0a, st));
  int rc = c2d_launch_vem(&P, (int)nc, st);
  if (rc) return fail(c, C2D_E_HIP, "vem launch: %s", hipGetErrorString((hipError_t)rc));
  HIPCHK(c, hipEventRecord(c->ev_g0b, st));
  /* NaN/Inf in the device electron state read, or in the tables written */
  if (!c->mono_flag) HIPCHK(c, dalloc(&c->mono_flag, 1));
  HIPCHK(c, hipMemsetAsync(c->mono_flag, 0, sizeof(int32_t), st));
  if (el_dev) check_finite(c, c->f_nt, (int64_t)nc * C2D_NUM_NT, 1, c->mono_flag, st);
  check_finite(c, c->vem_kap, (int64_t)nc * C2D_N_VOL, 2, c->mono_flag, st);
  check_finite(c, c->vem_et, (int64_t)nc * C2D_N_VOL, 2, c->mono_flag, st);
  check_finite(c, c->vem_eh, (int64_t)nc * C2D_N_VOL, 2, c->mono_flag, st);
  HIPCHK(c, hipGetLastError());
  int32_t vflag = 0;
  HIPCHK(c, hipMemcpyAsync(&vflag, c->mono_flag, sizeof vflag, hipMemcpyDeviceToHost, st));
  /* tables cross to the host only for the output views that are present */
  std::vector<double> kap(out->kappa_tot.data ? nc * C2D_N_VOL : 0),
      et(out->eps_tot.data ? nc * C2D_N_VOL : 0), eh(out->eps_th.data ? nc * C2D_N_VOL : 0), zo(nc * VO_N);
  if (!kap.empty())
    HIPCHK(c, hipMemcpyAsync(kap.data(), c->vem_kap, kap.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  if (!et.empty())
    HIPCHK(c, hipMemcpyAsync(et.data(), c->vem_et, et.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  if (!eh.empty())
    HIPCHK(c, hipMemcpyAsync(eh.data(), c->vem_eh, eh.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(zo.data(), c->vem_zout, zo.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  (void)hipEventElapsedTime(&c->last_vem_ms, c->ev_g0a, c->ev_g0b);
  if (vflag & 1) return fail(c, C2D_E_NONFINITE, "c2d_volume_em: NaN/Inf in the device f_nt");
  bool zo_ok = true;
  for (size_t cell = 0; cell < nc; cell++) zo_ok = zo_ok && all_finite(&zo[cell * VO_N], VO_ETOT + 1);
  if ((vflag & 2) || !zo_ok)
    return fail(c, C2D_E_NONFINITE, "c2d_volume_em: NaN/Inf in the emission/absorption tables or "
                "Eloss outputs (volume2d.f:343-390)");
  c->have_vem = true;
  if (out->E_ph) std::copy(eph.begin(), eph.end(), out->E_ph);
  auto put3 = [&](c2d_marray3& m, const std::vector<double>& v, size_t cell, int j, int k) {
    if (!m.data) return;
    for (int i = 0; i < C2D_N_VOL; i++)
      m.data[i * m.s_i + j * m.s_j + k * m.s_k] = v[cell * C2D_N_VOL + i];
  };
  auto put2 = [&](c2d_marray2& m, int j, int k, double v) {
    if (m.data) m.data[j * m.s_j + k * m.s_k] = v;
  };
  for (int j = 0; j < nz; j++)
    for (int k = 0; k < nr; k++) {
      const size_t cell = (size_t)j * nr + k;
      put3(out->kappa_tot, kap, cell, j, k);
      put3(out->eps_tot, et, cell, j, k);
      put3(out->eps_th, eh, cell, j, k);
      const double* o = &zo[cell * VO_N];
      put2(out->B_field, j, k, o[VO_B]);
      put2(out->Eloss_sy, j, k, o[VO_ESY]);
      put2(out->Eloss_cy, j, k, o[VO_ECY]);
      put2(out->Eloss_th, j, k, o[VO_ETH]);
      put2(out->Eloss_tot, j, k, o[VO_ETOT]);
    }
  return C2D_OK;
}

extern "C" int c2d_last_vem_ms(c2d_ctx* c, double* ms) {
  if (!c || !ms) return C2D_E_ARG;
  *ms = c->last_vem_ms;
  return C2D_OK;
}

/* ------------------------------------------------------------------ */
/* observer-frame binning (postprocessing/pspt.c, plcm.c)               */
/* ------------------------------------------------------------------ */
static int obs_settle(c2d_ctx* c);

extern "C" int c2d_obs_begin(c2d_ctx* c, const c2d_obs_bins* b) {
  if (!c || !b) return C2D_E_ARG;
  if ((b->mode != C2D_OBS_SED && b->mode != C2D_OBS_LC) || b->n_t < 1 || b->n_t > C2D_OBS_MAX_T ||
      b->n_mu < 1 || b->n_mu > C2D_OBS_MAX_MU || b->n_e < 1 || b->n_e > C2D_OBS_MAX_E ||
      !b->t0 || !b->t1 || !b->mu0 || !b->mu1 || !b->E0 || !b->E1 || !(b->gam_bulk >= 1.0))
    return fail(c, C2D_E_ARG, "c2d_obs_begin: bad binning");
  if (b->mode == C2D_OBS_SED && b->n_mu != 1)
    return fail(c, C2D_E_ARG, "c2d_obs_begin: the SED mode has one angular window");
  /* a new binning ends any pspt deck: c2d_obs_begin_pspt sets it again */
  c->pspt_on = false;
  c->obs_ready = false;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  { const int rc = obs_settle(c); if (rc) return rc; }   /* the histogram is about to go */
  if (c->obs_edges) (void)hipFree(c->obs_edges);
  if (c->obs_hist) (void)hipFree(c->obs_hist);
  c->obs_edges = c->obs_hist = nullptr;
  const int ne = 2 * (b->n_t + b->n_mu + b->n_e);
  std::vector<double> h;
  h.reserve(ne);
  h.insert(h.end(), b->t0, b->t0 + b->n_t);
  h.insert(h.end(), b->t1, b->t1 + b->n_t);
  h.insert(h.end(), b->mu0, b->mu0 + b->n_mu);
  h.insert(h.end(), b->mu1, b->mu1 + b->n_mu);
  h.insert(h.end(), b->E0, b->E0 + b->n_e);
  h.insert(h.end(), b->E1, b->E1 + b->n_e);
  HIPCHK(c, dalloc(&c->obs_edges, (size_t)ne));
  HIPCHK(c, hipMemcpy(c->obs_edges, h.data(), ne * sizeof(double), hipMemcpyHostToDevice));
  const size_t nh = (size_t)b->n_t * b->n_mu * b->n_e;
  HIPCHK(c, dalloc(&c->obs_hist, 3 * nh));
  HIPCHK(c, hipMemset(c->obs_hist, 0, 3 * nh * sizeof(double)));
  ObsDev& O = c->obs;
  O.gam_bulk = b->gam_bulk; O.rmax = b->rmax; O.t_offset = b->t_offset;
  O.mode = b->mode; O.n_t = b->n_t; O.n_mu = b->n_mu; O.n_e = b->n_e;
  O.t0 = c->obs_edges; O.t1 = O.t0 + b->n_t; O.mu0 = O.t1 + b->n_t; O.mu1 = O.mu0 + b->n_mu;
  O.E0 = O.mu1 + b->n_mu; O.E1 = O.E0 + b->n_e;
  O.F = c->obs_hist; O.F2 = O.F + nh; O.cnt = O.F2 + nh;
  /* privatise in LDS when the three histograms fit next to the edges */
  /* privatise as many leading time rows in LDS as fit (all of them for the
   * usual SED); later rows go to wave-aggregated global atomics */
  {
    const size_t edges = c2d_obs_lds_bytes(b->n_t, b->n_mu, b->n_e, 0);
    const size_t row = c2d_obs_lds_bytes(0, b->n_mu, b->n_e, 1) - c2d_obs_lds_bytes(0, b->n_mu, b->n_e, 0);
    /* 1 KiB for the kernel's static segment table (observe.hip ObsSegs) */
    const size_t avail = c->lds_max > edges + 1024 ? c->lds_max - edges - 1024 : 0;
    O.lds_rows = (int)std::min<size_t>((size_t)b->n_t, avail / row);
    const size_t bytes = c2d_obs_lds_bytes(b->n_t, b->n_mu, b->n_e, O.lds_rows);
    /* workgroups per CU that fit the CU's 160 KiB of LDS, at most 4 */
    c->obs_wg_per_cu = (int)std::max<size_t>(1, std::min<size_t>(4, (160 * 1024) / (bytes + 1024)));
  }
  auto sorted = [](const double* lo, const double* hi, int n) {
    for (int i = 1; i < n; i++)
      if (!(lo[i] >= lo[i - 1]) || !(hi[i] >= hi[i - 1])) return 0;
    return 1;
  };
  O.sorted_t = sorted(b->t0, b->t1, b->n_t);
  O.sorted_mu = sorted(b->mu0, b->mu1, b->n_mu);
  O.sorted_e = sorted(b->E0, b->E1, b->n_e);
  c->obs_ms = 0.0;
  c->obs_ready = true;
  return C2D_OK;
}

/* Wait for an asynchronous binning of the context's own events (obs_stream)
 * and add its kernel time. */
static int obs_settle(c2d_ctx* c) {
  if (!c->obs_inflight) return C2D_OK;
  c->obs_inflight = false;
  HIPCHK(c, hipEventSynchronize(c->ev_obs_b));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ev_obs_a, c->ev_obs_b);
  c->obs_ms += ms;
  return C2D_OK;
}

/* Bin `nseg` event segments (device pointer, count) back to back on the
 * context's stream; one event pair and one synchronisation around them all. */
static int obs_launch_segments(c2d_ctx* c, const double* const* ev, const int64_t* m, int nseg) {
  int64_t tot = 0;
  for (int s = 0; s < nseg; s++) tot += m[s];
  if (tot == 0) return C2D_OK;
  /* enough blocks to fill the chip, each privatising its own histogram */
  const int64_t bs = c2d_obs_block();
  HIPCHK(c, hipEventRecord(c->ev_g0a, c->stream));
  {   /* every segment in one launch */
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->n_cu * c->obs_wg_per_cu, (tot + bs - 1) / bs));
    int rc = c2d_launch_obs_segs(&c->obs, ev, m, nseg, grid, c->stream);
    if (rc) return fail(c, C2D_E_HIP, "obs launch: %s", hipGetErrorString((hipError_t)rc));
  }
  HIPCHK(c, hipEventRecord(c->ev_g0b, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ev_g0a, c->ev_g0b);
  c->obs_ms += ms;
  return C2D_OK;
}

static int obs_launch(c2d_ctx* c, const double* ev, int64_t m) {
  return obs_launch_segments(c, &ev, &m, 1);
}

extern "C" int c2d_obs_accumulate(c2d_ctx* c, const double* events, int64_t n) {
  if (!c) return C2D_E_ARG;
  if (!c->obs_ready) return fail(c, C2D_E_STATE, "c2d_obs_begin must precede c2d_obs_accumulate");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  { const int rc = obs_settle(c); if (rc) return rc; }
  if (!events) {
    const double* seg[C2D_EV_SHARDS];
    int64_t cnt[C2D_EV_SHARDS];
    int64_t tot = 0;
    for (int sh = 0; sh < C2D_EV_SHARDS; sh++) {
      seg[sh] = c->ev + (size_t)sh * c->ev_cap_sh * C2D_EVENT_WORDS;
      cnt[sh] = c->ev_cnt[sh];
      tot += cnt[sh];
    }
    const char* e = getenv("C2D_OBS_ASYNC");
    if ((e && e[0] == '0') || tot == 0) return obs_launch_segments(c, seg, cnt, C2D_EV_SHARDS);
    /* on obs_stream, after the step that wrote the events; the next
     * generation-0 launch waits for it (run_step_body) */
    HIPCHK(c, hipEventRecord(c->ev_obs_src, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->obs_stream, c->ev_obs_src, 0));
    const int64_t bs = c2d_obs_block();
    HIPCHK(c, hipEventRecord(c->ev_obs_a, c->obs_stream));
    /* one launch per shard: between the short launches the FP update's
     * workgroups (69 KB of LDS each) find room beside them (binning all
     * shards in one launch beside the FP slowed it 1.26 -> 2.3-2.8 ms,
     * at one or two workgroups per CU) */
    for (int s = 0; s < C2D_EV_SHARDS; s++) {
      if (cnt[s] == 0) continue;
      const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)c->n_cu * c->obs_wg_per_cu, (cnt[s] + bs - 1) / bs));
      int rc = c2d_launch_obs(&c->obs, seg[s], cnt[s], grid, c->obs_stream);
      if (rc) return fail(c, C2D_E_HIP, "obs launch: %s", hipGetErrorString((hipError_t)rc));
    }
    HIPCHK(c, hipEventRecord(c->ev_obs_b, c->obs_stream));
    c->obs_inflight = true;
    return C2D_OK;
  }
  if (n < 0) return C2D_E_ARG;
  if (n > c->obs_ev_cap) {
    if (c->obs_ev) (void)hipFree(c->obs_ev);
    c->obs_ev = nullptr;
    HIPCHK(c, dalloc(&c->obs_ev, (size_t)n * C2D_EVENT_WORDS));
    c->obs_ev_cap = n;
  }
  if (n) HIPCHK(c, hipMemcpy(c->obs_ev, events, (size_t)n * C2D_EVENT_WORDS * sizeof(double),
                             hipMemcpyHostToDevice));
  return obs_launch(c, c->obs_ev, n);
}

extern "C" int c2d_obs_accumulate_device(c2d_ctx* c, const double* d_events, int64_t n) {
  if (!c || !d_events || n < 0) return C2D_E_ARG;
  if (!c->obs_ready) return fail(c, C2D_E_STATE, "c2d_obs_begin must precede c2d_obs_accumulate_device");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  { const int rc = obs_settle(c); if (rc) return rc; }
  return obs_launch(c, d_events, n);
}

extern "C" int c2d_obs_result(c2d_ctx* c, double* F, double* F2, double* count, double* kernel_ms) {
  if (!c) return C2D_E_ARG;
  if (!c->obs_ready) return fail(c, C2D_E_STATE, "c2d_obs_begin must precede c2d_obs_result");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  { const int rc = obs_settle(c); if (rc) return rc; }
  const size_t nh = (size_t)c->obs.n_t * c->obs.n_mu * c->obs.n_e;
  if (F) HIPCHK(c, hipMemcpy(F, c->obs.F, nh * sizeof(double), hipMemcpyDeviceToHost));
  if (F2) HIPCHK(c, hipMemcpy(F2, c->obs.F2, nh * sizeof(double), hipMemcpyDeviceToHost));
  if (count) HIPCHK(c, hipMemcpy(count, c->obs.cnt, nh * sizeof(double), hipMemcpyDeviceToHost));
  if (kernel_ms) *kernel_ms = c->obs_ms;
  return C2D_OK;
}

/* pspt's dialogue -> the SED binning (postprocessing/pspt.c:105-205) */
extern "C" int c2d_obs_begin_pspt(c2d_ctx* c, const char* deck) {
  if (!c) return C2D_E_ARG;
  c2d_pspt_deck d;
  if (c2d_pspt_parse(deck ? deck : "", &d))
    return fail(c, C2D_E_ARG, "c2d_obs_begin_pspt: the deck's grid has no bins or more than %d energy channels",
                C2D_PSPT_CHMAX);
  c2d_obs_bins b;
  b.mode = C2D_OBS_SED; b.gam_bulk = d.gam_bulk; b.rmax = d.rmax; b.t_offset = 0.0;
  b.n_t = d.n_t; b.t0 = d.t0; b.t1 = d.t1;
  b.n_mu = 1; b.mu0 = &d.mu0; b.mu1 = &d.mu1;
  b.n_e = d.n_e; b.E0 = d.E0; b.E1 = d.E1;
  const int rc = c2d_obs_begin(c, &b);
  if (rc != C2D_OK) return rc;
  /* the world_sum reduction buffer lives as long as the deck, so a rank can
   * no longer fail an allocation and skip the collective the others enter */
  if (c->pspt_red) (void)hipFree(c->pspt_red);
  c->pspt_red = nullptr;
  HIPCHK(c, dalloc(&c->pspt_red, 2 * (size_t)d.n_t * d.n_e));
  c->pspt = d;
  c->pspt_on = true;
  return C2D_OK;
}

/* pspt's output file from the histogram so far (postprocessing/pspt.c:323-353);
 * world_sum: summed over the context's communicator first (every rank calls,
 * rank 0 writes) */
extern "C" int c2d_obs_write_pspt(c2d_ctx* c, const char* path, int32_t factor, int32_t world_sum) {
  if (!c) return C2D_E_ARG;
  if (!c->pspt_on || !c->obs_ready) return fail(c, C2D_E_STATE, "c2d_obs_write_pspt: c2d_obs_begin_pspt first");
  { const int rc = obs_settle(c); if (rc) return rc; }
  if (c->obs.mode != C2D_OBS_SED || c->obs.n_mu != 1 || c->obs.n_t != c->pspt.n_t || c->obs.n_e != c->pspt.n_e ||
      !c->pspt_red)
    return fail(c, C2D_E_STATE, "c2d_obs_write_pspt: the binning is not the pspt deck's");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const size_t nh = (size_t)c->obs.n_t * c->obs.n_mu * c->obs.n_e;
  std::vector<double> F(nh), cnt(nh);
  if (world_sum) {
    if (!c->comm) return fail(c, C2D_E_STATE, "c2d_obs_write_pspt: world_sum needs c2d_comm_init");
    double* w = c->pspt_red;
    HIPCHK(c, hipMemcpyAsync(w, c->obs.F, nh * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(w + nh, c->obs.cnt, nh * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    const ncclResult_t r = ncclAllReduce(w, w, 2 * nh, ncclDouble, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return fail(c, C2D_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    HIPCHK(c, hipMemcpyAsync(F.data(), w, nh * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(cnt.data(), w + nh, nh * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->comm_rank != 0) return C2D_OK;
  } else {
    const int rc = c2d_obs_result(c, F.data(), nullptr, cnt.data(), nullptr);
    if (rc != C2D_OK) return rc;
  }
  const char* out = (path && path[0]) ? path : c->pspt.outfile;
  if (c2d_pspt_write(out, &c->pspt, F.data(), cnt.data(), factor))
    return fail(c, C2D_E_IO, "c2d_obs_write_pspt: cannot write '%s'", out);
  return C2D_OK;
}

/* ------------------------------------------------------------------ */
/* RCCL tally all-reduce (xec_add/graphics_collect, src/xec2d.f:325-399; */
/* cens_add_up/E_add_up, src/update2d.f:1929-2078)                      */
/* ------------------------------------------------------------------ */
static_assert(sizeof(ncclUniqueId) == C2D_COMM_ID_BYTES, "RCCL unique id size");

extern "C" int c2d_device_count(int32_t* n) {
  if (!n) return C2D_E_ARG;
  int d = 0;
  *n = 0;
  if (hipGetDeviceCount(&d) != hipSuccess) return C2D_E_HIP;
  *n = d;
  return C2D_OK;
}

extern "C" int c2d_comm_unique_id(void* id, int64_t cap) {
  if (!id || cap < C2D_COMM_ID_BYTES) return C2D_E_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return C2D_E_RCCL;
  memcpy(id, &u, sizeof u);
  return C2D_OK;
}

extern "C" int c2d_comm_init(c2d_ctx* c, const void* id, int32_t rank, int32_t world) {
  if (!c || !id || world < 1 || rank < 0 || rank >= world) return C2D_E_ARG;
  if (c->comm) return fail(c, C2D_E_STATE, "c2d_comm_init: the context already has a communicator");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&comm, world, u, rank);
  if (r != ncclSuccess)
    return fail(c, C2D_E_RCCL, "ncclCommInitRank(rank %d of %d): %s", rank, world, ncclGetErrorString(r));
  c->comm = comm;
  c->comm_rank = rank;
  c->comm_world = world;
  return C2D_OK;
}

extern "C" int c2d_allreduce_tallies(c2d_ctx* c) {
  if (!c) return C2D_E_ARG;
  if (!c->comm) return fail(c, C2D_E_STATE, "c2d_allreduce_tallies: c2d_comm_init first");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const ncclResult_t r = ncclAllReduce(c->T, c->T, (size_t)c->L.total, ncclDouble, ncclSum, c->comm,
                                       c->stream);
  if (r != ncclSuccess) return fail(c, C2D_E_RCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return C2D_OK;
}
