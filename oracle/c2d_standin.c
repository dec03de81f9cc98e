/*
 * c2d_standin.c — TEST INFRASTRUCTURE ONLY (this container).
 *
 * A stand-in for compton2d_amd/libcompton2d.so that implements the C-ABI
 * entry points the drop-in Fortran shim (examples/c2d_shim.f) calls, by
 * delegating to the C oracle (oracle/c2d_oracle.c, c2d_fp_oracle.c) in its
 * reference mode: the reference's lagged-Fibonacci zone streams with its
 * reseeding points, per-copy split1 probes, the stale t_bound of hazard H4
 * and glibc libm -- bit for bit the reference's worker routines
 * (tests/test_oracle_golden.py).  With it, oracle/ref/build_shim.sh links
 * the reference's OWN main program + the shim into an executable that
 * runs on a machine without a GPU, so tests/test_fortran_shim.py can run
 * the reference's time loop through the shim and compare what it writes
 * with the unmodified reference on the same deck.
 *
 * Built only by oracle/ref/build_shim.sh into oracle/_ref/standin/ (never
 * linked into the product, never shipped to the GPU box).
 *
 * The multi-worker tally exchange (c2d_comm_*) is emulated for the shim's
 * N-worker mode: every worker context of one process group registers its
 * tally buffer in a shared file under C2D_STANDIN_COMM_DIR, and
 * c2d_allreduce_tallies sums them in rank order (a file-based stand-in for
 * RCCL; the product uses ncclAllReduce, compton2d_amd/csrc/capi.cpp).
 *
 * Environment: C2D_STANDIN_RNG = fib (default) | lineage,
 * C2D_STANDIN_RAND_SWITCH (default 1), C2D_STANDIN_H4 (default 1: stale
 * t_bound), C2D_STANDIN_DT_LAG (default 1: the MPI workers' previous-step
 * dt for census and volume packets, hazard H11), C2D_STANDIN_GRID_LAG
 * (default 1: bins 0 for the first step's census and volume packets, hazard
 * H12), C2D_STANDIN_RSEED (the
 * deck's rseed: the oracle replays the master's seed_zone chain from it).
 */
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../include/compton2d.h"
#include "../compton2d_amd/csrc/pspt_host.h"   /* the product's pspt dialogue/file code */

typedef struct c2o_ctx c2o_ctx;
c2o_ctx* c2o_create(const c2d_config* cfg, int rng_mode, int rand_switch, int32_t rseed, int h4_stale);
void c2o_destroy(c2o_ctx* c);
int c2o_step(c2o_ctx* c, const c2d_step_in* in);
const double* c2o_tallies(c2o_ctx* c, int64_t* n);
int64_t c2o_event_count(c2o_ctx* c);
int64_t c2o_events(c2o_ctx* c, double* out, int64_t cap);
int64_t c2o_census_count(c2o_ctx* c);
int64_t c2o_census_export(c2o_ctx* c, double* d6, int32_t* i5, uint64_t* keys, int64_t cap);
int c2o_census_import(c2o_ctx* c, const double* d6, const int32_t* i5, const uint64_t* keys, int64_t n);
void c2o_set_dt_lag(c2o_ctx* c, int on);
void c2o_set_grid_lag(c2o_ctx* c, int on);
int c2o_fp_step(const c2d_config* g, const c2d_fp_config* fc, const c2d_fp_step_in* in,
                c2d_fp_step_out* out);
int c2o_obs_bin(const c2d_obs_bins* b, const double* ev, int64_t n, double* F, double* F2, double* cnt);

enum { RNG_FIB = 1, RNG_LINEAGE = 3 };

struct c2d_ctx {
  c2o_ctx* o;
  c2d_config cfg;
  c2d_tally_layout L;
  c2d_fp_config fc;
  double* fic;
  int fp_ready;
  double* T;            /* this context's tally buffer (the last step's, then all-reduced) */
  int comm_rank, comm_world;
  char comm_id[C2D_COMM_ID_BYTES];
  int64_t comm_round;
  int64_t obs_round;
  c2d_pspt_deck pspt;   /* c2d_obs_begin_pspt */
  int pspt_on;
  double *oF, *oF2, *ocnt;
  char err[512];
};

static int fail(c2d_ctx* c, int rc, const char* fmt, ...) {
  if (c) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(c->err, sizeof c->err, fmt, ap);
    va_end(ap);
  }
  return rc;
}

static long envl(const char* name, long dflt) {
  const char* e = getenv(name);
  return e && *e ? strtol(e, NULL, 10) : dflt;
}

const char* c2d_version(void) { return "c2d_standin (C oracle, reference mode; test infrastructure)"; }

int c2d_device_count(int32_t* n) {
  if (!n) return C2D_E_ARG;
  *n = 1;
  return C2D_OK;
}

int c2d_init(const c2d_config* cfg, c2d_ctx** out) {
  if (!cfg || !out) return C2D_E_ARG;
  c2d_ctx* c = (c2d_ctx*)calloc(1, sizeof *c);
  if (!c) return C2D_E_NOMEM;
  *out = c;
  const char* rng = getenv("C2D_STANDIN_RNG");
  const int mode = (rng && strcmp(rng, "lineage") == 0) ? RNG_LINEAGE : RNG_FIB;
  c->cfg = *cfg;
  /* the oracle's fib mode replays the master's seed_zone chain from the
   * run's input rseed (the shim's seed is the master's rseed after the first
   * imcgen2d): C2D_STANDIN_RSEED gives the deck's value */
  const int32_t rs = (int32_t)envl("C2D_STANDIN_RSEED", (long)cfg->seed);
  c->o = c2o_create(cfg, mode, (int)envl("C2D_STANDIN_RAND_SWITCH", 1), rs,
                    (int)envl("C2D_STANDIN_H4", 1));
  if (!c->o) return fail(c, C2D_E_ARG, "c2d_standin: c2o_create rejected the configuration");
  /* hazard H11: the reference's MPI workers transport census and volume
   * packets with the dt of the previous z_surf_bcast (0 in the first step) */
  c2o_set_dt_lag(c->o, (int)envl("C2D_STANDIN_DT_LAG", 1));
  /* hazard H12: the workers' spectral / light-curve grids are unset during
   * the first step's census and volume jobs, so those packets carry bins 0
   * and their escapes never reach fout / edout */
  c2o_set_grid_lag(c->o, (int)envl("C2D_STANDIN_GRID_LAG", 1));
  c2d_tally_layout_for(cfg->nz, cfg->nr, cfg->nmu, &c->L);
  c->T = (double*)calloc((size_t)c->L.total, sizeof(double));
  if (!c->T) return fail(c, C2D_E_NOMEM, "c2d_standin: tally buffer");
  return C2D_OK;
}

void c2d_finalize(c2d_ctx* c) {
  if (!c) return;
  if (c->o) c2o_destroy(c->o);
  free(c->oF);
  free(c->oF2);
  free(c->ocnt);
  free(c->fic);
  free(c->T);
  free(c);
}

const char* c2d_last_error(c2d_ctx* c) { return c ? c->err : "c2d_standin: no context"; }

int c2d_tally_layout_get(c2d_ctx* c, c2d_tally_layout* L) {
  if (!c || !L) return C2D_E_ARG;
  *L = c->L;
  return C2D_OK;
}

int c2d_transport_step(c2d_ctx* c, const c2d_step_in* in) {
  if (!c || !in) return C2D_E_ARG;
  const int rc = c2o_step(c->o, in);
  if (rc) return fail(c, rc, "c2d_standin: oracle step failed (%d)", rc);
  int64_t n = 0;
  const double* t = c2o_tallies(c->o, &n);
  memcpy(c->T, t, sizeof(double) * (size_t)n);
  return C2D_OK;
}

int c2d_tally_download(c2d_ctx* c, double* host, int64_t n) {
  if (!c || !host || n < c->L.total) return C2D_E_ARG;
  memcpy(host, c->T, sizeof(double) * (size_t)c->L.total);
  return C2D_OK;
}

int c2d_events(c2d_ctx* c, double* buf, int64_t cap, int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  *n = c2o_event_count(c->o);
  if (buf && cap > 0) c2o_events(c->o, buf, cap);
  return C2D_OK;
}

int c2d_census_count(c2d_ctx* c, int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  *n = c2o_census_count(c->o);
  return C2D_OK;
}

int c2d_census_export(c2d_ctx* c, double* d6, int32_t* i5, uint64_t* keys, int64_t cap, int64_t* n) {
  if (!c || !n) return C2D_E_ARG;
  *n = c2o_census_count(c->o);
  if (cap > 0) c2o_census_export(c->o, d6, i5, keys, cap);
  return C2D_OK;
}

int c2d_census_import(c2d_ctx* c, const double* d6, const int32_t* i5, const uint64_t* keys, int64_t n) {
  if (!c || n < 0) return C2D_E_ARG;
  const int rc = c2o_census_import(c->o, d6, i5, keys, n);
  return rc ? fail(c, rc, "c2d_standin: census import of %lld records", (long long)n) : C2D_OK;
}

int c2d_fp_set_config(c2d_ctx* c, const c2d_fp_config* fc) {
  if (!c || !fc || !fc->F_IC) return C2D_E_ARG;
  free(c->fic);
  c->fic = (double*)malloc(sizeof(double) * C2D_NUM_NT * C2D_NPHFIELD);
  if (!c->fic) return C2D_E_NOMEM;
  for (int i = 0; i < C2D_NUM_NT; i++)
    for (int ph = 0; ph < C2D_NPHFIELD; ph++)
      c->fic[i + (size_t)ph * C2D_NUM_NT] = fc->F_IC[i * fc->F_IC_s_i + ph * fc->F_IC_s_ph];
  c->fc = *fc;
  c->fc.F_IC = c->fic;
  c->fc.F_IC_s_i = 1;
  c->fc.F_IC_s_ph = C2D_NUM_NT;
  c->fp_ready = 1;
  return C2D_OK;
}

/* the oracle has one FP arithmetic (the reference's order): either mode maps to it */
int c2d_fp_set_mode(c2d_ctx* c, int32_t mode) {
  if (!c || (mode != C2D_FP_EXACT && mode != C2D_FP_FAST && mode != C2D_FP_AUTO)) return C2D_E_ARG;
  return C2D_OK;
}

/* the stand-in always runs the oracle's FP_calc (the exact arithmetic) */
int c2d_last_fp_mode(c2d_ctx* c, int32_t* mode) {
  if (!c || !mode) return C2D_E_ARG;
  *mode = C2D_FP_EXACT;
  return C2D_OK;
}

int c2d_fp_step(c2d_ctx* c, const c2d_fp_step_in* in, c2d_fp_step_out* out) {
  if (!c || !in || !out) return C2D_E_ARG;
  if (!c->fp_ready) return fail(c, C2D_E_STATE, "c2d_fp_set_config must precede c2d_fp_step");
  const int rc = c2o_fp_step(&c->cfg, &c->fc, in, out);
  return rc ? fail(c, rc, "c2d_standin: oracle FP step failed (%d)", rc) : C2D_OK;
}

/* ---- the tally exchange, emulated through files (one directory per group) ----
 * The id is a directory name made by rank 0's c2d_comm_unique_id; rank r
 * writes round k's buffer to <dir>/r<rank>.<k> and waits until all
 * `world` buffers of round k exist, then sums them in rank order. */
int c2d_comm_unique_id(void* id, int64_t nbytes) {
  if (!id || nbytes < C2D_COMM_ID_BYTES) return C2D_E_ARG;
  const char* base = getenv("C2D_STANDIN_COMM_DIR");
  char tmpl[C2D_COMM_ID_BYTES];
  snprintf(tmpl, sizeof tmpl, "%s/c2dcommXXXXXX", base && *base ? base : "/tmp");
  if (!mkdtemp(tmpl)) return C2D_E_RCCL;
  memset(id, 0, (size_t)nbytes);
  memcpy(id, tmpl, strlen(tmpl));
  return C2D_OK;
}

int c2d_comm_init(c2d_ctx* c, const void* id, int32_t rank, int32_t world) {
  if (!c || !id || rank < 0 || world < 1 || rank >= world) return C2D_E_ARG;
  memcpy(c->comm_id, id, C2D_COMM_ID_BYTES);
  c->comm_id[C2D_COMM_ID_BYTES - 1] = 0;
  c->comm_rank = rank;
  c->comm_world = world;
  c->comm_round = 0;
  return C2D_OK;
}

/* sum `n` doubles over the group's ranks in rank order, round `round` of
 * the exchange named `tag` */
static int file_allreduce(c2d_ctx* c, double* v, int64_t n, const char* tag, int64_t round) {
  const size_t bytes = sizeof(double) * (size_t)n;
  char path[C2D_COMM_ID_BYTES + 64], tmp[C2D_COMM_ID_BYTES + 64];
  snprintf(tmp, sizeof tmp, "%s/.%s%d.%lld", c->comm_id, tag, c->comm_rank, (long long)round);
  snprintf(path, sizeof path, "%s/%s%d.%lld", c->comm_id, tag, c->comm_rank, (long long)round);
  FILE* f = fopen(tmp, "wb");
  if (!f || fwrite(v, 1, bytes, f) != bytes || fclose(f)) return fail(c, C2D_E_RCCL, "write %s", tmp);
  if (rename(tmp, path)) return fail(c, C2D_E_RCCL, "rename %s", path);
  double* sum = (double*)calloc((size_t)n, sizeof(double));
  double* buf = (double*)malloc(bytes);
  if (!sum || !buf) return fail(c, C2D_E_NOMEM, "allreduce buffers");
  for (int r = 0; r < c->comm_world; r++) {
    snprintf(path, sizeof path, "%s/%s%d.%lld", c->comm_id, tag, r, (long long)round);
    for (int tries = 0;; tries++) {
      f = fopen(path, "rb");
      if (f) break;
      if (tries > 600000) {
        free(sum);
        free(buf);
        return fail(c, C2D_E_RCCL, "timeout waiting for %s", path);
      }
      struct timespec ts = {0, 1000000};
      nanosleep(&ts, NULL);
    }
    const size_t got = fread(buf, 1, bytes, f);
    fclose(f);
    if (got != bytes) {
      free(sum);
      free(buf);
      return fail(c, C2D_E_RCCL, "short read %s", path);
    }
    for (int64_t i = 0; i < n; i++) sum[i] = sum[i] + buf[i];
  }
  memcpy(v, sum, bytes);
  free(sum);
  free(buf);
  return C2D_OK;
}

int c2d_allreduce_tallies(c2d_ctx* c) {
  if (!c) return C2D_E_ARG;
  if (c->comm_world < 1) return fail(c, C2D_E_STATE, "c2d_comm_init must precede c2d_allreduce_tallies");
  const int rc = file_allreduce(c, c->T, c->L.total, "r", c->comm_round);
  if (rc) return rc;
  c->comm_round++;
  return C2D_OK;
}

/* ---- observer-frame SED binning (the oracle's restatement of pspt's loop,
 * oracle/c2d_obs_oracle.c) with the product's pspt dialogue and file code ---- */
int c2d_obs_begin_pspt(c2d_ctx* c, const char* deck) {
  if (!c) return C2D_E_ARG;
  if (c2d_pspt_parse(deck ? deck : "", &c->pspt)) return fail(c, C2D_E_ARG, "c2d_standin: pspt deck");
  const size_t nh = (size_t)c->pspt.n_t * c->pspt.n_e;
  free(c->oF);
  free(c->oF2);
  free(c->ocnt);
  c->oF = (double*)calloc(nh, sizeof(double));
  c->oF2 = (double*)calloc(nh, sizeof(double));
  c->ocnt = (double*)calloc(nh, sizeof(double));
  if (!c->oF || !c->oF2 || !c->ocnt) return fail(c, C2D_E_NOMEM, "c2d_standin: histogram");
  c->pspt_on = 1;
  return C2D_OK;
}

int c2d_obs_accumulate(c2d_ctx* c, const double* events, int64_t n) {
  if (!c) return C2D_E_ARG;
  if (!c->pspt_on) return fail(c, C2D_E_STATE, "c2d_standin: c2d_obs_begin_pspt first");
  double* ev = NULL;
  if (!events) {                                   /* the last step's events */
    n = c2o_event_count(c->o);
    ev = (double*)malloc(sizeof(double) * C2D_EVENT_WORDS * (size_t)(n > 0 ? n : 1));
    if (!ev) return fail(c, C2D_E_NOMEM, "c2d_standin: events");
    if (n > 0) c2o_events(c->o, ev, n);
    events = ev;
  }
  c2d_obs_bins b;
  b.mode = C2D_OBS_SED; b.gam_bulk = c->pspt.gam_bulk; b.rmax = c->pspt.rmax; b.t_offset = 0.0;
  b.n_t = c->pspt.n_t; b.t0 = c->pspt.t0; b.t1 = c->pspt.t1;
  b.n_mu = 1; b.mu0 = &c->pspt.mu0; b.mu1 = &c->pspt.mu1;
  b.n_e = c->pspt.n_e; b.E0 = c->pspt.E0; b.E1 = c->pspt.E1;
  const int rc = c2o_obs_bin(&b, events, n, c->oF, c->oF2, c->ocnt);
  free(ev);
  return rc ? fail(c, rc, "c2d_standin: c2o_obs_bin") : C2D_OK;
}

int c2d_obs_write_pspt(c2d_ctx* c, const char* path, int32_t factor, int32_t world_sum) {
  if (!c) return C2D_E_ARG;
  if (!c->pspt_on) return fail(c, C2D_E_STATE, "c2d_standin: c2d_obs_begin_pspt first");
  const int64_t nh = (int64_t)c->pspt.n_t * c->pspt.n_e;
  double* w = (double*)malloc(sizeof(double) * 2 * (size_t)nh);
  if (!w) return fail(c, C2D_E_NOMEM, "c2d_standin: histogram copy");
  memcpy(w, c->oF, sizeof(double) * (size_t)nh);
  memcpy(w + nh, c->ocnt, sizeof(double) * (size_t)nh);
  if (world_sum) {
    if (c->comm_world < 1) {
      free(w);
      return fail(c, C2D_E_STATE, "c2d_standin: world_sum needs c2d_comm_init");
    }
    const int rc = file_allreduce(c, w, 2 * nh, "s", c->obs_round++);
    if (rc || c->comm_rank != 0) {
      free(w);
      return rc;
    }
  }
  const char* out = (path && path[0]) ? path : c->pspt.outfile;
  const int rc = c2d_pspt_write(out, &c->pspt, w, w + nh, factor);
  free(w);
  return rc ? fail(c, C2D_E_IO, "c2d_standin: cannot write %s", out) : C2D_OK;
}
