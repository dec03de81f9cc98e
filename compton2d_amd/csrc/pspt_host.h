/* The SED tool's input dialogue and output file, on the host
 * (postprocessing/pspt.c:105-205 and :323-353), for c2d_obs_begin_pspt /
 * c2d_obs_write_pspt: the shim bins every step's escapes on the device with
 * pspt's own binning and writes pspt's file, so no event text is needed.
 *
 * Header-only C that also compiles as C++ (capi.cpp, and the test-only
 * oracle stand-in oracle/c2d_standin.c); no device code. */
#ifndef C2D_PSPT_HOST_H
#define C2D_PSPT_HOST_H

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define C2D_PSPT_TMAX 90     /* pspt.c:10 t_max  */
#define C2D_PSPT_CHMAX 200   /* pspt.c:8  ch_max */

typedef struct c2d_pspt_deck {
  char infile[64], outfile[64];
  double gam_bulk, rmax, t_start, t_end, dt, mu0, mu1;
  int n_t, n_e;
  double t0[C2D_PSPT_TMAX], t1[C2D_PSPT_TMAX];
  double E0[C2D_PSPT_CHMAX], E1[C2D_PSPT_CHMAX];
} c2d_pspt_deck;

/* the next line of the dialogue (gets() on stdin: up to the newline) */
static int c2d_pspt_line(const char** p, char* a, int cap) {
  int n = 0;
  const char* s = *p;
  while (*s && *s != '\n') {
    if (n < cap - 1) a[n++] = *s;
    s++;
  }
  if (*s == '\n') s++;
  a[n] = '\0';
  *p = s;
  return n;
}

/* add_dat (pspt.c:36-49): ".dat" unless the name has a 3-letter extension */
static void c2d_pspt_add_dat(char* s, int cap) {
  const int n = (int)strlen(s);
  if (!(n >= 4 && s[n - 4] == '.') && n + 4 < cap) strcat(s, ".dat");
}

/* dinput / iinput (pspt.c:52-71): an empty line keeps the default */
static double c2d_pspt_d(const char** p, double x) {
  char a[256];
  return c2d_pspt_line(p, a, (int)sizeof a) ? atof(a) : x;
}
static int c2d_pspt_i(const char** p, int x) {
  char a[256];
  return c2d_pspt_line(p, a, (int)sizeof a) ? atoi(a) : x;
}

/* pspt.c:105-205 over `text` (one answer a line, e.g.
 * postprocessing/mrk421_sed.input; "" = every default).  0, or -1 when the
 * energy grid exceeds ch_max channels (pspt asks again; here an error). */
static int c2d_pspt_parse(const char* text, c2d_pspt_deck* d) {
  const char* p = text ? text : "";
  char a[256];
  int reg, k, regions = 1, n_r = 100;
  double E_lower = 1.e-7, E_upper = 1.e10, dE;
  memset(d, 0, sizeof *d);
  strcpy(d->infile, "p001_evb.dat");
  strcpy(d->outfile, "seds_30.dat");
  if (c2d_pspt_line(&p, a, (int)sizeof a)) {
    if (a[0] >= '0' && a[0] <= '9') {              /* p0 + the digits given */
      d->infile[2] = '\0';
      strncat(d->infile, a, sizeof d->infile - 8);
    } else {
      strncpy(d->infile, a, sizeof d->infile - 8);
    }
    c2d_pspt_add_dat(d->infile, (int)sizeof d->infile);
  }
  d->gam_bulk = c2d_pspt_d(&p, 33.);
  d->rmax = c2d_pspt_d(&p, 1.e16);
  if (c2d_pspt_line(&p, a, (int)sizeof a)) {
    strncpy(d->outfile, a, sizeof d->outfile - 8);
    c2d_pspt_add_dat(d->outfile, (int)sizeof d->outfile);
  }
  d->n_t = c2d_pspt_i(&p, 30);
  if (d->n_t > C2D_PSPT_TMAX) d->n_t = C2D_PSPT_TMAX;
  if (d->n_t < 1) return -1;
  d->t_start = c2d_pspt_d(&p, 1.6e4);
  d->t_end = c2d_pspt_d(&p, 6e4);
  d->dt = (d->t_end - d->t_start) / d->n_t;
  for (k = 0; k < d->n_t; k++) {                   /* pspt.c:143-146 */
    d->t0[k] = d->t_start + k * d->dt;
    d->t1[k] = d->t_start + k * d->dt + d->dt;
  }
  d->mu0 = c2d_pspt_d(&p, 0.99944);
  d->mu1 = c2d_pspt_d(&p, 0.99964);
  regions = c2d_pspt_i(&p, regions);
  d->n_e = 0;
  for (reg = 0; reg < regions; reg++) {            /* pspt.c:159-193 */
    E_lower = c2d_pspt_d(&p, E_lower);
    E_upper = c2d_pspt_d(&p, E_upper);
    n_r = c2d_pspt_i(&p, n_r);
    if (n_r < 1 || n_r + d->n_e > C2D_PSPT_CHMAX) return -1;
    c2d_pspt_line(&p, a, (int)sizeof a);
    const int n0 = d->n_e;
    if (a[0] == '1') {
      dE = (E_upper - E_lower) / ((double)(n_r));
      d->E0[n0] = E_lower;
      for (k = n0; k < n0 + n_r - 1; k++) d->E1[k] = d->E0[k + 1] = d->E0[k] + dE;
      d->E1[n0 + n_r - 1] = d->E0[n0 + n_r - 1] + dE;
    } else {
      dE = exp(log(E_upper / E_lower) / ((double)(n_r)));
      d->E0[n0] = E_lower;
      for (k = n0; k < n0 + n_r - 1; k++) d->E1[k] = d->E0[k + 1] = d->E0[k] * dE;
      d->E1[n0 + n_r - 1] = d->E0[n0 + n_r - 1] * dE;
    }
    d->n_e += n_r;
    E_lower = E_upper;
  }
  return d->n_e > 0 ? 0 : -1;
}

/* max() of pspt.c:14-20 (a NaN second argument wins) */
static double c2d_pspt_max(double x, double y) { return x > y ? x : y; }

/* The output file of pspt.c:323-353 from the raw sums of ew and the counts
 * per [n_t][n_e] bin (c2d_obs_result's F and count with n_mu = 1).
 * 0, or -1 when the file cannot be written. */
static int c2d_pspt_write(const char* path, const c2d_pspt_deck* d, const double* F, const double* cnt,
                          int factor) {
  int k, n;
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  fprintf(f, "#time(s): %e %e dt(s): %e\n", d->t_start, d->t_end, d->dt);
  fprintf(f, "#angle: %f %f\n", d->mu0, d->mu1);
  fprintf(f, "#factor: %i\n", factor);
  fprintf(f, "#Energy(keV)   Luminosity(erg/s/keV)\n");
  for (k = 0; k < d->n_e; k++) {
    const double den = d->dt * (d->E1[k] - d->E0[k]) * (d->mu1 - d->mu0) / 2.;
    fprintf(f, "%e ", c2d_pspt_max(1.e-20, sqrt(d->E0[k] * d->E1[k])));
    for (n = 0; n < d->n_t - 1; n++) fprintf(f, "%e ", c2d_pspt_max(1.e-20, F[(size_t)n * d->n_e + k] / den));
    n = d->n_t - 1;
    fprintf(f, "%e %i\n", c2d_pspt_max(1.e-20, F[(size_t)n * d->n_e + k] / den), (int)cnt[(size_t)n * d->n_e + k]);
  }
  return fclose(f) == 0 ? 0 : -1;
}

#endif /* C2D_PSPT_HOST_H */
