/*
 * observe.hip — observer-frame binning of escape events on gfx950
 * (SURVEY.md §8(f)#3): the loops of the reference's post-processing tools
 * postprocessing/pspt.c:245-294 (SED: time x energy, one angular window) and
 * postprocessing/plcm.c:382-456 (light curves: time x angular bins x
 * possibly overlapping energy bands, with sum of ew^2), run on the device's
 * escape-event buffer so the 105-byte ASCII event lines (imcleak2d.f:171,
 * format 105) need not be written and re-parsed.
 *
 * One lane per event: Lorentz boost with the bulk factor, light-travel time,
 * bin search over LDS-staged edges (the tools' first-match semantics; a
 * binary search when the edges are sorted, else their linear scan), then
 * accumulation.  The leading time rows of the histogram that fit in LDS
 * (all of them for a pspt SED; ~290 of plcm's 1024 rows) are privatised per
 * workgroup and flushed with one global atomic per non-zero bin; events in
 * later rows use wave-aggregated global atomics (one atomic per distinct bin
 * per wave), so hot bins never serialise lane by lane.  The event stream is
 * read once: 56 B per event (HBM-bound).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/compton2d.h"
#include "c2d_device.hpp"
#include "c2d_math.h"

namespace c2d {

constexpr int OBS_BLOCK = 512;

__device__ inline double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

/* Wave-aggregated histogram add: every lane with h >= 0 adds (w, w^2, 1) to
 * bin h.  Lanes that share a bin are reduced first and one lane per distinct
 * bin issues the atomics, so a hot bin costs one atomic per wave instead of
 * one per lane (hot bins are the norm: most events fall in a few time bins).
 * Called by all lanes of the wave together. */
__device__ inline void agg_add(double* F, double* F2, double* C, int h, double w) {
  uint64_t pending = __ballot(h >= 0);
  const int lane = __lane_id();
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const int hl = __shfl(h, leader, 64);
    const bool mine = (h == hl) && ((pending >> lane) & 1);
    const uint64_t m = __ballot(mine);
    const double s = wave_sum(mine ? w : 0.0);
    const double s2 = wave_sum(mine ? w * w : 0.0);
    if (lane == leader) {
      atomicAdd(&F[hl], s);
      atomicAdd(&F2[hl], s2);
      atomicAdd(&C[hl], (double)__popcll(m));
    }
    pending &= ~m;
  }
}

/* First k with lo[k] <= x < hi[k] (the tools' linear first-match scan), or n.
 * When lo[] and hi[] are both non-decreasing (`sorted`, checked on the host)
 * the matching k form a contiguous range whose first element is the first k
 * with hi[k] > x: a binary search then gives the same answer, NaN included. */
__device__ inline int first_bin(const double* lo, const double* hi, int n, bool sorted, double x) {
  if (!sorted) {
    int k;
    for (k = 0; k < n; k++)
      if (x >= lo[k] && x < hi[k]) break;
    return k;
  }
  int a = 0, b = n;                      /* first k in [a, b) with hi[k] > x */
  while (a < b) {
    const int m = (a + b) >> 1;
    if (hi[m] > x) b = m; else a = m + 1;
  }
  return (a < n && x >= lo[a]) ? a : n;
}

/* the event segments of one launch (the transport's event shards, back to
 * back): event e lies in segment s with pre[s] <= e < pre[s + 1] */
struct ObsSegs {
  const double* base[C2D_EV_SHARDS];
  int64_t pre[C2D_EV_SHARDS + 1];
  int32_t nseg;
};

__global__ void __launch_bounds__(OBS_BLOCK) c2d_obs_kernel(const ObsDev O, const ObsSegs S) {
  __shared__ int64_t seg_pre[C2D_EV_SHARDS + 1];
  __shared__ const double* seg_base[C2D_EV_SHARDS];
  if (threadIdx.x <= (unsigned)S.nseg) seg_pre[threadIdx.x] = S.pre[threadIdx.x];
  if (threadIdx.x < (unsigned)S.nseg) seg_base[threadIdx.x] = S.base[threadIdx.x];
  const int64_t n = S.pre[S.nseg];
  extern __shared__ double sh[];
  double* t0 = sh;
  double* t1 = t0 + O.n_t;
  double* mu0 = t1 + O.n_t;
  double* mu1 = mu0 + O.n_mu;
  double* E0 = mu1 + O.n_mu;
  double* E1 = E0 + O.n_e;
  /* bins h = row * row_len + col, row = time bin; rows < lds_rows live in LDS */
  const int row_len = O.n_mu * O.n_e;
  const int nl = O.lds_rows * row_len;
  double* hF = E1 + O.n_e;
  double* hF2 = hF + nl;
  double* hC = hF2 + nl;
  for (int i = threadIdx.x; i < O.n_t; i += OBS_BLOCK) { t0[i] = O.t0[i]; t1[i] = O.t1[i]; }
  for (int i = threadIdx.x; i < O.n_mu; i += OBS_BLOCK) { mu0[i] = O.mu0[i]; mu1[i] = O.mu1[i]; }
  for (int i = threadIdx.x; i < O.n_e; i += OBS_BLOCK) { E0[i] = O.E0[i]; E1[i] = O.E1[i]; }
  for (int i = threadIdx.x; i < 3 * nl; i += OBS_BLOCK) hF[i] = 0.0;
  __syncthreads();
  /* LDS bins: plain per-lane LDS atomics; the rest: wave-aggregated global atomics */
  auto add = [&](int h, double w) {
    if (h >= 0 && h < nl) {
      atomicAdd(&hF[h], w);
      atomicAdd(&hF2[h], w * w);
      atomicAdd(&hC[h], 1.0);
    }
    agg_add(O.F, O.F2, O.cnt, h >= nl ? h : -1, w);
  };
  const double G = O.gam_bulk;
  const double betta = __builtin_sqrt(1. - 1. / (G * G));
  /* wave-uniform trip count so the aggregation's cross-lane ops see the whole wave */
  for (int64_t base = (int64_t)blockIdx.x * OBS_BLOCK; base < n; base += (int64_t)gridDim.x * OBS_BLOCK) {
    const int64_t e = base + threadIdx.x;
    const bool valid = e < n;
    const int64_t ee = valid ? e : 0;
    int sg = 0;                            /* last segment with seg_pre[sg] <= ee */
    for (int hi = S.nseg - 1; sg < hi;) {
      const int m = (sg + hi + 1) >> 1;
      if (seg_pre[m] <= ee) sg = m; else hi = m - 1;
    }
    const double* v = seg_base[sg] + (ee - seg_pre[sg]) * C2D_EVENT_WORDS;
    double t_bound = v[0], E = v[1], ew = v[2];
    const double r = v[3], z = v[4];
    double mu = v[5];
    const double phi = v[6];
    /* pspt.c:253-272 / plcm.c:390-399 */
    mu = -mu;
    const double doppler = G * (1. + mu * betta);
    t_bound = (t_bound - betta * z * 3.33333333e-11) / doppler;
    E = E * doppler;
    ew = ew * doppler;
    mu = (mu + betta) / (1. + mu * betta);
    const double cdt = z * mu / G + __builtin_sqrt(1. - mu * mu) * (O.rmax - r * c2d_cos(phi));
    double time = t_bound + 3.33333333e-11 * cdt;
    if (O.mode == C2D_OBS_SED) {
      int h = -1;
      if (valid && !(mu < mu0[0] || mu > mu1[0])) {            /* pspt.c:274 */
        const int k = first_bin(E0, E1, O.n_e, O.sorted_e, E);
        const int m = first_bin(t0, t1, O.n_t, O.sorted_t, time);
        if (k < O.n_e && m < O.n_t) h = m * O.n_e + k;
      }
      add(h, ew);
    } else {
      time -= O.t_offset;                                      /* plcm.c:407-408 */
      int row = -1;
      if (valid && !(time < 0.)) {
        const int k = first_bin(t0, t1, O.n_t, O.sorted_t, time);
        const int m = first_bin(mu0, mu1, O.n_mu, O.sorted_mu, mu);
        if (k < O.n_t && m < O.n_mu) row = (k * O.n_mu + m) * O.n_e;
      }
      for (int l = 0; l < O.n_e; l++)                          /* every band containing E */
        add((row >= 0 && E >= E0[l] && E < E1[l]) ? row + l : -1, ew);
    }
  }
  if (nl) {
    __syncthreads();
    for (int i = threadIdx.x; i < nl; i += OBS_BLOCK) {
      if (hC[i] != 0.0) {
        atomicAdd(&O.F[i], hF[i]);
        atomicAdd(&O.F2[i], hF2[i]);
        atomicAdd(&O.cnt[i], hC[i]);
      }
    }
  }
}

}  // namespace c2d

extern "C" size_t c2d_obs_lds_bytes(int n_t, int n_mu, int n_e, int lds_rows) {
  return sizeof(double) * (2 * (size_t)(n_t + n_mu + n_e) + 3 * (size_t)lds_rows * n_mu * n_e);
}

extern "C" int c2d_obs_block(void) { return c2d::OBS_BLOCK; }

/* one launch over nseg event segments (ev[s], n[s] events each; at most
 * C2D_EV_SHARDS): the transport's event shards binned together */
extern "C" int c2d_launch_obs_segs(const c2d::ObsDev* O, const double* const* ev, const int64_t* n, int nseg,
                                   int grid, hipStream_t stream) {
  if (nseg < 1 || nseg > C2D_EV_SHARDS) return (int)hipErrorInvalidValue;
  c2d::ObsSegs S;
  int k = 0;
  S.pre[0] = 0;
  for (int s = 0; s < nseg; s++) {
    if (n[s] <= 0) continue;
    S.base[k] = ev[s];
    S.pre[k + 1] = S.pre[k] + n[s];
    k++;
  }
  if (k == 0) return 0;
  S.nseg = k;
  const size_t lds = c2d_obs_lds_bytes(O->n_t, O->n_mu, O->n_e, O->lds_rows);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)c2d::c2d_obs_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(c2d::c2d_obs_kernel, dim3(grid), dim3(c2d::OBS_BLOCK), lds, stream, *O, S);
  return (int)hipGetLastError();
}

extern "C" int c2d_launch_obs(const c2d::ObsDev* O, const double* ev, int64_t n, int grid,
                              hipStream_t stream) {
  return c2d_launch_obs_segs(O, &ev, &n, 1, grid, stream);
}
