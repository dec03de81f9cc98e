/*
 * fp.hip — Fokker-Planck electron-solve kernels (gfx950).
 *
 * Batched Chang-Cooper tridiagonal solve of src/update2d.f:2476-2518
 * (`tridag`, called from FP_calc :1398 once per zone and sub-step) with the
 * reference's semantics kept exactly: the |b(1)| <= 1e-100 early return
 * (x left untouched), the |bet| <= 1e-100 zeroing, and the clipping of
 * negative values during back-substitution (every entry but x(1)).
 * The Thomas recurrence is sequential in the energy index, so one zone is
 * one lane (the zone count, <= 9801, is far below one wave per CU: this
 * solve is latency-bound and tiny next to transport).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace c2d {

constexpr int TRI_BLOCK = 64;
constexpr int TRI_MAXN = 256;

__global__ void __launch_bounds__(TRI_BLOCK) c2d_tridag_kernel(const double* __restrict__ a,
                                                               const double* __restrict__ b,
                                                               const double* __restrict__ c,
                                                               const double* __restrict__ r,
                                                               double* __restrict__ x, int ncell,
                                                               int nt) {
  const int cell = blockIdx.x * TRI_BLOCK + threadIdx.x;
  if (cell >= ncell) return;
  const size_t o = (size_t)cell * nt;
  double gam[TRI_MAXN];
  double f[TRI_MAXN];
  const double b1 = b[o];
  if (fabs(b1) <= 1.0e-100) {   /* 'Error: b(1) = 0.' -> return, x unchanged */
    return;
  }
  double bet = b1;
  f[0] = r[o] / bet;
  for (int i = 1; i < nt; i++) {
    gam[i] = c[o + i - 1] / bet;
    bet = b[o + i] - a[o + i] * gam[i];
    if (fabs(bet) <= 1.0e-100) {
      for (int n = 0; n < nt; n++) x[o + n] = 0.0;
      return;
    }
    f[i] = (r[o + i] - a[o + i] * f[i - 1]) / bet;
  }
  for (int i = nt - 2; i >= 0; i--) {
    f[i] = f[i] - gam[i + 1] * f[i + 1];
    if (f[i + 1] < 0.0) f[i + 1] = 0.0;
  }
  for (int i = 0; i < nt; i++) x[o + i] = f[i];
}

}  // namespace c2d

extern "C" int c2d_launch_tridag(const double* a, const double* b, const double* c,
                                 const double* r, double* x, int ncell, int nt,
                                 hipStream_t stream) {
  if (nt > c2d::TRI_MAXN) return (int)hipErrorInvalidValue;
  const int grid = (ncell + c2d::TRI_BLOCK - 1) / c2d::TRI_BLOCK;
  hipLaunchKernelGGL(c2d::c2d_tridag_kernel, dim3(grid), dim3(c2d::TRI_BLOCK), 0, stream, a, b, c,
                     r, x, ncell, nt);
  return (int)hipGetLastError();
}
