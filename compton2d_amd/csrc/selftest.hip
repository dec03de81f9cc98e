/*
 * selftest.hip — device-side diagnostics exported through the C-ABI:
 * evaluates the deterministic elementary functions (c2d_math.h), the
 * lineage RNG (c2d_rng.h) and McDonald's series (c2d_wave.hpp) on the GPU so
 * tests can check them bit for bit against the host build of the same code.
 */
#include <hip/hip_runtime.h>

#include <vector>

#include "c2d_device.hpp"
#include "c2d_math.h"
#include "c2d_rng.h"
#include "c2d_wave.hpp"

namespace c2d {
__global__ void c2d_selftest_math_kernel(int fn, const double* x, double* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double r;
  switch (fn) {
    case 0: r = c2d_log(v); break;
    case 1: r = c2d_exp(v); break;
    case 2: r = c2d_cos(v); break;
    case 3: r = c2d_acos(v); break;
    case 4: r = c2d_pow(v, 1.0 / 3.0); break;
    case 5: r = __builtin_sqrt(v); break;
    case 6: r = v / 3.0; break;
    case 8: r = c2d_log_pos(v); break;
    case 9: r = c2d_exp_bf(v); break;
    /* the fast build's reciprocal / reciprocal-sqrt sequences (transport.hip):
     * the hardware estimate alone and after one Newton step */
    case 10: r = __builtin_amdgcn_rcp(v); break;
    case 11: {
      const double q = __builtin_amdgcn_rcp(v);
      r = __builtin_fma(q, __builtin_fma(-v, q, 1.0), q);
      break;
    }
    case 12: r = __builtin_amdgcn_rsq(v); break;
    case 13: {
      const double q = __builtin_amdgcn_rsq(v);
      r = q * __builtin_fma(-0.5 * v, q * q, 1.5);
      break;
    }
    /* the fast build's optical depth log (transport.hip TAU_LOG) */
    case 14: r = c2d_tau_log_f32(v); break;
    default: r = c2d_draw((uint64_t)(int64_t)v, (uint32_t)i); break;
  }
  y[i] = r;
}
}  // namespace c2d

extern "C" int c2d_selftest_math(int device, int fn, const double* x_host, double* y_host,
                                 int64_t n) {
  if (n <= 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return -2;
  double *x = nullptr, *y = nullptr;
  if (hipMalloc((void**)&x, n * sizeof(double)) != hipSuccess) return -2;
  if (hipMalloc((void**)&y, n * sizeof(double)) != hipSuccess) return -2;
  int rc = 0;
  if (hipMemcpy(x, x_host, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(c2d::c2d_selftest_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, 0, fn, x, y, n);
    if (hipDeviceSynchronize() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(y_host, y, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  (void)hipFree(x);
  (void)hipFree(y);
  return rc;
}

/* The r-boundary distance of a flight step (src/imctrk2d.f:251-277) with the
 * fast build's reciprocal / square-root sequences after NR Newton steps --
 * the same sequences as transport.hip rcp_pos / fsqrt_nn -- or (NR = 0) IEEE
 * sqrt and division as the exact build. */
namespace c2d {
template <int NR>
__device__ __forceinline__ double st_rcp(double b) {
  double y = __builtin_amdgcn_rcp(b);
#pragma unroll
  for (int k = 0; k < NR; k++) y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  return y;
}
template <int NR>
__device__ __forceinline__ double st_sqrt(double x) {
  x = fmax(x, 1.0e-300);
  const double h = 0.5 * x;
  double y = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int k = 0; k < NR; k++) y = y * __builtin_fma(-h, y * y, 1.5);
  return x * y;
}
template <int NR>
__global__ void c2d_selftest_geom_kernel(const double* in, double* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  /* rbnd < 0: the inner boundary |rbnd| (inout = -1, imctrk2d.f:254-264) */
  const double rpre = in[4 * i], Eta = in[4 * i + 1], wmu = in[4 * i + 2];
  const double rbnd = fabs(in[4 * i + 3]);
  const double inout = in[4 * i + 3] < 0.0 ? -1.0 : 1.0;
  const double disp = Eta * rpre;
  const double psq = rpre * rpre * (1.0 - Eta * Eta);
  double dpbsq = rbnd * rbnd - psq;
  if (dpbsq < 1.0e-6) dpbsq = 1.0e-6;
  double disbr, trldb;
  if (NR == 0) {
    disbr = inout * __builtin_sqrt(dpbsq) - disp;
    trldb = disbr / __builtin_sqrt(1.0 - wmu * wmu);
  } else {
    disbr = inout * st_sqrt<NR>(dpbsq) - disp;
    trldb = disbr * st_rcp<NR>(st_sqrt<NR>(1.0 - wmu * wmu));
  }
  out[2 * i] = disbr;
  out[2 * i + 1] = trldb;
}
}  // namespace c2d

extern "C" int c2d_selftest_geom(int device, int nr, const double* in_host, double* out_host, int64_t n) {
  if (n <= 0) return 0;
  if (nr < 0 || nr > 2) return -1;
  if (hipSetDevice(device) != hipSuccess) return -2;
  double *in = nullptr, *out = nullptr;
  if (hipMalloc((void**)&in, 4 * n * sizeof(double)) != hipSuccess) return -2;
  if (hipMalloc((void**)&out, 2 * n * sizeof(double)) != hipSuccess) { (void)hipFree(in); return -2; }
  int rc = 0;
  if (hipMemcpy(in, in_host, 4 * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) rc = -2;
  if (!rc) {
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    if (nr == 0) hipLaunchKernelGGL(c2d::c2d_selftest_geom_kernel<0>, g, b, 0, 0, in, out, n);
    else if (nr == 1) hipLaunchKernelGGL(c2d::c2d_selftest_geom_kernel<1>, g, b, 0, 0, in, out, n);
    else hipLaunchKernelGGL(c2d::c2d_selftest_geom_kernel<2>, g, b, 0, 0, in, out, n);
    if (hipDeviceSynchronize() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out_host, out, 2 * n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) rc = -2;
  (void)hipFree(in);
  (void)hipFree(out);
  return rc;
}

/* McDonald K2, K3 at n arguments z (one wavefront each, c2d_wave.hpp's
 * mcdonald23_w) and the shader cycles each evaluation took: parity with the
 * oracle's sequential McDonald (src/volume2d.f:598-626) and a latency probe. */

namespace c2d {
__global__ void __launch_bounds__(64) c2d_selftest_mcd_kernel(const double* z, const double* tab,
                                                             double* out, int n) {
  const int i = blockIdx.x;
  if (i >= n) return;
  const int lane = threadIdx.x;
  __shared__ double scr[4 * wave::FPB];
  long long guard = 0;
  double K2, K3;
  const long long t0 = clock64();
  wave::mcdonald23_w(z[i], lane, tab, K2, K3, guard, scr);
  const long long t1 = clock64();
  if (lane == 0) {
    out[3 * i] = K2;
    out[3 * i + 1] = K3;
    out[3 * i + 2] = (double)(t1 - t0);
  }
}
}  // namespace c2d

/* the abscissa table as capi.cpp ensure_mcd builds it */
static std::vector<double> mcd_abscissae() {
  std::vector<double> mt((size_t)C2D_FP_MCD_N * 4);
  const double dtm = 1.001, sm = 5.0e-1 * (1.0 + dtm);
  double t = 1.0;
  for (int k = 0; k < C2D_FP_MCD_N; k++) {
    const double ts = t * sm;
    mt[(size_t)k * 4 + 0] = t;
    mt[(size_t)k * 4 + 1] = ts;
    mt[(size_t)k * 4 + 2] = c2d_pow(ts * ts - 1.0, 1.5);
    mt[(size_t)k * 4 + 3] = c2d_pow(ts * ts - 1.0, 2.5);
    t = t * dtm;
  }
  return mt;
}

extern "C" int c2d_selftest_mcdonald(int device, const double* z_host, int n, double* out_host) {
  if (n <= 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return -2;
  const std::vector<double> mt = mcd_abscissae();
  double *z = nullptr, *tab = nullptr, *out = nullptr;
  int rc = 0;
  if (hipMalloc((void**)&z, n * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&tab, mt.size() * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&out, 3 * (size_t)n * sizeof(double)) != hipSuccess)
    rc = -2;
  if (!rc && (hipMemcpy(z, z_host, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(tab, mt.data(), mt.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
    rc = -2;
  if (!rc) {
    hipLaunchKernelGGL(c2d::c2d_selftest_mcd_kernel, dim3((unsigned)n), dim3(64), 0, 0, z, tab, out, n);
    if (hipDeviceSynchronize() != hipSuccess) rc = -2;
  }
  if (!rc && hipMemcpy(out_host, out, 3 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = -2;
  if (z) (void)hipFree(z);
  if (tab) (void)hipFree(tab);
  if (out) (void)hipFree(out);
  return rc;
}

/* The fast FP kernel's McDonald pair from its moment table against the same
 * kernel's term-by-term series (fp_fast.hip mcd_mtab / mcdonald23_fast), per
 * z: K2, K3 (table), K2, K3 (series), 1 if the table answered, and the
 * shader cycles of each. */
extern "C" int c2d_fp_mom_build(const double* mcd, double* mom, hipStream_t stream);
extern "C" int c2d_fp_mtab_test(const double* mcd, const double* mom, const double* z, double* out, int n,
                                hipStream_t stream);
extern "C" int c2d_selftest_mcd_fast(int device, const double* z_host, int n, double* out_host) {
  if (n <= 0) return 0;
  if (hipSetDevice(device) != hipSuccess) return -2;
  const std::vector<double> mt = mcd_abscissae();
  double *z = nullptr, *tab = nullptr, *mom = nullptr, *out = nullptr;
  int rc = 0;
  if (hipMalloc((void**)&z, n * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&tab, mt.size() * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&mom, (size_t)C2D_FPF_MT_N * C2D_FPF_MT_W * sizeof(double)) != hipSuccess ||
      hipMalloc((void**)&out, 8 * (size_t)n * sizeof(double)) != hipSuccess)
    rc = -2;
  if (!rc && (hipMemcpy(z, z_host, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
              hipMemcpy(tab, mt.data(), mt.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
    rc = -2;
  if (!rc && (c2d_fp_mom_build(tab, mom, 0) != 0 || c2d_fp_mtab_test(tab, mom, z, out, n, 0) != 0)) rc = -2;
  if (!rc && hipDeviceSynchronize() != hipSuccess) rc = -2;
  if (!rc && hipMemcpy(out_host, out, 8 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = -2;
  if (z) (void)hipFree(z);
  if (tab) (void)hipFree(tab);
  if (mom) (void)hipFree(mom);
  if (out) (void)hipFree(out);
  return rc;
}
