/*
 * selftest.hip — device-side diagnostics exported through the C-ABI:
 * evaluates the deterministic elementary functions (c2d_math.h) and the
 * lineage RNG (c2d_rng.h) on the GPU so tests can check them bit for bit
 * against the host build of the same code.
 */
#include <hip/hip_runtime.h>

#include "c2d_math.h"
#include "c2d_rng.h"

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
