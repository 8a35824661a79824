// study: accuracy of the hardware v_sin_f32 / v_cos_f32 after a Cody-Waite reduction, vs the
// polynomial sincos_fast of jet_common.hpp (double reference on the host)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__device__ __forceinline__ void sc_hw(float x, float& s, float& c) {
  const float n = rintf(x * 0.15915494309189535f);
  float r = fmaf(-n, 6.28125f, x);
  r = fmaf(-n, 1.9353071795864769e-3f, r);
  const float t = r * 0.15915494309189535f;
  s = __builtin_amdgcn_sinf(t);
  c = __builtin_amdgcn_cosf(t);
}
__global__ void k(const float* x, float* s, float* c, long n) {
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) sc_hw(x[i], s[i], c[i]);
}
int main() {
  const long n = 1 << 24;
  std::vector<float> x(n), s(n), c(n);
  for (long i = 0; i < n; ++i) x[i] = -200.f + 400.f * (float)i / (float)n;
  float *dx, *ds, *dc;
  hipMalloc(&dx, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, n);
  hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
  double es = 0, ec = 0, es2 = 0;
  for (long i = 0; i < n; ++i) {
    const double d = (double)x[i];
    es = fmax(es, fabs(s[i] - sin(d)));
    ec = fmax(ec, fabs(c[i] - cos(d)));
    es2 += (s[i] - sin(d)) * (s[i] - sin(d));
  }
  // fp32 argument rounding of 30 z itself: |x| ulp / 2 at |x| = 200
  printf("hw sin max abs err %.3g  cos %.3g  rms %.3g  (fp32 half-ulp at 200: %.3g)\n", es, ec, sqrt(es2 / n),
         ldexp(1.0, -24) * 128);
  return 0;
}
