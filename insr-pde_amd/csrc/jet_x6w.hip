// jet_x6w.hip -- the two-kernel backward (jet_x6w.hpp) at fp32-level accuracy (NQ = 3), and
// the host helpers of the wide path.
#include "jet_x6w.hpp"

namespace insr {
template int dispatch_wide_bwd_q<3>(int, int, bool, const FbJobs&, int, int, int, int, const float*, float*, float*, int, int, int,
                                    const AdamArgs&, hipStream_t);
long wide_work_floats(long n, int din, int dout, int L, int W, int S) {
  return wide_work_floats_impl(n, din, dout, L, W, S);
}
int wsplit_launch(const float* prm, int din, int dout, int L, int W, float* planes, hipStream_t st) {
  if (L < 1) return 0;
  const long threads = 4L * L * (W / 16) * (W / 32) * 64;  // two bf16 orientations + two fp16 ones
  const dim3 grid((unsigned)((threads + 255) / 256));
  u32x4* out = reinterpret_cast<u32x4*>(planes);
  // the status quad after the planes: cleared, then set by any out-of-range weight of this split
  unsigned* status = reinterpret_cast<unsigned*>(planes + 5L * L * W * W);
  if (const int rc = (int)hipMemsetAsync(status, 0, 4 * sizeof(unsigned), st)) return rc;
  switch (W) {
    case 32: hipLaunchKernelGGL((wsplit_kernel<2>), grid, dim3(256), 0, st, prm, din, L, out, status); break;
    case 64: hipLaunchKernelGGL((wsplit_kernel<4>), grid, dim3(256), 0, st, prm, din, L, out, status); break;
    case 128: hipLaunchKernelGGL((wsplit_kernel<8>), grid, dim3(256), 0, st, prm, din, L, out, status); break;
    case 256: hipLaunchKernelGGL((wsplit_kernel<16>), grid, dim3(256), 0, st, prm, din, L, out, status); break;
    default: return INSR_EWIDTH;
  }
  (void)dout;
  return (int)hipGetLastError();
}
void wide_launch_threads(long n, int din, int dout, int L, int W, int S, long* out) {
  wide_launch_threads_impl(n, din, dout, L, W, S, out);
}
}  // namespace insr
