// jet_x6w.hip -- the two-kernel backward (jet_x6w.hpp) at fp32-level accuracy (NQ = 3), and
// the host helpers of the wide path.
#include "jet_x6w.hpp"

namespace insr {
template int dispatch_wide_bwd_q<3>(int, int, bool, const float*, int, int, int, int, const float*, const float*,
                                    const float*, const float*, const float*, float*, float*, int, hipStream_t);
long wide_work_floats(long n, int din, int dout, int L, int W, int S) {
  return wide_work_floats_impl(n, din, dout, L, W, S);
}
void wide_launch_threads(long n, int din, int dout, int L, int W, int S, long* out) {
  wide_launch_threads_impl(n, din, dout, L, W, S, out);
}
}  // namespace insr
