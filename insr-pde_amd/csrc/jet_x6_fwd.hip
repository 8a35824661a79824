// jet_x6_fwd.hip -- instantiations + dispatch of the split-bf16 forward (jet_x6.hpp).
#include "jet_x6.hpp"

namespace insr {

template <int NT, int S, bool LAP>
int launch_fwd_x6(int T, const float* x, int N, int din, int dout, int L, const float* prm, float* y, float* dy,
                  float* lap, float* act, hipStream_t st) {
  switch (T) {
    case 1: return launch_fwd_x6_t<NT, S, LAP, 1>(x, N, din, dout, L, prm, y, dy, lap, act, st);
    case 2: return launch_fwd_x6_t<NT, S, LAP, 2>(x, N, din, dout, L, prm, y, dy, lap, act, st);
    case 4: return launch_fwd_x6_t<NT, S, LAP, 4>(x, N, din, dout, L, prm, y, dy, lap, act, st);
    default: return INSR_EINVAL;
  }
}

int dispatch_fwd_x6(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                    const float* prm, float* y, float* dy, float* lap, float* act, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_fwd_x6, T, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 4: INSR_DISPATCH(4, launch_fwd_x6, T, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 8: INSR_DISPATCH(8, launch_fwd_x6, T, x, N, din, dout, L, prm, y, dy, lap, act, st)
    case 16: INSR_DISPATCH(16, launch_fwd_x6, T, x, N, din, dout, L, prm, y, dy, lap, act, st)
    default: return INSR_EWIDTH;
  }
}

}  // namespace insr
