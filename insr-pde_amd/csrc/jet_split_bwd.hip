// jet_split_bwd.hip -- instantiations + dispatch of the tile-split backward (jet_split.hpp).
#include "jet_split.hpp"

namespace insr {

template <int NT, int S, bool LAP>
int launch_bwd_split(int T, const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
                     const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st) {
  switch (T) {
    case 1: return launch_bwd_split_t<NT, S, LAP, 1>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    case 2: return launch_bwd_split_t<NT, S, LAP, 2>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    case 4: return launch_bwd_split_t<NT, S, LAP, 4>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    default: return INSR_EINVAL;
  }
}

int dispatch_bwd_split(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                       const float* prm, const float* act, const float* gy, const float* gdy, const float* glap,
                       float* part, long P, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_bwd_split, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 4: INSR_DISPATCH(4, launch_bwd_split, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 8: INSR_DISPATCH(8, launch_bwd_split, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 16: INSR_DISPATCH(16, launch_bwd_split, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    default: return INSR_EWIDTH;
  }
}

}  // namespace insr

#ifdef INSR_STAMPS
// diagnostic build only (make diag): read / clear the phase stamps of the backward
extern "C" int insr_diag_stamps(unsigned long long* host, int n) {
  if (n > insr::kStampSlots) n = insr::kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(insr::g_insr_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int insr_diag_clear(void) {
  static unsigned long long zero[insr::kStampSlots];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(insr::g_insr_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif
