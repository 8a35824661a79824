// jet_x6_bwd.hip -- instantiations + dispatch of the split-bf16 backward (jet_x6.hpp).
#include "jet_x6.hpp"

namespace insr {

template <int NT, int S, bool LAP>
int launch_bwd_x6(int T, const float* x, int N, int din, int dout, int L, const float* prm, const float* act,
                  const float* gy, const float* gdy, const float* glap, float* part, long P, hipStream_t st) {
  switch (T) {
    case 1: return launch_bwd_x6_t<NT, S, LAP, 1>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    case 2: return launch_bwd_x6_t<NT, S, LAP, 2>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    case 4: return launch_bwd_x6_t<NT, S, LAP, 4>(x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st);
    default: return INSR_EINVAL;
  }
}

// width 256 (NT = 16) has no x6 backward (its dW accumulators would not fit the register
// file across stream groups): the host routes it to the fp32 tile-split kernel
int dispatch_bwd_x6(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                    const float* prm, const float* act, const float* gy, const float* gdy, const float* glap,
                    float* part, long P, hipStream_t st) {
  switch (NT) {
    case 2: INSR_DISPATCH(2, launch_bwd_x6, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 4: INSR_DISPATCH(4, launch_bwd_x6, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    case 8: INSR_DISPATCH(8, launch_bwd_x6, T, x, N, din, dout, L, prm, act, gy, gdy, glap, part, P, st)
    default: return INSR_EWIDTH;
  }
}

}  // namespace insr

#ifdef INSR_STAMPS
// diagnostic build only (make diag): the x6 backward's phase stamps (this translation unit's copy)
extern "C" int insr_diag_stamps_x6(unsigned long long* host, int n) {
  if (n > insr::kStampSlots) n = insr::kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(insr::g_insr_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
