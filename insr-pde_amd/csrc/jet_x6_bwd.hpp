// jet_x6_bwd.hpp -- launch + dispatch templates of the split-bf16 backward (jet_x6.hpp),
// instantiated per precision (NQ) by jet_x6_bwd.hip (NQ = 3) and jet_bf_bwd.hip (NQ = 1, 2).
#pragma once
#include "jet_x6.hpp"

namespace insr {

// T in {1, 2, 4}; the balanced modes add T = 3 (2-3 stream jets) and T = 5 (value jets)
template <int NQ, int NT, int S, bool LAP>
int launch_bwd_x6(int T, const BwdJobsX6* J, int din, int dout, int L, const float* prm, float* part, long P,
                  hipStream_t st) {
  switch (T) {
    case 1: return launch_bwd_x6_t<NQ, NT, S, LAP, 1>(J, din, dout, L, prm, part, P, st);
    case 2: return launch_bwd_x6_t<NQ, NT, S, LAP, 2>(J, din, dout, L, prm, part, P, st);
    case 4: return launch_bwd_x6_t<NQ, NT, S, LAP, 4>(J, din, dout, L, prm, part, P, st);
    case 3:
      if constexpr ((S == 2 || S == 3) && !LAP)
        return launch_bwd_x6_t<NQ, NT, S, LAP, 3>(J, din, dout, L, prm, part, P, st);
      return INSR_EINVAL;
    case 5:
      if constexpr (S == 1)
        return launch_bwd_x6_t<NQ, NT, S, LAP, 5>(J, din, dout, L, prm, part, P, st);
      return INSR_EINVAL;
    default: return INSR_EINVAL;
  }
}

// width 256 (NT = 16) has no fused split-bf16 backward (its dW accumulators would not fit the
// register file across stream groups): the host routes it to the two-kernel path
template <int NQ>
int dispatch_bwd_q(int NT, int S, bool LAP, int T, const BwdJobsX6* J, int din, int dout, int L,
                   const float* prm, float* part, long P, hipStream_t st) {
#define INSR_BWD_Q(NTV)                                                                                       \
  switch (S * 2 + (LAP ? 1 : 0)) {                                                                            \
    case 2: return launch_bwd_x6<NQ, NTV, 1, false>(T, J, din, dout, L, prm, part, P, st); \
    case 4: return launch_bwd_x6<NQ, NTV, 2, false>(T, J, din, dout, L, prm, part, P, st); \
    case 6: return launch_bwd_x6<NQ, NTV, 3, false>(T, J, din, dout, L, prm, part, P, st); \
    case 8: return launch_bwd_x6<NQ, NTV, 4, false>(T, J, din, dout, L, prm, part, P, st); \
    case 7: return launch_bwd_x6<NQ, NTV, 3, true>(T, J, din, dout, L, prm, part, P, st);  \
    case 9: return launch_bwd_x6<NQ, NTV, 4, true>(T, J, din, dout, L, prm, part, P, st);  \
    case 11: return launch_bwd_x6<NQ, NTV, 5, true>(T, J, din, dout, L, prm, part, P, st); \
    default: return INSR_EINVAL;                                                                              \
  }
  switch (NT) {
    case 2: INSR_BWD_Q(2)
    case 4: INSR_BWD_Q(4)
    case 8: INSR_BWD_Q(8)
    default: return INSR_EWIDTH;
  }
#undef INSR_BWD_Q
}

}  // namespace insr
