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

template <int NT, int S, bool LAP>
int launch_fwd_x6_multi(int T, const InsrJetJob* jobs, const int* small, int njobs, int din, int dout, int L,
                        hipStream_t st) {
  switch (T) {
    case 1: return launch_fwd_x6_multi_t<NT, S, LAP, 1>(jobs, small, njobs, din, dout, L, st);
    case 2: return launch_fwd_x6_multi_t<NT, S, LAP, 2>(jobs, small, njobs, din, dout, L, st);
    case 4: return launch_fwd_x6_multi_t<NT, S, LAP, 4>(jobs, small, njobs, din, dout, L, st);
    default: return INSR_EINVAL;
  }
}

// value and gradient jets (the fused pairs the models issue are value jets; the Laplacian
// jet is never paired), widths 64 / 128 / 256
int dispatch_fwd_x6_multi(int NT, int S, bool LAP, int T, const InsrJetJob* jobs, const int* small, int njobs,
                          int din, int dout, int L, hipStream_t st) {
  if (LAP) return INSR_EINVAL;
#define INSR_MULTI_S(NTV)                                                          \
  switch (S) {                                                                     \
    case 1: return launch_fwd_x6_multi<NTV, 1, false>(T, jobs, small, njobs, din, dout, L, st); \
    case 2: return launch_fwd_x6_multi<NTV, 2, false>(T, jobs, small, njobs, din, dout, L, st); \
    case 3: return launch_fwd_x6_multi<NTV, 3, false>(T, jobs, small, njobs, din, dout, L, st); \
    case 4: return launch_fwd_x6_multi<NTV, 4, false>(T, jobs, small, njobs, din, dout, L, st); \
    default: return INSR_EINVAL;                                                   \
  }
  switch (NT) {
    case 4: INSR_MULTI_S(4)
    case 8: INSR_MULTI_S(8)
    case 16: INSR_MULTI_S(16)
    default: return INSR_EWIDTH;
  }
#undef INSR_MULTI_S
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
