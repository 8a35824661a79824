// jet_x6_fwd.hpp -- launch + dispatch templates of the split-bf16 forward (jet_x6.hpp),
// instantiated per precision (NQ) by jet_x6_fwd.hip (NQ = 3) and jet_bf_fwd.hip (NQ = 1, 2).
#pragma once
#include "jet_x6.hpp"

namespace insr {

// T in {1, 2, 4}; the balanced modes add T = 3 (2-3 stream jets) and T = 5 (value jets) at W <= 128
template <int NQ, int NT, int S, bool LAP>
int launch_fwd_x6(int T, const float* x, int N, int din, int dout, int L, const float* prm, float* y, float* dy,
                  float* lap, float* act, int nbal, hipStream_t st) {
  switch (T) {
    case 1: return launch_fwd_x6_t<NQ, NT, S, LAP, 1>(x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);
    case 2: return launch_fwd_x6_t<NQ, NT, S, LAP, 2>(x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);
    case 4: return launch_fwd_x6_t<NQ, NT, S, LAP, 4>(x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);
    case 3:
      if constexpr (NT <= 8 && (S == 2 || S == 3) && !LAP)
        return launch_fwd_x6_t<NQ, NT, S, LAP, 3>(x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);
      return INSR_EINVAL;
    case 5:
      if constexpr (NT <= 8 && S == 1)
        return launch_fwd_x6_t<NQ, NT, S, LAP, 5>(x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);
      return INSR_EINVAL;
    default: return INSR_EINVAL;
  }
}

template <int NQ, int NT, int S, bool LAP>
int launch_fwd_x6_multi(int T, const InsrJetJob* jobs, const int* small, const int* nbal, int njobs, int din,
                        int dout, int L, hipStream_t st) {
  switch (T) {
    case 1: return launch_fwd_x6_multi_t<NQ, NT, S, LAP, 1>(jobs, small, nbal, njobs, din, dout, L, st);
    case 2: return launch_fwd_x6_multi_t<NQ, NT, S, LAP, 2>(jobs, small, nbal, njobs, din, dout, L, st);
    case 4: return launch_fwd_x6_multi_t<NQ, NT, S, LAP, 4>(jobs, small, nbal, njobs, din, dout, L, st);
    case 5:
      if constexpr (NT <= 8 && S == 1)
        return launch_fwd_x6_multi_t<NQ, NT, S, LAP, 5>(jobs, small, nbal, njobs, din, dout, L, st);
      return INSR_EINVAL;
    default: return INSR_EINVAL;
  }
}

// value and gradient jets (the fused pairs the models issue are value jets; the Laplacian
// jet is never paired), widths 64 / 128 / 256
template <int NQ>
int dispatch_fwd_multi_q(int NT, int S, bool LAP, int T, const InsrJetJob* jobs, const int* small, const int* nbal,
                         int njobs, int din, int dout, int L, hipStream_t st) {
  if (LAP) return INSR_EINVAL;
#define INSR_MULTI_S(NTV)                                                                        \
  switch (S) {                                                                                   \
    case 1: return launch_fwd_x6_multi<NQ, NTV, 1, false>(T, jobs, small, nbal, njobs, din, dout, L, st); \
    case 2: return launch_fwd_x6_multi<NQ, NTV, 2, false>(T, jobs, small, nbal, njobs, din, dout, L, st); \
    case 3: return launch_fwd_x6_multi<NQ, NTV, 3, false>(T, jobs, small, nbal, njobs, din, dout, L, st); \
    case 4: return launch_fwd_x6_multi<NQ, NTV, 4, false>(T, jobs, small, nbal, njobs, din, dout, L, st); \
    default: return INSR_EINVAL;                                                                 \
  }
  switch (NT) {
    case 4: INSR_MULTI_S(4)
    case 8: INSR_MULTI_S(8)
    case 16: INSR_MULTI_S(16)
    default: return INSR_EWIDTH;
  }
#undef INSR_MULTI_S
}

// mixed-mode fused forward (W = 128 only: the tile policy it encodes is the W = 128 one)
template <int NQ>
int dispatch_fwd_mixed_q(int NT, int din, const InsrJetJob* jobs, const int* modes, const float* scalars, int njobs,
                         int dout, int L, hipStream_t st) {
  if (NT != 8) return INSR_EWIDTH;
  int need = 0;
  for (int k = 0; k < njobs; ++k) need |= 1 << modes[k];
  // the smallest compiled body set that covers the jobs
#define INSR_MIX_DIN(B)                                                                  \
  switch (din) {                                                                         \
    case 1: return launch_fwd_x6_mixed_t<NQ, 8, 1, B>(jobs, modes, scalars, njobs, dout, L, st); \
    case 2: return launch_fwd_x6_mixed_t<NQ, 8, 2, B>(jobs, modes, scalars, njobs, dout, L, st); \
    case 3: return launch_fwd_x6_mixed_t<NQ, 8, 3, B>(jobs, modes, scalars, njobs, dout, L, st); \
    default: return INSR_EINVAL;                                                         \
  }
  if ((need & ~(kMixV | kMixA)) == 0) INSR_MIX_DIN(kMixV | kMixA)
  if ((need & ~(kMixV | kMixG)) == 0) INSR_MIX_DIN(kMixV | kMixG)
  if ((need & ~(kMixG | kMixL)) == 0) INSR_MIX_DIN(kMixG | kMixL)
  INSR_MIX_DIN(kMixV | kMixG | kMixL | kMixA)
#undef INSR_MIX_DIN
}

template <int NQ>
int dispatch_fwd_q(int NT, int S, bool LAP, int T, const float* x, int N, int din, int dout, int L,
                   const float* prm, float* y, float* dy, float* lap, float* act, int nbal, hipStream_t st) {
#define INSR_FWD_Q(NTV)                                                                                  \
  switch (S * 2 + (LAP ? 1 : 0)) {                                                                       \
    case 2: return launch_fwd_x6<NQ, NTV, 1, false>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);    \
    case 4: return launch_fwd_x6<NQ, NTV, 2, false>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);    \
    case 6: return launch_fwd_x6<NQ, NTV, 3, false>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);    \
    case 8: return launch_fwd_x6<NQ, NTV, 4, false>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);    \
    case 7: return launch_fwd_x6<NQ, NTV, 3, true>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);     \
    case 9: return launch_fwd_x6<NQ, NTV, 4, true>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);     \
    case 11: return launch_fwd_x6<NQ, NTV, 5, true>(T, x, N, din, dout, L, prm, y, dy, lap, act, nbal, st);    \
    default: return INSR_EINVAL;                                                                         \
  }
  switch (NT) {
    case 2: INSR_FWD_Q(2)
    case 4: INSR_FWD_Q(4)
    case 8: INSR_FWD_Q(8)
    case 16: INSR_FWD_Q(16)
    default: return INSR_EWIDTH;
  }
#undef INSR_FWD_Q
}

}  // namespace insr
