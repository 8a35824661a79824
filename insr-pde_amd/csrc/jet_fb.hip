// jet_fb.hip -- the recompute backward (jet_fb.hpp): W = 128, 4 hidden layers (the fluid nets:
// velocity 2 -> 2, pressure 2 -> 1), products f16x3 (fp32-level) with per-tile power-of-two scales.
#include "jet_fb.hpp"

namespace insr {

// (S, LAP) served: the 2-d Laplacian jet (S = 4), the 2-d gradient jet (S = 3), the value jet (S = 1);
// ZR = hidden layers whose z-streams stay in registers (the rest in LDS)
bool fb_supported(int S, bool LAP, int L) {
  if (L != 4) return false;
  return (S == 4 && LAP) || (S == 3 && !LAP) || (S == 1 && !LAP);
}
// the saved-stream sweep also serves the 2-d gradient jet of 5 hidden layers (round 6: the
// elasticity2Dstretch deformation net's Jacobian, elasticity/model.py:143; 255 VGPRs, no spills)
bool fb_saved_supported(int S, bool LAP, int L) { return fb_supported(S, LAP, L) || (L == 5 && S == 3 && !LAP); }

// saved = 0: the recompute backward (reruns the forward per tile); 1: the same reverse sweep on the
// forward's saved streams (J.act) -- dW resident per CU, f16x3 products, no z̄ round trip
int dispatch_fb_bwd(int S, bool LAP, int L, const FbJobs& J, int din, int dout, const float* prm, float* work,
                    float* grad, int accumulate, int saved, int phases, const AdamArgs& A, hipStream_t st) {
  if (L == 5) {
    if (S == 3 && !LAP && saved) return fb_bwd_t<3, false, 5, 1, true>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    return INSR_EINVAL;
  }
  if (!fb_supported(S, LAP, L)) return INSR_EINVAL;
  switch ((S * 2 + (LAP ? 1 : 0)) * 2 + (saved ? 1 : 0)) {
    case 18: return fb_bwd_t<4, true, 4, 2, false>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    case 12: return fb_bwd_t<3, false, 4, 2, false>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    case 4: return fb_bwd_t<1, false, 4, 4, false>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    case 19: return fb_bwd_t<4, true, 4, 1, true>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    case 13: return fb_bwd_t<3, false, 4, 1, true>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    case 5: return fb_bwd_t<1, false, 4, 1, true>(J, din, dout, prm, work, grad, accumulate, phases, A, st);
    default: return INSR_EINVAL;
  }
}

long fb_work_floats(long tiles, int din, int dout, int L) { return fb_work_floats_impl(tiles, din, dout, L); }
int fb_launch_blocks(long tiles) { return fb_blocks(tiles); }

}  // namespace insr

#ifdef INSR_STAMPS
// diagnostic build only: the recompute kernel's phase stamps of its last launch
extern "C" int insr_diag_fb_stamps(unsigned long long* out, int n) {
  const int m = n < 8 * 8 * insr::kFbStampPts ? n : 8 * 8 * insr::kFbStampPts;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(insr::g_fb_stamps), (size_t)m * sizeof(unsigned long long));
}
#endif

namespace insr {

}  // namespace insr
