// jet_x6r.hip -- the resident-dW backward (jet_x6r.hpp) at fp32-level accuracy (NQ = 3), W = 128,
// 4 hidden layers (the fluid nets: velocity 2 -> 2, pressure 2 -> 1).
#include "jet_x6r.hpp"

namespace insr {

template <int RPW>
static int resident_rpw(int S, bool LAP, const float* x, int N, int din, int dout, const float* prm, const float* act,
                        const float* gy, const float* gdy, const float* glap, float* work, float* grad, int accumulate,
                        hipStream_t st) {
  switch (S * 2 + (LAP ? 1 : 0)) {
    case 2: return resident_bwd_t<3, 1, false, 4, RPW>(x, N, din, dout, prm, act, gy, gdy, glap, work, grad, accumulate, st);
    case 6: return resident_bwd_t<3, 3, false, 4, RPW>(x, N, din, dout, prm, act, gy, gdy, glap, work, grad, accumulate, st);
    case 9: return resident_bwd_t<3, 4, true, 4, RPW>(x, N, din, dout, prm, act, gy, gdy, glap, work, grad, accumulate, st);
    default: return INSR_EINVAL;
  }
}

// 8-wave blocks (one row tile per wave, two waves per SIMD).  4-wave blocks (two row tiles per
// wave, the dW of 32 rows per wave in AGPRs, one wave per SIMD) measured slower on every size
// (r3b: headline 55.7 vs 68.5 M pts/s, fluid2DtlgnM 84.1 vs 102.1) and are not instantiated.
int dispatch_resident_bwd(int S, bool LAP, int L, const float* x, int N, int din, int dout, const float* prm,
                          const float* act, const float* gy, const float* gdy, const float* glap, float* work,
                          float* grad, int accumulate, hipStream_t st) {
  if (L != 4) return INSR_EINVAL;
  return resident_rpw<1>(S, LAP, x, N, din, dout, prm, act, gy, gdy, glap, work, grad, accumulate, st);
}

long resident_work_floats(long n, int din, int dout, int L) { return x6r_work_floats(n, din, dout, L); }
int resident_blocks(long n) { return x6r_blocks(n); }

}  // namespace insr
