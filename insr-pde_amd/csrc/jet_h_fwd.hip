// jet_h_fwd.hip -- the fp16 two-term forward at fp32-level accuracy (NQ = 4, "f16x3": three
// v_mfma_f32_16x16x32_f16 products per K chunk, jet_x6.hpp).  Forward only: its backward runs
// the split-bf16 x6 kernels (capi.hip call_prec).
#include "jet_x6_fwd.hpp"

namespace insr {
template int dispatch_fwd_q<4>(int, int, bool, int, const float*, int, int, int, int, const float*, float*, float*,
                               float*, float*, int, hipStream_t);
template int dispatch_fwd_multi_q<4>(int, int, bool, int, const InsrJetJob*, const int*, const int*, int, int, int,
                                     int, hipStream_t);
template int dispatch_fwd_mixed_q<4>(int, int, const InsrJetJob*, const int*, const float*, int, int, int,
                                     hipStream_t);
}  // namespace insr
