// jet_x6_fwd.hip -- the split-bf16 forward at fp32-level accuracy (NQ = 3, "x6").
#include "jet_x6_fwd.hpp"

namespace insr {
template int dispatch_fwd_q<3>(int, int, bool, int, const float*, int, int, int, int, const float*, float*, float*,
                               float*, float*, int, hipStream_t);
template int dispatch_fwd_multi_q<3>(int, int, bool, int, const InsrJetJob*, const int*, const int*, int, int, int,
                                     int, hipStream_t);
template int dispatch_fwd_mixed_q<3>(int, int, const InsrJetJob*, const int*, const float*, int, int, int,
                                     hipStream_t);
}  // namespace insr
