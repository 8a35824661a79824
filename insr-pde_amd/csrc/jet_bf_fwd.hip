// jet_bf_fwd.hip -- the reduced-precision forward jets: NQ = 2 ("x3", 3 bf16 products per
// fp32 product) and NQ = 1 (plain bf16 operands, fp32 accumulation).
#include "jet_x6_fwd.hpp"

namespace insr {
template int dispatch_fwd_q<1>(int, int, bool, int, const float*, int, int, int, int, const float*, float*, float*,
                               float*, float*, int, hipStream_t);
template int dispatch_fwd_multi_q<1>(int, int, bool, int, const InsrJetJob*, const int*, const int*, int, int, int,
                                     int, hipStream_t);
template int dispatch_fwd_q<2>(int, int, bool, int, const float*, int, int, int, int, const float*, float*, float*,
                               float*, float*, int, hipStream_t);
template int dispatch_fwd_multi_q<2>(int, int, bool, int, const InsrJetJob*, const int*, const int*, int, int, int,
                                     int, hipStream_t);
template int dispatch_fwd_mixed_q<1>(int, int, const InsrJetJob*, const int*, const float*, int, int, int,
                                     hipStream_t);
template int dispatch_fwd_mixed_q<2>(int, int, const InsrJetJob*, const int*, const float*, int, int, int,
                                     hipStream_t);
}  // namespace insr
