// jet_h_bwd.hip -- the fused tile-split backward with its products on the fp16 matrix cores
// (NQ = 4, f16x3 with power-of-two adjoint scales: the x6 backward under INSR_BWD_F16_FUSED).
#include "jet_x6_bwd.hpp"

namespace insr {
template int dispatch_bwd_q<4>(int, int, bool, int, const BwdJobsX6*, int, int, int, const float*, float*, long,
                               hipStream_t);
}  // namespace insr
