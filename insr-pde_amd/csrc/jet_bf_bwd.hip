// jet_bf_bwd.hip -- the reduced-precision backward jets (NQ = 2 "x3", NQ = 1 bf16).
#include "jet_x6_bwd.hpp"

namespace insr {
template int dispatch_bwd_q<1>(int, int, bool, int, const BwdJobsX6*, int, int, int, const float*, float*, long,
                               hipStream_t);
template int dispatch_bwd_q<2>(int, int, bool, int, const BwdJobsX6*, int, int, int, const float*, float*, long,
                               hipStream_t);
}  // namespace insr
