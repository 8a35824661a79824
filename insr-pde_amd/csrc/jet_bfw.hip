// jet_bfw.hip -- the two-kernel backward (jet_x6w.hpp) at reduced precision (NQ = 2, 1).
#include "jet_x6w.hpp"

namespace insr {
template int dispatch_wide_bwd_q<1>(int, int, bool, const FbJobs&, int, int, int, int, const float*, float*, float*, int, int, int,
                                    const AdamArgs&, hipStream_t);
template int dispatch_wide_bwd_q<2>(int, int, bool, const FbJobs&, int, int, int, int, const float*, float*, float*, int, int, int,
                                    const AdamArgs&, hipStream_t);
}  // namespace insr
