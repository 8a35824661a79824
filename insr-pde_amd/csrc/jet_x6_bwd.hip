// jet_x6_bwd.hip -- the split-bf16 backward at fp32-level accuracy (NQ = 3, "x6").
#include "jet_x6_bwd.hpp"

namespace insr {
template int dispatch_bwd_q<3>(int, int, bool, int, const BwdJobsX6*, int, int, int, const float*, float*, long,
                               hipStream_t);
}  // namespace insr

#ifdef INSR_STAMPS
// diagnostic build only (make diag): the x6 backward's phase stamps (this translation unit's copy)
extern "C" int insr_diag_stamps_x6(unsigned long long* host, int n) {
  if (n > insr::kStampSlots) n = insr::kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(insr::g_insr_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
