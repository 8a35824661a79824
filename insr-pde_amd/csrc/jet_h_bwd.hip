// jet_h_bwd.hip -- the fused tile-split backward with its products on the fp16 matrix cores
// (NQ = 4, f16x3 with power-of-two adjoint scales: the x6 backward under INSR_BWD_F16_FUSED).
#include "jet_x6_bwd.hpp"

namespace insr {
template int dispatch_bwd_q<4>(int, int, bool, int, const BwdJobsX6*, int, int, int, const float*, float*, long,
                               hipStream_t);
}  // namespace insr

#ifdef INSR_STAMPS
// diagnostic build only (make diag): the f16x3 fused backward's phase stamps (this translation unit's copy)
extern "C" int insr_diag_stamps_h(unsigned long long* host, int n) {
  if (n > insr::kStampSlots) n = insr::kStampSlots;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(insr::g_insr_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
