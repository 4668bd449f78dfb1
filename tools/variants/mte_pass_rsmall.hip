// Round phases for pass-1-sized documents (mte_rsmall.h) in their own
// translation unit.
#include "mte_passes.h"
#include "mte_rsmall.h"

namespace mte {

template <int K>
hipError_t launch_rsmall(const ReplayArgs& a, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((rsmall_kernel<K>), dim3(blocks), dim3(kRsW * kWave), 0, s, a);
  return hipGetLastError();
}
template hipError_t launch_rsmall<0>(const ReplayArgs&, uint32_t, hipStream_t);
template hipError_t launch_rsmall<4>(const ReplayArgs&, uint32_t, hipStream_t);
template hipError_t launch_rsmall<8>(const ReplayArgs&, uint32_t, hipStream_t);

}  // namespace mte
