// Passes 1-3 of the flat replay (mte_replay.h, mte_stream.h) in their own
// translation unit.
#include "mte_passes.h"
#include "mte_replay.h"
#include "mte_stream.h"

namespace mte {

template <int K, bool S>
hipError_t launch_pair(const ReplayArgs& a, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((pair_kernel<K, S, kPairsPerBlock, MTE_PAIR_WAVES>), dim3(blocks), dim3(kPairsPerBlock * kWave),
                     0, s, a);
  return hipGetLastError();
}

int pass1_waves() { return MTE_PAIR_WAVES; }

template <int K, bool S>
hipError_t launch_big(const ReplayArgs& a, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((big_kernel<K, S>), dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int K, bool S>
hipError_t launch_stream(const ReplayArgs& a, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((stream_kernel<K, S>), dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

#define MTE_INST(K, S)                                                              \
  template hipError_t launch_pair<K, S>(const ReplayArgs&, uint32_t, hipStream_t); \
  template hipError_t launch_big<K, S>(const ReplayArgs&, uint32_t, hipStream_t);  \
  template hipError_t launch_stream<K, S>(const ReplayArgs&, uint32_t, hipStream_t);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST
// pass 1 with the four property planes packed into one register (kPack4)
template hipError_t launch_pair<kPack4, false>(const ReplayArgs&, uint32_t, hipStream_t);
template hipError_t launch_pair<kPack4, true>(const ReplayArgs&, uint32_t, hipStream_t);

}  // namespace mte
