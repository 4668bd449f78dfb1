// The tree pass (mte_tree.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_tree.h"

namespace mte {

template <int K, bool S>
hipError_t launch_tree(const ReplayArgs& a, const TreeArgs& t, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((tree_kernel<K, S, 0>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, t);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tree_kernel<K, S, 1>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, t);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((tree_kernel<K, S, 2>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, t);
  return hipGetLastError();
}

#define MTE_INST(K, S) template hipError_t launch_tree<K, S>(const ReplayArgs&, const TreeArgs&, uint32_t, hipStream_t);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST

}  // namespace mte
