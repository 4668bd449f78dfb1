// The tree pass (mte_tree.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_tree.h"

namespace mte {

// TIER 0 / TIER 1 alternate `rounds` times (documents move between them as
// they grow and shrink; the last TIER 1 keeps its documents), then TIER 2.
template <int K, bool S>
hipError_t launch_tree(const ReplayArgs& a, const TreeArgs& t, uint32_t blocks, hipStream_t s, int rounds) {
  hipError_t e;
  for (int r = 0; r < rounds; r++) {
    TreeArgs tr = t;
    tr.final_round = r + 1 == rounds;
    hipLaunchKernelGGL((tree_kernel<K, S, 0>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, tr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((tree_kernel<K, S, 1>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, tr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  hipLaunchKernelGGL((tree_kernel<K, S, 2>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, t);
  return hipGetLastError();
}

#define MTE_INST(K, S) \
  template hipError_t launch_tree<K, S>(const ReplayArgs&, const TreeArgs&, uint32_t, hipStream_t, int);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST

}  // namespace mte
