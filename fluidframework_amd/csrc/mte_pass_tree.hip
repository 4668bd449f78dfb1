// The tree pass (mte_tree.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_tree.h"

namespace mte {

// TIER 0 / TIER 1 alternate `rounds` times; round r lets every document run
// up to op (r + 1) * per_round of the batch, so a document that briefly
// outgrows TIER 0 waits for at most one round's share of the others instead of
// the whole batch (the last round has no cap and its TIER 1 keeps its
// documents), then TIER 2.
template <int K, bool S>
hipError_t launch_tree(const ReplayArgs& a, const TreeArgs& t, uint32_t blocks, hipStream_t s, int rounds,
                       uint32_t per_round) {
  hipError_t e;
  for (int r = 0; r < rounds; r++) {
    TreeArgs tr = t;
    tr.final_round = r + 1 == rounds;
    tr.k_cap = tr.final_round ? 0xffffffffu : (uint32_t)(r + 1) * per_round;
    hipLaunchKernelGGL((tree_kernel<K, S, 0>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, tr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL((tree_kernel<K, S, 1>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, tr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  TreeArgs tb = t;
  tb.k_cap = 0xffffffffu;
  hipLaunchKernelGGL((tree_kernel<K, S, 2>), dim3(blocks), dim3(kDocsPerBlock * kWave), 0, s, a, tb);
  return hipGetLastError();
}

#define MTE_INST(K, S) \
  template hipError_t launch_tree<K, S>(const ReplayArgs&, const TreeArgs&, uint32_t, hipStream_t, int, uint32_t);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST

}  // namespace mte
