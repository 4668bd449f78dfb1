// The HBM tree pass (mte_htree.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_htree.h"

namespace mte {

template <int K, bool S>
hipError_t launch_htree(const ReplayArgs& a, const HtreeArgs& t, hipStream_t s) {
  if (!t.n_docs) return hipSuccess;
  // dynamic LDS: (nP + 5) words per item of lcap (ht_to_lds), nP of a local-client document
  const size_t lds = t.lcap ? ((size_t)(kLocalPlanes<K> + 5) * t.lcap + 2) * 4 : 0;
  if (t.maint) hipLaunchKernelGGL((htree_kernel<K, S, true>), dim3(t.n_docs), dim3(kWave), lds, s, a, t);
  else hipLaunchKernelGGL((htree_kernel<K, S, false>), dim3(t.n_docs), dim3(kWave), lds, s, a, t);
  return hipGetLastError();
}

#define MTE_INST(K, S) template hipError_t launch_htree<K, S>(const ReplayArgs&, const HtreeArgs&, hipStream_t);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST

}  // namespace mte
