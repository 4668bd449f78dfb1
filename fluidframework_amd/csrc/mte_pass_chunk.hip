// The chunked pass (mte_chunk.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_chunk.h"

namespace mte {

template <int K, bool S>
hipError_t launch_chunk(const ReplayArgs& a, const ChunkArgs& ch, uint32_t n_docs, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((chunk_kernel<K, S>), dim3(n_docs), dim3(kChWaves * kWave), lds, s, a, ch);
  return hipGetLastError();
}

#define MTE_INST(K, S) \
  template hipError_t launch_chunk<K, S>(const ReplayArgs&, const ChunkArgs&, uint32_t, size_t, hipStream_t);
MTE_INST(0, false) MTE_INST(0, true) MTE_INST(4, false) MTE_INST(4, true) MTE_INST(8, false) MTE_INST(8, true)
#undef MTE_INST

}  // namespace mte
