// The chunked pass (mte_chunk.h) in its own translation unit.
#include "mte_passes.h"
#include "mte_chunk.h"
#include "mte_round.h"

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

hipError_t launch_round_plan(const ReplayArgs& a, const RoundArgs& rd, uint32_t n_docs, hipStream_t s) {
  hipLaunchKernelGGL(rnd_plan_kernel, dim3((n_docs + 3) / 4), dim3(256), 0, s, a, rd);
  return hipGetLastError();
}

template <int K>
hipError_t launch_round_run(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, uint32_t n_docs,
                            hipStream_t s) {
  const dim3 blk(kChWaves * kWave);
  hipLaunchKernelGGL((rnd_scatter_kernel<K>), dim3(n_docs), blk, 0, s, a, ch, rd);
  hipLaunchKernelGGL((rnd_resolve_kernel<K>), dim3(n_docs), blk, 0, s, a, ch, rd);
  const uint64_t waves = (uint64_t)n_docs * ch.nch_cap;
  hipLaunchKernelGGL((rnd_apply_kernel<K>), dim3((uint32_t)((waves + 3) / 4)), dim3(4 * kWave), 0, s, a, ch, rd);
  hipLaunchKernelGGL((rnd_gather_kernel<K>), dim3(n_docs), blk, 0, s, a, ch, rd);
  return hipGetLastError();
}
template hipError_t launch_round_run<0>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);
template hipError_t launch_round_run<4>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);
template hipError_t launch_round_run<8>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);

}  // namespace mte
