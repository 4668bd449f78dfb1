// The chunked pass (mte_chunk.h) in its own translation unit.
#include <algorithm>
#include <cstdio>

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

hipError_t launch_round_plan(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, uint32_t n_docs,
                             hipStream_t s) {
  hipLaunchKernelGGL(rnd_plan_kernel, dim3(n_docs), dim3(kChWaves * kWave), 0, s, a, ch, rd);
  return hipGetLastError();
}

template <int K>
static void round_gather(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, hipStream_t s) {
  const uint64_t chunks = (uint64_t)rd.nd * ch.nch_cap;
  hipLaunchKernelGGL(rnd_gscan_kernel, dim3(rd.nd), dim3(kChWaves * kWave), 0, s, a, ch, rd);
  hipLaunchKernelGGL((rnd_gmove_kernel<K>), dim3((uint32_t)std::min<uint64_t>((chunks + 3) / 4, 2048)), dim3(4 * kWave),
                     0, s, a, ch, rd);
}

template <int K>
hipError_t launch_round_gather(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, int final,
                               hipStream_t s) {
  hipLaunchKernelGGL(rnd_live_kernel, dim3(rd.nd), dim3(256), 0, s, a, ch, rd, final);
  round_gather<K>(a, ch, rd, s);
  return hipGetLastError();
}

template <int K>
hipError_t launch_round_run(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, uint32_t,
                            hipStream_t s) {
#if MTE_RND_DIAG
  {  // the counters so far (diagnostic builds)
    unsigned long long h[16] = {};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rnd_diag), sizeof h) == hipSuccess)
      fprintf(stderr,
              "rnd_diag blocks %llu serial %llu ops %llu clk_block %llu clk_gather %llu clk_serial %llu recs %llu "
              "back %llu find %llu fwd %llu out %llu apply_waves %llu apply_load %llu apply_ops %llu apply_subops %llu "
              "apply_head %llu\n",
              h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12], h[13], h[14], h[15]);
  }
#endif
  const uint32_t n_docs = rd.nd;  // this launch's slice of the documents
  const uint32_t tpd = (a.cap + kT - 1) / kT;  // flat tiles per document
  const uint64_t tiles = (uint64_t)n_docs * tpd, chunks = (uint64_t)n_docs * ch.nch_cap;
  const dim3 w4(4 * kWave);
  // documents whose carried chunks go back to the flat planes first (their run
  // is not a round, or a chunk is full: the latter are re-laid out below)
  hipLaunchKernelGGL(rnd_live_kernel, dim3(n_docs), dim3(256), 0, s, a, ch, rd, 0);
  round_gather<K>(a, ch, rd, s);
  // re-layout of the documents the arena does not hold: flat -> chunks (zamboni
  // at M); then every round document's round-start column
  hipLaunchKernelGGL((rnd_count_kernel<K>), dim3((uint32_t)((tiles + 3) / 4)), w4, 0, s, a, ch, rd, tpd);
  hipLaunchKernelGGL(rnd_scan_kernel, dim3(n_docs), dim3(kChWaves * kWave), 0, s, a, ch, rd, 0);
  hipLaunchKernelGGL((rnd_move_kernel<K>), dim3((uint32_t)((tiles + 3) / 4)), w4, 0, s, a, ch, rd, tpd);
  // a fixed grid walking the chunk slots (rnd_cols skips a carried document's)
  hipLaunchKernelGGL(rnd_cols_kernel, dim3((uint32_t)std::min<uint64_t>((chunks + 3) / 4, 2048)), w4, 0, s, a, ch, rd);
  // resolve: the client chains, columns in LDS (two waves per workgroup when they fit)
  const size_t col = (size_t)rnd_resolve_lds(rd.col_cap, rd.col_cap / kChGroup);
  if (2 * col <= kRoundLdsMax) {
    hipError_t e = hipFuncSetAttribute((const void*)rnd_resolve_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(2 * col));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rnd_resolve_kernel<2>, dim3(n_docs * (kChWaves / 2)), dim3(2 * kWave), 2 * col, s, a, ch, rd);
  } else {
    hipError_t e = hipFuncSetAttribute((const void*)rnd_resolve_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)col);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rnd_resolve_kernel<1>, dim3(n_docs * kChWaves), dim3(kWave), col, s, a, ch, rd);
  }
  // (the resolve wrote each sub-op into its chunk's bucket: rnd_emit)
  hipLaunchKernelGGL(rnd_room_kernel, dim3((uint32_t)((chunks + 255) / 256)), dim3(256), 0, s, a, ch, rd);
  // apply: every chunk with sub-ops on its own wave
  {  // a fixed grid (rnd_apply_kernel walks the chunk slots): 2 workgroups per SIMD's worth
    const uint32_t g = (uint32_t)std::min<uint64_t>((chunks + 3) / 4, 2048);
    hipLaunchKernelGGL((rnd_apply_kernel<K>), dim3(g), w4, 0, s, a, ch, rd);
  }
  // the header past the run (the segments stay in the arena); the refused runs'
  // carried documents back to the flat planes
  hipLaunchKernelGGL(rnd_scan_kernel, dim3(n_docs), dim3(kChWaves * kWave), 0, s, a, ch, rd, 1);
  hipLaunchKernelGGL(rnd_post_kernel, dim3((n_docs + 63) / 64), dim3(64), 0, s, a, ch, rd);
  round_gather<K>(a, ch, rd, s);
  return hipGetLastError();
}
template hipError_t launch_round_run<0>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);
template hipError_t launch_round_gather<0>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, int, hipStream_t);
template hipError_t launch_round_gather<4>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, int, hipStream_t);
template hipError_t launch_round_gather<8>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, int, hipStream_t);
template hipError_t launch_round_run<4>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);
template hipError_t launch_round_run<8>(const ReplayArgs&, const ChunkArgs&, const RoundArgs&, uint32_t, hipStream_t);

}  // namespace mte
