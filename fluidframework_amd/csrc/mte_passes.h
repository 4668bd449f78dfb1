// mte_passes.h — host launchers of the replay passes.  Each pass lives in its
// own translation unit (mte_pass_tree.hip, mte_pass_flat.hip,
// mte_pass_chunk.hip) so the passes compile in parallel and one can be rebuilt
// alone; mte_engine.hip drives them (launch_replay).
#pragma once

#include <hip/hip_runtime.h>

#include "mte_kernels.h"

namespace mte {

struct ReplayArgs;
struct TreeArgs;
struct HtreeArgs;
struct ChunkArgs;

// round phases of the chunked pass (mte_round.h)
constexpr int kRB = 62;              // sub-ops per chunk and run: 128 + 2 x 62 slots <= 254
constexpr uint32_t kRoundMin = 256;  // the shortest run the round phases take
constexpr int kMaxPhases = 16;       // phases per launch before the rest runs op after op
// a document's chunks stay laid out from one run to the next (rnd_live) while
// no chunk holds more than this many segments; a run whose sub-ops would not
// fit a carried chunk (count + 2 per sub-op > kChSlots) is re-laid out and run
// again in the next phase
constexpr uint32_t kLiveFull = 192;
struct RoundArgs {
  uint4* plan;      // [doc] x mode, y k0, z k1, w M
  uint32_t* rcnt;   // [doc][nch_cap] sub-ops per chunk
  uint2* rbuf;      // [doc][nch_cap][kRB] (op index - k0, chunk start in the op's perspective)
  uint4* rrec;      // [doc][nch_cap][kRB][2] the sub-op's record, copied there by the resolve (rnd_emit)
  uint32_t* rflag;  // [doc] non-zero: the run replays op after op
  uint32_t* nch;    // [doc] chunks after the re-layout
  uint32_t* nnew;   // [doc] segments after the re-layout
  uint32_t* count;  // [0] round docs, [1] op-after-op docs, [2] active docs
  uint2* rchain;    // [doc][MTE_MAX_CLIENTS] (list offset, entries) of each client chain
  // [doc] where the document's segments are: 0 the flat planes; 1 the chunk
  // arena, carried from the previous run (the flat planes are stale); 2 the
  // arena, re-laid out for this run
  uint32_t* live;
  uint32_t* gfl;    // [doc] 1: this launch gathers the arena back into the flat planes
  uint32_t last;    // this phase sends every active document op after op
  uint32_t col_cap; // chunks a resolve column holds (the phase's largest document, rounded to 64: rnd_plan's count[3])
  uint32_t d0, nd;  // the documents [d0, d0 + nd) one launch_round_run covers
  // [doc] the bytes the round phases of the last mte_run had to read and write
  // (their algorithmic bytes: records, planes re-laid out / applied /
  // gathered, sub-op lists), added per document and phase; planes = the
  // segment planes a move carries (kFieldPlanes + K)
  unsigned long long* acct;
  uint32_t planes;
};
// the round phases fit a context whose per-wave column (nch_cap + ng_cap
// entries, mte_round.h rnd_resolve_kernel) fits this much LDS
constexpr uint32_t kRoundLdsMax = 150u * 1024u;
// the documents leaving the arena (their next run is not a round, a chunk is
// full, or final: every one) gathered back into the flat planes
template <int K>
hipError_t launch_round_gather(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, int final,
                               hipStream_t s);
inline uint64_t rnd_resolve_lds(uint32_t nch_cap, uint32_t ng_cap) {
  return (uint64_t)(nch_cap + 2 * ((ng_cap + 63) / 64 * 64) + 64 + 1024) * 4u;  // + GD rows, the staging ring (kRing)
}

// the tree pass over the legacy documents (mte_tree.h): `rounds` of TIER 0
// (E <= 2) / TIER 1 (E = 4), then TIER 2 (E = 8, 16)
template <int K, bool S>
hipError_t launch_tree(const ReplayArgs& a, const TreeArgs& t, uint32_t blocks, hipStream_t s, int rounds,
                       uint32_t per_round);
// the HBM tree pass (mte_htree.h): one wavefront per candidate document
template <int K, bool S>
hipError_t launch_htree(const ReplayArgs& a, const HtreeArgs& t, hipStream_t s);
// pass 1 (ReplayArgs::group documents per wavefront) and pass 2 (one per
// wavefront); pass1_waves() = the waves per SIMD pass 1's register budget is
// built for (the host sizes the groups so the batch is resident at once)
template <int K, bool S>
hipError_t launch_pair(const ReplayArgs& a, uint32_t blocks, hipStream_t s);
int pass1_waves();
template <int K, bool S>
hipError_t launch_big(const ReplayArgs& a, uint32_t blocks, hipStream_t s);
// pass 3: HBM-streamed (mte_stream.h) or chunked (mte_chunk.h)
template <int K, bool S>
hipError_t launch_stream(const ReplayArgs& a, uint32_t blocks, hipStream_t s);
template <int K, bool S>
hipError_t launch_chunk(const ReplayArgs& a, const ChunkArgs& ch, uint32_t n_docs, size_t lds, hipStream_t s);
// the round phases: plan, then (scatter, resolve, apply, gather) for the
// documents the plan gives a run
hipError_t launch_round_plan(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, uint32_t n_docs,
                             hipStream_t s);
template <int K>
hipError_t launch_round_run(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, uint32_t n_docs,
                            hipStream_t s);

}  // namespace mte
