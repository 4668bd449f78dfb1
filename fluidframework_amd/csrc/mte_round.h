// mte_round.h — round phases of the chunked pass (mte_chunk.h): a run of
// concurrent ops replayed chunk-parallel instead of op after op.
//
// A *run* of a document is a stretch of ops k0 .. k1 - 1 that all carry
// refSeq R = the document's currentSeq at k0 and one minSeq M (every op of a
// conflict-farm round: BASELINE config 5).  Within a run the perspective of an
// op of client c is the state at k0 plus c's own earlier ops of the run: every
// other client's insert of the run is invisible to it (seq > R) and every other
// client's remove of the run leaves its segments visible (removedSeq > R).  So
//   * client c's chunk length column (mte_chunk.h: sum[c][i], the chunk-level
//     PartialSequenceLengths.getPartialLength, partialLengths.ts:667-702)
//     changes only by c's own ops — by +inserted units and -the units a remove
//     covers, arithmetic on the column with no segment in sight — and starts
//     from the same round-start column for every client;
//   * so each client's ops resolve to (chunk, the chunk's start in the op's
//     perspective) on their own column, all clients at once (rnd_resolve: one
//     wave per client chain);
//   * an op changes only the chunks it resolved to, and what it does to a chunk
//     depends only on that chunk's content (the segment step seg_op_v, with the
//     op's positions taken relative to the chunk start, as the sequential chunk
//     pass runs it), so replaying every chunk's ops in seq order — each chunk
//     on its own wave, all chunks at once (rnd_apply) — gives every chunk the
//     content the op-after-op replay gives it.
// An insert goes to the chunk holding the unit before its position (the first
// chunk for position 0) and appends there if no slot of that chunk follows
// the position: in a new-length-calc run no segment is undefined to the
// perspective (tombstones with removedSeq <= M are dropped at the re-layout,
// those of the run have removedSeq > R >= M), so the end of chunk i is the
// place the op-after-op pass reaches at the start of chunk i + 1
// (insertingWalk's "before the first leaf at or after pos", mergeTree.ts:1743,
// 1788-1797).  minSeq moves to M before the run instead of after its first op:
// tombstones at or below M are zero-length to every op of the run, so the op
// lands in the same place relative to every segment that stays.
//
// Phases per launch of the chunked pass (host loop, mte_engine.hip):
//   rnd_plan     a workgroup per document: the run at its op cursor (mode kRound
//                if long enough, else the rest goes to the sequential pass);
//   re-layout    flat planes -> chunks of kChFill segments, dropping
//                removedSeq <= M (zamboni, mergeTree.ts:1077-1093): keep
//                counts per 256-slot tile (rnd_count, a wave per tile), their
//                prefix per document (rnd_scan), the moves (rnd_move, a wave
//                per tile), then per chunk its count and round-start column
//                entry, the visible length (rnd_cols, a wave per chunk);
//   rnd_resolve  one wave per client chain, its column in LDS: positions ->
//                (chunk, start), each sub-op written into its chunk's bucket
//                with its record (rnd_emit);
//   rnd_apply    one wave per chunk with sub-ops: sort them by op index, load
//                the chunk into registers, seg_op_v each, store;
//   gather       chunk counts -> prefix (rnd_scan), chunks -> flat planes
//                (rnd_gmove, a wave per chunk), the header advanced to k1.
// Anything the run cannot take — an insert past the end (the op-after-op pass
// reports MTE_E_INSERT_FAILED at that op), a bucket over kRB sub-ops — sets
// the document's flag before any segment is written, and the sequential chunk
// pass replays the same run from the untouched flat planes.  Statistics runs
// (mte_set_stats) always take the sequential pass.
#pragma once

#include "mte_chunk.h"
#include "mte_passes.h"

namespace mte {

// segments per chunk a re-layout aims at (measured: 128 beats 96 / 80 / 64 --
// more chunks cost the apply more waves than the narrower registers save); the
// chunk count stays within nch_cap, the fill is total / chunks rounded up (rnd_fill)
#ifndef MTE_RND_FILL
#define MTE_RND_FILL 128
#endif

// diagnostic builds (tools/variants.sh ...:"-DMTE_RND_DIAG=1"): per resolve
// [0] blocks, [1] blocks sent op by op, [2] ops, [3] clocks in blocks,
// [4] clocks gathering, [5] clocks in the serial fallback, in rnd_block [6]
// to the records, [7] back pass, [8] search, [9] forward pass, [10] outputs
// and fold; printed per launch
#ifndef MTE_RND_DIAG
#define MTE_RND_DIAG 0
#endif
#if MTE_RND_DIAG
__device__ unsigned long long g_rnd_diag[16];
#define RND_DIAG(i, v) \
  do {                                                                           \
    if (lane_id() == 0) atomicAdd(&g_rnd_diag[i], (unsigned long long)(v));     \
  } while (0)
#define RND_CLK(t) const long long t = clock64()
#else
#define RND_DIAG(i, v) \
  do {                 \
  } while (0)
#define RND_CLK(t)
#endif

__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// the resolve's column and ring live in the wave's own LDS, whose operations
// complete in issue order: ordering them needs a compiler barrier and the LDS
// counter only -- not fence_wave's vmcnt(0), which would wait out the sub-op
// list stores and the records in flight
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// one workgroup per document: its 8 waves scan the records from the cursor
// in interleaved batches of 64 for the first op that ends the run
__global__ __launch_bounds__(512) void rnd_plan_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  __shared__ uint32_t first_bad, full;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int doc = (int)blockIdx.x;
  const DocHdr h = a.hdr[doc];
  const uint64_t kb = a.op_off[doc];
  const uint32_t ktot = (uint32_t)(a.op_off[doc + 1] - kb);
  const bool active = (h.flags & kHdrNeedsEsc) && h.status == 0 && h.resume < ktot;
  const uint32_t k0 = h.resume, nleft = active ? ktot - k0 : 0u;
  const bool newcalc = (h.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  if (threadIdx.x == 0) first_bad = nleft, full = 0u;
  __syncthreads();
  // a carried layout with a chunk past kLiveFull is re-laid out this phase (rnd_live)
  if (rd.live[doc] == 1u) {
    const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
    uint32_t mx = 0;
    for (int q = (int)threadIdx.x; q < (int)rd.nch[doc]; q += (int)blockDim.x) mx = cnt[q] > mx ? cnt[q] : mx;
    if (mx > kLiveFull) atomicOr(&full, 1u);
  }
  const uint4* recp = a.recs + 2 * (kb + k0);
  const int32_t M = active ? (int32_t)reinterpret_cast<const uint32_t*>(recp)[2] : 0;
  if (active && !rd.last && newcalc) {
    const int32_t R = h.cur_seq;
    constexpr uint32_t kAllowed = MTE_F_MSG_END | MTE_F_MARKER | MTE_F_REWRITE;
    for (uint32_t base = (uint32_t)w * kWave; base < nleft; base += kChWaves * kWave) {
      if (base >= *(volatile uint32_t*)&first_bad) break;  // an earlier op already ends the run
      uint32_t b[8];
      ch_rec_batch(b, recp, base);
      const int32_t s = (int32_t)b[0], r = (int32_t)b[1], m = (int32_t)b[2];
      const uint32_t type = b[3] & 0xffu, c = (b[3] >> 8) & 0xffu, fl = b[3] >> 16;
      // the seq of the op before (lane 0: the record before the batch)
      const int32_t up = __shfl_up(s, 1);
      const int32_t before = base > 0 ? (int32_t)reinterpret_cast<const uint32_t*>(recp + 2 * (base - 1))[0] : R;
      const int32_t below = l == 0 ? before : up;
      const bool in = base + (uint32_t)l < nleft;
      const bool ok = r == R && m == M && type <= MTE_OP_ANNOTATE && c < MTE_MAX_CLIENTS &&
                      (fl & MTE_F_MSG_END) && !(fl & ~kAllowed) && s > below && M >= h.min_seq && M <= R &&
                      (int32_t)b[4] >= 0 && (int32_t)b[5] >= 0;
      const uint64_t bad = __ballot(in && !ok);
      if (bad) {
        if (l == 0) atomicMin(&first_bad, base + (uint32_t)(__ffsll((long long)bad) - 1));
        break;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint4 p = make_uint4(kModeIdle, 0u, 0u, 0u);
  if (active) {
    const uint32_t len = (!rd.last && newcalc) ? first_bad : 0u;
    const uint32_t k1 = k0 + len;
    // room for every op's segments (an insert or a range op adds at most 3)
    const bool room = (uint64_t)h.nseg + 3ull * len + 2ull <= (uint64_t)a.cap;
    if (len >= kRoundMin && room) {
      p = make_uint4(kModeRound, k0, k1, (uint32_t)M);
      // the chunks this document's column may need: a carried layout's count,
      // at most the re-layout's (its segments only drop) -- sizes the resolve's LDS
      uint32_t nb = (uint32_t)((h.nseg + MTE_RND_FILL - 1) / MTE_RND_FILL);
      if (rd.live[doc] == 1u) nb = full ? (rd.nch[doc] > nb ? rd.nch[doc] : nb) : rd.nch[doc];
      atomicMax(rd.count + 3, nb);
    }
    else if (len >= kRoundMin) p = make_uint4(kModeSeq, k0, k1, 0u);  // this run, op after op
    else p = make_uint4(kModeSeq, k0, ktot, 0u);  // not round-shaped: the rest op after op
    atomicAdd(rd.count + (p.x == kModeRound ? 0 : 1), 1u);
    atomicAdd(rd.count + 2, 1u);
  }
  rd.plan[doc] = p;
}

// ---- re-layout and gather: many waves per document ---------------------------

// a fixed grid of waves walking the (document, chunk) slots with a stride
// (launched at most 2048 x 4 waves): a slot past a document's chunk count, or
// of a document the kernel skips, costs a test, not a wave launch
template <typename F>
__device__ __forceinline__ void chunk_walk(const ChunkArgs& ch, const RoundArgs& rd, F&& f) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
  const uint64_t n = (uint64_t)rd.nd * ch.nch_cap, stride = (uint64_t)gridDim.x * 4;
  for (uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w; wi < n; wi += stride)
    f((int)rd.d0 + (int)(wi / ch.nch_cap), (int)(wi % ch.nch_cap));
}

// the same walk document by document: a document the (wave-uniform) test
// turns down costs one test per wave, not one per chunk slot
template <class P, class F>
__device__ __forceinline__ void chunk_walk_docs(const ChunkArgs& ch, const RoundArgs& rd, P&& take, F&& f) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
  const uint32_t wid = (uint32_t)blockIdx.x * 4u + (uint32_t)w, nw = gridDim.x * 4u;
  for (uint32_t d = 0; d < rd.nd; d++) {
    const int doc = (int)rd.d0 + (int)d;
    if (!__builtin_amdgcn_readfirstlane((int)take(doc))) continue;
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)rd.nch[doc]);
    for (uint32_t q = wid; q < m; q += nw) f(doc, (int)q);
  }
}

constexpr int kT = kChE * kWave;  // flat slots per tile
__device__ __forceinline__ uint32_t rnd_fill(uint32_t total, uint32_t nch) { return nch ? (total + nch - 1) / nch : 1u; }

// keep counts of the flat tiles (removedSeq > M), one wave per tile
template <int K>
__global__ __launch_bounds__(256) void rnd_count_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd, uint32_t tpd) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
  const int doc = (int)rd.d0 + (int)(wi / tpd), t = (int)(wi % tpd);
  if (doc >= (int)(rd.d0 + rd.nd)) return;
  const uint4 p = rd.plan[doc];
  const int n = a.hdr[doc].nseg;
  if (p.x != kModeRound || rd.live[doc] != 0u || t * kT >= n) return;
  const int32_t M = (int32_t)p.w;
  const uint32_t* rs = a.planes + 2 * a.stride + (uint64_t)doc * a.cap;
  int32_t k = 0;
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const int i = t * kT + j * kWave + l;
    k += (i < n && (int32_t)rs[i] > M) ? 1 : 0;
  }
  const int32_t tot = rdlane(wave_incl_scan(k), kWave - 1);
  if (l == 0) ch.kc[(uint64_t)doc * ch.nch_cap + t] = (uint32_t)tot;
}

// per document: exclusive prefix of kc (scatter: the tiles' keep counts) or of
// cnt (gather: the chunks' segment counts, into kc); the gather also advances
// the header past the run
__global__ __launch_bounds__(512) void rnd_scan_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd, int gather) {
  __shared__ ChCtl ctl;
  const int doc = (int)rd.d0 + (int)blockIdx.x;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound || (gather && rd.rflag[doc] != 0u) || (!gather && rd.live[doc] != 0u)) return;
  uint32_t* kc = ch.kc + (uint64_t)doc * ch.nch_cap;
  int m;
  int32_t total;
  if (gather) {
    // the chunks' segment counts summed; kc keeps the column entries the
    // apply wrote (the next run's resolve reads them)
    m = (int)rd.nch[doc];
    const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
    __shared__ int32_t tsum;
    if (threadIdx.x == 0) tsum = 0;
    __syncthreads();
    int32_t v = 0;
    for (int i = (int)threadIdx.x; i < m; i += (int)blockDim.x) v += (int32_t)cnt[i];
    v = rdlane(wave_incl_scan(v), kWave - 1);
    if (lane_id() == 0) atomicAdd(&tsum, v);
    __syncthreads();
    total = tsum;
  } else {
    m = (a.hdr[doc].nseg + kT - 1) / kT;
    total = ch_block_scan(kc, m, &ctl);
  }
  if (threadIdx.x == 0) {
    const unsigned long long pb = 4ull * rd.planes;  // bytes of one segment's planes
    if (!gather) {
      int nch = (total + MTE_RND_FILL - 1) / MTE_RND_FILL;
      nch = nch < 1 ? 1 : (nch > (int)ch.nch_cap ? (int)ch.nch_cap : nch);
      rd.nch[doc] = (uint32_t)nch;
      rd.nnew[doc] = (uint32_t)total;
      rd.live[doc] = 2u;  // the arena holds it from here (rnd_move)
      // the plan's record scan, the keep counts' removedSeq reads, the kept
      // segments' planes moved into the chunks, the columns' length and
      // removedSeq reads, the chunk counts and column entries
      const unsigned long long n_old = (unsigned long long)a.hdr[doc].nseg;
      atomicAdd(rd.acct + doc, 32ull * (p.z - p.y) + 4ull * n_old + 2ull * pb * (unsigned long long)total +
                                   8ull * (unsigned long long)total + 8ull * (unsigned long long)nch);
    } else {
      // the run applied: the header past it, the segments stay in the arena
      // (rnd_live decides when they go back to the flat planes); the counts read
      atomicAdd(rd.acct + doc, 4ull * (unsigned long long)m);
      rd.live[doc] = 1u;
      const uint64_t kb = a.op_off[doc];
      const uint32_t ktot = (uint32_t)(a.op_off[doc + 1] - kb);
      DocHdr h = a.hdr[doc];
      h.nseg = total;
      h.min_seq = (int32_t)p.w;
      h.cur_seq = (int32_t)reinterpret_cast<const uint32_t*>(a.recs + 2 * (kb + p.z - 1))[0];
      h.resume = p.z;
      if (p.z >= ktot) h.flags &= ~kHdrNeedsEsc;
      a.hdr[doc] = h;
    }
  }
}

// flat tile -> its kept segments at kChFill per chunk, one wave per tile
template <int K>
__global__ __launch_bounds__(256) void rnd_move_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd, uint32_t tpd) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
  const int doc = (int)rd.d0 + (int)(wi / tpd), t = (int)(wi % tpd);
  if (doc >= (int)(rd.d0 + rd.nd)) return;
  const uint4 p = rd.plan[doc];
  const int n = a.hdr[doc].nseg;
  if (p.x != kModeRound || rd.live[doc] != 2u || t * kT >= n) return;
  const int32_t M = (int32_t)p.w;
  const uint32_t* pl = a.planes + (uint64_t)doc * a.cap;
  bool keep[kChE];
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const int i = t * kT + j * kWave + l;
    keep[j] = i < n && (int32_t)pl[2 * a.stride + i] > M;
  }
  // destinations in document order: slot j * 64 + l of the tile
  int32_t dst[kChE];
  int32_t run = (int32_t)ch.kc[(uint64_t)doc * ch.nch_cap + t];
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const uint64_t mk = __ballot(keep[j]);
    dst[j] = run + (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
    run += __popcll(mk);
  }
  const uint32_t nch = rd.nch[doc], fill = rnd_fill(rd.nnew[doc], nch);
  const uint32_t lim = nch * fill;
  uint64_t xs[kChE];
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const uint32_t ci = (uint32_t)dst[j] / fill;
    xs[j] = ch_slot(ch, doc, (int)ci) + ((uint32_t)dst[j] - ci * fill);
  }
  // every plane's loads in flight before the stores (as rnd_gmove)
  constexpr int NP = kFieldPlanes + K;
  uint32_t v[NP][kChE];
#pragma unroll
  for (int q = 0; q < NP; q++)
#pragma unroll
    for (int j = 0; j < kChE; j++) {
      const int i = t * kT + j * kWave + l;
      v[q][j] = pl[(uint64_t)q * a.stride + (i < n ? i : 0)];
    }
#pragma unroll
  for (int q = 0; q < NP; q++)
#pragma unroll
    for (int j = 0; j < kChE; j++)
      if (keep[j] && (uint32_t)dst[j] < lim) ch.arena[(uint64_t)q * ch.astride + xs[j]] = v[q][j];
}

// per chunk after the moves: its segment count and its round-start column
// entry (the visible length: every segment is seen at refSeq R), into kc
__global__ __launch_bounds__(256) void rnd_cols_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  const int l = lane_id();
  // a carried document's counts and column entries are current: the apply
  // wrote each chunk it changed (rnd_apply_one), the rest did not change
  chunk_walk_docs(ch, rd, [&](int doc) { return rd.plan[doc].x == kModeRound && rd.live[doc] != 1u; },
                  [&](int doc, int q) {
    // a re-laid-out document: kChFill per chunk
    const int n_new = (int)rd.nnew[doc], fill = (int)rnd_fill(rd.nnew[doc], rd.nch[doc]);
    const int cn = n_new - q * fill < fill ? (n_new - q * fill > 0 ? n_new - q * fill : 0) : fill;
    const uint64_t x0 = ch_slot(ch, doc, q);
    int32_t v = 0;
#pragma unroll
    for (int j = 0; j < kChSlots / kWave; j++) {
      const int s = j * kWave + l;
      if (s < cn) v += (int32_t)ch.arena[2 * ch.astride + x0 + s] == kNone ? (int32_t)ch.arena[x0 + s] : 0;
    }
    const int32_t tot = rdlane(wave_incl_scan(v), kWave - 1);
    if (l == 0) {
      ch.cnt[(uint64_t)doc * ch.nch_cap + q] = (uint32_t)cn;
      ch.kc[(uint64_t)doc * ch.nch_cap + q] = (uint32_t)tot;
    }
  });
}

// chunk -> flat planes at its prefix (nothing is dropped: the run's
// tombstones have removedSeq > R >= M), one wave per chunk
template <int K>
__global__ __launch_bounds__(256) void rnd_gmove_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  const int l = lane_id();
  chunk_walk_docs(ch, rd, [&](int doc) { return rd.gfl[doc] != 0u; }, [&](int doc, int q) {
    const int cn = (int)ch.cnt[(uint64_t)doc * ch.nch_cap + q];
    const uint32_t d0 = ch.kc[(uint64_t)doc * ch.nch_cap + q];
    const uint64_t x0 = ch_slot(ch, doc, q);
    uint32_t* pl = a.planes + (uint64_t)doc * a.cap;
    // every plane's loads in flight before the stores (the two may alias as
    // far as the compiler knows: interleaved, each plane waited for the last)
    constexpr int NP = kFieldPlanes + K;
    uint32_t v[NP][kChE];
#pragma unroll
    for (int qq = 0; qq < NP; qq++)
#pragma unroll
      for (int j = 0; j < kChE; j++) {
        const int s = j * kWave + l;
        v[qq][j] = ch.arena[(uint64_t)qq * ch.astride + x0 + (s < cn ? s : 0)];
      }
#pragma unroll
    for (int qq = 0; qq < NP; qq++)
#pragma unroll
      for (int j = 0; j < kChE; j++) {
        const int s = j * kWave + l;
        if (s < cn && d0 + (uint32_t)s < a.cap) pl[(uint64_t)qq * a.stride + d0 + (uint32_t)s] = v[qq][j];
      }
  });
}

// ---- carried layouts ------------------------------------------------------------
// per document (a workgroup): does its arena go back to the flat planes in this
// launch?  It does when it holds the document (live 1) and the next run is not
// a round, a chunk is past kLiveFull, or this is the launch's last gather
__global__ __launch_bounds__(256) void rnd_live_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd, int final) {
  __shared__ uint32_t full;
  const int doc = (int)rd.d0 + (int)blockIdx.x;
  const uint32_t lv = rd.live[doc];
  if (threadIdx.x == 0) full = 0u;
  __syncthreads();
  const bool leave = lv == 1u && (final || rd.plan[doc].x != kModeRound);
  if (lv == 1u && !leave) {
    const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
    const int nch = (int)rd.nch[doc];
    uint32_t mx = 0;
    for (int q = (int)threadIdx.x; q < nch; q += (int)blockDim.x) mx = cnt[q] > mx ? cnt[q] : mx;
    if (mx > kLiveFull) atomicOr(&full, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) rd.gfl[doc] = (leave || full) ? 1u : 0u;
}

// per document after the apply: a run the round phases refused (rflag) left
// the arena untouched -- a re-laid-out document's flat planes are still
// current, a carried one's go back (rflag & 4: its chunks had no room, the run
// is re-laid out and taken again next phase, not op after op)
__global__ __launch_bounds__(64) void rnd_post_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  const int doc = (int)rd.d0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (doc >= (int)(rd.d0 + rd.nd)) return;
  uint32_t g = 0;
  const uint4 p = rd.plan[doc];
  const uint32_t f = rd.rflag[doc];
  if (p.x == kModeRound && f != 0u) {
    const uint32_t lv = rd.live[doc];
    if (lv == 2u) rd.live[doc] = 0u;
    if (lv == 1u) {
      g = 1u;
      if (f & 4u) rd.plan[doc] = make_uint4(kModeIdle, 0u, 0u, 0u);
    }
  }
  rd.gfl[doc] = g;
}

// the gather documents: exclusive prefix of their chunk counts (into kc); they
// leave the arena
__global__ __launch_bounds__(512) void rnd_gscan_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  __shared__ ChCtl ctl;
  const int doc = (int)rd.d0 + (int)blockIdx.x;
  if (rd.gfl[doc] == 0u) return;
  uint32_t* kc = ch.kc + (uint64_t)doc * ch.nch_cap;
  const int m = (int)rd.nch[doc];
  const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  for (int i = (int)threadIdx.x; i < m; i += (int)blockDim.x) kc[i] = cnt[i];
  __syncthreads();
  const int32_t total = ch_block_scan(kc, m, &ctl);
  if (threadIdx.x == 0) {
    const unsigned long long pb = 4ull * rd.planes;
    atomicAdd(rd.acct + doc, 2ull * pb * (unsigned long long)total + 8ull * (unsigned long long)m);
    a.hdr[doc].nseg = total;
    rd.live[doc] = 0u;
  }
}

// a carried document's chunks must hold the run's sub-ops: count + 2 per
// sub-op <= kChSlots (a re-laid-out one's always do: kChFill + 2 kRB); one
// thread per chunk
__global__ __launch_bounds__(256) void rnd_room_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  const uint64_t wi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int doc = (int)rd.d0 + (int)(wi / ch.nch_cap), q = (int)(wi % ch.nch_cap);
  if (doc >= (int)(rd.d0 + rd.nd)) return;
  // (a failed chain's run goes op after op anyway: its partial buckets are moot)
  if (rd.plan[doc].x != kModeRound || rd.live[doc] != 1u || q >= (int)rd.nch[doc] || (rd.rflag[doc] & 2u)) return;
  const uint64_t i = (uint64_t)doc * ch.nch_cap + q;
  if (ch.cnt[i] + 2u * rd.rcnt[i] > (uint32_t)kChSlots) atomicOr(rd.rflag + doc, 4u);
}

// ---- resolve: one wave per client chain, the column as prefix sums -----------
// The column is kept in LDS as three levels of inclusive prefix sums over rows
// of 64: CI[i] = chunk i's prefix within its group of 64 chunks, GS[g] = group
// g's prefix within its supergroup of 64 groups, SS[s] = supergroup s's prefix
// over the document.  A position resolves with one LDS read and one ballot
// per level and no scan; a change d to chunk i adds d to the later entries of
// the three rows it lies in (one LDS write per lane and level, from the values
// the search just read).
struct Col {
  int32_t* CI;  // nch_cap entries
  int32_t* GS;  // ng_cap rounded up to 64
  int32_t* SS;  // 64
  int32_t* GD;  // ng_cap rounded up to 64: a block's length changes per group (zero between blocks)
  int nch;
  int ng, nsg;
};

struct ColHit {
  int i, g, sg;          // chunk, its group and supergroup (i = nch: none)
  int lc, lg;            // lane of the chunk in its group row, of the group in its supergroup row
  int32_t excl, csum;    // the chunk's exclusive prefix and length
  int32_t total;         // the column's total
  int32_t ci, gs, ss;    // this lane's entries of the three rows, as read
};

// the first chunk whose inclusive prefix is > x (strict) or >= x
__device__ __forceinline__ ColHit col_find(const Col& C, int32_t x, bool strict) {
  const int l = lane_id();
  ColHit h;
  h.g = h.sg = h.lc = h.lg = 0;
  h.ci = h.gs = 0;
  h.ss = l < C.nsg ? C.SS[l] : INT32_MAX / 2;
  h.total = C.nsg > 0 ? rdlane(h.ss, C.nsg - 1) : 0;
  const uint64_t ms = __ballot(l < C.nsg && (strict ? h.ss > x : h.ss >= x));
  if (!ms) {
    h.i = C.nch;
    h.excl = h.total;
    h.csum = 0;
    return h;
  }
  h.sg = __ffsll((long long)ms) - 1;
  const int32_t es = h.sg > 0 ? rdlane(h.ss, h.sg - 1) : 0;
  const int gi = h.sg * kWave + l;
  h.gs = gi < C.ng ? C.GS[gi] : INT32_MAX / 2;
  const uint64_t mg = __ballot(gi < C.ng && (strict ? es + h.gs > x : es + h.gs >= x));
  h.lg = mg ? __ffsll((long long)mg) - 1 : 0;
  h.g = h.sg * kWave + h.lg;
  const int32_t eg = es + (h.lg > 0 ? rdlane(h.gs, h.lg - 1) : 0);
  const int ci = h.g * kChGroup + l;
  h.ci = ci < C.nch ? C.CI[ci] : INT32_MAX / 2;
  const uint64_t mc = __ballot(ci < C.nch && (strict ? eg + h.ci > x : eg + h.ci >= x));
  h.lc = mc ? __ffsll((long long)mc) - 1 : 0;
  h.i = h.g * kChGroup + h.lc;
  const int32_t prev = h.lc > 0 ? rdlane(h.ci, h.lc - 1) : 0;
  h.excl = eg + prev;
  h.csum = rdlane(h.ci, h.lc) - prev;
  return h;
}

// chunk h.i changed by d: the later entries of its three rows
__device__ __forceinline__ void col_add(const Col& C, const ColHit& h, int32_t d) {
  const int l = lane_id();
  const int ci = h.g * kChGroup + l, gi = h.sg * kWave + l;
  if (l >= h.lc && ci < C.nch) C.CI[ci] = h.ci + d;
  if (l >= h.lg && gi < C.ng) C.GS[gi] = h.gs + d;
  if (l >= h.sg && l < C.nsg) C.SS[l] = h.ss + d;
}

// group gg's row changed by the per-lane amounts o (lane j: chunk gg * 64 + j):
// CI of the row minus their running sum, the group's and later groups' GS /
// SS minus their total
__device__ __forceinline__ void col_sub_row(const Col& C, int gg, int32_t ci_row, int32_t o) {
  const int l = lane_id();
  const int32_t oi = wave_incl_scan(o);
  const int32_t og = rdlane(oi, kWave - 1);
  const int ci = gg * kChGroup + l;
  if (ci < C.nch) C.CI[ci] = ci_row - oi;
  const int sg = gg / kWave, lg = gg % kWave;
  const int gi = sg * kWave + l;
  if (l >= lg && gi < C.ng) C.GS[gi] = C.GS[gi] - og;
  if (l >= sg && l < C.nsg) C.SS[l] = C.SS[l] - og;
}

// A resolved sub-op straight into its chunk's bucket: the entry (op index,
// chunk start in the op's perspective) and the op's record beside it, so the
// apply reads its chunk's records in one contiguous load; a bucket past kRB
// refuses the run (rflag 1).  The record loads go out with the slot's atomic.
struct Emit {
  uint32_t* rcnt;      // the document's per-chunk counts
  uint2* rbuf;         // its buckets
  uint4* rrec;         // their records
  const uint4* recp;   // the run's records
  uint32_t* rflag;     // the document's refusal flags
  uint64_t base;       // doc * nch_cap
};
__device__ __forceinline__ void rnd_emit(const Emit& E, uint32_t chunk, uint32_t k, uint32_t excl) {
  const uint4 q0 = E.recp[2 * k], q1 = E.recp[2 * k + 1];
  const uint32_t pos = atomicAdd(E.rcnt + chunk, 1u);
  if (pos < (uint32_t)kRB) {
    const uint64_t slot = (E.base + chunk) * kRB + pos;
    E.rbuf[slot] = make_uint2(k, excl);
    E.rrec[2 * slot] = q0;
    E.rrec[2 * slot + 1] = q1;
  } else {
    atomicOr(E.rflag, 1u);
  }
}

// one op of a chain against the column, op after op: emits its sub-ops
// (counted in m) and changes the column; false = the run cannot take it (an insert
// past the end: MTE_E_INSERT_FAILED op after op; the list full)
__device__ __forceinline__ bool rnd_serial_op(const Col& C, uint32_t k, uint32_t w3, int32_t pos1, int32_t pos2,
                                              const Emit& E, uint32_t& m, uint32_t cap_c) {
  const int l = lane_id();
  const uint32_t type = w3 & 0xffu, flags = w3 >> 16;
  if (type == MTE_OP_INSERT) {
    const ColHit h = col_find(C, pos1, false);
    if (pos1 > h.total || h.i >= C.nch || m >= cap_c) return false;
    const int32_t nlen = (flags & MTE_F_MARKER) ? 1 : pos2;
    if (l == 0) rnd_emit(E, (uint32_t)h.i, k, (uint32_t)h.excl);
    m++;
    if (nlen > 0) col_add(C, h, nlen);
    lds_fence();
    return true;
  }
  const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
  const ColHit h = col_find(C, b1, true);
  if (h.i < C.nch) {
    if (b1 == b2) {
      // ensureIntervalBoundary alone: a split strictly inside a leaf
      if (h.excl < b1) {
        if (m >= cap_c) return false;
        if (l == 0) rnd_emit(E, (uint32_t)h.i, k, (uint32_t)h.excl);
        m++;
      }
    } else {
      // group by group from the first chunk's while the chunk starts are
      // before b2, in the op's perspective before it (eg: the group's start then)
      int32_t eg = h.excl - (h.lc > 0 ? rdlane(h.ci, h.lc - 1) : 0);
      for (int gg = h.g; gg < C.ng; gg++) {
        const int i = gg * kChGroup + l;
        const int32_t ci = i < C.nch ? C.CI[i] : 0;
        const int32_t cprev0 = __shfl_up(ci, 1);
        const int32_t cprev = l == 0 ? 0 : cprev0;
        const int32_t st = eg + cprev, incl = eg + ci, v = ci - cprev;
        const bool hit = i < C.nch && i >= h.i && v > 0 && st < b2;
        const uint64_t hm = __ballot(hit);
        m += (uint32_t)__popcll(hm);
        if (m > cap_c) return false;
        if (hit) rnd_emit(E, (uint32_t)i, k, (uint32_t)st);
        // the group's end before this op
        const int last = C.nch - gg * kChGroup < kWave ? C.nch - gg * kChGroup - 1 : kWave - 1;
        const int32_t gend = eg + rdlane(ci, last);
        if (type == MTE_OP_REMOVE && hm) {
          const int32_t lo = b1 > st ? b1 : st, hi = b2 < incl ? b2 : incl;
          col_sub_row(C, gg, ci, hit ? hi - lo : 0);
          lds_fence();
        }
        eg = gend;
        if (gend >= b2) break;
      }
    }
  }
  lds_fence();
  return true;
}

// ---- block-parallel chain resolve ----------------------------------------------
// A chain's ops resolve 64 at a time, lane t = the block's t-th op.  An op
// changes its chain's column only through the chunk boundaries B_c (inclusive
// prefixes) it moves, a monotone map on positions -- exactly what col_add /
// col_sub_row do to the rows:
//   insert of n at p:  B -> B + n if p <= B (the first chunk with B >= p takes it)
//   remove [b1, b2):   B -> B if B <= b1;  b1 if b1 < B < b2;  B - (b2 - b1) if B >= b2
//   annotate:          identity.
// Op t's chunk is the first c whose boundary, carried through the block's
// earlier ops, is > x (x = b1; an insert's "first with >= pos" is "> pos - 1"),
// and as every map is monotone that condition pulls back to the block-start
// column: B_c > y, y = x carried back through the earlier ops, latest first:
//   insert (p, n):  y -> y if y < p;  y - n if y >= p + n;  p - 1 otherwise (inside it: its chunk)
//   remove (b1, r): y -> y if y < b1;  y + r otherwise.
// So every lane finds its chunk with one search of the block-start column, the
// chunk's start and end in its perspective are block-start boundaries carried
// forward through the earlier ops, and the block's length changes fold into the
// column afterwards (one LDS add per chunk row and change, group rows by a
// scan of the block's per-group changes).  A range that
// reaches a third chunk sends the block op by op (rnd_serial_op).

// first t in [0, V) with R[t] > lim over a nondecreasing row, >= V if none
// (this lane's row: two rounds of 8 LDS reads)
__device__ __forceinline__ int row_first_gt(const int32_t* R, int V, int32_t lim) {
  int q = 0;
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const int t = 8 * s + 7;
    q += (t < V && R[t] <= lim) ? 1 : 0;
  }
  if (q == 8) return kWave;
  int u = 0;
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const int t = 8 * q + s;
    u += (t < V && R[t] <= lim) ? 1 : 0;
  }
  return 8 * q + u;
}

struct ColPos {
  int c;                // the first chunk with B_c > y (nch: none)
  int32_t bm, bc, bn;   // B_{c-1} (-1 for chunk 0), B_c, B_{c+1} (B_c for the last chunk)
};

__device__ __forceinline__ ColPos col_find_lane(const Col& C, int32_t y, bool act) {
  ColPos r;
  r.c = C.nch;
  r.bm = r.bc = r.bn = 0;
  if (!act) return r;
  const int sg = row_first_gt(C.SS, C.nsg, y);
  if (sg >= C.nsg) return r;
  const int32_t es = sg > 0 ? C.SS[sg - 1] : 0;
  const int vg = C.ng - sg * kWave < kWave ? C.ng - sg * kWave : kWave;
  const int t = row_first_gt(C.GS + sg * kWave, vg, y - es);
  if (t >= vg) return r;  // the rows disagree: not found (the run falls back)
  const int g = sg * kWave + t;
  const int32_t eg = es + (t > 0 ? C.GS[g - 1] : 0);
  const int vc = C.nch - g * kChGroup < kChGroup ? C.nch - g * kChGroup : kChGroup;
  const int u = row_first_gt(C.CI + g * kChGroup, vc, y - eg);
  if (u >= vc) return r;
  r.c = g * kChGroup + u;
  r.bm = u > 0 ? eg + C.CI[r.c - 1] : (r.c == 0 ? -1 : eg);
  r.bc = eg + C.CI[r.c];
  r.bn = r.bc;
  if (r.c + 1 < C.nch) {
    if (u + 1 < kChGroup) {
      r.bn = eg + C.CI[r.c + 1];
    } else {  // the next group's first chunk
      const int g1 = g + 1, sg1 = g1 / kWave;
      const int32_t es1 = sg1 == sg ? es : C.SS[sg1 - 1];
      r.bn = es1 + ((g1 % kWave) ? C.GS[g1 - 1] : 0) + C.CI[r.c + 1];
    }
  }
  return r;
}

// the block of nb ops (lane t < nb: op t -- record index k, w3, pos1, pos2):
// sub-ops appended at list[m..], the column advanced past the block.  false:
// nothing done, the block goes op by op.  failed: an insert past the end.
__device__ __forceinline__ bool rnd_block(const Col& C, int nb, uint32_t k, uint32_t w3, int32_t pos1, int32_t pos2,
                                          const Emit& E, uint32_t& m, uint32_t cap_c, bool& failed) {
  if (m + 2u * (uint32_t)nb > cap_c) return false;  // at most two sub-ops an op; else op by op, checked
  RND_CLK(c0);
  const int l = lane_id();
  const bool v = l < nb;
  const uint32_t type = w3 & 0xffu;
  const bool ins = v && type == MTE_OP_INSERT, rem = v && type == MTE_OP_REMOVE;
  const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
  const int32_t nlen = ((w3 >> 16) & MTE_F_MARKER) ? 1 : pos2;
  // the op as a map: tn > 0 an insert of tn at tp, tn < 0 a remove of -tn at tp
  const int32_t tp = ins ? pos1 : b1;
  const int32_t tn = ins ? (nlen > 0 ? nlen : 0) : (rem ? b1 - b2 : 0);
  int32_t y = ins ? pos1 - 1 : b1;
  RND_CLK(c1);
  // The passes visit the block's inserts and removes only (an annotate is the
  // identity), the lanes after j taking op j; one uniform branch on the op's
  // kind per step, selects inside.
  const uint64_t xm = __ballot(tn != 0);
  // back, latest first: y -> y if y < p; y - n if y >= p + n; p - 1 otherwise
  // (insert of n at p); y + r if y >= p (remove of r at p)
  for (uint64_t m = xm; m;) {
    const int j = 63 - __clzll((long long)m);
    m ^= 1ull << j;
    const int32_t tj = rdlane(tn, j), pj = rdlane(tp, j);
    const bool take = l > j && y >= pj;
    if (tj > 0) {
      const int32_t y1 = y >= pj + tj ? y - tj : pj - 1;
      y = take ? y1 : y;
    } else {
      y = take ? y - tj : y;
    }
  }
  RND_CLK(c2);
  const ColPos P = col_find_lane(C, y, v);
  const bool found = v && P.c < C.nch;
  int32_t bm = P.bm, bc = P.bc, bn = P.bn;
  RND_CLK(c3);
  // forward: B -> B + n if p <= B (insert); B - clamp(B - p, 0, r) (remove)
  for (uint64_t m = xm; m; m &= m - 1) {
    const int j = __ffsll((long long)m) - 1;
    const int32_t tj = rdlane(tn, j), pj = rdlane(tp, j);
    if (tj > 0) {
      const int32_t a = l > j ? tj : 0;
      bm += pj <= bm ? a : 0;
      bc += pj <= bc ? a : 0;
      bn += pj <= bn ? a : 0;
    } else {
      const int32_t r = l > j ? -tj : 0;
      bm -= min(max(bm - pj, 0), r);
      bc -= min(max(bc - pj, 0), r);
      bn -= min(max(bn - pj, 0), r);
    }
  }
  RND_CLK(c4);
  const int c = P.c;
  const int32_t st = c == 0 ? 0 : bm;
  bool s0 = false, s1 = false, more = false, bad = false;
  int32_t d0 = 0, d1 = 0;
  if (ins) {
    if (!found) bad = true;
    else {
      s0 = true;
      d0 = nlen > 0 ? nlen : 0;
    }
  } else if (found) {
    if (b1 == b2) {
      s0 = st < b1;  // a split strictly inside the chunk
    } else {
      s0 = true;
      if (rem) d0 = (b1 > st ? b1 : st) - (b2 < bc ? b2 : bc);
      if (bc < b2 && c + 1 < C.nch) {
        if (bn > bc) {
          s1 = true;
          if (rem) d1 = bc - (b2 < bn ? b2 : bn);
        }
        if (bn < b2 && c + 2 < C.nch) more = true;
      }
    }
  }
  if (__ballot(more)) return false;
  if (__ballot(bad)) {
    failed = true;
    return true;
  }
  if (s0) rnd_emit(E, (uint32_t)c, k, (uint32_t)st);
  if (s1) rnd_emit(E, (uint32_t)c + 1u, k, (uint32_t)bc);
  m += (uint32_t)(__popcll(__ballot(s0)) + __popcll(__ballot(s1)));
  // fold: each change into its chunk row (one add per change, no divergence),
  // the changes per group lane-parallel into GD, then per supergroup row the
  // groups' running sums into GS and the row totals into SS
  const uint32_t lanes4 = (uint32_t)l;
  for (uint64_t e = __ballot(d0 != 0); e; e &= e - 1) {
    const int t = __ffsll((long long)e) - 1;
    const uint32_t cc = (uint32_t)rdlane(c, t);
    const int32_t dd = rdlane(d0, t);
    const uint32_t g0 = cc & ~63u, ci = g0 + lanes4;
    atomicAdd(&C.CI[ci], (lanes4 >= (cc & 63u) && ci < (uint32_t)C.nch) ? dd : 0);
  }
  for (uint64_t e = __ballot(d1 != 0); e; e &= e - 1) {
    const int t = __ffsll((long long)e) - 1;
    const uint32_t cc = (uint32_t)rdlane(c, t) + 1u;
    const int32_t dd = rdlane(d1, t);
    const uint32_t g0 = cc & ~63u, ci = g0 + lanes4;
    atomicAdd(&C.CI[ci], (lanes4 >= (cc & 63u) && ci < (uint32_t)C.nch) ? dd : 0);
  }
  if (d0 != 0) atomicAdd(&C.GD[(uint32_t)c >> 6], d0);
  if (d1 != 0) atomicAdd(&C.GD[((uint32_t)c + 1u) >> 6], d1);
  lds_fence();
  for (int sg = 0; sg < C.nsg; sg++) {
    const int gi = sg * kWave + l;
    const bool in = gi < C.ng;
    const int32_t dv = in ? C.GD[gi] : 0;
    const int32_t inc = wave_incl_scan(dv);
    if (in) {
      C.GD[gi] = 0;
      C.GS[gi] += inc;
    }
    const int32_t tot = rdlane(inc, kWave - 1);
    if (l >= sg && l < C.nsg) C.SS[l] += tot;
  }
  lds_fence();
  RND_DIAG(6, c1 - c0);
  RND_DIAG(7, c2 - c1);
  RND_DIAG(8, c3 - c2);
  RND_DIAG(9, c4 - c3);
  RND_DIAG(10, clock64() - c4);
  return true;
}

constexpr uint32_t kRing = 1024;  // a chain wave's staging ring of record indices (LDS)

// WPB waves per workgroup, 8 / WPB workgroups per document; wave u = 0..7 of
// the document takes the clients c = u, u + 8, ...; dynamic LDS: per wave a
// CI column of nch_cap entries
template <int WPB>
__global__ __launch_bounds__(WPB * kWave) void rnd_resolve_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  extern __shared__ uint32_t rs_lds[];
  __shared__ uint32_t ccount[MTE_MAX_CLIENTS];
  constexpr int kBlocksPerDoc = kChWaves / WPB;
  const int doc = (int)rd.d0 + (int)blockIdx.x / kBlocksPerDoc;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound) return;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int u = ((int)blockIdx.x % kBlocksPerDoc) * WPB + w;
  const uint32_t nops = p.z - p.y;
  const uint4* recp = a.recs + 2 * (a.op_off[doc] + p.y);
  Col C;
  C.nch = (int)rd.nch[doc];
  C.ng = (C.nch + kChGroup - 1) / kChGroup;
  C.nsg = (C.ng + kWave - 1) / kWave;
  {
    // the column sized for this phase's largest document (rd.col_cap, a multiple of 64)
    const uint32_t gs_cap = (rd.col_cap / kChGroup + kWave - 1) / kWave * kWave;
    int32_t* base = reinterpret_cast<int32_t*>(rs_lds) + (uint64_t)w * (rd.col_cap + 2 * gs_cap + kWave + kRing);
    C.CI = base;
    C.GS = base + rd.col_cap;
    C.SS = base + rd.col_cap + gs_cap;
    C.GD = C.SS + kWave;
  }
  uint32_t* const ring = reinterpret_cast<uint32_t*>(C.GD + (rd.col_cap / kChGroup + kWave - 1) / kWave * kWave);
  const int32_t* sum0 = reinterpret_cast<const int32_t*>(ch.kc + (uint64_t)doc * ch.nch_cap);
  const Emit E{rd.rcnt + (uint64_t)doc * ch.nch_cap, rd.rbuf, rd.rrec, recp, rd.rflag + doc,
               (uint64_t)doc * ch.nch_cap};
  // ops per client (every workgroup of the document counts them all)
  for (int c = (int)threadIdx.x; c < MTE_MAX_CLIENTS; c += (int)blockDim.x) ccount[c] = 0u;
  __syncthreads();
  for (uint32_t i0 = threadIdx.x; i0 < nops; i0 += 8 * blockDim.x) {  // 8 records in flight per thread
    uint32_t w3[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t i = i0 + (uint32_t)q * blockDim.x;
      w3[q] = i < nops ? reinterpret_cast<const uint32_t*>(recp + 2 * i)[3] : 0xffffffffu;
    }
#pragma unroll
    for (int q = 0; q < 8; q++)
      if (w3[q] != 0xffffffffu) atomicAdd(&ccount[(w3[q] >> 8) & 31u], 1u);
  }
  __syncthreads();
  // each chain's list region: twice its ops (+ 8) from the prefix over clients
  uint32_t off = 0;
  for (int c = 0; c < MTE_MAX_CLIENTS; c++) {
    const uint32_t nc = ccount[c];
    const uint32_t cap_c = nc ? 2u * nc + 8u : 0u;
    if ((c % kChWaves) == u && nc) {
      // column c = the round-start column as prefix sums: the chunk rows, then
      // the group rows from the chunk rows' totals, then the supergroup row
      for (int g = 0; g < C.ng; g++) {
        const int i = g * kChGroup + l;
        const int32_t v = i < C.nch ? sum0[i] : 0;
        const int32_t incl = wave_incl_scan(v);
        if (i < C.nch) C.CI[i] = incl;
        if (l == 0) C.GS[g] = rdlane(incl, kWave - 1);  // the group's total, for now
      }
      lds_fence();
      for (int sg = 0; sg < C.nsg; sg++) {
        const int g = sg * kWave + l;
        const int32_t v = g < C.ng ? C.GS[g] : 0;
        const int32_t incl = wave_incl_scan(v);
        if (g < C.ng) C.GS[g] = incl;
        if (l == 0) C.SS[sg] = rdlane(incl, kWave - 1);
      }
      for (int g = l; g < C.ng; g += kWave) C.GD[g] = 0;
      lds_fence();
      {
        const int32_t v = l < C.nsg ? C.SS[l] : 0;
        const int32_t incl = wave_incl_scan(v);
        if (l < C.nsg) C.SS[l] = incl;
      }
      lds_fence();
      uint32_t m = 0;  // entries in the chain's list
      bool failed = false;
      // the chain's ops in blocks of 64: the records' client bytes 512 at a time
      // (the next 512 in flight meanwhile), the chain's record indices staged in
      // an LDS ring, each block's records read back per lane
      uint32_t head = 0, tail = 0;
      uint32_t cw[8], nw[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t r = (uint32_t)(q * kWave + l);
        cw[q] = r < nops ? reinterpret_cast<const uint32_t*>(recp + 2 * r)[3] : 0xffffffffu;
      }
      for (uint32_t sb = 0; sb < nops && !failed; sb += 8 * kWave) {
        RND_CLK(tg0);
        const bool last = sb + 8 * kWave >= nops;
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t r = sb + 8 * kWave + (uint32_t)(q * kWave + l);
          nw[q] = r < nops ? reinterpret_cast<const uint32_t*>(recp + 2 * r)[3] : 0xffffffffu;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const uint32_t r = sb + (uint32_t)(q * kWave + l);
          const uint64_t mine = __ballot(r < nops && ((cw[q] >> 8) & 0xffu) == (uint32_t)c);
          if ((mine >> l) & 1ull) ring[(tail + lanes_below(mine)) & (kRing - 1)] = r;
          tail += (uint32_t)__popcll(mine);
        }
        lds_fence();
        RND_DIAG(4, clock64() - tg0);
        while (!failed && (tail - head >= (uint32_t)kWave || (last && tail > head))) {
          RND_CLK(tb0);
          const int nb = tail - head < (uint32_t)kWave ? (int)(tail - head) : kWave;
          uint32_t k = 0, w3 = 0;
          int32_t p1 = 0, p2 = 0;
          if (l < nb) {
            k = ring[(head + (uint32_t)l) & (kRing - 1)];
            const uint32_t* rp = reinterpret_cast<const uint32_t*>(recp + 2 * k);
            w3 = rp[3];
            p1 = (int32_t)rp[4];
            p2 = (int32_t)rp[5];
          }
          const bool par = rnd_block(C, nb, k, w3, p1, p2, E, m, cap_c, failed);
          RND_CLK(tb1);
          if (!par) {
            for (int t = 0; t < nb && !failed; t++)
              failed = !rnd_serial_op(C, rdlane(k, t), rdlane(w3, t), rdlane(p1, t), rdlane(p2, t), E, m,
                                      cap_c);
            RND_DIAG(1, 1);
            RND_DIAG(5, clock64() - tb1);
          }
          RND_DIAG(0, 1);
          RND_DIAG(2, nb);
          RND_DIAG(3, tb1 - tb0);
          head += (uint32_t)nb;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) cw[q] = nw[q];
      }
      if (l == 0) {
        if (failed) atomicOr(rd.rflag + doc, 2u);
        rd.rchain[(uint64_t)doc * MTE_MAX_CLIENTS + (uint32_t)c] = make_uint2(off, failed ? 0u : m);
        // the chain's records; per sub-op its record read again and copied
        // with its bucket entry into the chunk's bucket
        atomicAdd(rd.acct + doc, 32ull * nc + 72ull * m);
      }
    } else if ((c % kChWaves) == u && l == 0) {
      rd.rchain[(uint64_t)doc * MTE_MAX_CLIENTS + (uint32_t)c] = make_uint2(off, 0u);
    }
    off += cap_c;
  }
}

// a chunk's first E * 64 slots into registers (E = 2: one 8-byte load per
// plane and lane; E = 4: ch_load), padding past n; and back
template <int E, int K>
__device__ __forceinline__ void ch_load_e(Regs<E, K>& R, const ChunkArgs& ch, uint64_t x0, int n) {
  if constexpr (E == kChE) {
    ch_load<K>(R, ch, x0, n);
  } else {
    static_assert(E == 2, "two or four slots per lane");
    const uint32_t* pl = ch.arena + x0 + (uint32_t)lane_id() * E;
    const uint64_t st = ch.astride;
    uint2 q[kFieldPlanes + K];
    const int base = lane_id() * E;
#pragma unroll
    for (int p = 0; p < kFieldPlanes + K; p++)
      q[p] = base < n ? *reinterpret_cast<const uint2*>(pl + p * st) : make_uint2(0u, 0u);
#pragma unroll
    for (int j = 0; j < E; j++) {
      const bool v = base + j < n;
      auto el = [&](int p) -> uint32_t { return j == 0 ? q[p].x : q[p].y; };
      R.len[j] = v ? (int32_t)el(0) : 0;
      R.seq[j] = v ? (int32_t)el(1) : 0;
      R.rseq[j] = v ? (int32_t)el(2) : kPad;
      R.rmask[j] = v ? el(3) : 0u;
      R.meta[j] = v ? el(4) : 0u;
      R.toff[j] = v ? el(5) : 0u;
#pragma unroll
      for (int k = 0; k < K; k++) R.pr[k][j] = v ? el(kFieldPlanes + k) : 0u;
    }
  }
}

template <int E, int K>
__device__ __forceinline__ void ch_store_e(const Regs<E, K>& R, const ChunkArgs& ch, uint64_t x0, int n,
                                           int32_t* vis = nullptr) {
  uint32_t* pl = ch.arena;
  const uint64_t st = ch.astride;
  const int base = lane_id() * E;
  if (vis) *vis = 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    if (i < n) {
      const uint64_t x = x0 + (uint32_t)i;
      if (vis) *vis += R.rseq[j] == kNone ? R.len[j] : 0;
      pl[x] = (uint32_t)R.len[j];
      pl[st + x] = (uint32_t)R.seq[j];
      pl[2 * st + x] = (uint32_t)R.rseq[j];
      pl[3 * st + x] = R.rmask[j];
      pl[4 * st + x] = R.meta[j];
      pl[5 * st + x] = R.toff[j];
#pragma unroll
      for (int k = 0; k < K; k++) pl[(kFieldPlanes + k) * st + x] = R.pr[k][j];
    }
  }
}

// the chunk's sub-ops in op order through seg_op_v at E slots per lane
template <int E, int K>
__device__ __forceinline__ int rnd_apply_chunk(const ReplayArgs& a, const ChunkArgs& ch, uint64_t x0, int& ni,
                                               uint32_t nb, int from, const uint2& e, const uint4& r0,
                                               const uint4& r1, int32_t M, int32_t& vis) {
  RND_CLK(a0);
  Regs<E, K> R;
  ch_load_e<E, K>(R, ch, x0, ni);
  uint32_t st[kNumStats] = {};
  int rcs = 0;
#if MTE_RND_DIAG
  R.len[0] += __builtin_amdgcn_readfirstlane(0);  // (the planes are in)
#endif
  RND_CLK(a1);
  for (uint32_t j = 0; j < nb; j++) {
    const int q = rdlane(from, (int)j);
    const int32_t ex = (int32_t)rdlane(e.y, q);
    s8v op;
    op[0] = (int32_t)rdlane(r0.x, q);
    op[1] = (int32_t)rdlane(r0.y, q);
    op[2] = (int32_t)rdlane(r0.z, q);
    op[3] = (int32_t)rdlane(r0.w, q);
    op[4] = (int32_t)rdlane(r1.x, q);
    op[5] = (int32_t)rdlane(r1.y, q);
    op[6] = (int32_t)rdlane(r1.z, q);
    op[7] = (int32_t)rdlane(r1.w, q);
    const uint32_t w3 = (uint32_t)op[3];
    int32_t tot = 0, dlen = 0;
    const int rc = seg_op_v<E, K, false, true>(R, ni, op, w3 & 0xffu, (w3 >> 8) & 0xffu, w3 >> 16, M, true, ex, true,
                                               tot, dlen, a, st);
    rcs = rc != 0 ? rc : rcs;
  }
  RND_CLK(a2);
  // the chunk's column entry for the next run (rnd_cols: its visible length,
  // every segment seen at that run's refSeq): the segments not removed
  ch_store_e<E, K>(R, ch, x0, ni, &vis);
  RND_DIAG(12, a1 - a0);
  RND_DIAG(13, a2 - a1);
  RND_DIAG(14, nb);
  return rcs;
}

// one wave per chunk of a run: its sub-ops in op order (MTE_APPLY_E2: a chunk
// that stays within 128 slots -- its segments + 2 per sub-op -- at two slots
// per lane; off: both paths' registers cost the kernel half its occupancy)
#ifndef MTE_APPLY_E2
#define MTE_APPLY_E2 0
#endif
template <int K>
__device__ __forceinline__ void rnd_apply_one(const ReplayArgs& a, const ChunkArgs& ch, const RoundArgs& rd, int doc,
                                              int i) {
  const int l = lane_id();
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound || rd.rflag[doc] != 0u || i >= (int)rd.nch[doc]) return;
  // the sub-op count and bucket and the segment count, issued together; then
  // each sub-op's record (bucket order)
  RND_CLK(w0);
  const uint32_t nb = rd.rcnt[(uint64_t)doc * ch.nch_cap + i];
  const uint64_t bslot = ((uint64_t)doc * ch.nch_cap + i) * kRB + (l < kRB ? l : 0);
  const uint2 e0 = rd.rbuf[bslot];
  const uint4 q0 = rd.rrec[2 * bslot], q1 = rd.rrec[2 * bslot + 1];
  uint32_t* cntp = ch.cnt + (uint64_t)doc * ch.nch_cap;
  int ni = (int)cntp[i];
  const int n_before = ni;
  const uint64_t x0 = ch_slot(ch, doc, i);
  if (nb == 0u) return;
  const uint2 e = l < (int)nb ? e0 : make_uint2(0xffffffffu, 0u);
  const uint4 r0 = l < (int)nb ? q0 : make_uint4(0u, 0u, 0u, 0u), r1 = l < (int)nb ? q1 : make_uint4(0u, 0u, 0u, 0u);
  // the bucket in op order: each entry's rank, and per rank the lane holding it
  uint32_t rank = 0;
  for (uint32_t j = 0; j < nb; j++) rank += rdlane(e.x, (int)j) < e.x ? 1u : 0u;
  const int dst = (l < (int)nb ? (int)rank : l) << 2;
  const int from = __builtin_amdgcn_ds_permute(dst, l);
  const int32_t M = (int32_t)p.w;
#if MTE_RND_DIAG
  RND_DIAG(11, 1);
  RND_DIAG(15, clock64() - w0 + 0 * (r0.x + r1.w + (uint32_t)from));
#endif
#if MTE_APPLY_E2
  int32_t vis = 0;
  const int rcs = ni + 2 * (int)nb <= 2 * kWave ? rnd_apply_chunk<2, K>(a, ch, x0, ni, nb, from, e, r0, r1, M, vis)
                                                : rnd_apply_chunk<kChE, K>(a, ch, x0, ni, nb, from, e, r0, r1, M, vis);
#else
  int32_t vis = 0;
  const int rcs = rnd_apply_chunk<kChE, K>(a, ch, x0, ni, nb, from, e, r0, r1, M, vis);
#endif
  vis = rdlane(wave_incl_scan(vis), kWave - 1);
  if (l == 0) {
    // the chunk's sub-ops (record + bucket entry), its planes in and out, its count
    atomicAdd(rd.acct + doc, 40ull * nb + 4ull * rd.planes * (unsigned long long)(n_before + ni) + 8ull);
    cntp[i] = (uint32_t)ni;
    ch.kc[(uint64_t)doc * ch.nch_cap + i] = (uint32_t)vis;  // read by the next run's resolve
    if (rcs != 0) a.hdr[doc].status = MTE_E_STATE;  // resolve guarantees every sub-op fits: an engine bug
  }
}

// a fixed grid of waves walking the (document, chunk) slots with a stride: the
// slots past a document's chunk count cost a test, not a wave launch
template <int K>
// MTE_APPLY_WPE: a waves-per-SIMD floor for the register allocator (A/B builds)
#ifndef MTE_APPLY_WPE
#define MTE_APPLY_WPE 0
#endif
#if MTE_APPLY_WPE > 0
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MTE_APPLY_WPE)))
#else
__global__ __launch_bounds__(256)
#endif
void rnd_apply_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  chunk_walk_docs(ch, rd, [&](int doc) { return rd.plan[doc].x == kModeRound && rd.rflag[doc] == 0u; },
                  [&](int doc, int q) { rnd_apply_one<K>(a, ch, rd, doc, q); });
}

}  // namespace mte
