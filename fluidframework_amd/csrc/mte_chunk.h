// mte_chunk.h — pass 3 for big-document contexts (seg_capacity >=
// kChunkMinCap): documents beyond the register tiers (> 1,022 segments, up
// to millions: BASELINE config 5) replayed one workgroup per document over a
// chunked segment layout with per-client chunk length summaries.
//
// Layout (per document, in a ctx-wide arena next to the flat planes):
//   chunk i = 256 slots, segments [0, cnt[i]) in document order, the same
//             planes as the flat layout (len seq rseq rmask meta toff props);
//   sum[c][i] = chunk i's length in the perspective (rr[c], client c) — the
//             flat counterpart of PartialSequenceLengths.getPartialLength
//             (partialLengths.ts:667-702) at chunk granularity;
//   G[c][g]  = sum over the 64 chunks of group g (LDS).
// An op of client c at refSeq r resolves its position with two wavefront
// scans (G column in LDS, then the group's 64 sums), applies the same
// segment step as the register tiers (seg_op_v, mte_step1.h) to the one chunk
// holding the position (a range op: each chunk of the range), and adds its
// length change to column c.  The summaries are exact incrementally because a
// sequenced op changes no perspective length except its own client's (proof
// in DESIGN.md §5); a column is rebuilt (all waves, O(S)) when an op of its
// client arrives with another refSeq, and all are dropped at a re-layout.
//
// Re-layout (all 8 waves): gather the chunks into the flat planes dropping
// tombstones with removedSeq <= minSeq (zamboni, mergeTree.ts:1077-1093),
// then scatter 128 segments per chunk.  It runs at entry, when minSeq
// advances, and when a chunk op could overflow its 256 slots; the pass ends
// with a final gather, so every other kernel sees the flat layout.
#pragma once

#include "mte_replay.h"

namespace mte {

constexpr uint32_t kChunkMinCap = 8192;  // ctxs with a smaller capacity use pass 3 = stream_kernel
constexpr int kChE = 4;                  // slots per lane
constexpr int kChSlots = kWave * kChE;   // 256 slots per chunk
constexpr int kChFill = 128;             // segments per chunk after a re-layout
constexpr int kChGroup = 64;             // chunks per summary group
constexpr int kChWaves = 8;              // one document per 512-thread workgroup
constexpr uint32_t kChMaxGroups = 500;   // G in LDS: 32 x 500 x 4 B
constexpr int32_t kColInvalid = INT32_MIN;

struct ChunkArgs {
  uint32_t* arena;   // plane p, doc d, chunk i, slot j: arena[p * astride + (d * nch_cap + i) * 256 + j]
  uint64_t astride;
  uint32_t nch_cap;  // chunks per doc
  uint32_t ng_cap;   // groups per doc (<= kChMaxGroups)
  uint32_t* cnt;     // [doc][nch_cap] segments per chunk
  uint32_t* kc;      // [doc][nch_cap] re-layout scratch
  int32_t* sum;      // [doc][MTE_MAX_CLIENTS][nch_cap]
  // round phases (mte_round.h): with a plan, chunk_kernel replays only the
  // documents the plan sends op after op, up to their run's end
  const uint4* plan;      // [doc] x mode, y k0, z k1, w M (null: every escalated doc to its end)
  const uint32_t* rflag;  // [doc] non-zero: the round phases left the run to this pass
};

enum : uint32_t { kModeIdle = 0, kModeRound = 1, kModeSeq = 2 };

// wave-0 -> workgroup requests
enum ChReq : int32_t { kReqNone = 0, kReqRelayout, kReqRebuild, kReqDone };

struct ChCtl {
  int32_t req, arg_c, arg_r;
  int32_t n;        // segments of the doc
  int32_t nch;      // chunks in use
  int32_t min_seq;  // for the re-layout's zamboni and the rebuilds
  int32_t status;
  int32_t part[kChWaves];
  int32_t rr[MTE_MAX_CLIENTS];  // refSeq each summary column is valid for
  int32_t pf_k;     // wave 0's current op (the prefetch wave runs ahead of it)
  int32_t pf_stop;  // wave 0 left its op loop
};

// Data this kernel writes is read back with agent-scope loads (vector, L1
// bypassed): never through the scalar cache, never a stale L1 line.
__device__ __forceinline__ uint32_t ld_ag(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_ag(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t ch_slot(const ChunkArgs& ch, int doc, int i) {
  return ((uint64_t)doc * ch.nch_cap + (uint32_t)i) * kChSlots;
}

// A chunk's planes into registers: one 16-byte load per plane and lane (every
// slot of a chunk is allocated, so slots >= n are read and replaced by
// padding).  Plain loads: the chunk data is written by this workgroup only,
// and the CU's L1 is shared by its waves (workgroup-scope coherence).
__device__ __forceinline__ uint4 ld4(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }

template <int K>
__device__ __forceinline__ void ch_load(Regs<kChE, K>& R, const ChunkArgs& ch, uint64_t x0, int n) {
  const uint32_t* pl = ch.arena + x0 + (uint32_t)lane_id() * kChE;
  const uint64_t st = ch.astride;
  uint4 q[kFieldPlanes + K];
  const int base = lane_id() * kChE;
  // the lanes past the chunk's segments read nothing (their slots are padding)
#pragma unroll
  for (int p = 0; p < kFieldPlanes + K; p++) q[p] = base < n ? ld4(pl + p * st) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const bool v = base + j < n;
    auto el = [&](int p) -> uint32_t { return j == 0 ? q[p].x : (j == 1 ? q[p].y : (j == 2 ? q[p].z : q[p].w)); };
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

template <int K>
__device__ __forceinline__ void ch_store(const Regs<kChE, K>& R, const ChunkArgs& ch, uint64_t x0, int n) {
  uint32_t* pl = ch.arena;
  const uint64_t st = ch.astride;
  const int base = lane_id() * kChE;
#pragma unroll
  for (int j = 0; j < kChE; j++) {
    const int i = base + j;
    if (i < n) {
      const uint64_t x = x0 + (uint32_t)i;
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

// op records: 1 = 64 at a time through vector loads, 0 = scalar loads one ahead
#ifndef MTE_CH_VREC
#define MTE_CH_VREC 1
#endif

// 64 op records from record `base` on: lane l holds record base + l, one
// dword per register
__device__ __forceinline__ void ch_rec_batch(uint32_t (&b)[8], const uint4* recp, uint32_t base) {
  const uint4* p = recp + 2 * (base + (uint32_t)lane_id());
  const uint4 x = p[0], y = p[1];
  b[0] = x.x, b[1] = x.y, b[2] = x.z, b[3] = x.w;
  b[4] = y.x, b[5] = y.y, b[6] = y.z, b[7] = y.w;
}

// First chunk whose inclusive prefix (column c) is > x (strict) or >= x.
// Returns the chunk (nch if none) and its exclusive prefix in *excl; *total =
// the doc's length in the column's perspective.
__device__ __forceinline__ int ch_find(const uint32_t* G, uint32_t ng, const int32_t* sumc, const uint32_t* cnt,
                                       int nch, int32_t x, bool strict, int32_t* excl, int32_t* total,
                                       int32_t* csum, int* ccnt) {
  const int l = lane_id();
  const uint32_t gpl = (ng + kWave - 1) / kWave;  // groups per lane (<= 8)
  int32_t s = 0;
  for (uint32_t k = 0; k < gpl; k++) {
    const uint32_t g = (uint32_t)l * gpl + k;
    s += g < ng ? (int32_t)G[g] : 0;
  }
  const int32_t incl = wave_incl_scan(s);
  *total = rdlane(incl, kWave - 1);
  // the lane whose groups cross x, then the group inside it
  const bool hit = strict ? incl > x : incl >= x;
  const uint64_t hm = __ballot(hit);
  if (!hm) {
    *excl = *total;
    *csum = 0;
    *ccnt = 0;
    return nch;
  }
  const int ls = __ffsll((long long)hm) - 1;
  int32_t run = rdlane(incl - s, ls);
  uint32_t g = (uint32_t)ls * gpl;
  for (uint32_t k = 0; k < gpl; k++, g++) {
    const int32_t v = (int32_t)G[g];  // wave-uniform address: one LDS broadcast
    if (strict ? run + v > x : run + v >= x) break;
    run += v;
  }
  // the 64 chunks of group g (their segment counts come along)
  const int i = (int)g * kChGroup + l;
  const int32_t v = i < nch ? ld_ag(sumc + i) : 0;
  const int32_t nc = i < nch ? (int32_t)ld_ag(cnt + i) : 0;
  const int32_t ci = wave_incl_scan(v) + run;
  const uint64_t cm = __ballot(strict ? ci > x : ci >= x);
  const int lc = cm ? __ffsll((long long)cm) - 1 : kWave - 1;  // (cm != 0 by construction)
  *excl = rdlane(ci - v, lc);
  *csum = rdlane(v, lc);
  *ccnt = rdlane(nc, lc);
  return (int)g * kChGroup + lc;
}

// ---- workgroup phases (all 8 waves) ---------------------------------------

// block-wide exclusive scan of kc[0, nch) in place; returns the total
__device__ __forceinline__ int32_t ch_block_scan(uint32_t* kc, int nch, ChCtl* ctl) {
  const int t = (int)threadIdx.x, w = __builtin_amdgcn_readfirstlane(t / kWave);
  const int per = (nch + kChWaves * kWave - 1) / (kChWaves * kWave);
  const int i0 = t * per;
  int32_t s = 0;
  for (int k = 0; k < per; k++)
    if (i0 + k < nch) s += (int32_t)ld_ag(kc + i0 + k);
  const int32_t incl = wave_incl_scan(s);
  if (lane_id() == kWave - 1) ctl->part[w] = incl;
  __syncthreads();
  int32_t wbase = 0, total = 0;
  for (int v = 0; v < kChWaves; v++) {
    const int32_t pv = ctl->part[v];
    wbase += v < w ? pv : 0;
    total += pv;
  }
  int32_t run = wbase + incl - s;
  for (int k = 0; k < per; k++)
    if (i0 + k < nch) {
      const int32_t x = (int32_t)ld_ag(kc + i0 + k);
      kc[i0 + k] = (uint32_t)run;
      run += x;
    }
  __syncthreads();
  return total;
}

// chunks -> flat planes, dropping tombstones with rseq <= m; returns the new n
template <int K>
__device__ int32_t ch_gather(const ReplayArgs& a, const ChunkArgs& ch, int doc, ChCtl* ctl, int nch, int32_t m) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  uint32_t* kc = ch.kc + (uint64_t)doc * ch.nch_cap;
  for (int i = w; i < nch; i += kChWaves) {
    const uint64_t x0 = ch_slot(ch, doc, i);
    const int n = (int)ld_ag(cnt + i);
    int32_t k = 0;
#pragma unroll
    for (int j = 0; j < kChE; j++) {
      const int s = l * kChE + j;
      k += (s < n && (int32_t)ld_ag(ch.arena + 2 * ch.astride + x0 + s) > m) ? 1 : 0;
    }
    const int32_t tot = rdlane(wave_incl_scan(k), kWave - 1);
    if (l == 0) kc[i] = (uint32_t)tot;
  }
  __syncthreads();
  const int32_t n_new = ch_block_scan(kc, nch, ctl);
  uint32_t* pl = a.planes + (uint64_t)doc * a.cap;
  const int nplanes = kFieldPlanes + K;
  for (int i = w; i < nch; i += kChWaves) {
    const uint64_t x0 = ch_slot(ch, doc, i);
    const int n = (int)ld_ag(cnt + i);
    bool keep[kChE];
    int32_t k = 0;
#pragma unroll
    for (int j = 0; j < kChE; j++) {
      const int s = l * kChE + j;
      keep[j] = s < n && (int32_t)ld_ag(ch.arena + 2 * ch.astride + x0 + s) > m;
      k += keep[j] ? 1 : 0;
    }
    int32_t d = (int32_t)ld_ag(kc + i) + wave_incl_scan(k) - k;
    for (int p = 0; p < nplanes; p++) {
      int32_t dd = d;
#pragma unroll
      for (int j = 0; j < kChE; j++) {
        if (keep[j] && (uint32_t)dd < a.cap)
          pl[(uint64_t)p * a.stride + dd] = ld_ag(ch.arena + (uint64_t)p * ch.astride + x0 + l * kChE + j);
        dd += keep[j] ? 1 : 0;
      }
    }
  }
  __syncthreads();
  return n_new;
}

// flat planes -> chunks of kChFill segments; returns the chunk count
template <int K>
__device__ int ch_scatter(const ReplayArgs& a, const ChunkArgs& ch, int doc, int n) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  int nch = (n + kChFill - 1) / kChFill;
  if (nch < 1) nch = 1;
  if (nch > (int)ch.nch_cap) nch = (int)ch.nch_cap;  // n <= cap keeps this unreachable
  const uint32_t* pl = a.planes + (uint64_t)doc * a.cap;
  const int nplanes = kFieldPlanes + K;
  for (int i = w; i < nch; i += kChWaves) {
    const uint64_t x0 = ch_slot(ch, doc, i);
    const int f0 = i * kChFill;
    const int cn = n - f0 < kChFill ? (n - f0 > 0 ? n - f0 : 0) : kChFill;
    for (int p = 0; p < nplanes; p++) {
#pragma unroll
      for (int j = 0; j < kChFill / kWave; j++) {
        const int s = j * kWave + l;
        if (s < cn) ch.arena[(uint64_t)p * ch.astride + x0 + s] = ld_ag(pl + (uint64_t)p * a.stride + f0 + s);
      }
    }
    if (l == 0) cnt[i] = (uint32_t)cn;
  }
  __syncthreads();
  return nch;
}

// summary column c for (r, client c): sum[c][i] for every chunk, then G[c][g]
template <int K>
__device__ void ch_rebuild(const ChunkArgs& ch, int doc, uint32_t* Gc, int nch, int c, int32_t r, int32_t m,
                           bool newcalc) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  int32_t* sumc = ch.sum + ((uint64_t)doc * MTE_MAX_CLIENTS + (uint32_t)c) * ch.nch_cap;
  for (int i = w; i < nch; i += kChWaves) {
    Regs<kChE, 0> R;
    ch_load<0>(R, ch, ch_slot(ch, doc, i), (int)ld_ag(cnt + i));
    int32_t L[kChE];
    leaf_lengths<kChE, 0>(R, r, (uint32_t)c + 1u, c, m, newcalc, L);
    int32_t s = 0;
#pragma unroll
    for (int j = 0; j < kChE; j++) s += L[j] > 0 ? L[j] : 0;
    const int32_t tot = rdlane(wave_incl_scan(s), kWave - 1);
    if (l == 0) sumc[i] = tot;
  }
  __syncthreads();
  const int ng = (nch + kChGroup - 1) / kChGroup;
  for (int g = w; g < ng; g += kChWaves) {
    const int i = g * kChGroup + l;
    const int32_t v = i < nch ? ld_ag(sumc + i) : 0;
    const int32_t tot = rdlane(wave_incl_scan(v), kWave - 1);
    if (l == 0) Gc[g] = (uint32_t)tot;
  }
  __syncthreads();
}

// ---- diagnostics: MTE_CH_PROF=1 phase clocks (tools/chunk_prof.py) ------------
// Per document, in its stats slots at the end of the pass (s_memtime cycles):
// 0 ops, 1 position lookups (ch_find), 2 chunk loads (issue -> data), 3 the
// register step, 4 stores + summary updates, 5 the pass (max over docs),
// 6 column rebuilds, 7 re-layouts.  A diagnostic build, never the product.
#ifndef MTE_CH_PROF
#define MTE_CH_PROF 0
#endif
#if MTE_CH_PROF
#define CHPROF(...) __VA_ARGS__
__device__ __forceinline__ uint64_t ch_clock() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  return __builtin_amdgcn_s_memtime();
}
#else
#define CHPROF(...)
#endif

// ---- wave 1: chunk prefetch ---------------------------------------------------
// While wave 0 applies op k, wave 1 resolves ops k+1 .. k+kPfAhead against the
// summaries as they stand and touches their chunks, so wave 0's chunk loads
// hit L2 instead of HBM.  A column only changes for its own client's ops, so
// the guess is exact unless an op of the same client lies in between; a wrong
// guess costs bandwidth only: this wave reads, never writes (the summaries
// and G may be mid-update — every index it forms is range-checked).
#ifndef MTE_CH_PREFETCH
#define MTE_CH_PREFETCH 1
#endif
constexpr int kPfAhead = 4;

template <int K>
__device__ void ch_prefetch(const DocRun& D0, const ReplayArgs& a, const ChunkArgs& ch, const uint32_t* G,
                            uint32_t ng_cap, ChCtl* ctl, int doc) {
  const int nch = ctl->nch;
  const uint32_t ng = (uint32_t)((nch + kChGroup - 1) / kChGroup);
  const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  const uint64_t kb = a.op_off[doc];
  const uint4* recp = a.recs + 2 * kb;
  const uint32_t k1 = (uint32_t)(a.op_off[doc + 1] - kb);
  uint32_t done = 0;  // ops below this are prefetched
  uint32_t sink = 0;
  for (;;) {
    if (*(volatile int32_t*)&ctl->pf_stop) break;
    const uint32_t k = (uint32_t)uni(*(volatile int32_t*)&ctl->pf_k);
    uint32_t j = done > k + 1 ? done : k + 1;
    if (j >= k + 1 + kPfAhead || j >= k1) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    done = j + 1;
    const uint32_t rw = lane_id() < 8 ? reinterpret_cast<const uint32_t*>(recp + 2 * j)[lane_id()] : 0u;
    const uint32_t w3 = rdlane(rw, 3);
    const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu;
    if (type > MTE_OP_ANNOTATE || c >= MTE_MAX_CLIENTS) continue;
    if (ctl->rr[c] != (int32_t)rdlane(rw, 1)) continue;  // column c not built for this refSeq
    const int32_t pos1 = (int32_t)rdlane(rw, 4), pos2 = (int32_t)rdlane(rw, 5);
    const int32_t x = type == MTE_OP_INSERT ? pos1 : (pos1 < pos2 ? pos1 : pos2);
    const int32_t* sumc = ch.sum + ((uint64_t)doc * MTE_MAX_CLIENTS + c) * ch.nch_cap;
    int32_t ex, total, cs;
    int cn;
    const int i = ch_find(G + c * ng_cap, ng, sumc, cnt, nch, x, type != MTE_OP_INSERT, &ex, &total, &cs, &cn);
    if (i < 0 || i >= nch) continue;
    const uint32_t* pl = ch.arena + ch_slot(ch, doc, i) + (uint32_t)lane_id() * kChE;
#pragma unroll
    for (int p = 0; p < kFieldPlanes + K; p++) sink ^= ld4(pl + p * ch.astride).x;
  }
  if (sink == 0x9e3779b9u && doc < 0) a.stats[0] = sink;  // keeps the touches alive
  (void)D0;
}

// ---- wave 0: the op loop ------------------------------------------------------

// Runs ops of the doc until the workgroup must act (re-layout, column
// rebuild) or the batch ends.  Returns the request.
template <int K, bool S>
__device__ int ch_ops(DocRun& D, const ReplayArgs& a, const ChunkArgs& ch, uint32_t* G, uint32_t ng_cap, ChCtl* ctl,
                      uint32_t (&st)[kNumStats], uint64_t* prof) {
  const int doc = D.doc;
  const int nch = ctl->nch;
  const uint32_t ng = (uint32_t)((nch + kChGroup - 1) / kChGroup);
  uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  const bool newcalc = (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  // MTE_CH_VREC: op records 64 at a time through vector loads (lane l:
  // record base + l), the next batch loading while this one is used, so the
  // LDS scans never wait behind a scalar load in flight (SMEM and LDS share
  // lgkmcnt).  Past the doc's last op the loads read the next doc's records
  // or the zeroed tail (kRecPad).
#if MTE_CH_VREC
  uint32_t rbase = D.k & ~(uint32_t)(kWave - 1);
  uint32_t rc0[8], rc1[8];
  ch_rec_batch(rc0, D.recp, rbase);
  ch_rec_batch(rc1, D.recp, rbase + kWave);
#else
  s8v cur = sload8(D.recp + 2 * D.k);
#endif
  while (D.k < D.k1) {
    if constexpr (S) {
      if (st[kStOps] >= 256) run_flush_stats(D, st, a);
    }
#if MTE_CH_VREC
    if (D.k - rbase >= (uint32_t)kWave) {  // the next batch; load the one after
      rbase += kWave;
#pragma unroll
      for (int i = 0; i < 8; i++) rc0[i] = rc1[i];
      ch_rec_batch(rc1, D.recp, rbase + kWave);
    }
    s8v op;
#pragma unroll
    for (int i = 0; i < 8; i++) op[i] = (int32_t)rdlane(rc0[i], (int)(D.k - rbase));
#else
    // this op's record was prefetched; the next one is in flight meanwhile
    // (past the last op it reads the next doc's record or the zeroed tail)
    const s8v op = cur;
    uint64_t next = uni64(reinterpret_cast<uint64_t>(D.recp + 2 * (D.k + 1)));
    asm volatile("" : "+s"(next) : "s"(op));
    cur = sload8(reinterpret_cast<const uint4*>(next));
#endif
    CHPROF(uint64_t tq = ch_clock(); uint64_t tn;)
    if (MTE_CH_PREFETCH && lane_id() == 0) *(volatile int32_t*)&ctl->pf_k = (int32_t)D.k;
    const uint32_t w3 = (uint32_t)op[3];
    const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
    const int32_t s = op[0], r = op[1], msn = op[2];
    if (c >= MTE_MAX_CLIENTS) {
      D.status = MTE_E_CLIENT_RANGE;
      return kReqDone;
    }
    if (type > MTE_OP_NOOP) {
      D.status = MTE_E_INVALID_ARG;
      return kReqDone;
    }
    if (type != MTE_OP_NOOP) {
      if (ctl->rr[c] != r) {  // column c is for another refSeq: rebuild, then retry
        ctl->arg_c = (int32_t)c;
        ctl->arg_r = r;
        return kReqRebuild;
      }
      if (D.n + 2 > (int)a.cap) {
        D.status = MTE_E_CAPACITY;
        return kReqDone;
      }
    }
    const int n_before = D.n;
    uint32_t scan = 0;  // chunk slots + summary entries this op scans
    uint32_t* Gc = G + c * ng_cap;
    int32_t* sumc = ch.sum + ((uint64_t)doc * MTE_MAX_CLIENTS + c) * ch.nch_cap;
    if (type != MTE_OP_NOOP) {
      const int32_t pos1 = op[4], pos2 = op[5];
      int i0, i1;
      int32_t ex = 0, total = 0, ex2 = 0, cs0 = 0, cs1 = 0;
      int cn0 = 0, cn1 = 0;
      if (type == MTE_OP_INSERT) {
        i0 = ch_find(Gc, ng, sumc, cnt, nch, pos1, false, &ex, &total, &cs0, &cn0);
        scan += ng + kChGroup;
        if (pos1 > total) {  // no slot anywhere (mergeTree.ts:1666-1672)
          D.status = MTE_E_INSERT_FAILED;
          return kReqDone;
        }
        if (i0 >= nch) {
          i0 = nch - 1;
          cn0 = (int)ld_ag(cnt + i0);
        }
        i1 = nch - 1;  // an insert may move on to later chunks (kNextChunk)
      } else {
        const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
        i0 = ch_find(Gc, ng, sumc, cnt, nch, b1, true, &ex, &total, &cs0, &cn0);
        scan += ng + kChGroup;
        if (i0 >= nch) {
          i1 = -1;  // the range starts past the end: nothing to split or mark
        } else if (b1 == b2) {
          i1 = ex < b1 ? i0 : -1;  // a split strictly inside a leaf, or nothing
        } else if (ex + cs0 >= b2) {
          i1 = i0;  // the range ends in its first chunk
          cn1 = cn0;
        } else {
          int32_t t2;
          i1 = ch_find(Gc, ng, sumc, cnt, nch, b2, false, &ex2, &t2, &cs1, &cn1);
          scan += ng + kChGroup;
          if (i1 >= nch) {
            i1 = nch - 1;
            cn1 = (int)ld_ag(cnt + i1);
          }
        }
        // only the two boundary chunks can grow (one split each)
        if (i1 >= i0 && (cn0 + 2 > kChSlots - 2 || cn1 + 2 > kChSlots - 2)) return kReqRelayout;
      }
      CHPROF(tn = ch_clock(); prof[1] += tn - tq; tq = tn;)
      for (int i = i0; i <= i1; i++) {
        int ni = i == i0 ? cn0 : (int)ld_ag(cnt + i);
        // an insert touches one chunk and nothing is applied before this
        // check; a range op checked its two boundary chunks above (the chunks
        // between them cannot split)
        if (type == MTE_OP_INSERT && ni + 2 > kChSlots - 2) return kReqRelayout;
        const uint64_t x0 = ch_slot(ch, doc, i);
        Regs<kChE, K> R;
        ch_load<K>(R, ch, x0, ni);
        CHPROF(tn = ch_clock(); prof[2] += tn - tq; tq = tn;)
        const int n0 = ni;
        scan += (uint32_t)ni;
        int32_t tot = 0, dlen = 0;
        const int rc = seg_op_v<kChE, K, S, true>(R, ni, op, type, c, flags, D.min_seq, newcalc, ex, i == nch - 1,
                                                  tot, dlen, a, st);
        CHPROF(tn = ch_clock(); prof[3] += tn - tq; tq = tn;)
        if (rc == kNextChunk) {  // insert at the end of chunk i's perspective: the slot is further on
          ex = pos1;
          continue;
        }
        if (rc < 0) {
          D.status = rc;
          return kReqDone;
        }
        ch_store<K>(R, ch, x0, ni);
        if (dlen != 0) {
          // chunk i0's sum came with ch_find: no second round trip for it
          const int32_t prev = i == i0 ? cs0 : ld_ag(sumc + i);
          if (lane_id() == 0) {
            sumc[i] = prev + dlen;
            Gc[i / kChGroup] += (uint32_t)dlen;
          }
        }
        if (lane_id() == 0) cnt[i] = (uint32_t)ni;
        D.n += ni - n0;
        ex += tot;
        CHPROF(tn = ch_clock(); prof[4] += tn - tq; tq = tn;)
        if (type == MTE_OP_INSERT) break;
      }
      fence_wave();
    }
    // counted once the op is applied (a re-layout or rebuild retries it)
    CHPROF(prof[0]++;)
    MTE_STAT(st[kStOps]++;)
    MTE_STAT(st[kStMaxSegs] = (uint32_t)n_before > st[kStMaxSegs] ? (uint32_t)n_before : st[kStMaxSegs];)
    MTE_STAT(if (type != MTE_OP_NOOP) {
      st[kStScanned] += (uint32_t)n_before;
      st[kStChunkCanon] += (uint32_t)n_before;
      st[kStChunkScan] += scan;
    })
    D.k++;
    // collab window (doc_step, mte_replay.h)
    const bool live = type != MTE_OP_NOOP, end = (flags & MTE_F_MSG_END) != 0;
    const bool bad = (live & (s <= D.cur_seq)) | (end & (s < D.cur_seq)) | ((live | end) & (msn < D.min_seq)) |
                     (end & (msn > s));
    if (bad) {
      D.status = window_error(D, live, end, s, msn);
      return kReqDone;
    }
    if (end) {
      D.cur_seq = s;
      if (msn > D.min_seq) {
        D.min_seq = msn;
        return kReqRelayout;  // zamboni
      }
    }
  }
  return kReqDone;
}

// pass 3 (big-doc contexts): one document per 512-thread workgroup, for the
// documents pass 2 escalated
template <int K, bool S>
__global__ __launch_bounds__(512) void chunk_kernel(ReplayArgs a, ChunkArgs ch) {
  extern __shared__ uint32_t ch_lds[];
  const int doc = (int)blockIdx.x;
  if (doc >= (int)a.n_docs) return;
  if (!(a.hdr[doc].flags & kHdrNeedsEsc)) return;  // untouched doc: leave the header alone
  uint32_t kend = 0xffffffffu;
  if (ch.plan) {
    const uint4 pp = ch.plan[doc];
    if (!(pp.x == kModeSeq || (pp.x == kModeRound && ch.rflag[doc] != 0u))) return;
    kend = pp.z;
  }
  uint32_t* G = ch_lds;  // [MTE_MAX_CLIENTS][ng_cap]
  ChCtl* ctl = reinterpret_cast<ChCtl*>(ch_lds + (size_t)MTE_MAX_CLIENTS * ch.ng_cap);
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
  DocRun D;
  uint32_t st[kNumStats] = {};
  uint64_t prof[8] = {};
  CHPROF(const uint64_t t_start = ch_clock(); uint64_t tph = 0;)
  uint32_t ktot = 0;
  if (w == 0) {
    run_init(D, a, doc, true);
    ktot = D.k1;
    if (D.k1 > kend) D.k1 = kend;
    D.running = D.running && D.k < D.k1;
    if (lane_id() == 0) {
      ctl->n = D.n;
      ctl->min_seq = D.min_seq;
      ctl->req = D.running ? kReqRelayout : kReqDone;
      ctl->nch = 0;
    }
  }
  __syncthreads();
  bool chunked = false;  // the doc is in the chunk layout
  for (;;) {
    const int req = ctl->req;
    CHPROF(tph = ch_clock();)
    if (req == kReqRelayout || req == kReqDone) {
      int n = ctl->n;
      if (chunked) n = ch_gather<K>(a, ch, doc, ctl, ctl->nch, ctl->min_seq);
      chunked = false;
      if (req == kReqRelayout) {
        const int nch = ch_scatter<K>(a, ch, doc, n);
        chunked = true;
        if (threadIdx.x == 0) ctl->nch = nch;
      }
      if (threadIdx.x < MTE_MAX_CLIENTS) ctl->rr[threadIdx.x] = kColInvalid;
      if (threadIdx.x == 0) ctl->n = n;
      __syncthreads();
      CHPROF(prof[7] += ch_clock() - tph;)
      if (req == kReqDone) break;
    } else if (req == kReqRebuild) {
      const int c = ctl->arg_c;
      ch_rebuild<K>(ch, doc, G + (uint32_t)c * ch.ng_cap, ctl->nch, c, ctl->arg_r, ctl->min_seq,
                    (a.hdr[doc].flags & MTE_DOC_NEW_LENGTH_CALC) != 0);
      if (threadIdx.x == 0) ctl->rr[c] = ctl->arg_r;
      __syncthreads();
      CHPROF(prof[6] += ch_clock() - tph;)
    }
    if (MTE_CH_PREFETCH && threadIdx.x == 0) {
      ctl->pf_stop = 0;
      ctl->pf_k = D.k;
    }
    __syncthreads();
    if (w == 0) {
      D.n = ctl->n;
      const int nreq = D.status == 0 ? ch_ops<K, S>(D, a, ch, G, ch.ng_cap, ctl, st, prof) : (int)kReqDone;
      if (lane_id() == 0) {
        ctl->req = nreq;
        ctl->n = D.n;
        ctl->min_seq = D.min_seq;
        if (MTE_CH_PREFETCH) *(volatile int32_t*)&ctl->pf_stop = 1;
      }
    } else if (MTE_CH_PREFETCH && w == 1) {
      ch_prefetch<K>(D, a, ch, G, ch.ng_cap, ctl, doc);
    }
    __syncthreads();
  }
  if (w == 0) {
    D.n = ctl->n;
    D.running = false;
    if constexpr (S) run_flush_stats(D, st, a);
    run_finish(D, a);
    // a plan's run ended before the batch: the document stays escalated
    if (ch.plan && lane_id() == 0 && D.status == 0 && D.k < ktot) a.hdr[doc].flags |= kHdrNeedsEsc;
    CHPROF(prof[5] = ch_clock() - t_start;
           if (lane_id() == 0) for (int t = 0; t < 8; t++) a.stats[(size_t)doc * kNumStats + t] = prof[t];)
  }
}

}  // namespace mte
