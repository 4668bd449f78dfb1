// mte_replay.h — the replay kernels.
//
//   pair_kernel  — pass 1: two documents per wavefront, E in {1, 2} (<= 126
//                  segments each).  The wave alternates between its two
//                  documents op by op, so all documents of a 10k-doc batch
//                  are resident on the chip at once (one wave per doc would
//                  need 10k resident waves; the chip holds 8 per SIMD).
//   big_kernel   — pass 2: one document per wavefront, E in {4, 8, 16}
//                  (<= 1022 segments), for documents pass 1 escalated.
//   stream_kernel — pass 3 (mte_stream.h): larger documents, HBM-resident.
//
// Both run the same per-op step (doc_step) on a register-resident document.
// Op records (64 B compiled records, mte_kernels.h) are read with scalar
// loads straight into SGPRs (the op index is wave-uniform): the next op's
// first 32 bytes are in flight while the current op runs, and every 64 ops a
// vector load touches the next 64 records so the scalar loads hit L2.
#pragma once

#include <type_traits>

#include "mte_kernels.h"

// Build-time knobs (tools/variants.sh builds A/B variants; defaults are the product build).
// MTE_FAIR_PRIO: 0 = hardware age order, 1 = 4 linear bands of work left, 2 = geometric bands,
// 3 = bands around the global progress (one returning atomic per burst; measured 33.9 ms vs
// 23.9 ms on config 3: the single contended counter costs more than the balance gains),
// 4 = bands around the previous run's schedule (product: 22.6 ms; band 1 on the first run).
#ifndef MTE_PAIR_WAVES  // pass-1 waves per SIMD the register budget is sized for (5: 96 VGPRs, 4: 128)
#define MTE_PAIR_WAVES 5
#endif
#ifndef MTE_BURST
#define MTE_BURST 128
#endif
#ifndef MTE_PASS1_EMAX
#define MTE_PASS1_EMAX 4
#endif
#ifndef MTE_FAIR_PRIO  // pass-1 issue priority policy (below)
#define MTE_FAIR_PRIO 4
#endif
#ifndef MTE_VREC  // 1: pass-1 op records fetched with vector loads (vmcnt), 0: scalar loads (lgkmcnt)
// 1 since round 6 (profiles/r06/ab/vrec/): config 3 at 10k documents 22.3 -> 21.6 ms (an LDS wait
// no longer waits for the next record's scalar load too); 1,250 documents 8.01 -> 8.07 ms
#define MTE_VREC 1
#endif
#ifndef MTE_E1_DPP  // 1: the E = 1 shift moves slots with DPP instead of ds_bpermute
#define MTE_E1_DPP 0
#endif
#ifndef MTE_OUTLINE  // 1: pass-1 tiers as out-of-line functions (measured: same time, 1.7x the HBM traffic)
#define MTE_OUTLINE 0
#endif
#ifndef MTE_STEPV_EMAX  // tiers up to this E run the per-slot-flag step (doc_step_v), larger ones doc_step
#define MTE_STEPV_EMAX 4
#endif
#ifndef MTE_EARLY_PROPS  // 1: pass-1 tiers load an op's compiled propset at the op's start
#define MTE_EARLY_PROPS 0
#endif
#ifndef MTE_DIAG_NOPAYLOAD  // diagnostics only (wrong results): pass-1 tiers skip the text-offset / property planes
#define MTE_DIAG_NOPAYLOAD 0
#endif
#ifndef MTE_OUTLINE_E4  // 1: only the rare E = 4 tier out of line (the E <= 2 loops get the registers)
#define MTE_OUTLINE_E4 0
#endif

namespace mte {

constexpr uint32_t kBurst = MTE_BURST;  // ops per burst in pass 1

// per-document replay state (wave-uniform); op cursors are 32-bit, relative
// to the document's first record of the batch
struct DocRun {
  int doc;
  int n;
  int32_t min_seq, cur_seq;
  int32_t status;
  uint32_t flags;
  bool running;
  const uint4* recp;  // the doc's first op record (2 x uint4 each)
  uint32_t k, k1;     // current op, end
};

__device__ __forceinline__ void fence_wave() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- scalar op fetch -------------------------------------------------------
// Records are read through the constant address space: the op index is
// wave-uniform, so the compiler emits s_load straight into SGPRs (no vector
// load, no readfirstlane) and tracks the lgkmcnt wait itself.  The records
// are never written while a replay kernel runs.
typedef int32_t s8v __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) s8v* cs8p;

__device__ __forceinline__ s8v sload8(const uint4* p) { return *(cs8p)(const void*)p; }
// compiled propset `psi` (mte_kernels.h)
__device__ __forceinline__ s8v sload_props(const ReplayArgs& a, uint32_t psi) { return sload8(a.cps + 2 * psi); }

// op record through a vector load: dword i in lane i < 8.  Its wait is on
// vmcnt, so the LDS traffic of an op (shift permutes, zamboni) never waits for
// the next record as it does for a scalar load in flight (SMEM and LDS share
// lgkmcnt, and SMEM returns out of order, so any LDS wait becomes lgkmcnt(0)).
__device__ __forceinline__ uint32_t vload_rec8(const uint4* rec) {
  const int l = __lane_id();
  return l < 8 ? reinterpret_cast<const uint32_t*>(rec)[l] : 0u;
}
#if MTE_VREC
typedef uint32_t RecV;  // the prefetched record of the pass-1 tiers (doc_step_v)
#else
typedef s8v RecV;
#endif
__device__ __forceinline__ void swait(s8v&) {}

// L2 prefetch: lane l touches record `from + 4 l` (one 128-B line per lane,
// 256 records).  The loaded word is folded into `sink` one prefetch later, so
// the wait for it never stalls.
constexpr uint32_t kTouchSpan = 4 * kWave;
__device__ __forceinline__ void touch_records(const DocRun& D, uint32_t from, uint32_t& pending, uint32_t& sink) {
  sink ^= pending;
  const uint32_t r = from + 4u * (uint32_t)lane_id();
  pending = r < D.k1 + kRecPad ? reinterpret_cast<const uint32_t*>(D.recp + 2 * r)[0] : 0u;
}

// ISegment.addProperties for a remote op (segmentPropertiesManager.ts:63-151):
// entries in order, value 0 (null) deletes.  The first two entries come with
// the compiled propset record; longer sets are read here.  Applied to the slots with
// sel[j] set (E slots per lane, K planes); no lambdas, so the register arrays
// never need an address.
#ifndef MTE_SET_PLANE_SWITCH
#define MTE_SET_PLANE_SWITCH 1
#endif

template <int E>
__device__ __forceinline__ void set_one_plane(uint32_t (&p)[E], const bool (&sel)[E], uint32_t val) {
#pragma unroll
  for (int jj = 0; jj < E; jj++) {
    uint32_t x = sel[jj] ? val : p[jj];
    asm volatile("" : "+v"(x));  // keeps each case's selects distinct, so no case merging into p[key]
    p[jj] = x;
  }
}

template <int E, int K>
__device__ __forceinline__ void set_plane(uint32_t (&pr)[kRP<K>][E], const bool (&sel)[E], uint32_t key,
                                          uint32_t val) {
  if constexpr (K == kPack4) {
    // byte `key` of the packed plane (key < 4 and val < 256: the host's choice)
    const uint32_t sh = key * 8u, keep = ~(0xffu << sh), v = val << sh;
#pragma unroll
    for (int jj = 0; jj < E; jj++) pr[0][jj] = sel[jj] ? ((pr[0][jj] & keep) | v) : pr[0][jj];
    return;
  }
#if MTE_SET_PLANE_SWITCH
  // `key` is wave-uniform: one scalar branch picks the plane, so only that
  // plane's E selects issue (the branch-free form costs K x E selects)
  switch (key) {
    case 0: if constexpr (K > 0) set_one_plane<E>(pr[K > 0 ? 0 : 0], sel, val); break;
    case 1: if constexpr (K > 1) set_one_plane<E>(pr[K > 1 ? 1 : 0], sel, val); break;
    case 2: if constexpr (K > 2) set_one_plane<E>(pr[K > 2 ? 2 : 0], sel, val); break;
    case 3: if constexpr (K > 3) set_one_plane<E>(pr[K > 3 ? 3 : 0], sel, val); break;
    case 4: if constexpr (K > 4) set_one_plane<E>(pr[K > 4 ? 4 : 0], sel, val); break;
    case 5: if constexpr (K > 5) set_one_plane<E>(pr[K > 5 ? 5 : 0], sel, val); break;
    case 6: if constexpr (K > 6) set_one_plane<E>(pr[K > 6 ? 6 : 0], sel, val); break;
    case 7: if constexpr (K > 7) set_one_plane<E>(pr[K > 7 ? 7 : 0], sel, val); break;
    default: break;
  }
#else
  // branch-free over planes: a `kk == key` branch gets folded into pr[key],
  // a dynamic index that would push the whole register file to scratch
#pragma unroll
  for (int kk = 0; kk < K; kk++) {
    const bool hit = (uint32_t)kk == key;
#pragma unroll
    for (int jj = 0; jj < E; jj++) pr[kk][jj] = (hit && sel[jj]) ? val : pr[kk][jj];
  }
#endif
}

template <int E, int K>
__device__ __forceinline__ void apply_props(uint32_t (&pr)[kRP<K>][E], const bool (&sel)[E], uint32_t pk,
                                            uint32_t v0, uint32_t v1, uint32_t psi, const ReplayArgs& a) {
  const uint32_t k0 = pk & 0xffu, k1 = (pk >> 8) & 0xffu;
  // kPack4: the side key never goes into the packed bytes (ReplayArgs::side_key)
  const uint32_t skip = K == kPack4 ? a.side_key : kNoKey;
  if (k0 != kNoKey && k0 != skip) set_plane<E, K>(pr, sel, k0, v0);
  if (k1 != kNoKey && k1 != skip) set_plane<E, K>(pr, sel, k1, v1);
  if (pk >> 16) {
    const mte_propset ps = a.ps[psi];
    for (uint32_t t = 2; t < ps.count; t++) {
      const mte_prop p = a.pe[ps.first + t];
      if (p.key < a.n_keys && p.key != skip) set_plane<E, K>(pr, sel, uni(p.key), uni(p.value));
    }
  }
}

// one plane of the zamboni stream compaction: scatter kept slots to their
// compacted index in LDS, gather back lane-major
template <int E, typename T>
__device__ __forceinline__ void compact_plane(T (&F)[E], const bool (&keep)[E], const int32_t (&dst)[E],
                                              uint32_t* zlds) {
  const int base = lane_id() * E;
#pragma unroll
  for (int jj = 0; jj < E; jj++)
    if (keep[jj]) zlds[dst[jj]] = (uint32_t)F[jj];
  fence_wave();
#pragma unroll
  for (int jj = 0; jj < E; jj++) F[jj] = (T)zlds[base + jj];
  fence_wave();
}

template <int E, int NF, typename T>
__device__ __forceinline__ void shift_grab(uint32_t (&last)[NF], uint32_t (&last2)[NF], int f, const T (&F)[E]) {
  last[f] = (uint32_t)F[E - 1];
  last2[f] = (uint32_t)F[E >= 2 ? E - 2 : 0];
}

template <int E, int NF, typename T>
__device__ __forceinline__ void shift_apply(T (&F)[E], const uint32_t (&p1)[NF], const uint32_t (&p2)[NF], int f,
                                            const bool (&g1)[E], const bool (&g2)[E]) {
#pragma unroll
  for (int j = E - 1; j >= 0; j--) {
    const T m1 = (j >= 1) ? F[j >= 1 ? j - 1 : 0] : (T)p1[f];
    const T m2 = (j >= 2) ? F[j >= 2 ? j - 2 : 0] : ((j == 1) ? (T)p1[f] : (T)p2[f]);
    F[j] = g2[j] ? m2 : (g1[j] ? m1 : F[j]);
  }
}

// Shift every plane (and, for range ops, the L / P planes): new[i] =
// old[i - d(i)] with d(i) = (i > t1) + (i > t2), as pull_shift does for one
// plane.  The cross-lane moves of all planes are issued first and the selects
// after, so no DPP read waits on the VALU write just before it (a chained
// move per plane costs two hazard nops each).
template <int E, typename T>
__device__ __forceinline__ void shift_perm(T (&F)[E], int addr) {
  F[0] = (T)__builtin_amdgcn_ds_bpermute(addr, (int32_t)F[0]);
}

template <int E, int K, bool LP>
__device__ __forceinline__ void shift_all(Regs<E, K>& R, int32_t (&L)[E], int32_t (&P)[E], int t1, int t2) {
  if constexpr (E == 1) {
    // one slot per lane: lane l pulls lane l - d(l) through the LDS crossbar
    // (ds_bpermute: one LDS-pipe instruction per plane instead of two DPP
    // moves and two selects on the VALU)
    const int l = lane_id();
    const int addr = (l - (l > t1 ? 1 : 0) - (l > t2 ? 1 : 0)) << 2;
    shift_perm<E>(R.len, addr);
    shift_perm<E>(R.seq, addr);
    shift_perm<E>(R.rseq, addr);
    shift_perm<E>(R.rmask, addr);
    shift_perm<E>(R.meta, addr);
    shift_perm<E>(R.toff, addr);
#pragma unroll
    for (int k = 0; k < kRegPlanes<K>; k++) shift_perm<E>(R.pr[k], addr);
    if constexpr (LP) {
      shift_perm<E>(L, addr);
      shift_perm<E>(P, addr);
    }
    return;
  }
  constexpr int NF = kFieldPlanes + kRegPlanes<K> + (LP ? 2 : 0);
  uint32_t last[NF], last2[NF];
  shift_grab<E, NF>(last, last2, 0, R.len);
  shift_grab<E, NF>(last, last2, 1, R.seq);
  shift_grab<E, NF>(last, last2, 2, R.rseq);
  shift_grab<E, NF>(last, last2, 3, R.rmask);
  shift_grab<E, NF>(last, last2, 4, R.meta);
  shift_grab<E, NF>(last, last2, 5, R.toff);
#pragma unroll
  for (int k = 0; k < kRegPlanes<K>; k++) shift_grab<E, NF>(last, last2, kFieldPlanes + k, R.pr[k]);
  if constexpr (LP) {
    shift_grab<E, NF>(last, last2, NF - 2, L);
    shift_grab<E, NF>(last, last2, NF - 1, P);
  }
  uint32_t p1[NF], p2[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) p1[f] = (uint32_t)lane_prev((int32_t)last[f]);  // old[base - 1]
#pragma unroll
  for (int f = 0; f < NF; f++) p2[f] = (uint32_t)lane_prev((int32_t)(E >= 2 ? last2[f] : p1[f]));  // old[base - 2]
  const int base = lane_id() * E;
  bool g1[E], g2[E];
#pragma unroll
  for (int j = 0; j < E; j++) {
    g1[j] = base + j > t1;
    g2[j] = base + j > t2;
  }
  shift_apply<E, NF>(R.len, p1, p2, 0, g1, g2);
  shift_apply<E, NF>(R.seq, p1, p2, 1, g1, g2);
  shift_apply<E, NF>(R.rseq, p1, p2, 2, g1, g2);
  shift_apply<E, NF>(R.rmask, p1, p2, 3, g1, g2);
  shift_apply<E, NF>(R.meta, p1, p2, 4, g1, g2);
  shift_apply<E, NF>(R.toff, p1, p2, 5, g1, g2);
#pragma unroll
  for (int k = 0; k < kRegPlanes<K>; k++) shift_apply<E, NF>(R.pr[k], p1, p2, kFieldPlanes + k, g1, g2);
  if constexpr (LP) {
    shift_apply<E, NF>(L, p1, p2, NF - 2, g1, g2);
    shift_apply<E, NF>(P, p1, p2, NF - 1, g1, g2);
  }
}

template <int E, int K>
__device__ __forceinline__ void load_regs(Regs<E, K>& R, const DocRun& D, const ReplayArgs& a) {
  const uint32_t* pl = a.planes + (uint64_t)D.doc * a.cap;
  const uint64_t st = a.stride;
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    const bool v = i < D.n;
    const uint32_t x = (uint32_t)(v ? i : 0);
    R.len[j] = v ? (int32_t)pl[x] : 0;
    R.seq[j] = v ? (int32_t)pl[st + x] : 0;
    R.rseq[j] = v ? (int32_t)pl[2 * st + x] : kPad;
    R.rmask[j] = v ? pl[3 * st + x] : 0u;
    R.meta[j] = v ? pl[4 * st + x] : 0u;
    R.toff[j] = v ? pl[5 * st + x] : 0u;
    if constexpr (K == kPack4) {
      // the side key's value of a marker rides in its toff register
      uint32_t w = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t pv = v ? pl[(kFieldPlanes + k) * st + x] : 0u;
        if ((uint32_t)k == a.side_key) R.toff[j] = (R.meta[j] >> 8) ? pv : R.toff[j];
        else w |= pv << (8 * k);
      }
      R.pr[0][j] = w;
    } else {
#pragma unroll
      for (int k = 0; k < K; k++) R.pr[k][j] = v ? pl[(kFieldPlanes + k) * st + x] : 0u;
    }
  }
}

template <int E, int K>
__device__ __forceinline__ void store_regs(const Regs<E, K>& R, const DocRun& D, const ReplayArgs& a) {
  uint32_t* pl = a.planes + (uint64_t)D.doc * a.cap;
  const uint64_t st = a.stride;
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    if (i < D.n) {
      const uint32_t x = (uint32_t)i;
      pl[x] = (uint32_t)R.len[j];
      pl[st + x] = (uint32_t)R.seq[j];
      pl[2 * st + x] = (uint32_t)R.rseq[j];
      pl[3 * st + x] = R.rmask[j];
      pl[4 * st + x] = R.meta[j];
      if constexpr (K == kPack4) {
        const bool mk = (R.meta[j] >> 8) != 0 && a.side_key < 4u;
        pl[5 * st + x] = mk ? 0u : R.toff[j];
#pragma unroll
        for (int k = 0; k < 4; k++)
          pl[(kFieldPlanes + k) * st + x] =
              (uint32_t)k == a.side_key ? (mk ? R.toff[j] : 0u) : (R.pr[0][j] >> (8 * k)) & 0xffu;
      } else {
        pl[5 * st + x] = R.toff[j];
#pragma unroll
        for (int k = 0; k < K; k++) pl[(kFieldPlanes + k) * st + x] = R.pr[k][j];
      }
    }
  }
}

// A split of one leaf, applied after the shift: the head keeps [0, o) at
// slot h, the tail [o, len) lands at slot tl with its text offset advanced.
struct SplitPatch {
  int h, tl;      // -1: none
  int32_t o, len; // offset, length of the leaf before the split
  uint32_t toff;  // text offset of the leaf before the split
  int32_t pos;    // document position of the tail (P of the tail slot)
};

// Statistics (mte_stats: the Client.measureOps-style accounting and the
// algorithmic byte count) are a compile-time option of the replay kernels:
// S = false drops every counter update from the per-op path.
#define MTE_STAT(...) \
  if constexpr (S) {    \
    __VA_ARGS__         \
  }

// The collab-window error of an applied op, checked in the reference's order:
// completeAndLogOp (client.ts:525-528), then updateSeqNumbers (937-945) ->
// setMinSeq (mergeTree.ts:1078-1084), which sets currentSeq before its asserts.
__device__ __forceinline__ int window_error(DocRun& D, bool live, bool end, int32_t s, int32_t msn) {
  if (live) {
    if (!(D.cur_seq < s)) return MTE_E_SEQ_ORDER;
    if (!(D.min_seq <= msn)) return MTE_E_MSN_ORDER;
  }
  if (end) {
    if (!(D.cur_seq <= s)) return MTE_E_SEQ_ORDER;
    D.cur_seq = s;
    if (!(msn <= s)) return MTE_E_MSN_GT_SEQ;
    if (!(D.min_seq <= msn)) return MTE_E_MSN_ORDER;
  }
  return MTE_E_STATE;  // unreachable: the caller saw a violation
}

// One op record of one document: Client.applyMsg -> applyRemoteOp ->
// insertSegments / markRangeRemoved / annotateRange -> updateSeqNumbers
// (client.ts:918-945).  Returns 0 (applied), 1 (re-pick the register tier
// before this op, or after a compaction that shrank the doc), or a negative
// MTE_E_* (the doc stops).
//
// Structure: a scalar decision phase (visibility lengths, prefix scan and the
// split / insert-slot lookups, then wave-uniform shift thresholds and split
// patches) followed by ONE vector apply phase shared by all op types, so the
// register state flows through a single path (no per-branch copies).
template <int E, int K, bool S>
__device__ __forceinline__ int doc_step(Regs<E, K>& R, DocRun& D, uint32_t (&st)[kNumStats], s8v& cur,
                                        const ReplayArgs& a, uint32_t* zlds, int emin) {
  const int l = lane_id();
  const int base = l * E;
  const int lim = kWave * E < (int)a.cap ? kWave * E : (int)a.cap;
  if (D.n + 2 > lim) return 1;
  if constexpr (S) {
    if (st[kStOps] >= (1u << 20)) return 1;
  }

  // ---- op record: words 0..7 were prefetched into `cur` -------------------
  const s8v op = cur;
  const uint4* rec = D.recp + 2 * D.k;
  // next op, in flight during this one; past a doc's last op this reads the
  // next doc's first record or the zeroed kRecPad tail (never used).  Scalar
  // loads complete out of order, so a wait for `op` is an lgkmcnt(0) that
  // would also wait for this prefetch: the empty asm takes `op` as an input
  // and hands the prefetch its address, so the wait lands before the issue.
  uint64_t next = reinterpret_cast<uint64_t>(rec + 2);
  asm volatile("" : "+s"(next) : "s"(op));
  cur = sload8(reinterpret_cast<const uint4*>(next));
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  MTE_STAT(st[kStOps]++;)
  MTE_STAT(st[kStMaxSegs] = (uint32_t)D.n > st[kStMaxSegs] ? (uint32_t)D.n : st[kStMaxSegs];)
  const int32_t s = op[0];
  const int32_t msn = op[2];
  int n = D.n;

  if (type == MTE_OP_INSERT || type == MTE_OP_REMOVE || type == MTE_OP_ANNOTATE) {
    const bool ins = type == MTE_OP_INSERT;
    MTE_STAT(st[kStScanned] += (uint32_t)n;)
    const int32_t r = op[1];
    const int32_t pos1 = op[4], pos2 = op[5];
    int32_t L[E], P[E];
    leaf_lengths<E, K>(R, r, c + 1, (int)c, D.min_seq, (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0, L);
    const int32_t total = prefix<E>(L, P);

    // ---- scalar decisions ------------------------------------------------
    int t1 = INT32_MAX, t2 = INT32_MAX;  // shift thresholds (pull_shift)
    SplitPatch pa{-1, -1, 0, 0, 0u, 0}, pb{-1, -1, 0, 0, 0u, 0};
    int g = -1;  // slot of the new segment
    if (ins) {
      // Client.applyInsertOp -> MergeTree.insertSegments (client.ts:470-505,
      // mergeTree.ts:1394-1422): ensureIntervalBoundary, then insertingWalk
      const int32_t nlen = (flags & MTE_F_MARKER) ? 1 : pos2;  // markers have length 1
      int32_t off = 0;
      const int xs = find_split<E>(L, P, pos1, &off);
      if (xs >= 0) {
        pa.h = xs;
        pa.o = off;
        pa.len = bcast<E>(R.len, xs);
        pa.toff = bcast<E>(R.toff, xs);
        t1 = xs;
        if (nlen > 0) {  // [head][new][tail]
          t2 = xs + 1;
          g = xs + 1;
          pa.tl = xs + 2;
          MTE_STAT(st[kStWritten] += 3;)
        } else {
          pa.tl = xs + 1;
          MTE_STAT(st[kStWritten] += 2;)
        }
        n += 1;
      } else if (nlen > 0) {
        g = find_slot<E>(L, P, pos1);
        if (g < 0) {
          if (pos1 > total) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
          g = n;
        }
        t1 = g - 1;
        MTE_STAT(st[kStWritten] += 1;)
      }
      if (nlen > 0) n += 1;
    } else {
      // markRangeRemoved (mergeTree.ts:1908-2000) / annotateRange
      // (1864-1906): the two ensureIntervalBoundary calls, ordered by position
      const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
      int32_t o1 = 0, o2 = 0;
      int x1 = find_split<E>(L, P, b1, &o1);
      int x2 = b2 != b1 ? find_split<E>(L, P, b2, &o2) : -1;
      int32_t bb1 = b1;
      if (x1 < 0) {
        x1 = x2;
        o1 = o2;
        bb1 = b2;
        x2 = -1;
      }
      if (x1 >= 0) {
        pa.h = x1;
        pa.tl = x1 + 1;
        pa.o = o1;
        pa.len = bcast<E>(R.len, x1);
        pa.toff = bcast<E>(R.toff, x1);
        pa.pos = bb1;
        t1 = x1;
        n += 1;
        MTE_STAT(st[kStWritten] += 2;)
        if (x2 >= 0) {
          // after the first split the second leaf sits at x2 + 1; when both
          // boundaries fall in one leaf it is the first split's tail
          const bool same = x2 == x1;
          pb.h = x2 + 1;
          pb.tl = x2 + 2;
          pb.o = same ? o2 - o1 : o2;
          pb.len = same ? pa.len - o1 : bcast<E>(R.len, x2);
          pb.toff = same ? pa.toff + (uint32_t)o1 : bcast<E>(R.toff, x2);
          pb.pos = b2;
          t2 = x2 + 1;
          n += 1;
          MTE_STAT(st[kStWritten] += 2;)
        }
      }
    }

    // ---- vector apply ----------------------------------------------------
    if (t1 != INT32_MAX) {
      if (ins) shift_all<E, K, false>(R, L, P, t1, t2);
      else shift_all<E, K, true>(R, L, P, t1, t2);
    }
#pragma unroll
    for (int pi = 0; pi < 2; pi++) {
      const SplitPatch& p = pi == 0 ? pa : pb;
      if (p.h >= 0) {
#pragma unroll
        for (int jj = 0; jj < E; jj++) {
          const bool hd = base + jj == p.h, tl = base + jj == p.tl;
          R.len[jj] = hd ? p.o : (tl ? p.len - p.o : R.len[jj]);
          R.toff[jj] = tl ? p.toff + (uint32_t)p.o : R.toff[jj];
          if (!ins) {
            L[jj] = hd ? p.o : (tl ? p.len - p.o : L[jj]);
            P[jj] = tl ? p.pos : P[jj];
          }
        }
      }
    }
    if (g >= 0) {
      // the new segment (mergeTree.ts:1599-1611, textSegment.ts:40-48,
      // mergeTreeNodes.ts:602-609)
      const bool marker = (flags & MTE_F_MARKER) != 0;
      const uint32_t meta = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
      const uint32_t toff = marker ? 0u : a.text_base + (uint32_t)op[6];
      const uint32_t psi = (uint32_t)op[7];
      uint32_t pr[kRP<K>][1];
      const bool one[1] = {true};
#pragma unroll
      for (int kk = 0; kk < kRP<K>; kk++) pr[kk][0] = 0;
      if (K > 0 && psi != MTE_NO_PROPS) {
        const s8v q2 = sload_props(a, psi);
        apply_props<1, K>(pr, one, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
        MTE_STAT(st[kStPwrites] += (uint32_t)q2[3];)
      }
      MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
      const int32_t nlen = marker ? 1 : pos2;
#pragma unroll
      for (int jj = 0; jj < E; jj++) {
        const bool at = base + jj == g;
        R.len[jj] = at ? nlen : R.len[jj];
        R.seq[jj] = at ? s : R.seq[jj];
        R.rseq[jj] = at ? kNone : R.rseq[jj];
        R.rmask[jj] = at ? 0u : R.rmask[jj];
        R.meta[jj] = at ? meta : R.meta[jj];
        R.toff[jj] = at ? toff : R.toff[jj];
#pragma unroll
        for (int kk = 0; kk < kRegPlanes<K>; kk++) R.pr[kk][jj] = at ? pr[kk][0] : R.pr[kk][jj];
      }
    }
    if (!ins && pos2 != pos1) {
      // nodeMap (mergeTree.ts:2274-2330): after the splits no visible leaf
      // straddles start or end, so a leaf is in range iff start <= P < end
      bool in[E];
      uint32_t cnt = 0;
#pragma unroll
      for (int jj = 0; jj < E; jj++) {
        in[jj] = L[jj] > 0 && P[jj] >= pos1 && P[jj] < pos2;
        cnt += (uint32_t)__popcll(__ballot(in[jj]));
      }
      MTE_STAT(st[kStWritten] += cnt;)
      if (type == MTE_OP_REMOVE) {
        // markRemoved (mergeTree.ts:1924-1962): keep the earliest removedSeq,
        // add the client to removedClientIds
        const uint32_t bit = 1u << c;
#pragma unroll
        for (int jj = 0; jj < E; jj++) {
          R.rseq[jj] = (in[jj] && R.rseq[jj] == kNone) ? s : R.rseq[jj];
          R.rmask[jj] = in[jj] ? (R.rmask[jj] | bit) : R.rmask[jj];
        }
      } else if (cnt > 0) {
        // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
        const uint32_t psi = (uint32_t)op[6];
        const s8v q2 = sload_props(a, psi);
        if (flags & MTE_F_REWRITE) {
#pragma unroll
          for (int kk = 0; kk < kRegPlanes<K>; kk++)
#pragma unroll
            for (int jj = 0; jj < E; jj++) R.pr[kk][jj] = in[jj] ? 0u : R.pr[kk][jj];
        }
        apply_props<E, K>(R.pr, in, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
        MTE_STAT(st[kStPwrites] += cnt * (uint32_t)q2[3];)
      }
    }
  } else if (type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  D.n = n;
  D.k++;

  // Client.completeAndLogOp (client.ts:525-528) and updateSeqNumbers
  // (client.ts:937-945) -> setMinSeq (mergeTree.ts:1077-1093): one combined
  // test on the fast path, the exact code (in the reference's order) after
  const bool live = type != MTE_OP_NOOP, end = (flags & MTE_F_MSG_END) != 0;
  const bool bad = (live & (s <= D.cur_seq)) | (end & (s < D.cur_seq)) | ((live | end) & (msn < D.min_seq)) |
                   (end & (msn > s));
  if (bad) return window_error(D, live, end, s, msn);
  if (end) {
    D.cur_seq = s;
    if (msn > D.min_seq) {
      D.min_seq = msn;
      // zamboni: drop tombstones with removedSeq <= minSeq (padding included)
      // by a stream compaction staged through LDS
      bool keep[E];
      int32_t cntl = 0;
#pragma unroll
      for (int jj = 0; jj < E; jj++) {
        keep[jj] = R.rseq[jj] > msn;
        cntl += keep[jj] ? 1 : 0;
      }
      const int32_t incl = wave_incl_scan(cntl);
      const int n_new = rdlane(incl, kWave - 1);
      if (n_new != n) {
        int32_t dst[E];
        int32_t d0 = incl - cntl;
#pragma unroll
        for (int jj = 0; jj < E; jj++) {
          dst[jj] = d0;
          d0 += keep[jj] ? 1 : 0;
        }
        compact_plane<E>(R.len, keep, dst, zlds);
        compact_plane<E>(R.seq, keep, dst, zlds);
        compact_plane<E>(R.rseq, keep, dst, zlds);
        compact_plane<E>(R.rmask, keep, dst, zlds);
        compact_plane<E>(R.meta, keep, dst, zlds);
        compact_plane<E>(R.toff, keep, dst, zlds);
#pragma unroll
        for (int kk = 0; kk < kRegPlanes<K>; kk++) compact_plane<E>(R.pr[kk], keep, dst, zlds);
#pragma unroll
        for (int jj = 0; jj < E; jj++) {
          const bool pad = base + jj >= n_new;
          R.rseq[jj] = pad ? kPad : R.rseq[jj];
          R.len[jj] = pad ? 0 : R.len[jj];
        }
        D.n = n_new;
        // drop to a smaller register tier once the doc fits in half of it
        if (E > emin && n_new + 2 + 16 <= 32 * E) return 1;
      }
    }
  }
  return 0;
}

}  // namespace mte

#include "mte_step1.h"

namespace mte {

__device__ __forceinline__ void run_init(DocRun& D, const ReplayArgs& a, int doc, bool escalated_only) {
  D.doc = doc;
  D.running = false;
  D.n = 0;
  D.status = 0;
  D.k = D.k1 = 0;
  if (doc < 0) return;
  const DocHdr h = a.hdr[doc];
  const uint64_t kb = a.op_off[doc];
  D.n = h.nseg;
  D.min_seq = h.min_seq;
  D.cur_seq = h.cur_seq;
  D.status = h.status;
  D.flags = h.flags;
  D.recp = a.recs + 2 * kb;
  D.k = h.resume;
  D.k1 = (uint32_t)(a.op_off[doc + 1] - kb);
  if (h.status != 0) return;
  if (escalated_only && !(h.flags & kHdrNeedsEsc)) return;
  D.flags &= ~kHdrNeedsEsc;
  D.running = D.k < D.k1;
}

// add the 32-bit per-doc counters into the doc's 64-bit stats in HBM
__device__ __forceinline__ void run_flush_stats(const DocRun& D, uint32_t (&st)[kNumStats], const ReplayArgs& a) {
  if (D.doc >= 0 && lane_id() == 0) {
    unsigned long long* sd = a.stats + (size_t)D.doc * kNumStats;
#pragma unroll
    for (int t = 0; t < kNumStats; t++) {
      if (t == kStMaxSegs) sd[t] = sd[t] > st[t] ? sd[t] : st[t];
      else sd[t] += st[t];
    }
  }
#pragma unroll
  for (int t = 0; t < kNumStats; t++) st[t] = 0;
}

__device__ __forceinline__ void run_finish(DocRun& D, const ReplayArgs& a) {
  if (D.doc < 0) return;
  if (lane_id() == 0) {
    DocHdr h;
    h.nseg = D.n;
    h.min_seq = D.min_seq;
    h.cur_seq = D.cur_seq;
    h.status = D.status;
    h.flags = D.flags;
    h.resume = D.k;
    h.pad0 = a.hdr[D.doc].pad0;  // MTE_DOC_ROUND_SYNC check state (round_sync_kernel)
    h.pad1 = a.hdr[D.doc].pad1;
    a.hdr[D.doc] = h;
  }
}

// handle a doc_step result: 0 keep going, otherwise the doc leaves the loop
__device__ __forceinline__ bool step_done(DocRun& D, int rc) {
  if (rc < 0) {
    D.status = rc;
    D.running = false;
    return true;
  }
  if (D.k >= D.k1) D.running = false;
  return rc != 0 || !D.running;
}

// One burst of up to `limit` ops of one document at register tier E: load
// its segments into VGPRs, replay, write them back.  Returns early when the
// document needs another tier or stops.
template <int E, int K, bool S>
__device__ __forceinline__ void burst_run(DocRun& D, const ReplayArgs& a, uint32_t* zlds, int emin, uint32_t limit) {
  Regs<E, K> R;
  uint32_t st[kNumStats] = {};
  load_regs<E, K>(R, D, a);
  const uint32_t kend = D.k1 - D.k > limit ? D.k + limit : D.k1;
  s8v cur;
  RecV vcur;
  if constexpr (E <= MTE_STEPV_EMAX) {
#if MTE_VREC
    vcur = vload_rec8(D.recp + 2 * D.k);
#else
    vcur = sload8(D.recp + 2 * D.k);
#endif
  } else {
    cur = sload8(D.recp + 2 * D.k);
  }
  uint32_t pending = 0, sink = 0;
  // L2 prefetch of the records: short bursts (pass 1) touch the span after
  // this burst once, at its start (the first burst its own span too); long
  // runs touch ahead every kTouchSpan / 2 ops
  const bool per_burst = limit <= kTouchSpan / 2;
  if (per_burst) touch_records(D, D.k == 0 ? 0u : D.k + limit, pending, sink);
  else touch_records(D, D.k + 16, pending, sink);
  for (;;) {
    if (!per_burst && (D.k & (kTouchSpan / 2 - 1)) == 0) touch_records(D, D.k + kTouchSpan / 2, pending, sink);
    int rc;
    if constexpr (E <= MTE_STEPV_EMAX) rc = doc_step_v<E, K, S>(R, D, st, vcur, a, zlds, emin);
    else rc = doc_step<E, K, S>(R, D, st, cur, a, zlds, emin);
    if (rc != 0) {
      if (rc < 0) {
        D.status = rc;
        D.running = false;
      }
      break;
    }
    if (D.k >= kend) break;
  }
  if (D.k >= D.k1) D.running = false;
  if constexpr (E > MTE_STEPV_EMAX) swait(cur);  // no scalar load may be left in flight
#if !MTE_VREC
  if constexpr (E <= MTE_STEPV_EMAX) swait(vcur);
#endif
  store_regs<E, K>(R, D, a);
  if constexpr (S) run_flush_stats(D, st, a);
  sink ^= pending;
  if (sink == 0x9e3779b9u && D.doc < 0) a.stats[0] = sink;  // keeps the prefetch loads alive
}

// tier for the next burst in pass 1 (E <= 4, 254 segments); larger documents
// continue in pass 2
__device__ __forceinline__ int pick_pass1_tier(DocRun& D, uint32_t cap) {
  if (D.n + 2 > (int)cap) {
    D.status = MTE_E_CAPACITY;
    D.running = false;
    return 0;
  }
  if (D.n + 2 <= kWave) return 1;
  if (D.n + 2 <= 2 * kWave) return 2;
  if (MTE_PASS1_EMAX == 3 && D.n + 2 <= 3 * kWave) return 3;
  if (MTE_PASS1_EMAX >= 4 && D.n + 2 <= 4 * kWave) return 4;
  D.flags |= kHdrNeedsEsc;  // continue in the big-doc pass
  D.running = false;
  return 0;
}

// ---- out-of-line pass-1 bursts (MTE_OUTLINE=1, an A/B variant) -------------
// Each register tier as its own (non-inlined) function, so the register
// allocator sizes each tier's op loop on its own: inlined together, the E = 4
// tier's pressure leaves spill code in the E = 1 / 2 loops.  Measured on
// config 3 (profiles/r01): no change in time (the spills are off the per-op
// dependency chain) and 1.7x the HBM traffic (caller/callee register saves per
// burst), so the product build inlines.  Arguments arrive in VGPRs under the
// call ABI; every one is wave-uniform, so it is made scalar again at entry.
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)uni((uint32_t)v) | ((uint64_t)uni((uint32_t)(v >> 32)) << 32);
}
template <typename T>
__device__ __forceinline__ T* unip(T* p) {
  return reinterpret_cast<T*>(uni64(reinterpret_cast<uint64_t>(p)));
}

__device__ __forceinline__ ReplayArgs uni_args(const ReplayArgs& a) {
  ReplayArgs u;
  u.hdr = unip(a.hdr);
  u.planes = unip(a.planes);
  u.stride = uni64(a.stride);
  u.cap = uni(a.cap);
  u.n_docs = uni(a.n_docs);
  u.recs = unip(a.recs);
  u.cps = unip(a.cps);
  u.op_off = unip(a.op_off);
  u.ps = unip(a.ps);
  u.pe = unip(a.pe);
  u.n_keys = uni(a.n_keys);
  u.text_base = uni(a.text_base);
  u.stats = unip(a.stats);
  u.pair_docs = unip(a.pair_docs);
  u.n_pairs = uni(a.n_pairs);
  return u;
}

struct BurstState {  // the mutable part of DocRun
  int32_t n, min_seq, cur_seq, status;
  uint32_t flags, k;
  int32_t running;
};

typedef __attribute__((address_space(3))) uint32_t* lds_u32p;

template <int E, int K, bool S>
__device__ __attribute__((noinline)) BurstState burst_call(BurstState io, int doc, const uint4* recp, uint32_t k1,
                                                           ReplayArgs a0, lds_u32p zl) {
  const ReplayArgs a = uni_args(a0);
  DocRun D;
  D.doc = uni((int32_t)doc);
  D.recp = unip(recp);
  D.k1 = uni(k1);
  D.n = uni(io.n);
  D.min_seq = uni(io.min_seq);
  D.cur_seq = uni(io.cur_seq);
  D.status = uni(io.status);
  D.flags = uni(io.flags);
  D.k = uni(io.k);
  D.running = uni(io.running) != 0;
  burst_run<E, K, S>(D, a, (uint32_t*)zl, 1, kBurst);
  return BurstState{D.n, D.min_seq, D.cur_seq, D.status, D.flags, D.k, D.running ? 1 : 0};
}

template <int E, int K, bool S>
__device__ __forceinline__ void burst_out(DocRun& D, const ReplayArgs& a, uint32_t* zlds) {
  const BurstState r = burst_call<E, K, S>(BurstState{D.n, D.min_seq, D.cur_seq, D.status, D.flags, D.k,
                                                      D.running ? 1 : 0},
                                           D.doc, D.recp, D.k1, a, (lds_u32p)zlds);
  D.n = uni(r.n);
  D.min_seq = uni(r.min_seq);
  D.cur_seq = uni(r.cur_seq);
  D.status = uni(r.status);
  D.flags = uni(r.flags);
  D.k = uni(r.k);
  D.running = uni(r.running) != 0;
}

template <int K, bool S>
__device__ __forceinline__ void pass1_burst(DocRun& D, const ReplayArgs& a, uint32_t* zlds) {
  const int e = pick_pass1_tier(D, a.cap);
#if MTE_OUTLINE
  if (e == 1) burst_out<1, K, S>(D, a, zlds);
  else if (e == 2) burst_out<2, K, S>(D, a, zlds);
  else if constexpr (MTE_PASS1_EMAX >= 4) {
    if (e == 4) burst_out<4, K, S>(D, a, zlds);
  }
#elif defined(MTE_ISA_STUDY)  // ISA inspection only: one tier
  if (e) burst_run<MTE_ISA_STUDY, K, S>(D, a, zlds, 1, kBurst);
#else
  if (e == 1) burst_run<1, K, S>(D, a, zlds, 1, kBurst);
  else if (e == 2) burst_run<2, K, S>(D, a, zlds, 1, kBurst);
  else if constexpr (MTE_PASS1_EMAX == 3) {
    if (e == 3) burst_run<3, K, S>(D, a, zlds, 1, kBurst);
  } else if constexpr (MTE_PASS1_EMAX >= 4) {
#if MTE_OUTLINE_E4
    if (e == 4) burst_out<4, K, S>(D, a, zlds);
#else
    if (e == 4) burst_run<4, K, S>(D, a, zlds, 1, kBurst);
#endif
  }
#endif
}

// DocRun <-> a DocHdr image in LDS (pass 1 keeps both documents of a pair
// there between bursts, so only the running document's state occupies SGPRs)
__device__ __forceinline__ bool run_from_lds(DocRun& D, const DocHdr* hl, int doc, const ReplayArgs& a) {
  const uint4 h0 = reinterpret_cast<const uint4*>(hl)[0], h1 = reinterpret_cast<const uint4*>(hl)[1];
  D.doc = doc;
  D.n = uni((int32_t)h0.x);
  D.min_seq = uni((int32_t)h0.y);
  D.cur_seq = uni((int32_t)h0.z);
  D.status = uni((int32_t)h0.w);
  D.flags = uni(h1.x);
  D.k = uni(h1.y);
  const uint64_t kb = a.op_off[doc];
  D.recp = a.recs + 2 * kb;
  D.k1 = (uint32_t)(a.op_off[doc + 1] - kb);
  D.running = D.status == 0 && D.k < D.k1 && !(D.flags & kHdrNeedsEsc);
  return D.running;
}

__device__ __forceinline__ void run_to_lds(const DocRun& D, DocHdr* hl) {
  if (lane_id() == 0) {
    uint4* p = reinterpret_cast<uint4*>(hl);
    p[0] = make_uint4((uint32_t)D.n, (uint32_t)D.min_seq, (uint32_t)D.cur_seq, (uint32_t)D.status);
    reinterpret_cast<uint2*>(hl)[2] = make_uint2(D.flags, D.k);  // pad0 / pad1 kept
  }
  fence_wave();
}

// Fair issue between the waves sharing a SIMD.  The SIMD arbiter favours the
// oldest wave, so with equal work per wave the youngest starves, then runs
// alone (latency-bound) at the end: measured on config 3 the pass-1 waves
// ended in five steps by dispatch order, 14.9 ms to 26.3 ms (tools/
// wave_clock.py).  Setting the priority from the work left (4 levels) keeps
// the waves of a SIMD abreast, so they finish together.
__device__ __forceinline__ void fair_prio(uint32_t left, uint32_t total) {
  if constexpr (MTE_FAIR_PRIO == 1) {
    const uint32_t q = (uint32_t)(((uint64_t)left * 4u) / (total ? total : 1u));
    if (q >= 3) __builtin_amdgcn_s_setprio(3);
    else if (q == 2) __builtin_amdgcn_s_setprio(2);
    else if (q == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  } else if constexpr (MTE_FAIR_PRIO >= 3) {
    // (pair_kernel computes the level itself)
  } else if constexpr (MTE_FAIR_PRIO == 2) {
    // geometric bands (> 1/4, > 3/32, > 1/32 of the work left): the last band,
    // where the waves fall back to age order, is short
    const uint64_t l32 = (uint64_t)left * 32u, t = total ? total : 1u;
    if (l32 > 8 * t) __builtin_amdgcn_s_setprio(3);
    else if (l32 > 3 * t) __builtin_amdgcn_s_setprio(2);
    else if (l32 > t) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
}

// pass 1: `a.group` documents per wavefront (1 when the batch fits the chip
// at one per wave), replayed in turn one burst each, so a 10k-document batch is
// resident on the chip at once with the register budget of one document
// (E <= 4); W = waves per SIMD the register budget is sized for
template <int K, bool S, int WPB, int W>
__global__ __launch_bounds__(WPB * kWave, W * 4 / WPB) void pair_kernel(ReplayArgs a) {
  __shared__ uint32_t zlds_all[WPB][kWave * 4];
  __shared__ DocHdr hl_all[WPB][kGroupMax];
  const int w = WPB == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int pair = (int)blockIdx.x * WPB + w;
  if (pair >= (int)a.n_pairs) return;
  if (a.wclock && lane_id() == 0) a.wclock[2 * pair] = __builtin_amdgcn_s_memrealtime();
  const int g = (int)a.group;
  DocHdr* hl = hl_all[w];
  uint32_t* zlds = zlds_all[w];
  uint32_t live = 0;  // bit t: document t still has ops to run in this pass
  uint32_t total = 0;  // ops of the group in this pass, and those left (for fair_prio)
  for (int t = 0; t < g; t++) {
    const int doc = (int)a.pair_docs[(uint32_t)g * (uint32_t)pair + (uint32_t)t];
    if (doc >= 0) {
      DocHdr h = a.hdr[doc];
      const bool rel = (h.flags & kHdrRel) != 0;  // the streamed pass's this batch
      if (!rel) h.flags &= ~kHdrNeedsEsc;
      if (lane_id() == 0) hl[t] = h;
      if (!rel) {
        live |= 1u << t;
        total += (uint32_t)(a.op_off[doc + 1] - a.op_off[doc]) - h.resume;
      }
    }
  }
  fence_wave();
  total = uni(total);
  uint32_t left = total;
  [[maybe_unused]] const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  if constexpr (MTE_FAIR_PRIO == 4) __builtin_amdgcn_s_setprio(2);
  else fair_prio(left, total);
  // one burst per iteration, the documents in turn; a single copy of the
  // burst code serves them all (the document is a runtime index)
  for (int t = 0; live; t = (t + 1 == g) ? 0 : t + 1) {
    if (!(live & (1u << t))) continue;
    const int doc = (int)a.pair_docs[(uint32_t)g * (uint32_t)pair + (uint32_t)t];
    DocRun D;
    const uint32_t k0 = hl[t].resume;
    if (run_from_lds(D, &hl[t], doc, a)) pass1_burst<K, S>(D, a, zlds);
    run_to_lds(D, &hl[t]);
    if (!D.running) live &= ~(1u << t);
    const uint32_t ran = uni(hl[t].resume - k0);
    left -= ran;
    if constexpr (MTE_FAIR_PRIO == 3) {
      // progress relative to all waves: the global count of applied ops comes
      // back from the atomic that adds this burst (its old value)
      unsigned long long gl = 0;
      if (lane_id() == 0) gl = atomicAdd(a.gdone, (unsigned long long)ran);
      gl = ((unsigned long long)uni((uint32_t)(gl >> 32)) << 32) | uni((uint32_t)gl);
      const unsigned long long mine = (unsigned long long)(total - left) * a.n_ops;  // my fraction x n_ops x total
      const unsigned long long all = gl * total;
      const unsigned long long band = (unsigned long long)total * a.n_ops / 64;  // 1/64 of the work
      if (mine + band < all) __builtin_amdgcn_s_setprio(3);
      else if (mine < all) __builtin_amdgcn_s_setprio(2);
      else if (mine < all + band) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    } else if constexpr (MTE_FAIR_PRIO == 4) {
      // against the schedule of the previous run (a.eta ticks for the whole
      // pass): behind it -> higher priority; without an estimate, by work left
      if (a.eta) {
        const unsigned long long el = __builtin_amdgcn_s_memrealtime() - t_start;
        const unsigned long long mine = (unsigned long long)(total - left) * a.eta;  // done/total vs el/eta
        const unsigned long long sched = el * total;
        const unsigned long long band = (unsigned long long)total * a.eta / 32;
        if (mine + band < sched) __builtin_amdgcn_s_setprio(3);
        else if (mine < sched) __builtin_amdgcn_s_setprio(2);
        else if (mine < sched + band) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      } else {
        fair_prio(left, total);
      }
    } else {
      fair_prio(left, total);
    }
  }
  if (lane_id() == 0) {
    for (int t = 0; t < g; t++) {
      const int doc = (int)a.pair_docs[(uint32_t)g * (uint32_t)pair + (uint32_t)t];
      if (doc >= 0) a.hdr[doc] = hl[t];  // resume = the op cursor
    }
    if (a.wclock) a.wclock[2 * pair + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// pass 2: one document per wavefront, for the documents pass 1 escalated
template <int K, bool S>
__global__ __launch_bounds__(256) void big_kernel(ReplayArgs a) {
  __shared__ uint32_t zlds_all[kDocsPerBlock][kWave * 16];
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int doc = (int)blockIdx.x * kDocsPerBlock + w;
  if (doc >= (int)a.n_docs) return;
  DocRun D;
  run_init(D, a, doc, true);
  if (!D.running && !(a.hdr[doc].flags & kHdrNeedsEsc)) return;  // untouched doc: leave the header alone
  if (D.flags & kHdrRel) {  // relative positions: on to the streamed pass
    D.flags |= kHdrNeedsEsc;
    D.running = false;
  }
  uint32_t* zlds = zlds_all[w];
  while (D.running) {
    const int n = D.n;
    if (n + 2 > (int)a.cap) {
      D.status = MTE_E_CAPACITY;
      break;
    }
    if (n + 2 > 16 * kWave) {  // beyond the register tiers: continue in pass 3 (mte_stream.h)
      D.flags |= kHdrNeedsEsc;
      break;
    }
    if (n + 2 <= 4 * kWave) burst_run<4, K, S>(D, a, zlds, 4, 1u << 19);
    else if (n + 2 <= 8 * kWave) burst_run<8, K, S>(D, a, zlds, 4, 1u << 19);
    else burst_run<16, K, S>(D, a, zlds, 4, 1u << 19);
  }
  run_finish(D, a);
}

}  // namespace mte
