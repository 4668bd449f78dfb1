// mte_kernels.h — gfx950 device code of the batched sequence-merge engine.
//
// Execution model (DESIGN.md "Kernels"): one 64-lane wavefront replays one
// document.  The document's segments live in VGPRs for the whole batch,
// lane-major: segment i is slot (i % E) of lane (i / E), E in {1,2,4,8,16}
// chosen from the segment count (a doc that outgrows 64*E - 2 segments is
// written back to HBM and resumed with a larger E).  Per op:
//   * perspective length of every segment for (refSeq, clientId, minSeq)
//     (mergeTree.ts:1003-1054), lane-local sums + a wavefront prefix scan
//     (replaces PartialSequenceLengths.getPartialLength, partialLengths.ts:667);
//   * split / insert-slot / range lookups by ballot over lanes;
//   * the split + insert is a "pull" shift of every field by 0/1/2 slots
//     (register moves inside a lane + one cross-lane shuffle);
//   * remove / annotate mark the segments of [start, end) in place;
//   * when minSeq advances, tombstones with removedSeq <= minSeq are dropped
//     by a stream compaction staged through LDS (zamboni, mergeTree.ts:800-838).
// Op records are wave-uniform and read through the scalar unit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mte.h"

namespace mte {

constexpr int kWave = 64;
constexpr int32_t kNone = INT32_MAX;     // "removedSeq undefined"
constexpr int kDocsPerBlock = 4;         // 4 independent waves per workgroup

// per-doc header in HBM (32 B)
struct DocHdr {
  int32_t nseg;
  int32_t min_seq;
  int32_t cur_seq;
  int32_t status;
  uint32_t flags;   // MTE_DOC_* | kHdrNeedsEsc
  uint32_t resume;  // ops of this batch already applied
  uint32_t pad0, pad1;
};
constexpr uint32_t kHdrNeedsEsc = 0x80000000u;

enum StatIdx { kStOps = 0, kStScanned, kStWritten, kStPwrites, kStUnits, kStMaxSegs, kNumStats };

// segment state, structure of arrays, doc-major: field[doc * cap + i]
struct SegSoA {
  int32_t* len;
  int32_t* seq;
  int32_t* rseq;
  uint32_t* rmask;
  uint32_t* meta;   // bits 0-7: clientId + 1 (0 = LocalClientId); 8-31: kind (0 text, 1+refType marker)
  uint32_t* toff;   // text offset in the ctx text arena
  uint32_t* props;  // plane k at props[k * plane_stride + doc * cap + i]
  uint64_t plane_stride;
};

struct ReplayArgs {
  DocHdr* hdr;
  SegSoA soa;
  uint32_t cap;
  uint32_t n_docs;
  const mte_op* ops;
  const uint64_t* op_off;
  const mte_propset* ps;
  const mte_prop* pe;
  uint32_t n_keys;
  uint32_t text_base;
  unsigned long long* stats;  // n_docs * kNumStats
};

// ---- wavefront primitives --------------------------------------------------

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int32_t t = __shfl_up(v, d, kWave);
    if (l >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ int32_t rdlane(int32_t v, int lane) {
  return __builtin_amdgcn_readlane(v, lane);
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

template <int E, typename T>
__device__ __forceinline__ T pick(const T (&F)[E], int j) {
  T v = F[0];
#pragma unroll
  for (int jj = 1; jj < E; jj++) v = (j == jj) ? F[jj] : v;
  return v;
}

// broadcast field value of global segment index idx (wave-uniform)
template <int E, typename T>
__device__ __forceinline__ T bcast(const T (&F)[E], int idx) {
  return rdlane(pick<E>(F, idx % E), idx / E);
}

template <int E, typename T>
__device__ __forceinline__ void put(T (&F)[E], int idx, T v) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++)
    if (base + j == idx) F[j] = v;
}

// new[i] = old[i - d(i)], d(i) = (i > s1) + (i > s2); slots s1, s2 are left for
// the caller to fill (s2 may be INT_MAX for a single special slot).
template <int E, typename T>
__device__ __forceinline__ void pull_shift(T (&F)[E], int s1, int s2) {
  const int l = lane_id();
  const int base = l * E;
  int32_t p1 = __shfl_up((int32_t)F[E - 1], 1, kWave);  // old[base - 1]
  int32_t p2;
  if constexpr (E >= 2) p2 = __shfl_up((int32_t)F[E - 2], 1, kWave);  // old[base - 2]
  else p2 = __shfl_up((int32_t)F[0], 2, kWave);
  T out[E];
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    T m1 = (j >= 1) ? F[j - 1] : (T)p1;
    T m2 = (j >= 2) ? F[j - 2] : ((j == 1) ? (T)p1 : (T)p2);
    const int d = (i > s1) + (i > s2);
    out[j] = d == 0 ? F[j] : (d == 1 ? m1 : m2);
  }
#pragma unroll
  for (int j = 0; j < E; j++) F[j] = out[j];
}

// ---- register-resident document --------------------------------------------

template <int E, int K>
struct Regs {
  int32_t len[E], seq[E], rseq[E];
  uint32_t rmask[E], meta[E], toff[E];
  uint32_t pr[K > 0 ? K : 1][E];
};

template <int E, int K>
__device__ __forceinline__ void shift_all(Regs<E, K>& R, int s1, int s2) {
  pull_shift<E>(R.len, s1, s2);
  pull_shift<E>(R.seq, s1, s2);
  pull_shift<E>(R.rseq, s1, s2);
  pull_shift<E>(R.rmask, s1, s2);
  pull_shift<E>(R.meta, s1, s2);
  pull_shift<E>(R.toff, s1, s2);
#pragma unroll
  for (int k = 0; k < K; k++) pull_shift<E>(R.pr[k], s1, s2);
}

// a whole segment, wave-uniform
template <int K>
struct Seg {
  int32_t len, seq, rseq;
  uint32_t rmask, meta, toff;
  uint32_t pr[K > 0 ? K : 1];
};

template <int E, int K>
__device__ __forceinline__ Seg<K> get_seg(const Regs<E, K>& R, int idx) {
  Seg<K> s;
  s.len = bcast<E>(R.len, idx);
  s.seq = bcast<E>(R.seq, idx);
  s.rseq = bcast<E>(R.rseq, idx);
  s.rmask = bcast<E>(R.rmask, idx);
  s.meta = bcast<E>(R.meta, idx);
  s.toff = bcast<E>(R.toff, idx);
#pragma unroll
  for (int k = 0; k < K; k++) s.pr[k] = bcast<E>(R.pr[k], idx);
  return s;
}

template <int E, int K>
__device__ __forceinline__ void put_seg(Regs<E, K>& R, int idx, const Seg<K>& s) {
  put<E>(R.len, idx, s.len);
  put<E>(R.seq, idx, s.seq);
  put<E>(R.rseq, idx, s.rseq);
  put<E>(R.rmask, idx, s.rmask);
  put<E>(R.meta, idx, s.meta);
  put<E>(R.toff, idx, s.toff);
#pragma unroll
  for (int k = 0; k < K; k++) put<E>(R.pr[k], idx, s.pr[k]);
}

// Perspective length (mergeTree.ts:1003-1026 new calc, 1028-1054 legacy);
// -1 = undefined.  Slots >= n are undefined.
template <int E, int K>
__device__ __forceinline__ void leaf_lengths(const Regs<E, K>& R, int n, int32_t r, int c, int32_t m,
                                             bool newcalc, int32_t (&L)[E]) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const bool removed = R.rseq[j] != kNone;
    const bool by_c = (R.rmask[j] >> c) & 1u;
    const int cli = (int)(R.meta[j] & 0xffu) - 1;
    const bool mine_or_seen = (R.seq[j] <= r) || (cli == c);
    int32_t l;
    if (newcalc) {
      const int32_t vis = mine_or_seen ? R.len[j] : 0;
      l = removed ? (R.rseq[j] <= m ? -1 : ((R.rseq[j] <= r || by_c) ? 0 : vis)) : vis;
    } else {
      if (removed && R.rseq[j] <= r) l = -1;
      else if (mine_or_seen) l = (removed && by_c) ? 0 : R.len[j];
      else l = removed ? -1 : 0;
    }
    L[j] = (base + j < n) ? l : -1;
  }
}

// exclusive prefix P of max(L,0); returns the total
template <int E>
__device__ __forceinline__ int32_t prefix(const int32_t (&L)[E], int32_t (&P)[E]) {
  int32_t s = 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    P[j] = s;
    s += L[j] > 0 ? L[j] : 0;
  }
  const int32_t incl = wave_incl_scan(s);
  const int32_t excl = incl - s;
#pragma unroll
  for (int j = 0; j < E; j++) P[j] += excl;
  return rdlane(incl, kWave - 1);
}

// ensureIntervalBoundary lookup (mergeTree.ts:1698-1702, 1681-1696): the leaf
// with L > 0 and P < pos < P + L.  Markers (L == 1) can never satisfy it.
// Returns the global index or -1; *off = pos - P.
template <int E>
__device__ __forceinline__ int find_split(const int32_t (&L)[E], const int32_t (&P)[E], int32_t pos,
                                          int32_t* off) {
  int jsel = -1;
  int32_t o = 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const bool cnd = L[j] > 0 && P[j] < pos && pos < P[j] + L[j];
    jsel = cnd ? j : jsel;
    o = cnd ? pos - P[j] : o;
  }
  const unsigned long long m = __ballot(jsel >= 0);
  if (!m) return -1;
  const int ls = __ffsll((long long)m) - 1;
  *off = rdlane(o, ls);
  return ls * E + rdlane(jsel, ls);
}

// insertingWalk slot (mergeTree.ts:1723-1825 with breakTie 1705-1721): the
// first defined leaf (L >= 0) with P >= pos, or -1.
template <int E>
__device__ __forceinline__ int find_slot(const int32_t (&L)[E], const int32_t (&P)[E], int32_t pos) {
  int jsel = E;
#pragma unroll
  for (int j = E - 1; j >= 0; j--) jsel = (L[j] >= 0 && P[j] >= pos) ? j : jsel;
  const unsigned long long m = __ballot(jsel < E);
  if (!m) return -1;
  const int ls = __ffsll((long long)m) - 1;
  return ls * E + rdlane(jsel, ls);
}

}  // namespace mte
