// mte_kernels.h — gfx950 device code of the batched sequence-merge engine.
//
// Execution model (DESIGN.md "Kernels"): one 64-lane wavefront replays one
// document.  The document's segments live in VGPRs for the whole batch,
// lane-major: segment i is slot (i % E) of lane (i / E), E in {1,2,4,8,16}
// chosen from the segment count (a doc that outgrows 64*E - 2 segments is
// written back to HBM and resumed with a larger E, possibly in a later pass).
// Per op:
//   * perspective length of every segment for (refSeq, clientId, minSeq)
//     (mergeTree.ts:1003-1054), lane-local sums + a DPP wavefront prefix scan
//     (replaces PartialSequenceLengths.getPartialLength, partialLengths.ts:667);
//   * split / insert-slot / range lookups by ballot over lanes;
//   * the split + insert is a "pull" shift of every field by 0/1/2 slots
//     (register moves inside a lane + DPP wave_shr across lanes);
//   * remove / annotate mark the segments of [start, end) in place;
//   * when minSeq advances, tombstones with removedSeq <= minSeq are dropped
//     by a stream compaction staged through LDS (zamboni, mergeTree.ts:800-838).
// Op records are fetched 64 at a time (one coalesced 2 KiB load per wave, lane l
// holds op l of the chunk) and broadcast per op with v_readlane.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mte.h"

namespace mte {

constexpr int kWave = 64;
constexpr int32_t kNone = INT32_MAX;  // "removedSeq undefined"
constexpr int kDocsPerBlock = 4;      // 4 independent waves (docs) per workgroup

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

// DPP controls (GFX9 encoding)
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143, kWaveShr1 = 0x138;

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int32_t dpp(int32_t v) {
  // disabled / out-of-range source lanes produce `old` = 0
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xf, false);
}

// inclusive prefix sum over the 64 lanes (Kogge-Stone in rows + row broadcasts)
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
  v += dpp<kRowShr1>(v);
  v += dpp<kRowShr2>(v);
  v += dpp<kRowShr4>(v);
  v += dpp<kRowShr8>(v);
  v += dpp<kRowBcast15, 0xa>(v);
  v += dpp<kRowBcast31, 0xc>(v);
  return v;
}

// value of lane l-1 (lane 0 gets 0)
__device__ __forceinline__ int32_t lane_prev(int32_t v) { return dpp<kWaveShr1>(v); }

__device__ __forceinline__ int32_t rdlane(int32_t v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
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
  for (int j = 0; j < E; j++) F[j] = (base + j == idx) ? v : F[j];
}

// new[i] = old[i - d(i)] with d(i) = (i > t1) + (i > t2), t1 <= t2 (t2 may be
// INT_MAX).  Slot t1+1 thus receives a copy of old[t1] (a split tail), slot
// t2+1 a copy of old[t2 - 1] or old[t1] when t2 == t1 + 1.
template <int E, typename T>
__device__ __forceinline__ void pull_shift(T (&F)[E], int t1, int t2) {
  const int base = lane_id() * E;
  const T p1 = (T)lane_prev((int32_t)F[E - 1]);  // old[base - 1]
  T p2;
  if constexpr (E >= 2) p2 = (T)lane_prev((int32_t)F[E - 2]);  // old[base - 2]
  else p2 = (T)lane_prev((int32_t)p1);
  T out[E];
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    const T m1 = (j >= 1) ? F[j - 1] : p1;
    const T m2 = (j >= 2) ? F[j - 2] : ((j == 1) ? p1 : p2);
    out[j] = (i > t2) ? m2 : ((i > t1) ? m1 : F[j]);
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

// write a new segment (wave-uniform values) into slot idx
template <int E, int K>
__device__ __forceinline__ void put_new(Regs<E, K>& R, int idx, int32_t len, int32_t seq, uint32_t meta,
                                        uint32_t toff, const uint32_t (&pr)[K > 0 ? K : 1]) {
  put<E>(R.len, idx, len);
  put<E>(R.seq, idx, seq);
  put<E>(R.rseq, idx, kNone);
  put<E>(R.rmask, idx, 0u);
  put<E>(R.meta, idx, meta);
  put<E>(R.toff, idx, toff);
#pragma unroll
  for (int k = 0; k < K; k++) put<E>(R.pr[k], idx, pr[k]);
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
      const int32_t seen = (removed && by_c) ? 0 : R.len[j];
      l = (removed && R.rseq[j] <= r) ? -1 : (mine_or_seen ? seen : (removed ? -1 : 0));
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
    const bool cnd = L[j] > 0 && P[j] < pos && pos - P[j] < L[j];
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

// ---- op chunk: 64 consecutive op records, lane l holds record l ----------
struct OpChunk {
  uint32_t w[8];    // the 32-byte record
  uint32_t pcnt;    // propset: entry count (0 if none)
  uint32_t pk0, pv0, pk1, pv1;  // first two entries
};

__device__ __forceinline__ void chunk_load_ops(OpChunk& c, const mte_op* ops, uint64_t base, uint64_t k1) {
  const uint32_t l = (uint32_t)lane_id();
  if (base + l < k1) {
    const uint4* __restrict__ p = reinterpret_cast<const uint4*>(ops + base) + 2u * l;
    const uint4 a = p[0], b = p[1];
    c.w[0] = a.x; c.w[1] = a.y; c.w[2] = a.z; c.w[3] = a.w;
    c.w[4] = b.x; c.w[5] = b.y; c.w[6] = b.z; c.w[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) c.w[i] = 0;
    c.w[3] = MTE_OP_NOOP;
  }
}

// gather each lane's propset header + first two entries (dependent on w)
__device__ __forceinline__ void chunk_load_props(OpChunk& c, const mte_propset* ps, const mte_prop* pe) {
  const uint32_t type = c.w[3] & 0xffu;
  uint32_t psi = MTE_NO_PROPS;
  if (type == MTE_OP_ANNOTATE) psi = c.w[6];
  else if (type == MTE_OP_INSERT) psi = c.w[7];
  c.pcnt = 0;
  c.pk0 = c.pv0 = c.pk1 = c.pv1 = 0;
  if (psi != MTE_NO_PROPS) {
    const mte_propset s = ps[psi];
    c.pcnt = s.count;
    if (s.count > 0) {
      const mte_prop e = pe[s.first];
      c.pk0 = e.key;
      c.pv0 = e.value;
    }
    if (s.count > 1) {
      const mte_prop e = pe[s.first + 1];
      c.pk1 = e.key;
      c.pv1 = e.value;
    }
  }
}

struct OpView {  // wave-uniform (SGPR) copy of one record
  int32_t seq, ref_seq, min_seq;
  uint32_t type, client, flags;
  int32_t pos1, pos2;
  uint32_t a, b;
  uint32_t pcnt, pk0, pv0, pk1, pv1;
};

__device__ __forceinline__ OpView chunk_op(const OpChunk& c, int j) {
  OpView v;
  v.seq = (int32_t)rdlane(c.w[0], j);
  v.ref_seq = (int32_t)rdlane(c.w[1], j);
  v.min_seq = (int32_t)rdlane(c.w[2], j);
  const uint32_t w3 = rdlane(c.w[3], j);
  v.type = w3 & 0xffu;
  v.client = (w3 >> 8) & 0xffu;
  v.flags = w3 >> 16;
  v.pos1 = (int32_t)rdlane(c.w[4], j);
  v.pos2 = (int32_t)rdlane(c.w[5], j);
  v.a = rdlane(c.w[6], j);
  v.b = rdlane(c.w[7], j);
  v.pcnt = rdlane(c.pcnt, j);
  v.pk0 = rdlane(c.pk0, j);
  v.pv0 = rdlane(c.pv0, j);
  v.pk1 = rdlane(c.pk1, j);
  v.pv1 = rdlane(c.pv1, j);
  return v;
}

}  // namespace mte
