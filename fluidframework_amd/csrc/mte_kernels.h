// mte_kernels.h — data layout and wavefront primitives of the gfx950 engine.
//
// Execution model: a document is replayed by one 64-lane
// wavefront with its segments held in VGPRs for the whole batch, lane-major:
// segment i is slot (i % E) of lane (i / E), E in {1,2,4,8,16} chosen from the
// segment count.  Small documents (<= 126 segments) are replayed two per
// wavefront (the wave alternates between them op by op, so 10k documents fit
// on the chip at once); larger ones one per wavefront.
//
// Slots >= n hold *padding*: len 0 and removedSeq INT32_MIN, which is
// "undefined" (UNDEF) for every perspective in both length modes, so no
// per-op validity test is needed and shifts carry padding along for free.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mte.h"

namespace mte {

constexpr int kWave = 64;
constexpr int32_t kNone = INT32_MAX;  // removedSeq undefined (not removed)
constexpr int32_t kPad = INT32_MIN;   // removedSeq of a padding slot
constexpr int kDocsPerBlock = 4;      // big-doc kernel: 4 waves (docs) per workgroup
constexpr int kPairsPerBlock = 4;     // pass-1 kernel: 4 waves per workgroup
constexpr int kGroupMax = 8;          // pass 1: at most this many documents per wave

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
// the document's batch holds MTE_OP_RELPOS records: passes 1 and 2 leave it to
// the HBM-streamed pass (set per batch by the engine, mte_engine.hip)
constexpr uint32_t kHdrRel = 0x08000000u;

// kStChunkCanon / kStChunkScan (chunk pass only): the canonical S_live of its
// ops, and the chunk slots + summary entries those ops actually scanned
enum StatIdx {
  kStOps = 0,
  kStScanned,
  kStWritten,
  kStPwrites,
  kStUnits,
  kStMaxSegs,
  kStChunkCanon,
  kStChunkScan,
  kNumStats
};

// segment state, structure of arrays, doc-major: field[doc * cap + i].  All
// planes live in one allocation at a common stride (plane_stride elements):
// len seq rseq rmask meta toff, then the property planes.
constexpr int kFieldPlanes = 6;
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

// ---- op records --------------------------------------------------------------
// The replay kernels read the submitted mte_op records (32 B = one s_load_dwordx8)
// in place: w0 seq | w1 ref_seq | w2 min_seq | w3 type | client << 8 | flags << 16
// | w4 pos1 | w5 pos2 | w6 a | w7 b (include/mte.h).  Property sets are compiled
// per run into 32-B records (props_kernel): w0 k0 | k1 << 8 | (count > 2) << 16
// (key 0xff = none) | w1 v0 | w2 v1 | w3 keys < n_keys in the set | w4-7 0.
constexpr uint32_t kNoKey = 0xffu;
constexpr uint32_t kRecPad = 512;  // zeroed records after the last op (L2 prefetch runs ahead)

struct ReplayArgs {
  DocHdr* hdr;
  uint32_t* planes;       // SegSoA base: plane p of slot x at planes[p * stride + x]
  uint64_t stride;
  uint32_t cap;
  uint32_t n_docs;
  const uint4* recs;       // the batch's mte_op records, 2 x uint4 each (+ kRecPad)
  const uint4* cps;        // compiled propsets, 2 x uint4 each
  const uint64_t* op_off;  // n_docs + 1
  const mte_propset* ps;
  const mte_prop* pe;
  uint32_t n_keys;
  uint32_t text_base;      // arena offset of the batch's text (mte_op.a of inserts)
  unsigned long long* stats;  // n_docs * kNumStats
  const uint32_t* pair_docs;  // pass 1: `group` document indices per wave (-1: none)
  uint32_t n_pairs;           // pass-1 waves
  uint32_t group;             // pass 1: documents per wave (1 .. kGroupMax)
  unsigned long long* wclock;  // diagnostics (MTE_WAVE_CLOCK): pass-1 start / end time per pair, or null
  unsigned long long* gdone;   // pass 1: ops applied so far by all waves (fair priority), zeroed per run
  unsigned long long n_ops;    // ops of the batch
  unsigned long long eta;      // expected pass-1 duration in s_memrealtime ticks (0 = unknown)
  // kPack4 with a side key: the key (< 4) whose value ids may exceed a byte
  // because only marker inserts ever set it (markerId); pass 1 holds a
  // marker's value of it in the marker's toff register (a marker has no text)
  // and the key's byte stays 0.  kNoKey: none.
  uint32_t side_key;
  // MTE_DOC_EVENTS documents: delta events of doc d go to dl[dl_off[d] ..
  // dl_off[d + 1]); dl_n[d] = how many the batch produced (more = overflow)
  mte_delta* dl;
  const uint64_t* dl_off;
  uint32_t* dl_n;
  // MTE_DOC_REFS documents: local reference slots of doc d at refs[d * ref_cap ..]
  // (x = the arena offset of the unit the reference sits on, y = kRefLive |
  // kRefDetached | refType; mte_stream.h)
  uint2* refs;
  uint32_t ref_cap;
  // the streamed pass's document order (stream_kernel: wave i replays document
  // sorder[i]), or null for index order
  const uint32_t* sorder;
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

// value of lane l-1 (lane 0 gets 0: bound_ctrl, so no zero-initialised
// destination is needed and the move is a single v_mov_b32_dpp)
__device__ __forceinline__ int32_t lane_prev(int32_t v) {
  return __builtin_amdgcn_mov_dpp(v, kWaveShr1, 0xf, 0xf, true);
}

__device__ __forceinline__ int32_t rdlane(int32_t v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// F[j] with a wave-uniform j.  Each element passes through an empty asm so
// the select chain stays on register values: a chain of selects on loads
// gets folded into one load through a selected pointer, which turns the
// register array into a scratch array.
template <int E, typename T>
__device__ __forceinline__ T pick(const T (&F)[E], int j) {
  T v = F[0];
#pragma unroll
  for (int jj = 1; jj < E; jj++) {
    T x = F[jj];
    asm("" : "+v"(x));
    v = (j == jj) ? x : v;
  }
  return v;
}

// broadcast field value of global segment index idx (wave-uniform)
template <int E, typename T>
__device__ __forceinline__ T bcast(const T (&F)[E], int idx) {
  if constexpr (E == 1) return rdlane(F[0], idx);
  else return rdlane(pick<E>(F, (int)((uint32_t)idx % (uint32_t)E)), (int)((uint32_t)idx / (uint32_t)E));
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
#pragma unroll
  for (int j = E - 1; j >= 0; j--) {  // in place, highest slot first
    const int i = base + j;
    const T m1 = (j >= 1) ? F[j - 1] : p1;
    const T m2 = (j >= 2) ? F[j - 2] : ((j == 1) ? p1 : p2);
    F[j] = (i > t2) ? m2 : ((i > t1) ? m1 : F[j]);
  }
}

// ---- register-resident document --------------------------------------------

// Property planes in registers.  K = kPack4: four keys whose value ids all fit
// in 8 bits held as the bytes of ONE register plane (pass 1 when the context's
// values allow it): shifts, inserts and compactions move one plane instead of
// four; HBM keeps the four planes (load_regs / store_regs pack and unpack).
constexpr int kPack4 = -4;
template <int K>
constexpr int kRegPlanes = K == kPack4 ? 1 : K;  // register planes
template <int K>
constexpr int kRP = kRegPlanes<K> > 0 ? kRegPlanes<K> : 1;  // array extent
template <int K>
constexpr int kKeys = K == kPack4 ? 4 : K;  // keys (HBM planes)

template <int E, int K>
struct Regs {
  int32_t len[E], seq[E], rseq[E];
  uint32_t rmask[E], meta[E], toff[E];
  uint32_t pr[kRP<K>][E];
};

// Perspective length of every slot (mergeTree.ts:1003-1026 new calc,
// 1028-1054 legacy calc); -1 = undefined.  Written as selects on compare
// results so no per-slot mask arithmetic lands on the scalar unit.
//   new:    rseq <= m ? UNDEF : (rseq <= r || c in rcli) ? 0 : seen ? len : 0
//   legacy: rseq <= r ? UNDEF : seen ? (c in rcli ? 0 : len) : removed ? UNDEF : 0
// with seen = seq <= r || cli == c.  Padding (rseq INT32_MIN) is UNDEF in both.
template <int E, int K>
__device__ __forceinline__ void leaf_lengths(const Regs<E, K>& R, int32_t r, uint32_t cm1, int c, int32_t m,
                                             bool newcalc, int32_t (&L)[E]) {
  if (newcalc) {
#pragma unroll
    for (int j = 0; j < E; j++) {
      const int32_t seqe = ((R.meta[j] & 0xffu) == cm1) ? INT32_MIN : R.seq[j];
      const int32_t vis = (seqe <= r) ? R.len[j] : 0;
      const int32_t rse = ((R.rmask[j] >> c) & 1u) ? INT32_MIN : R.rseq[j];
      const int32_t v2 = (rse <= r) ? 0 : vis;
      L[j] = (R.rseq[j] <= m) ? -1 : v2;
    }
  } else {
#pragma unroll
    for (int j = 0; j < E; j++) {
      const int32_t seqe = ((R.meta[j] & 0xffu) == cm1) ? INT32_MIN : R.seq[j];
      const int32_t lenc = ((R.rmask[j] >> c) & 1u) ? 0 : R.len[j];
      const int32_t unseen = (R.rseq[j] != kNone) ? -1 : 0;
      const int32_t sel = (seqe <= r) ? lenc : unseen;
      L[j] = (R.rseq[j] <= r) ? -1 : sel;
    }
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
// with L > 0 and P < pos < P + L, i.e. (pos - 1 - P) <u (L - 1).  Markers
// (L == 1) can never satisfy it.  Returns the global index or -1; *off = pos - P.
template <int E>
__device__ __forceinline__ int find_split(const int32_t (&L)[E], const int32_t (&P)[E], int32_t pos,
                                          int32_t* off) {
  int jsel = -1;
  int32_t o = 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint32_t lim = L[j] > 1 ? (uint32_t)(L[j] - 1) : 0u;
    const bool cnd = ((uint32_t)pos - 1u - (uint32_t)P[j]) < lim;
    jsel = cnd ? j : jsel;
    o = cnd ? pos - P[j] : o;
  }
  const unsigned long long msk = __ballot(jsel >= 0);
  if (!msk) return -1;
  const int ls = __ffsll((long long)msk) - 1;
  *off = rdlane(o, ls);
  if constexpr (E == 1) return ls;
  else return ls * E + rdlane(jsel, ls);
}

// insertingWalk slot (mergeTree.ts:1723-1825 with breakTie 1705-1721): the
// first defined leaf (L >= 0) with P >= pos, or -1.
template <int E>
__device__ __forceinline__ int find_slot(const int32_t (&L)[E], const int32_t (&P)[E], int32_t pos) {
  int jsel = E;
#pragma unroll
  for (int j = E - 1; j >= 0; j--) jsel = (L[j] >= 0 && P[j] >= pos) ? j : jsel;
  const unsigned long long msk = __ballot(jsel < E);
  if (!msk) return -1;
  const int ls = __ffsll((long long)msk) - 1;
  if constexpr (E == 1) return ls;
  else return ls * E + rdlane(jsel, ls);
}

}  // namespace mte
