// mte_step1.h — the per-op step of the pass-1 register tiers (E <= 4 slots
// per lane, documents of <= 254 segments: nearly every op of a conflict-farm
// batch).
//
// Same semantics as doc_step (mte_replay.h, which cites the reference for
// every rule), but the split / insert decisions stay per slot instead of
// going through scalar lookups: a slot learns "I am after the split leaf"
// from the popcount of the candidate ballot in the lanes below (v_mbcnt) plus
// its own lane's earlier slots, "I am right after it" from its neighbour's
// flag, and every piece of a split leaf is rebuilt from the values the slot
// pulled in the shift.  The scalar unit — one per CU, shared by four SIMDs —
// then only decodes the op, branches on the op type and on "is there a
// split", and keeps the collab window; the rest is VALU work on each SIMD.
#pragma once

#include "mte_kernels.h"

namespace mte {

// number of set bits of m in the lanes below this one
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A[j] = some flagged slot lies before slot j (in this lane or a lower one)
template <int E>
__device__ __forceinline__ void after_flag(const bool (&F)[E], bool (&A)[E]) {
  bool any = false;
#pragma unroll
  for (int j = 0; j < E; j++) any = any || F[j];
  bool run = lanes_below(__ballot(any)) != 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    A[j] = run;
    run = run || F[j];
  }
}

// F1[j] / F2[j] = the flag of the slot 1 / 2 positions before slot j
template <int E>
__device__ __forceinline__ void prev_flags(const bool (&F)[E], bool (&F1)[E], bool (&F2)[E]) {
  const bool p1 = lane_prev(F[E - 1] ? 1 : 0) != 0;
  bool p2;
  if constexpr (E >= 2) p2 = lane_prev(F[E >= 2 ? E - 2 : 0] ? 1 : 0) != 0;
  else p2 = lane_prev(p1 ? 1 : 0) != 0;
#pragma unroll
  for (int j = 0; j < E; j++) {
    F1[j] = j >= 1 ? F[j >= 1 ? j - 1 : 0] : p1;
    F2[j] = j >= 2 ? F[j >= 2 ? j - 2 : 0] : (j == 1 ? p1 : p2);
  }
}

template <typename T>
__device__ __forceinline__ T perm1(T v, int addr) {
  return (T)__builtin_amdgcn_ds_bpermute(addr, (int32_t)v);
}

template <int E, typename T>
__device__ __forceinline__ void perm_plane(T (&F)[E], int addr) {
  F[0] = perm1(F[0], addr);
}

#ifndef MTE_SHIFT_SEQ_EMIN  // tiers with E >= this shift one plane at a time (register-light)
#define MTE_SHIFT_SEQ_EMIN 4
#endif

// one plane of shift_v: its two cross-lane moves, then its selects.  The E = 4
// tier shifts plane by plane: moving all 13 planes' neighbours first needs 52
// temporaries on top of 40 state registers, which spilled the whole pass-1
// kernel (its register budget is that of its largest tier)
template <int E, typename T>
__device__ __forceinline__ void shift_plane(T (&F)[E], const bool (&g1)[E], const bool (&g2)[E]) {
  const T p1 = (T)lane_prev((int32_t)F[E - 1]);
  const T p2 = (T)lane_prev((int32_t)F[E >= 2 ? E - 2 : 0]);
#pragma unroll
  for (int j = E - 1; j >= 0; j--) {
    const T m1 = (j >= 1) ? F[j >= 1 ? j - 1 : 0] : p1;
    const T m2 = (j >= 2) ? F[j >= 2 ? j - 2 : 0] : ((j == 1) ? p1 : p2);
    F[j] = g2[j] ? m2 : (g1[j] ? m1 : F[j]);
  }
}

template <typename T>
__device__ __forceinline__ void shift1_dpp(T (&F)[1], bool g1, bool g2) {
  const int32_t p1 = lane_prev((int32_t)F[0]);
  const int32_t p2 = lane_prev(p1);
  F[0] = g2 ? (T)p2 : (g1 ? (T)p1 : F[0]);
}

// new[i] = old[i - d(i)], d = g1 + g2 (g2 implies g1), for every plane and
// the NX extra per-slot values X.  E == 1: one ds_bpermute per plane.  E > 1:
// the two cross-lane moves of every plane first (DPP), then the selects.
template <int E, int K, int NX>
__device__ __forceinline__ void shift_v(Regs<E, K>& R, int32_t (&X)[NX > 0 ? NX : 1][E], const bool (&g1)[E],
                                        const bool (&g2)[E]) {
  if constexpr (E == 1 && MTE_E1_DPP) {
    // new = d == 2 ? old[l-2] : d == 1 ? old[l-1] : old, two wave_shr:1 moves per plane
    shift1_dpp(R.len, g1[0], g2[0]);
    shift1_dpp(R.seq, g1[0], g2[0]);
    shift1_dpp(R.rseq, g1[0], g2[0]);
    shift1_dpp(R.rmask, g1[0], g2[0]);
    shift1_dpp(R.meta, g1[0], g2[0]);
    if constexpr (!MTE_DIAG_NOPAYLOAD) shift1_dpp(R.toff, g1[0], g2[0]);
#pragma unroll
    for (int k = 0; k < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); k++) shift1_dpp(R.pr[k], g1[0], g2[0]);
#pragma unroll
    for (int x = 0; x < NX; x++) shift1_dpp(X[x], g1[0], g2[0]);
  } else if constexpr (E == 1) {
    const int addr = (lane_id() - (g1[0] ? 1 : 0) - (g2[0] ? 1 : 0)) << 2;
    perm_plane<E>(R.len, addr);
    perm_plane<E>(R.seq, addr);
    perm_plane<E>(R.rseq, addr);
    perm_plane<E>(R.rmask, addr);
    perm_plane<E>(R.meta, addr);
    if constexpr (!MTE_DIAG_NOPAYLOAD) perm_plane<E>(R.toff, addr);
#pragma unroll
    for (int k = 0; k < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); k++) perm_plane<E>(R.pr[k], addr);
#pragma unroll
    for (int x = 0; x < NX; x++) perm_plane<E>(X[x], addr);
  } else if constexpr (E >= MTE_SHIFT_SEQ_EMIN) {
    shift_plane<E>(R.len, g1, g2);
    shift_plane<E>(R.seq, g1, g2);
    shift_plane<E>(R.rseq, g1, g2);
    shift_plane<E>(R.rmask, g1, g2);
    shift_plane<E>(R.meta, g1, g2);
    if constexpr (!MTE_DIAG_NOPAYLOAD) shift_plane<E>(R.toff, g1, g2);
#pragma unroll
    for (int k = 0; k < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); k++) shift_plane<E>(R.pr[k], g1, g2);
#pragma unroll
    for (int x = 0; x < NX; x++) shift_plane<E>(X[x], g1, g2);
  } else {
    constexpr int NF = kFieldPlanes + kRegPlanes<K> + NX;
    uint32_t last[NF], last2[NF];
    shift_grab<E, NF>(last, last2, 0, R.len);
    shift_grab<E, NF>(last, last2, 1, R.seq);
    shift_grab<E, NF>(last, last2, 2, R.rseq);
    shift_grab<E, NF>(last, last2, 3, R.rmask);
    shift_grab<E, NF>(last, last2, 4, R.meta);
    shift_grab<E, NF>(last, last2, 5, R.toff);
#pragma unroll
    for (int k = 0; k < kRegPlanes<K>; k++) shift_grab<E, NF>(last, last2, kFieldPlanes + k, R.pr[k]);
#pragma unroll
    for (int x = 0; x < NX; x++) shift_grab<E, NF>(last, last2, kFieldPlanes + kRegPlanes<K> + x, X[x]);
    uint32_t p1[NF], p2[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) p1[f] = (uint32_t)lane_prev((int32_t)last[f]);
#pragma unroll
    for (int f = 0; f < NF; f++) p2[f] = (uint32_t)lane_prev((int32_t)last2[f]);
    shift_apply<E, NF>(R.len, p1, p2, 0, g1, g2);
    shift_apply<E, NF>(R.seq, p1, p2, 1, g1, g2);
    shift_apply<E, NF>(R.rseq, p1, p2, 2, g1, g2);
    shift_apply<E, NF>(R.rmask, p1, p2, 3, g1, g2);
    shift_apply<E, NF>(R.meta, p1, p2, 4, g1, g2);
    if constexpr (!MTE_DIAG_NOPAYLOAD) shift_apply<E, NF>(R.toff, p1, p2, 5, g1, g2);
#pragma unroll
    for (int k = 0; k < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); k++) shift_apply<E, NF>(R.pr[k], p1, p2, kFieldPlanes + k, g1, g2);
#pragma unroll
    for (int x = 0; x < NX; x++) shift_apply<E, NF>(X[x], p1, p2, kFieldPlanes + kRegPlanes<K> + x, g1, g2);
  }
}

// the inserted segment at the slots with `at` (mergeTree.ts:1599-1611,
// textSegment.ts:40-48, mergeTreeNodes.ts:602-609)
template <int E, int K, bool S>
__device__ __forceinline__ void put_new_v(Regs<E, K>& R, const bool (&at)[E], const s8v& op, uint32_t c,
                                          uint32_t flags, const ReplayArgs& a, uint32_t (&st)[kNumStats],
                                          const s8v* pq) {
  const int32_t s = op[0], pos2 = op[5];
  const bool marker = (flags & MTE_F_MARKER) != 0;
  const int32_t nlen = marker ? 1 : pos2;
  const uint32_t meta = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
  uint32_t toff = marker ? 0u : a.text_base + (uint32_t)op[6];
  const uint32_t psi = MTE_DIAG_NOPAYLOAD ? MTE_NO_PROPS : (uint32_t)op[7];
  uint32_t pr[kRP<K>][1];
  const bool one[1] = {true};
#pragma unroll
  for (int kk = 0; kk < kRP<K>; kk++) pr[kk][0] = 0;
  if (kKeys<K> > 0 && psi != MTE_NO_PROPS) {
    const s8v q2 = pq ? *pq : sload_props(a, psi);
    apply_props<1, K>(pr, one, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
    MTE_STAT(st[kStPwrites] += (uint32_t)q2[3];)
    if constexpr (K == kPack4) {
      // a marker's side-key value goes to its toff register (ReplayArgs::side_key)
      if (marker && a.side_key < 4u) {
        const uint32_t pk = (uint32_t)q2[0];
        if ((pk & 0xffu) == a.side_key) toff = (uint32_t)q2[1];
        if (((pk >> 8) & 0xffu) == a.side_key) toff = (uint32_t)q2[2];
        if (pk >> 16) {
          const mte_propset ps = a.ps[psi];
          for (uint32_t t = 2; t < ps.count; t++) {
            const mte_prop p = a.pe[ps.first + t];
            if (p.key == a.side_key) toff = uni(p.value);
          }
        }
      }
    }
  }
  MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
#pragma unroll
  for (int j = 0; j < E; j++) {
    R.len[j] = at[j] ? nlen : R.len[j];
    R.seq[j] = at[j] ? s : R.seq[j];
    R.rseq[j] = at[j] ? kNone : R.rseq[j];
    R.rmask[j] = at[j] ? 0u : R.rmask[j];
    R.meta[j] = at[j] ? meta : R.meta[j];
    R.toff[j] = at[j] ? toff : R.toff[j];
#pragma unroll
    for (int kk = 0; kk < kRegPlanes<K>; kk++) R.pr[kk][j] = at[j] ? pr[kk][0] : R.pr[kk][j];
  }
}

// chunk pass (mte_chunk.h): the insert slot lies in a later chunk
constexpr int kNextChunk = 2;

// The segment part of one insert / remove / annotate on a register-resident
// run of segments — a whole document (doc_step_v) or one chunk of a big one
// (mte_chunk.h, CH = true).  Returns 0, MTE_E_INSERT_FAILED or (CH, insert
// only, unless `last`) kNextChunk with the registers untouched.  With CH the
// op's positions are taken relative to `off`, the chunk's first position in
// the op's perspective; *tot is the chunk's length in that perspective before
// the op and *dlen its change (+ inserted units, - units the remover saw).
template <int E, int K, bool S, bool CH>
__device__ __forceinline__ int seg_op_v(Regs<E, K>& R, int& n, const s8v& op, uint32_t type, uint32_t c,
                                        uint32_t flags, int32_t m, bool newcalc, int32_t off, bool last,
                                        int32_t& tot, int32_t& dlen, const ReplayArgs& a,
                                        uint32_t (&st)[kNumStats], const s8v* pq = nullptr) {
  const int base = lane_id() * E;
  const int32_t s = op[0], r = op[1];
  const int32_t pos1 = op[4] - (CH ? off : 0);
  const int32_t pos2 = (CH && type != MTE_OP_INSERT) ? op[5] - off : op[5];
  int32_t L[E], P[E];
  leaf_lengths<E, K>(R, r, c + 1, (int)c, m, newcalc, L);
  const int32_t total = prefix<E>(L, P);
  if constexpr (CH) {
    tot = total;
    dlen = 0;
  }
  // split candidate at b: the visible leaf with P < b < P + L
  uint32_t slim[E];
#pragma unroll
  for (int j = 0; j < E; j++) slim[j] = L[j] > 1 ? (uint32_t)(L[j] - 1) : 0u;

  if (type == MTE_OP_INSERT) {
    // applyInsertOp -> insertSegments (client.ts:470-505, mergeTree.ts:1394-1422)
    const bool marker = (flags & MTE_F_MARKER) != 0;
    const int32_t nlen = marker ? 1 : pos2;
    int32_t X[1][E];  // split offset, meaningful at the split leaf
    bool sp[E], any = false;
#pragma unroll
    for (int j = 0; j < E; j++) {
      X[0][j] = pos1 - P[j];
      sp[j] = ((uint32_t)X[0][j] - 1u) < slim[j];
      any = any || sp[j];
    }
    bool at[E];
#pragma unroll
    for (int j = 0; j < E; j++) at[j] = false;
    if (__ballot(any)) {
      // ensureIntervalBoundary: [head][new][tail], the tail a copy of the leaf
      bool A[E], nb[E], nb2[E], g2[E];
      after_flag<E>(sp, A);
      prev_flags<E>(sp, nb, nb2);
#pragma unroll
      for (int j = 0; j < E; j++) g2[j] = nlen > 0 && A[j] && !nb[j];
      bool own[E];
#pragma unroll
      for (int j = 0; j < E; j++) own[j] = sp[j];
      shift_v<E, K, 1>(R, X, A, g2);
#pragma unroll
      for (int j = 0; j < E; j++) {
        const bool tail = nlen > 0 ? nb2[j] : nb[j];
        R.len[j] = own[j] ? X[0][j] : (tail ? R.len[j] - X[0][j] : R.len[j]);
        R.toff[j] = tail ? R.toff[j] + (uint32_t)X[0][j] : R.toff[j];
        at[j] = nlen > 0 && nb[j];
      }
      n += nlen > 0 ? 2 : 1;
      MTE_STAT(st[kStWritten] += nlen > 0 ? 3u : 2u;)
    } else if (nlen > 0) {
      // insertingWalk: before the first defined leaf with P >= pos
      bool cand[E], anyc = false;
#pragma unroll
      for (int j = 0; j < E; j++) {
        cand[j] = L[j] >= 0 && P[j] >= pos1;
        anyc = anyc || cand[j];
      }
      if (__ballot(anyc)) {
        bool A[E], g1[E], g2[E];
        after_flag<E>(cand, A);
#pragma unroll
        for (int j = 0; j < E; j++) {
          at[j] = cand[j] && !A[j];
          g1[j] = A[j] || cand[j];
          g2[j] = false;
        }
        int32_t none[1][E];
        shift_v<E, K, 0>(R, none, g1, g2);
      } else {
        if (CH && !last) return kNextChunk;  // the slot is in a later chunk
        if (pos1 > total) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
#pragma unroll
        for (int j = 0; j < E; j++) at[j] = base + j == n;  // append: the slot is padding
      }
      n += 1;
      MTE_STAT(st[kStWritten] += 1;)
    }
    if (nlen > 0) put_new_v<E, K, S>(R, at, op, c, flags, a, st, pq);
    if constexpr (CH) dlen = nlen > 0 ? nlen : 0;
  } else {
    // markRangeRemoved / annotateRange: ensureIntervalBoundary at both ends
    // (ordered by position), then mark start <= P < end
    const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
    bool s1[E], s2[E], any1 = false, any2 = false;
#pragma unroll
    for (int j = 0; j < E; j++) {
      s1[j] = ((uint32_t)(b1 - P[j]) - 1u) < slim[j];
      s2[j] = b2 != b1 && ((uint32_t)(b2 - P[j]) - 1u) < slim[j];
      any1 = any1 || s1[j];
      any2 = any2 || s2[j];
    }
    uint64_t m1 = __ballot(any1), m2 = __ballot(any2);
    int32_t bA = b1;
    if (!m1) {  // only the end splits: it acts as the first split
#pragma unroll
      for (int j = 0; j < E; j++) {
        s1[j] = s2[j];
        s2[j] = false;
      }
      m1 = m2;
      m2 = 0;
      bA = b2;
    }
    if (m1) {
      bool A[E], AB[E], nbB[E], nbB2[E], B[E];
      after_flag<E>(s1, A);
      after_flag<E>(s2, AB);
      prev_flags<E>(s2, nbB, nbB2);
      int32_t X[3][E];  // L, P and the split flags travel with the slot
#pragma unroll
      for (int j = 0; j < E; j++) {
        B[j] = m2 != 0 && AB[j] && !nbB[j];
        X[0][j] = L[j];
        X[1][j] = P[j];
        X[2][j] = (s1[j] ? 1 : 0) | (s2[j] ? 2 : 0);
      }
      shift_v<E, K, 3>(R, X, A, B);
#pragma unroll
      for (int j = 0; j < E; j++) {
        // which piece of its source leaf slot j now holds
        const int d = (A[j] ? 1 : 0) + (B[j] ? 1 : 0);
        const bool h1 = (X[2][j] & 1) != 0, h2 = (X[2][j] & 2) != 0;
        const int32_t oA = bA - X[1][j], oB = b2 - X[1][j];
        const int kp = h1 ? d : d - 1;
        const int32_t cutA = h1 ? oA : oB;
        const int32_t st0 = (h1 || h2) ? (kp == 0 ? 0 : (kp == 1 ? cutA : oB)) : 0;
        const int32_t en = (h1 || h2) ? (kp == 0 ? cutA : ((kp == 1 && h1 && h2) ? oB : R.len[j])) : R.len[j];
        const int32_t nl = en - st0;
        L[j] = (h1 || h2) ? nl : X[0][j];
        P[j] = X[1][j] + st0;
        R.len[j] = nl;
        R.toff[j] += (uint32_t)st0;
      }
      n += m2 ? 2 : 1;
      MTE_STAT(st[kStWritten] += m2 ? 4u : 2u;)
    }
    if (pos2 != pos1) {
      // nodeMap (mergeTree.ts:2274-2330): no visible leaf straddles a boundary
      bool in[E];
      uint32_t cnt = 0;
#pragma unroll
      for (int j = 0; j < E; j++) {
        in[j] = L[j] > 0 && P[j] >= pos1 && P[j] < pos2;
        cnt += (uint32_t)__popcll(__ballot(in[j]));
      }
      MTE_STAT(st[kStWritten] += cnt;)
      if (type == MTE_OP_REMOVE) {
        // markRemoved (mergeTree.ts:1924-1962)
        const uint32_t bit = 1u << c;
#pragma unroll
        for (int j = 0; j < E; j++) {
          R.rseq[j] = (in[j] && R.rseq[j] == kNone) ? s : R.rseq[j];
          R.rmask[j] = in[j] ? (R.rmask[j] | bit) : R.rmask[j];
        }
        if constexpr (CH) {  // the remover's own view loses the marked units
          int32_t rl = 0;
#pragma unroll
          for (int j = 0; j < E; j++) rl += in[j] ? L[j] : 0;
          dlen = -rdlane(wave_incl_scan(rl), kWave - 1);
        }
      } else if (cnt > 0 && !MTE_DIAG_NOPAYLOAD) {
        // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
        const uint32_t psi = (uint32_t)op[6];
        const s8v q2 = pq ? *pq : sload_props(a, psi);
        if (flags & MTE_F_REWRITE) {
#pragma unroll
          for (int kk = 0; kk < kRegPlanes<K>; kk++)
#pragma unroll
            for (int j = 0; j < E; j++) R.pr[kk][j] = in[j] ? 0u : R.pr[kk][j];
        }
        apply_props<E, K>(R.pr, in, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
        MTE_STAT(st[kStPwrites] += cnt * (uint32_t)q2[3];)
      }
    }
  }
  return 0;
}

template <int E, int K, bool S>
__device__ __forceinline__ int doc_step_v(Regs<E, K>& R, DocRun& D, uint32_t (&st)[kNumStats], RecV& cur,
                                          const ReplayArgs& a, uint32_t* zlds, int emin) {
  const int l = lane_id();
  const int base = l * E;
  const int lim = kWave * E < (int)a.cap ? kWave * E : (int)a.cap;
  if (D.n + 2 > lim) return 1;
  if constexpr (S) {
    if (st[kStOps] >= (1u << 20)) return 1;
  }

  // ---- op record (prefetched into `cur`; see doc_step) ----------------------
  const uint4* rec = D.recp + 2 * D.k;
#if MTE_VREC
  s8v op;
#pragma unroll
  for (int i = 0; i < 8; i++) op[i] = (int32_t)rdlane(cur, i);
  cur = vload_rec8(rec + 2);  // the next record (zeroed pad after the last)
#else
  const s8v op = cur;
  uint64_t next = reinterpret_cast<uint64_t>(rec + 2);
  asm volatile("" : "+s"(next) : "s"(op));
  cur = sload8(reinterpret_cast<const uint4*>(next));
#endif
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  MTE_STAT(st[kStOps]++;)
  MTE_STAT(st[kStMaxSegs] = (uint32_t)D.n > st[kStMaxSegs] ? (uint32_t)D.n : st[kStMaxSegs];)
  const int32_t s = op[0];
  const int32_t msn = op[2];
  int n = D.n;

  if (type <= MTE_OP_ANNOTATE) {
    MTE_STAT(st[kStScanned] += (uint32_t)n;)
    int32_t tot, dlen;
#if MTE_EARLY_PROPS
    // the op's compiled propset, loaded before the lengths and the scan so its
    // latency hides behind them (annotates, and inserts that carry props)
    s8v q2e;
    const s8v* pq = nullptr;
    if constexpr (kKeys<K> > 0) {
      const uint32_t psi = type == MTE_OP_ANNOTATE ? (uint32_t)op[6] : (uint32_t)op[7];
      const bool want = type == MTE_OP_ANNOTATE || (type == MTE_OP_INSERT && psi != MTE_NO_PROPS);
      q2e = sload_props(a, want ? psi : 0u);
      pq = &q2e;
    }
#else
    const s8v* pq = nullptr;
#endif
    const int rc = seg_op_v<E, K, S, false>(R, n, op, type, c, flags, D.min_seq, (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0,
                                            0, true, tot, dlen, a, st, pq);
    if (rc) return rc;
  } else if (type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  D.n = n;
  D.k++;

  // collab window (see doc_step)
  const bool live = type != MTE_OP_NOOP, end = (flags & MTE_F_MSG_END) != 0;
  const bool bad = (live & (s <= D.cur_seq)) | (end & (s < D.cur_seq)) | ((live | end) & (msn < D.min_seq)) |
                   (end & (msn > s));
  if (bad) return window_error(D, live, end, s, msn);
  if (end) {
    D.cur_seq = s;
    if (msn > D.min_seq) {
      D.min_seq = msn;
      // zamboni: drop tombstones with removedSeq <= minSeq (padding included)
      if constexpr (E == 1) {
        // each kept slot pushes its fields to its compacted lane (ds_permute)
        const bool keep = R.rseq[0] > msn;
        const uint64_t mk = __ballot(keep);
        const int n_new = __popcll(mk);
        if (n_new != n) {
          const int addr = (keep ? (int)lanes_below(mk) : kWave - 1) << 2;
          R.len[0] = __builtin_amdgcn_ds_permute(addr, R.len[0]);
          R.seq[0] = __builtin_amdgcn_ds_permute(addr, R.seq[0]);
          R.rseq[0] = __builtin_amdgcn_ds_permute(addr, R.rseq[0]);
          R.rmask[0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.rmask[0]);
          R.meta[0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.meta[0]);
          if constexpr (!MTE_DIAG_NOPAYLOAD) R.toff[0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.toff[0]);
#pragma unroll
          for (int kk = 0; kk < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); kk++)
            R.pr[kk][0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.pr[kk][0]);
          const bool pad = l >= n_new;
          R.rseq[0] = pad ? kPad : R.rseq[0];
          R.len[0] = pad ? 0 : R.len[0];
          D.n = n_new;
        }
      } else {
        // stream compaction staged through LDS
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
          if constexpr (!MTE_DIAG_NOPAYLOAD) compact_plane<E>(R.toff, keep, dst, zlds);
#pragma unroll
          for (int kk = 0; kk < (MTE_DIAG_NOPAYLOAD ? 0 : kRegPlanes<K>); kk++) compact_plane<E>(R.pr[kk], keep, dst, zlds);
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
  }
  return 0;
}

}  // namespace mte
