// mte_step1.h — the per-op step of the one-slot-per-lane tier (E == 1,
// documents of <= 62 segments: most of the ops of a conflict-farm batch).
//
// Same semantics as doc_step (mte_replay.h, which cites the reference for
// every rule), but the split / insert decisions stay per lane instead of
// going through scalar lookups: a lane learns "my slot is after the split
// leaf" from the popcount of the candidate ballot below it (v_mbcnt), "I am
// the slot right after it" from its neighbour's flag (DPP), and every
// half of a split leaf is rebuilt from the values the lane pulled in the
// shift.  The scalar unit — one per CU, shared by four SIMDs — then only
// decodes the op, branches on the op type and on "is there a split", and
// keeps the collab window; the rest is VALU work on each SIMD.
#pragma once

#include "mte_kernels.h"

namespace mte {

// number of set bits of m in the lanes below this one
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <typename T>
__device__ __forceinline__ T perm1(T v, int addr) {
  return (T)__builtin_amdgcn_ds_bpermute(addr, (int32_t)v);
}

// new[l] = old[l - d(l)] for every plane; addr = (l - d(l)) * 4
template <int K>
__device__ __forceinline__ void shift1(Regs<1, K>& R, int addr) {
  R.len[0] = perm1(R.len[0], addr);
  R.seq[0] = perm1(R.seq[0], addr);
  R.rseq[0] = perm1(R.rseq[0], addr);
  R.rmask[0] = perm1(R.rmask[0], addr);
  R.meta[0] = perm1(R.meta[0], addr);
  R.toff[0] = perm1(R.toff[0], addr);
#pragma unroll
  for (int k = 0; k < K; k++) R.pr[k][0] = perm1(R.pr[k][0], addr);
}

// the inserted segment at the lanes with `at` (mergeTree.ts:1599-1611,
// textSegment.ts:40-48, mergeTreeNodes.ts:602-609)
template <int K, bool S>
__device__ __forceinline__ void put_new1(Regs<1, K>& R, bool at, const s8v& op, uint32_t c, uint32_t flags,
                                         const ReplayArgs& a, uint32_t (&st)[kNumStats]) {
  const int32_t s = op[0], pos2 = op[5];
  const bool marker = (flags & MTE_F_MARKER) != 0;
  const int32_t nlen = marker ? 1 : pos2;
  const uint32_t meta = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
  const uint32_t toff = marker ? 0u : a.text_base + (uint32_t)op[6];
  const uint32_t psi = (uint32_t)op[7];
  uint32_t pr[K > 0 ? K : 1][1];
  const bool one[1] = {true};
#pragma unroll
  for (int kk = 0; kk < (K > 0 ? K : 1); kk++) pr[kk][0] = 0;
  if (K > 0 && psi != MTE_NO_PROPS) {
    const s8v q2 = sload_props(a, psi);
    apply_props<1, K>(pr, one, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
    MTE_STAT(st[kStPwrites] += (uint32_t)q2[3];)
  }
  MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
  R.len[0] = at ? nlen : R.len[0];
  R.seq[0] = at ? s : R.seq[0];
  R.rseq[0] = at ? kNone : R.rseq[0];
  R.rmask[0] = at ? 0u : R.rmask[0];
  R.meta[0] = at ? meta : R.meta[0];
  R.toff[0] = at ? toff : R.toff[0];
#pragma unroll
  for (int kk = 0; kk < K; kk++) R.pr[kk][0] = at ? pr[kk][0] : R.pr[kk][0];
}

template <int K, bool S>
__device__ __forceinline__ int doc_step1(Regs<1, K>& R, DocRun& D, uint32_t (&st)[kNumStats], s8v& cur,
                                         const ReplayArgs& a, uint32_t* zlds) {
  const int l = lane_id();
  const int lim = kWave < (int)a.cap ? kWave : (int)a.cap;
  if (D.n + 2 > lim) return 1;
  if constexpr (S) {
    if (st[kStOps] >= (1u << 20)) return 1;
  }

  // ---- op record (prefetched into `cur`; see doc_step) ----------------------
  const s8v op = cur;
  const uint4* rec = D.recp + 2 * D.k;
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

  if (type <= MTE_OP_ANNOTATE) {
    const int32_t r = op[1], pos1 = op[4], pos2 = op[5];
    MTE_STAT(st[kStScanned] += (uint32_t)n;)
    int32_t L[1], P[1];
    leaf_lengths<1, K>(R, r, c + 1, (int)c, D.min_seq, (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0, L);
    const int32_t total = prefix<1>(L, P);
    // split candidate at b: the visible leaf with P < b < P + L
    const uint32_t slim = L[0] > 1 ? (uint32_t)(L[0] - 1) : 0u;

    if (type == MTE_OP_INSERT) {
      // applyInsertOp -> insertSegments (client.ts:470-505, mergeTree.ts:1394-1422)
      const bool marker = (flags & MTE_F_MARKER) != 0;
      const int32_t nlen = marker ? 1 : pos2;
      const int32_t q = pos1 - P[0];  // split offset, at the split leaf
      const bool sp = ((uint32_t)q - 1u) < slim;
      const uint64_t msp = __ballot(sp);
      bool at = false;
      if (msp) {
        // ensureIntervalBoundary: [head][new][tail], the tail a copy of the leaf
        const bool after = lanes_below(msp) != 0;        // slot > split leaf
        const bool nb = lane_prev(sp ? 1 : 0) != 0;       // slot == split leaf + 1
        const int d = after ? ((nlen > 0 && !nb) ? 2 : 1) : 0;
        const int addr = (l - d) << 2;
        shift1<K>(R, addr);
        const int32_t qp = perm1(q, addr);
        const bool tail = nlen > 0 ? (lane_prev(nb ? 1 : 0) != 0) : nb;
        R.len[0] = sp ? q : (tail ? R.len[0] - qp : R.len[0]);
        R.toff[0] = tail ? R.toff[0] + (uint32_t)qp : R.toff[0];
        at = nlen > 0 && nb;
        n += nlen > 0 ? 2 : 1;
        MTE_STAT(st[kStWritten] += nlen > 0 ? 3u : 2u;)
      } else if (nlen > 0) {
        // insertingWalk: before the first defined leaf with P >= pos
        const bool cand = L[0] >= 0 && P[0] >= pos1;
        const uint64_t mg = __ballot(cand);
        if (mg) {
          const bool pre = lanes_below(mg) != 0;
          at = cand && !pre;
          const int addr = (l - ((pre || cand) ? 1 : 0)) << 2;
          shift1<K>(R, addr);
        } else {
          if (pos1 > total) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
          at = l == n;                                   // append: the slot is padding
        }
        n += 1;
        MTE_STAT(st[kStWritten] += 1;)
      }
      if (nlen > 0) put_new1<K, S>(R, at, op, c, flags, a, st);
    } else {
      // markRangeRemoved / annotateRange: ensureIntervalBoundary at both ends
      // (ordered by position), then mark start <= P < end
      const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
      bool s1 = ((uint32_t)(b1 - P[0]) - 1u) < slim;
      bool s2 = b2 != b1 && ((uint32_t)(b2 - P[0]) - 1u) < slim;
      uint64_t m1 = __ballot(s1), m2 = __ballot(s2);
      int32_t bA = b1;
      if (!m1) {  // only the end splits: it acts as the first split
        s1 = s2;
        s2 = false;
        m1 = m2;
        m2 = 0;
        bA = b2;
      }
      if (m1) {
        const bool A = lanes_below(m1) != 0;              // slot > first split leaf
        const bool nbB = lane_prev(s2 ? 1 : 0) != 0;       // slot == second split leaf + 1
        const bool B = m2 != 0 && lanes_below(m2) != 0 && !nbB;
        const int d = (A ? 1 : 0) + (B ? 1 : 0);
        const int addr = (l - d) << 2;
        shift1<K>(R, addr);
        L[0] = perm1(L[0], addr);
        P[0] = perm1(P[0], addr);
        const int fs = perm1((s1 ? 1 : 0) | (s2 ? 2 : 0), addr);
        // which piece of its source leaf this slot now holds
        const bool h1 = (fs & 1) != 0, h2 = (fs & 2) != 0;
        const int32_t oA = bA - P[0], oB = b2 - P[0];
        const int kp = h1 ? d : d - 1;
        const int32_t cutA = h1 ? oA : oB;
        const int32_t st0 = (h1 || h2) ? (kp == 0 ? 0 : (kp == 1 ? cutA : oB)) : 0;
        const int32_t en = (h1 || h2) ? (kp == 0 ? cutA : ((kp == 1 && h1 && h2) ? oB : R.len[0])) : R.len[0];
        const int32_t nl = en - st0;
        L[0] = (h1 || h2) ? nl : L[0];
        P[0] += st0;
        R.len[0] = nl;
        R.toff[0] += (uint32_t)st0;
        n += m2 ? 2 : 1;
        MTE_STAT(st[kStWritten] += m2 ? 4u : 2u;)
      }
      if (pos2 != pos1) {
        // nodeMap (mergeTree.ts:2274-2330): no visible leaf straddles a boundary
        const bool in = L[0] > 0 && P[0] >= pos1 && P[0] < pos2;
        MTE_STAT(st[kStWritten] += (uint32_t)__popcll(__ballot(in));)
        if (type == MTE_OP_REMOVE) {
          // markRemoved (mergeTree.ts:1924-1962)
          R.rseq[0] = (in && R.rseq[0] == kNone) ? s : R.rseq[0];
          R.rmask[0] = in ? (R.rmask[0] | (1u << c)) : R.rmask[0];
        } else {
          // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
          const uint64_t min = __ballot(in);
          if (min) {
            const uint32_t psi = (uint32_t)op[6];
            const s8v q2 = sload_props(a, psi);
            const bool sel[1] = {in};
            if (flags & MTE_F_REWRITE) {
#pragma unroll
              for (int kk = 0; kk < K; kk++) R.pr[kk][0] = in ? 0u : R.pr[kk][0];
            }
            apply_props<1, K>(R.pr, sel, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
            MTE_STAT(st[kStPwrites] += (uint32_t)__popcll(min) * (uint32_t)q2[3];)
          }
        }
      }
    }
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
      // zamboni: each kept slot pushes its fields to its compacted lane
      // (ds_permute); the lanes past the new count become padding
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
        R.toff[0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.toff[0]);
#pragma unroll
        for (int kk = 0; kk < K; kk++) R.pr[kk][0] = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int32_t)R.pr[kk][0]);
        const bool pad = l >= n_new;
        R.rseq[0] = pad ? kPad : R.rseq[0];
        R.len[0] = pad ? 0 : R.len[0];
        D.n = n_new;
      }
    }
  }
  (void)zlds;
  return 0;
}

}  // namespace mte
