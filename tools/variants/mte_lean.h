// mte_lean.h — the pass-1 per-op step of the E = 1 / 2 register tiers (documents
// of <= 126 segments: ~all ops of configs 2-4), written for instruction count.
//
// Same rules as doc_step / doc_step_v (mte_replay.h / mte_step1.h, which cite
// the reference for each), restated so that every per-slot condition lives in
// a lane mask (an SGPR pair from one v_cmp) instead of a bool array in VGPRs:
//   * decisions: the split / insert-slot candidates are lane masks; the slot
//     comes from s_ff1 of their union and the candidate mask it hit (scalar);
//   * single slots are written on their lane only (the new segment, the
//     pieces of a split leaf): one select per plane, not one per slot;
//   * the shift is specialised for one threshold (an insert without a split)
//     and two (a split), its selects read lane masks made once per op;
//   * a range op's "in range" flags stay lane masks: computed before the
//     shift on the leaves as they are, carried through it by mask shifts on
//     the scalar unit, and fixed at the split pieces -- instead of carrying the
//     L and P planes through the shift (two more planes of DPP moves and
//     selects).
// The scalar unit then decodes the op and moves masks; the VALU does the
// lengths, the scan, the plane moves and the marks.
#pragma once

#include "mte_kernels.h"

namespace mte {

// lane mask of slot j (slot = lane * E + j): bit l <-> slot l * E + j
typedef uint64_t lmask;

// lane l's bit of a uniform lane mask as the select condition: b where set,
// else a (one v_cndmask reading the mask's SGPR pair; written as asm because
// the compiler would otherwise extract the bit per lane with VALU shifts)
__device__ __forceinline__ uint32_t msel(lmask m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}
__device__ __forceinline__ int32_t msel(lmask m, int32_t a, int32_t b) {
  return (int32_t)msel(m, (uint32_t)a, (uint32_t)b);
}

// value of F at global slot x (x uniform, its lane l and sub-slot j given)
template <int E, typename T>
__device__ __forceinline__ T lean_at(const T (&F)[E], int l, int j) {
  if constexpr (E == 1) return rdlane(F[0], l);
  else return j ? rdlane(F[1], l) : rdlane(F[0], l);
}

// F at slot (l, j) := v (all uniform): one select on lane l of the register
// holding sub-slot j (the compare lane == l is shared by every plane written
// at that slot)
template <int E, typename T>
__device__ __forceinline__ void lean_put(T (&F)[E], int l, int j, T v) {
  const bool at = lane_id() == l;
  if constexpr (E == 1) {
    F[0] = at ? v : F[0];
  } else {
    if (j) F[1] = at ? v : F[1];
    else F[0] = at ? v : F[0];
  }
}

// slot-index masks of the shift: D[j] = lanes whose slot j is > t
template <int E>
__device__ __forceinline__ void lean_dmask(int t, lmask (&D)[E]) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) D[j] = __ballot(base + j > t);
}

// new[i] = old[i - d(i)], d = (i > t1) + (i > t2), one plane; TWO: t2 < inf.
// The conditions are the per-lane compares themselves (each one v_cmp into an
// SGPR pair that the selects read).
template <int E, bool TWO, typename T>
__device__ __forceinline__ void lean_shift_plane(T (&F)[E], const bool (&a)[E], const bool (&b)[E], int addr) {
  if constexpr (E == 1) {
    F[0] = (T)__builtin_amdgcn_ds_bpermute(addr, (int32_t)F[0]);
  } else {
    // E == 2: slot 2l+1 takes F0 (d = 1) or F1 of lane l-1 (d = 2); slot 2l
    // takes F1 (d = 1) or F0 (d = 2) of lane l-1
    const T p1 = (T)lane_prev((int32_t)F[1]);
    if constexpr (TWO) {
      const T p0 = (T)lane_prev((int32_t)F[0]);
      const T n1 = b[1] ? p1 : (a[1] ? F[0] : F[1]);
      const T n0 = b[0] ? p0 : (a[0] ? p1 : F[0]);
      F[1] = n1;
      F[0] = n0;
    } else {
      const T n1 = a[1] ? F[0] : F[1];
      const T n0 = a[0] ? p1 : F[0];
      F[1] = n1;
      F[0] = n0;
    }
  }
}

template <int E, int K, bool TWO>
__device__ __forceinline__ void lean_shift(Regs<E, K>& R, int t1, int t2) {
  const int base = lane_id() * E;
  bool a[E], b[E];
#pragma unroll
  for (int j = 0; j < E; j++) {
    a[j] = base + j > t1;
    b[j] = TWO && base + j > t2;
  }
  int addr = 0;
  if constexpr (E == 1) addr = (base - (a[0] ? 1 : 0) - (b[0] ? 1 : 0)) << 2;
  lean_shift_plane<E, TWO>(R.len, a, b, addr);
  lean_shift_plane<E, TWO>(R.seq, a, b, addr);
  lean_shift_plane<E, TWO>(R.rseq, a, b, addr);
  lean_shift_plane<E, TWO>(R.rmask, a, b, addr);
  lean_shift_plane<E, TWO>(R.meta, a, b, addr);
  lean_shift_plane<E, TWO>(R.toff, a, b, addr);
#pragma unroll
  for (int k = 0; k < K; k++) lean_shift_plane<E, TWO>(R.pr[k], a, b, addr);
}

// the same shift on lane masks (a range op's in-range flags), scalar unit
template <int E>
__device__ __forceinline__ void lean_shift_masks(lmask (&M)[E], int t1, int t2) {
  lmask D1[E], D2[E];
  lean_dmask<E>(t1, D1);
  lean_dmask<E>(t2, D2);
  if constexpr (E == 1) {
    const lmask m = M[0];
    M[0] = (~D1[0] & m) | (D1[0] & ~D2[0] & (m << 1)) | (D2[0] & (m << 2));
  } else {
    const lmask m0 = M[0], m1 = M[1];
    M[1] = (~D1[1] & m1) | (D1[1] & ~D2[1] & m0) | (D2[1] & (m1 << 1));
    M[0] = (~D1[0] & m0) | (D1[0] & ~D2[0] & (m1 << 1)) | (D2[0] & (m0 << 1));
  }
}

template <int E>
__device__ __forceinline__ void lean_mask_set(lmask (&M)[E], int x, bool on) {
  const int l = x / E, j = x % E;
  const lmask b = 1ull << l;
  if constexpr (E == 1) M[0] = on ? (M[0] | b) : (M[0] & ~b);
  else {
    if (j) M[1] = on ? (M[1] | b) : (M[1] & ~b);
    else M[0] = on ? (M[0] | b) : (M[0] & ~b);
  }
}

// the first slot (lowest index) set in the lane masks, or -1; its lane / sub-slot
template <int E>
__device__ __forceinline__ int lean_first(const lmask (&M)[E], int& l, int& j) {
  lmask any = M[0];
  if constexpr (E == 2) any |= M[1];
  if (!any) return -1;
  l = __ffsll((long long)any) - 1;
  j = (E == 2 && !((M[0] >> l) & 1)) ? 1 : 0;
  return l * E + j;
}

// ensureIntervalBoundary candidates at b (mergeTree.ts:1698-1702, 1681-1696):
// the visible leaf with P < b < P + L, as lane masks
template <int E>
__device__ __forceinline__ void lean_split_masks(const int32_t (&L)[E], const int32_t (&P)[E], int32_t b,
                                                 lmask (&M)[E]) {
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint32_t lim = (uint32_t)(L[j] > 1 ? L[j] - 1 : 0);
    M[j] = __ballot(((uint32_t)b - 1u - (uint32_t)P[j]) < lim);
  }
}

// the new segment (mergeTree.ts:1599-1611, textSegment.ts:40-48,
// mergeTreeNodes.ts:602-609) at slot (l, j)
template <int E, int K, bool S>
__device__ __forceinline__ void lean_new(Regs<E, K>& R, int l, int j, const s8v& op, uint32_t c, uint32_t flags,
                                         const ReplayArgs& a, uint32_t (&st)[kNumStats]) {
  const int32_t s = op[0], pos2 = op[5];
  const bool marker = (flags & MTE_F_MARKER) != 0;
  const int32_t nlen = marker ? 1 : pos2;
  const uint32_t meta = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
  const uint32_t toff = marker ? 0u : a.text_base + (uint32_t)op[6];
  const uint32_t psi = (uint32_t)op[7];
  uint32_t pv[K > 0 ? K : 1];
#pragma unroll
  for (int kk = 0; kk < (K > 0 ? K : 1); kk++) pv[kk] = 0u;
  if (K > 0 && psi != MTE_NO_PROPS) {
    // addProperties on a fresh segment: entries in order, a null deletes
    const s8v q2 = sload_props(a, psi);
    const uint32_t pk = (uint32_t)q2[0], k0 = pk & 0xffu, k1 = (pk >> 8) & 0xffu;
#pragma unroll
    for (int kk = 0; kk < K; kk++) {
      pv[kk] = (k0 == (uint32_t)kk) ? (uint32_t)q2[1] : pv[kk];
      pv[kk] = (k1 == (uint32_t)kk) ? (uint32_t)q2[2] : pv[kk];
    }
    if (pk >> 16) {
      const mte_propset ps = a.ps[psi];
      for (uint32_t t = 2; t < ps.count; t++) {
        const mte_prop p = a.pe[ps.first + t];
        const uint32_t key = uni(p.key), val = uni(p.value);
#pragma unroll
        for (int kk = 0; kk < K; kk++) pv[kk] = (key == (uint32_t)kk) ? val : pv[kk];
      }
    }
    MTE_STAT(st[kStPwrites] += (uint32_t)q2[3];)
  }
  MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
  lean_put<E>(R.len, l, j, nlen);
  lean_put<E>(R.seq, l, j, s);
  lean_put<E>(R.rseq, l, j, kNone);
  lean_put<E>(R.rmask, l, j, 0u);
  lean_put<E>(R.meta, l, j, meta);
  lean_put<E>(R.toff, l, j, toff);
#pragma unroll
  for (int kk = 0; kk < K; kk++) lean_put<E>(R.pr[kk], l, j, pv[kk]);
}

// a property write on the slots of the lane masks
template <int E, int K>
__device__ __forceinline__ void lean_set_key(Regs<E, K>& R, const lmask (&in)[E], uint32_t key, uint32_t val) {
#pragma unroll
  for (int kk = 0; kk < K; kk++) {
    if (key != (uint32_t)kk) continue;  // key is uniform: one plane's selects run
#pragma unroll
    for (int j = 0; j < E; j++) R.pr[kk][j] = msel(in[j], R.pr[kk][j], val);
  }
}

// One remote insert / remove / annotate on a register-resident document of
// n segments (n updated).  Returns 0 or MTE_E_INSERT_FAILED.
template <int E, int K, bool S>
__device__ __forceinline__ int lean_seg_op(Regs<E, K>& R, int& n, const s8v& op, uint32_t type, uint32_t c,
                                           uint32_t flags, int32_t m, bool newcalc, const ReplayArgs& a,
                                           uint32_t (&st)[kNumStats]) {
  const int32_t r = op[1], pos1 = op[4], pos2 = op[5];
  int32_t L[E], P[E];
  leaf_lengths<E, K>(R, r, c + 1, (int)c, m, newcalc, L);
  const int32_t total = prefix<E>(L, P);

  if (type == MTE_OP_INSERT) {
    // applyInsertOp -> insertSegments (client.ts:470-505, mergeTree.ts:1394-1422)
    const int32_t nlen = (flags & MTE_F_MARKER) ? 1 : pos2;
    lmask sm[E];
    lean_split_masks<E>(L, P, pos1, sm);
    int sl = 0, sj = 0;
    const int xs = lean_first<E>(sm, sl, sj);
    if (xs >= 0) {
      // ensureIntervalBoundary: [head][new][tail], the tail a copy of the leaf
      const int32_t o = pos1 - lean_at<E>(P, sl, sj);
      const int32_t lx = lean_at<E>(R.len, sl, sj);
      const uint32_t tx = lean_at<E>(R.toff, sl, sj);
      int tl;
      if (nlen > 0) {
        lean_shift<E, K, true>(R, xs, xs + 1);
        tl = xs + 2;
        lean_new<E, K, S>(R, (xs + 1) / E, (xs + 1) % E, op, c, flags, a, st);
        n += 2;
        MTE_STAT(st[kStWritten] += 3;)
      } else {
        lean_shift<E, K, false>(R, xs, INT32_MAX);
        tl = xs + 1;
        n += 1;
        MTE_STAT(st[kStWritten] += 2;)
      }
      lean_put<E>(R.len, sl, sj, o);
      lean_put<E>(R.len, tl / E, tl % E, lx - o);
      lean_put<E>(R.toff, tl / E, tl % E, tx + (uint32_t)o);
    } else if (nlen > 0) {
      // insertingWalk: before the first defined leaf with P >= pos
      lmask cm[E];
#pragma unroll
      for (int j = 0; j < E; j++) cm[j] = __ballot(L[j] >= 0 && P[j] >= pos1);
      int gl = 0, gj = 0;
      int g = lean_first<E>(cm, gl, gj);
      if (g < 0) {
        if (pos1 > total) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
        g = n;  // append: the slot is padding
        gl = g / E;
        gj = g % E;
      } else {
        lean_shift<E, K, false>(R, g - 1, INT32_MAX);
      }
      lean_new<E, K, S>(R, gl, gj, op, c, flags, a, st);
      n += 1;
      MTE_STAT(st[kStWritten] += 1;)
    }
    return 0;
  }

  // markRangeRemoved / annotateRange: ensureIntervalBoundary at both ends
  // (ordered by position), then mark start <= P < end
  const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
  // in range before the splits: visible, starting in [start, end) -- a leaf
  // straddling start is out (its tail goes in below), one straddling end in
  // (its tail goes out)
  lmask in[E];
#pragma unroll
  for (int j = 0; j < E; j++) in[j] = __ballot(L[j] > 0 && P[j] >= pos1 && P[j] < pos2);
  lmask s1[E], s2[E];
  lean_split_masks<E>(L, P, b1, s1);
  int l1 = 0, j1 = 0, l2 = 0, j2 = 0;
  int x1 = lean_first<E>(s1, l1, j1);
  int x2 = -1;
  if (b2 != b1) {
    lean_split_masks<E>(L, P, b2, s2);
    x2 = lean_first<E>(s2, l2, j2);
  }
  int32_t bA = b1;
  if (x1 < 0) {  // only the end splits: it acts as the first split
    x1 = x2;
    l1 = l2;
    j1 = j2;
    x2 = -1;
    bA = b2;
  }
  if (x1 >= 0) {
    const int32_t o1 = bA - lean_at<E>(P, l1, j1);
    const int32_t lx1 = lean_at<E>(R.len, l1, j1);
    const uint32_t tx1 = lean_at<E>(R.toff, l1, j1);
    if (x2 >= 0) {
      const bool same = x2 == x1;
      const int32_t o2 = b2 - lean_at<E>(P, l2, j2);  // offset in leaf x2
      const int32_t lx2 = same ? lx1 : lean_at<E>(R.len, l2, j2);
      const uint32_t tx2 = same ? tx1 : lean_at<E>(R.toff, l2, j2);
      lean_shift<E, K, true>(R, x1, x2 + 1);
      lean_shift_masks<E>(in, x1, x2 + 1);
      if (same) {
        // [head][mid][tail] of one leaf: head out, mid in, tail out
        lean_put<E>(R.len, l1, j1, o1);
        lean_put<E>(R.len, (x1 + 1) / E, (x1 + 1) % E, o2 - o1);
        lean_put<E>(R.toff, (x1 + 1) / E, (x1 + 1) % E, tx1 + (uint32_t)o1);
        lean_put<E>(R.len, (x1 + 2) / E, (x1 + 2) % E, lx1 - o2);
        lean_put<E>(R.toff, (x1 + 2) / E, (x1 + 2) % E, tx1 + (uint32_t)o2);
        lean_mask_set<E>(in, x1 + 1, true);
      } else {
        // leaf x1: head (x1) out, tail (x1 + 1) in; leaf x2 moved to x2 + 1:
        // head in, tail (x2 + 2) out
        lean_put<E>(R.len, l1, j1, o1);
        lean_put<E>(R.len, (x1 + 1) / E, (x1 + 1) % E, lx1 - o1);
        lean_put<E>(R.toff, (x1 + 1) / E, (x1 + 1) % E, tx1 + (uint32_t)o1);
        lean_put<E>(R.len, (x2 + 1) / E, (x2 + 1) % E, o2);
        lean_put<E>(R.len, (x2 + 2) / E, (x2 + 2) % E, lx2 - o2);
        lean_put<E>(R.toff, (x2 + 2) / E, (x2 + 2) % E, tx2 + (uint32_t)o2);
        lean_mask_set<E>(in, x1 + 1, true);
        lean_mask_set<E>(in, x2 + 2, false);
      }
      n += 2;
      MTE_STAT(st[kStWritten] += 4;)
    } else {
      lean_shift<E, K, false>(R, x1, INT32_MAX);
      lean_shift_masks<E>(in, x1, INT32_MAX);
      lean_put<E>(R.len, l1, j1, o1);
      lean_put<E>(R.len, (x1 + 1) / E, (x1 + 1) % E, lx1 - o1);
      lean_put<E>(R.toff, (x1 + 1) / E, (x1 + 1) % E, tx1 + (uint32_t)o1);
      // split at start: the tail is in; at end: the head stays in, the tail out
      lean_mask_set<E>(in, x1 + 1, bA == b1);
      n += 1;
      MTE_STAT(st[kStWritten] += 2;)
    }
  }
  if (pos2 <= pos1) return 0;  // nodeMap over an empty range: nothing visited
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < E; j++) cnt += (uint32_t)__popcll(in[j]);
  MTE_STAT(st[kStWritten] += cnt;)
  if (type == MTE_OP_REMOVE) {
    // markRemoved (mergeTree.ts:1924-1962): keep the earliest removedSeq, add
    // the client to removedClientIds
    const int32_t s = op[0];
    const uint32_t bit = 1u << c;
#pragma unroll
    for (int j = 0; j < E; j++) {
      const lmask fresh = in[j] & __ballot(R.rseq[j] == kNone);
      R.rseq[j] = msel(fresh, R.rseq[j], s);
      R.rmask[j] = msel(in[j], R.rmask[j], R.rmask[j] | bit);
    }
  } else if (cnt > 0 && K > 0) {
    // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
    const uint32_t psi = (uint32_t)op[6];
    const s8v q2 = sload_props(a, psi);
    if (flags & MTE_F_REWRITE) {
#pragma unroll
      for (int kk = 0; kk < K; kk++)
#pragma unroll
        for (int j = 0; j < E; j++) R.pr[kk][j] = msel(in[j], R.pr[kk][j], 0u);
    }
    const uint32_t pk = (uint32_t)q2[0], k0 = pk & 0xffu, k1 = (pk >> 8) & 0xffu;
    if (k0 != kNoKey) lean_set_key<E, K>(R, in, k0, (uint32_t)q2[1]);
    if (k1 != kNoKey) lean_set_key<E, K>(R, in, k1, (uint32_t)q2[2]);
    if (pk >> 16) {
      const mte_propset ps = a.ps[psi];
      for (uint32_t t = 2; t < ps.count; t++) {
        const mte_prop p = a.pe[ps.first + t];
        if (p.key < a.n_keys) lean_set_key<E, K>(R, in, uni(p.key), uni(p.value));
      }
    }
    MTE_STAT(st[kStPwrites] += cnt * (uint32_t)q2[3];)
  }
  return 0;
}

}  // namespace mte
