// mte_stream.h — pass 3: documents pass 2 escalated (> 1,022 segments) and
// new length-calc documents of remote clients with delta events, replayed
// one wavefront per document with the segment planes left in HBM and streamed
// per op in tiles of 128 slots (2 per lane, lane-major, coalesced; 2 per lane
// keeps the registers low enough for 5-8 waves per SIMD, which hide the
// per-op chain of L2 round trips better than wider tiles).
//
// Per op, the same algorithm as doc_step (mte_replay.h), restated over tiles:
//   A  scan tiles front to back: perspective lengths, running prefix, the
//      split / insert-slot lookups (stops once every target is found and the
//      prefix has passed the op's positions);
//   B  the split + insert shift as a back-to-front tiled move of every plane
//      (new[i] = old[i - d(i)], d(i) = (i > t1) + (i > t2)), then the split
//      patches and the new segment (single-lane stores);
//   C  for remove / annotate, a second front-to-back scan on the new layout
//      that marks the leaves with start <= P < end;
// and, when minSeq advances, a tiled stream compaction (zamboni).
// Loads bypass L1 (agent-scope relaxed atomics = sc1) and every phase ends
// with s_waitcnt vmcnt(0), so each phase reads what the previous one wrote.
// This path is bandwidth- and latency-bound by design (O(n) bytes per op); it
// exists so that no document size is refused below the ctx capacity.
#pragma once

#include "mte_replay.h"
#include "mte_tree.h"

namespace mte {

constexpr int kTileE = 2;
constexpr int kTile = kWave * kTileE;  // slots per tile

__device__ __forceinline__ uint32_t ld_l2(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// plane p, slot i of a doc's planes as a 32-bit offset from the doc's base
// (global_load saddr + voffset: no 64-bit address per lane and plane)
__device__ __forceinline__ uint32_t ld_l2o(const uint32_t* pl, uint32_t off) {
  return __hip_atomic_load(pl + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Every slot index this path computes is checked against the doc's capacity
// before it touches memory; a violation (an engine bug) stops the document
// with MTE_E_STATE instead of faulting the device.
#define MTE_SLOT_OK(i, cap) ((unsigned)(i) < (unsigned)(cap))

// hot planes (len seq rseq rmask meta toff) of tile [tb, tb + kTile); slots >= n are padding
template <int K>
__device__ __forceinline__ void tile_load_hot(Regs<kTileE, K>& R, const uint32_t* pl, uint64_t st, int tb, int n) {
  const int base = tb + lane_id() * kTileE;
#pragma unroll
  for (int j = 0; j < kTileE; j++) {
    const int i = base + j;
    const bool v = i < n;
    // unconditional loads (slot 0 stands in for padding), selected after:
    // no branch around each load
    const uint32_t x = (uint32_t)(v ? i : 0);
    const uint32_t l0 = ld_l2(pl + x), l1 = ld_l2(pl + st + x), l2 = ld_l2(pl + 2 * st + x);
    const uint32_t l3 = ld_l2(pl + 3 * st + x), l4 = ld_l2(pl + 4 * st + x), l5 = ld_l2(pl + 5 * st + x);
    R.len[j] = v ? (int32_t)l0 : 0;
    R.seq[j] = v ? (int32_t)l1 : 0;
    R.rseq[j] = v ? (int32_t)l2 : kPad;
    R.rmask[j] = v ? l3 : 0u;
    R.meta[j] = v ? l4 : 0u;
    R.toff[j] = v ? l5 : 0u;
  }
}

// ---- documents with a local client (MTE_DOC_LOCAL_CLIENT, include/mte.h) ----
// They replay on the HBM tree pass (mte_htree.h); the plane layout and the
// event / reference helpers below are shared with it.  Pending seqs are kLocalBase + localSeq (UnassignedSequenceNumber, normalised
// above every sequenced seq as breakTie / nodeLength do, mergeTree.ts:1009-1016,
// 1713-1714).  K more planes after the property planes hold, per slot and key,
// the localSeq of the last pending local annotate that set the key (0 = none):
// the pendingKeyUpdateCount of segmentPropertiesManager.ts:94-135 (acks come in
// order, so "count > 0" is "last pending localSeq not yet acked").  One more
// plane after them holds the mask of the pending annotate segment groups the
// slot belongs to (MTE_ANNOTATE_SLOTS, include/mte.h).
constexpr int32_t kLocalBase = MTE_LOCAL_SEQ_BASE;
template <int K>
constexpr int kAnnPlane = kFieldPlanes + 2 * K;
constexpr int kPlaneGroup = 5;  // planes moved per batch of loads (all in flight, then the stores)

// ---- delta events (MTE_DOC_EVENTS, include/mte.h) ----------------------------
// The doc's own view: removed -> 0, else the length (Client.getPosition,
// client.ts:345-350, through nodeLength for the local client).
struct EvOut {
  mte_delta* p;   // the doc's region
  uint64_t cap;   // its size
  uint32_t n;     // events so far (may pass cap: overflow)
  uint32_t op;    // the record being applied
};
__device__ __forceinline__ void ev_one(EvOut& ev, uint32_t kind, int32_t pos, int32_t len) {
  if (lane_id() == 0 && ev.n < ev.cap) ev.p[ev.n] = mte_delta{ev.op, kind, pos, len, 0u};
  ev.n++;
}
// the own view's length of slots [0, g)
__device__ __forceinline__ int32_t own_prefix(const uint32_t* pl, uint64_t sd, int g) {
  int32_t acc = 0;
  for (int tb = 0; tb < g; tb += kTile) {
#pragma unroll
    for (int j = 0; j < kTileE; j++) {
      const int i = tb + lane_id() * kTileE + j;
      const int ic = i < g ? i : 0;  // unconditional loads, selected after
      const int32_t rs = (int32_t)ld_l2(pl + 2 * sd + ic), ln = (int32_t)ld_l2(pl + ic);
      acc += (i < g && rs == kNone) ? ln : 0;
    }
  }
  return rdlane(wave_incl_scan(acc), kWave - 1);
}

// ---- local references (MTE_DOC_REFS, include/mte.h) -------------------------
// A reference is kept as the text unit it sits on -- its arena offset (a
// marker's is its reserved unit): splits never copy text, so the unit names the
// same place in whatever segment holds it, which is what LocalReferenceCollection
// keeps as (segment, offset) and moves on split (localReference.ts:391-416).
// kRefOff (with kRefDetached): a reference slideAckedRemovedSegmentReferences
// took off its segment's list for want of a segment to slide to
// (mergeTree.ts:935-942, removeLocalRef keeps the segment): detached for
// every read but mte_read_refs_transient, which still finds its segment.
constexpr uint32_t kRefLive = 0x80000000u, kRefDetached = 0x40000000u, kRefOff = 0x20000000u;
// a Transient reference (localReference.ts:263: never on its segment's list, so
// nothing moves or slides it): kRefLive | kRefDetached | kRefTrans | its offset
// in its segment, x = that segment's leaf id (mte_htree.h ht_ref_transient;
// titems.c REF_TRANS): read as its segment's position + the offset, the offset
// dropped once the segment is removed, -1 once the segment is gone
constexpr uint32_t kRefTrans = 0x10000000u, kRefTransOff = 0x0fffffffu;

// a segment references may slide to (_getSlideToSegment, mergeTree.ts:893-913):
// not a pending insert and not removed-and-acked (a pending removal is fine)
__device__ __forceinline__ bool slide_ok(int32_t sq, int32_t rs) { return sq < kLocalBase && rs >= kLocalBase; }

// the first slot a reference may slide to after x (dir > 0) or before it
// (dir < 0), or -1; x is wave-uniform.  grp != 0: the removals of one ack
// (removedSeq grp) are acked segment by segment in group order (gp: the
// group-order plane), so the ones after `cur` in it are still pending when x's
// references slide (ackPendingSegment, mergeTree.ts:1285-1304)
// tw (the tree words, or nullptr): a merged leaf's items are one segment, so
// the search starts past x's leaf (its kTCont continuations / its head)
// gm / gid: a group member's word in plane gm is gid (its localSeq)
__device__ __forceinline__ int find_slide_target(const uint32_t* pl, uint64_t sd, int n, int x, int dir,
                                                 int32_t grp = 0, const uint32_t* gp = nullptr, uint32_t cur = 0,
                                                 const uint32_t* tw = nullptr, const uint32_t* gm = nullptr,
                                                 uint32_t gid = 0) {
  const int l = lane_id();
  if (dir > 0) {
    int b0 = x + 1;
    if (tw)
      while (b0 < n && (uni(ld_l2(tw + b0)) & kTCont)) b0++;
    for (int b = b0; b < n; b += kWave) {
      const int i = b + l;
      const int ic = i < n ? i : 0;  // unconditional loads, selected after
      const int32_t sq = (int32_t)ld_l2(pl + sd + ic), rs = (int32_t)ld_l2(pl + 2 * sd + ic);
      const bool pend = grp != 0 && rs == grp && sq < kLocalBase && ld_l2(gp + ic) > cur && ld_l2(gm + ic) == gid;
      const uint64_t m = __ballot(i < n && (slide_ok(sq, rs) || pend));
      if (m) return b + __ffsll((long long)m) - 1;
    }
  } else {
    int e0 = x;
    if (tw)
      while (e0 > 0 && (uni(ld_l2(tw + e0)) & kTCont)) e0--;
    for (int e = e0; e > 0; e -= kWave) {  // slots [e - 64, e)
      const int i = e - kWave + l;
      const int ic = i >= 0 ? i : 0;
      const int32_t sq = (int32_t)ld_l2(pl + sd + ic), rs = (int32_t)ld_l2(pl + 2 * sd + ic);
      const bool pend = grp != 0 && rs == grp && sq < kLocalBase && ld_l2(gp + ic) > cur && ld_l2(gm + ic) == gid;
      const uint64_t m = __ballot(i >= 0 && (slide_ok(sq, rs) || pend));
      if (m) return e - kWave + (63 - __builtin_clzll(m));
    }
  }
  return -1;
}

// slideAckedRemovedSegmentReferences (mergeTree.ts:921-950) for every segment
// the op of seq s made removed-and-acked -- its removedSeq is now s: a remote
// remove's new removals and the pending ones it overtook (:1936-1938,
// 1986-1993), or the local removals an ack sequenced (:1302-1304).  Each such
// segment's SlideOnRemove references move to offset 0 of the first following
// segment they may slide to (addBeforeTombstones), else to the last offset of
// the last preceding one (addAfterTombstones), else come off the segment's list
// (kRefOff); Simple references detach, or come off the list when there is no
// segment to slide to (localReference.ts:422-485).  Slots [0, rhi) of the table rt.
// ev (MTE_DOC_EVENTS documents): one MTE_DELTA_SLIDE record per reference that
// slid or came off its segment -- the reference calls its beforeSlide /
// afterSlide callbacks there (mergeTree.ts:936-942, localReference.ts:436-447,
// 471-480), which an interval collection turns into "changeInterval" events
// mid-op (intervalCollection.ts:1042-1053): pos = the own-view position of the
// removed segment it sat on, len = the unit it left (mte_htree.h
// ht_slide_keys makes it the unit's order key), removed = its slot,
// kind = MTE_DELTA_SLIDE | 1 if
// it moved to a segment | 2 if to the end of a preceding one | its offset in
// the removed segment << 16 (clamped):
// the host orders one segment's references as its LocalReferenceCollection
// iterates them.
enum { kSlideAll = 0, kSlideAck = 1, kSlideOverlap = 2, kSlideNew = 3 };
// one removed segment x's references (grp / gp / cur: find_slide_target)
__device__ __forceinline__ void slide_segment(const uint32_t* pl, uint64_t sd, int n, uint2* rt, uint32_t rhi, int x,
                                              EvOut* ev, int32_t grp, const uint32_t* gp, uint32_t cur,
                                              const uint32_t* tw, const uint32_t* gm = nullptr, uint32_t gid = 0) {
  const int l = lane_id();
  const uint32_t toff = uni(ld_l2(pl + 5 * sd + x)), len = uni(ld_l2(pl + x));
  // an item continuing a merged leaf is one segment with the items before it:
  // offsets count from the leaf's first unit
  uint32_t lead = 0;
  if (tw)
    for (int y = x; y > 0 && (uni(ld_l2(tw + y)) & kTCont); y--) lead += uni(ld_l2(pl + y - 1));
  int t = find_slide_target(pl, sd, n, x, 1, grp, gp, cur, tw, gm, gid);
  bool after = false;
  if (t < 0) {
    t = find_slide_target(pl, sd, n, x, -1, grp, gp, cur, tw, gm, gid);
    after = t >= 0;
  }
  uint32_t to = 0;
  if (t >= 0) {
    const uint32_t tt = uni(ld_l2(pl + 5 * sd + t)), tl = uni(ld_l2(pl + t));
    to = after ? tt + tl - 1u : tt;
  }
  const int32_t xpos = ev ? own_prefix(pl, sd, x) : 0;
  for (uint32_t rb = 0; rb < rhi; rb += kWave) {
    const uint32_t r = rb + (uint32_t)l;
    const uint32_t rc = r < rhi ? r : 0u;  // unconditional loads, selected after
    const uint32_t anc = ld_l2(&rt[rc].x), st = ld_l2(&rt[rc].y);
    const bool hit = r < rhi && (st & kRefLive) && !(st & (kRefDetached | MTE_REF_STAY_ON_REMOVE)) && anc - toff < len;
    const bool moves = (st & MTE_REF_SLIDE_ON_REMOVE) && t >= 0;
    if (hit) {
      if (moves) rt[r].x = to;
      else rt[r].y = st | kRefDetached | (t < 0 ? kRefOff : 0u);
    }
    if (ev) {
      const uint64_t hm = __ballot(hit);
      if (hm) {
        const uint32_t idx = ev->n + __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
        const uint32_t off = lead + (anc - toff) < 0xffffu ? lead + (anc - toff) : 0xffffu;
        if (hit && idx < ev->cap)
          ev->p[idx] = mte_delta{ev->op, MTE_DELTA_SLIDE | (moves ? 1u : 0u) | (moves && after ? 2u : 0u) | (off << 16), xpos,
                                 (int32_t)anc, r};
        ev->n += (uint32_t)__popcll(hm);
      }
    }
  }
  vm_drain();
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
    v = w < v ? w : v;
  }
  return v;
}

// mode: kSlideAll every such segment; kSlideAck the removals of one localSeq's
// group (gm / gid: its members hold gid there) in group order (gp: the
// group-order plane), each slid while the later ones are still pending (a reference can slide again from a later one: one record per
// slide); kSlideOverlap / kSlideNew a remote remove's segments that the local
// client had removed already (lrp: the local-removal plane, non-zero) -- slid
// before the delta callback -- then the newly removed ones, after it
// (mergeTree.ts:1970-1993).  lrp: the local-removal plane (overlap modes) or
// the group-order plane (kSlideAck).
__device__ __forceinline__ void stream_slide(const uint32_t* pl, uint64_t sd, int n, uint2* rt, uint32_t rhi, int32_t s,
                                             EvOut* ev = nullptr, int mode = kSlideAll,
                                             const uint32_t* lrp = nullptr, const uint32_t* tw = nullptr,
                                             const uint32_t* gm = nullptr, uint32_t gid = 0) {
  const int l = lane_id();
  if (mode == kSlideAck) {
    const uint32_t* gp = lrp;
    uint32_t cur = 0;
    for (bool first = true;; first = false) {
      // the group's next segment: the lowest order above cur among removedSeq s
      uint32_t best = 0xffffffffu;
      int bx = -1;
      for (int tb = 0; tb < n; tb += kWave) {
        const int i = tb + l;
        const int ic = i < n ? i : 0;
        const int32_t rs = (int32_t)ld_l2(pl + 2 * sd + ic);
        const uint32_t g = ld_l2(gp + ic);
        const bool c = i < n && rs == s && ld_l2(gm + ic) == gid && (first || g > cur);
        const uint32_t mn = wave_min_u32(c ? g : 0xffffffffu);
        const uint64_t at = __ballot(c && g == mn);
        if (at && (bx < 0 || mn < best)) {
          best = mn;
          bx = tb + __ffsll((long long)at) - 1;
        }
      }
      if (bx < 0) return;
      cur = best;
      slide_segment(pl, sd, n, rt, rhi, bx, ev, s, gp, cur, tw, gm, gid);
    }
  }
  for (int tb = 0; tb < n; tb += kWave) {
    const int i = tb + l;
    const int ic = i < n ? i : 0;
    const int32_t rs = (int32_t)ld_l2(pl + 2 * sd + ic);
    const bool lr = mode >= kSlideOverlap && ld_l2(lrp + ic) != 0u;
    uint64_t m = __ballot(i < n && rs == s && (mode < kSlideOverlap || lr == (mode == kSlideOverlap)));
    while (m) {
      const int x = tb + __ffsll((long long)m) - 1;
      m &= m - 1;
      slide_segment(pl, sd, n, rt, rhi, x, ev, 0, nullptr, 0u, tw);
    }
  }
}

// the anchor a reference on slot x moves to when x is removed and acked
// (_getSlideToSegment, mergeTree.ts:893-913; Client.getSlideToSegment's offset,
// client.ts:1117-1130), or false when there is none; x is wave-uniform
__device__ __forceinline__ bool slide_anchor(const uint32_t* pl, uint64_t sd, int n, int x, uint32_t& to) {
  int t = find_slide_target(pl, sd, n, x, 1);
  bool after = false;
  if (t < 0) {
    t = find_slide_target(pl, sd, n, x, -1);
    after = true;
  }
  if (t < 0) return false;
  const uint32_t tt = uni(ld_l2(pl + 5 * sd + t)), tl = uni(ld_l2(pl + t));
  to = after ? tt + tl - 1u : tt;
  return true;
}

// MTE_OP_REF (include/mte.h):
//   b = 0: createLocalReferencePosition on the segment and offset
//     getContainingSegment(pos1) finds in the local view (client.ts:360-364,
//     1107-1110; mergeTree.ts:872-885, 2124-2143);
//   b = 1: removeLocalReferencePosition (mergeTree.ts:2113-2123);
//   b = 2: a reference a sequenced op creates (createPositionReference with an
//     op, intervalCollection.ts:639-658): getContainingSegment in the op's
//     perspective (ref_seq, client), then getSlideToSegment; no segment: detached;
//   b = 3: the reference becomes SlideOnRemove (a = its new type) and slides if
//     its segment is removed and acked (ackInterval, :1805-1902).
// rhi: slots in use so far.
template <int K>
__device__ __forceinline__ int stream_ref(const uint32_t* pl, uint64_t sd, int n, uint2* rt, uint32_t& rhi, const s8v& op,
                          int32_t m, bool newcalc) {
  const uint32_t slot = (uint32_t)op[5], b = (uint32_t)op[7], typ = (uint32_t)op[6];
  const int l = lane_id();
  if (b == 1u) {
    if (l == 0) rt[slot] = make_uint2(0u, 0u);
    vm_drain();
    return 0;
  }
  if (typ & MTE_REF_TRANSIENT) return MTE_E_UNSUPPORTED;
  if ((typ & MTE_REF_SLIDE_ON_REMOVE) && (typ & MTE_REF_STAY_ON_REMOVE)) return MTE_E_INVALID_ARG;
  if (b == 3u) {
    const uint32_t st0 = ld_l2(&rt[slot].y), anc = ld_l2(&rt[slot].x);
    if (!(st0 & kRefLive)) return MTE_E_INVALID_ARG;
    uint32_t st = (st0 & (kRefLive | kRefDetached | kRefOff)) | (typ & 0xffffu), to = anc;
    if (!(st & kRefDetached) && (st & MTE_REF_SLIDE_ON_REMOVE)) {
      // the slot holding the reference's unit
      for (int tb = 0; tb < n; tb += kWave) {
        const int i = tb + l;
        const int ic = i < n ? i : 0;  // unconditional loads, selected after
        const uint32_t tf = ld_l2(pl + 5 * sd + ic), ln = ld_l2(pl + ic);
        const uint64_t mk = __ballot(i < n && anc - tf < ln);
        if (mk) {
          const int x = tb + __ffsll((long long)mk) - 1;
          const int32_t rs = (int32_t)uni(ld_l2(pl + 2 * sd + x));
          if (rs != kNone && rs < kLocalBase && !slide_anchor(pl, sd, n, x, to)) st |= kRefDetached;
          break;
        }
      }
    }
    if (l == 0) rt[slot] = make_uint2(to, st);
    vm_drain();
    return 0;
  }
  const bool remote = b == 2u;
  const int32_t pos = op[4], r = op[1];
  const uint32_t c = ((uint32_t)op[3] >> 8) & 0xffu;
  int32_t carry = 0;
  for (int tb = 0; tb < n; tb += kTile) {
    Regs<kTileE, K> R;
    tile_load_hot<K>(R, pl, sd, tb, n);
    int32_t L[kTileE], P[kTileE];
    if (remote) {
      leaf_lengths<kTileE, K>(R, r, c + 1, (int)c, m, newcalc, L);
    } else {
#pragma unroll
      for (int j = 0; j < kTileE; j++) L[j] = R.rseq[j] == kNone ? R.len[j] : 0;  // the local view: removed -> 0
    }
#pragma unroll
    for (int j = 0; j < kTileE; j++) L[j] = L[j] > 0 ? L[j] : 0;  // padding / undefined: nothing
    const int32_t tot = prefix<kTileE>(L, P);
    bool hit = false;
    uint32_t anc = 0;
    int jx = 0;
#pragma unroll
    for (int j = 0; j < kTileE; j++) {
      const bool h = L[j] > 0 && pos >= carry + P[j] && pos < carry + P[j] + L[j];
      anc = h ? R.toff[j] + (uint32_t)(pos - carry - P[j]) : anc;
      jx = h ? j : jx;
      hit = hit || h;
    }
    const uint64_t mk = __ballot(hit);
    if (mk) {
      const int ls = __ffsll((long long)mk) - 1;
      uint32_t a0 = rdlane(anc, ls), st = kRefLive | (typ & 0xffffu);
      if (remote) {
        const int x = tb + ls * kTileE + rdlane(jx, ls);
        const int32_t rs = (int32_t)uni(ld_l2(pl + 2 * sd + x));
        if (rs != kNone && rs < kLocalBase && !slide_anchor(pl, sd, n, x, a0)) st |= kRefDetached;
      }
      if (l == 0) rt[slot] = make_uint2(a0, st);
      vm_drain();
      if (slot + 1 > rhi) rhi = slot + 1;
      return 0;
    }
    carry += tot;
  }
  if (!remote) return MTE_E_INVALID_ARG;  // no segment holds pos in the local view
  if (l == 0) rt[slot] = make_uint2(0u, kRefLive | kRefDetached | (typ & 0xffffu));  // detached
  vm_drain();
  if (slot + 1 > rhi) rhi = slot + 1;
  return 0;
}

// MTE_OP_RELPOS (include/mte.h): the position of the first marker whose key
// plane `key` holds `vid`, in the view (r, c) -- getPosition (mergeTree.ts:
// 853-870) sums the lengths of everything before it; undefined leaves count 0
// -- or -1 when no held marker carries the id (posFromRelativePos,
// mergeTree.ts:1369-1392).  One front-to-back tile scan with early exit.
template <int K>
__device__ int32_t stream_marker_pos(const uint32_t* pl, uint64_t sd, int n, uint32_t key, uint32_t vid, int32_t r,
                                     uint32_t c, int32_t m, bool newcalc) {
  if (key >= (uint32_t)K || vid == 0u) return -1;
  constexpr int E = kTileE;
  const uint32_t* kp = pl + (uint64_t)(kFieldPlanes + key) * sd;
  int32_t carry = 0;
  for (int tb = 0; tb < n; tb += kTile) {
    Regs<E, K> R;
    tile_load_hot<K>(R, pl, sd, tb, n);
    int32_t L[E], P[E];
    leaf_lengths<E, K>(R, r, c + 1, (int)c, m, newcalc, L);
    const int32_t tot = prefix<E>(L, P);
    int jsel = E;
#pragma unroll
    for (int j = E - 1; j >= 0; j--) {
      const int i = tb + lane_id() * E + j;
      const uint32_t v = ld_l2(kp + (i < n ? i : 0));  // unconditional, selected after
      jsel = (i < n && (R.meta[j] >> 8) != 0u && v == vid) ? j : jsel;
    }
    const uint64_t msk = __ballot(jsel < E);
    if (msk) {
      const int ls = __ffsll((long long)msk) - 1;
      int32_t pv = P[0];
#pragma unroll
      for (int j = 1; j < E; j++) pv = jsel == j ? P[j] : pv;
      return carry + (int32_t)rdlane(pv, ls);
    }
    carry += tot;
  }
  return -1;
}

// One op of one HBM-resident document of remote clients (see the file
// comment).  Returns 0 or a negative MTE_E_*.  ev: its delta events
// (MTE_DOC_EVENTS docs).
template <int K, bool S>
__device__ int stream_step(DocRun& D, uint32_t (&st)[kNumStats], s8v& cur, const ReplayArgs& a, EvOut& ev) {
  constexpr int E = kTileE;
  const int l = lane_id();
  uint32_t* pl = a.planes + (uint64_t)D.doc * a.cap;
  const uint64_t sd = a.stride;
  const bool evd = (D.flags & MTE_DOC_EVENTS) != 0;
  ev.op = D.k;
  const int nplanes = kFieldPlanes + K;

  const s8v op = cur;
  const uint4* rec = D.recp + 2 * D.k;
  if (D.k + 1 < D.k1) cur = sload8(rec + 2);
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  if (type == MTE_OP_RELPOS) {
    // the next record's positions, in its view (the engine checked that an
    // insert, remove or annotate of this document follows)
    if (D.k + 1 >= D.k1) return MTE_E_INVALID_ARG;
    const uint32_t nw3 = (uint32_t)cur[3];
    const uint32_t nt = nw3 & 0xffu, nc = (nw3 >> 8) & 0xffu;
    if (nt > MTE_OP_ANNOTATE || nc >= MTE_MAX_CLIENTS || ((nw3 >> 16) & MTE_F_LOCAL)) return MTE_E_INVALID_ARG;
    const bool newcalc = (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
    const uint32_t key = (uint32_t)op[6];
    if (flags & MTE_RP_POS1) {
      int32_t p = stream_marker_pos<K>(pl, sd, D.n, key, (uint32_t)op[4], cur[1], nc, D.min_seq, newcalc);
      if (p >= 0) p = (flags & MTE_RP_BEFORE1) ? p - op[0] : p + 1 + op[0];
      else if (nt == MTE_OP_INSERT) return MTE_E_UNSUPPORTED;
      cur[4] = p;
    }
    if ((flags & MTE_RP_POS2) && nt != MTE_OP_INSERT) {
      int32_t p = stream_marker_pos<K>(pl, sd, D.n, key, (uint32_t)op[5], cur[1], nc, D.min_seq, newcalc);
      if (p >= 0) p = (flags & MTE_RP_BEFORE2) ? p - op[1] : p + 1 + op[1];
      cur[5] = p;
    }
    D.k++;
    return 0;
  }
  // local ops, acks, rollbacks, regenerations and references belong to a
  // local client's document (the HBM tree pass)
  if (type == MTE_OP_REF || (flags & MTE_F_LOCAL) || type >= MTE_OP_ACK) return MTE_E_UNSUPPORTED;
  MTE_STAT(st[kStOps]++;)
  MTE_STAT(st[kStMaxSegs] = (uint32_t)D.n > st[kStMaxSegs] ? (uint32_t)D.n : st[kStMaxSegs];)
  const int32_t s = op[0], r = op[1], msn = op[2];
  const int32_t pos1 = op[4], pos2 = op[5];
  const bool ins = type == MTE_OP_INSERT;
  const bool marker = ins && (flags & MTE_F_MARKER) != 0;
  const int32_t nlen = marker ? 1 : pos2;  // insert: length of the new segment
  const bool rng = type == MTE_OP_REMOVE || type == MTE_OP_ANNOTATE;
  const bool newcalc = (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  int n = D.n;

  if (ins || rng) {
    MTE_STAT(st[kStScanned] += (uint32_t)n;)
    // ---- A: scan -----------------------------------------------------------
    const int32_t b1 = ins ? pos1 : (pos1 < pos2 ? pos1 : pos2);
    const int32_t b2 = ins ? pos1 : (pos1 < pos2 ? pos2 : pos1);
    int xa = -1, xb = -1, gs = -1;  // split at b1, split at b2 (range only), first defined leaf with P >= pos
    int32_t oa = 0, ob = 0, lena = 0, lenb = 0;
    uint32_t toffa = 0, toffb = 0;
    int32_t carry = 0;
    bool complete = true;  // the scan reached the end of the document
    for (int tb = 0; tb < n; tb += kTile) {
      Regs<E, K> R;
      tile_load_hot<K>(R, pl, sd, tb, n);
      int32_t L[E], P[E];
      leaf_lengths<E, K>(R, r, c + 1, (int)c, D.min_seq, newcalc, L);
      const int32_t tot = prefix<E>(L, P);
#pragma unroll
      for (int j = 0; j < E; j++) P[j] += carry;
      if (xa < 0) {
        int32_t o = 0;
        const int x = find_split<E>(L, P, b1, &o);
        if (x >= 0) {
          xa = tb + x;
          oa = o;
          lena = bcast<E>(R.len, x);
          toffa = bcast<E>(R.toff, x);
        }
      }
      if (rng && b2 != b1 && xb < 0) {
        int32_t o = 0;
        const int x = find_split<E>(L, P, b2, &o);
        if (x >= 0) {
          xb = tb + x;
          ob = o;
          lenb = bcast<E>(R.len, x);
          toffb = bcast<E>(R.toff, x);
        }
      }
      if (ins && gs < 0) {
        const int x = find_slot<E>(L, P, pos1);
        if (x >= 0) gs = tb + x;
      }
      carry += tot;
      // every later leaf has P >= carry > both positions: nothing more to find
      if (carry > b2 && (!ins || gs >= 0 || xa >= 0) && tb + kTile < n) {
        complete = false;
        break;
      }
    }
    // ---- decisions (as doc_step) --------------------------------------------
    int t1 = INT32_MAX, t2 = INT32_MAX, g = -1;
    SplitPatch pa{-1, -1, 0, 0, 0u, 0}, pb{-1, -1, 0, 0, 0u, 0};
    if (ins) {
      if (xa >= 0) {
        pa = SplitPatch{xa, nlen > 0 ? xa + 2 : xa + 1, oa, lena, toffa, pos1};
        t1 = xa;
        if (nlen > 0) {
          t2 = xa + 1;
          g = xa + 1;
        }
        MTE_STAT(st[kStWritten] += nlen > 0 ? 3 : 2;)
        n += 1;
      } else if (nlen > 0) {
        g = gs;
        if (g < 0) {
          if (complete && pos1 > carry) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
          g = n;
        }
        t1 = g - 1;
        MTE_STAT(st[kStWritten] += 1;)
      }
      if (nlen > 0) n += 1;
    } else {
      int x1 = xa, x2 = xb;
      int32_t o1 = oa, o2 = ob, l1 = lena, l2 = lenb, bb1 = b1;
      uint32_t f1 = toffa, f2 = toffb;
      if (x1 < 0) {
        x1 = x2;
        o1 = o2;
        l1 = l2;
        f1 = f2;
        bb1 = b2;
        x2 = -1;
      }
      if (x1 >= 0) {
        pa = SplitPatch{x1, x1 + 1, o1, l1, f1, bb1};
        t1 = x1;
        n += 1;
        MTE_STAT(st[kStWritten] += 2;)
        if (x2 >= 0) {
          const bool same = x2 == x1;
          pb = SplitPatch{x2 + 1, x2 + 2, same ? o2 - o1 : o2, same ? l1 - o1 : l2, same ? f1 + (uint32_t)o1 : f2, b2};
          t2 = x2 + 1;
          n += 1;
          MTE_STAT(st[kStWritten] += 2;)
        }
      }
    }
    if (n + 2 > (int)a.cap) return MTE_E_CAPACITY;
    // ---- B: shift back to front, then patches and the new segment --------------
    if (t1 != INT32_MAX) {
      const int lo = t1 + 1;
      // back to front: a tile's sources lie in it or the tile below, which is
      // moved later, so a tile's planes move kPlaneGroup at a time: their loads
      // all in flight at once, then their stores
      for (int tb = ((n - 1) / kTile) * kTile; tb + kTile > lo; tb -= kTile) {
        const int base = tb + l * E;
#pragma nounroll
        for (int p0 = 0; p0 < nplanes; p0 += kPlaneGroup) {
          uint32_t v[kPlaneGroup][E];
#pragma unroll
          for (int g = 0; g < kPlaneGroup; g++) {
            // unconditional loads from a valid plane and slot, selected after
            const int pg = p0 + g < nplanes ? p0 + g : nplanes - 1;
            const uint32_t pb = (uint32_t)((uint64_t)pg * sd);
#pragma unroll
            for (int j = 0; j < E; j++) {
              const int i = base + j;
              const int src = i - ((i > t1 ? 1 : 0) + (i > t2 ? 1 : 0));
              // src is -1 only for the new segment's slot 0 (t1 == -1), which the
              // new-segment stores below overwrite: never read before the doc
              const bool ok = p0 + g < nplanes && i < n && i >= lo && MTE_SLOT_OK(src, a.cap);
              const uint32_t x = ld_l2o(pl, pb + (uint32_t)(ok ? src : 0));
              v[g][j] = ok ? x : 0u;
            }
          }
#pragma unroll
          for (int g = 0; g < kPlaneGroup; g++) {
            const uint32_t pb = (uint32_t)((uint64_t)(p0 + g) * sd);
#pragma unroll
            for (int j = 0; j < E; j++) {
              const int i = base + j;
              if (p0 + g < nplanes && i < n && i >= lo && MTE_SLOT_OK(i, a.cap)) pl[pb + (uint32_t)i] = v[g][j];
            }
          }
        }
      }
      vm_drain();
    }
    if ((pa.h >= 0 && !(MTE_SLOT_OK(pa.h, a.cap) && MTE_SLOT_OK(pa.tl, a.cap))) ||
        (pb.h >= 0 && !(MTE_SLOT_OK(pb.h, a.cap) && MTE_SLOT_OK(pb.tl, a.cap))) || (g >= 0 && !MTE_SLOT_OK(g, a.cap)))
      return MTE_E_STATE;
    if (l == 0) {
#pragma unroll
      for (int pi = 0; pi < 2; pi++) {
        const SplitPatch& p = pi == 0 ? pa : pb;
        if (p.h >= 0) {
          pl[p.h] = (uint32_t)p.o;
          pl[p.tl] = (uint32_t)(p.len - p.o);
          pl[5 * sd + p.tl] = p.toff + (uint32_t)p.o;
        }
      }
      if (g >= 0) {
        pl[g] = (uint32_t)nlen;
        pl[sd + g] = (uint32_t)s;
        pl[2 * sd + g] = (uint32_t)kNone;
        pl[3 * sd + g] = 0u;
        pl[4 * sd + g] = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
        pl[5 * sd + g] = marker ? 0u : a.text_base + (uint32_t)op[6];
      }
    }
    if (g >= 0) {
      uint32_t pr[K > 0 ? K : 1][1];
      const bool one[1] = {true};
#pragma unroll
      for (int kk = 0; kk < (K > 0 ? K : 1); kk++) pr[kk][0] = 0;
      const uint32_t psi = (uint32_t)op[7];
      if (K > 0 && psi != MTE_NO_PROPS) {
        const s8v q2 = sload_props(a, psi);
        apply_props<1, K>(pr, one, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
        MTE_STAT(st[kStPwrites] += (uint32_t)q2[3];)
      }
      if (l == 0) {
#pragma unroll
        for (int kk = 0; kk < K; kk++) pl[(kFieldPlanes + kk) * sd + g] = pr[kk][0];
      }
      MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
    }
    vm_drain();
    if (evd && ins) {  // insertSegments' delta callback (mergeTree.ts:1409-1416)
      if (g >= 0) ev_one(ev, MTE_OP_INSERT, own_prefix(pl, sd, g), nlen);
      else if (nlen <= 0) ev_one(ev, MTE_OP_INSERT, -1, 0);  // a zero-length segment is never linked
    }
    // ---- C: mark [start, end) on the new layout ---------------------------------
    if (rng && pos2 > pos1) {
      s8v q2 = {0, 0, 0, 0, 0, 0, 0, 0};
      if (type == MTE_OP_ANNOTATE) q2 = sload_props(a, (uint32_t)op[6]);
      const bool rem = type == MTE_OP_REMOVE;
      int32_t cy = 0, ocy = 0;  // ocy: the own view's prefix after the op (events)
      uint32_t cnt_all = 0;
      for (int tb = 0; tb < n && cy < pos2; tb += kTile) {
        Regs<E, K> R;
        tile_load_hot<K>(R, pl, sd, tb, n);
        int32_t L[E], P[E];
        leaf_lengths<E, K>(R, r, c + 1, (int)c, D.min_seq, newcalc, L);
        const int32_t tot = prefix<E>(L, P);
        bool in[E];
        uint32_t cnt = 0;
#pragma unroll
        for (int j = 0; j < E; j++) {
          P[j] += cy;
          in[j] = L[j] > 0 && P[j] >= pos1 && P[j] < pos2;
          cnt += (uint32_t)__popcll(__ballot(in[j]));
        }
        cy += tot;
        if (evd) {
          // markRangeRemoved reports the segments it newly removes, annotateRange
          // every one it visits (mergeTree.ts:1954-1959, 1893-1900), at their
          // positions in the own view after the op, in document order
          const bool rem0 = type == MTE_OP_REMOVE;
          bool evf[E];
          int32_t OL[E], OP[E];
#pragma unroll
          for (int j = 0; j < E; j++) {
            evf[j] = in[j] && (!rem0 || R.rseq[j] == kNone);
            const bool gone = rem0 && in[j];
            OL[j] = (R.rseq[j] == kNone && !gone) ? R.len[j] : 0;
          }
          const int32_t otot = prefix<E>(OL, OP);
          uint32_t ecnt = 0;
#pragma unroll
          for (int j = 0; j < E; j++) ecnt += evf[j] ? 1u : 0u;
          const int32_t eincl = wave_incl_scan((int32_t)ecnt);
          uint32_t e = ev.n + (uint32_t)(eincl - (int32_t)ecnt);
#pragma unroll
          for (int j = 0; j < E; j++) {
            if (evf[j]) {
              if (e < ev.cap) ev.p[e] = mte_delta{ev.op, type, ocy + OP[j], R.len[j], OL[j] == 0 ? 1u : 0u};
              e++;
            }
          }
          ev.n += (uint32_t)rdlane(eincl, kWave - 1);
          ocy += otot;
        }
        if (cnt == 0) continue;
        cnt_all += cnt;
        const int base = tb + l * E;
        if (rem) {
          // markRemoved (mergeTree.ts:1924-1962)
#pragma unroll
          for (int j = 0; j < E; j++) {
            if (in[j]) {
              // an earlier removedSeq stays; the remover joins the mask
              pl[2 * sd + base + j] = (uint32_t)(R.rseq[j] == kNone ? s : R.rseq[j]);
              pl[3 * sd + base + j] = R.rmask[j] | (1u << c);
            }
          }
        } else if (K > 0) {
          // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
          // loads unconditional (padding reads slot 0), padding selected away
          // after: no branch per load
          uint32_t pr[K > 0 ? K : 1][E];
#pragma unroll
          for (int kk = 0; kk < K; kk++)
#pragma unroll
            for (int j = 0; j < E; j++) {
              const int i = base + j;
              const uint32_t o = ld_l2(pl + (kFieldPlanes + kk) * sd + (i < n ? i : 0));
              pr[kk][j] = ((flags & MTE_F_REWRITE) && in[j]) ? 0u : (i < n ? o : 0u);
            }
          apply_props<E, K>(pr, in, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], (uint32_t)op[6], a);
#pragma unroll
          for (int kk = 0; kk < K; kk++)
#pragma unroll
            for (int j = 0; j < E; j++)
              if (in[j]) pl[(kFieldPlanes + kk) * sd + base + j] = pr[kk][j];
        }
      }
      MTE_STAT(st[kStWritten] += cnt_all;)
      if (type == MTE_OP_ANNOTATE) st[kStPwrites] += cnt_all * (uint32_t)q2[3];
      vm_drain();
    }
  }
  D.n = n;
  D.k++;

  if (type != MTE_OP_NOOP) {  // Client.completeAndLogOp (client.ts:525-528)
    if (!(D.cur_seq < s)) return MTE_E_SEQ_ORDER;
    if (!(D.min_seq <= msn)) return MTE_E_MSN_ORDER;
  }
  if (flags & MTE_F_MSG_END) {
    // updateSeqNumbers (client.ts:937-945) -> setMinSeq (mergeTree.ts:1077-1093)
    if (!(D.cur_seq <= s)) return MTE_E_SEQ_ORDER;
    D.cur_seq = s;
    if (!(msn <= s)) return MTE_E_MSN_GT_SEQ;
    if (!(D.min_seq <= msn)) return MTE_E_MSN_ORDER;
    if (msn > D.min_seq) {
      D.min_seq = msn;
      // zamboni as a tiled stream compaction, front to back (dst <= src)
      int32_t w = 0;
      for (int tb = 0; tb < n; tb += kTile) {
        const int base = tb + l * E;
        bool keep[E];
        int32_t cntl = 0;
#pragma unroll
        for (int j = 0; j < E; j++) {
          const int i = base + j;
          const int32_t rs = (int32_t)ld_l2(pl + 2 * sd + (i < n ? i : 0));  // unconditional, selected after
          keep[j] = i < n && rs > msn;
          cntl += keep[j] ? 1 : 0;
        }
        const int32_t incl = wave_incl_scan(cntl);
        const int32_t tot = rdlane(incl, kWave - 1);
        if (tot != kTile || w != tb) {
          int32_t dst = w + incl - cntl;
          // kPlaneGroup planes' loads in flight at once, then their stores (dst
          // <= src: a tile's stores land at or below it, after its own loads)
  #pragma nounroll
        for (int p0 = 0; p0 < nplanes; p0 += kPlaneGroup) {
            uint32_t v[kPlaneGroup][E];
#pragma unroll
            for (int g = 0; g < kPlaneGroup; g++) {
              const int pg = p0 + g < nplanes ? p0 + g : nplanes - 1;
              const uint32_t pb = (uint32_t)((uint64_t)pg * sd);
#pragma unroll
              for (int j = 0; j < E; j++) {
                const bool ok = p0 + g < nplanes && keep[j];  // keep implies base + j < n
                const uint32_t x = ld_l2o(pl, pb + (uint32_t)(ok ? base + j : 0));
                v[g][j] = ok ? x : 0u;
              }
            }
#pragma unroll
            for (int g = 0; g < kPlaneGroup; g++) {
              const uint32_t pb = (uint32_t)((uint64_t)(p0 + g) * sd);
              int32_t d0 = dst;
#pragma unroll
              for (int j = 0; j < E; j++) {
                if (p0 + g < nplanes && keep[j] && MTE_SLOT_OK(d0, a.cap)) pl[pb + (uint32_t)d0] = v[g][j];
                d0 += keep[j] ? 1 : 0;
              }
            }
          }
          vm_drain();
        }
        w += tot;
      }
      D.n = w;
    }
  }
  return 0;
}

// pass 3: documents pass 2 escalated (more than 1,022 segments)
template <int K, bool S>
__global__ __launch_bounds__(256) void stream_kernel(ReplayArgs a) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int idx = (int)blockIdx.x * kDocsPerBlock + w;
  if (idx >= (int)a.n_docs) return;
  // longest batch first (a.sorder): the long local-client chains start first
  const int doc = a.sorder ? (int)__builtin_amdgcn_readfirstlane((int)a.sorder[idx]) : idx;
  // documents pass 2 escalated, and the new length-calc documents with delta
  // events and no local client (a local client's go to the HBM tree pass)
  const uint32_t hf = a.hdr[doc].flags;
  if (hf & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) return;  // the HBM tree pass's
  const bool own = (hf & (MTE_DOC_EVENTS | MTE_DOC_NEW_LENGTH_CALC)) == (MTE_DOC_EVENTS | MTE_DOC_NEW_LENGTH_CALC);
  if (!(hf & kHdrNeedsEsc) && !own) return;  // untouched doc: leave the header alone
  DocRun D;
  run_init(D, a, doc, !own);
  uint32_t st[kNumStats] = {};
  EvOut ev{nullptr, 0, 0u, 0u};
  if ((hf & MTE_DOC_EVENTS) && a.dl_off) {
    ev.p = a.dl + a.dl_off[doc];
    ev.cap = a.dl_off[doc + 1] - a.dl_off[doc];
  }
  if (D.running) {
    s8v cur = sload8(D.recp + 2 * D.k);
    while (D.running) {
      const int rc = stream_step<K, S>(D, st, cur, a, ev);
      if (rc < 0) {
        D.status = rc;
        D.running = false;
      } else if (D.k >= D.k1) {
        D.running = false;
      } else if (S && st[kStOps] >= (1u << 20)) {
        run_flush_stats(D, st, a);
      }
    }
    if constexpr (S) run_flush_stats(D, st, a);
  }
  if ((hf & MTE_DOC_EVENTS) && a.dl_n && lane_id() == 0) a.dl_n[doc] = ev.n;
  run_finish(D, a);
}

}  // namespace mte
