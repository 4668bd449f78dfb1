// mte_htree.h — the HBM tree pass: the reference's B+tree over an item array
// left in HBM, one wavefront per document (DESIGN.md §5 "HBM tree pass").
//
// Two kinds of documents replay here:
//   * legacy length-calc documents that outgrow the register tree tiers
//     (mte_tree.h holds at most 1,020 items in registers);
//   * every document with a local client (MTE_DOC_LOCAL_CLIENT), in either
//     length mode: the reference places a sequenced insert next to the
//     client's pending segments by its block edges (continuePredicate's
//     forward excursion, mergeTree.ts:1599-1611, 1788-1793), holds the
//     segments of pending groups in scourNode (:686-688) and runs the lazy
//     zamboni after acks and rollbacks (:1329, 2052-2061), so only the tree
//     replays such a document exactly.
// Its executable spec is oracle/titems.c (doc_apply and the local records);
// every function here names the titems.c function it restates.
//
// Layout per document: the segment planes of the SoA (len seq rseq rmask meta
// toff, K property planes; a local-client document also K pending-key planes,
// the annotate-group mask, K base-value planes and the localRemovedSeq plane),
// the tree word plane (TreeArgs::tree, mte_tree.h), the LRU heap (hcap
// entries) and a small state record, all in HBM; the perspective lengths L and
// their prefix P of the op being applied in a scratch pair, computed lazily
// front to back only as far as the op looks (lp_n).  Items are visited in
// tiles of 64 x kHE, j-major (item tb + 64 j + lane), so each load instruction
// reads 256 contiguous bytes.  Control flow is wave-uniform: the O(n) walks
// (lengths, searches, moves, compactions) run across the wave, the tree's
// bookkeeping (splits, LRU heap, scour's append chain, packParent) as uniform
// scalar code over single-item loads.  Loads bypass L1 (ld_l2) and every phase
// that stores ends with vm_drain, as in mte_stream.h.
#pragma once

#include "mte_stream.h"
#include "mte_tree.h"

namespace mte {

#ifndef MTE_HTREE_KHE
#define MTE_HTREE_KHE 2
#endif
constexpr int kHE = MTE_HTREE_KHE;     // items per lane per tile
constexpr int kHT = kWave * kHE;       // items per tile
constexpr uint32_t kHdrTreeHbm = kHdrTreeHbmFlag;  // a legacy document continues on the HBM tree pass
constexpr int kHtState = 8;            // state words per document

// state words (HtreeArgs::st)
enum HtSt { kHsDepth = 0, kHsNextId, kHsHeapN, kHsLseq, kHsRhi, kHsEntered, kHsWin };

// MTE_HTREE_PROF (a profiling build only, `make prof`): per-phase clocks
// (s_memrealtime ticks, 100 MHz) summed over every document into
// HtreeArgs::prof: 0 insert, 1 remove / annotate, 2 ack, 3 zamboni (inside the
// others too), 4 rollback / regen, 5 references / relative positions, 6 every
// record, 7 records.
constexpr int kHtProf = 8;
#ifdef MTE_HTREE_PROF
#define HPROF_BEGIN(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime();
#define HPROF_END(h, i, v) (h).prof[i] += __builtin_amdgcn_s_memrealtime() - (v);
#else
#define HPROF_BEGIN(v)
#define HPROF_END(h, i, v)
#endif

struct HtreeArgs {
  uint32_t* tree;        // tree words: tree[doc * cap + i]
  const uint2* rheap;    // the register tiers' heaps (kTreeHeapCap + 1 per doc): an escalating doc's
  uint2* heap;           // HBM tree heaps: heap[doc * (hcap + 1) + k], k = 1 .. hn
  uint32_t hcap;
  uint32_t lcap;         // items a document may hold in LDS (0: none; the launch's dynamic LDS)
  uint32_t* st;          // kHtState words per document
  int32_t* scr;          // L at scr[doc * 2 cap + i], P at scr[doc * 2 cap + cap + i]
  const uint32_t* docs;  // the documents this pass may replay
  uint32_t n_docs;
  const uint16_t* arena;
  unsigned long long* prof;  // kHtProf phase clocks (MTE_HTREE_PROF builds), or nullptr
  uint32_t maint;        // some document records maintenance (the htree_kernel<K, S, true> build)
};

// plane indices of a local-client document (after the K property planes)
template <int K> constexpr int kPkPlane = kFieldPlanes + K;
template <int K> constexpr int kLrsPlane = kFieldPlanes + 3 * K + 1;
// kLrsPlane: localRemovedSeq, | kLrsReleased once a regeneration dequeued the
// segment from its group -- it keeps the value, the group no longer holds it
// (resetPendingDeltaToOps, client.ts:802-857; titems.c LRS_RELEASED)
constexpr uint32_t kLrsReleased = 0x40000000u;
// kGrpPlane: the item's place in its pending removal group (SegmentGroup.segments,
// the order an ack walks them, mergeTree.ts:1285): its index at the local
// remove, 0x80000000 | the tail's id for a tail split off later (splitAt's
// segmentGroups.copyTo appends it, mergeTreeNodes.ts:505-534; titems.c gord)
template <int K> constexpr int kGrpPlane = kFieldPlanes + 3 * K + 2;
// kBornPlane: the first localSeq whose segment group can hold the item as one
// of the segments its op marked -- an item split off later joins the groups
// before it as a tail, appended (titems.c item.born); kRgPlane: a regenerated
// segment's group, 1 + its id at its last regeneration, shared by the tails
// split off it since (titems.c item.rg, MTE_F_REGENERATED)
template <int K> constexpr int kBornPlane = kFieldPlanes + 3 * K + 3;
template <int K> constexpr int kRgPlane = kFieldPlanes + 3 * K + 4;
// kRmHiPlane: removedClientIds of short ids 32 .. 63 (MTE_MAX_CLIENTS_TREE;
// plane 3 holds 0 .. 31), zero while the item is not removed; the last plane
// of every document with nP = kLocalPlanes (local-client and MTE_DOC_TREE ones)
template <int K> constexpr int kRmHiPlane = kFieldPlanes + 3 * K + 5;
template <int K> constexpr int kLocalPlanes = kFieldPlanes + 3 * K + 6;  // planes of a local-client / MTE_DOC_TREE document

struct HT {
  uint32_t* pl;   // the document's plane base
  uint64_t sd;    // plane stride
  uint32_t* tw;   // tree words
  int32_t* L;
  int32_t* P;
  uint32_t* hp;   // heap entries as uint32 pairs (index 1 .. hn)
  uint32_t hcap;
  int cap;
  int nP;         // planes an item carries (moves and compactions)
  int n;
  int depth;
  uint32_t next_id, hn;
  int32_t min_seq, cur_seq;
  bool newcalc, ldoc;
  // the perspective of L / P and how far they are valid
  bool plocal;
  int32_t pr;
  int pc;
  int lp_n;
  int32_t lp_carry;
  const uint16_t* arena;
  bool maint;     // MTE_DOC_MAINT_EVENTS: maintenance records (ht_maint)
  uint32_t born;  // kBornPlane of an item made by the record being applied
  // MTE_OP_RELPOS: positions for the next record (rpf: MTE_RP_POS1 / POS2 given)
  uint32_t rpf;
  // the window of the reference's cached local partial lengths (ht_view_window), -1: none
  int32_t wcache;
  int32_t rp1, rp2;
  // LDS residency: the document's planes, tree words, L / P and heap in the
  // workgroup's LDS while they fit (every access goes through the pointers
  // above); its HBM home below
  bool lds;
  uint32_t* g_pl;
  uint64_t g_sd;
  uint32_t* g_tw;
  int32_t* g_L;
  int32_t* g_P;
  uint32_t* g_hp;
  uint32_t g_hcap;
  int g_cap;
#ifdef MTE_HTREE_PROF
  unsigned long long prof[kHtProf];
#endif
};

// ---- single-item access (wave-uniform) ----------------------------------------

__device__ __forceinline__ uint32_t uld(const uint32_t* p) { return uni(ld_l2(p)); }
__device__ __forceinline__ void lane0_st(uint32_t* p, uint32_t v) {
  if (lane_id() == 0) *p = v;
}
__device__ __forceinline__ uint32_t ht_T(const HT& h, int i) { return uld(h.tw + i); }
__device__ __forceinline__ uint32_t ht_pl(const HT& h, int p, int i) { return uld(h.pl + (uint64_t)p * h.sd + i); }
__device__ __forceinline__ void ht_setT(HT& h, int i, uint32_t v) { lane0_st(h.tw + i, v); }
__device__ __forceinline__ void ht_setpl(HT& h, int p, int i, uint32_t v) { lane0_st(h.pl + (uint64_t)p * h.sd + i, v); }

// ---- perspective lengths (titems.c leaf_len / lengths_local) -------------------

__device__ __forceinline__ int32_t ht_item_len(const HT& h, int32_t len, int32_t seq, int32_t rseq, uint32_t rmask,
                                               uint32_t meta, uint32_t t) {
  if (t & kTEmpty) return -1;
  const bool removed = rseq != kNone;
  if (h.plocal) {
    // localNetLength without localSeq (mergeTree.ts:553-573)
    if (!removed) return len;
    return (h.newcalc || rseq > h.min_seq) ? 0 : -1;
  }
  const int c = h.pc;
  const int32_t r = h.pr;
  const bool by_c = ((rmask >> (c & 31)) & 1u) != 0;  // rmask: the half of the mask that holds c (ht_ensure)
  const int cli = (int)(meta & 0xffu) - 1;
  if (h.newcalc) {  // mergeTree.ts:1003-1026
    if (removed) {
      if (rseq <= h.min_seq) return -1;
      if (rseq <= r || by_c) return 0;
    }
    return (seq <= r || cli == c) ? len : 0;
  }
  // mergeTree.ts:1028-1054; a pending local removal (removedSeq Unassigned) is not undefined
  if (removed && rseq <= r) return -1;
  if (cli == c || seq <= r) return (removed && by_c) ? 0 : len;
  return (removed && rseq < kLocalBase) ? -1 : 0;
}

__device__ __forceinline__ void ht_persp(HT& h, bool local, int32_t r, int c) {
  h.plocal = local;
  h.pr = r;
  h.pc = c;
  h.lp_n = 0;
  h.lp_carry = 0;
}

// L / P of the items before `from` stay valid (a split or move at `from`)
__device__ __forceinline__ void ht_inval(HT& h, int from) {
  if (from < h.lp_n) {
    h.lp_n = from;
    h.lp_carry = from > 0 ? (int32_t)uld((const uint32_t*)h.P + from) : 0;
  }
}

// L / P valid through item `upto` (or the document's end)
__device__ __forceinline__ void ht_ensure(HT& h, int upto) {
  const int l = lane_id();
  bool wrote = false;
  // the removers plane holding the perspective's client (ht_item_len)
  const uint32_t* rmp = h.pl + (uint64_t)(h.pc < 32 ? 3 : h.nP - 1) * h.sd;
  while (h.lp_n <= upto && h.lp_n < h.n) {
    const int tb = h.lp_n;
    int32_t len[kHE], seq[kHE], rseq[kHE];
    uint32_t rmask[kHE], meta[kHE], t[kHE];
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const int ic = i < h.n ? i : 0;  // unconditional loads, selected after
      len[j] = (int32_t)ld_l2(h.pl + ic);
      seq[j] = (int32_t)ld_l2(h.pl + h.sd + ic);
      rseq[j] = (int32_t)ld_l2(h.pl + 2 * h.sd + ic);
      rmask[j] = ld_l2(rmp + ic);
      meta[j] = ld_l2(h.pl + 4 * h.sd + ic);
      t[j] = ld_l2(h.tw + ic);
    }
    int32_t carry = h.lp_carry;
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const int32_t Lv = i < h.n ? ht_item_len(h, len[j], seq[j], rseq[j], rmask[j], meta[j], t[j]) : -1;
      const int32_t v = Lv > 0 ? Lv : 0;
      const int32_t incl = wave_incl_scan(v);
      if (i < h.n) {
        h.L[i] = Lv;
        h.P[i] = carry + incl - v;
      }
      carry += rdlane(incl, kWave - 1);
    }
    h.lp_carry = carry;
    h.lp_n = tb + kHT < h.n ? tb + kHT : h.n;
    wrote = true;
  }
  if (wrote) vm_drain();
}

// ---- searches (wave-parallel, early exit) ----------------------------------------

// first i in [lo, hi) with pred(i) (evaluated per lane), or -1
template <typename F>
__device__ __forceinline__ int ht_first(int lo, int hi, F pred) {
  const int l = lane_id();
  for (int tb = lo; tb < hi; tb += kHT) {
    bool p[kHE];
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      p[j] = i < hi && pred(i < hi ? i : lo);
    }
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const uint64_t m = __ballot(p[j]);
      if (m) return tb + j * kWave + (__ffsll((long long)m) - 1);
    }
  }
  return -1;
}

// last i in [lo, hi) with pred(i), or -1
template <typename F>
__device__ __forceinline__ int ht_last(int lo, int hi, F pred) {
  const int l = lane_id();
  for (int te = hi; te > lo; te -= kHT) {
    const int tb = te - kHT;
    bool p[kHE];
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      p[j] = i >= lo && i < te && pred(i >= lo && i < te ? i : lo);
    }
#pragma unroll
    for (int j = kHE - 1; j >= 0; j--) {
      const uint64_t m = __ballot(p[j]);
      if (m) return tb + j * kWave + (63 - __clzll((long long)m));
    }
  }
  return -1;
}

// number of i in [lo, hi) with pred(i)
template <typename F>
__device__ __forceinline__ int ht_count(int lo, int hi, F pred) {
  const int l = lane_id();
  int c = 0;
  for (int tb = lo; tb < hi; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      c += __popcll(__ballot(i < hi && pred(i < hi ? i : lo)));
    }
  }
  return c;
}

// the r-th (0-based) i in [lo, hi) with pred(i), or -1
template <typename F>
__device__ __forceinline__ int ht_nth(int lo, int hi, int r, F pred) {
  const int l = lane_id();
  for (int tb = lo; tb < hi; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      uint64_t m = __ballot(i < hi && pred(i < hi ? i : lo));
      const int c = __popcll(m);
      if (r < c) {
        for (int q = 0; q < r; q++) m &= m - 1;
        return tb + j * kWave + (__ffsll((long long)m) - 1);
      }
      r -= c;
    }
  }
  return -1;
}

// search over L / P: they are extended tile by tile as the search advances
template <typename F>
__device__ __forceinline__ int ht_first_lp(HT& h, int lo, F pred) {
  for (int tb = lo; tb < h.n; tb += kHT) {
    const int te = tb + kHT < h.n ? tb + kHT : h.n;
    ht_ensure(h, te - 1);
    const int x = ht_first(tb, te, pred);
    if (x >= 0) return x;
  }
  return -1;
}

// ---- moves -------------------------------------------------------------------------

// planes moved per batch of loads: kHtGroup planes' loads in flight at once,
// then their stores (one memory round trip per group, not per plane)
constexpr int kHtGroup = 8;

__device__ __forceinline__ uint32_t* ht_plane(const HT& h, int p) {  // p == nP: the tree word
  return p < h.nP ? h.pl + (uint64_t)p * h.sd : h.tw;
}

// open an empty slot at g: items [g, n) move up by one (titems.c open_slot)
__device__ __forceinline__ void ht_open(HT& h, int g) {
  const int l = lane_id();
  for (int te = h.n; te > g; te -= kHT) {
    const int tb = te - kHT > g ? te - kHT : g;
    for (int p0 = 0; p0 <= h.nP; p0 += kHtGroup) {
      uint32_t v[kHtGroup][kHE];
#pragma unroll
      for (int q = 0; q < kHtGroup; q++) {
        const int p = p0 + q <= h.nP ? p0 + q : h.nP;  // past the last plane: reload it, stored never
        const uint32_t* base = ht_plane(h, p);
#pragma unroll
        for (int j = 0; j < kHE; j++) {
          const int i = tb + j * kWave + l;
          v[q][j] = ld_l2(base + (i < te ? i : tb));
        }
      }
#pragma unroll
      for (int q = 0; q < kHtGroup; q++) {
        if (p0 + q > h.nP) break;
        uint32_t* base = ht_plane(h, p0 + q);
#pragma unroll
        for (int j = 0; j < kHE; j++) {
          const int i = tb + j * kWave + l;
          if (i < te) base[i + 1] = v[q][j];
        }
      }
    }
  }
  h.n++;
  vm_drain();
  ht_inval(h, g);
}

// copy every plane of item `from` into slot `to` (one lane per plane)
__device__ __forceinline__ void ht_copy_item(HT& h, int from, int to) {
  const int l = lane_id();
  if (l < h.nP) {
    uint32_t* b = h.pl + (uint64_t)l * h.sd;
    b[to] = ld_l2(b + from);
  }
  vm_drain();
}

// drop the items i in [lo, hi] whose flag (L scratch) is set; the others keep
// their order (titems.c compact)
__device__ __forceinline__ void ht_compact(HT& h, int lo, int hi) {
  const int l = lane_id();
  int w = lo;
  for (int tb = lo; tb < h.n; tb += kHT) {
    bool keep[kHE];
    int32_t dst[kHE];
    int kept = 0;
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const int32_t f = (int32_t)ld_l2((const uint32_t*)h.L + (i < h.n ? i : 0));
      keep[j] = i < h.n && !(i <= hi && f != 0);
      const int32_t incl = wave_incl_scan(keep[j] ? 1 : 0);
      dst[j] = w + kept + incl - (keep[j] ? 1 : 0);
      kept += rdlane(incl, kWave - 1);
    }
    if (w != tb || kept != (h.n - tb < kHT ? h.n - tb : kHT)) {
      for (int p0 = 0; p0 <= h.nP; p0 += kHtGroup) {
        uint32_t v[kHtGroup][kHE];
#pragma unroll
        for (int q = 0; q < kHtGroup; q++) {
          const int p = p0 + q <= h.nP ? p0 + q : h.nP;
          const uint32_t* base = ht_plane(h, p);
#pragma unroll
          for (int j = 0; j < kHE; j++) {
            const int i = tb + j * kWave + l;
            v[q][j] = ld_l2(base + (keep[j] ? i : tb));
          }
        }
#pragma unroll
        for (int q = 0; q < kHtGroup; q++) {
          if (p0 + q > h.nP) break;
          uint32_t* base = ht_plane(h, p0 + q);
#pragma unroll
          for (int j = 0; j < kHE; j++)
            if (keep[j]) base[dst[j]] = v[q][j];
        }
      }
    }
    w += kept;
    if (tb >= hi && w == tb + kept) {  // past the range with nothing moved: the rest stays
      w = h.n;
      break;
    }
  }
  vm_drain();
  h.n = w;
  h.lp_n = 0;
  h.lp_carry = 0;
}

// ---- block spans (titems.c span_start / span_end / children) -----------------------

__device__ __forceinline__ int ht_span_start(const HT& h, int i, int k) {
  const uint32_t* tw = h.tw;
  const int s = ht_last(0, i + 1, [&](int x) { return (int)t_h(ld_l2(tw + x)) >= k; });
  return s < 0 ? 0 : s;
}
__device__ __forceinline__ int ht_span_end(const HT& h, int s, int k) {
  const uint32_t* tw = h.tw;
  const int e = ht_first(s + 1, h.n, [&](int x) { return (int)t_h(ld_l2(tw + x)) >= k; });
  return e < 0 ? h.n - 1 : e - 1;
}
__device__ __forceinline__ bool is_child_t(uint32_t t, int k) {
  return k == 1 ? (t & (kTCont | kTEmpty)) == 0 : (int)t_h(t) >= k - 1;
}
__device__ __forceinline__ int ht_children(const HT& h, int s, int e, int k) {
  const uint32_t* tw = h.tw;
  return ht_count(s, e + 1, [&](int x) { return is_child_t(ld_l2(tw + x), k); });
}
__device__ __forceinline__ void ht_set_h(HT& h, int i, uint32_t hv, bool clear_ns) {
  const uint32_t t = ht_T(h, i);
  ht_setT(h, i, (t & ~(kTH | (clear_ns ? kTNs : 0u))) | hv);
  vm_drain();
}

// split_cascade (titems.c): a leaf block gained a child at item i
__device__ __forceinline__ void ht_split_cascade(HT& h, int i) {
  for (int k = 1;; k++) {
    const int s = ht_span_start(h, i, k), e = ht_span_end(h, s, k);
    if (ht_children(h, s, e, k) < kMaxNodes) return;
    const uint32_t* tw = h.tw;
    const int z = ht_nth(s, e + 1, kMaxNodes / 2, [&](int x) { return is_child_t(ld_l2(tw + x), k); });
    ht_set_h(h, z, (uint32_t)k, k == 1);
    if (k == h.depth) {  // the root split: a new root above both halves
      h.depth++;
      ht_set_h(h, 0, (uint32_t)h.depth, false);
      return;
    }
  }
}

// ---- LRU heap (collections/heap.ts; titems.c heap_add / heap_get) ----------------------

__device__ __forceinline__ uint2 ht_hget(const HT& h, uint32_t k) {
  return make_uint2(uld(h.hp + 2 * k), uld(h.hp + 2 * k + 1));
}
__device__ __forceinline__ void ht_hput(HT& h, uint32_t k, uint2 v) {
  if (lane_id() == 0) {
    h.hp[2 * k] = v.x;
    h.hp[2 * k + 1] = v.y;
  }
}

__device__ __forceinline__ int ht_heap_add(HT& h, int32_t key, uint32_t id) {
  if (h.hn >= h.hcap) return MTE_E_CAPACITY;
  uint32_t k = ++h.hn;
  while (k > 1) {  // the same comparisons as heap.ts fixup, moving a hole
    const uint2 par = ht_hget(h, k >> 1);
    if (!((int32_t)par.x - key > 0)) break;
    ht_hput(h, k, par);
    vm_drain();
    k >>= 1;
  }
  ht_hput(h, k, make_uint2((uint32_t)key, id));
  vm_drain();
  return 0;
}

__device__ __forceinline__ uint2 ht_heap_pop(HT& h) {
  const uint2 x = ht_hget(h, 1);
  const uint2 cur = ht_hget(h, h.hn);
  h.hn--;
  uint32_t k = 1;
  while ((k << 1) <= h.hn) {
    uint32_t j = k << 1;
    uint2 c = ht_hget(h, j);
    if (j < h.hn) {
      const uint2 c1 = ht_hget(h, j + 1);
      if ((int32_t)c.x - (int32_t)c1.x > 0) {
        j++;
        c = c1;
      }
    }
    if ((int32_t)cur.x - (int32_t)c.x <= 0) break;
    ht_hput(h, k, c);
    vm_drain();
    k = j;
  }
  if (h.hn > 0) ht_hput(h, k, cur);
  vm_drain();
  return x;
}

// add_lru (titems.c): addToLRUSet for the leaf headed at item i
__device__ __forceinline__ int ht_add_lru(HT& h, int i, int32_t seq, int& bs_cache, int& be_cache) {
  int bs;
  if (i >= bs_cache && i <= be_cache) {
    bs = bs_cache;
  } else {
    bs = ht_span_start(h, i, 1);
    bs_cache = bs;
    be_cache = ht_span_end(h, bs, 1);
  }
  const uint32_t tb = ht_T(h, bs);
  if (t_ns(tb) != kNsTrue && seq > h.cur_seq) {
    ht_setT(h, bs, (tb & ~kTNs) | (kNsTrue << kTNsShift));
    vm_drain();
    return ht_heap_add(h, seq, t_id(ht_T(h, i)));
  }
  return 0;
}

// ---- scour / pack (titems.c scour, drop_keep_starts, pack_parent) -----------------------

// end (exclusive) of the logical leaf headed at i (titems.c leaf_end)
__device__ __forceinline__ int ht_leaf_end(const HT& h, int i) {
  const uint32_t* tw = h.tw;
  const int e = ht_first(i + 1, h.n, [&](int x) { return (ld_l2(tw + x) & kTCont) == 0; });
  return e < 0 ? h.n : e;
}
__device__ __forceinline__ int32_t ht_sum_len(const HT& h, int a, int b) {
  const int l = lane_id();
  int32_t s = 0;
  for (int tb = a; tb < b; tb += kHT)
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const int32_t v = (int32_t)ld_l2(h.pl + (i < b ? i : a));
      s += i < b ? v : 0;
    }
  return rdlane(wave_incl_scan(s), kWave - 1);
}

// one segment of a maintenance callback (MTE_DELTA_MAINT, include/mte.h;
// titems.c maint_push): named by its leaf's id until the message's end
// (ht_maint_positions), -1 out of the tree; idx its index in the callback
__device__ __forceinline__ void ht_maint(const HT& h, EvOut& ev, uint32_t type, int32_t id, int32_t len, uint32_t idx) {
  if (!h.maint) return;
  if (lane_id() == 0 && ev.n < ev.cap) ev.p[ev.n] = mte_delta{ev.op, MTE_DELTA_MAINT | type, id, len, idx};
  ev.n++;
}
__device__ __forceinline__ int ht_leaf_start(const HT& h, int i) {
  const uint32_t* tw = h.tw;
  const int s = ht_last(0, i + 1, [&](int x) { return (ld_l2(tw + x) & kTCont) == 0; });
  return s < 0 ? 0 : s;
}
// the SPLIT callback (splitLeafSegment, mergeTree.ts:1682-1694): the leaf
// ending before item i and the one starting there (titems.c maint_split)
__device__ __forceinline__ void ht_maint_split(HT& h, EvOut& ev, int i) {
  if (!h.maint) return;
  const int hd = ht_leaf_start(h, i - 1);
  ht_maint(h, ev, MTE_MAINT_SPLIT, (int32_t)t_id(ht_T(h, hd)), ht_sum_len(h, hd, i), 0u);
  ht_maint(h, ev, MTE_MAINT_SPLIT, (int32_t)t_id(ht_T(h, i)), ht_sum_len(h, i, ht_leaf_end(h, i)), 1u);
}

// mark items [a, b) for dropping (the L scratch is the flag plane)
__device__ __forceinline__ void ht_mark(HT& h, int a, int b, int32_t f) {
  const int l = lane_id();
  for (int tb = a; tb < b; tb += kHT)
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      if (i < b) h.L[i] = f;
    }
}

// scourNode over the leaf block [s, e] (mergeTree.ts:681-747): marks the
// unlinked items, turns appended leaves into continuations; returns the
// logical leaves held.  The caller cleared the flags of [s, e].
template <int K>
__device__ __forceinline__ int ht_scour(HT& h, int s, int e, uint32_t n_keys, EvOut& ev) {
  int held = 0;
  int prev = -1;             // head of the leaf appends go to
  int32_t prev_len = 0;
  int prev_end = 0;
  for (int i = s; i <= e;) {
    const uint32_t tx = ht_T(h, i);
    if (tx & kTEmpty) {
      i++;
      continue;
    }
    const int xe = ht_leaf_end(h, i);
    const int32_t xl = ht_sum_len(h, i, xe);
    const int32_t seq = (int32_t)ht_pl(h, 1, i), rseq = (int32_t)ht_pl(h, 2, i);
    bool grouped = seq >= kLocalBase;  // a pending insert
    if (h.ldoc && !grouped) {
      const uint32_t lr = ht_pl(h, kLrsPlane<K>, i);
      grouped = (lr != 0u && !(lr & kLrsReleased)) || ht_pl(h, kAnnPlane<K>, i) != 0u;
    }
    if (grouped) {
      // a segment of a pending group is held and ends the append run (:686, 736-739)
      held++;
      prev = -1;
    } else if (rseq != kNone) {
      if (rseq > h.min_seq) {
        held++;
      } else {
        ht_mark(h, i, xe, 1);
        ht_maint(h, ev, MTE_MAINT_UNLINK, -1, xl, 0u);  // mergeTree.ts:692-703
      }
      prev = -1;
    } else if (seq <= h.min_seq) {
      bool app = false;
      if (prev >= 0) {
        const uint32_t tp = ht_T(h, prev);
        const uint32_t mp = ht_pl(h, 4, prev), mx = ht_pl(h, 4, i);
        // the last text of the leaf appended to ends in '\n' (only texts that held one are read)
        const int pe = prev_end - 1;
        const uint32_t tpe = ht_T(h, pe);
        bool nl = false;
        if (tpe & kTNl) {
          const uint32_t pel = ht_pl(h, 0, pe), pet = ht_pl(h, 5, pe);
          nl = pel > 0 && uni((uint32_t)h.arena[pet + pel - 1u]) == (uint32_t)'\n';
        }
        bool match = (tp & kTPo) == (tx & kTPo);
        for (uint32_t k = 0; k < n_keys && k < (uint32_t)K && match; k++) {
          const uint32_t vx = ht_pl(h, kFieldPlanes + (int)k, i);
          match = ht_pl(h, kFieldPlanes + (int)k, prev) == vx && !(vx & MTE_VALUE_UNEQUAL);  // NaN !== NaN
        }
        app = (mp >> 8) == 0 && (mx >> 8) == 0 && !nl && (prev_len <= kTextGranularity || xl <= kTextGranularity) &&
              match && xl > 0;
      }
      if (app) {
        ht_setT(h, i, (tx & ((0xffu & ~kTNs) | kTNl)) | kTCont);  // id 0: a continuation
        prev_len += xl;
        prev_end = xe;
        // mergeTree.ts:715-727: the segment appended to, then this one
        ht_maint(h, ev, MTE_MAINT_APPEND, (int32_t)t_id(ht_T(h, prev)), prev_len, 0u);
        ht_maint(h, ev, MTE_MAINT_APPEND, -1, xl, 1u);
      } else {
        held++;
        if (xl > 0) {
          prev = i;
          prev_len = xl;
          prev_end = xe;
        } else {
          prev = -1;
        }
      }
    } else {
      held++;
      prev = -1;
    }
    i = xe;
  }
  vm_drain();
  return held;
}

// titems.c drop_keep_starts over [s, e]: every block start moves to a kept
// item of its block; a block left with no leaf keeps a placeholder
__device__ __forceinline__ void ht_drop_keep_starts(HT& h, int s, int e) {
  const int32_t* Lf = h.L;
  for (int b = s; b <= e;) {
    const int be = ht_span_end(h, b, 1);
    const int j = ht_first(b, be + 1, [&](int x) { return ld_l2((const uint32_t*)Lf + x) == 0u; });
    const uint32_t tb = ht_T(h, b);
    if (j < 0) {
      // placeholder(h) with the block's ns (titems.c placeholder)
      ht_setpl(h, 0, b, 0u);
      ht_setpl(h, 1, b, 0u);
      ht_setpl(h, 2, b, (uint32_t)kPad);
      ht_setpl(h, 3, b, 0u);
      ht_setpl(h, 4, b, 0u);
      ht_setpl(h, 5, b, 0u);
      for (int p = kFieldPlanes; p < h.nP; p++) ht_setpl(h, p, b, 0u);
      ht_setT(h, b, (tb & (kTH | kTNs)) | kTEmpty);
      lane0_st((uint32_t*)h.L + b, 0u);
    } else if (j != b) {
      const uint32_t tj = ht_T(h, j);
      ht_setT(h, j, (tj & ~(kTH | kTNs)) | (tb & (kTH | kTNs)));
    }
    vm_drain();
    b = be + 1;
  }
}

__device__ __forceinline__ bool group_start_h(int r, int base, int rem) {
  const int big = rem * (base + 1);
  if (r < big) return r % (base + 1) == 0;
  return (r - big) % base == 0;
}

// the items [s, e]'s group starts: rank r (counted over items with pred) of
// cnt starts a group of the base + 1 / base split (packParent,
// mergeTree.ts:764-786), setting h = top for the first, else `hv`, and `other`
// on the rest of the ranked items (other < 0: left alone)
template <typename F>
__device__ __forceinline__ void ht_regroup(HT& h, int s, int e, int total, uint32_t top, uint32_t hv, int other, bool clear_ns,
                           F pred) {
  int cc = total / (kMaxNodes / 2) < kMaxNodes - 1 ? total / (kMaxNodes / 2) : kMaxNodes - 1;
  if (cc < 1) cc = 1;
  const int gb = total / cc, rem = total % cc;
  const int l = lane_id();
  int r0 = 0;
  for (int tb = s; tb <= e; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const bool in = i <= e;
      const uint32_t t = ld_l2(h.tw + (in ? i : s));
      const bool q = in && pred(t);
      const int32_t incl = wave_incl_scan(q ? 1 : 0);
      const int r = r0 + incl - (q ? 1 : 0);
      if (q) {
        if (group_start_h(r, gb, rem)) {
          h.tw[i] = (t & ~(kTH | (clear_ns ? kTNs : 0u))) | (r == 0 ? top : hv);
        } else if (other >= 0) {
          h.tw[i] = (t & ~kTH) | (uint32_t)other;
        }
      }
      r0 += rdlane(incl, kWave - 1);
    }
  }
  vm_drain();
}

template <int K>
__device__ __forceinline__ int ht_pack_parent(HT& h, int s, int p, uint32_t n_keys, int& status, EvOut& ev);

// zamboniSegments (titems.c zamboni): at most two scours
template <int K>
__device__ __forceinline__ int ht_zamboni_body(HT& h, uint32_t n_keys, EvOut& ev);
template <int K>
__device__ __forceinline__ int ht_zamboni(HT& h, uint32_t n_keys, EvOut& ev) {
  HPROF_BEGIN(t0)
  const int rc = ht_zamboni_body<K>(h, n_keys, ev);
  HPROF_END(h, 3, t0)
  return rc;
}
template <int K>
__device__ __forceinline__ int ht_zamboni_body(HT& h, uint32_t n_keys, EvOut& ev) {
  int status = 0;
  for (int z = 0; z < 2; z++) {
    if (h.hn == 0) break;
    const uint2 top = ht_hget(h, 1);
    if ((int32_t)top.x > h.min_seq) break;
    const uint2 ent = ht_heap_pop(h);
    const uint32_t* tw = h.tw;
    const int i = ht_first(0, h.n, [&](int x) {
      const uint32_t t = ld_l2(tw + x);
      return t_id(t) == ent.y && (t & (kTCont | kTEmpty)) == 0;
    });
    if (i < 0) continue;  // unlinked
    const int bs = ht_span_start(h, i, 1), be = ht_span_end(h, bs, 1);
    const uint32_t tbs = ht_T(h, bs);
    if (t_ns(tbs) == kNsFalse) continue;
    const int before = ht_children(h, bs, be, 1);
    ht_mark(h, bs, be + 1, 0);
    h.lp_n = 0;
    const int held = ht_scour<K>(h, bs, be, n_keys, ev);
    {
      const uint32_t t2 = ht_T(h, bs);
      ht_setT(h, bs, (t2 & ~kTNs) | (kNsFalse << kTNsShift));
      vm_drain();
    }
    if (held < before) {
      ht_drop_keep_starts(h, bs, be);
      ht_compact(h, bs, be);
      if (held < kMaxNodes / 2 && h.depth >= 2) {
        ht_pack_parent<K>(h, ht_span_start(h, bs, 2), 2, n_keys, status, ev);
        if (status) return status;
      }
    }
  }
  return status;
}

// packParent (mergeTree.ts:750-798) of the level-p block starting at s
template <int K>
__device__ __forceinline__ int ht_pack_parent(HT& h, int s, int p, uint32_t n_keys, int& status, EvOut& ev) {
  for (;;) {
    int e = ht_span_end(h, s, p);
    const uint32_t top = t_h(ht_T(h, s));
    if (p == 2) {
      ht_mark(h, s, e + 1, 0);
      h.lp_n = 0;
      for (int b = s; b <= e;) {
        const int be = ht_span_end(h, b, 1);
        ht_scour<K>(h, b, be, n_keys, ev);
        b = be + 1;
      }
      // the held leaves, re-packed: drop the scoured-out items and the placeholders
      {
        const int l = lane_id();
        for (int tb = s; tb <= e; tb += kHT)
#pragma unroll
          for (int j = 0; j < kHE; j++) {
            const int i = tb + j * kWave + l;
            if (i <= e) {
              const uint32_t t = ld_l2(h.tw + i);
              if (t & kTEmpty) h.L[i] = 1;
              h.tw[i] = t & ~kTH;
            }
          }
        vm_drain();
      }
      const int n0 = h.n;
      ht_compact(h, s, e);
      e -= n0 - h.n;
      if (e < s) {
        // no leaf left: one empty leaf block
        if (h.n + 2 > h.cap) {
          status = MTE_E_CAPACITY;
          return h.n;
        }
        ht_open(h, s);
        ht_setpl(h, 0, s, 0u);
        ht_setpl(h, 1, s, 0u);
        ht_setpl(h, 2, s, (uint32_t)kPad);
        ht_setpl(h, 3, s, 0u);
        ht_setpl(h, 4, s, 0u);
        ht_setpl(h, 5, s, 0u);
        for (int q = kFieldPlanes; q < h.nP; q++) ht_setpl(h, q, s, 0u);
        ht_setT(h, s, top | kTEmpty);
        vm_drain();
      } else {
        const uint32_t* tw = h.tw;
        const int total = ht_count(s, e + 1, [&](int x) { return (ld_l2(tw + x) & kTCont) == 0; });
        ht_regroup(h, s, e, total, top, 1u, -1, true, [](uint32_t t) { return (t & kTCont) == 0; });
      }
    } else {
      // level p >= 3: the level-(p-2) blocks regrouped under new level-(p-1) blocks
      const uint32_t* tw = h.tw;
      const int pm2 = p - 2;
      const int total = ht_count(s, e + 1, [&](int x) { return (int)t_h(ld_l2(tw + x)) >= pm2; });
      ht_regroup(h, s, e, total, top, (uint32_t)(p - 1), p - 2, false,
                 [pm2](uint32_t t) { return (int)t_h(t) >= pm2; });
    }
    // the parent's own child count: an underflow re-packs its parent too
    if (p >= h.depth) return h.n;
    const int cc = ht_children(h, s, ht_span_end(h, s, p), p);
    if (cc >= kMaxNodes / 2) return h.n;
    s = ht_span_start(h, s, p + 1);
    p++;
  }
}

// ---- ensureIntervalBoundary (titems.c boundary) ---------------------------------------

template <int K, bool S>
__device__ __forceinline__ int ht_boundary(HT& h, int32_t pos, uint32_t (&st)[kNumStats], EvOut& ev) {
  const int32_t* Lp = h.L;
  const int32_t* Pp = h.P;
  const int i = ht_first_lp(h, 0, [&](int x) {
    const int32_t l = (int32_t)ld_l2((const uint32_t*)Lp + x);
    return l > 0 && (int32_t)ld_l2((const uint32_t*)Pp + x) + l > pos;
  });
  if (i < 0) return 0;
  const int32_t P = (int32_t)uld((const uint32_t*)h.P + i);
  if (P > pos) return 0;
  const uint32_t t = ht_T(h, i);
  if (P == pos) {
    if (t & kTCont) {  // between two texts of one merged leaf
      MTE_STAT(st[kStWritten] += 1;)
      ht_setT(h, i, (t & (kTPo | kTNl)) | (h.next_id++ << 8));
      vm_drain();
      ht_split_cascade(h, i);
      ht_maint_split(h, ev, i);
    }
    return 0;
  }
  // split the leaf at pos - P (the tail copies everything but the length)
  const int32_t off = pos - P;
  if (h.n + 1 > h.cap) return MTE_E_CAPACITY;
  const uint32_t len = ht_pl(h, 0, i), toff = ht_pl(h, 5, i);
  ht_open(h, i + 1);
  ht_copy_item(h, i, i + 1);  // the tail inherits everything (mergeTreeNodes.ts:505-534)
  ht_setpl(h, 0, i, (uint32_t)off);
  ht_setpl(h, 0, i + 1, len - (uint32_t)off);
  ht_setpl(h, 5, i + 1, toff + (uint32_t)off);
  if (h.ldoc) {
    ht_setpl(h, kGrpPlane<K>, i + 1, 0x80000000u | h.next_id);
    ht_setpl(h, kBornPlane<K>, i + 1, h.born);
  }
  ht_setT(h, i + 1, (t & (kTPo | kTNl)) | (h.next_id++ << 8));
  vm_drain();
  ht_inval(h, i);
  MTE_STAT(st[kStWritten] += 2;)
  ht_split_cascade(h, i + 1);
  ht_maint_split(h, ev, i + 1);
  return 0;
}

// ---- the op's new item ---------------------------------------------------------------

// write the planes of a new segment at slot g (one lane per plane): the
// insert's spec (textSegment.ts:40-48, mergeTreeNodes.ts:602-609), its props,
// nothing pending
template <int K>
__device__ __forceinline__ void ht_put_new(HT& h, int g, const s8v& op, bool local, uint32_t refd, const ReplayArgs& a) {
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  const bool marker = (flags & MTE_F_MARKER) != 0;
  const int32_t s = op[0], pos2 = op[5];
  const uint32_t psi = (uint32_t)op[7];
  const int l = lane_id();
  uint32_t v = 0u;
  if (l == 0) v = marker ? 1u : (uint32_t)pos2;
  else if (l == 1) v = (uint32_t)(local ? kLocalBase + s : s);
  else if (l == 2) v = (uint32_t)kNone;
  else if (l == 3) v = 0u;
  else if (l == 4) v = (c + 1u) | (marker ? (1u + (uint32_t)pos2) << 8 : 0u);
  else if (l == 5) v = (marker && !refd) ? 0u : a.text_base + (uint32_t)op[6];
  else if (l == kBornPlane<K>) v = h.born;
  if (K > 0 && psi != MTE_NO_PROPS) {
    const mte_propset ps = a.ps[psi];
    for (uint32_t t = 0; t < ps.count; t++) {
      const mte_prop p = a.pe[ps.first + t];
      if (p.key < a.n_keys && p.key < (uint32_t)K && l == kFieldPlanes + (int)p.key) v = p.value;
    }
  }
  if (l < h.nP) h.pl[(uint64_t)l * h.sd + g] = v;
  vm_drain();
}

// ---- insert (titems.c tree_insert) ---------------------------------------------------

// insertSegments -> blockInsert -> insertingWalk (mergeTree.ts:1394-1422,
// 1590-1680, 1723-1825); *at = the new item or -1
template <int K, bool S>
__device__ __forceinline__ int ht_insert(HT& h, const s8v& op, bool local, bool refd, const ReplayArgs& a, uint32_t (&st)[kNumStats],
                         int& at, EvOut& ev) {
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  const int32_t s = op[0], r = op[1], pos = op[4], pos2 = op[5];
  at = -1;
  ht_persp(h, local, r, (int)c);
  int rc = ht_boundary<K, S>(h, pos, st, ev);
  if (rc) return rc;
  const bool marker = (flags & MTE_F_MARKER) != 0;
  const int32_t len = marker ? 1 : pos2;
  if (len <= 0) return 0;  // blockInsert skips zero-length segments (:1645)
  const int32_t* Lp = h.L;
  const int32_t* Pp = h.P;
  const uint32_t* tw = h.tw;
  const uint32_t* seqp = h.pl + h.sd;
  // the leaf block insertingWalk enters: the first whose end reaches pos
  int ks = ht_first_lp(h, 0, [&](int x) {
    const int32_t l = (int32_t)ld_l2((const uint32_t*)Lp + x);
    return (int32_t)ld_l2((const uint32_t*)Pp + x) + (l > 0 ? l : 0) >= pos;
  });
  if (ks < 0) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
  int bs = ht_span_start(h, ks, 1), be = ht_span_end(h, bs, 1);
  int slot;
  bool replace = false;
  for (;;) {
    slot = -1;
    if (!(ht_T(h, bs) & kTEmpty)) {
      ht_ensure(h, be);
      // before the first defined leaf at pos: pos < len, or a zero-length leaf
      // breakTie prefers (every sequenced one; a pending one only for a local
      // insert: Unassigned is MAX vs MAX - 1, :1705-1721)
      slot = ht_first(ks, be + 1, [&](int x) {
        const int32_t l = (int32_t)ld_l2((const uint32_t*)Lp + x);
        const int32_t p = (int32_t)ld_l2((const uint32_t*)Pp + x);
        const uint32_t t = ld_l2(tw + x);
        const int32_t sq = (int32_t)ld_l2(seqp + x);
        return l >= 0 && p >= pos && !(t & kTEmpty) && !(!local && l == 0 && sq >= kLocalBase);
      });
      if (slot >= 0) break;
    }
    // _pos == 0 at the block's end: a sequenced insert asks continuePredicate,
    // whose forward excursion looks at the first segment after the block and
    // moves past the block when it is a pending local one (:1599-1611, 1788-1793)
    if (!local) {
      const int x = ht_first(be + 1, h.n, [&](int y) { return (ld_l2(tw + y) & kTEmpty) == 0; });
      if (x >= 0 && (int32_t)ht_pl(h, 1, x) >= kLocalBase) {
        ks = x;
        bs = ht_span_start(h, x, 1);
        be = ht_span_end(h, bs, 1);
        continue;
      }
    }
    if (ht_T(h, bs) & kTEmpty) {
      slot = bs;
      replace = true;
    } else {
      slot = be + 1;
    }
    break;
  }
  if (!replace && h.n + 1 > h.cap) return MTE_E_CAPACITY;
  if (h.next_id + 2 >= kIdLimit) return MTE_E_CAPACITY;
  const uint32_t psi = (uint32_t)op[7];
  uint32_t tw_new = (h.next_id++ << 8) | (psi != MTE_NO_PROPS ? kTPo : 0u) | ((flags & kRecNl) ? kTNl : 0u);
  if (replace) {
    tw_new |= ht_T(h, slot) & (kTH | kTNs);
  } else {
    ht_open(h, slot);
    if (slot == bs) {  // the new leaf becomes the block's first child
      const uint32_t t1 = ht_T(h, slot + 1);
      tw_new |= t1 & (kTH | kTNs);
      ht_setT(h, slot + 1, t1 & ~(kTH | kTNs));
    }
  }
  ht_put_new<K>(h, slot, op, local, refd ? 1u : 0u, a);
  ht_setT(h, slot, tw_new);
  vm_drain();
  ht_inval(h, slot);
  MTE_STAT(st[kStWritten] += 1;)
  MTE_STAT(if (!marker) st[kStUnits] += (uint32_t)len;)
  if (K > 0 && psi != MTE_NO_PROPS) {
    const mte_propset ps = a.ps[psi];
    uint32_t w = 0;
    for (uint32_t t = 0; t < ps.count; t++) w += a.pe[ps.first + t].key < a.n_keys ? 1u : 0u;
    MTE_STAT(st[kStPwrites] += w;)
  }
  if (!replace) ht_split_cascade(h, slot);
  // saveIfLocal (:1614-1627): a local segment joins the pending list, a sequenced one the LRU set
  if (!local) {
    int bc = -1, bec = -2;
    if ((rc = ht_add_lru(h, slot, s, bc, bec))) return rc;
  }
  at = slot;
  return 0;
}

// ---- remove / annotate (titems.c tree_range) -------------------------------------------

// joins per-item delta records into one per segment: an item that continues
// the leaf of the item just before it (both visited) adds its length to that
// item's record (the leaf is one segment of the reference)
struct EvRun {
  int64_t last_item;  // the item of the last record, or -2
};

template <int K, bool S>
__device__ __forceinline__ int ht_range(HT& h, const s8v& op, bool local, const ReplayArgs& a, uint32_t (&st)[kNumStats], EvOut& ev,
                        bool evd, uint2* rt, uint32_t rhi, bool evs) {
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  const int32_t s = op[0], r = op[1], start = op[4], end = op[5];
  ht_persp(h, local, r, (int)c);
  int rc = ht_boundary<K, S>(h, start, st, ev);
  if (rc) return rc;
  if ((rc = ht_boundary<K, S>(h, end, st, ev))) return rc;
  if (end == start) return 0;
  const int32_t* Lp = h.L;
  const int32_t* Pp = h.P;
  const int i0 = ht_first_lp(h, 0, [&](int x) {
    const int32_t l = (int32_t)ld_l2((const uint32_t*)Lp + x);
    return l > 0 && (int32_t)ld_l2((const uint32_t*)Pp + x) + l > start;
  });
  if (i0 < 0) return 0;
  const bool rem = type == MTE_OP_REMOVE;
  const uint32_t apsi = (uint32_t)op[6];
  const mte_propset aps = rem ? mte_propset{0u, 0u} : a.ps[apsi];
  const uint32_t slot = (uint32_t)op[7];
  const int l = lane_id();
  int32_t ocy = evd ? own_prefix(h.pl, h.sd, i0) : 0;  // the own view's prefix after the op (events)
  int64_t last_ev = -2;
  uint32_t cnt_all = 0;
  int bc = -1, bec = -2;
  bool done = false;
  for (int tb = i0; tb < h.n && !done; tb += kHT) {
    const int te = tb + kHT < h.n ? tb + kHT : h.n;
    ht_ensure(h, te - 1);
    bool in[kHE];
    uint32_t tt[kHE];
    int32_t rs[kHE], ln[kHE];
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const bool v = i < te;
      const int ic = v ? i : tb;
      const int32_t Lv = (int32_t)ld_l2((const uint32_t*)Lp + ic), Pv = (int32_t)ld_l2((const uint32_t*)Pp + ic);
      tt[j] = ld_l2(h.tw + ic);
      rs[j] = (int32_t)ld_l2(h.pl + 2 * h.sd + ic);
      ln[j] = (int32_t)ld_l2(h.pl + ic);
      in[j] = v && Lv > 0 && Pv < end;
      if (__ballot(v && Lv > 0 && Pv >= end)) done = true;  // nodeMap stops at pos >= end
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < kHE; j++) cnt += (uint32_t)__popcll(__ballot(in[j]));
    // ---- delta events: per segment, at its own-view position after the op ----
    if (evd) {
#pragma unroll
      for (int j = 0; j < kHE; j++) {
        const int i = tb + j * kWave + l;
        const bool e = in[j] && (!rem || rs[j] == kNone);
        const int32_t ol = (i < te && rs[j] == kNone && !(rem && in[j])) ? ln[j] : 0;
        const int32_t oincl = wave_incl_scan(ol);
        // an item that continues the leaf of the item just before, both
        // reported: one segment, one record
        const uint64_t em = __ballot(e);
        const bool eprev = l > 0 ? ((em >> (l - 1)) & 1ull) != 0 : last_ev == (int64_t)i - 1;
        const bool ext = e && (tt[j] & kTCont) && eprev;
        const bool st0 = e && !ext;
        const int32_t sincl = wave_incl_scan(st0 ? 1 : 0);
        const uint32_t base = ev.n;
        if (st0) {
          const uint32_t idx = base + (uint32_t)(sincl - 1);
          if (idx < ev.cap)
            ev.p[idx] = mte_delta{ev.op, type, ocy + oincl - ol, ln[j], (rem || rs[j] != kNone) ? 1u : 0u};
        }
        vm_drain();
        if (ext) {  // the record of the last start at or before it (sincl == 0: an earlier row's)
          const uint32_t idx = base + (uint32_t)sincl - 1u;
          if (idx < ev.cap) atomicAdd((int*)&ev.p[idx].len, ln[j]);
        }
        ev.n += (uint32_t)rdlane(sincl, kWave - 1);
        ocy += rdlane(oincl, kWave - 1);
        if (em) last_ev = tb + j * kWave + (63 - __clzll((long long)em));
      }
      vm_drain();
    }
    if (cnt == 0) continue;
    cnt_all += cnt;
    // ---- the marks ----
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      if (!in[j]) continue;
      if (rem) {
        if (local) {
          h.pl[2 * h.sd + i] = (uint32_t)(kLocalBase + s);
          h.pl[3 * h.sd + i] = 1u;
          h.pl[(uint64_t)kLrsPlane<K> * h.sd + i] = (uint32_t)s;
          h.pl[(uint64_t)kGrpPlane<K> * h.sd + i] = (uint32_t)i;
        } else {
          // removers: plane 3 for short ids < 32, the last plane (kRmHiPlane) for the rest
          uint32_t* rmp = h.pl + (uint64_t)(c < 32 ? 3 : h.nP - 1) * h.sd + i;
          const uint32_t rm = ld_l2(rmp);
          if (rs[j] == kNone) {
            h.pl[2 * h.sd + i] = (uint32_t)s;
            *rmp = 1u << (c & 31);  // the other half is zero while the item is not removed
          } else {
            if (rs[j] >= kLocalBase) h.pl[2 * h.sd + i] = (uint32_t)s;  // overtaking our pending removal (:1928-1938)
            *rmp = rm | (1u << (c & 31));
          }
        }
      } else {
        h.tw[i] = tt[j] | kTPo;
        if (K > 0) {
          if (!local && !h.ldoc && (flags & MTE_F_REWRITE))
            for (int k = 0; k < K; k++) h.pl[(uint64_t)(kFieldPlanes + k) * h.sd + i] = 0u;
          if (!local && h.ldoc && (flags & MTE_F_REWRITE))
            for (int k = 0; k < K; k++)
              if (ld_l2(h.pl + (uint64_t)(kPkPlane<K> + k) * h.sd + i) == 0u)
                h.pl[(uint64_t)(kFieldPlanes + k) * h.sd + i] = 0u;
          for (uint32_t t = 0; t < aps.count; t++) {
            const mte_prop p = a.pe[aps.first + t];
            if (p.key >= a.n_keys || p.key >= (uint32_t)K) continue;
            uint32_t* vp = h.pl + (uint64_t)(kFieldPlanes + p.key) * h.sd + i;
            if (flags & MTE_F_COMBINE) {
              // combine(op, current, undefined, seq): the host's map of every value
              // the key can hold; pending keys are no exception (shouldModifyKey)
              const uint32_t old = ld_l2(vp);
              uint32_t nv = old;
              for (uint32_t u = 1; u <= p.value; u++) {
                const mte_prop q = a.pe[aps.first + t + u];
                if ((q.key & ~MTE_COMBINE_PAIR) == old) {
                  nv = q.value;
                  break;
                }
              }
              if (local) {  // a local incr / consensus: the key pending as for any local annotate
                uint32_t* pk = h.pl + (uint64_t)(kPkPlane<K> + p.key) * h.sd + i;
                if (ld_l2(pk) == 0u) h.pl[(uint64_t)(kAnnPlane<K> + 1 + p.key) * h.sd + i] = old;
                *pk = (uint32_t)s;
              }
              *vp = nv;
            } else if (local) {
              // the value before the first pending annotate of the key, then pending
              uint32_t* pk = h.pl + (uint64_t)(kPkPlane<K> + p.key) * h.sd + i;
              if (ld_l2(pk) == 0u) h.pl[(uint64_t)(kAnnPlane<K> + 1 + p.key) * h.sd + i] = ld_l2(vp);
              *vp = p.value;
              *pk = (uint32_t)s;
            } else if (h.ldoc) {
              // shouldModifyKey: a key with a pending local update keeps its value
              if (ld_l2(h.pl + (uint64_t)(kPkPlane<K> + p.key) * h.sd + i) == 0u) *vp = p.value;
            } else {
              *vp = p.value;
            }
          }
        }
        if (local && slot < MTE_ANNOTATE_SLOTS) {
          uint32_t* am = h.pl + (uint64_t)kAnnPlane<K> * h.sd + i;
          *am = ld_l2(am) | (1u << slot);  // the annotate's segment group (:1874-1880)
        }
      }
    }
    vm_drain();
    // ---- a sequenced op adds each visited segment to the LRU set, in order (:1881-1884, 1955-1958) ----
    if (!local) {
#pragma unroll
      for (int j = 0; j < kHE; j++) {
        uint64_t m = __ballot(in[j] && !(tt[j] & kTCont));
        while (m) {
          const int i = tb + j * kWave + (__ffsll((long long)m) - 1);
          m &= m - 1;
          if ((rc = ht_add_lru(h, i, s, bc, bec))) return rc;
        }
      }
    }
  }
  MTE_STAT(st[kStWritten] += cnt_all;)
  if (!rem) {
    uint32_t w = 0;
    for (uint32_t t = 0; t < aps.count; t++) w += a.pe[aps.first + t].key < a.n_keys ? 1u : 0u;
    MTE_STAT(st[kStPwrites] += cnt_all * w;)
  }
  h.lp_n = 0;  // the marks changed lengths
  if (rem && !local && rt && rhi) {
    const uint32_t* lrp = h.pl + (uint64_t)kLrsPlane<K> * h.sd;
    stream_slide(h.pl, h.sd, h.n, rt, rhi, s, evs ? &ev : nullptr, kSlideOverlap, lrp, h.tw);
    stream_slide(h.pl, h.sd, h.n, rt, rhi, s, evs ? &ev : nullptr, kSlideNew, lrp, h.tw);
  }
  return 0;
}

// ---- local records (titems.c doc_ack, doc_rollback, doc_rollback_annotate, doc_regen) ----------

// createLocalReferencePosition of a Transient reference (titems.c doc_ref):
// getContainingSegment(pos) in the local view -- the leaf holding pos and the
// offset in it -- kept as (leaf id, offset), never moved (kRefTrans)
template <int K>
__device__ __forceinline__ int ht_ref_transient(HT& h, uint2* rt, uint32_t& rhi, const s8v& op) {
  const uint32_t slot = (uint32_t)op[5], typ = (uint32_t)op[6];
  const int32_t pos = op[4];
  if (typ & (MTE_REF_SLIDE_ON_REMOVE | MTE_REF_STAY_ON_REMOVE)) return MTE_E_INVALID_ARG;
  ht_persp(h, true, 0, 0);  // the local view
  const int32_t* Lp = h.L;
  const int32_t* Pp = h.P;
  const int x = ht_first_lp(h, 0, [&](int i) {
    const int32_t l = (int32_t)ld_l2((const uint32_t*)Lp + i);
    const int32_t p = (int32_t)ld_l2((const uint32_t*)Pp + i);
    return l > 0 && pos >= p && pos < p + l;
  });
  if (x < 0) return MTE_E_INVALID_ARG;  // no segment holds pos in the local view
  const int hd = ht_leaf_start(h, x);
  const int32_t off = pos - own_prefix(h.pl, h.sd, hd);
  if (off < 0 || (uint32_t)off > kRefTransOff) return MTE_E_UNSUPPORTED;
  lane0_st(&rt[slot].x, t_id(ht_T(h, hd)));
  lane0_st(&rt[slot].y, kRefLive | kRefDetached | kRefTrans | (uint32_t)off);
  vm_drain();
  if (slot + 1 > rhi) rhi = slot + 1;
  return 0;
}

// an item the ack of ls still has to take: inserted, removed or annotated by
// ls (am_mask: ls's annotate slot), or a removal of ls a remote one overtook
// (titems.c ack_pending)
template <int K>
__device__ __forceinline__ bool ht_ack_pending(const HT& h, int i, int32_t ls, uint32_t am_mask) {
  if (ld_l2(h.tw + i) & kTEmpty) return false;
  return (int32_t)ld_l2(h.pl + h.sd + i) == kLocalBase + ls || (int32_t)ld_l2(h.pl + 2 * h.sd + i) == kLocalBase + ls ||
         (int32_t)ld_l2(h.pl + (uint64_t)kLrsPlane<K> * h.sd + i) == ls ||
         (ld_l2(h.pl + (uint64_t)kAnnPlane<K> * h.sd + i) & am_mask) != 0u;
}

// the group's next tail split off after ls (a member flagged in L whose born >
// ls), by id from `last` on: (its index or -1, its id)
__device__ __forceinline__ uint2 ht_next_tail(const uint32_t* Lf, const uint32_t* bnp, const uint32_t* tw,
                                                        int n, uint32_t ls, uint32_t last) {
  const int l = lane_id();
  uint32_t best = 0xffffffffu;
  for (int tb = 0; tb < n; tb += kWave) {
    const int i = tb + l;
    if (i < n && ld_l2(Lf + i) == 1u && ld_l2(bnp + i) > ls) {
      const uint32_t id = t_id(ld_l2(tw + i));
      if (id >= last && id < best) best = id;
    }
  }
  best = uni(wave_min_u32(best));
  if (best == 0xffffffffu) return make_uint2(0xffffffffu, 0u);
  const int i = ht_first(0, n, [&](int x) { return ld_l2(Lf + x) == 1u && ld_l2(bnp + x) > ls && t_id(ld_l2(tw + x)) == best; });
  return make_uint2((uint32_t)i, best);
}

// ackPendingSegment (mergeTree.ts:1278-1331, mergeTreeNodes.ts:475-503) for one
// segment group of ls (titems.c ack_group): the items of regeneration group
// `key` (keyed) or every item of ls get the seq, each segment is added to the
// LRU set in the group's order -- the segments the op marked in document
// order, then the tails split off since, as they were made -- the references
// of the acked removals slide, the ACKNOWLEDGED record reports the group, then
// zamboniSegments runs.  The group's segments are flagged in the L scratch.
template <int K>
__device__ __forceinline__ int ht_ack_group(HT& h, int32_t ls, int32_t s, uint32_t am_mask, uint32_t stamp, bool keyed,
                                            uint32_t key, const ReplayArgs& a, uint2* rt, uint32_t rhi, EvOut& ev,
                                            bool evs) {
  const int l = lane_id();
  int rc;
  int bc = -1, bec = -2;
  uint32_t tails = 0;
  const uint32_t* rgp = h.pl + (uint64_t)kRgPlane<K> * h.sd;
  const uint32_t* bnp = h.pl + (uint64_t)kBornPlane<K> * h.sd;
  for (int tb = 0; tb < h.n; tb += kHT) {
    bool member[kHE], orig[kHE];
    uint32_t tt[kHE];
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const bool v = i < h.n;
      const int ic = v ? i : 0;
      tt[j] = ld_l2(h.tw + ic);
      const int32_t sq = (int32_t)ld_l2(h.pl + h.sd + ic), rs = (int32_t)ld_l2(h.pl + 2 * h.sd + ic);
      const int32_t lr = (int32_t)ld_l2(h.pl + (uint64_t)kLrsPlane<K> * h.sd + ic);
      const uint32_t am = ld_l2(h.pl + (uint64_t)kAnnPlane<K> * h.sd + ic);
      const uint32_t rg = ld_l2(rgp + ic);
      orig[j] = ld_l2(bnp + ic) <= (uint32_t)ls;
      member[j] = false;
      if (v) h.L[i] = 0;
      if (!v || (tt[j] & kTEmpty) || (keyed && rg != key)) continue;
      if (sq == kLocalBase + ls) {
        h.pl[h.sd + i] = (uint32_t)s;
        member[j] = true;
      }
      if (lr == ls) {  // acked, or overtaken by a remote remove before (:1928-1938)
        h.pl[(uint64_t)kLrsPlane<K> * h.sd + i] = 0u;
        member[j] = true;
      }
      if (rs == kLocalBase + ls) {
        h.pl[2 * h.sd + i] = (uint32_t)s;
        // the group's removals hold ls until they have slid (stream_slide's
        // group mark; a regenerated one's localRemovedSeq is its old op's)
        // (acked: localRemovedSeq undefined, mergeTreeNodes.ts:493)
        h.pl[(uint64_t)kLrsPlane<K> * h.sd + i] = (rt && rhi) ? (uint32_t)ls : 0u;
      }
      if (am & am_mask) {
        h.pl[(uint64_t)kAnnPlane<K> * h.sd + i] = am & ~am_mask;
        member[j] = true;
        // updateConsensusProperty (client.ts:646-650, 1083-1090): a local
        // consensus's ack stamps its marker's value with the seq, outside the
        // pending-key rules (titems.c ack_group)
        if (K > 0 && stamp != MTE_NO_PROPS) {
          const mte_propset sp = a.ps[stamp];
          for (uint32_t t = 0; t < sp.count; t++) {
            const mte_prop hd = a.pe[sp.first + t];
            if ((hd.key & MTE_COMBINE_PAIR) || hd.key >= a.n_keys || hd.key >= (uint32_t)K) continue;
            uint32_t* vp = h.pl + (uint64_t)(kFieldPlanes + hd.key) * h.sd + i;
            const uint32_t old = ld_l2(vp);
            for (uint32_t u = 1; u <= hd.value; u++) {
              const mte_prop q = a.pe[sp.first + t + u];
              if ((q.key & ~MTE_COMBINE_PAIR) == old) {
                *vp = q.value;
                break;
              }
            }
          }
        }
      }
    }
    vm_drain();
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const bool mem = member[j] && !(tt[j] & kTCont);
      if (mem) h.L[tb + j * kWave + l] = 1;
      tails += (uint32_t)__popcll(__ballot(mem && !orig[j]));
      uint64_t m = __ballot(mem && orig[j]);
      while (m) {
        const int i = tb + j * kWave + (__ffsll((long long)m) - 1);
        m &= m - 1;
        if ((rc = ht_add_lru(h, i, s, bc, bec))) return rc;
      }
    }
  }
  vm_drain();
  const int32_t* Lf = h.L;
  for (uint32_t last = 0; tails; tails--) {
    const uint2 nx = ht_next_tail((const uint32_t*)Lf, bnp, h.tw, h.n, (uint32_t)ls, last);
    if ((int)nx.x < 0) break;
    if ((rc = ht_add_lru(h, (int)nx.x, s, bc, bec))) return rc;
    last = nx.y + 1u;
  }
  if (rt && rhi) {
    // the group slides in its order, the later groups still pending
    // (ackPendingSegment per group op, mergeTree.ts:1278-1304)
    uint32_t* lrp = h.pl + (uint64_t)kLrsPlane<K> * h.sd;
    stream_slide(h.pl, h.sd, h.n, rt, rhi, s, evs ? &ev : nullptr, kSlideAck, h.pl + (uint64_t)kGrpPlane<K> * h.sd,
                 h.tw, lrp, (uint32_t)ls);
    for (int tb = 0; tb < h.n; tb += kWave) {
      const int i = tb + l;
      if (i < h.n && (int32_t)ld_l2(lrp + i) == ls && (!keyed || ld_l2(rgp + i) == key)) lrp[i] = 0u;
    }
    vm_drain();
  }
  if (h.maint) {
    // ACKNOWLEDGED (mergeTree.ts:1313-1320): the group's segments in document
    // order, after their slides (titems.c ack_group)
    uint32_t idx = 0;
    for (int i = ht_first(0, h.n, [&](int x) { return ld_l2((const uint32_t*)Lf + x) == 1u; }); i >= 0;
         i = ht_first(i + 1, h.n, [&](int x) { return ld_l2((const uint32_t*)Lf + x) == 1u; }))
      ht_maint(h, ev, MTE_MAINT_ACK, (int32_t)t_id(ht_T(h, i)), ht_sum_len(h, i, ht_leaf_end(h, i)), idx++);
  }
  h.lp_n = 0;  // the L scratch held the flags
  return ht_zamboni<K>(h, a.n_keys, ev);
}

// MTE_OP_ACK for localSeqs pos1..pos2 (titems.c doc_ack): per localSeq,
// ackPendingSegment acks its group; a regenerated message (MTE_F_REGENERATED)
// acks each re-sent segment of it as a group of its own, in document order
// (resetPendingDeltaToOps, client.ts:802-857)
template <int K>
__device__ __forceinline__ int ht_ack(HT& h, const s8v& op, const ReplayArgs& a, uint2* rt, uint32_t rhi, EvOut& ev,
                                      bool evs) {
  const int32_t lo = op[4], hi = op[5], s = op[0];
  const uint32_t mask = (uint32_t)op[6];
  const uint32_t oflags = ((uint32_t)op[3]) >> 16;
  const bool regen = (oflags & MTE_F_REGENERATED) != 0u;
  const int l = lane_id();
  int rc;
  for (int32_t ls = lo; ls <= hi; ls++) {
    const uint32_t am_mask = ls == hi ? mask : 0u;
    // the stamp of a local consensus (MTE_F_COMBINE: b = its propset), with the last localSeq's group
    const uint32_t stamp = (ls == hi && (oflags & MTE_F_COMBINE)) ? (uint32_t)op[7] : MTE_NO_PROPS;
    // the pending property keys of ls stop blocking remote annotates
    for (int tb = 0; tb < h.n; tb += kWave) {
      const int i = tb + l;
      if (i < h.n) {
#pragma unroll
        for (int k = 0; k < K; k++) {
          uint32_t* pk = h.pl + (uint64_t)(kPkPlane<K> + k) * h.sd + i;
          const uint32_t v = ld_l2(pk);
          if (v != 0u && v <= (uint32_t)ls) *pk = 0u;
        }
      }
    }
    vm_drain();
    // one group, or (regenerated) one per re-sent segment; one call site keeps
    // the inlined group body single
    for (;;) {
      uint32_t key = 0u;
      if (regen) {
        const int f = ht_first(0, h.n, [&](int x) { return ht_ack_pending<K>(h, x, ls, am_mask); });
        if (f < 0) break;
        key = uld(h.pl + (uint64_t)kRgPlane<K> * h.sd + f);
      }
      if ((rc = ht_ack_group<K>(h, ls, s, am_mask, stamp, regen, key, a, rt, rhi, ev, evs))) return rc;
      if (!regen) break;
    }
  }
  return 0;
}

// the first item of a pending group from `from` on: an insert group by its
// seq, a remove group by its removedSeq, an annotate group by its slot bit
template <int K>
__device__ __forceinline__ int ht_member(const HT& h, int from, uint32_t t, int32_t ls, uint32_t slot) {
  const uint32_t* pl = h.pl;
  const uint64_t sd = h.sd;
  const uint32_t* tw = h.tw;
  return ht_first(from, h.n, [&](int x) {
    if (ld_l2(tw + x) & kTEmpty) return false;
    if (t == MTE_OP_INSERT) return (int32_t)ld_l2(pl + sd + x) == kLocalBase + ls;
    if (t == MTE_OP_REMOVE) return (int32_t)ld_l2(pl + 2 * sd + x) == kLocalBase + ls;
    return ((ld_l2(pl + (uint64_t)kAnnPlane<K> * sd + x) >> slot) & 1u) != 0u;
  });
}

// MTE_OP_ROLLBACK (MergeTree.rollback, mergeTree.ts:2005-2083): an insert's
// segments become seq / removedSeq UniversalSequenceNumber through
// markRangeRemoved at seq 0, each followed by zamboniSegments; a remove's are
// restored
template <int K>
__device__ __forceinline__ int ht_rollback(HT& h, const s8v& op, const ReplayArgs& a, bool evd, EvOut& ev) {
  const int32_t ls = op[0];
  const uint32_t t = (uint32_t)op[4];
  int rc;
  if (t == MTE_OP_INSERT) {
    for (int i = ht_member<K>(h, 0, t, ls, 0); i >= 0; i = ht_member<K>(h, 0, t, ls, 0)) {
      const int32_t len = (int32_t)ht_pl(h, 0, i);
      const int32_t lp = evd ? own_prefix(h.pl, h.sd, i) : 0;
      ht_setpl(h, 1, i, 0u);
      ht_setpl(h, 2, i, 0u);
      ht_setpl(h, 3, i, 1u);
      ht_setpl(h, kRmHiPlane<K>, i, 0u);
      vm_drain();
      if (evd) ev_one(ev, MTE_OP_REMOVE, lp, len);
      if ((rc = ht_zamboni<K>(h, a.n_keys, ev))) return rc;
    }
    return 0;
  }
  for (int i = ht_member<K>(h, 0, t, ls, 0); i >= 0; i = ht_member<K>(h, i + 1, t, ls, 0)) {
    ht_setpl(h, 2, i, (uint32_t)kNone);
    ht_setpl(h, 3, i, 0u);
    ht_setpl(h, kRmHiPlane<K>, i, 0u);
    ht_setpl(h, kLrsPlane<K>, i, 0u);
    vm_drain();
    if (evd) ev_one(ev, MTE_OP_INSERT, own_prefix(h.pl, h.sd, i), (int32_t)ht_pl(h, 0, i));
  }
  return 0;
}

// MTE_OP_ROLLBACK of an annotate (group slot b) with its MTE_OP_RBKEY records at
// aux (titems.c doc_rollback_annotate): each segment of the group re-annotated
// by annotateRange at seq 0, which runs zamboniSegments after it
template <int K>
__device__ __forceinline__ int ht_rollback_annotate(HT& h, uint32_t b, const uint4* aux, uint32_t n_aux, const ReplayArgs& a,
                                    bool evd, EvOut& ev) {
  int rc;
  for (int i = ht_member<K>(h, 0, MTE_OP_ANNOTATE, 0, b); i >= 0; i = ht_member<K>(h, 0, MTE_OP_ANNOTATE, 0, b)) {
    if ((int32_t)ht_pl(h, 2, i) != kNone) return MTE_E_UNSUPPORTED;
    const int e = ht_leaf_end(h, i);
    const uint32_t am = ht_pl(h, kAnnPlane<K>, i);
    for (uint32_t q = 0; q < n_aux;) {
      const uint32_t key = uni((uint32_t)sload8(aux + 2 * q)[4]);
      if (key >= (uint32_t)K) return MTE_E_INVALID_ARG;
      bool found = false;
      uint32_t val = 0u, pk = 0u;
      for (;;) {  // the key's candidates, latest first, then its base entry
        if (q >= n_aux) return MTE_E_INVALID_ARG;
        const s8v rr = sload8(aux + 2 * q);
        q++;
        if ((uint32_t)rr[4] != key) return MTE_E_INVALID_ARG;
        const uint32_t sl = (uint32_t)rr[5];
        if (sl >= MTE_ANNOTATE_SLOTS) break;
        if (!found && ((am >> sl) & 1u)) {
          found = true;
          val = (uint32_t)rr[6];
          pk = (uint32_t)rr[0];
        }
      }
      for (int x = i; x < e; x++) {
        const uint32_t v = found ? val : ht_pl(h, kAnnPlane<K> + 1 + (int)key, x);
        ht_setpl(h, kFieldPlanes + (int)key, x, v);
        ht_setpl(h, kPkPlane<K> + (int)key, x, pk);
      }
      vm_drain();
    }
    int32_t tl = 0;
    for (int x = i; x < e; x++) {
      ht_setpl(h, kAnnPlane<K>, x, ht_pl(h, kAnnPlane<K>, x) & ~(1u << b));
      tl += (int32_t)ht_pl(h, 0, x);
    }
    vm_drain();
    if (evd) ev_one(ev, MTE_OP_ANNOTATE, own_prefix(h.pl, h.sd, i), tl);
    if ((rc = ht_zamboni<K>(h, a.n_keys, ev))) return rc;
  }
  return 0;
}

// ---- LDS residency -------------------------------------------------------------------------
// A document's state is moved whole: rows [0, n) of its nP planes and tree
// words, and heap entries 1 .. hn.  L / P are scratch (recomputed lazily).
// Items a record may add at most (splits, a new leaf, placeholders): the
// document leaves LDS before a record that could pass its LDS capacity.
constexpr int kLdsMargin = 16;

__device__ __forceinline__ void ht_move(uint32_t* dpl, uint64_t dsd, uint32_t* dtw, uint32_t* dhp, const uint32_t* spl, uint64_t ssd,
                        const uint32_t* stw, const uint32_t* shp, int nP, int n, uint32_t hn) {
  const int l = lane_id();
  // tiles of kHT items, kHtGroup planes' loads in flight before their stores
  for (int tb = 0; tb < n; tb += kHT) {
    for (int p0 = 0; p0 <= nP; p0 += kHtGroup) {
      uint32_t v[kHtGroup][kHE];
#pragma unroll
      for (int q = 0; q < kHtGroup; q++) {
        const int p = p0 + q <= nP ? p0 + q : nP;
        const uint32_t* sp = p < nP ? spl + (uint64_t)p * ssd : stw;
#pragma unroll
        for (int j = 0; j < kHE; j++) {
          const int i = tb + j * kWave + l;
          v[q][j] = ld_l2(sp + (i < n ? i : 0));
        }
      }
#pragma unroll
      for (int q = 0; q < kHtGroup; q++) {
        if (p0 + q > nP) break;
        const int p = p0 + q;
        uint32_t* dp = p < nP ? dpl + (uint64_t)p * dsd : dtw;
#pragma unroll
        for (int j = 0; j < kHE; j++) {
          const int i = tb + j * kWave + l;
          if (i < n) dp[i] = v[q][j];
        }
      }
    }
  }
  for (uint32_t k = 1 + (uint32_t)l; k <= hn; k += kWave) {
    dhp[2 * k] = ld_l2(shp + 2 * k);
    dhp[2 * k + 1] = ld_l2(shp + 2 * k + 1);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// into the workgroup's LDS (lds: (nP + 5) x lcap + 2 words)
__device__ __forceinline__ void ht_to_lds(HT& h, uint32_t* lds, uint32_t lcap) {
  h.g_pl = h.pl;
  h.g_sd = h.sd;
  h.g_tw = h.tw;
  h.g_L = h.L;
  h.g_P = h.P;
  h.g_hp = h.hp;
  h.g_hcap = h.hcap;
  h.g_cap = h.cap;
  uint32_t* pl = lds;
  uint32_t* tw = pl + (uint64_t)h.nP * lcap;
  int32_t* L = reinterpret_cast<int32_t*>(tw + lcap);
  int32_t* P = L + lcap;
  uint32_t* hp = reinterpret_cast<uint32_t*>(P + lcap);
  ht_move(pl, lcap, tw, hp, h.pl, h.sd, h.tw, h.hp, h.nP, h.n, h.hn);
  h.pl = pl;
  h.sd = lcap;
  h.tw = tw;
  h.L = L;
  h.P = P;
  h.hp = hp;
  h.hcap = lcap;
  h.cap = (int)lcap;
  h.lds = true;
  h.lp_n = 0;
  h.lp_carry = 0;
}

// back to HBM (before a record that could outgrow LDS, and at the end)
__device__ __forceinline__ void ht_spill(HT& h) {
  ht_move(h.g_pl, h.g_sd, h.g_tw, h.g_hp, h.pl, h.sd, h.tw, h.hp, h.nP, h.n, h.hn);
  h.pl = h.g_pl;
  h.sd = h.g_sd;
  h.tw = h.g_tw;
  h.L = h.g_L;
  h.P = h.g_P;
  h.hp = h.g_hp;
  h.hcap = h.g_hcap;
  h.cap = h.g_cap;
  h.lds = false;
  h.lp_n = 0;
  h.lp_carry = 0;
}

__device__ __forceinline__ bool ht_lds_room(const HT& h) {
  return h.n + kLdsMargin <= h.cap && (int)h.hn + h.n + kLdsMargin <= (int)h.hcap;
}

// ---- one record (titems.c doc_apply / doc_apply_local) ----------------------------------

// MTE_OP_RELPOS (include/mte.h): the position of the first marker whose key
// plane `key` holds `vid` in the view of the record it serves (getPosition,
// mergeTree.ts:853-870, the lengths before it; posFromRelativePos :1369-1392),
// -1 when no held marker carries the id
template <int K>
__device__ __forceinline__ int32_t ht_marker_pos(HT& h, uint32_t key, uint32_t vid, bool local, int32_t r, int c) {
  if (key >= (uint32_t)K || vid == 0u) return -1;
  const uint32_t* kp = h.pl + (uint64_t)(kFieldPlanes + key) * h.sd;
  const uint32_t* mp = h.pl + 4 * h.sd;
  const uint32_t* tw = h.tw;
  const int x = ht_first(0, h.n, [&](int i) {
    return (ld_l2(mp + i) >> 8) != 0u && ld_l2(kp + i) == vid && !(ld_l2(tw + i) & kTEmpty);
  });
  if (x < 0) return -1;
  ht_persp(h, local, r, c);
  ht_ensure(h, x);
  return (int32_t)uld((const uint32_t*)h.P + x);
}

// ---- reconnection of pending interval ops (MTE_OP_REF b = 4 / 5) --------------------------
// The local client's view at refSeq rs0 and localSeq ls (localNetLength with a
// localSeq, mergeTree.ts:575-593): acked text up to rs0 less acked removals up
// to rs0, own pending inserts up to ls, less own removals up to ls.
template <int K>
__device__ __forceinline__ int32_t ht_view_len(const HT& h, int i, int32_t rs0, int32_t ls) {
  const uint32_t tt = ld_l2(h.tw + i);
  const int32_t len = (int32_t)ld_l2(h.pl + i), sq = (int32_t)ld_l2(h.pl + h.sd + i);
  const int32_t rs = (int32_t)ld_l2(h.pl + 2 * h.sd + i);
  const int32_t lr = (int32_t)ld_l2(h.pl + (uint64_t)kLrsPlane<K> * h.sd + i);
  if (tt & kTEmpty) return 0;
  if (lr != 0 && (lr & ~(int32_t)kLrsReleased) <= ls) return 0;
  if (sq >= kLocalBase && sq != kNone) return sq - kLocalBase > ls ? 0 : len;
  if (sq > rs0) return 0;
  if (rs != kNone && rs >= kLocalBase) return rs - kLocalBase <= ls ? 0 : len;
  return (rs != kNone && rs <= rs0) ? 0 : len;
}

// The reference takes a block's length in these views from its local partial
// lengths (titems.c item_partial / block_len, which cite the rules): per item
// a sequenced part, a local part counted only when the block holds a local
// record at or below localSeq, less the overlapping removes; W the window of
// the cached partials (ht_view_window).
template <int K>
__device__ __forceinline__ void ht_item_partial(const HT& h, int i, int32_t R, int32_t L, int32_t W, int32_t& a, int32_t& b,
                                                int32_t& o, bool& fl) {
  const uint32_t tt = ld_l2(h.tw + i);
  const int32_t c = (int32_t)ld_l2(h.pl + i), sq = (int32_t)ld_l2(h.pl + h.sd + i);
  const int32_t rs = (int32_t)ld_l2(h.pl + 2 * h.sd + i);
  const uint32_t rm = ld_l2(h.pl + 3 * h.sd + i), rmh = ld_l2(h.pl + (uint64_t)kRmHiPlane<K> * h.sd + i);
  const int32_t lr = (int32_t)(ld_l2(h.pl + (uint64_t)kLrsPlane<K> * h.sd + i) & ~kLrsReleased);
  if (tt & kTEmpty) return;
  if (sq < kLocalBase) {
    if (sq <= W || sq <= R) a += c;
  } else if (sq - kLocalBase <= L) {
    b += c;
    fl = true;
  }
  if (rs == kNone) return;
  if (rs >= kLocalBase) {
    if (rs - kLocalBase <= L) {
      b -= c;
      fl = true;
    }
    return;
  }
  if (rs <= W) {
    a -= c;
    return;
  }
  if (rs <= R) a -= c;
  if (__popc(rm) + __popc(rmh) > 1 && lr != 0 && lr <= L) {
    b -= c;
    fl = true;
    if (rs <= R) o -= c;
  }
}

// the window of the reference's cached local partials: the first block length
// a query evaluates since the last length update computes them, with that
// query's refSeq (nodeLength :984-995 -> computeLocalPartials :964-982)
__device__ __forceinline__ int32_t ht_view_window(HT& h, int32_t R) {
  if (h.wcache < 0) h.wcache = h.min_seq < R ? h.min_seq : R;
  return h.wcache;
}

template <int K>
__device__ __forceinline__ int32_t ht_block_len(HT& h, int s, int e, int32_t R, int32_t L) {
  const int32_t W = ht_view_window(h, R);
  int32_t a = 0, b = 0, o = 0;
  bool fl = false;
  for (int tb = s; tb <= e; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + lane_id();
      if (i <= e) ht_item_partial<K>(h, i, R, L, W, a, b, o, fl);
    }
  }
  a = rdlane(wave_incl_scan(a), kWave - 1);
  b = rdlane(wave_incl_scan(b), kWave - 1);
  o = rdlane(wave_incl_scan(o), kWave - 1);
  return a + (__ballot(fl) ? b - o : 0);
}

// the leaf-rule length of items [s, e]
template <int K>
__device__ __forceinline__ int32_t ht_range_view(const HT& h, int s, int e, int32_t R, int32_t L) {
  int32_t acc = 0;
  for (int tb = s; tb <= e; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + lane_id();
      const int32_t v = ht_view_len<K>(h, i <= e ? i : s, R, L);
      acc += i <= e ? v : 0;
    }
  }
  return rdlane(wave_incl_scan(acc), kWave - 1);
}

// the last item of the child of a level-k block (ending at e) that starts at c
__device__ __forceinline__ int ht_child_last(const HT& h, int c, int e, int k) {
  if (k == 1) return ht_leaf_end(h, c) - 1;
  const uint32_t* tw = h.tw;
  const int j = ht_first(c + 1, e + 1, [&](int x) { return (int)t_h(ld_l2(tw + x)) >= k - 1; });
  return j < 0 ? e : j - 1;
}

template <int K>
__device__ __forceinline__ int32_t ht_child_len(HT& h, int c, int ce, int k, int32_t R, int32_t L) {
  return k > 1 ? ht_block_len<K>(h, c, ce, R, L) : ht_range_view<K>(h, c, ce, R, L);
}


// getPosition of the leaf starting at item x (mergeTree.ts:853-870): the
// lengths of the children before it at every level
template <int K>
__device__ __forceinline__ int32_t ht_view_prefix(HT& h, int x, int32_t R, int32_t L) {
  const int s1 = ht_span_start(h, x, 1);
  int32_t pos = s1 < x ? ht_range_view<K>(h, s1, x - 1, R, L) : 0;
  for (int k = 2; k <= h.depth; k++) {
    const int s = ht_span_start(h, x, k), cx = ht_span_start(h, x, k - 1), e = ht_span_end(h, s, k);
    for (int c = s; c < cx;) {
      const int ce = ht_child_last(h, c, e, k);
      pos += ht_block_len<K>(h, c, ce, R, L);
      c = ce + 1;
    }
  }
  return pos;
}

// getContainingSegment(pos) in the view (mergeTree.ts:872-885 -> nodeMap
// :2274-2330, depth first from the root's children): a zero length skips a
// child, a negative one moves the running position back.  The item holding pos
// and the offset there; -1 past the end.
template <int K>
__device__ __forceinline__ int ht_view_find(HT& h, int32_t pos, int32_t R, int32_t L, int32_t& off) {
  int k = h.depth, e = h.n - 1, c = 0, found = -1;
  int32_t p = 0;
  while (h.n > 0) {
    if (c > e) {  // this block's children are done: its parent goes on after it
      if (k >= h.depth) break;
      k++;
      e = ht_span_end(h, ht_span_start(h, c - 1, k), k);
      continue;
    }
    if (!is_child_t(uni(ld_l2(h.tw + c)), k)) {  // a continuation or a placeholder
      c++;
      continue;
    }
    if (pos + 1 <= p) break;
    const int ce = ht_child_last(h, c, e, k);
    const int32_t len = ht_child_len<K>(h, c, ce, k, R, L);
    if (len != 0) {
      if (pos >= p + len) {
        p += len;
      } else if (k == 1) {
        found = c;
        off = pos - p;
        break;
      } else {
        k--;
        e = ce;
        continue;
      }
    }
    c = ce + 1;
  }
  if (found < 0) return -1;
  // the offset within the leaf -> the item of the leaf holding it
  const int le = ht_leaf_end(h, found);
  while (found + 1 < le && off >= (int32_t)uni(ld_l2(h.pl + found))) {
    off -= (int32_t)uni(ld_l2(h.pl + found));
    found++;
  }
  return found;
}

// the units of its leaf before item i
__device__ __forceinline__ int32_t ht_leaf_offset(const HT& h, int i) {
  const int s = ht_leaf_start(h, i);
  return s < i ? ht_sum_len(h, s, i) : 0;
}

__device__ __forceinline__ bool ht_removed_acked(const HT& h, int i) {
  const int32_t rs = (int32_t)uni(ld_l2(h.pl + 2 * h.sd + i));
  return !(uni(ld_l2(h.tw + i)) & kTEmpty) && rs != kNone && rs < kLocalBase;
}

// Client.getSlideToSegment (client.ts:1117-1130 -> _getSlideToSegment,
// mergeTree.ts:893-913) from item x, removed and acked: offset 0 of the first
// following item a reference may slide to, else the last unit of the last
// preceding one; false when there is none
__device__ __forceinline__ bool ht_slide_item(const HT& h, int x, int& t, int32_t& off) {
  auto ok = [&](int i) {
    const int32_t sq = (int32_t)ld_l2(h.pl + h.sd + i), rs = (int32_t)ld_l2(h.pl + 2 * h.sd + i);
    return !(ld_l2(h.tw + i) & kTEmpty) && slide_ok(sq, rs);
  };
  t = ht_first(x + 1, h.n, ok);
  off = 0;
  if (t >= 0) return true;
  t = ht_last(0, x, ok);
  if (t < 0) return false;
  off = (int32_t)uni(ld_l2(h.pl + t)) - 1;
  return true;
}

// b = 4: Client.rebasePosition(pos1, ref_seq, a) (client.ts:755-786) as an
// MTE_DELTA_REBASE event: the item holding pos1 in the view at (ref_seq, a),
// else the last item at offset 0; slid if removed and acked; its position in
// the view at (currentSeq, a) (findReconnectionPosition :709-713) plus the
// offset, -1 (DetachedReferencePosition) when it slid off the string.
// b = 5: rebaseLocalInterval's slide of a pending interval end
// (intervalCollection.ts:1782-1799): the reference in slot pos2, live on an
// item removed and acked, moves to what createPositionReference finds, in the
// view at (currentSeq, a), at its slide target's position there; the event's
// position is that position, -1 when it stays.
// MTE_OP_REGEN (titems.c doc_regen): the group's segments in document order at
// their positions in the view at localSeq ls, a merged leaf one record
template <int K>
__device__ __forceinline__ void ht_regen(HT& h, int32_t ls, uint32_t t, uint32_t slot, EvOut& ev) {
  const int l = lane_id();
  bool prev_hit = false;  // the tile's last item was a record's item (a continuation joins it)
  for (int tb = 0; tb < h.n; tb += kHT) {
#pragma unroll
    for (int j = 0; j < kHE; j++) {
      const int i = tb + j * kWave + l;
      const bool v = i < h.n;
      const int ic = v ? i : 0;
      const uint32_t tt = ld_l2(h.tw + ic);
      const int32_t len = (int32_t)ld_l2(h.pl + ic), sq = (int32_t)ld_l2(h.pl + h.sd + ic);
      const int32_t rs = (int32_t)ld_l2(h.pl + 2 * h.sd + ic);
      const int32_t lr = (int32_t)ld_l2(h.pl + (uint64_t)kLrsPlane<K> * h.sd + ic);
      const uint32_t am = ld_l2(h.pl + (uint64_t)kAnnPlane<K> * h.sd + ic);
      const uint32_t tf = ld_l2(h.pl + 5 * h.sd + ic);
      const bool rp = rs >= kLocalBase && rs != kNone;  // a pending local removal
      bool hit = false;
      if (v && !(tt & kTEmpty)) {
        if (t == MTE_OP_INSERT) hit = sq == kLocalBase + ls;
        else if (t == MTE_OP_REMOVE) hit = rs == kLocalBase + ls;
        else hit = ((am >> slot) & 1u) && (rs == kNone || rp);
        // a member that re-sends nothing leaves the group (resetPendingDeltaToOps
        // enqueues only the segments with a new op, client.ts:803-852): the
        // zamboni stops holding it for the group; it keeps its localRemovedSeq
        // (titems.c doc_regen)
        if (!hit && t == MTE_OP_REMOVE && lr == ls)
          h.pl[(uint64_t)kLrsPlane<K> * h.sd + i] = (uint32_t)ls | kLrsReleased;
        // each re-sent segment heads a group of its own, the old group's taken
        // by ordinal (client.ts:802, 852): the ack slides them in document order
        if (hit && t == MTE_OP_REMOVE) h.pl[(uint64_t)kGrpPlane<K> * h.sd + i] = (uint32_t)i;
        // and a segment group of its own (client.ts:851-854), which the
        // tails split off it later join (a continuation: its leaf's, below)
        if (hit && !(tt & kTCont)) h.pl[(uint64_t)kRgPlane<K> * h.sd + i] = 1u + t_id(tt);
        if (!hit && t == MTE_OP_ANNOTATE && ((am >> slot) & 1u))
          h.pl[(uint64_t)kAnnPlane<K> * h.sd + i] = am & ~(1u << slot);
      }
      // a member that leaves has its position taken all the same
      // (resetPendingDeltaToOps :806, before the op is chosen), which may compute
      // the cached local partials (titems.c doc_regen)
      const bool gone = v && !(tt & kTEmpty) && !hit && !(tt & kTCont) &&
                        ((t == MTE_OP_REMOVE && lr == ls) || (t == MTE_OP_ANNOTATE && ((am >> slot) & 1u)));
      uint64_t gm = h.wcache < 0 ? __ballot(gone) : 0ull;
      while (gm && h.wcache < 0) {
        const int ln = __ffsll((long long)gm) - 1;
        gm &= gm - 1;
        (void)ht_view_prefix<K>(h, tb + j * kWave + ln, h.cur_seq, ls);
      }
      // hit(i - 1): the lane before, or the previous row's / tile's last item
      uint64_t cm = __ballot(hit && (tt & kTCont));
      if (cm) {  // a merged leaf's continuations: its head's group
        uint32_t* rgp = h.pl + (uint64_t)kRgPlane<K> * h.sd;
        vm_drain();
        while (cm) {
          const int x = tb + j * kWave + (__ffsll((long long)cm) - 1);
          cm &= cm - 1;
          lane0_st(rgp + x, uld(rgp + x - 1));
          vm_drain();
        }
      }
      const uint64_t hm = __ballot(hit);
      const bool hprev = l > 0 ? ((hm >> (l - 1)) & 1ull) != 0 : prev_hit;
      const bool ext = hit && (tt & kTCont) && hprev;
      const bool st0 = hit && !ext;
      const int32_t sincl = wave_incl_scan(st0 ? 1 : 0);
      const uint32_t base = ev.n;
      if (st0) {
        const uint32_t idx = base + (uint32_t)(sincl - 1);
        if (idx < ev.cap) ev.p[idx] = mte_delta{ev.op, MTE_DELTA_REGEN | t, 0, len, t == MTE_OP_INSERT ? tf : 0u};
      }
      vm_drain();
      if (ext) {
        const uint32_t idx = base + (uint32_t)sincl - 1u;
        if (idx < ev.cap) atomicAdd((int*)&ev.p[idx].len, len);
      }
      // positions: findReconnectionPosition (client.ts:709-713), getPosition with
      // the localSeq, block lengths from the local partials (ht_view_prefix)
      uint64_t sm = __ballot(st0);
      while (sm) {
        const int ln = __ffsll((long long)sm) - 1;
        sm &= sm - 1;
        const int x = tb + j * kWave + ln;
        const int32_t pos = ht_view_prefix<K>(h, ht_leaf_start(h, x), h.cur_seq, ls) + ht_leaf_offset(h, x);
        const uint32_t idx = base + (uint32_t)rdlane(sincl, ln) - 1u;
        if (l == 0 && idx < ev.cap) ev.p[idx].pos = pos;
      }
      vm_drain();
      ev.n += (uint32_t)rdlane(sincl, kWave - 1);
      prev_hit = ((hm >> 63) & 1ull) != 0;
    }
  }
  vm_drain();
}

template <int K>
__device__ __forceinline__ int ht_ref_rebase(HT& h, const s8v& op, int32_t lseq, uint2* rt, EvOut& ev) {
  const uint32_t b = (uint32_t)op[7];
  const int32_t ls = op[6];
  if (ls < 0 || ls > lseq) return MTE_E_INVALID_ARG;
  if (b == 4u) {
    int32_t off = 0;
    int x = ht_view_find<K>(h, op[4], op[1], ls, off);
    if (x < 0) {  // past every segment of the view: the tree's last leaf, offset 0
      x = ht_last(0, h.n, [&](int i) { return !(ld_l2(h.tw + i) & kTEmpty); });
      off = 0;
    }
    int32_t p = -1;
    if (x >= 0) {
      int t = x;
      bool ok = true;
      if (ht_removed_acked(h, x)) ok = ht_slide_item(h, x, t, off);
      if (ok) p = ht_view_prefix<K>(h, ht_leaf_start(h, t), h.cur_seq, ls) + ht_leaf_offset(h, t) + off;
    }
    ev_one(ev, MTE_DELTA_REBASE, p, 0);
    return 0;
  }
  const uint32_t slot = (uint32_t)op[5];
  const uint32_t stt = uni(ld_l2(&rt[slot].y)), anc = uni(ld_l2(&rt[slot].x));
  // a slot not in use answers -1 (titems.c the same); no return between here
  // and the end: an early one tripled the pass's VGPRs (148 against 53, three
  // waves per SIMD instead of seven)
  int32_t p = -1;
  if ((stt & kRefLive) && !(stt & kRefDetached)) {
    const int x = ht_first(0, h.n, [&](int i) {
      return !(ld_l2(h.tw + i) & kTEmpty) && anc - ld_l2(h.pl + 5 * h.sd + i) < ld_l2(h.pl + i);
    });
    int t = -1;
    int32_t off = 0;
    if (x >= 0 && ht_removed_acked(h, x)) {
      uint32_t to = 0, st2 = stt;
      if (ht_slide_item(h, x, t, off)) {
        p = ht_view_prefix<K>(h, ht_leaf_start(h, t), h.cur_seq, ls) + ht_leaf_offset(h, t) + off;
        int32_t o2 = 0;
        const int y = ht_view_find<K>(h, p, h.cur_seq, ls, o2);
        if (y >= 0) to = uni(ld_l2(h.pl + 5 * h.sd + y)) + (uint32_t)o2;
        else st2 |= kRefDetached;  // the reference throws: no segment there
      } else {
        st2 |= kRefDetached;
      }
      if (lane_id() == 0) rt[slot] = make_uint2(to, st2);
      vm_drain();
      h.wcache = -1;  // createLocalReferencePosition updates lengths (mergeTree.ts:2124-2143)
    }
  }
  ev_one(ev, MTE_DELTA_REBASE, p, 0);
  return 0;
}

// The MTE_DELTA_SLIDE records of one message, [from, ev.n): the unit each
// reference left -> that unit's order key after the message (its zambonis
// included): the held units before it, as mte_read_ref_order counts them, -1
// if it is gone (titems.c slide_keys).  One wave-wide search per record.
// (Out of line, its arguments by value: a reference to the pass's state would
// keep that state in scratch for the whole kernel.)
// Returns the number of slide records.
__device__ __noinline__ uint32_t ht_slide_keys(const uint32_t* pl, uint64_t sd, int n, mte_delta* evp, uint32_t to,
                                               uint32_t from) {
  if (from >= to) return 0;
  vm_drain();  // this wave's record stores are visible to its loads
  const int l = lane_id();
  uint32_t slid = 0;
  for (uint32_t q = from; q < to; q++) {
    const uint32_t kind = uni(ld_l2(&evp[q].kind));
    if ((kind & 0xc0u) != MTE_DELTA_SLIDE) continue;
    slid++;
    const uint32_t u = uni(ld_l2(reinterpret_cast<const uint32_t*>(&evp[q].len)));
    int32_t key = -1, carry = 0;
    for (int tb = 0; tb < n; tb += kWave) {
      const int i = tb + l;
      const int ic = i < n ? i : 0;  // unconditional loads, selected after
      const uint32_t ln = ld_l2(pl + ic), tf = ld_l2(pl + 5 * sd + ic);
      const int32_t L = i < n ? (int32_t)ln : 0;
      const int32_t incl = wave_incl_scan(L);
      const uint64_t m = __ballot(i < n && u - tf < ln);
      if (m) {
        const int j = __ffsll((long long)m) - 1;
        key = carry + rdlane(incl - L + (int32_t)(u - tf), j);
        break;
      }
      carry += rdlane(incl, kWave - 1);
    }
    if (l == 0) evp[q].len = key;
  }
  vm_drain();
  return slid;
}

// The MTE_DELTA_MAINT records of one message, [from, to): each segment's leaf
// id -> its position in the own view now, -1 when no leaf of that id is in the
// tree (titems.c maint_positions).  Out of line, its arguments by value.
__device__ __noinline__ void ht_maint_positions(const uint32_t* pl, uint64_t sd, const uint32_t* tw, int n, mte_delta* evp,
                                                uint32_t to, uint32_t from) {
  if (from >= to) return;
  vm_drain();
  for (uint32_t q = from; q < to; q++) {
    const uint32_t kind = uni(ld_l2(&evp[q].kind));
    const int32_t id = (int32_t)uni(ld_l2(reinterpret_cast<const uint32_t*>(&evp[q].pos)));
    if ((kind & 0xff00u) != MTE_DELTA_MAINT || id < 0) continue;
    const int i = ht_first(0, n, [&](int x) {
      const uint32_t t = ld_l2(tw + x);
      return t_id(t) == (uint32_t)id && (t & (kTCont | kTEmpty)) == 0;
    });
    const int32_t p = i < 0 ? -1 : own_prefix(pl, sd, i);
    if (lane_id() == 0) evp[q].pos = p;
  }
  vm_drain();
}

// MTE_DELTA_REFPOS (include/mte.h): every live reference of slots [0, rhi) as
// a record that slid one left the document -- its position (as mte_read_refs;
// -2 - its Transient position for one off the string, as
// mte_read_refs_transient finds it) and its order key (as mte_read_ref_order):
// what the reference's slide callbacks read mid-op (intervalCollection.ts:
// 1042-1053; titems.c ref_snapshot).  A lane per reference walks the items
// with wave-uniform loads: rare (records that slid something), so simple.
// Returns the event count after the records (ev.n).
__device__ __noinline__ uint32_t ht_ref_snapshot(const uint32_t* pl, uint64_t sd, int n, const uint2* rt, uint32_t rhi,
                                                 mte_delta* evp, uint64_t cap, uint32_t en, uint32_t op) {
  const int l = lane_id();
  for (uint32_t rb = 0; rb < rhi; rb += kWave) {
    const uint32_t r = rb + (uint32_t)l;
    const uint32_t rc = r < rhi ? r : 0u;  // unconditional loads, selected after
    const uint32_t anc = ld_l2(&rt[rc].x), st = ld_l2(&rt[rc].y);
    const bool live = r < rhi && (st & kRefLive) && !(st & kRefTrans);  // a Transient one slides no interval
    const bool det = (st & kRefDetached) != 0, off = (st & kRefOff) != 0;
    int32_t pos = -1, tpos = -1, key = -1, own = 0, all = 0;
    bool found = false;
    for (int i = 0; i < n; i++) {
      const uint32_t ln = uni(ld_l2(pl + i)), tf = uni(ld_l2(pl + 5 * sd + i));
      const int32_t rs = (int32_t)uni(ld_l2(pl + 2 * sd + i));
      const bool hit = !found && anc - tf < ln;
      if (hit) {
        const int32_t p = own + (rs != kNone ? 0 : (int32_t)(anc - tf));
        tpos = p;
        pos = det ? -1 : p;
        key = (det && !off) ? -1 : all + (int32_t)(anc - tf);
        found = true;
      }
      own += rs == kNone ? (int32_t)ln : 0;
      all += (int32_t)ln;
    }
    if (det) pos = (off && tpos >= 0) ? -2 - tpos : -1;
    const uint64_t lm = __ballot(live);
    const uint32_t idx = en + lanes_below(lm);
    if (live && idx < cap) evp[idx] = mte_delta{op, MTE_DELTA_REFPOS, pos, key, r};
    en += (uint32_t)__popcll(lm);
  }
  vm_drain();
  return en;
}

template <int K, bool S>
__device__ __forceinline__ int ht_step(HT& h, DocRun& D, uint32_t (&st)[kNumStats], const ReplayArgs& a, int32_t& lseq, EvOut& ev,
                       uint32_t& rhi) {
  s8v op = sload8(D.recp + 2 * D.k);
  const uint4* rec = D.recp + 2 * D.k;
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  if (h.rpf) {  // the positions an MTE_OP_RELPOS record resolved for this one
    if (h.rpf & MTE_RP_POS1) op[4] = h.rp1;
    if (h.rpf & MTE_RP_POS2) op[5] = h.rp2;
    h.rpf = 0;
  }
  const bool ldoc = h.ldoc;
  const bool evd = (D.flags & MTE_DOC_EVENTS) != 0;
  const bool refd = (D.flags & MTE_DOC_REFS) != 0 && a.refs != nullptr;
  const bool evs = evd && refd && (D.flags & MTE_DOC_SLIDE_EVENTS) != 0;  // slide records (and snapshots)
  uint2* const rt = refd ? a.refs + (uint64_t)D.doc * a.ref_cap : nullptr;
  ev.op = D.k;
  const uint32_t ev_from = ev.n;  // this record's first event
  if (h.n + 4 > h.cap) return MTE_E_CAPACITY;
  // short ids: 64 where the removers' upper half has its plane (kRmHiPlane)
  const uint32_t max_c = h.nP == kLocalPlanes<K> ? MTE_MAX_CLIENTS_TREE : MTE_MAX_CLIENTS;
  if (c >= max_c) return MTE_E_CLIENT_RANGE;
  const int32_t s = op[0], msn = op[2];
  const bool lop = (flags & MTE_F_LOCAL) != 0;
  int rc;
  h.born = (uint32_t)lseq + 1u;  // an item split off now is a tail of the pending groups
  h.min_seq = D.min_seq;
  h.cur_seq = D.cur_seq;
  if (type == MTE_OP_RELPOS) {
    // the next record's positions, in its view (the engine checked that an
    // insert, remove or annotate of this document follows)
    if (D.k + 1 >= D.k1) return MTE_E_INVALID_ARG;
    HPROF_BEGIN(t0)
    const s8v nx = sload8(rec + 2);
    const uint32_t nw3 = (uint32_t)nx[3];
    const uint32_t nt = nw3 & 0xffu, nc = (nw3 >> 8) & 0xffu;
    const bool nloc = ((nw3 >> 16) & MTE_F_LOCAL) != 0;
    if (nt > MTE_OP_ANNOTATE || nc >= max_c) return MTE_E_INVALID_ARG;
    const uint32_t key = (uint32_t)op[6];
    h.rpf = 0;
    if (flags & MTE_RP_POS1) {
      int32_t p = ht_marker_pos<K>(h, key, (uint32_t)op[4], nloc, nx[1], (int)nc);
      if (p >= 0) p = (flags & MTE_RP_BEFORE1) ? p - op[0] : p + 1 + op[0];
      else if (nt == MTE_OP_INSERT) return MTE_E_UNSUPPORTED;
      h.rp1 = p;
      h.rpf |= MTE_RP_POS1;
    }
    if ((flags & MTE_RP_POS2) && nt != MTE_OP_INSERT) {
      int32_t p = ht_marker_pos<K>(h, key, (uint32_t)op[5], nloc, nx[1], (int)nc);
      if (p >= 0) p = (flags & MTE_RP_BEFORE2) ? p - op[1] : p + 1 + op[1];
      h.rp2 = p;
      h.rpf |= MTE_RP_POS2;
    }
    HPROF_END(h, 5, t0)
    D.k++;
    return 0;
  }
  // a length update drops the reference's cached local partials
  // (mergeTree.ts:2105-2110, 2188-2191; ht_view_window): every record but a
  // regeneration; references below
  if (type != MTE_OP_REF && type != MTE_OP_REGEN) h.wcache = -1;
  if (type == MTE_OP_REF) {
    if (!lop || !ldoc || !refd) return MTE_E_UNSUPPORTED;
    if ((uint32_t)op[5] >= a.ref_cap || (uint32_t)op[7] > 5u) return MTE_E_INVALID_ARG;
    if ((uint32_t)op[7] == 2u && c == 0) return MTE_E_INVALID_ARG;
    if ((uint32_t)op[7] >= 4u && !evd) return MTE_E_UNSUPPORTED;
    MTE_STAT(st[kStOps]++;)
    MTE_STAT(if ((uint32_t)op[7] != 1u) st[kStScanned] += (uint32_t)h.n;)
    HPROF_BEGIN(t0)
    if ((uint32_t)op[7] >= 4u) {
      rc = ht_ref_rebase<K>(h, op, lseq, rt, ev);
    } else {
      // createLocalReferencePosition updates lengths (mergeTree.ts:2124-2143): a
      // reference made on a segment (b = 0 / 2), or one ackInterval re-makes (b = 3)
      const uint32_t slot = (uint32_t)op[5];
      const uint2 before = make_uint2(uni(ld_l2(&rt[slot].x)), uni(ld_l2(&rt[slot].y)));
      if ((uint32_t)op[7] == 0u && ((uint32_t)op[6] & MTE_REF_TRANSIENT)) rc = ht_ref_transient<K>(h, rt, rhi, op);
      else rc = stream_ref<K>(h.pl, h.sd, h.n, rt, rhi, op, D.min_seq, h.newcalc);
      const uint2 after = make_uint2(uni(ld_l2(&rt[slot].x)), uni(ld_l2(&rt[slot].y)));
      const uint32_t b = (uint32_t)op[7];
      if ((b == 0u || b == 2u) ? !(after.y & kRefDetached)
                               : (b == 3u && (after.x != before.x || ((after.y ^ before.y) & kRefDetached))))
        h.wcache = -1;
    }
    HPROF_END(h, 5, t0)
    if (rc) return rc;
    D.k++;
    return 0;
  }
  if (type > MTE_OP_REGEN) return MTE_E_INVALID_ARG;  // MTE_OP_RBKEY only after an annotate's rollback
  if ((lop || type >= MTE_OP_ACK) && !ldoc) return MTE_E_UNSUPPORTED;
  MTE_STAT(st[kStOps]++;)
  MTE_STAT(st[kStMaxSegs] = (uint32_t)h.n > st[kStMaxSegs] ? (uint32_t)h.n : st[kStMaxSegs];)
  if (type != MTE_OP_NOOP) MTE_STAT(st[kStScanned] += (uint32_t)h.n;)
  if (type == MTE_OP_ROLLBACK) {
    if (!lop || !(s > 0 && s <= lseq)) return MTE_E_INVALID_ARG;
    const int32_t t = op[4];
    if (t == MTE_OP_ANNOTATE) {
      const uint32_t n_aux = (uint32_t)op[5];
      if ((uint64_t)D.k + 1 + n_aux > D.k1 || (uint32_t)op[6] >= MTE_ANNOTATE_SLOTS) return MTE_E_INVALID_ARG;
      HPROF_BEGIN(t0)
      rc = ht_rollback_annotate<K>(h, (uint32_t)op[6], rec + 2, n_aux, a, evd, ev);
      HPROF_END(h, 4, t0)
      if (rc) return rc;
      D.k += 1 + n_aux;
      return 0;
    }
    if (t != MTE_OP_INSERT && t != MTE_OP_REMOVE) return MTE_E_INVALID_ARG;
    HPROF_BEGIN(t0)
    rc = ht_rollback<K>(h, op, a, evd, ev);
    HPROF_END(h, 4, t0)
    if (rc) return rc;
    D.k++;
    return 0;
  }
  if (type == MTE_OP_REGEN) {
    const int32_t t = op[4];
    if (!lop || !(s > 0 && s <= lseq)) return MTE_E_INVALID_ARG;
    if (t != MTE_OP_INSERT && t != MTE_OP_REMOVE && t != MTE_OP_ANNOTATE) return MTE_E_INVALID_ARG;
    if (t == MTE_OP_ANNOTATE && (uint32_t)op[6] >= MTE_ANNOTATE_SLOTS) return MTE_E_INVALID_ARG;
    if (!evd) return MTE_E_UNSUPPORTED;
    HPROF_BEGIN(t0)
    ht_regen<K>(h, s, (uint32_t)t, (uint32_t)op[6], ev);
    HPROF_END(h, 4, t0)
    D.k++;
    return 0;
  }
  if (lop) {
    if (!(s > lseq && s < kLocalBase) || c != 0) return MTE_E_INVALID_ARG;
    if (type == MTE_OP_ANNOTATE && (flags & MTE_F_REWRITE)) return MTE_E_UNSUPPORTED;
    if (type == MTE_OP_ANNOTATE && (uint32_t)op[7] != MTE_NO_PROPS && (uint32_t)op[7] >= MTE_ANNOTATE_SLOTS)
      return MTE_E_INVALID_ARG;
    lseq = s;
    h.born = (uint32_t)s;  // an item this op makes is one of its group's own
  } else if (ldoc && type <= MTE_OP_ANNOTATE && c == 0) {
    return MTE_E_INVALID_ARG;  // a remote op from the local client's own slot
  }
  if (type == MTE_OP_INSERT) {
    int at = -1;
    HPROF_BEGIN(t0)
    rc = ht_insert<K, S>(h, op, lop, refd, a, st, at, ev);
    HPROF_END(h, 0, t0)
    if (rc) return rc;
    if (evd) {  // insertSegments' delta callback (mergeTree.ts:1409-1416)
      if (at >= 0) ev_one(ev, MTE_OP_INSERT, own_prefix(h.pl, h.sd, at), (flags & MTE_F_MARKER) ? 1 : op[5]);
      else ev_one(ev, MTE_OP_INSERT, -1, 0);  // a zero-length segment is never linked
    }
  } else if (type == MTE_OP_REMOVE || type == MTE_OP_ANNOTATE) {
    HPROF_BEGIN(t0)
    rc = ht_range<K, S>(h, op, lop, a, st, ev, evd, rt, rhi, evs);
    HPROF_END(h, 1, t0)
    if (rc) return rc;
  } else if (type == MTE_OP_ACK) {
    if (!(op[4] > 0 && op[4] <= op[5] && op[5] <= lseq)) return MTE_E_INVALID_ARG;
    HPROF_BEGIN(t0)
    rc = ht_ack<K>(h, op, a, rt, refd ? rhi : 0u, ev, evs);
    HPROF_END(h, 2, t0)
    if (rc) return rc;
  } else if (type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  D.k++;
  if (lop) return 0;  // a local op moves no window and runs no zamboni
  if (type == MTE_OP_INSERT || type == MTE_OP_REMOVE || type == MTE_OP_ANNOTATE)
    if ((rc = ht_zamboni<K>(h, a.n_keys, ev))) return rc;
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
      h.min_seq = msn;
      h.cur_seq = D.cur_seq;
      if ((rc = ht_zamboni<K>(h, a.n_keys, ev))) return rc;
    }
  }
  // the slides of this record, keyed by the units they left as they stand now,
  // then every reference as this record left them
  if (evs && ev.n > ev_from) {
    const uint32_t slid = ht_slide_keys(h.pl, h.sd, h.n, ev.p, ev.n < ev.cap ? ev.n : (uint32_t)ev.cap, ev_from);
    if (slid) ev.n = ht_ref_snapshot(h.pl, h.sd, h.n, rt, rhi, ev.p, ev.cap, ev.n, ev.op);
  }
  return 0;
}

// The HBM tree pass: one wavefront (workgroup) per candidate document — every
// local-client document, and the legacy documents the register tiers handed
// over (kHdrTreeHbm; their heap and tree state move over on first entry).
// M: the build with the maintenance records (MTE_DOC_MAINT_EVENTS), launched
// only for a batch that asks for them -- their code costs the kernel registers
// (189 VGPRs against 80 without, two waves per SIMD instead of six)
#ifndef MTE_HTREE_WPE  // a waves-per-SIMD floor for the register allocator (A/B builds)
#define MTE_HTREE_WPE 0
#endif
#if MTE_HTREE_WPE > 0
#define MTE_HTREE_ATTR __attribute__((amdgpu_waves_per_eu(MTE_HTREE_WPE)))
#else
#define MTE_HTREE_ATTR
#endif
template <int K, bool S, bool M>
__global__ __launch_bounds__(64) MTE_HTREE_ATTR void htree_kernel(ReplayArgs a, HtreeArgs t) {
  const int idx = (int)blockIdx.x;
  if (idx >= (int)t.n_docs) return;
  const int doc = uni((int)t.docs[idx]);
  const uint32_t hf = uni(a.hdr[doc].flags);
  const bool ldoc = (hf & MTE_DOC_LOCAL_CLIENT) != 0;
  // its own documents from the start (a local client's, MTE_DOC_TREE, legacy
  // ones with delta events), the other legacy ones once TIER 2 hands them over
  const bool own = ldoc || (hf & MTE_DOC_TREE) || ((hf & MTE_DOC_EVENTS) && !(hf & MTE_DOC_NEW_LENGTH_CALC));
  if (!own && !(hf & kHdrTreeHbm)) return;
  DocRun D;
  run_init(D, a, doc, false);
  uint32_t* stp = t.st + (uint64_t)doc * kHtState;
  HT h;
  h.pl = a.planes + (uint64_t)doc * a.cap;
  h.sd = a.stride;
  h.tw = t.tree + (uint64_t)doc * a.cap;
  h.L = t.scr + (uint64_t)doc * 2 * a.cap;
  h.P = h.L + a.cap;
  h.hp = reinterpret_cast<uint32_t*>(t.heap + (uint64_t)doc * (t.hcap + 1));
  h.hcap = t.hcap;
  h.cap = (int)a.cap;
  h.nP = (ldoc || (hf & MTE_DOC_TREE)) ? kLocalPlanes<K> : kFieldPlanes + K;
  h.n = D.n;
  h.newcalc = (hf & MTE_DOC_NEW_LENGTH_CALC) != 0;
  h.ldoc = ldoc;
  h.arena = t.arena;
  h.min_seq = D.min_seq;
  h.cur_seq = D.cur_seq;
  h.lp_n = 0;
  h.lp_carry = 0;
  h.plocal = false;
  h.pr = 0;
  h.pc = 0;
  h.rpf = 0;
  h.lds = false;
  h.maint = false;
#ifdef MTE_HTREE_PROF
  for (int q = 0; q < kHtProf; q++) h.prof[q] = 0;
#endif
  if (!ldoc && uld(stp + kHsEntered) == 0u) {
    // a legacy document leaves the register tiers: its depth / next id / heap
    // (DocHdr pad0 / pad1, TreeArgs::heap) move to the HBM tree's state
    const uint32_t p0 = uni(a.hdr[doc].pad0), p1 = uni(a.hdr[doc].pad1);
    h.depth = (int)(p1 & 0xffu);
    h.hn = p1 >> 8;
    h.next_id = p0;
    const uint2* src = t.rheap + (uint64_t)doc * (kTreeHeapCap + 1);
    for (uint32_t k = 1 + (uint32_t)lane_id(); k <= h.hn; k += kWave) {
      const uint2 v = src[k];
      h.hp[2 * k] = v.x;
      h.hp[2 * k + 1] = v.y;
    }
    lane0_st(stp + kHsEntered, 1u);
    vm_drain();
  } else {
    h.depth = (int)uld(stp + kHsDepth);
    h.next_id = uld(stp + kHsNextId);
    h.hn = uld(stp + kHsHeapN);
  }
  int32_t lseq = (int32_t)uld(stp + kHsLseq);
  uint32_t rhi = uld(stp + kHsRhi);
  h.wcache = (int32_t)uld(stp + kHsWin) - 1;
  uint32_t st[kNumStats] = {};
  EvOut ev{nullptr, 0, 0u, 0u};
  if ((hf & MTE_DOC_EVENTS) && a.dl_off) {
    ev.p = a.dl + a.dl_off[doc];
    ev.cap = a.dl_off[doc + 1] - a.dl_off[doc];
    h.maint = M && (hf & MTE_DOC_MAINT_EVENTS) != 0;
  }
  uint32_t msg_ev = 0;   // MTE_DELTA_MAINT: the first event of the message being applied
  bool msg_open = false;  // its MSG_END not applied yet
  D.running = D.status == 0 && D.k < D.k1;
  extern __shared__ uint32_t ht_lds[];
  // LDS-resident while the document fits (ht_lds_room's margins)
  if (D.running && t.lcap && h.n + kLdsMargin <= (int)t.lcap && (int)h.hn + h.n + kLdsMargin <= (int)t.lcap)
    ht_to_lds(h, ht_lds, t.lcap);
  while (D.running) {
    if (h.lds && !ht_lds_room(h)) ht_spill(h);
    HPROF_BEGIN(t_rec)
    uint32_t w3 = 0u;
    if (h.maint) {
      if (!msg_open) msg_ev = ev.n;
      w3 = (uint32_t)sload8(D.recp + 2 * D.k)[3];
    }
    const int rc = ht_step<K, S>(h, D, st, a, lseq, ev, rhi);
    if (h.maint && rc >= 0) {
      // maintenance positions once the message (a local record: itself) is applied
      msg_open = (w3 & 0xffu) == MTE_OP_RELPOS || !((w3 >> 16) & (MTE_F_MSG_END | MTE_F_LOCAL));
      if (!msg_open && ev.n > msg_ev)
        ht_maint_positions(h.pl, h.sd, h.tw, h.n, ev.p, ev.n < ev.cap ? ev.n : (uint32_t)ev.cap, msg_ev);
    }
    HPROF_END(h, 6, t_rec)
#ifdef MTE_HTREE_PROF
    h.prof[7]++;
#endif
    D.n = h.n;
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
  if (h.lds) ht_spill(h);
#ifdef MTE_HTREE_PROF
  if (t.prof && lane_id() == 0)
    for (int q = 0; q < kHtProf; q++) atomicAdd(t.prof + q, h.prof[q]);
#endif
  lane0_st(stp + kHsDepth, (uint32_t)h.depth);
  lane0_st(stp + kHsNextId, h.next_id);
  lane0_st(stp + kHsHeapN, h.hn);
  lane0_st(stp + kHsLseq, (uint32_t)lseq);
  lane0_st(stp + kHsRhi, rhi);
  lane0_st(stp + kHsWin, (uint32_t)(h.wcache + 1));
  if ((hf & MTE_DOC_EVENTS) && a.dl_n && lane_id() == 0) a.dl_n[doc] = ev.n;
  vm_drain();
  run_finish(D, a);
}

}  // namespace mte
