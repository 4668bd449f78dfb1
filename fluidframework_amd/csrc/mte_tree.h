// mte_tree.h — the tree pass: legacy length-calc documents replayed with the
// reference's B+tree shape.
//
// With the legacy length calculation an insert next to tombstones lands where
// the reference's insertingWalk puts it: at the end of the first leaf block
// whose perspective length reaches the position (mergeTree.ts:1743,
// 1788-1797), which depends on the block edges of its B+tree, and those on
// every split (1800-1840) and on the lazy LRU zamboni (665-675, 681-838).  This
// pass carries that tree beside the segments.  Its executable spec is
// oracle/titems.c (checked against the linked-block tree.c and the reference
// itself); each function below names the titems.c function it restates.
//
// Layout: one wavefront per document, the segments register-resident
// lane-major as in the flat passes (segment i = slot i % E of lane i / E), plus
// one more plane, the tree word
//   bits 0-2  h: block levels this item starts (0 inside a leaf block)
//   bit  3    cont: continues the previous item's leaf (an append-merge)
//   bits 4-5  ns: needsScour of the leaf block it starts (0 undefined, 1 false, 2 true)
//   bit  6    po: segment.properties exists
//   bit  7    empty: placeholder of an empty leaf block (len 0, undefined to all)
//   bits 8-30 id: the name the LRU heap entries use
//   bit  31   nl: the text may hold a '\n' (its insert's text did; mte_submit
//             marks those records kRecNl), so an append-merge must look at its
//             last unit in the arena; without it no load is needed
// and the LRU heap (collections/heap.ts) in LDS, 8 B per entry.  The op
// records are prefetched with vector loads: a scalar prefetch would share the
// LDS accesses' wait counter and stall every heap access on it.  Between
// launches the tree word lives in TreeArgs::tree, the heap in TreeArgs::heap,
// depth / next id / heap size in DocHdr pad0 / pad1.
#pragma once

#include "mte_replay.h"

namespace mte {

constexpr int kTreeHeapCap = 255;  // entries per document (+ the unused index 0)
constexpr uint32_t kHdrTreeEsc = 0x40000000u;  // tree pass: the document is TIER 1's (E = 4)
constexpr uint32_t kHdrTreeBig = 0x20000000u;  // tree pass: the document is TIER 2's (E = 8, 16)
constexpr uint32_t kHdrTreeHbmFlag = 0x10000000u;  // past TIER 2: the HBM tree pass (mte_htree.h kHdrTreeHbm)
constexpr uint32_t kTH = 0x7u, kTCont = 0x8u, kTNsShift = 4, kTNs = 0x30u, kTPo = 0x40u, kTEmpty = 0x80u;
constexpr uint32_t kTNl = 0x80000000u;
constexpr uint16_t kRecNl = 0x8000u;  // op record flag (engine-internal): the insert's text holds a '\n'
constexpr uint32_t kNsUndef = 0, kNsFalse = 1, kNsTrue = 2;
constexpr int kMaxNodes = 8;       // MaxNodesInBlock, mergeTreeNodes.ts:373
constexpr int32_t kTextGranularity = 256;  // textSegment.ts:19
constexpr uint32_t kIdLimit = 1u << 23;

// MTE_TREE_PROF (a profiling build only, `make prof`): with statistics on, the
// tree pass's counters become phase clocks (s_memrealtime ticks, 100 MHz):
// segs_scanned = lengths + boundaries, segs_written = insert / range marks +
// LRU, prop_writes = the op's zamboni, units_inserted = the whole op,
// max_segs = the largest per-doc zamboni time at msn advances.
#ifdef MTE_TREE_PROF
#define TSTAT(...)
#define TPROF(...) MTE_STAT(__VA_ARGS__)
#else
#define TSTAT(...) MTE_STAT(__VA_ARGS__)
#define TPROF(...)
#endif

struct TreeArgs {
  uint32_t* tree;        // tree word of slot x of doc d: tree[d * cap + x]
  uint2* heap;           // doc d: heap[d * (kTreeHeapCap + 1) + k], k = 1 .. size
  const uint32_t* docs;  // the legacy documents
  uint32_t n_docs;
  const uint16_t* arena; // text (an append-merge looks at the last unit of a leaf)
  uint32_t final_round;  // TIER 1: keep documents that shrink (no return to TIER 0)
  uint32_t k_cap;        // this round's op cursor limit (TIER 0 / 1): documents advance together
};

__device__ __forceinline__ uint32_t t_h(uint32_t t) { return t & kTH; }
__device__ __forceinline__ uint32_t t_ns(uint32_t t) { return (t & kTNs) >> kTNsShift; }
__device__ __forceinline__ uint32_t t_id(uint32_t t) { return (t >> 8) & (kIdLimit - 1u); }

// ---- wave-wide index helpers (E slots per lane, index = lane * E + j) --------

// first index >= lo with pred, or -1
template <int E>
__device__ __forceinline__ int first_where(const bool (&p)[E], int lo) {
  const int base = lane_id() * E;
  int best = INT32_MAX;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint64_t m = __ballot(p[j] && base + j >= lo);
    if (m) {
      const int c = (__ffsll((long long)m) - 1) * E + j;
      best = c < best ? c : best;
    }
  }
  return best == INT32_MAX ? -1 : best;
}

// last index <= hi with pred, or -1
template <int E>
__device__ __forceinline__ int last_where(const bool (&p)[E], int hi) {
  const int base = lane_id() * E;
  int best = -1;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint64_t m = __ballot(p[j] && base + j <= hi);
    if (m) {
      const int c = (63 - __clzll((long long)m)) * E + j;
      best = c > best ? c : best;
    }
  }
  return best;
}

template <int E>
__device__ __forceinline__ int count_where(const bool (&p)[E], int lo, int hi) {
  const int base = lane_id() * E;
  int c = 0;
#pragma unroll
  for (int j = 0; j < E; j++) c += __popcll(__ballot(p[j] && base + j >= lo && base + j <= hi));
  return c;
}

// index of the r-th (0-based) index in [lo, hi] with pred, or -1
template <int E>
__device__ __forceinline__ int nth_where(const bool (&p)[E], int lo, int hi, int r) {
  const int base = lane_id() * E;
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < E; j++) cnt += (p[j] && base + j >= lo && base + j <= hi) ? 1 : 0;
  const int incl = wave_incl_scan(cnt);
  const int excl = incl - cnt;
  const bool mine = excl <= r && r < incl;
  int at = -1, k = excl;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const bool q = p[j] && base + j >= lo && base + j <= hi;
    if (q && k == r && at < 0) at = base + j;
    k += q ? 1 : 0;
  }
  const uint64_t m = __ballot(mine);
  if (!m) return -1;
  return rdlane(at, __ffsll((long long)m) - 1);
}

// sum of v over [lo, hi)
template <int E>
__device__ __forceinline__ int32_t sum_range(const int32_t (&v)[E], int lo, int hi) {
  const int base = lane_id() * E;
  int32_t s = 0;
#pragma unroll
  for (int j = 0; j < E; j++) s += (base + j >= lo && base + j < hi) ? v[j] : 0;
  return rdlane(wave_incl_scan(s), kWave - 1);
}

// ---- per-document tree state ----------------------------------------------------

struct TreeRun {
  int depth;
  uint32_t next_id;
  uint32_t hn;   // LRU heap entries
  volatile uint2* hp;  // LDS heap of this wave, hp[1 .. hn] (16-byte aligned)
  const uint16_t* arena;
};

template <int E, int K>
struct TReg {
  Regs<E, K> R;
  uint32_t T[E];
};

// open slot g (new[i] = old[i - 1] for i >= g), every plane
template <int E, int K>
__device__ __forceinline__ void open_slot(TReg<E, K>& X, int g) {
  pull_shift<E>(X.R.len, g - 1, INT32_MAX);
  pull_shift<E>(X.R.seq, g - 1, INT32_MAX);
  pull_shift<E>(X.R.rseq, g - 1, INT32_MAX);
  pull_shift<E>(X.R.rmask, g - 1, INT32_MAX);
  pull_shift<E>(X.R.meta, g - 1, INT32_MAX);
  pull_shift<E>(X.R.toff, g - 1, INT32_MAX);
#pragma unroll
  for (int k = 0; k < K; k++) pull_shift<E>(X.R.pr[k], g - 1, INT32_MAX);
  pull_shift<E>(X.T, g - 1, INT32_MAX);
}

// drop the slots without `keep` (stream compaction through LDS)
template <int E, int K>
__device__ __forceinline__ int compact_slots(TReg<E, K>& X, const bool (&keep)[E], int n, uint32_t* zlds) {
  const int base = lane_id() * E;
  int32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < E; j++) cnt += (keep[j] && base + j < n) ? 1 : 0;
  const int32_t incl = wave_incl_scan(cnt);
  const int n_new = rdlane(incl, kWave - 1);
  if (n_new == n) return n;
  bool kp[E];
  int32_t dst[E];
  int32_t d0 = incl - cnt;
#pragma unroll
  for (int j = 0; j < E; j++) {
    kp[j] = keep[j] && base + j < n;
    dst[j] = d0;
    d0 += kp[j] ? 1 : 0;
  }
  compact_plane<E>(X.R.len, kp, dst, zlds);
  compact_plane<E>(X.R.seq, kp, dst, zlds);
  compact_plane<E>(X.R.rseq, kp, dst, zlds);
  compact_plane<E>(X.R.rmask, kp, dst, zlds);
  compact_plane<E>(X.R.meta, kp, dst, zlds);
  compact_plane<E>(X.R.toff, kp, dst, zlds);
#pragma unroll
  for (int k = 0; k < K; k++) compact_plane<E>(X.R.pr[k], kp, dst, zlds);
  compact_plane<E>(X.T, kp, dst, zlds);
#pragma unroll
  for (int j = 0; j < E; j++) {
    const bool pad = base + j >= n_new;
    X.R.rseq[j] = pad ? kPad : X.R.rseq[j];
    X.R.len[j] = pad ? 0 : X.R.len[j];
    X.T[j] = pad ? 0u : X.T[j];
  }
  return n_new;
}

// block spans: the last index <= i that starts a level-k block, and the last
// index of that block
template <int E>
__device__ __forceinline__ int span_start(const uint32_t (&T)[E], int i, int k) {
  bool p[E];
#pragma unroll
  for (int j = 0; j < E; j++) p[j] = (int)t_h(T[j]) >= k;
  const int s = last_where<E>(p, i);
  return s < 0 ? 0 : s;
}
template <int E>
__device__ __forceinline__ int span_end(const uint32_t (&T)[E], int s, int k, int n) {
  bool p[E];
#pragma unroll
  for (int j = 0; j < E; j++) p[j] = (int)t_h(T[j]) >= k;
  const int e = first_where<E>(p, s + 1);
  return (e < 0 || e >= n) ? n - 1 : e - 1;
}

// children of a level-k block: logical leaves (k = 1) or level-(k-1) starts
template <int E>
__device__ __forceinline__ void child_pred(const uint32_t (&T)[E], int k, bool (&p)[E]) {
#pragma unroll
  for (int j = 0; j < E; j++)
    p[j] = k == 1 ? (T[j] & (kTCont | kTEmpty)) == 0 : (int)t_h(T[j]) >= k - 1;
}

template <int E>
__device__ __forceinline__ void set_h(uint32_t (&T)[E], int i, uint32_t h, bool clear_ns) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++)
    if (base + j == i) T[j] = (T[j] & ~(kTH | (clear_ns ? kTNs : 0u))) | h;
}

template <int E>
__device__ __forceinline__ void set_ns(uint32_t (&T)[E], int i, uint32_t ns) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++)
    if (base + j == i) T[j] = (T[j] & ~kTNs) | (ns << kTNsShift);
}

// split_cascade (titems.c): a leaf block gained a child at item i
template <int E>
__device__ __forceinline__ void split_cascade(uint32_t (&T)[E], int i, int n, TreeRun& tr) {
  for (int k = 1;; k++) {
    const int s = span_start<E>(T, i, k), e = span_end<E>(T, s, k, n);
    bool p[E];
    child_pred<E>(T, k, p);
    if (count_where<E>(p, s, e) < kMaxNodes) return;
    const int z = nth_where<E>(p, s, e, kMaxNodes / 2);
    set_h<E>(T, z, (uint32_t)k, k == 1);
    if (k == tr.depth) {  // the root split: a new root above both halves
      tr.depth++;
      set_h<E>(T, 0, (uint32_t)tr.depth, false);
      return;
    }
  }
}

// ---- LRU heap (collections/heap.ts), uniform code over the LDS array ------------
// The sifts move a hole instead of swapping (the same comparisons as heap.ts's
// fixup / fixdown, so the same final array): the element being placed stays
// in registers, each level of fixdown is one 16-byte read of both children
// and one write, and LDS accesses through the volatile pointer stay in order
// (a wave's LDS operations complete in order), so only reads are waited on.

__device__ __forceinline__ void hp_put(volatile uint2* hp, uint32_t k, uint2 v) {
  if (lane_id() == 0) {
    hp[k].x = v.x;
    hp[k].y = v.y;
  }
}
__device__ __forceinline__ uint2 hp_get(volatile uint2* hp, uint32_t k) {
  const uint32_t x = hp[k].x, y = hp[k].y;
  return make_uint2(uni(x), uni(y));
}

__device__ __forceinline__ int heap_add(TreeRun& tr, int32_t key, uint32_t id) {
  if (tr.hn >= (uint32_t)kTreeHeapCap) return MTE_E_CAPACITY;
  uint32_t k = ++tr.hn;
  // fixup: while the parent compares greater, it moves down into the hole
  while (k > 1) {
    const uint2 par = hp_get(tr.hp, k >> 1);
    if (!((int32_t)par.x - key > 0)) break;
    hp_put(tr.hp, k, par);
    k >>= 1;
  }
  hp_put(tr.hp, k, make_uint2((uint32_t)key, id));
  return 0;
}

__device__ __forceinline__ uint2 heap_pop(TreeRun& tr) {
  const uint2 x = hp_get(tr.hp, 1);
  const uint2 cur = hp_get(tr.hp, tr.hn);  // the last entry, re-placed from the root
  tr.hn--;
  uint32_t k = 1;
  while ((k << 1) <= tr.hn) {
    uint32_t j = k << 1;
    // both children in one read (entries 2k, 2k + 1 are 16-byte aligned)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u cc = *reinterpret_cast<const volatile v4u*>(tr.hp + j);
    uint2 c = make_uint2(uni(cc[0]), uni(cc[1]));
    if (j < tr.hn) {
      const uint2 c1 = make_uint2(uni(cc[2]), uni(cc[3]));
      if ((int32_t)c.x - (int32_t)c1.x > 0) {
        j++;
        c = c1;
      }
    }
    if ((int32_t)cur.x - (int32_t)c.x <= 0) break;
    hp_put(tr.hp, k, c);
    k = j;
  }
  if (tr.hn > 0) hp_put(tr.hp, k, cur);
  return x;
}

// add_lru (titems.c): addToLRUSet for the leaf headed at item i
template <int E>
__device__ __forceinline__ int add_lru(uint32_t (&T)[E], int i, int32_t seq, int32_t cur_seq, TreeRun& tr) {
  const int bs = span_start<E>(T, i, 1);
  const uint32_t tb = bcast<E>(T, bs);
  if (t_ns(tb) != kNsTrue && seq > cur_seq) {
    set_ns<E>(T, bs, kNsTrue);
    return heap_add(tr, seq, t_id(bcast<E>(T, i)));
  }
  return 0;
}

// ---- scour / pack (titems.c scour, drop_keep_starts, pack_parent) ----------------

// scourNode over the leaf block [s, e]: sets drop[] on unlinked items and the
// cont bit on appended leaves; returns the logical leaves held.
//
// Vector form of mergeTree.ts:681-757 (titems.c scour): every leaf of the
// block is summarised in parallel — removed / kept tombstone / below minSeq /
// text, "same properties and text as the leaf before it", "the leaf before it
// ends in '\n'", its prefix length — and the summaries are gathered through
// LDS so that leaf r sits in lane r.  The append chain (TextSegment.canAppend
// with the running length of the leaf appended to) then runs as a scalar loop
// over those lanes, and its drop / append masks are applied in one pass.  The
// leaf appended to is always the one just before: a run's leaves carry its
// head's properties, and an append needs a match with the run.
constexpr uint32_t kScRemoved = 1u, kScKeep = 2u, kScElig = 4u, kScText = 8u, kScMatch = 16u, kScNl = 32u;

template <int E, int K>
__device__ __forceinline__ int scour(TReg<E, K>& X, int s, int e, int n, int32_t min_seq, bool (&drop)[E],
                                     const TreeRun& tr, int n_keys, uint32_t* zlds) {
  const int l = lane_id();
  const int base = l * E;
  // previous item's T / len / toff (item base + j - 1)
  uint32_t pT[E], pO[E];
  int32_t pL[E];
  pT[0] = (uint32_t)lane_prev((int32_t)X.T[E - 1]);
  pL[0] = lane_prev(X.R.len[E - 1]);
  pO[0] = (uint32_t)lane_prev((int32_t)X.R.toff[E - 1]);
#pragma unroll
  for (int j = 1; j < E; j++) {
    pT[j] = X.T[j - 1];
    pL[j] = X.R.len[j - 1];
    pO[j] = X.R.toff[j - 1];
  }
  bool head[E];
  int32_t hc = 0, lsum = 0, PX[E];
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    head[j] = i >= s && i <= e && (X.T[j] & (kTCont | kTEmpty)) == 0;
    hc += head[j] ? 1 : 0;
    PX[j] = lsum;
    lsum += i < n ? X.R.len[j] : 0;
  }
  const int32_t hin = wave_incl_scan(hc), lin = wave_incl_scan(lsum);
  const int m = rdlane(hin, kWave - 1);
  const int32_t ltot = rdlane(lin, kWave - 1);
#pragma unroll
  for (int j = 0; j < E; j++) PX[j] += lin - lsum;
  if (m == 0) return 0;
  // the leaf before a head ends in '\n' (only texts that held one are loaded)
  bool nlc[E];
  bool any_nl = false;
#pragma unroll
  for (int j = 0; j < E; j++) {
    nlc[j] = head[j] && (pT[j] & kTNl) && pL[j] > 0;
    any_nl = any_nl || nlc[j];
  }
  uint32_t nlb[E];
#pragma unroll
  for (int j = 0; j < E; j++) nlb[j] = 0;
  if (__ballot(any_nl)) {
#pragma unroll
    for (int j = 0; j < E; j++)
      nlb[j] = (nlc[j] && tr.arena[pO[j] + (uint32_t)pL[j] - 1u] == (uint16_t)'\n') ? kScNl : 0u;
  }
  // leaf records by rank: [bits, PX, po, props...] (W words)
  constexpr int W = 3 + K;
  int32_t r0 = hin - hc;
#pragma unroll
  for (int j = 0; j < E; j++) {
    if (head[j]) {
      uint32_t* rec = zlds + r0 * W;
      const uint32_t meta = X.R.meta[j];
      uint32_t bits = nlb[j];
      bits |= X.R.rseq[j] != kNone ? kScRemoved : 0u;
      bits |= X.R.rseq[j] > min_seq ? kScKeep : 0u;
      bits |= X.R.seq[j] <= min_seq ? kScElig : 0u;
      bits |= (meta >> 8) == 0 ? kScText : 0u;
      rec[0] = bits;
      rec[1] = (uint32_t)PX[j];
      rec[2] = X.T[j] & kTPo;
#pragma unroll
      for (int k = 0; k < K; k++) rec[3 + k] = k < n_keys ? X.R.pr[k][j] : 0u;
      r0++;
    }
  }
  fence_wave();
  // lane r: leaf r's bits, with the match against leaf r - 1
  uint32_t bits = 0, pxh = 0;
  if (l < m) {
    const uint32_t* rc = zlds + l * W;
    bits = rc[0];
    pxh = rc[1];
    if (l > 0) {
      const uint32_t* rp = rc - W;
      bool match = (rp[0] & kScText) && (bits & kScText) && rp[2] == rc[2];
#pragma unroll
      for (int k = 0; k < K; k++) match = match && rp[3 + k] == rc[3 + k] && !(rc[3 + k] & MTE_VALUE_UNEQUAL);
      bits |= match ? kScMatch : 0u;
    }
  }
  fence_wave();
  const int32_t pend = e + 1 < n ? bcast<E>(PX, e + 1) : ltot;
  // the append chain, leaf by leaf (scalar)
  int held = 0;
  uint64_t dropm = 0, contm = 0;
  bool run = false;  // the leaf before can be appended to
  int32_t run_len = 0;
  for (int r = 0; r < m; r++) {
    const uint32_t b = rdlane(bits, r);
    const int32_t xl = (int32_t)((r + 1 < m ? rdlane(pxh, r + 1) : (uint32_t)pend) - rdlane(pxh, r));
    if (b & kScRemoved) {
      if (b & kScKeep) held++;
      else dropm |= 1ull << r;
      run = false;
    } else if (b & kScElig) {
      const bool app = run && (b & kScMatch) && !(b & kScNl) &&
                       (run_len <= kTextGranularity || xl <= kTextGranularity) && xl > 0;
      if (app) {
        contm |= 1ull << r;
        run_len += xl;
      } else {
        held++;
        run = xl > 0;
        run_len = xl;
      }
    } else {
      held++;
      run = false;
    }
  }
  // apply: items of dropped leaves, heads of appended ones
  const int32_t hex = hin - hc;  // heads before this lane
  int32_t rk = hex - 1;          // rank of the leaf the item belongs to
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    rk += head[j] ? 1 : 0;
    const bool inb = i >= s && i <= e && rk >= 0;
    drop[j] = drop[j] || (inb && ((dropm >> rk) & 1ull));
    if (head[j] && ((contm >> rk) & 1ull)) X.T[j] = (X.T[j] & ((0xffu & ~kTNs) | kTNl)) | kTCont;
  }
  return held;
}

// titems.c drop_keep_starts over one leaf block [bs, be], then the compaction
template <int E, int K>
__device__ __forceinline__ int drop_block(TReg<E, K>& X, int bs, int be, bool (&drop)[E], int n, uint32_t* zlds) {
  const int base = lane_id() * E;
  const int j0 = [&] {
    bool keep[E];
#pragma unroll
    for (int j = 0; j < E; j++) keep[j] = !drop[j];
    return first_where<E>(keep, bs);
  }();
  const uint32_t tbs = bcast<E>(X.T, bs);
  if (j0 < 0 || j0 > be) {
    // the block lost every leaf: keep a placeholder
#pragma unroll
    for (int j = 0; j < E; j++)
      if (base + j == bs) {
        drop[j] = false;
        X.R.len[j] = 0;
        X.R.rseq[j] = kPad;
        X.R.rmask[j] = 0;
        X.R.meta[j] = 0;
        X.T[j] = (tbs & (kTH | kTNs)) | kTEmpty;
      }
  } else if (j0 != bs) {
#pragma unroll
    for (int j = 0; j < E; j++)
      if (base + j == j0) X.T[j] = (X.T[j] & ~(kTH | kTNs)) | (tbs & (kTH | kTNs));
  }
  bool keep[E];
#pragma unroll
  for (int j = 0; j < E; j++) keep[j] = !drop[j];
  return compact_slots<E, K>(X, keep, n, zlds);
}

// group starts of re-packed children: rank r starts a group of the
// base + 1 / base split (packParent, mergeTree.ts:764-786)
__device__ __forceinline__ bool group_start(int r, int base, int rem) {
  const int big = rem * (base + 1);
  if (r < big) return r % (base + 1) == 0;
  return (r - big) % base == 0;
}

// packParent of the level-p block starting at s (titems.c pack_parent)
template <int E, int K>
__device__ __forceinline__ int pack_parent(TReg<E, K>& X, int s, int p, int n, int32_t min_seq, TreeRun& tr, uint32_t* zlds,
                           int n_keys, int& status) {
  const int base = lane_id() * E;
  for (;;) {
    int e = span_end<E>(X.T, s, p, n);
    const uint32_t top = t_h(bcast<E>(X.T, s));
    if (p == 2) {
      bool drop[E];
#pragma unroll
      for (int j = 0; j < E; j++) drop[j] = false;
      for (int b = s; b <= e;) {
        const int be = span_end<E>(X.T, b, 1, n);
        scour<E, K>(X, b, be, n, min_seq, drop, tr, n_keys, zlds);
        b = be + 1;
      }
      // held leaves (placeholders go too), re-packed
      bool keep[E];
#pragma unroll
      for (int j = 0; j < E; j++) {
        const int i = base + j;
        keep[j] = !(i >= s && i <= e && (drop[j] || (X.T[j] & kTEmpty)));
        if (i >= s && i <= e) X.T[j] &= ~kTH;
      }
      const int n0 = n;
      n = compact_slots<E, K>(X, keep, n, zlds);
      e -= n0 - n;
      if (e < s) {
        // no leaf left: one empty leaf block
        if (n + 2 > E * kWave) {
          status = MTE_E_CAPACITY;
          return n;
        }
        open_slot<E, K>(X, s);
#pragma unroll
        for (int j = 0; j < E; j++)
          if (base + j == s) {
            X.R.len[j] = 0;
            X.R.rseq[j] = kPad;
            X.R.rmask[j] = 0;
            X.R.meta[j] = 0;
            X.T[j] = top | kTEmpty;
          }
        n++;
      } else {
        bool hd[E];
#pragma unroll
        for (int j = 0; j < E; j++) hd[j] = (X.T[j] & kTCont) == 0;
        const int total = count_where<E>(hd, s, e);
        int cc = total / (kMaxNodes / 2) < kMaxNodes - 1 ? total / (kMaxNodes / 2) : kMaxNodes - 1;
        if (cc < 1) cc = 1;
        const int gb = total / cc, rem = total % cc;
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < E; j++) cnt += (hd[j] && base + j >= s && base + j <= e) ? 1 : 0;
        const int incl = wave_incl_scan(cnt);
        int r = incl - cnt;
#pragma unroll
        for (int j = 0; j < E; j++) {
          const int i = base + j;
          if (hd[j] && i >= s && i <= e) {
            if (group_start(r, gb, rem)) X.T[j] = (X.T[j] & ~(kTH | kTNs)) | (r == 0 ? top : 1u);
            r++;
          }
        }
      }
    } else {
      // level p >= 3: the level-(p-2) blocks regrouped under new level-(p-1) blocks
      bool ch[E];
#pragma unroll
      for (int j = 0; j < E; j++) ch[j] = (int)t_h(X.T[j]) >= p - 2;
      const int total = count_where<E>(ch, s, e);
      int cc = total / (kMaxNodes / 2) < kMaxNodes - 1 ? total / (kMaxNodes / 2) : kMaxNodes - 1;
      if (cc < 1) cc = 1;
      const int gb = total / cc, rem = total % cc;
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < E; j++) cnt += (ch[j] && base + j >= s && base + j <= e) ? 1 : 0;
      const int incl = wave_incl_scan(cnt);
      int r = incl - cnt;
#pragma unroll
      for (int j = 0; j < E; j++) {
        const int i = base + j;
        if (ch[j] && i >= s && i <= e) {
          const uint32_t h = group_start(r, gb, rem) ? (r == 0 ? top : (uint32_t)(p - 1)) : (uint32_t)(p - 2);
          X.T[j] = (X.T[j] & ~kTH) | h;
          r++;
        }
      }
    }
    // the parent's own children: an underflow re-packs its parent too
    if (p >= tr.depth) return n;
    bool ch[E];
    child_pred<E>(X.T, p, ch);
    const int cc = count_where<E>(ch, s, span_end<E>(X.T, s, p, n));
    if (cc >= kMaxNodes / 2) return n;
    s = span_start<E>(X.T, s, p + 1);
    p++;
  }
}

// zamboniSegments (titems.c zamboni): at most two scours
template <int E, int K>
__device__ __forceinline__ int zamboni(TReg<E, K>& X, int n, int32_t min_seq, TreeRun& tr, uint32_t* zlds, int n_keys,
                       int& status) {
  for (int z = 0; z < 2; z++) {
    if (tr.hn == 0) break;
    const uint2 top = hp_get(tr.hp, 1);
    if ((int32_t)top.x > min_seq) break;
    const uint2 ent = heap_pop(tr);
    bool hit[E];
    const int base = lane_id() * E;
#pragma unroll
    for (int j = 0; j < E; j++) hit[j] = base + j < n && t_id(X.T[j]) == ent.y && (X.T[j] & (kTCont | kTEmpty)) == 0;
    const int i = first_where<E>(hit, 0);
    if (i < 0) continue;  // unlinked
    const int bs = span_start<E>(X.T, i, 1), be = span_end<E>(X.T, bs, 1, n);
    if (t_ns(bcast<E>(X.T, bs)) == kNsFalse) continue;
    bool ch[E];
    child_pred<E>(X.T, 1, ch);
    const int before = count_where<E>(ch, bs, be);
    bool drop[E];
#pragma unroll
    for (int j = 0; j < E; j++) drop[j] = false;
    const int held = scour<E, K>(X, bs, be, n, min_seq, drop, tr, n_keys, zlds);
    set_ns<E>(X.T, bs, kNsFalse);
    if (held < before) {
      n = drop_block<E, K>(X, bs, be, drop, n, zlds);
      if (held < kMaxNodes / 2 && tr.depth >= 2)
        n = pack_parent<E, K>(X, span_start<E>(X.T, bs, 2), 2, n, min_seq, tr, zlds, n_keys, status);
      if (status) return n;
    }
  }
  return n;
}

// ensureIntervalBoundary (titems.c boundary); returns the new item count
template <int E, int K, bool S>
__device__ __forceinline__ int tree_boundary(TReg<E, K>& X, const int32_t (&L)[E], const int32_t (&P)[E], int32_t pos, int n,
                             TreeRun& tr, uint32_t (&st)[kNumStats], bool& changed) {
  int32_t off = 0;
  const int xs = find_split<E>(L, P, pos, &off);
  const int base = lane_id() * E;
  if (xs >= 0) {
    const int32_t len = bcast<E>(X.R.len, xs);
    open_slot<E, K>(X, xs + 1);
    const uint32_t id = tr.next_id++;
#pragma unroll
    for (int j = 0; j < E; j++) {
      const int i = base + j;
      if (i == xs) X.R.len[j] = off;
      if (i == xs + 1) {
        X.R.len[j] = len - off;
        X.R.toff[j] += (uint32_t)off;
        X.T[j] = (X.T[j] & (kTPo | kTNl)) | (id << 8);
      }
    }
    n++;
    TSTAT(st[kStWritten] += 2;)
    split_cascade<E>(X.T, xs + 1, n, tr);
    changed = true;
    return n;
  }
  // between two texts of one merged leaf
  bool c[E];
#pragma unroll
  for (int j = 0; j < E; j++) c[j] = (X.T[j] & kTCont) && L[j] > 0 && P[j] == pos;
  const int ic = first_where<E>(c, 0);
  if (ic >= 0) {
    const uint32_t id = tr.next_id++;
#pragma unroll
    for (int j = 0; j < E; j++)
      if (base + j == ic) X.T[j] = (X.T[j] & (kTPo | kTNl)) | (id << 8);
    TSTAT(st[kStWritten] += 1;)
    split_cascade<E>(X.T, ic, n, tr);
    changed = true;
  }
  return n;
}

// op record k through vector loads: dword i in lane i < 8 (vmcnt, not lgkmcnt)
__device__ __forceinline__ uint32_t vload_rec(const uint4* rec) {
  const int l = lane_id();
  return l < 8 ? reinterpret_cast<const uint32_t*>(rec)[l] : 0u;
}

// One op record of a legacy document (titems.c doc_apply).  Returns 0, 1 (the
// document needs the next register tier) or a negative MTE_E_*.
template <int E, int K, bool S>
__device__ __forceinline__ int tree_step(TReg<E, K>& X, DocRun& D, TreeRun& tr, uint32_t (&st)[kNumStats],
                                         uint32_t& cur, const ReplayArgs& a, uint32_t* zlds) {
  const int base = lane_id() * E;
  const int lim = kWave * E < (int)a.cap ? kWave * E : (int)a.cap;
  if (D.n + 4 > lim) return 1;
  if (tr.next_id + 4 >= kIdLimit) return MTE_E_CAPACITY;
  s8v op;
#pragma unroll
  for (int i = 0; i < 8; i++) op[i] = (int32_t)rdlane(cur, i);
  cur = vload_rec(D.recp + 2 * (D.k + 1));  // the next record (zeroed pad after the last)
  const uint32_t w3 = (uint32_t)op[3];
  const uint32_t type = w3 & 0xffu, c = (w3 >> 8) & 0xffu, flags = w3 >> 16;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  TSTAT(st[kStOps]++;)
  TSTAT(st[kStMaxSegs] = (uint32_t)D.n > st[kStMaxSegs] ? (uint32_t)D.n : st[kStMaxSegs];)
  const int32_t s = op[0], r = op[1], msn = op[2];
  const int32_t pos1 = op[4], pos2 = op[5];
  int n = D.n;
  int status = 0;
  const bool newcalc = (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  [[maybe_unused]] uint64_t tq0 = 0, tq1 = 0, tq2 = 0, tq3 = 0;
  TPROF(tq0 = wall_clock64(); tq1 = tq2 = tq3 = tq0;)

  if (type == MTE_OP_INSERT || type == MTE_OP_REMOVE || type == MTE_OP_ANNOTATE) {
    TSTAT(st[kStScanned] += (uint32_t)n;)
    int32_t L[E], P[E];
    leaf_lengths<E, K>(X.R, r, c + 1, (int)c, D.min_seq, newcalc, L);
    int32_t total = prefix<E>(L, P);
    bool changed = false;
    n = tree_boundary<E, K, S>(X, L, P, pos1, n, tr, st, changed);
    if (type != MTE_OP_INSERT) {
      if (changed) {
        leaf_lengths<E, K>(X.R, r, c + 1, (int)c, D.min_seq, newcalc, L);
        total = prefix<E>(L, P);
        changed = false;
      }
      n = tree_boundary<E, K, S>(X, L, P, pos2, n, tr, st, changed);
    }
    if (changed) {
      leaf_lengths<E, K>(X.R, r, c + 1, (int)c, D.min_seq, newcalc, L);
      total = prefix<E>(L, P);
    }
    TPROF(tq1 = wall_clock64();)
    if (type == MTE_OP_INSERT) {
      const bool marker = (flags & MTE_F_MARKER) != 0;
      const int32_t nlen = marker ? 1 : pos2;
      if (nlen > 0) {
        // the leaf block insertingWalk enters: the first whose end reaches pos
        bool q[E];
#pragma unroll
        for (int j = 0; j < E; j++) q[j] = base + j < n && P[j] + (L[j] > 0 ? L[j] : 0) >= pos1;
        const int ks = first_where<E>(q, 0);
        if (ks < 0 || pos1 > total) return MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
        const int bs = span_start<E>(X.T, ks, 1), be = span_end<E>(X.T, bs, 1, n);
        const uint32_t tbs = bcast<E>(X.T, bs);
        int slot;
        bool replace = false;
        if (tbs & kTEmpty) {
          slot = bs;
          replace = true;
        } else {
          bool f[E];
#pragma unroll
          for (int j = 0; j < E; j++) f[j] = L[j] >= 0 && P[j] >= pos1 && !(X.T[j] & kTEmpty);
          slot = first_where<E>(f, ks);
          if (slot < 0 || slot > be) slot = be + 1;
        }
        // the new segment (mergeTree.ts:1599-1611, textSegment.ts:40-48, mergeTreeNodes.ts:602-609)
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
          TSTAT(st[kStPwrites] += (uint32_t)q2[3];)
        }
        TSTAT(if (!marker) st[kStUnits] += (uint32_t)pos2;)
        TSTAT(st[kStWritten] += 1;)
        const uint32_t id = tr.next_id++;
        uint32_t tw = (id << 8) | (psi != MTE_NO_PROPS ? kTPo : 0u) | ((flags & kRecNl) ? kTNl : 0u);
        if (replace) {
          tw |= tbs & (kTH | kTNs);
        } else {
          open_slot<E, K>(X, slot);
          n++;
          if (slot == bs) {  // the new leaf becomes the block's first child
            tw |= tbs & (kTH | kTNs);
#pragma unroll
            for (int j = 0; j < E; j++)
              if (base + j == slot + 1) X.T[j] &= ~(kTH | kTNs);
          }
        }
#pragma unroll
        for (int j = 0; j < E; j++) {
          if (base + j != slot) continue;
          X.R.len[j] = nlen;
          X.R.seq[j] = s;
          X.R.rseq[j] = kNone;
          X.R.rmask[j] = 0;
          X.R.meta[j] = meta;
          X.R.toff[j] = toff;
#pragma unroll
          for (int kk = 0; kk < K; kk++) X.R.pr[kk][j] = pr[kk][0];
          X.T[j] = tw;
        }
        if (!replace) split_cascade<E>(X.T, slot, n, tr);
        const int rc = add_lru<E>(X.T, slot, s, D.cur_seq, tr);
        if (rc) return rc;
      }
    } else if (pos2 != pos1) {
      // nodeMap over [start, end) (mergeTree.ts:2274-2330)
      bool in[E];
      uint32_t cnt = 0;
#pragma unroll
      for (int j = 0; j < E; j++) {
        in[j] = L[j] > 0 && P[j] >= pos1 && P[j] < pos2;
        cnt += (uint32_t)__popcll(__ballot(in[j]));
      }
      TSTAT(st[kStWritten] += cnt;)
      if (type == MTE_OP_REMOVE) {
        const uint32_t bit = 1u << c;
#pragma unroll
        for (int j = 0; j < E; j++) {
          X.R.rseq[j] = (in[j] && X.R.rseq[j] == kNone) ? s : X.R.rseq[j];
          X.R.rmask[j] = in[j] ? (X.R.rmask[j] | bit) : X.R.rmask[j];
        }
      } else if (cnt > 0) {
        const uint32_t psi = (uint32_t)op[6];
        const s8v q2 = sload_props(a, psi);
        if (flags & MTE_F_REWRITE) {
#pragma unroll
          for (int kk = 0; kk < K; kk++)
#pragma unroll
            for (int j = 0; j < E; j++) X.R.pr[kk][j] = in[j] ? 0u : X.R.pr[kk][j];
        }
        apply_props<E, K>(X.R.pr, in, (uint32_t)q2[0], (uint32_t)q2[1], (uint32_t)q2[2], psi, a);
#pragma unroll
        for (int j = 0; j < E; j++) X.T[j] |= in[j] ? kTPo : 0u;
        TSTAT(st[kStPwrites] += cnt * (uint32_t)q2[3];)
      }
      // addToLRUSet for every touched leaf: the first one of each leaf block
      bool th[E];
#pragma unroll
      for (int j = 0; j < E; j++) th[j] = in[j] && (X.T[j] & kTCont) == 0;
      for (int i = first_where<E>(th, 0); i >= 0;) {
        const int rc = add_lru<E>(X.T, i, s, D.cur_seq, tr);
        if (rc) return rc;
        const int be = span_end<E>(X.T, span_start<E>(X.T, i, 1), 1, n);
        i = first_where<E>(th, be + 1);
      }
    }
    TPROF(tq2 = wall_clock64();)
    n = zamboni<E, K>(X, n, D.min_seq, tr, zlds, a.n_keys, status);
    TPROF(tq3 = wall_clock64();)
    if (status) return status;
  } else if (type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  D.n = n;
  D.k++;
  const bool live = type != MTE_OP_NOOP, end = (flags & MTE_F_MSG_END) != 0;
  const bool bad = (live & (s <= D.cur_seq)) | (end & (s < D.cur_seq)) | ((live | end) & (msn < D.min_seq)) |
                   (end & (msn > s));
  if (bad) return window_error(D, live, end, s, msn);
  if (end) {
    D.cur_seq = s;
    if (msn > D.min_seq) {
      D.min_seq = msn;
      [[maybe_unused]] uint64_t tz = 0;
      TPROF(tz = wall_clock64();)
      D.n = zamboni<E, K>(X, D.n, D.min_seq, tr, zlds, a.n_keys, status);
      TPROF(st[kStMaxSegs] += (uint32_t)(wall_clock64() - tz);)
      if (status) return status;
    }
  }
  TPROF(st[kStScanned] += (uint32_t)(tq1 - tq0); st[kStWritten] += (uint32_t)(tq2 - tq1);
        st[kStPwrites] += (uint32_t)(tq3 - tq2); st[kStUnits] += (uint32_t)(wall_clock64() - tq0);)
  return 0;
}

template <int E, int K>
__device__ __forceinline__ void tree_load(TReg<E, K>& X, const DocRun& D, const ReplayArgs& a, const TreeArgs& t) {
  load_regs<E, K>(X.R, D, a);
  const uint32_t* tp = t.tree + (uint64_t)D.doc * a.cap;
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) X.T[j] = base + j < D.n ? tp[base + j] : 0u;
}

template <int E, int K>
__device__ __forceinline__ void tree_store(const TReg<E, K>& X, const DocRun& D, const ReplayArgs& a,
                                           const TreeArgs& t) {
  store_regs<E, K>(X.R, D, a);
  uint32_t* tp = t.tree + (uint64_t)D.doc * a.cap;
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++)
    if (base + j < D.n) tp[base + j] = X.T[j];
}

// one run of a legacy document at tier E: until it ends, stops or needs
// another tier
template <int E, int K, bool S>
__device__ __forceinline__ void tree_burst(DocRun& D, TreeRun& tr, const ReplayArgs& a, const TreeArgs& t, uint32_t* zlds,
                           int emin) {
  TReg<E, K> X;
  uint32_t st[kNumStats] = {};
  tree_load<E, K>(X, D, a, t);
  uint32_t cur = vload_rec(D.recp + 2 * D.k);
  for (;;) {
    const int rc = tree_step<E, K, S>(X, D, tr, st, cur, a, zlds);
    if (rc < 0) {
      D.status = rc;
      D.running = false;
      break;
    }
    if (rc > 0) break;  // needs the next tier
    if (D.k >= D.k1) {
      D.running = false;
      break;
    }
    if (E > emin && D.n + 4 + 16 <= 32 * E) break;  // fits the tier below
    if constexpr (S) {
      if (st[kStOps] >= (1u << 20)) {
        run_flush_stats(D, st, a);
      }
    }
  }
  tree_store<E, K>(X, D, a, t);
  if constexpr (S) run_flush_stats(D, st, a);
}

// The tree pass.  A kernel's register allocation is that of its largest tier,
// so the tiers are separate kernels: TIER 0 runs E = 1, 2 (documents up to 124
// items, bounded to MTE_TREE0_WAVES waves per SIMD), TIER 1 E = 4 (up to 252
// items, ~225 VGPRs: 2 waves), TIER 2 E = 8, 16 (up to 1,020 items).  A document that
// outgrows TIER 0 is flagged kHdrTreeEsc and continues in the TIER 1 launch
// that follows; one that shrinks back (20 items of slack) returns to the next
// TIER 0 launch, so a passing peak does not keep it at low occupancy for the
// rest of the batch.  The host alternates TIER 0 / TIER 1 a few rounds (the
// last TIER 1 keeps its documents), then runs TIER 2 (kHdrTreeBig) once.
// TIER 0's register budget in waves per SIMD (5: 96 VGPRs, 40 spilled).  It
// decides how many of a batch's documents are resident at once: config 3's
// 5,000 legacy documents (one wave each) fit the chip's 1,024 SIMDs at five
// waves, but not at four, where the last 904 start only as the first finish --
// 82.5 -> 68.6 ms per step, digests unchanged (round 6)
#ifndef MTE_TREE0_WAVES
#define MTE_TREE0_WAVES 5
#endif
#ifndef MTE_TREE1_WAVES  // TIER 1's (1: no bound, 224 VGPRs = 2 waves per SIMD)
#define MTE_TREE1_WAVES 1
#endif
template <int K, bool S, int TIER>
__global__ __launch_bounds__(256, TIER == 0 ? MTE_TREE0_WAVES : TIER == 1 ? MTE_TREE1_WAVES : 1) void tree_kernel(
    ReplayArgs a, TreeArgs t) {
  constexpr int EMAX = TIER == 2 ? 16 : TIER == 1 ? 4 : 2;
  constexpr uint32_t kTierFlags = kHdrTreeEsc | kHdrTreeBig | kHdrTreeHbmFlag;
  __shared__ uint32_t zlds_all[kDocsPerBlock][kWave * EMAX];
  __shared__ __attribute__((aligned(16))) uint2 heap_all[kDocsPerBlock][kTreeHeapCap + 1];
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int idx = (int)blockIdx.x * kDocsPerBlock + w;
  if (idx >= (int)t.n_docs) return;
  const int doc = uni((int)t.docs[idx]);
  const uint4 h0 = reinterpret_cast<const uint4*>(a.hdr + doc)[0], h1 = reinterpret_cast<const uint4*>(a.hdr + doc)[1];
  const uint32_t hflags = uni(h1.x);
  if (TIER == 0 && (hflags & kTierFlags)) return;
  if (TIER == 1 && (hflags & kTierFlags) != kHdrTreeEsc) return;
  if (TIER == 2 && !(hflags & kHdrTreeBig)) return;
  DocRun D;
  D.doc = doc;
  D.n = uni((int32_t)h0.x);
  D.min_seq = uni((int32_t)h0.y);
  D.cur_seq = uni((int32_t)h0.z);
  D.status = uni((int32_t)h0.w);
  D.flags = hflags & ~kTierFlags;
  D.k = uni(h1.y);
  const uint64_t kb = uni64(a.op_off[doc]);
  D.recp = a.recs + 2 * kb;
  D.k1 = (uint32_t)(uni64(a.op_off[doc + 1]) - kb);
  if (TIER < 2 && D.k1 > t.k_cap) D.k1 = t.k_cap;  // the round's share of the batch
  D.running = D.status == 0 && D.k < D.k1;
  if (!D.running) return;
  TreeRun tr;
  tr.depth = (int)uni(h1.w & 0xffu);
  tr.hn = uni(h1.w >> 8);
  tr.next_id = uni(h1.z);
  tr.hp = heap_all[w];
  tr.arena = t.arena;
  const uint2* hg = t.heap + (uint64_t)doc * (kTreeHeapCap + 1);
  for (uint32_t k = (uint32_t)lane_id(); k <= tr.hn; k += kWave) {
    const uint2 v = hg[k];
    tr.hp[k].x = v.x;
    tr.hp[k].y = v.y;
  }
  fence_wave();
  uint32_t* zlds = zlds_all[w];
  while (D.running) {
    const int n = D.n;
    if (n + 4 > (int)a.cap) {
      D.status = MTE_E_CAPACITY;
      break;
    }
    if (n + 4 > 16 * kWave) {  // past the registers: the HBM tree pass goes on (mte_htree.h)
      D.flags |= kHdrTreeHbmFlag;
      break;
    }
    if constexpr (TIER == 0) {
      if (n + 4 <= kWave) tree_burst<1, K, S>(D, tr, a, t, zlds, 1);
      else if (n + 4 <= 2 * kWave) tree_burst<2, K, S>(D, tr, a, t, zlds, 1);
      else {
        D.flags |= kHdrTreeEsc;
        break;
      }
    } else if constexpr (TIER == 1) {
      if (n + 4 > 4 * kWave) {
        D.flags |= kHdrTreeBig;
        break;
      }
      if (!t.final_round && n + 4 + 16 <= 2 * kWave) break;  // back to TIER 0
      tree_burst<4, K, S>(D, tr, a, t, zlds, t.final_round ? 4 : 2);
    } else {
      if (n + 4 <= 8 * kWave) tree_burst<8, K, S>(D, tr, a, t, zlds, 8);
      else tree_burst<16, K, S>(D, tr, a, t, zlds, 8);
    }
  }
  uint2* hw = t.heap + (uint64_t)doc * (kTreeHeapCap + 1);
  fence_wave();
  for (uint32_t k = (uint32_t)lane_id(); k <= tr.hn; k += kWave) hw[k] = make_uint2(tr.hp[k].x, tr.hp[k].y);
  if (lane_id() == 0) {
    DocHdr o;
    o.nseg = D.n;
    o.min_seq = D.min_seq;
    o.cur_seq = D.cur_seq;
    o.status = D.status;
    o.flags = D.flags;
    o.resume = D.k;
    o.pad0 = tr.next_id;
    o.pad1 = (uint32_t)tr.depth | (tr.hn << 8);
    a.hdr[doc] = o;
  }
}

}  // namespace mte
