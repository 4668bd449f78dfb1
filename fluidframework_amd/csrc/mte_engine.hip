// mte_engine.hip — C-ABI (include/mte.h) + gfx950 kernels of the batched
// sequence-merge engine.  See DESIGN.md for the data layout and the mapping
// to the reference (packages/dds/merge-tree/src).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>
#include <atomic>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "mte_kernels.h"
#include "mte_replay.h"
#include "mte_stream.h"
#include "mte_chunk.h"

namespace mte {
}  // namespace mte
#include "mte_tree.h"
#include "mte_htree.h"
#include "mte_passes.h"

#include <rccl/rccl.h>

using namespace mte;

namespace {

// reset resume/escalation flags and stats at the start of a batch
__global__ void begin_batch_kernel(DocHdr* hdr, unsigned long long* stats, uint32_t n_docs,
                                   unsigned long long* gdone) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d == 0) *gdone = 0;
  if (d >= n_docs) return;
  hdr[d].resume = 0;
  hdr[d].flags &= ~(kHdrNeedsEsc | kHdrTreeEsc | kHdrTreeBig | kHdrRel);
#pragma unroll
  for (int t = 0; t < kNumStats; t++) stats[(size_t)d * kNumStats + t] = 0;
}

// MTE_DOC_ROUND_SYNC check (include/mte.h; oracle.c round_sync_ok): one wave
// per declared legacy document, 64 records per step.  A live record violates
// the declaration when its refSeq is below the highest refSeq so far, or above
// it but below the highest live seq so far; both maxima are exclusive wave
// max-scans continued from the header (pad0 = highest refSeq, pad1 = highest
// live seq, the load's currentSeq to start with).  A violation stops the
// document before any op of the batch.
__device__ __forceinline__ int32_t dpp_max(int32_t v, int32_t x) { return v > x ? v : x; }
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ int32_t dppm(int32_t v) {
  return __builtin_amdgcn_update_dpp(INT32_MIN, v, CTRL, ROWMASK, 0xf, false);
}
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
  v = dpp_max(v, dppm<kRowShr1>(v));
  v = dpp_max(v, dppm<kRowShr2>(v));
  v = dpp_max(v, dppm<kRowShr4>(v));
  v = dpp_max(v, dppm<kRowShr8>(v));
  v = dpp_max(v, dppm<kRowBcast15, 0xa>(v));
  v = dpp_max(v, dppm<kRowBcast31, 0xc>(v));
  return v;
}

__global__ __launch_bounds__(256) void round_sync_kernel(DocHdr* hdr, const uint4* recs, const uint64_t* op_off,
                                                         const uint32_t* docs, uint32_t n) {
  const uint32_t w = blockIdx.x * 4 + threadIdx.x / kWave;
  if (w >= n) return;
  const int doc = (int)uni(docs[w]);
  const int l = lane_id();
  if (uni(hdr[doc].status) != 0) return;
  int32_t ref = (int32_t)uni(hdr[doc].pad0), seq = (int32_t)uni(hdr[doc].pad1);
  const uint64_t k0 = op_off[doc], k1 = op_off[doc + 1];
  bool bad = false;
  for (uint64_t k = k0; k < k1 && !bad; k += kWave) {
    const bool in = k + (uint64_t)l < k1;
    const uint4 w0 = in ? recs[2 * (k + (uint64_t)l)] : make_uint4(0u, 0u, 0u, (uint32_t)MTE_OP_NOOP);
    const uint32_t ty = w0.w & 0xffu;
    const bool live = in && ty != MTE_OP_NOOP && ty != MTE_OP_RELPOS;  // RELPOS: seq / ref_seq are offsets
    const int32_t r = (int32_t)w0.y, sq = (int32_t)w0.x;
    // maxima over the live records before this one (exclusive scans)
    const int32_t rin = wave_incl_max(live ? r : INT32_MIN), sin = wave_incl_max(live ? sq : INT32_MIN);
    int32_t rb = (int32_t)__builtin_amdgcn_mov_dpp(rin, kWaveShr1, 0xf, 0xf, false);
    int32_t sb = (int32_t)__builtin_amdgcn_mov_dpp(sin, kWaveShr1, 0xf, 0xf, false);
    rb = l == 0 ? INT32_MIN : rb;
    sb = l == 0 ? INT32_MIN : sb;
    rb = dpp_max(rb, ref);
    sb = dpp_max(sb, seq);
    bad = __ballot(live && (r < rb || (r > rb && r < sb))) != 0;
    ref = dpp_max(ref, (int32_t)rdlane(rin, kWave - 1));
    seq = dpp_max(seq, (int32_t)rdlane(sin, kWave - 1));
  }
  if (l == 0) {
    if (bad) hdr[doc].status = MTE_E_UNSUPPORTED;
    else {
      hdr[doc].pad0 = (uint32_t)ref;
      hdr[doc].pad1 = (uint32_t)seq;
    }
  }
}

// Documents whose batch holds MTE_OP_RELPOS records (include/mte.h): the flat
// ones replay this batch on the HBM-streamed pass (kHdrRel: passes 1 and 2
// hand them on), the legacy tree ones move to the HBM tree pass for good
// (their state enters it as from TIER 2, mte_htree.h); the HBM tree pass's own
// already resolve them.  The chunked pass does not: MTE_E_UNSUPPORTED.
__global__ void rel_route_kernel(DocHdr* hdr, const uint32_t* docs, uint32_t n, int chunked) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DocHdr* h = hdr + docs[i];
  if (h->status != 0) return;
  const uint32_t f = h->flags;
  if (f & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) return;
  if (!(f & (MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_ROUND_SYNC))) {
    if (!(f & MTE_DOC_EVENTS)) h->flags = f | kHdrTreeHbmFlag;
    return;
  }
  if (chunked) h->status = MTE_E_UNSUPPORTED;
  else h->flags = f | kHdrRel | kHdrNeedsEsc;
}

// (re)initialise docs from their load description: one seq-0 LocalClientId
// text segment (client.replay.spec.ts:22-23)
// Legacy length-calc documents also carry the reference's B+tree (mte_tree.h):
// the load text is one leaf in the root leaf block (MergeTree starts with an
// empty root, mergeTree.ts:495-498; the replay harness's insertTextLocal adds
// one leaf), an empty document one placeholder; a loaded body has
// reloadFromSegments' blocks of 7 (image_kernel writes the tree words).
// device copy of mte_doc_init::flags: the load text holds a '\n' (engine-internal)
constexpr uint32_t kInitNl = 0x80000000u;

__global__ void reset_kernel(DocHdr* hdr, SegSoA soa, uint32_t cap, const mte_doc_init* inits,
                             const uint32_t* init_props, uint32_t n_keys, uint32_t n_docs,
                             const uint64_t* img_off, uint32_t* tree, uint32_t kt, uint32_t* hst) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_docs) return;
  const mte_doc_init in = inits[d];
  const uint32_t n_img = img_off ? (uint32_t)(img_off[d + 1] - img_off[d]) : 0u;
  const bool flat_legacy = (in.flags & (MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_ROUND_SYNC)) == MTE_DOC_ROUND_SYNC;
  // documents with the reference's tree: legacy ones (register tiers, then the
  // HBM tree pass) and the HBM tree pass's own (a local client, or legacy with
  // delta events)
  const bool legacy = tree != nullptr && (!(in.flags & (MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_ROUND_SYNC)) ||
                                          (in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)));
  DocHdr h;
  h.nseg = n_img ? (int32_t)n_img : (in.text_len > 0 || legacy ? 1 : 0);
  h.min_seq = in.min_seq;
  h.cur_seq = in.cur_seq;
  h.status = 0;
  h.flags = in.flags & (MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_ROUND_SYNC | MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS | MTE_DOC_REFS |
                        MTE_DOC_SLIDE_EVENTS | MTE_DOC_MAINT_EVENTS | MTE_DOC_TREE);
  h.resume = 0;
  h.pad0 = h.pad1 = 0;
  if (legacy) {
    int depth = 1;
    for (uint64_t w = 7; n_img && w < n_img; w *= 7) depth++;
    h.pad0 = n_img ? n_img + 1 : 2;  // next segment id
    h.pad1 = (uint32_t)depth;         // depth | heap size << 8
  }
  if (flat_legacy) {
    h.pad0 = (uint32_t)INT32_MIN;  // round-sync check: no refSeq yet
    h.pad1 = (uint32_t)in.cur_seq;  // every later increase must reach it
  }
  hdr[d] = h;
  if (hst) {  // the HBM tree pass's state (mte_htree.h): a legacy doc enters it from the register tiers
    uint32_t* st = hst + (uint64_t)d * kHtState;
    st[kHsDepth] = h.pad1 & 0xffu;
    st[kHsNextId] = h.pad0;
    st[kHsHeapN] = 0u;
    st[kHsLseq] = 0u;
    st[kHsRhi] = 0u;
    st[kHsEntered] = (in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) ? 1u : 0u;
    st[kHsWin] = 0u;  // no cached local partials
  }
  if (in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) {  // nothing pending, no removers >= 32 (mte_htree.h planes)
    const uint32_t nz = n_img ? n_img : 1u;
    for (uint32_t k = 0; k < 2 * kt + 6; k++)  // the local planes (mte_htree.h kLocalPlanes)
      for (uint32_t x = 0; x < nz; x++) soa.props[(kt + k) * soa.plane_stride + (uint64_t)d * cap + x] = 0u;
  }
  if (n_img) return;  // image_kernel writes the segments
  const uint64_t i = (uint64_t)d * cap;
  soa.len[i] = (int32_t)in.text_len;
  soa.seq[i] = 0;
  soa.rseq[i] = (legacy && in.text_len == 0) ? kPad : kNone;
  soa.rmask[i] = 0;
  soa.meta[i] = 0;  // clientId -1, text
  soa.toff[i] = in.text_off;
  uint32_t po = 0;
  for (uint32_t k = 0; k < n_keys; k++) soa.props[k * soa.plane_stride + i] = init_props[(size_t)d * MTE_MAX_KEYS + k];
  if (in.propset != MTE_NO_PROPS) po = kTPo;
  if (legacy) tree[i] = in.text_len > 0 ? (1u | po | (1u << 8) | ((in.flags & kInitNl) ? kTNl : 0u)) : (1u | kTEmpty);
}

// the image planes that hold one value for every segment (found at load):
// written from the kernel argument instead of read back each reset
struct ImgConst {
  uint32_t mask;     // bit p: plane p is uniform
  uint32_t val[16];  // its value
};

// the mte_load_segments image -> the flat planes (one thread per segment)
// (the image's last plane is the tree word, for the tree pass)
__global__ void image_kernel(SegSoA soa, uint32_t cap, uint32_t n_planes, const uint32_t* img, uint64_t img_stride,
                             const uint32_t* img_doc, const uint64_t* img_off, uint64_t n_img, uint32_t* tree,
                             ImgConst uc) {
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_img;
       g += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = img_doc[g];
    const uint64_t x = (uint64_t)d * cap + (g - img_off[d]);
    uint32_t* pl = reinterpret_cast<uint32_t*>(soa.len);
    for (uint32_t p = 0; p < n_planes; p++)
      pl[p * soa.plane_stride + x] = ((uc.mask >> p) & 1u) ? uc.val[p] : img[p * img_stride + g];
    if (tree) tree[x] = img[n_planes * img_stride + g];
  }
}

// Compile the batch's property sets into the 32-byte records the replay
// kernels fetch with one scalar load (mte_kernels.h): the first two entries
// inlined, the count of keys < n_keys.  One thread per set; runs at the start
// of every mte_run (inside the timed region).
__global__ void props_kernel(const mte_propset* __restrict__ ps, uint32_t n_ps, const mte_prop* __restrict__ pe,
                             uint32_t n_keys, uint4* __restrict__ cps) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ps) return;
  const mte_propset s = ps[i];
  uint32_t k0 = kNoKey, k1 = kNoKey, v0 = 0, v1 = 0, nw = 0;
  for (uint32_t t = 0; t < s.count; t++) {
    const mte_prop p = pe[s.first + t];
    const bool ok = p.key < n_keys;
    nw += ok ? 1u : 0u;
    if (t == 0) {
      k0 = ok ? p.key : kNoKey;
      v0 = p.value;
    } else if (t == 1) {
      k1 = ok ? p.key : kNoKey;
      v1 = p.value;
    }
  }
  cps[2 * i] = make_uint4(k0 | (k1 << 8) | ((s.count > 2 ? 1u : 0u) << 16), v0, v1, nw);
  cps[2 * i + 1] = make_uint4(0, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// digest (DESIGN.md "Digest"): H = sum_p x_p * B^(n-1-p) mod 2^61-1
// ---------------------------------------------------------------------------
constexpr uint64_t kM61 = (1ull << 61) - 1;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fold61(uint64_t x) {
  uint64_t r = (x & kM61) + (x >> 61);
  return r >= kM61 ? r - kM61 : r;
}
__device__ __forceinline__ uint64_t mulmod61(uint64_t a, uint64_t b) {
  const uint64_t lo = a * b;
  const uint64_t hi = __umul64hi(a, b);
  uint64_t r = (lo & kM61) + ((hi << 3) | (lo >> 61));
  r = (r & kM61) + (r >> 61);
  return r >= kM61 ? r - kM61 : r;
}
__device__ __forceinline__ uint64_t addmod61(uint64_t a, uint64_t b) {
  uint64_t r = a + b;
  return r >= kM61 ? r - kM61 : r;
}
__device__ __forceinline__ uint64_t powmod61(const uint64_t* tab, uint32_t e) {
  uint64_t r = 1;
  for (int i = 0; e; i++, e >>= 1)
    if (e & 1u) r = mulmod61(r, tab[i]);
  return r;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
  return ((uint64_t)hi << 32) | lo;
}

struct DigestArgs {
  const DocHdr* hdr;
  SegSoA soa;
  uint32_t cap;
  uint32_t n_keys;
  uint32_t n_docs;
  const uint16_t* arena;
  const uint64_t* pow1;  // B1^(2^i), i < 32
  const uint64_t* pow2;
  uint64_t* out;
};

__global__ __launch_bounds__(256) void digest_kernel(DigestArgs a) {
  const int w = threadIdx.x / kWave;
  const int l = lane_id();
  const int doc = blockIdx.x * kDocsPerBlock + w;
  if (doc >= (int)a.n_docs) return;
  const int n = a.hdr[doc].nseg;
  const uint64_t db = (uint64_t)doc * a.cap;
  int32_t tot = 0;
  for (int c0 = 0; c0 < n; c0 += kWave) {
    const int i = c0 + l;
    const int32_t L = (i < n && a.soa.rseq[db + i] == kNone) ? a.soa.len[db + i] : 0;
    tot += rdlane(wave_incl_scan(L), kWave - 1);
  }
  uint64_t h1 = 0, h2 = 0, xs = 0;
  int32_t carry = 0;
  for (int c0 = 0; c0 < n; c0 += kWave) {
    const int i = c0 + l;
    const bool vis = i < n && a.soa.rseq[db + i] == kNone;
    const int32_t L = vis ? a.soa.len[db + i] : 0;
    const int32_t incl = wave_incl_scan(L);
    const int32_t P = carry + incl - L;
    uint64_t c1 = 0, c2 = 0, xl = 0;
    if (L > 0) {
      uint64_t ph = 0;
      for (uint32_t k = 0; k < a.n_keys; k++) {
        const uint32_t v = a.soa.props[k * a.soa.plane_stride + db + i];
        if (v) ph += mix64(((uint64_t)(k + 1) << 32) | v);
      }
      const uint32_t kind = a.soa.meta[db + i] >> 8;
      const uint32_t toff = a.soa.toff[db + i];
      uint64_t s1 = 0, s2 = 0;
      for (int32_t u = 0; u < L; u++) {
        const uint64_t rec = kind == 0 ? (uint64_t)a.arena[toff + (uint32_t)u] : ((1ull << 32) | (uint64_t)(kind - 1));
        const uint64_t x = fold61(mix64(rec * 0x9E3779B97F4A7C15ull + ph));
        s1 = addmod61(mulmod61(s1, a.pow1[0]), x);
        s2 = addmod61(mulmod61(s2, a.pow2[0]), x);
        xl += x;
      }
      const uint32_t e = (uint32_t)(tot - P - L);
      c1 = mulmod61(s1, powmod61(a.pow1, e));
      c2 = mulmod61(s2, powmod61(a.pow2, e));
    }
#pragma unroll
    for (int m = 1; m < kWave; m <<= 1) {
      c1 = addmod61(c1, shfl_xor64(c1, m));
      c2 = addmod61(c2, shfl_xor64(c2, m));
      xl += shfl_xor64(xl, m);
    }
    h1 = addmod61(h1, c1);
    h2 = addmod61(h2, c2);
    xs += xl;
    carry += rdlane(incl, kWave - 1);
  }
  if (l == 0) {
    a.out[4 * (size_t)doc + 0] = (uint64_t)tot;
    a.out[4 * (size_t)doc + 1] = h1;
    a.out[4 * (size_t)doc + 2] = h2;
    a.out[4 * (size_t)doc + 3] = xs;
  }
}

// ---- the digest of big documents, tile-parallel ------------------------------
// digest_kernel walks a document on one wave; a document of a million segments
// (config 5) is 16k rows of it.  Every segment's contribution depends only on
// its own units and its position P (c . B^(n - P - L)), so the same sums come
// from tiles of kDgTile segments on waves of their own: the tiles' visible
// lengths (dg_len_kernel), their prefix per document (dg_scan_kernel), each
// tile's contributions at those positions (dg_tile_kernel), the tiles' sums
// per document (dg_final_kernel).  Same value as digest_kernel, bit for bit.
constexpr int kDgTile = 4 * kWave;  // segments per tile (4 per lane, row-major like digest_kernel)
constexpr uint32_t kDgWaveMaxCap = 4096;  // contexts up to this capacity keep one wave per document

struct DigestTiles {
  uint32_t tpd;        // tiles per document (cap / kDgTile, rounded up)
  int32_t* tsum;       // [doc][tpd] visible length, then its exclusive prefix
  int32_t* tot;        // [doc] visible length of the document
  uint64_t* part;      // [doc][tpd][3] h1, h2, sum of x
};

__device__ __forceinline__ int32_t dg_vis_len(const DigestArgs& a, uint64_t db, int i, int n) {
  return (i < n && a.soa.rseq[db + i] == kNone) ? a.soa.len[db + i] : 0;
}

__global__ __launch_bounds__(256) void dg_len_kernel(DigestArgs a, DigestTiles t) {
  const int w = threadIdx.x / kWave, l = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
  const int doc = (int)(wi / t.tpd), tile = (int)(wi % t.tpd);
  if (doc >= (int)a.n_docs) return;
  const int n = a.hdr[doc].nseg;
  if (tile * kDgTile >= n) return;
  const uint64_t db = (uint64_t)doc * a.cap;
  int32_t v = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) v += dg_vis_len(a, db, tile * kDgTile + j * kWave + l, n);
  const int32_t s = rdlane(wave_incl_scan(v), kWave - 1);
  if (l == 0) t.tsum[(uint64_t)doc * t.tpd + tile] = s;
}

// one 256-thread workgroup per document: exclusive prefix of its tiles' lengths
__global__ __launch_bounds__(256) void dg_scan_kernel(DigestArgs a, DigestTiles t) {
  __shared__ int32_t wsum[4];
  __shared__ int32_t carry_s;
  const int doc = (int)blockIdx.x;
  const int w = threadIdx.x / kWave, l = lane_id();
  const int n = a.hdr[doc].nseg;
  const int m = (n + kDgTile - 1) / kDgTile;
  int32_t* ts = t.tsum + (uint64_t)doc * t.tpd;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int b = 0; b < m; b += 256) {
    const int i = b + (int)threadIdx.x;
    const int32_t v = i < m ? ts[i] : 0;
    const int32_t incl = wave_incl_scan(v);
    if (l == kWave - 1) wsum[w] = incl;
    __syncthreads();
    int32_t before = carry_s;
    for (int q = 0; q < w; q++) before += wsum[q];
    if (i < m) ts[i] = before + incl - v;
    __syncthreads();
    if (threadIdx.x == 0) carry_s += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) t.tot[doc] = carry_s;
}

__global__ __launch_bounds__(256) void dg_tile_kernel(DigestArgs a, DigestTiles t) {
  const int w = threadIdx.x / kWave, l = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
  const int doc = (int)(wi / t.tpd), tile = (int)(wi % t.tpd);
  if (doc >= (int)a.n_docs) return;
  const int n = a.hdr[doc].nseg;
  if (tile * kDgTile >= n) return;
  const uint64_t db = (uint64_t)doc * a.cap;
  const int32_t tot = t.tot[doc];
  int32_t carry = t.tsum[(uint64_t)doc * t.tpd + tile];
  uint64_t h1 = 0, h2 = 0, xs = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int i = tile * kDgTile + j * kWave + l;
    const int32_t L = dg_vis_len(a, db, i, n);
    const int32_t incl = wave_incl_scan(L);
    const int32_t P = carry + incl - L;
    if (L > 0) {
      uint64_t ph = 0;
      for (uint32_t k = 0; k < a.n_keys; k++) {
        const uint32_t v = a.soa.props[k * a.soa.plane_stride + db + i];
        if (v) ph += mix64(((uint64_t)(k + 1) << 32) | v);
      }
      const uint32_t kind = a.soa.meta[db + i] >> 8;
      const uint32_t toff = a.soa.toff[db + i];
      uint64_t s1 = 0, s2 = 0;
      for (int32_t u = 0; u < L; u++) {
        const uint64_t rec = kind == 0 ? (uint64_t)a.arena[toff + (uint32_t)u] : ((1ull << 32) | (uint64_t)(kind - 1));
        const uint64_t x = fold61(mix64(rec * 0x9E3779B97F4A7C15ull + ph));
        s1 = addmod61(mulmod61(s1, a.pow1[0]), x);
        s2 = addmod61(mulmod61(s2, a.pow2[0]), x);
        xs += x;
      }
      const uint32_t e = (uint32_t)(tot - P - L);
      h1 = addmod61(h1, mulmod61(s1, powmod61(a.pow1, e)));
      h2 = addmod61(h2, mulmod61(s2, powmod61(a.pow2, e)));
    }
    carry += rdlane(incl, kWave - 1);
  }
#pragma unroll
  for (int m = 1; m < kWave; m <<= 1) {
    h1 = addmod61(h1, shfl_xor64(h1, m));
    h2 = addmod61(h2, shfl_xor64(h2, m));
    xs += shfl_xor64(xs, m);
  }
  if (l == 0) {
    uint64_t* p = t.part + 3 * ((uint64_t)doc * t.tpd + tile);
    p[0] = h1;
    p[1] = h2;
    p[2] = xs;
  }
}

__global__ __launch_bounds__(256) void dg_final_kernel(DigestArgs a, DigestTiles t) {
  const int w = threadIdx.x / kWave, l = lane_id();
  const int doc = (int)blockIdx.x * 4 + w;
  if (doc >= (int)a.n_docs) return;
  const int m = (a.hdr[doc].nseg + kDgTile - 1) / kDgTile;
  uint64_t h1 = 0, h2 = 0, xs = 0;
  for (int i = l; i < m; i += kWave) {
    const uint64_t* p = t.part + 3 * ((uint64_t)doc * t.tpd + (uint32_t)i);
    h1 = addmod61(h1, p[0]);
    h2 = addmod61(h2, p[1]);
    xs += p[2];
  }
#pragma unroll
  for (int s = 1; s < kWave; s <<= 1) {
    h1 = addmod61(h1, shfl_xor64(h1, s));
    h2 = addmod61(h2, shfl_xor64(h2, s));
    xs += shfl_xor64(xs, s);
  }
  if (l == 0) {
    a.out[4 * (size_t)doc + 0] = (uint64_t)t.tot[doc];
    a.out[4 * (size_t)doc + 1] = h1;
    a.out[4 * (size_t)doc + 2] = h2;
    a.out[4 * (size_t)doc + 3] = xs;
  }
}

// host helpers for the digest constants (must match oracle/oracle.c)
uint64_t h_mulmod61(uint64_t a, uint64_t b) {
  unsigned __int128 p = (unsigned __int128)a * b;
  uint64_t r = (uint64_t)(p & kM61) + (uint64_t)(p >> 61);
  return r >= kM61 ? r - kM61 : r;
}
const uint64_t kDigB1 = 0x1d8e4e27c47d124full % kM61;
const uint64_t kDigB2 = 0x0a0761d6478bd642ull % kM61;

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------

// An RCCL communicator and the number of contexts using it (mte_comm_share).
struct CommRef {
  ncclComm_t comm = nullptr;
  std::atomic<int> refs{1};
};

struct mte_ctx {
  int device = 0;
  uint32_t n_keys = 0, kt = 0;  // kt: template planes (0/4/8)
  uint32_t cap = 1024;
  uint32_t n_docs = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // the tree pass runs on its own stream beside the flat passes (disjoint
  // documents), forked after the batch set-up and joined before the read-outs
  hipStream_t tree_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool ran = false, submitted = false;
  bool stats_on = true;
  std::string err;

  DocHdr* hdr = nullptr;
  SegSoA soa{};
  unsigned long long* stats = nullptr;
  mte_doc_init* d_inits = nullptr;
  uint32_t* d_init_props = nullptr;
  uint64_t* d_pow = nullptr;  // pow1[32], pow2[32]

  // mte_load_segments image (SoA, 6 + kt planes at stride n_img)
  uint32_t* d_img = nullptr;
  uint32_t* d_img_doc = nullptr;
  uint64_t* d_img_off = nullptr;
  uint64_t n_img = 0;
  ImgConst img_uc = {};  // the image's uniform planes (image_kernel)

  // pinned staging for op-record uploads (mte_submit), allocated on first use
  static constexpr int kStages = 3;
  static constexpr size_t kStageBytes = 64ull << 20;
  void* stage[kStages] = {nullptr, nullptr, nullptr};
  hipEvent_t stage_ev[kStages] = {nullptr, nullptr, nullptr};

  // diagnostics: MTE_WAVE_CLOCK=<file> dumps pass-1 start / end times per
  // pair (s_memrealtime, 100 MHz) at every mte_sync
  unsigned long long* d_wclock = nullptr;
  unsigned long long* d_gdone = nullptr;  // pass-1 global progress (fair priority)
  double last_ms = 0, last_ops = 0;       // previous run (pass-1 schedule estimate, MTE_FAIR_PRIO 4)
  const char* wclock_path = nullptr;

  // chunked big-document pass (seg_capacity >= kChunkMinCap, mte_chunk.h)
  bool chunked = false;
  ChunkArgs ch{};
  uint64_t* d_digest = nullptr;
  // tile-parallel digest of big-document contexts (dg_*_kernel), allocated at
  // the first digest of such a context
  void* d_dgt = nullptr;
  DigestTiles dgt{};

  // text arena
  uint16_t* arena = nullptr;
  uint64_t arena_n = 0, arena_cap = 0;
  std::vector<uint16_t> h_arena;
  std::vector<mte_propset> h_load_ps;  // mte_load_docs propsets (for mte_load_segments)
  std::vector<mte_prop> h_load_pe;

  // batch
  // Two batch slots: mte_submit fills one (validation, pinned staging, DMA on
  // up_stream) while a replay of the other may still run on `stream`; a slot is
  // rewritten only after the last run that read it (slot_ev).  mte_run replays
  // the slot last submitted (rslot).
  hipStream_t up_stream = nullptr;
  int rslot = 0;
  hipEvent_t slot_ev[2] = {nullptr, nullptr};
  mte_op* d_ops_s[2] = {nullptr, nullptr};
  uint64_t ops_cap_s[2] = {0, 0};
  uint4* d_cps_s[2] = {nullptr, nullptr};  // compiled propsets, 2 x uint4 each (props_kernel)
  uint64_t cps_cap_s[2] = {0, 0};
  uint64_t* d_off_s[2] = {nullptr, nullptr};
  uint64_t off_cap_s[2] = {0, 0};
  mte_propset* d_ps_s[2] = {nullptr, nullptr};
  uint64_t ps_cap_s[2] = {0, 0};
  mte_prop* d_pe_s[2] = {nullptr, nullptr};
  uint64_t pe_cap_s[2] = {0, 0};
  uint64_t n_ops_s[2] = {0, 0}, n_propsets_s[2] = {0, 0};
  uint32_t text_base_s[2] = {0, 0};
  uint64_t max_doc_ops_s[2] = {0, 0};  // the batch's largest per-document op count
  // the batch mte_run replays (= slot rslot)
  mte_op* d_ops = nullptr;
  uint4* d_cps = nullptr;
  uint64_t n_ops = 0, n_propsets = 0;
  uint32_t* d_pairs = nullptr;  // pass-1 doc pairs (new length calc documents)
  uint32_t n_pairs = 0;         // pass-1 waves
  uint32_t pass1_group = 1;     // documents per pass-1 wave
  // tree pass (legacy length calc documents, mte_tree.h)
  uint32_t* d_tree = nullptr;       // tree word per slot
  uint2* d_heap = nullptr;          // LRU heap per document
  uint32_t* d_tree_docs = nullptr;  // the legacy documents
  uint32_t n_tree = 0;
  // the HBM tree pass (mte_htree.h): legacy documents past the register tiers
  // and every document with a local client (or legacy with delta events)
  uint2* d_hheap = nullptr;         // heaps, hcap + 1 entries per document
  uint32_t hcap = 0;
  uint32_t* d_hst = nullptr;        // kHtState words per document
  int32_t* d_hscr = nullptr;        // L / P scratch, 2 x cap per document
  uint32_t* d_htree_docs = nullptr; // the candidates
  uint32_t n_htree = 0;
  std::vector<uint8_t> h_legacy;    // per doc
  std::vector<uint8_t> h_local;     // per doc: 1 MTE_DOC_LOCAL_CLIENT, 2 MTE_DOC_TREE (the HBM tree pass's)
  std::vector<uint8_t> h_events;    // per doc: MTE_DOC_EVENTS
  // delta events per batch slot: region offsets (n_docs + 1, host and device),
  // the events, their counts; ev_slot = the slot of the last mte_run
  uint32_t ev_per_op = 8;
  std::vector<uint64_t> h_dl_off_s[2];
  uint64_t* d_dl_off_s[2] = {nullptr, nullptr};
  uint64_t dl_off_cap_s[2] = {0, 0};
  mte_delta* d_dl_s[2] = {nullptr, nullptr};
  uint64_t dl_cap_s[2] = {0, 0};
  uint32_t* d_dl_n_s[2] = {nullptr, nullptr};
  uint64_t dl_n_cap_s[2] = {0, 0};
  // the streamed pass's document order (longest batch first, so the longest
  // chains start first): the local-client / event documents by this batch's op
  // count, then the rest; empty without such documents
  std::vector<uint32_t> h_sdocs;
  uint32_t* d_sorder_s[2] = {nullptr, nullptr};
  uint64_t sorder_cap_s[2] = {0, 0};
  // per batch slot: the documents with MTE_OP_RELPOS records (upload_ops)
  std::vector<uint32_t> h_rel_s[2];
  uint32_t* d_rel_s[2] = {nullptr, nullptr};
  uint64_t rel_cap_s[2] = {0, 0};
  int ev_slot = -1;
  // local references of the MTE_DOC_REFS documents (mte_stream.h): ref_cap slots
  // per document, zeroed at every reset
  std::vector<uint8_t> h_refs;      // per doc: MTE_DOC_REFS
  std::vector<uint8_t> h_slides;    // per doc: MTE_DOC_SLIDE_EVENTS (with REFS and EVENTS)
  bool any_maint = false;           // a document records maintenance (the HBM tree pass's M build)
  std::vector<uint32_t> h_ref_hi;   // per doc: reference slots its MTE_OP_REF records used so far (+1)
  uint32_t ref_cap = 1024;
  uint2* d_refs = nullptr;
  uint32_t* d_rs_docs = nullptr;    // legacy documents declared MTE_DOC_ROUND_SYNC (flat)
  int tree_rounds = 0;              // TIER 0 / TIER 1 rounds (MTE_TREE_ROUNDS; 0 = from the batch)
  // node level (mte_comm_*): the RCCL communicator and its staging buffers
  // the communicator is shared by reference count (mte_comm_share): the last
  // context to release it destroys it, whatever order contexts go in
  CommRef* cref = nullptr;
  ncclComm_t comm = nullptr;  // cref->comm, or null
  int world = 1, rank = 0;
  uint64_t* d_comm = nullptr;  // digests of all ranks / scalar reductions
  uint64_t comm_cap = 0;       // uint64 elements
  uint32_t n_rs = 0;
  // per key, the largest property value id the context was given (load +
  // every batch) and whether any text segment or annotate ever carried it:
  // pass 1 packs the 4 property planes into one (kPack4) when every key's ids
  // fit a byte, or all but a side key that only marker inserts ever set
  // (ReplayArgs::side_key, config 3's markerId); sticky per context
  uint32_t max_vid_k[MTE_MAX_KEYS] = {};
  uint8_t key_text[MTE_MAX_KEYS] = {};
  std::vector<uint8_t> h_text_ps;  // the batch's propsets a text insert or an annotate used
  // the largest property value id the context was given (load + every batch):
  // below 256 pass 1 packs the 4 property planes into one (kPack4);
  // MTE_PACK_PROPS=0 turns that off
  uint32_t max_vid = 0;
  bool pack_props = true;
  // round phases of the chunked pass (mte_round.h); MTE_ROUND_PHASES=0 turns them off
  RoundArgs rd{};
  bool round_phases = true;
  uint32_t htree_lds = 0;  // LDS bytes a document of the HBM tree pass may hold (MTE_HTREE_LDS)
  std::vector<uint32_t> h_htree_docs, h_hord;
  uint32_t* d_hord_s[2] = {nullptr, nullptr};  // per batch slot: the candidates, most records first
  uint64_t hord_cap_s[2] = {0, 0};
  bool hord_ok_s[2] = {false, false};  // the slot's order is of the loaded documents
  // MTE_HTREE_PROF=<file>: the HBM tree pass's phase clocks (a `make prof`
  // build) appended to <file> at each mte_stats_get
  const char* hprof_path = nullptr;
  unsigned long long* d_hprof = nullptr;
  uint32_t* h_rcount = nullptr;  // pinned: the plan's counts
  // The round phases' host loop (launch_replay) reads each phase's counts back
  // before launching the next, so it cannot be enqueued ahead: mte_run starts
  // it on this thread and returns (include/mte.h: mte_run does not wait); every
  // later call that uses the context's stream or state joins it first
  // (join_tail), and its error, if any, is returned there.
  std::thread tail;
  std::function<int()> tail_fn;
  int tail_rc = 0;
  int tail_slot = -1;  // the batch slot the running tail replays
  uint64_t* d_off = nullptr;
  mte_propset* d_ps = nullptr;
  mte_prop* d_pe = nullptr;
  uint32_t batch_text_base = 0;
};

namespace {

int set_err(mte_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

// Join the round phases' tail thread of the last mte_run, if any, and hand on
// its status (mte_ctx::tail).
int join_tail(mte_ctx* c) {
  if (c->tail.joinable()) c->tail.join();
  const int rc = c->tail_rc;
  c->tail_rc = 0;
  return rc;
}
#define JOIN_TAIL(c)                              \
  do {                                            \
    if (const int jr_ = join_tail(c)) return jr_; \
  } while (0)

// drop this context's reference to its communicator; the last one destroys it
ncclResult_t comm_release(mte_ctx* c) {
  ncclResult_t r = ncclSuccess;
  if (c->cref && c->cref->refs.fetch_sub(1) == 1) {
    r = ncclCommDestroy(c->cref->comm);
    delete c->cref;
  }
  c->cref = nullptr;
  c->comm = nullptr;
  c->world = 1;
  c->rank = 0;
  return r;
}

#define HIPCHK(ctx, expr)                                                                  \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return set_err(ctx, MTE_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                     __LINE__);                                                            \
  } while (0)

template <typename T>
int grow(mte_ctx* c, T** p, uint64_t* cap, uint64_t need, bool keep = false, uint64_t keep_n = 0) {
  if (need <= *cap && *p) return MTE_OK;
  uint64_t nc = *cap ? *cap : 256;
  while (nc < need) nc *= 2;
  T* q = nullptr;
  HIPCHK(c, hipMalloc((void**)&q, nc * sizeof(T)));
  if (keep && *p && keep_n) HIPCHK(c, hipMemcpyAsync(q, *p, keep_n * sizeof(T), hipMemcpyDeviceToDevice, c->stream));
  if (*p) {
    // every kernel that may still read the old buffer has to be done: the
    // round phases' tail thread (mte_ctx::tail) enqueues onto the engine
    // stream after this call could sync it, and the tree passes run on their
    // own stream, which only the tail's finish() joins back (the
    // HBM tree pass reads the text arena).  The tail's status stays in
    // tail_rc for the next JOIN_TAIL.
    if (c->tail.joinable()) c->tail.join();
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->tree_stream) HIPCHK(c, hipStreamSynchronize(c->tree_stream));
    HIPCHK(c, hipFree(*p));
  }
  *p = q;
  *cap = nc;
  return MTE_OK;
}

void free_image(mte_ctx* c) {
  void* ps[] = {c->d_img, c->d_img_doc, c->d_img_off};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  c->d_img = nullptr;
  c->d_img_doc = nullptr;
  c->d_img_off = nullptr;
  c->n_img = 0;
}

void free_docs(mte_ctx* c) {
  free_image(c);
  void* cs[] = {c->ch.arena, c->ch.cnt, c->ch.kc, c->ch.sum, c->rd.plan, c->rd.acct, c->rd.rcnt, c->rd.rbuf, c->rd.rflag,
                c->rd.nch, c->rd.nnew, c->rd.count, c->rd.rchain, c->rd.live, c->rd.gfl, c->rd.rrec};
  for (void* p : cs)
    if (p) (void)hipFree(p);
  c->ch = ChunkArgs{};
  c->rd = RoundArgs{};
  c->chunked = false;
  if (c->d_wclock) (void)hipFree(c->d_wclock);
  c->d_wclock = nullptr;
  if (c->d_dgt) (void)hipFree(c->d_dgt);
  c->d_dgt = nullptr;
  c->dgt = DigestTiles{};
  void* ps[] = {c->hdr, c->soa.len, c->stats, c->d_inits, c->d_init_props, c->d_digest, c->d_pairs,
                c->d_tree, c->d_heap, c->d_tree_docs, c->d_rs_docs, c->d_refs, c->d_hheap, c->d_hst, c->d_hscr,
                c->d_htree_docs};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  c->d_refs = nullptr;
  c->d_rs_docs = nullptr;
  c->n_rs = 0;
  c->d_tree = nullptr;
  c->d_heap = nullptr;
  c->d_tree_docs = nullptr;
  c->n_tree = 0;
  c->d_hheap = nullptr;
  c->d_hst = nullptr;
  c->d_hscr = nullptr;
  c->d_htree_docs = nullptr;
  c->n_htree = 0;
  c->h_htree_docs.clear();
  c->hord_ok_s[0] = c->hord_ok_s[1] = false;
  c->hdr = nullptr;
  c->soa = SegSoA{};
  c->stats = nullptr;
  c->d_inits = nullptr;
  c->d_init_props = nullptr;
  c->d_digest = nullptr;
  c->d_pairs = nullptr;
  c->n_pairs = 0;
  c->n_docs = 0;
}

int launch_reset(mte_ctx* c) {
  if (!c->n_docs) return MTE_OK;
  const uint32_t blocks = (c->n_docs + 255) / 256;
  hipLaunchKernelGGL(reset_kernel, dim3(blocks), dim3(256), 0, c->stream, c->hdr, c->soa, c->cap,
                     c->d_inits, c->d_init_props, c->n_keys, c->n_docs, (const uint64_t*)c->d_img_off, c->d_tree,
                     c->kt, c->d_hst);
  HIPCHK(c, hipGetLastError());
  if (c->d_refs)
    HIPCHK(c, hipMemsetAsync(c->d_refs, 0, sizeof(uint2) * (size_t)c->ref_cap * c->n_docs, c->stream));
  std::fill(c->h_ref_hi.begin(), c->h_ref_hi.end(), 0u);  // the references are gone
  if (c->n_img) {
    const uint64_t nb = std::min<uint64_t>((c->n_img + 255) / 256, 65536);
    hipLaunchKernelGGL(image_kernel, dim3((uint32_t)nb), dim3(256), 0, c->stream, c->soa, c->cap,
                       (uint32_t)(kFieldPlanes + c->kt), c->d_img, c->n_img, c->d_img_doc,
                       (const uint64_t*)c->d_img_off, c->n_img, c->d_tree, c->img_uc);
    HIPCHK(c, hipGetLastError());
  }
  c->ran = false;
  return MTE_OK;
}

// The round phases of the chunked pass (mte_round.h), run by the context's tail
// thread (mte_ctx::tail): per phase the plan's counts come back to the host,
// which stops when no document is left or launches the phase's runs.
template <int K>
int round_phase_loop(mte_ctx* c, const ReplayArgs& a, size_t lds) {
  HIPCHK(c, hipSetDevice(c->device));
  ChunkArgs ch = c->ch;
  RoundArgs rd = c->rd;
  ch.plan = rd.plan;
  ch.rflag = rd.rflag;
  rd.planes = kFieldPlanes + (uint32_t)(K > 0 ? K : 0);
  HIPCHK(c, hipMemsetAsync(rd.acct, 0, sizeof(unsigned long long) * c->n_docs, c->stream));
  // no document starts in the arena (rd.live: a run's chunks stay laid out for
  // the document's next run and go back to the flat planes when it leaves)
  HIPCHK(c, hipMemsetAsync(rd.live, 0, 4 * (uint64_t)c->n_docs, c->stream));
  rd.d0 = 0;
  rd.nd = c->n_docs;
  bool carried = false;  // some document may be in the arena
  const uint64_t nch_all = (uint64_t)c->n_docs * ch.nch_cap;
  for (int ph = 0; ph < kMaxPhases; ph++) {
    rd.last = ph == kMaxPhases - 1 ? 1u : 0u;
    HIPCHK(c, hipMemsetAsync(rd.count, 0, 16, c->stream));
    HIPCHK(c, launch_round_plan(a, ch, rd, c->n_docs, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_rcount, rd.count, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint32_t n_round = c->h_rcount[0], n_active = c->h_rcount[2];
    if (n_active == 0) break;
    if (n_round) {
      // the resolve's columns: the largest round document's chunks (rnd_plan)
      const uint32_t want = c->h_rcount[3] < 64u ? 64u : c->h_rcount[3];
      rd.col_cap = (want + 63u) / 64u * 64u;
      HIPCHK(c, hipMemsetAsync(rd.rcnt, 0, nch_all * 4, c->stream));
      HIPCHK(c, hipMemsetAsync(rd.rflag, 0, 4 * (uint64_t)c->n_docs, c->stream));
      HIPCHK(c, (launch_round_run<K>(a, ch, rd, c->n_docs, c->stream)));
      carried = true;
    } else if (carried) {  // the carried documents' runs are not rounds: back to the flat planes
      HIPCHK(c, (launch_round_gather<K>(a, ch, rd, 0, c->stream)));
    }
    HIPCHK(c, (launch_chunk<K, false>(a, ch, c->n_docs, lds, c->stream)));
  }
  if (carried) HIPCHK(c, (launch_round_gather<K>(a, ch, rd, 1, c->stream)));
  return MTE_OK;
}

template <int K, bool S>
int launch_replay(mte_ctx* c, const ReplayArgs& a) {
  // the tree pass: legacy length calc documents (mte_tree.h), up to 252
  // items at E <= 4, then up to 1,020 at E = 8 / 16; then the HBM tree pass
  // (mte_htree.h): the legacy documents past that and every document with a
  // local client
  if (c->n_tree || c->n_htree) {
    if (!c->tree_stream) {
      HIPCHK(c, hipStreamCreateWithFlags(&c->tree_stream, hipStreamNonBlocking));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    }
    // the flat passes only touch documents pass 1 owns or escalates (never a
    // tree document), so the two streams share no document state
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->tree_stream, c->ev_fork, 0));
    if (c->n_tree) {
      TreeArgs t{c->d_tree, c->d_heap, c->d_tree_docs, c->n_tree, c->arena, 0u, 0u};
      // rounds of at most ~625 ops per document (MTE_TREE_ROUNDS overrides the count)
      const uint64_t mx = c->max_doc_ops_s[c->rslot];
      int rounds = c->tree_rounds > 0 ? c->tree_rounds : (int)std::min<uint64_t>(32, std::max<uint64_t>(1, (mx + 624) / 625));
      const uint32_t per = (uint32_t)((mx + (uint64_t)rounds - 1) / (uint64_t)rounds);
      HIPCHK(c, (launch_tree<K, S>(a, t, (c->n_tree + kDocsPerBlock - 1) / kDocsPerBlock, c->tree_stream, rounds,
                                   per ? per : 1u)));
    }
    if (c->n_htree) {
      // LDS residency: (nP + 5) words per item (mte_htree.h ht_to_lds), whole wavefronts' worth
      const uint32_t words = (uint32_t)(kLocalPlanes<K> + 5);
      uint32_t lcap = c->htree_lds >= 8 ? (c->htree_lds / 4 - 2) / words / kWave * kWave : 0u;
      if (lcap > c->cap) lcap = c->cap / kWave * kWave;
      const uint32_t* order = c->hord_ok_s[c->rslot] ? c->d_hord_s[c->rslot] : c->d_htree_docs;
      if (c->hprof_path && !c->d_hprof) {
        HIPCHK(c, hipMalloc((void**)&c->d_hprof, kHtProf * 8));
        HIPCHK(c, hipMemsetAsync(c->d_hprof, 0, kHtProf * 8, c->tree_stream));
      }
      HtreeArgs ht{c->d_tree, c->d_heap, c->d_hheap, c->hcap, lcap, c->d_hst, c->d_hscr, order, c->n_htree,
                   c->arena, c->d_hprof, c->any_maint ? 1u : 0u};
      HIPCHK(c, (launch_htree<K, S>(a, ht, c->tree_stream)));
    }
    HIPCHK(c, hipEventRecord(c->ev_join, c->tree_stream));
  }
  // pass 1: two documents per wavefront (docs up to 126 segments)
  const uint32_t b1 = (c->n_pairs + kPairsPerBlock - 1) / kPairsPerBlock;
  // with 4 keys whose value ids all fit in a byte (every value the context was
  // ever given), pass 1 holds the four planes as one packed register plane
  if (b1) {
    if constexpr (K == 4) {
      uint32_t side = kNoKey;
      bool pack = c->pack_props;
      for (uint32_t k = 0; k < 4 && pack; k++) {
        if (c->max_vid_k[k] < 256) continue;
        if (side == kNoKey && !c->key_text[k]) side = k;  // set on markers only
        else pack = false;
      }
      for (uint32_t k = 4; k < MTE_MAX_KEYS; k++) pack = pack && c->max_vid_k[k] == 0;  // kt = 4: 4 keys at most
      ReplayArgs ap = a;
      ap.side_key = side;
      if (pack) HIPCHK(c, (launch_pair<kPack4, S>(ap, b1, c->stream)));
      else HIPCHK(c, (launch_pair<K, S>(a, b1, c->stream)));
    } else {
      HIPCHK(c, (launch_pair<K, S>(a, b1, c->stream)));
    }
  }
  // pass 2: docs that outgrew pass 1 continue one per wavefront (up to 1022 segments)
  const uint32_t b2 = (c->n_docs + kDocsPerBlock - 1) / kDocsPerBlock;
  HIPCHK(c, (launch_big<K, S>(a, b2, c->stream)));
  // pass 3: larger docs (up to the ctx capacity): the chunked pass in big-doc
  // contexts, otherwise HBM-resident and streamed per op
  if (c->chunked) {
    const size_t lds = sizeof(uint32_t) * MTE_MAX_CLIENTS * c->ch.ng_cap + sizeof(ChCtl);
    const uint64_t col_bytes = rnd_resolve_lds(c->ch.nch_cap, c->ch.ng_cap);
    if (!S && c->round_phases && col_bytes <= kRoundLdsMax) {
      // round phases (mte_round.h): each phase plans every escalated
      // document's next run, replays the round-shaped runs chunk-parallel and
      // the rest op after op; the host reads the plan's counts to stop.  The
      // loop runs on the context's tail thread (mte_run returns at once).
      c->tail_fn = [c, a, lds]() -> int { return round_phase_loop<K>(c, a, lds); };
      return MTE_OK;  // the tail joins the tree stream after the loop
    } else {
      HIPCHK(c, (launch_chunk<K, S>(a, c->ch, c->n_docs, lds, c->stream)));
    }
  } else {
    HIPCHK(c, (launch_stream<K, S>(a, b2, c->stream)));
  }
  return MTE_OK;  // mte_run joins the tree stream (finish)
}

// Validation of one op record (the kernels index with these fields, so a bad
// record must never reach them).  Returns nullptr or the reason.
const char* bad_op(const mte_op& o, const mte_batch* b, bool local_doc, bool tree_doc, bool refs_doc, uint32_t ref_cap) {
  if (o.type > MTE_OP_RELPOS) return "type";
  if (o.type == MTE_OP_RELPOS) {  // the record after it is checked by the caller
    const uint32_t rp = MTE_RP_POS1 | MTE_RP_BEFORE1 | MTE_RP_POS2 | MTE_RP_BEFORE2;
    if ((o.flags & ~rp) || !(o.flags & (MTE_RP_POS1 | MTE_RP_POS2))) return "relative position record: flags";
    return nullptr;
  }
  if (o.type >= MTE_OP_ROLLBACK && !(o.flags & MTE_F_LOCAL)) return "rollback / regen without MTE_F_LOCAL";
  if (o.type == MTE_OP_REF) {
    if (!refs_doc) return "local reference record in a document without MTE_DOC_REFS";
    if (o.seq != 0 || o.pos2 < 0 || (uint32_t)o.pos2 >= ref_cap || o.b > 5 || o.client >= MTE_MAX_CLIENTS ||
        (o.b == 2 && o.client == 0))
      return "local reference record: seq, slot (mte_set_ref_capacity), b or client out of range";
    if (o.b >= 4 && (!local_doc || o.a >= MTE_LOCAL_SEQ_BASE))
      return "rebase record: not a local-client document, or localSeq out of range";
    return nullptr;
  }
  if ((o.flags & MTE_F_LOCAL) && o.type == MTE_OP_ANNOTATE && o.b != MTE_NO_PROPS && o.b >= MTE_ANNOTATE_SLOTS)
    return "annotate group slot out of range";
  if ((o.flags & MTE_F_LOCAL) || o.type == MTE_OP_ACK) {
    if (!local_doc) return "local op or ack in a document without MTE_DOC_LOCAL_CLIENT";
    if ((o.flags & MTE_F_LOCAL) && o.type != MTE_OP_RBKEY &&
        (o.type == MTE_OP_ACK || o.seq <= 0 || o.seq >= MTE_LOCAL_SEQ_BASE))
      return "local record: type or localSeq out of range";
    if (o.type == MTE_OP_RBKEY && (o.seq < 0 || o.seq >= MTE_LOCAL_SEQ_BASE || o.pos1 < 0 ||
                                   o.pos1 >= MTE_MAX_KEYS || o.pos2 < 0 || o.pos2 > MTE_ANNOTATE_SLOTS))
      return "rollback key record out of range";
    if (o.type == MTE_OP_ROLLBACK && o.pos1 == MTE_OP_ANNOTATE &&
        (o.a >= MTE_ANNOTATE_SLOTS || o.pos2 < 0 || o.pos2 > MTE_MAX_KEYS * (MTE_ANNOTATE_SLOTS + 1)))
      return "annotate rollback: group slot or key record count out of range";
    if (o.type == MTE_OP_ACK && (o.pos1 <= 0 || o.pos1 > o.pos2)) return "ack: localSeq range";
  }
  if (local_doc && !(o.flags & MTE_F_LOCAL) && o.seq >= MTE_LOCAL_SEQ_BASE) return "seq >= MTE_LOCAL_SEQ_BASE";
  if (o.type == MTE_OP_INSERT) {
    if (!(o.flags & MTE_F_MARKER) && o.pos2 > 0 && (uint64_t)o.a + (uint64_t)o.pos2 > b->text_units)
      return "text out of range";
    if ((o.flags & MTE_F_MARKER) && (o.pos2 < 0 || o.pos2 >= (1 << 23))) return "refType out of range";
    if (!(o.flags & MTE_F_MARKER) && o.pos2 < 0) return "negative text length";
    if (o.b != MTE_NO_PROPS && o.b >= b->n_propsets) return "propset out of range";
  } else if (o.type == MTE_OP_ANNOTATE && o.a >= b->n_propsets) {
    return "propset out of range";
  }
  if (o.flags & MTE_F_COMBINE) {
    // a sequenced or local incr / consensus annotate, or the ack of a local
    // consensus (b = the stamp's value map)
    const bool ack = o.type == MTE_OP_ACK;
    if ((o.type != MTE_OP_ANNOTATE && !ack) || (o.flags & MTE_F_REWRITE) || (ack && (o.flags & MTE_F_LOCAL)))
      return "combining record: type or flags";
    if (!local_doc && (ack || !tree_doc))
      return "combiningOp incr / consensus outside an MTE_DOC_LOCAL_CLIENT or MTE_DOC_TREE document";
    const uint32_t psi = ack ? o.b : o.a;
    if (psi >= b->n_propsets) return "combining propset out of range";
    const mte_propset& ps = b->propsets[psi];
    if ((uint64_t)ps.first + ps.count > b->n_props) return "combining propset out of range";
    for (uint32_t t = 0; t < ps.count;) {  // headers and their pairs tile the set exactly
      const mte_prop& h = b->props[ps.first + t];
      if ((h.key & MTE_COMBINE_PAIR) || h.value > ps.count - t - 1) return "combining propset: header";
      for (uint32_t u = 1; u <= h.value; u++)
        if (!(b->props[ps.first + t + u].key & MTE_COMBINE_PAIR)) return "combining propset: pair";
      t += 1 + h.value;
    }
  }
  return nullptr;
}

unsigned host_workers() {
  const unsigned hw = std::thread::hardware_concurrency();
  return hw == 0 ? 1u : (hw > 16 ? 16u : hw);
}

// Host op records -> HBM: validated and copied in one pass by host_workers()
// threads into pinned staging buffers, each buffer's DMA overlapping the
// filling of the next (pageable hipMemcpy runs at a fraction of PCIe speed).
// Returns MTE_OK or MTE_E_INVALID_ARG with *bad = the first bad record.
int upload_ops(mte_ctx* c, const mte_batch* b, int w, uint64_t* bad, const char** why) {
  for (int i = 0; i < mte_ctx::kStages; i++) {
    if (!c->stage[i]) HIPCHK(c, hipHostMalloc(&c->stage[i], mte_ctx::kStageBytes, hipHostMallocDefault));
    if (!c->stage_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
  }
  const uint64_t per_stage = mte_ctx::kStageBytes / sizeof(mte_op);
  const unsigned nw = host_workers();
  std::atomic<uint64_t> first_bad{UINT64_MAX};
  std::vector<const char*> reasons(nw, nullptr);
  // per worker: the propsets a text insert or an annotate used (kPack4 side key)
  std::vector<std::vector<uint8_t>> tps(nw, std::vector<uint8_t>(b->n_propsets, 0));
  // per worker: the documents with MTE_OP_RELPOS records
  std::vector<std::vector<uint32_t>> rels(nw);
  for (uint64_t k0 = 0, it = 0; k0 < b->n_ops; k0 += per_stage, it++) {
    const int si = (int)(it % mte_ctx::kStages);
    const uint64_t n = std::min(per_stage, b->n_ops - k0);
    HIPCHK(c, hipEventSynchronize(c->stage_ev[si]));  // its previous DMA has drained
    mte_op* dst = static_cast<mte_op*>(c->stage[si]);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nw; w++) {
      th.emplace_back([&, w]() {
        const uint64_t a = n * w / nw, e = n * (w + 1) / nw;
        // the document of record k0 + a, then a cursor over op_offsets
        uint32_t d = (uint32_t)(std::upper_bound(b->op_offsets, b->op_offsets + b->n_docs + 1, k0 + a) -
                                b->op_offsets) - 1;
        for (uint64_t k = a; k < e; k++) {
          while (d + 1 < b->n_docs && b->op_offsets[d + 1] <= k0 + k) d++;
          const mte_op& o = b->ops[k0 + k];
          const uint8_t hl = c->h_local.empty() ? 0 : c->h_local[d];
          const char* r = bad_op(o, b, (hl & 1) != 0, (hl & 2) != 0, !c->h_refs.empty() && c->h_refs[d], c->ref_cap);
          if (!r && o.type == MTE_OP_RELPOS) {
            const mte_op* nx = k0 + k + 1 < b->op_offsets[d + 1] ? &b->ops[k0 + k + 1] : nullptr;
            if (!nx || nx->type > MTE_OP_ANNOTATE) r = "relative position record not followed by an insert, remove "
                                                      "or annotate of its document";
            else if (rels[w].empty() || rels[w].back() != d) rels[w].push_back(d);
          }
          if (r) {
            uint64_t cur = first_bad.load();
            while (k0 + k < cur && !first_bad.compare_exchange_weak(cur, k0 + k)) {
            }
            if (first_bad.load() == k0 + k) reasons[w] = r;
            return;
          }
        }
        std::memcpy(dst + a, b->ops + k0 + a, (e - a) * sizeof(mte_op));
        // kRecNl: the insert's text holds a '\n' (the tree pass's append-merge
        // looks at a leaf's last unit only then, mte_tree.h)
        std::vector<uint8_t>& tp = tps[w];
        for (uint64_t k = a; k < e; k++) {
          mte_op& o = dst[k];
          if (o.type == MTE_OP_ANNOTATE && o.a < b->n_propsets) tp[o.a] = 1;
          if (o.type == MTE_OP_INSERT && !(o.flags & MTE_F_MARKER) && o.b != MTE_NO_PROPS && o.b < b->n_propsets)
            tp[o.b] = 1;
          o.flags = (uint16_t)(o.flags & ~kRecNl);
          if (o.type == MTE_OP_INSERT && !(o.flags & MTE_F_MARKER) && o.pos2 > 0) {
            const uint16_t* t = b->text + o.a;
            for (int32_t u = 0; u < o.pos2; u++)
              if (t[u] == 0x0A) {
                o.flags = (uint16_t)(o.flags | kRecNl);
                break;
              }
          }
        }
      });
    }
    for (auto& t : th) t.join();
    if (first_bad.load() != UINT64_MAX) break;
    HIPCHK(c, hipMemcpyAsync(c->d_ops_s[w] + k0, dst, n * sizeof(mte_op), hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(c, hipEventRecord(c->stage_ev[si], c->up_stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->up_stream));
  if (first_bad.load() != UINT64_MAX) {
    *bad = first_bad.load();
    *why = "bad record";
    for (const char* r : reasons)
      if (r) *why = r;
    return MTE_E_INVALID_ARG;
  }
  c->h_text_ps.assign(b->n_propsets, 0);
  for (const auto& v : tps)
    for (uint32_t i = 0; i < b->n_propsets; i++) c->h_text_ps[i] |= v[i];
  std::vector<uint32_t>& rd = c->h_rel_s[w];
  rd.clear();
  for (const auto& v : rels) rd.insert(rd.end(), v.begin(), v.end());
  std::sort(rd.begin(), rd.end());
  rd.erase(std::unique(rd.begin(), rd.end()), rd.end());
  return MTE_OK;
}

}  // namespace

extern "C" {

int mte_abi_version(void) { return MTE_ABI_VERSION; }


const char* mte_strerror(int code) {
  switch (code) {
    case MTE_OK: return "ok";
    case MTE_E_INVALID_ARG: return "invalid argument";
    case MTE_E_NO_DEVICE: return "no HIP device";
    case MTE_E_HIP: return "HIP runtime error";
    case MTE_E_CAPACITY: return "segment capacity exceeded";
    case MTE_E_SEQ_ORDER: return "0x030: remote op sequence number <= currentSeq";
    case MTE_E_MSN_ORDER: return "0x031: remote op minSequenceNumber < minSeq";
    case MTE_E_MSN_GT_SEQ: return "0x039: sequence number < minSequenceNumber";
    case MTE_E_INSERT_FAILED: return "MergeTree insert failed";
    case MTE_E_UNSUPPORTED: return "unsupported op";
    case MTE_E_STATE: return "call out of order";
    case MTE_E_OOM: return "out of memory";
    case MTE_E_CLIENT_RANGE: return "client id out of range";
    default: return "unknown error";
  }
}

const char* mte_last_error(const mte_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int mte_create(const mte_config* cfg, mte_ctx** out) {
  if (!cfg || !out || cfg->n_keys > MTE_MAX_KEYS) return MTE_E_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MTE_E_NO_DEVICE;
  if (cfg->device < 0 || cfg->device >= ndev) return MTE_E_NO_DEVICE;
  mte_ctx* c = new (std::nothrow) mte_ctx();
  if (!c) return MTE_E_OOM;
  c->device = cfg->device;
  c->n_keys = cfg->n_keys;
  c->kt = cfg->n_keys == 0 ? 0 : (cfg->n_keys <= 4 ? 4 : 8);
  c->cap = cfg->seg_capacity ? cfg->seg_capacity : 1024;
  c->wclock_path = std::getenv("MTE_WAVE_CLOCK");
  if (const char* pp = std::getenv("MTE_PACK_PROPS")) c->pack_props = std::atoi(pp) != 0;
  if (const char* rp = std::getenv("MTE_ROUND_PHASES")) c->round_phases = std::atoi(rp) != 0;
  c->hprof_path = std::getenv("MTE_HTREE_PROF");
  if (const char* hl = std::getenv("MTE_HTREE_LDS")) c->htree_lds = (uint32_t)std::min(160l << 10, std::max(0l, std::atol(hl)));
  if (const char* r = std::getenv("MTE_TREE_ROUNDS")) {
    const int v = std::atoi(r);
    c->tree_rounds = v < 0 ? 0 : (v > 64 ? 64 : v);
  }
  if (c->cap < 64) c->cap = 64;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    delete c;
    return MTE_E_NO_DEVICE;
  }
  uint64_t pw[64];
  pw[0] = kDigB1;
  pw[32] = kDigB2;
  for (int i = 1; i < 32; i++) {
    pw[i] = h_mulmod61(pw[i - 1], pw[i - 1]);
    pw[32 + i] = h_mulmod61(pw[32 + i - 1], pw[32 + i - 1]);
  }
  if (hipMalloc((void**)&c->d_pow, sizeof(pw)) != hipSuccess ||
      hipMemcpy(c->d_pow, pw, sizeof(pw), hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return MTE_E_OOM;
  }
  *out = c;
  return MTE_OK;
}

int mte_destroy(mte_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  (void)join_tail(c);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  free_docs(c);
  void* ps[] = {c->arena, c->d_pow, c->d_gdone, c->d_hprof};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  for (int w = 0; w < 2; w++) {
    void* sl[] = {c->d_ops_s[w], c->d_cps_s[w], c->d_off_s[w], c->d_ps_s[w], c->d_pe_s[w],
                  c->d_dl_off_s[w], c->d_dl_s[w], c->d_dl_n_s[w], c->d_sorder_s[w], c->d_rel_s[w], c->d_hord_s[w]};
    for (void* p : sl)
      if (p) (void)hipFree(p);
    if (c->slot_ev[w]) (void)hipEventDestroy(c->slot_ev[w]);
  }
  if (c->up_stream) (void)hipStreamDestroy(c->up_stream);
  for (int i = 0; i < mte_ctx::kStages; i++) {
    if (c->stage[i]) (void)hipHostFree(c->stage[i]);
    if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
  }
  comm_release(c);
  if (c->h_rcount) (void)hipHostFree(c->h_rcount);
  if (c->d_comm) (void)hipFree(c->d_comm);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->tree_stream) (void)hipStreamDestroy(c->tree_stream);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MTE_OK;
}

int mte_load_docs(mte_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props) {
  if (!c || (n_docs && !docs) || (text_units && !text)) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<uint32_t> iprops((size_t)n_docs * MTE_MAX_KEYS, 0u);
  for (uint32_t d = 0; d < n_docs; d++) {
    const mte_doc_init& in = docs[d];
    if ((uint64_t)in.text_off + in.text_len > text_units || in.text_len > 0x7fffffffu)
      return set_err(c, MTE_E_INVALID_ARG, "doc %u: initial text out of range", d);
    if ((in.flags & MTE_DOC_REFS) && !(in.flags & MTE_DOC_LOCAL_CLIENT))
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: local references need MTE_DOC_LOCAL_CLIENT", d);
    // maintenance records come from the HBM tree pass, which keeps the
    // reference's segments (a local client's, MTE_DOC_TREE or a legacy document)
    if ((in.flags & MTE_DOC_MAINT_EVENTS) &&
        (!(in.flags & MTE_DOC_EVENTS) ||
         !((in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) || !(in.flags & MTE_DOC_NEW_LENGTH_CALC))))
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: maintenance events need MTE_DOC_EVENTS on the HBM tree pass "
                     "(MTE_DOC_LOCAL_CLIENT, MTE_DOC_TREE or the legacy length calculation)", d);
    if ((in.flags & MTE_DOC_TREE) && (in.flags & MTE_DOC_ROUND_SYNC))
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: MTE_DOC_TREE with MTE_DOC_ROUND_SYNC", d);
    // delta events of a new length-calc document without a local client come
    // from the HBM-streamed flat pass, which big-document contexts do not run
    if ((in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS | MTE_DOC_TREE)) == MTE_DOC_EVENTS &&
        (in.flags & MTE_DOC_NEW_LENGTH_CALC) && c->cap >= kChunkMinCap)
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: delta events of a document without a local client need a "
                     "context below %u segments", d, kChunkMinCap);
    if ((in.flags & MTE_DOC_ROUND_SYNC) && (in.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS)))
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: MTE_DOC_ROUND_SYNC with a local client or delta events", d);
    if (in.propset != MTE_NO_PROPS) {
      if (in.propset >= n_propsets || !propsets) return set_err(c, MTE_E_INVALID_ARG, "doc %u: bad propset", d);
      const mte_propset ps = propsets[in.propset];
      if ((uint64_t)ps.first + ps.count > n_props) return set_err(c, MTE_E_INVALID_ARG, "doc %u: bad propset", d);
      for (uint32_t t = 0; t < ps.count; t++) {
        const mte_prop p = props[ps.first + t];
        if (p.key < c->n_keys) iprops[(size_t)d * MTE_MAX_KEYS + p.key] = p.value;
      }
    }
  }
  free_docs(c);
  c->n_docs = n_docs;
  c->submitted = false;
  c->max_vid = 0;
  for (uint32_t i = 0; props && i < n_props; i++) c->max_vid = std::max(c->max_vid, props[i].value);
  for (uint32_t k = 0; k < MTE_MAX_KEYS; k++) c->max_vid_k[k] = 0, c->key_text[k] = 0;
  for (uint32_t i = 0; props && i < n_props; i++)
    if (props[i].key < MTE_MAX_KEYS) c->max_vid_k[props[i].key] = std::max(c->max_vid_k[props[i].key], props[i].value);
  for (uint32_t d = 0; d < n_docs; d++)  // the initial text's properties
    if (docs[d].propset != MTE_NO_PROPS) {
      const mte_propset ps = propsets[docs[d].propset];
      for (uint32_t t = 0; t < ps.count; t++)
        if (props[ps.first + t].key < MTE_MAX_KEYS) c->key_text[props[ps.first + t].key] = 1;
    }
  c->ev_slot = -1;
  c->n_ops = 0;
  const uint64_t nslots = (uint64_t)(n_docs ? n_docs : 1) * c->cap;
  c->soa.plane_stride = nslots;
  c->h_local.assign(n_docs, 0);
  c->h_events.assign(n_docs, 0);
  c->h_refs.assign(n_docs, 0);
  c->h_slides.assign(n_docs, 0);
  c->any_maint = false;
  for (uint32_t d = 0; d < n_docs; d++)
    if (docs[d].flags & MTE_DOC_MAINT_EVENTS) c->any_maint = true;
  c->h_ref_hi.assign(n_docs, 0);
  bool any_local = false, any_refs = false;
  c->h_sdocs.clear();
  for (uint32_t d = 0; d < n_docs; d++) {
    // the flat HBM-streamed pass's own: new length-calc documents with delta events and no local client
    if ((docs[d].flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS | MTE_DOC_NEW_LENGTH_CALC | MTE_DOC_TREE)) ==
        (MTE_DOC_EVENTS | MTE_DOC_NEW_LENGTH_CALC))
      c->h_sdocs.push_back(d);
    if (docs[d].flags & MTE_DOC_LOCAL_CLIENT) c->h_local[d] = 1, any_local = true;
    else if (docs[d].flags & MTE_DOC_TREE) c->h_local[d] = 2, any_local = true;
    if (docs[d].flags & MTE_DOC_EVENTS) c->h_events[d] = 1;
    if (docs[d].flags & MTE_DOC_REFS) c->h_refs[d] = 1, any_refs = true;
    const uint32_t sl = MTE_DOC_REFS | MTE_DOC_EVENTS | MTE_DOC_SLIDE_EVENTS;
    if ((docs[d].flags & sl) == sl) c->h_slides[d] = 1;
  }
  if (any_refs) HIPCHK(c, hipMalloc((void**)&c->d_refs, sizeof(uint2) * (size_t)c->ref_cap * n_docs));
  // documents with a local client hold 2 kt + 6 more planes (mte_htree.h): the
  // pending property keys, the annotate-group mask, the keys' values before
  // their first pending annotate, localRemovedSeq, the removal-group order, the
  // first group an item is one of the marked segments of, the regeneration
  // group, the removers of short ids 32 .. 63 (the last one MTE_DOC_TREE
  // documents use too)
  const uint64_t prop_planes = (c->kt ? c->kt : 1) + (any_local ? 2 * c->kt + 6 : 0);
  HIPCHK(c, hipMalloc((void**)&c->hdr, sizeof(DocHdr) * (n_docs ? n_docs : 1)));
  // one allocation, planes at stride nslots: len seq rseq rmask meta toff props[kt]
  // (kt >= n_keys planes, so the register-resident kernels never index past it)
  {
    const uint64_t planes = kFieldPlanes + prop_planes;
    uint32_t* base = nullptr;
    HIPCHK(c, hipMalloc((void**)&base, nslots * 4 * planes));
    c->soa.len = (int32_t*)base;
    c->soa.seq = (int32_t*)(base + 1 * nslots);
    c->soa.rseq = (int32_t*)(base + 2 * nslots);
    c->soa.rmask = base + 3 * nslots;
    c->soa.meta = base + 4 * nslots;
    c->soa.toff = base + 5 * nslots;
    c->soa.props = base + kFieldPlanes * nslots;
  }
  HIPCHK(c, hipMemsetAsync(c->soa.props, 0, nslots * 4 * prop_planes, c->stream));
  if (c->cap >= kChunkMinCap && n_docs) {
    // chunk arena: every doc can be re-laid out at kChFill segments per chunk
    const uint32_t nch_cap = c->cap / kChFill + 2;
    const uint32_t ng_cap = (nch_cap + kChGroup - 1) / kChGroup;
    if (ng_cap <= kChMaxGroups) {
      ChunkArgs& ch = c->ch;
      ch.nch_cap = nch_cap;
      ch.ng_cap = ng_cap;
      const uint64_t nch_all = (uint64_t)n_docs * nch_cap;
      ch.astride = nch_all * kChSlots;
      const uint64_t planes = kFieldPlanes + (c->kt ? c->kt : 1);
      HIPCHK(c, hipMalloc((void**)&ch.arena, ch.astride * 4 * planes));
      HIPCHK(c, hipMalloc((void**)&ch.cnt, nch_all * 4));
      HIPCHK(c, hipMalloc((void**)&ch.kc, nch_all * 4));
      HIPCHK(c, hipMalloc((void**)&ch.sum, nch_all * 4 * MTE_MAX_CLIENTS));
      RoundArgs& rd = c->rd;
      HIPCHK(c, hipMalloc((void**)&rd.plan, sizeof(uint4) * n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.acct, sizeof(unsigned long long) * n_docs));
      HIPCHK(c, hipMemsetAsync(rd.acct, 0, sizeof(unsigned long long) * n_docs, c->stream));
      HIPCHK(c, hipMalloc((void**)&rd.rcnt, nch_all * 4));
      HIPCHK(c, hipMalloc((void**)&rd.rbuf, nch_all * kRB * sizeof(uint2)));
      HIPCHK(c, hipMalloc((void**)&rd.rrec, nch_all * kRB * 2 * sizeof(uint4)));
      HIPCHK(c, hipMalloc((void**)&rd.rflag, 4 * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.nch, 4 * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.nnew, 4 * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.rchain, sizeof(uint2) * MTE_MAX_CLIENTS * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.live, 4 * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.gfl, 4 * (uint64_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&rd.count, 16));
      if (!c->h_rcount) HIPCHK(c, hipHostMalloc((void**)&c->h_rcount, 16, 0));
      c->chunked = true;
    }
  }
  HIPCHK(c, hipMalloc((void**)&c->stats, sizeof(unsigned long long) * kNumStats * (n_docs ? n_docs : 1)));
  HIPCHK(c, hipMemsetAsync(c->stats, 0, sizeof(unsigned long long) * kNumStats * (n_docs ? n_docs : 1), c->stream));
  HIPCHK(c, hipMalloc((void**)&c->d_inits, sizeof(mte_doc_init) * (n_docs ? n_docs : 1)));
  HIPCHK(c, hipMalloc((void**)&c->d_init_props, sizeof(uint32_t) * iprops.size() + 4));
  HIPCHK(c, hipMalloc((void**)&c->d_digest, sizeof(uint64_t) * 4 * (n_docs ? n_docs : 1)));
  {
    // pass-1 groups: g consecutive documents per wave, g the smallest count
    // that puts the whole batch on the chip at once (CUs x 4 SIMDs x
    // pass1_waves() waves), so a batch that fits at one document per wave
    // (config 2's 1k docs, the 1,250 per GPU of an 8-GPU 10k job) runs one per
    // wave: grouping it would leave SIMDs idle and serialise its documents.
    // Legacy length-calc documents go to the tree pass instead (mte_tree.h).
    // Round-synchronous legacy documents (MTE_DOC_ROUND_SYNC) stay flat, behind
    // the per-batch check of round_sync_kernel.
    std::vector<uint32_t> flat_docs, tree_docs, rs_docs, htree_docs;
    c->h_legacy.assign(n_docs, 0);  // the document carries tree words (read-outs join merged leaves)
    for (uint32_t d = 0; d < n_docs; d++) {
      const uint32_t f = docs[d].flags;
      if ((f & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) || ((f & MTE_DOC_EVENTS) && !(f & MTE_DOC_NEW_LENGTH_CALC))) {
        htree_docs.push_back(d);  // the HBM tree pass's own (mte_htree.h)
        c->h_legacy[d] = 1;
      } else if (f & MTE_DOC_EVENTS) {
        continue;  // the HBM-streamed flat pass replays them (mte_stream.h)
      } else if (docs[d].flags & MTE_DOC_NEW_LENGTH_CALC) {
        flat_docs.push_back(d);
      } else if (docs[d].flags & MTE_DOC_ROUND_SYNC) {
        flat_docs.push_back(d);
        rs_docs.push_back(d);
      } else {
        tree_docs.push_back(d);
        c->h_legacy[d] = 1;
      }
    }
    const uint32_t nf = (uint32_t)flat_docs.size();
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) n_cu = 0;
    const uint64_t resident = (n_cu > 0 ? (uint64_t)n_cu : 256) * 4 * (uint64_t)pass1_waves();
    const uint32_t g = (uint32_t)std::min<uint64_t>(kGroupMax, std::max<uint64_t>(1, (nf + resident - 1) / resident));
    c->pass1_group = g;
    c->n_pairs = (nf + g - 1) / g;
    std::vector<uint32_t> pairs((size_t)c->n_pairs * g + g, 0xffffffffu);
    for (uint32_t i = 0; i < nf; i++) pairs[i] = flat_docs[i];
    HIPCHK(c, hipMalloc((void**)&c->d_pairs, pairs.size() * 4));
    HIPCHK(c, hipMemcpy(c->d_pairs, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice));
    c->n_rs = (uint32_t)rs_docs.size();
    if (c->n_rs) {
      HIPCHK(c, hipMalloc((void**)&c->d_rs_docs, rs_docs.size() * 4));
      HIPCHK(c, hipMemcpy(c->d_rs_docs, rs_docs.data(), rs_docs.size() * 4, hipMemcpyHostToDevice));
    }
    c->n_tree = (uint32_t)tree_docs.size();
    if (c->n_tree) {
      HIPCHK(c, hipMalloc((void**)&c->d_heap, sizeof(uint2) * (kTreeHeapCap + 1) * (size_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&c->d_tree_docs, tree_docs.size() * 4));
      HIPCHK(c, hipMemcpy(c->d_tree_docs, tree_docs.data(), tree_docs.size() * 4, hipMemcpyHostToDevice));
    }
    // the HBM tree pass takes its own documents and the legacy ones the
    // register tiers hand over (past 1,020 items)
    // (past 1,020 items, or from a batch with relative positions)
    for (uint32_t d : tree_docs) htree_docs.push_back(d);
    c->n_htree = (uint32_t)htree_docs.size();
    if (c->n_tree || c->n_htree) {
      HIPCHK(c, hipMalloc((void**)&c->d_tree, nslots * 4));
      HIPCHK(c, hipMemsetAsync(c->d_tree, 0, nslots * 4, c->stream));
    }
    if (c->n_htree) {
      c->hcap = c->cap;  // one heap entry per slot
      HIPCHK(c, hipMalloc((void**)&c->d_hheap, sizeof(uint2) * ((size_t)c->hcap + 1) * n_docs));
      HIPCHK(c, hipMalloc((void**)&c->d_hst, sizeof(uint32_t) * kHtState * (size_t)n_docs));
      HIPCHK(c, hipMalloc((void**)&c->d_hscr, sizeof(int32_t) * 2 * nslots));
      c->h_htree_docs = htree_docs;
      HIPCHK(c, hipMalloc((void**)&c->d_htree_docs, htree_docs.size() * 4));
      HIPCHK(c, hipMemcpy(c->d_htree_docs, htree_docs.data(), htree_docs.size() * 4, hipMemcpyHostToDevice));
    }
  }
  if (n_docs) {
    std::vector<mte_doc_init> dinit(docs, docs + n_docs);
    for (mte_doc_init& di : dinit) {
      di.flags &= ~kInitNl;
      for (uint32_t u = 0; u < di.text_len; u++)
        if (text[di.text_off + u] == 0x0A) {
          di.flags |= kInitNl;
          break;
        }
    }
    HIPCHK(c, hipMemcpy(c->d_inits, dinit.data(), sizeof(mte_doc_init) * n_docs, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpyAsync(c->d_init_props, iprops.data(), sizeof(uint32_t) * iprops.size(),
                             hipMemcpyHostToDevice, c->stream));
  }
  c->h_load_ps.assign(propsets, propsets + (propsets ? n_propsets : 0));
  c->h_load_pe.assign(props, props + (props ? n_props : 0));
  for (const mte_propset& ps : c->h_load_ps)
    if ((uint64_t)ps.first + ps.count > c->h_load_pe.size()) return set_err(c, MTE_E_INVALID_ARG, "bad load propset");
  // text arena restarts with the load text
  c->arena_n = 0;
  c->h_arena.assign(text, text + text_units);
  int rc = grow(c, &c->arena, &c->arena_cap, text_units + 1);
  if (rc) return rc;
  if (text_units)
    HIPCHK(c, hipMemcpyAsync(c->arena, text, text_units * 2, hipMemcpyHostToDevice, c->stream));
  c->arena_n = text_units;
  rc = launch_reset(c);
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MTE_OK;
}

int mte_load_segments(mte_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs) {
  if (!c || !seg_offsets || (n_segs && !segs)) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!c->n_docs) return MTE_OK;
  if (seg_offsets[0] != 0 || seg_offsets[c->n_docs] != n_segs)
    return set_err(c, MTE_E_INVALID_ARG, "seg_offsets must run from 0 to n_segs");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t np = kFieldPlanes + c->kt;
  // planes + the tree word (reloadFromSegments' blocks of 7 per level,
  // mergeTree.ts:607-652), used by the tree pass
  std::vector<uint32_t> img((size_t)(np + 1) * (n_segs ? n_segs : 1), 0u), doc((size_t)(n_segs ? n_segs : 1), 0u);
  // propsets of the load: the load propsets/props were consumed by
  // mte_load_docs; the per-doc initial props are kept, so segment propsets
  // arrive here through the host copy (set by mte_load_docs)
  for (uint32_t d = 0; d < c->n_docs; d++) {
    const uint64_t b = seg_offsets[d], e = seg_offsets[d + 1];
    if (e < b || e - b > c->cap) return set_err(c, MTE_E_CAPACITY, "doc %u: %llu segments > capacity %u", d,
                                                (unsigned long long)(e - b), c->cap);
    for (uint64_t g = b; g < e; g++) {
      const mte_seg& sg = segs[g];
      const bool marker = sg.kind != 0;
      if ((marker && sg.len != 1) || (!marker && (sg.len == 0 || sg.len > 0x7fffffffu)) ||
          (!marker && (uint64_t)sg.text_off + sg.len > c->h_arena.size()) || sg.client < -1 ||
          sg.client >= MTE_MAX_CLIENTS || sg.kind > 0xfffffeu || sg.seq < 0 ||
          (sg.removed_seq != MTE_NOT_REMOVED && sg.removers == 0))
        return set_err(c, MTE_E_INVALID_ARG, "doc %u segment %llu: bad segment", d, (unsigned long long)(g - b));
      img[0 * n_segs + g] = sg.len;
      img[1 * n_segs + g] = (uint32_t)sg.seq;
      img[2 * n_segs + g] = (uint32_t)(sg.removed_seq == MTE_NOT_REMOVED ? kNone : sg.removed_seq);
      img[3 * n_segs + g] = sg.removed_seq == MTE_NOT_REMOVED ? 0u : sg.removers;
      img[4 * n_segs + g] = (uint32_t)(sg.client + 1) | (sg.kind << 8);
      // a marker of an MTE_DOC_REFS document is named by its index in the load
      // (above every arena offset), as an inserted one by its reserved unit
      img[5 * n_segs + g] = marker ? (c->h_refs[d] ? 0x80000000u + (uint32_t)(g - b) : 0u) : sg.text_off;
      {
        const uint64_t nd = e - b, k = g - b;
        int depth = 1;
        for (uint64_t w = 7; w < nd; w *= 7) depth++;
        uint32_t h = 0;
        if (k == 0) h = (uint32_t)depth;
        else {
          uint64_t w = 7;
          for (int lv = 1; lv < depth && k % w == 0; lv++, w *= 7) h = (uint32_t)lv;
        }
        bool nl = false;
        for (uint32_t u = 0; !marker && u < sg.len && !nl; u++) nl = c->h_arena[sg.text_off + u] == 0x0A;
        img[(size_t)np * n_segs + g] = h | (sg.propset != MTE_NO_PROPS ? kTPo : 0u) | ((uint32_t)(k + 1) << 8) |
                                       (nl ? kTNl : 0u);
      }
      if (sg.propset != MTE_NO_PROPS) {
        if (sg.propset >= c->h_load_ps.size())
          return set_err(c, MTE_E_INVALID_ARG, "doc %u segment %llu: bad propset", d, (unsigned long long)(g - b));
        const mte_propset ps = c->h_load_ps[sg.propset];
        for (uint32_t t = 0; t < ps.count; t++) {
          const mte_prop p = c->h_load_pe[ps.first + t];
          if (p.key < c->n_keys) img[(uint64_t)(kFieldPlanes + p.key) * n_segs + g] = p.value;
          if (p.key < MTE_MAX_KEYS && sg.kind == 0) c->key_text[p.key] = 1;  // a text segment's key (kPack4 side key)
        }
      }
      doc[g] = d;
    }
  }
  free_image(c);
  if (!n_segs) return launch_reset(c);
  // planes with one value throughout (config 5's preloaded one-unit segments:
  // all but the text offsets and tree words) are not read back at each reset
  c->img_uc = ImgConst{};
  for (uint32_t p = 0; p < np && p < 16; p++) {
    const uint32_t* v = img.data() + (size_t)p * n_segs;
    bool same = true;
    for (uint64_t g = 1; g < n_segs && same; g++) same = v[g] == v[0];
    if (same) {
      c->img_uc.mask |= 1u << p;
      c->img_uc.val[p] = v[0];
    }
  }
  HIPCHK(c, hipMalloc((void**)&c->d_img, img.size() * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_img_doc, doc.size() * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_img_off, ((size_t)c->n_docs + 1) * 8));
  HIPCHK(c, hipMemcpy(c->d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_img_doc, doc.data(), doc.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_img_off, seg_offsets, ((size_t)c->n_docs + 1) * 8, hipMemcpyHostToDevice));
  c->n_img = n_segs;
  int rc = launch_reset(c);
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MTE_OK;
}

int mte_submit(mte_ctx* c, const mte_batch* b) {
  if (!c || !b || b->n_docs != c->n_docs || !b->op_offsets) return MTE_E_INVALID_ARG;
  if (b->op_offsets[0] != 0 || b->op_offsets[b->n_docs] != b->n_ops) return set_err(c, MTE_E_INVALID_ARG, "op_offsets");
  for (uint32_t d = 0; d < b->n_docs; d++)
    if (b->op_offsets[d + 1] < b->op_offsets[d]) return set_err(c, MTE_E_INVALID_ARG, "op_offsets not sorted");
  for (uint32_t i = 0; i < b->n_propsets; i++)
    if ((uint64_t)b->propsets[i].first + b->propsets[i].count > b->n_props)
      return set_err(c, MTE_E_INVALID_ARG, "propset %u out of range", i);
  if (c->arena_n + b->text_units >= (1ull << 32)) return set_err(c, MTE_E_OOM, "text arena exceeds 2^32 units");
  if (c->d_refs && c->arena_n + b->text_units >= (1ull << 31))  // loaded markers are named above 2^31
    return set_err(c, MTE_E_OOM, "text arena of a context with local references exceeds 2^31 units");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if (!c->up_stream) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) HIPCHK(c, hipEventCreateWithFlags(&c->slot_ev[i], hipEventDisableTiming));
  }
  // the other slot than the one mte_run replays now; its buffers are written
  // once the last run that read them is done
  const int w = c->submitted ? c->rslot ^ 1 : c->rslot;
  if (c->tail.joinable() && w == c->tail_slot) JOIN_TAIL(c);  // a second submit without mte_run
  HIPCHK(c, hipStreamWaitEvent(c->up_stream, c->slot_ev[w], 0));
  // the replay kernels read the records in place; kRecPad zeroed records
  // follow the last one for the L2 prefetch that runs ahead
  if ((rc = grow(c, &c->d_ops_s[w], &c->ops_cap_s[w], b->n_ops + kRecPad))) return rc;
  HIPCHK(c, hipMemsetAsync(c->d_ops_s[w] + b->n_ops, 0, kRecPad * sizeof(mte_op), c->up_stream));
  if ((rc = grow(c, &c->d_off_s[w], &c->off_cap_s[w], (uint64_t)b->n_docs + 1))) return rc;
  if ((rc = grow(c, &c->d_ps_s[w], &c->ps_cap_s[w], (uint64_t)b->n_propsets + 1))) return rc;
  if ((rc = grow(c, &c->d_pe_s[w], &c->pe_cap_s[w], (uint64_t)b->n_props + 1))) return rc;
  if ((rc = grow(c, &c->d_cps_s[w], &c->cps_cap_s[w], 2 * ((uint64_t)b->n_propsets + 1)))) return rc;
  if (b->n_ops) {
    // every record is validated on the way (no kernel may index out of bounds);
    // the host validates and stages while the previous batch may replay
    uint64_t bad = 0;
    const char* why = "";
    if ((rc = upload_ops(c, b, w, &bad, &why)))
      return rc == MTE_E_INVALID_ARG ? set_err(c, rc, "op %llu: %s", (unsigned long long)bad, why) : rc;
  } else {
    c->h_text_ps.clear();
    c->h_rel_s[w].clear();
  }
  // append batch text to the arena (a running replay reads only below arena_n;
  // growing it waits for the replay)
  if ((rc = grow(c, &c->arena, &c->arena_cap, c->arena_n + b->text_units + 1, true, c->arena_n))) return rc;
  if (b->text_units)
    HIPCHK(c, hipMemcpyAsync(c->arena + c->arena_n, b->text, b->text_units * 2, hipMemcpyHostToDevice, c->up_stream));
  c->h_arena.insert(c->h_arena.end(), b->text, b->text + b->text_units);
  c->text_base_s[w] = (uint32_t)c->arena_n;
  c->arena_n += b->text_units;
  HIPCHK(c, hipMemcpyAsync(c->d_off_s[w], b->op_offsets, ((uint64_t)b->n_docs + 1) * 8, hipMemcpyHostToDevice,
                           c->up_stream));
  if (b->n_propsets)
    HIPCHK(c, hipMemcpyAsync(c->d_ps_s[w], b->propsets, b->n_propsets * sizeof(mte_propset), hipMemcpyHostToDevice,
                             c->up_stream));
  if (b->n_props)
    HIPCHK(c, hipMemcpyAsync(c->d_pe_s[w], b->props, b->n_props * sizeof(mte_prop), hipMemcpyHostToDevice,
                             c->up_stream));
  if (!c->h_sdocs.empty()) {
    std::vector<uint32_t> order(c->h_sdocs);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
      return b->op_offsets[x + 1] - b->op_offsets[x] > b->op_offsets[y + 1] - b->op_offsets[y];
    });
    std::vector<uint8_t> in(b->n_docs, 0);
    for (uint32_t d : order) in[d] = 1;
    for (uint32_t d = 0; d < b->n_docs; d++)
      if (!in[d]) order.push_back(d);
    if ((rc = grow(c, &c->d_sorder_s[w], &c->sorder_cap_s[w], (uint64_t)b->n_docs))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_sorder_s[w], order.data(), (size_t)b->n_docs * 4, hipMemcpyHostToDevice,
                             c->up_stream));
    HIPCHK(c, hipStreamSynchronize(c->up_stream));  // `order` goes out of scope
  }
  if (!c->h_htree_docs.empty()) {
    // the HBM tree pass's documents, most records first (the long chains start first)
    std::vector<uint32_t>& ho = c->h_hord;
    ho = c->h_htree_docs;
    std::stable_sort(ho.begin(), ho.end(), [&](uint32_t x, uint32_t y) {
      return b->op_offsets[x + 1] - b->op_offsets[x] > b->op_offsets[y + 1] - b->op_offsets[y];
    });
    if ((rc = grow(c, &c->d_hord_s[w], &c->hord_cap_s[w], (uint64_t)ho.size()))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_hord_s[w], ho.data(), ho.size() * 4, hipMemcpyHostToDevice, c->up_stream));
  }
  c->hord_ok_s[w] = !c->h_htree_docs.empty();
  if (!c->h_rel_s[w].empty()) {
    if ((rc = grow(c, &c->d_rel_s[w], &c->rel_cap_s[w], (uint64_t)c->h_rel_s[w].size()))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_rel_s[w], c->h_rel_s[w].data(), c->h_rel_s[w].size() * 4, hipMemcpyHostToDevice,
                             c->up_stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->up_stream));  // host buffers may be freed after return
  // delta event regions of the MTE_DOC_EVENTS docs (per_op x records + 256
  // each); a document with slide events also gets 2 x its reference slots in
  // use for each record that can slide references (a remote remove, an ack):
  // its slides and the MTE_DELTA_REFPOS snapshot after them
  {
    std::vector<uint64_t>& off = c->h_dl_off_s[w];
    off.assign((size_t)b->n_docs + 1, 0);
    bool any = false;
    for (uint32_t d = 0; d < b->n_docs; d++) {
      const bool e = d < c->h_events.size() && c->h_events[d];
      any = any || e;
      uint64_t extra = 0;
      if (e && d < c->h_slides.size() && c->h_slides[d]) {
        uint32_t hi = c->h_ref_hi[d];
        uint64_t sliding = 0;
        for (uint64_t i = b->op_offsets[d]; i < b->op_offsets[d + 1]; i++) {
          const mte_op& o = b->ops[i];
          if (o.type == MTE_OP_REF && (uint32_t)o.pos2 + 1 > hi) hi = (uint32_t)o.pos2 + 1;
          if ((o.type == MTE_OP_REMOVE && !(o.flags & MTE_F_LOCAL)) || o.type == MTE_OP_ACK) sliding++;
        }
        c->h_ref_hi[d] = hi;
        extra = sliding * 2 * (uint64_t)hi;
      }
      off[d + 1] = off[d] + (e ? (uint64_t)c->ev_per_op * (b->op_offsets[d + 1] - b->op_offsets[d]) + 256 + extra : 0);
    }
    if (any) {
      if ((rc = grow(c, &c->d_dl_off_s[w], &c->dl_off_cap_s[w], (uint64_t)b->n_docs + 1))) return rc;
      if ((rc = grow(c, &c->d_dl_s[w], &c->dl_cap_s[w], off[b->n_docs] + 1))) return rc;
      if ((rc = grow(c, &c->d_dl_n_s[w], &c->dl_n_cap_s[w], (uint64_t)b->n_docs + 1))) return rc;
      HIPCHK(c, hipMemcpyAsync(c->d_dl_off_s[w], off.data(), off.size() * 8, hipMemcpyHostToDevice, c->up_stream));
      HIPCHK(c, hipMemsetAsync(c->d_dl_n_s[w], 0, ((size_t)b->n_docs + 1) * 4, c->up_stream));
      HIPCHK(c, hipStreamSynchronize(c->up_stream));
    } else {
      off.clear();
    }
  }
  for (uint32_t i = 0; b->props && i < b->n_props; i++) {
    c->max_vid = std::max(c->max_vid, b->props[i].value);
    if (b->props[i].key < MTE_MAX_KEYS)
      c->max_vid_k[b->props[i].key] = std::max(c->max_vid_k[b->props[i].key], b->props[i].value);
  }
  // the keys of every propset a text insert or an annotate used (upload_ops)
  for (uint32_t i = 0; i < b->n_propsets && i < c->h_text_ps.size(); i++)
    if (c->h_text_ps[i]) {
      const mte_propset ps = b->propsets[i];
      for (uint32_t t = 0; t < ps.count; t++)
        if (b->props[ps.first + t].key < MTE_MAX_KEYS) c->key_text[b->props[ps.first + t].key] = 1;
    }
  c->n_ops_s[w] = b->n_ops;
  c->n_propsets_s[w] = b->n_propsets;
  uint64_t mx = 0;
  for (uint32_t d = 0; d < b->n_docs; d++) mx = std::max<uint64_t>(mx, b->op_offsets[d + 1] - b->op_offsets[d]);
  c->max_doc_ops_s[w] = mx;
  c->rslot = w;
  c->d_ops = c->d_ops_s[w];
  c->d_cps = c->d_cps_s[w];
  c->d_off = c->d_off_s[w];
  c->d_ps = c->d_ps_s[w];
  c->d_pe = c->d_pe_s[w];
  c->n_ops = b->n_ops;
  c->n_propsets = b->n_propsets;
  c->batch_text_base = c->text_base_s[w];
  c->submitted = true;
  return MTE_OK;
}

int mte_run(mte_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!c->submitted) return set_err(c, MTE_E_STATE, "mte_run before mte_submit");
  if (!c->n_docs) return MTE_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));  // kernel_ms covers every kernel of the run
  if (!c->d_gdone) HIPCHK(c, hipMalloc((void**)&c->d_gdone, 64));
  hipLaunchKernelGGL(begin_batch_kernel, dim3((c->n_docs + 255) / 256), dim3(256), 0, c->stream, c->hdr, c->stats,
                     c->n_docs, c->d_gdone);
  HIPCHK(c, hipGetLastError());
  ReplayArgs a;
  a.hdr = c->hdr;
  a.planes = (uint32_t*)c->soa.len;
  a.stride = c->soa.plane_stride;
  a.cap = c->cap;
  a.n_docs = c->n_docs;
  a.recs = reinterpret_cast<const uint4*>(c->d_ops);
  a.cps = c->d_cps;
  a.op_off = c->d_off;
  a.ps = c->d_ps;
  a.pe = c->d_pe;
  a.n_keys = c->n_keys;
  a.text_base = c->batch_text_base;
  a.stats = c->stats;
  a.pair_docs = c->d_pairs;
  a.n_pairs = c->n_pairs;
  a.group = c->pass1_group;
  a.wclock = nullptr;
  a.gdone = c->d_gdone;
  a.n_ops = c->n_ops;
  const bool evs = !c->h_dl_off_s[c->rslot].empty();
  a.dl = evs ? c->d_dl_s[c->rslot] : nullptr;
  a.dl_off = evs ? c->d_dl_off_s[c->rslot] : nullptr;
  a.dl_n = evs ? c->d_dl_n_s[c->rslot] : nullptr;
  c->ev_slot = evs ? c->rslot : -1;
  a.refs = c->d_refs;
  a.ref_cap = c->ref_cap;
  a.sorder = c->h_sdocs.empty() ? nullptr : c->d_sorder_s[c->rslot];
  // s_memrealtime runs at 100 MHz: ticks = ms x 1e5, scaled to this batch's
  // ops.  A context's first run has no previous duration: it is estimated from
  // the batch, the larger of a saturated chip's throughput (0.215 ns per op,
  // configs 3 and 4 on one MI355X) and one wave's chain over its documents'
  // ops (0.85 us per op alone on its SIMD, the 1,250-document and config-2
  // batches) -- within a few per cent of the measured pass-1 times
  // (DESIGN.md §6), which is what the schedule's bands need
  double eta_ms = 0.0;
  if (c->last_ms > 0 && c->last_ops > 0) {
    eta_ms = c->last_ms * (double)c->n_ops / c->last_ops;
  } else if (c->n_ops) {
    const double thr = 2.15e-7 * (double)c->n_ops;
    const double chain = 8.5e-4 * (double)c->max_doc_ops_s[c->rslot] * (double)c->pass1_group;
    eta_ms = std::max(thr, chain);
  }
  a.eta = (unsigned long long)(eta_ms * 1e5);
  if (c->wclock_path) {
    if (!c->d_wclock) HIPCHK(c, hipMalloc((void**)&c->d_wclock, 16ull * (c->n_pairs + 1)));
    a.wclock = c->d_wclock;
  }
  if (c->n_rs) {
    hipLaunchKernelGGL(round_sync_kernel, dim3((c->n_rs + 3) / 4), dim3(256), 0, c->stream, c->hdr, a.recs, c->d_off,
                       c->d_rs_docs, c->n_rs);
    HIPCHK(c, hipGetLastError());
  }
  if (const uint32_t nr = (uint32_t)c->h_rel_s[c->rslot].size()) {
    hipLaunchKernelGGL(rel_route_kernel, dim3((nr + 255) / 256), dim3(256), 0, c->stream, c->hdr,
                       c->d_rel_s[c->rslot], nr, c->chunked ? 1 : 0);
    HIPCHK(c, hipGetLastError());
  }
  if (c->n_propsets) {
    hipLaunchKernelGGL(props_kernel, dim3((uint32_t)((c->n_propsets + 255) / 256)), dim3(256), 0, c->stream, c->d_ps,
                       (uint32_t)c->n_propsets, c->d_pe, c->n_keys, c->d_cps);
    HIPCHK(c, hipGetLastError());
  }
  int rc;
  if (c->stats_on)
    rc = c->kt == 0 ? launch_replay<0, true>(c, a) : (c->kt == 4 ? launch_replay<4, true>(c, a) : launch_replay<8, true>(c, a));
  else
    rc = c->kt == 0 ? launch_replay<0, false>(c, a)
                    : (c->kt == 4 ? launch_replay<4, false>(c, a) : launch_replay<8, false>(c, a));
  if (rc) return rc;
  c->ran = true;
  const int slot = c->rslot;
  auto finish = [c, slot]() -> int {
    if (c->n_tree || c->n_htree) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipEventRecord(c->slot_ev[slot], c->stream));  // the slot may be rewritten after this
    return MTE_OK;
  };
  if (!c->tail_fn) return finish();
  // the round phases' host loop goes on on the tail thread; mte_run returns
  std::function<int()> fn = std::move(c->tail_fn);
  c->tail_fn = nullptr;
  c->tail_slot = slot;
  c->tail = std::thread([c, fn, finish]() {
    int r = fn();
    if (!r) r = finish();
    c->tail_rc = r;
  });
  return MTE_OK;
}

int mte_sync(mte_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->ran) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess && ms > 0.f) {
      c->last_ms = ms;
      c->last_ops = (double)c->n_ops;
    }
  }
  if (c->wclock_path && c->d_wclock) {
    std::vector<unsigned long long> w(2ull * c->n_pairs);
    HIPCHK(c, hipMemcpy(w.data(), c->d_wclock, w.size() * 8, hipMemcpyDeviceToHost));
    if (FILE* f = std::fopen(c->wclock_path, "wb")) {
      std::fwrite(w.data(), 8, w.size(), f);
      std::fclose(f);
    }
  }
  return MTE_OK;
}

int mte_reset(mte_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  return launch_reset(c);
}

int mte_digest_device(mte_ctx* c, void* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!n_docs) return MTE_OK;
  HIPCHK(c, hipSetDevice(c->device));
  DigestArgs a;
  a.hdr = c->hdr;
  a.soa = c->soa;
  a.cap = c->cap;
  a.n_keys = c->n_keys;
  a.n_docs = c->n_docs;
  a.arena = c->arena;
  a.pow1 = c->d_pow;
  a.pow2 = c->d_pow + 32;
  a.out = (uint64_t*)out;
  if (c->cap > kDgWaveMaxCap) {
    // documents of up to `cap` segments: tile-parallel (dg_*_kernel)
    if (!c->d_dgt) {
      DigestTiles& t = c->dgt;
      t.tpd = (c->cap + kDgTile - 1) / kDgTile;
      const uint64_t nt = (uint64_t)c->n_docs * t.tpd;
      HIPCHK(c, hipMalloc(&c->d_dgt, nt * (4 + 24) + 4ull * c->n_docs + 64));
      t.part = (uint64_t*)c->d_dgt;
      t.tsum = (int32_t*)(t.part + 3 * nt);
      t.tot = t.tsum + nt;
    }
    const uint64_t nt = (uint64_t)n_docs * c->dgt.tpd;
    const uint32_t tb = (uint32_t)((nt + 3) / 4);
    hipLaunchKernelGGL(dg_len_kernel, dim3(tb), dim3(256), 0, c->stream, a, c->dgt);
    hipLaunchKernelGGL(dg_scan_kernel, dim3(n_docs), dim3(256), 0, c->stream, a, c->dgt);
    hipLaunchKernelGGL(dg_tile_kernel, dim3(tb), dim3(256), 0, c->stream, a, c->dgt);
    hipLaunchKernelGGL(dg_final_kernel, dim3((n_docs + 3) / 4), dim3(256), 0, c->stream, a, c->dgt);
  } else {
    hipLaunchKernelGGL(digest_kernel, dim3((n_docs + kDocsPerBlock - 1) / kDocsPerBlock), dim3(256), 0, c->stream, a);
  }
  HIPCHK(c, hipGetLastError());
  return MTE_OK;
}

int mte_digest(mte_ctx* c, uint64_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!n_docs) return MTE_OK;
  int rc = mte_digest_device(c, c->d_digest, n_docs);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(out, c->d_digest, sizeof(uint64_t) * 4 * n_docs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MTE_OK;
}

int mte_doc_status(mte_ctx* c, int32_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!n_docs) return MTE_OK;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<DocHdr> h(n_docs);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->hdr, sizeof(DocHdr) * n_docs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < n_docs; i++) out[i] = h[i].status;
  return MTE_OK;
}

int mte_read_doc(mte_ctx* c, uint32_t doc, mte_doc_view* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  DocHdr h;
  HIPCHK(c, hipMemcpyAsync(&h, c->hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t n = (uint32_t)std::max(h.nseg, 0);
  const uint64_t db = (uint64_t)doc * c->cap;
  std::vector<int32_t> len(n + 1), rseq(n + 1);
  std::vector<uint32_t> meta(n + 1), toff(n + 1), props((size_t)(n + 1) * (c->n_keys ? c->n_keys : 1));
  std::vector<uint32_t> tw(n + 1, 0u);  // tree words (legacy documents)
  if (n && c->d_tree && c->h_legacy[doc])
    HIPCHK(c, hipMemcpyAsync(tw.data(), c->d_tree + db, n * 4, hipMemcpyDeviceToHost, c->stream));
  if (n) {
    HIPCHK(c, hipMemcpyAsync(len.data(), c->soa.len + db, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(rseq.data(), c->soa.rseq + db, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(meta.data(), c->soa.meta + db, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(toff.data(), c->soa.toff + db, n * 4, hipMemcpyDeviceToHost, c->stream));
    for (uint32_t k = 0; k < c->n_keys; k++)
      HIPCHK(c, hipMemcpyAsync(props.data() + (size_t)k * n, c->soa.props + k * c->soa.plane_stride + db, n * 4,
                               hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  v->status = h.status;
  v->cur_seq = h.cur_seq;
  v->min_seq = h.min_seq;
  uint32_t length = 0, nt = 0, ns = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (rseq[i] != kNone) continue;  // gatherText: only segments not removed
    const uint32_t kind = meta[i] >> 8;
    if ((tw[i] & kTCont) && ns > 0) {  // a merged leaf reads as one segment
      if (ns - 1 < v->seg_cap && v->seg_len) v->seg_len[ns - 1] += (uint32_t)len[i];
    } else {
      if (ns < v->seg_cap) {
        if (v->seg_len) v->seg_len[ns] = (uint32_t)len[i];
        if (v->seg_kind) v->seg_kind[ns] = kind;
        if (v->seg_props)
          for (uint32_t k = 0; k < c->n_keys; k++) v->seg_props[(size_t)ns * c->n_keys + k] = props[(size_t)k * n + i];
      }
      ns++;
    }
    length += (uint32_t)len[i];
    if (kind == 0) {
      for (int32_t u = 0; u < len[i]; u++) {
        if (nt < v->text_cap && v->text) v->text[nt] = c->h_arena[toff[i] + (uint32_t)u];
        nt++;
      }
    }
  }
  v->length = length;
  v->n_text = nt;
  v->n_segs = ns;
  return MTE_OK;
}

int mte_set_event_capacity(mte_ctx* c, uint32_t per_op) {
  if (!c || per_op == 0 || per_op > (1u << 16)) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  c->ev_per_op = per_op;
  return MTE_OK;
}

int mte_set_ref_capacity(mte_ctx* c, uint32_t per_doc) {
  if (!c || per_doc == 0 || per_doc > (1u << 20)) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (c->d_refs) return set_err(c, MTE_E_STATE, "mte_set_ref_capacity after mte_load_docs of MTE_DOC_REFS documents");
  c->ref_cap = per_doc;
  return MTE_OK;
}

// referencePositionToLocalPosition (mergeTree.ts:1095-1112) of slots [0, n):
// the own-view position of the segment holding the reference's unit plus its
// offset there (0 on a removed segment); -1 for a detached or unused slot or a
// unit no segment holds any more (a tombstone compacted at minSeq)
static int read_refs_view(mte_ctx* c, uint32_t doc, int32_t* pos, uint32_t n, bool transient) {
  if (!c || (n && !pos) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (c->h_refs.empty() || !c->h_refs[doc]) return set_err(c, MTE_E_INVALID_ARG, "doc %u: no MTE_DOC_REFS", doc);
  if (n > c->ref_cap) return set_err(c, MTE_E_INVALID_ARG, "%u reference slots > capacity %u", n, c->ref_cap);
  HIPCHK(c, hipSetDevice(c->device));
  DocHdr h;
  HIPCHK(c, hipMemcpyAsync(&h, c->hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t ns = (uint32_t)std::max(h.nseg, 0);
  const uint64_t db = (uint64_t)doc * c->cap;
  std::vector<int32_t> len(ns + 1), rseq(ns + 1);
  std::vector<uint32_t> toff(ns + 1);
  std::vector<uint2> rt(n + 1);
  std::vector<uint32_t> tw;  // tree words, for Transient references (their leaf ids)
  if (ns) {
    HIPCHK(c, hipMemcpyAsync(len.data(), c->soa.len + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(rseq.data(), c->soa.rseq + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(toff.data(), c->soa.toff + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
    if (c->d_tree) {
      tw.resize(ns);
      HIPCHK(c, hipMemcpyAsync(tw.data(), c->d_tree + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
    }
  }
  if (n)
    HIPCHK(c, hipMemcpyAsync(rt.data(), c->d_refs + (uint64_t)doc * c->ref_cap, n * sizeof(uint2),
                             hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t r = 0; r < n; r++) {
    pos[r] = -1;
    if ((rt[r].y & kRefLive) && (rt[r].y & kRefTrans)) {
      // a Transient reference: its segment (leaf id) + its offset, the offset
      // dropped once removed; -1 once the segment is gone (mergeTree.ts:1095-1112)
      int64_t p = 0;
      for (uint32_t i = 0; i < ns && i < (uint32_t)tw.size(); i++) {
        const bool head = !(tw[i] & (kTCont | kTEmpty));
        if (head && ((tw[i] >> 8) & (kIdLimit - 1u)) == rt[r].x) {
          pos[r] = (int32_t)(p + (rseq[i] != kNone ? 0 : (int64_t)(rt[r].y & kRefTransOff)));
          break;
        }
        p += rseq[i] == kNone ? len[i] : 0;
      }
      continue;
    }
    if (!(rt[r].y & kRefLive) || ((rt[r].y & kRefDetached) && !(transient && (rt[r].y & kRefOff)))) continue;
    int64_t p = 0;
    for (uint32_t i = 0; i < ns; i++) {
      if (rt[r].x - toff[i] < (uint32_t)len[i]) {
        pos[r] = (int32_t)(p + (rseq[i] != kNone ? 0 : (int64_t)(rt[r].x - toff[i])));
        break;
      }
      p += rseq[i] == kNone ? len[i] : 0;
    }
  }
  return MTE_OK;
}

int mte_read_refs(mte_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) { return read_refs_view(c, doc, pos, n, false); }

int mte_read_refs_transient(mte_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) {
  return read_refs_view(c, doc, pos, n, true);
}

int mte_read_ref_order(mte_ctx* c, uint32_t doc, int64_t* key, uint32_t n) {
  if (!c || (n && !key) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (c->h_refs.empty() || !c->h_refs[doc]) return set_err(c, MTE_E_INVALID_ARG, "doc %u: no MTE_DOC_REFS", doc);
  if (n > c->ref_cap) return set_err(c, MTE_E_INVALID_ARG, "%u reference slots > capacity %u", n, c->ref_cap);
  HIPCHK(c, hipSetDevice(c->device));
  DocHdr h;
  HIPCHK(c, hipMemcpyAsync(&h, c->hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t ns = (uint32_t)std::max(h.nseg, 0);
  const uint64_t db = (uint64_t)doc * c->cap;
  std::vector<int32_t> len(ns + 1);
  std::vector<uint32_t> toff(ns + 1);
  std::vector<uint2> rt(n + 1);
  if (ns) {
    HIPCHK(c, hipMemcpyAsync(len.data(), c->soa.len + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(toff.data(), c->soa.toff + db, ns * 4, hipMemcpyDeviceToHost, c->stream));
  }
  if (n)
    HIPCHK(c, hipMemcpyAsync(rt.data(), c->d_refs + (uint64_t)doc * c->ref_cap, n * sizeof(uint2),
                             hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t r = 0; r < n; r++) {
    key[r] = -1;
    // a reference off the string still sits on its segment (compareReferencePositions
    // compares its segment's ordinal, referencePositions.ts:81-89)
    if (!(rt[r].y & kRefLive) || ((rt[r].y & kRefDetached) && !(rt[r].y & kRefOff))) continue;
    int64_t p = 0;
    for (uint32_t i = 0; i < ns; i++) {
      if (rt[r].x - toff[i] < (uint32_t)len[i]) {
        key[r] = p + (int64_t)(rt[r].x - toff[i]);
        break;
      }
      p += len[i];
    }
  }
  return MTE_OK;
}

int mte_read_deltas(mte_ctx* c, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  *n = 0;
  if (c->h_events.empty() || !c->h_events[doc]) return set_err(c, MTE_E_INVALID_ARG, "doc %u: no MTE_DOC_EVENTS", doc);
  if (c->ev_slot < 0) return MTE_OK;  // no batch with events ran yet
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int sl = c->ev_slot;
  uint32_t cnt = 0;
  HIPCHK(c, hipMemcpy(&cnt, c->d_dl_n_s[sl] + doc, 4, hipMemcpyDeviceToHost));
  const uint64_t b0 = c->h_dl_off_s[sl][doc], room = c->h_dl_off_s[sl][doc + 1] - b0;
  *n = cnt;
  if (cnt > room) return set_err(c, MTE_E_CAPACITY, "doc %u: %u delta events, room for %llu (mte_set_event_capacity)",
                                 doc, cnt, (unsigned long long)room);
  const uint64_t k = std::min<uint64_t>(cap, cnt);
  if (out && k) HIPCHK(c, hipMemcpy(out, c->d_dl_s[sl] + b0, k * sizeof(mte_delta), hipMemcpyDeviceToHost));
  return MTE_OK;
}

int mte_read_segments(mte_ctx* c, uint32_t doc, mte_seg_list* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  DocHdr h;
  HIPCHK(c, hipMemcpyAsync(&h, c->hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint32_t n = (uint32_t)std::max(h.nseg, 0);
  const uint64_t db = (uint64_t)doc * c->cap;
  const uint32_t np = kFieldPlanes + c->n_keys;
  std::vector<uint32_t> pl((size_t)np * (n + 1));
  std::vector<uint32_t> tw(n + 1, 0u);
  if (n && c->d_tree && c->h_legacy[doc])
    HIPCHK(c, hipMemcpyAsync(tw.data(), c->d_tree + db, n * 4, hipMemcpyDeviceToHost, c->stream));
  for (uint32_t p = 0; p < np && n; p++)
    HIPCHK(c, hipMemcpyAsync(pl.data() + (size_t)p * n, reinterpret_cast<const uint32_t*>(c->soa.len) +
                                                             p * c->soa.plane_stride + db,
                             n * 4, hipMemcpyDeviceToHost, c->stream));
  // the removers of short ids >= 32 (mte_htree.h kRmHiPlane): mte_seg.removers has 32 bits
  std::vector<uint32_t> rmh;
  if (n && !c->h_local.empty() && c->h_local[doc]) {
    rmh.resize(n);
    HIPCHK(c, hipMemcpyAsync(rmh.data(), reinterpret_cast<const uint32_t*>(c->soa.len) +
                                             (uint64_t)(kFieldPlanes + 3 * c->kt + 5) * c->soa.plane_stride + db,
                             n * 4, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < (uint32_t)rmh.size(); i++)
    if (rmh[i] && !(tw[i] & kTEmpty) && (int32_t)pl[2 * (size_t)n + i] != kNone)
      return set_err(c, MTE_E_UNSUPPORTED, "doc %u: a segment removed by a short id >= 32 (mte_seg.removers)", doc);
  uint64_t nt = 0;
  uint64_t m = 0;  // segments out (a tree pass placeholder is none, a merged leaf one)
  for (uint32_t i = 0; i < n; i++) {
    const int32_t len = (int32_t)pl[i], rseq = (int32_t)pl[2 * (size_t)n + i];
    const uint32_t meta = pl[4 * (size_t)n + i], kind = meta >> 8;
    if (tw[i] & kTEmpty) continue;
    if ((tw[i] & kTCont) && m > 0) {
      if (m - 1 < v->seg_cap && v->segs) v->segs[m - 1].len += (uint32_t)len;
      const uint32_t toff = pl[5 * (size_t)n + i];
      for (int32_t u = 0; u < len; u++, nt++)
        if (nt < v->text_cap && v->text) v->text[nt] = c->h_arena[toff + (uint32_t)u];
      continue;
    }
    const uint64_t io = m++;
    if (io < v->seg_cap && v->segs) {
      mte_seg& s = v->segs[io];
      s.text_off = kind == 0 ? (uint32_t)nt : 0u;
      s.len = (uint32_t)len;
      s.seq = (int32_t)pl[(size_t)n + i];
      s.removed_seq = rseq == kNone ? MTE_NOT_REMOVED : rseq;
      s.removers = rseq == kNone ? 0u : pl[3 * (size_t)n + i];
      s.client = (int32_t)(meta & 0xffu) - 1;
      s.kind = kind;
      s.propset = MTE_NO_PROPS;
      if (v->props)
        for (uint32_t k = 0; k < c->n_keys; k++)
          v->props[(size_t)io * c->n_keys + k] = pl[(size_t)(kFieldPlanes + k) * n + i];
    }
    if (kind == 0) {
      const uint32_t toff = pl[5 * (size_t)n + i];
      for (int32_t u = 0; u < len; u++, nt++)
        if (nt < v->text_cap && v->text) v->text[nt] = c->h_arena[toff + (uint32_t)u];
    }
  }
  v->n_segs = m;
  v->n_text = nt;
  return MTE_OK;
}

int mte_set_stats(mte_ctx* c, int enable) {
  if (!c) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  c->stats_on = enable != 0;
  return MTE_OK;
}

// ---- node level over RCCL (include/mte.h) ----------------------------------

#define NCCLCHK(ctx, expr)                                                                        \
  do {                                                                                            \
    ncclResult_t r_ = (expr);                                                                     \
    if (r_ != ncclSuccess) return set_err(ctx, MTE_E_HIP, "%s: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

int mte_comm_unique_id(uint8_t id[MTE_COMM_ID_BYTES]) {
  if (!id) return MTE_E_INVALID_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return MTE_E_HIP;
  static_assert(sizeof(u) == MTE_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, MTE_COMM_ID_BYTES);
  return MTE_OK;
}

int mte_comm_init(mte_ctx* c, int world, int rank, const uint8_t id[MTE_COMM_ID_BYTES]) {
  if (!c || !id || world < 1 || rank < 0 || rank >= world) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (c->comm) return set_err(c, MTE_E_STATE, "mte_comm_init: already initialised");
  HIPCHK(c, hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, MTE_COMM_ID_BYTES);
  ncclComm_t comm = nullptr;
  NCCLCHK(c, ncclCommInitRank(&comm, world, u, rank));
  c->cref = new CommRef;
  c->cref->comm = comm;
  c->comm = comm;
  c->world = world;
  c->rank = rank;
  return MTE_OK;
}

int mte_comm_share(mte_ctx* c, const mte_ctx* src) {
  if (!c || !src || !src->comm || src->device != c->device) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (c->comm) return set_err(c, MTE_E_STATE, "mte_comm_share: already has a communicator");
  src->cref->refs.fetch_add(1);
  c->cref = src->cref;
  c->comm = src->comm;
  c->world = src->world;
  c->rank = src->rank;
  return MTE_OK;
}

namespace {
int comm_staging(mte_ctx* c, uint64_t n) {
  if (n <= c->comm_cap) return MTE_OK;
  if (c->d_comm) HIPCHK(c, hipFree(c->d_comm));
  c->d_comm = nullptr;
  HIPCHK(c, hipMalloc((void**)&c->d_comm, n * sizeof(uint64_t)));
  c->comm_cap = n;
  return MTE_OK;
}
}  // namespace

int mte_comm_allreduce_f64(mte_ctx* c, double* v, int op) {
  if (!c || !v || (op != MTE_COMM_SUM && op != MTE_COMM_MAX)) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!c->comm) return set_err(c, MTE_E_STATE, "mte_comm_init first");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = comm_staging(c, 1);
  if (rc) return rc;
  double* d = reinterpret_cast<double*>(c->d_comm);
  HIPCHK(c, hipMemcpyAsync(d, v, sizeof(double), hipMemcpyHostToDevice, c->stream));
  NCCLCHK(c, ncclAllReduce(d, d, 1, ncclFloat64, op == MTE_COMM_SUM ? ncclSum : ncclMax, c->comm, c->stream));
  HIPCHK(c, hipMemcpyAsync(v, d, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MTE_OK;
}

int mte_comm_barrier(mte_ctx* c) {
  double one = 1.0;
  return mte_comm_allreduce_f64(c, &one, MTE_COMM_SUM);
}

int mte_comm_world(const mte_ctx* c, int32_t* world, int32_t* rank) {
  if (!c || !world || !rank) return MTE_E_INVALID_ARG;
  *world = c->world;
  *rank = c->rank;
  return MTE_OK;
}

int mte_comm_gather_digests(mte_ctx* c, uint64_t* out, uint64_t out_cap, uint32_t docs_per_rank) {
  if (!c || !out || docs_per_rank < c->n_docs) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  if (!c->comm) return set_err(c, MTE_E_STATE, "mte_comm_init first");
  if (out_cap < 4ull * docs_per_rank * (uint64_t)c->world)
    return set_err(c, MTE_E_INVALID_ARG, "mte_comm_gather_digests: out holds %llu uint64, needs world %d x %u docs x 4",
                   (unsigned long long)out_cap, c->world, docs_per_rank);
  HIPCHK(c, hipSetDevice(c->device));
  const uint64_t per = 4ull * docs_per_rank;
  int rc = comm_staging(c, per * (uint64_t)(c->world + 1));
  if (rc) return rc;
  uint64_t* send = c->d_comm + per * (uint64_t)c->world;  // after the receive area
  HIPCHK(c, hipMemsetAsync(send, 0, per * sizeof(uint64_t), c->stream));
  if (c->n_docs && (rc = mte_digest_device(c, send, c->n_docs))) return rc;
  NCCLCHK(c, ncclAllGather(send, c->d_comm, per, ncclUint64, c->comm, c->stream));
  HIPCHK(c, hipMemcpyAsync(out, c->d_comm, per * (uint64_t)c->world * sizeof(uint64_t), hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MTE_OK;
}

int mte_comm_destroy(mte_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  HIPCHK(c, hipSetDevice(c->device));
  const ncclResult_t r = comm_release(c);
  if (r != ncclSuccess) return set_err(c, MTE_E_HIP, "ncclCommDestroy: %s", ncclGetErrorString(r));
  c->world = 1;
  c->rank = 0;
  return MTE_OK;
}

int mte_stats_get(mte_ctx* c, mte_stats* o) {
  if (!c || !o) return MTE_E_INVALID_ARG;
  JOIN_TAIL(c);
  std::memset(o, 0, sizeof(*o));
  if (!c->n_docs) return MTE_OK;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<unsigned long long> s((size_t)c->n_docs * kNumStats);
  unsigned long long chunk_canon = 0;
  HIPCHK(c, hipMemcpyAsync(s.data(), c->stats, s.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t d = 0; d < c->n_docs; d++) {
    const unsigned long long* x = &s[(size_t)d * kNumStats];
    o->ops_applied += x[kStOps];
    o->segs_scanned += x[kStScanned];
    o->segs_written += x[kStWritten];
    o->prop_writes += x[kStPwrites];
    o->units_inserted += x[kStUnits];
    if (x[kStMaxSegs] > o->max_segs) o->max_segs = x[kStMaxSegs];
    chunk_canon += x[kStChunkCanon];
    o->chunk_scanned += x[kStChunkScan];
  }
  if (c->ran) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) o->kernel_ms = ms;
  }
  if (c->d_hprof) {  // MTE_HTREE_PROF: one line of phase clocks, then zeroed
    unsigned long long hp[kHtProf];
    HIPCHK(c, hipMemcpyAsync(hp, c->d_hprof, sizeof(hp), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_hprof, 0, sizeof(hp), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (FILE* f = std::fopen(c->hprof_path, "a")) {
      for (int q = 0; q < kHtProf; q++) std::fprintf(f, q ? " %llu" : "%llu", hp[q]);
      std::fprintf(f, "\n");
      std::fclose(f);
    }
  }
  // ops of the chunked pass count the slots and summary
  // entries they scanned instead of the document's S_live
  // the round phases' own bytes of the last run (RoundArgs::acct)
  o->round_bytes = 0.0;
  if (c->chunked && c->rd.acct && c->n_docs) {
    std::vector<unsigned long long> ac(c->n_docs);
    HIPCHK(c, hipMemcpyAsync(ac.data(), c->rd.acct, sizeof(unsigned long long) * c->n_docs, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (unsigned long long v : ac) o->round_bytes += (double)v;
  }
  const double scanned = (double)(o->segs_scanned - chunk_canon) + (double)o->chunk_scanned;
  o->algo_bytes = 32.0 * (double)o->ops_applied + 20.0 * scanned + 20.0 * (double)o->segs_written +
                  4.0 * (double)o->prop_writes + 2.0 * (double)o->units_inserted;
  return MTE_OK;
}

}  // extern "C"
