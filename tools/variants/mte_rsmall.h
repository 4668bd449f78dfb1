// mte_rsmall.h — round phases for pass-1-sized documents: a workgroup of four
// waves per document when the batch is too small to fill the SIMDs.
//
// At 1,250 documents per GPU (the 10k-document job on 8 GPUs) pass 1 holds one
// document per wave and a SIMD about one wave, so every op costs its full
// instruction latency.  The round phases' argument (mte_round.h)
// holds for any document: within a run — ops that all carry refSeq R = the
// document's currentSeq and one minSeq M — the perspective of an op of client
// c is the run-start state plus c's own earlier ops of the run, so each
// client's ops resolve to (chunk, chunk start) on a column of its own, and
// each chunk can apply its ops in seq order alone.  Here the document sits in
// LDS; per run (up to 64 ops, one record batch):
//   1. four chunk boundaries, each at a segment that is not removed, so no chunk
//      starts with a leaf a perspective could skip as undefined (legacy
//      calc: removed before its refSeq, or a concurrent insert its own client
//      removed); an insert therefore always belongs to the chunk holding the
//      unit before its position, and appending there is where the
//      op-after-op pass puts it;
//   2. wave 0 resolves the run: per op, the column of its client (four chunk
//      lengths, one lane per client) gives the chunk(s) and their starts in
//      the op's perspective, as scalar arithmetic; the sub-ops land in each
//      chunk's bucket already in seq order;
//   3. each wave loads its chunk into registers and applies its bucket with
//      the segment step every pass shares (seg_op_v, positions relative to
//      the chunk start); the chunks go back to LDS end to end, and if minSeq
//      moved to M the tombstones at or below it go (zamboni,
//      mergeTree.ts:1077-1093) — after the run instead of after its first op,
//      which leaves every op's place among the segments that stay unchanged.
// A run that does not fit (an insert past the end — the op-after-op pass
// reports MTE_E_INSERT_FAILED at that op —, a full bucket, a chunk over 126
// slots) replays op after op on wave 0 with the whole document in registers;
// a document that outgrows that, or reaches an op that is not part of a run,
// is written back at its cursor and pass 1 / 2 go on from there.  Statistics
// runs never take this path.
#pragma once

#include "mte_replay.h"

namespace mte {

constexpr int kRsW = 4;                          // waves (chunks) per document
constexpr int kRsE = 2;                          // chunk registers: 128 slots per wave
constexpr int kRsCap = kRsW * kRsE * kWave;      // 512 LDS slots per document
constexpr int kRsChunkMax = kRsE * kWave - 2;    // 126
constexpr int kRsBucket = 60;                    // sub-ops per chunk and run
constexpr int kRsGrowMax = 400;                  // past this the document goes back to pass 1 / 2

template <int K>
struct RsLds {
  uint32_t pl[kFieldPlanes + K][kRsCap];
  uint2 bk[kRsW][kRsBucket];  // per chunk: (op index in the run, chunk start)
  int32_t b[kRsW + 1];        // chunk boundaries
  int32_t cnt[kRsW];          // chunk sizes after the apply / kept slots in the zamboni
  int32_t vis[kRsW];          // run-start visible length per chunk
  int32_t bn[kRsW];           // sub-ops per chunk
  int32_t col[MTE_MAX_CLIENTS][kRsW];  // each client's column during the resolve
  int32_t n, k, cur, minq, status, flag, stop;
  int32_t seqr;     // a run left part-way by the op-after-op path: its refSeq (else INT32_MIN)
  int32_t diag[4];  // diagnostics (MTE_WAVE_CLOCK runs): parallel runs, op-after-op runs, stop reason, ops
};

// chunk [b, b + n) of the LDS planes into registers (lane-major, padding past n)
template <int E, int K>
__device__ __forceinline__ void rs_load(Regs<E, K>& R, const RsLds<K>& S, int b, int n) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    const bool v = i < n;
    const int x = b + (v ? i : 0);
    R.len[j] = v ? (int32_t)S.pl[0][x] : 0;
    R.seq[j] = v ? (int32_t)S.pl[1][x] : 0;
    R.rseq[j] = v ? (int32_t)S.pl[2][x] : kPad;
    R.rmask[j] = v ? S.pl[3][x] : 0u;
    R.meta[j] = v ? S.pl[4][x] : 0u;
    R.toff[j] = v ? S.pl[5][x] : 0u;
#pragma unroll
    for (int k = 0; k < K; k++) R.pr[k][j] = v ? S.pl[kFieldPlanes + k][x] : 0u;
  }
}

template <int E, int K>
__device__ __forceinline__ void rs_store(const Regs<E, K>& R, RsLds<K>& S, int b, int n) {
  const int base = lane_id() * E;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const int i = base + j;
    if (i < n && b + i < kRsCap) {
      const int x = b + i;
      S.pl[0][x] = (uint32_t)R.len[j];
      S.pl[1][x] = (uint32_t)R.seq[j];
      S.pl[2][x] = (uint32_t)R.rseq[j];
      S.pl[3][x] = R.rmask[j];
      S.pl[4][x] = R.meta[j];
      S.pl[5][x] = R.toff[j];
#pragma unroll
      for (int k = 0; k < K; k++) S.pl[kFieldPlanes + k][x] = R.pr[k][j];
    }
  }
}

// record q of the batch each lane holds (lane j: record j), as the op vector
__device__ __forceinline__ s8v rs_rec(const uint32_t (&rb)[8], int q) {
  s8v op;
#pragma unroll
  for (int i = 0; i < 8; i++) op[i] = (int32_t)rdlane(rb[i], q);
  return op;
}

// zamboni at M (mergeTree.ts:1077-1093): drop removedSeq <= M, all waves
template <int K>
__device__ __forceinline__ void rs_zamboni(RsLds<K>& S, int32_t M) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int n0 = S.n;
  bool keep[kRsE];
  uint32_t v[kFieldPlanes + K][kRsE];
  int32_t kc = 0;
#pragma unroll
  for (int j = 0; j < kRsE; j++) {
    const int i = w * kRsE * kWave + l * kRsE + j;
    keep[j] = i < n0 && (int32_t)S.pl[2][i] > M;
    kc += keep[j] ? 1 : 0;
#pragma unroll
    for (int p = 0; p < kFieldPlanes + K; p++) v[p][j] = i < n0 ? S.pl[p][i] : 0u;
  }
  const int32_t incl = wave_incl_scan(kc);
  if (l == kWave - 1) S.cnt[w] = incl;
  __syncthreads();
  int32_t d = incl - kc;
  int32_t tot = 0;
  for (int u = 0; u < kRsW; u++) {
    d += u < w ? S.cnt[u] : 0;
    tot += S.cnt[u];
  }
  __syncthreads();  // every slot is in registers before any is overwritten
#pragma unroll
  for (int j = 0; j < kRsE; j++) {
    if (keep[j]) {
#pragma unroll
      for (int p = 0; p < kFieldPlanes + K; p++) S.pl[p][d] = v[p][j];
    }
    d += keep[j] ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) S.n = tot;
  __syncthreads();
}

// one document per workgroup of kRsW waves: a.pair_docs[blockIdx.x] (pass 1
// with one document per slot)
template <int K>
__global__ __launch_bounds__(kRsW * kWave, 5) void rsmall_kernel(ReplayArgs a) {
  __shared__ RsLds<K> S;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int doc = (int)a.pair_docs[blockIdx.x];
  if (doc < 0) return;
  DocRun D;
  run_init(D, a, doc, false);
  if (!D.running || (D.flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS)) || D.n > kRsGrowMax) return;
  const bool newcalc = (D.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  uint32_t* hp = a.planes + (uint64_t)doc * a.cap;
  for (int i = (int)threadIdx.x; i < D.n; i += kRsW * kWave) {
#pragma unroll
    for (int p = 0; p < kFieldPlanes + K; p++) S.pl[p][i] = hp[(uint64_t)p * a.stride + i];
  }
  if (threadIdx.x == 0) {
    S.n = D.n;
    S.k = (int32_t)D.k;
    S.cur = D.cur_seq;
    S.minq = D.min_seq;
    S.status = 0;
    S.stop = 0;
    S.seqr = INT32_MIN;
    S.diag[0] = S.diag[1] = S.diag[2] = S.diag[3] = 0;
  }
  __syncthreads();
  uint32_t st[kNumStats] = {};
  constexpr uint32_t kAllowed = MTE_F_MSG_END | MTE_F_MARKER | MTE_F_REWRITE;
  for (;;) {
    const uint32_t k = (uint32_t)S.k;
    const int32_t R = S.cur, m0 = S.minq;
    // a run the op-after-op path left part-way goes on op after op: its ops
    // carry the run's refSeq, below the document's currentSeq by now
    const bool cont = S.seqr != INT32_MIN;
    const int32_t Rr = cont ? S.seqr : R;
    if (S.stop || S.status || k >= D.k1) break;
    // ---- the run: up to 64 records from the cursor (every wave holds them)
    uint32_t rb[8];
    {
      const uint4* p = D.recp + 2 * (k + (uint32_t)l);
      const bool in = k + (uint32_t)l < D.k1;
      const uint4 x = in ? p[0] : make_uint4(0u, 0u, 0u, 0u), y = in ? p[1] : make_uint4(0u, 0u, 0u, 0u);
      rb[0] = x.x, rb[1] = x.y, rb[2] = x.z, rb[3] = x.w, rb[4] = y.x, rb[5] = y.y, rb[6] = y.z, rb[7] = y.w;
    }
    const int32_t M = (int32_t)rdlane(rb[2], 0);
    int len;
    {
      const int32_t s = (int32_t)rb[0];
      const uint32_t type = rb[3] & 0xffu, c = (rb[3] >> 8) & 0xffu, fl = rb[3] >> 16;
      const int32_t up = __shfl_up(s, 1);
      const int32_t below = l == 0 ? R : up;
      const bool in = k + (uint32_t)l < D.k1;
      const bool ok = in && (int32_t)rb[1] == Rr && (int32_t)rb[2] == M && type <= MTE_OP_ANNOTATE &&
                      c < MTE_MAX_CLIENTS && (fl & MTE_F_MSG_END) && !(fl & ~kAllowed) && s > below && M >= m0 &&
                      M <= Rr && (int32_t)rb[4] >= 0 && (int32_t)rb[5] >= 0;
      const uint64_t stopm = __ballot(!ok);
      len = stopm ? __ffsll((long long)stopm) - 1 : kWave;
    }
    if (len == 0) {  // not a run: pass 1 goes on from this op
      if (threadIdx.x == 0) S.diag[2] = 1;
      break;
    }
    const int n = S.n;
    // ---- chunk boundaries: about n / 4 each, every chunk starting at a segment not removed
    if (threadIdx.x == 0) {
      const int q = (n + kRsW - 1) / kRsW;
      S.b[0] = 0;
      for (int u = 1; u < kRsW; u++) {
        int bu = u * q < n ? u * q : n;
        if (bu < S.b[u - 1]) bu = S.b[u - 1];
        while (bu < n && (int32_t)S.pl[2][bu] != kNone) bu++;
        S.b[u] = bu;
      }
      S.b[kRsW] = n;
    }
    __syncthreads();
    const int cb = S.b[w], ce = S.b[w + 1];
    {
      int32_t vs = 0;
      for (int i = cb + l; i < ce; i += kWave) vs += (int32_t)S.pl[2][i] == kNone ? (int32_t)S.pl[0][i] : 0;
      const int32_t t = rdlane(wave_incl_scan(vs), kWave - 1);
      if (l == 0) S.vis[w] = t;
    }
    __syncthreads();
    // ---- resolve (wave 0), all clients at once: step t takes every client's
    // t-th op of the run (lane j: op j), each against its client's column
    if (w == 0 && cont) {
      if (l == 0) S.flag = 4;  // the rest of a run op after op
    } else if (w == 0) {
      const uint32_t w3 = rb[3];
      const int cj = (int)((w3 >> 8) & 31u);
      const bool inrun = l < len;
      // the clients of the run, and each op's rank among its client's ops
      uint32_t pres = inrun ? 1u << cj : 0u;
      for (int off = 32; off >= 1; off >>= 1) pres |= (uint32_t)__shfl_xor((int)pres, off);
      pres = __builtin_amdgcn_readfirstlane(pres);
      int rank = 0, maxrank = 0;
      for (uint32_t m = pres; m; m &= m - 1) {
        const int c = __ffs((int)m) - 1;
        const uint64_t mc = __ballot(inrun && cj == c);
        if (inrun && cj == c)
          rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mc, 0u));
        const int nc = __popcll(mc);
        maxrank = nc > maxrank ? nc : maxrank;
      }
      // every present client's column = the run-start visible lengths
      if (l < MTE_MAX_CLIENTS && ((pres >> l) & 1u)) {
#pragma unroll
        for (int u = 0; u < kRsW; u++) S.col[l][u] = S.vis[u];
      }
      if (l < kRsW) S.bn[l] = 0;
      if (l == 0) S.flag = 0;
      fence_wave();
      const uint32_t type = w3 & 0xffu, flags = w3 >> 16;
      const int32_t pos1 = (int32_t)rb[4], pos2 = (int32_t)rb[5];
      for (int t = 0; t < maxrank; t++) {
        if (inrun && rank == t) {
          int32_t cc[kRsW];
#pragma unroll
          for (int u = 0; u < kRsW; u++) cc[u] = S.col[cj][u];
          if (type == MTE_OP_INSERT) {
            int i0 = -1;
            int32_t ex = 0, run = 0;
#pragma unroll
            for (int u = 0; u < kRsW; u++) {
              const int32_t incl = run + cc[u];
              if (i0 < 0 && incl >= pos1) {
                i0 = u;
                ex = run;
              }
              run = incl;
            }
            if (i0 < 0 || pos1 > run) {
              atomicOr(&S.flag, 1);  // MTE_E_INSERT_FAILED at this op: pass 1 replays it
            } else {
              const int q = atomicAdd(&S.bn[i0], 1);
              if (q < kRsBucket) S.bk[i0][q] = make_uint2((uint32_t)l, (uint32_t)ex);
              const int32_t nlen = (flags & MTE_F_MARKER) ? 1 : pos2;
              S.col[cj][i0] = cc[i0] + nlen;
            }
          } else {
            const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
            int32_t run = 0;
            bool first = true;
#pragma unroll
            for (int u = 0; u < kRsW; u++) {
              const int32_t stu = run, incl = run + cc[u];
              run = incl;
              bool emit = false;
              if (b1 == b2) {
                // ensureIntervalBoundary alone: the first chunk reaching past b1, a split strictly inside it
                if (first && incl > b1) {
                  first = false;
                  emit = stu < b1;
                }
              } else if (cc[u] > 0 && incl > b1 && stu < b2) {
                emit = true;
                if (type == MTE_OP_REMOVE) {
                  const int32_t lo = b1 > stu ? b1 : stu, hi = b2 < incl ? b2 : incl;
                  S.col[cj][u] = cc[u] - (hi - lo);
                }
              }
              if (emit) {
                const int q = atomicAdd(&S.bn[u], 1);
                if (q < kRsBucket) S.bk[u][q] = make_uint2((uint32_t)l, (uint32_t)stu);
              }
            }
          }
        }
        fence_wave();
      }
      if (l < kRsW && (S.bn[l] > kRsBucket || S.b[l + 1] - S.b[l] + 2 * S.bn[l] > kRsChunkMax)) atomicOr(&S.flag, 2);
    }
    __syncthreads();
    if (S.flag) {
      // a run the chunks cannot take (a young document's first rounds land in
      // one chunk): op after op on wave 0 with the whole document in one
      // chunk's registers while it fits, else pass 1 goes on from this run
      if (w == 0) {
        if (n + 2 > kRsChunkMax) {
          if (l == 0) {
            S.stop = 1;
            S.diag[2] = 2;
          }
        } else {
          // as many of the run's ops as the chunk's registers hold (the rest
          // start the next run)
          Regs<kRsE, K> Rg;
          rs_load<kRsE, K>(Rg, S, 0, n);
          int nn = n;
          int32_t cur = R;
          int done = 0, rc = 0;
          for (int j = 0; j < len; j++) {
            if (nn + 2 > kRsChunkMax) break;
            const s8v op = rs_rec(rb, j);
            const uint32_t w3 = (uint32_t)op[3];
            int32_t tot = 0, dlen = 0;
            rc = seg_op_v<kRsE, K, false, false>(Rg, nn, op, w3 & 0xffu, (w3 >> 8) & 0xffu, w3 >> 16, M, newcalc, 0,
                                                 true, tot, dlen, a, st);
            if (rc < 0) break;
            cur = op[0];
            done++;
          }
          rs_store<kRsE, K>(Rg, S, 0, nn);
          if (l == 0) {
            S.n = nn;
            S.k = (int32_t)(k + (uint32_t)done);
            S.cur = cur;
            if (done > 0) S.minq = M;  // the window moves after the run's first op
            if (rc < 0) S.status = rc;
            S.seqr = done < len ? Rr : INT32_MIN;
            if (done == 0 && rc == 0) {
              S.stop = 1;
              S.diag[2] = 2;
            }
            S.diag[1]++;
            S.diag[3] += done;
          }
        }
      }
      __syncthreads();
      // minSeq moved to M after the first op: its tombstones go (as op after op)
      if (S.minq == M && M > m0) rs_zamboni<K>(S, M);
    } else {
      // ---- each wave its chunk and its bucket, in op order
      const int nb = S.bn[w];
      // the bucket sorted by op index: lane q holds entry q, its rank among them
      const uint2 e = l < nb ? S.bk[w][l] : make_uint2(0xffffffffu, 0u);
      uint32_t rk = 0;
      for (int q = 0; q < nb; q++) rk += rdlane(e.x, q) < e.x ? 1u : 0u;
      const int dst = (l < nb ? (int)rk : l) << 2;
      const uint32_t ks = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)e.x);
      const int32_t exs = __builtin_amdgcn_ds_permute(dst, (int)e.y);
      Regs<kRsE, K> Rg;
      int ni = ce - cb;
      rs_load<kRsE, K>(Rg, S, cb, ni);
      int rcs = 0;
      for (int q = 0; q < nb; q++) {
        const int j = (int)uni(rdlane(ks, q));
        const int32_t ex = rdlane(exs, q);
        s8v op = rs_rec(rb, j);
        const uint32_t w3 = (uint32_t)op[3];
        const uint32_t type = w3 & 0xffu;
        // positions relative to the chunk start: the whole-document step on the chunk
        op[4] -= ex;
        if (type != MTE_OP_INSERT) op[5] -= ex;
        int32_t tot = 0, dlen = 0;
        const int rc = seg_op_v<kRsE, K, false, false>(Rg, ni, op, type, (w3 >> 8) & 0xffu, w3 >> 16, M, newcalc, 0,
                                                       true, tot, dlen, a, st);
        rcs = rc != 0 ? rc : rcs;
      }
      if (l == 0) S.cnt[w] = ni;
      __syncthreads();  // every chunk is in registers before any is written back
      int off = 0, tot = 0;
      for (int u = 0; u < kRsW; u++) {
        off += u < w ? S.cnt[u] : 0;
        tot += S.cnt[u];
      }
      rs_store<kRsE, K>(Rg, S, off, ni);
      if (rcs != 0 && l == 0) S.status = MTE_E_STATE;  // resolve guarantees every sub-op fits: an engine bug
      __syncthreads();
      if (threadIdx.x == 0) {
        S.n = tot;
        S.k = (int32_t)(k + (uint32_t)len);
        S.cur = (int32_t)rdlane(rb[0], len - 1);
        S.minq = M;
        S.diag[0]++;
        S.diag[3] += len;
      }
      __syncthreads();
      if (M > m0) rs_zamboni<K>(S, M);
      if (threadIdx.x == 0 && S.n > kRsGrowMax) {
        S.stop = 1;
        S.diag[2] = 3;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  // ---- write back: planes, then the header at the cursor
  const int n = S.n;
  for (int i = (int)threadIdx.x; i < n; i += kRsW * kWave) {
#pragma unroll
    for (int p = 0; p < kFieldPlanes + K; p++) hp[(uint64_t)p * a.stride + i] = S.pl[p][i];
  }
  if (threadIdx.x == 0) {
    DocHdr h = a.hdr[doc];
    h.nseg = n;
    h.min_seq = S.minq;
    h.cur_seq = S.cur;
    h.resume = (uint32_t)S.k;
    if (S.status) h.status = S.status;
    a.hdr[doc] = h;
    if (a.wclock) {  // diagnostics: the run counts in the document's statistics slots
      unsigned long long* sd = a.stats + (size_t)doc * kNumStats;
      sd[0] = (unsigned long long)S.diag[3];
      sd[1] = (unsigned long long)S.diag[0];
      sd[2] = (unsigned long long)S.diag[1];
      sd[3] = S.diag[2] == 0 ? 0ull : 1ull << (20 * (S.diag[2] - 1));  // stop reasons, summable
    }
  }
}

}  // namespace mte
