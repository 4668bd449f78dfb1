// mte_round.h — round phases of the chunked pass (mte_chunk.h): a run of
// concurrent ops replayed chunk-parallel instead of op after op.
//
// A *run* of a document is a stretch of ops k0 .. k1 - 1 that all carry
// refSeq R = the document's currentSeq at k0 and one minSeq M (every op of a
// conflict-farm round: BASELINE config 5).  Within a run the perspective of an
// op of client c is the state at k0 plus c's own earlier ops of the run: every
// other client's insert of the run is invisible to it (seq > R) and every other
// client's remove of the run leaves its segments visible (removedSeq > R).  So
//   * client c's chunk length column (mte_chunk.h: sum[c][i], the chunk-level
//     PartialSequenceLengths.getPartialLength, partialLengths.ts:667-702)
//     changes only by c's own ops — by +inserted units and -the units a remove
//     covers, arithmetic on the column with no segment in sight — and starts
//     from the same round-start column for every client;
//   * so each client's ops resolve to (chunk, the chunk's start in the op's
//     perspective) on their own column, all clients at once (rnd_resolve: one
//     wave per client chain);
//   * an op changes only the chunks it resolved to, and what it does to a chunk
//     depends only on that chunk's content (the segment step seg_op_v, with the
//     op's positions taken relative to the chunk start, as the sequential chunk
//     pass runs it), so replaying every chunk's ops in seq order — each chunk
//     on its own wave, all chunks at once (rnd_apply) — gives every chunk the
//     content the op-after-op replay gives it.
// An insert goes to the chunk holding the unit before its position (the first
// chunk for position 0) and appends there if no slot of that chunk follows
// the position: in a new-length-calc run no segment is undefined to the
// perspective (tombstones with removedSeq <= M are dropped at the re-layout,
// those of the run have removedSeq > R >= M), so the end of chunk i is the
// place the op-after-op pass reaches at the start of chunk i + 1
// (insertingWalk's "before the first leaf at or after pos", mergeTree.ts:1743,
// 1788-1797).  minSeq moves to M before the run instead of after its first op:
// tombstones at or below M are zero-length to every op of the run, so the op
// lands in the same place relative to every segment that stays.
//
// Phases per launch of the chunked pass (host loop, mte_engine.hip):
//   rnd_plan     one wave per document: the run at its op cursor (mode kRound
//                if long enough, else the rest goes to the sequential pass);
//   rnd_scatter  flat planes -> chunks of kChFill segments, dropping
//                removedSeq <= M (zamboni, mergeTree.ts:1077-1093), and the
//                round-start column (visible length per chunk);
//   rnd_resolve  one wave per client chain: positions -> (chunk, start) on the
//                client's column, each sub-op into the chunk's bucket;
//   rnd_apply    one wave per chunk with sub-ops: sort them by op index, load
//                the chunk into registers, seg_op_v each, store;
//   rnd_gather   chunks -> flat planes, the document header advanced to k1.
// Anything the run cannot take — an insert past the end (the op-after-op pass
// reports MTE_E_INSERT_FAILED at that op), a bucket over kRB sub-ops — sets
// the document's flag before any segment is written, and the sequential chunk
// pass replays the same run from the untouched flat planes.  Statistics runs
// (mte_set_stats) always take the sequential pass.
#pragma once

#include "mte_chunk.h"
#include "mte_passes.h"

namespace mte {

__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// one wave per document
__global__ __launch_bounds__(256) void rnd_plan_kernel(ReplayArgs a, RoundArgs rd) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int doc = (int)blockIdx.x * 4 + w;
  if (doc >= (int)a.n_docs) return;
  const DocHdr h = a.hdr[doc];
  const uint64_t kb = a.op_off[doc];
  const uint32_t ktot = (uint32_t)(a.op_off[doc + 1] - kb);
  const bool active = (h.flags & kHdrNeedsEsc) && h.status == 0 && h.resume < ktot;
  uint4 p = make_uint4(kModeIdle, 0u, 0u, 0u);
  if (active) {
    const uint32_t k0 = h.resume;
    uint32_t k1 = k0;
    int32_t M = 0;
    const bool newcalc = (h.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
    if (!rd.last && newcalc) {
      const uint4* recp = a.recs + 2 * (kb + k0);
      const int32_t R = h.cur_seq;
      const uint32_t nleft = ktot - k0;
      int32_t prev = R;  // seq of the op before this batch of 64
      constexpr uint32_t kAllowed = MTE_F_MSG_END | MTE_F_MARKER | MTE_F_REWRITE;
      for (uint32_t base = 0; base < nleft; base += kWave) {
        uint32_t b[8];
        ch_rec_batch(b, recp, base);
        const int32_t s = (int32_t)b[0], r = (int32_t)b[1], m = (int32_t)b[2];
        const uint32_t type = b[3] & 0xffu, c = (b[3] >> 8) & 0xffu, fl = b[3] >> 16;
        if (base == 0) M = rdlane(m, 0);
        // the seq of the lane below (lane 0: the previous batch's last)
        int32_t below = __shfl_up(s, 1);
        below = l == 0 ? prev : below;
        const bool in = base + (uint32_t)l < nleft;
        const bool ok = r == R && m == M && type <= MTE_OP_ANNOTATE && c < MTE_MAX_CLIENTS &&
                        (fl & MTE_F_MSG_END) && !(fl & ~kAllowed) && s > below && M >= h.min_seq && M <= R &&
                        (int32_t)b[4] >= 0 && (int32_t)b[5] >= 0;
        const uint64_t bad = __ballot(in && !ok);
        if (bad) {
          k1 = k0 + base + (uint32_t)(__ffsll((long long)bad) - 1);
          break;
        }
        prev = rdlane(s, kWave - 1);
        k1 = k0 + base + kWave;
      }
      k1 = k1 < ktot ? k1 : ktot;
    }
    const uint32_t len = k1 - k0;
    // room for every op's segments (an insert or a range op adds at most 3)
    const bool room = (uint64_t)h.nseg + 3ull * len + 2ull <= (uint64_t)a.cap;
    if (len >= kRoundMin && room) p = make_uint4(kModeRound, k0, k1, (uint32_t)M);
    else if (len >= kRoundMin) p = make_uint4(kModeSeq, k0, k1, 0u);  // this run, op after op
    else p = make_uint4(kModeSeq, k0, ktot, 0u);  // not round-shaped: the rest op after op
    if (l == 0) {
      atomicAdd(rd.count + (p.x == kModeRound ? 0 : 1), 1u);
      atomicAdd(rd.count + 2, 1u);
    }
  }
  if (l == 0) rd.plan[doc] = p;
}

// flat planes -> chunks of kChFill, dropping removedSeq <= M; the round-start
// column (visible length of each chunk) into ch.kc
template <int K>
__global__ __launch_bounds__(512) void rnd_scatter_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  __shared__ ChCtl ctl;
  const int doc = (int)blockIdx.x;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound) return;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const int32_t M = (int32_t)p.w;
  const int n = a.hdr[doc].nseg;
  const uint32_t* pl = a.planes + (uint64_t)doc * a.cap;
  uint32_t* kc = ch.kc + (uint64_t)doc * ch.nch_cap;
  uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  constexpr int kT = kChE * kWave;  // 256 flat slots per tile
  const int ntile = (n + kT - 1) / kT;
  for (int t = w; t < ntile; t += kChWaves) {
    int32_t k = 0;
#pragma unroll
    for (int j = 0; j < kChE; j++) {
      const int i = t * kT + l * kChE + j;
      k += (i < n && (int32_t)pl[2 * a.stride + i] > M) ? 1 : 0;
    }
    const int32_t tot = rdlane(wave_incl_scan(k), kWave - 1);
    if (l == 0) kc[t] = (uint32_t)tot;
  }
  __syncthreads();
  const int32_t n_new = ch_block_scan(kc, ntile, &ctl);
  const int nplanes = kFieldPlanes + K;
  for (int t = w; t < ntile; t += kChWaves) {
    bool keep[kChE];
    int32_t k = 0;
#pragma unroll
    for (int j = 0; j < kChE; j++) {
      const int i = t * kT + l * kChE + j;
      keep[j] = i < n && (int32_t)pl[2 * a.stride + i] > M;
      k += keep[j] ? 1 : 0;
    }
    const int32_t d0 = (int32_t)ld_ag(kc + t) + wave_incl_scan(k) - k;
    for (int q = 0; q < nplanes; q++) {
      int32_t d = d0;
#pragma unroll
      for (int j = 0; j < kChE; j++) {
        const int i = t * kT + l * kChE + j;
        if (keep[j] && d < (int32_t)(ch.nch_cap * kChFill)) {
          const uint64_t x = ch_slot(ch, doc, d / kChFill) + (uint32_t)(d % kChFill);
          ch.arena[(uint64_t)q * ch.astride + x] = pl[(uint64_t)q * a.stride + i];
        }
        d += keep[j] ? 1 : 0;
      }
    }
  }
  __syncthreads();  // (every wave has read its tile's prefix before kc is reused)
  int nch = (n_new + kChFill - 1) / kChFill;
  nch = nch < 1 ? 1 : (nch > (int)ch.nch_cap ? (int)ch.nch_cap : nch);
  for (int q = w; q < nch; q += kChWaves) {
    const int cn = n_new - q * kChFill < kChFill ? (n_new - q * kChFill > 0 ? n_new - q * kChFill : 0) : kChFill;
    const uint64_t x0 = ch_slot(ch, doc, q);
    int32_t v = 0;
#pragma unroll
    for (int j = 0; j < kChFill / kWave; j++) {
      const int s = j * kWave + l;
      if (s < cn) {
        const int32_t rs = (int32_t)ld_ag(ch.arena + 2 * ch.astride + x0 + s);
        v += rs == kNone ? (int32_t)ld_ag(ch.arena + x0 + s) : 0;
      }
    }
    const int32_t tot = rdlane(wave_incl_scan(v), kWave - 1);
    if (l == 0) {
      cnt[q] = (uint32_t)cn;
      kc[q] = (uint32_t)tot;
    }
  }
  if (threadIdx.x == 0) rd.nch[doc] = (uint32_t)nch;
}

// one sub-op into chunk i's bucket (any lane; returns false on overflow)
__device__ __forceinline__ void rnd_emit(const RoundArgs& rd, uint32_t* rcnt, uint2* rbuf, int doc, int i,
                                         uint32_t k, int32_t ex) {
  const uint32_t pos = atomicAdd(rcnt + i, 1u);
  if (pos < (uint32_t)kRB) rbuf[(uint64_t)i * kRB + pos] = make_uint2(k, (uint32_t)ex);
  else atomicOr(rd.rflag + doc, 1u);
}

// one wave per client chain (clients c = w, w + 8, ... with ops in the run)
template <int K>
__global__ __launch_bounds__(512) void rnd_resolve_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  __shared__ uint32_t Gs[kChWaves][kChMaxGroups];
  __shared__ uint32_t present;
  const int doc = (int)blockIdx.x;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound) return;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const uint32_t k0 = p.y, nops = p.z - p.y;
  const uint4* recp = a.recs + 2 * (a.op_off[doc] + k0);
  const int nch = (int)rd.nch[doc];
  const uint32_t ng = (uint32_t)((nch + kChGroup - 1) / kChGroup);
  const uint32_t* cnt = ch.cnt + (uint64_t)doc * ch.nch_cap;
  const int32_t* sum0 = reinterpret_cast<const int32_t*>(ch.kc + (uint64_t)doc * ch.nch_cap);
  uint32_t* rcnt = rd.rcnt + (uint64_t)doc * ch.nch_cap;
  uint2* rbuf = rd.rbuf + (uint64_t)doc * ch.nch_cap * kRB;
  uint32_t* G = Gs[w];
  // the clients with ops in the run
  if (threadIdx.x == 0) present = 0u;
  __syncthreads();
  uint32_t mask = 0u;
  for (uint32_t base = (uint32_t)w * kWave; base < nops; base += kChWaves * kWave) {
    const uint32_t i = base + (uint32_t)l;
    const uint32_t w3 = i < nops ? reinterpret_cast<const uint32_t*>(recp + 2 * i)[3] : 0u;
    mask |= i < nops ? 1u << ((w3 >> 8) & 31u) : 0u;
  }
  for (int off = 32; off >= 1; off >>= 1) mask |= (uint32_t)__shfl_xor((int)mask, off);
  if (l == 0 && mask) atomicOr(&present, mask);
  __syncthreads();
  const uint32_t pres = present;
  for (int c = w; c < MTE_MAX_CLIENTS; c += kChWaves) {
    if (!((pres >> c) & 1u)) continue;
    int32_t* sumc = ch.sum + ((uint64_t)doc * MTE_MAX_CLIENTS + (uint32_t)c) * ch.nch_cap;
    // column c = the round-start column
    for (int i = l; i < nch; i += kWave) sumc[i] = ld_ag(sum0 + i);
    for (uint32_t g = 0; g < ng; g++) {
      const int i = (int)g * kChGroup + l;
      const int32_t v = i < nch ? ld_ag(sum0 + i) : 0;
      const int32_t tot = rdlane(wave_incl_scan(v), kWave - 1);
      if (l == 0) G[g] = (uint32_t)tot;
    }
    vm_wait();
    fence_wave();
    bool failed = false;
    for (uint32_t base = 0; base < nops && !failed; base += kWave) {
      uint32_t b[8];
      ch_rec_batch(b, recp, base);
      uint64_t mine = __ballot(base + (uint32_t)l < nops && ((b[3] >> 8) & 0xffu) == (uint32_t)c);
      while (mine) {
        const int j = __ffsll((long long)mine) - 1;
        mine &= mine - 1;
        const uint32_t k = base + (uint32_t)j;
        const uint32_t w3 = rdlane(b[3], j);
        const uint32_t type = w3 & 0xffu, flags = w3 >> 16;
        const int32_t pos1 = (int32_t)rdlane(b[4], j), pos2 = (int32_t)rdlane(b[5], j);
        int32_t ex = 0, total = 0, cs = 0;
        int cn = 0;
        if (type == MTE_OP_INSERT) {
          const int i0 = ch_find(G, ng, sumc, cnt, nch, pos1, false, &ex, &total, &cs, &cn);
          if (pos1 > total || i0 >= nch) {  // MTE_E_INSERT_FAILED at this op: the run goes op after op
            if (l == 0) atomicOr(rd.rflag + doc, 2u);
            failed = true;
            break;
          }
          const int32_t nlen = (flags & MTE_F_MARKER) ? 1 : pos2;
          if (l == 0) {
            rnd_emit(rd, rcnt, rbuf, doc, i0, k, ex);
            if (nlen > 0) {
              sumc[i0] = cs + nlen;
              G[(uint32_t)i0 / kChGroup] += (uint32_t)nlen;
            }
          }
        } else {
          const int32_t b1 = pos1 < pos2 ? pos1 : pos2, b2 = pos1 < pos2 ? pos2 : pos1;
          const int i0 = ch_find(G, ng, sumc, cnt, nch, b1, true, &ex, &total, &cs, &cn);
          if (i0 < nch) {
            if (b1 == b2) {
              // ensureIntervalBoundary alone: a split strictly inside a leaf
              if (ex < b1 && l == 0) rnd_emit(rd, rcnt, rbuf, doc, i0, k, ex);
            } else {
              // chunks i0 .. while their start is before b2, 64 at a time
              int32_t run = ex;
              for (int cb = i0; cb < nch; cb += kWave) {
                const int i = cb + l;
                const int32_t v = i < nch ? ld_ag(sumc + i) : 0;
                const int32_t incl = wave_incl_scan(v) + run;
                const int32_t st = incl - v;
                const bool hit = i < nch && v > 0 && st < b2;
                if (hit) {
                  rnd_emit(rd, rcnt, rbuf, doc, i, k, st);
                  if (type == MTE_OP_REMOVE) {
                    const int32_t lo = b1 > st ? b1 : st, hi = b2 < incl ? b2 : incl;
                    sumc[i] = v - (hi - lo);
                    atomicSub(&G[(uint32_t)i / kChGroup], (uint32_t)(hi - lo));
                  }
                }
                run = rdlane(incl, kWave - 1);
                if (run >= b2) break;
              }
            }
          }
        }
        vm_wait();
        fence_wave();
      }
    }
  }
}

// one wave per chunk of a run: its sub-ops in op order through seg_op_v
template <int K>
__global__ __launch_bounds__(256) void rnd_apply_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave), l = lane_id();
  const uint64_t wi = (uint64_t)blockIdx.x * 4 + (uint32_t)w;
  const int doc = (int)(wi / ch.nch_cap), i = (int)(wi % ch.nch_cap);
  if (doc >= (int)a.n_docs) return;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound || rd.rflag[doc] != 0u || i >= (int)rd.nch[doc]) return;
  const uint32_t nb = rd.rcnt[(uint64_t)doc * ch.nch_cap + i];
  if (nb == 0u) return;
  const uint2 e = l < (int)nb ? rd.rbuf[((uint64_t)doc * ch.nch_cap + i) * kRB + l] : make_uint2(0xffffffffu, 0u);
  // sort the bucket by op index: each entry's rank, then a push to that lane
  uint32_t rank = 0;
  for (uint32_t j = 0; j < nb; j++) rank += rdlane(e.x, (int)j) < e.x ? 1u : 0u;
  const int dst = (l < (int)nb ? (int)rank : l) << 2;
  const uint32_t ks = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)e.x);
  const int32_t exs = __builtin_amdgcn_ds_permute(dst, (int)e.y);
  uint32_t* cntp = ch.cnt + (uint64_t)doc * ch.nch_cap;
  int ni = (int)cntp[i];
  const uint64_t x0 = ch_slot(ch, doc, i);
  Regs<kChE, K> R;
  ch_load<K>(R, ch, x0, ni);
  uint32_t st[kNumStats] = {};
  const int32_t M = (int32_t)p.w;
  const uint4* recp = a.recs + 2 * (a.op_off[doc] + p.y);
  int rcs = 0;
  for (uint32_t j = 0; j < nb; j++) {
    const uint32_t k = uni(rdlane(ks, (int)j));
    const int32_t ex = rdlane(exs, (int)j);
    const s8v op = sload8(recp + 2 * k);
    const uint32_t w3 = (uint32_t)op[3];
    int32_t tot = 0, dlen = 0;
    const int rc = seg_op_v<kChE, K, false, true>(R, ni, op, w3 & 0xffu, (w3 >> 8) & 0xffu, w3 >> 16, M, true, ex,
                                                  true, tot, dlen, a, st);
    rcs = rc != 0 ? rc : rcs;
  }
  ch_store<K>(R, ch, x0, ni);
  if (l == 0) {
    cntp[i] = (uint32_t)ni;
    if (rcs != 0) a.hdr[doc].status = MTE_E_STATE;  // resolve guarantees every sub-op fits: an engine bug
  }
}

// chunks -> flat planes; the header advanced past the run
template <int K>
__global__ __launch_bounds__(512) void rnd_gather_kernel(ReplayArgs a, ChunkArgs ch, RoundArgs rd) {
  __shared__ ChCtl ctl;
  const int doc = (int)blockIdx.x;
  const uint4 p = rd.plan[doc];
  if (p.x != kModeRound || rd.rflag[doc] != 0u) return;
  const int32_t M = (int32_t)p.w;
  const int32_t n_new = ch_gather<K>(a, ch, doc, &ctl, (int)rd.nch[doc], M);
  if (threadIdx.x == 0) {
    const uint64_t kb = a.op_off[doc];
    const uint32_t ktot = (uint32_t)(a.op_off[doc + 1] - kb);
    DocHdr h = a.hdr[doc];
    h.nseg = n_new;
    h.min_seq = M;
    h.cur_seq = (int32_t)reinterpret_cast<const uint32_t*>(a.recs + 2 * (kb + p.z - 1))[0];
    h.resume = p.z;
    if (p.z >= ktot) h.flags &= ~kHdrNeedsEsc;
    a.hdr[doc] = h;
  }
}

}  // namespace mte
