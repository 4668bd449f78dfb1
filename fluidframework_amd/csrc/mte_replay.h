// mte_replay.h — the replay kernel: one wavefront per document, segments in
// VGPRs (see mte_kernels.h for the layout and primitives).
#pragma once

#include <type_traits>

#include "mte_kernels.h"

namespace mte {

// ISegment.addProperties for a remote op (segmentPropertiesManager.ts:63-151):
// each key of the set is written (value 0 = null = delete).  The first two
// entries come prefetched with the op; longer sets are read here.
template <typename F>
__device__ __forceinline__ uint32_t for_each_prop(const OpView& op, uint32_t psi, const ReplayArgs& a, F&& f) {
  uint32_t w = 0;
  if (op.pcnt > 0 && op.pk0 < a.n_keys) { f(op.pk0, op.pv0); w++; }
  if (op.pcnt > 1 && op.pk1 < a.n_keys) { f(op.pk1, op.pv1); w++; }
  if (op.pcnt > 2) {
    const mte_propset ps = a.ps[psi];
    for (uint32_t t = 2; t < ps.count; t++) {
      const mte_prop p = a.pe[ps.first + t];
      if (p.key < a.n_keys) { f(p.key, p.value); w++; }
    }
  }
  return w;
}

// Returns 0 = batch range done, 1 = re-pick E, or a negative MTE_E_*.
template <int E, int K>
__device__ int run_ops(const ReplayArgs& a, int doc, DocHdr& h, uint64_t& k, uint64_t k1, int emin,
                       uint32_t* lds, uint32_t (&st)[kNumStats]) {
  const int l = lane_id();
  const int base = l * E;
  const uint64_t dbase = (uint64_t)doc * a.cap;
  const bool newcalc = (h.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  int n = h.nseg;

  // uniform per-field base pointers (SGPR) + 32-bit lane offsets: saddr addressing
  int32_t* __restrict__ p_len = a.soa.len + dbase;
  int32_t* __restrict__ p_seq = a.soa.seq + dbase;
  int32_t* __restrict__ p_rseq = a.soa.rseq + dbase;
  uint32_t* __restrict__ p_rmask = a.soa.rmask + dbase;
  uint32_t* __restrict__ p_meta = a.soa.meta + dbase;
  uint32_t* __restrict__ p_toff = a.soa.toff + dbase;
  uint32_t* __restrict__ p_props = a.soa.props + dbase;
  const uint64_t pstride = a.soa.plane_stride;

  Regs<E, K> R;
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint32_t i = (uint32_t)(base + j);
    const bool v = (int)i < n;
    R.len[j] = v ? p_len[i] : 0;
    R.seq[j] = v ? p_seq[i] : 0;
    R.rseq[j] = v ? p_rseq[i] : 0;
    R.rmask[j] = v ? p_rmask[i] : 0u;
    R.meta[j] = v ? p_meta[i] : 0u;
    R.toff[j] = v ? p_toff[i] : 0u;
#pragma unroll
    for (int kk = 0; kk < K; kk++) R.pr[kk][j] = v ? p_props[kk * pstride + i] : 0u;
  }

  const int lim = kWave * E < (int)a.cap ? kWave * E : (int)a.cap;
  // op chunks, double-buffered without register copies: chunk q (records
  // [kq, kq + 64)) lives in buf[q & 1]; entering chunk q issues the load of
  // chunk q+1 into the other buffer and the propset gather of chunk q.
  OpChunk bufA, bufB;
  uint64_t cbase = k;
  int par = 0;
  chunk_load_ops(bufA, a.ops, cbase, k1);
  chunk_load_ops(bufB, a.ops, cbase + kWave, k1);
  chunk_load_props(bufA, a.ps, a.pe);

  int reason = 0;
  for (; k < k1; k++) {
    // re-pick E when the doc no longer fits; also return every 2^20 ops so the
    // 32-bit stat counters never wrap
    if (n + 2 > lim || st[kStOps] >= (1u << 20)) {
      reason = 1;
      break;
    }
    int j = (int)(k - cbase);
    if (j == kWave) {
      cbase += kWave;
      j = 0;
      par ^= 1;
      if (par) {
        chunk_load_ops(bufA, a.ops, cbase + kWave, k1);
        chunk_load_props(bufB, a.ps, a.pe);
      } else {
        chunk_load_ops(bufB, a.ops, cbase + kWave, k1);
        chunk_load_props(bufA, a.ps, a.pe);
      }
    }
    const OpView op = par ? chunk_op(bufB, j) : chunk_op(bufA, j);
    st[kStOps]++;
    st[kStMaxSegs] = (uint32_t)n > st[kStMaxSegs] ? (uint32_t)n : st[kStMaxSegs];
    const int c = (int)op.client;
    if (c >= MTE_MAX_CLIENTS) {
      reason = MTE_E_CLIENT_RANGE;
      break;
    }
    const int32_t r = op.ref_seq, s = op.seq, m = h.min_seq;

    if (op.type == MTE_OP_INSERT) {
      // Client.applyInsertOp -> MergeTree.insertSegments (client.ts:470-505,
      // mergeTree.ts:1394-1422)
      st[kStScanned] += (uint32_t)n;
      int32_t L[E], P[E];
      leaf_lengths<E, K>(R, n, r, c, m, newcalc, L);
      const int32_t total = prefix<E>(L, P);
      const int32_t pos = op.pos1;
      int32_t off = 0;
      const int xs = find_split<E>(L, P, pos, &off);  // ensureIntervalBoundary
      const bool marker = (op.flags & MTE_F_MARKER) != 0;
      const int32_t nlen = marker ? 1 : op.pos2;
      int g = -1;
      if (xs < 0 && nlen > 0) {
        g = find_slot<E>(L, P, pos);
        if (g < 0) {
          if (pos > total) {
            reason = MTE_E_INSERT_FAILED;  // mergeTree.ts:1666-1672
            break;
          }
          g = n;
        }
      }
      if (xs >= 0) {
        // split: head keeps [0, off), the shift copies it into the tail slot
        const int32_t xlen = bcast<E>(R.len, xs);
        const uint32_t xtoff = bcast<E>(R.toff, xs);
        if (nlen > 0) {
          shift_all<E, K>(R, xs, xs + 1);  // slot xs+1: new segment, xs+2: tail
          g = xs + 1;
          st[kStWritten] += 3;
        } else {
          shift_all<E, K>(R, xs, INT32_MAX);
          st[kStWritten] += 2;
        }
        const int tail = nlen > 0 ? xs + 2 : xs + 1;
        put<E>(R.len, xs, off);
        put<E>(R.len, tail, xlen - off);
        put<E>(R.toff, tail, xtoff + (uint32_t)off);
        n += 1;
      } else if (nlen > 0) {
        shift_all<E, K>(R, g - 1, INT32_MAX);
        st[kStWritten] += 1;
      }
      if (nlen > 0) {
        uint32_t pr[K > 0 ? K : 1];
#pragma unroll
        for (int kk = 0; kk < (K > 0 ? K : 1); kk++) pr[kk] = 0;
        if (op.b != MTE_NO_PROPS)
          st[kStPwrites] += for_each_prop(op, op.b, a, [&](uint32_t key, uint32_t val) {
#pragma unroll
            for (int kk = 0; kk < K; kk++) pr[kk] = ((uint32_t)kk == key) ? val : pr[kk];
          });
        if (!marker) st[kStUnits] += (uint32_t)nlen;
        const uint32_t meta = (uint32_t)(c + 1) | ((marker ? 1u + (uint32_t)op.pos2 : 0u) << 8);
        put_new<E, K>(R, g, nlen, s, meta, marker ? 0u : a.text_base + op.a, pr);
        n += 1;
      }
    } else if (op.type == MTE_OP_REMOVE || op.type == MTE_OP_ANNOTATE) {
      // markRangeRemoved (mergeTree.ts:1908-2000) / annotateRange (1864-1906)
      st[kStScanned] += (uint32_t)n;
      const int32_t start = op.pos1, end = op.pos2;
      int32_t L[E], P[E];
      leaf_lengths<E, K>(R, n, r, c, m, newcalc, L);
      prefix<E>(L, P);
      int32_t oa = 0, ob = 0;
      const int xa = find_split<E>(L, P, start, &oa);
      const int xb = find_split<E>(L, P, end, &ob);
      // order the (at most two) split events by (index, offset)
      int x1 = xa, x2 = xb;
      int32_t o1 = oa, o2 = ob;
      if (x1 < 0 || (x2 >= 0 && (x2 < x1 || (x2 == x1 && ob < oa)))) {
        x1 = xb;
        x2 = xa;
        o1 = ob;
        o2 = oa;
      }
      if (x2 >= 0 && x1 == x2 && o1 == o2) x2 = -1;  // same boundary twice
      if (x1 < 0) {
        x1 = x2;
        o1 = o2;
        x2 = -1;
      }
      if (x1 >= 0 && x2 < 0) {
        const int32_t xlen = bcast<E>(R.len, x1);
        const uint32_t xtoff = bcast<E>(R.toff, x1);
        shift_all<E, K>(R, x1, INT32_MAX);  // slot x1+1 = copy of x1
        put<E>(R.len, x1, o1);
        put<E>(R.len, x1 + 1, xlen - o1);
        put<E>(R.toff, x1 + 1, xtoff + (uint32_t)o1);
        n += 1;
        st[kStWritten] += 2;
      } else if (x1 >= 0) {
        const int32_t len1 = bcast<E>(R.len, x1);
        const uint32_t toff1 = bcast<E>(R.toff, x1);
        const int32_t len2 = bcast<E>(R.len, x2);
        const uint32_t toff2 = bcast<E>(R.toff, x2);
        if (x2 == x1) {  // three pieces of one segment: [0,o1) [o1,o2) [o2,len)
          shift_all<E, K>(R, x1, x1 + 1);
          put<E>(R.len, x1, o1);
          put<E>(R.len, x1 + 1, o2 - o1);
          put<E>(R.toff, x1 + 1, toff1 + (uint32_t)o1);
          put<E>(R.len, x1 + 2, len1 - o2);
          put<E>(R.toff, x1 + 2, toff1 + (uint32_t)o2);
        } else {  // x1 < x2: tails at x1+1 and x2+2, second head at x2+1
          shift_all<E, K>(R, x1, x2 + 1);
          put<E>(R.len, x1, o1);
          put<E>(R.len, x1 + 1, len1 - o1);
          put<E>(R.toff, x1 + 1, toff1 + (uint32_t)o1);
          put<E>(R.len, x2 + 1, o2);
          put<E>(R.len, x2 + 2, len2 - o2);
          put<E>(R.toff, x2 + 2, toff2 + (uint32_t)o2);
        }
        n += 2;
        st[kStWritten] += 4;
      }
      if (end != start) {
        // nodeMap (mergeTree.ts:2274-2330): leaves with len > 0 overlapping [start, end)
        leaf_lengths<E, K>(R, n, r, c, m, newcalc, L);
        prefix<E>(L, P);
        bool in[E];
        unsigned cnt = 0;
#pragma unroll
        for (int j2 = 0; j2 < E; j2++) {
          in[j2] = L[j2] > 0 && P[j2] < end && P[j2] + L[j2] > start;
          cnt += (unsigned)__popcll(__ballot(in[j2]));
        }
        st[kStWritten] += cnt;
        if (op.type == MTE_OP_REMOVE) {
          // markRemoved (mergeTree.ts:1924-1962): keep the earliest removedSeq,
          // add the client to removedClientIds
          const uint32_t bit = 1u << c;
#pragma unroll
          for (int j2 = 0; j2 < E; j2++) {
            R.rseq[j2] = (in[j2] && R.rseq[j2] == kNone) ? s : R.rseq[j2];
            R.rmask[j2] = in[j2] ? (R.rmask[j2] | bit) : R.rmask[j2];
          }
        } else if (cnt > 0) {
          // PropertiesManager.addProperties (segmentPropertiesManager.ts:63-151)
          if (op.flags & MTE_F_REWRITE) {
#pragma unroll
            for (int kk = 0; kk < K; kk++)
#pragma unroll
              for (int j2 = 0; j2 < E; j2++) R.pr[kk][j2] = in[j2] ? 0u : R.pr[kk][j2];
          }
          const uint32_t nw = for_each_prop(op, op.a, a, [&](uint32_t key, uint32_t val) {
#pragma unroll
            for (int kk = 0; kk < K; kk++) {
              if ((uint32_t)kk == key) {
#pragma unroll
                for (int j2 = 0; j2 < E; j2++) R.pr[kk][j2] = in[j2] ? val : R.pr[kk][j2];
              }
            }
          });
          st[kStPwrites] += cnt * nw;
        }
      }
    } else if (op.type != MTE_OP_NOOP) {
      reason = MTE_E_INVALID_ARG;
      break;
    }

    if (op.type != MTE_OP_NOOP) {  // Client.completeAndLogOp (client.ts:525-528)
      if (!(h.cur_seq < s)) { reason = MTE_E_SEQ_ORDER; k++; break; }
      if (!(h.min_seq <= op.min_seq)) { reason = MTE_E_MSN_ORDER; k++; break; }
    }
    if (op.flags & MTE_F_MSG_END) {
      // updateSeqNumbers (client.ts:937-945) -> setMinSeq (mergeTree.ts:1077-1093)
      if (!(h.cur_seq <= s)) { reason = MTE_E_SEQ_ORDER; k++; break; }
      h.cur_seq = s;
      if (!(op.min_seq <= s)) { reason = MTE_E_MSN_GT_SEQ; k++; break; }
      if (!(h.min_seq <= op.min_seq)) { reason = MTE_E_MSN_ORDER; k++; break; }
      if (op.min_seq > h.min_seq) {
        h.min_seq = op.min_seq;
        // zamboni: drop tombstones with removedSeq <= minSeq (stream compaction through LDS)
        bool keep[E];
        int32_t cntl = 0;
#pragma unroll
        for (int j2 = 0; j2 < E; j2++) {
          keep[j2] = (base + j2 < n) && !(R.rseq[j2] != kNone && R.rseq[j2] <= h.min_seq);
          cntl += keep[j2] ? 1 : 0;
        }
        const int32_t incl = wave_incl_scan(cntl);
        const int n_new = rdlane(incl, kWave - 1);
        if (n_new != n) {
          int32_t dst[E];
          int32_t d0 = incl - cntl;
#pragma unroll
          for (int j2 = 0; j2 < E; j2++) {
            dst[j2] = d0;
            d0 += keep[j2] ? 1 : 0;
          }
          auto compact = [&](auto& F) {
#pragma unroll
            for (int j2 = 0; j2 < E; j2++)
              if (keep[j2]) lds[dst[j2]] = (uint32_t)F[j2];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (int j2 = 0; j2 < E; j2++) F[j2] = (std::remove_reference_t<decltype(F[0])>)lds[base + j2];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          };
          compact(R.len);
          compact(R.seq);
          compact(R.rseq);
          compact(R.rmask);
          compact(R.meta);
          compact(R.toff);
#pragma unroll
          for (int kk = 0; kk < K; kk++) compact(R.pr[kk]);
          n = n_new;
          // drop to a smaller register tier once the doc fits in half of it
          if (E > emin && n + 2 + 16 <= 32 * E) {
            k++;
            reason = 1;
            break;
          }
        }
      }
    }
  }

  // write back (also on error / escalation)
#pragma unroll
  for (int j = 0; j < E; j++) {
    const uint32_t i = (uint32_t)(base + j);
    if ((int)i < n) {
      p_len[i] = R.len[j];
      p_seq[i] = R.seq[j];
      p_rseq[i] = R.rseq[j];
      p_rmask[i] = R.rmask[j];
      p_meta[i] = R.meta[j];
      p_toff[i] = R.toff[j];
#pragma unroll
      for (int kk = 0; kk < K; kk++) p_props[kk * pstride + i] = R.pr[kk][j];
    }
  }
  h.nseg = n;
  return reason;
}

template <int EMIN, int EMAX, int K, bool LAST>
__global__ __launch_bounds__(256) void replay_kernel(ReplayArgs a, int pass) {
  __shared__ uint32_t lds_all[kDocsPerBlock][kWave * EMAX];
  // wave index: uniform by construction; readfirstlane tells the compiler, so
  // every doc-derived value (header, pointers, op cursor) lives in SGPRs
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int doc = (int)blockIdx.x * kDocsPerBlock + w;
  if (doc >= (int)a.n_docs) return;
  uint32_t* lds = lds_all[w];
  DocHdr h = a.hdr[doc];
  if (h.status != 0) return;
  if (pass > 0 && !(h.flags & kHdrNeedsEsc)) return;
  h.flags &= ~kHdrNeedsEsc;
  const uint64_t kb = a.op_off[doc];
  uint64_t k = kb + h.resume;
  const uint64_t k1 = a.op_off[doc + 1];
  unsigned long long st[kNumStats] = {0, 0, 0, 0, 0, 0};
  while (k < k1) {
    const int n = h.nseg;
    int E = 0;
    if (EMIN <= 1 && EMAX >= 1 && n + 2 <= kWave * 1) E = 1;
    else if (EMIN <= 2 && EMAX >= 2 && n + 2 <= kWave * 2) E = 2;
    else if (EMIN <= 4 && EMAX >= 4 && n + 2 <= kWave * 4) E = 4;
    else if (EMIN <= 8 && EMAX >= 8 && n + 2 <= kWave * 8) E = 8;
    else if (EMIN <= 16 && EMAX >= 16 && n + 2 <= kWave * 16) E = 16;
    if (E == 0 || n + 2 > (int)a.cap) {
      if (LAST || n + 2 > (int)a.cap) h.status = MTE_E_CAPACITY;
      else h.flags |= kHdrNeedsEsc;
      break;
    }
    int rc = 0;
    uint32_t s32[kNumStats] = {0, 0, 0, 0, 0, 0};
    if constexpr (EMIN <= 1 && EMAX >= 1) if (E == 1) rc = run_ops<1, K>(a, doc, h, k, k1, EMIN, lds, s32);
    if constexpr (EMIN <= 2 && EMAX >= 2) if (E == 2) rc = run_ops<2, K>(a, doc, h, k, k1, EMIN, lds, s32);
    if constexpr (EMIN <= 4 && EMAX >= 4) if (E == 4) rc = run_ops<4, K>(a, doc, h, k, k1, EMIN, lds, s32);
    if constexpr (EMIN <= 8 && EMAX >= 8) if (E == 8) rc = run_ops<8, K>(a, doc, h, k, k1, EMIN, lds, s32);
    if constexpr (EMIN <= 16 && EMAX >= 16) if (E == 16) rc = run_ops<16, K>(a, doc, h, k, k1, EMIN, lds, s32);
#pragma unroll
    for (int t = 0; t < kNumStats; t++) {
      if (t == kStMaxSegs) st[t] = st[t] > s32[t] ? st[t] : s32[t];
      else st[t] += s32[t];
    }
    if (rc < 0) {
      h.status = rc;
      break;
    }
  }
  h.resume = (uint32_t)(k - kb);
  if (lane_id() == 0) {
    a.hdr[doc] = h;
    unsigned long long* sd = a.stats + (size_t)doc * kNumStats;
#pragma unroll
    for (int t = 0; t < kNumStats; t++) {
      if (t == kStMaxSegs) sd[t] = sd[t] > st[t] ? sd[t] : st[t];
      else sd[t] += st[t];
    }
  }
}

}  // namespace mte
