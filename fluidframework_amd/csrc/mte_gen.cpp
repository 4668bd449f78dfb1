// mte_gen.cpp — synthetic sequenced-op streams (see mte_gen.h).
//
// The generator needs each author's perspective length L(refSeq, client) to
// draw valid positions.  It keeps a per-UNIT model of the document (one record
// per UTF-16 unit / marker), which is enough for lengths: a unit is visible to
// (r, c) iff it was inserted at seq <= r or by c, and it is not removed at
// rseq <= r or by c (the perspective rule of mergeTree.ts:1003-1054 summed
// over leaves; both length modes give the same sums).  Placement of
// concurrent, invisible units does not change any length, so the model never
// needs the tie-break rules.
#include "mte_gen.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

namespace {

constexpr int32_t kNone = INT32_MAX;

// MT19937 (Matsumoto & Nishimura), with init_by_array.
struct MT {
  uint32_t mt[624];
  int mti = 625;
  void init(uint32_t s) {
    mt[0] = s;
    for (mti = 1; mti < 624; mti++)
      mt[mti] = 1812433253u * (mt[mti - 1] ^ (mt[mti - 1] >> 30)) + (uint32_t)mti;
  }
  void init_by_array(const uint32_t* key, int len) {
    init(19650218u);
    int i = 1, j = 0;
    for (int k = (624 > len ? 624 : len); k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      i++, j++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= len) j = 0;
    }
    for (int k = 623; k; k--) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      i++;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
  }
  uint32_t next() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (mti >= 624) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < 624 - 397; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // uniform integer in [lo, hi] (rejection sampling, no modulo bias)
  int64_t uniform(int64_t lo, int64_t hi) {
    uint64_t range = (uint64_t)(hi - lo) + 1u;
    if (range == 0 || range > 0xFFFFFFFFull) return lo;  // not used for such ranges
    uint32_t r32 = (uint32_t)range;
    uint32_t limit = (uint32_t)(0x100000000ull - (0x100000000ull % r32));
    uint32_t x;
    do { x = next(); } while (limit != 0 && x >= limit);
    return lo + (int64_t)(x % r32);
  }
};

struct Unit {
  int32_t seq, rseq;
  uint32_t rmask;
  int32_t cli;
};

inline bool visible(const Unit& u, int32_t r, int c) {
  if (!(u.seq <= r || u.cli == c)) return false;
  if (u.rseq != kNone && (u.rseq <= r || ((u.rmask >> c) & 1u))) return false;
  return true;
}

// the unit's leaf has a defined perspective length (mergeTree.ts:1003-1054):
// new calc -> every unit still held (tombstones at or below minSeq are gone
// from the model); legacy -> not a tombstone the perspective saw removed, and
// not a removed unit it never saw inserted
inline bool defined(const Unit& u, int32_t r, int c, bool newcalc) {
  if (newcalc || u.rseq == kNone) return true;
  if (u.rseq <= r) return false;
  return u.seq <= r || u.cli == c;
}

struct DocOut {
  std::vector<mte_op> ops;
  std::vector<uint16_t> text;
  std::vector<mte_propset> psets;  // per-doc (markers); index fixed up at fill
  std::vector<mte_prop> props;
  std::vector<uint16_t> init_text;
  uint32_t flags = 0;
};

// Fixed annotate propsets: [0,27) single key, [27,270) two keys.
constexpr uint32_t kFixedSets = 270;
void fixed_propsets(std::vector<mte_propset>& ps, std::vector<mte_prop>& pe) {
  auto val = [](uint32_t key, uint32_t v) -> uint32_t {  // v == 8 -> null
    if (v == 8) return 0;
    if (key == MTEG_KEY_CLIENT) return 1 + v;
    if (key == MTEG_KEY_BOLD) return 33 + v;
    return 41 + v;
  };
  for (uint32_t k = 0; k < 3; k++)
    for (uint32_t v = 0; v < 9; v++) {
      ps.push_back({(uint32_t)pe.size(), 1});
      pe.push_back({k, val(k, v)});
    }
  for (uint32_t k1 = 0; k1 < 3; k1++)
    for (uint32_t k2 = k1 + 1; k2 < 3; k2++)
      for (uint32_t v1 = 0; v1 < 9; v1++)
        for (uint32_t v2 = 0; v2 < 9; v2++) {
          ps.push_back({(uint32_t)pe.size(), 2});
          pe.push_back({k1, val(k1, v1)});
          pe.push_back({k2, val(k2, v2)});
        }
}
uint32_t single_set(uint32_t k, uint32_t v) { return k * 9 + v; }
uint32_t pair_set(uint32_t k1, uint32_t k2, uint32_t v1, uint32_t v2) {
  // pairs in order (0,1), (0,2), (1,2)
  uint32_t pi = (k1 == 0) ? (k2 == 1 ? 0 : 1) : 2;
  return 27 + pi * 81 + v1 * 9 + v2;
}

// annotate props: 1-2 keys of {client, bold, color}, values of <= 8 per key,
// 10% null -> one of the fixed propsets
uint32_t annotate_set(MT& rng) {
  const uint32_t nk = (uint32_t)rng.uniform(1, 2);
  auto pick_val = [&]() -> uint32_t { return rng.uniform(0, 9) == 0 ? 8u : (uint32_t)rng.uniform(0, 7); };
  if (nk == 1) {
    const uint32_t k1 = (uint32_t)rng.uniform(0, 2);
    return single_set(k1, pick_val());
  }
  uint32_t k1 = (uint32_t)rng.uniform(0, 2), k2 = (uint32_t)rng.uniform(0, 1);
  if (k2 >= k1) k2++;
  if (k2 < k1) std::swap(k1, k2);
  const uint32_t v1 = pick_val(), v2 = pick_val();
  return pair_set(k1, k2, v1, v2);
}

// n units of the author's name; with newline_every, 1 in N texts has one unit
// (any of them) replaced by '\n' (TextSegment.canAppend refuses to append to a
// text ending in one, textSegment.ts:72-77).  No draw is made without the option.
void push_text(const mteg_config& cfg, MT& rng, uint32_t author, int32_t n, DocOut& out) {
  int32_t nl = -1;
  if (cfg.newline_every && rng.uniform(0, cfg.newline_every - 1) == 0) nl = (int32_t)rng.uniform(0, (uint32_t)n - 1);
  for (int32_t i = 0; i < n; i++) out.text.push_back(i == nl ? (uint16_t)'\n' : (uint16_t)('B' + author));
}

// an insert of 1-3 units of the author's name, or (1 in marker_every) a
// marker {marker:{refType:1}, props:{markerId:"m<seq>"}}; returns its length
int32_t gen_insert(const mteg_config& cfg, MT& rng, uint32_t author, int32_t s, mte_op& op, DocOut& out) {
  const bool marker = cfg.marker_every && rng.uniform(0, cfg.marker_every - 1) == 0;
  if (marker) {
    op.flags |= MTE_F_MARKER;
    op.pos2 = 1;                         // refType
    op.b = (uint32_t)out.psets.size();   // per-doc index, fixed up at fill
    out.psets.push_back({(uint32_t)out.props.size(), 1});
    out.props.push_back({MTEG_KEY_MARKER_ID, 64u + (uint32_t)s});
    return 1;
  }
  const int32_t n = (int32_t)rng.uniform(1, 3);
  op.pos2 = n;
  op.a = (uint32_t)out.text.size();  // per-doc offset, fixed up at fill
  push_text(cfg, rng, author, n, out);
  return n;
}

// Long documents (config 5: a preloaded body of init_segs one-unit segments,
// loaded through mte_load_segments).  The per-unit model of gen_doc would cost
// O(document) per op, so each author's perspective length is kept instead:
// within a round (refSeq = round start for every op) an author sees the base
// text plus its own ops only, so L(r, c) = L0 + inserted_c - removed_c
// exactly.  The next round's L0 is bounded below by L0 + all inserted - all
// removed (a unit removed by two authors counts twice), and positions are
// drawn against that bound, so every op is valid; the stream departs from the
// farm rule (mergeTreeOperationRunner.ts:164-176) only in drawing from
// [0, bound] instead of [0, L].  Ranges are short (1..max_range units).
void gen_doc_long(const mteg_config& cfg, uint32_t d, DocOut& out) {
  MT rng;
  const uint32_t key[4] = {0xDEADBEEFu, 0xFEEDBEDu, cfg.config_id, cfg.doc_ids ? cfg.doc_ids[d] : cfg.doc_base + d};
  rng.init_by_array(key, 4);
  const uint32_t C = cfg.clients < 1 ? 1 : (cfg.clients > 31 ? 31 : cfg.clients);
  if (cfg.length_mode == 0) out.flags = (rng.next() & 1u) ? MTE_DOC_NEW_LENGTH_CALC : 0u;
  else if (cfg.length_mode == 2) out.flags = MTE_DOC_NEW_LENGTH_CALC;
  out.init_text.resize(cfg.init_segs);
  for (uint32_t i = 0; i < cfg.init_segs; i++) out.init_text[i] = (uint16_t)('a' + (i % 26));
  int short_of[32];
  for (int i = 0; i < 32; i++) short_of[i] = -1;
  int next_short = 1;
  std::vector<uint32_t> mix;
  if (cfg.mix & MTEG_MIX_INSERT) mix.push_back(MTE_OP_INSERT);
  if (cfg.mix & MTEG_MIX_REMOVE) mix.push_back(MTE_OP_REMOVE);
  if (cfg.mix & MTEG_MIX_ANNOTATE) mix.push_back(MTE_OP_ANNOTATE);
  if (mix.empty()) mix.push_back(MTE_OP_INSERT);
  out.ops.reserve(cfg.ops_per_doc);
  const uint32_t R = cfg.round_ops ? cfg.round_ops : 1;
  const int64_t max_range = cfg.max_range ? cfg.max_range : INT32_MAX;
  int64_t L0 = cfg.init_segs;
  int32_t seq = 0;
  uint32_t done = 0;
  while (done < cfg.ops_per_doc) {
    const int32_t round_start = seq;
    int64_t ins[32] = {0}, rem[32] = {0}, all_ins = 0, all_rem = 0;
    for (uint32_t k = 0; k < R && done < cfg.ops_per_doc; k++, done++) {
      const uint32_t author = (uint32_t)rng.uniform(0, C - 1);
      if (short_of[author] < 0) short_of[author] = next_short++;
      const int c = short_of[author];
      const int32_t r = round_start;
      const int32_t s = ++seq;
      const int64_t L = L0 + ins[c] - rem[c];
      const uint32_t type = (L <= 0 || L < (int64_t)cfg.min_length)
                                ? MTE_OP_INSERT
                                : mix[(size_t)rng.uniform(0, (int64_t)mix.size() - 1)];
      mte_op op;
      std::memset(&op, 0, sizeof(op));
      op.seq = s;
      op.ref_seq = r;
      op.min_seq = r;
      op.type = (uint8_t)type;
      op.client = (uint8_t)c;
      op.flags = MTE_F_MSG_END;
      op.b = MTE_NO_PROPS;
      if (type == MTE_OP_INSERT) {
        op.pos1 = (int32_t)rng.uniform(0, L > 0 ? L : 0);
        const int32_t n = gen_insert(cfg, rng, author, s, op, out);
        ins[c] += n;
        all_ins += n;
      } else {
        const int64_t start = rng.uniform(0, L - 1);
        const int64_t span = L - start < max_range ? L - start : max_range;
        const int64_t end = start + rng.uniform(1, span);
        op.pos1 = (int32_t)start;
        op.pos2 = (int32_t)end;
        if (type == MTE_OP_REMOVE) {
          rem[c] += end - start;
          all_rem += end - start;
        } else {
          op.a = annotate_set(rng);
        }
      }
      out.ops.push_back(op);
    }
    L0 = L0 + all_ins - all_rem;
    if (L0 < 0) L0 = 0;
  }
}

void gen_doc(const mteg_config& cfg, uint32_t d, DocOut& out) {
  if (cfg.init_segs) {
    gen_doc_long(cfg, d, out);
    return;
  }
  MT rng;
  const uint32_t key[4] = {0xDEADBEEFu, 0xFEEDBEDu, cfg.config_id, cfg.doc_ids ? cfg.doc_ids[d] : cfg.doc_base + d};
  rng.init_by_array(key, 4);
  const uint32_t C = cfg.clients < 1 ? 1 : (cfg.clients > 31 ? 31 : cfg.clients);
  if (cfg.length_mode == 0) out.flags = (rng.next() & 1u) ? MTE_DOC_NEW_LENGTH_CALC : 0u;
  else if (cfg.length_mode == 2) out.flags = MTE_DOC_NEW_LENGTH_CALC;

  std::vector<Unit> units;
  units.reserve(256);
  for (uint32_t i = 0; i < cfg.init_len; i++) {
    out.init_text.push_back((uint16_t)('a' + (i % 26)));
    units.push_back({0, kNone, 0u, -1});
  }
  // author k (0-based) -> short id in first-seen order (observer "A" = 0)
  int short_of[32];
  for (int i = 0; i < 32; i++) short_of[i] = -1;
  int next_short = 1;

  std::vector<uint32_t> mix;
  if (cfg.mix & MTEG_MIX_INSERT) mix.push_back(MTE_OP_INSERT);
  if (cfg.mix & MTEG_MIX_REMOVE) mix.push_back(MTE_OP_REMOVE);
  if (cfg.mix & MTEG_MIX_ANNOTATE) mix.push_back(MTE_OP_ANNOTATE);
  if (mix.empty()) mix.push_back(MTE_OP_INSERT);

  out.ops.reserve(cfg.ops_per_doc);
  const uint32_t R = cfg.max_lag ? 1u : (cfg.round_ops ? cfg.round_ops : 1);
  int32_t seq = 0;
  int32_t min_seq = 0;
  int32_t cref[32] = {0};  // max_lag: each author's refSeq (its last seen seq)
  uint32_t done = 0;
  while (done < cfg.ops_per_doc) {
    const int32_t round_start = seq;  // rounds: refSeq == msn for the whole round
    if (!cfg.max_lag && round_start > min_seq) {
      min_seq = round_start;
      // zamboni in the model: drop units removed at or below minSeq
      size_t w = 0;
      for (size_t i = 0; i < units.size(); i++)
        if (!(units[i].rseq != kNone && units[i].rseq <= min_seq)) units[w++] = units[i];
      units.resize(w);
    }
    for (uint32_t k = 0; k < R && done < cfg.ops_per_doc; k++, done++) {
      const uint32_t author = (uint32_t)rng.uniform(0, C - 1);
      if (short_of[author] < 0) short_of[author] = next_short++;
      const int c = short_of[author];
      int32_t r = round_start, msn = round_start;
      if (cfg.max_lag) {
        // the author catches up to a seq at most max_lag behind; the
        // sequencer's msn is the lowest refSeq of all authors
        const int32_t lo = seq - (int32_t)cfg.max_lag;
        const int32_t want = (int32_t)rng.uniform(lo > 0 ? lo : 0, seq);
        if (want > cref[author]) cref[author] = want;
        r = cref[author];
        msn = cref[0];
        for (uint32_t a = 1; a < C; a++) msn = cref[a] < msn ? cref[a] : msn;
      }
      const int32_t s = ++seq;
      int64_t L = 0;
      for (const Unit& u : units) L += visible(u, r, c) ? 1 : 0;
      uint32_t type = (L == 0 || L < (int64_t)cfg.min_length)
                          ? MTE_OP_INSERT
                          : mix[(size_t)rng.uniform(0, (int64_t)mix.size() - 1)];
      mte_op op;
      std::memset(&op, 0, sizeof(op));
      op.seq = s;
      op.ref_seq = r;
      op.min_seq = msn;
      op.type = (uint8_t)type;
      op.client = (uint8_t)c;
      op.flags = MTE_F_MSG_END;
      op.b = MTE_NO_PROPS;
      if (type == MTE_OP_INSERT) {
        const int64_t pos = rng.uniform(0, L);
        const bool marker = cfg.marker_every && rng.uniform(0, cfg.marker_every - 1) == 0;
        int32_t n = 1;
        op.pos1 = (int32_t)pos;
        if (marker) {
          op.flags |= MTE_F_MARKER;
          op.pos2 = 1;  // refType
          op.b = (uint32_t)out.psets.size();  // per-doc index, fixed up at fill
          out.psets.push_back({(uint32_t)out.props.size(), 1});
          out.props.push_back({MTEG_KEY_MARKER_ID, 64u + (uint32_t)s});
        } else {
          n = (int32_t)rng.uniform(1, 3);
          op.pos2 = n;
          op.a = (uint32_t)out.text.size();  // per-doc offset, fixed up at fill
          push_text(cfg, rng, author, n, out);
        }
        // model: the engine's placement: before the first
        // defined unit with P >= pos.  Lengths alone would not need the exact
        // place, but with lagging refSeqs a later range op of another
        // perspective removes units by position, so the order must match.
        const bool newcalc = (out.flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
        size_t at = units.size();
        int64_t seen = 0;
        for (size_t i = 0; i < units.size(); i++) {
          if (seen >= pos && defined(units[i], r, c, newcalc)) { at = i; break; }
          if (visible(units[i], r, c)) seen++;
        }
        units.insert(units.begin() + (ptrdiff_t)at, (size_t)n, Unit{s, kNone, 0u, c});
      } else {
        const int64_t start = rng.uniform(0, L - 1);
        const int64_t end = rng.uniform(start + 1, L);
        op.pos1 = (int32_t)start;
        op.pos2 = (int32_t)end;
        if (type == MTE_OP_REMOVE) {
          int64_t seen = 0;
          for (Unit& u : units) {
            if (!visible(u, r, c)) continue;
            if (seen >= start && seen < end) {
              if (u.rseq == kNone) { u.rseq = s; u.rmask = 1u << c; }
              else u.rmask |= 1u << c;
            }
            if (++seen >= end) break;
          }
        } else {
          op.a = annotate_set(rng);
        }
      }
      out.ops.push_back(op);
      if (cfg.max_lag && msn > min_seq) {
        min_seq = msn;  // the window moves after the message (client.ts:934)
        size_t w = 0;
        for (size_t i = 0; i < units.size(); i++)
          if (!(units[i].rseq != kNone && units[i].rseq <= min_seq)) units[w++] = units[i];
        units.resize(w);
      }
    }
  }
}

}  // namespace

struct mteg_stream {
  mteg_config cfg;
  std::vector<DocOut> docs;
  std::vector<mte_propset> fixed_ps;
  std::vector<mte_prop> fixed_pe;
};

extern "C" int mteg_generate(const mteg_config* cfg, mteg_stream** out) {
  if (!cfg || !out || cfg->n_docs == 0) return MTE_E_INVALID_ARG;
  mteg_stream* s = new (std::nothrow) mteg_stream();
  if (!s) return MTE_E_OOM;
  s->cfg = *cfg;
  try {
    s->docs.resize(cfg->n_docs);
    fixed_propsets(s->fixed_ps, s->fixed_pe);
    uint32_t nt = cfg->n_threads ? cfg->n_threads : 1;
    if (nt > cfg->n_docs) nt = cfg->n_docs;
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; t++)
      th.emplace_back([s, t, nt]() {
        for (uint32_t d = t; d < s->cfg.n_docs; d += nt) gen_doc(s->cfg, d, s->docs[d]);
      });
    for (auto& x : th) x.join();
  } catch (...) {
    delete s;
    return MTE_E_OOM;
  }
  *out = s;
  return MTE_OK;
}

extern "C" int mteg_get_sizes(const mteg_stream* s, mteg_sizes* o) {
  if (!s || !o) return MTE_E_INVALID_ARG;
  std::memset(o, 0, sizeof(*o));
  o->n_propsets = (uint32_t)s->fixed_ps.size();
  o->n_props = (uint32_t)s->fixed_pe.size();
  for (const DocOut& d : s->docs) {
    o->n_ops += d.ops.size();
    o->text_units += d.text.size();
    o->init_units += d.init_text.size();
    o->n_propsets += (uint32_t)d.psets.size();
    o->n_props += (uint32_t)d.props.size();
  }
  return MTE_OK;
}

extern "C" int mteg_fill(const mteg_stream* s, mte_doc_init* inits, uint16_t* init_text,
                         uint64_t* op_offsets, mte_op* ops, uint16_t* text, mte_propset* psets,
                         mte_prop* props) {
  if (!s || !inits || !op_offsets || !ops || !psets || !props) return MTE_E_INVALID_ARG;
  std::memcpy(psets, s->fixed_ps.data(), s->fixed_ps.size() * sizeof(mte_propset));
  std::memcpy(props, s->fixed_pe.data(), s->fixed_pe.size() * sizeof(mte_prop));
  uint64_t op_n = 0, text_n = 0, init_n = 0;
  uint32_t ps_n = (uint32_t)s->fixed_ps.size(), pe_n = (uint32_t)s->fixed_pe.size();
  for (size_t di = 0; di < s->docs.size(); di++) {
    const DocOut& d = s->docs[di];
    inits[di] = mte_doc_init{(uint32_t)init_n, (uint32_t)d.init_text.size(), d.flags, MTE_NO_PROPS, 0, 0};
    if (!d.init_text.empty() && init_text)
      std::memcpy(init_text + init_n, d.init_text.data(), d.init_text.size() * 2);
    init_n += d.init_text.size();
    op_offsets[di] = op_n;
    for (const mte_op& o0 : d.ops) {
      mte_op o = o0;
      if (o.type == MTE_OP_INSERT) {
        if (o.flags & MTE_F_MARKER) o.b += ps_n;
        else o.a += (uint32_t)text_n;
      }
      ops[op_n++] = o;
    }
    if (!d.text.empty() && text) std::memcpy(text + text_n, d.text.data(), d.text.size() * 2);
    text_n += d.text.size();
    for (const mte_propset& p : d.psets) psets[ps_n++] = mte_propset{p.first + pe_n, p.count};
    for (const mte_prop& p : d.props) props[pe_n++] = p;
  }
  op_offsets[s->docs.size()] = op_n;
  return MTE_OK;
}

extern "C" int mteg_free(mteg_stream* s) {
  delete s;
  return MTE_OK;
}

extern "C" int mteg_value_json(uint32_t id, char* buf, uint32_t cap) {
  if (!buf || cap == 0) return -1;
  int n;
  if (id >= 1 && id <= 32) n = std::snprintf(buf, cap, "\"%c\"", (char)('B' + id - 1));
  else if (id >= 33 && id <= 40) n = std::snprintf(buf, cap, "%u", id - 33);
  else if (id >= 41 && id <= 48) n = std::snprintf(buf, cap, "\"c%u\"", id - 41);
  else if (id >= 64) n = std::snprintf(buf, cap, "\"m%u\"", id - 64);
  else return -1;
  return (n < 0 || (uint32_t)n >= cap) ? -1 : n;
}
