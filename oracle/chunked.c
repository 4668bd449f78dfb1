/*
 * chunked.c — the flat restatement (oracle.c) with a chunk index, for
 * documents of millions of segments (TEST INFRASTRUCTURE: config 5's full-size
 * checker and CPU baseline).
 *
 * oracle.c recomputes every perspective length and prefix per op, O(S) per op:
 * at config 5 (2^20 segments per document) that is a strawman.  This file keeps
 * the same document -- the same segments, split on op boundaries, never
 * append-merged, tombstones dropped when removedSeq <= minSeq -- as a list of
 * chunks of at most CH segments, and per client a column of chunk lengths in
 * that client's perspective: the flat counterpart of the per-client entries of
 * PartialSequenceLengths.getPartialLength (partialLengths.ts:667-702) at chunk
 * granularity, as the GPU's chunk pass keeps them.  An op of
 * client c with refSeq r resolves its position on column c (rebuilt when c's
 * refSeq or the window's minSeq changed since it was built), then applies the
 * flat rules of oracle.c (doc_split_at, the insert slot, the range marks) to
 * the chunk(s) it lands in; per op O(chunks + CH), not O(S).
 *
 * Why a column stays exact across other clients' ops (new length calculation,
 * mergeTree.ts:1003-1026): an op (seq s, client c) makes a segment of seq s --
 * visible only to c in every held perspective, whose refSeqs are < s -- or
 * marks removals at s > every held refSeq, or adds c to removedClientIds; none
 * of that changes L(x; r', c') for c' != c.  Splits move no length between
 * chunks.  Only column c moves, by the op's own length change.
 *
 * Only remote (observer) replay with the new length calculation: the config-5
 * documents.  Other documents are refused (MTE_E_UNSUPPORTED).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 */
#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "chunked.h"
#include "orc_common.h"

#define NONE_SEQ ORC_NONE_SEQ
#define CH 512           /* segments per chunk at most */
#define CH_FILL 256      /* segments per chunk after a rebuild */

typedef struct {
  int32_t len, seq, rseq;
  uint32_t rmask;
  int32_t cli;
  uint32_t kind, toff;
  uint32_t props[MTE_MAX_KEYS];
} cseg;

typedef struct {
  cseg s[CH];
  uint32_t n;
} chunk;

typedef struct {
  chunk** ch;
  uint32_t nch, cap_ch;
  int32_t min_seq, cur_seq;
  uint32_t flags;
  int32_t status;
  /* per client: the perspective (refSeq, minSeq) column `col` holds, and the
   * chunk lengths in it (undefined leaves count 0) */
  int32_t col_r[MTE_MAX_CLIENTS], col_m[MTE_MAX_CLIENTS];
  int32_t* col[MTE_MAX_CLIENTS];
  uint32_t col_cap;
  uint64_t ops, rebuilds;
  mte_doc_init init;
  uint32_t init_props[MTE_MAX_KEYS];
} __attribute__((aligned(128))) cdoc;

struct och_ctx {
  uint32_t n_keys, n_docs;
  cdoc* docs;
  uint16_t* arena;
  uint64_t arena_n, arena_cap, load_units;
  mte_propset* load_ps;
  uint32_t n_load_ps;
  mte_prop* load_pe;
  uint32_t n_load_pe;
};

/* ---- lengths (oracle.c leaf_len, new calculation) -------------------------- */

static inline int32_t leaf_len(const cseg* s, int32_t r, int c, int32_t m) {
  if (s->rseq != NONE_SEQ) {
    if (s->rseq <= m) return -1;
    if (s->rseq <= r || ((s->rmask >> c) & 1u)) return 0;
  }
  return (s->seq <= r || s->cli == c) ? s->len : 0;
}

static int32_t chunk_len(const chunk* k, int32_t r, int c, int32_t m) {
  int32_t t = 0;
  for (uint32_t i = 0; i < k->n; i++) {
    const int32_t l = leaf_len(&k->s[i], r, c, m);
    if (l > 0) t += l;
  }
  return t;
}

/* ---- chunk list ---------------------------------------------------------------- */

static int cols_reserve(cdoc* d, uint32_t need) {
  if (need <= d->col_cap) return MTE_OK;
  uint32_t nc = d->col_cap ? d->col_cap : 64;
  while (nc < need) nc *= 2;
  for (int c = 0; c < MTE_MAX_CLIENTS; c++) {
    int32_t* x = (int32_t*)realloc(d->col[c], (size_t)nc * sizeof(int32_t));
    if (!x) return MTE_E_OOM;
    d->col[c] = x;
  }
  d->col_cap = nc;
  return MTE_OK;
}

static int chunks_reserve(cdoc* d, uint32_t need) {
  if (need > d->cap_ch) {
    uint32_t nc = d->cap_ch ? d->cap_ch : 16;
    while (nc < need) nc *= 2;
    chunk** x = (chunk**)realloc(d->ch, (size_t)nc * sizeof(chunk*));
    if (!x) return MTE_E_OOM;
    d->ch = x;
    d->cap_ch = nc;
  }
  return cols_reserve(d, need);
}

static void invalidate_cols(cdoc* d) {
  for (int c = 0; c < MTE_MAX_CLIENTS; c++) d->col_r[c] = INT32_MIN;
}

/* column c for (r, m): rebuilt from the chunks when it holds another perspective */
static void ensure_col(cdoc* d, int c, int32_t r, int32_t m) {
  if (d->col_r[c] == r && d->col_m[c] == m) return;
  for (uint32_t k = 0; k < d->nch; k++) d->col[c][k] = chunk_len(d->ch[k], r, c, m);
  d->col_r[c] = r;
  d->col_m[c] = m;
  d->rebuilds++;
}

/* split chunk k in two halves (it is full); every valid column gets the halves' lengths */
static int split_chunk(cdoc* d, uint32_t k) {
  int rc = chunks_reserve(d, d->nch + 1);
  if (rc) return rc;
  chunk* a = d->ch[k];
  chunk* b = (chunk*)malloc(sizeof(chunk));
  if (!b) return MTE_E_OOM;
  const uint32_t h = a->n / 2;
  b->n = a->n - h;
  memcpy(b->s, a->s + h, (size_t)b->n * sizeof(cseg));
  a->n = h;
  memmove(d->ch + k + 2, d->ch + k + 1, (size_t)(d->nch - k - 1) * sizeof(chunk*));
  d->ch[k + 1] = b;
  for (int c = 0; c < MTE_MAX_CLIENTS; c++) {
    if (d->col_r[c] == INT32_MIN) continue;
    memmove(d->col[c] + k + 2, d->col[c] + k + 1, (size_t)(d->nch - k - 1) * sizeof(int32_t));
    const int32_t la = chunk_len(a, d->col_r[c], c, d->col_m[c]);
    d->col[c][k + 1] = d->col[c][k] - la;
    d->col[c][k] = la;
  }
  d->nch++;
  return MTE_OK;
}

/* open a slot at index i of chunk k (splitting a full chunk first); returns
 * the slot's (chunk, index) through *k / *i */
static int open_slot(cdoc* d, uint32_t* k, uint32_t* i) {
  if (d->ch[*k]->n == CH) {
    int rc = split_chunk(d, *k);
    if (rc) return rc;
    const uint32_t h = d->ch[*k]->n;
    if (*i > h) {
      *i -= h;
      (*k)++;
    }
  }
  chunk* ck = d->ch[*k];
  memmove(ck->s + *i + 1, ck->s + *i, (size_t)(ck->n - *i) * sizeof(cseg));
  ck->n++;
  return MTE_OK;
}

/* rebuild the chunk list: drop tombstones at or below minSeq (setMinSeq's
 * zamboni, content-equivalent, oracle.c doc_compact), CH_FILL per chunk */
static int relayout(cdoc* d) {
  uint32_t total = 0;
  for (uint32_t k = 0; k < d->nch; k++) total += d->ch[k]->n;
  cseg* all = (cseg*)malloc((size_t)(total ? total : 1) * sizeof(cseg));
  if (!all) return MTE_E_OOM;
  uint32_t w = 0;
  for (uint32_t k = 0; k < d->nch; k++) {
    const chunk* ck = d->ch[k];
    for (uint32_t i = 0; i < ck->n; i++)
      if (!(ck->s[i].rseq != NONE_SEQ && ck->s[i].rseq <= d->min_seq)) all[w++] = ck->s[i];
  }
  const uint32_t need = w ? (w + CH_FILL - 1) / CH_FILL : 1;
  for (uint32_t k = need; k < d->nch; k++) free(d->ch[k]);
  int rc = chunks_reserve(d, need);
  if (rc) {
    free(all);
    return rc;
  }
  for (uint32_t k = d->nch; k < need; k++) {
    d->ch[k] = (chunk*)malloc(sizeof(chunk));
    if (!d->ch[k]) {
      free(all);
      return MTE_E_OOM;
    }
  }
  d->nch = need;
  for (uint32_t k = 0; k < need; k++) {
    const uint32_t a = k * CH_FILL, b = a + CH_FILL < w ? a + CH_FILL : w;
    d->ch[k]->n = b > a ? b - a : 0;
    if (b > a) memcpy(d->ch[k]->s, all + a, (size_t)(b - a) * sizeof(cseg));
  }
  free(all);
  invalidate_cols(d);
  return MTE_OK;
}

/* ---- position lookups on column c ----------------------------------------------- */

/* the first chunk whose end (prefix + length) satisfies end > pos (strict) or
 * end >= pos; *pre = the prefix before it; nch when none */
static uint32_t find_chunk(const cdoc* d, int c, int64_t pos, int strict, int64_t* pre) {
  int64_t p = 0;
  const int32_t* col = d->col[c];
  for (uint32_t k = 0; k < d->nch; k++) {
    const int64_t e = p + col[k];
    if (strict ? e > pos : e >= pos) {
      *pre = p;
      return k;
    }
    p = e;
  }
  *pre = p;
  return d->nch;
}

/* ensureIntervalBoundary(pos) (oracle.c doc_split_at): split the leaf with
 * L > 0 and P < pos < P + L; column c is unchanged by a split */
static int split_at(cdoc* d, int c, int32_t r, int32_t m, int64_t pos) {
  int64_t p;
  uint32_t k = find_chunk(d, c, pos, 1, &p);
  if (k == d->nch) return MTE_OK;
  chunk* ck = d->ch[k];
  for (uint32_t i = 0; i < ck->n; i++) {
    const int32_t l = leaf_len(&ck->s[i], r, c, m);
    if (l <= 0) continue;
    if (pos < p) return MTE_OK;
    if (pos < p + l) {
      const int64_t off = pos - p;
      if (off == 0 || ck->s[i].kind != 0) return MTE_OK;
      uint32_t kk = k, ii = i + 1;
      int rc = open_slot(d, &kk, &ii);
      if (rc) return rc;
      /* after a chunk split the head may have moved too: locate it again */
      uint32_t kh = kk, ih = ii;
      if (ih == 0) {
        kh = kk - 1;
        ih = d->ch[kh]->n - 1;
      } else {
        ih--;
      }
      cseg* head = &d->ch[kh]->s[ih];
      cseg* tail = &d->ch[kk]->s[ii];
      *tail = *head;
      tail->len = head->len - (int32_t)off;
      tail->toff = head->toff + (uint32_t)off;
      head->len = (int32_t)off;
      /* a split moves no length between chunks except when head and tail land
       * in different chunks: then the columns of both chunks move */
      if (kh != kk) {
        for (int cc = 0; cc < MTE_MAX_CLIENTS; cc++) {
          if (d->col_r[cc] == INT32_MIN) continue;
          const int32_t lt = leaf_len(tail, d->col_r[cc], cc, d->col_m[cc]);
          if (lt > 0) {
            d->col[cc][kh] -= lt;
            d->col[cc][kk] += lt;
          }
        }
      }
      return MTE_OK;
    }
    p += l;
  }
  return MTE_OK;
}

/* ---- one op ------------------------------------------------------------------------------ */

typedef struct {
  const mte_batch* b;
  uint64_t text_base;
  uint32_t n_keys;
} env_t;

static int doc_apply(cdoc* d, const mte_op* op, const env_t* env) {
  const int32_t r = op->ref_seq, s = op->seq, m = d->min_seq;
  const int c = op->client;
  int rc;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  if (op->flags & MTE_F_LOCAL) return MTE_E_UNSUPPORTED;
  if (op->type > MTE_OP_ANNOTATE && op->type != MTE_OP_NOOP) return MTE_E_UNSUPPORTED;
  d->ops++;
  if (op->type == MTE_OP_INSERT) {
    ensure_col(d, c, r, m);
    if ((rc = split_at(d, c, r, m, op->pos1))) return rc;
    const int is_marker = (op->flags & MTE_F_MARKER) != 0;
    const int32_t len = is_marker ? 1 : op->pos2;
    if (len > 0) {
      /* before the first defined leaf with P >= pos, else at the end
       * (oracle.c doc_apply); pos past the length fails */
      const int64_t pos = op->pos1;
      int64_t p;
      uint32_t k = find_chunk(d, c, pos, 0, &p), at_k = d->nch, at_i = 0;
      for (; k < d->nch && at_k == d->nch; k++) {
        const chunk* ck = d->ch[k];
        for (uint32_t i = 0; i < ck->n; i++) {
          const int32_t l = leaf_len(&ck->s[i], r, c, m);
          if (l >= 0 && p >= pos) {
            at_k = k;
            at_i = i;
            break;
          }
          if (l > 0) p += l;
        }
      }
      if (at_k == d->nch) {
        if (pos > p) return MTE_E_INSERT_FAILED;
        at_k = d->nch - 1;
        at_i = d->ch[at_k]->n;
      }
      if ((rc = open_slot(d, &at_k, &at_i))) return rc;
      cseg* ns = &d->ch[at_k]->s[at_i];
      memset(ns, 0, sizeof(*ns));
      ns->len = len;
      ns->seq = s;
      ns->cli = c;
      ns->rseq = NONE_SEQ;
      if (is_marker) {
        ns->kind = 1u + (uint32_t)op->pos2;
      } else {
        ns->toff = (uint32_t)(env->text_base + op->a);
      }
      if (op->b != MTE_NO_PROPS) orc_apply_props(ns->props, env->n_keys, &env->b->propsets[op->b], env->b->props, 0);
      d->col[c][at_k] += len; /* only the inserting client sees it */
    }
  } else if (op->type == MTE_OP_REMOVE || op->type == MTE_OP_ANNOTATE) {
    const int64_t start = op->pos1, end = op->pos2;
    ensure_col(d, c, r, m);
    if ((rc = split_at(d, c, r, m, start))) return rc;
    if ((rc = split_at(d, c, r, m, end))) return rc;
    if (end > start) {
      int64_t p;
      uint32_t k = find_chunk(d, c, start, 1, &p);
      for (; k < d->nch && p < end; k++) {
        chunk* ck = d->ch[k];
        for (uint32_t i = 0; i < ck->n && p < end; i++) {
          cseg* g = &ck->s[i];
          const int32_t l = leaf_len(g, r, c, m);
          if (l <= 0) continue;
          if (p + l > start) {
            if (op->type == MTE_OP_REMOVE) {
              if (g->rseq == NONE_SEQ) {
                g->rseq = s;
                g->rmask = 1u << c;
              } else {
                g->rmask |= 1u << c;
              }
              d->col[c][k] -= l; /* removed for c (by_c); no one else's length moves */
            } else {
              orc_apply_props(g->props, env->n_keys, &env->b->propsets[op->a], env->b->props,
                              (op->flags & MTE_F_REWRITE) != 0);
            }
          }
          p += l;
        }
      }
    }
  } else if (op->type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  if (op->type != MTE_OP_NOOP) {
    if (!(d->cur_seq < s)) return MTE_E_SEQ_ORDER;
    if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
  }
  if (op->flags & MTE_F_MSG_END) {
    if (!(d->cur_seq <= s)) return MTE_E_SEQ_ORDER;
    d->cur_seq = s;
    if (!(op->min_seq <= s)) return MTE_E_MSN_GT_SEQ;
    if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
    if (op->min_seq > d->min_seq) {
      d->min_seq = op->min_seq;
      if ((rc = relayout(d))) return rc;
    }
  }
  return MTE_OK;
}

/* ---- API --------------------------------------------------------------------------------- */

static int arena_append(och_ctx* c, const uint16_t* t, uint64_t n, uint64_t* base) {
  if (c->arena_n + n > c->arena_cap) {
    uint64_t nc = c->arena_cap ? c->arena_cap : 1024;
    while (nc < c->arena_n + n) nc *= 2;
    uint16_t* a = (uint16_t*)realloc(c->arena, nc * sizeof(uint16_t));
    if (!a) return MTE_E_OOM;
    c->arena = a;
    c->arena_cap = nc;
  }
  *base = c->arena_n;
  if (n) memcpy(c->arena + c->arena_n, t, n * sizeof(uint16_t));
  c->arena_n += n;
  return MTE_OK;
}

int och_create(uint32_t n_keys, och_ctx** out) {
  if (!out || n_keys > MTE_MAX_KEYS) return MTE_E_INVALID_ARG;
  och_ctx* c = (och_ctx*)calloc(1, sizeof(och_ctx));
  if (!c) return MTE_E_OOM;
  c->n_keys = n_keys;
  *out = c;
  return MTE_OK;
}

static void free_doc(cdoc* d) {
  for (uint32_t k = 0; k < d->nch; k++) free(d->ch[k]);
  free(d->ch);
  for (int c = 0; c < MTE_MAX_CLIENTS; c++) free(d->col[c]);
  memset(d, 0, sizeof(*d));
}

static void free_docs(och_ctx* c) {
  for (uint32_t i = 0; i < c->n_docs; i++) free_doc(&c->docs[i]);
  free(c->docs);
  free(c->load_ps);
  free(c->load_pe);
  c->docs = NULL;
  c->load_ps = NULL;
  c->load_pe = NULL;
  c->n_docs = 0;
}

int och_destroy(och_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  free_docs(c);
  free(c->arena);
  free(c);
  return MTE_OK;
}

/* a document from one segment list (the load text or a summary body) */
static int doc_from(cdoc* d, const cseg* segs, uint32_t n) {
  for (uint32_t k = 0; k < d->nch; k++) free(d->ch[k]);
  d->nch = 0;
  const uint32_t need = n ? (n + CH_FILL - 1) / CH_FILL : 1;
  int rc = chunks_reserve(d, need);
  if (rc) return rc;
  for (uint32_t k = 0; k < need; k++) {
    d->ch[k] = (chunk*)malloc(sizeof(chunk));
    if (!d->ch[k]) return MTE_E_OOM;
    const uint32_t a = k * CH_FILL, b = a + CH_FILL < n ? a + CH_FILL : n;
    d->ch[k]->n = b > a ? b - a : 0;
    if (b > a) memcpy(d->ch[k]->s, segs + a, (size_t)(b - a) * sizeof(cseg));
  }
  d->nch = need;
  invalidate_cols(d);
  return MTE_OK;
}

int och_load_docs(och_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text, uint64_t text_units,
                  const mte_propset* propsets, uint32_t n_propsets, const mte_prop* props, uint32_t n_props) {
  if (!c || (n_docs && !docs)) return MTE_E_INVALID_ARG;
  free_docs(c);
  c->arena_n = 0;
  uint64_t base = 0;
  int rc = arena_append(c, text, text_units, &base);
  if (rc) return rc;
  c->load_units = text_units;
  c->docs = (cdoc*)aligned_alloc(128, (size_t)(n_docs ? n_docs : 1) * sizeof(cdoc));
  if (!c->docs) return MTE_E_OOM;
  memset(c->docs, 0, (size_t)(n_docs ? n_docs : 1) * sizeof(cdoc));
  c->n_docs = n_docs;
  if (n_propsets) {
    c->load_ps = (mte_propset*)malloc((size_t)n_propsets * sizeof(mte_propset));
    if (!c->load_ps) return MTE_E_OOM;
    memcpy(c->load_ps, propsets, (size_t)n_propsets * sizeof(mte_propset));
    c->n_load_ps = n_propsets;
  }
  if (n_props) {
    c->load_pe = (mte_prop*)malloc((size_t)n_props * sizeof(mte_prop));
    if (!c->load_pe) return MTE_E_OOM;
    memcpy(c->load_pe, props, (size_t)n_props * sizeof(mte_prop));
    c->n_load_pe = n_props;
  }
  for (uint32_t i = 0; i < n_docs; i++) {
    cdoc* d = &c->docs[i];
    const mte_doc_init* in = &docs[i];
    if ((uint64_t)in->text_off + in->text_len > text_units) return MTE_E_INVALID_ARG;
    d->init = *in;
    d->flags = in->flags;
    d->min_seq = in->min_seq;
    d->cur_seq = in->cur_seq;
    if (!(in->flags & MTE_DOC_NEW_LENGTH_CALC) || (in->flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS)))
      d->status = MTE_E_UNSUPPORTED;
    cseg g;
    memset(&g, 0, sizeof g);
    g.len = (int32_t)in->text_len;
    g.cli = -1;
    g.rseq = NONE_SEQ;
    g.toff = (uint32_t)(base + in->text_off);
    if (in->propset != MTE_NO_PROPS) {
      if (in->propset >= n_propsets) return MTE_E_INVALID_ARG;
      orc_apply_props(g.props, c->n_keys, &propsets[in->propset], props, 0);
    }
    if ((rc = doc_from(d, &g, in->text_len > 0 ? 1u : 0u))) return rc;
  }
  return MTE_OK;
}

int och_load_segments(och_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs) {
  if (!c || !seg_offsets || (n_segs && !segs)) return MTE_E_INVALID_ARG;
  if (seg_offsets[0] != 0 || seg_offsets[c->n_docs] != n_segs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < c->n_docs; di++) {
    const uint64_t b = seg_offsets[di], e = seg_offsets[di + 1];
    if (e < b) return MTE_E_INVALID_ARG;
    if (e == b) continue;
    const uint32_t n = (uint32_t)(e - b);
    cseg* tmp = (cseg*)calloc(n, sizeof(cseg));
    if (!tmp) return MTE_E_OOM;
    for (uint32_t k = 0; k < n; k++) {
      const mte_seg* sg = &segs[b + k];
      const int marker = sg->kind != 0;
      if ((marker && sg->len != 1) || (!marker && (sg->len == 0 || (uint64_t)sg->text_off + sg->len > c->load_units)) ||
          sg->client < -1 || sg->client >= MTE_MAX_CLIENTS || sg->seq < 0 ||
          (sg->removed_seq != MTE_NOT_REMOVED && sg->removers == 0)) {
        free(tmp);
        return MTE_E_INVALID_ARG;
      }
      cseg* g = &tmp[k];
      g->len = (int32_t)sg->len;
      g->seq = sg->seq;
      g->cli = sg->client;
      g->rseq = sg->removed_seq == MTE_NOT_REMOVED ? NONE_SEQ : sg->removed_seq;
      g->rmask = sg->removed_seq == MTE_NOT_REMOVED ? 0u : sg->removers;
      g->kind = sg->kind;
      g->toff = marker ? 0u : sg->text_off;
      if (sg->propset != MTE_NO_PROPS) {
        if (sg->propset >= c->n_load_ps) {
          free(tmp);
          return MTE_E_INVALID_ARG;
        }
        orc_apply_props(g->props, c->n_keys, &c->load_ps[sg->propset], c->load_pe, 0);
      }
    }
    const int rc = doc_from(&c->docs[di], tmp, n);
    free(tmp);
    if (rc) return rc;
  }
  return MTE_OK;
}

typedef struct {
  och_ctx* c;
  const mte_batch* b;
  uint64_t base;
  uint32_t d0, d1, stride;
} worker_arg;

static void* worker(void* p) {
  worker_arg* w = (worker_arg*)p;
  env_t env = {w->b, w->base, w->c->n_keys};
  for (uint32_t di = w->d0; di < w->d1; di += w->stride) {
    cdoc* d = &w->c->docs[di];
    if (d->status) continue;
    for (uint64_t k = w->b->op_offsets[di]; k < w->b->op_offsets[di + 1]; k++) {
      const int rc = doc_apply(d, &w->b->ops[k], &env);
      if (rc) {
        d->status = rc;
        break;
      }
    }
  }
  return NULL;
}

int och_apply_batch(och_ctx* c, const mte_batch* b, int n_threads) {
  if (!c || !b || b->n_docs != c->n_docs || !b->op_offsets) return MTE_E_INVALID_ARG;
  if (b->op_offsets[b->n_docs] != b->n_ops) return MTE_E_INVALID_ARG;
  for (uint64_t k = 0; k < b->n_ops; k++) {
    const mte_op* op = &b->ops[k];
    if (op->type == MTE_OP_INSERT && !(op->flags & MTE_F_MARKER) && op->pos2 > 0 &&
        (uint64_t)op->a + (uint64_t)op->pos2 > b->text_units)
      return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_INSERT && op->b != MTE_NO_PROPS && op->b >= b->n_propsets) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_ANNOTATE && op->a >= b->n_propsets) return MTE_E_INVALID_ARG;
  }
  uint64_t base = 0;
  int rc = arena_append(c, b->text, b->text_units, &base);
  if (rc) return rc;
  if (n_threads < 1) n_threads = 1;
  if ((uint32_t)n_threads > c->n_docs) n_threads = c->n_docs ? (int)c->n_docs : 1;
  worker_arg* args = (worker_arg*)calloc((size_t)n_threads, sizeof(worker_arg));
  pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
  if (!args || !th) {
    free(args);
    free(th);
    return MTE_E_OOM;
  }
  for (int t = 0; t < n_threads; t++) args[t] = (worker_arg){c, b, base, (uint32_t)t, c->n_docs, (uint32_t)n_threads};
  if (n_threads == 1) {
    worker(&args[0]);
  } else {
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, worker, &args[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  }
  free(args);
  free(th);
  return MTE_OK;
}

int och_digest(och_ctx* c, uint64_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < n_docs; di++) {
    const cdoc* d = &c->docs[di];
    orc_digest_acc acc = {0, 0, 0, 0};
    for (uint32_t k = 0; k < d->nch; k++) {
      const chunk* ck = d->ch[k];
      for (uint32_t i = 0; i < ck->n; i++) {
        const cseg* g = &ck->s[i];
        if (g->rseq != NONE_SEQ) continue;
        orc_digest_seg(&acc, g->kind, g->kind == 0 ? c->arena + g->toff : NULL, g->len, g->props, c->n_keys);
      }
    }
    out[4 * (size_t)di + 0] = acc.n;
    out[4 * (size_t)di + 1] = acc.h1;
    out[4 * (size_t)di + 2] = acc.h2;
    out[4 * (size_t)di + 3] = acc.sum;
  }
  return MTE_OK;
}

int och_doc_status(och_ctx* c, int32_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < n_docs; i++) out[i] = c->docs[i].status;
  return MTE_OK;
}

int och_doc_nsegs(och_ctx* c, uint32_t doc, uint32_t* out) {
  if (!c || !out || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  uint32_t n = 0;
  for (uint32_t k = 0; k < c->docs[doc].nch; k++) n += c->docs[doc].ch[k]->n;
  *out = n;
  return MTE_OK;
}

int och_read_doc(och_ctx* c, uint32_t doc, mte_doc_view* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const cdoc* d = &c->docs[doc];
  v->status = d->status;
  v->cur_seq = d->cur_seq;
  v->min_seq = d->min_seq;
  uint32_t length = 0, nt = 0, ns = 0;
  for (uint32_t k = 0; k < d->nch; k++) {
    const chunk* ck = d->ch[k];
    for (uint32_t i = 0; i < ck->n; i++) {
      const cseg* g = &ck->s[i];
      if (g->rseq != NONE_SEQ) continue;
      if (ns < v->seg_cap) {
        if (v->seg_len) v->seg_len[ns] = (uint32_t)g->len;
        if (v->seg_kind) v->seg_kind[ns] = g->kind;
        if (v->seg_props)
          for (uint32_t q = 0; q < c->n_keys; q++) v->seg_props[(size_t)ns * c->n_keys + q] = g->props[q];
      }
      ns++;
      length += (uint32_t)g->len;
      if (g->kind == 0)
        for (int32_t u = 0; u < g->len; u++, nt++)
          if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
    }
  }
  v->length = length;
  v->n_text = nt;
  v->n_segs = ns;
  return MTE_OK;
}

/* every held segment, tombstones included, in document order (as
 * mte_read_segments / orc_read_segments) */
int och_read_segments(och_ctx* c, uint32_t doc, mte_seg_list* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const cdoc* d = &c->docs[doc];
  uint64_t nt = 0;
  uint32_t i = 0;
  for (uint32_t k = 0; k < d->nch; k++) {
    const chunk* ck = d->ch[k];
    for (uint32_t j = 0; j < ck->n; j++, i++) {
      const cseg* g = &ck->s[j];
      if (i < v->seg_cap && v->segs) {
        mte_seg* s = &v->segs[i];
        s->text_off = g->kind == 0 ? (uint32_t)nt : 0u;
        s->len = (uint32_t)g->len;
        s->seq = g->seq;
        s->removed_seq = g->rseq == NONE_SEQ ? MTE_NOT_REMOVED : g->rseq;
        s->removers = g->rseq == NONE_SEQ ? 0u : g->rmask;
        s->client = g->cli;
        s->kind = g->kind;
        s->propset = MTE_NO_PROPS;
        if (v->props)
          for (uint32_t q = 0; q < c->n_keys; q++) v->props[(size_t)i * c->n_keys + q] = g->props[q];
      }
      if (g->kind == 0)
        for (int32_t u = 0; u < g->len; u++, nt++)
          if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
    }
  }
  v->n_segs = i;
  v->n_text = nt;
  return MTE_OK;
}

int och_stats_get(och_ctx* c, mte_stats* o) {
  if (!c || !o) return MTE_E_INVALID_ARG;
  memset(o, 0, sizeof(*o));
  for (uint32_t i = 0; i < c->n_docs; i++) o->ops_applied += c->docs[i].ops;
  return MTE_OK;
}
