/*
 * titems.c — the reference B+tree restated on a FLAT ITEM ARRAY
 * (TEST INFRASTRUCTURE: the executable spec of the GPU tree pass).
 *
 * tree.c keeps the reference's tree as linked blocks; the GPU cannot.  This
 * file keeps the same tree as the GPU kernel does (mte_tree.h): the segments
 * in document order, each with a small tree word
 *   h      the number of block levels this item starts (0: inside a leaf
 *          block; 1: starts a leaf block; 2: also its parent; ...);
 *   cont   the item continues the previous item's leaf (an append-merge of
 *          scourNode, mergeTree.ts:716-728: two texts that became one leaf
 *          stay two items, so no text is ever copied);
 *   ns     needsScour of the leaf block the item starts (mergeTreeNodes.ts:98);
 *   po     segment.properties exists ({} vs undefined for matchProperties);
 *   empty  a placeholder for an empty leaf block (packParent can make one,
 *          mergeTree.ts:764-786; the empty root, 495-498);
 *   id     the identity the LRU heap entries name (mergeTree.ts:452-455),
 * and the heap itself as an array (collections/heap.ts).  Every rule cites the
 * reference in tree.c; this file only re-expresses them over the item array.
 * It must agree with tree.c on every document (tests/test_tree_items.py).
 */
#include <limits.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"
#include "titems.h"

#define NONE_SEQ ORC_NONE_SEQ
#define UNDEF_SEQ INT32_MIN /* removedSeq of a placeholder: undefined to every perspective */
#define MAX_NODES 8
#define TEXT_GRANULARITY 256
#define ZAMBONI_MAX 2
#define NS_UNDEF 0
#define NS_FALSE 1
#define NS_TRUE 2

typedef struct {
  int32_t len, seq, rseq;
  uint32_t rmask;
  int32_t cli;
  uint32_t kind, toff;
  uint32_t props[MTE_MAX_KEYS];
  uint8_t h, cont, ns, po, empty, drop;
  uint32_t id;
} item;

typedef struct {
  int32_t max_seq;
  uint32_t id;
} hent;

typedef struct {
  item* it;
  uint32_t n, cap;
  int32_t depth;
  uint32_t next_id;
  hent* heap;
  uint32_t hn, hcap;
  int32_t min_seq, cur_seq;
  uint32_t flags;
  int32_t status;
  int32_t* L;
  int64_t* P;
  uint32_t scap;
  /* the GPU tree pass's statistics (mte_stats), counted the same way */
  uint64_t ops, scanned, written, pwrites, units, max_segs;
  mte_doc_init init;
} __attribute__((aligned(128))) idoc;

struct oti_ctx {
  uint32_t n_keys, n_docs;
  uint32_t limit; /* items + 4 of headroom a document may reach (the GPU tree pass: min(1024, cap)) */
  idoc* docs;
  uint16_t* arena;
  uint64_t arena_n, arena_cap, load_units;
  mte_propset* load_ps;
  uint32_t n_load_ps;
  mte_prop* load_pe;
  uint32_t n_load_pe;
};

typedef struct {
  const mte_batch* b;
  uint64_t text_base;
  uint32_t n_keys;
  const uint16_t* arena;
  uint32_t limit;
} env_t;

/* ---- storage --------------------------------------------------------------- */

static int reserve(idoc* d, uint32_t need) {
  if (need > d->cap) {
    uint32_t nc = d->cap ? d->cap : 64;
    while (nc < need) nc *= 2;
    item* x = (item*)realloc(d->it, (size_t)nc * sizeof(item));
    if (!x) return MTE_E_OOM;
    d->it = x;
    d->cap = nc;
  }
  if (need > d->scap) {
    uint32_t nc = d->cap;
    int32_t* L = (int32_t*)realloc(d->L, (size_t)nc * sizeof(int32_t));
    int64_t* P = (int64_t*)realloc(d->P, (size_t)nc * sizeof(int64_t));
    if (!L || !P) return MTE_E_OOM;
    d->L = L;
    d->P = P;
    d->scap = nc;
  }
  return MTE_OK;
}

/* open an empty slot at index g */
static int open_slot(idoc* d, uint32_t g) {
  int rc = reserve(d, d->n + 1);
  if (rc) return rc;
  memmove(d->it + g + 1, d->it + g, (size_t)(d->n - g) * sizeof(item));
  memset(&d->it[g], 0, sizeof(item));
  d->n++;
  return MTE_OK;
}

static void compact(idoc* d) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < d->n; i++)
    if (!d->it[i].drop) d->it[w++] = d->it[i];
  d->n = w;
}

static uint32_t new_id(idoc* d) { return d->next_id++; }

static item placeholder(uint8_t h) {
  item e;
  memset(&e, 0, sizeof e);
  e.rseq = UNDEF_SEQ;
  e.h = h;
  e.empty = 1;
  return e;
}

/* ---- lengths ------------------------------------------------------------------ */

static inline int32_t leaf_len(const item* s, int32_t r, int c, int32_t m, int newcalc) {
  const int removed = s->rseq != NONE_SEQ;
  const int by_c = (int)((s->rmask >> c) & 1u);
  if (newcalc) {
    if (removed) {
      if (s->rseq <= m) return -1;
      if (s->rseq <= r || by_c) return 0;
    }
    return (s->seq <= r || s->cli == c) ? s->len : 0;
  }
  if (removed && s->rseq <= r) return -1;
  if (s->cli == c || s->seq <= r) return (removed && by_c) ? 0 : s->len;
  return removed ? -1 : 0;
}

static int64_t lengths(idoc* d, int32_t r, int c, int32_t m, int newcalc) {
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = leaf_len(&d->it[i], r, c, m, newcalc);
    d->L[i] = l;
    d->P[i] = p;
    if (l > 0) p += l;
  }
  return p;
}

/* ---- block spans ------------------------------------------------------------------ */

static uint32_t span_start(const idoc* d, uint32_t i, int k) {
  while (i > 0 && d->it[i].h < k) i--;
  return i;
}
static uint32_t span_end(const idoc* d, uint32_t i, int k) {
  uint32_t j = i + 1;
  while (j < d->n && d->it[j].h < k) j++;
  return j - 1;
}
/* children of the level-k block spanning [s, e]: logical leaves (k = 1) or
 * level-(k-1) block starts */
static int is_child(const item* x, int k) { return k == 1 ? (!x->cont && !x->empty) : x->h >= k - 1; }
static int children(const idoc* d, uint32_t s, uint32_t e, int k) {
  int c = 0;
  for (uint32_t i = s; i <= e; i++) c += is_child(&d->it[i], k);
  return c;
}

/* a leaf block gained a child at item i: split full blocks bottom-up
 * (insertingWalk 1800-1821, split 1827-1840, updateRoot 1263-1272) */
static void split_cascade(idoc* d, uint32_t i) {
  for (int k = 1;; k++) {
    const uint32_t s = span_start(d, i, k), e = span_end(d, s, k);
    if (children(d, s, e, k) < MAX_NODES) return;
    int seen = 0;
    uint32_t z = s;
    for (uint32_t j = s; j <= e; j++)
      if (is_child(&d->it[j], k) && seen++ == MAX_NODES / 2) {
        z = j;
        break;
      }
    d->it[z].h = (uint8_t)k;
    if (k == 1) d->it[z].ns = NS_UNDEF;
    if (k == d->depth) { /* the root split: a new root above both halves */
      d->depth++;
      d->it[0].h = (uint8_t)d->depth;
      return;
    }
  }
}

/* ---- LRU heap (collections/heap.ts) ---------------------------------------------------- */

static int heap_add(idoc* d, int32_t key, uint32_t id) {
  if (d->hn + 2 > d->hcap) {
    uint32_t nc = d->hcap ? 2 * d->hcap : 64;
    hent* h = (hent*)realloc(d->heap, (size_t)nc * sizeof(hent));
    if (!h) return MTE_E_OOM;
    d->heap = h;
    d->hcap = nc;
  }
  hent* L = d->heap;
  L[++d->hn] = (hent){key, id};
  for (uint32_t k = d->hn; k > 1 && L[k >> 1].max_seq - L[k].max_seq > 0; k >>= 1) {
    hent t = L[k >> 1];
    L[k >> 1] = L[k];
    L[k] = t;
  }
  return MTE_OK;
}

static hent heap_get(idoc* d) {
  hent* L = d->heap;
  hent x = L[1];
  L[1] = L[d->hn];
  d->hn--;
  uint32_t k = 1;
  while ((k << 1) <= d->hn) {
    uint32_t j = k << 1;
    if (j < d->hn && L[j].max_seq - L[j + 1].max_seq > 0) j++;
    if (L[k].max_seq - L[j].max_seq <= 0) break;
    hent t = L[k];
    L[k] = L[j];
    L[j] = t;
    k = j;
  }
  return x;
}

/* addToLRUSet for the leaf headed at item i */
static int add_lru(idoc* d, uint32_t i, int32_t seq) {
  const uint32_t bs = span_start(d, i, 1);
  if (d->it[bs].ns != NS_TRUE && seq > d->cur_seq) {
    d->it[bs].ns = NS_TRUE;
    return heap_add(d, seq, d->it[i].id);
  }
  return MTE_OK;
}

/* ---- scour / pack ---------------------------------------------------------------------------- */

/* end (exclusive) of the logical leaf headed at i */
static uint32_t leaf_end(const idoc* d, uint32_t i) {
  uint32_t j = i + 1;
  while (j < d->n && d->it[j].cont) j++;
  return j;
}

static int64_t leaf_total(const idoc* d, uint32_t a, uint32_t b) {
  int64_t s = 0;
  for (uint32_t j = a; j < b; j++) s += d->it[j].len;
  return s;
}

/* scourNode over the leaf block [s, e] (mergeTree.ts:681-747): marks the
 * unlinked items `drop`, turns appended leaves into continuations.  Returns
 * the logical leaves held. */
static int scour(idoc* d, uint32_t s, uint32_t e, const uint16_t* arena, uint32_t n_keys) {
  int held = 0;
  int64_t prev = -1;  /* head of the leaf appends go to */
  int64_t prev_len = 0;
  uint32_t prev_end = 0;
  for (uint32_t i = s; i <= e;) {
    item* x = &d->it[i];
    if (x->empty) {
      i++;
      continue;
    }
    const uint32_t xe = leaf_end(d, i);
    const int64_t xl = leaf_total(d, i, xe);
    if (x->rseq != NONE_SEQ) {
      if (x->rseq > d->min_seq) {
        held++;
      } else {
        for (uint32_t j = i; j < xe; j++) d->it[j].drop = 1;
      }
      prev = -1;
    } else if (x->seq <= d->min_seq) {
      int app = 0;
      if (prev >= 0) {
        const item* p = &d->it[prev];
        const item* pl = &d->it[prev_end - 1]; /* the last text of the leaf appended to */
        const int nl = pl->len > 0 && arena[pl->toff + (uint32_t)pl->len - 1] == (uint16_t)'\n';
        int match = p->po == x->po;
        for (uint32_t k = 0; k < n_keys && match; k++) match = p->props[k] == x->props[k];
        app = p->kind == 0 && x->kind == 0 && !nl && (prev_len <= TEXT_GRANULARITY || xl <= TEXT_GRANULARITY) &&
              match && xl > 0;
      }
      if (app) {
        x->cont = 1;
        x->id = 0;
        prev_len += xl;
        prev_end = xe;
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
  return held;
}

/* drop the marked items, keeping every block start on a surviving item of
 * its block; a leaf block left with no leaf keeps a placeholder */
static void drop_keep_starts(idoc* d, uint32_t s, uint32_t e) {
  for (uint32_t b = s; b <= e;) {
    const uint32_t be = span_end(d, b, 1);
    uint32_t j = b;
    while (j <= be && d->it[j].drop) j++;
    if (j > be) {
      const uint8_t h = d->it[b].h, ns = d->it[b].ns;
      d->it[b] = placeholder(h);
      d->it[b].ns = ns;
    } else if (j != b) {
      d->it[j].h = d->it[b].h;
      d->it[j].ns = d->it[b].ns;
    }
    b = be + 1;
  }
}

/* packParent (mergeTree.ts:750-798) of the level-p block spanning [s, e] */
static void pack_parent(idoc* d, uint32_t s, int p, const uint16_t* arena, uint32_t n_keys) {
  uint32_t e = span_end(d, s, p);
  const uint8_t top = d->it[s].h;
  if (p == 2) {
    for (uint32_t b = s; b <= e; b = span_end(d, b, 1) + 1) scour(d, b, span_end(d, b, 1), arena, n_keys);
    /* the held leaves, re-packed */
    uint32_t w = s;
    for (uint32_t i = s; i <= e; i++) {
      if (d->it[i].drop || d->it[i].empty) continue;
      d->it[w] = d->it[i];
      d->it[w].h = 0;
      w++;
    }
    const uint32_t removed = (e + 1) - w;
    memmove(d->it + w, d->it + e + 1, (size_t)(d->n - e - 1) * sizeof(item));
    d->n -= removed;
    e = w == s ? s : w - 1;
    if (w == s) { /* no leaf left: one empty leaf block */
      if (open_slot(d, s)) return;
      d->it[s] = placeholder(top);
      e = s;
    } else {
      int total = 0;
      for (uint32_t i = s; i <= e; i++) total += !d->it[i].cont;
      int cc = total / (MAX_NODES / 2) < MAX_NODES - 1 ? total / (MAX_NODES / 2) : MAX_NODES - 1;
      if (cc < 1) cc = 1;
      const int base = total / cc;
      int rem = total % cc, left = 0, blk = 0;
      for (uint32_t i = s; i <= e; i++) {
        if (d->it[i].cont) continue;
        if (left == 0) {
          left = base + (rem > 0 ? 1 : 0);
          if (rem > 0) rem--;
          d->it[i].h = blk == 0 ? top : 1;
          d->it[i].ns = NS_UNDEF;
          blk++;
        }
        left--;
      }
    }
  } else {
    /* level p >= 3: the level-(p-2) blocks regrouped under new level-(p-1) blocks */
    int total = 0;
    for (uint32_t i = s; i <= e; i++) total += d->it[i].h >= p - 2;
    int cc = total / (MAX_NODES / 2) < MAX_NODES - 1 ? total / (MAX_NODES / 2) : MAX_NODES - 1;
    if (cc < 1) cc = 1;
    const int base = total / cc;
    int rem = total % cc, left = 0, blk = 0;
    for (uint32_t i = s; i <= e; i++) {
      if (d->it[i].h < p - 2) continue;
      if (left == 0) {
        left = base + (rem > 0 ? 1 : 0);
        if (rem > 0) rem--;
        d->it[i].h = (uint8_t)(blk == 0 ? top : p - 1);
        blk++;
      } else {
        d->it[i].h = (uint8_t)(p - 2);
      }
      left--;
    }
  }
  /* the parent's own child count: underflow -> its parent re-packs too */
  if (p < d->depth) {
    const int cc = children(d, s, span_end(d, s, p), p);
    if (cc < MAX_NODES / 2) pack_parent(d, span_start(d, s, p + 1), p + 1, arena, n_keys);
  }
}

/* zamboniSegments (mergeTree.ts:800-838) */
static void zamboni(idoc* d, const uint16_t* arena, uint32_t n_keys) {
  for (int z = 0; z < ZAMBONI_MAX; z++) {
    if (d->hn == 0 || d->heap[1].max_seq > d->min_seq) break;
    const hent e = heap_get(d);
    uint32_t i = 0;
    while (i < d->n && !(d->it[i].id == e.id && !d->it[i].cont && !d->it[i].empty)) i++;
    if (i == d->n) continue; /* unlinked: parent undefined */
    const uint32_t bs = span_start(d, i, 1), be = span_end(d, bs, 1);
    if (d->it[bs].ns == NS_FALSE) continue;
    const int before = children(d, bs, be, 1);
    const int held = scour(d, bs, be, arena, n_keys);
    d->it[bs].ns = NS_FALSE;
    if (held < before) {
      drop_keep_starts(d, bs, be);
      const uint32_t bs2 = bs;
      compact(d);
      if (held < MAX_NODES / 2 && d->depth >= 2) pack_parent(d, span_start(d, bs2, 2), 2, arena, n_keys);
    }
    for (uint32_t j = 0; j < d->n; j++) d->it[j].drop = 0;
  }
}

/* ---- ensureIntervalBoundary ------------------------------------------------------------------ */

static int boundary(idoc* d, int64_t pos) {
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = d->L[i];
    if (l <= 0) continue;
    if (pos < d->P[i]) return MTE_OK;
    if (pos == d->P[i] && d->it[i].cont) { /* between two texts of one merged leaf */
      d->written += 1;
      d->it[i].cont = 0;
      d->it[i].id = new_id(d);
      split_cascade(d, i);
      return MTE_OK;
    }
    if (pos > d->P[i] && pos < d->P[i] + l) {
      const int32_t off = (int32_t)(pos - d->P[i]);
      int rc = open_slot(d, i + 1);
      if (rc) return rc;
      memmove(d->L + i + 2, d->L + i + 1, (size_t)(d->n - i - 2) * sizeof(int32_t));
      memmove(d->P + i + 2, d->P + i + 1, (size_t)(d->n - i - 2) * sizeof(int64_t));
      item* hd = &d->it[i];
      item* tl = &d->it[i + 1];
      *tl = *hd;
      tl->len = hd->len - off;
      tl->toff = hd->toff + (uint32_t)off;
      tl->h = 0;
      tl->cont = 0;
      tl->id = new_id(d);
      d->written += 2;
      hd->len = off;
      d->L[i] = off;
      d->L[i + 1] = tl->len;
      d->P[i + 1] = d->P[i] + off;
      split_cascade(d, i + 1);
      return MTE_OK;
    }
  }
  return MTE_OK;
}

/* ---- one op ------------------------------------------------------------------------------------ */

static int check_op_window(const idoc* d, const mte_op* op) {
  if (!(d->cur_seq < op->seq)) return MTE_E_SEQ_ORDER;
  if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
  return MTE_OK;
}

static int doc_apply(idoc* d, const mte_op* op, const env_t* env) {
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  const int32_t r = op->ref_seq, s = op->seq, m = d->min_seq;
  const int c = op->client;
  int rc;
  if (d->n + 4 > env->limit) return MTE_E_CAPACITY;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  d->ops++;
  if (d->n > d->max_segs) d->max_segs = d->n;
  if (op->type != MTE_OP_NOOP) d->scanned += d->n;
  if (op->type == MTE_OP_INSERT) {
    if ((rc = reserve(d, d->n + 3))) return rc;
    lengths(d, r, c, m, newcalc);
    if ((rc = boundary(d, op->pos1))) return rc;
    const int64_t total = lengths(d, r, c, m, newcalc);
    const int is_marker = (op->flags & MTE_F_MARKER) != 0;
    const int32_t len = is_marker ? 1 : op->pos2;
    if (len > 0) {
      const int64_t pos = op->pos1;
      /* the leaf block insertingWalk enters: the first whose end reaches pos */
      uint32_t ks = d->n;
      for (uint32_t i = 0; i < d->n; i++)
        if (d->P[i] + (d->L[i] > 0 ? d->L[i] : 0) >= pos) {
          ks = i;
          break;
        }
      if (ks == d->n || pos > total) return MTE_E_INSERT_FAILED;
      const uint32_t bs = span_start(d, ks, 1), be = span_end(d, bs, 1);
      uint32_t slot;
      int replace = 0;
      if (d->it[bs].empty) {
        slot = bs;
        replace = 1;
      } else {
        slot = be + 1;
        for (uint32_t i = ks; i <= be; i++)
          if (d->L[i] >= 0 && d->P[i] >= pos && !d->it[i].empty) {
            slot = i;
            break;
          }
      }
      item nw;
      memset(&nw, 0, sizeof nw);
      nw.len = len;
      nw.seq = s;
      nw.cli = c;
      nw.rseq = NONE_SEQ;
      nw.id = new_id(d);
      d->written += 1;
      if (is_marker) {
        nw.kind = 1u + (uint32_t)op->pos2;
      } else {
        nw.toff = (uint32_t)(env->text_base + op->a);
        d->units += (uint64_t)len;
      }
      if (op->b != MTE_NO_PROPS) {
        nw.po = 1;
        d->pwrites += orc_apply_props(nw.props, env->n_keys, &env->b->propsets[op->b], env->b->props, 0);
      }
      if (replace) {
        nw.h = d->it[slot].h;
        nw.ns = d->it[slot].ns;
        d->it[slot] = nw;
      } else {
        if ((rc = open_slot(d, slot))) return rc;
        if (slot == bs) { /* the new leaf becomes the block's first child */
          nw.h = d->it[slot + 1].h;
          nw.ns = d->it[slot + 1].ns;
          d->it[slot + 1].h = 0;
        }
        d->it[slot] = nw;
        split_cascade(d, slot);
      }
      if ((rc = add_lru(d, slot, s))) return rc;
    }
    zamboni(d, env->arena, env->n_keys);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_REMOVE || op->type == MTE_OP_ANNOTATE) {
    const int64_t start = op->pos1, end = op->pos2;
    if ((rc = reserve(d, d->n + 3))) return rc;
    lengths(d, r, c, m, newcalc);
    if ((rc = boundary(d, start))) return rc;
    lengths(d, r, c, m, newcalc);
    if ((rc = boundary(d, end))) return rc;
    if (end != start) {
      lengths(d, r, c, m, newcalc);
      for (uint32_t i = 0; i < d->n; i++) {
        const int32_t l = d->L[i];
        if (l <= 0) continue;
        if (d->P[i] >= end) break;
        if (d->P[i] + l <= start) continue;
        item* g = &d->it[i];
        d->written += 1;
        if (op->type == MTE_OP_REMOVE) {
          if (g->rseq == NONE_SEQ) {
            g->rseq = s;
            g->rmask = 1u << c;
          } else {
            g->rmask |= 1u << c;
          }
        } else {
          g->po = 1;
          d->pwrites += orc_apply_props(g->props, env->n_keys, &env->b->propsets[op->a], env->b->props,
                                        (op->flags & MTE_F_REWRITE) != 0);
        }
        if (!g->cont && (rc = add_lru(d, i, s))) return rc;
      }
    }
    zamboni(d, env->arena, env->n_keys);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }
  if (op->flags & MTE_F_MSG_END) {
    if (!(d->cur_seq <= s)) return MTE_E_SEQ_ORDER;
    d->cur_seq = s;
    if (!(op->min_seq <= s)) return MTE_E_MSN_GT_SEQ;
    if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
    if (op->min_seq > d->min_seq) {
      d->min_seq = op->min_seq;
      zamboni(d, env->arena, env->n_keys);
    }
  }
  return MTE_OK;
}

/* ---- API ------------------------------------------------------------------------------------------ */

static int arena_append(oti_ctx* c, const uint16_t* t, uint64_t n, uint64_t* base) {
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

int oti_create(uint32_t n_keys, oti_ctx** out) {
  if (!out || n_keys > MTE_MAX_KEYS) return MTE_E_INVALID_ARG;
  oti_ctx* c = (oti_ctx*)calloc(1, sizeof(oti_ctx));
  if (!c) return MTE_E_OOM;
  c->n_keys = n_keys;
  c->limit = 1024;
  *out = c;
  return MTE_OK;
}

static void free_docs(oti_ctx* c) {
  for (uint32_t i = 0; i < c->n_docs; i++) {
    free(c->docs[i].it);
    free(c->docs[i].heap);
    free(c->docs[i].L);
    free(c->docs[i].P);
  }
  free(c->docs);
  free(c->load_ps);
  free(c->load_pe);
  c->docs = NULL;
  c->load_ps = NULL;
  c->load_pe = NULL;
  c->n_docs = 0;
}

int oti_destroy(oti_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  free_docs(c);
  free(c->arena);
  free(c);
  return MTE_OK;
}

int oti_load_docs(oti_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text, uint64_t text_units,
                  const mte_propset* propsets, uint32_t n_propsets, const mte_prop* props, uint32_t n_props) {
  if (!c || (n_docs && !docs)) return MTE_E_INVALID_ARG;
  free_docs(c);
  c->arena_n = 0;
  uint64_t base = 0;
  int rc = arena_append(c, text, text_units, &base);
  if (rc) return rc;
  c->load_units = text_units;
  c->docs = (idoc*)aligned_alloc(128, (size_t)(n_docs ? n_docs : 1) * sizeof(idoc));
  if (!c->docs) return MTE_E_OOM;
  memset(c->docs, 0, (size_t)(n_docs ? n_docs : 1) * sizeof(idoc));
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
    idoc* d = &c->docs[i];
    const mte_doc_init* in = &docs[i];
    if ((uint64_t)in->text_off + in->text_len > text_units) return MTE_E_INVALID_ARG;
    d->init = *in;
    d->flags = in->flags;
    d->min_seq = in->min_seq;
    d->cur_seq = in->cur_seq;
    d->depth = 1;
    d->next_id = 1;
    if ((rc = reserve(d, 64))) return rc;
    d->n = 1;
    if (in->text_len > 0) {
      item* g = &d->it[0];
      memset(g, 0, sizeof(*g));
      g->len = (int32_t)in->text_len;
      g->cli = -1;
      g->rseq = NONE_SEQ;
      g->toff = (uint32_t)(base + in->text_off);
      g->h = 1;
      g->id = new_id(d);
      if (in->propset != MTE_NO_PROPS) {
        if (in->propset >= n_propsets) return MTE_E_INVALID_ARG;
        g->po = 1;
        orc_apply_props(g->props, c->n_keys, &propsets[in->propset], props, 0);
      }
    } else {
      d->it[0] = placeholder(1);
    }
  }
  return MTE_OK;
}

/* reloadFromSegments (mergeTree.ts:607-652): blocks of 7 children per level */
int oti_load_segments(oti_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs) {
  if (!c || !seg_offsets || (n_segs && !segs)) return MTE_E_INVALID_ARG;
  if (seg_offsets[0] != 0 || seg_offsets[c->n_docs] != n_segs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < c->n_docs; di++) {
    const uint64_t b = seg_offsets[di], e = seg_offsets[di + 1];
    if (e < b) return MTE_E_INVALID_ARG;
    if (e == b) continue;
    idoc* d = &c->docs[di];
    const uint32_t n = (uint32_t)(e - b);
    int rc = reserve(d, n + 64);
    if (rc) return rc;
    int depth = 1;
    for (uint64_t w = 7; w < n; w *= 7) depth++;
    d->depth = depth;
    for (uint32_t k = 0; k < n; k++) {
      const mte_seg* sg = &segs[b + k];
      const int marker = sg->kind != 0;
      if ((marker && sg->len != 1) || (!marker && (sg->len == 0 || (uint64_t)sg->text_off + sg->len > c->load_units)) ||
          sg->client < -1 || sg->client >= MTE_MAX_CLIENTS || sg->seq < 0 ||
          (sg->removed_seq != MTE_NOT_REMOVED && sg->removers == 0))
        return MTE_E_INVALID_ARG;
      item* g = &d->it[k];
      memset(g, 0, sizeof(*g));
      g->len = (int32_t)sg->len;
      g->seq = sg->seq;
      g->cli = sg->client;
      g->rseq = sg->removed_seq == MTE_NOT_REMOVED ? NONE_SEQ : sg->removed_seq;
      g->rmask = sg->removed_seq == MTE_NOT_REMOVED ? 0u : sg->removers;
      g->kind = sg->kind;
      g->toff = marker ? 0u : sg->text_off;
      g->id = new_id(d);
      uint64_t w = 7;
      int h = 0;
      if (k == 0) h = depth;
      else
        for (int lv = 1; lv < depth && k % w == 0; lv++, w *= 7) h = lv;
      g->h = (uint8_t)h;
      if (sg->propset != MTE_NO_PROPS) {
        if (sg->propset >= c->n_load_ps) return MTE_E_INVALID_ARG;
        g->po = 1;
        orc_apply_props(g->props, c->n_keys, &c->load_ps[sg->propset], c->load_pe, 0);
      }
    }
    d->n = n;
  }
  return MTE_OK;
}

typedef struct {
  oti_ctx* c;
  const mte_batch* b;
  uint64_t base;
  uint32_t d0, d1, stride;
} worker_arg;

static void* worker(void* p) {
  worker_arg* w = (worker_arg*)p;
  env_t env = {w->b, w->base, w->c->n_keys, w->c->arena, w->c->limit};
  for (uint32_t di = w->d0; di < w->d1; di += w->stride) {
    idoc* d = &w->c->docs[di];
    if (d->status) continue;
    for (uint64_t k = w->b->op_offsets[di]; k < w->b->op_offsets[di + 1]; k++) {
      int rc = doc_apply(d, &w->b->ops[k], &env);
      if (rc) {
        d->status = rc;
        break;
      }
    }
  }
  return NULL;
}

int oti_apply_batch(oti_ctx* c, const mte_batch* b, int n_threads) {
  if (!c || !b || b->n_docs != c->n_docs || !b->op_offsets) return MTE_E_INVALID_ARG;
  if (b->op_offsets[b->n_docs] != b->n_ops) return MTE_E_INVALID_ARG;
  uint64_t base = 0;
  int rc = arena_append(c, b->text, b->text_units, &base);
  if (rc) return rc;
  for (uint32_t i = 0; i < c->n_docs; i++) {
    idoc* d = &c->docs[i];
    d->ops = d->scanned = d->written = d->pwrites = d->units = d->max_segs = 0;
  }
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
  if (n_threads == 1) worker(&args[0]);
  else {
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, worker, &args[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  }
  free(args);
  free(th);
  return MTE_OK;
}

int oti_read_doc(oti_ctx* c, uint32_t doc, mte_doc_view* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  idoc* d = &c->docs[doc];
  v->status = d->status;
  v->cur_seq = d->cur_seq;
  v->min_seq = d->min_seq;
  uint32_t length = 0, nt = 0, ns = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const item* g = &d->it[i];
    if (g->rseq != NONE_SEQ) continue;
    /* a merged leaf reads as one segment */
    if (g->cont && ns > 0) {
      if (ns - 1 < v->seg_cap && v->seg_len) v->seg_len[ns - 1] += (uint32_t)g->len;
    } else {
      if (ns < v->seg_cap) {
        if (v->seg_len) v->seg_len[ns] = (uint32_t)g->len;
        if (v->seg_kind) v->seg_kind[ns] = g->kind;
        if (v->seg_props)
          for (uint32_t k = 0; k < c->n_keys; k++) v->seg_props[(size_t)ns * c->n_keys + k] = g->props[k];
      }
      ns++;
    }
    length += (uint32_t)g->len;
    if (g->kind == 0)
      for (int32_t u = 0; u < g->len; u++, nt++)
        if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
  }
  v->length = length;
  v->n_text = nt;
  v->n_segs = ns;
  return MTE_OK;
}

int oti_digest(oti_ctx* c, uint64_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < n_docs; di++) {
    idoc* d = &c->docs[di];
    orc_digest_acc acc = {0, 0, 0, 0};
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (g->rseq != NONE_SEQ) continue;
      orc_digest_seg(&acc, g->kind, g->kind == 0 ? c->arena + g->toff : NULL, g->len, g->props, c->n_keys);
    }
    out[4 * (size_t)di + 0] = acc.n;
    out[4 * (size_t)di + 1] = acc.h1;
    out[4 * (size_t)di + 2] = acc.h2;
    out[4 * (size_t)di + 3] = acc.sum;
  }
  return MTE_OK;
}

int oti_doc_status(oti_ctx* c, int32_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < n_docs; i++) out[i] = c->docs[i].status;
  return MTE_OK;
}

int oti_doc_nsegs(oti_ctx* c, uint32_t doc, uint32_t* out) {
  if (!c || !out || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  uint32_t k = 0;
  const idoc* d = &c->docs[doc];
  for (uint32_t i = 0; i < d->n; i++) k += !d->it[i].cont && !d->it[i].empty;
  *out = k;
  return MTE_OK;
}

/* the same shape string as ort_doc_shape, from the block levels */
int oti_doc_shape(oti_ctx* c, uint32_t doc, char* buf, uint32_t cap) {
  if (!c || !buf || !cap || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const idoc* d = &c->docs[doc];
  uint32_t k = 0;
#define PUT(ch) \
  do {          \
    if (k + 1 < cap) buf[k++] = (ch); \
  } while (0)
  for (uint32_t i = 0; i < d->n;) {
    const item* g = &d->it[i];
    if (i > 0) {
      /* close the blocks that end before item i, open the ones it starts */
      for (int lv = 0; lv < g->h; lv++) PUT(']');
      if (g->h > 0) PUT(' ');
      else PUT(' ');
    }
    for (int lv = 0; lv < g->h; lv++) PUT('[');
    if (!g->empty) {
      const uint32_t e = leaf_end(d, i);
      char tmp[32];
      int m = snprintf(tmp, sizeof tmp, "%lld%s", (long long)leaf_total(d, i, e), g->rseq != NONE_SEQ ? "r" : "");
      for (int q = 0; q < m; q++) PUT(tmp[q]);
      i = e;
    } else {
      i++;
    }
  }
  for (int lv = 0; lv < d->depth; lv++) PUT(']');
  buf[k] = 0;
#undef PUT
  return (int)d->hn;
}

int oti_stats_get(oti_ctx* c, mte_stats* o) {
  if (!c || !o) return MTE_E_INVALID_ARG;
  memset(o, 0, sizeof(*o));
  for (uint32_t i = 0; i < c->n_docs; i++) {
    const idoc* d = &c->docs[i];
    o->ops_applied += d->ops;
    o->segs_scanned += d->scanned;
    o->segs_written += d->written;
    o->prop_writes += d->pwrites;
    o->units_inserted += d->units;
    if (d->max_segs > o->max_segs) o->max_segs = d->max_segs;
  }
  o->algo_bytes = 32.0 * (double)o->ops_applied + 20.0 * (double)o->segs_scanned +
                  20.0 * (double)o->segs_written + 4.0 * (double)o->prop_writes +
                  2.0 * (double)o->units_inserted;
  return MTE_OK;
}

/* every item a document holds, placeholders skipped and merged leaves joined
 * (as mte_read_segments) */
int oti_read_segments(oti_ctx* c, uint32_t doc, mte_seg_list* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const idoc* d = &c->docs[doc];
  uint64_t nt = 0, m = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const item* g = &d->it[i];
    if (g->empty) continue;
    if (g->cont && m > 0) {
      if (m - 1 < v->seg_cap && v->segs) v->segs[m - 1].len += (uint32_t)g->len;
    } else {
      const uint64_t io = m++;
      if (io < v->seg_cap && v->segs) {
        mte_seg* s = &v->segs[io];
        s->text_off = g->kind == 0 ? (uint32_t)nt : 0u;
        s->len = (uint32_t)g->len;
        s->seq = g->seq;
        s->removed_seq = g->rseq == NONE_SEQ ? MTE_NOT_REMOVED : g->rseq;
        s->removers = g->rseq == NONE_SEQ ? 0u : g->rmask;
        s->client = g->cli;
        s->kind = g->kind;
        s->propset = MTE_NO_PROPS;
        if (v->props)
          for (uint32_t k = 0; k < c->n_keys; k++) v->props[(size_t)io * c->n_keys + k] = g->props[k];
      }
    }
    if (g->kind == 0)
      for (int32_t u = 0; u < g->len; u++, nt++)
        if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
  }
  v->n_segs = m;
  v->n_text = nt;
  return MTE_OK;
}

int oti_set_limit(oti_ctx* c, uint32_t limit) {
  if (!c || limit < 8) return MTE_E_INVALID_ARG;
  c->limit = limit;
  return MTE_OK;
}
