/*
 * tree.c — TREE-EXACT CPU restatement of merge-tree observer replay
 * (TEST INFRASTRUCTURE, the second oracle).
 *
 * oracle.c restates the replay on a flat segment array.  That is exact for
 * everything a document shows, except where the reference's *B+tree shape*
 * decides an insert's place relative to tombstones (VERDICT r1
 * Weak #1): insertingWalk enters the first block whose perspective length
 * reaches the insert position and appends at that block's end
 * (mergeTree.ts:1743, 1788-1797), so a new segment lands *before* tombstones
 * that start the next block, where the flat rule puts it after them.  With the
 * legacy length calculation such a tombstone can be visible again to a later
 * op whose refSeq lies before its removal, and the text then differs.
 *
 * This file therefore keeps the reference's tree itself — blocks of up to
 * MaxNodesInBlock = 8 children (mergeTreeNodes.ts:373), split 4 + 4 when a
 * block fills (mergeTree.ts:1808-1821, 1827-1840), the root replaced on a
 * split (1263-1272) — and the lazy zamboni that shapes it: the LRU heap of
 * segments to scour (665-675, collections/heap.ts), at most two scours per
 * call (466, 800-838) after every sequenced insert / remove / annotate
 * (1418-1421, 1995-1999, 1901-1905) and every minSeq advance (1077-1093),
 * scourNode's unlinking and append-merging (681-747, textSegment.ts:72-87,
 * properties.ts:66-100) and packParent's re-packing (750-798).  Lengths are
 * recomputed by brute force over the leaves (what PartialSequenceLengths
 * caches: partialLengths.ts:667-702 == the leaf sum, test/testUtils.ts:173-248).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 */
#include <limits.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"
#include "tree.h"

#define NONE_SEQ ORC_NONE_SEQ
#define MAX_NODES 8          /* MaxNodesInBlock, mergeTreeNodes.ts:373       */
#define TEXT_GRANULARITY 256 /* TextSegmentGranularity, textSegment.ts:19   */
#define ZAMBONI_MAX 2        /* zamboniSegmentsMaxCount, mergeTree.ts:466   */

typedef struct tnode {
  struct tnode* parent;
  int32_t leaf;
  /* block */
  int32_t cc;
  struct tnode* ch[MAX_NODES];
  int32_t scour; /* needsScour: -1 undefined, 0 false, 1 true (mergeTreeNodes.ts:98) */
  /* leaf */
  int32_t len, seq, rseq;
  uint32_t rmask;
  int32_t cli;
  uint32_t kind;
  int32_t po; /* segment.properties is an object (undefined vs {}: matchProperties) */
  uint16_t* text;
  uint32_t props[MTE_MAX_KEYS];
  int32_t hrefs; /* heap entries pointing here */
  int32_t dead;  /* unlinked (parent = undefined) */
} tnode;

typedef struct {
  int32_t max_seq;
  tnode* seg;
} lru_ent;

typedef struct {
  tnode* root;
  int32_t min_seq, cur_seq;
  uint32_t flags;
  int32_t status;
  lru_ent* heap; /* heap[0] = comparer min; heap[1 .. hn] (collections/heap.ts) */
  uint32_t hn, hcap;
  tnode** flat; /* scratch: leaves in order */
  int32_t* L;
  int64_t* P;
  uint32_t flat_cap;
  uint64_t ops;
  uint64_t n_push, n_pop, n_scour, n_split, n_pack, n_merge;  /* structure counters (tests, tuning) */
  mte_doc_init init;
} __attribute__((aligned(128))) tdoc;

struct ort_ctx {
  uint32_t n_keys;
  uint32_t n_docs;
  tdoc* docs;
  uint16_t* load_text;
  uint64_t load_units;
  mte_propset* load_ps;
  uint32_t n_load_ps;
  mte_prop* load_pe;
  uint32_t n_load_pe;
};

/* ---- nodes ---------------------------------------------------------------- */

static tnode* make_block(void) {
  tnode* b = (tnode*)calloc(1, sizeof(tnode));
  if (b) b->scour = -1;
  return b;
}

static tnode* make_leaf(void) {
  tnode* l = (tnode*)calloc(1, sizeof(tnode));
  if (l) {
    l->leaf = 1;
    l->rseq = NONE_SEQ;
  }
  return l;
}

static void free_leaf(tnode* l) {
  free(l->text);
  free(l);
}

/* a leaf leaves the tree (scourNode unlink / append, mergeTree.ts:705, 727);
 * it lives on while the LRU heap still points at it */
static void unlink_leaf(tnode* l) {
  l->parent = NULL;
  l->dead = 1;
  if (l->hrefs == 0) free_leaf(l);
}

static void free_tree(tnode* n) {
  if (!n) return;
  if (n->leaf) {
    if (n->hrefs == 0) free_leaf(n);
    else {
      n->parent = NULL;
      n->dead = 1;
    }
    return;
  }
  for (int i = 0; i < n->cc; i++) free_tree(n->ch[i]);
  free(n);
}

static void assign_child(tnode* b, tnode* c, int i) {
  c->parent = b;
  b->ch[i] = c;
}

/* ---- lengths -------------------------------------------------------------- */

/* nodeLength of a leaf for a remote perspective (mergeTree.ts:1003-1054);
 * -1 = undefined.  Same rule as oracle.c leaf_len. */
static inline int32_t leaf_len(const tnode* s, int32_t r, int c, int32_t m, int newcalc) {
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

typedef struct {
  int32_t r, m;
  int c, newcalc;
} persp;

/* nodeLength of a block: partialLengths.getPartialLength, i.e. the sum of the
 * defined leaf lengths below it */
static int64_t block_len(const tnode* b, const persp* v) {
  int64_t s = 0;
  for (int i = 0; i < b->cc; i++) {
    const tnode* x = b->ch[i];
    if (x->leaf) {
      int32_t l = leaf_len(x, v->r, v->c, v->m, v->newcalc);
      if (l > 0) s += l;
    } else {
      s += block_len(x, v);
    }
  }
  return s;
}

static int64_t node_len(const tnode* x, const persp* v) {
  return x->leaf ? (int64_t)leaf_len(x, v->r, v->c, v->m, v->newcalc) : block_len(x, v);
}

/* ---- insertingWalk --------------------------------------------------------- */

/* split(node), mergeTree.ts:1827-1840: the upper half moves to a new block */
static tnode* split_block(tnode* b) {
  tnode* nb = make_block();
  if (!nb) return NULL;
  const int half = MAX_NODES / 2;
  for (int i = 0; i < half; i++) {
    assign_child(nb, b->ch[half + i], i);
    b->ch[half + i] = NULL;
  }
  nb->cc = half;
  b->cc = half;
  return nb;
}

/* BaseSegment.splitAt / TextSegment.createSplitSegmentAt
 * (mergeTreeNodes.ts:505-547, textSegment.ts:105-113) */
static tnode* split_leaf(tnode* s, int32_t off) {
  tnode* t = make_leaf();
  if (!t) return NULL;
  *t = *s;
  t->parent = s->parent;
  t->hrefs = 0;
  t->dead = 0;
  t->len = s->len - off;
  t->text = (uint16_t*)malloc((size_t)(t->len > 0 ? t->len : 1) * sizeof(uint16_t));
  if (!t->text) {
    free(t);
    return NULL;
  }
  memcpy(t->text, s->text + off, (size_t)t->len * sizeof(uint16_t));
  s->len = off;
  return t;
}

enum { WALK_SPLIT = 0, WALK_INSERT = 1 };

typedef struct {
  int mode;      /* WALK_SPLIT: ensureIntervalBoundary; WALK_INSERT: blockInsert */
  int32_t seq;   /* TreeMaintenanceSequenceNumber (-2) or the op's seq */
  tnode* cand;   /* the new segment (insert) */
  int oom;
  uint64_t* counter; /* block splits */
} walk_ctx;

/* breakTie (mergeTree.ts:1705-1721), called only when pos == len */
static int break_tie(int64_t pos, const tnode* node, int32_t seq) {
  if (node->leaf) {
    if (pos == 0) return seq > node->seq; /* sequenced: no Unassigned normalisation */
    return 0;
  }
  return 1;
}

/* insertingWalk (mergeTree.ts:1723-1825); returns the new sibling of `block`
 * when it split, else NULL.  continuePredicate (1790-1793) asks whether the
 * segment after the block is a local unacked one: never, for an observer. */
static tnode* inserting_walk(tnode* block, int64_t pos, const persp* v, walk_ctx* w) {
  int64_t p = pos;
  int ci;
  tnode* nn = NULL;
  for (ci = 0; ci < block->cc; ci++) {
    tnode* child = block->ch[ci];
    const int64_t len = node_len(child, v);
    if (len < 0) continue; /* undefined leaf: skipped (1735-1738) */
    if (p < len || (p == len && break_tie(p, child, w->seq))) {
      if (!child->leaf) {
        tnode* sp = inserting_walk(child, p, v, w);
        if (!sp) return NULL;
        nn = sp;
        ci++;
      } else if (w->mode == WALK_SPLIT) {
        /* splitLeafSegment (1681-1696) */
        if (!(p > 0)) return NULL;
        nn = split_leaf(child, (int32_t)p);
        if (!nn) {
          w->oom = 1;
          return NULL;
        }
        ci++;
      } else {
        /* blockInsert onLeaf (1629-1639): the new segment takes the child's
         * index, the child moves after it */
        assign_child(block, w->cand, ci);
        nn = child;
        ci++;
      }
      break;
    }
    p -= len;
  }
  if (!nn && p == 0 && w->mode == WALK_INSERT) nn = w->cand; /* append at the block's end */
  if (!nn) return NULL;
  for (int i = block->cc; i > ci; i--) block->ch[i] = block->ch[i - 1];
  assign_child(block, nn, ci);
  block->cc++;
  if (block->cc < MAX_NODES) return NULL;
  tnode* sp = split_block(block);
  if (w->counter) (*w->counter)++;
  if (!sp) w->oom = 1;
  return sp;
}

/* updateRoot (mergeTree.ts:1263-1272) */
static int update_root(tdoc* d, tnode* split) {
  if (!split) return MTE_OK;
  tnode* nr = make_block();
  if (!nr) return MTE_E_OOM;
  assign_child(nr, d->root, 0);
  assign_child(nr, split, 1);
  nr->cc = 2;
  d->root = nr;
  return MTE_OK;
}

/* ensureIntervalBoundary (mergeTree.ts:1698-1702) */
static int ensure_boundary(tdoc* d, int64_t pos, const persp* v) {
  walk_ctx w = {WALK_SPLIT, -2, NULL, 0, &d->n_split};
  tnode* sp = inserting_walk(d->root, pos, v, &w);
  if (w.oom) return MTE_E_OOM;
  return update_root(d, sp);
}

/* ---- LRU heap of segments to scour (collections/heap.ts; LRUSegmentComparer
 * mergeTree.ts:120-123 compares maxSeq) ---------------------------------------- */

static int heap_add(tdoc* d, tnode* seg, int32_t max_seq) {
  if (d->hn + 2 > d->hcap) {
    uint32_t nc = d->hcap ? 2 * d->hcap : 64;
    lru_ent* h = (lru_ent*)realloc(d->heap, (size_t)nc * sizeof(lru_ent));
    if (!h) return MTE_E_OOM;
    d->heap = h;
    d->hcap = nc;
  }
  lru_ent* L = d->heap;
  d->n_push++;
  L[++d->hn] = (lru_ent){max_seq, seg};
  seg->hrefs++;
  for (uint32_t k = d->hn; k > 1 && L[k >> 1].max_seq - L[k].max_seq > 0; k >>= 1) {
    lru_ent t = L[k >> 1];
    L[k >> 1] = L[k];
    L[k] = t;
  }
  return MTE_OK;
}

static lru_ent heap_get(tdoc* d) {
  lru_ent* L = d->heap;
  lru_ent x = L[1];
  L[1] = L[d->hn];
  d->hn--;
  uint32_t k = 1;
  while ((k << 1) <= d->hn) {
    uint32_t j = k << 1;
    if (j < d->hn && L[j].max_seq - L[j + 1].max_seq > 0) j++;
    if (L[k].max_seq - L[j].max_seq <= 0) break;
    lru_ent t = L[k];
    L[k] = L[j];
    L[j] = t;
    k = j;
  }
  return x;
}

/* addToLRUSet (mergeTree.ts:665-675) */
static int add_to_lru(tdoc* d, tnode* seg, int32_t seq) {
  if (seg->parent->scour != 1 && seq > d->cur_seq) {
    seg->parent->scour = 1;
    return heap_add(d, seg, seq);
  }
  return MTE_OK;
}

/* ---- zamboni ---------------------------------------------------------------- */

typedef struct {
  tnode** v;
  int n, cap;
} nodevec;

static int nv_push(nodevec* h, tnode* x) {
  if (h->n == h->cap) {
    int nc = h->cap ? 2 * h->cap : 16;
    tnode** v = (tnode**)realloc(h->v, (size_t)nc * sizeof(tnode*));
    if (!v) return MTE_E_OOM;
    h->v = v;
    h->cap = nc;
  }
  h->v[h->n++] = x;
  return MTE_OK;
}

/* matchProperties (properties.ts:66-100) on interned values: an absent
 * properties object matches only another absent one; two objects match when
 * every key has the same value */
static int match_props(const tnode* a, const tnode* b, uint32_t n_keys) {
  if (a->po != b->po) return 0;
  for (uint32_t k = 0; k < n_keys; k++)
    if (a->props[k] != b->props[k] || (a->props[k] & MTE_VALUE_UNEQUAL)) return 0; /* NaN !== NaN */
  return 1;
}

/* TextSegment.canAppend (textSegment.ts:72-77) */
static int can_append(const tnode* prev, const tnode* seg) {
  if (prev->kind != 0 || seg->kind != 0) return 0; /* markers never append */
  if (prev->len > 0 && prev->text[prev->len - 1] == (uint16_t)'\n') return 0;
  return prev->len <= TEXT_GRANULARITY || seg->len <= TEXT_GRANULARITY;
}

/* scourNode (mergeTree.ts:681-747) */
static int scour_node(tdoc* d, tnode* node, nodevec* hold, uint32_t n_keys) {
  tnode* prev = NULL;
  int rc;
  for (int k = 0; k < node->cc; k++) {
    tnode* x = node->ch[k];
    if (!x->leaf) {
      if ((rc = nv_push(hold, x))) return rc;
      prev = NULL;
      continue;
    }
    if (x->rseq != NONE_SEQ) {
      if (x->rseq > d->min_seq) {
        if ((rc = nv_push(hold, x))) return rc;
      } else {
        unlink_leaf(x);
      }
      prev = NULL;
    } else if (x->seq <= d->min_seq) {
      /* localNetLength of a segment not removed is its length (> 0) */
      if (prev && can_append(prev, x) && match_props(prev, x, n_keys) && x->len > 0) {
        /* TextSegment.append (textSegment.ts:83-87, mergeTreeNodes.ts:551-563) */
        uint16_t* t = (uint16_t*)realloc(prev->text, (size_t)(prev->len + x->len) * sizeof(uint16_t));
        if (!t) return MTE_E_OOM;
        memcpy(t + prev->len, x->text, (size_t)x->len * sizeof(uint16_t));
        prev->text = t;
        prev->len += x->len;
        d->n_merge++;
        unlink_leaf(x);
      } else {
        if ((rc = nv_push(hold, x))) return rc;
        prev = x->len > 0 ? x : NULL;
      }
    } else {
      if ((rc = nv_push(hold, x))) return rc;
      prev = NULL;
    }
  }
  return MTE_OK;
}

/* packParent (mergeTree.ts:750-798) */
static int pack_parent(tdoc* d, tnode* parent, uint32_t n_keys) {
  nodevec hold = {NULL, 0, 0};
  d->n_pack++;
  int rc = MTE_OK;
  for (int i = 0; i < parent->cc; i++) {
    tnode* cb = parent->ch[i];
    if ((rc = scour_node(d, cb, &hold, n_keys))) goto out;
  }
  for (int i = 0; i < parent->cc; i++) free(parent->ch[i]); /* replaced by packed blocks */
  const int total = hold.n;
  const int half = MAX_NODES / 2;
  int count = total / half < MAX_NODES - 1 ? total / half : MAX_NODES - 1;
  if (count < 1) count = 1;
  const int base = total / count;
  int rem = total % count;
  int packed = 0;
  for (int b = 0; b < count; b++) {
    int n = base;
    if (rem > 0) {
      n++;
      rem--;
    }
    tnode* pb = make_block();
    if (!pb) {
      rc = MTE_E_OOM;
      goto out;
    }
    for (int j = 0; j < n; j++) assign_child(pb, hold.v[packed++], j);
    pb->cc = n;
    assign_child(parent, pb, b);
  }
  for (int b = count; b < MAX_NODES; b++) parent->ch[b] = NULL;
  parent->cc = count;
  if (parent->cc < MAX_NODES / 2 && parent->parent) rc = pack_parent(d, parent->parent, n_keys);
out:
  free(hold.v);
  return rc;
}

/* zamboniSegments (mergeTree.ts:800-838) */
static int zamboni(tdoc* d, uint32_t n_keys) {
  int rc;
  for (int i = 0; i < ZAMBONI_MAX; i++) {
    if (d->hn == 0 || d->heap[1].max_seq > d->min_seq) break;
    lru_ent e = heap_get(d);
    d->n_pop++;
    tnode* seg = e.seg; /* its entry still counts in hrefs: a scour below cannot free it */
    if (seg->parent && seg->parent->scour != 0) {
      tnode* block = seg->parent;
      nodevec hold = {NULL, 0, 0};
      if ((rc = scour_node(d, block, &hold, n_keys))) {
        free(hold.v);
        return rc;
      }
      block->scour = 0;
      d->n_scour++;
      if (hold.n < block->cc) {
        for (int j = 0; j < hold.n; j++) assign_child(block, hold.v[j], j);
        for (int j = hold.n; j < MAX_NODES; j++) block->ch[j] = NULL;
        block->cc = hold.n;
        if (block->cc < MAX_NODES / 2 && block->parent) rc = pack_parent(d, block->parent, n_keys);
        else rc = MTE_OK;
        if (rc) {
          free(hold.v);
          return rc;
        }
      }
      free(hold.v);
    }
    if (--seg->hrefs == 0 && seg->dead) free_leaf(seg);
  }
  return MTE_OK;
}

/* ---- leaves in order -------------------------------------------------------- */

static int flat_reserve(tdoc* d, uint32_t need) {
  if (need <= d->flat_cap) return MTE_OK;
  uint32_t nc = d->flat_cap ? d->flat_cap : 64;
  while (nc < need) nc *= 2;
  tnode** f = (tnode**)realloc(d->flat, (size_t)nc * sizeof(tnode*));
  if (!f) return MTE_E_OOM;
  d->flat = f;
  int32_t* L = (int32_t*)realloc(d->L, (size_t)nc * sizeof(int32_t));
  if (!L) return MTE_E_OOM;
  d->L = L;
  int64_t* P = (int64_t*)realloc(d->P, (size_t)nc * sizeof(int64_t));
  if (!P) return MTE_E_OOM;
  d->P = P;
  d->flat_cap = nc;
  return MTE_OK;
}

static uint32_t count_leaves(const tnode* n) {
  if (n->leaf) return 1;
  uint32_t s = 0;
  for (int i = 0; i < n->cc; i++) s += count_leaves(n->ch[i]);
  return s;
}

static void collect(tnode* n, tnode** out, uint32_t* k) {
  if (n->leaf) {
    out[(*k)++] = n;
    return;
  }
  for (int i = 0; i < n->cc; i++) collect(n->ch[i], out, k);
}

/* leaves in document order -> d->flat[0 .. n) */
static int flatten(tdoc* d, uint32_t* n) {
  const uint32_t cnt = count_leaves(d->root);
  int rc = flat_reserve(d, cnt + 1);
  if (rc) return rc;
  *n = 0;
  collect(d->root, d->flat, n);
  return MTE_OK;
}

/* ---- one op record ------------------------------------------------------------ */

typedef struct {
  const mte_batch* b;
  const uint16_t* batch_text;
  uint32_t n_keys;
} apply_env;

static int check_op_window(const tdoc* d, const mte_op* op) {
  if (!(d->cur_seq < op->seq)) return MTE_E_SEQ_ORDER;
  if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
  return MTE_OK;
}

static int doc_apply(tdoc* d, const mte_op* op, const apply_env* env) {
  /* combiningOp incr / consensus: the HBM tree pass's restatement (titems.c) only */
  if (op->flags & MTE_F_COMBINE) return MTE_E_UNSUPPORTED;
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  const int32_t s = op->seq;
  const int c = op->client;
  const persp v = {op->ref_seq, d->min_seq, c, newcalc};
  int rc;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  d->ops++;

  if (op->type == MTE_OP_INSERT) {
    /* applyInsertOp -> insertSegments (client.ts:470-505, mergeTree.ts:1394-1422) */
    if ((rc = ensure_boundary(d, op->pos1, &v))) return rc;
    const int is_marker = (op->flags & MTE_F_MARKER) != 0;
    const int32_t len = is_marker ? 1 : op->pos2;
    if (len > 0) { /* blockInsert skips zero-length segments (1645) */
      tnode* ns = make_leaf();
      if (!ns) return MTE_E_OOM;
      ns->len = len;
      ns->seq = s;
      ns->cli = c;
      if (is_marker) {
        ns->kind = 1u + (uint32_t)op->pos2;
      } else {
        ns->text = (uint16_t*)malloc((size_t)len * sizeof(uint16_t));
        if (!ns->text) {
          free(ns);
          return MTE_E_OOM;
        }
        memcpy(ns->text, env->batch_text + op->a, (size_t)len * sizeof(uint16_t));
      }
      if (op->b != MTE_NO_PROPS) {
        /* TextSegment.make / Marker.make: props given -> addProperties */
        ns->po = 1;
        orc_apply_props(ns->props, env->n_keys, &env->b->propsets[op->b], env->b->props, 0);
      }
      walk_ctx w = {WALK_INSERT, s, ns, 0, &d->n_split};
      tnode* sp = inserting_walk(d->root, op->pos1, &v, &w);
      if (w.oom) return MTE_E_OOM;
      if (!ns->parent) { /* "MergeTree insert failed" (1666-1672) */
        free_leaf(ns);
        return MTE_E_INSERT_FAILED;
      }
      if ((rc = update_root(d, sp))) return rc;
      /* saveIfLocal (1614-1628) */
      if (ns->seq > d->min_seq && (rc = add_to_lru(d, ns, ns->seq))) return rc;
    }
    if ((rc = zamboni(d, env->n_keys))) return rc;
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_REMOVE || op->type == MTE_OP_ANNOTATE) {
    /* markRangeRemoved (1908-2000) / annotateRange (1864-1906): the two
     * ensureIntervalBoundary calls in the reference's order, then nodeMap
     * (2274-2330) over the leaves with length > 0 overlapping [start, end) */
    const int64_t start = op->pos1, end = op->pos2;
    if ((rc = ensure_boundary(d, start, &v))) return rc;
    if ((rc = ensure_boundary(d, end, &v))) return rc;
    if (end != start) {
      uint32_t n = 0;
      if ((rc = flatten(d, &n))) return rc;
      int64_t p = 0;
      for (uint32_t i = 0; i < n; i++) {
        tnode* g = d->flat[i];
        const int32_t l = leaf_len(g, v.r, v.c, v.m, v.newcalc);
        if (l <= 0) continue;
        if (p >= end) break;
        if (p + l > start) {
          if (op->type == MTE_OP_REMOVE) {
            /* markRemoved (1924-1962) */
            if (g->rseq == NONE_SEQ) {
              g->rseq = s;
              g->rmask = 1u << c;
            } else {
              g->rmask |= 1u << c;
            }
          } else {
            /* annotateSegment -> BaseSegment.addProperties (mergeTreeNodes.ts:426-442) */
            g->po = 1;
            orc_apply_props(g->props, env->n_keys, &env->b->propsets[op->a], env->b->props,
                            (op->flags & MTE_F_REWRITE) != 0);
          }
          if ((rc = add_to_lru(d, g, s))) return rc;
        }
        p += l;
      }
    }
    if ((rc = zamboni(d, env->n_keys))) return rc;
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }

  if (op->flags & MTE_F_MSG_END) {
    /* updateSeqNumbers (client.ts:937-945) -> setMinSeq (mergeTree.ts:1077-1093) */
    if (!(d->cur_seq <= s)) return MTE_E_SEQ_ORDER;
    d->cur_seq = s;
    if (!(op->min_seq <= s)) return MTE_E_MSN_GT_SEQ;
    if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
    if (op->min_seq > d->min_seq) {
      d->min_seq = op->min_seq;
      if ((rc = zamboni(d, env->n_keys))) return rc;
    }
  }
  return MTE_OK;
}

/* ---- API -------------------------------------------------------------------- */

int ort_create(uint32_t n_keys, ort_ctx** out) {
  if (!out || n_keys > MTE_MAX_KEYS) return MTE_E_INVALID_ARG;
  ort_ctx* c = (ort_ctx*)calloc(1, sizeof(ort_ctx));
  if (!c) return MTE_E_OOM;
  c->n_keys = n_keys;
  *out = c;
  return MTE_OK;
}

static void free_doc(tdoc* d) {
  /* heap entries first: a dead leaf is freed when its last entry goes */
  for (uint32_t k = 1; k <= d->hn; k++) {
    tnode* s = d->heap[k].seg;
    if (--s->hrefs == 0 && s->dead) free_leaf(s);
  }
  /* live leaves still counted by nothing now */
  if (d->root) {
    uint32_t n = 0;
    if (flatten(d, &n) == MTE_OK)
      for (uint32_t i = 0; i < n; i++) d->flat[i]->hrefs = 0;
  }
  free_tree(d->root);
  free(d->heap);
  free(d->flat);
  free(d->L);
  free(d->P);
  memset(d, 0, sizeof(*d));
}

static void free_docs(ort_ctx* c) {
  for (uint32_t i = 0; i < c->n_docs; i++) free_doc(&c->docs[i]);
  free(c->docs);
  c->docs = NULL;
  c->n_docs = 0;
  free(c->load_text);
  free(c->load_ps);
  free(c->load_pe);
  c->load_text = NULL;
  c->load_ps = NULL;
  c->load_pe = NULL;
  c->load_units = 0;
  c->n_load_ps = c->n_load_pe = 0;
}

int ort_destroy(ort_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  free_docs(c);
  free(c);
  return MTE_OK;
}

int ort_load_docs(ort_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props) {
  if (!c || (n_docs && !docs)) return MTE_E_INVALID_ARG;
  free_docs(c);
  c->docs = (tdoc*)aligned_alloc(128, (size_t)(n_docs ? n_docs : 1) * sizeof(tdoc));
  if (!c->docs) return MTE_E_OOM;
  memset(c->docs, 0, (size_t)(n_docs ? n_docs : 1) * sizeof(tdoc));
  c->n_docs = n_docs;
  c->load_text = (uint16_t*)malloc((size_t)(text_units ? text_units : 1) * sizeof(uint16_t));
  if (!c->load_text) return MTE_E_OOM;
  if (text_units) memcpy(c->load_text, text, (size_t)text_units * sizeof(uint16_t));
  c->load_units = text_units;
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
    tdoc* d = &c->docs[i];
    const mte_doc_init* in = &docs[i];
    if ((uint64_t)in->text_off + in->text_len > text_units) return MTE_E_INVALID_ARG;
    d->init = *in;
    d->flags = in->flags;
    d->min_seq = in->min_seq;
    d->cur_seq = in->cur_seq;
    d->root = make_block(); /* MergeTree constructor: an empty root (mergeTree.ts:495-498) */
    if (!d->root) return MTE_E_OOM;
    if (in->text_len > 0) {
      /* the harness's insertTextLocal before collaboration
       * (client.replay.spec.ts:22-23): one seq-0 LocalClientId leaf */
      tnode* g = make_leaf();
      if (!g) return MTE_E_OOM;
      g->len = (int32_t)in->text_len;
      g->seq = 0;
      g->cli = -1;
      g->text = (uint16_t*)malloc((size_t)in->text_len * sizeof(uint16_t));
      if (!g->text) return MTE_E_OOM;
      memcpy(g->text, text + in->text_off, (size_t)in->text_len * sizeof(uint16_t));
      if (in->propset != MTE_NO_PROPS) {
        if (in->propset >= n_propsets) return MTE_E_INVALID_ARG;
        g->po = 1;
        orc_apply_props(g->props, c->n_keys, &propsets[in->propset], props, 0);
      }
      assign_child(d->root, g, 0);
      d->root->cc = 1;
    }
  }
  return MTE_OK;
}

/* A summary body loaded as MergeTree.reloadFromSegments does for the header
 * chunk (mergeTree.ts:607-652): blocks of MaxNodesInBlock - 1 nodes per level,
 * bottom up.  (Body chunks beyond the header, appended through insertSegments by
 * SnapshotLoader.loadBody, snapshotLoader.ts:168-240, are not restated here.) */
static tnode* build_level(tnode** nodes, uint32_t n, int* oom) {
  const uint32_t maxc = MAX_NODES - 1;
  const uint32_t nb = (n + maxc - 1) / maxc;
  tnode** blocks = (tnode**)malloc((size_t)(nb ? nb : 1) * sizeof(tnode*));
  if (!blocks) {
    *oom = 1;
    return NULL;
  }
  for (uint32_t b = 0, k = 0; b < nb; b++) {
    tnode* blk = make_block();
    if (!blk) {
      *oom = 1;
      free(blocks);
      return NULL;
    }
    for (uint32_t j = 0; j < maxc && k < n; j++, k++) assign_child(blk, nodes[k], (int)j);
    blk->cc = (int32_t)(n - (uint64_t)b * maxc < maxc ? n - (uint64_t)b * maxc : maxc);
    blocks[b] = blk;
  }
  tnode* r = nb == 1 ? blocks[0] : build_level(blocks, nb, oom);
  free(blocks);
  return r;
}

int ort_load_segments(ort_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs) {
  if (!c || !seg_offsets || (n_segs && !segs)) return MTE_E_INVALID_ARG;
  if (seg_offsets[0] != 0 || seg_offsets[c->n_docs] != n_segs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < c->n_docs; i++) {
    const uint64_t b = seg_offsets[i], e = seg_offsets[i + 1];
    if (e < b) return MTE_E_INVALID_ARG;
    if (e == b) continue;
    tdoc* d = &c->docs[i];
    tnode** leaves = (tnode**)malloc((size_t)(e - b) * sizeof(tnode*));
    if (!leaves) return MTE_E_OOM;
    for (uint64_t k = b; k < e; k++) {
      const mte_seg* sg = &segs[k];
      const int marker = sg->kind != 0;
      if ((marker && sg->len != 1) || (!marker && (sg->len == 0 || (uint64_t)sg->text_off + sg->len > c->load_units)) ||
          sg->client < -1 || sg->client >= MTE_MAX_CLIENTS || sg->seq < 0 ||
          (sg->removed_seq != MTE_NOT_REMOVED && sg->removers == 0)) {
        for (uint64_t q = b; q < k; q++) free_leaf(leaves[q - b]);
        free(leaves);
        return MTE_E_INVALID_ARG;
      }
      tnode* g = make_leaf();
      if (!g) return MTE_E_OOM;
      g->len = (int32_t)sg->len;
      g->seq = sg->seq;
      g->cli = sg->client;
      g->rseq = sg->removed_seq == MTE_NOT_REMOVED ? NONE_SEQ : sg->removed_seq;
      g->rmask = sg->removed_seq == MTE_NOT_REMOVED ? 0u : sg->removers;
      g->kind = sg->kind;
      if (!marker) {
        g->text = (uint16_t*)malloc((size_t)sg->len * sizeof(uint16_t));
        if (!g->text) return MTE_E_OOM;
        memcpy(g->text, c->load_text + sg->text_off, (size_t)sg->len * sizeof(uint16_t));
      }
      if (sg->propset != MTE_NO_PROPS) {
        if (sg->propset >= c->n_load_ps) return MTE_E_INVALID_ARG;
        g->po = 1;
        orc_apply_props(g->props, c->n_keys, &c->load_ps[sg->propset], c->load_pe, 0);
      }
      leaves[k - b] = g;
    }
    int oom = 0;
    tnode* root = build_level(leaves, (uint32_t)(e - b), &oom);
    free(leaves);
    if (oom || !root) return MTE_E_OOM;
    free_tree(d->root);
    d->root = root;
  }
  return MTE_OK;
}

typedef struct {
  ort_ctx* c;
  const mte_batch* b;
  uint32_t d0, d1, stride;
} worker_arg;

static void* worker(void* p) {
  worker_arg* w = (worker_arg*)p;
  apply_env env = {w->b, w->b->text, w->c->n_keys};
  for (uint32_t di = w->d0; di < w->d1; di += w->stride) {
    tdoc* d = &w->c->docs[di];
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

int ort_apply_batch(ort_ctx* c, const mte_batch* b, int n_threads) {
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
  for (uint32_t i = 0; i < c->n_docs; i++) {
    tdoc* d = &c->docs[i];
    d->ops = d->n_push = d->n_pop = d->n_scour = d->n_split = d->n_pack = d->n_merge = 0;
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
  for (int t = 0; t < n_threads; t++) args[t] = (worker_arg){c, b, (uint32_t)t, c->n_docs, (uint32_t)n_threads};
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

int ort_read_doc(ort_ctx* c, uint32_t doc, mte_doc_view* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  tdoc* d = &c->docs[doc];
  v->status = d->status;
  v->cur_seq = d->cur_seq;
  v->min_seq = d->min_seq;
  uint32_t n = 0;
  int rc = flatten(d, &n);
  if (rc) return rc;
  uint32_t length = 0, nt = 0, ns = 0;
  for (uint32_t i = 0; i < n; i++) {
    const tnode* g = d->flat[i];
    if (g->rseq != NONE_SEQ) continue; /* gatherText: removed -> not visible */
    if (ns < v->seg_cap) {
      if (v->seg_len) v->seg_len[ns] = (uint32_t)g->len;
      if (v->seg_kind) v->seg_kind[ns] = g->kind;
      if (v->seg_props)
        for (uint32_t k = 0; k < c->n_keys; k++) v->seg_props[(size_t)ns * c->n_keys + k] = g->props[k];
    }
    ns++;
    length += (uint32_t)g->len;
    if (g->kind == 0) {
      for (int32_t u = 0; u < g->len; u++) {
        if (nt < v->text_cap && v->text) v->text[nt] = g->text[u];
        nt++;
      }
    }
  }
  v->length = length;
  v->n_text = nt;
  v->n_segs = ns;
  return MTE_OK;
}

int ort_read_segments(ort_ctx* c, uint32_t doc, mte_seg_list* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  tdoc* d = &c->docs[doc];
  uint32_t n = 0;
  int rc = flatten(d, &n);
  if (rc) return rc;
  uint64_t nt = 0;
  for (uint32_t i = 0; i < n; i++) {
    const tnode* g = d->flat[i];
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
        for (uint32_t k = 0; k < c->n_keys; k++) v->props[(size_t)i * c->n_keys + k] = g->props[k];
    }
    if (g->kind == 0)
      for (int32_t u = 0; u < g->len; u++, nt++)
        if (nt < v->text_cap && v->text) v->text[nt] = g->text[u];
  }
  v->n_segs = n;
  v->n_text = nt;
  return MTE_OK;
}

int ort_digest(ort_ctx* c, uint64_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < n_docs; di++) {
    tdoc* d = &c->docs[di];
    uint32_t n = 0;
    int rc = flatten(d, &n);
    if (rc) return rc;
    orc_digest_acc acc = {0, 0, 0, 0};
    for (uint32_t i = 0; i < n; i++) {
      const tnode* g = d->flat[i];
      if (g->rseq != NONE_SEQ) continue;
      orc_digest_seg(&acc, g->kind, g->text, g->len, g->props, c->n_keys);
    }
    out[4 * (size_t)di + 0] = acc.n;
    out[4 * (size_t)di + 1] = acc.h1;
    out[4 * (size_t)di + 2] = acc.h2;
    out[4 * (size_t)di + 3] = acc.sum;
  }
  return MTE_OK;
}

int ort_doc_status(ort_ctx* c, int32_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < n_docs; i++) out[i] = c->docs[i].status;
  return MTE_OK;
}

int ort_stats_get(ort_ctx* c, mte_stats* o) {
  if (!c || !o) return MTE_E_INVALID_ARG;
  memset(o, 0, sizeof(*o));
  /* structure counters of the last batch, in the spare fields: segs_scanned =
   * LRU pushes, segs_written = pops, prop_writes = block scours, units_inserted
   * = block splits, max_segs = packParent calls, chunk_scanned = append-merges */
  for (uint32_t i = 0; i < c->n_docs; i++) {
    const tdoc* d = &c->docs[i];
    o->ops_applied += d->ops;
    o->segs_scanned += d->n_push;
    o->segs_written += d->n_pop;
    o->prop_writes += d->n_scour;
    o->units_inserted += d->n_split;
    o->max_segs += d->n_pack;
    o->chunk_scanned += d->n_merge;
  }
  return MTE_OK;
}

int ort_doc_nsegs(ort_ctx* c, uint32_t doc, uint32_t* out) {
  if (!c || !out || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  *out = count_leaves(c->docs[doc].root);
  return MTE_OK;
}

/* The tree's shape as text: blocks in brackets, leaves as their length
 * ("r" marks a removed leaf), e.g. "[[3 1r][2]]".  For tests. */
static void shape_rec(const tnode* n, char* buf, uint32_t cap, uint32_t* k) {
  char tmp[32];
  if (n->leaf) {
    int m = snprintf(tmp, sizeof tmp, "%d%s", n->len, n->rseq != NONE_SEQ ? "r" : "");
    for (int i = 0; i < m; i++)
      if (*k + 1 < cap) buf[(*k)++] = tmp[i];
    return;
  }
  if (*k + 1 < cap) buf[(*k)++] = '[';
  for (int i = 0; i < n->cc; i++) {
    if (i && *k + 1 < cap) buf[(*k)++] = ' ';
    shape_rec(n->ch[i], buf, cap, k);
  }
  if (*k + 1 < cap) buf[(*k)++] = ']';
}

int ort_doc_shape(ort_ctx* c, uint32_t doc, char* buf, uint32_t cap) {
  if (!c || !buf || !cap || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  uint32_t k = 0;
  shape_rec(c->docs[doc].root, buf, cap, &k);
  buf[k] = 0;
  return (int)c->docs[doc].hn; /* heap entries, for tests */
}
