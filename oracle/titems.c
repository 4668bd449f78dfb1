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
 *
 * Documents with a local client (MTE_DOC_LOCAL_CLIENT) run here too, with the
 * flat restatement's local records (oracle.c: local ops, acks, rollback,
 * regeneration, references, delta events) on the tree: the reference places
 * a remote insert next to the client's pending segments by its block edges
 * (continuePredicate's forward excursion, mergeTree.ts:1599-1611, 1788-1797),
 * holds every segment of a pending group in scourNode (:686-688), runs the
 * lazy zamboni after acks and rollbacks (:1329, 2052-2061) and adds acked
 * segments to the LRU set (:1303-1305).  This is the spec of the GPU's HBM
 * tree pass (csrc/mte_htree.h).
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
  uint64_t rmask; /* removedClientIds: short ids < MTE_MAX_CLIENTS_TREE */
  int32_t cli;
  uint32_t kind, toff;
  uint32_t props[MTE_MAX_KEYS];
  uint8_t h, cont, ns, po, empty, drop;
  uint32_t id;
  /* MTE_DOC_LOCAL_CLIENT (as oracle.c's pk rows): per key the localSeq of the
   * last pending local annotate that set it, the mask of the pending annotate
   * segment groups the item belongs to, per key the value before the first
   * pending annotate set it */
  uint32_t pk[MTE_MAX_KEYS];
  uint32_t am;
  uint32_t basev[MTE_MAX_KEYS];
  /* localRemovedSeq: the localSeq of the client's pending removal, kept when
   * a remote remove overtakes it (the segment stays in that removal's group
   * until the ack, mergeTreeNodes.ts:487-497), 0 = none */
  int32_t lrs; /* localRemovedSeq; | LRS_RELEASED once a regeneration dequeued the
                 segment from its group (it keeps the value, the group no longer
                 holds it: resetPendingDeltaToOps, client.ts:802-857) */
  /* the item's place in its pending removal group (SegmentGroup.segments, the
   * order an ack walks them, mergeTree.ts:1285): the doc index at the local
   * remove for the segments it marked, 0x80000000 | the new item's id for a
   * tail split off later (splitAt's segmentGroups.copyTo appends it,
   * mergeTreeNodes.ts:505-534) */
  uint32_t gord;
  /* the first localSeq whose segment group can hold this item as one of the
   * segments its op marked (an item split off later joins the groups before it
   * as a tail, appended: mergeTreeNodes.ts:505-534) */
  uint32_t born;
  /* a regenerated segment's group (resetPendingDeltaToOps gives each re-sent
   * segment one, client.ts:851-854): 1 + the segment's id at its last
   * regeneration, shared by the tails split off it since (MTE_F_REGENERATED) */
  uint32_t rg;
  uint8_t member; /* doc_ack: in the group being acked */
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
  /* MTE_DOC_LOCAL_CLIENT: the last localSeq; the window the reference's
   * cached local partial lengths were computed with (block_views), -1: none */
  int32_t local_seq;
  int64_t wcache;
  /* MTE_DOC_REFS: reference slots (as oracle.c) */
  uint32_t *ref_anchor, *ref_state;
  uint32_t ref_cap, ref_hi;
  int32_t slide_gid; /* the localSeq whose removal group an ack is sliding (doc_ack) */
  uint8_t in_lop;    /* applying a local op (item.born) */
  /* MTE_DOC_EVENTS: the last batch's delta events, the record being applied */
  mte_delta* dl;
  uint64_t dl_n, dl_cap;
  uint32_t cur_op;
  int ev_rc; /* an event push that failed where no status could be returned (scour) */
  uint64_t msg_dl; /* the first event of the message being applied (maint_positions) */
  int msg_open;    /* a message's records are being applied (its MSG_END not yet) */
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
  const mte_op* aux; /* the records after the one applied (an annotate rollback's MTE_OP_RBKEY) */
} env_t;

#define LOCAL_BASE MTE_LOCAL_SEQ_BASE
#define LRS_RELEASED 0x40000000 /* item.lrs: see there (localSeqs stay below it) */
static inline int is_pending(int32_t seq) { return seq >= LOCAL_BASE && seq != NONE_SEQ; }

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
/* item.born for an item made now: during local op ls it is one of ls's own */
static uint32_t born_now(const idoc* d) { return (uint32_t)d->local_seq + (d->in_lop ? 0u : 1u); }

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
  const int by_c = (int)((s->rmask >> c) & 1u); /* c < 64 */
  if (newcalc) {
    if (removed) {
      if (s->rseq <= m) return -1;
      if (s->rseq <= r || by_c) return 0;
    }
    return (s->seq <= r || s->cli == c) ? s->len : 0;
  }
  if (removed && s->rseq <= r) return -1;
  if (s->cli == c || s->seq <= r) return (removed && by_c) ? 0 : s->len;
  /* inserted and removed before this perspective: undefined, unless the
   * removal is the local client's pending one (removedSeq Unassigned,
   * mergeTree.ts:1049-1052) */
  return (removed && !is_pending(s->rseq)) ? -1 : 0;
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

/* The local client's own view (nodeLength with clientId == collabWindow.clientId
 * -> localNetLength without localSeq, mergeTree.ts:985-987, 553-573): a segment
 * not removed counts its length; a removed one 0 -- with the legacy calculation
 * undefined once its (sequenced) removal is at or below minSeq; a placeholder
 * is no segment. */
static int64_t lengths_local(idoc* d) {
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const item* s = &d->it[i];
    int32_t l;
    if (s->empty) l = -1;
    else if (s->rseq == NONE_SEQ) l = s->len;
    else l = (newcalc || is_pending(s->rseq) || s->rseq > d->min_seq) ? 0 : -1;
    d->L[i] = l;
    d->P[i] = p;
    if (l > 0) p += l;
  }
  return p;
}

/* ---- relative positions (MTE_OP_RELPOS, include/mte.h) ---------------------------
 * posFromRelativePos (mergeTree.ts:1369-1392) for the record nx that follows:
 * the first marker whose key-`key` value is vid (idToSegment, :490, 597-599),
 * at getPosition (:853-870) -- the length before it in nx's view, undefined
 * leaves 0 -- minus the offset (before) or plus 1 + offset; -1 when no held
 * marker carries the id.  nx's pos1 / pos2 are replaced (as oracle.c). */
static int32_t marker_pos(idoc* d, const mte_op* nx, uint32_t key, uint32_t vid, uint32_t n_keys) {
  if (key >= n_keys || vid == 0) return -1;
  uint32_t x = d->n;
  for (uint32_t i = 0; i < d->n && x == d->n; i++)
    if (!d->it[i].empty && d->it[i].kind != 0 && d->it[i].props[key] == vid) x = i;
  if (x == d->n) return -1;
  if (nx->flags & MTE_F_LOCAL) lengths_local(d);
  else lengths(d, nx->ref_seq, nx->client, d->min_seq, (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0);
  return (int32_t)d->P[x];
}

static int doc_relpos(idoc* d, const mte_op* rp, mte_op* nx, uint32_t n_keys) {
  if (rp->flags & MTE_RP_POS1) {
    int32_t p = marker_pos(d, nx, rp->a, (uint32_t)rp->pos1, n_keys);
    if (p >= 0) p = (rp->flags & MTE_RP_BEFORE1) ? p - rp->seq : p + 1 + rp->seq;
    else if (nx->type == MTE_OP_INSERT) return MTE_E_UNSUPPORTED;
    nx->pos1 = p;
  }
  if ((rp->flags & MTE_RP_POS2) && nx->type != MTE_OP_INSERT) {
    int32_t p = marker_pos(d, nx, rp->a, (uint32_t)rp->pos2, n_keys);
    if (p >= 0) p = (rp->flags & MTE_RP_BEFORE2) ? p - rp->ref_seq : p + 1 + rp->ref_seq;
    nx->pos2 = p;
  }
  return MTE_OK;
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
static uint32_t leaf_start(const idoc* d, uint32_t i) {
  while (i > 0 && d->it[i].cont) i--;
  return i;
}
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

static int maint_push(idoc* d, uint32_t type, int64_t id, int64_t len, uint32_t idx);

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
    if (is_pending(x->seq) || (x->lrs && !(x->lrs & LRS_RELEASED)) || x->am) {
      /* a segment of a pending group (segmentGroups not empty, mergeTree.ts:686,
       * 736-739) is held and ends the append run */
      held++;
      prev = -1;
    } else if (x->rseq != NONE_SEQ) {
      if (x->rseq > d->min_seq) {
        held++;
      } else {
        for (uint32_t j = i; j < xe; j++) d->it[j].drop = 1;
        /* UNLINK (mergeTree.ts:692-703) */
        const int rc = maint_push(d, MTE_MAINT_UNLINK, -1, xl, 0);
        if (rc) d->ev_rc = rc;
      }
      prev = -1;
    } else if (x->seq <= d->min_seq) {
      int app = 0;
      if (prev >= 0) {
        const item* p = &d->it[prev];
        const item* pl = &d->it[prev_end - 1]; /* the last text of the leaf appended to */
        const int nl = pl->len > 0 && arena[pl->toff + (uint32_t)pl->len - 1] == (uint16_t)'\n';
        int match = p->po == x->po;
        for (uint32_t k = 0; k < n_keys && match; k++)
          match = p->props[k] == x->props[k] && !(x->props[k] & MTE_VALUE_UNEQUAL); /* NaN !== NaN */
        app = p->kind == 0 && x->kind == 0 && !nl && (prev_len <= TEXT_GRANULARITY || xl <= TEXT_GRANULARITY) &&
              match && xl > 0;
      }
      if (app) {
        x->cont = 1;
        x->id = 0;
        prev_len += xl;
        prev_end = xe;
        /* APPEND (mergeTree.ts:715-727): the segment appended to, then this one */
        int rc = maint_push(d, MTE_MAINT_APPEND, d->it[prev].id, prev_len, 0);
        if (!rc) rc = maint_push(d, MTE_MAINT_APPEND, -1, xl, 1);
        if (rc) d->ev_rc = rc;
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

/* the SPLIT callback of splitLeafSegment (mergeTree.ts:1682-1694): the leaf
 * ending before item i and the one starting there */
static int maint_split(idoc* d, uint32_t i) {
  if (!(d->flags & MTE_DOC_MAINT_EVENTS)) return MTE_OK;
  const uint32_t h = leaf_start(d, i - 1);
  int rc = maint_push(d, MTE_MAINT_SPLIT, d->it[h].id, leaf_total(d, h, i), 0);
  if (!rc) rc = maint_push(d, MTE_MAINT_SPLIT, d->it[i].id, leaf_total(d, i, leaf_end(d, i)), 1);
  return rc;
}

static int boundary(idoc* d, int64_t pos) {
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = d->L[i];
    if (l <= 0) continue;
    if (pos < d->P[i]) return MTE_OK;
    if (pos == d->P[i] && d->it[i].cont) { /* between two texts of one merged leaf */
      d->written += 1;
      d->it[i].cont = 0;
      d->it[i].id = new_id(d);
      d->it[i].born = born_now(d);
      split_cascade(d, i);
      return maint_split(d, i);
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
      tl->born = born_now(d);
      tl->gord = 0x80000000u | tl->id;
      d->written += 2;
      hd->len = off;
      d->L[i] = off;
      d->L[i + 1] = tl->len;
      d->P[i + 1] = d->P[i] + off;
      split_cascade(d, i + 1);
      return maint_split(d, i + 1);
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

/* ---- delta events (MTE_DOC_EVENTS, as oracle.c) ------------------------------
 * One record per segment of the reference: a merged leaf (a head and its
 * continuations) is one segment, so its items' records are joined. */
static int delta_push(idoc* d, uint32_t kind, int64_t pos, int32_t len, uint32_t removed) {
  if (d->dl_n == d->dl_cap) {
    uint64_t nc = d->dl_cap ? 2 * d->dl_cap : 64;
    mte_delta* x = (mte_delta*)realloc(d->dl, nc * sizeof(mte_delta));
    if (!x) return MTE_E_OOM;
    d->dl = x;
    d->dl_cap = nc;
  }
  d->dl[d->dl_n++] = (mte_delta){d->cur_op, kind, (int32_t)pos, len, removed};
  return MTE_OK;
}
/* MTE_DELTA_MAINT (include/mte.h): one segment of a maintenance callback,
 * named by its leaf's id (the reference's segment object: splitAt keeps the
 * head, append keeps the segment appended to) until the record's end, when
 * maint_positions makes it a position; -1: out of the tree */
static int maint_push(idoc* d, uint32_t type, int64_t id, int64_t len, uint32_t idx) {
  if (!(d->flags & MTE_DOC_MAINT_EVENTS)) return MTE_OK;
  return delta_push(d, MTE_DELTA_MAINT | type, id, (int32_t)len, idx);
}
static inline int32_t own_len(const item* g) { return g->rseq == NONE_SEQ ? g->len : 0; }
static int64_t own_prefix(const idoc* d, uint32_t at) {
  int64_t p = 0;
  for (uint32_t i = 0; i < at; i++) p += own_len(&d->it[i]);
  return p;
}

/* annotateRange on one item for a sequenced op in a document with a local
 * client: keys with a pending local update keep their value (shouldModifyKey,
 * segmentPropertiesManager.ts:94-102, 105-135) */
static uint64_t apply_props_pending(uint32_t* props, const uint32_t* pk, uint32_t n_keys, const mte_propset* ps,
                                    const mte_prop* pe, int rewrite) {
  uint64_t w = 0;
  if (rewrite)
    for (uint32_t k = 0; k < n_keys; k++)
      if (!pk[k]) props[k] = 0;
  for (uint32_t j = 0; j < ps->count; j++) {
    const mte_prop* p = &pe[ps->first + j];
    if (p->key < n_keys) {
      if (!pk[p->key]) props[p->key] = p->value;
      w++;
    }
  }
  return w;
}

/* annotateRange with combiningOp incr / consensus (MTE_F_COMBINE): each key
 * becomes combine(op, current, undefined, seq) (segmentPropertiesManager.ts:141,
 * properties.ts:24-62), pending keys included (shouldModifyKey :94-102); the
 * host's per-key map lists {old | MTE_COMBINE_PAIR, new} after a {key, n}
 * header, an old value not listed stays */
static uint64_t apply_combine(uint32_t* props, uint32_t n_keys, const mte_propset* ps, const mte_prop* pe) {
  uint64_t w = 0;
  for (uint32_t t = 0; t < ps->count; t++) {
    const mte_prop* h = &pe[ps->first + t];
    if ((h->key & MTE_COMBINE_PAIR) || h->key >= n_keys) continue;
    const uint32_t old = props[h->key];
    for (uint32_t u = 1; u <= h->value; u++)
      if ((pe[ps->first + t + u].key & ~MTE_COMBINE_PAIR) == old) {
        props[h->key] = pe[ps->first + t + u].value;
        break;
      }
    w++;
  }
  return w;
}

/* ---- local references (MTE_DOC_REFS, as oracle.c) ---------------------------- */
#define REF_LIVE 0x80000000u
#define REF_DETACHED 0x40000000u
/* with REF_DETACHED: taken off its segment's list for want of a segment to
 * slide to (mergeTree.ts:935-942; removeLocalRef keeps the segment) */
#define REF_OFF 0x20000000u
/* a Transient reference (localReference.ts:263: never on its segment's list,
 * so nothing moves or slides it): REF_LIVE | REF_DETACHED | REF_TRANS | the
 * offset in its segment; the anchor is that segment's leaf id -- the segment
 * keeps it across splits (splitAt keeps the head), loses it for good when the
 * zamboni appends it to the one before (a later split there makes a new
 * segment, a new id) or unlinks it (position -1, mergeTree.ts:1095-1112) */
#define REF_TRANS 0x10000000u
#define REF_TRANS_OFF 0x0fffffffu
#define REF_LIMIT (1u << 24)

/* a segment references may slide to (_getSlideToSegment, mergeTree.ts:893-913):
 * not a pending insert, not removed-and-acked (a pending removal is fine), not
 * a placeholder */
static inline int slide_target_ok(const item* g) { return !g->empty && g->seq < LOCAL_BASE && g->rseq >= LOCAL_BASE; }
static inline int removed_and_acked(const item* g) { return g->rseq != NONE_SEQ && !is_pending(g->rseq) && !g->empty; }

/* where a reference on item i slides to (forwardExcursion / backwardExcursion,
 * client.ts:1117-1130): offset 0 of the first following segment, else the last
 * unit of the last preceding one; -1: nowhere */
static inline int grp_pending(const item* g, int32_t grp, uint32_t cur, int32_t gid) {
  return grp && g->rseq == grp && !g->empty && g->seq < LOCAL_BASE && g->gord > cur && g->lrs == gid;
}
static int64_t slide_to_grp(const idoc* d, uint32_t i, uint32_t* anchor, int32_t grp, uint32_t cur) {
  /* a merged leaf's items are one segment: search past i's leaf */
  uint32_t j0 = i + 1;
  while (j0 < d->n && d->it[j0].cont) j0++;
  for (uint32_t j = j0; j < d->n; j++)
    if (slide_target_ok(&d->it[j]) || grp_pending(&d->it[j], grp, cur, d->slide_gid)) {
      *anchor = d->it[j].toff;
      return j;
    }
  int64_t h0 = i;
  while (h0 > 0 && d->it[h0].cont) h0--;
  for (int64_t j = h0 - 1; j >= 0; j--)
    if (slide_target_ok(&d->it[j]) || grp_pending(&d->it[j], grp, cur, d->slide_gid)) {
      *anchor = d->it[j].toff + (uint32_t)d->it[j].len - 1u;
      return j;
    }
  return -1;
}
static int64_t slide_to(const idoc* d, uint32_t i, uint32_t* anchor) { return slide_to_grp(d, i, anchor, 0, 0); }

static int ref_reserve(idoc* d, uint32_t slot) {
  if (slot < d->ref_cap) return MTE_OK;
  uint32_t nc = d->ref_cap ? d->ref_cap : 64;
  while (nc <= slot) nc *= 2;
  uint32_t* a = (uint32_t*)realloc(d->ref_anchor, (size_t)nc * sizeof(uint32_t));
  if (!a) return MTE_E_OOM;
  d->ref_anchor = a;
  uint32_t* st = (uint32_t*)realloc(d->ref_state, (size_t)nc * sizeof(uint32_t));
  if (!st) return MTE_E_OOM;
  d->ref_state = st;
  memset(d->ref_state + d->ref_cap, 0, (size_t)(nc - d->ref_cap) * sizeof(uint32_t));
  d->ref_cap = nc;
  return MTE_OK;
}

static int delta_push(idoc* d, uint32_t kind, int64_t pos, int32_t len, uint32_t removed);

/* the length of an item in the local client's view at refSeq rs0 and localSeq
 * ls (localNetLength with a localSeq, mergeTree.ts:575-593): acked text up to
 * rs0 less acked removals up to rs0, own pending inserts up to ls, less own
 * removals up to ls */
static inline int32_t view_len(const item* g, int32_t rs0, int32_t ls) {
  if (g->empty) return 0;
  if (g->lrs && (g->lrs & ~LRS_RELEASED) <= ls) return 0;
  if (is_pending(g->seq)) return g->seq - LOCAL_BASE > ls ? 0 : g->len;
  if (g->seq > rs0) return 0;
  if (is_pending(g->rseq)) return g->rseq - LOCAL_BASE <= ls ? 0 : g->len;
  return (g->rseq != NONE_SEQ && g->rseq <= rs0) ? 0 : g->len;
}

/* ---- the reference's localSeq views at block level -----------------------------
 * getContainingSegment / getPosition with a localSeq (mergeTree.ts:853-885, 2274-2330)
 * take a block's length from its local partial lengths (nodeLength :984-995 ->
 * PartialSequenceLengths.getPartialLength, partialLengths.ts:667-700): minLength
 * plus the sequenced records up to refSeq, and -- when the block holds a local
 * record at or below localSeq -- the local records up to localSeq less the
 * overlapping removes (a remote remove that overtook a local one).  Summed per
 * item (fromLeaves / insertSegment :330-505), which can disagree with the leaf
 * rule view_len: a local removal of a segment inserted after refSeq is
 * subtracted while its insertion is not counted (a block can come out
 * negative).  The partials are computed by the first such query after a length
 * update, with the window's minSeq lowered to that query's refSeq
 * (computeLocalPartials :964-982): W, kept in idoc.wcache. */
typedef struct {
  int64_t a, b, o;
  int flag;
} pl_acc;

static void item_partial(const item* g, int32_t R, int32_t L, int64_t W, pl_acc* x) {
  if (g->empty) return;
  const int64_t c = g->len;
  if (!is_pending(g->seq)) {
    if (g->seq <= W || g->seq <= R) x->a += c;
  } else if (g->seq - LOCAL_BASE <= L) {
    x->b += c;
    x->flag = 1;
  }
  if (g->rseq == NONE_SEQ) return;
  if (is_pending(g->rseq)) {
    if (g->rseq - LOCAL_BASE <= L) {
      x->b -= c;
      x->flag = 1;
    }
    return;
  }
  if (g->rseq <= W) {
    x->a -= c;
    return;
  }
  if (g->rseq <= R) x->a -= c;
  const int32_t lrs = g->lrs & ~LRS_RELEASED;
  if (__builtin_popcountll(g->rmask) > 1 && lrs != 0 && lrs <= L) { /* an overlapping remove */
    x->b -= c;
    x->flag = 1;
    if (g->rseq <= R) x->o -= c;
  }
}

/* the window of the cached local partials: the first block length a query
 * evaluates computes them, with that query's refSeq (nodeLength :984-995) */
static int64_t view_window(idoc* d, int32_t R) {
  if (d->wcache < 0) d->wcache = d->min_seq < R ? d->min_seq : R;
  return d->wcache;
}

static int64_t block_len(idoc* d, uint32_t s, uint32_t e, int32_t R, int32_t L) {
  const int64_t W = view_window(d, R);
  pl_acc x = {0, 0, 0, 0};
  for (uint32_t i = s; i <= e; i++) item_partial(&d->it[i], R, L, W, &x);
  return x.a + (x.flag ? x.b - x.o : 0);
}

/* the last item of the child of the level-k block [.., e] that starts at c */
static uint32_t child_last(const idoc* d, uint32_t c, uint32_t e, int k) {
  if (k == 1) return leaf_end(d, c) - 1;
  uint32_t j = c + 1;
  while (j <= e && d->it[j].h < k - 1) j++;
  return j - 1;
}

/* a child's length in the view: a leaf by the leaf rule, a block by its partials */
static int64_t child_len(idoc* d, uint32_t c, uint32_t ce, int k, int32_t R, int32_t L) {
  if (k > 1) return block_len(d, c, ce, R, L);
  int64_t v = 0;
  for (uint32_t i = c; i <= ce; i++) v += view_len(&d->it[i], R, L);
  return v;
}

/* nodeMap from the root's children (depthFirstNodeWalk): a zero length skips,
 * a negative one moves the running position back */
static int walk_find(idoc* d, uint32_t s, uint32_t e, int k, int64_t pos, int32_t R, int32_t L, int64_t* p,
                     int64_t* leaf, int64_t* off) {
  for (uint32_t c = s; c <= e; c++) {
    if (!is_child(&d->it[c], k)) continue;
    if (pos + 1 <= *p) return 1;
    const uint32_t ce = child_last(d, c, e, k);
    const int64_t len = child_len(d, c, ce, k, R, L);
    if (len != 0) {
      if (pos >= *p + len) {
        *p += len;
      } else if (k == 1) {
        *leaf = c;
        *off = pos - *p;
        return 1;
      } else if (walk_find(d, c, ce, k - 1, pos, R, L, p, leaf, off)) {
        return 1;
      }
    }
    c = ce;
  }
  return 0;
}

/* getContainingSegment(pos) in the view at (R, L) (mergeTree.ts:872-885): the
 * item holding pos and the offset there; -1 past the end */
static int64_t view_find(idoc* d, int64_t pos, int32_t R, int32_t L, int32_t* off) {
  if (!d->n) return -1;
  int64_t p = 0, leaf = -1, o = 0;
  walk_find(d, 0, d->n - 1, d->depth, pos, R, L, &p, &leaf, &o);
  if (leaf < 0) return -1;
  /* the offset within the leaf -> the item of the leaf holding it */
  uint32_t i = (uint32_t)leaf;
  const uint32_t le = leaf_end(d, i);
  while (i + 1 < le && o >= d->it[i].len) {
    o -= d->it[i].len;
    i++;
  }
  *off = (int32_t)o;
  return i;
}

/* getPosition of the leaf starting at item x (mergeTree.ts:853-870): the
 * lengths of the children before it at every level */
static int64_t view_prefix(idoc* d, uint32_t x, int32_t R, int32_t L) {
  int64_t pos = 0;
  for (int k = 1; k <= d->depth; k++) {
    const uint32_t s = span_start(d, x, k), e = span_end(d, s, k);
    const uint32_t cx = k == 1 ? x : span_start(d, x, k - 1);
    for (uint32_t c = s; c < cx; c++) {
      if (!is_child(&d->it[c], k)) continue;
      const uint32_t ce = child_last(d, c, e, k);
      pos += child_len(d, c, ce, k, R, L);
      c = ce;
    }
  }
  return pos;
}


/* the item a leaf starts at */
/* the units of its leaf before item i */
static int32_t leaf_offset(const idoc* d, uint32_t i) {
  int32_t o = 0;
  for (uint32_t j = leaf_start(d, i); j < i; j++) o += d->it[j].len;
  return o;
}

/* Client.getSlideToSegment (client.ts:1117-1130) from item x, removed and
 * acked: offset 0 of the first following item a reference may slide to, else
 * the last unit of the last preceding one; -1 when there is none */
static int64_t slide_item(const idoc* d, uint32_t x, int32_t* off) {
  for (uint32_t j = x + 1; j < d->n; j++)
    if (slide_target_ok(&d->it[j])) {
      *off = 0;
      return j;
    }
  for (int64_t j = (int64_t)x - 1; j >= 0; j--)
    if (slide_target_ok(&d->it[j])) {
      *off = d->it[j].len - 1;
      return j;
    }
  return -1;
}

/* MTE_OP_REF b = 4 (include/mte.h): Client.rebasePosition (client.ts:755-786)
 * of pos1 from the view at (ref_seq, a) to the view at (currentSeq, a); b = 5:
 * rebaseLocalInterval's slide of a pending interval end
 * (intervalCollection.ts:1782-1799).  One MTE_DELTA_REBASE event each. */
static int doc_ref_rebase(idoc* d, const mte_op* op) {
  const int32_t ls = (int32_t)op->a;
  if (!(d->flags & MTE_DOC_LOCAL_CLIENT) || ls < 0 || ls > d->local_seq) return MTE_E_INVALID_ARG;
  if (!(d->flags & MTE_DOC_EVENTS)) return MTE_E_UNSUPPORTED;
  d->scanned += d->n;
  if (op->b == 4) {
    int32_t off = 0;
    int64_t x = view_find(d, op->pos1, op->ref_seq, ls, &off);
    if (x < 0) { /* past every segment of the view: the tree's last leaf, offset 0 */
      for (int64_t j = (int64_t)d->n - 1; j >= 0 && x < 0; j--)
        if (!d->it[j].empty) x = j;
      off = 0;
    }
    int64_t p = -1;
    if (x >= 0) {
      int64_t t = x;
      if (removed_and_acked(&d->it[x])) t = slide_item(d, (uint32_t)x, &off);
      if (t >= 0) p = view_prefix(d, leaf_start(d, (uint32_t)t), d->cur_seq, ls) + leaf_offset(d, (uint32_t)t) + off;
    }
    return delta_push(d, MTE_DELTA_REBASE, p, 0, 0);
  }
  const uint32_t slot = (uint32_t)op->pos2;
  int64_t p = -1;
  const uint32_t st = slot < d->ref_hi ? d->ref_state[slot] : 0u;
  if ((st & REF_LIVE) && !(st & REF_DETACHED)) { /* a slot not in use answers -1 */
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (g->empty || d->ref_anchor[slot] - g->toff >= (uint32_t)g->len) continue;
      if (removed_and_acked(g)) {
        int32_t off = 0, o2 = 0;
        const int64_t t = slide_item(d, i, &off);
        int64_t y = -1;
        if (t >= 0) {
          p = view_prefix(d, leaf_start(d, (uint32_t)t), d->cur_seq, ls) + leaf_offset(d, (uint32_t)t) + off;
          y = view_find(d, p, d->cur_seq, ls, &o2);
        }
        if (y >= 0) d->ref_anchor[slot] = d->it[y].toff + (uint32_t)o2;
        else { /* the reference throws: no segment there */
          d->ref_anchor[slot] = 0;
          d->ref_state[slot] = st | REF_DETACHED;
        }
        d->wcache = -1; /* createLocalReferencePosition updates lengths (mergeTree.ts:2124-2143) */
      }
      break;
    }
  }
  return delta_push(d, MTE_DELTA_REBASE, p, 0, 0);
}

/* MTE_OP_REF (oracle.c doc_ref): b = 0 create in the local view, 1 remove,
 * 2 create in a sequenced op's perspective, 3 become SlideOnRemove, 4 / 5
 * reconnection (doc_ref_rebase) */
static int doc_ref(idoc* d, const mte_op* op) {
  if (!(d->flags & MTE_DOC_REFS)) return MTE_E_UNSUPPORTED;
  if (op->pos2 < 0 || (uint32_t)op->pos2 >= REF_LIMIT || op->b > 5) return MTE_E_INVALID_ARG;
  if (op->b >= 4) {
    d->ops++;
    return doc_ref_rebase(d, op);
  }
  const uint32_t slot = (uint32_t)op->pos2;
  int rc;
  if ((rc = ref_reserve(d, slot))) return rc;
  d->ops++;
  if (op->b == 1) {
    d->ref_state[slot] = 0;
    return MTE_OK;
  }
  if ((op->a & MTE_REF_TRANSIENT) && op->b != 0) return MTE_E_UNSUPPORTED;
  if ((op->a & MTE_REF_SLIDE_ON_REMOVE) && (op->a & MTE_REF_STAY_ON_REMOVE)) return MTE_E_INVALID_ARG;
  if (op->a & MTE_REF_TRANSIENT) {
    /* createLocalReferencePosition(getContainingSegment(pos)) in the local view */
    d->scanned += d->n;
    int64_t p = 0;
    for (uint32_t i = 0; i < d->n; i++) {
      const int32_t l = d->it[i].empty ? 0 : own_len(&d->it[i]);
      if (l > 0 && op->pos1 >= p && op->pos1 < p + l) {
        const uint32_t h = leaf_start(d, i);
        const int64_t off = op->pos1 - own_prefix(d, h);
        if (off < 0 || off > (int64_t)REF_TRANS_OFF) return MTE_E_UNSUPPORTED;
        if (slot + 1 > d->ref_hi) d->ref_hi = slot + 1;
        d->ref_anchor[slot] = d->it[h].id;
        d->ref_state[slot] = REF_LIVE | REF_DETACHED | REF_TRANS | (uint32_t)off;
        return MTE_OK;
      }
      if (l > 0) p += l;
    }
    return MTE_E_INVALID_ARG;
  }
  d->scanned += d->n;
  if (op->b == 3) {
    uint32_t st = d->ref_state[slot];
    if (!(st & REF_LIVE)) return MTE_E_INVALID_ARG;
    d->ref_state[slot] = st = (st & (REF_LIVE | REF_DETACHED | REF_OFF)) | (op->a & 0xffffu);
    if (st & REF_DETACHED) return MTE_OK;
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (g->empty || d->ref_anchor[slot] - g->toff >= (uint32_t)g->len) continue;
      if (removed_and_acked(g) && (st & MTE_REF_SLIDE_ON_REMOVE)) {
        uint32_t to = 0;
        if (slide_to(d, i, &to) >= 0) d->ref_anchor[slot] = to;
        else d->ref_state[slot] = st | REF_DETACHED;
        d->wcache = -1; /* ackInterval re-creates the end (createLocalReferencePosition) */
      }
      break;
    }
    return MTE_OK;
  }
  const int remote = op->b == 2;
  if (remote && (op->client >= MTE_MAX_CLIENTS || op->client == 0)) return MTE_E_INVALID_ARG;
  if (remote) lengths(d, op->ref_seq, op->client, d->min_seq, (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0);
  int64_t p = 0;
  if (slot + 1 > d->ref_hi) d->ref_hi = slot + 1;
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = remote ? d->L[i] : (d->it[i].empty ? 0 : own_len(&d->it[i]));
    if (l > 0 && op->pos1 >= p && op->pos1 < p + l) {
      uint32_t anchor = d->it[i].toff + (uint32_t)(op->pos1 - p);
      uint32_t st = REF_LIVE | (op->a & 0xffffu);
      if (remote && removed_and_acked(&d->it[i]) && slide_to(d, i, &anchor) < 0) st |= REF_DETACHED;
      else d->wcache = -1; /* createLocalReferencePosition (mergeTree.ts:2124-2143) */
      d->ref_anchor[slot] = anchor;
      d->ref_state[slot] = st;
      return MTE_OK;
    }
    if (l > 0) p += l;
  }
  if (remote) {
    d->ref_anchor[slot] = 0;
    d->ref_state[slot] = REF_LIVE | REF_DETACHED | (op->a & 0xffffu);
    return MTE_OK;
  }
  return MTE_E_INVALID_ARG;
}

/* slideAckedRemovedSegmentReferences for every item whose removedSeq is now s
 * (oracle.c doc_slide_refs); an MTE_DOC_EVENTS document gets one
 * MTE_DELTA_SLIDE record per reference that slid or came off (include/mte.h:
 * the reference's beforeSlide / afterSlide callbacks, localReference.ts:436-447) */
static int delta_push(idoc* d, uint32_t kind, int64_t pos, int32_t len, uint32_t removed);
static int64_t own_prefix(const idoc* d, uint32_t at);
/* mode (mte_stream.h stream_slide): 0 every such item; 1 the removals of one
 * ack, in order, each slid while the later ones are still pending
 * (ackPendingSegment, mergeTree.ts:1285-1304: a reference can slide again);
 * 2 / 3 a remote remove's items the local client had removed already (lrs),
 * slid before its delta callback, then the newly removed ones (:1970-1993) */
static int slide_item_refs(idoc* d, uint32_t i, int32_t grp, uint32_t cur, int evd) {
  const item* g = &d->it[i];
  uint32_t to = 0;
  const int64_t t = slide_to_grp(d, i, &to, grp, cur);
  const int64_t xpos = evd ? own_prefix(d, i) : 0;
  for (uint32_t r = 0; r < d->ref_hi; r++) {
    const uint32_t st = d->ref_state[r];
    if (!(st & REF_LIVE) || (st & REF_DETACHED) || (st & MTE_REF_STAY_ON_REMOVE)) continue;
    const uint32_t off = d->ref_anchor[r] - g->toff;
    if (off >= (uint32_t)g->len) continue;
    const int moves = (st & MTE_REF_SLIDE_ON_REMOVE) && t >= 0;
    const uint32_t left = d->ref_anchor[r];
    if (moves) d->ref_anchor[r] = to;
    else d->ref_state[r] = st | REF_DETACHED | (t < 0 ? REF_OFF : 0u);
    if (evd) {
      /* len: the unit it left, made its order key once the message is done (slide_keys) */
      /* offsets count from the merged leaf's first unit (its items are one segment) */
      uint32_t lead = 0;
      for (uint32_t y = i; y > 0 && d->it[y].cont; y--) lead += (uint32_t)d->it[y - 1].len;
      const uint32_t lo = lead + off;
      const int rc = delta_push(d, MTE_DELTA_SLIDE | (moves ? 1u : 0u) | (moves && t < (int64_t)i ? 2u : 0u) |
                                         ((lo < 0xffffu ? lo : 0xffffu) << 16), xpos,
                                (int32_t)left, r);
      if (rc) return rc;
    }
  }
  return MTE_OK;
}
static int doc_slide_refs(idoc* d, int32_t s, int mode) {
  if (!(d->flags & MTE_DOC_REFS) || !d->ref_hi) return MTE_OK;
  const int evd = (d->flags & MTE_DOC_EVENTS) && (d->flags & MTE_DOC_SLIDE_EVENTS);  /* slide records */
  int rc;
  if (mode == 1) {
    /* the group's segments in group order, each slid while the later ones are pending */
    uint32_t cur = 0;
    for (int first = 1;; first = 0) {
      int64_t bx = -1;
      for (uint32_t i = 0; i < d->n; i++) {
        const item* g = &d->it[i];
        if (g->rseq != s || g->empty || g->lrs != d->slide_gid || (!first && g->gord <= cur)) continue;
        if (bx < 0 || g->gord < d->it[bx].gord) bx = i;
      }
      if (bx < 0) return MTE_OK;
      cur = d->it[bx].gord;
      if ((rc = slide_item_refs(d, (uint32_t)bx, s, cur, evd))) return rc;
    }
  }
  for (uint32_t i = 0; i < d->n; i++) {
    const item* g = &d->it[i];
    if (g->rseq != s || g->empty) continue;
    if (mode >= 2 && (g->lrs != 0) != (mode == 2)) continue;
    if ((rc = slide_item_refs(d, i, 0, 0, evd))) return rc;
  }
  return MTE_OK;
}

/* ---- insert, range ops (remote and local) -------------------------------------------------------- */

/* insertSegments -> blockInsert -> insertingWalk (mergeTree.ts:1394-1422,
 * 1590-1680, 1723-1825) for a remote op (local = 0: lengths in the op's
 * perspective, seq s) or a local one (local = 1: the local view, seq
 * Unassigned = LOCAL_BASE + localSeq).  Returns the new item's index through
 * *at (-1 when nothing was linked). */
static int tree_insert(idoc* d, const mte_op* op, const env_t* env, int local, int64_t* at) {
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  const int32_t r = op->ref_seq, s = op->seq, m = d->min_seq;
  const int c = op->client;
  int rc;
  *at = -1;
  if ((rc = reserve(d, d->n + 3))) return rc;
  if (local) lengths_local(d);
  else lengths(d, r, c, m, newcalc);
  if ((rc = boundary(d, op->pos1))) return rc;
  const int64_t total = local ? lengths_local(d) : lengths(d, r, c, m, newcalc);
  const int is_marker = (op->flags & MTE_F_MARKER) != 0;
  const int32_t len = is_marker ? 1 : op->pos2;
  if (len <= 0) return MTE_OK; /* blockInsert skips zero-length segments (:1645) */
  const int64_t pos = op->pos1;
  /* the leaf block insertingWalk enters: the first whose end reaches pos */
  uint32_t ks = d->n;
  for (uint32_t i = 0; i < d->n; i++)
    if (d->P[i] + (d->L[i] > 0 ? d->L[i] : 0) >= pos) {
      ks = i;
      break;
    }
  if (ks == d->n || pos > total) return MTE_E_INSERT_FAILED;
  uint32_t bs = span_start(d, ks, 1), be = span_end(d, bs, 1);
  uint32_t slot;
  int replace = 0;
  for (;;) {
    slot = UINT32_MAX;
    if (!d->it[bs].empty) {
      /* before the first defined leaf at pos (pos < len, or a zero-length leaf
       * breakTie prefers: every sequenced one, but a pending one only for a
       * local insert -- Unassigned normalises to MAX vs MAX - 1, :1705-1721) */
      for (uint32_t i = ks; i <= be; i++) {
        const item* g = &d->it[i];
        if (d->L[i] >= 0 && d->P[i] >= pos && !g->empty && !(!local && d->L[i] == 0 && is_pending(g->seq))) {
          slot = i;
          break;
        }
      }
      if (slot != UINT32_MAX) break;
    }
    /* _pos == 0 at the block's end: a sequenced insert asks continuePredicate,
     * whose forward excursion looks at the first segment after the block and
     * moves on past the block when it is a pending local one (:1599-1611,
     * 1788-1793); otherwise the segment goes at the block's end */
    if (!local) {
      uint32_t x = be + 1;
      while (x < d->n && d->it[x].empty) x++;
      if (x < d->n && is_pending(d->it[x].seq)) {
        ks = x;
        bs = span_start(d, x, 1);
        be = span_end(d, bs, 1);
        continue;
      }
    }
    if (d->it[bs].empty) {
      slot = bs;
      replace = 1;
    } else {
      slot = be + 1;
    }
    break;
  }
  item nw;
  memset(&nw, 0, sizeof nw);
  nw.len = len;
  nw.seq = local ? LOCAL_BASE + s : s;
  nw.cli = c;
  nw.rseq = NONE_SEQ;
  nw.id = new_id(d);
  nw.born = born_now(d);
  d->written += 1;
  if (is_marker) {
    nw.kind = 1u + (uint32_t)op->pos2;
    if (d->flags & MTE_DOC_REFS) nw.toff = (uint32_t)(env->text_base + op->a); /* its reserved unit */
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
  /* saveIfLocal (:1614-1627): a local segment joins the pending list, a
   * sequenced one the LRU set */
  if (!local && (rc = add_lru(d, slot, s))) return rc;
  *at = slot;
  return MTE_OK;
}

/* markRangeRemoved / annotateRange (mergeTree.ts:1864-2000) for a remote op or
 * a local one (the local view, removedSeq / pending keys Unassigned) */
static int tree_range(idoc* d, const mte_op* op, const env_t* env, int local) {
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  const int32_t r = op->ref_seq, s = op->seq, m = d->min_seq;
  const int c = op->client;
  const int local_doc = (d->flags & MTE_DOC_LOCAL_CLIENT) != 0;
  const int ev = (d->flags & MTE_DOC_EVENTS) != 0;
  const int64_t start = op->pos1, end = op->pos2;
  int rc;
  if ((rc = reserve(d, d->n + 3))) return rc;
  if (local) lengths_local(d);
  else lengths(d, r, c, m, newcalc);
  if ((rc = boundary(d, start))) return rc;
  if (local) lengths_local(d);
  else lengths(d, r, c, m, newcalc);
  if ((rc = boundary(d, end))) return rc;
  if (end == start) return MTE_OK;
  if (local) lengths_local(d);
  else lengths(d, r, c, m, newcalc);
  int64_t lp = 0;         /* the own view's prefix after the op, for the events */
  int64_t last_ev = -2;   /* the item of the last event (a continuation joins it) */
  for (uint32_t i = 0; i < d->n; lp += own_len(&d->it[i]), i++) {
    const int32_t l = d->L[i];
    if (l <= 0) continue;
    if (d->P[i] >= end) break;
    if (d->P[i] + l <= start) continue;
    item* g = &d->it[i];
    d->written += 1;
    const int is_rem = op->type == MTE_OP_REMOVE;
    /* a remove reports the segments it newly removes, an annotate every one it
     * visits (removedSegments / deltaSegments, :1954-1959, 1893-1900) */
    if (ev && (!is_rem || g->rseq == NONE_SEQ)) {
      const uint32_t removed = is_rem || g->rseq != NONE_SEQ;
      if (g->cont && last_ev == (int64_t)i - 1 && d->dl_n) {
        d->dl[d->dl_n - 1].len += g->len;
      } else if ((rc = delta_push(d, op->type, lp, g->len, removed))) {
        return rc;
      }
      last_ev = i;
    }
    if (is_rem) {
      if (local) {
        g->rseq = LOCAL_BASE + s;
        g->rmask = 1u;
        g->lrs = s;
        g->gord = i;
      } else if (g->rseq == NONE_SEQ) {
        g->rseq = s;
        g->rmask = 1ull << c;
      } else {
        if (is_pending(g->rseq)) g->rseq = s; /* overtaking our pending removal (:1928-1938) */
        g->rmask |= 1ull << c;
      }
    } else {
      const mte_propset* ps = &env->b->propsets[op->a];
      g->po = 1;
      if ((op->flags & MTE_F_COMBINE) && local) {
        /* a local incr / consensus: pending keys and group as any local
         * annotate, each key's value mapped (segmentPropertiesManager.ts:117-147) */
        for (uint32_t t = 0; t < ps->count; t++) {
          const mte_prop* h = &env->b->props[ps->first + t];
          if (!(h->key & MTE_COMBINE_PAIR) && h->key < env->n_keys && !g->pk[h->key]) g->basev[h->key] = g->props[h->key];
        }
        d->pwrites += apply_combine(g->props, env->n_keys, ps, env->b->props);
        for (uint32_t t = 0; t < ps->count; t++) {
          const mte_prop* h = &env->b->props[ps->first + t];
          if (!(h->key & MTE_COMBINE_PAIR) && h->key < env->n_keys) g->pk[h->key] = (uint32_t)s;
        }
        if (op->b != MTE_NO_PROPS) g->am |= 1u << op->b;
      } else if (op->flags & MTE_F_COMBINE) {
        d->pwrites += apply_combine(g->props, env->n_keys, ps, env->b->props);
      } else if (local) {
        for (uint32_t j = 0; j < ps->count; j++) {
          const mte_prop* p = &env->b->props[ps->first + j];
          if (p->key < env->n_keys && !g->pk[p->key]) g->basev[p->key] = g->props[p->key];
        }
        d->pwrites += orc_apply_props(g->props, env->n_keys, ps, env->b->props, 0);
        for (uint32_t j = 0; j < ps->count; j++) {
          const mte_prop* p = &env->b->props[ps->first + j];
          if (p->key < env->n_keys) g->pk[p->key] = (uint32_t)s;
        }
        if (op->b != MTE_NO_PROPS) g->am |= 1u << op->b; /* the annotate's segment group */
      } else if (local_doc) {
        d->pwrites += apply_props_pending(g->props, g->pk, env->n_keys, ps, env->b->props,
                                          (op->flags & MTE_F_REWRITE) != 0);
      } else {
        d->pwrites += orc_apply_props(g->props, env->n_keys, ps, env->b->props, (op->flags & MTE_F_REWRITE) != 0);
      }
    }
    /* a sequenced op adds each visited segment to the LRU set (:1881-1884, 1955-1958) */
    if (!local && !g->cont && (rc = add_lru(d, i, s))) return rc;
  }
  return MTE_OK;
}

/* ---- local records --------------------------------------------------------------------------------- */

static int doc_rollback(idoc* d, const mte_op* op, const env_t* env);
static int doc_regen(idoc* d, const mte_op* op);

/* A local op (MTE_F_LOCAL): insertSegmentLocal / removeRangeLocal /
 * annotateRangeLocal (client.ts:131-229) with seq Unassigned, or one of the
 * local records (rollback, regeneration, reference). */
static int doc_apply_local_op(idoc* d, const mte_op* op, const env_t* env);
static int doc_apply_local(idoc* d, const mte_op* op, const env_t* env) {
  d->in_lop = 1;
  const int rc = doc_apply_local_op(d, op, env);
  d->in_lop = 0;
  return rc;
}
static int doc_apply_local_op(idoc* d, const mte_op* op, const env_t* env) {
  const int32_t ls = op->seq;
  int rc;
  /* a length update drops the cached local partials (mergeTree.ts:2105-2110,
   * 2188-2191): every local op; references: doc_ref */
  if (op->type != MTE_OP_REGEN && op->type != MTE_OP_REF) d->wcache = -1;
  if (op->type == MTE_OP_ROLLBACK) return doc_rollback(d, op, env);
  if (op->type == MTE_OP_REGEN) return doc_regen(d, op);
  if (op->type == MTE_OP_REF) return doc_ref(d, op);
  if (!(ls > d->local_seq && ls < LOCAL_BASE)) return MTE_E_INVALID_ARG;
  if (op->client != 0) return MTE_E_INVALID_ARG;
  if (op->type == MTE_OP_ANNOTATE && (op->flags & MTE_F_REWRITE)) return MTE_E_UNSUPPORTED;
  d->local_seq = ls;
  d->ops++;
  if (d->n > d->max_segs) d->max_segs = d->n;
  if (op->type == MTE_OP_NOOP) return MTE_OK;
  d->scanned += d->n;
  if (op->type == MTE_OP_INSERT) {
    int64_t at;
    if ((rc = tree_insert(d, op, env, 1, &at))) return rc;
    if (d->flags & MTE_DOC_EVENTS) {
      const int is_marker = (op->flags & MTE_F_MARKER) != 0;
      return at >= 0 ? delta_push(d, MTE_OP_INSERT, own_prefix(d, (uint32_t)at), is_marker ? 1 : op->pos2, 0)
                     : delta_push(d, MTE_OP_INSERT, -1, 0, 0);
    }
    return MTE_OK;
  }
  if (op->type != MTE_OP_REMOVE && op->type != MTE_OP_ANNOTATE) return MTE_E_INVALID_ARG;
  return tree_range(d, op, env, 1);
}

/* the next item of a pending group, from i on: an insert / remove group by its
 * seq / removedSeq, an annotate group by its slot bit */
static int64_t next_member(const idoc* d, uint32_t i, uint32_t t, int32_t ls, uint32_t slot) {
  for (; i < d->n; i++) {
    const item* g = &d->it[i];
    if (g->empty) continue;
    if (t == MTE_OP_INSERT ? g->seq == LOCAL_BASE + ls
                           : (t == MTE_OP_REMOVE ? g->rseq == LOCAL_BASE + ls : ((g->am >> slot) & 1u) != 0))
      return i;
  }
  return -1;
}

/* MTE_OP_ROLLBACK of an annotate (as oracle.c doc_rollback_annotate), each
 * segment re-annotated by annotateRange at seq UniversalSequenceNumber, which
 * runs zamboniSegments after it (mergeTree.ts:2036-2072, 1901-1905) */
static int doc_rollback_annotate(idoc* d, const mte_op* op, const env_t* env) {
  const uint32_t b = op->a;
  const mte_op* aux = env->aux;
  const uint32_t n_aux = (uint32_t)op->pos2;
  int rc;
  if (b >= MTE_ANNOTATE_SLOTS || !aux) return MTE_E_INVALID_ARG;
  d->ops++;
  d->scanned += d->n;
  for (int64_t i = next_member(d, 0, MTE_OP_ANNOTATE, 0, b); i >= 0; i = next_member(d, 0, MTE_OP_ANNOTATE, 0, b)) {
    item* g = &d->it[i];
    if (g->rseq != NONE_SEQ) return MTE_E_UNSUPPORTED;
    /* a merged leaf of the group is one segment: its items together */
    uint32_t e = (uint32_t)i + 1;
    while (e < d->n && d->it[e].cont) e++;
    uint32_t j = 0;
    while (j < n_aux) {
      const uint32_t key = (uint32_t)aux[j].pos1;
      if (key >= env->n_keys) return MTE_E_INVALID_ARG;
      uint32_t val = g->basev[key], pk = 0;
      for (; j < n_aux; j++) {
        const uint32_t slot = (uint32_t)aux[j].pos2;
        if ((uint32_t)aux[j].pos1 != key) return MTE_E_INVALID_ARG;
        if (slot >= MTE_ANNOTATE_SLOTS) break;
        if ((g->am >> slot) & 1u) {
          val = aux[j].a;
          pk = (uint32_t)aux[j].seq;
          break;
        }
      }
      while (j < n_aux && (uint32_t)aux[j].pos2 < MTE_ANNOTATE_SLOTS) j++;
      if (j >= n_aux) return MTE_E_INVALID_ARG;
      j++;
      for (uint32_t q = (uint32_t)i; q < e; q++) {
        d->it[q].props[key] = val;
        d->it[q].pk[key] = pk;
      }
      d->pwrites += 1;
    }
    int32_t tl = 0;
    for (uint32_t q = (uint32_t)i; q < e; q++) {
      d->it[q].am &= ~(1u << b);
      tl += d->it[q].len;
    }
    if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_ANNOTATE, own_prefix(d, (uint32_t)i), tl, 0)))
      return rc;
    d->written += 1;
    zamboni(d, env->arena, env->n_keys);
  }
  return MTE_OK;
}

/* MTE_OP_ROLLBACK (MergeTree.rollback, mergeTree.ts:2005-2083): an insert's
 * segments get seq and removedSeq UniversalSequenceNumber through
 * markRangeRemoved at seq 0, which runs zamboniSegments after each; a remove's
 * are restored */
static int doc_rollback(idoc* d, const mte_op* op, const env_t* env) {
  const int32_t ls = op->seq;
  int rc;
  if (!(ls > 0 && ls <= d->local_seq)) return MTE_E_INVALID_ARG;
  if (op->pos1 == MTE_OP_ANNOTATE) return doc_rollback_annotate(d, op, env);
  if (op->pos1 != MTE_OP_INSERT && op->pos1 != MTE_OP_REMOVE) return MTE_E_INVALID_ARG;
  d->ops++;
  d->scanned += d->n;
  const uint32_t t = (uint32_t)op->pos1;
  for (int64_t i = next_member(d, 0, t, ls, 0); i >= 0; i = next_member(d, t == MTE_OP_INSERT ? 0 : (uint32_t)i + 1, t, ls, 0)) {
    item* g = &d->it[i];
    const int64_t lp = own_prefix(d, (uint32_t)i);
    if (t == MTE_OP_INSERT) {
      g->seq = 0;
      g->rseq = 0;
      g->rmask = 1u;
      if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_REMOVE, lp, g->len, 1))) return rc;
      d->written += 1;
      zamboni(d, env->arena, env->n_keys);
    } else {
      g->rseq = NONE_SEQ;
      g->rmask = 0;
      g->lrs = 0;
      if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_INSERT, lp, g->len, 0))) return rc;
      d->written += 1;
    }
  }
  return MTE_OK;
}


/* MTE_OP_REGEN (as oracle.c doc_regen): the group's segments in document order
 * at their positions in the view at that localSeq -- a merged leaf one record */
static int doc_regen(idoc* d, const mte_op* op) {
  const int32_t ls = op->seq;
  const uint32_t t = (uint32_t)op->pos1;
  int rc;
  if (!(ls > 0 && ls <= d->local_seq)) return MTE_E_INVALID_ARG;
  if (t != MTE_OP_INSERT && t != MTE_OP_REMOVE && t != MTE_OP_ANNOTATE) return MTE_E_INVALID_ARG;
  if (t == MTE_OP_ANNOTATE && op->a >= MTE_ANNOTATE_SLOTS) return MTE_E_INVALID_ARG;
  if (!(d->flags & MTE_DOC_EVENTS)) return MTE_E_UNSUPPORTED;
  d->ops++;
  d->scanned += d->n;
  int64_t last = -2;
  for (uint32_t i = 0; i < d->n; i++) {
    item* g = &d->it[i];
    int hit;
    if (g->empty) hit = 0;
    else if (t == MTE_OP_INSERT) hit = g->seq == LOCAL_BASE + ls;
    else if (t == MTE_OP_REMOVE) hit = g->rseq == LOCAL_BASE + ls;
    else hit = ((g->am >> op->a) & 1u) && (g->rseq == NONE_SEQ || is_pending(g->rseq));
    /* a member that re-sends nothing leaves the group (resetPendingDeltaToOps
     * dequeues every segment and enqueues only those with a new op,
     * client.ts:803-852): a removal a remote remove overtook, an annotated
     * segment removed since -- the zamboni no longer holds it for the group */
    if (!g->empty && !hit) {
      const int member = (t == MTE_OP_REMOVE && g->lrs == ls) || (t == MTE_OP_ANNOTATE && ((g->am >> op->a) & 1u));
      if (t == MTE_OP_REMOVE && g->lrs == ls) g->lrs |= LRS_RELEASED;
      if (t == MTE_OP_ANNOTATE) g->am &= ~(1u << op->a);
      /* its position is taken all the same (resetPendingDeltaToOps :806, before
       * the op is chosen): that may compute the cached local partials */
      if (member && !g->cont && d->wcache < 0) (void)view_prefix(d, i, d->cur_seq, ls);
    }
    if (hit) {
      /* each re-sent segment heads a group of its own, the old group's segments
       * taken by ordinal (client.ts:802, 852): the ack slides them in document
       * order, split tails included */
      if (t == MTE_OP_REMOVE) g->gord = i;
      g->rg = g->cont ? d->it[i - 1].rg : 1u + g->id;
      /* findReconnectionPosition (client.ts:709-713): getPosition with the
       * localSeq, block lengths from the local partials (view_prefix) */
      if (g->cont && last == (int64_t)i - 1 && d->dl_n) d->dl[d->dl_n - 1].len += g->len;
      else if ((rc = delta_push(d, MTE_DELTA_REGEN | t,
                                view_prefix(d, leaf_start(d, i), d->cur_seq, ls) + leaf_offset(d, i), g->len,
                                t == MTE_OP_INSERT ? g->toff : 0u)))
        return rc;
      last = i;
    }
  }
  return MTE_OK;
}

/* an item the ack of ls still has to take: inserted, removed or annotated by
 * ls (am_mask: ls's annotate slot), or a removal of ls a remote one overtook */
static inline int ack_pending(const item* g, int32_t ls, uint32_t am_mask) {
  return !g->empty && (g->seq == LOCAL_BASE + ls || g->lrs == ls || g->rseq == LOCAL_BASE + ls || (g->am & am_mask));
}

/* ackPendingSegment (mergeTree.ts:1278-1331) for one segment group of ls: the
 * items whose regeneration key is `key` (-1: every item of ls) get the seq,
 * each is added to the LRU set in the group's order, the references of the
 * acked removals slide, the ACKNOWLEDGED callback reports the group, then
 * zamboniSegments runs. */
static int ack_group(idoc* d, int32_t ls, int32_t s, uint32_t am_mask, int64_t key, const mte_propset* stamp,
                     const env_t* env) {
  int rc;
  for (uint32_t i = 0; i < d->n; i++) {
    item* g = &d->it[i];
    if (g->empty || (key >= 0 && g->rg != (uint32_t)key)) continue;
    int member = 0;
    if (g->seq == LOCAL_BASE + ls) {
      g->seq = s;
      member = 1;
    }
    if (g->lrs == ls) { /* acked, or overtaken by a remote remove before (:1928-1938) */
      g->lrs = 0;
      member = 1;
    }
    if (g->rseq == LOCAL_BASE + ls) {
      g->rseq = s;
      /* the group's removals hold ls until they have slid (doc_slide_refs'
       * group mark; a regenerated one's localRemovedSeq is its old op's);
       * acked: localRemovedSeq undefined (mergeTreeNodes.ts:493) */
      g->lrs = ((d->flags & MTE_DOC_REFS) && d->ref_hi) ? ls : 0;
    }
    if (g->am & am_mask) {
      /* updateConsensusProperty (client.ts:646-650, 1083-1090): the ack of a
       * local consensus stamps its marker's value with the seq, outside the
       * pending-key rules (addProperties without a collab window) */
      if (stamp) (void)apply_combine(g->props, env->n_keys, stamp, env->b->props);
      g->am &= ~am_mask;
      member = 1;
    }
    g->member = member && !g->cont;
  }
  /* addToLRUSet per segment in the group's order: the segments the op marked
   * in document order, then the tails split off since, as they were made */
  for (uint32_t i = 0; i < d->n; i++)
    if (d->it[i].member && d->it[i].born <= (uint32_t)ls && (rc = add_lru(d, i, s))) return rc;
  for (uint32_t last = 0, any = 1; any;) {
    int64_t bx = -1;
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (g->member && g->born > (uint32_t)ls && g->id >= last && (bx < 0 || g->id < d->it[bx].id)) bx = i;
    }
    any = bx >= 0;
    if (any) {
      if ((rc = add_lru(d, (uint32_t)bx, s))) return rc;
      last = d->it[bx].id + 1u;
    }
  }
  d->slide_gid = ls;  /* this localSeq's group, in its order (ackPendingSegment per group op) */
  if ((rc = doc_slide_refs(d, s, 1))) return rc;
  /* ACKNOWLEDGED (mergeTree.ts:1313-1320): the group's segments, after their slides */
  if (d->flags & MTE_DOC_MAINT_EVENTS) {
    uint32_t idx = 0;
    for (uint32_t i = 0; i < d->n; i++)
      if (d->it[i].member && (rc = maint_push(d, MTE_MAINT_ACK, d->it[i].id, leaf_total(d, i, leaf_end(d, i)), idx++)))
        return rc;
  }
  for (uint32_t i = 0; i < d->n; i++) {
    item* g = &d->it[i];
    if (key >= 0 && g->rg != (uint32_t)key) continue;
    if (g->lrs == ls) g->lrs = 0;
    g->member = 0;
  }
  zamboni(d, env->arena, env->n_keys);
  return MTE_OK;
}

/* MTE_OP_ACK for localSeqs pos1..pos2 (client.ts:640-672 acks a GROUP's members
 * one by one): per localSeq, ackPendingSegment acks its group.  A regenerated
 * message (MTE_F_REGENERATED) re-sent each segment of a localSeq as an op of
 * its own with a group of its own (resetPendingDeltaToOps, client.ts:802-857):
 * it acks them one by one, in document order, each group the segment and the
 * tails split off it since.  The slot mask op->a frees the annotate groups (all of them
 * with the last localSeq of the record). */
static int doc_ack(idoc* d, const mte_op* op, const env_t* env) {
  const int32_t lo = op->pos1, hi = op->pos2, s = op->seq;
  int rc;
  if (!(lo > 0 && lo <= hi && hi <= d->local_seq)) return MTE_E_INVALID_ARG;
  for (int32_t ls = lo; ls <= hi; ls++) {
    const uint32_t am_mask = ls == hi ? op->a : 0u;
    const mte_propset* stamp = (ls == hi && (op->flags & MTE_F_COMBINE)) ? &env->b->propsets[op->b] : NULL;
    for (uint32_t i = 0; i < d->n; i++) {
      item* g = &d->it[i];
      for (uint32_t k = 0; k < MTE_MAX_KEYS; k++)
        if (g->pk[k] && g->pk[k] <= (uint32_t)ls) g->pk[k] = 0;
    }
    if (!(op->flags & MTE_F_REGENERATED)) {
      if ((rc = ack_group(d, ls, s, am_mask, -1, stamp, env))) return rc;
      continue;
    }
    for (;;) {
      int64_t first = -1;
      for (uint32_t i = 0; i < d->n && first < 0; i++)
        if (ack_pending(&d->it[i], ls, am_mask)) first = i;
      if (first < 0) break;
      if ((rc = ack_group(d, ls, s, am_mask, d->it[first].rg, stamp, env))) return rc;
    }
  }
  return MTE_OK;
}

/* The MTE_DELTA_SLIDE records of the message that starts at record `from`:
 * the unit each reference left -> that unit's order key once the message's
 * zamboni has run (the held units before it, as mte_read_ref_order counts
 * them; -1 if it is gone), so a host compares the ends as they were with the
 * others as they are. */
static void slide_keys(idoc* d, uint64_t from) {
  for (uint64_t q = from; q < d->dl_n; q++) {
    mte_delta* e = &d->dl[q];
    if ((e->kind & 0xc0u) != MTE_DELTA_SLIDE) continue;
    const uint32_t u = (uint32_t)e->len;
    int64_t p = 0, key = -1;
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (!g->empty && u - g->toff < (uint32_t)g->len) {
        key = p + (int64_t)(u - g->toff);
        break;
      }
      p += g->len;
    }
    e->len = (int32_t)key;
  }
}

static int32_t ref_position(const idoc* d, uint32_t r, int transient);
static int64_t ref_order_key(const idoc* d, uint32_t r);

/* MTE_DELTA_REFPOS (include/mte.h): after a record that slid references,
 * every live reference as it left the document -- its position (-2 - the
 * Transient one for a reference off the string) and order key: what the
 * reference's slide callbacks read mid-op (intervalCollection.ts:1042-1053) */
static int ref_snapshot(idoc* d) {
  for (uint32_t r = 0; r < d->ref_hi; r++) {
    if (!(d->ref_state[r] & REF_LIVE) || (d->ref_state[r] & REF_TRANS)) continue;  /* no interval end */
    const int32_t p = ref_position(d, r, 0), tp = ref_position(d, r, 1);
    const int rc = delta_push(d, MTE_DELTA_REFPOS, p >= 0 ? p : (tp >= 0 ? -2 - tp : -1), (int32_t)ref_order_key(d, r), r);
    if (rc) return rc;
  }
  return MTE_OK;
}

/* the record's MTE_DELTA_MAINT segments, named by leaf id -> their positions
 * in the own view now (-1: no leaf of that id is in the tree any more) */
static void maint_positions(idoc* d, uint64_t from) {
  for (uint64_t q = from; q < d->dl_n; q++) {
    mte_delta* e = &d->dl[q];
    if ((e->kind & 0xff00u) != MTE_DELTA_MAINT || e->pos < 0) continue;
    int64_t p = -1;
    for (uint32_t i = 0; i < d->n; i++)
      if (d->it[i].id == (uint32_t)e->pos && !d->it[i].cont && !d->it[i].empty) {
        p = own_prefix(d, i);
        break;
      }
    e->pos = (int32_t)p;
  }
}

static int doc_apply_op(idoc* d, const mte_op* op, const env_t* env);
static int doc_apply(idoc* d, const mte_op* op, const env_t* env) {
  const uint64_t from = d->dl_n;
  if (!d->msg_open) d->msg_dl = from;
  int rc = doc_apply_op(d, op, env);
  if (!rc && d->ev_rc) rc = d->ev_rc;
  /* maintenance positions once the message (a local record: itself) is applied */
  d->msg_open = !(op->flags & (MTE_F_MSG_END | MTE_F_LOCAL)) && op->type != MTE_OP_RELPOS ? 1 : 0;
  if (op->type == MTE_OP_RELPOS) d->msg_open = 1;
  if (!rc && (d->flags & MTE_DOC_MAINT_EVENTS) && !d->msg_open && d->dl_n > d->msg_dl) maint_positions(d, d->msg_dl);
  if (!rc && (d->flags & MTE_DOC_SLIDE_EVENTS) && d->dl_n > from) {
    slide_keys(d, from);
    int slid = 0;
    for (uint64_t q = from; q < d->dl_n; q++) slid |= (d->dl[q].kind & 0xc0u) == MTE_DELTA_SLIDE;
    if (slid) rc = ref_snapshot(d);
  }
  return rc;
}

static int doc_apply_op(idoc* d, const mte_op* op, const env_t* env) {
  const int32_t s = op->seq;
  const int c = op->client;
  const int local_doc = (d->flags & MTE_DOC_LOCAL_CLIENT) != 0;
  int rc;
  if (d->n + 4 > env->limit) return MTE_E_CAPACITY;
  /* short ids: 32 on the flat passes (a 32-bit removers plane), 64 on the HBM
   * tree pass (local-client and MTE_DOC_TREE documents: a second plane) */
  if (c >= ((d->flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_TREE)) ? MTE_MAX_CLIENTS_TREE : MTE_MAX_CLIENTS))
    return MTE_E_CLIENT_RANGE;
  if (op->flags & MTE_F_LOCAL) {
    if ((op->flags & MTE_F_COMBINE) && op->type != MTE_OP_ANNOTATE) return MTE_E_UNSUPPORTED;
    return local_doc ? doc_apply_local(d, op, env) : MTE_E_UNSUPPORTED;
  }
  /* a combining annotate, or the ack of a local consensus (its stamp) */
  if ((op->flags & MTE_F_COMBINE) && (!(local_doc || (d->flags & MTE_DOC_TREE)) ||
                                       (op->type != MTE_OP_ANNOTATE && op->type != MTE_OP_ACK)))
    return MTE_E_UNSUPPORTED;
  d->wcache = -1; /* a sequenced message updates lengths */
  if (op->type == MTE_OP_ACK && !local_doc) return MTE_E_UNSUPPORTED;
  if (local_doc && op->type != MTE_OP_ACK && op->type != MTE_OP_NOOP && c == 0) return MTE_E_INVALID_ARG;
  d->ops++;
  if (d->n > d->max_segs) d->max_segs = d->n;
  if (op->type != MTE_OP_NOOP) d->scanned += d->n;
  if (op->type == MTE_OP_INSERT) {
    int64_t at;
    if ((rc = tree_insert(d, op, env, 0, &at))) return rc;
    if (d->flags & MTE_DOC_EVENTS) {
      const int is_marker = (op->flags & MTE_F_MARKER) != 0;
      rc = at >= 0 ? delta_push(d, MTE_OP_INSERT, own_prefix(d, (uint32_t)at), is_marker ? 1 : op->pos2, 0)
                   : delta_push(d, MTE_OP_INSERT, -1, 0, 0);
      if (rc) return rc;
    }
    zamboni(d, env->arena, env->n_keys);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_REMOVE || op->type == MTE_OP_ANNOTATE) {
    if ((rc = tree_range(d, op, env, 0))) return rc;
    if (op->type == MTE_OP_REMOVE && ((rc = doc_slide_refs(d, s, 2)) || (rc = doc_slide_refs(d, s, 3)))) return rc;
    zamboni(d, env->arena, env->n_keys);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_ACK) {
    if ((rc = doc_ack(d, op, env))) return rc;
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
    free(c->docs[i].ref_anchor);
    free(c->docs[i].ref_state);
    free(c->docs[i].dl);
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
    d->wcache = -1;
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
  env_t env = {w->b, w->base, w->c->n_keys, w->c->arena, w->c->limit, NULL};
  for (uint32_t di = w->d0; di < w->d1; di += w->stride) {
    idoc* d = &w->c->docs[di];
    if (d->status) continue;
    d->dl_n = 0;
    for (uint64_t k = w->b->op_offsets[di]; k < w->b->op_offsets[di + 1]; k++) {
      const mte_op* op = &w->b->ops[k];
      mte_op nx;
      int rc = 0;
      if (op->type == MTE_OP_RELPOS) {  /* the next record, at the resolved positions */
        if (d->n + 4 > env.limit) rc = MTE_E_CAPACITY;
        nx = op[1];
        if (!rc) rc = doc_relpos(d, op, &nx, env.n_keys);
        op = &nx;
        k++;
      }
      d->cur_op = (uint32_t)(k - w->b->op_offsets[di]);
      env.aux = &w->b->ops[k] + 1;
      if (!rc) rc = doc_apply(d, op, &env);
      if (rc) {
        d->status = rc;
        break;
      }
      if (op->type == MTE_OP_ROLLBACK && op->pos1 == MTE_OP_ANNOTATE) k += (uint64_t)op->pos2; /* its RBKEY records */
    }
  }
  return NULL;
}

int oti_apply_batch(oti_ctx* c, const mte_batch* b, int n_threads) {
  if (!c || !b || b->n_docs != c->n_docs || !b->op_offsets) return MTE_E_INVALID_ARG;
  if (b->op_offsets[b->n_docs] != b->n_ops) return MTE_E_INVALID_ARG;
  /* the records as mte_submit validates them (oracle.c orc_apply_batch) */
  uint32_t dcur = 0;
  uint64_t rbkey_end = 0;
  for (uint64_t k = 0; k < b->n_ops; k++) {
    const mte_op* op = &b->ops[k];
    while (dcur + 1 < b->n_docs && b->op_offsets[dcur + 1] <= k) dcur++;
    const int local_doc = (c->docs[dcur].flags & MTE_DOC_LOCAL_CLIENT) != 0;
    if ((op->type == MTE_OP_RBKEY) != (k < rbkey_end)) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_ROLLBACK && op->pos1 == MTE_OP_ANNOTATE) {
      if (op->pos2 < 0 || k + 1 + (uint64_t)op->pos2 > b->op_offsets[dcur + 1]) return MTE_E_INVALID_ARG;
      rbkey_end = k + 1 + (uint64_t)op->pos2;
    }
    if (op->type > MTE_OP_RELPOS) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_RELPOS) {
      const uint32_t rp = MTE_RP_POS1 | MTE_RP_BEFORE1 | MTE_RP_POS2 | MTE_RP_BEFORE2;
      if ((op->flags & ~rp) || !(op->flags & (MTE_RP_POS1 | MTE_RP_POS2)) || k + 1 >= b->op_offsets[dcur + 1] ||
          op[1].type > MTE_OP_ANNOTATE)
        return MTE_E_INVALID_ARG;
      continue;
    }
    if (op->type >= MTE_OP_ROLLBACK && !(op->flags & MTE_F_LOCAL)) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_REF) {
      if (!(c->docs[dcur].flags & MTE_DOC_REFS) || op->seq != 0 || op->pos2 < 0 || op->b > 5 ||
          op->client >= MTE_MAX_CLIENTS)
        return MTE_E_INVALID_ARG;
      continue;
    }
    if ((op->flags & MTE_F_LOCAL) && op->type == MTE_OP_ANNOTATE && op->b != MTE_NO_PROPS &&
        op->b >= MTE_ANNOTATE_SLOTS)
      return MTE_E_INVALID_ARG;
    if ((op->flags & MTE_F_LOCAL) || op->type == MTE_OP_ACK) {
      if (!local_doc) return MTE_E_INVALID_ARG;
      if ((op->flags & MTE_F_LOCAL) && op->type != MTE_OP_RBKEY &&
          (op->type == MTE_OP_ACK || op->seq <= 0 || op->seq >= MTE_LOCAL_SEQ_BASE))
        return MTE_E_INVALID_ARG;
      if (op->type == MTE_OP_RBKEY && (op->seq < 0 || op->seq >= MTE_LOCAL_SEQ_BASE || op->pos1 < 0 ||
                                       op->pos1 >= MTE_MAX_KEYS || op->pos2 < 0 || op->pos2 > MTE_ANNOTATE_SLOTS))
        return MTE_E_INVALID_ARG;
      if (op->type == MTE_OP_ACK && (op->pos1 <= 0 || op->pos1 > op->pos2)) return MTE_E_INVALID_ARG;
    }
    if (local_doc && !(op->flags & MTE_F_LOCAL) && op->seq >= MTE_LOCAL_SEQ_BASE) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_INSERT && !(op->flags & MTE_F_MARKER) && op->pos2 > 0 &&
        (uint64_t)op->a + (uint64_t)op->pos2 > b->text_units)
      return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_INSERT && op->b != MTE_NO_PROPS && op->b >= b->n_propsets) return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_ANNOTATE && op->a >= b->n_propsets) return MTE_E_INVALID_ARG;
  }
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
        /* mte_seg.removers holds short ids < 32 */
        if (g->rseq != NONE_SEQ && (g->rmask >> 32)) return MTE_E_UNSUPPORTED;
        s->removers = g->rseq == NONE_SEQ ? 0u : (uint32_t)g->rmask;
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

int oti_read_deltas(oti_ctx* c, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const idoc* d = &c->docs[doc];
  *n = d->dl_n;
  if (out) memcpy(out, d->dl, (size_t)(cap < d->dl_n ? cap : d->dl_n) * sizeof(mte_delta));
  return MTE_OK;
}

/* referencePositionToLocalPosition (mergeTree.ts:1095-1112) of slots [0, n),
 * as oracle.c: -1 for a detached or unused slot or a unit no item holds (its
 * segment unlinked by the zamboni) */
/* mte_read_ref_order: the index, among every unit the document holds, of the
 * unit each reference sits on (-1 detached / unused) */
/* the order key of reference slot r: the index, among every unit the document
 * holds, of the unit it sits on (-1 detached / unused) */
static int64_t ref_order_key(const idoc* d, uint32_t r) {
  if (r >= d->ref_hi) return -1;
  const uint32_t st = d->ref_state[r], u = d->ref_anchor[r];
  if (!(st & REF_LIVE) || ((st & REF_DETACHED) && !(st & REF_OFF))) return -1; /* off the string: on its segment */
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const item* g = &d->it[i];
    if (!g->empty && u - g->toff < (uint32_t)g->len) return p + (int64_t)(u - g->toff);
    p += g->empty ? 0 : g->len;
  }
  return -1;
}

int oti_read_ref_order(oti_ctx* c, uint32_t doc, int64_t* key, uint32_t n) {
  if (!c || (n && !key) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const idoc* d = &c->docs[doc];
  for (uint32_t r = 0; r < n; r++) key[r] = ref_order_key(d, r);
  return MTE_OK;
}

/* the position of reference slot r (-1 detached / unused / a unit no segment
 * holds); transient: one taken off its segment's list still finds it */
static int32_t ref_position(const idoc* d, uint32_t r, int transient) {
  if (r >= d->ref_hi) return -1;
  const uint32_t st = d->ref_state[r], u = d->ref_anchor[r];
  if ((st & REF_LIVE) && (st & REF_TRANS)) {
    /* referencePositionToLocalPosition of a Transient one: its segment's
     * position, plus the offset unless the segment is removed; -1 unlinked */
    for (uint32_t i = 0; i < d->n; i++) {
      const item* g = &d->it[i];
      if (!g->empty && !g->cont && g->id == u)
        return (int32_t)(own_prefix(d, i) + (g->rseq != NONE_SEQ ? 0 : (int64_t)(st & REF_TRANS_OFF)));
    }
    return -1;
  }
  if (!(st & REF_LIVE) || ((st & REF_DETACHED) && !(transient && (st & REF_OFF)))) return -1;
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const item* g = &d->it[i];
    if (!g->empty && u - g->toff < (uint32_t)g->len) return (int32_t)(p + (g->rseq != NONE_SEQ ? 0 : (int64_t)(u - g->toff)));
    p += g->empty ? 0 : own_len(g);
  }
  return -1;
}

static int read_refs_view(oti_ctx* c, uint32_t doc, int32_t* pos, uint32_t n, int transient) {
  if (!c || (n && !pos) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const idoc* d = &c->docs[doc];
  for (uint32_t r = 0; r < n; r++) pos[r] = ref_position(d, r, transient);
  return MTE_OK;
}

int oti_read_refs(oti_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) { return read_refs_view(c, doc, pos, n, 0); }

/* mte_read_refs_transient: as oti_read_refs with every reference Transient
 * (emitChange, intervalCollection.ts:1387-1410): a reference taken off its
 * segment's list still finds the segment while it is held */
int oti_read_refs_transient(oti_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) {
  return read_refs_view(c, doc, pos, n, 1);
}
