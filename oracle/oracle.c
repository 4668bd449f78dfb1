/*
 * oracle.c — CPU restatement of merge-tree observer replay (TEST INFRASTRUCTURE).
 *
 * This file restates, for a client that only receives sequenced remote ops,
 * the semantics of the reference TypeScript merge-tree
 * (/root/reference/packages/dds/merge-tree/src, cited below as file:line).
 * It is a *flat* restatement: a document is an ordered array of segments and
 * every perspective length is recomputed by a linear scan, instead of the
 * reference's B+tree with PartialSequenceLengths.  SURVEY.md Appendix A and
 * DESIGN.md ("Flat restatement") argue the equivalence; the golden fixtures
 * pin it.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 */
#include "oracle.h"
#include "orc_common.h"

#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define NONE_SEQ ORC_NONE_SEQ

typedef struct {
  int32_t len;   /* cachedLength (text: UTF-16 units, marker: 1)          */
  int32_t seq;   /* insert seq (UniversalSequenceNumber 0 for load text)  */
  int32_t rseq;  /* removedSeq or NONE_SEQ                                */
  uint32_t rmask;/* removedClientIds as a set (mergeTreeNodes.ts:134-150) */
  int32_t cli;   /* clientId (-1 = LocalClientId, constants.ts:14)        */
  uint32_t kind; /* 0 text, 1 + refType for a marker                      */
  uint32_t toff; /* text offset into the ctx text arena                   */
  uint32_t props[MTE_MAX_KEYS];
} oseg;

typedef struct {
  oseg* s;
  uint32_t n, cap;
  int32_t min_seq, cur_seq;
  uint32_t flags;
  int32_t status;
  int32_t rs_ref, rs_seq; /* MTE_DOC_ROUND_SYNC: highest refSeq, highest live seq so far */
  /* MTE_DOC_LOCAL_CLIENT: per segment and key, the localSeq of the last pending
   * local annotate that set the key (0 = none pending), a row of MTE_MAX_KEYS
   * per segment kept in step with s[] (the pendingKeyUpdateCount of
   * segmentPropertiesManager.ts:20-60, see doc_apply_local); the last localSeq */
  uint32_t* pk;
  int32_t local_seq;
  /* MTE_DOC_REFS: local reference slots -- the arena offset of the unit the
   * reference sits on (a marker's is its reserved unit) and REF_LIVE |
   * REF_DETACHED | refType; slots [0, ref_hi) were ever used */
  uint32_t* ref_anchor;
  uint32_t* ref_state;
  uint32_t ref_cap, ref_hi;
  /* MTE_DOC_EVENTS: the last batch's delta events, and the record being applied */
  mte_delta* dl;
  uint64_t dl_n, dl_cap;
  uint32_t cur_op;
  /* stats */
  uint64_t ops, scanned, written, pwrites, units, max_segs;
  /* scratch */
  int32_t* L;
  int64_t* P;
  uint32_t scratch_cap;
  /* loaded state, for reload */
  mte_doc_init init;
  uint32_t init_props[MTE_MAX_KEYS];
} __attribute__((aligned(128))) odoc; /* one cache-line pair per doc: no false sharing between threads */

struct orc_ctx {
  uint32_t n_keys;
  uint32_t n_docs;
  odoc* docs;
  uint64_t load_units;     /* text units given to orc_load_docs */
  mte_propset* load_ps;    /* propsets given to orc_load_docs (for orc_load_segments) */
  uint32_t n_load_ps;
  mte_prop* load_pe;
  uint32_t n_load_pe;
  uint16_t* arena;
  uint64_t arena_n, arena_cap;
};

/* ------------------------------------------------------------------------ */

static int arena_append(orc_ctx* c, const uint16_t* t, uint64_t n, uint64_t* base) {
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

/* a pk row: MTE_MAX_KEYS pending-key localSeqs, the mask of the pending
 * annotate groups (MTE_ANNOTATE_SLOTS) the segment belongs to, then per key the
 * value it had before the first pending annotate set it (what an annotate
 * rollback puts back when no older pending annotate set the key) */
#define PKW (2 * MTE_MAX_KEYS + 1)
#define PK(d, i) ((d)->pk + (size_t)(i) * PKW)
#define AM(d, i) (PK(d, i)[MTE_MAX_KEYS])
#define BASEV(d, i) (PK(d, i) + MTE_MAX_KEYS + 1)

static int doc_reserve(odoc* d, uint32_t need) {
  if (need <= d->cap) return MTE_OK;
  uint32_t nc = d->cap ? d->cap : 64;
  while (nc < need) nc *= 2;
  oseg* s = (oseg*)realloc(d->s, (size_t)nc * sizeof(oseg));
  if (!s) return MTE_E_OOM;
  d->s = s;
  if (d->flags & MTE_DOC_LOCAL_CLIENT) {
    uint32_t* pk = (uint32_t*)realloc(d->pk, (size_t)nc * PKW * sizeof(uint32_t));
    if (!pk) return MTE_E_OOM;
    d->pk = pk;
  }
  d->cap = nc;
  return MTE_OK;
}

static int doc_scratch(odoc* d) {
  if (d->n <= d->scratch_cap) return MTE_OK;
  uint32_t nc = d->cap;
  int32_t* L = (int32_t*)realloc(d->L, (size_t)nc * sizeof(int32_t));
  if (!L) return MTE_E_OOM;
  d->L = L;
  int64_t* P = (int64_t*)realloc(d->P, (size_t)nc * sizeof(int64_t));
  if (!P) return MTE_E_OOM;
  d->P = P;
  d->scratch_cap = nc;
  return MTE_OK;
}

/* Insert `cnt` empty slots at index `at` (shifting the tail right). */
static int doc_open(odoc* d, uint32_t at, uint32_t cnt) {
  int rc = doc_reserve(d, d->n + cnt);
  if (rc) return rc;
  memmove(d->s + at + cnt, d->s + at, (size_t)(d->n - at) * sizeof(oseg));
  if (d->pk) {
    memmove(PK(d, at + cnt), PK(d, at), (size_t)(d->n - at) * PKW * sizeof(uint32_t));
    memset(PK(d, at), 0, (size_t)cnt * PKW * sizeof(uint32_t));
  }
  d->n += cnt;
  return MTE_OK;
}

/*
 * Perspective length of a leaf for (refSeq r, clientId c), with m = the
 * window minSeq before this message.  Returns -1 for "undefined".
 *   new calc:  mergeTree.ts:1003-1026
 *   legacy:    mergeTree.ts:1028-1054
 * The observer never sends, so the local branch (mergeTree.ts:985-995,
 * localNetLength 553-594) is never taken for op application.
 */
static inline int32_t leaf_len(const oseg* s, int32_t r, int c, int32_t m, int newcalc) {
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

/* L[i] and exclusive prefix P[i] (undefined leaves contribute 0).  Returns the
 * total perspective length.  This is the flat restatement of nodeLength on
 * blocks (partialLengths.ts:667-702 == sum of leaf lengths, test/testUtils.ts
 * :173-248). */
static int64_t doc_lengths(odoc* d, int32_t r, int c, int32_t m, int newcalc) {
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    int32_t l = leaf_len(&d->s[i], r, c, m, newcalc);
    d->L[i] = l;
    d->P[i] = p;
    if (l > 0) p += l;
  }
  return p;
}

/*
 * ensureIntervalBoundary(pos) (mergeTree.ts:1698-1702): the insertingWalk with
 * TreeMaintenanceSequenceNumber enters the first leaf with pos < len (breakTie
 * is false for it, 1705-1721) and splitLeafSegment splits it when the offset is
 * > 0 (1681-1696).  The tail inherits seq/clientId/removal/props
 * (mergeTreeNodes.ts:505-534, textSegment.ts:105-113); markers never split
 * (mergeTreeNodes.ts:644-646).  L/P are kept consistent.  Returns the index of
 * the new tail segment or -1.
 */
static int64_t doc_split_at(odoc* d, int64_t pos, uint64_t* written) {
  for (uint32_t i = 0; i < d->n; i++) {
    int32_t l = d->L[i];
    if (l <= 0) continue;
    if (pos < d->P[i]) return -1;
    if (pos < d->P[i] + l) {
      int64_t off = pos - d->P[i];
      if (off == 0 || d->s[i].kind != 0) return -1;
      if (doc_open(d, i + 1, 1)) return -2;
      /* keep scratch arrays in step */
      if (doc_scratch(d)) return -2;
      memmove(d->L + i + 2, d->L + i + 1, (size_t)(d->n - i - 2) * sizeof(int32_t));
      memmove(d->P + i + 2, d->P + i + 1, (size_t)(d->n - i - 2) * sizeof(int64_t));
      oseg* head = &d->s[i];
      oseg* tail = &d->s[i + 1];
      *tail = *head;
      /* the tail keeps the pending key counts (copyPropertiesTo,
       * mergeTreeNodes.ts:505-534 -> PropertiesManager.copyTo) */
      if (d->pk) memcpy(PK(d, i + 1), PK(d, i), PKW * sizeof(uint32_t));
      tail->len = head->len - (int32_t)off;
      tail->toff = head->toff + (uint32_t)off;
      head->len = (int32_t)off;
      d->L[i] = (int32_t)off;
      d->L[i + 1] = tail->len;
      d->P[i + 1] = d->P[i] + off;
      *written += 2;
      return (int64_t)i + 1;
    }
  }
  return -1;
}

typedef struct {
  const mte_batch* b;
  uint64_t text_base;
  uint32_t n_keys;
  const uint16_t* arena;
  const mte_op* aux;  /* the records after the one applied (an annotate rollback's MTE_OP_RBKEY) */
} apply_env;

/* Client.completeAndLogOp asserts (client.ts:525-528). */
static int check_op_window(const odoc* d, const mte_op* op) {
  if (!(d->cur_seq < op->seq)) return MTE_E_SEQ_ORDER;
  if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER;
  return MTE_OK;
}

/* Canonical zamboni: drop tombstones with removedSeq <= minSeq.  The reference
 * unlinks the same segments lazily (scourNode, mergeTree.ts:681-747); the
 * difference is not observable (such leaves are "undefined" for every later
 * op in both length modes, and never visible). */
static void doc_compact(odoc* d) {
  uint32_t w = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    if (d->s[i].rseq != NONE_SEQ && d->s[i].rseq <= d->min_seq) continue;
    if (w != i) {
      d->s[w] = d->s[i];
      if (d->pk) memcpy(PK(d, w), PK(d, i), PKW * sizeof(uint32_t));
    }
    w++;
  }
  d->n = w;
}

#define LOCAL_BASE MTE_LOCAL_SEQ_BASE

/* ---- delta events (MTE_DOC_EVENTS, include/mte.h) --------------------------
 * mergeTreeDeltaCallback after an insert / remove / annotate
 * (mergeTree.ts:1409-1416, 1893-1900, 1978-1985) as SharedString's
 * sequenceDelta listener reads it right away: per affected segment its
 * position in the doc's own view (Client.getPosition, client.ts:345-350 ->
 * nodeLength for the local client: removed 0, else the length) and its
 * cachedLength. */
static int delta_push(odoc* d, uint32_t kind, int64_t pos, int32_t len, uint32_t removed) {
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
static inline int32_t own_len(const oseg* g) { return g->rseq == NONE_SEQ ? g->len : 0; }
static int64_t own_prefix(const odoc* d, uint32_t at) {
  int64_t p = 0;
  for (uint32_t i = 0; i < at; i++) p += own_len(&d->s[i]);
  return p;
}
static inline int is_pending(int32_t seq) { return seq >= LOCAL_BASE && seq != NONE_SEQ; }

/* annotateRange on one segment for a sequenced (remote) op in a document with
 * a local client: PropertiesManager.addProperties skips every key with a
 * pending local update (shouldModifyKey, segmentPropertiesManager.ts:94-102,
 * 121-135), the rewrite's clear included (105-119). */
static uint64_t apply_props_pending(uint32_t* props, const uint32_t* pk, uint32_t n_keys, const mte_propset* ps,
                                    const mte_prop* pe, int rewrite) {
  uint64_t w = 0;
  if (rewrite) {
    for (uint32_t k = 0; k < n_keys; k++)
      if (!pk[k]) props[k] = 0;
  }
  for (uint32_t j = 0; j < ps->count; j++) {
    const mte_prop* p = &pe[ps->first + j];
    if (p->key < n_keys) {
      if (!pk[p->key]) props[p->key] = p->value;
      w++;
    }
  }
  return w;
}

/* The local client's own view (nodeLength with clientId == collabWindow.clientId
 * -> localNetLength without localSeq, mergeTree.ts:985-987, 553-573, new length
 * calculation): every segment not removed counts its length, a removed one 0
 * (its own pending removals included). */
static int64_t doc_lengths_local(odoc* d) {
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = d->s[i].rseq != NONE_SEQ ? 0 : d->s[i].len;
    d->L[i] = l;
    d->P[i] = p;
    p += l;
  }
  return p;
}

static int doc_rollback(odoc* d, const mte_op* op, const apply_env* env);
static int doc_regen(odoc* d, const mte_op* op);

/* ---- relative positions (MTE_OP_RELPOS, include/mte.h) ------------------------
 * posFromRelativePos (mergeTree.ts:1369-1392) for the record nx that follows:
 * the marker idToSegment holds for the id -- the first marker segment whose
 * key-`key` value is vid (ids unique per document, :490, 597-599) -- at
 * getPosition (:853-870), the length of everything before it in nx's view
 * (undefined leaves count 0), minus the offset (before) or plus 1 + offset;
 * -1 when no held marker carries the id.  nx's pos1 / pos2 are replaced. */
static int32_t marker_pos(odoc* d, const mte_op* nx, uint32_t key, uint32_t vid, uint32_t n_keys) {
  if (key >= n_keys || vid == 0) return -1;
  uint32_t x = d->n;
  for (uint32_t i = 0; i < d->n && x == d->n; i++)
    if (d->s[i].kind != 0 && d->s[i].props[key] == vid) x = i;
  if (x == d->n) return -1;
  if (nx->flags & MTE_F_LOCAL) doc_lengths_local(d);
  else doc_lengths(d, nx->ref_seq, nx->client, d->min_seq, (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0);
  return (int32_t)d->P[x];
}

static int doc_relpos(odoc* d, const mte_op* rp, mte_op* nx, uint32_t n_keys) {
  int rc;
  if ((rc = doc_scratch(d))) return rc;
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

/* ---- local references (MTE_DOC_REFS, include/mte.h) --------------------------
 * A reference is kept as the text unit it sits on (its arena offset: splits
 * never copy text, so the unit names the same place in whatever segment holds
 * it) -- LocalReferenceCollection keeps it as (segment, offset) and moves it on
 * split / append (localReference.ts:330-416), which names the same unit. */
#define REF_LIVE 0x80000000u
#define REF_DETACHED 0x40000000u
/* with REF_DETACHED: taken off its segment's list for want of a segment to
 * slide to (mergeTree.ts:935-942; removeLocalRef keeps the segment) */
#define REF_OFF 0x20000000u
#define REF_LIMIT (1u << 24)

/* a segment references may slide to (_getSlideToSegment, mergeTree.ts:893-913):
 * not a pending insert and not removed-and-acked (a pending removal is fine) */
static inline int slide_target_ok(const oseg* g) { return g->seq < LOCAL_BASE && g->rseq >= LOCAL_BASE; }

/* where a reference on segment i slides to when that segment is removed and
 * acked (_getSlideToSegment, mergeTree.ts:893-913; Client.getSlideToSegment's
 * offset, client.ts:1117-1130): the first following segment it may slide to at
 * offset 0, else the last preceding one at its last offset; -1: nowhere */
static int64_t slide_to(const odoc* d, uint32_t i, uint32_t* anchor) {
  for (uint32_t j = i + 1; j < d->n; j++)
    if (slide_target_ok(&d->s[j])) {
      *anchor = d->s[j].toff;
      return j;
    }
  for (int64_t j = (int64_t)i - 1; j >= 0; j--)
    if (slide_target_ok(&d->s[j])) {
      *anchor = d->s[j].toff + (uint32_t)d->s[j].len - 1u;
      return j;
    }
  return -1;
}
static inline int removed_and_acked(const oseg* g) { return g->rseq != NONE_SEQ && !is_pending(g->rseq); }

/* MTE_OP_REF (include/mte.h):
 *   b = 0: createLocalReferencePosition on getContainingSegment(pos1) in the
 *     local view (client.ts:360-364, 1107-1110; mergeTree.ts:872-885, 2124-2143);
 *   b = 1: removeLocalReferencePosition (mergeTree.ts:2113-2123);
 *   b = 2: a reference a sequenced op creates (createPositionReference with an
 *     op, intervalCollection.ts:639-658): getContainingSegment(pos1, op) in the
 *     op's perspective (ref_seq, client), then getSlideToSegment -- a segment
 *     removed and acked since hands it on at once; no segment: detached
 *     (createDetachedLocalReferencePosition, :621-637);
 *   b = 3: the reference becomes SlideOnRemove (a = its new type) and slides
 *     if its segment is removed and acked (ackInterval's setSlideOnRemove and
 *     getSlideToSegment, :1805-1902). */
static int doc_ref(odoc* d, const mte_op* op) {
  if (!(d->flags & MTE_DOC_REFS)) return MTE_E_UNSUPPORTED;
  /* b = 4 / 5 (reconnection of pending interval ops): titems.c, the HBM tree
   * pass's restatement, only */
  if (op->b == 4 || op->b == 5) return MTE_E_UNSUPPORTED;
  if (op->pos2 < 0 || (uint32_t)op->pos2 >= REF_LIMIT || op->b > 3) return MTE_E_INVALID_ARG;
  const uint32_t slot = (uint32_t)op->pos2;
  if (slot >= d->ref_cap) {
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
  }
  d->ops++;
  if (op->b == 1) {
    d->ref_state[slot] = 0;
    return MTE_OK;
  }
  if (op->a & MTE_REF_TRANSIENT) return MTE_E_UNSUPPORTED;
  if ((op->a & MTE_REF_SLIDE_ON_REMOVE) && (op->a & MTE_REF_STAY_ON_REMOVE)) return MTE_E_INVALID_ARG;
  d->scanned += d->n;
  if (op->b == 3) {
    uint32_t st = d->ref_state[slot];
    if (!(st & REF_LIVE)) return MTE_E_INVALID_ARG;
    d->ref_state[slot] = st = (st & (REF_LIVE | REF_DETACHED | REF_OFF)) | (op->a & 0xffffu);
    if (st & REF_DETACHED) return MTE_OK;
    for (uint32_t i = 0; i < d->n; i++) {
      const oseg* g = &d->s[i];
      if (d->ref_anchor[slot] - g->toff >= (uint32_t)g->len) continue;
      if (removed_and_acked(g) && (st & MTE_REF_SLIDE_ON_REMOVE)) {
        uint32_t to = 0;
        if (slide_to(d, i, &to) >= 0) d->ref_anchor[slot] = to;
        else d->ref_state[slot] = st | REF_DETACHED;
      }
      break;
    }
    return MTE_OK;
  }
  const int remote = op->b == 2;
  if (remote && (op->client >= MTE_MAX_CLIENTS || op->client == 0)) return MTE_E_INVALID_ARG;
  int rc;
  if (remote && (rc = doc_scratch(d))) return rc;
  if (remote) doc_lengths(d, op->ref_seq, op->client, d->min_seq, (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0);
  int64_t p = 0;
  if (slot + 1 > d->ref_hi) d->ref_hi = slot + 1;
  for (uint32_t i = 0; i < d->n; i++) {
    const int32_t l = remote ? d->L[i] : own_len(&d->s[i]);
    if (l > 0 && op->pos1 >= p && op->pos1 < p + l) {
      uint32_t anchor = d->s[i].toff + (uint32_t)(op->pos1 - p);
      uint32_t st = REF_LIVE | (op->a & 0xffffu);
      if (remote && removed_and_acked(&d->s[i]) && slide_to(d, i, &anchor) < 0) st |= REF_DETACHED;
      d->ref_anchor[slot] = anchor;
      d->ref_state[slot] = st;
      return MTE_OK;
    }
    if (l > 0) p += l;
  }
  if (remote) {  /* no segment holds pos1 in the op's view: a detached reference */
    d->ref_anchor[slot] = 0;
    d->ref_state[slot] = REF_LIVE | REF_DETACHED | (op->a & 0xffffu);
    return MTE_OK;
  }
  return MTE_E_INVALID_ARG; /* no segment holds pos1 in the local view */
}

/* slideAckedRemovedSegmentReferences (mergeTree.ts:921-950) for every segment
 * the op of seq s made removed-and-acked (its removedSeq is now s: a remote
 * remove's new removals and overtaken pending ones, :1936-1938 / 1986-1993, or
 * the ack of a local removal, :1302-1304): SlideOnRemove references go to
 * offset 0 of the first following segment a reference may slide to
 * (forwardExcursion, addBeforeTombstones), else to the last offset of the last
 * preceding one (backwardExcursion, addAfterTombstones), else detach; Simple
 * references detach (localReference.ts:422-485). */
static void doc_slide_refs(odoc* d, int32_t s) {
  if (!(d->flags & MTE_DOC_REFS) || !d->ref_hi) return;
  for (uint32_t i = 0; i < d->n; i++) {
    const oseg* g = &d->s[i];
    if (g->rseq != s) continue;
    uint32_t to = 0;
    const int64_t t = slide_to(d, i, &to);
    for (uint32_t r = 0; r < d->ref_hi; r++) {
      const uint32_t st = d->ref_state[r];
      if (!(st & REF_LIVE) || (st & REF_DETACHED) || (st & MTE_REF_STAY_ON_REMOVE)) continue;
      if (d->ref_anchor[r] - g->toff >= (uint32_t)g->len) continue;
      if ((st & MTE_REF_SLIDE_ON_REMOVE) && t >= 0) d->ref_anchor[r] = to;
      else d->ref_state[r] = st | REF_DETACHED | (t < 0 ? REF_OFF : 0u);
    }
  }
}

/* A local op (MTE_F_LOCAL, include/mte.h): insertSegmentLocal /
 * removeRangeLocal / annotateRangeLocal (client.ts:131-229) with seq =
 * UnassignedSequenceNumber, held as LOCAL_BASE + localSeq.
 *   insert: ensureIntervalBoundary + insertingWalk in the local view; breakTie
 *     normalises the new seq to MAX_SAFE_INTEGER (mergeTree.ts:1713), so the
 *     segment goes before the first leaf at P >= pos, as a remote insert does;
 *     no continuePredicate for a local insert (:1790).  The segment joins the
 *     pending list (saveIfLocal, :1614-1619).
 *   remove: markRemoved on the leaves the local view sees in [start, end):
 *     removedSeq = Unassigned, removedClientIds = [local] (:1954-1959).
 *   annotate: set / delete each key now and count it pending
 *     (segmentPropertiesManager.ts:121-135); a local rewrite is unsupported. */
static int doc_apply_local(odoc* d, const mte_op* op, const apply_env* env) {
  const int32_t ls = op->seq;
  int rc;
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
  if ((rc = doc_scratch(d))) return rc;
  const int64_t total = doc_lengths_local(d);
  if (op->type == MTE_OP_INSERT) {
    const int64_t pos = op->pos1;
    const int64_t tail = doc_split_at(d, pos, &d->written);
    if (tail == -2) return MTE_E_OOM;
    const int is_marker = (op->flags & MTE_F_MARKER) != 0;
    const int32_t len = is_marker ? 1 : op->pos2;
    if (len <= 0) return (d->flags & MTE_DOC_EVENTS) ? delta_push(d, MTE_OP_INSERT, -1, 0, 0) : MTE_OK;
    uint32_t at = d->n;
    if (tail >= 0) {
      at = (uint32_t)tail;
    } else {
      for (uint32_t i = 0; i < d->n; i++)
        if (d->P[i] >= pos) { at = i; break; }
      if (at == d->n && pos > total) return MTE_E_INSERT_FAILED;
    }
    if ((rc = doc_open(d, at, 1))) return rc;
    oseg* ns = &d->s[at];
    memset(ns, 0, sizeof(*ns));
    ns->len = len;
    ns->seq = LOCAL_BASE + ls;
    ns->cli = 0;
    ns->rseq = NONE_SEQ;
    if (is_marker) {
      ns->kind = 1u + (uint32_t)op->pos2;
      if (d->flags & MTE_DOC_REFS) ns->toff = (uint32_t)(env->text_base + op->a); /* its reserved unit */
    } else {
      ns->toff = (uint32_t)(env->text_base + op->a);
      d->units += (uint64_t)len;
    }
    if (op->b != MTE_NO_PROPS)
      d->pwrites += orc_apply_props(ns->props, env->n_keys, &env->b->propsets[op->b], env->b->props, 0);
    d->written += 1;
    if (d->flags & MTE_DOC_EVENTS) return delta_push(d, MTE_OP_INSERT, own_prefix(d, at), len, 0);
    return MTE_OK;
  }
  if (op->type != MTE_OP_REMOVE && op->type != MTE_OP_ANNOTATE) return MTE_E_INVALID_ARG;
  const int64_t start = op->pos1, end = op->pos2;
  if (doc_split_at(d, start, &d->written) == -2) return MTE_E_OOM;
  if (doc_split_at(d, end, &d->written) == -2) return MTE_E_OOM;
  int64_t lp = 0;  /* the own view's prefix after the op, for the events */
  for (uint32_t i = 0; i < d->n && end > start; lp += own_len(&d->s[i]), i++) {
    const int32_t l = d->L[i];
    if (l <= 0) continue;
    if (d->P[i] >= end) break;
    if (d->P[i] + l <= start) continue;
    oseg* g = &d->s[i];
    if ((d->flags & MTE_DOC_EVENTS) &&
        (rc = delta_push(d, op->type, lp, g->len, op->type == MTE_OP_REMOVE || g->rseq != NONE_SEQ)))
      return rc;
    if (op->type == MTE_OP_REMOVE) {
      g->rseq = LOCAL_BASE + ls;
      g->rmask = 1u;
    } else {
      const mte_propset* ps = &env->b->propsets[op->a];
      /* the value a key had before the first pending annotate set it (the
       * previousProps of that annotate, mergeTree.ts:1874-1880) */
      for (uint32_t j = 0; j < ps->count; j++) {
        const mte_prop* p = &env->b->props[ps->first + j];
        if (p->key < env->n_keys && !PK(d, i)[p->key]) BASEV(d, i)[p->key] = g->props[p->key];
      }
      d->pwrites += orc_apply_props(g->props, env->n_keys, ps, env->b->props, 0);
      for (uint32_t j = 0; j < ps->count; j++) {
        const mte_prop* p = &env->b->props[ps->first + j];
        if (p->key < env->n_keys) PK(d, i)[p->key] = (uint32_t)ls;
      }
      /* the segment joins the annotate's segment group (addToPendingList) */
      if (op->b != MTE_NO_PROPS) AM(d, i) |= 1u << op->b;
    }
    d->written += 1;
  }
  return MTE_OK;
}

/* MTE_OP_ROLLBACK of an annotate (group slot op->a), followed by its op->pos2
 * MTE_OP_RBKEY records (env->aux): MergeTree.rollback -> annotateRange of
 * each segment of the group with its previousProps under
 * PropertiesRollback.Rollback (mergeTree.ts:2036-2072): the pending count of
 * each key drops (decrementPendingCounts, segmentPropertiesManager.ts:73-84)
 * and the key takes its value from before the annotate -- the latest older
 * pending annotate of the segment's groups that set it (its localSeq becomes
 * the key's pending one), else the value before the first pending annotate.
 * Each segment's annotate event at its own-view position (findRollbackPosition
 * :2088-2103).  A segment of the group removed since would make the reference
 * re-annotate the range after it (its local length is 0): MTE_E_UNSUPPORTED. */
static int doc_rollback_annotate(odoc* d, const mte_op* op, const apply_env* env) {
  const uint32_t b = op->a;
  const mte_op* aux = env->aux;
  const uint32_t n_aux = (uint32_t)op->pos2;
  int rc;
  if (b >= MTE_ANNOTATE_SLOTS || !aux) return MTE_E_INVALID_ARG;
  d->ops++;
  d->scanned += d->n;
  int64_t lp = 0;
  for (uint32_t i = 0; i < d->n; lp += own_len(&d->s[i]), i++) {
    if (!((AM(d, i) >> b) & 1u)) continue;
    oseg* g = &d->s[i];
    if (g->rseq != NONE_SEQ) return MTE_E_UNSUPPORTED;
    uint32_t j = 0;
    while (j < n_aux) {
      const uint32_t key = (uint32_t)aux[j].pos1;
      if (key >= env->n_keys) return MTE_E_INVALID_ARG;
      uint32_t val = BASEV(d, i)[key], pk = 0;
      for (; j < n_aux; j++) {  /* the key's candidates, latest first, then the base entry */
        const uint32_t slot = (uint32_t)aux[j].pos2;
        if ((uint32_t)aux[j].pos1 != key) return MTE_E_INVALID_ARG;
        if (slot >= MTE_ANNOTATE_SLOTS) break;
        if ((AM(d, i) >> slot) & 1u) {
          val = aux[j].a;
          pk = (uint32_t)aux[j].seq;
          break;
        }
      }
      while (j < n_aux && (uint32_t)aux[j].pos2 < MTE_ANNOTATE_SLOTS) j++;  /* to the run's base entry */
      if (j >= n_aux) return MTE_E_INVALID_ARG;
      j++;
      g->props[key] = val;
      PK(d, i)[key] = pk;
      d->pwrites += 1;
    }
    AM(d, i) &= ~(1u << b);
    if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_ANNOTATE, lp, g->len, 0))) return rc;
    d->written += 1;
  }
  return MTE_OK;
}

/* MTE_OP_ROLLBACK (a local record): MergeTree.rollback of the pending op of
 * localSeq op->seq, type op->pos1 (mergeTree.ts:2005-2083).  Its inserted
 * segments get seq and removedSeq UniversalSequenceNumber (markRangeRemoved
 * at seq 0 by the local client: gone for every view, zamboni drops them);
 * its removed ones are restored.  Each segment's delta event comes at its
 * own-view position once it is done (findRollbackPosition :2088-2103). */
static int doc_rollback(odoc* d, const mte_op* op, const apply_env* env) {
  const int32_t ls = op->seq;
  int rc;
  if (!(ls > 0 && ls <= d->local_seq)) return MTE_E_INVALID_ARG;
  if (op->pos1 == MTE_OP_ANNOTATE) return doc_rollback_annotate(d, op, env);
  if (op->pos1 != MTE_OP_INSERT && op->pos1 != MTE_OP_REMOVE) return MTE_E_INVALID_ARG;
  d->ops++;
  d->scanned += d->n;
  int64_t lp = 0;
  for (uint32_t i = 0; i < d->n; lp += own_len(&d->s[i]), i++) {
    oseg* g = &d->s[i];
    if (op->pos1 == MTE_OP_INSERT && g->seq == LOCAL_BASE + ls) {
      g->seq = 0;
      g->rseq = 0;
      g->rmask = 1u;
      if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_REMOVE, lp, g->len, 1))) return rc;
      d->written += 1;
    } else if (op->pos1 == MTE_OP_REMOVE && g->rseq == LOCAL_BASE + ls) {
      g->rseq = NONE_SEQ;
      g->rmask = 0;
      if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_INSERT, lp, g->len, 0))) return rc;
      d->written += 1;
    }
  }
  return MTE_OK;
}

/* The length of a segment in the local client's view at localSeq ls
 * (localNetLength with localSeq and refSeq = currentSeq, mergeTree.ts:575-593):
 * an own pending insert after ls is not there yet, an own pending removal up to
 * ls is; a sequenced removal always is (removedSeq <= currentSeq). */
static inline int32_t len_at_local_seq(const oseg* g, int32_t ls) {
  if (is_pending(g->seq) && g->seq - LOCAL_BASE > ls) return 0;
  if (g->rseq != NONE_SEQ && (!is_pending(g->rseq) || g->rseq - LOCAL_BASE <= ls)) return 0;
  return g->len;
}

/* MTE_OP_REGEN (a local record): Client.regeneratePendingOp of the pending op
 * of localSeq op->seq, type op->pos1 (client.ts:972-1002 ->
 * resetPendingDeltaToOps :788-860).  Its segment group, sorted by ordinal
 * (document order), each at findReconnectionPosition (:709-713) -- the view at
 * that localSeq -- with its cachedLength, as MTE_DELTA_REGEN | type records:
 *   insert: every segment the op inserted (the record's removed field: its
 *     text offset);
 *   remove: only while the removal is still pending (a remote remove that
 *     overtook it leaves nothing to send, :839-845);
 *   annotate: the segments of group slot op->a not removed, or removed only by
 *     a pending local remove (:809-823).
 * The document itself does not change. */
static int doc_regen(odoc* d, const mte_op* op) {
  const int32_t ls = op->seq;
  const uint32_t t = (uint32_t)op->pos1;
  int rc;
  if (!(ls > 0 && ls <= d->local_seq)) return MTE_E_INVALID_ARG;
  if (t != MTE_OP_INSERT && t != MTE_OP_REMOVE && t != MTE_OP_ANNOTATE) return MTE_E_INVALID_ARG;
  if (t == MTE_OP_ANNOTATE && op->a >= MTE_ANNOTATE_SLOTS) return MTE_E_INVALID_ARG;
  if (!(d->flags & MTE_DOC_EVENTS)) return MTE_E_UNSUPPORTED;
  d->ops++;
  d->scanned += d->n;
  int64_t p = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const oseg* g = &d->s[i];
    int hit;
    if (t == MTE_OP_INSERT) hit = g->seq == LOCAL_BASE + ls;
    else if (t == MTE_OP_REMOVE) hit = g->rseq == LOCAL_BASE + ls;
    else hit = ((AM(d, i) >> op->a) & 1u) && (g->rseq == NONE_SEQ || is_pending(g->rseq));
    if (hit && (rc = delta_push(d, MTE_DELTA_REGEN | t, p, g->len, t == MTE_OP_INSERT ? g->toff : 0u))) return rc;
    p += len_at_local_seq(g, ls);
  }
  return MTE_OK;
}

/* MTE_OP_ACK: ackPendingSegment for the groups of localSeq pos1..pos2
 * (mergeTree.ts:1278-1331, BaseSegment.ack mergeTreeNodes.ts:475-503): a
 * pending insert takes the seq, a pending removal too unless a remote remove
 * overtook it (then removedSeq is already that op's, :1928-1938), and the
 * annotate's keys stop being pending (ackPendingProperties). */
static int doc_ack(odoc* d, const mte_op* op) {
  const int32_t lo = op->pos1, hi = op->pos2, s = op->seq;
  if (!(lo > 0 && lo <= hi && hi <= d->local_seq)) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < d->n; i++) {
    oseg* g = &d->s[i];
    if (g->seq >= LOCAL_BASE + lo && g->seq <= LOCAL_BASE + hi) g->seq = s;
    if (g->rseq >= LOCAL_BASE + lo && g->rseq <= LOCAL_BASE + hi) g->rseq = s;
    uint32_t* pk = PK(d, i);
    for (uint32_t k = 0; k < MTE_MAX_KEYS; k++)
      if (pk[k] && pk[k] <= (uint32_t)hi) pk[k] = 0;
    pk[MTE_MAX_KEYS] &= ~op->a; /* the acked annotates' groups */
  }
  return MTE_OK;
}

/* One op record.  Client.applyMsg -> applyRemoteOp (client.ts:918-935,
 * 862-889) -> updateSeqNumbers (937-945). */
static int doc_apply(odoc* d, const mte_op* op, const apply_env* env) {
  /* combiningOp incr / consensus: the HBM tree pass's restatement (titems.c) only */
  if (op->flags & MTE_F_COMBINE) return MTE_E_UNSUPPORTED;
  const int newcalc = (d->flags & MTE_DOC_NEW_LENGTH_CALC) != 0;
  const int32_t r = op->ref_seq, s = op->seq, m = d->min_seq;
  const int c = op->client;
  const int local_doc = (d->flags & MTE_DOC_LOCAL_CLIENT) != 0;
  int rc;
  if (c >= MTE_MAX_CLIENTS) return MTE_E_CLIENT_RANGE;
  if (op->flags & MTE_F_LOCAL) return local_doc ? doc_apply_local(d, op, env) : MTE_E_UNSUPPORTED;
  if (op->type == MTE_OP_ACK && !local_doc) return MTE_E_UNSUPPORTED;
  if (local_doc && op->type != MTE_OP_ACK && op->type != MTE_OP_NOOP && c == 0) return MTE_E_INVALID_ARG;
  d->ops++;
  if (d->n > d->max_segs) d->max_segs = d->n;
  if (op->type != MTE_OP_NOOP) d->scanned += d->n;

  if (op->type == MTE_OP_INSERT) {
    /* applyInsertOp (client.ts:470-505) -> insertSegments (mergeTree.ts:1394-1422) */
    if ((rc = doc_scratch(d))) return rc;
    int64_t total = doc_lengths(d, r, c, m, newcalc);
    int64_t pos = op->pos1;
    int64_t tail = doc_split_at(d, pos, &d->written); /* ensureIntervalBoundary */
    if (tail == -2) return MTE_E_OOM;
    const int is_marker = (op->flags & MTE_F_MARKER) != 0;
    int32_t len = is_marker ? 1 : op->pos2;
    if (len > 0) { /* blockInsert skips zero-length segments, mergeTree.ts:1645 */
      /* insertingWalk + breakTie (mergeTree.ts:1723-1825, 1705-1721): the new
       * segment goes before the first defined leaf whose prefix equals pos
       * (a zero-length leaf at pos ties in favour of the newer seq), else at
       * the end; undefined leaves are skipped.  pos > length fails
       * (mergeTree.ts:1666-1672). */
      uint32_t at = d->n;
      if (tail >= 0) {
        at = (uint32_t)tail;
      } else {
        /* a pending local segment (zero-length for every remote view) is
         * passed over: breakTie normalises its seq to MAX_SAFE_INTEGER - 1
         * (mergeTree.ts:1714), and at a block's end continuePredicate's
         * forward excursion moves on when it comes next (:1599-1611, 1790) */
        for (uint32_t i = 0; i < d->n; i++) {
          if (d->L[i] >= 0 && d->P[i] >= pos && !(local_doc && is_pending(d->s[i].seq))) { at = i; break; }
        }
        if (at == d->n && pos > total) return MTE_E_INSERT_FAILED;
      }
      if ((rc = doc_open(d, at, 1))) return rc;
      oseg* ns = &d->s[at];
      memset(ns, 0, sizeof(*ns));
      ns->len = len;
      ns->seq = s;
      ns->cli = c;
      ns->rseq = NONE_SEQ;
      ns->rmask = 0;
      if (is_marker) {
        ns->kind = 1u + (uint32_t)op->pos2;
        ns->toff = (d->flags & MTE_DOC_REFS) ? (uint32_t)(env->text_base + op->a) : 0u; /* its reserved unit */
      } else {
        ns->kind = 0;
        ns->toff = (uint32_t)(env->text_base + op->a);
        d->units += (uint64_t)len;
      }
      if (op->b != MTE_NO_PROPS)
        d->pwrites += orc_apply_props(ns->props, env->n_keys, &env->b->propsets[op->b], env->b->props, 0);
      d->written += 1;
      if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_INSERT, own_prefix(d, at), len, 0))) return rc;
    } else if ((d->flags & MTE_DOC_EVENTS) && (rc = delta_push(d, MTE_OP_INSERT, -1, 0, 0))) {
      return rc;  /* a zero-length segment is reported unlinked (getPosition -1) */
    }
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_REMOVE || op->type == MTE_OP_ANNOTATE) {
    /* markRangeRemoved (mergeTree.ts:1908-2000) / annotateRange (1864-1906):
     * two ensureIntervalBoundary, then nodeMap (2274-2330) visits the leaves
     * with len > 0 overlapping [start, end). */
    if ((rc = doc_scratch(d))) return rc;
    int64_t start = op->pos1, end = op->pos2;
    doc_lengths(d, r, c, m, newcalc);
    if (doc_split_at(d, start, &d->written) == -2) return MTE_E_OOM;
    if (doc_split_at(d, end, &d->written) == -2) return MTE_E_OOM;
    if (end != start) {
      int64_t lp = 0; /* the own view's prefix after the op, for the events */
      const int ev = (d->flags & MTE_DOC_EVENTS) != 0;
      for (uint32_t i = 0; i < d->n; lp += own_len(&d->s[i]), i++) {
        int32_t l = d->L[i];
        if (l <= 0) continue;
        if (d->P[i] >= end) break;
        if (d->P[i] + l <= start) continue;
        oseg* g = &d->s[i];
        if (ev && (op->type == MTE_OP_ANNOTATE || g->rseq == NONE_SEQ) &&
            (rc = delta_push(d, op->type, lp, g->len, op->type == MTE_OP_REMOVE || g->rseq != NONE_SEQ)))
          return rc; /* a remove reports the segments it newly removes (removedSegments) */
        if (op->type == MTE_OP_REMOVE) {
          /* markRemoved closure (mergeTree.ts:1924-1962): keep the earlier
           * removedSeq and add the client to removedClientIds (1939-1942). */
          if (g->rseq == NONE_SEQ) {
            g->rseq = s;
            g->rmask = 1u << c;
          } else {
            /* overtaking our pending removal: this op's seq becomes the
             * removedSeq (1928-1938) */
            if (is_pending(g->rseq)) g->rseq = s;
            g->rmask |= 1u << c;
          }
        } else if (local_doc) {
          d->pwrites += apply_props_pending(g->props, PK(d, i), env->n_keys, &env->b->propsets[op->a],
                                            env->b->props, (op->flags & MTE_F_REWRITE) != 0);
        } else {
          d->pwrites += orc_apply_props(g->props, env->n_keys, &env->b->propsets[op->a], env->b->props,
                                    (op->flags & MTE_F_REWRITE) != 0);
        }
        d->written += 1;
      }
    }
    if (op->type == MTE_OP_REMOVE) doc_slide_refs(d, s);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type == MTE_OP_ACK) {
    if ((rc = doc_ack(d, op))) return rc;
    doc_slide_refs(d, s);
    if ((rc = check_op_window(d, op))) return rc;
  } else if (op->type != MTE_OP_NOOP) {
    return MTE_E_INVALID_ARG;
  }

  if (op->flags & MTE_F_MSG_END) {
    /* updateSeqNumbers (client.ts:937-945) -> setMinSeq (mergeTree.ts:1077-1093) */
    if (!(d->cur_seq <= s)) return MTE_E_SEQ_ORDER;          /* 0x038 */
    d->cur_seq = s;
    if (!(op->min_seq <= s)) return MTE_E_MSN_GT_SEQ;        /* 0x039 / 0x04e */
    if (!(d->min_seq <= op->min_seq)) return MTE_E_MSN_ORDER; /* 0x04f */
    if (op->min_seq > d->min_seq) {
      d->min_seq = op->min_seq;
      doc_compact(d);
    }
  }
  return MTE_OK;
}

/* ------------------------------------------------------------------------ */

int orc_create(uint32_t n_keys, orc_ctx** out) {
  if (!out || n_keys > MTE_MAX_KEYS) return MTE_E_INVALID_ARG;
  orc_ctx* c = (orc_ctx*)calloc(1, sizeof(orc_ctx));
  if (!c) return MTE_E_OOM;
  c->n_keys = n_keys;
  *out = c;
  return MTE_OK;
}

static void free_docs(orc_ctx* c) {
  for (uint32_t i = 0; i < c->n_docs; i++) {
    free(c->docs[i].s);
    free(c->docs[i].L);
    free(c->docs[i].P);
    free(c->docs[i].pk);
    free(c->docs[i].dl);
    free(c->docs[i].ref_anchor);
    free(c->docs[i].ref_state);
  }
  free(c->docs);
  c->docs = NULL;
  c->n_docs = 0;
  free(c->load_ps);
  free(c->load_pe);
  c->load_ps = NULL;
  c->load_pe = NULL;
  c->n_load_ps = c->n_load_pe = 0;
}

int orc_destroy(orc_ctx* c) {
  if (!c) return MTE_E_INVALID_ARG;
  free_docs(c);
  free(c->arena);
  free(c);
  return MTE_OK;
}

int orc_load_docs(orc_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props) {
  (void)n_props;
  if (!c || (n_docs && !docs)) return MTE_E_INVALID_ARG;
  free_docs(c);
  c->arena_n = 0;
  uint64_t base = 0;
  int rc = arena_append(c, text, text_units, &base);
  if (rc) return rc;
  c->docs = (odoc*)aligned_alloc(128, (size_t)(n_docs ? n_docs : 1) * sizeof(odoc));
  if (c->docs) memset(c->docs, 0, (size_t)(n_docs ? n_docs : 1) * sizeof(odoc));
  if (!c->docs) return MTE_E_OOM;
  c->n_docs = n_docs;
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
    odoc* d = &c->docs[i];
    const mte_doc_init* in = &docs[i];
    if ((uint64_t)in->text_off + in->text_len > text_units) return MTE_E_INVALID_ARG;
    d->init = *in;
    d->flags = in->flags;
    if ((in->flags & (MTE_DOC_LOCAL_CLIENT | MTE_DOC_EVENTS)) && !(in->flags & MTE_DOC_NEW_LENGTH_CALC))
      return MTE_E_UNSUPPORTED;
    if ((in->flags & MTE_DOC_REFS) && !(in->flags & MTE_DOC_LOCAL_CLIENT)) return MTE_E_UNSUPPORTED;
    d->min_seq = in->min_seq;
    d->cur_seq = in->cur_seq;
    d->rs_ref = INT32_MIN;
    d->rs_seq = in->cur_seq;
    if (in->text_len > 0) {
      if ((rc = doc_reserve(d, 64))) return rc;
      oseg* g = &d->s[0];
      memset(g, 0, sizeof(*g));
      g->len = (int32_t)in->text_len;
      g->seq = 0;   /* UniversalSequenceNumber */
      g->cli = -1;  /* LocalClientId */
      g->rseq = NONE_SEQ;
      g->toff = (uint32_t)(base + in->text_off);
      if (d->pk) memset(PK(d, 0), 0, PKW * sizeof(uint32_t));
      if (in->propset != MTE_NO_PROPS) {
        if (in->propset >= n_propsets) return MTE_E_INVALID_ARG;
        orc_apply_props(g->props, c->n_keys, &propsets[in->propset], props, 0);
      }
      d->n = 1;
    }
  }
  return MTE_OK;
}

/* Snapshot body -> segments with their merge info (SnapshotLoader.loadBody,
 * snapshotLoader.ts:85-125; IJSONSegmentWithMergeInfo, snapshotChunks.ts:48-78):
 * seq, clientId, removedSeq and removedClientIds are taken as given. */
int orc_load_segments(orc_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs) {
  if (!c || !seg_offsets || (n_segs && !segs)) return MTE_E_INVALID_ARG;
  if (seg_offsets[0] != 0 || seg_offsets[c->n_docs] != n_segs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < c->n_docs; i++) {
    const uint64_t b = seg_offsets[i], e = seg_offsets[i + 1];
    if (e < b) return MTE_E_INVALID_ARG;
    if (e == b) continue;
    odoc* d = &c->docs[i];
    int rc = doc_reserve(d, (uint32_t)(e - b) + 64);
    if (rc) return rc;
    for (uint64_t k = b; k < e; k++) {
      const mte_seg* sg = &segs[k];
      const int marker = sg->kind != 0;
      if ((marker && sg->len != 1) || (!marker && (sg->len == 0 || (uint64_t)sg->text_off + sg->len > c->load_units)) ||
          sg->client < -1 || sg->client >= MTE_MAX_CLIENTS || sg->seq < 0 ||
          (sg->removed_seq != MTE_NOT_REMOVED && sg->removers == 0))
        return MTE_E_INVALID_ARG;
      oseg* g = &d->s[k - b];
      memset(g, 0, sizeof(*g));
      if (d->pk) memset(PK(d, k - b), 0, PKW * sizeof(uint32_t));
      g->len = (int32_t)sg->len;
      g->seq = sg->seq;
      g->cli = sg->client;
      g->rseq = sg->removed_seq == MTE_NOT_REMOVED ? NONE_SEQ : sg->removed_seq;
      g->rmask = sg->removed_seq == MTE_NOT_REMOVED ? 0u : sg->removers;
      g->kind = sg->kind;
      /* a marker of an MTE_DOC_REFS document is named by its index in the load
       * (above every arena offset), as an inserted one by its reserved unit */
      g->toff = marker ? ((d->flags & MTE_DOC_REFS) ? 0x80000000u + (uint32_t)(k - b) : 0u) : sg->text_off;
      if (sg->propset != MTE_NO_PROPS) {
        if (sg->propset >= c->n_load_ps) return MTE_E_INVALID_ARG;
        orc_apply_props(g->props, c->n_keys, &c->load_ps[sg->propset], c->load_pe, 0);
      }
    }
    d->n = (uint32_t)(e - b);
  }
  return MTE_OK;
}

typedef struct {
  orc_ctx* c;
  const mte_batch* b;
  uint64_t base;
  uint32_t d0, d1, stride;
} worker_arg;

/* MTE_DOC_ROUND_SYNC (include/mte.h) on a legacy-calc document: the batch's
 * live ops keep refSeq non-decreasing and each increase reaches every earlier
 * live op's seq (the load's currentSeq included).  Checked before the batch
 * applies; a violation stops the document with MTE_E_UNSUPPORTED. */
static int round_sync_ok(odoc* d, const mte_op* ops, uint64_t k0, uint64_t k1) {
  int32_t ref = d->rs_ref, seq = d->rs_seq;
  for (uint64_t k = k0; k < k1; k++) {
    const mte_op* o = &ops[k];
    if (o->type == MTE_OP_NOOP || o->type == MTE_OP_RELPOS) continue;
    if (o->ref_seq < ref) return 0;
    if (o->ref_seq > ref) {
      if (o->ref_seq < seq) return 0;
      ref = o->ref_seq;
    }
    if (o->seq > seq) seq = o->seq;
  }
  d->rs_ref = ref;
  d->rs_seq = seq;
  return 1;
}

static void* worker(void* p) {
  worker_arg* w = (worker_arg*)p;
  apply_env env = {w->b, w->base, w->c->n_keys, w->c->arena, NULL};
  for (uint32_t di = w->d0; di < w->d1; di += w->stride) {
    odoc* d = &w->c->docs[di];
    if (d->status) continue;
    if ((d->flags & (MTE_DOC_ROUND_SYNC | MTE_DOC_NEW_LENGTH_CALC)) == MTE_DOC_ROUND_SYNC &&
        !round_sync_ok(d, w->b->ops, w->b->op_offsets[di], w->b->op_offsets[di + 1])) {
      d->status = MTE_E_UNSUPPORTED;
      continue;
    }
    d->dl_n = 0;
    for (uint64_t k = w->b->op_offsets[di]; k < w->b->op_offsets[di + 1]; k++) {
      const mte_op* op = &w->b->ops[k];
      mte_op nx;
      int rc = 0;
      if (op->type == MTE_OP_RELPOS) {  /* the next record, at the resolved positions */
        nx = op[1];
        rc = doc_relpos(d, op, &nx, env.n_keys);
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
      if (op->type == MTE_OP_ROLLBACK && op->pos1 == MTE_OP_ANNOTATE) k += (uint64_t)op->pos2;  /* its RBKEY records */
    }
  }
  return NULL;
}

int orc_apply_batch(orc_ctx* c, const mte_batch* b, int n_threads) {
  if (!c || !b || b->n_docs != c->n_docs || !b->op_offsets) return MTE_E_INVALID_ARG;
  if (b->op_offsets[b->n_docs] != b->n_ops) return MTE_E_INVALID_ARG;
  uint32_t dcur = 0;
  uint64_t rbkey_end = 0;  /* records up to here are an annotate rollback's MTE_OP_RBKEY */
  for (uint64_t k = 0; k < b->n_ops; k++) {
    const mte_op* op = &b->ops[k];
    while (dcur + 1 < b->n_docs && b->op_offsets[dcur + 1] <= k) dcur++;
    /* local records (as mte_submit validates them) */
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
    if (op->type == MTE_OP_INSERT && op->b != MTE_NO_PROPS && op->b >= b->n_propsets)
      return MTE_E_INVALID_ARG;
    if (op->type == MTE_OP_ANNOTATE && op->a >= b->n_propsets) return MTE_E_INVALID_ARG;
  }
  uint64_t base = 0;
  int rc = arena_append(c, b->text, b->text_units, &base);
  if (rc) return rc;
  /* stats describe the last batch, like mte_stats_get */
  for (uint32_t i = 0; i < c->n_docs; i++) {
    odoc* d = &c->docs[i];
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
  for (int t = 0; t < n_threads; t++) {
    args[t] = (worker_arg){c, b, base, (uint32_t)t, c->n_docs, (uint32_t)n_threads};
  }
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

int orc_read_doc(orc_ctx* c, uint32_t doc, mte_doc_view* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  odoc* d = &c->docs[doc];
  v->status = d->status;
  v->cur_seq = d->cur_seq;
  v->min_seq = d->min_seq;
  uint32_t length = 0, nt = 0, ns = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const oseg* g = &d->s[i];
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
        if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
        nt++;
      }
    }
  }
  v->length = length;
  v->n_text = nt;
  v->n_segs = ns;
  return MTE_OK;
}

int orc_read_segments(orc_ctx* c, uint32_t doc, mte_seg_list* v) {
  if (!c || !v || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  odoc* d = &c->docs[doc];
  uint64_t nt = 0;
  for (uint32_t i = 0; i < d->n; i++) {
    const oseg* g = &d->s[i];
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
        if (nt < v->text_cap && v->text) v->text[nt] = c->arena[g->toff + (uint32_t)u];
  }
  v->n_segs = d->n;
  v->n_text = nt;
  return MTE_OK;
}

/* ---- canonical digest (DESIGN.md "Digest", orc_common.h) ------------------ */
int orc_digest(orc_ctx* c, uint64_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t di = 0; di < n_docs; di++) {
    odoc* d = &c->docs[di];
    orc_digest_acc acc = {0, 0, 0, 0};
    for (uint32_t i = 0; i < d->n; i++) {
      const oseg* g = &d->s[i];
      if (g->rseq != NONE_SEQ) continue;
      orc_digest_seg(&acc, g->kind, g->kind == 0 ? c->arena + g->toff : NULL, g->len, g->props, c->n_keys);
    }
    const uint64_t n = acc.n, h1 = acc.h1, h2 = acc.h2, sum = acc.sum;
    out[4 * (size_t)di + 0] = n;
    out[4 * (size_t)di + 1] = h1;
    out[4 * (size_t)di + 2] = h2;
    out[4 * (size_t)di + 3] = sum;
  }
  return MTE_OK;
}

int orc_doc_status(orc_ctx* c, int32_t* out, uint32_t n_docs) {
  if (!c || !out || n_docs != c->n_docs) return MTE_E_INVALID_ARG;
  for (uint32_t i = 0; i < n_docs; i++) out[i] = c->docs[i].status;
  return MTE_OK;
}

int orc_stats_get(orc_ctx* c, mte_stats* o) {
  if (!c || !o) return MTE_E_INVALID_ARG;
  memset(o, 0, sizeof(*o));
  for (uint32_t i = 0; i < c->n_docs; i++) {
    odoc* d = &c->docs[i];
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

int orc_doc_nsegs(orc_ctx* c, uint32_t doc, uint32_t* out) {
  if (!c || !out || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  *out = c->docs[doc].n;
  return MTE_OK;
}

int orc_read_deltas(orc_ctx* c, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const odoc* d = &c->docs[doc];
  *n = d->dl_n;
  if (out) memcpy(out, d->dl, (size_t)(cap < d->dl_n ? cap : d->dl_n) * sizeof(mte_delta));
  return MTE_OK;
}

/* referencePositionToLocalPosition (mergeTree.ts:1095-1112) of slots [0, n):
 * the own-view position of the segment holding the reference's unit plus its
 * offset there (0 on a removed segment); -1 for a detached or unused slot or a
 * unit no segment holds any more. */
/* mte_read_ref_order: the index, among every unit the document holds, of the
 * unit each reference sits on (-1 detached / unused) */
int orc_read_ref_order(orc_ctx* c, uint32_t doc, int64_t* key, uint32_t n) {
  if (!c || (n && !key) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const odoc* d = &c->docs[doc];
  for (uint32_t r = 0; r < n; r++) {
    key[r] = -1;
    if (r >= d->ref_hi) continue;
    const uint32_t st = d->ref_state[r], u = d->ref_anchor[r];
    if (!(st & REF_LIVE) || ((st & REF_DETACHED) && !(st & REF_OFF))) continue; /* off the string: on its segment */
    int64_t p = 0;
    for (uint32_t i = 0; i < d->n; i++) {
      const oseg* g = &d->s[i];
      if (u - g->toff < (uint32_t)g->len) {
        key[r] = p + (int64_t)(u - g->toff);
        break;
      }
      p += g->len;
    }
  }
  return MTE_OK;
}

static int read_refs_view(orc_ctx* c, uint32_t doc, int32_t* pos, uint32_t n, int transient) {
  if (!c || (n && !pos) || doc >= c->n_docs) return MTE_E_INVALID_ARG;
  const odoc* d = &c->docs[doc];
  for (uint32_t r = 0; r < n; r++) {
    pos[r] = -1;
    if (r >= d->ref_hi) continue;
    const uint32_t st = d->ref_state[r], u = d->ref_anchor[r];
    if (!(st & REF_LIVE) || ((st & REF_DETACHED) && !(transient && (st & REF_OFF)))) continue;
    int64_t p = 0;
    for (uint32_t i = 0; i < d->n; i++) {
      const oseg* g = &d->s[i];
      if (u - g->toff < (uint32_t)g->len) {
        pos[r] = (int32_t)(p + (g->rseq != NONE_SEQ ? 0 : (int64_t)(u - g->toff)));
        break;
      }
      p += own_len(g);
    }
  }
  return MTE_OK;
}

int orc_read_refs(orc_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) { return read_refs_view(c, doc, pos, n, 0); }

/* mte_read_refs_transient: as orc_read_refs with every reference Transient
 * (emitChange, intervalCollection.ts:1387-1410): a reference taken off its
 * segment's list still finds the segment while it is held */
int orc_read_refs_transient(orc_ctx* c, uint32_t doc, int32_t* pos, uint32_t n) {
  return read_refs_view(c, doc, pos, n, 1);
}
