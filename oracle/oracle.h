/*
 * oracle.h — CPU restatement of the reference merge-tree observer replay.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libmte.so) never links,
 * loads or calls it.
 *
 * Pinning: the restatement is checked against all 1,920 round checkpoints of
 * the 30 golden replay fixtures of the reference
 * (packages/dds/merge-tree/src/test/results/ JSON files, replayed as in
 * test/client.replay.spec.ts:16-60) and against known-answer scenarios
 * transcribed from test/client.applyMsg.spec.ts, mergeTree.markRangeRemoved
 * .spec.ts and mergeTree.annotate.spec.ts (tests/test_oracle_*.py).
 *
 * It takes the same op records / batches as include/mte.h.
 */
#ifndef MTE_ORACLE_H_
#define MTE_ORACLE_H_

#include "../include/mte.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_ctx orc_ctx;

int orc_create(uint32_t n_keys, orc_ctx** out);
int orc_destroy(orc_ctx* c);
int orc_load_docs(orc_ctx* c, uint32_t n_docs, const mte_doc_init* docs,
                  const uint16_t* text, uint64_t text_units,
                  const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props);
/* Replace docs' loaded content with segment lists (as mte_load_segments). */
int orc_load_segments(orc_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs);
/* Apply a batch immediately, docs spread over n_threads pthreads. */
int orc_apply_batch(orc_ctx* c, const mte_batch* b, int n_threads);
int orc_read_doc(orc_ctx* c, uint32_t doc, mte_doc_view* v);
/* Delta events of the last batch of an MTE_DOC_EVENTS doc (as mte_read_deltas, no cap). */
int orc_read_deltas(orc_ctx* c, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n);
int orc_read_refs(orc_ctx* c, uint32_t doc, int32_t* pos, uint32_t n);
int orc_read_refs_transient(orc_ctx* c, uint32_t doc, int32_t* pos, uint32_t n);
int orc_read_ref_order(orc_ctx* c, uint32_t doc, int64_t* key, uint32_t n);
int orc_read_segments(orc_ctx* c, uint32_t doc, mte_seg_list* v);
int orc_digest(orc_ctx* c, uint64_t* out, uint32_t n_docs);
int orc_doc_status(orc_ctx* c, int32_t* out, uint32_t n_docs);
int orc_stats_get(orc_ctx* c, mte_stats* out);
/* Segments currently held by a doc (canonical model: tombstones included). */
int orc_doc_nsegs(orc_ctx* c, uint32_t doc, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
