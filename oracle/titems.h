/*
 * titems.h — the reference B+tree on a flat item array (titems.c): the
 * executable spec of the GPU tree pass.  TEST INFRASTRUCTURE ONLY (same rules
 * as oracle.h).  Same calls as oracle.h, prefix oti_.
 */
#ifndef MTE_ORACLE_TITEMS_H_
#define MTE_ORACLE_TITEMS_H_

#include "../include/mte.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oti_ctx oti_ctx;

int oti_create(uint32_t n_keys, oti_ctx** out);
int oti_destroy(oti_ctx* c);
int oti_load_docs(oti_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props);
int oti_load_segments(oti_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs);
int oti_apply_batch(oti_ctx* c, const mte_batch* b, int n_threads);
int oti_read_doc(oti_ctx* c, uint32_t doc, mte_doc_view* v);
int oti_digest(oti_ctx* c, uint64_t* out, uint32_t n_docs);
int oti_doc_status(oti_ctx* c, int32_t* out, uint32_t n_docs);
int oti_doc_nsegs(oti_ctx* c, uint32_t doc, uint32_t* out);
int oti_doc_shape(oti_ctx* c, uint32_t doc, char* buf, uint32_t cap);
int oti_stats_get(oti_ctx* c, mte_stats* out);
/* a document stops with MTE_E_CAPACITY once items + 4 > limit (default 1024) */
int oti_set_limit(oti_ctx* c, uint32_t limit);
int oti_read_segments(oti_ctx* c, uint32_t doc, mte_seg_list* v);
int oti_read_deltas(oti_ctx* c, uint32_t doc, mte_delta* out, uint64_t cap, uint64_t* n);
int oti_read_refs(oti_ctx* c, uint32_t doc, int32_t* pos, uint32_t n);
int oti_read_refs_transient(oti_ctx* c, uint32_t doc, int32_t* pos, uint32_t n);
int oti_read_ref_order(oti_ctx* c, uint32_t doc, int64_t* key, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
