/*
 * chunked.h — the flat restatement with a chunk index (chunked.c), for
 * documents of millions of segments (config 5).  TEST INFRASTRUCTURE ONLY
 * (same rules as oracle.h).  New length-calc observer documents only.
 */
#ifndef MTE_ORACLE_CHUNKED_H_
#define MTE_ORACLE_CHUNKED_H_

#include "../include/mte.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct och_ctx och_ctx;

int och_create(uint32_t n_keys, och_ctx** out);
int och_destroy(och_ctx* c);
int och_load_docs(och_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props);
int och_load_segments(och_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs);
int och_apply_batch(och_ctx* c, const mte_batch* b, int n_threads);
int och_read_doc(och_ctx* c, uint32_t doc, mte_doc_view* v);
int och_digest(och_ctx* c, uint64_t* out, uint32_t n_docs);
int och_doc_status(och_ctx* c, int32_t* out, uint32_t n_docs);
int och_doc_nsegs(och_ctx* c, uint32_t doc, uint32_t* out);
int och_read_segments(och_ctx* c, uint32_t doc, mte_seg_list* v);
int och_stats_get(och_ctx* c, mte_stats* out);

#ifdef __cplusplus
}
#endif
#endif
