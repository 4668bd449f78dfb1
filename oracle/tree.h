/*
 * tree.h — tree-exact CPU restatement of merge-tree observer replay (tree.c).
 *
 * TEST INFRASTRUCTURE ONLY, like oracle.h: tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, only as a checker / timed baseline.
 * Same calls and records as oracle.h (and include/mte.h), prefix ort_.
 */
#ifndef MTE_ORACLE_TREE_H_
#define MTE_ORACLE_TREE_H_

#include "../include/mte.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ort_ctx ort_ctx;

int ort_create(uint32_t n_keys, ort_ctx** out);
int ort_destroy(ort_ctx* c);
int ort_load_docs(ort_ctx* c, uint32_t n_docs, const mte_doc_init* docs, const uint16_t* text,
                  uint64_t text_units, const mte_propset* propsets, uint32_t n_propsets,
                  const mte_prop* props, uint32_t n_props);
int ort_load_segments(ort_ctx* c, const uint64_t* seg_offsets, const mte_seg* segs, uint64_t n_segs);
int ort_apply_batch(ort_ctx* c, const mte_batch* b, int n_threads);
int ort_read_doc(ort_ctx* c, uint32_t doc, mte_doc_view* v);
int ort_read_segments(ort_ctx* c, uint32_t doc, mte_seg_list* v);
int ort_digest(ort_ctx* c, uint64_t* out, uint32_t n_docs);
int ort_doc_status(ort_ctx* c, int32_t* out, uint32_t n_docs);
int ort_stats_get(ort_ctx* c, mte_stats* out);
int ort_doc_nsegs(ort_ctx* c, uint32_t doc, uint32_t* out);
/* shape string of a doc's tree; returns the LRU heap size */
int ort_doc_shape(ort_ctx* c, uint32_t doc, char* buf, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif
