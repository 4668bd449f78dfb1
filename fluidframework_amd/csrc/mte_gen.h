/*
 * mte_gen.h — seeded synthetic op streams for the benchmark configs
 * (SURVEY.md 8(d)).  CPU tooling that produces engine *inputs*; it is not on
 * the replay path and not a checker.
 *
 * Stream model, following the reference conflict farm
 * (test/mergeTreeOperationRunner.ts:149-199, test/client.conflictFarm.spec.ts):
 * rounds of R ops whose refSeq == msn == the round's start seq (or, with
 * max_lag, per-client lagging refSeqs and msn = their minimum); the author of
 * each op is uniform among C clients; positions are drawn from the author's
 * perspective length; below minLength the op is an insert of the author's
 * name repeated 1-3 times.  PRNG: MT19937 init_by_array([0xDEADBEEF,
 * 0xFEEDBED, config_id, doc_index]).  random-js (the reference's generator,
 * not vendored) is not reproduced: the streams are "parity-unpinned" inputs;
 * parity is engine vs oracle on the same stream.
 */
#ifndef MTE_GEN_H_
#define MTE_GEN_H_

#include "../../include/mte.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MTEG_MIX_INSERT 0x1u
#define MTEG_MIX_REMOVE 0x2u
#define MTEG_MIX_ANNOTATE 0x4u

/* property planes used by generated streams */
#define MTEG_KEY_CLIENT 0
#define MTEG_KEY_BOLD 1
#define MTEG_KEY_COLOR 2
#define MTEG_KEY_MARKER_ID 3
#define MTEG_N_KEYS 4

typedef struct mteg_config {
  uint32_t config_id;    /* seed word 3                                 */
  uint32_t n_docs;
  uint32_t ops_per_doc;
  uint32_t doc_base;     /* global index of doc 0 (seed word 4)         */
  uint32_t clients;      /* authors, observer excluded (1..31)          */
  uint32_t min_length;
  uint32_t round_ops;    /* R                                           */
  uint32_t mix;          /* MTEG_MIX_*                                  */
  uint32_t marker_every; /* 1 in N inserts is a marker (0 = none)       */
  uint32_t length_mode;  /* 0: per doc 50/50, 1: all legacy, 2: all new */
  uint32_t init_len;     /* initial text units per doc                  */
  uint32_t n_threads;
  uint32_t init_segs;    /* > 0: preload this many one-unit segments per doc
                            (mte_load_segments) and use the long-doc generator */
  uint32_t max_range;    /* remove / annotate span cap (0 = farm rule)     */
  uint32_t max_lag;      /* 0: rounds (refSeq == msn == round start).  > 0:
                            every client keeps its own refSeq, which moves up
                            to a seq in [seq - max_lag, seq - 1] when it sends;
                            msn = the minimum over the clients (the sequencer
                            rule, deli clientSeqManager.ts:130-137), so ops
                            see each other's concurrent edits partially */
  uint32_t newline_every; /* 1 in N inserted texts holds a '\n' (0 = none) */
  const uint32_t* doc_ids; /* NULL: doc d is global doc doc_base + d; else the
                              global index of doc d (seed word 4), e.g. a
                              rank's shard from a work-balanced assignment   */
} mteg_config;

typedef struct mteg_stream mteg_stream;

typedef struct mteg_sizes {
  uint64_t n_ops;
  uint64_t text_units;     /* batch text                              */
  uint64_t init_units;     /* load text                               */
  uint32_t n_propsets;
  uint32_t n_props;
} mteg_sizes;

int mteg_generate(const mteg_config* cfg, mteg_stream** out);
int mteg_get_sizes(const mteg_stream* s, mteg_sizes* out);
/* Copy out.  Arrays sized per mteg_get_sizes; op_offsets has n_docs+1. */
int mteg_fill(const mteg_stream* s, mte_doc_init* inits, uint16_t* init_text,
              uint64_t* op_offsets, mte_op* ops, uint16_t* text,
              mte_propset* propsets, mte_prop* props);
int mteg_free(mteg_stream* s);

/* Canonical JSON of a generated value id into buf (NUL-terminated).  Returns
 * the length, or -1 if unknown / too small. */
int mteg_value_json(uint32_t value_id, char* buf, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif
