/*
 * orc_common.h — pieces shared by the two CPU restatements (TEST INFRASTRUCTURE):
 * oracle.c (flat) and tree.c (tree-exact).  The canonical digest (DESIGN.md
 * "Digest") and the remote-observer PropertiesManager.addProperties.
 */
#ifndef MTE_ORC_COMMON_H_
#define MTE_ORC_COMMON_H_

#include <stdint.h>

#include "../include/mte.h"

#define ORC_NONE_SEQ INT32_MAX /* "removedSeq undefined" */

/* ---- canonical digest --------------------------------------------------- */
#define ORC_M61 ((1ull << 61) - 1)
static const uint64_t ORC_DIG_B1 = 0x1d8e4e27c47d124full % ((1ull << 61) - 1);
static const uint64_t ORC_DIG_B2 = 0x0a0761d6478bd642ull % ((1ull << 61) - 1);

static inline uint64_t orc_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline uint64_t orc_mulmod61(uint64_t a, uint64_t b) {
  unsigned __int128 p = (unsigned __int128)a * b;
  uint64_t lo = (uint64_t)(p & ORC_M61), hi = (uint64_t)(p >> 61);
  uint64_t r = lo + hi;
  if (r >= ORC_M61) r -= ORC_M61;
  return r;
}
static inline uint64_t orc_addmod61(uint64_t a, uint64_t b) {
  uint64_t r = a + b;
  if (r >= ORC_M61) r -= ORC_M61;
  return r;
}

/* running digest state of one document */
typedef struct {
  uint64_t n, h1, h2, sum;
} orc_digest_acc;

/* feed one visible segment: `units` (text) or a marker of `kind` (1 + refType) */
static inline void orc_digest_seg(orc_digest_acc* a, uint32_t kind, const uint16_t* units, int32_t len,
                                  const uint32_t* props, uint32_t n_keys) {
  uint64_t ph = 0;
  for (uint32_t k = 0; k < n_keys; k++)
    if (props[k]) ph += orc_mix64(((uint64_t)(k + 1) << 32) | props[k]);
  for (int32_t u = 0; u < len; u++) {
    uint64_t rec = kind == 0 ? (uint64_t)units[u] : ((1ull << 32) | (uint64_t)(kind - 1));
    uint64_t x = orc_mix64(rec * 0x9E3779B97F4A7C15ull + ph) % ORC_M61;
    a->h1 = orc_addmod61(orc_mulmod61(a->h1, ORC_DIG_B1), x);
    a->h2 = orc_addmod61(orc_mulmod61(a->h2, ORC_DIG_B2), x);
    a->sum += x;
    a->n++;
  }
}

/* PropertiesManager.addProperties for a remote observer (collaborating, no
 * pending local keys, so shouldModifyKey is true for every key):
 * segmentPropertiesManager.ts:63-151.  rewrite first clears the keys not in
 * newProps (105-119); then null deletes, anything else sets (121-148).  The
 * falsy-value test of the rewrite loop cancels against the set loop, so the net
 * effect is "clear all, then apply". */
static inline uint64_t orc_apply_props(uint32_t* props, uint32_t n_keys, const mte_propset* ps,
                                       const mte_prop* pe, int rewrite) {
  uint64_t w = 0;
  if (rewrite) {
    for (uint32_t k = 0; k < n_keys; k++) props[k] = 0;
  }
  for (uint32_t j = 0; j < ps->count; j++) {
    const mte_prop* p = &pe[ps->first + j];
    if (p->key < n_keys) {
      props[p->key] = p->value; /* value 0 == null == delete */
      w++;
    }
  }
  return w;
}

#endif
