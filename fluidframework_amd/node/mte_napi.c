/*
 * mte_napi.c — Node N-API addon over the C-ABI of libmte.so (include/mte.h).
 *
 * This is the "thin C-ABI exposed as a Node N-API addon" of BASELINE.json's
 * north star: the JavaScript host layer (index.js, BatchClient) packs
 * ISequencedDocumentMessage objects into 32-byte op records and hands them to
 * the engine through these functions.  Every function takes plain typed
 * arrays; nothing here interprets merge-tree semantics.
 *
 * Errors: a negative mte status becomes a thrown JS Error whose `code` is the
 * MTE_E_* value and whose message carries mte_strerror + mte_last_error (the
 * reference raises asserts with hex codes, client.ts:525-528; the JS layer
 * adds `assertCode` where a 1:1 equivalent exists).
 *
 * Built with gcc against /usr/include/node (N-API v8), linked to libmte.so
 * with an $ORIGIN rpath, so no node-gyp run is needed (Makefile).
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mte.h"

#define NAPI_CALL(env, call)                                          \
  do {                                                                \
    napi_status s_ = (call);                                          \
    if (s_ != napi_ok) {                                              \
      const napi_extended_error_info* ei_ = NULL;                     \
      napi_get_last_error_info((env), &ei_);                          \
      napi_throw_error((env), NULL,                                   \
                       ei_ && ei_->error_message ? ei_->error_message \
                                                 : "N-API call failed"); \
      return NULL;                                                    \
    }                                                                 \
  } while (0)

/* Throw Error(code) for rc < 0; returns 1 if thrown. */
static int throw_rc(napi_env env, int rc, mte_ctx* ctx, const char* what) {
  if (rc >= 0) return 0;
  char msg[768];
  snprintf(msg, sizeof msg, "%s: %s%s%s", what, mte_strerror(rc), ctx ? ": " : "",
           ctx ? mte_last_error(ctx) : "");
  napi_value m, err, code;
  napi_create_string_utf8(env, msg, NAPI_AUTO_LENGTH, &m);
  napi_create_error(env, NULL, m, &err);
  napi_create_int32(env, rc, &code);
  napi_set_named_property(env, err, "code", code);
  napi_throw(env, err);
  return 1;
}

typedef struct {
  mte_ctx* ctx;
  uint32_t n_keys; /* the context's property planes: the read-outs size their buffers by it */
} ctx_box;

static void ctx_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  ctx_box* b = (ctx_box*)data;
  if (b->ctx) mte_destroy(b->ctx);
  free(b);
}

static int get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
  size_t argc = want;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return 0;
  if (argc < want) {
    napi_throw_type_error(env, NULL, "too few arguments");
    return 0;
  }
  return 1;
}

static ctx_box* get_box(napi_env env, napi_value v) {
  ctx_box* b = NULL;
  if (napi_get_value_external(env, v, (void**)&b) != napi_ok || !b || !b->ctx) {
    napi_throw_type_error(env, NULL, "expected a live engine context");
    return NULL;
  }
  return b;
}

static mte_ctx* get_ctx(napi_env env, napi_value v) {
  ctx_box* b = get_box(env, v);
  return b ? b->ctx : NULL;
}

/* The read-outs write the context's n_keys values per segment: a caller's nKeys
   that differs would size the property buffers wrongly (MTE_E_INVALID_ARG). */
static int check_nkeys(napi_env env, const ctx_box* b, uint32_t nk) {
  if (nk == b->n_keys) return 1;
  throw_rc(env, MTE_E_INVALID_ARG, b->ctx, "nKeys differs from the context's n_keys");
  return 0;
}

/* Raw bytes of any TypedArray (or null/undefined -> NULL, 0). */
static int get_bytes(napi_env env, napi_value v, void** data, size_t* nbytes) {
  napi_valuetype t;
  *data = NULL;
  *nbytes = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return 0;
  if (t == napi_null || t == napi_undefined) return 1;
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (!is_ta) {
    napi_throw_type_error(env, NULL, "expected a TypedArray");
    return 0;
  }
  napi_typedarray_type tt;
  size_t len = 0, off = 0;
  napi_value ab;
  if (napi_get_typedarray_info(env, v, &tt, &len, data, &ab, &off) != napi_ok) return 0;
  size_t el = 1;
  switch (tt) {
    case napi_int8_array: case napi_uint8_array: case napi_uint8_clamped_array: el = 1; break;
    case napi_int16_array: case napi_uint16_array: el = 2; break;
    case napi_int32_array: case napi_uint32_array: case napi_float32_array: el = 4; break;
    default: el = 8; break;
  }
  *nbytes = len * el;
  return 1;
}

static napi_value js_abi_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value r;
  NAPI_CALL(env, napi_create_int32(env, mte_abi_version(), &r));
  return r;
}

static napi_value js_strerror(napi_env env, napi_callback_info info) {
  napi_value argv[1], r;
  if (!get_args(env, info, 1, argv)) return NULL;
  int32_t code = 0;
  NAPI_CALL(env, napi_get_value_int32(env, argv[0], &code));
  NAPI_CALL(env, napi_create_string_utf8(env, mte_strerror(code), NAPI_AUTO_LENGTH, &r));
  return r;
}

/* create(device, nKeys, segCapacity) -> external ctx */
static napi_value js_create(napi_env env, napi_callback_info info) {
  napi_value argv[3], r;
  if (!get_args(env, info, 3, argv)) return NULL;
  mte_config cfg;
  memset(&cfg, 0, sizeof cfg);
  uint32_t nk = 0, cap = 0;
  NAPI_CALL(env, napi_get_value_int32(env, argv[0], &cfg.device));
  NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &nk));
  NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &cap));
  cfg.n_keys = nk;
  cfg.seg_capacity = cap;
  mte_ctx* ctx = NULL;
  int rc = mte_create(&cfg, &ctx);
  if (throw_rc(env, rc, NULL, "mte_create")) return NULL;
  ctx_box* b = (ctx_box*)calloc(1, sizeof *b);
  if (!b) {
    mte_destroy(ctx);
    throw_rc(env, MTE_E_OOM, NULL, "mte_create");
    return NULL;
  }
  b->ctx = ctx;
  b->n_keys = nk;
  NAPI_CALL(env, napi_create_external(env, b, ctx_finalize, NULL, &r));
  return r;
}

static napi_value js_destroy(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  ctx_box* b = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&b));
  if (b && b->ctx) {
    mte_destroy(b->ctx);
    b->ctx = NULL;
  }
  return NULL;
}

static napi_value js_last_error(napi_env env, napi_callback_info info) {
  napi_value argv[1], r;
  if (!get_args(env, info, 1, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  NAPI_CALL(env, napi_create_string_utf8(env, mte_last_error(ctx), NAPI_AUTO_LENGTH, &r));
  return r;
}

/* loadDocs(ctx, inits Uint8Array(24*n), text Uint16Array, propsets Uint32Array, props Uint32Array) */
static napi_value js_load_docs(napi_env env, napi_callback_info info) {
  napi_value argv[5];
  if (!get_args(env, info, 5, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void *inits, *text, *ps, *pe;
  size_t ni, nt, nps, npe;
  if (!get_bytes(env, argv[1], &inits, &ni) || !get_bytes(env, argv[2], &text, &nt) ||
      !get_bytes(env, argv[3], &ps, &nps) || !get_bytes(env, argv[4], &pe, &npe))
    return NULL;
  if (ni % sizeof(mte_doc_init) || nt % 2 || nps % sizeof(mte_propset) || npe % sizeof(mte_prop)) {
    throw_rc(env, MTE_E_INVALID_ARG, ctx, "loadDocs: buffer sizes");
    return NULL;
  }
  int rc = mte_load_docs(ctx, (uint32_t)(ni / sizeof(mte_doc_init)), (const mte_doc_init*)inits,
                         (const uint16_t*)text, nt / 2, (const mte_propset*)ps,
                         (uint32_t)(nps / sizeof(mte_propset)), (const mte_prop*)pe,
                         (uint32_t)(npe / sizeof(mte_prop)));
  throw_rc(env, rc, ctx, "mte_load_docs");
  return NULL;
}

/* loadSegments(ctx, offsets BigUint64Array(n+1), segs Uint8Array(32*k)) -> mte_load_segments */
static napi_value js_load_segments(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void *offs, *segs;
  size_t no, ns;
  if (!get_bytes(env, argv[1], &offs, &no) || !get_bytes(env, argv[2], &segs, &ns)) return NULL;
  if (no % 8 || ns % sizeof(mte_seg)) {
    throw_rc(env, MTE_E_INVALID_ARG, ctx, "loadSegments: buffer sizes");
    return NULL;
  }
  int rc = mte_load_segments(ctx, (const uint64_t*)offs, (const mte_seg*)segs, ns / sizeof(mte_seg));
  throw_rc(env, rc, ctx, "mte_load_segments");
  return NULL;
}

/* submit(ctx, offsets BigUint64Array(n+1), ops Uint8Array(32*k), text Uint16Array,
 *        propsets Uint32Array, props Uint32Array) */
static napi_value js_submit(napi_env env, napi_callback_info info) {
  napi_value argv[6];
  if (!get_args(env, info, 6, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void *off, *ops, *text, *ps, *pe;
  size_t noff, nops, nt, nps, npe;
  if (!get_bytes(env, argv[1], &off, &noff) || !get_bytes(env, argv[2], &ops, &nops) ||
      !get_bytes(env, argv[3], &text, &nt) || !get_bytes(env, argv[4], &ps, &nps) ||
      !get_bytes(env, argv[5], &pe, &npe))
    return NULL;
  if (noff < 8 || noff % 8 || nops % sizeof(mte_op) || nt % 2 || nps % sizeof(mte_propset) ||
      npe % sizeof(mte_prop)) {
    throw_rc(env, MTE_E_INVALID_ARG, ctx, "submit: buffer sizes");
    return NULL;
  }
  mte_batch b;
  memset(&b, 0, sizeof b);
  b.n_docs = (uint32_t)(noff / 8 - 1);
  b.op_offsets = (const uint64_t*)off;
  b.ops = (const mte_op*)ops;
  b.n_ops = nops / sizeof(mte_op);
  b.text = (const uint16_t*)text;
  b.text_units = nt / 2;
  b.propsets = (const mte_propset*)ps;
  b.n_propsets = (uint32_t)(nps / sizeof(mte_propset));
  b.props = (const mte_prop*)pe;
  b.n_props = (uint32_t)(npe / sizeof(mte_prop));
  throw_rc(env, mte_submit(ctx, &b), ctx, "mte_submit");
  return NULL;
}

#define SIMPLE(name, fn)                                                  \
  static napi_value name(napi_env env, napi_callback_info info) {        \
    napi_value argv[1];                                                   \
    if (!get_args(env, info, 1, argv)) return NULL;                       \
    mte_ctx* ctx = get_ctx(env, argv[0]);                                 \
    if (!ctx) return NULL;                                                \
    throw_rc(env, fn(ctx), ctx, #fn);                                     \
    return NULL;                                                          \
  }
SIMPLE(js_run, mte_run)
SIMPLE(js_sync, mte_sync)
SIMPLE(js_reset, mte_reset)

/* digest(ctx, out BigUint64Array(4*n)) */
static napi_value js_digest(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void* out;
  size_t n;
  if (!get_bytes(env, argv[1], &out, &n)) return NULL;
  throw_rc(env, mte_digest(ctx, (uint64_t*)out, (uint32_t)(n / 32)), ctx, "mte_digest");
  return NULL;
}

/* docStatus(ctx, out Int32Array(n)) */
static napi_value js_doc_status(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void* out;
  size_t n;
  if (!get_bytes(env, argv[1], &out, &n)) return NULL;
  throw_rc(env, mte_doc_status(ctx, (int32_t*)out, (uint32_t)(n / 4)), ctx, "mte_doc_status");
  return NULL;
}

static void set_i32(napi_env env, napi_value o, const char* k, int32_t v) {
  napi_value x;
  napi_create_int32(env, v, &x);
  napi_set_named_property(env, o, k, x);
}
static void set_f64(napi_env env, napi_value o, const char* k, double v) {
  napi_value x;
  napi_create_double(env, v, &x);
  napi_set_named_property(env, o, k, x);
}

static napi_value u32_array(napi_env env, const uint32_t* src, size_t n) {
  napi_value ab, ta;
  void* p = NULL;
  if (napi_create_arraybuffer(env, n * 4, &p, &ab) != napi_ok) return NULL;
  if (n) memcpy(p, src, n * 4);
  if (napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &ta) != napi_ok) return NULL;
  return ta;
}

/* readDoc(ctx, doc, nKeys) -> {status, curSeq, minSeq, length, text, segLen, segKind, segProps} */
/* readSegments(ctx, doc, nKeys) -> {segs Uint8Array(32*n) (mte_seg, text_off into text),
   props Uint32Array(n*nKeys), text Uint16Array} (mte_read_segments) */
static napi_value js_read_segments(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  ctx_box* box = get_box(env, argv[0]);
  if (!box) return NULL;
  mte_ctx* ctx = box->ctx;
  uint32_t doc = 0, nk = 0;
  NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
  NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &nk));
  if (!check_nkeys(env, box, nk)) return NULL;
  mte_seg_list v;
  memset(&v, 0, sizeof v);
  if (throw_rc(env, mte_read_segments(ctx, doc, &v), ctx, "mte_read_segments")) return NULL;  // sizes
  napi_value o = NULL, ab_s, ab_p, ab_t, ts, tp, tt;
  void *ps, *pp, *pt;
  const size_t ns = (size_t)v.n_segs, nt = (size_t)v.n_text, npv = ns * nk;
  NAPI_CALL(env, napi_create_arraybuffer(env, ns * sizeof(mte_seg), &ps, &ab_s));
  NAPI_CALL(env, napi_create_arraybuffer(env, npv * 4, &pp, &ab_p));
  NAPI_CALL(env, napi_create_arraybuffer(env, nt * 2, &pt, &ab_t));
  v.segs = (mte_seg*)ps;
  v.props = nk ? (uint32_t*)pp : NULL;
  v.seg_cap = ns;
  v.text = (uint16_t*)pt;
  v.text_cap = nt;
  if (throw_rc(env, mte_read_segments(ctx, doc, &v), ctx, "mte_read_segments")) return NULL;
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, ns * sizeof(mte_seg), ab_s, 0, &ts));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint32_array, npv, ab_p, 0, &tp));
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint16_array, nt, ab_t, 0, &tt));
  NAPI_CALL(env, napi_create_object(env, &o));
  napi_set_named_property(env, o, "segs", ts);
  napi_set_named_property(env, o, "props", tp);
  napi_set_named_property(env, o, "text", tt);
  return o;
}

static napi_value js_read_doc(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  ctx_box* box = get_box(env, argv[0]);
  if (!box) return NULL;
  mte_ctx* ctx = box->ctx;
  uint32_t doc = 0, nk = 0;
  NAPI_CALL(env, napi_get_value_uint32(env, argv[1], &doc));
  NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &nk));
  if (!check_nkeys(env, box, nk)) return NULL;
  mte_doc_view v;
  memset(&v, 0, sizeof v);
  if (throw_rc(env, mte_read_doc(ctx, doc, &v), ctx, "mte_read_doc")) return NULL;  // sizes
  const size_t nt = v.n_text, ns = v.n_segs;
  uint16_t* text = (uint16_t*)malloc((nt + 1) * 2);
  uint32_t* sl = (uint32_t*)malloc((ns + 1) * 4);
  uint32_t* sk = (uint32_t*)malloc((ns + 1) * 4);
  uint32_t* sp = (uint32_t*)malloc((ns * (nk ? nk : 1) + 1) * 4);
  napi_value o = NULL;
  if (!text || !sl || !sk || !sp) {
    throw_rc(env, MTE_E_OOM, ctx, "readDoc");
    goto done;
  }
  v.text = text;
  v.text_cap = (uint32_t)nt;
  v.seg_len = sl;
  v.seg_kind = sk;
  v.seg_props = nk ? sp : NULL;
  v.seg_cap = (uint32_t)ns;
  if (throw_rc(env, mte_read_doc(ctx, doc, &v), ctx, "mte_read_doc")) goto done;
  napi_create_object(env, &o);
  set_i32(env, o, "status", v.status);
  set_i32(env, o, "curSeq", v.cur_seq);
  set_i32(env, o, "minSeq", v.min_seq);
  set_f64(env, o, "length", (double)v.length);
  {
    napi_value s;
    napi_create_string_utf16(env, (const char16_t*)text, v.n_text, &s);
    napi_set_named_property(env, o, "text", s);
    napi_set_named_property(env, o, "segLen", u32_array(env, sl, v.n_segs));
    napi_set_named_property(env, o, "segKind", u32_array(env, sk, v.n_segs));
    napi_set_named_property(env, o, "segProps", u32_array(env, sp, nk ? (size_t)v.n_segs * nk : 0));
  }
done:
  free(text);
  free(sl);
  free(sk);
  free(sp);
  return o;
}

static napi_value js_stats(napi_env env, napi_callback_info info) {
  napi_value argv[1], o;
  if (!get_args(env, info, 1, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  mte_stats s;
  if (throw_rc(env, mte_stats_get(ctx, &s), ctx, "mte_stats_get")) return NULL;
  NAPI_CALL(env, napi_create_object(env, &o));
  set_f64(env, o, "opsApplied", (double)s.ops_applied);
  set_f64(env, o, "segsScanned", (double)s.segs_scanned);
  set_f64(env, o, "segsWritten", (double)s.segs_written);
  set_f64(env, o, "propWrites", (double)s.prop_writes);
  set_f64(env, o, "unitsInserted", (double)s.units_inserted);
  set_f64(env, o, "maxSegs", (double)s.max_segs);
  set_f64(env, o, "kernelMs", s.kernel_ms);
  set_f64(env, o, "algoBytes", s.algo_bytes);
  set_f64(env, o, "chunkScanned", (double)s.chunk_scanned);
  set_f64(env, o, "roundBytes", s.round_bytes);
  return o;
}

/* ---- node level over RCCL (mte_comm_*) ---- */
/* commUniqueId() -> Uint8Array(128) */
static napi_value js_comm_unique_id(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value ab, ta;
  void* p = NULL;
  NAPI_CALL(env, napi_create_arraybuffer(env, MTE_COMM_ID_BYTES, &p, &ab));
  if (throw_rc(env, mte_comm_unique_id((uint8_t*)p), NULL, "mte_comm_unique_id")) return NULL;
  NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, MTE_COMM_ID_BYTES, ab, 0, &ta));
  return ta;
}

/* commInit(ctx, world, rank, id Uint8Array(128)) */
static napi_value js_comm_init(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  int32_t world = 0, rank = 0;
  NAPI_CALL(env, napi_get_value_int32(env, argv[1], &world));
  NAPI_CALL(env, napi_get_value_int32(env, argv[2], &rank));
  void* id;
  size_t n;
  if (!get_bytes(env, argv[3], &id, &n)) return NULL;
  if (n != MTE_COMM_ID_BYTES) {
    throw_rc(env, MTE_E_INVALID_ARG, ctx, "commInit: id must be 128 bytes");
    return NULL;
  }
  throw_rc(env, mte_comm_init(ctx, world, rank, (const uint8_t*)id), ctx, "mte_comm_init");
  return NULL;
}

/* commShare(ctx, srcCtx) */
static napi_value js_comm_share(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  mte_ctx* src = get_ctx(env, argv[1]);
  if (!src) return NULL;
  throw_rc(env, mte_comm_share(ctx, src), ctx, "mte_comm_share");
  return NULL;
}

/* commBarrier(ctx) */
static napi_value js_comm_barrier(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  throw_rc(env, mte_comm_barrier(ctx), ctx, "mte_comm_barrier");
  return NULL;
}

/* commAllreduce(ctx, value, op 0 sum / 1 max) -> number */
static napi_value js_comm_allreduce(napi_env env, napi_callback_info info) {
  napi_value argv[3], r;
  if (!get_args(env, info, 3, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  double v = 0;
  int32_t op = 0;
  NAPI_CALL(env, napi_get_value_double(env, argv[1], &v));
  NAPI_CALL(env, napi_get_value_int32(env, argv[2], &op));
  if (throw_rc(env, mte_comm_allreduce_f64(ctx, &v, op), ctx, "mte_comm_allreduce_f64")) return NULL;
  NAPI_CALL(env, napi_create_double(env, v, &r));
  return r;
}

/* commGatherDigests(ctx, out BigUint64Array(world * docsPerRank * 4), docsPerRank) */
static napi_value js_comm_gather_digests(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  void* out;
  size_t n;
  if (!get_bytes(env, argv[1], &out, &n)) return NULL;
  uint32_t per = 0;
  NAPI_CALL(env, napi_get_value_uint32(env, argv[2], &per));
  /* the byte length of the caller's array bounds the gather (mte.h) */
  throw_rc(env, mte_comm_gather_digests(ctx, (uint64_t*)out, (uint64_t)(n / sizeof(uint64_t)), per), ctx,
           "mte_comm_gather_digests");
  return NULL;
}

/* commDestroy(ctx) */
static napi_value js_comm_destroy(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  throw_rc(env, mte_comm_destroy(ctx), ctx, "mte_comm_destroy");
  return NULL;
}

/* readDeltas(ctx, doc) -> Int32Array(5 n): op, kind, pos, len, removed per
   event (mte_read_deltas) */
static napi_value js_read_deltas(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t doc = 0;
  if (napi_get_value_uint32(env, argv[1], &doc) != napi_ok) {
    napi_throw_type_error(env, NULL, "doc must be a number");
    return NULL;
  }
  uint64_t n = 0;
  if (throw_rc(env, mte_read_deltas(ctx, doc, NULL, 0, &n), ctx, "mte_read_deltas")) return NULL;
  mte_delta* buf = (mte_delta*)malloc((size_t)(n ? n : 1) * sizeof(mte_delta));
  if (!buf) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  if (throw_rc(env, mte_read_deltas(ctx, doc, buf, n, &n), ctx, "mte_read_deltas")) {
    free(buf);
    return NULL;
  }
  napi_value out = u32_array(env, (const uint32_t*)buf, (size_t)n * 5);
  free(buf);
  return out;
}

/* setEventCapacity(ctx, perOp) (mte_set_event_capacity) */
static napi_value js_set_event_capacity(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t per = 0;
  if (napi_get_value_uint32(env, argv[1], &per) != napi_ok) {
    napi_throw_type_error(env, NULL, "setEventCapacity: the per-op capacity must be a number");
    return NULL;
  }
  throw_rc(env, mte_set_event_capacity(ctx, per), ctx, "mte_set_event_capacity");
  return NULL;
}

/* setRefCapacity(ctx, perDoc) (mte_set_ref_capacity) */
static napi_value js_set_ref_capacity(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t per = 0;
  if (napi_get_value_uint32(env, argv[1], &per) != napi_ok) {
    napi_throw_type_error(env, NULL, "setRefCapacity: the per-document capacity must be a number");
    return NULL;
  }
  throw_rc(env, mte_set_ref_capacity(ctx, per), ctx, "mte_set_ref_capacity");
  return NULL;
}

/* readRefs(ctx, doc, n[, transient]) -> Int32Array(n): positions of reference
   slots [0, n) (mte_read_refs; -1 detached / unused); transient true: as
   Transient references (mte_read_refs_transient) */
static napi_value js_read_refs(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  size_t argc = 4;
  if (napi_get_cb_info(env, info, &argc, argv, NULL, NULL) != napi_ok) return NULL;
  if (argc < 3) {
    napi_throw_type_error(env, NULL, "too few arguments");
    return NULL;
  }
  bool transient = false;
  if (argc > 3 && napi_get_value_bool(env, argv[3], &transient) != napi_ok) transient = false;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t doc = 0, n = 0;
  if (napi_get_value_uint32(env, argv[1], &doc) != napi_ok || napi_get_value_uint32(env, argv[2], &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "readRefs: doc and n must be numbers");
    return NULL;
  }
  int32_t* buf = (int32_t*)malloc((size_t)(n ? n : 1) * sizeof(int32_t));
  if (!buf) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  if (throw_rc(env, (transient ? mte_read_refs_transient : mte_read_refs)(ctx, doc, buf, n), ctx, "mte_read_refs")) {
    free(buf);
    return NULL;
  }
  napi_value out = u32_array(env, (const uint32_t*)buf, (size_t)n);
  free(buf);
  return out;
}

/* readRefOrder(ctx, doc, n) -> Float64Array(n): document order of reference
   slots [0, n) (mte_read_ref_order; -1 detached / unused) */
static napi_value js_read_ref_order(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return NULL;
  mte_ctx* ctx = get_ctx(env, argv[0]);
  if (!ctx) return NULL;
  uint32_t doc = 0, n = 0;
  if (napi_get_value_uint32(env, argv[1], &doc) != napi_ok || napi_get_value_uint32(env, argv[2], &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "readRefOrder: doc and n must be numbers");
    return NULL;
  }
  int64_t* buf = (int64_t*)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
  if (!buf) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  if (throw_rc(env, mte_read_ref_order(ctx, doc, buf, n), ctx, "mte_read_ref_order")) {
    free(buf);
    return NULL;
  }
  napi_value ab, out;
  void* data = NULL;
  if (napi_create_arraybuffer(env, (size_t)n * 8, &data, &ab) != napi_ok ||
      napi_create_typedarray(env, napi_float64_array, n, ab, 0, &out) != napi_ok) {
    free(buf);
    napi_throw_error(env, NULL, "readRefOrder: allocation");
    return NULL;
  }
  for (uint32_t i = 0; i < n; i++) ((double*)data)[i] = (double)buf[i];
  free(buf);
  return out;
}

static napi_value init(napi_env env, napi_value exports) {
  const napi_property_descriptor d[] = {
      {"abiVersion", NULL, js_abi_version, NULL, NULL, NULL, napi_enumerable, NULL},
      {"strerror", NULL, js_strerror, NULL, NULL, NULL, napi_enumerable, NULL},
      {"create", NULL, js_create, NULL, NULL, NULL, napi_enumerable, NULL},
      {"destroy", NULL, js_destroy, NULL, NULL, NULL, napi_enumerable, NULL},
      {"lastError", NULL, js_last_error, NULL, NULL, NULL, napi_enumerable, NULL},
      {"loadDocs", NULL, js_load_docs, NULL, NULL, NULL, napi_enumerable, NULL},
      {"loadSegments", NULL, js_load_segments, NULL, NULL, NULL, napi_enumerable, NULL},
      {"submit", NULL, js_submit, NULL, NULL, NULL, napi_enumerable, NULL},
      {"run", NULL, js_run, NULL, NULL, NULL, napi_enumerable, NULL},
      {"sync", NULL, js_sync, NULL, NULL, NULL, napi_enumerable, NULL},
      {"reset", NULL, js_reset, NULL, NULL, NULL, napi_enumerable, NULL},
      {"digest", NULL, js_digest, NULL, NULL, NULL, napi_enumerable, NULL},
      {"docStatus", NULL, js_doc_status, NULL, NULL, NULL, napi_enumerable, NULL},
      {"readDoc", NULL, js_read_doc, NULL, NULL, NULL, napi_enumerable, NULL},
      {"readSegments", NULL, js_read_segments, NULL, NULL, NULL, napi_enumerable, NULL},
      {"stats", NULL, js_stats, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commUniqueId", NULL, js_comm_unique_id, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commInit", NULL, js_comm_init, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commShare", NULL, js_comm_share, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commBarrier", NULL, js_comm_barrier, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commAllreduce", NULL, js_comm_allreduce, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commGatherDigests", NULL, js_comm_gather_digests, NULL, NULL, NULL, napi_enumerable, NULL},
      {"commDestroy", NULL, js_comm_destroy, NULL, NULL, NULL, napi_enumerable, NULL},
      {"readDeltas", NULL, js_read_deltas, NULL, NULL, NULL, napi_enumerable, NULL},
      {"setEventCapacity", NULL, js_set_event_capacity, NULL, NULL, NULL, napi_enumerable, NULL},
      {"setRefCapacity", NULL, js_set_ref_capacity, NULL, NULL, NULL, napi_enumerable, NULL},
      {"readRefs", NULL, js_read_refs, NULL, NULL, NULL, napi_enumerable, NULL},
      {"readRefOrder", NULL, js_read_ref_order, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  if (napi_define_properties(env, exports, sizeof d / sizeof d[0], d) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
