"use strict";
/*
 * packing.js — host half of Client.applyMsg for the device engine: turns
 * ISequencedDocumentMessage objects into 32-byte op records (include/mte.h
 * mte_op) plus a UTF-16 text arena and property tables.
 *
 * Reference behaviour mirrored (packages/dds/merge-tree/src):
 *  - short client ids in first-seen order, the observer's own id first
 *    (Client.getOrAddShortClientId / startOrUpdateCollaboration,
 *    client.ts:683-698, 1163-1183); every message registers its sender
 *    (client.ts:920), "op" or not;
 *  - only type "op" messages carry a merge-tree op, every message advances
 *    currentSeq / minSeq (client.ts:922-934): non-op messages become NOOP
 *    records;
 *  - GROUP ops apply their members in order under one sequenced message
 *    (client.ts:876-884): one record per member, MSG_END on the last;
 *  - insert specs: string -> text, {text, props}, {marker:{refType}, props}
 *    (test/testClient.ts:32-44, textSegment.ts:40-48, mergeTreeNodes.ts:602-609);
 *    an insert without seg is a no-op (client.ts:481-487);
 *  - annotate: null deletes a key, anything else sets it; combiningOp
 *    "rewrite" is supported, other combining ops are rejected.
 * Property keys are interned to plane indices and values to ids of their
 * canonical JSON (sorted keys), so id equality == matchProperties
 * (properties.ts:66-100).
 *
 * Written in the Node-12-compatible subset of JavaScript (no ?. / ??), see
 * DESIGN.md "Host language".  Mirrors fluidframework_amd/packing.py record
 * for record (tests/test_node_host.py checks the bytes are identical).
 */

const OP_INSERT = 0, OP_REMOVE = 1, OP_ANNOTATE = 2, OP_NOOP = 3, OP_ACK = 4, OP_ROLLBACK = 5, OP_REGEN = 6;
const OP_RBKEY = 7;          // MTE_OP_RBKEY: an annotate rollback's previous-value candidates
const OP_REF = 8;            // MTE_OP_REF: create / remove a local reference
const OP_RELPOS = 9;         // MTE_OP_RELPOS: relative positions of the record that follows
const RP_POS1 = 0x100, RP_BEFORE1 = 0x200, RP_POS2 = 0x400, RP_BEFORE2 = 0x800;
const MARKER_ID_KEY = "markerId";  // reservedMarkerIdKey (mergeTreeNodes.ts)
const REF_SLIDE_ON_REMOVE = 0x40, REF_STAY_ON_REMOVE = 0x80, REF_TRANSIENT = 0x100;  // ReferenceType (ops.ts)
const DELTA_REGEN = 0x10;    // MTE_DELTA_REGEN: kind flag of a regenerated op's records
const ANNOTATE_SLOTS = 32;   // MTE_ANNOTATE_SLOTS: pending local annotate groups tracked per document
const F_MARKER = 0x1, F_MSG_END = 0x2, F_REWRITE = 0x4, F_LOCAL = 0x8;
const F_COMBINE = 0x10, COMBINE_PAIR = 0x80000000;
const F_REGENERATED = 0x20;  // an ack of a regenerated message (include/mte.h)  // incr / consensus value maps (include/mte.h)
// a value id matching no other, itself included: NaN (matchProperties' !==, include/mte.h)
const VALUE_UNEQUAL = 0x40000000;
const LOCAL_SEQ_BASE = 0x40000000; // MTE_LOCAL_SEQ_BASE
const NO_PROPS = 0xffffffff;
const MAX_CLIENTS = 32;
// local-client and MTE_DOC_TREE documents (the HBM tree pass: a second removers plane)
const MAX_CLIENTS_TREE = 64;
const OP_BYTES = 32;
const DOC_INIT_BYTES = 24;
const DOC_NEW_LENGTH_CALC = 0x1;

// MergeTreeDeltaType, ops.ts:43-48
const INSERT = 0, REMOVE = 1, ANNOTATE = 2, GROUP = 3;

const DOC_ROUND_SYNC = 0x2; // MTE_DOC_ROUND_SYNC (include/mte.h)
const DOC_LOCAL_CLIENT = 0x4; // MTE_DOC_LOCAL_CLIENT
const DOC_REFS = 0x10;       // MTE_DOC_REFS
const DOC_EVENTS = 0x8; // MTE_DOC_EVENTS
const DOC_SLIDE_EVENTS = 0x20;  // MTE_DOC_SLIDE_EVENTS: the references' slides and their snapshots
const DOC_MAINT_EVENTS = 0x40;  // MTE_DOC_MAINT_EVENTS: mergeTreeMaintenanceCallback records
const DOC_TREE = 0x80;  // MTE_DOC_TREE: the HBM tree pass (the reference's segmentation)
const E_INVALID_ARG = -1, E_CAPACITY = -4, E_UNSUPPORTED = -9, E_STATE = -10, E_CLIENT_RANGE = -12;
const COMBINE_DOMAIN_MAX = 4096;  // distinct values of one key a combining op's value map may cover
const DEFAULT_REF_CAPACITY = 1024;  // mte_set_ref_capacity's default (include/mte.h)

class MergeTreeError extends Error {
  constructor(code, message) {
    super(message);
    this.code = code;
  }
}

function canonicalJson(v) {
  if (v === null || typeof v !== "object") return JSON.stringify(v);
  if (Array.isArray(v)) return "[" + v.map(canonicalJson).join(",") + "]";
  const keys = Object.keys(v).sort();
  return "{" + keys.map((k) => JSON.stringify(k) + ":" + canonicalJson(v[k])).join(",") + "}";
}

function checkI32(v, what) {
  if ((v | 0) === v) return v;  // an int32 number (fast path; the test below gives the same answer)
  if (typeof v !== "number" || !Number.isInteger(v) || v < -2147483648 || v > 2147483647) {
    throw new MergeTreeError(E_INVALID_ARG, what + "=" + String(v) + " is not an int32");
  }
  return v;
}

/** Key -> plane index, canonical JSON value -> id (0 is reserved for null). */
class Interner {
  constructor(nKeys) {
    this.nKeys = nKeys;
    this.keys = new Map();
    this.keyNames = [];
    this.values = new Map();
    this.valueJson = [null];
    this.numIds = new Map();
    this.strIds = new Map();
    // per value index, the keys it was ever given (bit k), and per key how
    // many: the combining ops' domain (packing.py Interner.note_value)
    this.keyMask = new Uint32Array(256);
    this.keyCount = new Uint32Array(Math.max(1, nKeys));
    // a ShardedHost worker's interner logs [key, value index] the first time a
    // key is given a value, so the host's interner learns the combining ops'
    // domains (shards.js); null elsewhere
    this.noteLog = null;
  }
  /** [key, value id] of one property, noting the value under its key */
  kv(name, v) {
    const k = this.key(name), id = this.value(v);
    if (id) this.noteValue(k, id);
    return [k, id];
  }
  /** value id `id` was given to key `k` (the combining ops' domain) */
  noteValue(k, id) {
    const x = id & ~VALUE_UNEQUAL;
    if (x >= this.keyMask.length) {
      const m = new Uint32Array(Math.max(x + 1, this.keyMask.length * 2));
      m.set(this.keyMask);
      this.keyMask = m;
    }
    if (!(this.keyMask[x] & (1 << k))) {
      this.keyMask[x] |= 1 << k;
      this.keyCount[k]++;
      if (this.noteLog) this.noteLog.push(k, x);
    }
  }
  /** the value ids key k was ever given, ascending; a key given more than
   *  COMBINE_DOMAIN_MAX values is refused (its combining value map) */
  domainOf(k) {
    if (this.keyCount[k] > COMBINE_DOMAIN_MAX) {
      throw new MergeTreeError(E_UNSUPPORTED, "combiningOp over key " + this.keyNames[k] + ", given " +
        this.keyCount[k] + " distinct values (> " + COMBINE_DOMAIN_MAX + ")");
    }
    const out = [], b = 1 << k, M = this.keyMask;
    for (let x = 1; x < this.valueJson.length && x < M.length; x++) {
      if (M[x] & b) out.push((x | (this.valueJson[x] === "NaN" ? VALUE_UNEQUAL : 0)) >>> 0);
    }
    return out;
  }
  key(name) {
    let k = this.keys.get(name);
    if (k === undefined) {
      if (this.keyNames.length >= this.nKeys) {
        throw new MergeTreeError(E_UNSUPPORTED, "more than nKeys=" + this.nKeys + " property keys (" + name + ")");
      }
      k = this.keyNames.length;
      this.keys.set(name, k);
      this.keyNames.push(name);
    }
    return k;
  }
  value(v) {
    if (v === null || v === undefined) return 0;
    // numbers and strings: their canonical JSON is a function of the value, so
    // a map keyed by the value skips the stringify (same ids)
    const prim = typeof v === "number" ? this.numIds : (typeof v === "string" ? this.strIds : null);
    if (prim !== null) {
      const id = prim.get(v);
      if (id !== undefined) return id;
    }
    // NaN (an incr's result) is a value of its own, not JSON's null, and
    // matches nothing (VALUE_UNEQUAL)
    const nan = typeof v === "number" && v !== v;
    const cj = nan ? "NaN" : canonicalJson(v);
    let i = this.values.get(cj);
    if (i === undefined) {
      i = this.valueJson.length | (nan ? VALUE_UNEQUAL : 0);
      this.values.set(cj, i);
      this.valueJson.push(cj);
    }
    if (prim !== null && !(typeof v === "number" && Object.is(v, -0))) prim.set(v, i);
    return i;
  }
  /** the id of a value given as its canonical JSON (a shard's interned value, shards.js) */
  valueOfJson(cj) {
    let i = this.values.get(cj);
    if (i === undefined) {
      i = this.valueJson.length | (cj === "NaN" ? VALUE_UNEQUAL : 0);
      this.values.set(cj, i);
      this.valueJson.push(cj);
    }
    return i;
  }
  /** canonical JSON of a value id */
  jsonOf(id) {
    return this.valueJson[id & ~VALUE_UNEQUAL];
  }
  /** plane values of one segment -> PropertySet (undefined when empty) */
  decode(planes) {
    let out;
    for (let k = 0; k < planes.length; k++) {
      if (planes[k]) {
        if (out === undefined) out = {};
        const cj = this.jsonOf(planes[k]);
        out[this.keyNames[k]] = cj === "NaN" ? NaN : JSON.parse(cj);
      }
    }
    return out;
  }
}

/** Per-document long -> short client id map (client.ts:683-698) over the
 *  engine's MAX_CLIENTS slots (MAX_CLIENTS_TREE in local-client and tree
 *  documents).  A slot is recycled for a new client once the
 *  window's minSeq has passed every seq its client used: its segments are then
 *  visible to every perspective and its tombstones compacted
 *  (mergeTree.ts:1003-1054, 1077-1093), so the slot number decides no
 *  visibility rule any more (same rule as fluidframework_amd/packing.py). */
const NEVER = 0x7fffffff;
class DocClients {
  constructor(observerId, minSeq, local, tree) {
    this.observer = observerId;
    // an MTE_DOC_TREE document (the HBM tree pass without a local client): it
    // takes sequenced combining ops too
    this.tree = !!tree;
    this.maxClients = local || tree ? MAX_CLIENTS_TREE : MAX_CLIENTS;
    this.ids = new Map([[observerId, 0]]);
    this.last = new Int32Array(MAX_CLIENTS_TREE).fill(NEVER); // slot -> highest seq its client used
    this.lastId = observerId;  // the last sender and its slot (messages come in runs per sender)
    this.lastSlot = 0;
    this.minSeq = minSeq || 0;          // the window's minSeq before the next message
    // a document whose own client sends (MTE_DOC_LOCAL_CLIENT): collabWindow.localSeq
    // and the [first, last] localSeqs of each unacked local message, oldest first
    // (MergeTree.pendingSegments, mergeTree.ts:1333-1355)
    this.local = !!local;
    this.localSeq = 0;
    this.pending = [];
    this.pendingTypes = [];  // the record types of each pending message (rollback)
    // the first localSeqs of the pending messages regenerated since sent (their
    // acks carry F_REGENERATED)
    this.regenerated = new Set();
    // acks of annotates made while every slot was taken: the engine cannot
    // tell their segments (no ACKNOWLEDGED maintenance record)
    this.untrackedAcks = 0;
    // segment groups of pending local annotates: localSeq -> group slot; an
    // annotate made while all are taken is not tracked (cannot be regenerated)
    this.annSlot = new Map();
    // the key -> value id each pending local annotate set (its rollback puts the
    // older values back), and the annotates whose rollback the engine cannot
    // restate exactly (as packing.py)
    this.annProps = new Map();
    // the pending local incr / consensus annotates: localSeq -> [props, combiningOp]
    this.annComb = new Map();
    this.noRollback = new Set();
    // local reference slots (MTE_DOC_REFS documents): the next unused one and the
    // removed ones, reused first (as packing.py)
    this.refNext = 0;
    this.refFree = [];
    // the context's reference slots per document (MergeTreeEngine refCapacity,
    // mte_set_ref_capacity): a slot past it would fail the whole batch at
    // mte_submit, so the packer refuses the reference for this document alone
    this.refCap = DEFAULT_REF_CAPACITY;
  }
  short(longId, seq) {
    let i = longId === this.lastId ? this.lastSlot : this.ids.get(longId);
    if (i === undefined) {
      i = this._freeSlot();
      if (i >= this.maxClients) return i; // the caller throws E_CLIENT_RANGE
      this.ids.set(longId, i);
      this.last[i] = seq === undefined ? NEVER : seq;
    } else if (seq !== undefined && this.last[i] !== NEVER) {
      if (seq > this.last[i]) this.last[i] = seq;
    }
    this.lastId = longId;
    this.lastSlot = i;
    return i;
  }
  _freeSlot() {
    const used = new Set(this.ids.values());
    for (let s = 1; s < this.maxClients; s++) if (!used.has(s)) return s;
    let best = -1, bestSeq = NEVER;
    for (const v of used) {
      if (v !== 0 && (best < 0 || this.last[v] < bestSeq || (this.last[v] === bestSeq && v < best))) {
        best = v;
        bestSeq = this.last[v];
      }
    }
    if (best < 0 || bestSeq > this.minSeq) return this.maxClients;
    for (const [k, v] of this.ids) if (v === best) { this.ids.delete(k); break; }
    if (this.lastSlot === best) this.lastId = undefined;  // its client leaves the cache with its slot
    return best;
  }
  advance(msn) {
    if (msn > this.minSeq) this.minSeq = msn;
  }
}

/** Property sets of one batch (mte_propset / mte_prop arrays). */
class PropTable {
  constructor(interner) {
    this.interner = interner;
    this.sets = [];
    this.entries = [];
    this.combOf = new Map();  // a local combining set's index -> [props, combiningOp]
    this.deferred = null;  // addDeferred: [set index, key names, combiningOp, seq]
  }
  /** A sequenced incr / consensus annotate packed where the keys' value
   *  domains are not all known (a ShardedHost worker sees its own documents'
   *  values only): a placeholder set whose entries the host computes with
   *  addCombining over its own interner once every shard's values are merged
   *  (shards.js _merge).  combineValue ignores the op's values: only the key
   *  names travel. */
  addDeferred(props, comb, seq) {
    if (props === null || typeof props !== "object" || Array.isArray(props)) {
      throw new MergeTreeError(E_INVALID_ARG, "props must be an object");
    }
    const names = Object.keys(props);
    for (const name of names) this.interner.key(name);  // nKeys is checked here, as addCombining does
    if (!this.deferred) this.deferred = [];
    const s = this.sets.length >> 1;
    this.sets.push(this.entries.length >> 1, 0);
    this.deferred.push([s, names, { name: comb.name, defaultValue: comb.defaultValue, minValue: comb.minValue }, seq]);
    return s;
  }
  add(props) {
    if (props === undefined || props === null) return NO_PROPS;
    if (typeof props !== "object" || Array.isArray(props)) {
      throw new MergeTreeError(E_INVALID_ARG, "props must be an object");
    }
    const first = this.entries.length / 2;
    const it = this.interner, E = this.entries;
    for (const name in props) {
      if (!Object.prototype.hasOwnProperty.call(props, name)) continue;
      const k = it.key(name), id = it.value(props[name]);
      if (id) it.noteValue(k, id);
      E.push(k, id);
    }
    this.sets.push(first, this.entries.length / 2 - first);
    return this.sets.length / 2 - 1;
  }
  /** An annotate with combiningOp incr / consensus (as packing.py
   *  add_combining): per key a header [key, n] and n pairs [old | COMBINE_PAIR,
   *  new] -- combineValue over every value the key was ever given, 0 = absent. */
  addCombining(props, comb, seq) {
    if (props === null || typeof props !== "object" || Array.isArray(props)) {
      throw new MergeTreeError(E_INVALID_ARG, "props must be an object");
    }
    const it = this.interner;
    const first = this.entries.length / 2;
    for (const name of Object.keys(props)) {
      const k = it.key(name);
      const dom = it.domainOf(k).sort((x, y) => x - y);
      dom.push(0);
      const pairs = [];
      for (const old of dom) {
        const cj = it.jsonOf(old);
        const cur = old === 0 ? undefined : (cj === "NaN" ? NaN : JSON.parse(cj));
        const nv = combineValue(comb, cur, seq);
        const nid = nv === undefined ? 0 : it.value(nv);
        if (nid !== old) pairs.push(old, nid);
      }
      for (let q = 1; q < pairs.length; q += 2) if (pairs[q]) it.noteValue(k, pairs[q]);
      this.entries.push(k, pairs.length / 2);
      for (let q = 0; q < pairs.length; q += 2) this.entries.push((pairs[q] | COMBINE_PAIR) >>> 0, pairs[q + 1]);
    }
    this.sets.push(first, this.entries.length / 2 - first);
    return this.sets.length / 2 - 1;
  }
}

/** The value an incr / consensus annotate leaves on a segment whose value is
 *  cur (undefined: absent): the reference passes undefined for the op's own
 *  value (segmentPropertiesManager.ts:141), so incr adds undefined to the value
 *  (or its defaultValue) and then lets a truthy minValue replace anything
 *  below it, and consensus makes {value: undefined, seq} of an absent value and
 *  stamps the seq of an object whose seq is -1 (properties.ts:24-62).  Pure:
 *  the reference mutates that object in place. */
function combineValue(comb, cur, seq) {
  let v = cur === undefined ? comb.defaultValue : cur;
  if (comb.name === "incr") {
    v += undefined;
    if (comb.minValue && v < comb.minValue) v = comb.minValue;
    return v;
  }
  if (comb.name === "consensus") {
    if (v === undefined || v === null) return { seq };
    if (typeof v === "object" && v.seq === -1) return Object.assign({}, v, { seq });
    return v;
  }
  throw new MergeTreeError(E_UNSUPPORTED, "combiningOp " + String(comb.name));
}

function utf16(s) {
  const u = new Uint16Array(s.length);
  for (let i = 0; i < s.length; i++) u[i] = s.charCodeAt(i); // JS strings are UTF-16 (textSegment.ts:52-55)
  return u;
}

/** Collects messages for nDocs documents and emits one mte_batch. */
class BatchBuilder {
  constructor(nDocs, interner, trackDocs, capHint) {
    this.nDocs = nDocs;
    this.interner = interner;
    // documents whose delta events are read back (MTE_DOC_EVENTS): per record,
    // {msg, op, local} — the message (or local op) and the (GROUP member) op
    this.track = trackDocs || null;
    this.recSrc = trackDocs ? trackDocs.map((t) => (t ? [] : null)) : null;
    this.props = new PropTable(interner);
    // records in arrival order, 8 int32 words each (the mte_op layout), and
    // their documents; build() sorts them by document (counting sort)
    this.cap = Math.max(1024, capHint || 0);  // records (capHint: the expected count, no regrowth)
    this.rec = new Int32Array(this.cap * 8);
    this.recDoc = new Uint32Array(this.cap);
    this.docCount = new Uint32Array(nDocs);
    this.count = 0;
    this.textBuf = new Uint16Array(4096);
    this.textUnits = 0;
  }

  _grow() {
    this.cap *= 2;
    const r = new Int32Array(this.cap * 8);
    r.set(this.rec);
    this.rec = r;
    const d = new Uint32Array(this.cap);
    d.set(this.recDoc);
    this.recDoc = d;
  }

  /** one record (mte_op): seq, ref_seq, min_seq, type | client << 8 | flags << 16, pos1, pos2, a, b */
  _put(doc, seq, ref, msn, type, client, flags, p1, p2, a, b) {
    if (this.count === this.cap) this._grow();
    const w = this.count * 8, R = this.rec;
    R[w] = seq;
    R[w + 1] = ref;
    R[w + 2] = msn;
    R[w + 3] = type | (client << 8) | (flags << 16);
    R[w + 4] = p1;
    R[w + 5] = p2;
    R[w + 6] = a;
    R[w + 7] = b;
    this.recDoc[this.count] = doc;
    this.docCount[doc]++;
    this.count++;
  }

  _truncate(k0) {
    for (let k = k0; k < this.count; k++) this.docCount[this.recDoc[k]]--;
    this.count = k0;
  }

  /** the records of document d as [seq, ref, msn, type, client, flags, pos1, pos2, a, b] (tests) */
  get docOps() {
    const out = [];
    for (let d = 0; d < this.nDocs; d++) out.push([]);
    const R = this.rec;
    for (let k = 0; k < this.count; k++) {
      const w = k * 8, w3 = R[w + 3];
      out[this.recDoc[k]].push([R[w], R[w + 1], R[w + 2], w3 & 0xff, (w3 >>> 8) & 0xff, w3 >>> 16, R[w + 4],
        R[w + 5], R[w + 6] >>> 0, R[w + 7] >>> 0]);
    }
    return out;
  }

  _text(s) {
    const off = this._textOff(s);
    return [off, s.length];
  }

  /** s's UTF-16 units appended to the batch text; their offset */
  _textOff(s) {
    if (typeof s !== "string") throw new MergeTreeError(E_INVALID_ARG, "text must be a string");
    const off = this.textUnits, n = s.length;
    if (off + n > this.textBuf.length) {
      let c = this.textBuf.length * 2;
      while (c < off + n) c *= 2;
      const t = new Uint16Array(c);
      t.set(this.textBuf.subarray(0, off));
      this.textBuf = t;
    }
    const T = this.textBuf;
    for (let i = 0; i < n; i++) T[off + i] = s.charCodeAt(i);  // UTF-16 code units (textSegment.ts:52-55)
    this.textUnits = off + n;
    return off;
  }

  /** Client.applyMsg(msg, local=false) for one document (client.ts:918-935). */
  addMessage(doc, clients, msg) {
    const sender = msg.clientId;
    const seq = checkI32(msg.sequenceNumber, "sequenceNumber");
    const ref = checkI32(msg.referenceSequenceNumber === undefined ? 0 : msg.referenceSequenceNumber,
      "referenceSequenceNumber");
    const msn = checkI32(msg.minimumSequenceNumber, "minimumSequenceNumber");
    // a recycled slot is only sound while every op sees past minSeq (DocClients)
    if (ref < clients.minSeq) {
      throw new MergeTreeError(E_INVALID_ARG, "referenceSequenceNumber " + ref + " < minSeq " + clients.minSeq);
    }
    const k0 = this.count;
    this._srcOps = null;
    if ((msg.type === undefined ? "op" : msg.type) === "op") {
      if (sender === clients.observer) {
        // our own op, sequenced: ackPendingSegment (client.ts:925-928)
        if (!clients.local) throw new MergeTreeError(E_UNSUPPORTED, "ack of a local op in an observer document");
        if (clients.pending.length === 0) throw new MergeTreeError(E_STATE, "ack without a pending local op");
        const [lo, hi] = clients.pending[0];
        // as packing.py: an earlier annotate still pending would lose its keys
        for (let q = 1; q < clients.pending.length; q++) {
          if (clients.pending[q][0] < lo && clients.pendingTypes[q].includes(OP_ANNOTATE)) {
            throw new MergeTreeError(E_UNSUPPORTED,
              "ack out of localSeq order past a pending annotate (regenerate every pending op, in order)");
          }
        }
        clients.pending.shift();
        clients.pendingAckTypes = clients.pendingTypes.shift();
        let mask = 0;
        for (let ls = lo; ls <= hi; ls++) {
          if (clients.annSlot.has(ls)) {
            mask |= 1 << clients.annSlot.get(ls);
            clients.annSlot.delete(ls);
          } else if (clients.pendingAckTypes && clients.pendingAckTypes[ls - lo] === OP_ANNOTATE) {
            clients.untrackedAcks++;
          }
          // an annotate acked under a later pending one on the same key (packing.py)
          const keys = clients.annProps.get(ls);
          if (keys) {
            clients.annProps.delete(ls);
            for (const [ls2, kv] of clients.annProps) {
              if (ls2 > hi && Array.from(keys.keys()).some((k) => kv.has(k))) clients.noRollback.add(ls2);
            }
          }
          clients.noRollback.delete(ls);
        }
        const regen = clients.regenerated.delete(lo);
        let flags = regen ? F_REGENERATED : 0, stamp = NO_PROPS;
        const comb = clients.annComb.get(hi);
        if (comb && comb[1].name === "consensus") {
          // updateConsensusProperty: the marker's consensus value takes the seq
          stamp = this.props.addCombining(comb[0], comb[1], seq);
          flags |= F_COMBINE;
        }
        for (let ls = lo; ls <= hi; ls++) clients.annComb.delete(ls);
        this._put(doc, seq, ref, msn, OP_ACK, 0, flags, lo, hi, mask, stamp);
      } else {
        this._combLocal = clients.local || clients.tree;
        try {
          this._opPut(doc, seq, ref, msn, msg.contents, this._src(doc));
        } catch (e) {
          this._combLocal = false;
          this._truncate(k0);
          throw e;
        }
        this._combLocal = false;
      }
    }
    // the slot is taken only once the message has validated
    let short;
    try {
      short = slotOf(clients, sender, seq);
    } catch (e) {
      this._truncate(k0);
      throw e;
    }
    if (this.count === k0) this._put(doc, seq, ref, msn, OP_NOOP, 0, 0, 0, 0, 0, NO_PROPS);
    const src = this._src(doc);
    if (src) {  // one entry per record of this message
      const ops = this._srcOps || [];
      for (let i = 0; i < this.count - k0; i++) src.push({ msg, op: ops[i], local: false });
      this._srcOps = null;
    }
    const R = this.rec;
    for (let k = k0; k < this.count; k++) R[k * 8 + 3] |= short << 8;
    R[(this.count - 1) * 8 + 3] |= F_MSG_END << 16;
    clients.advance(msn);
    clients.mergeSeq = seq;  // collabWindow.currentSeq after updateSeqNumbers (client.ts:937-945)
  }

  /** the records of a remote op (client.ts:862-889), as _opRecords, written
   *  straight into the batch (client 0, no MSG_END: addMessage sets both) */
  _opPut(doc, seq, ref, msn, op, track) {
    if (track && op && typeof op === "object" && op.type !== GROUP) {
      if (!this._srcOps) this._srcOps = [];
      this._srcOps.push(op);
    }
    if (op === null || typeof op !== "object") throw new MergeTreeError(E_INVALID_ARG, "op contents must be an object");
    const t = op.type;
    if (t === GROUP) {
      for (const member of op.ops || []) this._opPut(doc, seq, ref, msn, member, track);
      return;
    }
    const rel = this._relpos(op, t);
    if ((t === REMOVE || t === ANNOTATE) && !("pos2" in op) && !(rel && (rel[0] & RP_POS2))) {
      throw new MergeTreeError(E_UNSUPPORTED, "range op without pos2");
    }
    if ((t === REMOVE || t === ANNOTATE) && !("pos1" in op) && !(rel && (rel[0] & RP_POS1))) {
      throw new MergeTreeError(E_UNSUPPORTED, "range op without pos1");
    }
    if (rel && (t !== INSERT || (op.seg !== undefined && op.seg !== null))) {
      this._put(doc, rel[4], rel[5], 0, OP_RELPOS, 0, rel[0], rel[1], rel[2], rel[3], 0);
      if (track) this._srcOps.push(op);  // the RELPOS record's entry
    }
    if (t === INSERT) {
      const seg = op.seg;
      if (seg === undefined || seg === null) { // applyInsertOp returns false: no segment
        this._put(doc, seq, ref, msn, OP_NOOP, 0, 0, 0, 0, 0, NO_PROPS);
        return;
      }
      const pos = checkI32(op.pos1 === undefined ? 0 : op.pos1, "pos1");
      if (typeof seg === "string") {
        const off = this._textOff(seg);
        this._put(doc, seq, ref, msn, OP_INSERT, 0, 0, pos, seg.length, off, NO_PROPS);
      } else if (typeof seg === "object" && "text" in seg) {
        const off = this._textOff(seg.text);
        this._put(doc, seq, ref, msn, OP_INSERT, 0, 0, pos, seg.text.length, off, this.props.add(seg.props));
      } else if (typeof seg === "object" && "marker" in seg) {
        const rt = checkI32(seg.marker.refType === undefined ? 0 : seg.marker.refType, "refType");
        const off = this._textOff("\ufffc");  // one reserved unit names the marker in MTE_DOC_REFS documents
        this._put(doc, seq, ref, msn, OP_INSERT, 0, F_MARKER, pos, rt, off, this.props.add(seg.props));
      } else {
        throw new MergeTreeError(E_INVALID_ARG, "Unrecognized IJSONSegment type: " + JSON.stringify(seg));
      }
      return;
    }
    const p1 = op.pos1 === undefined ? 0 : op.pos1, p2 = op.pos2 === undefined ? 0 : op.pos2;
    if (t === REMOVE) {
      this._put(doc, seq, ref, msn, OP_REMOVE, 0, 0, checkI32(p1, "pos1"), checkI32(p2, "pos2"), 0, NO_PROPS);
    } else if (t === ANNOTATE) {
      let flags = 0;
      const comb = op.combiningOp;
      if (comb !== undefined && comb !== null && (comb.name === "incr" || comb.name === "consensus")) {
        if (!this._combLocal) {
          throw new MergeTreeError(E_UNSUPPORTED, "combiningOp " + comb.name +
            " outside a local-client or tree document (the HBM tree pass)");
        }
        if (comb.name === "consensus" && "defaultValue" in comb) {
          throw new MergeTreeError(E_UNSUPPORTED, "consensus with a defaultValue");
        }
        const pv = op.props === undefined ? {} : op.props;
        const ps = this.shard ? this.props.addDeferred(pv, comb, seq) : this.props.addCombining(pv, comb, seq);
        this._put(doc, seq, ref, msn, OP_ANNOTATE, 0, F_COMBINE, checkI32(p1, "pos1"), checkI32(p2, "pos2"), ps, NO_PROPS);
        return;
      }
      if (comb !== undefined && comb !== null) {
        if (comb.name !== "rewrite") throw new MergeTreeError(E_UNSUPPORTED, "combiningOp " + String(comb.name));
        flags = F_REWRITE;
      }
      const ps = this.props.add(op.props === undefined ? {} : op.props);  // before the checks, as packing.py
      this._put(doc, seq, ref, msn, OP_ANNOTATE, 0, flags, checkI32(p1, "pos1"), checkI32(p2, "pos2"), ps, NO_PROPS);
    } else {
      throw new MergeTreeError(E_INVALID_ARG, "unknown op type " + String(t));
    }
  }

  /** A local op of the document's own client (insertSegmentLocal /
   *  removeRangeLocal / annotateRangeLocal, client.ts:131-229): one F_LOCAL record
   *  per (GROUP member) op, each with the next localSeq; the message's localSeqs
   *  join the pending list, acked in order by addMessage (as packing.py add_local). */
  addLocal(doc, clients, op) {
    if (!clients.local) throw new MergeTreeError(E_UNSUPPORTED, "local op in an observer document");
    const recs = [];
    this._srcOps = null;
    this._opRecords(op, recs, this._src(doc));
    if (recs.length === 0) recs.push([OP_NOOP, 0, 0, 0, 0, NO_PROPS]);
    if (recs.some((r) => r[0] !== OP_RELPOS && (r[1] & F_REWRITE))) {
      throw new MergeTreeError(E_UNSUPPORTED, "local combiningOp rewrite");
    }
    // a local consensus is annotateMarkerNotifyConsensus's: alone in its message,
    // with a group slot (its ack's stamp, packing.py add_local)
    if (recs.some((r) => r[0] === OP_ANNOTATE && (r[1] & F_COMBINE) && this.props.combOf.get(r[4])[1].name === "consensus")) {
      if (recs.filter((r) => r[0] !== OP_RELPOS).length !== 1 || recs[0][0] !== OP_RELPOS) {
        throw new MergeTreeError(E_UNSUPPORTED,
          "a local consensus annotate is a marker's (annotateMarkerNotifyConsensus), alone in its message");
      }
      if (clients.annSlot.size >= ANNOTATE_SLOTS) {
        throw new MergeTreeError(E_UNSUPPORTED, "a local consensus annotate with " + ANNOTATE_SLOTS + " annotates pending");
      }
    }
    const first = clients.localSeq + 1;
    const nOps = recs.filter((r) => r[0] !== OP_RELPOS).length;  // a RELPOS record takes no localSeq
    if (first + nOps >= LOCAL_SEQ_BASE) throw new MergeTreeError(E_INVALID_ARG, "localSeq overflow");
    // every check that can throw is above: the event sources stay aligned with the records
    const src = this._src(doc);
    if (src) {
      const ops = this._srcOps || [];
      for (let i = 0; i < recs.length; i++) src.push({ msg: null, op: ops[i], local: true });
    }
    this._srcOps = null;
    let i = 0;
    for (const r of recs) {
      if (r[0] === OP_RELPOS) {
        this._put(doc, r[5][0], r[5][1], 0, OP_RELPOS, 0, r[1], r[2], r[3], r[4], 0);
        continue;
      }
      let b = r[5];
      if (r[0] === OP_ANNOTATE) {
        const used = new Set(clients.annSlot.values());
        let free = -1;
        for (let x = 0; x < ANNOTATE_SLOTS && free < 0; x++) if (!used.has(x)) free = x;
        if (free >= 0) {
          clients.annSlot.set(first + i, free);
          b = free;
        }
        const kv = new Map();
        const f0 = this.props.sets[2 * r[4]], cnt = this.props.sets[2 * r[4] + 1];
        if (r[1] & F_COMBINE) {
          // its keys (the map's headers); no rollback restates it, nor one past it
          for (let t = f0; t < f0 + cnt; t++) {
            if (!(this.props.entries[2 * t] & COMBINE_PAIR)) kv.set(this.props.entries[2 * t], null);
          }
          clients.annComb.set(first + i, this.props.combOf.get(r[4]));
          clients.noRollback.add(first + i);
        } else {
          for (let t = f0; t < f0 + cnt; t++) kv.set(this.props.entries[2 * t], this.props.entries[2 * t + 1]);
        }
        clients.annProps.set(first + i, kv);
      }
      this._put(doc, first + i, 0, 0, r[0], 0, r[1] | F_LOCAL, r[2], r[3], r[4], b);
      i++;
    }
    clients.localSeq += nOps;
    clients.pending.push([first, clients.localSeq]);
    clients.pendingTypes.push(recs.filter((r) => r[0] !== OP_RELPOS).map((r) => r[0]));
  }

  /** Client.rollback of the latest pending local op (client.ts:396-398 ->
   *  MergeTree.rollback, mergeTree.ts:2005-2083), as packing.py add_rollback. */
  addRollback(doc, clients) {
    if (!clients.local || clients.pending.length === 0) {
      throw new MergeTreeError(E_STATE, "rollback without a pending local op");
    }
    const types = clients.pendingTypes[clients.pendingTypes.length - 1];
    const [lo, hi] = clients.pending[clients.pending.length - 1];
    // an annotate's MTE_OP_RBKEY records (packing.py add_rollback): per key it
    // set, the older pending annotates that set the key, latest first, then the
    // base entry; every check that can throw comes before any record
    const aux = new Map();
    for (let ls = hi; ls >= lo; ls--) {
      if (types[ls - lo] !== OP_ANNOTATE) continue;
      if (!clients.annSlot.has(ls) || clients.noRollback.has(ls)) {
        throw new MergeTreeError(E_UNSUPPORTED, "rollback of an annotate the engine does not track");
      }
      const mine = clients.annProps.get(ls);
      for (const [x, kv] of clients.annProps) {
        if (x > ls && (x < lo || x > hi) && Array.from(mine.keys()).some((k) => kv.has(k))) {
          throw new MergeTreeError(E_UNSUPPORTED, "rollback under a newer pending annotate of the same key");
        }
      }
      const recs = [];
      for (const k of mine.keys()) {
        const older = Array.from(clients.annProps.keys()).filter((x) => x < ls && clients.annProps.get(x).has(k))
          .sort((p, q) => q - p);
        if (older.some((x) => !clients.annSlot.has(x))) {
          throw new MergeTreeError(E_UNSUPPORTED, "rollback past an untracked pending annotate");
        }
        if (older.some((x) => clients.annComb.has(x))) {
          throw new MergeTreeError(E_UNSUPPORTED, "rollback past a pending local incr / consensus");
        }
        for (const x of older) {
          recs.push([x, 0, 0, OP_RBKEY, 0, F_LOCAL, k, clients.annSlot.get(x), clients.annProps.get(x).get(k), NO_PROPS]);
        }
        recs.push([0, 0, 0, OP_RBKEY, 0, F_LOCAL, k, ANNOTATE_SLOTS, 0, NO_PROPS]);
      }
      aux.set(ls, recs);
    }
    clients.regenerated.delete(lo);
    clients.pending.pop();
    clients.pendingTypes.pop();
    const src = this._src(doc);
    const push = (r) => {
      this._put(doc, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9]);
      if (src) src.push({ msg: null, op: undefined, local: true });
    };
    for (let ls = hi; ls >= lo; ls--) {
      const t = types[ls - lo];
      if (t === OP_ANNOTATE) {
        const recs = aux.get(ls);
        push([ls, 0, 0, OP_ROLLBACK, 0, F_LOCAL, t, recs.length, clients.annSlot.get(ls), NO_PROPS]);
        recs.forEach(push);
        clients.annSlot.delete(ls);
        clients.annProps.delete(ls);
      } else if (t !== OP_NOOP) {
        push([ls, 0, 0, OP_ROLLBACK, 0, F_LOCAL, t, 0, 0, NO_PROPS]);
      }
    }
  }

  /** Client.regeneratePendingOp of the oldest pending local message
   *  (client.ts:972-1002), as packing.py add_regen: one MTE_OP_REGEN record per
   *  record of it; the message moves to the end of the pending list.  Returns
   *  [[record index in the doc's part of the batch, localSeq, type], ...]. */
  addRegen(doc, clients) {
    if (!clients.local || clients.pending.length === 0) {
      throw new MergeTreeError(E_STATE, "regenerate without a pending local op");
    }
    const [lo, hi] = clients.pending[0];
    const types = clients.pendingTypes[0];
    const idx = [];
    for (let ls = lo; ls <= hi; ls++) {
      const t = types[ls - lo];
      if (t === OP_NOOP) continue;
      let slot = 0;
      if (t === OP_ANNOTATE) {
        if (!clients.annSlot.has(ls)) {
          throw new MergeTreeError(E_UNSUPPORTED, "regenerate an untracked annotate (more than " + ANNOTATE_SLOTS +
            " pending)");
        }
        slot = clients.annSlot.get(ls);
      }
      idx.push([this.docCount[doc], ls, t]);
      this._put(doc, ls, 0, 0, OP_REGEN, 0, F_LOCAL, t, 0, slot, NO_PROPS);
      const src = this._src(doc);
      if (src) src.push({ msg: null, op: undefined, local: true, regen: true });
    }
    clients.regenerated.add(lo);
    clients.pending.push(clients.pending.shift());
    clients.pendingTypes.push(clients.pendingTypes.shift());
    return idx;
  }

  /** Client.createLocalReferencePosition on getContainingSegment(pos) in the
   *  local view (client.ts:360-364, 1107-1110): an MTE_OP_REF record in an
   *  MTE_DOC_REFS document (as packing.py add_ref).  Returns the slot. */
  addRef(doc, clients, pos, refType) {
    if (!clients.local) throw new MergeTreeError(E_UNSUPPORTED, "local reference in an observer document");
    const rt = checkI32(refType === undefined ? REF_SLIDE_ON_REMOVE : refType, "refType");
    if (rt < 0 || ((rt & REF_TRANSIENT) && (rt & (REF_SLIDE_ON_REMOVE | REF_STAY_ON_REMOVE)))) {
      throw new MergeTreeError(E_INVALID_ARG, "Transient with SlideOnRemove or StayOnRemove (localReference.ts:27-38)");
    }
    if ((rt & REF_SLIDE_ON_REMOVE) && (rt & REF_STAY_ON_REMOVE)) {
      throw new MergeTreeError(E_INVALID_ARG, "SlideOnRemove and StayOnRemove together");
    }
    const p = checkI32(pos, "pos");
    const slot = this._refSlot(clients);
    this._put(doc, 0, 0, 0, OP_REF, 0, F_LOCAL, p, slot, rt, 0);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true });
    return slot;
  }

  _refSlot(clients) {
    if (clients.refFree.length) return clients.refFree.pop();
    if (clients.refNext >= clients.refCap) {
      throw new MergeTreeError(E_CAPACITY, "more than " + clients.refCap +
        " live local references in one document (MergeTreeEngine refCapacity)");
    }
    return clients.refNext++;
  }

  /** A reference a sequenced op creates (createPositionReference with an op,
   *  intervalCollection.ts:639-658): getContainingSegment(pos) in the op's
   *  perspective (its refSeq and sender), then getSlideToSegment; detached when
   *  no segment holds pos there (MTE_OP_REF, b = 2).  The sender takes a short
   *  id as for a message (getClientSequenceArgsForMessage).  Returns the slot. */
  addRefRemote(doc, clients, msg, pos, refType) {
    if (!clients.local) throw new MergeTreeError(E_UNSUPPORTED, "local reference in an observer document");
    const rt = checkI32(refType, "refType");
    if (!(rt & REF_SLIDE_ON_REMOVE) || (rt & (REF_STAY_ON_REMOVE | REF_TRANSIENT))) {
      throw new MergeTreeError(E_INVALID_ARG, "an op creates SlideOnRemove references");
    }
    const seq = checkI32(msg.sequenceNumber, "sequenceNumber");
    const ref = checkI32(msg.referenceSequenceNumber, "referenceSequenceNumber");
    if (ref < clients.minSeq) {
      throw new MergeTreeError(E_INVALID_ARG, "referenceSequenceNumber " + ref + " < minSeq " + clients.minSeq);
    }
    if (msg.clientId === clients.observer) throw new MergeTreeError(E_INVALID_ARG, "a remote op of the local client");
    const short = slotOf(clients, msg.clientId, seq);
    if (short >= MAX_CLIENTS) throw new MergeTreeError(E_CLIENT_RANGE, "an op's reference: short id " + short + " >= 32");
    const slot = this._refSlot(clients);
    this._put(doc, 0, ref, 0, OP_REF, short, F_LOCAL, checkI32(pos, "pos"), slot, rt, 2);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true });
    return slot;
  }

  /** The reference in slot becomes refType (SlideOnRemove) and slides if its
   *  segment is removed and acked (ackInterval, intervalCollection.ts:1819-1902;
   *  MTE_OP_REF, b = 3). */
  setRefSlide(doc, clients, slot, refType) {
    const rt = checkI32(refType, "refType");
    if (!(rt & REF_SLIDE_ON_REMOVE) || (rt & (REF_STAY_ON_REMOVE | REF_TRANSIENT))) {
      throw new MergeTreeError(E_INVALID_ARG, "setRefSlide takes a SlideOnRemove type");
    }
    this._put(doc, 0, 0, 0, OP_REF, 0, F_LOCAL, 0, slot, rt, 3);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true });
  }

  /** removeLocalReferencePosition (mergeTree.ts:2113-2123). */
  removeRef(doc, clients, slot) {
    if (!(slot >= 0 && slot < clients.refNext) || clients.refFree.includes(slot)) {
      throw new MergeTreeError(E_INVALID_ARG, "no local reference in slot " + slot);
    }
    clients.refFree.push(slot);
    this._put(doc, 0, 0, 0, OP_REF, 0, F_LOCAL, -1, slot, 0, 1);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true });
  }

  /** Client.rebasePosition(pos, seqFrom, localSeq) (client.ts:755-786) for a
   *  pending interval op's reconnection (MTE_OP_REF, b = 4; packing.py
   *  add_rebase): answered by one MTE_DELTA_REBASE event of the returned
   *  record index. */
  addRebase(doc, clients, pos, seqFrom, localSeq) {
    if (!clients.local) throw new MergeTreeError(E_UNSUPPORTED, "rebase in an observer document");
    if (!(localSeq >= 0 && localSeq <= clients.localSeq)) {
      throw new MergeTreeError(E_INVALID_ARG, "localSeq " + localSeq + " > the client's " + clients.localSeq);
    }
    const idx = this.docCount[doc];
    this._put(doc, 0, checkI32(seqFrom, "seq"), 0, OP_REF, 0, F_LOCAL, checkI32(pos, "pos"), 0, localSeq, 4);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true, rebase: true });
    return idx;
  }

  /** rebaseLocalInterval's slide of a pending interval end
   *  (intervalCollection.ts:1782-1799; MTE_OP_REF, b = 5): one MTE_DELTA_REBASE
   *  event, the position it moved to or -1. */
  addRefRebase(doc, clients, slot, localSeq) {
    if (!(slot >= 0 && slot < clients.refNext) || clients.refFree.includes(slot)) {
      throw new MergeTreeError(E_INVALID_ARG, "no local reference in slot " + slot);
    }
    if (!(localSeq >= 0 && localSeq <= clients.localSeq)) {
      throw new MergeTreeError(E_INVALID_ARG, "localSeq " + localSeq + " > the client's " + clients.localSeq);
    }
    const idx = this.docCount[doc];
    this._put(doc, 0, 0, 0, OP_REF, 0, F_LOCAL, 0, slot, localSeq, 5);
    const src = this._src(doc);
    if (src) src.push({ msg: null, op: undefined, local: true, rebase: true });
    return idx;
  }

  /** One MergeTree-level call (insertSegments / markRangeRemoved / annotateRange):
   *  a record that does not close a message (no window update). */
  addRaw(doc, seq, ref, msn, client, op) {
    if (client < 0 || client >= MAX_CLIENTS) throw new MergeTreeError(E_CLIENT_RANGE, "client " + client);
    const recs = [];
    this._opRecords(op, recs);
    for (const r of recs) {
      this._put(doc, checkI32(seq, "seq"), checkI32(ref, "refSeq"), msn, r[0], client, r[1], r[2], r[3], r[4], r[5]);
    }
  }

  _src(doc) {
    return this.recSrc ? this.recSrc[doc] : null;
  }

  /** getValidOpRange (client.ts:541-560): a position given as relativePos (no
   *  pos1 / pos2) -> [flags, vid1, vid2, key, offset1, offset2] of an
   *  MTE_OP_RELPOS record the engine resolves (posFromRelativePos,
   *  mergeTree.ts:1369-1392), or null (as packing.py _relpos) */
  _relpos(op, t) {
    // the plain-op fast path: no relative position, nothing allocated
    if (op.relativePos1 === undefined && op.relativePos2 === undefined) return null;
    let flags = 0;
    const vids = [0, 0], offs = [0, 0];
    const spec = [["pos1", "relativePos1", RP_POS1, RP_BEFORE1], ["pos2", "relativePos2", RP_POS2, RP_BEFORE2]];
    for (let i = 0; i < 2; i++) {
      const [pk, rk, pf, bf] = spec[i];
      const rp = op[rk];
      if (pk in op || rp === undefined || rp === null || (i === 1 && op.type === INSERT)) continue;
      if (typeof rp !== "object") throw new MergeTreeError(E_INVALID_ARG, rk + " must be an object");
      flags |= pf;
      if (rp.before) flags |= bf;
      if (rp.offset !== undefined && rp.offset !== null) offs[i] = checkI32(rp.offset, rk + ".offset");
      // an id no marker was ever given cannot match (value 0); a shard interns
      // it, as its documents' markers may be loaded ones the host interned
      // (buildInto renames it to the engine's id, which no other marker has)
      if (rp.id) {
        const v = this.shard ? this.interner.value(rp.id) : this.interner.values.get(canonicalJson(rp.id));
        vids[i] = v === undefined ? 0 : v;
      }
    }
    if (!flags) return null;
    let key = this.interner.keys.get(MARKER_ID_KEY);
    if (key === undefined && this.shard && this.interner.keyNames.length < this.interner.nKeys) {
      key = this.interner.key(MARKER_ID_KEY);
    }
    return [flags, vids[0], vids[1], key === undefined ? NO_PROPS : key, offs[0], offs[1]];
  }

  _opRecords(op, recs, track) {
    if (track && op && typeof op === "object" && op.type !== GROUP) {
      if (!this._srcOps) this._srcOps = [];
      this._srcOps.push(op);  // the op behind the record pushed below
    }
    if (op === null || typeof op !== "object") throw new MergeTreeError(E_INVALID_ARG, "op contents must be an object");
    const t = op.type;
    if (t === GROUP) {
      for (const member of op.ops || []) this._opRecords(member, recs, track);
      return;
    }
    const rel = this._relpos(op, t);
    if ((t === REMOVE || t === ANNOTATE) && !("pos2" in op) && !(rel && (rel[0] & RP_POS2))) {
      throw new MergeTreeError(E_UNSUPPORTED, "range op without pos2");
    }
    if ((t === REMOVE || t === ANNOTATE) && !("pos1" in op) && !(rel && (rel[0] & RP_POS1))) {
      throw new MergeTreeError(E_UNSUPPORTED, "range op without pos1");
    }
    if (rel && (t !== INSERT || (op.seg !== undefined && op.seg !== null))) {
      recs.push([OP_RELPOS, rel[0], rel[1], rel[2], rel[3], [rel[4], rel[5]]]);
      if (track) this._srcOps.push(op);  // the RELPOS record's entry
    }
    if (t === INSERT) {
      const seg = op.seg;
      if (seg === undefined || seg === null) { // applyInsertOp returns false: no segment
        recs.push([OP_NOOP, 0, 0, 0, 0, NO_PROPS]);
        return;
      }
      const pos = checkI32(op.pos1 === undefined ? 0 : op.pos1, "pos1");
      if (typeof seg === "string") {
        const tx = this._text(seg);
        recs.push([OP_INSERT, 0, pos, tx[1], tx[0], NO_PROPS]);
      } else if (typeof seg === "object" && "text" in seg) {
        const tx = this._text(seg.text);
        recs.push([OP_INSERT, 0, pos, tx[1], tx[0], this.props.add(seg.props)]);
      } else if (typeof seg === "object" && "marker" in seg) {
        const rt = checkI32(seg.marker.refType === undefined ? 0 : seg.marker.refType, "refType");
        const off = this._text("\ufffc")[0];  // one reserved unit names the marker in MTE_DOC_REFS documents
        recs.push([OP_INSERT, F_MARKER, pos, rt, off, this.props.add(seg.props)]);
      } else {
        throw new MergeTreeError(E_INVALID_ARG, "Unrecognized IJSONSegment type: " + JSON.stringify(seg));
      }
    } else if (t === REMOVE) {
      recs.push([OP_REMOVE, 0, checkI32(op.pos1 === undefined ? 0 : op.pos1, "pos1"),
        checkI32(op.pos2 === undefined ? 0 : op.pos2, "pos2"), 0, NO_PROPS]);
    } else if (t === ANNOTATE) {
      let flags = 0;
      const comb = op.combiningOp;
      if (comb !== undefined && comb !== null && (comb.name === "incr" || comb.name === "consensus")) {
        // a local incr / consensus: its value map at seq UnassignedSequenceNumber
        // (segmentPropertiesManager.ts:141), as packing.py add_local
        if (this.noCombining) {
          throw new MergeTreeError(E_UNSUPPORTED, "combiningOp " + comb.name + " in a sharded (worker) packer");
        }
        if (comb.name === "consensus" && "defaultValue" in comb) {
          throw new MergeTreeError(E_UNSUPPORTED, "consensus with a defaultValue");
        }
        const props = op.props === undefined ? {} : op.props;
        const ps = this.props.addCombining(props, comb, -1);
        this.props.combOf.set(ps, [props, comb]);
        recs.push([OP_ANNOTATE, F_COMBINE, checkI32(op.pos1 === undefined ? 0 : op.pos1, "pos1"),
          checkI32(op.pos2 === undefined ? 0 : op.pos2, "pos2"), ps, NO_PROPS]);
        return;
      }
      if (comb !== undefined && comb !== null) {
        if (comb.name !== "rewrite") throw new MergeTreeError(E_UNSUPPORTED, "combiningOp " + String(comb.name));
        flags = F_REWRITE;
      }
      const ps = this.props.add(op.props === undefined ? {} : op.props);
      recs.push([OP_ANNOTATE, flags, checkI32(op.pos1 === undefined ? 0 : op.pos1, "pos1"),
        checkI32(op.pos2 === undefined ? 0 : op.pos2, "pos2"), ps, NO_PROPS]);
    } else {
      throw new MergeTreeError(E_INVALID_ARG, "unknown op type " + String(t));
    }
  }

  /** -> {offsets: BigUint64Array, ops: Uint8Array, text: Uint16Array, propsets, props: Uint32Array} */
  build() {
    // counting sort of the records by document, arrival order kept within one
    const nd = this.nDocs, n = this.count;
    const offsets = new BigUint64Array(nd + 1);
    const cur = new Uint32Array(nd);
    let acc = 0;
    for (let d = 0; d < nd; d++) {
      offsets[d] = BigInt(acc);
      cur[d] = acc;
      acc += this.docCount[d];
    }
    offsets[nd] = BigInt(acc);
    const out = new Int32Array(n * 8), R = this.rec, D = this.recDoc;
    for (let k = 0; k < n; k++) {
      const o = cur[D[k]]++ * 8, w = k * 8;
      out[o] = R[w];
      out[o + 1] = R[w + 1];
      out[o + 2] = R[w + 2];
      out[o + 3] = R[w + 3];
      out[o + 4] = R[w + 4];
      out[o + 5] = R[w + 5];
      out[o + 6] = R[w + 6];
      out[o + 7] = R[w + 7];
    }
    const text = this.textBuf.slice(0, this.textUnits);
    return {
      offsets,
      ops: new Uint8Array(out.buffer, 0, n * OP_BYTES),
      text,
      propsets: new Uint32Array(this.props.sets),
      props: new Uint32Array(this.props.entries),
    };
  }

  /** build() straight into a shared batch: the records sorted by document into
   *  `out` (an Int32Array of count * 8), their text offsets (insert a) moved by
   *  textBase and their propset indices (insert b, annotate a) by psBase.
   *  Returns the per-document record offsets relative to `out`. */
  buildInto(out, textBase, psBase, map) {
    const nd = this.nDocs, n = this.count;
    const offsets = new Uint32Array(nd + 1);
    const cur = new Uint32Array(nd);
    let acc = 0;
    for (let d = 0; d < nd; d++) {
      offsets[d] = acc;
      cur[d] = acc;
      acc += this.docCount[d];
    }
    offsets[nd] = acc;
    const R = this.rec, D = this.recDoc;
    for (let k = 0; k < n; k++) {
      const o = cur[D[k]]++ * 8, w = k * 8;
      const w3 = R[w + 3], t = w3 & 0xff;
      let a = R[w + 6], b = R[w + 7];
      if (t === OP_INSERT) {
        a += textBase;
        if ((b >>> 0) !== NO_PROPS) b += psBase;
      } else if (t === OP_ANNOTATE) {
        a += psBase;
      }
      let p1 = R[w + 4], p2 = R[w + 5];
      if (t === OP_RELPOS && map) {
        // a shard's markerId key and marker-id values -> the engine's ids (shards.js)
        if ((a >>> 0) !== NO_PROPS) a = map.keys[a];
        p1 = map.values[p1];
        p2 = map.values[p2];
      }
      out[o] = R[w];
      out[o + 1] = R[w + 1];
      out[o + 2] = R[w + 2];
      out[o + 3] = w3;
      out[o + 4] = p1;
      out[o + 5] = p2;
      out[o + 6] = a;
      out[o + 7] = b;
    }
    return offsets;
  }
}

/** mte_doc_init records + load text for documents created before start(). */
function packDocInits(docs, interner) {
  const buf = Buffer.alloc(docs.length * DOC_INIT_BYTES);
  const props = new PropTable(interner);
  let off = 0;
  const parts = [];
  docs.forEach((d, i) => {
    const o = i * DOC_INIT_BYTES;
    buf.writeUInt32LE(off, o);
    buf.writeUInt32LE(d.text.length, o + 4);
    buf.writeUInt32LE((d.newLengthCalc ? DOC_NEW_LENGTH_CALC : 0) | (d.roundSync ? DOC_ROUND_SYNC : 0) |
      (d.localClient ? DOC_LOCAL_CLIENT : 0) | (d.events ? DOC_EVENTS : 0) | (d.refs ? DOC_REFS : 0) |
      (d.slideEvents ? DOC_SLIDE_EVENTS : 0) | (d.maintenanceEvents ? DOC_MAINT_EVENTS : 0) |
      (d.tree ? DOC_TREE : 0), o + 8);
    buf.writeUInt32LE(props.add(d.props) >>> 0, o + 12);
    buf.writeInt32LE(d.minSeq || 0, o + 16);
    buf.writeInt32LE(d.currentSeq || 0, o + 20);
    parts.push(d.text);
    off += d.text.length;
  });
  const text = utf16(parts.join(""));
  return {
    inits: new Uint8Array(buf.buffer, buf.byteOffset, buf.length),
    text,
    propsets: Uint32Array.from(props.sets),
    props: Uint32Array.from(props.entries),
  };
}

/**
 * A summary body per document -> mte_seg records (include/mte.h) appended to
 * the load text of packDocInits.  Each spec is an IJSONSegmentWithMergeInfo
 * (snapshotChunks.ts:48-78): {json: "text" | {text, props} | {marker:{refType},
 * props}, client?, seq?, removedSeq?, removedClientIds?}; client ids are
 * registered in the document's DocClients in order, as SnapshotLoader.loadBody
 * does (snapshotLoader.ts:90-118); a missing client / seq means NonCollabClient
 * / UniversalSequenceNumber.
 */
function slotOf(clients, longId, seq, max) {
  const s = clients.short(longId, seq);
  if (s >= (max || clients.maxClients)) {
    const hint = !max && clients.maxClients < MAX_CLIENTS_TREE ? " ({tree: true} takes " + MAX_CLIENTS_TREE + ")" : "";
    throw new MergeTreeError(E_CLIENT_RANGE, "client " + String(longId) + ": more than " + (max || clients.maxClients) +
      " clients inside the collab window" + hint);
  }
  return s;
}

function packSegments(docs, clientsOf, inits) {
  const SEG_BYTES = 32;
  let n = 0;
  docs.forEach((d) => { n += d.segments ? d.segments.length : 0; });
  const buf = Buffer.alloc(n * SEG_BYTES);
  const offsets = new BigUint64Array(docs.length + 1);
  const props = new PropTable(inits.interner);
  props.sets = inits.propsetsArr;
  props.entries = inits.propsArr;
  const extra = [];
  let textOff = inits.textUnits;
  let k = 0;
  docs.forEach((d, i) => {
    offsets[i] = BigInt(k);
    for (const sp of d.segments || []) {
      const j = sp.json;
      let text = null, kind = 0, segProps;
      if (typeof j === "string") text = j;
      else if (j && typeof j.text === "string") { text = j.text; segProps = j.props; }
      else if (j && j.marker) { kind = 1 + (j.marker.refType >>> 0); segProps = j.props; }
      else throw new MergeTreeError(E_INVALID_ARG, "segment spec");
      const o = k * SEG_BYTES;
      buf.writeUInt32LE(text === null ? 0 : textOff, o);
      buf.writeUInt32LE(text === null ? 1 : text.length, o + 4);
      buf.writeInt32LE(sp.seq === undefined ? 0 : sp.seq, o + 8);
      const removed = sp.removedSeq !== undefined;
      buf.writeInt32LE(removed ? sp.removedSeq : 0x7fffffff, o + 12);
      // loaded clients are tied to the seq they inserted / removed at, so their
      // slots recycle once minSeq passes it like those of live senders
      let mask = 0;
      const rc = sp.removedClientIds || (sp.removedClient !== undefined ? [sp.removedClient] : []);
      // a loaded segment's ids fit mte_seg (removers: 32 bits)
      for (const id of rc) mask |= 1 << slotOf(clientsOf(i), id, removed ? sp.removedSeq : undefined, MAX_CLIENTS);
      buf.writeUInt32LE(mask >>> 0, o + 16);
      buf.writeInt32LE(sp.client === undefined ? -1 : slotOf(clientsOf(i), sp.client, sp.seq, MAX_CLIENTS), o + 20);
      buf.writeUInt32LE(kind, o + 24);
      buf.writeUInt32LE(props.add(segProps) >>> 0, o + 28);
      if (text !== null) { extra.push(text); textOff += text.length; }
      k++;
    }
  });
  offsets[docs.length] = BigInt(k);
  return { offsets, segs: new Uint8Array(buf.buffer, buf.byteOffset, buf.length), extraText: extra.join("") };
}

/** The op Client.regeneratePendingOp returns (client.ts:972-1002,
 *  resetPendingDeltaToOps :788-860), from the engine's MTE_DELTA_REGEN records,
 *  as packing.py regen_ops: op = the pending message's original contents, idx =
 *  addRegen's result, recs = [[record, kind, pos, len, textOffset], ...].  One
 *  op per segment of each member's group in document order: an insert re-sends
 *  its part of the original text (with the original seg.props, :829-832). */
function regenOps(op, idx, recs) {
  const flat = [];
  const walk = (o) => {
    if (o && o.type === GROUP) for (const m of o.ops || []) walk(m);
    else if (!(o.type === INSERT && (o.seg === undefined || o.seg === null))) flat.push(o);
  };
  walk(op);
  const byRec = new Map();
  for (const r of recs) {
    if (!(r[1] & DELTA_REGEN)) continue;
    if (!byRec.has(r[0])) byRec.set(r[0], []);
    byRec.get(r[0]).push(r);
  }
  const out = [];
  idx.forEach(([k, , t], j) => {
    const m = flat[j];
    const rs = byRec.get(k) || [];
    if (t === OP_INSERT) {
      const seg = m.seg;
      let base = Infinity;
      for (const r of rs) base = Math.min(base, r[4]);
      for (const r of rs) {
        const text = typeof seg === "string" ? seg : seg.text;
        if (text === undefined) {  // a marker
          out.push({ pos1: r[2], seg, type: INSERT });
          continue;
        }
        const piece = text.substr(r[4] - base, r[3]);
        out.push({ pos1: r[2], seg: typeof seg === "string" || seg.props === undefined ? piece :
          { text: piece, props: seg.props }, type: INSERT });
      }
    } else if (t === OP_REMOVE) {
      for (const r of rs) out.push({ pos1: r[2], pos2: r[2] + r[3], type: REMOVE });
    } else {
      for (const r of rs) {
        const a = { pos1: r[2], pos2: r[2] + r[3], props: m.props, type: ANNOTATE };
        if (m.combiningOp) a.combiningOp = m.combiningOp;
        out.push(a);
      }
    }
  });
  return out.length === 1 ? out[0] : { ops: out, type: GROUP };
}

module.exports = {
  OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_NOOP, OP_ACK, OP_REGEN, DELTA_REGEN, ANNOTATE_SLOTS, F_MARKER, F_MSG_END, F_REWRITE,
  F_LOCAL, NO_PROPS, MAX_CLIENTS, MAX_CLIENTS_TREE, OP_REF, REF_SLIDE_ON_REMOVE, REF_STAY_ON_REMOVE, REF_TRANSIENT,
  INSERT, REMOVE, ANNOTATE, GROUP,
  MergeTreeError, Interner, DocClients, PropTable, BatchBuilder, canonicalJson, packDocInits, packSegments, utf16,
  regenOps,
};
