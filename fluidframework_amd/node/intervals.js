"use strict";
// SharedString interval collections on the engine's local references
// (packages/dds/sequence/src/intervalCollection.ts): an interval's two ends are
// local references of its document (MTE_DOC_REFS, include/mte.h), so the
// engine moves them with their text and slides them on removal; this module
// keeps the collection's bookkeeping -- ids, pending changes, the interval
// properties' pending keys, which end is which reference, the order of the
// interval tree, events, the summary -- as the reference's IntervalCollection
// does, and turns each interval op into the reference records the engine needs:
//   local add / change           StayOnRemove references in the local view
//                                (createSequenceInterval / modify without an op,
//                                intervalCollection.ts:573-609, 660-707)
//   remote add / change          SlideOnRemove references in the op's
//                                perspective, slid at once if their segment is
//                                removed and acked (createPositionReference with
//                                an op, :639-658; MTE_OP_REF b = 2)
//   ack of a local add / change  the ends that no later local change holds
//                                become SlideOnRemove and slide if their
//                                segment is removed and acked (ackInterval,
//                                :1826-1902; MTE_OP_REF b = 3)
//   load from a summary          SlideOnRemove references in the local view
//                                (attachGraph with fromSnapshot, :1337-1374)
// Positions are read back from the engine (localReferencePositionToPosition),
// the tree order from the units the ends sit on (mte_read_ref_order, as
// compareReferencePositions orders them).  Events (IIntervalCollectionEvent,
// :1257-1300) fire for the collection's own edits and the interval ops it
// processes; an end the engine slides off a removed segment inside a merge-tree
// op raises "changeInterval" as the reference's position-change listeners do
// mid-op (:1023-1058): the engine reports the slide (MTE_DELTA_SLIDE) with
// every reference as that record left the document (MTE_DELTA_REFPOS), and the
// events are raised when the batch holding the op is delivered (_onSlides).
// Each entry point first replays what its document has queued (_settle), so
// those events come before the collection's own.
const { MergeTreeError } = require("./packing");
const { RedBlackTree, KeyMovedError } = require("./rbtree");

// ReferenceType (merge-tree ops.ts) and IntervalType (intervalCollection.ts:48-66)
const RefType = { Simple: 0x0, Tile: 0x1, NestBegin: 0x2, NestEnd: 0x4, RangeBegin: 0x10, RangeEnd: 0x20,
  SlideOnRemove: 0x40, StayOnRemove: 0x80, Transient: 0x100 };
const IntervalType = { Simple: 0x0, Nest: 0x1, SlideOnRemove: 0x2, Transient: 0x4 };
const reservedIntervalIdKey = "intervalId";            // intervalCollection.ts:46
const reservedRangeLabelsKey = "referenceRangeLabels";  // merge-tree referencePositions.ts
const UnassignedSequenceNumber = -1;                   // merge-tree constants.ts

// Client.getCurrentSeq without a replay: the last sequenced message the host
// packed (collabWindow.currentSeq after it, client.ts:937-945)
const curSeq = (client) => client.clients.mergeSeq || 0;

/** PropertiesManager (merge-tree segmentPropertiesManager.ts:29-160) for the
 *  interval properties: a key with a pending local change keeps its value
 *  against remote changes until the local change is acked. */
class PropertiesManager {
  constructor() {
    this.pending = new Map();  // key -> pendingKeyUpdateCount
  }
  ackPendingProperties(props) {
    for (const key of Object.keys(props || {})) {
      const n = this.pending.get(key);
      if (n === undefined) continue;
      if (n <= 1) this.pending.delete(key);
      else this.pending.set(key, n - 1);
    }
  }
  addProperties(oldProps, newProps, seq, collaborating) {
    const deltas = {};
    for (const key of Object.keys(newProps)) {
      if (collaborating) {
        if (seq === UnassignedSequenceNumber) {
          this.pending.set(key, (this.pending.get(key) || 0) + 1);
        } else if (this.pending.has(key)) {
          continue;  // shouldModifyKey: a pending local change wins
        }
      }
      const prev = oldProps[key];
      deltas[key] = prev === undefined ? null : prev;
      if (newProps[key] === null) delete oldProps[key];
      else oldProps[key] = newProps[key];
    }
    return deltas;
  }
}

/** compareReferencePositions (merge-tree referencePositions.ts:81-89) on the
 *  engine's order keys: the same unit compares equal; a detached end (-1, no
 *  segment) before every other. */
function compareKeys(a, b) {
  if (a === b) return 0;
  if (a < 0) return -1;
  if (b < 0) return 1;
  return a < b ? -1 : 1;
}

/** SequenceInterval (intervalCollection.ts:387-619): two local references and
 *  the interval's properties. */
class SequenceInterval {
  constructor(collection, start, end, intervalType) {
    this.collection = collection;
    this.start = start;
    this.end = end;
    this.intervalType = intervalType;
    this.properties = {};
    this.propertyManager = new PropertiesManager();
  }
  getIntervalId() {
    return this.properties[reservedIntervalIdKey];
  }
  getProperties() {
    return this.properties;
  }
  addProperties(newProps, collab, seq) {
    return this.propertyManager.addProperties(this.properties, newProps, seq, !!collab);
  }
  /** [start, end] positions in the client's view (-1: detached). */
  positions() {
    const c = this.collection.client;
    return [c.localReferencePositionToPosition(this.start), c.localReferencePositionToPosition(this.end)];
  }
  _keys() {
    if (this._pinKeys) return this._pinKeys;  // the ends as they were (an index removal before they moved)
    const v = this.collection._keyView;  // inside a group op: as one of its members left them
    if (v) return [v(this.start), v(this.end)];
    const c = this.collection.client;
    return [c._refOrder(this.start), c._refOrder(this.end)];
  }
  /** compare (:483-506): start, then end, then id. */
  compare(b) {
    const x = this._keys(), y = b._keys();
    const r = compareKeys(x[0], y[0]) || compareKeys(x[1], y[1]);
    if (r) return r;
    const i = this.getIntervalId(), j = b.getIntervalId();
    return i && j ? (i > j ? 1 : i < j ? -1 : 0) : 0;
  }
  compareStart(b) {
    return compareKeys(this._keys()[0], b._keys()[0]);
  }
  compareEnd(b) {
    return compareKeys(this._keys()[1], b._keys()[1]);
  }
  /** overlaps (:522-527): ends inclusive. */
  overlaps(b) {
    const x = this._keys(), y = b._keys();
    return compareKeys(x[0], y[1]) <= 0 && compareKeys(x[1], y[0]) >= 0;
  }
  /** serialize (:456-474). */
  serialize() {
    const [start, end] = this.positions();
    const out = { end, intervalType: this.intervalType, sequenceNumber: curSeq(this.collection.client), start };
    if (this.properties) out.properties = this.properties;
    return out;
  }
}

/** A Transient interval at positions of the client's view, for queries
 *  (createPositionReference with Transient, :639-658: no unit there ->
 *  detached). */
class TransientInterval {
  constructor(client, start, end) {
    this.k = [start === undefined ? undefined : client._unitKeyAt(start),
      end === undefined ? undefined : client._unitKeyAt(end)];
  }
  _keys() {
    return this.k;
  }
}

/** The ends of an interval as they were, for a "changeInterval" event's
 *  previousInterval (position information only): read as Transient references,
 *  as emitChange makes them (:1387-1410) -- an end that slid off the string
 *  still finds its removed segment while the document holds it
 *  (mte_read_refs_transient).  _src: the ends themselves, for the ones the
 *  changed interval keeps. */
function snapshotInterval(ival) {
  const c = ival.collection.client;
  const ref = (r) => {
    r.transientRead = true;
    const position = c.localReferencePositionToPosition(r);
    delete r.transientRead;
    return { snapshot: true, position, refType: RefType.Transient };
  };
  const prev = new SequenceInterval(ival.collection, ref(ival.start), ref(ival.end), ival.intervalType);
  prev.properties = Object.assign({}, ival.properties);
  prev._src = [ival.start, ival.end];
  return prev;
}

function endpointTypes(intervalType, op, fromSnapshot) {
  if (intervalType & IntervalType.Transient) throw new MergeTreeError(-9, "Can not add transient intervals");
  let b = RefType.RangeBegin, e = RefType.RangeEnd;
  if (intervalType === IntervalType.Nest) {
    b = RefType.NestBegin;
    e = RefType.NestEnd;
  }
  // createSequenceInterval (:679-689): SlideOnRemove once created by an op or
  // from a summary, StayOnRemove while a local creation is pending
  const slide = op || fromSnapshot ? RefType.SlideOnRemove : RefType.StayOnRemove;
  return [b | slide, e | slide];
}

/** decompressInterval / compressInterval (:123-149). */
function decompressInterval(x, label) {
  return { start: x[0], end: x[1], sequenceNumber: x[2], intervalType: x[3],
    properties: Object.assign({}, x[4], { [reservedRangeLabelsKey]: [label] }) };
}
function compressInterval(v) {
  const props = Object.assign({}, v.properties);
  delete props[reservedRangeLabelsKey];  // {..., referenceRangeLabels: undefined} drops it from the JSON
  return [v.start, v.end, v.sequenceNumber, v.intervalType, props];
}

/** IntervalCollection (intervalCollection.ts:1309-2102) of one label on one
 *  BatchClient ({localClient, refs} document).  emitter.emit(opName, undefined,
 *  value, metadata) receives the ops to send, as SharedString's value-type
 *  emitter does; the sequenced messages come back through process().
 *  serialized: a summary of the collection (serializeInternal's
 *  ISerializedIntervalCollectionV2, or a V1 array) to load. */
class IntervalCollection {
  constructor(client, label, emitter, serialized) {
    this.client = client;
    this.label = label;
    this.emitter = emitter || { emit() {} };
    this.byId = new Map();
    this.pendingStart = new Map();  // id -> pending local changes of the start (FIFO)
    this.pendingEnd = new Map();
    this.nextLocalId = 0;
    this.listeners = new Map();
    this.stamp = 0;  // index insertion order
    // the end tree (LocalIntervalCollection.endIntervalTree, :728-757): the
    // reference's red-black tree keyed by the intervals' ends
    // (compareSequenceIntervalEnds, :1025-1026), put / removed exactly where
    // the reference puts / removes (addIntervalToIndex, removeIntervalFromIndex),
    // with no conflict resolver (IntervalCollection.addConflictResolver is the
    // application's to call): previousInterval / nextInterval read it
    this.endTree = new RedBlackTree((a, b) => compareKeys(a._keys()[1], b._keys()[1]));
    this._endOrder = 0;
    if (serialized) this._load(serialized);
  }

  // ---- the end tree ----------------------------------------------------------------
  /** The end tree follows every put / remove of the reference only when the
   *  document reports its references' slides (createClient {events: true}):
   *  an end that slides re-enters the tree there (_onSlides).  Without them
   *  the tree is rebuilt at each query, the intervals put in index order --
   *  the reference's tree where no end has slid. */
  _tracksSlides() {
    const e = this.client.engine;
    return !!(e && e.docs && e.docs[this.client.doc] && e.docs[this.client.doc].events);
  }
  _endPut(ival) {
    if (this.client.traceEnd) process.stderr.write(`    PUT ${ival.getIntervalId()} ${JSON.stringify(ival._keys())}\n`);
    if (this._tracksSlides()) this.endTree.put(ival, ival);
  }
  _endRemove(ival) {
    if (this.client.traceEnd) process.stderr.write(`    DEL ${ival.getIntervalId()} ${JSON.stringify(ival._keys())}\n`);
    if (!this._tracksSlides()) return;
    try {
      this.endTree.remove(ival);
    } catch (e) {
      if (!(e instanceof KeyMovedError)) throw e;
      // an end whose unit the zamboni took no longer compares as it did (the
      // reference keeps comparing the removed segment's stale ordinal,
      // referencePositions.ts:81-89): the descent left the tree -- rebuilt,
      // the intervals put in index order, without this one
      this.endTree = new RedBlackTree(this.endTree.compare);
      for (const x of Array.from(this.byId.values()).sort((a, b) => a.stamp - b.stamp)) {
        if (x !== ival) this.endTree.put(x, x);
      }
      this.endRebuilds = (this.endRebuilds || 0) + 1;
    }
  }
  _ends() {
    if (this._tracksSlides()) return this.endTree;
    const t = new RedBlackTree(this.endTree.compare);
    for (const x of Array.from(this.byId.values()).sort((a, b) => a.stamp - b.stamp)) t.put(x, x);
    return t;
  }

  // ---- events (TypedEventEmitter<IIntervalCollectionEvent>) ------------------------
  on(event, listener) {
    if (!this.listeners.has(event)) this.listeners.set(event, []);
    this.listeners.get(event).push(listener);
    return this;
  }
  off(event, listener) {
    const l = this.listeners.get(event);
    if (l) {
      const i = l.indexOf(listener);
      if (i >= 0) l.splice(i, 1);
    }
    return this;
  }
  _has(event) {
    const l = this.listeners.get(event);
    return !!l && l.length > 0;
  }
  _emit(event, ...args) {
    const l = this.listeners.get(event);
    if (l) for (const f of l.slice()) f(...args);
  }
  /** emitChange (:1387-1410): while the listeners run, the ends the changed
   *  interval shares with the previous one are Transient too. */
  _emitChange(ival, prev, local, op) {
    const shared = [ival.start, ival.end].filter((r) => prev._src && prev._src.includes(r));
    for (const r of shared) r.transientRead = true;
    try {
      this._emit("changeInterval", ival, prev, local, op);
    } finally {
      for (const r of shared) delete r.transientRead;
    }
  }


  // ---- references ------------------------------------------------------------
  _localRef(pos, type) {
    return this.client.createLocalReferencePosition(pos, 0, type);
  }
  _opRef(pos, type, op) {
    // createPositionReference with an op asserts SlideOnRemove (0x2f5)
    if (!(type & RefType.SlideOnRemove)) throw new MergeTreeError(-1, "op create references must be SlideOnRemove");
    return this.client._createRefFromOp(op, pos, type);
  }
  _drop(ref) {
    if (ref) this.client.removeLocalReferencePosition(ref);
  }

  _create(start, end, intervalType, op, fromSnapshot) {
    const [bt, et] = endpointTypes(intervalType, op, fromSnapshot);
    const s = op ? this._opRef(start, bt, op) : this._localRef(start, bt);
    const e = op ? this._opRef(end, et, op) : this._localRef(end, et);
    const ival = new SequenceInterval(this, s, e, intervalType);
    ival.addProperties({ [reservedRangeLabelsKey]: [this.label] });
    return ival;
  }

  _index(ival) {
    ival.stamp = ++this.stamp;
    this.byId.set(ival.getIntervalId(), ival);
    this._endPut(ival);  // addIntervalToIndex (:975-987)
  }

  _addInterval(start, end, intervalType, props, op, fromSnapshot) {
    const ival = this._create(start, end, intervalType, op, fromSnapshot);
    if (props) ival.addProperties(props);
    if (ival.properties[reservedIntervalIdKey] === undefined) {
      ival.properties[reservedIntervalIdKey] = `${this.client.longClientId}-${this.label}-${this.nextLocalId++}`;
    }
    this._index(ival);
    return ival;
  }

  /** attachGraph with saved intervals (:1337-1374): each end a SlideOnRemove
   *  reference at its position in the local view; no events. */
  _load(serialized) {
    const list = Array.isArray(serialized) ? serialized
      : serialized.intervals.map((x) => decompressInterval(x, serialized.label));
    const n = list.length ? this.client.getLength() : 0;
    for (const v of list) {
      // createPositionReferenceFromSegoff without a segment (:629-636)
      if (!(v.start >= 0 && v.start < n && v.end >= 0 && v.end < n)) {
        throw new MergeTreeError(-1, "Non-transient references need segment");
      }
    }
    for (const v of list) {
      this._ensureId(v);
      const ival = this._create(v.start, v.end, v.intervalType, undefined, true);
      if (v.properties) ival.addProperties(v.properties);
      this._index(ival);
    }
  }

  /** LocalIntervalCollection.changeInterval -> SequenceInterval.modify
   *  (:573-609, 999-1012): new references for the ends given (StayOnRemove
   *  without an op), the others kept. */
  _changeInterval(ival, start, end, op) {
    const retype = (t) => (op ? t : ((t & ~RefType.SlideOnRemove) | RefType.StayOnRemove));
    this._endRemove(ival);  // removeExistingInterval of the interval modify replaced (:999-1012)
    if (start !== undefined) {
      const old = ival.start;
      ival.start = op ? this._opRef(start, retype(old.refType), op) : this._localRef(start, retype(old.refType));
      this._drop(old);
    }
    if (end !== undefined) {
      const old = ival.end;
      ival.end = op ? this._opRef(end, retype(old.refType), op) : this._localRef(end, retype(old.refType));
      this._drop(old);
    }
    ival.stamp = ++this.stamp;
    this._endPut(ival);  // add(newInterval)
    return ival;
  }

  _remove(ival) {
    this._endRemove(ival);  // removeIntervalFromIndex (:960-968), while its ends still compare
    this.byId.delete(ival.getIntervalId());
    this._drop(ival.start);
    this._drop(ival.end);
  }

  // ---- local edits (each returns as the reference does and emits its op) ------
  getIntervalById(id) {
    return this.byId.get(id);
  }

  /** The local op metadata an emitted op carries ({localSeq}, :1454): the
   *  client's merge-tree localSeq when it was made (its pending ops up to there
   *  are in the view the op's positions refer to) -- what rebaseLocalInterval
   *  takes back on reconnection. */
  _meta() {
    return { localSeq: this.client.clients.localSeq };
  }

  /** The value type's rebase of a pending op for re-sending (makeOpsMap,
   *  :1163-1172, 1191-1200): a delete goes out unchanged (by id), an add or a
   *  change through rebaseLocalInterval.  meta: the op's local metadata. */
  rebaseOp(opName, value, meta) {
    if (opName === "delete") return value;
    return this.rebaseLocalInterval(opName, value, meta.localSeq);
  }

  /** rebaseLocalInterval (:1735-1803) for reconnection (the ops map's rebase,
   *  :1163-1172): a pending add / change re-made at the positions
   *  Client.rebasePosition gives its ends (from the view it was made in: its
   *  sequenceNumber and localSeq) and the current seq, its pending change
   *  re-queued; undefined -- the op is sent empty -- when an end slid off the
   *  string (the interval is dropped, no event).  An end of the interval whose
   *  segment was removed and acked since moves to its slide target at that
   *  localSeq (changeInterval with localSeq, :1782-1799).  Replays what is
   *  queued (flush + sync). */
  rebaseLocalInterval(opName, v, localSeq) {
    this.client._settle();
    const id = v.properties && v.properties[reservedIntervalIdKey];
    const ival = id === undefined ? undefined : this.byId.get(id);
    const reqs = [];
    if (v.start !== undefined) reqs.push({ pos: v.start, seqFrom: v.sequenceNumber, localSeq });
    if (v.end !== undefined) reqs.push({ pos: v.end, seqFrom: v.sequenceNumber, localSeq });
    const nPos = reqs.length;
    // the slides ride in the same replay (ignored if an end detaches); the
    // interval leaves the end tree with its ends as they were (removeExistingInterval
    // of the unmodified interval)
    const before = ival && this._tracksSlides() ? ival._keys() : null;
    if (ival) reqs.push({ slot: ival.start.slot, localSeq }, { slot: ival.end.slot, localSeq });
    const r = reqs.length ? this.client._rebase(reqs) : [];
    let k = 0;
    const start = v.start === undefined ? undefined : r[k++];
    const end = v.end === undefined ? undefined : r[k++];
    const rebased = { start, end, intervalType: v.intervalType, sequenceNumber: curSeq(this.client),
      properties: v.properties };
    if (opName === "change" && id !== undefined && (this.pendingStart.has(id) || this.pendingEnd.has(id))) {
      this._removePending(v);
      this._addPending(id, rebased);
    }
    if (start === -1 || end === -1) {
      if (ival) this._remove(ival);  // removeExistingInterval: no event
      return undefined;
    }
    if (ival && (r[nPos] !== -1 || r[nPos + 1] !== -1)) {  // re-added by changeInterval (removeExisting + add)
      // modify makes each moved end a new reference (createPositionReference,
      // :573-609), pushed onto the "at" list of its offset, start first
      for (const [k, lref] of [[nPos, ival.start], [nPos + 1, ival.end]]) {
        if (r[k] === -1) continue;
        lref.list = 1;
        lref.listOrder = lref.constructor.pushStamp();
      }
      ival.stamp = ++this.stamp;
      ival._pinKeys = before;
      this._endRemove(ival);
      delete ival._pinKeys;
      this._endPut(ival);
    }
    return rebased;
  }

  /** IntervalCollection.add (:1430-1460). */
  add(start, end, intervalType, props) {
    this.client._settle();
    const ival = this._addInterval(start, end, intervalType, props);
    this.emitter.emit("add", undefined, { end, intervalType, properties: Object.assign({}, ival.properties),
      sequenceNumber: curSeq(this.client), start }, this._meta());
    this._emit("addInterval", ival, true, undefined);
    return ival;
  }

  /** IntervalCollection.removeIntervalById (:1493-1502) -> deleteExistingInterval (:1462-1491). */
  removeIntervalById(id) {
    this.client._settle();
    const ival = this.byId.get(id);
    if (ival) {
      // serialize() without the ends' positions (a replay per delete; receivers
      // look the interval up by id, ackDelete :1943-1963)
      const v = { intervalType: ival.intervalType, sequenceNumber: curSeq(this.client),
        properties: Object.assign({}, ival.properties) };
      this._remove(ival);
      this.emitter.emit("delete", undefined, v, this._meta());
      this._emit("deleteInterval", ival, true, undefined);
    }
    return ival;
  }

  /** IntervalCollection.changeProperties (:1510-1537). */
  changeProperties(id, props) {
    this.client._settle();
    if (typeof id !== "string") throw new MergeTreeError(-1, "Change API requires an ID that is a string");
    if (!props) throw new MergeTreeError(-1, "changeProperties should be called with a property set");
    const ival = this.byId.get(id);
    if (ival) {
      const deltas = ival.addProperties(props, true, UnassignedSequenceNumber);
      this.emitter.emit("change", undefined, { intervalType: ival.intervalType,
        sequenceNumber: curSeq(this.client),
        properties: Object.assign({}, props, { [reservedIntervalIdKey]: id }) }, this._meta());
      this._emit("propertyChanged", ival, deltas, true, undefined);
    }
  }

  /** IntervalCollection.change (:1546-1577): the ends given move (StayOnRemove
   *  until the change is acked); a pending change per end. */
  change(id, start, end) {
    this.client._settle();
    if (typeof id !== "string") throw new MergeTreeError(-1, "Change API requires an ID that is a string");
    const ival = this.byId.get(id);
    if (!ival) return undefined;
    const prev = this._has("changeInterval") ? snapshotInterval(ival) : null;
    this._changeInterval(ival, start, end);
    const v = { start, end, intervalType: ival.intervalType, sequenceNumber: curSeq(this.client),
      properties: { [reservedIntervalIdKey]: id } };
    this.emitter.emit("change", undefined, v, this._meta());
    this._addPending(id, v);
    if (prev) this._emitChange(ival, prev, true, undefined);
    return ival;
  }

  _addPending(id, v) {
    const put = (m) => {
      if (!m.has(id)) m.set(id, []);
      m.get(id).push(v);
    };
    if (v.start !== undefined) put(this.pendingStart);
    if (v.end !== undefined) put(this.pendingEnd);
  }
  _removePending(v) {
    const id = v.properties && v.properties[reservedIntervalIdKey];
    const take = (m) => {
      const q = m.get(id);
      if (!q) return;
      const p = q.shift();
      if (q.length === 0) m.delete(id);
      if (p.start !== v.start || p.end !== v.end) throw new MergeTreeError(-1, "Mismatch in pending changes");
    };
    if (v.start !== undefined) take(this.pendingStart);
    if (v.end !== undefined) take(this.pendingEnd);
  }

  // ---- sequenced interval messages (makeOpsMap, :1163-1221) --------------------
  /** One sequenced interval op (SharedSegmentSequence.processCore ->
   *  intervalCollections.tryProcessMessage, sequence.ts:628-648): the merge-tree
   *  window does not move. */
  process(opName, value, local, op) {
    this.client._settle();
    if (!value) return;  // deleted while rebasing
    if (opName === "add") this.ackAdd(value, local, op);
    else if (opName === "delete") this.ackDelete(value, local, op);
    else if (opName === "change") this.ackChange(value, local, op);
    else throw new MergeTreeError(-1, "unknown interval op " + String(opName));
  }

  _ensureId(v) {
    let id = v.properties && v.properties[reservedIntervalIdKey];
    if (id === undefined) {  // ensureSerializedId (:777-796): a legacy id from the ends
      id = `legacy${v.start}-${v.end}`;
      v.properties = Object.assign({}, v.properties || {}, { [reservedIntervalIdKey]: id });
    }
    return id;
  }

  /** ackAdd (:1905-1940). */
  ackAdd(v, local, op) {
    if (local) {
      const ival = this.byId.get(v.properties && v.properties[reservedIntervalIdKey]);
      if (ival) this._ackInterval(ival, op);
      return;
    }
    this._ensureId(v);
    const ival = this._addInterval(v.start, v.end, v.intervalType, v.properties, op);
    this._emit("addInterval", ival, false, op);
  }

  /** ackDelete (:1943-1963). */
  ackDelete(v, local, op) {
    if (local) return;
    const ival = this.byId.get(this._ensureId(v));
    if (ival) {
      this._remove(ival);
      this._emit("deleteInterval", ival, false, op);
    }
  }

  /** ackChange (:1641-1704). */
  ackChange(v, local, op) {
    if (local) this._removePending(v);
    const props = Object.assign({}, v.properties || {});
    const id = props[reservedIntervalIdKey];
    if (id === undefined) throw new MergeTreeError(-1, "id must exist on the interval");
    delete props[reservedIntervalIdKey];
    const ival = this.byId.get(id);
    if (!ival) return;  // removed locally
    if (local) {
      ival.propertyManager.ackPendingProperties(v.properties || {});
      this._ackInterval(ival, op);
      return;
    }
    const start = this.pendingStart.has(id) ? undefined : v.start;
    const end = this.pendingEnd.has(id) ? undefined : v.end;
    let prev = null;
    if (start !== undefined || end !== undefined) {
      prev = this._has("changeInterval") ? snapshotInterval(ival) : null;
      this._changeInterval(ival, start, end, op);
    }
    const deltas = ival.addProperties(props, true, op.sequenceNumber);
    if (prev) this._emitChange(ival, prev, false, op);
    if (Object.keys(props).length > 0) this._emit("propertyChanged", ival, deltas, false, op);
  }

  /** ackInterval (:1826-1902): the StayOnRemove ends no pending change holds
   *  become SlideOnRemove and slide if their segment is removed and acked;
   *  "changeInterval" when one slid. */
  _ackInterval(ival, op) {
    const stay = (r) => (r.refType & RefType.StayOnRemove) !== 0;
    if (!stay(ival.start) && !stay(ival.end)) return;
    const id = ival.getIntervalId();
    const watch = this._has("changeInterval");
    const prev = watch ? snapshotInterval(ival) : null;
    const before = ival._keys();
    const slide = (r) => (r.refType & ~RefType.StayOnRemove) | RefType.SlideOnRemove;
    if (!this.pendingStart.has(id) && stay(ival.start)) this.client._setRefSlide(ival.start, slide(ival.start));
    if (!this.pendingEnd.has(id) && stay(ival.end)) this.client._setRefSlide(ival.end, slide(ival.end));
    const after = ival._keys();
    // an end that moved is a new reference there (createPositionReferenceFromSegoff,
    // :1862-1890): pushed onto its offset's "at" list
    for (const w of [0, 1]) {
      if (after[w] === before[w]) continue;
      const r = w ? ival.end : ival.start;
      r.list = 1;
      r.listOrder = r.constructor.pushStamp();
    }
    if (after[0] !== before[0] || after[1] !== before[1]) {
      // removeExistingInterval (with the ends as they were) + add (:1862-1899)
      ival._pinKeys = before;
      this._endRemove(ival);
      delete ival._pinKeys;
      this._endPut(ival);
      ival.stamp = ++this.stamp;
      if (watch) this._emitChange(ival, prev, true, op);
    }
  }

  // ---- ends sliding inside merge-tree ops --------------------------------------
  /** The references one merge-tree op slid off removed-and-acked segments
   *  (MTE_DELTA_SLIDE records, BatchClient._deliver; back: the references
   *  as that record left the document, MTE_DELTA_REFPOS -- positions and order
   *  keys are read from it, not from the document after the batch).  The reference calls each
   *  sliding end's beforeSlide / afterSlide (localReference.ts:436-447,
   *  471-480, mergeTree.ts:921-950), which for an interval end are the
   *  collection's position-change listeners (addIntervalListeners,
   *  intervalCollection.ts:1023-1058): the interval leaves the index, its end
   *  moves, it is re-added and one "changeInterval" is raised, local = true and
   *  no op (attachGraph's onPositionChange -> emitChange, :1350-1353).
   *  The engine reports the removed segments in the order the reference slides
   *  them (a remote remove's overlapped segments, then its new ones; an ack's
   *  segments one by one, a reference sliding again off a later one), each
   *  segment's references together; within a segment the reference walks its
   *  LocalReferenceCollection -- by offset, then the before / at / after lists
   *  in list order (localReference.ts:181-215), which the ends' list places
   *  track.  previousInterval holds the ends as they were (Transient clones: a
   *  removed segment's position), the interval the ends as they are at that
   *  moment: an end that slides later in the same op still sits where it was. */
  _onSlides(slides, back) {
    if (this.byId.size === 0) return;
    const owner = new Map();  // slot -> [interval, 0 start | 1 end]
    for (const x of this.byId.values()) {
      if (x.start && x.start.slot >= 0) owner.set(x.start.slot, [x, 0]);
      if (x.end && x.end.slot >= 0) owner.set(x.end.slot, [x, 1]);
    }
    const mine = slides.filter((r) => owner.has(r.slot));
    if (mine.length === 0) return;
    if (!back) throw new MergeTreeError(-1, "slide records without the references' snapshot (MTE_DELTA_REFPOS)");
    const ref = (r) => { const [x, w] = owner.get(r.slot); return w ? x.end : x.start; };
    // runs of one removed segment each, in the engine's order (r.seg: the unit
    // the end left, as an order key after the op, so r.seg - r.off keys its
    // segment; -1 once the zamboni took it)
    // (r.off counts from the segment's first unit, a merged leaf's items too)
    const runs = [];
    let run = null, runId;
    for (const r of mine) {
      const id = r.seg >= 0 ? r.seg - r.off : -2 - r.pos;
      if (!run || id !== runId) {
        run = [];
        runs.push(run);
        runId = id;
      }
      run.push(r);
    }
    const c = this.client;
    // positions as the op left them; inside a remote group op, as its member
    // that slid these left them (back: the later members undone)
    const now = (lref) => back.at(lref.slot, false);
    const nowT = (lref) => back.at(lref.slot, true);
    // each sliding end's records in order: where it sits before each one
    const queue = new Map();
    for (const r of mine) {
      if (!queue.has(r.slot)) queue.set(r.slot, []);
      queue.get(r.slot).push(r);
    }
    const posNow = new Map();
    for (const [slot, q] of queue) posNow.set(slot, q[0].pos);
    // an end that slid off the string keeps its removed segment (removeLocalRef
    // relinks it there, localReference.ts:299-316): the Transient clone a later
    // previousInterval takes of it (:1024-1039) reads that segment's position
    const ghost = new Map();
    // the end tree compares the ends as they stand at each slide: an end still
    // to slide keeps the key of the unit it sits on (pinned)
    // every end as this record left it
    this._keyView = (lref) => back.key(lref.slot);
    const keyNow = (lref) => back.key(lref.slot);
    const touched = new Set(mine.map((r) => owner.get(r.slot)[0]));
    for (const x of touched) x._pinKeys = x._keys();
    for (const [slot, q] of queue) if (q[0].seg >= 0) owner.get(slot)[0]._pinKeys[owner.get(slot)[1]] = q[0].seg;
    const watch = this._has("changeInterval");
    // the events below are the ones a merge-tree op raises (for listeners that
    // tell them apart: the op is applied, its batch being delivered)
    this.inMergeTreeOp = true;
    try {
      for (const seg of runs) {
        seg.sort((a, b) => (a.off - b.off) || (ref(a).list - ref(b).list) || (ref(a).listOrder - ref(b).listOrder));
        let base = null, idx = 0;
        for (const r of seg) {
          const [ival, which] = owner.get(r.slot);
          const lref = ref(r);
          const q = queue.get(r.slot);
          q.shift();
          const at = posNow.get(r.slot);
          const next = q.length ? q[0].pos : now(lref);
          const other = which ? ival.start : ival.end;
          const otherPos = posNow.has(other.slot) ? posNow.get(other.slot) : now(other);
          // a previous interval's end is a Transient clone (cloneRef, :1024-1039):
          // an end that slid off the string in an earlier op still reads its
          // removed segment's position
          const otherPrev = otherPos !== -1 ? otherPos
            : (ghost.has(other.slot) ? ghost.get(other.slot) : (posNow.has(other.slot) ? -1 : nowT(other)));
          // beforeSlide: out of the index (removeIntervalFromIndex, :1042-1047)
          this._endRemove(ival);
          posNow.set(r.slot, next);
          if (next === -1) ghost.set(r.slot, at);
          ival._pinKeys[which] = q.length && q[0].seg >= 0 ? q[0].seg : keyNow(lref);
          // its place among the new segment's references: addBeforeTombstones
          // puts one segment's references, in order, in front of offset 0's
          // before list; addAfterTombstones pushes them onto the last offset's
          // after list (localReference.ts:422-485)
          if (r.moves) {
            if (r.after) {
              lref.list = 2;
              lref.listOrder = lref.constructor.pushStamp();
            } else {
              if (base === null) base = -lref.constructor.pushStamp() * 65536;
              lref.list = 0;
              lref.listOrder = base + idx++;
            }
          }
          // afterSlide: back in (addIntervalToIndex), then onPositionChange (:1048-1053)
          ival.stamp = ++this.stamp;
          this._endPut(ival);
          if (watch) {
            const snap = (p) => ({ snapshot: true, position: p, refType: RefType.Transient });
            const prev = new SequenceInterval(this, snap(which ? otherPrev : at), snap(which ? at : otherPrev),
              ival.intervalType);
            prev.properties = Object.assign({}, ival.properties);
            ival.start.pinned = which ? otherPos : next;
            ival.end.pinned = which ? next : otherPos;
            try {
              this._emit("changeInterval", ival, prev, true, undefined);
            } finally {
              delete ival.start.pinned;
              delete ival.end.pinned;
            }
          }
        }
      }
    } finally {
      for (const x of touched) delete x._pinKeys;
      delete this._keyView;
      this.inMergeTreeOp = false;
    }
  }

  // ---- queries (LocalIntervalCollection, :760-913) ------------------------------
  /** The interval tree's order (compare, :483-506). */
  _sorted() {
    this.client._settle();
    return Array.from(this.byId.values()).sort((a, b) => a.compare(b));
  }

  [Symbol.iterator]() {
    return this._sorted()[Symbol.iterator]();
  }

  map(fn) {
    for (const x of this._sorted()) fn(x);
  }

  /** gatherIterationResults (:802-879): whole tree, or the intervals whose start
   *  (and end) equal those of a Transient interval at the positions given. */
  gatherIterationResults(results, iteratesForward, start, end) {
    let all = this._sorted();
    if (!iteratesForward) all = all.reverse();
    if (start === undefined && end === undefined) {
      results.push(...all);
      return;
    }
    const t = new TransientInterval(this.client, start, end);
    for (const x of all) {
      const k = x._keys();
      if (start !== undefined && compareKeys(t.k[0], k[0]) !== 0) continue;
      if (end !== undefined && compareKeys(t.k[1], k[1]) !== 0) continue;
      results.push(x);
    }
  }

  CreateForwardIteratorWithStartPosition(startPosition) {
    const r = [];
    this.gatherIterationResults(r, true, startPosition);
    return r[Symbol.iterator]();
  }
  CreateBackwardIteratorWithStartPosition(startPosition) {
    const r = [];
    this.gatherIterationResults(r, false, startPosition);
    return r[Symbol.iterator]();
  }
  CreateForwardIteratorWithEndPosition(endPosition) {
    const r = [];
    this.gatherIterationResults(r, true, undefined, endPosition);
    return r[Symbol.iterator]();
  }
  CreateBackwardIteratorWithEndPosition(endPosition) {
    const r = [];
    this.gatherIterationResults(r, false, undefined, endPosition);
    return r[Symbol.iterator]();
  }

  /** findOverlappingIntervals (:881-895): the intervals overlapping a
   *  Transient interval at [startPosition, endPosition] (ends inclusive), in
   *  tree order. */
  findOverlappingIntervals(startPosition, endPosition) {
    this.client._settle();
    if (endPosition < startPosition || this.byId.size === 0) return [];
    const t = new TransientInterval(this.client, startPosition, endPosition);
    return this._sorted().filter((x) => {
      const k = x._keys();
      return compareKeys(k[0], t.k[1]) <= 0 && compareKeys(k[1], t.k[0]) >= 0;
    });
  }

  /** previousInterval / nextInterval (:897-913): the data of the end tree's
   *  floor / ceil node of a Transient interval at pos. */
  previousInterval(pos) {
    this.client._settle();
    const n = this._ends().floor(new TransientInterval(this.client, pos, pos));
    return n ? n.data : undefined;
  }
  nextInterval(pos) {
    this.client._settle();
    const n = this._ends().ceil(new TransientInterval(this.client, pos, pos));
    return n ? n.data : undefined;
  }

  // ---- summary --------------------------------------------------------------------
  /** serializeInternal (:1968-1977) -> LocalIntervalCollection.serialize
   *  (:1014-1021): the intervals in tree order, compressed. */
  serializeInternal() {
    return { label: this.label, intervals: this._sorted().map((x) => compressInterval(x.serialize())), version: 2 };
  }
}

module.exports = { IntervalCollection, SequenceInterval, PropertiesManager, RefType, IntervalType, compressInterval,
  decompressInterval };
