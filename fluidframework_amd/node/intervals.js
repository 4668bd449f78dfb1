"use strict";
// SharedString interval collections on the engine's local references
// (packages/dds/sequence/src/intervalCollection.ts): an interval's two ends are
// local references of its document (MTE_DOC_REFS, include/mte.h), so the
// engine moves them with their text and slides them on removal; this module
// keeps the collection's bookkeeping -- ids, pending changes, the interval
// properties' pending keys, which end is which reference -- as the reference's
// IntervalCollection does, and turns each interval op into the reference
// records the engine needs:
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
// Positions are read back from the engine (localReferencePositionToPosition).
const { MergeTreeError } = require("./packing");

// ReferenceType (merge-tree ops.ts) and IntervalType (intervalCollection.ts:48-66)
const RefType = { Simple: 0x0, Tile: 0x1, NestBegin: 0x2, NestEnd: 0x4, RangeBegin: 0x10, RangeEnd: 0x20,
  SlideOnRemove: 0x40, StayOnRemove: 0x80, Transient: 0x100 };
const IntervalType = { Simple: 0x0, Nest: 0x1, SlideOnRemove: 0x2, Transient: 0x4 };
const reservedIntervalIdKey = "intervalId";            // intervalCollection.ts:46
const reservedRangeLabelsKey = "referenceRangeLabels";  // merge-tree referencePositions.ts
const UnassignedSequenceNumber = -1;                   // merge-tree constants.ts

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
  addProperties(newProps, collab, seq) {
    return this.propertyManager.addProperties(this.properties, newProps, seq, !!collab);
  }
  /** [start, end] positions in the client's view (-1: detached). */
  positions() {
    const c = this.collection.client;
    return [c.localReferencePositionToPosition(this.start), c.localReferencePositionToPosition(this.end)];
  }
  serialize() {
    const [start, end] = this.positions();
    return { end, intervalType: this.intervalType, sequenceNumber: this.collection.client.clients.mergeSeq || 0,
      start, properties: this.properties };
  }
}

function endpointTypes(intervalType, op) {
  if (intervalType & IntervalType.Transient) throw new MergeTreeError(-9, "Can not add transient intervals");
  let b = RefType.RangeBegin, e = RefType.RangeEnd;
  if (intervalType === IntervalType.Nest) {
    b = RefType.NestBegin;
    e = RefType.NestEnd;
  }
  // createSequenceInterval (:679-689): SlideOnRemove once created by an op,
  // StayOnRemove while a local creation is pending
  const slide = op ? RefType.SlideOnRemove : RefType.StayOnRemove;
  return [b | slide, e | slide];
}

/** IntervalCollection (intervalCollection.ts:1309-2102) of one label on one
 *  BatchClient ({localClient, refs} document).  emitter.emit(opName, undefined,
 *  value, metadata) receives the ops to send, as SharedString's value-type
 *  emitter does; the sequenced messages come back through process(). */
class IntervalCollection {
  constructor(client, label, emitter) {
    this.client = client;
    this.label = label;
    this.emitter = emitter || { emit() {} };
    this.byId = new Map();
    this.pendingStart = new Map();  // id -> pending local changes of the start (FIFO)
    this.pendingEnd = new Map();
    this.nextLocalId = 0;
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

  _create(start, end, intervalType, op) {
    const [bt, et] = endpointTypes(intervalType, op);
    const s = op ? this._opRef(start, bt, op) : this._localRef(start, bt);
    const e = op ? this._opRef(end, et, op) : this._localRef(end, et);
    const ival = new SequenceInterval(this, s, e, intervalType);
    ival.addProperties({ [reservedRangeLabelsKey]: [this.label] });
    return ival;
  }

  _addInterval(start, end, intervalType, props, op) {
    const ival = this._create(start, end, intervalType, op);
    if (props) ival.addProperties(props);
    if (ival.properties[reservedIntervalIdKey] === undefined) {
      ival.properties[reservedIntervalIdKey] = `${this.client.longClientId}-${this.label}-${this.nextLocalId++}`;
    }
    this.byId.set(ival.getIntervalId(), ival);
    return ival;
  }

  /** LocalIntervalCollection.changeInterval -> SequenceInterval.modify
   *  (:573-609, 999-1012): new references for the ends given (StayOnRemove
   *  without an op), the others kept. */
  _changeInterval(ival, start, end, op) {
    const retype = (t) => (op ? t : ((t & ~RefType.SlideOnRemove) | RefType.StayOnRemove));
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
    return ival;
  }

  _remove(ival) {
    this.byId.delete(ival.getIntervalId());
    this._drop(ival.start);
    this._drop(ival.end);
  }

  // ---- local edits (each returns as the reference does and emits its op) ------
  getIntervalById(id) {
    return this.byId.get(id);
  }

  /** IntervalCollection.add (:1430-1460). */
  add(start, end, intervalType, props) {
    const ival = this._addInterval(start, end, intervalType, props);
    this.emitter.emit("add", undefined, { end, intervalType, properties: Object.assign({}, ival.properties),
      sequenceNumber: this.client.clients.mergeSeq || 0, start }, {});
    return ival;
  }

  /** IntervalCollection.removeIntervalById (:1493-1502). */
  removeIntervalById(id) {
    const ival = this.byId.get(id);
    if (ival) {
      const v = { intervalType: ival.intervalType, sequenceNumber: this.client.clients.mergeSeq || 0,
        properties: Object.assign({}, ival.properties) };
      this._remove(ival);
      this.emitter.emit("delete", undefined, v, {});
    }
    return ival;
  }

  /** IntervalCollection.changeProperties (:1510-1537). */
  changeProperties(id, props) {
    if (typeof id !== "string") throw new MergeTreeError(-1, "Change API requires an ID that is a string");
    if (!props) throw new MergeTreeError(-1, "changeProperties should be called with a property set");
    const ival = this.byId.get(id);
    if (ival) {
      ival.addProperties(props, true, UnassignedSequenceNumber);
      this.emitter.emit("change", undefined, { intervalType: ival.intervalType,
        sequenceNumber: this.client.clients.mergeSeq || 0,
        properties: Object.assign({}, props, { [reservedIntervalIdKey]: id }) }, {});
    }
  }

  /** IntervalCollection.change (:1546-1577): the ends given move (StayOnRemove
   *  until the change is acked); a pending change per end. */
  change(id, start, end) {
    if (typeof id !== "string") throw new MergeTreeError(-1, "Change API requires an ID that is a string");
    const ival = this.byId.get(id);
    if (!ival) return undefined;
    this._changeInterval(ival, start, end);
    const v = { start, end, intervalType: ival.intervalType, sequenceNumber: this.client.clients.mergeSeq || 0,
      properties: { [reservedIntervalIdKey]: id } };
    this.emitter.emit("change", undefined, v, {});
    this._addPending(id, v);
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
      if (ival) this._ackInterval(ival);
      return;
    }
    this._ensureId(v);
    this._addInterval(v.start, v.end, v.intervalType, v.properties, op);
  }

  /** ackDelete (:1943-1963). */
  ackDelete(v, local) {
    if (local) return;
    const ival = this.byId.get(this._ensureId(v));
    if (ival) this._remove(ival);
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
      this._ackInterval(ival);
      return;
    }
    const start = this.pendingStart.has(id) ? undefined : v.start;
    const end = this.pendingEnd.has(id) ? undefined : v.end;
    if (start !== undefined || end !== undefined) this._changeInterval(ival, start, end, op);
    ival.addProperties(props, true, op.sequenceNumber);
  }

  /** ackInterval (:1826-1902): the StayOnRemove ends no pending change holds
   *  become SlideOnRemove and slide if their segment is removed and acked. */
  _ackInterval(ival) {
    const stay = (r) => (r.refType & RefType.StayOnRemove) !== 0;
    if (!stay(ival.start) && !stay(ival.end)) return;
    const id = ival.getIntervalId();
    const slide = (r) => (r.refType & ~RefType.StayOnRemove) | RefType.SlideOnRemove;
    if (!this.pendingStart.has(id) && stay(ival.start)) this.client._setRefSlide(ival.start, slide(ival.start));
    if (!this.pendingEnd.has(id) && stay(ival.end)) this.client._setRefSlide(ival.end, slide(ival.end));
  }

  // ---- queries -----------------------------------------------------------------
  /** Every interval in (start, end, id) order of their positions. */
  [Symbol.iterator]() {
    const all = Array.from(this.byId.values()).map((x) => [x.positions(), x]);
    all.sort((a, b) => a[0][0] - b[0][0] || a[0][1] - b[0][1] ||
      (a[1].getIntervalId() < b[1].getIntervalId() ? -1 : a[1].getIntervalId() > b[1].getIntervalId() ? 1 : 0));
    return all.map((x) => x[1])[Symbol.iterator]();
  }

  /** findOverlappingIntervals (:881-895): the intervals overlapping
   *  [startPosition, endPosition] (ends inclusive). */
  findOverlappingIntervals(startPosition, endPosition) {
    if (endPosition < startPosition) return [];
    const out = [];
    for (const x of this) {
      const [s, e] = x.positions();
      if (s <= endPosition && e >= startPosition) out.push(x);
    }
    return out;
  }
}

module.exports = { IntervalCollection, SequenceInterval, PropertiesManager, RefType, IntervalType };
