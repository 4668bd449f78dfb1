"use strict";
/*
 * index.js — drop-in host layer of the MI355X batched sequence-merge engine.
 *
 * `MergeTreeEngine` owns one engine context (one HIP device, many documents).
 * `BatchClient` is one document seen by an observer client and keeps the
 * surface of @fluidframework/merge-tree's Client for the remote-op path:
 *
 *   applyMsg(msg, local=false)           Client.applyMsg          client.ts:918-935
 *   getText()                            TestClient.getText       test/testClient.ts:148-150
 *   getLength()                          Client.getLength         client.ts:1161
 *   getPropertiesAtPosition(pos)         Client.getPropertiesAtPosition client.ts:1133-1141
 *   getCurrentSeq() / getCollabWindow()  Client.getCurrentSeq / CollaborationWindow
 *   getOrAddShortClientId(longId)        client.ts:683-698
 *   mergeTree.insertSegments(pos, segments, refSeq, clientId, seq)  mergeTree.ts:1394-1422
 *   mergeTree.markRangeRemoved(start, end, refSeq, clientId, seq)   mergeTree.ts:1908-2000
 *   mergeTree.annotateRange(start, end, props, combiningOp, refSeq, clientId, seq)
 *                                                                   mergeTree.ts:1864-1906
 *
 * Messages are queued per document; the first read-out (or flush()) packs the
 * queued messages of every document of the engine into one batch, uploads it
 * (N-API -> C-ABI mte_submit) and replays it on the GPU (mte_run + mte_sync).
 * There is no CPU fallback: without libmte.so / a HIP device the constructor
 * throws.  Delta / maintenance callbacks are not emitted (DESIGN.md
 * "Boundary"), local ops and combining ops other than "rewrite" throw.
 */
const path = require("path");
const packing = require("./packing");
const { IntervalCollection, IntervalType, RefType } = require("./intervals");

const { BatchBuilder, DocClients, Interner, MergeTreeError, packDocInits, packSegments, utf16 } = packing;

// UTF-16 code units -> JS string (chunked: apply() on a huge array overflows the stack)
function unitsToString(u) {
  let out = "";
  for (let i = 0; i < u.length; i += 8192) out += String.fromCharCode.apply(null, u.subarray(i, i + 8192));
  return out;
}

let addon = null;
function loadAddon() {
  if (addon === null) {
    // built in-tree by `make -C fluidframework_amd/node` (DESIGN.md "Build")
    addon = require(path.join(__dirname, "..", "_lib", "mte_napi.node"));
  }
  return addon;
}

// MTE_E_* -> the reference assert code with the same meaning (client.ts:525-528,
// 940-943; mergeTree.ts:1078-1084, 1666-1672)
const ASSERT_CODES = { "-5": 0x030, "-6": 0x031, "-7": 0x039 };
const DELTA_SLIDE = 0x40;  // MTE_DELTA_SLIDE (include/mte.h): a reference slid off a removed segment
const DELTA_REFPOS = 0x80;  // MTE_DELTA_REFPOS: the references' positions after a group op's member
const DELTA_MAINT = 0x100;  // MTE_DELTA_MAINT | type: a mergeTreeMaintenanceCallback segment
// MergeTreeMaintenanceType (mergeTreeDeltaCallback.ts): MTE_MAINT_* t -> -t
const MAINT_NAMES = { [-1]: "append", [-2]: "split", [-3]: "unlink", [-4]: "acknowledged" };

function docError(code, doc) {
  const a = loadAddon();
  const e = new MergeTreeError(code, "document " + doc + ": " + a.strerror(code));
  if (ASSERT_CODES[String(code)] !== undefined) e.assertCode = ASSERT_CODES[String(code)];
  return e;
}

function segmentSpec(seg) {
  // ISegment objects expose toJSONObject() (textSegment.ts:57-63, mergeTreeNodes.ts:611-621)
  if (seg && typeof seg.toJSONObject === "function") return seg.toJSONObject();
  return seg;
}

/** SharedSegmentSequence.createOpsFromDelta (sequence.ts:116-161) for one
 *  record's ranges: inserts as they landed, consecutive removes at one
 *  position merged, annotates that continue the last merged (one op: the same
 *  props, its keys with the values they now have). */
function opsFromDelta(kind, ranges, op) {
  const ops = [];
  for (const r of ranges) {
    if (kind === 0) {
      ops.push({ pos1: r.position, seg: r.segment, type: 0 });
    } else if (kind === 1) {
      const last = ops[ops.length - 1];
      if (last && last.pos1 === r.position) last.pos2 += r.length;
      else ops.push({ pos1: r.position, pos2: r.position + r.length, type: 1 });
    } else {
      const props = {};
      for (const key of Object.keys((op && op.props) || {})) props[key] = op.props[key] === undefined ? null : op.props[key];
      const last = ops[ops.length - 1];
      if (last && last.pos2 === r.position) last.pos2 += r.length;
      else ops.push({ pos1: r.position, pos2: r.position + r.length, props, type: 2 });
    }
  }
  return ops;
}

class MergeTreeEngine {
  /**
   * @param {{device?: number, nKeys?: number, segCapacity?: number}} [options]
   */
  constructor(options) {
    const o = options || {};
    this.nKeys = o.nKeys === undefined ? 8 : o.nKeys;
    this.addon = o.addon || loadAddon();  // o.addon: another binding of the same functions (tests)
    this.ctx = this.addon.create(o.device || 0, this.nKeys, o.segCapacity || 0);
    // reference slots per document (mte_set_ref_capacity, default 1024): every
    // document's packer refuses a reference past it
    this.refCapacity = o.refCapacity === undefined ? 1024 : o.refCapacity;
    if (o.refCapacity !== undefined) this.addon.setRefCapacity(this.ctx, o.refCapacity);
    this.interner = new Interner(this.nKeys);
    this.docs = [];
    this.clients = [];
    this.started = false;
    this.pending = null;
    this.views = [];
  }

  /** A new document (before the first flush).  initialText becomes one seq-0
   *  segment of LocalClientId, as the replay harness loads it
   *  (client.replay.spec.ts:22-23); options.segments instead loads a summary
   *  body — IJSONSegmentWithMergeInfo specs with seq / client / removedSeq /
   *  removedClientIds — as SnapshotLoader.loadBody does (snapshotLoader.ts:85-125);
   *  options.legacy loads a legacy summary (BatchClient.summarizeLegacy) and
   *  queues its catch-up ops; options.summary loads the blobs of either format
   *  (summarizeV1 / summarizeLegacy). */
  createClient(initialText, options) {
    if (this.started) throw new MergeTreeError(-10, "createClient after the engine started");
    let o = options || {};
    if (o.summary) o = Object.assign({}, o, { legacy: o.summary });
    if (o.legacy) o = Object.assign({}, o, loadLegacy(o.legacy));
    const doc = this.docs.length;
    if ((o.localClient || o.events) && o.roundSync) {
      throw new MergeTreeError(-9, "roundSync with a local client or delta events");
    }
    if (o.refs && !o.localClient) throw new MergeTreeError(-9, "local references need {localClient: true}");
    if (o.maintenanceEvents && !(o.events && (o.localClient || o.tree || !o.newLengthCalc))) {
      throw new MergeTreeError(-9, "maintenance events need {events: true} on the tree pass (localClient, tree or the legacy length calculation)");
    }
    if (o.tree && o.roundSync) throw new MergeTreeError(-9, "tree with roundSync");
    this.docs.push({ text: initialText || "", newLengthCalc: !!o.newLengthCalc, roundSync: !!o.roundSync, props: o.props,
      minSeq: o.minSeq || 0, currentSeq: o.currentSeq || 0, segments: o.segments, localClient: !!o.localClient,
      events: !!o.events, refs: !!o.refs,
      // an interval collection's mid-op events need the references' slides
      // (MTE_DOC_SLIDE_EVENTS): on with events and references unless asked off
      slideEvents: !!(o.events && o.refs && o.slideEvents !== false),
      // SharedString's "maintenance" events (MTE_DOC_MAINT_EVENTS)
      maintenanceEvents: !!o.maintenanceEvents,
      // the HBM tree pass for a document without a local client (MTE_DOC_TREE):
      // the reference's own segments, so sequenceDelta ranges are segment-exact
      tree: !!o.tree });
    const c = new BatchClient(this, doc, o.observerId === undefined ? (o.longClientId || "A") : o.observerId,
      !!o.localClient);
    this.clients.push(c);
    if (o.legacy && o.legacy.catchupOps) {
      // SharedSegmentSequence.loadCore (sequence.ts:588-609): catch-up ops above the window
      for (const m of o.legacy.catchupOps) {
        if (m.minimumSequenceNumber < o.minSeq || m.referenceSequenceNumber < o.minSeq ||
            m.sequenceNumber <= o.minSeq || m.sequenceNumber <= o.currentSeq) {
          throw new MergeTreeError(-1, "Invalid catchup operations in snapshot: seq " + m.sequenceNumber);
        }
      }
      this.docs[doc].catchup = o.legacy.catchupOps; // queued at start(), after the load
    }
    return c;
  }

  start() {
    if (this.started) return;
    const p = packDocInits(this.docs, this.interner);
    let body = null;
    if (this.docs.some((d) => d.segments)) {
      // summary bodies (options.segments): their text follows the load text
      const ps = Array.from(p.propsets), pe = Array.from(p.props);
      body = packSegments(this.docs, (i) => this.clients[i].clients,
        { interner: this.interner, propsetsArr: ps, propsArr: pe, textUnits: p.text.length });
      const t = new Uint16Array(p.text.length + body.extraText.length);
      t.set(p.text);
      t.set(utf16(body.extraText), p.text.length);
      p.text = t;
      p.propsets = Uint32Array.from(ps);
      p.props = Uint32Array.from(pe);
    }
    this.addon.loadDocs(this.ctx, p.inits, p.text, p.propsets, p.props);
    if (body) this.addon.loadSegments(this.ctx, body.offsets, body.segs);
    this.started = true;
    this.track = this.docs.some((d) => d.events) ? this.docs.map((d) => !!d.events) : null;
    this.pending = new BatchBuilder(this.docs.length, this.interner, this.track);
    this.views = new Array(this.docs.length).fill(null);
    this.refViews = new Array(this.docs.length).fill(null);
    this.refViewsT = new Array(this.docs.length).fill(null);
    this.orderViews = new Array(this.docs.length).fill(null);
    this.unitViews = new Array(this.docs.length).fill(null);
    this.docs.forEach((d, i) => { if (d.catchup) for (const m of d.catchup) this.clients[i].applyMsg(m); });
  }

  _batch() {
    this.start();
    return this.pending;
  }

  /** Replay every queued message of every document on the GPU.  Returns once
   *  the replay is launched: the next messages can be packed (and the next
   *  flush uploaded, into the engine's other batch slot) while it runs; every
   *  read-out waits for it. */
  flush() {
    this.start();
    if (this.pending.count === 0) return;
    const b = this.pending.build();
    // documents with delta events: the running replay delivers its events
    // before this batch takes the engine (the events of one run are read
    // back before the next run); otherwise this batch uploads while it runs
    if (this.track) this.sync();
    this.inflightSrc = this.pending.recSrc;
    this.pending = new BatchBuilder(this.docs.length, this.interner, this.track);
    this.views.fill(null);
    this.refViews.fill(null);
    this.refViewsT.fill(null);
    this.orderViews.fill(null);
    this.unitViews.fill(null);
    this.addon.submit(this.ctx, b.offsets, b.ops, b.text, b.propsets, b.props);
    this.addon.run(this.ctx);
    this.running = true;
  }

  /** Wait for the launched replay (read-outs call it).  Every document's
   *  delta events are read and delivered before any error is raised: a
   *  document whose event region overflowed (MTE_E_CAPACITY, see
   *  setEventCapacity) loses its events and is marked, so its later
   *  getMessagesSinceMSNChange / summarizeLegacy throw instead of returning an
   *  incomplete stash; the other documents of the batch are unaffected. */
  sync() {
    if (!this.running) return;
    this.addon.sync(this.ctx);
    this.running = false;
    const src = this.inflightSrc;
    this.inflightSrc = null;
    if (!src) return;
    let first = null;
    src.forEach((recs, doc) => {
      if (!recs || !recs.length) return;
      const c = this.clients[doc];
      let flat;
      try {
        flat = this.addon.readDeltas(this.ctx, doc);
      } catch (e) {
        c.eventsLost = e;
        if (!first) first = e;
        return;
      }
      try {
        c._deliver(flat, recs);
      } catch (e) {  // a listener threw: the other documents still get theirs
        if (!first) first = e;
      }
    });
    if (first) throw first;
  }

  /** Delta-event records per op record of MTE_DOC_EVENTS documents (+ 256 per
   *  document; mte_set_event_capacity, default 8).  Takes effect at the next
   *  flush; raise it before replaying ops that touch many segments. */
  setEventCapacity(perOp) {
    this.addon.setEventCapacity(this.ctx, perOp);
  }

  _view(doc) {
    this.flush();
    this.sync();
    let v = this.views[doc];
    if (v === null) {
      v = this.addon.readDoc(this.ctx, doc, this.nKeys);
      this.views[doc] = v;
    }
    if (v.status !== 0) throw docError(v.status, doc);
    return v;
  }

  /** Positions of a document's local reference slots after the last replay
   *  (mte_read_refs), read once per flush. */
  _refView(doc, transient) {
    this.flush();
    this.sync();
    const views = transient ? this.refViewsT : this.refViews;
    let v = views[doc];
    if (v === null) {
      v = new Int32Array(this.addon.readRefs(this.ctx, doc, this.clients[doc].clients.refNext, !!transient).buffer);
      views[doc] = v;
    }
    return v;
  }

  /** Document order of a document's reference slots (mte_read_ref_order: the
   *  index of the held text unit each sits on, -1 detached), once per flush. */
  _refOrderView(doc) {
    this.flush();
    this.sync();
    let v = this.orderViews[doc];
    if (v === null) {
      v = this.addon.readRefOrder(this.ctx, doc, this.clients[doc].clients.refNext);
      this.orderViews[doc] = v;
    }
    return v;
  }

  /** Per held segment of a document: [length, removed] (mte_read_segments),
   *  once per flush: the units behind positions of the document's own view. */
  _unitView(doc) {
    let v = this.unitViews[doc];
    if (v === null) {
      this._view(doc);
      const r = this.addon.readSegments(this.ctx, doc, this.nKeys);
      const dv = new DataView(r.segs.buffer, r.segs.byteOffset, r.segs.byteLength);
      const n = r.segs.byteLength / 32;
      v = new Int32Array(2 * n);
      for (let i = 0; i < n; i++) {
        v[2 * i] = dv.getUint32(i * 32 + 4, true);
        v[2 * i + 1] = dv.getInt32(i * 32 + 12, true) !== 0x7fffffff ? 1 : 0;
      }
      this.unitViews[doc] = v;
    }
    return v;
  }

  /** Per-doc canonical digests (4 x u64 each, DESIGN.md "Digest"). */
  digests() {
    this.flush();
    this.sync();
    const out = new BigUint64Array(this.docs.length * 4);
    this.addon.digest(this.ctx, out);
    return out;
  }

  statuses() {
    this.flush();
    this.sync();
    const out = new Int32Array(this.docs.length);
    this.addon.docStatus(this.ctx, out);
    return out;
  }

  stats() {
    return this.addon.stats(this.ctx);
  }

  // ---- node level: one process per GPU, RCCL over xGMI (mte_comm_*) ----

  /** 128-byte RCCL id; draw it on one rank and hand it to the others. */
  commUniqueId() {
    return this.addon.commUniqueId();
  }

  /** Join the node's communicator (every rank, with the same id). */
  joinNode(world, rank, id) {
    this.addon.commInit(this.ctx, world, rank, id);
    this.world = world;
    this.rank = rank;
  }

  /** Use another engine's communicator (one per process). */
  shareNode(other) {
    this.addon.commShare(this.ctx, other.ctx);
    this.world = other.world;
    this.rank = other.rank;
  }

  nodeBarrier() {
    this.addon.commBarrier(this.ctx);
  }

  /** value summed (op "sum") or maximised ("max") over the ranks. */
  nodeAllreduce(value, op) {
    return this.addon.commAllreduce(this.ctx, value, op === "max" ? 1 : 0);
  }

  /** Every rank's per-doc digests, rank-major, each rank padded to docsPerRank. */
  gatherDigests(docsPerRank) {
    this.flush();
    this.sync();
    const out = new BigUint64Array(this.world * docsPerRank * 4);
    this.addon.commGatherDigests(this.ctx, out, docsPerRank);
    return out;
  }

  leaveNode() {
    this.addon.commDestroy(this.ctx);
  }

  /**
   * Documents -> ranks, balanced by their expected replay work (SURVEY.md 8(e):
   * ops x mean live segments per document): longest first onto the least
   * loaded rank (LPT).  Returns the rank of every document.
   */
  static shardByWork(work, world) {
    const order = Array.from(work.keys()).sort((a, b) => work[b] - work[a] || a - b);
    const load = new Array(world).fill(0);
    const rankOf = new Array(work.length).fill(0);
    for (const d of order) {
      let r = 0;
      for (let k = 1; k < world; k++) if (load[k] < load[r]) r = k;
      rankOf[d] = r;
      load[r] += work[d];
    }
    return rankOf;
  }

  close() {
    if (this.ctx) {
      this.sync();
      this.addon.destroy(this.ctx);
      this.ctx = null;
    }
  }
}

/** A local reference (LocalReferencePosition, localReference.ts:44-118): its
 *  engine slot, ReferenceType and properties. */
let refCreated = 0;  // creation order of references (a segment's list order at one offset)
class LocalReferencePosition {
  constructor(client, slot, refType, properties) {
    this.client = client;
    this.slot = slot;
    this.refType = refType;
    this.properties = properties;
    this.created = ++refCreated;
    // where it sits among the references at its offset (IRefsAtOffset,
    // localReference.ts:139-215): list 0 before / 1 at / 2 after, then its
    // place in that list -- created: pushed onto "at"
    this.list = 1;
    this.listOrder = this.created;
  }
  /** the next stamp of a list push (at / after) */
  static pushStamp() {
    return ++refCreated;
  }
  addProperties(newProps) {
    this.properties = Object.assign({}, this.properties || {}, newProps);
    for (const k of Object.keys(newProps)) if (newProps[k] === null) delete this.properties[k];
  }
  getProperties() {
    return this.properties;
  }
}

class BatchClient {
  constructor(engine, doc, observerId, local) {
    this.engine = engine;
    this.doc = doc;
    this.longClientId = observerId;
    this.clients = new DocClients(observerId, engine.docs[doc].minSeq, local, engine.docs[doc].tree);
    this.clients.refCap = engine.refCapacity;
    this.lastMinSeq = 0;
    const self = this;
    // MergeTree-level entry points (clientId = short id, as in the reference)
    this.mergeTree = {
      insertSegments(pos, segments, refSeq, clientId, seq) {
        let p = pos;
        for (const s of segments) { // mergeTree.ts:1394-1422: insertPos += len per segment
          const spec = segmentSpec(s);
          self.engine._batch().addRaw(self.doc, seq, refSeq, self.lastMinSeq, clientId,
            { type: 0, pos1: p, seg: spec });
          p += typeof spec === "string" ? spec.length : ("marker" in spec ? 1 : spec.text.length);
        }
      },
      markRangeRemoved(start, end, refSeq, clientId, seq) {
        self.engine._batch().addRaw(self.doc, seq, refSeq, self.lastMinSeq, clientId,
          { type: 1, pos1: start, pos2: end });
      },
      annotateRange(start, end, props, combiningOp, refSeq, clientId, seq) {
        const op = { type: 2, pos1: start, pos2: end, props };
        if (combiningOp) op.combiningOp = combiningOp;
        self.engine._batch().addRaw(self.doc, seq, refSeq, self.lastMinSeq, clientId, op);
      },
    };
  }

  /** Client.applyMsg (client.ts:918-935): a remote message, or — in a
   *  document created with {localClient: true} — the sequenced message of one
   *  of this client's own local ops, which acks its oldest pending op
   *  (ackPendingSegment, mergeTree.ts:1278-1331). */
  applyMsg(msg, local) {
    if (local) throw new MergeTreeError(-9, "applyMsg(msg, local = true): pass the sequenced message");
    if (msg.contents && msg.contents.type === "act") {  // an interval op (SharedString's map kernel)
      this.applyIntervalMsg(msg);
      return;
    }
    this.engine._batch().addMessage(this.doc, this.clients, msg);
    if (msg.minimumSequenceNumber > this.lastMinSeq) this.lastMinSeq = msg.minimumSequenceNumber;
    if (this.pendingConsensus) this._consensus(msg);
    // an interval collection's ends slide inside merge-tree ops (a remote
    // remove, the ack of our own), where the reference raises "changeInterval"
    // (intervalCollection.ts:1042-1053): the engine reports each slide with
    // every reference as that record left the document (MTE_DELTA_SLIDE,
    // MTE_DELTA_REFPOS), so the message stays queued and the events come at
    // the flush (_deliver -> IntervalCollection._onSlides)
  }

  /** Replay this document's queued messages before an interval collection
   *  reads or changes its state (positions, the end tree): the engine-wide
   *  flush when anything of this document is queued. */
  _settle() {
    const e = this.engine;
    if (!e.started) return;
    if (e.pending.docCount[this.doc]) e.flush();
    e.sync();
  }

  // ---- local ops (documents created with {localClient: true}) ----
  // Each queues the op for this document's next replay, where it applies at
  // once in this client's view with seq UnassignedSequenceNumber, and returns
  // the op to send (client.ts:131-229).  Positions are in this client's view
  // (getLength() etc. flush first, as any read-out).

  _local(op) {
    this.engine._batch().addLocal(this.doc, this.clients, op);
    return op;
  }

  /** Client.insertSegmentLocal with a TextSegment (TestClient.insertTextLocal, test/testClient.ts:179-189). */
  insertTextLocal(pos, text, props) {
    return this._local({ type: 0, pos1: pos, seg: props ? { text, props } : text });
  }

  /** Client.insertSegmentLocal with a Marker (TestClient.insertMarkerLocal, test/testClient.ts:224-235). */
  insertMarkerLocal(pos, refType, props) {
    const seg = { marker: { refType } };
    if (props) seg.props = props;
    return this._local({ type: 0, pos1: pos, seg });
  }

  /** Client.insertSegmentLocal (client.ts:216-229) with a segment or its JSON spec. */
  insertSegmentLocal(pos, segment) {
    return this._local({ type: 0, pos1: pos, seg: segmentSpec(segment) });
  }

  /** Client.removeRangeLocal (client.ts:206-214). */
  removeRangeLocal(start, end) {
    return this._local({ type: 1, pos1: start, pos2: end });
  }

  /** Client.annotateRangeLocal (client.ts:183-204); combiningOp rewrite is not supported locally. */
  annotateRangeLocal(start, end, props, combiningOp) {
    const op = { type: 2, pos1: start, pos2: end, props };
    if (combiningOp) op.combiningOp = combiningOp;
    return this._local(op);
  }

  /** Client.annotateMarker (client.ts:166-174): the op createAnnotateMarkerOp
   *  makes (opBuilder.ts:26-40, relativePos1 {id, before: true} and
   *  relativePos2 {id}), resolved by the engine in this client's view
   *  (posFromRelativePos, mergeTree.ts:1369-1392).  marker: the marker's id,
   *  or an object with getId() / properties.markerId; undefined without an id. */
  annotateMarker(marker, props, combiningOp) {
    const id = typeof marker === "string" ? marker
      : (marker && typeof marker.getId === "function" ? marker.getId()
        : (marker && marker.properties ? marker.properties.markerId : undefined));
    if (!id) return undefined;
    const op = { props, relativePos1: { id, before: true }, relativePos2: { id }, type: 2 };
    if (combiningOp) op.combiningOp = combiningOp;
    return this._local(op);
  }

  /** Client.annotateMarkerNotifyConsensus (client.ts:137-158): annotateMarker
   *  with combiningOp consensus; the ack stamps the marker's consensus value
   *  with its seq (updateConsensusProperty, :1083-1090: MTE_F_COMBINE on the
   *  ack record) and consensusCallback(marker) runs once the window's minSeq
   *  reaches that seq (addMinSeqListener, mergeTree.ts:1059-1075). */
  annotateMarkerNotifyConsensus(marker, props, consensusCallback) {
    const op = this.annotateMarker(marker, props, { name: "consensus" });
    if (op) (this.pendingConsensus || (this.pendingConsensus = [])).push({ op, marker, callback: consensusCallback });
    return op;
  }

  // the consensus ops sequenced, then their callbacks as minSeq passes them
  _consensus(msg) {
    const pc = this.pendingConsensus;
    if (!pc || !pc.length) return;
    if (msg.clientId === this.longClientId) {
      const e = pc.find((x) => x.seq === undefined);
      if (e && (msg.contents === e.op || JSON.stringify(msg.contents) === JSON.stringify(e.op))) e.seq = msg.sequenceNumber;
    }
    const due = pc.filter((x) => x.seq !== undefined && x.seq <= msg.minimumSequenceNumber).sort((x, y) => x.seq - y.seq);
    if (!due.length) return;
    this.pendingConsensus = pc.filter((x) => !due.includes(x));
    for (const x of due) if (typeof x.callback === "function") x.callback(x.marker);
  }

  /** A local op given as its IMergeTreeDeltaOp JSON -- the Client's own op
   *  path, applyInsertOp / applyRemoveRangeOp / applyAnnotateRangeOp({op})
   *  (client.ts:405-500) -- relative positions included.  Returns the op. */
  applyLocalOp(op) {
    return this._local(op);
  }

  /** TestClient.makeOpMessage (test/testClient.ts:259-272): the message to
   *  sequence for a local op. */
  makeOpMessage(op, seq, refSeq, minSeq) {
    return {
      clientId: this.longClientId, sequenceNumber: seq === undefined ? -1 : seq,
      referenceSequenceNumber: refSeq === undefined ? this.getCurrentSeq() : refSeq,
      minimumSequenceNumber: minSeq === undefined ? 0 : minSeq, type: "op", contents: op,
    };
  }

  // ---- delta events (documents created with {events: true}) ----
  // After each replay the document's mergeTreeDeltaCallback ranges come back
  // from the engine (MTE_DOC_EVENTS) and are delivered in op order as
  // SharedString's "sequenceDelta" events (sequence.ts:203-211,
  // SequenceDeltaEvent / ISequenceDeltaRange, sequenceDeltaEvent.ts): one event
  // per insert / remove / annotate that changed something, its ranges
  // {position, length, removed, segment} in document order.  The segment is the
  // inserted spec for an insert, else undefined: the engine keeps no segment
  // objects.  They arrive at the flush, not synchronously with applyMsg.

  /** on("sequenceDelta", listener(event, client)); on("maintenance",
   *  listener(event, client)) in a document created with {maintenanceEvents:
   *  true}: SharedString's "maintenance" events (sequence.ts:212-216,
   *  SequenceMaintenanceEvent), one per mergeTreeMaintenanceCallback --
   *  deltaOperation the MergeTreeMaintenanceType (APPEND -1, SPLIT -2, UNLINK
   *  -3, ACKNOWLEDGED -4), opArgs {op, sequencedMessage} of the op that caused
   *  it (undefined for a local op's), ranges {operation, position, length,
   *  propertyDeltas, segment} in document order: the segments' positions once
   *  the op's message is applied (-1: unlinked) and their lengths at the
   *  callback; segment undefined (the engine keeps no segment objects). */
  on(name, listener) {
    if (name === "maintenance") {
      if (!this.engine.docs[this.doc].maintenanceEvents) {
        throw new MergeTreeError(-9, "createClient(..., {maintenanceEvents: true}) first");
      }
      (this.maintListeners || (this.maintListeners = [])).push(listener);
      return this;
    }
    if (name !== "sequenceDelta") throw new MergeTreeError(-9, "only sequenceDelta and maintenance events are delivered");
    if (!this.engine.docs[this.doc].events) throw new MergeTreeError(-9, "createClient(..., {events: true}) first");
    (this.listeners || (this.listeners = [])).push(listener);
    return this;
  }

  _maint(list, src) {
    for (const m of list) {
      const ev = { deltaOperation: m.t, operation: MAINT_NAMES[m.t], ranges: m.ranges, first: m.ranges[0],
        last: m.ranges[m.ranges.length - 1], clientId: this.longClientId,
        opArgs: src ? { op: src.op, sequencedMessage: src.local ? undefined : src.msg } : undefined };
      for (const fn of this.maintListeners || []) fn(ev, this);
    }
  }

  /** Messages since the last minSeq change, catch-up ops rewritten as
   *  SharedSegmentSequence.processMergeTreeMsg stashes them for a legacy
   *  summary (sequence.ts:688-725, createOpsFromDelta :116-161): a message whose
   *  refSeq is not seq - 1 becomes its effect as ops at refSeq = seq - 1. */
  getMessagesSinceMSNChange() {
    if (this.eventsLost) throw this.eventsLost;
    return (this.stash || []).slice();
  }

  _deliver(flat, recs) {
    if (!this.stash) this.stash = [];
    const kinds = ["insert", "remove", "annotate"];
    let i = 0;
    const n = flat.length / 5;
    // one group of events per record, then one stash entry per message
    let cur = null;  // {msg, ops: [...]} of the message being rewritten
    const flushMsg = () => {
      if (!cur) return;
      const m = cur.msg;
      if ((m.type === undefined ? "op" : m.type) !== "op") {  // only merge-tree ops reach processMergeTreeMsg
        cur = null;
        return;
      }
      if (m.referenceSequenceNumber !== m.sequenceNumber - 1) {
        this.stash.push(Object.assign({}, m, { referenceSequenceNumber: m.sequenceNumber - 1,
          contents: cur.ops.length !== 1 ? { type: 3, ops: cur.ops } : cur.ops[0] }));
      } else {
        this.stash.push(m);
      }
      // sequence.ts:719-723 / 727-738: drop what the window has passed
      const msn = m.minimumSequenceNumber;
      if (this.stash.length > 20 && this.stash[20].sequenceNumber < msn) {
        this.stash = this.stash.filter((x) => x.sequenceNumber > msn);
      }
      cur = null;
    };
    // each record's events: its delta ranges and the references it slid
    const parsed = new Array(recs.length);
    for (let k = 0; k < recs.length; k++) {
      const src = recs[k];
      if (src.rebase) {  // a reconnection query of an interval op (_rebase): its answer
        while (i < n && flat[5 * i] === k) {
          (this.rebaseRecs || (this.rebaseRecs = [])).push([k, flat[5 * i + 2] | 0]);
          i++;
        }
        continue;
      }
      if (src.regen) {  // a regenerated op (regeneratePendingOp): no event
        while (i < n && flat[5 * i] === k) {
          (this.regenRecs || (this.regenRecs = [])).push([k, flat[5 * i + 1], flat[5 * i + 2] | 0, flat[5 * i + 3],
            flat[5 * i + 4]]);
          i++;
        }
        continue;
      }
      const ranges = [];
      let kind = -1;
      let slides = null, snap = null, mBefore = null, mAfter = null;
      while (i < n && flat[5 * i] === k) {
        const kd = flat[5 * i + 1];
        if ((kd & 0xff00) === DELTA_MAINT) {
          // a maintenance callback's segment (MTE_DELTA_MAINT): the callbacks
          // before the op's delta ranges (its splits) and after them
          const t = -(kd & 0xff);
          const list = ranges.length ? (mAfter || (mAfter = [])) : (mBefore || (mBefore = []));
          const r = { operation: t, position: flat[5 * i + 2] | 0, length: flat[5 * i + 3], propertyDeltas: {},
            segment: undefined };
          if (flat[5 * i + 4] === 0 || !list.length || list[list.length - 1].t !== t) list.push({ t, ranges: [r] });
          else list[list.length - 1].ranges.push(r);
          i++;
          continue;
        }
        if ((kd & 0xff) === DELTA_REFPOS) {  // slot -> [position, Transient position, order key]
          const p = flat[5 * i + 2] | 0;
          (snap || (snap = new Map())).set(flat[5 * i + 4], [p < -1 ? -1 : p, p < -1 ? -2 - p : p, flat[5 * i + 3] | 0]);
          i++;
          continue;
        }
        if ((kd & 0xff) >= DELTA_SLIDE && (kd & 0xff) < 2 * DELTA_SLIDE) {
          // a reference slid off a removed-and-acked segment (MTE_DELTA_SLIDE)
          (slides || (slides = [])).push({ slot: flat[5 * i + 4], pos: flat[5 * i + 2] | 0, seg: flat[5 * i + 3] | 0,
            moves: (kd & 1) !== 0, after: (kd & 2) !== 0, off: kd >>> 16, at: slides ? slides.length : 0 });
          i++;
          continue;
        }
        kind = kd;
        ranges.push({ position: flat[5 * i + 2] | 0, length: flat[5 * i + 3], removed: flat[5 * i + 4] === 1,
          segment: kind === 0 && src.op ? src.op.seg : undefined });
        i++;
      }
      parsed[k] = { kind, ranges, slides, snap, mBefore, mAfter };
    }
    // the references as record k left the document (MTE_DELTA_REFPOS): a
    // reference sliding there sees the document at that moment -- inside a
    // remote group op, between its members (client.ts applyRemoteOp per
    // member), and in any case before the rest of the batch
    const backTo = (k) => {
      const snap = parsed[k] && parsed[k].snap;
      if (!snap) return null;
      return {
        at: (slot, transient) => (snap.has(slot) ? snap.get(slot)[transient ? 1 : 0] : -1),
        key: (slot) => (snap.has(slot) ? snap.get(slot)[2] : -1),
      };
    };
    for (let k = 0; k < recs.length; k++) {
      const src = recs[k];
      const pr = parsed[k];
      if (!pr) continue;
      if (!src.local && (!cur || cur.msg !== src.msg)) {
        flushMsg();
        cur = { msg: src.msg, ops: [] };
      }
      const { kind, ranges, slides, mBefore, mAfter } = pr;
      if (kind < 0) {  // an ack: its slides come before its ACKNOWLEDGED callback
        if (slides) this._slid(slides, backTo(k));
        if (mBefore) this._maint(mBefore, src);
        continue;
      }
      if (mBefore) this._maint(mBefore, src);
      if (cur) cur.ops.push(...opsFromDelta(kind, ranges, src.op));
      const ev = { deltaOperation: kind, operation: kinds[kind], isLocal: src.local,
        message: src.local ? undefined : src.msg, ranges, first: ranges[0], last: ranges[ranges.length - 1] };
      for (const fn of this.listeners || []) fn(ev, this);
      // markRangeRemoved slides the newly removed segments' references after
      // the delta callback (mergeTree.ts:1978-1993)
      if (slides) this._slid(slides, backTo(k));
      if (mAfter) this._maint(mAfter, src);
    }
    flushMsg();
  }

  /** The references one op slid (MTE_DELTA_SLIDE records, in the order of the
   *  segments they left) -> the interval collections' position listeners. */
  _slid(slides, back) {
    if (this.onSlideRecords) this.onSlideRecords(slides);  // a test hook (tests/node/interval_farm.js trace)
    if (!this.intervalCollections) return;
    for (const c of this.intervalCollections.values()) c._onSlides(slides, back);
  }

  /** Client.rollback (client.ts:396-398 -> MergeTree.rollback,
   *  mergeTree.ts:2005-2083) of this client's latest pending op, which must not
   *  have been sent: its inserts disappear, its removes are undone, its
   *  annotates put the previous values back (previousProps). */
  rollback(op) {  // eslint-disable-line no-unused-vars
    this.engine._batch().addRollback(this.doc, this.clients);
  }

  /** Client.regeneratePendingOp (client.ts:972-1002 -> resetPendingDeltaToOps
   *  :788-860) for reconnection: the op that re-sends the oldest pending op
   *  (resetOp, as it was sent), one member per segment of its group, at
   *  positions in the view at its localSeq; the op stays pending (acked by the
   *  sequenced message of the returned op).  Needs {localClient, events};
   *  replays what is queued (flush + sync). */
  regeneratePendingOp(resetOp) {
    if (!this.engine.docs[this.doc].events) throw new MergeTreeError(-9, "createClient(..., {events: true}) first");
    const idx = this.engine._batch().addRegen(this.doc, this.clients);
    this.regenRecs = [];
    this.engine.flush();
    this.engine.sync();
    if (this.engine.statuses()[this.doc] !== 0) throw docError(this.engine.statuses()[this.doc], this.doc);
    const op = packing.regenOps(resetOp, idx, this.regenRecs);
    this.regenRecs = null;
    return op;
  }

  /** The reconnection queries of a pending interval op
   *  (rebaseLocalInterval, intervalCollection.ts:1735-1803), answered at once
   *  (flush + sync): each request {pos, seqFrom, localSeq} -> Client.rebasePosition
   *  (client.ts:755-786: the position, -1 when it slid off the string), or
   *  {slot, localSeq} -> the slide of a pending interval end whose segment was
   *  removed and acked (the position it moved to, -1 when it stays). */
  _rebase(requests) {
    if (!this.engine.docs[this.doc].events) throw new MergeTreeError(-9, "createClient(..., {events: true}) first");
    const b = this.engine._batch();
    const idx = requests.map((q) => (q.slot !== undefined
      ? b.addRefRebase(this.doc, this.clients, q.slot, q.localSeq)
      : b.addRebase(this.doc, this.clients, q.pos, q.seqFrom, q.localSeq)));
    this.rebaseRecs = [];
    this.engine.flush();
    this.engine.sync();
    if (this.engine.statuses()[this.doc] !== 0) throw docError(this.engine.statuses()[this.doc], this.doc);
    const byIdx = new Map(this.rebaseRecs.map((r) => [r[0], r[1]]));
    this.rebaseRecs = null;
    return idx.map((k) => (byIdx.has(k) ? byIdx.get(k) : -1));
  }

  // ---- local references (documents created with {localClient: true, refs: true}) ----
  // LocalReferenceCollection (localReference.ts:139-567) held by the engine
  // (MTE_DOC_REFS): a reference sits on a text unit of this client's view and
  // slides with it (slideAckedRemovedSegmentReferences, mergeTree.ts:893-950).

  /** Client.getContainingSegment (client.ts:1107-1110) in this client's view:
   *  {segment: {start, length, kind}, offset}, or {segment: undefined} past the
   *  end.  The segment is a snapshot of the visible segment holding pos (the
   *  engine keeps no segment objects); pass it to createLocalReferencePosition
   *  before queuing another op. */
  getContainingSegment(pos) {
    const v = this.engine._view(this.doc);
    let start = 0;
    for (let i = 0; i < v.segLen.length; i++) {
      const n = v.segLen[i];
      if (pos >= start && pos < start + n) {
        return { segment: { start, length: n, kind: v.segKind[i] }, offset: pos - start };
      }
      start += n;
    }
    return { segment: undefined, offset: undefined };
  }

  /** Client.createLocalReferencePosition (client.ts:360-364): a reference at
   *  offset of segment (from getContainingSegment; a number is taken as a
   *  position of this client's view).  refType: ReferenceType flags --
   *  SlideOnRemove (0x40), StayOnRemove (0x80), Simple (0) or Transient
   *  (0x100: kept on its segment, never slid -- localReference.ts:263), with
   *  any label bits.  Queued with the document's next replay. */
  createLocalReferencePosition(segment, offset, refType, properties) {
    if (!this.engine.docs[this.doc].refs) throw new MergeTreeError(-9, "createClient(..., {refs: true}) first");
    const base = typeof segment === "number" ? segment : (segment && typeof segment.start === "number" ? segment.start : NaN);
    if (Number.isNaN(base)) throw new MergeTreeError(-1, "createLocalReferencePosition: no segment");
    const rt = refType === undefined ? 0 : refType;
    const slot = this.engine._batch().addRef(this.doc, this.clients, base + (offset || 0), rt);
    return new LocalReferencePosition(this, slot, rt, properties);
  }

  /** A reference a sequenced op creates in its own perspective (refSeq and
   *  sender): createPositionReference with an op (intervalCollection.ts:639-658),
   *  SlideOnRemove, detached when no segment holds pos there. */
  _createRefFromOp(msg, pos, refType) {
    if (!this.engine.docs[this.doc].refs) throw new MergeTreeError(-9, "createClient(..., {refs: true}) first");
    const slot = this.engine._batch().addRefRemote(this.doc, this.clients, msg, pos, refType);
    return new LocalReferencePosition(this, slot, refType, undefined);
  }

  /** The reference becomes refType (SlideOnRemove) and slides if its segment is
   *  removed and acked (ackInterval's setSlideOnRemove + getSlideToSegment). */
  _setRefSlide(lref, refType) {
    if (!lref || lref.client !== this || lref.slot < 0) return;
    this.engine._batch().setRefSlide(this.doc, this.clients, lref.slot, refType);
    lref.refType = refType;
  }

  /** SharedString.getIntervalCollection(label) (sequence.ts): the label's
   *  IntervalCollection over this client's references ({localClient, refs}
   *  documents); emitter.emit(opName, undefined, value) receives its ops. */
  getIntervalCollection(label, emitter, serialized) {
    if (!this.intervalCollections) this.intervalCollections = new Map();
    let c = this.intervalCollections.get(label);
    if (!c) {
      if (!this.engine.docs[this.doc].refs) throw new MergeTreeError(-9, "createClient(..., {refs: true}) first");
      c = new IntervalCollection(this, label, emitter, serialized);
      this.intervalCollections.set(label, c);
    } else if (emitter) {
      c.emitter = emitter;
    }
    return c;
  }

  /** A sequenced interval op as SharedString's map kernel carries it
   *  ({key: label, type: "act", value: {opName, value}}): processed by the
   *  label's collection; the merge-tree window does not move (sequence.ts:628-648). */
  applyIntervalMsg(msg) {
    const c = msg.contents;
    this.getIntervalCollection(c.key).process(c.value.opName, c.value.value, msg.clientId === this.longClientId, msg);
  }

  /** Client.removeLocalReferencePosition (client.ts:369-371). */
  removeLocalReferencePosition(lref) {
    if (!lref || lref.client !== this || lref.slot < 0) return undefined;
    this.engine._batch().removeRef(this.doc, this.clients, lref.slot);
    lref.slot = -1;
    return lref;
  }

  /** The document-order key of a reference (mte_read_ref_order; -1 detached). */
  _refOrder(lref) {
    if (!lref || lref.client !== this || lref.slot < 0) return -1;
    return this.engine._refOrderView(this.doc)[lref.slot];
  }

  /** The document-order key of the unit at pos of this client's view, as a
   *  Transient reference there would have it (createPositionReference ->
   *  getContainingSegment, intervalCollection.ts:639-658): -1 outside. */
  _unitKeyAt(pos) {
    const v = this.engine._unitView(this.doc);
    if (!(pos >= 0)) return -1;
    let p = 0, k = 0;
    for (let i = 0; i < v.length; i += 2) {
      const len = v[i];
      if (!v[i + 1]) {
        if (pos < p + len) return k + (pos - p);
        p += len;
      }
      k += len;
    }
    return -1;
  }

  /** Client.localReferencePositionToPosition (client.ts:376-378): the
   *  reference's position in this client's view, -1 (DetachedReferencePosition)
   *  once it is detached or removed. */
  localReferencePositionToPosition(lref) {
    if (lref && lref.snapshot) return lref.position;  // an interval event's previousInterval end
    // an end an interval event raised mid-op reads as it was at that moment
    // (IntervalCollection._onSlides)
    if (lref && lref.pinned !== undefined) return lref.pinned;
    if (!lref || lref.client !== this || lref.slot < 0) return -1;
    // transientRead: an end an interval event's previousInterval shares, read
    // as the reference reads it while emitChange holds it Transient
    return this.engine._refView(this.doc, lref.transientRead)[lref.slot];
  }

  /** Local ops sent but not acknowledged yet. */
  getPendingCount() {
    return this.clients.pending.length;
  }

  /** Client.getOrAddShortClientId (client.ts:683-698).  A short id handed out
   *  here (no seq attached) keeps its slot for good; ids the engine assigns to
   *  message senders are recycled behind the window (DocClients). */
  getOrAddShortClientId(longId) {
    const i = this.clients.short(longId);
    if (i >= this.clients.maxClients) throw new MergeTreeError(-12, "client " + String(longId) + ": no free client slot");
    return i;
  }

  getClientId() {
    return 0;
  }

  getLongClientId(shortId) {
    for (const [k, v] of this.clients.ids) if (v === shortId) return k;
    return undefined;
  }

  flush() {
    this.engine.flush();
  }

  /** TestClient.getText(start?, end?) (test/testClient.ts:148) =
   *  MergeTreeTextHelper.getText with placeholder "" (MergeTreeTextHelper.ts:20-74):
   *  text units of the visible text segments overlapping [start, end); markers
   *  occupy one position and contribute nothing. */
  getText(start, end) {
    const v = this.engine._view(this.doc);
    if (start === undefined && end === undefined) return v.text;
    const s0 = start === undefined ? 0 : start;
    const e0 = end === undefined ? v.length : end;
    let out = "";
    let p = 0, t = 0;
    for (let i = 0; i < v.segLen.length && p < e0; i++) {
      const len = v.segLen[i];
      if (v.segKind[i] === 0) {
        if (p + len > s0) out += v.text.substring(t + Math.max(s0 - p, 0), t + Math.min(e0 - p, len));
        t += len;
      }
      p += len;
    }
    return out;
  }

  getLength() {
    return this.engine._view(this.doc).length;
  }

  getCurrentSeq() {
    return this.engine._view(this.doc).curSeq;
  }

  getCollabWindow() {
    const v = this.engine._view(this.doc);
    return { clientId: 0, currentSeq: v.curSeq, minSeq: v.minSeq, collaborating: true };
  }

  /** Properties of the visible segment containing pos (undefined when it has none). */
  getPropertiesAtPosition(pos) {
    const v = this.engine._view(this.doc);
    const nk = this.engine.nKeys;
    let p = 0;
    for (let i = 0; i < v.segLen.length; i++) {
      const len = v.segLen[i];
      if (pos >= p && pos < p + len) {
        return this.engine.interner.decode(nk ? v.segProps.subarray(i * nk, (i + 1) * nk) : []);
      }
      p += len;
    }
    return undefined;
  }

  /** Visible segments in order: {kind: "text"|"marker", text?, refType?, length, props?} */
  getSegments() {
    const v = this.engine._view(this.doc);
    const nk = this.engine.nKeys;
    const out = [];
    let t = 0;
    for (let i = 0; i < v.segLen.length; i++) {
      const kind = v.segKind[i];
      const props = this.engine.interner.decode(nk ? v.segProps.subarray(i * nk, (i + 1) * nk) : []);
      if (kind === 0) {
        out.push({ kind: "text", text: v.text.substr(t, v.segLen[i]), length: v.segLen[i], props });
        t += v.segLen[i];
      } else {
        out.push({ kind: "marker", refType: kind - 1, length: 1, props });
      }
    }
    return out;
  }

  /**
   * Summary body of this document: SnapshotV1.extractSegment
   * (snapshotV1.ts:189-265) over the segments the engine holds
   * (mte_read_segments).  Segments removed at or below minSeq are elided;
   * segments inserted at or below minSeq and not removed lose their merge
   * info and coalesce (TextSegment.canAppend textSegment.ts:72-77 +
   * matchProperties); the rest keep seq / client / removedSeq /
   * removedClientIds.  Load it with createClient("", {segments, minSeq,
   * currentSeq}).  Returns {segments, minSeq, currentSeq}.
   */
  summarize() {
    const v = this.engine._view(this.doc);
    const minSeq = v.minSeq;
    const out = [];
    let prev = null;
    for (const sg of this._heldSegments()) {
      const removed = sg.rseq !== 0x7fffffff;
      if (removed && sg.rseq <= minSeq) continue;
      if (sg.seq <= minSeq && !removed) {
        if (prev === null) prev = sg;
        else if (canAppend(prev, sg) && sameProps(prev.props, sg.props)) prev = { kind: 0, props: prev.props, text: prev.text + sg.text };
        else { out.push({ json: segJson(prev) }); prev = sg; }
        continue;
      }
      if (prev !== null) { out.push({ json: segJson(prev) }); prev = null; }
      const raw = { json: segJson(sg) };
      if (sg.seq > minSeq) { raw.seq = sg.seq; raw.client = this.getLongClientId(sg.client); }
      if (removed) {
        const ids = [];
        for (let c = 0; c < 32; c++) if ((sg.removers >>> c) & 1) ids.push(this.getLongClientId(c));
        raw.removedSeq = sg.rseq;
        raw.removedClient = ids[0];
        raw.removedClientIds = ids;
      }
      out.push(raw);
    }
    if (prev !== null) out.push({ json: segJson(prev) });
    return { segments: out, minSeq, currentSeq: v.curSeq };
  }

  /**
   * V1 summary (newMergeTreeSnapshotFormat: true): SnapshotV1.emit
   * (snapshotV1.ts:117-165) over summarize()'s segments: a "header"
   * MergeTreeChunkV1 {version, segmentCount, length, segments, startIndex,
   * headerMetadata} and "body_0", "body_1", ... of ~chunkSize units each.
   * Segments below the MSN are plain specs, the others IJSONSegmentWithMergeInfo.
   * Load it with createClient("", {summary: blobs}).
   */
  summarizeV1(chunkSize) {
    const size = chunkSize === undefined ? SNAPSHOT_V1_CHUNK_SIZE : chunkSize;
    const s = this.summarize();
    const specs = s.segments.map((sp) => (Object.keys(sp).length === 1 ? sp.json : sp));
    const lengths = s.segments.map((sp) => specLength(sp.json));
    const md = { minSequenceNumber: s.minSeq, sequenceNumber: s.currentSeq, orderedChunkMetadata: [],
      totalLength: 0, totalSegmentCount: 0 };
    const chunks = [];
    do { // getSeqLengthSegs (snapshotV1.ts:76-110)
      const start = md.totalSegmentCount;
      let n = 0, length = 0;
      while (length < size && start + n < specs.length) { length += lengths[start + n]; n++; }
      chunks.push({ version: "1", segmentCount: n, length, segments: specs.slice(start, start + n), startIndex: start });
      md.totalSegmentCount += n;
      md.totalLength += length;
    } while (md.totalSegmentCount < specs.length);
    const header = chunks.shift();
    md.orderedChunkMetadata = [{ id: "header" }].concat(chunks.map((_, i) => ({ id: "body_" + i })));
    header.headerMetadata = md;
    const blobs = { header };
    chunks.forEach((c, i) => { blobs["body_" + i] = c; });
    return blobs;
  }

  /**
   * Legacy summary (the default when newMergeTreeSnapshotFormat !== true):
   * SnapshotLegacy.extractSync + emit (snapshotlegacy.ts:105-211).  The
   * document as it reads at minSeq for NonCollabClient — segments inserted at
   * or below minSeq and not removed at or below it, coalesced, no merge info —
   * split into a "header" chunk of ~chunkSize units (with headerMetadata,
   * snapshotChunks.ts:168-186) and a "body" chunk, plus "catchupOps": the
   * given messages above minSeq with their minimumSequenceNumber set to minSeq
   * (SharedSegmentSequence.summarizeMergeTree, sequence.ts:676-686).  Load it
   * with createClient("", {legacy: blobs}).
   */
  summarizeLegacy(catchUpMsgs, chunkSize) {
    const size = chunkSize === undefined ? SIZE_OF_FIRST_CHUNK : chunkSize;
    const minSeq = this.engine._view(this.doc).minSeq;
    const specs = [];
    let prev = null;
    for (const sg of this._heldSegments()) {
      if (sg.seq > minSeq || sg.rseq <= minSeq) continue;
      if (prev !== null && canAppend(prev, sg) && sameProps(prev.props, sg.props)) {
        prev = { kind: 0, props: prev.props, text: prev.text + sg.text };
      } else {
        if (prev !== null) specs.push(segJson(prev));
        prev = sg;
      }
    }
    if (prev !== null) specs.push(segJson(prev));
    const total = specs.reduce((a, sp) => a + specLength(sp), 0);
    const header = legacyChunk(specs, size, 0, total, minSeq);
    const ids = [{ id: "header" }];
    if (header.chunkLengthChars < total) ids.push({ id: "body" });
    header.headerMetadata = { orderedChunkMetadata: ids, sequenceNumber: minSeq, totalLength: total,
      totalSegmentCount: specs.length };
    const blobs = { header };
    if (header.chunkSegmentCount < specs.length) {
      blobs.body = legacyChunk(specs, total, header.chunkSegmentCount, total, minSeq);
    }
    const catchup = (catchUpMsgs || []).filter((m) => m.sequenceNumber > minSeq)
      .map((m) => Object.assign({}, m, { minimumSequenceNumber: minSeq }));
    if (catchup.length > 0) blobs.catchupOps = catchup;
    return blobs;
  }

  /** Segments the engine holds for this document (mte_read_segments), decoded. */
  _heldSegments() {
    const eng = this.engine;
    eng._view(this.doc);
    const nk = eng.nKeys;
    const r = eng.addon.readSegments(eng.ctx, this.doc, nk);
    const dv = new DataView(r.segs.buffer, r.segs.byteOffset, r.segs.byteLength);
    const n = r.segs.byteLength / 32;
    const out = [];
    for (let i = 0; i < n; i++) {
      const o = i * 32;
      const textOff = dv.getUint32(o, true), len = dv.getUint32(o + 4, true);
      const kind = dv.getUint32(o + 24, true);
      out.push({ kind, seq: dv.getInt32(o + 8, true), rseq: dv.getInt32(o + 12, true),
        removers: dv.getUint32(o + 16, true), client: dv.getInt32(o + 20, true),
        props: eng.interner.decode(nk ? r.props.subarray(i * nk, (i + 1) * nk) : []),
        text: kind === 0 ? unitsToString(r.text.subarray(textOff, textOff + len)) : null });
    }
    return out;
  }
}

const SIZE_OF_FIRST_CHUNK = 10000; // SnapshotLegacy.sizeOfFirstChunk, snapshotlegacy.ts:52
const SNAPSHOT_V1_CHUNK_SIZE = 10000; // SnapshotV1.chunkSize, snapshotV1.ts:43

function segJson(sg) {
  if (sg.kind === 0) return sg.props ? { text: sg.text, props: sg.props } : sg.text;
  return sg.props ? { marker: { refType: sg.kind - 1 }, props: sg.props } : { marker: { refType: sg.kind - 1 } };
}

function sameProps(a, b) { // matchProperties (properties.ts:66-100) as the summary writers use it: empty == undefined
  // NaN !== NaN: a segment holding one never coalesces (canonicalJson writes it as null)
  for (const k in b || {}) if (typeof b[k] === "number" && b[k] !== b[k]) return false;
  return packing.canonicalJson(a || {}) === packing.canonicalJson(b || {});
}

function canAppend(a, b) { // TextSegment.canAppend (textSegment.ts:72-77)
  return a.kind === 0 && b.kind === 0 && !a.text.endsWith("\n") && (a.text.length <= 256 || b.text.length <= 256);
}

function specLength(sp) {
  return typeof sp === "string" ? sp.length : ("marker" in sp ? 1 : sp.text.length);
}

function legacyChunk(specs, approxLength, start, totalLength, seq) { // getSeqLengthSegs, snapshotlegacy.ts:66-99
  let n = 0, length = 0;
  while (length < approxLength && start + n < specs.length) { length += specLength(specs[start + n]); n++; }
  return { chunkStartSegmentIndex: start, chunkSegmentCount: n, chunkLengthChars: length,
    totalLengthChars: totalLength, totalSegmentCount: specs.length, chunkSequenceNumber: seq,
    segmentTexts: specs.slice(start, start + n) };
}

/** toLatestVersion (snapshotChunks.ts:142-186): a legacy chunk read as MergeTreeChunkV1. */
function toLatest(path, c) {
  if (c.version === "1") return c;
  if (c.version !== undefined) throw new MergeTreeError(-1, "Unsupported chunk path: " + path + " version: " + c.version);
  let md;
  if (path === "header") {
    md = c.headerMetadata;
    if (md === undefined) {
      const ids = [{ id: "header" }];
      if (c.chunkLengthChars < c.totalLengthChars) ids.push({ id: "body" });
      md = { orderedChunkMetadata: ids, minSequenceNumber: c.chunkMinSequenceNumber,
        sequenceNumber: c.chunkSequenceNumber, totalLength: c.totalLengthChars, totalSegmentCount: c.totalSegmentCount };
    }
  }
  return { version: "1", length: c.chunkLengthChars, segmentCount: c.chunkSegmentCount, headerMetadata: md,
    segments: c.segmentTexts, startIndex: c.chunkStartSegmentIndex };
}

/** SnapshotLoader.loadHeader / loadBody (snapshotLoader.ts:126-246) over the
 *  blobs of either format -> {segments, minSeq, currentSeq}; throws the
 *  loader's asserts.  Plain specs become {json} (NonCollabClient at
 *  UniversalSequenceNumber); specs with merge info keep it (hasMergeInfo,
 *  snapshotChunks.ts:80-82). */
function loadLegacy(blobs) {
  const h = toLatest("header", blobs.header);
  const md = h.headerMetadata;
  if (md === undefined) throw new MergeTreeError(-1, "header metadata not available");
  const wrap = (sp) => (sp && typeof sp === "object" && "json" in sp ? sp : { json: sp });
  if (h.length > md.totalLength) throw new MergeTreeError(-1, "0x061: Mismatch in totalLength");
  if (h.segmentCount > md.totalSegmentCount) throw new MergeTreeError(-1, "0x062: Mismatch in totalSegmentCount");
  const specs = h.segments.map(wrap);
  if (h.segmentCount < md.totalSegmentCount) {
    let length = h.length;
    for (const m of md.orderedChunkMetadata.slice(1)) {
      const c = toLatest(m.id, blobs[m.id]);
      length += c.length;
      specs.push(...c.segments.map(wrap));
    }
    if (length !== md.totalLength) throw new MergeTreeError(-1, "0x063: Mismatch in totalLength");
    if (specs.length !== md.totalSegmentCount) throw new MergeTreeError(-1, "0x064: Mismatch in totalSegmentCount");
  }
  const seq = md.sequenceNumber;
  return { segments: specs, minSeq: md.minSequenceNumber !== undefined ? md.minSequenceNumber : seq, currentSeq: seq };
}

module.exports = { MergeTreeEngine, BatchClient, LocalReferencePosition, IntervalCollection, IntervalType, RefType,
  MergeTreeError, loadAddon, loadLegacy, packing };
