#!/usr/bin/env node
// ref_interval_farm.js — conflict farms of REFERENCE merge-tree Clients that
// also edit a SharedString interval collection (TEST INFRASTRUCTURE; build
// container only, never on the GPU box).
//
// Every client holds the reference's IntervalCollection over its Client
// (packages/dds/sequence/src/intervalCollection.ts, erased by oracle/ts_erase.py
// into _ref/ts/sequence/), attached as SharedString attaches it
// (attachGraph(client, label), intervalCollection.ts:1337-1374), and processes
// interval messages as SharedSegmentSequence.processCore does: through the
// value type's ops map (makeOpsMap: ackAdd / ackChange / ackDelete,
// :1163-1221) without touching the merge-tree window (sequence.ts:628-648).
// Merge-tree ops are made and sequenced as in oracle/ref_farm.js.  Interval
// ops: add (with an explicit intervalId), change of one or both ends,
// changeProperties, removeIntervalById, by any client but the observer.  A
// message's refSeq is the sender's last processed seq (any kind), msn the
// lowest of those over the clients.
//
// stdin:  {"sets": [{"seed", "clients", "steps", "initialText", "nCheckpoints",
//                    "maxText", "intervals": p (the chance a step is an interval op)}]}
//          ext: true also records, per client and checkpoint, the
//         collection's events since the previous checkpoint (addInterval /
//         deleteInterval / changeInterval / propertyChanged, with local and the
//         ends before and after, IIntervalCollectionEvent :1257-1300), its
//         iteration order (the interval tree's compare order, :276-316, 483-520),
//         serializeInternal() (:1968-1977, compressInterval :137-149), and
//         (each event's last field true when a merge-tree op raised it: an end
//         sliding off a removed segment, the position change listeners :1023-1058)
//         queries at seeded positions: findOverlappingIntervals, previousInterval,
//         nextInterval and the start / end position iterators (:881-913,
//         :1987-2067); the queries draw from their own generator
//          reconnect: the chance per step that a sending client goes offline,
//         or, offline, reconnects.  Offline, its merge-tree ops (["H", op]) and
//         interval ops (["J", {opName, value}]) stay pending, unsent;
//         reconnecting, it catches up with the whole log, then re-sends them
//         in order as the container runtime's reSubmit does: merge-tree ops
//         through Client.regeneratePendingOp (["G", logIndex]), interval ops
//         through the value type's rebase (makeOpsMap :1163-1172 ->
//         rebaseLocalInterval :1735-1803, with the op's localSeq metadata;
//         ["K", logIndex], the value undefined when the interval slid off)
// stdout: {"sets": [{..params, "names", "log": [[clientId, seq, ref, msn, kind, contents]]
//                    (kind "op": a merge-tree op; "iv": {opName, value}),
//                    "events": per client [["L"|"A", logIndex] | ["I", logIndex]
//                    (an interval op it made: the log entry holds it)],
//                    "checkpoints": [{"done", "states": [{"text", "intervals":
//                    [[id, start, end, props]] sorted by id}]}]}]}
"use strict";
const path = require("path");
const fs = require("fs");

const refdir = process.argv[2] || path.join(__dirname, "_ref", "ts");
const { Client } = require(path.join(refdir, "client.js"));
const { TextSegment } = require(path.join(refdir, "textSegment.js"));
const { Marker } = require(path.join(refdir, "mergeTreeNodes.js"));
const { MergeTreeTextHelper } = require(path.join(refdir, "MergeTreeTextHelper.js"));
const iv = require(path.join(refdir, "sequence", "intervalCollection.js"));

// MTE_REF_TRACE=<client name>: that client's reference slides on stderr (each
// removed-and-acked segment whose references slide: its text, ordinal, the
// references at each offset; each ack's pending group in order) -- a debugging
// aid for the slide order the Node host restates
if (process.env.MTE_REF_TRACE) {
  const { MergeTree } = require(path.join(refdir, "mergeTree.js"));
  const who = process.env.MTE_REF_TRACE;
  const mine = (mt) => mt.collabWindow && mt.collabWindow.clientId === 0 && mt.__traceName === who;
  const refName = (r) => {
    const ivl = r.properties && r.properties.interval;
    const id = ivl && ivl.properties ? ivl.properties.intervalId : "?";
    return `${id}.${ivl && ivl.start === r ? "s" : ivl && ivl.end === r ? "e" : "x"}:${r.refType}`;
  };
  const segName = (sg) => `${sg.text !== undefined ? JSON.stringify(sg.text) : "M"}@${sg.ordinal}` +
    `[seq ${sg.seq} rs ${sg.removedSeq} lrs ${sg.localRemovedSeq}]`;
  const slide = MergeTree.prototype.slideAckedRemovedSegmentReferences;
  MergeTree.prototype.slideAckedRemovedSegmentReferences = function (segment) {
    if (this.__traceName === who && segment.localRefs && !segment.localRefs.empty) {
      const refs = [];
      for (const r of segment.localRefs) refs.push(`${refName(r)}@${r.getOffset()}`);
      process.stderr.write(`  slide ${segName(segment)} refs ${refs.join(" ")}\n`);
    }
    return slide.call(this, segment);
  };
  const ack = MergeTree.prototype.ackPendingSegment;
  MergeTree.prototype.ackPendingSegment = function (opArgs) {
    if (this.__traceName === who && this.pendingSegments && this.pendingSegments.first) {
      const g = this.pendingSegments.first.data;
      process.stderr.write(`  ack seq ${opArgs.sequencedMessage.sequenceNumber} group ${g.segments.map(segName).join(" ")}\n`);
    }
    return ack.call(this, opArgs);
  };
  void mine;
}

function specToSegment(spec) {
  const t = TextSegment.fromJSONObject(spec);
  if (t) return t;
  const m = Marker.fromJSONObject(spec);
  if (m) return m;
  throw new Error(`Unrecognized IJSONSegment type: '${JSON.stringify(spec)}'`);
}
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

// mulberry32 (as oracle/ref_farm.js)
function rng(seed) {
  let a = seed >>> 0;
  const next = () => {
    a = (a + 0x6d2b79f5) >>> 0;
    let t = a;
    t = Math.imul(t ^ (t >>> 15), t | 1);
    t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
  return { next, int: (lo, hi) => lo + Math.floor(next() * (hi - lo + 1)) };
}
function sortKeys(v) {
  if (v && typeof v === "object" && !Array.isArray(v)) {
    const o = {};
    for (const k of Object.keys(v).sort()) o[k] = sortKeys(v[k]);
    return o;
  }
  return v;
}
const clone = (v) => JSON.parse(JSON.stringify(v));
const LABEL = "farm";
const KEYS = ["client", "bold", "color"];

// reconnect farms: each localSeq view the reference computes -- rebasePosition
// (client.ts:755-786), findReconnectionPosition (:709-713) and getPosition
// with a localSeq (:345-350) -- checked against the same view summed leaf by
// leaf with localNetLength (mergeTree.ts:575-593), the rule the engine
// restates.  The reference takes block lengths from its local partial lengths
// (partialLengths.ts:667-700), which can disagree with its own leaf rule (a
// local removal of a segment inserted after refSeq is subtracted while the
// insertion is not counted; the partials cached by computeLocalPartials keep
// the window of the first query since the last length update,
// mergeTree.ts:964-982); the farm counts the calls where they differ.
const leafViews = { calls: 0, differ: 0 };
function leafHooks() {
  const leaves = (mt) => {
    const out = [];
    const walk = (n) => { if (n.isLeaf()) out.push(n); else for (let i = 0; i < n.childCount; i++) walk(n.children[i]); };
    walk(mt.root);
    return out;
  };
  const prefix = (c, seg, refSeq, ls) => {
    let q = 0;
    for (const x of leaves(c._mergeTree)) {
      if (x === seg) return q;
      q += c._mergeTree.localNetLength(x, refSeq, ls) || 0;
    }
    return -1;
  };
  const P = Client.prototype;
  const rebase0 = P.rebasePosition, frp0 = P.findReconnectionPosition, gp0 = P.getPosition;
  let depth = 0;
  const check = (r, e) => { leafViews.calls++; if (r !== e) leafViews.differ++; };
  P.rebasePosition = function (pos, seqFrom, localSeq) {
    depth++;
    const r = rebase0.call(this, pos, seqFrom, localSeq);
    depth--;
    const mt = this._mergeTree;
    let p0 = 0, seg, off = 0;
    for (const x of leaves(mt)) {
      const l = mt.localNetLength(x, seqFrom, localSeq) || 0;
      if (l > 0 && pos >= p0 && pos < p0 + l) { seg = x; off = pos - p0; break; }
      p0 += l;
    }
    if (!seg) { let f = mt.root; while (!f.isLeaf()) f = f.children[f.childCount - 1]; seg = f; off = 0; }
    const so = this.getSlideToSegment({ segment: seg, offset: off });
    check(r, so.segment ? prefix(this, so.segment, this.getCurrentSeq(), localSeq) + so.offset : -1);
    return r;
  };
  P.findReconnectionPosition = function (segment, localSeq) {
    const r = frp0.call(this, segment, localSeq);
    if (!depth) check(r, prefix(this, segment, this.getCurrentSeq(), localSeq));
    return r;
  };
  P.getPosition = function (segment, localSeq) {
    const r = gp0.call(this, segment, localSeq);
    if (!depth && localSeq !== undefined && segment && segment.parent) {
      check(r, prefix(this, segment, this.getCurrentSeq(), localSeq));
    }
    return r;
  };
}

function runSet(p) {
  if (p.reconnect && !leafHooks.done) {
    leafHooks();
    leafHooks.done = true;
  }
  const v0 = { calls: leafViews.calls, differ: leafViews.differ };
  const R = rng(p.seed);
  const names = [];
  for (let i = 0; i < p.clients; i++) names.push(String.fromCharCode(65 + i));
  const ops = new iv.SequenceIntervalCollectionValueType().ops;
  const factory = new iv.SequenceIntervalCollectionValueType().factory;
  const sent = [];  // the interval op each emitter captures, per client
  const clients = names.map((n, i) => {
    const c = new Client(specToSegment, logger, { mergeTreeUseNewLengthCalculations: true });
    if (p.initialText) c.insertSegmentLocal(0, new TextSegment(p.initialText));
    c.startOrUpdateCollaboration(n);
    c._mergeTree.__traceName = n;  // MTE_REF_TRACE
    const emitter = { emit(opName, _prev, params, meta) { sent[i] = { opName, value: clone(params), meta }; } };
    const coll = factory.load(emitter, []);
    coll.attachGraph(c, LABEL);
    const X = { c, coll, lastSeq: 0, ids: [], ev: [], mt: false };
    if (process.env.MTE_REF_TRACE === n && coll.localCollection && coll.localCollection.endIntervalTree) {
      // the end tree's puts and removes (the host restates them, node/intervals.js)
      const t = coll.localCollection.endIntervalTree;
      const at = (x) => `${x.getIntervalId ? x.getIntervalId() : "?"} [${c.localReferencePositionToPosition(x.start)},` +
        `${c.localReferencePositionToPosition(x.end)}]`;
      const put = t.put.bind(t), remove = t.remove.bind(t);
      t.put = (k, d, cf) => { process.stderr.write(`    PUT ${at(k)}\n`); return put(k, d, cf); };
      t.remove = (k) => { process.stderr.write(`    DEL ${at(k)}\n`); return remove(k); };
    }
    if (p.ext) {
      const pos = (r) => c.localReferencePositionToPosition(r);
      coll.on("addInterval", (ival, local, op) => X.ev.push(["add", ival.getIntervalId(), local, !!op, X.mt]));
      coll.on("deleteInterval", (ival, local, op) => X.ev.push(["delete", ival.getIntervalId(), local, !!op, X.mt]));
      coll.on("changeInterval", (ival, prev, local, op) => X.ev.push(["change", ival.getIntervalId(), local, !!op,
        pos(prev.start), pos(prev.end), pos(ival.start), pos(ival.end), X.mt]));
      if (process.env.MTE_REF_TRACE === n) {
        // each mid-op event's positions beside the same positions summed leaf by leaf
        const lpos = (r) => {
          const sg = r.getSegment();
          if (!sg || !sg.parent) return -1;
          let q = 0;
          const walk = (x) => {
            if (x === sg) return true;
            if (x.isLeaf()) { q += c._mergeTree.localNetLength(x) || 0; return false; }
            for (let i = 0; i < x.childCount; i++) if (walk(x.children[i])) return true;
            return false;
          };
          walk(c._mergeTree.root);
          return q + (sg.removedSeq !== undefined ? 0 : r.getOffset());
        };
        coll.on("changeInterval", (ival, prev, local, op) => process.stderr.write(`  ev ${ival.getIntervalId()} ` +
          `${pos(prev.start)},${pos(prev.end)} -> ${pos(ival.start)},${pos(ival.end)} leaf ${lpos(ival.start)},${lpos(ival.end)}` +
          ` end ${(() => { const g = ival.end.getSegment(); return g ? JSON.stringify(g.text) + "@" + g.ordinal + " rs " + g.removedSeq + " off " + ival.end.getOffset() : "-"; })()}\n`));
      }
      coll.on("propertyChanged", (ival, deltas, local, op) => X.ev.push(["props", ival.getIntervalId(), local, !!op,
        sortKeys(clone(deltas)), X.mt]));
    }
    return X;
  });
  const Q = rng(p.seed ^ 0x5bd1e995);
  const offline = names.map(() => false);
  const held = names.map(() => []);
  const cursor = names.map(() => 0);
  const events = names.map(() => []);
  const log = [];
  let seq = 0, nextId = 0;
  const checkpoints = [];
  const every = Math.max(1, Math.floor(p.steps / Math.max(1, p.nCheckpoints)));
  const msnNow = () => clients.reduce((a, x) => Math.min(a, x.lastSeq), Infinity);

  const applyNext = (i) => {
    const m = log[cursor[i]];
    const msg = { clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
      type: "op", contents: m[5] };
    const X = clients[i];
    if (m[4] === "op") {
      X.mt = true;
      X.c.applyMsg(msg);
      X.mt = false;
    } else {
      const v = m[5].value === undefined ? undefined : clone(m[5].value);  // slid off while rebasing
      ops.get(m[5].opName).process(X.coll, v, m[0] === names[i], msg);
    }
    X.lastSeq = m[1];
    events[i].push(["A", cursor[i]]);
    cursor[i]++;
  };
  const readOut = (X) => {
    const helper = new MergeTreeTextHelper(X.c._mergeTree);
    const text = helper.getText(X.c.getCurrentSeq(), X.c.getClientId(), "");
    const out = [];
    for (const ival of X.coll) {
      const props = Object.assign({}, ival.properties);
      out.push([ival.getIntervalId(), X.c.localReferencePositionToPosition(ival.start),
        X.c.localReferencePositionToPosition(ival.end), sortKeys(props)]);
    }
    out.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
    if (!p.ext) return { text, intervals: out };
    const ids = (xs) => xs.map((x) => x.getIntervalId());
    const n = X.c.getLength();
    const queries = [];
    for (let q = 0; q < 4; q++) {
      const a = Q.int(0, n + 1), b = Q.int(a - 1, n + 2);
      // IntervalCollectionIterator is an Iterator, not an Iterable (:1222-1250): drain it with next()
      const it = (f) => {
        const out = [];
        for (let r = f.next(); !r.done; r = f.next()) out.push(r.value);
        return ids(out);
      };
      queries.push([a, b, ids(X.coll.findOverlappingIntervals(a, b)),
        ids([X.coll.previousInterval(a)].filter(Boolean)), ids([X.coll.nextInterval(a)].filter(Boolean)),
        it(X.coll.CreateForwardIteratorWithStartPosition(a)), it(X.coll.CreateBackwardIteratorWithStartPosition(a)),
        it(X.coll.CreateForwardIteratorWithEndPosition(b)), it(X.coll.CreateBackwardIteratorWithEndPosition(b))]);
    }
    const st = { text, intervals: out, order: ids(Array.from(X.coll)), events: X.ev,
      summary: clone(X.coll.serializeInternal()), queries };
    X.ev = [];
    return st;
  };
  const checkpoint = () => {
    checkpoints.push({ done: events.map((e) => e.length), states: clients.map(readOut) });
  };
  const send = (i, kind, contents, ev) => {
    seq++;
    log.push([names[i], seq, clients[i].lastSeq, msnNow(), kind, contents]);
    events[i].push([ev || (kind === "op" ? "L" : "I"), log.length - 1]);
  };
  const reconnect = (i) => {
    const X = clients[i];
    while (cursor[i] < log.length) applyNext(i);  // every op it sent is acked
    for (const h of held[i]) {
      if (h.op) {
        send(i, "op", clone(X.c.regeneratePendingOp(h.op, h.sg)), "G");
      } else {
        const { rebasedOp } = ops.get(h.opName).rebase(X.coll, { opName: h.opName, value: h.value }, h.meta);
        send(i, "iv", { opName: h.opName, value: rebasedOp.value === undefined ? undefined : clone(rebasedOp.value) },
          "K");
      }
    }
    held[i] = [];
    offline[i] = false;
  };

  for (let step = 0; step < p.steps; step++) {
    if (p.reconnect && R.next() < p.reconnect) {
      const r = R.int(1, p.clients - 1);
      if (offline[r]) reconnect(r);
      else offline[r] = true;
      if ((step + 1) % every === 0 && step + 1 < p.steps) checkpoint();
      continue;
    }
    const i = R.int(1, p.clients - 1);
    const X = clients[i];
    const len = X.c.getLength();
    if (R.next() < p.intervals) {
      // an interval op of client i (SharedString.getIntervalCollection(label).add / change / ...)
      const live = Array.from(X.coll).map((x) => x.getIntervalId());
      const pick = R.next();
      sent[i] = undefined;
      if (live.length === 0 || pick < 0.35) {
        if (len === 0) continue;
        const s0 = R.int(0, len - 1), e0 = R.int(s0, Math.min(len - 1, s0 + R.int(0, 12)));
        const id = `iv${nextId++}`;
        const props = { intervalId: id };
        if (R.next() < 0.3) props[KEYS[R.int(0, 2)]] = R.int(0, 3);
        X.coll.add(s0, e0, iv.IntervalType.SlideOnRemove, props);
      } else {
        const id = live[R.int(0, live.length - 1)];
        if (pick < 0.6) {
          if (len === 0) continue;
          const s0 = R.int(0, len - 1), e0 = R.int(s0, Math.min(len - 1, s0 + R.int(0, 12)));
          const which = R.int(0, 2);
          X.coll.change(id, which === 2 ? undefined : s0, which === 1 ? undefined : e0);
        } else if (pick < 0.8) {
          X.coll.changeProperties(id, { [KEYS[R.int(0, 2)]]: R.next() < 0.2 ? null : R.int(0, 5) });
        } else {
          X.coll.removeIntervalById(id);
        }
      }
      if (sent[i] && offline[i]) {
        // made offline: pending, not sent
        held[i].push({ opName: sent[i].opName, value: sent[i].value, meta: sent[i].meta });
        events[i].push(["J", { opName: sent[i].opName, value: sent[i].value }]);
      } else if (sent[i]) {
        send(i, "iv", { opName: sent[i].opName, value: sent[i].value });
      }
    } else if (R.next() < 0.5) {
      // a merge-tree op (as oracle/ref_farm.js)
      let op;
      X.mt = true;
      if (len < 4 || (R.next() < 0.4 && len < p.maxText)) {
        const pos = R.int(0, len);
        const seg = new TextSegment(names[i].repeat(R.int(1, 3)));
        op = X.c.insertSegmentLocal(pos, seg);
      } else {
        const start = R.int(0, len - 1);
        const end = R.int(start + 1, Math.min(len, start + 1 + R.int(0, 24)));
        if (R.next() < 0.7) op = X.c.removeRangeLocal(start, end);
        else op = X.c.annotateRangeLocal(start, end, { [KEYS[R.int(0, 2)]]: R.int(0, 5) }, undefined);
      }
      X.mt = false;
      if (op && offline[i]) {
        held[i].push({ op, sg: X.c.peekPendingSegmentGroups() });
        events[i].push(["H", clone(op)]);
      } else if (op) {
        send(i, "op", clone(op));
      }
    } else {
      const j = R.int(0, p.clients - 1);
      const k = R.int(1, 6);
      for (let q = 0; q < k && cursor[j] < log.length; q++) applyNext(j);
    }
    if ((step + 1) % every === 0 && step + 1 < p.steps) checkpoint();
  }
  for (let i = 0; i < p.clients; i++) if (offline[i]) reconnect(i);
  for (let i = 0; i < p.clients; i++) while (cursor[i] < log.length) applyNext(i);
  checkpoint();
  const last = checkpoints[checkpoints.length - 1].states;
  let diverged = null;  // allowDiverge: the clients' final states differ (recorded, not thrown)
  for (const s of last) {
    if (s.text !== last[0].text || JSON.stringify(s.intervals) !== JSON.stringify(last[0].intervals)) {
      if (!p.allowDiverge) throw new Error(`seed ${p.seed}: the reference clients did not converge`);
      diverged = s.text !== last[0].text ? "text" : "intervals";
    }
  }
  const lv = p.reconnect ? { leafViews: { calls: leafViews.calls - v0.calls, differ: leafViews.differ - v0.differ } } : {};
  return Object.assign({}, p, { names, log, events, checkpoints }, diverged ? { diverged } : {}, lv);
}

const input = JSON.parse(fs.readFileSync(0, "utf8"));
process.stdout.write(JSON.stringify({ sets: input.sets.map(runSet) }));
