#!/usr/bin/env node
// ref_farm.js — a conflict farm of REFERENCE merge-tree Clients with local ops,
// acks and lagging clients (TEST INFRASTRUCTURE; runs only in the build
// container, never on the GPU box).
//
// Like test/client.conflictFarm.spec.ts + test/mergeTreeOperationRunner.ts
// (every client a collaborating Client with the new length calculation, :84;
// ops made locally with insertSegmentLocal / removeRangeLocal /
// annotateRangeLocal, client.ts:131-229, and their sequenced messages applied
// by every client — its own as acks, client.ts:918-935), but the sequencer and
// the clients run as a service does: a message is sequenced as soon as it is
// sent, with refSeq = the sender's currentSeq and msn = the lowest currentSeq
// of any client, and every client catches up with the sequenced log at its own
// pace.  So ops see lagging refSeqs, a client's pending ops meet remote ops
// (breakTie / continuePredicate, mergeTree.ts:1599-1611, 1705-1721, 1790;
// overlapping removes, :1928-1938; pending property keys,
// segmentPropertiesManager.ts:94-135) and the window trails far behind.
//
// stdin:  {"sets": [{"seed": int, "clients": int, "steps": int, "initialText": str,
//                    "nCheckpoints": int, "maxText": int, "rollback": p}]}
//         (rollback: the chance that a local remove -- with rollbackInserts
//         also an insert, with rollbackTypes [MergeTreeDeltaType, ...] those
//         types, annotates included -- is rolled back instead of sent; the
//         event is ["R", op]: the client made the op locally, then rolled it
//         back.
//          reconnect: the chance per step that a sending client goes offline,
//         or, when offline, reconnects.  Offline, its local ops are held
//         (["H", op]); reconnecting, it catches up with the whole log, then
//         re-sends every held op through Client.regeneratePendingOp
//         (client.ts:972-1002), as test/client.reconnectFarm.spec.ts:25-59
//         does: ["G", logIndex], the log entry holding the regenerated op)
//          refs: the chance per step that a client (the observer included)
//         creates a local reference -- Client.createLocalReferencePosition on
//         getContainingSegment(pos) in its own view, SlideOnRemove or Simple
//         (client.ts:360-364, 1107-1110) -- or removes one of its own
//         (removeLocalReferencePosition): ["F", pos, refType] / ["X", index];
//         each checkpoint state then holds "refs", the client's references'
//         localReferencePositionToPosition in creation order (null: removed);
//          combine: the chance that an annotate carries a combining op
//         (incr with or without defaultValue / minValue, or consensus on an
//         id'd marker), its values sometimes strings
//          transient: the chance that a reference made is Transient (a
//         segment and offset the tree does not track: localReference.ts:263,
//         mergeTree.ts:1095-1112), drawn before stay;
//          stay: the chance that a reference made is StayOnRemove (drawn from
//         the same number, so the farms without it are unchanged)
// stdout: {"sets": [{..params, "names": [...], "log": [[clientId, seq, ref, msn, "op", contents]],
//                    "events": [[["L"|"A", logIndex] | ["R", op], ...] per client],
//                    "checkpoints": [{"done": [events applied per client],
//                                     "states": [{"text", "props": [[start, end, {..}]]}]}]}]}
//          legacy: the clients keep the default (legacy) length calculation
//         instead of mergeTreeUseNewLengthCalculations
//          relpos: the chance that a local op addresses a marker by its id
//         (IRelativePosition, ops.ts:62-76, resolved by posFromRelativePos,
//         mergeTree.ts:1369-1392, from getValidOpRange, client.ts:541-560):
//         Client.annotateMarker (client.ts:166-174, opBuilder.ts:26-40), or a
//         remove / insert whose relativePos1 / relativePos2 name a marker the
//         client sees, applied through the Client's own op path
//         (applyRemoveRangeOp / applyInsertOp, client.ts:405-500); with relpos
//         the marker ids are unique ("mk<n>")
//          maint: record every client's maintenance callbacks ("maint" in
//         the output: per client [event index, type, [[position, length]...]])
// Client 0 ("A") never sends: the observer.
"use strict";
const path = require("path");
const fs = require("fs");

const refdir = process.argv[2] || path.join(__dirname, "_ref", "ts");
const { Client } = require(path.join(refdir, "client.js"));
const { TextSegment } = require(path.join(refdir, "textSegment.js"));
const { Marker } = require(path.join(refdir, "mergeTreeNodes.js"));
const { MergeTreeTextHelper } = require(path.join(refdir, "MergeTreeTextHelper.js"));
const { ReferenceType } = require(path.join(refdir, "ops.js"));

function specToSegment(spec) {
  const t = TextSegment.fromJSONObject(spec);
  if (t) return t;
  const m = Marker.fromJSONObject(spec);
  if (m) return m;
  throw new Error(`Unrecognized IJSONSegment type: '${JSON.stringify(spec)}'`);
}
const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

// mulberry32: a small seeded generator (the farm's random-js is not vendored)
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

function readOut(client) {
  const helper = new MergeTreeTextHelper(client._mergeTree);
  const text = helper.getText(client.getCurrentSeq(), client.getClientId(), "");
  const length = client.getLength();
  const props = [];
  let cur = null;
  let start = 0;
  for (let p = 0; p < length; p++) {
    const pr = client.getPropertiesAtPosition(p);
    const key = pr && Object.keys(pr).length ? JSON.stringify(sortKeys(pr)) : "";
    if (key !== cur) {
      if (cur) props.push([start, p, JSON.parse(cur)]);
      cur = key;
      start = p;
    }
  }
  if (cur) props.push([start, length, JSON.parse(cur)]);
  return { text, length, props };
}

const KEYS = ["client", "bold", "color"];
const STRS = ["a", "zz", "m", "q"];
// combine: the combining ops a farm's annotates draw from (properties.ts:24-62)
const COMBINING = [{ name: "incr" }, { name: "incr", defaultValue: 2 }, { name: "incr", minValue: 3 },
  { name: "incr", defaultValue: "q", minValue: "r" }, { name: "incr", minValue: "n" }];

function runSet(p) {
  const R = rng(p.seed);
  const names = [];
  for (let i = 0; i < p.clients; i++) names.push(String.fromCharCode(65 + i));
  const clients = names.map((n) => {
    // legacy: the default length calculation (mergeTree.ts:386-399)
    const c = new Client(specToSegment, logger, { mergeTreeUseNewLengthCalculations: !p.legacy });
    if (p.initialText) c.insertSegmentLocal(0, new TextSegment(p.initialText));
    c.startOrUpdateCollaboration(n);
    return c;
  });
  // maint: each client's mergeTreeMaintenanceCallback (mergeTree.ts:695-725,
  // 1313-1320, 1687-1694), per event: [event index, MergeTreeMaintenanceType,
  // its ranges as SequenceMaintenanceEvent.ranges sorts them (segment ordinal,
  // sortedSegmentSet.ts) as [Client.getPosition once the event is applied (-1:
  // out of the tree), cachedLength when the callback ran]]
  const maint = names.map(() => []);
  const mbuf = names.map(() => []);
  if (p.maint) {
    clients.forEach((c, i) => {
      c.mergeTreeMaintenanceCallback = (args) => {
        mbuf[i].push([args.operation, args.deltaSegments.map((d) => [d.segment, d.segment.cachedLength,
          d.segment.ordinal])]);
      };
    });
  }
  // positions once the message (or local op) that raised them is applied;
  // the segments of an ACKNOWLEDGED callback in document order (the group's
  // order is the segments' pending order), a SPLIT's / an APPEND's in the
  // callback's (the pieces, the segment appended to and the one appended)
  const settle = (i, at = events[i].length - 1) => {
    for (const [t, segs] of mbuf[i]) {
      // (ordinals as the callback saw them: an unlinked segment keeps a stale one)
      const r = segs.map(([sg, len, ord]) => [ord, clients[i].getPosition(sg), len]);
      if (t === -4) r.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
      maint[i].push([at, t, r.map((x) => [x[1], x[2]])]);
    }
    mbuf[i] = [];
  };
  const cursor = names.map(() => 0);
  const offline = names.map(() => false);
  const held = names.map(() => []);  // [op, segment group] per held op
  const events = names.map(() => []);
  const refs = names.map(() => []);  // per client, in creation order (null: removed)
  const log = [];
  let seq = 0;
  const checkpoints = [];
  const every = Math.max(1, Math.floor(p.steps / Math.max(1, p.nCheckpoints)));
  let markerNo = 0;
  // the id'd markers a client's own view holds
  const idMarkers = (c) => {
    const out = [];
    const len = c.getLength();
    for (let pos = 0; pos < len; pos++) {
      const { segment } = c.getContainingSegment(pos);
      if (segment && Marker.is(segment) && segment.getId()) out.push(segment);
    }
    return out;
  };
  // combine: an annotate with a combining op -- incr through annotateRangeLocal,
  // or consensus on an id'd marker of the range through
  // annotateMarkerNotifyConsensus (client.ts:137-158; a range consensus would
  // fail at its own ack, updateConsensusProperty reading relativePos1)
  const combineOp = (c, start, end, props) => {
    if (R.next() < 0.3) {
      for (let pos = start; pos < end; pos++) {
        const { segment } = c.getContainingSegment(pos);
        if (segment && Marker.is(segment) && segment.getId()) {
          return c.annotateMarkerNotifyConsensus(segment, props, () => {});
        }
      }
    }
    const comb = COMBINING[R.int(0, COMBINING.length - 1)];
    return c.annotateRangeLocal(start, end, props, { ...comb });
  };
  const relPos = (id) => {
    const rp = { id };
    if (R.next() < 0.5) rp.before = true;
    if (R.next() < 0.5) rp.offset = R.int(0, 3);
    return rp;
  };
  // a local op through a relative position; undefined when the range is not
  // valid in the client's view (getValidOpRange throws)
  const relOp = (c, i) => {
    const ms = idMarkers(c);
    if (!ms.length) return undefined;
    const m = ms[R.int(0, ms.length - 1)];
    const pick = R.next();
    try {
      if (pick < 0.5) {
        const props = { [KEYS[R.int(0, 2)]]: R.next() < 0.15 ? null : R.int(0, 5) };
        return c.annotateMarker(m, props, undefined);
      }
      if (pick < 0.75) {
        const op = { type: 1, relativePos1: relPos(m.getId()), relativePos2: relPos(m.getId()) };
        if (R.next() < 0.5) op.relativePos1.before = true;
        return c.applyRemoveRangeOp({ op }) ? op : undefined;
      }
      const op = { type: 0, relativePos1: relPos(m.getId()), seg: new TextSegment(names[i].toLowerCase()).toJSONObject() };
      return c.applyInsertOp({ op }) ? op : undefined;
    } catch (e) {
      if (e && (e.message === "RangeOutOfBounds" || /RangeOutOfBounds/.test(String(e.message)))) return undefined;
      throw e;
    }
  };

  const applyNext = (i) => {
    const m = log[cursor[i]];
    clients[i].applyMsg({
      clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
      type: m[4], contents: m[5],
    });
    events[i].push(["A", cursor[i]]);
    settle(i);
    cursor[i]++;
  };
  const reconnect = (i) => {
    const c = clients[i];
    while (cursor[i] < log.length) applyNext(i);  // every op it sent is acked
    for (const [op, sg] of held[i]) {
      const regen = c.regeneratePendingOp(op, sg);
      let msn = Infinity;
      for (const x of clients) msn = Math.min(msn, x.getCurrentSeq());
      seq++;
      log.push([names[i], seq, c.getCurrentSeq(), msn, "op", JSON.parse(JSON.stringify(regen))]);
      events[i].push(["G", log.length - 1]);
      settle(i);
    }
    held[i] = [];
    offline[i] = false;
  };
  const checkpoint = () => {
    const states = clients.map(readOut);
    if (p.refs) {
      states.forEach((st, i) => {
        st.refs = refs[i].map((r) => (r === null ? null : clients[i].localReferencePositionToPosition(r)));
      });
    }
    checkpoints.push({ done: events.map((e) => e.length), states });
  };

  for (let step = 0; step < p.steps; step++) {
    if (p.refs && R.next() < p.refs) {
      // a local reference made or dropped by any client (its own, not sequenced)
      const i = R.int(0, p.clients - 1);
      const c = clients[i];
      const live = [];
      refs[i].forEach((r, k) => { if (r !== null) live.push(k); });
      const len = c.getLength();
      if (len > 0 && (live.length === 0 || R.next() < 0.75)) {
        const pos = R.int(0, len - 1);
        const u = R.next();
        const type = p.transient && u < p.transient ? ReferenceType.Transient
          : p.stay && u < p.stay ? ReferenceType.StayOnRemove
            : u < 0.8 ? ReferenceType.SlideOnRemove : ReferenceType.Simple;
        const { segment, offset } = c.getContainingSegment(pos);
        refs[i].push(c.createLocalReferencePosition(segment, offset, type, undefined));
        events[i].push(["F", pos, type]);
        settle(i);
      } else if (live.length > 0) {
        const k = live[R.int(0, live.length - 1)];
        c.removeLocalReferencePosition(refs[i][k]);
        refs[i][k] = null;
        events[i].push(["X", k]);
        settle(i);
      }
      if ((step + 1) % every === 0 && step + 1 < p.steps) checkpoint();
      continue;
    }
    if (p.reconnect && R.next() < p.reconnect) {
      const i = R.int(1, p.clients - 1);
      if (offline[i]) reconnect(i);
      else offline[i] = true;
    } else if (R.next() < 0.55) {
      // a local op of a sending client (client 0 only observes)
      const i = R.int(1, p.clients - 1);
      const c = clients[i];
      const len = c.getLength();
      const pick = R.next();
      let op;
      if (p.relpos && len >= 4 && R.next() < p.relpos) {
        op = relOp(c, i);
      } else if (len < 4 || (pick < 0.4 && len < p.maxText)) {
        const pos = R.int(0, len);
        if (R.next() < (p.relpos ? 0.2 : 0.08)) {
          const props = R.next() < 0.5 ? { markerId: p.relpos ? `mk${markerNo++}` : `m${seq}` } : undefined;
          op = c.insertSegmentLocal(pos, Marker.make(1, props));
        } else {
          const text = names[i].repeat(R.int(1, 3));
          const seg = new TextSegment(text);
          if (R.next() < 0.2) seg.addProperties({ [KEYS[R.int(0, 2)]]: R.int(0, 3) });
          op = c.insertSegmentLocal(pos, seg);
        }
      } else {
        const start = R.int(0, len - 1);
        const end = R.int(start + 1, Math.min(len, start + 1 + R.int(0, 24)));
        if (pick < 0.7) {
          op = c.removeRangeLocal(start, end);
        } else {
          const props = {};
          const nk = R.int(1, 2);
          for (let k = 0; k < nk; k++) props[KEYS[R.int(0, 2)]] = R.next() < 0.15 ? null : R.int(0, 5);
          if (p.combine && R.next() < 0.4) {
            // string values too, so that incr's string branch is reached
            for (const k of Object.keys(props)) if (R.next() < 0.3) props[k] = STRS[R.int(0, STRS.length - 1)];
          }
          if (p.combine && R.next() < p.combine) op = combineOp(c, start, end, props);
          else op = c.annotateRangeLocal(start, end, props, undefined);
        }
      }
      if (op && offline[i]) {
        // made while offline: pending, not sent
        events[i].push(["H", JSON.parse(JSON.stringify(op))]);
        settle(i);
        held[i].push([op, c.peekPendingSegmentGroups()]);
      } else if (op && p.rollback && (p.rollbackTypes ? p.rollbackTypes.includes(op.type)
        : (p.rollbackInserts ? op.type !== 2 : op.type === 1)) && R.next() < p.rollback) {
        // Client.rollback of the op just made (client.ts:396-398 ->
        // MergeTree.rollback, mergeTree.ts:2005-2083): it is never sent
        const opJson = JSON.parse(JSON.stringify(op));
        settle(i, events[i].length);  // the local op's, before the rollback
        c.rollback(op, c.peekPendingSegmentGroups());
        events[i].push(["R", opJson]);
        settle(i);
      } else if (op) {
        let msn = Infinity;
        for (const x of clients) msn = Math.min(msn, x.getCurrentSeq());
        seq++;
        log.push([names[i], seq, c.getCurrentSeq(), msn, "op", JSON.parse(JSON.stringify(op))]);
        events[i].push(["L", log.length - 1]);
        settle(i);
      }
    } else {
      // a client catches up with a few sequenced messages
      const i = R.int(0, p.clients - 1);
      const k = R.int(1, 6);
      for (let j = 0; j < k && cursor[i] < log.length; j++) applyNext(i);
    }
    if ((step + 1) % every === 0 && step + 1 < p.steps) checkpoint();
  }
  for (let i = 0; i < p.clients; i++) if (offline[i]) reconnect(i);
  for (let i = 0; i < p.clients; i++) while (cursor[i] < log.length) applyNext(i);
  checkpoint();
  let diverged = null;  // allowDiverge: the clients' final documents differ (recorded, not thrown)
  const t0 = checkpoints[checkpoints.length - 1].states[0];
  for (const s of checkpoints[checkpoints.length - 1].states) {
    if (s.text !== t0.text || JSON.stringify(s.props) !== JSON.stringify(t0.props)) {
      const what = s.text !== t0.text ? `text ${JSON.stringify(s.text)} vs ${JSON.stringify(t0.text)}`
        : `props ${JSON.stringify(s.props)} vs ${JSON.stringify(t0.props)}`;
      if (!p.allowDiverge) throw new Error(`seed ${p.seed}: the reference clients did not converge: ${what}`);
      diverged = what;
    }
  }
  return Object.assign({}, p, { names, log, events, checkpoints }, diverged ? { diverged } : {},
    p.maint ? { maint } : {});
}

const input = JSON.parse(fs.readFileSync(0, "utf8"));
process.stdout.write(JSON.stringify({ sets: input.sets.map(runSet) }));
