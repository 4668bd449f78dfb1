#!/usr/bin/env node
// ref_replay.js — observer replay through the REFERENCE merge-tree itself
// (TEST INFRASTRUCTURE; runs only in the build container, never on the GPU box).
//
// Loads the reference packages/dds/merge-tree Client as oracle/ts_erase.py
// downlevelled it into oracle/_ref/ts/ (git- and gpurun-ignored) and replays
// documents the way test/client.replay.spec.ts:16-60 does for its original
// client "A": the initial text is inserted locally before collaboration
// (insertTextLocal + startOrUpdateCollaboration("A")), then every sequenced
// message goes through Client.applyMsg (client.ts:918-935).  The read-out is
// TestClient.getText (test/testClient.ts:148-150) and getPropertiesAtPosition
// (client.ts:1133-1141) for every position.
//
// stdin:  {"docs": [{"initialText": str, "newCalc": bool,
//                    "msgs": [[clientId, seq, refSeq, msn, type, contents], ...]}]}
// stdout: {"docs": [{"text": str, "length": int, "props": [[start, end, {..}], ...],
//                    "error": str|null, "applied": int, "ms": float}]}
"use strict";
const path = require("path");
const fs = require("fs");

const refdir = process.argv[2] || path.join(__dirname, "_ref", "ts");
const { Client } = require(path.join(refdir, "client.js"));
const { TextSegment } = require(path.join(refdir, "textSegment.js"));
const { Marker } = require(path.join(refdir, "mergeTreeNodes.js"));
const { MergeTreeTextHelper } = require(path.join(refdir, "MergeTreeTextHelper.js"));
const { walkAllChildSegments } = require(path.join(refdir, "mergeTreeNodeWalk.js"));

// test/testClient.ts:32-44
function specToSegment(spec) {
  const t = TextSegment.fromJSONObject(spec);
  if (t) return t;
  const m = Marker.fromJSONObject(spec);
  if (m) return m;
  throw new Error(`Unrecognized IJSONSegment type: '${JSON.stringify(spec)}'`);
}

const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };

function sortKeys(v) {
  if (Array.isArray(v)) return v.map(sortKeys);
  if (v && typeof v === "object") {
    const o = {};
    for (const k of Object.keys(v).sort()) o[k] = sortKeys(v[k]);
    return o;
  }
  return v;
}

function replayDoc(d) {
  const t0 = process.hrtime.bigint();
  const client = new Client(specToSegment, logger, d.newCalc ? { mergeTreeUseNewLengthCalculations: true } : undefined);
  if (d.initialText) client.insertSegmentLocal(0, new TextSegment(d.initialText)); // TestClient.insertTextLocal (test/testClient.ts:179-189)
  client.startOrUpdateCollaboration("A");
  let error = null;
  let applied = 0;
  // d.deltas: record every mergeTreeDeltaCallback (mergeTree.ts:1409-1416,
  // 1893-1900, 1978-1985) as SharedString's sequenceDelta listener reads it
  // (sequence.ts:203-211, 688-725; SequenceEvent.ranges, sequenceDeltaEvent.ts):
  // [message index, operation, [[client.getPosition(segment), cachedLength, removed], ...]]
  const deltas = [];
  if (d.deltas) {
    client.mergeTreeDeltaCallback = (opArgs, deltaArgs) => {
      deltas.push([applied, deltaArgs.operation,
        deltaArgs.deltaSegments.map((ds) => [client.getPosition(ds.segment), ds.segment.cachedLength,
          ds.segment.removedSeq !== undefined ? 1 : 0])]);
    };
  }
  // d.maint: every mergeTreeMaintenanceCallback (mergeTree.ts:695-725,
  // 1687-1694) as [message index, MergeTreeMaintenanceType, [[Client.getPosition
  // once the message is applied (-1: unlinked), cachedLength at the callback],
  // ...]] -- the ranges SharedString's "maintenance" event reads (sequence.ts:212-216)
  const maint = [];
  let mbuf = [];
  if (d.maint) {
    client.mergeTreeMaintenanceCallback = (args) => {
      mbuf.push([applied, args.operation, args.deltaSegments.map((ds) => [ds.segment, ds.segment.cachedLength])]);
    };
  }
  const settle = () => {
    for (const [mi, t, segs] of mbuf) maint.push([mi, t, segs.map(([sg, len]) => [client.getPosition(sg), len])]);
    mbuf = [];
  };
  for (const m of d.msgs) {
    const msg = {
      clientId: m[0],
      sequenceNumber: m[1],
      referenceSequenceNumber: m[2],
      minimumSequenceNumber: m[3],
      type: m[4],
      contents: m[5],
    };
    try {
      client.applyMsg(msg);
    } catch (e) {
      error = String(e && e.message ? e.message : e);
      break;
    }
    if (d.maint) settle();
    applied++;
  }
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  const helper = new MergeTreeTextHelper(client._mergeTree); // as TestClient does (test/testClient.ts:115)
  const text = helper.getText(client.getCurrentSeq(), client.getClientId(), "");
  const length = client.getLength();
  // per-position properties as runs (empty == undefined, testClientLogger.ts:33-42)
  const props = [];
  if (d.props !== false) {
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
  }
  // the visible segments in order (gatherText's walk, MergeTreeTextHelper.ts:49-74):
  // [text, props] or [{"marker": refType}, props]
  const segs = [];
  if (d.segs) {
    walkAllChildSegments(client._mergeTree.root, (seg) => {
      if (seg.removedSeq === undefined) {
        const p = seg.properties && Object.keys(seg.properties).length ? seg.properties : null;
        segs.push([TextSegment.is(seg) ? seg.text : { marker: seg.refType }, p]);
      }
      return true;
    });
  }
  return { text, length, props, segs, error, applied, ms, deltas: d.deltas ? deltas : undefined,
    maint: d.maint ? maint : undefined };
}

const input = JSON.parse(fs.readFileSync(0, "utf8"));
const out = { docs: input.docs.map(replayDoc) };
process.stdout.write(JSON.stringify(out));
