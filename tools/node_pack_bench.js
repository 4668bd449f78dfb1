#!/usr/bin/env node
// Host packing alone (no device): BatchClient.applyMsg over message objects
// into the engine's batch, with a recording N-API stand-in -- the pack_ms of
// bench.py's end_to_end_node leg, measurable on the CPU.  stdin as
// bench_e2e.js ({"docs": [...], "reps": R}); prints {"pack_ms": [...], "ops"}.
"use strict";
const fs = require("fs");
const { MergeTreeEngine } = require("../fluidframework_amd/node");

const input = JSON.parse(fs.readFileSync(0, "utf8"));
const msgs = input.docs.map((d) => d.msgs.map((m) => ({
  clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
  type: m[4], contents: m[5],
})));
const nOps = msgs.reduce((a, m) => a + m.length, 0);
const addon = {
  create() { return {}; }, destroy() {}, loadDocs() {}, loadSegments() {}, submit() {}, run() {}, sync() {},
  readDeltas() { return new Uint32Array(0); },
};
const out = [];
for (let rep = 0; rep < (input.reps || 3); rep++) {
  const eng = new MergeTreeEngine({ nKeys: 4, addon });
  const clients = input.docs.map((d) => eng.createClient(d.initialText, { newLengthCalc: d.newCalc, roundSync: d.roundSync }));
  eng.start();
  const maxLen = msgs.reduce((a, m) => Math.max(a, m.length), 0);
  const t0 = process.hrtime.bigint();
  for (let i = 0; i < maxLen; i++) {
    for (let d = 0; d < clients.length; d++) if (i < msgs[d].length) clients[d].applyMsg(msgs[d][i]);
  }
  eng._batch();
  const t1 = process.hrtime.bigint();
  out.push(Number(t1 - t0) / 1e6);
  eng.flush();
}
process.stdout.write(JSON.stringify({ pack_ms: out, ops: nOps, mops: nOps / Math.min(...out) / 1e3 }) + "\n");
