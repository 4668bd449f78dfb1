#!/usr/bin/env node
// The Node host path end to end (bench.py's end_to_end_node leg): message
// objects -> BatchClient.applyMsg (JS packing into 32-byte records) ->
// MergeTreeEngine.flush (mte_submit upload + mte_run + mte_sync through
// N-API) -> digests.  stdin: {"docs": [{initialText, newCalc, roundSync,
// msgs: [[clientId, seq, refSeq, msn, type, contents], ...]}], "reps": R}.
// The messages are turned into ISequencedDocumentMessage objects before the
// clock starts (a host receives them as objects from its delta stream).
"use strict";
const fs = require("fs");
const { MergeTreeEngine } = require("./index.js");

const input = JSON.parse(fs.readFileSync(0, "utf8"));
const msgs = input.docs.map((d) => d.msgs.map((m) => ({
  clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
  type: m[4], contents: m[5],
})));
const nOps = msgs.reduce((a, m) => a + m.length, 0);
const runs = [];
let digests = null;
let texts = null;
for (let rep = 0; rep < (input.reps || 2); rep++) {
  const eng = new MergeTreeEngine({ nKeys: 4, segCapacity: input.segCapacity || 0 });
  const clients = input.docs.map((d) => eng.createClient(d.initialText,
    { newLengthCalc: d.newCalc, roundSync: d.roundSync }));
  eng.start();  // load (mte_load_docs) outside the clock
  const t0 = process.hrtime.bigint();
  // documents interleaved in arrival order: message i of every document, then i + 1
  const maxLen = msgs.reduce((a, m) => Math.max(a, m.length), 0);
  for (let i = 0; i < maxLen; i++) {
    for (let d = 0; d < clients.length; d++) if (i < msgs[d].length) clients[d].applyMsg(msgs[d][i]);
  }
  const t1 = process.hrtime.bigint();
  eng.flush();
  const t2 = process.hrtime.bigint();
  digests = eng.digests();
  const status = eng.statuses();
  texts = clients.map((c) => c.getText());
  const t3 = process.hrtime.bigint();
  runs.push({ pack_ms: Number(t1 - t0) / 1e6, flush_ms: Number(t2 - t1) / 1e6, readout_ms: Number(t3 - t2) / 1e6,
    errors: status.reduce((a, x) => a + (x !== 0 ? 1 : 0), 0) });
  eng.close();
}
// pipelined: the messages arrive in `parts` slices per document; each slice is
// flushed as it is packed, so packing and uploading slice i + 1 overlap the
// replay of slice i (the engine's two batch slots)
const parts = input.parts || 4;
const piped = [];
for (let rep = 0; rep < (input.reps || 2); rep++) {
  const eng = new MergeTreeEngine({ nKeys: 4, segCapacity: input.segCapacity || 0 });
  const clients = input.docs.map((d) => eng.createClient(d.initialText,
    { newLengthCalc: d.newCalc, roundSync: d.roundSync }));
  eng.start();
  const maxLen = msgs.reduce((a, m) => Math.max(a, m.length), 0);
  const t0 = process.hrtime.bigint();
  for (let p = 0; p < parts; p++) {
    const i0 = Math.floor((maxLen * p) / parts), i1 = Math.floor((maxLen * (p + 1)) / parts);
    for (let i = i0; i < i1; i++) {
      for (let d = 0; d < clients.length; d++) if (i < msgs[d].length) clients[d].applyMsg(msgs[d][i]);
    }
    eng.flush();
  }
  eng.sync();
  const t1 = process.hrtime.bigint();
  const dg = eng.digests();
  const same = dg.every((x, k) => x === digests[k]);
  piped.push({ ms: Number(t1 - t0) / 1e6, digest_equal: same });
  eng.close();
}
const bestPiped = piped.reduce((a, r) => (a === null || r.ms < a.ms ? r : a), null);

const best = runs.reduce((a, r) => (a === null || r.pack_ms + r.flush_ms < a.pack_ms + a.flush_ms ? r : a), null);
process.stdout.write(JSON.stringify({ ops: nOps, docs: input.docs.length, runs, best,
  ops_per_s: nOps / ((best.pack_ms + best.flush_ms) / 1e3),
  pipelined: { parts, ms: bestPiped.ms, ops_per_s: nOps / (bestPiped.ms / 1e3), digest_equal: bestPiped.digest_equal },
  texts }));
