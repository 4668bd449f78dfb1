"use strict";
// GPU test: legacy summaries through the Node host layer.  Engine A replays
// the golden fixtures' first half as observer "A"; every document writes a
// legacy summary (BatchClient.summarizeLegacy: SnapshotLegacy.extractSync +
// emit, snapshotlegacy.ts:105-211) with the messages it saw as catch-up
// candidates (sequence.ts:676-686), which engine B loads
// (createClient("", {legacy}): snapshotLoader.ts:130-246 + the catch-up replay
// of sequence.ts:588-609) before replaying the second half.  Every checkpoint
// text of the second half must hold.  A small first chunk (argv[2]) forces
// header + body.  Prints one JSON line.
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { loadFixtures, asMsg } = require("./fixtures");

const chunkSize = process.argv[2] ? parseInt(process.argv[2], 10) : undefined;
const fx = loadFixtures();
const half = 32;
const a = new MergeTreeEngine({ nKeys: 8 });
const ca = fx.map((f) => a.createClient(f.rounds[0].initialText));
const seen = fx.map(() => []);
for (let r = 0; r < half; r++) {
  fx.forEach((f, d) => {
    if (r < f.rounds.length) {
      for (const m of f.rounds[r].msgs) { const msg = asMsg(m); seen[d].push(msg); ca[d].applyMsg(msg); }
    }
  });
}
const sums = ca.map((c, d) => c.summarizeLegacy(seen[d], chunkSize));
const b = new MergeTreeEngine({ nKeys: 8 });
const cb = fx.map((f, d) => b.createClient("", { legacy: JSON.parse(JSON.stringify(sums[d])) }));
let passed = 0, withBody = 0, catchup = 0;
const failures = [];
sums.forEach((s) => { if (s.body) withBody++; catchup += (s.catchupOps || []).length; });
for (let r = half; r < 64; r++) {
  fx.forEach((f, d) => {
    if (r >= f.rounds.length) return;
    if (cb[d].getText() === f.rounds[r].initialText) passed++; else failures.push([f.name, r, "initial"]);
    for (const m of f.rounds[r].msgs) cb[d].applyMsg(asMsg(m));
  });
  fx.forEach((f, d) => {
    if (r >= f.rounds.length) return;
    if (cb[d].getText() === f.rounds[r].resultText) passed++; else failures.push([f.name, r, "result"]);
  });
}
process.stdout.write(JSON.stringify({ passed, nFailures: failures.length, failures: failures.slice(0, 5),
  withBody, catchup }) + "\n");
a.close();
b.close();
