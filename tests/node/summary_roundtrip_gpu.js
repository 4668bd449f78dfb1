"use strict";
// GPU test: summaries through the Node host layer.  Engine A replays the
// golden fixtures' first half as observer "A" (client.replay.spec.ts:16-60);
// every document is summarized (BatchClient.summarize: snapshotV1.ts:189-265
// rules over mte_read_segments) and loaded into engine B
// (createClient("", {segments, minSeq, currentSeq}): SnapshotLoader.loadBody
// -> mte_load_segments), which replays the second half.  Every checkpoint
// text of the second half must hold.  Prints one JSON line.
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { loadFixtures, asMsg } = require("./fixtures");

const fx = loadFixtures();
const half = 32;
const a = new MergeTreeEngine({ nKeys: 8 });
const ca = fx.map((f) => a.createClient(f.rounds[0].initialText));
for (let r = 0; r < half; r++) {
  fx.forEach((f, d) => {
    if (r < f.rounds.length) for (const m of f.rounds[r].msgs) ca[d].applyMsg(asMsg(m));
  });
}
const sums = ca.map((c) => c.summarize());
const b = new MergeTreeEngine({ nKeys: 8 });
const cb = fx.map((f, d) => b.createClient("", { segments: sums[d].segments, minSeq: sums[d].minSeq,
  currentSeq: sums[d].currentSeq }));
let passed = 0, withInfo = 0;
const failures = [];
sums.forEach((s) => { withInfo += s.segments.filter((x) => x.seq !== undefined || x.removedSeq !== undefined).length; });
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
  segmentsWithMergeInfo: withInfo }) + "\n");
a.close();
b.close();
