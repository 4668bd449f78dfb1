"use strict";
// GPU test: the Node host layer (BatchClient over the N-API addon) replays
// the reference's golden fixtures as client "A" (client.replay.spec.ts:16-60)
// and checks initialText / resultText of every round.  Prints one JSON line.
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { loadFixtures, asMsg } = require("./fixtures");

const fx = loadFixtures();
const eng = new MergeTreeEngine({ nKeys: 8 });
// argv "body": each initial text arrives as a summary body of 3-unit
// segments (SnapshotLoader.loadBody path, mte_load_segments) instead of one
// segment; segmentation is unobservable, so every checkpoint must still hold
const asBody = process.argv[2] === "body";
// argv "fresh": every round's senders get new long ids ("B" -> "B#r"), 512 per
// document through the 31 client slots (DocClients recycling)
const fresh = process.argv[2] === "fresh";
function body(t) {
  const segs = [];
  for (let i = 0; i < t.length; i += 3) segs.push({ json: t.slice(i, i + 3) });
  return segs;
}
const clients = fx.map((f) => (asBody
  ? eng.createClient("", { segments: body(f.rounds[0].initialText) })
  : eng.createClient(f.rounds[0].initialText)));
let passed = 0;
const failures = [];
const nRounds = Math.max.apply(null, fx.map((f) => f.rounds.length));
for (let r = 0; r < nRounds; r++) {
  fx.forEach((f, d) => {
    if (r >= f.rounds.length) return;
    const got = clients[d].getText();
    if (got === f.rounds[r].initialText) passed++; else failures.push([f.name, r, "initial"]);
    for (const m of f.rounds[r].msgs) {
      const msg = asMsg(m);
      if (fresh) msg.clientId = msg.clientId + "#" + r;
      clients[d].applyMsg(msg);
    }
  });
  fx.forEach((f, d) => {
    if (r >= f.rounds.length) return;
    const got = clients[d].getText();
    const want = f.rounds[r].resultText;
    const a = want.length >> 2, b = a + (want.length >> 1); // a ranged read-out (getText(start, end))
    if (got === want && clients[d].getLength() === got.length && clients[d].getText(a, b) === want.slice(a, b)) {
      passed++;
    } else failures.push([f.name, r, "result"]);
  });
}
const dig = eng.digests();
const hex = [];
for (let i = 0; i < dig.length; i++) hex.push(dig[i].toString(16));
process.stdout.write(JSON.stringify({ passed, failures: failures.slice(0, 5), nFailures: failures.length,
  digests: hex, stats: eng.stats() }) + "\n");
eng.close();
