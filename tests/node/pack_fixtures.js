"use strict";
// CPU test helper: packs every round of the golden fixtures with the JS host
// packer (all documents side by side, one batch per round, as
// tests/fixtures_util.py does) and prints one JSON line per round with the
// base64 of each buffer, for byte comparison with fluidframework_amd/packing.py.
const packing = require("../../fluidframework_amd/node/packing");
const { loadFixtures, asMsg } = require("./fixtures");

const fx = loadFixtures();
const fresh = process.argv[2] === "fresh"; // senders renamed per round ("B" -> "B#r")
const interner = new packing.Interner(8);
const clients = fx.map(() => new packing.DocClients("A"));
const nRounds = Math.max.apply(null, fx.map((f) => f.rounds.length));
const b64 = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString("base64");
for (let r = 0; r < nRounds; r++) {
  const bb = new packing.BatchBuilder(fx.length, interner);
  fx.forEach((f, d) => {
    if (r < f.rounds.length) {
      for (const m of f.rounds[r].msgs) {
        const msg = asMsg(m);
        if (fresh) msg.clientId = msg.clientId + "#" + r;
        bb.addMessage(d, clients[d], msg);
      }
    }
  });
  const b = bb.build();
  process.stdout.write(JSON.stringify({ round: r, offsets: b64(b.offsets), ops: b64(b.ops), text: b64(b.text),
    propsets: b64(b.propsets), props: b64(b.props) }) + "\n");
}
