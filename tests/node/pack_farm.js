"use strict";
// CPU test helper: packs the reference farm vectors (tests/golden/
// farm_vectors.json.gz) — every client a local-client document, its local ops
// and sequenced messages (acks included) in its own order, one batch per
// checkpoint — with the JS host packer and prints one JSON line per batch
// (base64 buffers) for byte comparison with fluidframework_amd/packing.py.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const packing = require("../../fluidframework_amd/node/packing");
const { asMsg } = require("./fixtures");

// argv: the vectors file (farm_vectors.json.gz, reconnect_vectors.json.gz: ops
// held offline "H" and regeneratePendingOp "G" as MTE_OP_REGEN records, or
// localref_vectors.json.gz: local references "F" / "X" as MTE_OP_REF records)
const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden",
  process.argv[2] || "farm_vectors.json.gz"))).toString("utf8")).sets;
const interner = new packing.Interner(8);
const layout = [];
// argv[3] "observers": each set's observer alone (the combining-op farms)
const observers = process.argv[3] === "observers";
sets.forEach((s, si) => s.names.forEach((name, ci) => {
  if (!observers || ci === 0) layout.push([si, ci, new packing.DocClients(name, 0, true)]);
}));
const prev = layout.map(() => 0);
const refSlots = layout.map(() => []);
const nCp = Math.max.apply(null, sets.map((s) => s.checkpoints.length));
const b64 = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString("base64");
for (let j = 0; j < nCp; j++) {
  const bb = new packing.BatchBuilder(layout.length, interner);
  layout.forEach(([si, ci, cl], d) => {
    const s = sets[si];
    if (j >= s.checkpoints.length) return;
    const done = s.checkpoints[j].done[ci];
    for (const ev of s.events[ci].slice(prev[d], done)) {
      const kind = ev[0], li = ev[1];
      if (kind === "F") {
        refSlots[d].push(bb.addRef(d, cl, li, ev[2]));
        continue;
      }
      if (kind === "X") {
        bb.removeRef(d, cl, refSlots[d][li]);
        continue;
      }
      if (kind === "R") {  // made locally, then rolled back
        bb.addLocal(d, cl, li);
        bb.addRollback(d, cl);
        continue;
      }
      if (kind === "H") {
        bb.addLocal(d, cl, li);
        continue;
      }
      if (kind === "G") {
        bb.addRegen(d, cl);
        continue;
      }
      const m = asMsg(s.log[li]);
      if (kind === "L") bb.addLocal(d, cl, m.contents);
      else bb.addMessage(d, cl, m);
    }
    prev[d] = done;
  });
  const b = bb.build();
  process.stdout.write(JSON.stringify({ offsets: b64(b.offsets), ops: b64(b.ops), text: b64(b.text),
    propsets: b64(b.propsets), props: b64(b.props) }) + "\n");
}
