"use strict";
// SharedString "maintenance" events through the Node host (BatchClient
// .on("maintenance"), createClient {maintenanceEvents: true}): the reference's
// maintenance farms (tests/golden/maint_farm_vectors.json.gz, made by
// tests/golden/make_farm_golden.py --maint through oracle/ref_farm.js) with
// every client a BatchClient -- local ops, rollbacks "R", ops held offline
// "H", regeneratePendingOp "G", local references "F" / "X", the sequenced
// messages (its own are acks).  Each step applies one event of every client,
// then one flush delivers them, so every maintenance event is attributed to
// its client's event index; per client the list [event, type, [[position,
// length], ...]] must be the reference callback list, except the ACKNOWLEDGED
// callbacks of acks of annotates made while every annotate slot was taken
// (DocClients.untrackedAcks; counted as "skipped").
//   argv[2] "oracle": the CPU restatement's addon (oracle/_build); "gpu": libmte.so's
// Prints one JSON line: {clients, equal, skipped, callbacks, first}.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { asMsg } = require("./fixtures");

const root = path.join(__dirname, "..", "..");
const addon = require(process.argv[2] === "gpu" ? path.join(root, "fluidframework_amd", "_lib", "mte_napi.node")
  : path.join(root, "oracle", "_build", "mte_napi_oracle.node"));
const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden",
  "maint_farm_vectors.json.gz"))).toString("utf8")).sets;

const eng = new MergeTreeEngine({ nKeys: 8, addon });
const layout = [];
sets.forEach((s, si) => {
  s.names.forEach((name, ci) => {
    const L = { si, ci, cur: -1, held: [], refs: [], got: [], untracked: new Set(),
      client: eng.createClient(s.initialText, { newLengthCalc: !s.legacy, localClient: true, events: true,
        refs: !!s.refs, maintenanceEvents: true, longClientId: name }) };
    L.client.on("maintenance", (ev) => L.got.push([L.cur, ev.deltaOperation, ev.ranges.map((r) => [r.position, r.length])]));
    layout.push(L);
  });
});
eng.start();
const local = (c, o) => (o.type === 0 ? c.insertSegmentLocal(o.pos1, o.seg)
  : o.type === 1 ? c.removeRangeLocal(o.pos1, o.pos2) : c.annotateRangeLocal(o.pos1, o.pos2, o.props));
const nSteps = Math.max(...layout.map((L) => sets[L.si].events[L.ci].length));
for (let k = 0; k < nSteps; k++) {
  for (const L of layout) {
    const s = sets[L.si];
    const ev = s.events[L.ci][k];
    if (!ev) continue;
    L.cur = k;
    const [kind, li] = ev;
    const c = L.client;
    if (kind === "F") L.refs.push(c.createLocalReferencePosition(li, 0, ev[2]));
    else if (kind === "X") {
      c.removeLocalReferencePosition(L.refs[li]);
      L.refs[li] = null;
    } else if (kind === "R") c.rollback(local(c, li));
    else if (kind === "H") L.held.push(local(c, li));
    else if (kind === "G") c.regeneratePendingOp(L.held.shift());
    else if (kind === "A") {
      const u0 = c.clients.untrackedAcks;
      c.applyMsg(asMsg(s.log[li]));
      if (c.clients.untrackedAcks !== u0) L.untracked.add(k);
    } else local(c, asMsg(s.log[li]).contents);
  }
  eng.flush();
  eng.sync();
}
let equal = 0, skipped = 0, callbacks = 0, first = null;
for (const L of layout) {
  let want = sets[L.si].maint[L.ci];
  callbacks += want.length;
  if (L.untracked.size) {
    const keep = want.filter((x) => !(x[1] === -4 && L.untracked.has(x[0])));
    skipped += want.length - keep.length;
    want = keep;
  }
  const g = JSON.stringify(L.got), w = JSON.stringify(want);
  if (g === w) equal++;
  else if (!first) {
    let q = 0;
    while (q < Math.min(L.got.length, want.length) && JSON.stringify(L.got[q]) === JSON.stringify(want[q])) q++;
    first = [L.si, L.ci, q, L.got.slice(q, q + 2), want.slice(q, q + 2)];
  }
}
process.stdout.write(JSON.stringify({ clients: layout.length, equal, skipped, callbacks, first }) + "\n");
eng.close();
