"use strict";
// GPU test: the reference's reconnect farms (tests/golden/reconnect_vectors.json.gz,
// made by tests/golden/make_reconnect_golden.py through oracle/ref_farm.js) with
// every client a BatchClient ({localClient: true, events: true}): local ops,
// ops held while offline ("H"), BatchClient.regeneratePendingOp on reconnect
// ("G": the regenerated op is printed beside the reference's for the Python
// side to compare, tests/test_reconnect.py) and the sequenced messages (the
// reference's regenerated ones among them; its own are acks).  At every
// checkpoint each client's text, length and per-position properties are
// compared with the reference client's.  argv: number of sets ("all"), the
// vectors file (default reconnect_vectors.json.gz; relpos_farm_vectors.json.gz
// adds ops through relative positions -- Client.annotateMarker and the op path
// for removes / inserts -- rollbacks "R" and legacy-calc sets).  Prints one
// JSON line.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { asMsg } = require("./fixtures");

const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden",
  process.argv[3] || "reconnect_vectors.json.gz"))).toString("utf8")).sets;
const nSets = process.argv[2] && process.argv[2] !== "all" ? Number(process.argv[2]) : sets.length;

function sortKeys(v) {
  if (v && typeof v === "object" && !Array.isArray(v)) {
    const o = {};
    for (const k of Object.keys(v).sort()) o[k] = sortKeys(v[k]);
    return o;
  }
  return v;
}
function propRuns(c) {
  const runs = [];
  let cur = null, start = 0;
  const n = c.getLength();
  for (let p = 0; p < n; p++) {
    const pr = c.getPropertiesAtPosition(p);
    const key = pr && Object.keys(pr).length ? JSON.stringify(sortKeys(pr)) : "";
    if (key !== cur) {
      if (cur) runs.push([start, p, JSON.parse(cur)]);
      cur = key;
      start = p;
    }
  }
  if (cur) runs.push([start, n, JSON.parse(cur)]);
  return runs;
}

const eng = new MergeTreeEngine({ nKeys: 8 });
const layout = [];
for (let si = 0; si < nSets; si++) {
  sets[si].names.forEach((name, ci) => {
    layout.push({ si, ci, held: [], client: eng.createClient(sets[si].initialText,
      { newLengthCalc: !sets[si].legacy, localClient: true, events: true, longClientId: name }) });
  });
}
const isMarkerAnnotate = (o) => o.type === 2 && o.relativePos1 && o.relativePos2 && !("pos1" in o) &&
  o.relativePos1.before === true && o.relativePos1.offset === undefined && !o.relativePos2.before &&
  o.relativePos2.offset === undefined && o.relativePos1.id === o.relativePos2.id;
const local = (c, o) => {
  if (isMarkerAnnotate(o)) return c.annotateMarker(o.relativePos1.id, o.props);
  if (o.relativePos1 || o.relativePos2) return c.applyLocalOp(o);
  return o.type === 0 ? c.insertSegmentLocal(o.pos1, o.seg)
    : o.type === 1 ? c.removeRangeLocal(o.pos1, o.pos2) : c.annotateRangeLocal(o.pos1, o.pos2, o.props);
};
const ops = [];  // [set, client, made, the reference's]
const states = [];  // [set, client, checkpoint, ok]
const regens = [];  // [set, client, got, want, original]
const prev = layout.map(() => 0);
const nCp = Math.max.apply(null, sets.slice(0, nSets).map((s) => s.checkpoints.length));
for (let j = 0; j < nCp; j++) {
  layout.forEach((L, d) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length) return;
    const done = s.checkpoints[j].done[L.ci];
    for (const [kind, li] of s.events[L.ci].slice(prev[d], done)) {
      if (kind === "H") {
        L.held.push(local(L.client, li));
      } else if (kind === "R") {  // made locally, then rolled back (Client.rollback)
        L.client.rollback(local(L.client, li));
      } else if (kind === "G") {
        const orig = L.held.shift();
        regens.push([L.si, L.ci, L.client.regeneratePendingOp(orig), s.log[li][5], orig]);
      } else if (kind === "A") {
        L.client.applyMsg(asMsg(s.log[li]));
      } else {
        const o = asMsg(s.log[li]).contents;
        ops.push([L.si, L.ci, local(L.client, o), o]);
      }
    }
    prev[d] = done;
  });
  layout.forEach((L) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length) return;
    const want = s.checkpoints[j].states[L.ci];
    const got = { text: L.client.getText(), length: L.client.getLength(), props: propRuns(L.client) };
    states.push([s.seed, L.ci, j, got.text === want.text && got.length === want.length &&
      JSON.stringify(got.props) === JSON.stringify(want.props)]);
  });
}
const pending = layout.reduce((a, L) => a + L.client.getPendingCount(), 0);
const badOps = ops.filter((x) => JSON.stringify(sortKeys(x[2])) !== JSON.stringify(sortKeys(x[3])));
process.stdout.write(JSON.stringify({ states, regens: regens.map((r) => [sets[r[0]].seed, r[1], r[2], r[3], r[4]]),
  pending, docs: layout.length, opsChecked: ops.length, badOps: badOps.slice(0, 3), nBadOps: badOps.length }) + "\n");
eng.close();
