"use strict";
// GPU test: conflict farms with EVERY client a BatchClient of its own
// ({localClient: true}).  The sets are the ones the reference ran
// (tests/golden/farm_vectors.json.gz, made by tests/golden/make_farm_golden.py
// through oracle/ref_farm.js): each client replays its own events in order —
// its local ops through insertSegmentLocal / removeRangeLocal /
// annotateRangeLocal (the returned op must be the op the reference sent), the
// sequenced messages through applyMsg (its own ones are acks) — and at every
// checkpoint its text, length and per-position properties must be the
// reference client's.  argv "sync": every local op reads the client's length
// first, as the farm's op generator does (a flush + replay per op).  argv[4]:
// the vectors file (default farm_vectors.json.gz; localref_vectors.json.gz adds
// local references "F" / "X" through createLocalReferencePosition /
// removeLocalReferencePosition, their positions checked at every checkpoint).
// Prints one JSON line.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { asMsg } = require("./fixtures");

// MTE_NODE_ADDON=oracle: the same host over the CPU restatement (oracle/mte_shim.c, tests only)
const oracleAddon = process.env.MTE_NODE_ADDON === "oracle"
  ? require(path.join(__dirname, "..", "..", "oracle", "_build", "mte_napi_oracle.node")) : null;
const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden",
  process.argv[4] || "farm_vectors.json.gz"))).toString("utf8")).sets;
const nSets = process.argv[3] && process.argv[3] !== "all" ? Number(process.argv[3]) : sets.length;
const withRefs = sets.some((s) => s.refs);
const sync = process.argv[2] === "sync";

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

// argv[5] "observers": each set's observer alone (the combining-op farms);
// "perset": every client, each set in an engine of its own (a context's
// combining value maps cover the values its documents gave a key)
const observersOnly = process.argv[5] === "observers";
const perSet = process.argv[5] === "perset";
let passed = 0, opsChecked = 0, pending = 0, nDocs = 0;
const failures = [];
const groups = perSet ? Array.from({ length: nSets }, (_, i) => [i]) : [Array.from({ length: nSets }, (_, i) => i)];
for (const group of groups) {
const eng = new MergeTreeEngine(oracleAddon ? { nKeys: 8, addon: oracleAddon } : { nKeys: 8 });
const layout = [];
for (const si of group) {
  sets[si].names.forEach((name, ci) => {
    if (observersOnly && ci !== 0) return;
    layout.push({ si, ci, refs: [], client: eng.createClient(sets[si].initialText,
      { newLengthCalc: !sets[si].legacy, localClient: true, longClientId: name, refs: withRefs }) });
  });
}
const prev = layout.map(() => 0);
const nCp = Math.max.apply(null, group.map((si) => sets[si].checkpoints.length));
for (let j = 0; j < nCp; j++) {
  layout.forEach((L, d) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length) return;
    const done = s.checkpoints[j].done[L.ci];
    for (const ev of s.events[L.ci].slice(prev[d], done)) {
      const kind = ev[0], li = ev[1];
      if (kind === "F") {  // a local reference at position li of the client's view
        L.refs.push(L.client.createLocalReferencePosition(li, 0, ev[2]));
        continue;
      }
      if (kind === "X") {
        L.client.removeLocalReferencePosition(L.refs[li]);
        L.refs[li] = null;
        continue;
      }
      if (kind === "R") {  // the op made locally, then rolled back (Client.rollback)
        if (sync) L.client.getLength();
        const o = li;
        const op = o.type === 0 ? L.client.insertSegmentLocal(o.pos1, o.seg)
          : (o.type === 1 ? L.client.removeRangeLocal(o.pos1, o.pos2) : L.client.annotateRangeLocal(o.pos1, o.pos2, o.props));
        L.client.rollback(op);
        opsChecked++;
        continue;
      }
      const m = asMsg(s.log[li]);
      if (kind === "A") {
        L.client.applyMsg(m);
        continue;
      }
      if (sync) L.client.getLength();
      const o = m.contents;
      let op;
      if (o.type === 0) op = L.client.insertSegmentLocal(o.pos1, o.seg);
      else if (o.type === 1) op = L.client.removeRangeLocal(o.pos1, o.pos2);
      else if (o.relativePos1 && o.combiningOp && o.combiningOp.name === "consensus") {
        op = L.client.annotateMarkerNotifyConsensus(o.relativePos1.id, o.props, () => {});
      } else if (o.relativePos1 || o.relativePos2) op = L.client.applyLocalOp(o);
      else op = L.client.annotateRangeLocal(o.pos1, o.pos2, o.props, o.combiningOp);
      if (JSON.stringify(sortKeys(op)) !== JSON.stringify(sortKeys(o))) failures.push([L.si, L.ci, j, "op", op, o]);
      opsChecked++;
    }
    prev[d] = done;
  });
  layout.forEach((L) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length) return;
    const want = s.checkpoints[j].states[L.ci];
    const got = { text: L.client.getText(), length: L.client.getLength(), props: propRuns(L.client) };
    if (want.refs) got.refs = L.refs.map((r) => (r === null ? null : L.client.localReferencePositionToPosition(r)));
    if (got.text === want.text && got.length === want.length &&
        JSON.stringify(got.props) === JSON.stringify(want.props) &&
        JSON.stringify(got.refs) === JSON.stringify(want.refs)) passed++;
    else failures.push([L.si, L.ci, j, "state"]);
  });
}
pending += layout.reduce((a, L) => a + L.client.getPendingCount(), 0);
nDocs += layout.length;
eng.close();
}
process.stdout.write(JSON.stringify({ passed, opsChecked, pending, failures: failures.slice(0, 5),
  nFailures: failures.length, docs: nDocs }) + "\n");
