"use strict";
// Interval-holding documents batch like any other (VERDICT r05 next #1): a
// document whose collection holds intervals queues its merge-tree messages
// until the flush, and the "changeInterval" events its ends raise sliding off
// removed segments come from the engine's MTE_DELTA_SLIDE / MTE_DELTA_REFPOS
// records of that one replay -- the same events, positions, end tree and
// summaries as replaying message by message (each message its own replay,
// which the reference farms pin: tests/test_intervals.py).
//   argv[2] "oracle": both replays on the CPU restatement (oracle/mte_shim.c)
//   argv[2] "gpu":    the batched replay on the engine (libmte.so), the
//                     message-by-message one on the restatement
//   argv[3] documents, argv[4] merge-tree messages per document.
// Prints one JSON line: {runs, docs, messages, events, equal, first}.
const path = require("path");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");

const mode = process.argv[2] || "oracle";
const nDocs = Number(process.argv[3] || 100);
const nMsgs = Number(process.argv[4] || 120);
const root = path.join(__dirname, "..", "..");
const oracleAddon = require(path.join(root, "oracle", "_build", "mte_napi_oracle.node"));
const deviceAddon = mode === "gpu" ? require(path.join(root, "fluidframework_amd", "_lib", "mte_napi.node")) : null;

// mulberry32 (as oracle/ref_farm.js)
function rng(seed) {
  let a = seed >>> 0;
  const next = () => {
    a = (a + 0x6d2b79f5) >>> 0;
    let t = a;
    t = Math.imul(t ^ (t >>> 15), t | 1);
    t ^= t + Math.imul(t ^ (t >>> 7), t | 61);
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
  return { next, int: (lo, hi) => lo + Math.floor(next() * (hi - lo + 1)) };
}

const LABEL = "farm";
const REMOTE = ["B", "C", "D"];

// one document's stream: interval adds by remote clients, then merge-tree
// messages whose refSeq is seq - 1 (every sender up to date), so the
// generator can keep the length the next op's positions must respect
function stream(d) {
  const R = rng(7919 * (d + 1));
  const text = "abcdefghijklmnopqrstuvwxyz0123".slice(0, 20 + R.int(0, 10));
  let len = text.length, seq = 0, msn = 0;
  const msgs = [];
  const msg = (client, contents) => {
    seq++;
    msn = Math.max(msn, seq - 8);
    msgs.push({ clientId: client, sequenceNumber: seq, referenceSequenceNumber: seq - 1,
      minimumSequenceNumber: Math.min(msn, seq - 1), type: "op", contents });
  };
  const nIv = R.int(4, 8);
  for (let i = 0; i < nIv; i++) {
    const a = R.int(0, len - 1), b = R.int(a, Math.min(len - 1, a + 6));
    msg(REMOTE[R.int(0, 2)], { key: LABEL, type: "act", value: { opName: "add", value: { start: a, end: b,
      intervalType: 2, sequenceNumber: seq, properties: { intervalId: `iv${d}-${i}` } } } });
  }
  const first = msgs.length;
  const one = () => {
    if (len < 8 || R.next() < 0.45) {
      const n = R.int(1, 3);
      const op = { type: 0, pos1: R.int(0, len), seg: "xyz".slice(0, n) };
      len += n;
      return op;
    }
    const a = R.int(0, len - 1), b = Math.min(len, a + R.int(1, 4));
    len -= b - a;
    return { type: 1, pos1: a, pos2: b };
  };
  for (let i = 0; i < nMsgs; i++) {
    const c = REMOTE[R.int(0, 2)];
    if (R.next() < 0.25) {
      const ops = [];
      for (let k = R.int(2, 3); k > 0; k--) ops.push(one());
      msg(c, { type: 3, ops });
    } else {
      msg(c, one());
    }
  }
  return { text, intervalMsgs: msgs.slice(0, first), mtMsgs: msgs.slice(first) };
}

// the engine with its addon's run() counted
function engine(addon) {
  const counted = Object.assign({}, addon);
  const e = new MergeTreeEngine({ nKeys: 4, addon: counted });
  e.runs = 0;
  counted.run = (ctx) => {
    e.runs++;
    return addon.run(ctx);
  };
  return e;
}

function setup(addon, streams) {
  const e = engine(addon);
  const docs = streams.map((s) => {
    const c = e.createClient(s.text, { newLengthCalc: true, localClient: true, refs: true, events: true,
      longClientId: "A" });
    const coll = c.getIntervalCollection(LABEL);
    const ev = [];
    const pos = (r) => c.localReferencePositionToPosition(r);
    coll.on("changeInterval", (x, prev, local, op) => ev.push(["change", x.getIntervalId(), local, !!op,
      pos(prev.start), pos(prev.end), pos(x.start), pos(x.end)]));
    coll.on("addInterval", (x, local, op) => ev.push(["add", x.getIntervalId(), local, !!op]));
    return { c, coll, ev };
  });
  e.setEventCapacity(64);
  e.start();
  // the intervals (each interval op settles its document first)
  streams.forEach((s, i) => { for (const m of s.intervalMsgs) docs[i].c.applyMsg(m); });
  return { e, docs };
}

function state(x) {
  const n = x.c.getLength();
  const ids = (v) => (v ? v.getIntervalId() : null);
  const q = [];
  for (let p = 0; p <= n; p++) q.push([ids(x.coll.previousInterval(p)), ids(x.coll.nextInterval(p))]);
  return { text: x.c.getText(), ev: x.ev, intervals: Array.from(x.coll).map((v) => [v.getIntervalId(), ...v.positions()]),
    summary: x.coll.serializeInternal(), prevNext: q,
    overlap: [0, 3, 7].map((a) => x.coll.findOverlappingIntervals(a, a + 4).map(ids)) };
}

const streams = [];
for (let d = 0; d < nDocs; d++) streams.push(stream(d));

// batched: every merge-tree message of every document queued, one flush
const A = setup(deviceAddon || oracleAddon, streams);
const runs0 = A.e.runs;
streams.forEach((s, i) => { for (const m of s.mtMsgs) A.docs[i].c.applyMsg(m); });
A.e.flush();
A.e.sync();
const runs = A.e.runs - runs0;
const got = A.docs.map(state);

// message by message, on the restatement
const B = setup(oracleAddon, streams);
const n = Math.max(...streams.map((s) => s.mtMsgs.length));
for (let k = 0; k < n; k++) {
  streams.forEach((s, i) => {
    if (k >= s.mtMsgs.length) return;
    B.docs[i].c.applyMsg(s.mtMsgs[k]);
    B.e.flush();
    B.e.sync();
  });
}
const want = B.docs.map(state);

let equal = 0, first = null, events = 0;
for (let d = 0; d < nDocs; d++) {
  events += want[d].ev.filter((x) => x[0] === "change").length;
  const g = JSON.stringify(got[d]), w = JSON.stringify(want[d]);
  if (g === w) equal++;
  else if (!first) first = [d, g.slice(0, 600), w.slice(0, 600)];
}
process.stdout.write(JSON.stringify({ runs, docs: nDocs, messages: streams.reduce((a, s) => a + s.mtMsgs.length, 0),
  events, equal, first }) + "\n");
A.e.close();
B.e.close();
