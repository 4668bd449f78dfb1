"use strict";
// Interval-collection farms (tests/golden/interval_vectors.json.gz, made by
// tests/golden/make_interval_golden.py through oracle/ref_interval_farm.js)
// replayed through the Node host: every client a BatchClient
// ({localClient, refs}) with the label's IntervalCollection
// (fluidframework_amd/node/intervals.js).  Each client replays its own events
// in order: "L" a local merge-tree op, "I" a local interval op (re-made through
// add / change / changeProperties / removeIntervalById; the op it emits must be
// the one the reference sent), "A" a sequenced message (merge-tree ops through
// applyMsg, interval ops through the collection's process).
//   argv[2] "gpu":  on the engine; at every checkpoint each client's text and
//                   intervals (id, start, end, properties) must equal the
//                   reference client's.  Prints one JSON line.
//   argv[2] "pack": no device (a recording addon): prints one JSON line per
//                   checkpoint with the batch (base64) and, per client, its
//                   intervals as [id, start slot, end slot, properties], for
//                   tests/test_intervals.py to replay on the restatement.
//   argv[2] "ext":  as "gpu" on interval_ext_vectors.json.gz (argv[4]), and at
//                   every checkpoint also the collection's events since the
//                   last one (those a merge-tree op raises excepted: ends that
//                   slid, see intervals.js), its iteration order,
//                   serializeInternal() and the recorded queries; then each
//                   set's final summary loads into a fresh client whose
//                   intervals must equal the reference's.
//   argv[2] "reconnect": as "ext" on interval_reconnect_vectors.json.gz, whose
//                   clients also go offline: "H" / "J" a merge-tree / interval op
//                   made offline (held), "G" / "K" its re-send on reconnection --
//                   BatchClient.regeneratePendingOp / the collection's
//                   rebaseLocalInterval with the op's localSeq metadata -- which
//                   must equal the op the reference re-sent.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");

const mode = process.argv[2] || "gpu";
const rec = mode === "reconnect";
const ext = mode === "ext" || rec;
const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden",
  process.argv[4] || (rec ? "interval_reconnect_vectors.json.gz"
    : ext ? "interval_ext_vectors.json.gz" : "interval_vectors.json.gz")))).toString("utf8")).sets
  // "reconnect-leaf": only the farms in which every localSeq view the
  // reference computed equals its own leaf rule (oracle/ref_interval_farm.js
  // leafViews) -- the engine restates the block-level rule, so all of them pass
  .filter((s) => process.argv[5] !== "leaf" || (s.leafViews && s.leafViews.differ === 0));
const nSets = process.argv[3] && process.argv[3] !== "all" ? Number(process.argv[3]) : sets.length;
const LABEL = "farm";

function sortKeys(v) {
  if (v && typeof v === "object" && !Array.isArray(v)) {
    const o = {};
    for (const k of Object.keys(v).sort()) o[k] = sortKeys(v[k]);
    return o;
  }
  return v;
}
const clone = (v) => JSON.parse(JSON.stringify(v));
const b64 = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString("base64");

// pack mode: the N-API surface the engine uses, recording the submitted batches
// (several per checkpoint: the end tree's comparisons read reference order,
// which flushes; here every reference reads as the same unit)
let batches = [];
const recorder = {
  create() { return {}; }, destroy() {}, loadDocs() {}, loadSegments() {},
  submit(ctx, offsets, ops, text, propsets, props) {
    batches.push({ offsets: b64(offsets), ops: b64(ops), text: b64(text), propsets: b64(propsets), props: b64(props) });
  },
  run() {}, sync() {}, readDeltas() { return new Uint32Array(0); },
  readRefOrder(ctx, doc, n) { return new Int32Array(n); },
};

// MTE_NODE_ADDON=oracle: the same host over the CPU restatement (oracle/mte_shim.c, tests only)
const oracleAddon = process.env.MTE_NODE_ADDON === "oracle"
  ? require(path.join(__dirname, "..", "..", "oracle", "_build", "mte_napi_oracle.node")) : null;
const eng = new MergeTreeEngine(mode === "pack" ? { nKeys: 8, addon: recorder }
  : (oracleAddon ? { nKeys: 8, addon: oracleAddon } : { nKeys: 8 }));
const layout = [];
for (let si = 0; si < nSets; si++) {
  sets[si].names.forEach((name, ci) => {
    const L = { si, ci, sent: null };
    L.client = eng.createClient(sets[si].initialText, { newLengthCalc: true, localClient: true, refs: true,
      longClientId: name, events: ext });
    L.held = [];
    L.coll = L.client.getIntervalCollection(LABEL, { emit(opName, _p, value, meta) { L.sent = { opName, value, meta }; } });
    if (ext) {
      L.ev = [];
      const pos = (r) => L.client.localReferencePositionToPosition(r);
      L.coll.on("addInterval", (x, local, op) => L.ev.push(["add", x.getIntervalId(), local, !!op, false]));
      L.coll.on("deleteInterval", (x, local, op) => L.ev.push(["delete", x.getIntervalId(), local, !!op, false]));
      // mt: raised inside a merge-tree op (an end sliding off a removed segment)
      L.coll.on("changeInterval", (x, prev, local, op) => L.ev.push(["change", x.getIntervalId(), local, !!op,
        pos(prev.start), pos(prev.end), pos(x.start), pos(x.end), !!(L.mt || L.coll.inMergeTreeOp)]));
      L.coll.on("propertyChanged", (x, deltas, local, op) => L.ev.push(["props", x.getIntervalId(), local, !!op,
        sortKeys(clone(deltas)), false]));
    }
    // MTE_FARM_TRACE="set,client": that client's steps, slide records and
    // events on stderr, with the reference's events at each checkpoint
    if (process.env.MTE_FARM_TRACE === `${si},${ci}`) {
      L.trace = true;
      L.client.traceEnd = true;
      L.client.onSlideRecords = (sl) => process.stderr.write("  slides " + JSON.stringify(sl) + "\n");
    }
    layout.push(L);
  });
}
// ext: a loader client per set, of its final text, for the summary load below
const loaders = [];
if (ext) {
  for (let si = 0; si < nSets; si++) {
    const s = sets[si];
    const last = s.checkpoints[s.checkpoints.length - 1].states[0];
    loaders.push(eng.createClient(last.text, { newLengthCalc: true, localClient: true, refs: true,
      longClientId: "loader" + si }));
  }
}
if (ext) eng.setEventCapacity(64);  // a remove can slide many interval ends (MTE_DELTA_SLIDE)
eng.start();
const prev = layout.map(() => 0);
const failures = [];
const extFail = {}, extFirst = {}, prevNext = { n: 0, equal: 0 };
const mtEvents = { n: 0, equal: 0, first: null };  // checkpoints whose whole event list (mid-op ones included) is the reference's
const regens = [];  // [got, want, original] of each regenerated merge-tree op
let orderOff = 0;  // checkpoints whose order differs only among intervals with an end off the string
let passed = 0, opsChecked = 0;
const nCp = Math.max.apply(null, sets.slice(0, nSets).map((s) => s.checkpoints.length));
for (let j = 0; j < nCp; j++) {
  layout.forEach((L, d) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length) return;
    const done = s.checkpoints[j].done[L.ci];
    if (L.broken) return;
    for (const [kind, li] of s.events[L.ci].slice(prev[d], done)) {
     try {
      const m = typeof li === "number" ? s.log[li] : [null, 0, 0, 0, kind === "H" ? "op" : "iv", li];
      if (L.trace) {
        process.stderr.write(`${kind} ${JSON.stringify(m)}\n`);
        if (L.ev) process.stderr.write("  ev-so-far " + L.ev.length + "\n");
      }
      const msg = { clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
        type: "op", contents: m[5] };
      if (kind === "A") {
        if (m[4] === "op") {
          L.mt = true;
          try {
            L.client.applyMsg(msg);
          } finally {
            L.mt = false;
          }
        }
        else L.coll.process(m[5].opName, m[5].value === undefined ? undefined : clone(m[5].value),
          m[0] === s.names[L.ci], msg);
        continue;
      }
      if (kind === "L" || kind === "H") {
        const o = m[5];
        let made;
        if (o.type === 0) made = L.client.insertSegmentLocal(o.pos1, o.seg);
        else if (o.type === 1) made = L.client.removeRangeLocal(o.pos1, o.pos2);
        else made = L.client.annotateRangeLocal(o.pos1, o.pos2, o.props);
        if (kind === "H") L.held.push({ op: made });
        continue;
      }
      if (kind === "G" || kind === "K") {
        // reconnection: the held ops re-sent in order
        const h = L.held.shift();
        const got = kind === "G" ? (h && h.op ? L.client.regeneratePendingOp(h.op) : null)
          : (h && h.iv ? L.coll.rebaseOp(h.iv.opName, h.iv.value, h.iv.meta) : null);
        let want = kind === "G" ? m[5] : m[5].value;
        if (kind === "K" && m[5].opName === "delete" && want) {  // a delete's positions are informational
          want = clone(want);
          delete want.start;
          delete want.end;
        }
        // regenerated ops: compared in Python (fixtures_util.canon_regen)
        if (kind === "G") regens.push([got, want, h && h.op]);
        else if (JSON.stringify(sortKeys(got === undefined ? null : clone(got))) !==
            JSON.stringify(sortKeys(want === undefined ? null : want))) {
          failures.push([L.si, L.ci, j, "rebase", got, want]);
        }
        opsChecked++;
        continue;
      }
      // "I" / "J": the client's own interval op, re-made through the collection API
      const { opName, value } = m[5];
      const id = value.properties && value.properties.intervalId;
      L.sent = null;
      if (opName === "add") {
        L.coll.add(value.start, value.end, value.intervalType, value.properties);
      } else if (opName === "delete") {
        L.coll.removeIntervalById(id);
      } else if (value.start !== undefined || value.end !== undefined) {
        L.coll.change(id, value.start, value.end);
      } else {
        const props = Object.assign({}, value.properties);
        delete props.intervalId;
        L.coll.changeProperties(id, props);
      }
      // the op the reference sent (a delete's positions are informational)
      const want = clone(value), got = L.sent ? clone(L.sent.value) : null;
      if (opName === "delete" && got) {
        delete want.start;
        delete want.end;
      }
      if (!L.sent || L.sent.opName !== opName || JSON.stringify(sortKeys(got)) !== JSON.stringify(sortKeys(want))) {
        failures.push([L.si, L.ci, j, "op", L.sent, m[5]]);
      }
      if (kind === "J" && L.sent) L.held.push({ iv: L.sent });
      opsChecked++;
     } catch (e) {  // the client stops here; the failure says where
      failures.push([L.si, L.ci, j, "throw", kind, String(e && e.message)]);
      L.broken = true;
      return;
     }
    }
    prev[d] = done;
  });
  if (mode === "pack") {
    eng.flush();
    const states = layout.map((L) => {
      if (j >= sets[L.si].checkpoints.length) return null;
      const ivs = Array.from(L.coll.byId.values()).map((x) => [x.getIntervalId(), x.start.slot, x.end.slot,
        sortKeys(x.properties)]);
      ivs.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
      return { intervals: ivs, nRefs: L.client.clients.refNext };
    });
    process.stdout.write(JSON.stringify({ batches, states }) + "\n");
    batches = [];
    continue;
  }
  layout.forEach((L) => {
    const s = sets[L.si];
    if (j >= s.checkpoints.length || L.broken) return;
    const want = s.checkpoints[j].states[L.ci];
    const ivs = Array.from(L.coll.byId.values()).map((x) => {
      const [a, b] = x.positions();
      return [x.getIntervalId(), a, b, sortKeys(x.properties)];
    });
    ivs.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
    const text = L.client.getText();
    let ok = text === want.text && JSON.stringify(ivs) === JSON.stringify(want.intervals);
    if (!ok) failures.push([L.si, L.ci, j, "state", ivs.slice(0, 3), want.intervals.slice(0, 3)]);
    if (L.trace) {
      process.stderr.write(`== checkpoint ${j}\n got  ${JSON.stringify(L.ev)}\n want ${JSON.stringify(want.events)}\n`);
      process.stderr.write(` intervals ${JSON.stringify(want.intervals)}\n`);
    }
    if (ext && ok) {
      const ids = (xs) => xs.map((x) => x.getIntervalId());
      // the events a merge-tree op raised (ends sliding, last field true) are
      // compared apart (mtEvents): the rest must be exact
      const noMt = (evs) => evs.filter((e) => !e[e.length - 1]);
      const evWant = noMt(want.events);
      mtEvents.n++;
      if (JSON.stringify(sortKeys(L.ev)) === JSON.stringify(sortKeys(want.events))) mtEvents.equal++;
      else if (!mtEvents.first) mtEvents.first = [L.si, L.ci, j];
      const got = { events: noMt(L.ev), order: ids(Array.from(L.coll)), summary: clone(L.coll.serializeInternal()),
        queries: want.queries.map(([a, b]) => [a, b, ids(L.coll.findOverlappingIntervals(a, b)),
          ids([L.coll.previousInterval(a)].filter(Boolean)), ids([L.coll.nextInterval(a)].filter(Boolean)),
          ids(Array.from(L.coll.CreateForwardIteratorWithStartPosition(a))),
          ids(Array.from(L.coll.CreateBackwardIteratorWithStartPosition(a))),
          ids(Array.from(L.coll.CreateForwardIteratorWithEndPosition(b))),
          ids(Array.from(L.coll.CreateBackwardIteratorWithEndPosition(b)))]) };
      // previousInterval / nextInterval (columns 3, 4) are compared apart: the
      // reference's end tree keeps one node per end and can lose an interval
      // sharing its end with one removed (rbTree put / remove by key)
      const strip = (qs) => qs.map((q) => q.filter((_, i) => i !== 3 && i !== 4));
      for (const q of got.queries.keys()) {
        const gq = got.queries[q], wq = want.queries[q];
        prevNext.n += 2;
        const eq = (JSON.stringify(gq[3]) === JSON.stringify(wq[3]) ? 1 : 0) +
          (JSON.stringify(gq[4]) === JSON.stringify(wq[4]) ? 1 : 0);
        prevNext.equal += eq;
        if (eq < 2 && !prevNext.first) prevNext.first = [L.si, L.ci, j, q, gq.slice(0, 5), wq.slice(0, 5)];
      }
      let offOrder = false;
      for (const k of ["events", "order", "summary", "queries"]) {
        const w = k === "events" ? evWant : (k === "queries" ? strip(want[k]) : want[k]);
        if (k === "queries") got[k] = strip(got[k]);
        if (k === "order" && JSON.stringify(got[k]) !== JSON.stringify(w)) {
          // an end that slid off the string on a segment the zamboni has since
          // unlinked: the reference still compares that segment's ordinal
          // (compareReferencePositions, referencePositions.ts:81-89), which no
          // held segment carries any more -- the order among such intervals is
          // counted apart when the rest agrees
          const off = new Set(want.intervals.filter((x) => x[1] < 0 || x[2] < 0).map((x) => x[0]));
          const rest = (xs) => JSON.stringify(xs.filter((x) => !off.has(x)));
          if (rest(got[k]) === rest(w)) {
            orderOff++;
            offOrder = true;
            continue;
          }
        }
        if (k === "summary" && offOrder) {  // the same intervals, listed in that order: compared as sets
          const bySet = (x) => JSON.stringify(Object.assign({}, sortKeys(x), {
            intervals: x.intervals.map((y) => JSON.stringify(sortKeys(y))).sort() }));
          if (bySet(got[k]) === bySet(w)) continue;
        }
        if (JSON.stringify(sortKeys(got[k])) !== JSON.stringify(sortKeys(w))) {
          ok = false;
          extFail[k] = (extFail[k] || 0) + 1;
          if (!extFirst[k]) {
            const g = Array.isArray(got[k]) ? got[k] : [got[k]], ww = Array.isArray(w) ? w : [w];
            let d = 0;
            while (d < Math.min(g.length, ww.length) && JSON.stringify(sortKeys(g[d])) === JSON.stringify(sortKeys(ww[d]))) d++;
            extFirst[k] = [L.si, L.ci, j, d, g.length, ww.length, g.slice(d, d + 3), ww.slice(d, d + 3)];
          }
          failures.push([L.si, L.ci, j, k, got[k], w]);
          break;
        }
      }
      L.ev = [];
    }
    if (ok) passed++;
  });
}
let loaded = 0, unloadable = 0;
if (ext) {
  // each set's observer summary (serializeInternal at the last checkpoint)
  // loaded into a fresh client of the same text: the reference's intervals
  for (let si = 0; si < nSets; si++) {
    const s = sets[si];
    const last = s.checkpoints[s.checkpoints.length - 1].states[0];
    // an end outside the text (detached) makes the reference's load throw
    // ("Non-transient references need segment", :629-636): those sets load nothing
    if (last.intervals.some((x) => x[1] < 0 || x[2] < 0 || x[1] >= last.text.length || x[2] >= last.text.length)) {
      unloadable++;
      continue;
    }
    const c = loaders[si];
    const coll = c.getIntervalCollection(LABEL, null, last.summary);
    const ivs = Array.from(coll.byId.values()).map((x) => {
      const [a, b] = x.positions();
      return [x.getIntervalId(), a, b, sortKeys(x.properties)];
    });
    ivs.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
    const gotSum = JSON.stringify(sortKeys(clone(coll.serializeInternal())));
    // serialize() stamps each interval with the serializing client's current
    // seq (intervalCollection.ts:456-470): the fresh loader's, not the observer's
    const want = clone(last.summary);
    for (const x of want.intervals) x[2] = c.getCurrentSeq();
    const wantSum = JSON.stringify(sortKeys(want));
    if (JSON.stringify(ivs) === JSON.stringify(last.intervals) && gotSum === wantSum) loaded++;
    else {
      // the first differing interval, or the summaries from their first difference
      let d = 0;
      while (d < ivs.length && JSON.stringify(ivs[d]) === JSON.stringify(last.intervals[d])) d++;
      let e = 0;
      while (e < gotSum.length && gotSum[e] === wantSum[e]) e++;
      failures.push([si, "load", d, ivs.length, last.intervals.length, ivs.slice(d, d + 2),
        last.intervals.slice(d, d + 2), gotSum.slice(Math.max(0, e - 80), e + 120),
        wantSum.slice(Math.max(0, e - 80), e + 120)]);
    }
  }
}
if (mode !== "pack") {
  const endRebuilds = layout.reduce((a, L) => a + (L.coll.endRebuilds || 0), 0);
  process.stdout.write(JSON.stringify({ passed, opsChecked, loaded, unloadable, extFail, extFirst, prevNext, mtEvents, regens, orderOff,
    endRebuilds,
    failures: failures.slice(0, 16),
    nFailures: failures.length, docs: layout.length }) + "\n");
} else {
  process.stdout.write(JSON.stringify({ done: true, opsChecked, failures: failures.slice(0, 16),
    nFailures: failures.length }) + "\n");
}
eng.close();
