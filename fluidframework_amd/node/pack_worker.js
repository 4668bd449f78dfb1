"use strict";
// One packing worker of ShardedHost (shards.js): documents [d0, d1) of the
// engine, their DocClients, a BatchBuilder and an Interner of its own.
//   load            source.load(d0, d1, sourceData): the documents' messages
//   pack {upto}     addMessage for messages [cursor .. upto) of each document
//                   (arrival order: message i of every document, then i + 1);
//                   replies with its sizes and the keys / values interned since
//   emit {base, map, sab}  writes its records (by document), text, propsets
//                   and props into the shared batch at its bases, with the
//                   text / propset offsets moved by the bases and the keys /
//                   values renamed to the engine's ids
const { parentPort, workerData } = require("worker_threads");
const { BatchBuilder, DocClients, Interner } = require("./packing");

const { d0, d1, observers, minSeq, nKeys, trees } = workerData;
const n = d1 - d0;
// MTE_DOC_TREE documents take sequenced combining ops (deferred to the host's merge)
const clients = observers.map((o, i) => new DocClients(o, minSeq[i], false, trees && trees[i]));
const interner = new Interner(nKeys);
interner.noteLog = [];
let msgs = null;
const cursor = new Uint32Array(n);
let bb = null;
let sentKeys = 0, sentValues = 1;

function load() {
  const src = require(workerData.source);
  msgs = src.load(d0, d1, workerData.sourceData);
  return { ok: true };
}

function pack(upto) {
  const t0 = process.hrtime.bigint();
  // arrival order: message i of every document, then i + 1
  let lo = Infinity, hi = 0, count = 0;
  const end = new Uint32Array(n);
  for (let d = 0; d < n; d++) {
    end[d] = Math.min(upto === undefined ? msgs[d].length : upto, msgs[d].length);
    if (cursor[d] < lo) lo = cursor[d];
    if (end[d] > hi) hi = end[d];
    if (end[d] > cursor[d]) count += end[d] - cursor[d];
  }
  bb = new BatchBuilder(n, interner, null, count + (count >> 4));
  // a shard's interner sees neither the loaded documents' values nor the other
  // shards', so a sequenced combining op's value map is left to the host's
  // merge (PropTable.addDeferred); a local one has no place in a worker
  bb.noCombining = true;
  bb.shard = true;
  for (let i = lo; i < hi; i++) {
    for (let d = 0; d < n; d++) {
      if (i >= cursor[d] && i < end[d]) {
        bb.addMessage(d, clients[d], msgs[d][i]);
        msgs[d][i] = null;  // packed: a server would not keep it either
      }
    }
  }
  for (let d = 0; d < n; d++) if (end[d] > cursor[d]) cursor[d] = end[d];
  // the keys / values interned since the last pack (the host keeps the rest)
  const keys = interner.keyNames.slice(sentKeys);
  const values = interner.valueJson.slice(sentValues);
  sentKeys = interner.keyNames.length;
  sentValues = interner.valueJson.length;
  // the [key, value index] pairs first noted since, and the deferred combining sets
  const notes = interner.noteLog;
  interner.noteLog = [];
  return { nrec: bb.count, ntext: bb.textUnits, nps: bb.props.sets.length / 2, npe: bb.props.entries.length / 2,
    keys, values, notes, deferred: bb.props.deferred || [], ms: Number(process.hrtime.bigint() - t0) / 1e6 };
}

function emit(base, map, sab) {
  const t0 = process.hrtime.bigint();
  // records sorted by document, text / propset offsets moved by the bases
  const out = new Int32Array(sab.ops, base.rec * 32, bb.count * 8);
  const rel = bb.buildInto(out, base.text, base.ps, map);
  new Uint16Array(sab.text, base.text * 2, bb.textUnits).set(bb.textBuf.subarray(0, bb.textUnits));
  const sets = bb.props.sets, ents = bb.props.entries;
  const ps = new Uint32Array(sab.propsets, base.ps * 8, sets.length);
  for (let i = 0; i < ps.length; i += 2) {
    ps[i] = sets[i] + base.pe;
    ps[i + 1] = sets[i + 1];
  }
  // the deferred combining sets: entries the host wrote past every shard's (map.deferred)
  const df = bb.props.deferred || [];
  for (let q = 0; q < df.length; q++) {
    ps[2 * df[q][0]] = map.deferred[2 * q];
    ps[2 * df[q][0] + 1] = map.deferred[2 * q + 1];
  }
  // keys / values renamed to the engine's ids
  const pe = new Uint32Array(sab.props, base.pe * 8, ents.length);
  for (let i = 0; i < pe.length; i += 2) {
    pe[i] = map.keys[ents[i]];
    pe[i + 1] = map.values[ents[i + 1]];
  }
  const offs = new BigUint64Array(sab.offsets);
  for (let d = 0; d < n; d++) offs[d0 + d] = BigInt(base.rec + rel[d]);
  bb = null;
  return { ok: true, ms: Number(process.hrtime.bigint() - t0) / 1e6 };
}

parentPort.on("message", (m) => {
  try {
    if (m.cmd === "load") parentPort.postMessage(load());
    else if (m.cmd === "pack") parentPort.postMessage(pack(m.upto));
    else if (m.cmd === "emit") parentPort.postMessage(emit(m.base, m.map, m.sab));
    else parentPort.postMessage({ error: "unknown command " + m.cmd });
  } catch (e) {
    parentPort.postMessage({ error: String(e && e.stack ? e.stack : e) });
  }
});
