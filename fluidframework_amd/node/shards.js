"use strict";
// Parallel host packing: one worker thread per core, each owning a contiguous
// shard of the documents — their DocClients, a BatchBuilder and a property
// interner of its own — turns its documents' sequenced messages into op
// records, and writes them straight into the shared batch the engine uploads
// (mte_submit).  The reference applies each document's messages in that
// document's own Client (client.ts:918-935); documents never interact, so the
// shards pack independently and the only cross-shard step is the merge of
// the interned property keys / values into the engine's ids.
//
//   const host = new ShardedHost(engine, { workers: 16, source: "/path/source.js" });
//   await host.start();            // workers load their documents' messages (source.load)
//   const n = await host.flush(i); // pack messages [.. i) of every document, submit, replay
//
// source.js exports load(d0, d1, workerData) -> per-document arrays of
// ISequencedDocumentMessage objects (in a server: the documents' delta streams).
const path = require("path");
const { Worker } = require("worker_threads");
const { PropTable } = require("./packing");

const OP_BYTES = 32;

class ShardedHost {
  /**
   * @param engine  a started MergeTreeEngine whose documents were created (createClient) in order
   * @param options {workers, source, sourceData, observerIds?: string[]}
   */
  constructor(engine, options) {
    this.engine = engine;
    const nDocs = engine.docs.length;
    const nw = Math.max(1, Math.min(options.workers || 1, nDocs));
    this.ranges = [];
    for (let w = 0; w < nw; w++) this.ranges.push([Math.floor((nDocs * w) / nw), Math.floor((nDocs * (w + 1)) / nw)]);
    this.options = options;
    this.workers = [];
  }

  _call(w, msg) {
    return new Promise((resolve, reject) => {
      const W = this.workers[w];
      W.once("message", (m) => (m && m.error ? reject(new Error(m.error)) : resolve(m)));
      W.postMessage(msg);
    });
  }

  async start() {
    this.engine.start();
    const file = path.join(__dirname, "pack_worker.js");
    const obs = this.engine.clients.map((c) => c.longClientId);
    const minSeq = this.engine.docs.map((d) => d.minSeq || 0);
    this.workers = this.ranges.map(([d0, d1]) => new Worker(file, {
      workerData: { d0, d1, source: this.options.source, sourceData: this.options.sourceData,
        observers: obs.slice(d0, d1), minSeq: minSeq.slice(d0, d1), nKeys: this.engine.nKeys,
        trees: this.engine.docs.slice(d0, d1).map((d) => !!d.tree) },
    }));
    await Promise.all(this.workers.map((_, w) => this._call(w, { cmd: "load" })));
  }

  /** Pack messages [from the last flush .. upto) of every document in the
   *  workers, merge their interned keys / values into the engine's ids, have
   *  the workers write the batch into shared memory, then submit + run it.
   *  Returns the number of records. */
  async flush(upto) {
    return this.flushParts([upto]);
  }

  /** flush(uptos[0]), flush(uptos[1]), ... pipelined: the workers pack part
   *  i + 1 while the host thread submits part i (mte_submit's upload runs on
   *  the host thread, the packing on the workers) and the device replays it.
   *  Returns the number of records of all parts. */
  async flushParts(uptos) {
    const eng = this.engine;
    const t = this.timing || (this.timing = { pack_ms: 0, pack_max_worker_ms: 0, merge_ms: 0, emit_ms: 0, submit_ms: 0 });
    const packAll = (upto) => Promise.all(this.workers.map((_, w) => this._call(w, { cmd: "pack", upto })));
    let total = 0;
    let tp = process.hrtime.bigint();
    let next = packAll(uptos[0]);
    for (let i = 0; i < uptos.length; i++) {
      const parts = await next;
      const tm = process.hrtime.bigint();
      t.pack_ms += Number(tm - tp) / 1e6;
      t.pack_max_worker_ms += Math.max(...parts.map((p) => p.ms));
      const { maps, bases, nrec, ntext, nps, npe, comb } = this._merge(parts);
      const nDocs = eng.docs.length;
      const sab = {
        ops: new SharedArrayBuffer(Math.max(1, nrec) * OP_BYTES),
        text: new SharedArrayBuffer(Math.max(1, ntext) * 2),
        propsets: new SharedArrayBuffer(Math.max(1, nps) * 8),
        props: new SharedArrayBuffer(Math.max(1, npe) * 8),
        offsets: new SharedArrayBuffer((nDocs + 1) * 8),
      };
      // the deferred combining sets' entries, past every shard's
      new Uint32Array(sab.props, comb.base * 8, comb.entries.length).set(comb.entries);
      const te = process.hrtime.bigint();
      await Promise.all(this.workers.map((_, w) => this._call(w, { cmd: "emit", base: bases[w], map: maps[w], sab })));
      const ts = process.hrtime.bigint();
      // the workers go on with the next part while this thread submits
      tp = ts;
      if (i + 1 < uptos.length) next = packAll(uptos[i + 1]);
      new BigUint64Array(sab.offsets)[nDocs] = BigInt(nrec);
      eng.sync();  // the previous replay may still read the other batch slot
      eng.views.fill(null);
      eng.refViews.fill(null);
      eng.addon.submit(eng.ctx, new BigUint64Array(sab.offsets), new Uint8Array(sab.ops, 0, nrec * OP_BYTES),
        new Uint16Array(sab.text, 0, ntext), new Uint32Array(sab.propsets, 0, 2 * nps),
        new Uint32Array(sab.props, 0, 2 * npe));
      eng.addon.run(eng.ctx);
      eng.running = true;
      t.merge_ms += Number(te - tm) / 1e6;
      t.emit_ms += Number(ts - te) / 1e6;
      t.submit_ms += Number(process.hrtime.bigint() - ts) / 1e6;
      total += nrec;
    }
    return total;
  }

  // the shards' keys / values interned since the last part -> the engine's
  // interner (the single id space its read-outs decode with); each shard's
  // base in the shared batch.  Sequenced incr / consensus annotates of
  // MTE_DOC_TREE documents: their value maps cover every value their key was
  // ever given in any shard (PropTable.addCombining over the engine's
  // interner, once the shards' key -> value notes are merged), written past
  // the shards' property entries (PropTable.addDeferred)
  _merge(parts) {
    const it = this.engine.interner;
    if (!this.maps) this.maps = this.workers.map(() => ({ keys: [], values: [0] }));
    const maps = parts.map((p, w) => {
      const m = this.maps[w];  // a shard's key / value ids -> the engine's
      for (const name of p.keys) m.keys.push(it.key(name));
      for (const j of p.values) m.values.push(it.valueOfJson(j));
      for (let i = 0; i < p.notes.length; i += 2) it.noteValue(m.keys[p.notes[i]], m.values[p.notes[i + 1]]);
      return { keys: Int32Array.from(m.keys), values: Uint32Array.from(m.values) };
    });
    const pt = new PropTable(it);
    parts.forEach((p, w) => {
      const dv = [];
      for (const [, names, comb, seq] of p.deferred) {
        const props = {};
        for (const name of names) props[name] = null;  // combineValue ignores the op's values
        const i = pt.addCombining(props, comb, seq);
        dv.push(pt.sets[2 * i], pt.sets[2 * i + 1]);
      }
      maps[w].deferred = Uint32Array.from(dv);
    });
    let nrec = 0, ntext = 0, nps = 0, npe = 0;
    const bases = parts.map((p) => {
      const b = { rec: nrec, text: ntext, ps: nps, pe: npe };
      nrec += p.nrec;
      ntext += p.ntext;
      nps += p.nps;
      npe += p.npe;
      return b;
    });
    for (const m of maps) for (let q = 0; q < m.deferred.length; q += 2) m.deferred[q] += npe;
    const comb = { base: npe, entries: Uint32Array.from(pt.entries) };
    npe += pt.entries.length / 2;
    return { maps, bases, nrec, ntext, nps, npe, comb };
  }

  async close() {
    await Promise.all(this.workers.map((W) => W.terminate()));
    this.workers = [];
  }
}

module.exports = { ShardedHost };
