#!/usr/bin/env node
// The Node host end to end with parallel packing (bench.py's
// end_to_end_node_sharded leg): ShardedHost (shards.js) workers, each owning a
// contiguous shard of the documents, pack their documents' messages — built
// from the generated stream in data.dir by stream_source.js before the clock,
// as a server holds them from its delta streams — into one shared batch; the
// host submits and replays it (mte_submit + mte_run over N-API), in `parts`
// slices so that packing slice i + 1 overlaps the submit and replay of slice i.
// argv: dir workers parts [recorder] ("recorder": no device, the N-API calls
// recorded — a CPU run of the packing alone).  Prints one JSON line.
"use strict";
const fs = require("fs");
const path = require("path");
const { MergeTreeEngine } = require("./index.js");
const { ShardedHost } = require("./shards.js");

async function main() {
  const [dir, workersArg, partsArg, mode] = process.argv.slice(2);
  const workers = Number(workersArg || 8), parts = Number(partsArg || 4);
  const inits = JSON.parse(fs.readFileSync(path.join(dir, "inits.json"), "utf8"));
  const recorder = {
    create() { return {}; }, destroy() {}, loadDocs() {}, loadSegments() {}, submit() {}, run() {}, sync() {},
    readDeltas() { return new Uint32Array(0); },
  };
  const eng = new MergeTreeEngine(mode === "recorder" ? { nKeys: 4, addon: recorder } : { nKeys: 4 });
  const clients = inits.map((d) => eng.createClient(d.text, { newLengthCalc: d.newCalc, roundSync: d.roundSync }));
  const host = new ShardedHost(eng, { workers, source: path.join(__dirname, "stream_source.js"), sourceData: { dir } });
  const tl0 = process.hrtime.bigint();
  await host.start();  // load + each worker builds its documents' message objects
  const tl1 = process.hrtime.bigint();
  const maxLen = inits.reduce((a, d) => Math.max(a, d.nMsgs), 0);
  const t0 = process.hrtime.bigint();
  const uptos = [];
  for (let p = 1; p <= parts; p++) uptos.push(Math.floor((maxLen * p) / parts));
  const nrec = await host.flushParts(uptos);
  eng.sync();
  const t1 = process.hrtime.bigint();
  const ms = Number(t1 - t0) / 1e6;
  const out = { ops: nrec, docs: inits.length, workers: host.workers.length, parts, ms, ops_per_s: nrec / (ms / 1e3),
    load_ms: Number(tl1 - tl0) / 1e6, timing: host.timing };
  if (mode !== "recorder") {
    const st = eng.statuses();
    out.errors = st.reduce((a, x) => a + (x !== 0 ? 1 : 0), 0);
    const sample = Math.min(inits.length, 64);
    out.texts = clients.slice(0, sample).map((c) => c.getText());
  }
  await host.close();
  eng.close();
  process.stdout.write(JSON.stringify(out) + "\n");
}

main().catch((e) => {
  process.stderr.write(String(e && e.stack ? e.stack : e) + "\n");
  process.exit(1);
});
