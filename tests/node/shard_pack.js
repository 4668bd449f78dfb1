"use strict";
// CPU test helper: ShardedHost (fluidframework_amd/node/shards.js) over a
// generated stream on disk, with a recording addon instead of the device:
// prints one JSON line per flush (the shared batch, base64) and a last line
// with the engine interner's key names and value JSON (to decode properties).
// argv: dir workers parts [pipelined] (pipelined: one flushParts call, the
// workers packing part i + 1 while part i is submitted)
const path = require("path");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { ShardedHost } = require("../../fluidframework_amd/node/shards");
const fs = require("fs");

const [dir, workers, parts, mode] = process.argv.slice(2);
const b64 = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength).toString("base64");
const lines = [];
const recorder = {
  create() { return {}; }, destroy() {}, loadDocs() {}, loadSegments() {}, run() {}, sync() {},
  readDeltas() { return new Uint32Array(0); },
  submit(ctx, offsets, ops, text, propsets, props) {
    lines.push({ offsets: b64(offsets), ops: b64(ops), text: b64(text), propsets: b64(propsets), props: b64(props) });
  },
};
(async () => {
  const inits = JSON.parse(fs.readFileSync(path.join(dir, "inits.json"), "utf8"));
  const eng = new MergeTreeEngine({ nKeys: 4, addon: recorder });
  inits.forEach((d) => eng.createClient(d.text, { newLengthCalc: d.newCalc, roundSync: d.roundSync }));
  const host = new ShardedHost(eng, { workers: Number(workers), source: path.join(__dirname, "..", "..",
    "fluidframework_amd", "node", "stream_source.js"), sourceData: { dir } });
  await host.start();
  const maxLen = inits.reduce((a, d) => Math.max(a, d.nMsgs), 0);
  const uptos = [];
  for (let p = 1; p <= Number(parts); p++) uptos.push(Math.floor((maxLen * p) / Number(parts)));
  if (mode === "pipelined") await host.flushParts(uptos);
  else for (const u of uptos) await host.flush(u);
  await host.close();
  for (const l of lines) process.stdout.write(JSON.stringify(l) + "\n");
  process.stdout.write(JSON.stringify({ keys: eng.interner.keyNames, values: eng.interner.valueJson }) + "\n");
})().catch((e) => {
  process.stderr.write(String(e.stack || e));
  process.exit(1);
});
