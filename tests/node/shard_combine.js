"use strict";
// Test: ShardedHost (fluidframework_amd/node/shards.js) packing the combining
// farms' observers (tests/golden/combine_farm_vectors.json.gz) as remote-only
// MTE_DOC_TREE documents on several worker threads: each worker defers its
// sequenced incr / consensus annotates' value maps to the host's merge, which
// closes them over every shard's values (PropTable.addDeferred).  At the end
// every observer's text, length and per-position properties must be the
// reference's last checkpoint.  argv: workers, sets per engine.
// MTE_NODE_ADDON=oracle: over the CPU restatement.  Prints one JSON line.
const path = require("path");
const fs = require("fs");
const zlib = require("zlib");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { ShardedHost } = require("../../fluidframework_amd/node/shards");

const oracleAddon = process.env.MTE_NODE_ADDON === "oracle"
  ? require(path.join(__dirname, "..", "..", "oracle", "_build", "mte_napi_oracle.node")) : null;
const FILE = "combine_farm_vectors.json.gz";
const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden", FILE)))
  .toString("utf8")).sets;
const workers = Number(process.argv[2] || 3), per = Number(process.argv[3] || 3);

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

(async () => {
  let passed = 0, combining = 0;
  const failures = [];
  for (let g0 = 0; g0 < sets.length; g0 += per) {
    const group = [];
    for (let si = g0; si < Math.min(sets.length, g0 + per); si++) group.push(si);
    const eng = new MergeTreeEngine(oracleAddon ? { nKeys: 8, addon: oracleAddon } : { nKeys: 8 });
    const clients = group.map((si) => eng.createClient(sets[si].initialText,
      { newLengthCalc: !sets[si].legacy, longClientId: sets[si].names[0], tree: true }));
    for (const si of group) {
      for (const e of sets[si].log) if (e[5] && e[5].combiningOp && e[5].combiningOp.name !== "rewrite") combining++;
    }
    const host = new ShardedHost(eng, { workers, source: path.join(__dirname, "farm_source.js"),
      sourceData: { file: FILE, sets: group } });
    await host.start();
    await host.flushParts([50, 150, 1 << 30]);  // pipelined parts: shards pack part i + 1 during part i
    await host.close();
    eng.sync();
    group.forEach((si, d) => {
      const s = sets[si], c = clients[d];
      const want = s.checkpoints[s.checkpoints.length - 1].states[0];
      const got = { text: c.getText(), length: c.getLength(), props: propRuns(c) };
      if (got.text === want.text && got.length === want.length && JSON.stringify(got.props) === JSON.stringify(want.props)) {
        passed++;
      } else {
        const gp = JSON.stringify(got.props), wp = JSON.stringify(want.props);
        let k = 0;
        while (k < gp.length && gp[k] === wp[k]) k++;
        failures.push([si, got.text === want.text, gp.slice(Math.max(0, k - 80), k + 80), wp.slice(Math.max(0, k - 80), k + 80)]);
      }
    });
    eng.close();
  }
  process.stdout.write(JSON.stringify({ passed, combining, failures: failures.slice(0, 5), nFailures: failures.length,
    sets: sets.length }) + "\n");
})().catch((e) => {
  process.stderr.write(String(e.stack || e));
  process.exit(1);
});
