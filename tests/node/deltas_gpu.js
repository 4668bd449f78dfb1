"use strict";
// GPU test: delta events through the Node host.  stdin: {"docs": [{"initialText",
// "msgs": [[clientId, seq, refSeq, msn, type, contents], ...]}]} (new length
// calculation).  Every document is a BatchClient created with {events: true};
// all messages are applied, then one flush.  Prints one JSON line: per doc the
// sequenceDelta events flattened as [message index, kind, position, length,
// removed] and the rewritten catch-up stash (getMessagesSinceMSNChange).
// input.tree: the documents on the tree pass ({tree: true}, MTE_DOC_TREE);
// MTE_NODE_ADDON=oracle: the CPU restatement's addon (tests only).
const fs = require("fs");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");
const { asMsg } = require("./fixtures");

const input = JSON.parse(fs.readFileSync(0, "utf8"));
const oracleAddon = process.env.MTE_NODE_ADDON === "oracle"
  ? require(require("path").join(__dirname, "..", "..", "oracle", "_build", "mte_napi_oracle.node")) : null;
const eng = new MergeTreeEngine(oracleAddon ? { nKeys: 8, addon: oracleAddon } : { nKeys: 8 });
const out = input.docs.map((d) => {
  const c = eng.createClient(d.initialText, { newLengthCalc: true, events: true, tree: !!input.tree });
  const rec = { events: [], stash: null };
  const index = new Map();
  c.on("sequenceDelta", (ev) => {
    const mi = index.get(ev.message);
    for (const r of ev.ranges) rec.events.push([mi, ev.deltaOperation, r.position, r.length, r.removed ? 1 : 0]);
  });
  return { c, rec, d, index };
});
for (const o of out) {
  o.d.msgs.forEach((m, i) => {
    const msg = asMsg(m);
    o.index.set(msg, i);
    o.c.applyMsg(msg);
  });
}
eng.flush();
eng.sync();
for (const o of out) o.rec.stash = o.c.getMessagesSinceMSNChange();
process.stdout.write(JSON.stringify({ docs: out.map((o) => o.rec) }) + "\n");
eng.close();
