#!/usr/bin/env node
// ref_fixture_replay.js — the reference's own replay test, run on the erased
// reference merge-tree (TEST INFRASTRUCTURE; build container only: the
// reference never travels to the GPU box).
//
// Mirrors packages/dds/merge-tree/src/test/client.replay.spec.ts:16-60 on the
// Client of oracle/_ref/ts (oracle/ts_erase.py): the original client "A"
// inserts the first round's initialText before collaboration; every sender
// gets a client of its own holding that same document (the spec loads one from
// A's legacy snapshot, TestClient.createFromClientSnapshot, testClient.ts:58-65;
// A holds only that text at that point, so the loaded client is the same
// document: one segment at UniversalSequenceNumber); per round every message
// is first applied locally by its sender (Client.localTransaction of the op as
// a group, client.ts:1062-1082, after the sender caught up to the message's
// refSeq), then every client applies every message through Client.applyMsg
// (the sender's own as its ack).  TestClientLogger.validate
// (testClientLogger.ts:173-229) compares all clients' getText
// (testClient.ts:148-150) at the start and end of every round.
//
// stdin:  the fixture list of tests/golden/replay_fixtures.json.gz
//         [{"name", "rounds": [{"initialText", "resultText", "msgs": [[clientId, seq, refSeq, msn, type, contents]]}]}]
// stdout: [{"name", "texts": [[initial, result] per round], "diverged": [[round, "initial"|"result", clientId]], "error"}]
"use strict";
const path = require("path");
const fs = require("fs");

const refdir = process.argv[2] || path.join(__dirname, "_ref", "ts");
const { Client } = require(path.join(refdir, "client.js"));
const { TextSegment } = require(path.join(refdir, "textSegment.js"));
const { Marker } = require(path.join(refdir, "mergeTreeNodes.js"));
const { MergeTreeTextHelper } = require(path.join(refdir, "MergeTreeTextHelper.js"));
const { createGroupOp } = require(path.join(refdir, "opBuilder.js"));

// test/testClient.ts:32-44
function specToSegment(spec) {
  const t = TextSegment.fromJSONObject(spec);
  if (t) return t;
  const m = Marker.fromJSONObject(spec);
  if (m) return m;
  throw new Error(`Unrecognized IJSONSegment type: '${JSON.stringify(spec)}'`);
}

const logger = { send() {}, sendTelemetryEvent() {}, sendErrorEvent() {}, sendPerformanceEvent() {} };
const GROUP = 3; // MergeTreeDeltaType.GROUP, ops.ts:43-48

function newClient(initialText, longId) {
  const c = new Client(specToSegment, logger); // TestClient: legacy length calc (test/testClient.ts:97-110)
  if (initialText) c.insertSegmentLocal(0, new TextSegment(initialText)); // insertTextLocal, testClient.ts:179-189
  c.startOrUpdateCollaboration(longId);
  return c;
}

function getText(c) {
  return new MergeTreeTextHelper(c._mergeTree).getText(c.getCurrentSeq(), c.getClientId(), "");
}

function replayFile(f) {
  const asMsg = (m) => ({ clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2],
    minimumSequenceNumber: m[3], type: m[4], contents: m[5] });
  const init = f.rounds[0].initialText;
  const clients = new Map([["A", { client: newClient(init, "A"), msgs: [] }]]);
  for (const g of f.rounds) {
    for (const m of g.msgs) if (!clients.has(m[0])) clients.set(m[0], { client: newClient(init, m[0]), msgs: [] });
  }
  const texts = [];
  const diverged = [];
  const validate = (r, what) => {
    const a = getText(clients.get("A").client);
    for (const [id, mc] of clients) if (getText(mc.client) !== a) diverged.push([r, what, id]);
    return a;
  };
  try {
    f.rounds.forEach((g, r) => {
      const initial = validate(r, "initial");
      for (const m of g.msgs) {
        const msg = asMsg(m);
        const mc = clients.get(msg.clientId);
        while (mc.msgs.length > 0 && msg.referenceSequenceNumber > mc.client.getCurrentSeq()) {
          mc.client.applyMsg(mc.msgs.shift());
        }
        const op = msg.contents;
        mc.client.localTransaction(op.type === GROUP ? op : createGroupOp(op));
        clients.forEach((x) => x.msgs.push(msg));
      }
      clients.forEach((x) => {
        while (x.msgs.length > 0) x.client.applyMsg(x.msgs.shift());
      });
      texts.push([initial, validate(r, "result")]);
    });
  } catch (e) {
    return { name: f.name, texts, diverged, error: String(e && e.message ? e.message : e) };
  }
  return { name: f.name, texts, diverged, error: null };
}

const input = JSON.parse(fs.readFileSync(0, "utf8"));
process.stdout.write(JSON.stringify(input.map(replayFile)));
