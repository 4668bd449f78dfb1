// Load each rebuilt fixture string (stdin: [{name, version, segments}]) as a
// summary body, emit it with summarizeV1 / summarizeLegacy, and load the
// emitted blobs back: stdout [{name, blobs, text}].
"use strict";
const fs = require("fs");
const { MergeTreeEngine } = require("../../fluidframework_amd/node");

const cases = JSON.parse(fs.readFileSync(0, "utf8"));
const out = [];
for (const c of cases) {
  const eng = new MergeTreeEngine({ nKeys: 8, segCapacity: 16384 });
  const cl = eng.createClient("", { segments: c.segments, minSeq: 0, currentSeq: 0 });
  eng.start();
  const blobs = c.version === "v1" ? cl.summarizeV1() : cl.summarizeLegacy();
  eng.close();
  const eng2 = new MergeTreeEngine({ nKeys: 8, segCapacity: 16384 });
  const cl2 = eng2.createClient("", { summary: blobs });
  const text = cl2.getText();
  eng2.close();
  out.push({ name: c.name, blobs, text });
}
process.stdout.write(JSON.stringify(out));
