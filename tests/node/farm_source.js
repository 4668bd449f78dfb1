"use strict";
// A ShardedHost source (fluidframework_amd/node/shards.js) over reference
// farm vectors (tests/golden/*.json.gz): document d is the observer of set
// data.sets[d], fed the sequenced messages its events apply up to its last
// checkpoint (the observer never sends).  Test infrastructure.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const { asMsg } = require("./fixtures");

function load(d0, d1, data) {
  const sets = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, "..", "golden", data.file)))
    .toString("utf8")).sets;
  const out = [];
  for (let d = d0; d < d1; d++) {
    const s = sets[data.sets[d]];
    const done = s.checkpoints[s.checkpoints.length - 1].done[0];
    out.push(s.events[0].slice(0, done).map((ev) => {
      if (ev[0] !== "A") throw new Error("set " + data.sets[d] + ": the observer sent an op");
      return asMsg(s.log[ev[1]]);
    }));
  }
  return out;
}

module.exports = { load };
