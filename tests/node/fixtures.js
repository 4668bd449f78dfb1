"use strict";
// Loads tests/golden/replay_fixtures.json.gz (the reference's golden replay
// fixtures, see tests/golden/make_golden.py) for the Node host tests.
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");

function loadFixtures() {
  const p = path.join(__dirname, "..", "golden", "replay_fixtures.json.gz");
  return JSON.parse(zlib.gunzipSync(fs.readFileSync(p)).toString("utf8"));
}

function asMsg(m) {
  return { clientId: m[0], sequenceNumber: m[1], referenceSequenceNumber: m[2], minimumSequenceNumber: m[3],
    type: m[4], contents: m[5] };
}

module.exports = { loadFixtures, asMsg };
