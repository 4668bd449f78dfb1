"use strict";
// A ShardedHost source (shards.js) over a generated stream on disk
// (bench.py writes it: fluidframework_amd/gen.py's batch arrays): documents
// [d0, d1) as the ISequencedDocumentMessage objects the reference would
// receive, as fluidframework_amd/messages.py builds them (sender short id c ->
// long id "c<c>", the observer "A").  Each worker reads only its documents'
// records.  Files in data.dir: offsets.u64 (n_docs + 1), ops.bin (32-byte
// records), text.u16, propsets.u32 (first, count), props.u32 (key, value),
// tables.json {keys: [names], values: {id: json}}.
const fs = require("fs");
const path = require("path");

const OP_INSERT = 0, OP_REMOVE = 1, OP_ANNOTATE = 2, F_MARKER = 1, F_REWRITE = 4, NO_PROPS = 0xffffffff;

function readSlice(file, byteOff, byteLen) {
  const buf = Buffer.alloc(byteLen);
  const fd = fs.openSync(file, "r");
  try {
    let got = 0;
    while (got < byteLen) got += fs.readSync(fd, buf, got, byteLen - got, byteOff + got);
  } finally {
    fs.closeSync(fd);
  }
  return buf;
}

function load(d0, d1, data) {
  const dir = data.dir;
  const offs = new BigUint64Array(readSlice(path.join(dir, "offsets.u64"), d0 * 8, (d1 - d0 + 1) * 8).buffer.slice(0));
  const k0 = Number(offs[0]), k1 = Number(offs[d1 - d0]);
  const ops = readSlice(path.join(dir, "ops.bin"), k0 * 32, (k1 - k0) * 32);
  const W = new Int32Array(ops.buffer, ops.byteOffset, (k1 - k0) * 8);
  const tb = fs.readFileSync(path.join(dir, "text.u16"));
  const text = new Uint16Array(tb.buffer, tb.byteOffset, tb.length / 2);
  const psb = fs.readFileSync(path.join(dir, "propsets.u32"));
  const ps = new Uint32Array(psb.buffer, psb.byteOffset, psb.length / 4);
  const peb = fs.readFileSync(path.join(dir, "props.u32"));
  const pe = new Uint32Array(peb.buffer, peb.byteOffset, peb.length / 4);
  const tables = JSON.parse(fs.readFileSync(path.join(dir, "tables.json"), "utf8"));
  const vals = new Map(Object.keys(tables.values).map((k) => [Number(k), JSON.parse(tables.values[k])]));
  const propsOf = (psi) => {
    const out = {};
    for (let k = ps[2 * psi]; k < ps[2 * psi] + ps[2 * psi + 1]; k++) {
      const vid = pe[2 * k + 1];
      out[tables.keys[pe[2 * k]]] = vid === 0 ? null : vals.get(vid);
    }
    return out;
  };
  const docs = [];
  for (let d = 0; d < d1 - d0; d++) {
    const msgs = [];
    for (let k = Number(offs[d]) - k0; k < Number(offs[d + 1]) - k0; k++) {
      const w = k * 8, w3 = W[w + 3] >>> 0;
      const t = w3 & 0xff, client = (w3 >>> 8) & 0xff, flags = w3 >>> 16;
      const a = W[w + 6] >>> 0, b = W[w + 7] >>> 0;
      let contents;
      if (t === OP_INSERT) {
        let seg;
        if (flags & F_MARKER) {
          seg = { marker: { refType: W[w + 5] } };
          if (b !== NO_PROPS) seg.props = propsOf(b);
        } else {
          const s = String.fromCharCode.apply(null, text.subarray(a, a + W[w + 5]));
          seg = b === NO_PROPS ? s : { text: s, props: propsOf(b) };
        }
        contents = { type: 0, pos1: W[w + 4], seg };
      } else if (t === OP_REMOVE) {
        contents = { type: 1, pos1: W[w + 4], pos2: W[w + 5] };
      } else if (t === OP_ANNOTATE) {
        contents = { type: 2, pos1: W[w + 4], pos2: W[w + 5], props: propsOf(a) };
        if (flags & F_REWRITE) contents.combiningOp = { name: "rewrite" };
      }
      msgs.push({ clientId: "c" + client, sequenceNumber: W[w], referenceSequenceNumber: W[w + 1],
        minimumSequenceNumber: W[w + 2], type: contents === undefined ? "noop" : "op", contents });
    }
    docs.push(msgs);
  }
  return docs;
}

module.exports = { load };
