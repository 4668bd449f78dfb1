"""Summaries pinned against the reference's own fixtures.

packages/dds/sequence/src/test/snapshots/{legacy,legacyWithCatchUp,v1,v1Intervals}
hold the merge-tree "content" blobs SharedString wrote for the strings
generateSharedStrings.ts:47-147 builds.  tests/golden/snapshot_digests.json
keeps, per blob, the SHA-256 of its chunk as canonical JSON plus its counters
(tests/golden/make_snapshot_golden.py; no fixture text is copied).

The strings are rebuilt here (tests/snapshot_strings.py) and loaded into an
engine as the reference holds them (one segment per edit, NonCollabClient at
UniversalSequenceNumber); the writers (snapshot.write_v1 = SnapshotV1.emit,
snapshot.write_legacy = SnapshotLegacy.emit) must reproduce every blob digest,
and the loader (summary_body + load_bodies) must read the blobs back into the
same text and properties."""
import hashlib
import json
import os

import pytest

import snapshot_strings as ss
from fluidframework_amd import snapshot
from oracle import OracleEngine

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "snapshot_digests.json")
with open(GOLD, encoding="utf-8") as fh:
    FIXTURES = json.load(fh)["fixtures"]

CASES = [(v, n) for v in ("legacy", "legacyWithCatchUp", "v1") for n in ss.NAMES] + [("v1Intervals", "withV1Intervals")]


def digest(chunk):
    return hashlib.sha256(json.dumps(chunk, sort_keys=True, separators=(",", ":"),
                                     ensure_ascii=False).encode("utf-8")).hexdigest()


def load_string(make, name, new_calc=False):
    seg = ss.build(name)
    it = ss.interner()
    body = ss.body(seg, it)
    inits, text, ps, pe, offs, segs = snapshot.load_bodies([body], [(0, 0)], [1 if new_calc else 0], 8)
    e = make(8)
    e.load_docs(inits, text, ps, pe)
    e.load_segments(offs, segs)
    return e, it, seg


def emit(e, it, version):
    if version == "v1":
        blobs = snapshot.write_v1(e, 0, 0, 0)
        for c in blobs.values():
            c["segments"] = [snapshot.to_json(sp, it) for sp in c["segments"]]
    else:
        blobs = snapshot.write_legacy(e, 0, 0)
        for c in blobs.values():
            c["segmentTexts"] = [snapshot.to_json(sp, it) for sp in c["segmentTexts"]]
    return blobs


def test_fixture_inventory():
    assert set(FIXTURES) == {f"{v}/{n}" for v, n in CASES}
    assert sum(len(b) for b in FIXTURES.values()) == 29  # header, body, body_0..2 blobs


def test_rebuilt_strings_match_fixture_counters():
    # the rebuilt strings have the fixtures' lengths (header metadata)
    for v, n in CASES:
        md = FIXTURES[f"{v}/{n}"]["header"]["meta"]["headerMetadata"]
        text, props = ss.expected_view(ss.build(n))
        assert md["totalLength"] == len(props), (v, n)


@pytest.mark.parametrize("version,name", CASES, ids=[f"{v}/{n}" for v, n in CASES])
def test_writer_reproduces_reference_blobs(oracle_lib, version, name):
    e, it, _ = load_string(lambda k: OracleEngine(k), name)
    blobs = emit(e, it, "v1" if version == "v1" else "legacy")  # v1Intervals: default (legacy) content format
    want = FIXTURES[f"{version}/{name}"]
    assert sorted(blobs) == sorted(want)
    for bid, c in blobs.items():
        meta = {k: v for k, v in c.items() if k not in ("segments", "segmentTexts")}
        assert meta == want[bid]["meta"], bid
        assert digest(c) == want[bid]["sha256"], bid


@pytest.mark.parametrize("version", ["v1", "legacy"])
@pytest.mark.parametrize("name", ["headerOnly", "withMarkers", "withAnnotations"])
def test_loader_reads_emitted_blobs(oracle_lib, version, name):
    # blob -> summary_body -> load_bodies -> engine: the string reads as built
    e, it, seg = load_string(lambda k: OracleEngine(k), name)
    blobs = emit(e, it, version)
    body, n_header = snapshot.summary_body(blobs)
    assert 0 < n_header <= len(body)
    window = snapshot.summary_window(blobs)
    assert window == (0, 0)
    inits, text, ps, pe, offs, segs = snapshot.load_bodies(
        [[{"json": snapshot.from_json(sp["json"], it)} for sp in body]], [window], [0], 8)
    o = OracleEngine(8)
    o.load_docs(inits, text, ps, pe)
    o.load_segments(offs, segs)
    v = o.read_doc(0)
    want_text, want_props = ss.expected_view(seg)
    assert v["text"] == want_text
    props = [it.decode_props(p) for ln, _, p in v["segs"] for _ in range(ln)]
    assert props == want_props


def test_loader_checks_chunk_counters():
    e, it, _ = load_string(lambda k: OracleEngine(k), "withMarkers")
    blobs = emit(e, it, "v1")
    blobs["body_1"]["length"] += 1
    with pytest.raises(snapshot.SnapshotLoadError, match="0x063"):
        snapshot.summary_body(blobs)
    blobs = emit(e, it, "v1")
    blobs["header"]["segmentCount"] = blobs["header"]["headerMetadata"]["totalSegmentCount"] + 1
    with pytest.raises(snapshot.SnapshotLoadError, match="0x062"):
        snapshot.summary_body(blobs)


@pytest.mark.gpu
@pytest.mark.parametrize("version,name", [(v, n) for v, n in CASES if v != "legacyWithCatchUp"],
                         ids=[f"{v}/{n}" for v, n in CASES if v != "legacyWithCatchUp"])
def test_gpu_writer_reproduces_reference_blobs(version, name):
    from fluidframework_amd.engine import DeviceEngine
    e, it, _ = load_string(lambda k: DeviceEngine(k, seg_capacity=16384), name)
    blobs = emit(e, it, "v1" if version == "v1" else "legacy")  # v1Intervals: default (legacy) content format
    want = FIXTURES[f"{version}/{name}"]
    for bid, c in blobs.items():
        assert digest(c) == want[bid]["sha256"], bid


@pytest.mark.gpu
def test_node_host_writer_reproduces_reference_blobs():
    # the Node host's summarizeV1 / summarizeLegacy over the same loaded strings,
    # and its loader reading them back (tests/node/snapshot_fixtures_gpu.js)
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = []
    for version, name in [("v1", "withMarkers"), ("v1", "withAnnotations"), ("legacy", "withMarkers"),
                          ("legacy", "headerAndBody")]:
        it = ss.interner()
        seg = ss.build(name)
        cases.append({"name": f"{version}/{name}", "version": version,
                      "segments": [{"json": snapshot.to_json(sp["json"], it)} for sp in ss.body(seg, it)],
                      "text": ss.expected_view(seg)[0]})
    r = subprocess.run([node, "tests/node/snapshot_fixtures_gpu.js"], cwd=root, input=json.dumps(cases),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    for c, got in zip(cases, json.loads(r.stdout)):
        want = FIXTURES[c["name"]]
        assert sorted(got["blobs"]) == sorted(want)
        for bid, chunk in got["blobs"].items():
            assert digest(chunk) == want[bid]["sha256"], (c["name"], bid)
        assert got["text"] == c["text"]
