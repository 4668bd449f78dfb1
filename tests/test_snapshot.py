"""Summary round trip: replay half of a batch, write
every document's body (snapshotV1.ts:189-265 rules, fluidframework_amd/
snapshot.py), load the bodies into a fresh engine (snapshotLoader.ts:85-125,
mte_load_segments) and replay the rest: the digests must equal the
uninterrupted replay's.  CPU on the restatement, GPU on the engine."""
import numpy as np
import pytest

from fluidframework_amd import gen, snapshot
from fluidframework_amd.engine import DeviceEngine
from oracle import OracleEngine, SpecOracle


def split_batch(stream, k):
    """(first k ops of every doc, the rest)."""
    b = stream["batch"]
    o = b["op_offsets"].astype(np.int64)
    first = gen.prefix_ops(stream, len(o) - 1, k)["batch"]
    rest_ops = np.concatenate([b["ops"][o[i] + min(k, o[i + 1] - o[i]):o[i + 1]] for i in range(len(o) - 1)])
    cnt = np.array([max(0, (o[i + 1] - o[i]) - k) for i in range(len(o) - 1)])
    offs = np.zeros(len(o), np.uint64)
    offs[1:] = np.cumsum(cnt)
    return first, dict(b, ops=rest_ops, op_offsets=offs)


def round_trip(make, stream, k):
    full = make(stream["n_keys"])
    gen.load_stream(full, stream)
    full.apply_batch(stream["batch"])
    first, rest = split_batch(stream, k)
    a = make(stream["n_keys"])
    gen.load_stream(a, stream)
    a.apply_batch(first)
    n = len(stream["inits"])
    views = [a.read_doc(d) for d in range(n)]
    bodies = [snapshot.write_body(a, d, views[d]["min_seq"]) for d in range(n)]
    windows = [(v["min_seq"], v["cur_seq"]) for v in views]
    inits, text, ps, pe, offs, segs = snapshot.load_bodies(bodies, windows, stream["inits"]["flags"],
                                                          stream["n_keys"])
    b = make(stream["n_keys"])
    b.load_docs(inits, text, ps, pe)
    b.load_segments(offs, segs)
    for d in range(n):  # the loaded summary reads out as the summarized doc
        assert b.read_doc(d)["text"] == views[d]["text"]
    b.apply_batch(rest)
    assert (full.statuses() == 0).all() and (b.statuses() == 0).all()
    np.testing.assert_array_equal(b.digest(), full.digest())
    return bodies


@pytest.mark.parametrize("spec", [False, True])
def test_summary_round_trip_oracle(spec):
    s = gen.generate(3, n_docs=24, ops_per_doc=1500)  # R = 64: cut at a round boundary and inside one
    make = (lambda nk: SpecOracle(nk, threads=8)) if spec else (lambda nk: OracleEngine(nk))
    for k in (640, 700):
        bodies = round_trip(make, s, k)
        assert any("removedSeq" in sp for body in bodies for sp in body)  # tombstones above the MSN kept
        assert any("seq" not in sp for body in bodies for sp in body)     # below-MSN text coalesced


def test_summary_writer_coalesces_and_elides():
    s = gen.generate(2, n_docs=4, ops_per_doc=600)
    o = OracleEngine(s["n_keys"])
    gen.load_stream(o, s)
    o.apply_batch(s["batch"])
    for d in range(4):
        v = o.read_doc(d)
        body = snapshot.write_body(o, d, v["cur_seq"])  # everything at or below the MSN
        assert all("seq" not in sp and "removedSeq" not in sp for sp in body)
        units = [u for sp in body for u in (sp["json"] if isinstance(sp["json"], list) else
                                            sp["json"].get("text", []))]
        assert "".join(map(chr, units)) == v["text"]


@pytest.mark.gpu
def test_gpu_summary_round_trip():
    s = gen.generate(3, n_docs=64, ops_per_doc=1500)
    bodies_d = round_trip(lambda nk: DeviceEngine(nk), s, 700)
    # the engine's specification (legacy docs: the tree, whose append-merges
    # coarsen segments that a later remove turns into one tombstone)
    bodies_o = round_trip(lambda nk: SpecOracle(nk, threads=8), s, 700)
    assert bodies_d == bodies_o  # the GPU's summary is the restatement's


@pytest.mark.gpu
def test_gpu_summary_round_trip_long_docs():
    s = gen.generate(5, n_docs=4, ops_per_doc=4000, init_segs=6000, round_ops=1000)
    round_trip(lambda nk: DeviceEngine(nk, seg_capacity=16384), s, 2000)


def legacy_round_trip(make, stream, k, chunk_size=snapshot.SIZE_OF_FIRST_CHUNK):
    """Legacy summary (snapshotlegacy.ts:105-211): the document at minSeq plus the
    catch-up messages above it (sequence.ts:676-686); load (snapshotLoader.ts:130-246),
    replay the catch-up ops (sequence.ts:588-609), then the rest of the stream."""
    full = make(stream["n_keys"])
    gen.load_stream(full, stream)
    full.apply_batch(stream["batch"])
    first, rest = split_batch(stream, k)
    a = make(stream["n_keys"])
    gen.load_stream(a, stream)
    a.apply_batch(first)
    n = len(stream["inits"])
    views = [a.read_doc(d) for d in range(n)]
    fo = first["op_offsets"].astype(np.int64)
    ro = rest["op_offsets"].astype(np.int64)
    blobs, bodies, windows, tails = [], [], [], []
    for d in range(n):
        ops = first["ops"][fo[d]:fo[d + 1]]
        catchup = ops[ops["seq"] > views[d]["min_seq"]]
        b = snapshot.write_legacy(a, d, views[d]["min_seq"], catchup, chunk_size)
        blobs.append(b)
        windows.append(snapshot.legacy_window(b))
        bodies.append(snapshot.legacy_body(b))
        snapshot.check_catchup(catchup, windows[d])
        tails.append(np.concatenate([catchup, rest["ops"][ro[d]:ro[d + 1]]]))
    inits, text, ps, pe, offs, segs = snapshot.load_bodies(bodies, windows, stream["inits"]["flags"],
                                                          stream["n_keys"])
    b = make(stream["n_keys"])
    b.load_docs(inits, text, ps, pe)
    b.load_segments(offs, segs)
    toffs = np.zeros(n + 1, np.uint64)
    toffs[1:] = np.cumsum([len(t) for t in tails])
    b.apply_batch(dict(rest, ops=np.concatenate(tails), op_offsets=toffs))
    assert (full.statuses() == 0).all() and (b.statuses() == 0).all()
    np.testing.assert_array_equal(b.digest(), full.digest())
    return blobs


def test_legacy_summary_round_trip_oracle():
    s = gen.generate(3, n_docs=24, ops_per_doc=1500)
    for k in (640, 700):
        blobs = legacy_round_trip(lambda nk: OracleEngine(nk), s, k)
        assert all("catchupOps" in b for b in blobs)  # ops above the MSN travel with the summary
    # a small first chunk forces header + body (snapshotlegacy.spec.ts:47-81)
    blobs = legacy_round_trip(lambda nk: OracleEngine(nk), s, 700, chunk_size=40)
    assert any("body" in b for b in blobs)
    for b in blobs:
        md = b["header"]["headerMetadata"]
        assert [c["id"] for c in md["orderedChunkMetadata"]] == ["header"] + (["body"] if "body" in b else [])
        assert "minSequenceNumber" not in md  # legacy: window = (seq, seq) on load


def test_legacy_loader_checks():
    s = gen.generate(3, n_docs=2, ops_per_doc=600)  # annotated: segments with differing props
    o = OracleEngine(s["n_keys"])
    gen.load_stream(o, s)
    o.apply_batch(s["batch"])
    v = o.read_doc(0)
    b = snapshot.write_legacy(o, 0, v["min_seq"], chunk_size=2)
    assert "body" in b
    b["body"]["chunkLengthChars"] += 1
    with pytest.raises(snapshot.SnapshotLoadError, match="0x063"):
        snapshot.legacy_body(b)
    ops = s["batch"]["ops"][:4]
    with pytest.raises(snapshot.SnapshotLoadError, match="Invalid catchup"):
        snapshot.check_catchup(ops, (v["min_seq"], v["min_seq"]))


@pytest.mark.gpu
def test_gpu_legacy_summary_round_trip():
    s = gen.generate(3, n_docs=64, ops_per_doc=1500)
    blobs_d = legacy_round_trip(lambda nk: DeviceEngine(nk), s, 700, chunk_size=64)
    blobs_o = legacy_round_trip(lambda nk: SpecOracle(nk, threads=8), s, 700, chunk_size=64)
    assert [{k: v for k, v in b.items() if k != "catchupOps"} for b in blobs_d] == \
        [{k: v for k, v in b.items() if k != "catchupOps"} for b in blobs_o]
