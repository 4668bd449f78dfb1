"""Relative positions (IRelativePosition, ops.ts:62-76): ops that address a
marker by its id instead of a position -- Client.annotateMarker
(client.ts:166-174, opBuilder.ts:26-40), and removes / inserts whose
relativePos1 / relativePos2 name a marker -- resolved by getValidOpRange
(client.ts:541-560) -> posFromRelativePos (mergeTree.ts:1369-1392) in each
op's own view.  The host packs an MTE_OP_RELPOS record before the op
(include/mte.h); the engine resolves it on the HBM-streamed pass (flat
documents: passes 1 and 2 hand such a document on for that batch) or on the
HBM tree pass (legacy and local-client documents).

Pinned by the reference's own farms (tests/golden/relpos_farm_vectors.json.gz,
oracle/ref_farm.js with relpos, made by tests/golden/make_farm_golden.py
--relpos): every client local (acks, rollbacks, reconnects and regenerated
ops), both length calculations; and each set's observer as a document of
remote clients only.  Marker ids in the farm are unique (idToSegment is a map
the reference never clears, mergeTree.ts:596-598: with duplicate ids its
answer depends on insert order and block maintenance; the engine takes the
first marker in document order -- parity unpinned there).
"""
import gzip
import json
import os

import numpy as np
import pytest

from fixtures_util import replay_ref_farm
from fluidframework_amd import gen
from fluidframework_amd.abi import (DOC_NEW_LENGTH_CALC, DOC_TREE, MTE_E_UNSUPPORTED, OP_ANNOTATE, OP_INSERT, OP_RELPOS,
                                    RP_BEFORE1, RP_POS1, RP_POS2)
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner

HERE = os.path.dirname(os.path.abspath(__file__))
NAME = "relpos_farm_vectors.json.gz"


def vector_sets():
    with gzip.open(os.path.join(HERE, "golden", NAME), "rt", encoding="utf-8") as fh:
        return json.load(fh)


def tree_factory(k):
    from oracle import OracleEngine
    e = OracleEngine(k, tree="items")
    e.lib.oti_set_limit(e.ctx, 1 << 20)
    return e


def spec_factory(k):
    from oracle import SpecOracle
    return SpecOracle(k, threads=4)


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def _all_clients(factory):
    sets = vector_sets()["sets"]
    checks = []
    passed, failures = replay_ref_farm(factory, sets, regen_checks=checks, exact_regen=True)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
    assert checks and all(checks)
    return passed, len(checks)


def _observers(factory, extra_flags=0):
    sets = vector_sets()["sets"]
    passed, failures = replay_ref_farm(factory, sets, observers_only=True, extra_flags=extra_flags)
    assert not failures, failures[:2]
    assert passed == sum(len(s["checkpoints"]) for s in sets)
    return passed


def test_relpos_vectors_shape():
    v = vector_sets()
    sets = v["sets"]
    assert len(sets) == 42 and sorted(v["seeds_the_reference_failed"]) == [9304, 9309]
    ops = [e[5] for s in sets for e in s["log"] if "relativePos1" in e[5]]
    assert len(ops) > 1000
    assert {o["type"] for o in ops} == {0, 1, 2}
    assert any(o.get("relativePos1", {}).get("offset") for o in ops)
    assert any(s.get("legacy") for s in sets) and any(not s.get("legacy") for s in sets)
    assert any(e[0] == "G" for s in sets for ev in s["events"] for e in ev)


def test_relpos_tree_oracle_every_client():
    passed, n_regen = _all_clients(tree_factory)
    assert passed == 768 and n_regen == 658


def test_relpos_spec_oracle_observers():
    assert _observers(spec_factory) == 176


def test_packer_relpos_record():
    it = Interner(4)
    bb = BatchBuilder(1, it)
    cl = DocClients("A")
    bb.add_message(0, cl, dict(clientId="b", sequenceNumber=1, referenceSequenceNumber=0, minimumSequenceNumber=0,
                               contents={"type": 0, "pos1": 0,
                                         "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1"}}}))
    bb.add_message(0, cl, dict(clientId="c", sequenceNumber=2, referenceSequenceNumber=1, minimumSequenceNumber=0,
                               contents={"type": 2, "props": {"k": 1}, "relativePos1": {"id": "m1", "before": True},
                                         "relativePos2": {"id": "m1", "offset": 2}}))
    ops = bb.build()["ops"]
    assert list(ops["type"]) == [OP_INSERT, OP_RELPOS, OP_ANNOTATE]
    rp = ops[1]
    assert int(rp["flags"]) == RP_POS1 | RP_BEFORE1 | RP_POS2
    assert int(rp["a"]) == it.keys["markerId"]
    assert int(rp["pos1"]) == int(rp["pos2"]) == it.values['"m1"']
    assert int(rp["seq"]) == 0 and int(rp["ref_seq"]) == 2  # the offsets
    assert int(ops[2]["flags"]) & 2  # MSG_END on the op, not on the RELPOS record


def _unknown_id_batch():
    it = Interner(4)
    bb = BatchBuilder(1, it)
    cl = DocClients("A")
    msgs = [{"type": 0, "pos1": 0, "seg": "hello"},
            {"type": 0, "pos1": 2, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1"}}},
            {"type": 2, "props": {"k": 1}, "relativePos1": {"id": "nope", "before": True},
             "relativePos2": {"id": "nope"}},   # not found: [-1, -1), nothing
            {"type": 1, "relativePos1": {"id": "m1", "before": True}, "relativePos2": {"id": "m1", "offset": 1}},
            {"type": 0, "relativePos1": {"id": "nope"}, "seg": "x"}]  # an insert not found: stops the doc
    for i, m in enumerate(msgs):
        bb.add_message(0, cl, dict(clientId="b", sequenceNumber=i + 1, referenceSequenceNumber=i,
                                   minimumSequenceNumber=0, contents=m))
    inits = np.zeros(1, gen.DOC_INIT_DTYPE)
    inits["flags"] = DOC_NEW_LENGTH_CALC
    inits["propset"] = 0xFFFFFFFF
    return it, inits, bb.build()


def _unknown_id(factory):
    it, inits, batch = _unknown_id_batch()
    e = factory(4)
    e.load_docs(inits, np.zeros(0, np.uint16))
    sub = dict(batch, ops=batch["ops"][:-2], op_offsets=np.array([0, len(batch["ops"]) - 2], np.uint64))
    e.apply_batch(sub)  # up to the remove around the marker
    mid = (e.statuses()[0], e.read_doc(0)["text"])
    rest = dict(batch, ops=batch["ops"][-2:], op_offsets=np.array([0, 2], np.uint64), text=batch["text"])
    e.apply_batch(rest)
    return mid, e.statuses()[0]


def test_relpos_unknown_id_oracle():
    from oracle import OracleEngine
    (st, text), last = _unknown_id(lambda k: OracleEngine(k))
    assert st == 0 and text == "helo"  # "he" + marker + "llo" minus [marker, marker + 2)
    assert last == MTE_E_UNSUPPORTED


@pytest.mark.gpu
def test_gpu_relpos_every_client():
    assert _all_clients(device_factory) == _all_clients(tree_factory)


@pytest.mark.gpu
def test_gpu_relpos_observers():
    # new length calculation: flat documents handed to the streamed pass for
    # the batch; legacy: tree documents moved to the HBM tree pass
    assert _observers(device_factory) == 176


@pytest.mark.gpu
def test_gpu_relpos_unknown_id():
    from oracle import OracleEngine
    assert _unknown_id(device_factory) == _unknown_id(lambda k: OracleEngine(k))


@pytest.mark.gpu
def test_gpu_relpos_beside_plain_documents():
    # one context: config-3 documents on pass 1 and the observers' documents
    # with relative positions, in the same batches; every document equals the
    # specification
    from fluidframework_amd.engine import DeviceEngine
    from oracle import SpecOracle
    s = gen.generate(3, n_docs=512, ops_per_doc=600, length_mode=2)
    o = SpecOracle(s["n_keys"], threads=8)
    d = DeviceEngine(s["n_keys"])
    for e in (o, d):
        gen.load_stream(e, s)
        e.apply_batch(s["batch"])
    np.testing.assert_array_equal(d.statuses(), o.statuses())
    np.testing.assert_array_equal(d.digest(), o.digest())
    assert _observers(device_factory) == 176


@pytest.mark.gpu
def test_gpu_relpos_chunked_context():
    # contexts of >= 8192 segments: a new length-calc document with relative
    # positions stops with MTE_E_UNSUPPORTED before the batch; a legacy one
    # replays on the HBM tree pass
    from fluidframework_amd.engine import DeviceEngine
    it, inits, batch = _unknown_id_batch()
    sub = dict(batch, ops=batch["ops"][:-2], op_offsets=np.array([0, len(batch["ops"]) - 2], np.uint64))
    d = DeviceEngine(4, seg_capacity=8192)
    d.load_docs(inits, np.zeros(0, np.uint16))
    d.apply_batch(sub)
    assert d.statuses()[0] == MTE_E_UNSUPPORTED
    inits2 = inits.copy()
    inits2["flags"] = 0
    d2 = DeviceEngine(4, seg_capacity=8192)
    d2.load_docs(inits2, np.zeros(0, np.uint16))
    d2.apply_batch(sub)
    assert d2.statuses()[0] == 0 and d2.read_doc(0)["text"] == "helo"
    # the same new length-calc document flagged MTE_DOC_TREE replays on the HBM tree pass
    inits3 = inits.copy()
    inits3["flags"] = int(inits["flags"][0]) | DOC_TREE
    d3 = DeviceEngine(4, seg_capacity=8192)
    d3.load_docs(inits3, np.zeros(0, np.uint16))
    d3.apply_batch(sub)
    assert d3.statuses()[0] == 0 and d3.read_doc(0)["text"] == "helo"


@pytest.mark.gpu
def test_gpu_relpos_observers_tree_documents_in_chunked_context():
    """Relative positions in new length-calc documents of a big-document
    context (>= 8,192 segments): flagged MTE_DOC_TREE they replay on the HBM
    tree pass, every observer of the 42 reference farms at every checkpoint."""
    from fluidframework_amd.engine import DeviceEngine
    assert _observers(lambda k: DeviceEngine(k, seg_capacity=8192), extra_flags=DOC_TREE) == 176


@pytest.mark.gpu
def test_node_relpos_every_client_on_gpu():
    """Every client a BatchClient ({localClient, events}) through the N-API host
    (tests/node/reconnect_gpu.js): annotateMarker and relative-position ops
    through applyLocalOp return the reference's ops, every state at every
    checkpoint and every regenerated op equal the reference's."""
    import shutil
    import subprocess

    from fixtures_util import canon_regen
    if shutil.which("node") is None:
        pytest.skip("node not installed")
    r = subprocess.run([shutil.which("node"), "tests/node/reconnect_gpu.js", "all", NAME], cwd=os.path.dirname(HERE),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["pending"] == 0 and j["nBadOps"] == 0, j["badOps"]
    bad = [x for x in j["states"] if not x[3]]
    assert not bad, bad[:3]
    assert len(j["states"]) == 768
    bad_regen = [x for x in j["regens"] if canon_regen(x[2], x[4], False) != canon_regen(x[3], x[4], False)]
    assert not bad_regen, bad_regen[:2]
    assert len(j["regens"]) == 658
