"""Local ops and acks: documents whose own client sends
(MTE_DOC_LOCAL_CLIENT) take MTE_F_LOCAL records for insertSegmentLocal /
removeRangeLocal / annotateRangeLocal (client.ts:131-229) and MTE_OP_ACK
records for the sequenced messages of those ops (client.ts:918-935 ->
ackPendingSegment, mergeTree.ts:1278-1331).

Pinned two ways:
  * the reference's 30 conflict-farm fixtures with EVERY client on the engine
    (replay_farm): each non-observer client applies its round's ops locally,
    then every message (its own as acks) — 8,960 round checkpoints, all clients
    must show the fixture's resultText;
  * 40 farms the reference itself ran with lagging clients, pending ops meeting
    remote ones and property keys (tests/golden/farm_vectors.json.gz, made by
    tests/golden/make_farm_golden.py through oracle/ref_farm.js): every client's
    text and per-position properties at every checkpoint.
"""
import gzip
import json
import os

import pytest

from fixtures_util import doc_inits, replay_farm, replay_ref_farm
from fluidframework_amd.abi import (DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, MTE_E_STATE, MTE_E_UNSUPPORTED,
                                    MergeTreeError)
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner

HERE = os.path.dirname(os.path.abspath(__file__))
FARM = os.path.join(HERE, "golden", "farm_vectors.json.gz")


def farm_sets():
    with gzip.open(FARM, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def oracle_factory(k):
    from oracle import OracleEngine
    return OracleEngine(k)


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def test_oracle_farm_fixtures_every_client():
    passed, failures, _ = replay_farm(oracle_factory)
    assert not failures, failures[:3]
    assert passed == 8960


def test_oracle_reference_farms():
    sets = farm_sets()
    passed, failures = replay_ref_farm(oracle_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def test_reference_farm_live():
    """Re-run the reference farm generator here and compare with the committed
    vectors (build container only: the reference does not travel)."""
    import ref_util
    if not ref_util.ref_available():
        pytest.skip("reference sources not in this container")
    import subprocess
    sets = farm_sets()[:3]
    inp = {"sets": [{k: s[k] for k in ("seed", "clients", "steps", "initialText", "nCheckpoints", "maxText")}
                    for s in sets]}
    p = subprocess.run(["node", os.path.join(os.path.dirname(HERE), "oracle", "ref_farm.js"), ref_util.build_ref()],
                       input=json.dumps(inp), capture_output=True, text=True, timeout=600, check=True)
    live = json.loads(p.stdout)["sets"]
    for a, b in zip(live, sets):
        assert a["log"] == b["log"] and a["events"] == b["events"] and a["checkpoints"] == b["checkpoints"]


def test_packer_local_rules():
    it = Interner(4)
    bb = BatchBuilder(1, it)
    obs = DocClients("A")
    with pytest.raises(MergeTreeError) as e:
        bb.add_local(0, obs, {"type": 0, "pos1": 0, "seg": "x"})
    assert e.value.code == MTE_E_UNSUPPORTED
    loc = DocClients("B", local=True)
    msg = {"clientId": "B", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
           "type": "op", "contents": {"type": 0, "pos1": 0, "seg": "x"}}
    with pytest.raises(MergeTreeError) as e:
        bb.add_message(0, loc, msg)  # an ack with nothing pending
    assert e.value.code == MTE_E_STATE
    with pytest.raises(MergeTreeError) as e:
        bb.add_local(0, loc, {"type": 2, "pos1": 0, "pos2": 1, "props": {"a": 1},
                              "combiningOp": {"name": "rewrite"}})
    assert e.value.code == MTE_E_UNSUPPORTED
    assert loc.local_seq == 0 and not loc.pending  # nothing taken by the rejected op
    bb.add_local(0, loc, {"type": 3, "ops": [{"type": 0, "pos1": 0, "seg": "ab"},
                                             {"type": 1, "pos1": 0, "pos2": 1}]})
    assert loc.pending == [(1, 2)]
    bb.add_message(0, loc, dict(msg, contents={"type": 3, "ops": []}))
    b = bb.build()
    assert list(b["ops"]["type"]) == [0, 1, 4]
    assert list(b["ops"]["seq"][:2]) == [1, 2] and (b["ops"]["flags"][:2] & 0x8).all()
    assert (b["ops"]["pos1"][2], b["ops"]["pos2"][2]) == (1, 2)


def _scenario(factory):
    """A hand-built case: B inserts locally while C's concurrent insert at the
    same position arrives first; B's pending segment stays before C's
    (breakTie, mergeTree.ts:1705-1721) and the ack keeps it there."""
    inits, text = doc_inits(["ab"], flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT)
    it = Interner(4)
    e = factory(4)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, it)
    bb.add_local(0, cl, {"type": 0, "pos1": 1, "seg": "BB"})
    bb.add_local(0, cl, {"type": 2, "pos1": 0, "pos2": 4, "props": {"k": 1}})
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": 1, "seg": "CC"}})
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 2, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op",
                           "contents": {"type": 2, "pos1": 0, "pos2": 2, "props": {"k": 2, "j": 3}}})
    e.apply_batch(bb.build())
    v1 = e.read_doc(0)
    bb = BatchBuilder(1, it)
    for s, c in ((3, {"type": 0, "pos1": 1, "seg": "BB"}), (4, {"type": 2, "pos1": 0, "pos2": 4, "props": {"k": 1}})):
        bb.add_message(0, cl, {"clientId": "B", "sequenceNumber": s, "referenceSequenceNumber": 0,
                               "minimumSequenceNumber": 0, "type": "op", "contents": c})
    e.apply_batch(bb.build())
    v2 = e.read_doc(0)
    return e, it, v1, v2


def test_oracle_local_scenario():
    e, it, v1, v2 = _scenario(oracle_factory)
    assert (e.statuses() == 0).all()
    assert v1["text"] == "aBBCCb" and v2["text"] == "aBBCCb"
    # k stays B's own pending value where B annotated; j (not pending) is C's
    props = [it.decode_props(p) for _, _, p in v2["segs"]]
    assert props[0] == {"k": 1, "j": 3} and props[1] == {"k": 1}


@pytest.mark.gpu
def test_gpu_local_scenario():
    e, it, v1, v2 = _scenario(device_factory)
    assert (e.statuses() == 0).all()
    assert v1["text"] == "aBBCCb" and v2["text"] == "aBBCCb"
    props = [it.decode_props(p) for _, _, p in v2["segs"]]
    assert props[0] == {"k": 1, "j": 3} and props[1] == {"k": 1}


@pytest.mark.gpu
def test_gpu_farm_fixtures_every_client():
    passed, failures, eng = replay_farm(device_factory)
    assert not failures, failures[:3]
    assert passed == 8960


@pytest.mark.gpu
def test_gpu_reference_farms():
    sets = farm_sets()
    passed, failures = replay_ref_farm(device_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
