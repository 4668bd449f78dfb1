"""Local references: LocalReferenceCollection
(localReference.ts:139-567) in MTE_DOC_REFS documents -- references created at
a position of the local view (createLocalReferencePosition on
getContainingSegment, client.ts:360-364, 1107-1110), removed
(removeLocalReferencePosition), carried across splits, and slid when their
segment becomes removed and acked (slideAckedRemovedSegmentReferences,
mergeTree.ts:893-950): SlideOnRemove to the next segment that is neither
removed-and-acked nor a pending insert, else the previous one, else detached;
Simple ones detach.  Positions through mte_read_refs
(localReferencePositionToPosition, mergeTree.ts:1095-1112).

Pinned by 40 farms the reference itself ran (oracle/ref_farm.js with refs ->
tests/golden/localref_vectors.json.gz, made by tests/golden/make_farm_golden.py
--refs): every client -- the observer included -- creates and removes
references while editing, with lagging refSeqs, rollbacks and annotates; at
every checkpoint every reference's position must equal the reference
client's.  Two mutations of the slide rule (pending inserts as targets, no
backward slide) fail 219 and 327 of the 880 checkpoints.

StayOnRemove references (localReference.ts:434, 469: they stay on their
removed segment, at its position) are pinned by 32 more farms
(tests/golden/localref_stay_vectors.json.gz, make_farm_golden.py --stay):
there the reference's lazy zamboni (mergeTree.ts:680-705) decides when such a
reference reads detached -- the unlink of its tombstone -- so they hold for
the local-client documents' tree pass (titems.c, mte_htree.h), which keeps that
zamboni; the flat restatement's compaction at minSeq detaches them at other
times and is not held to them.

Transient references (localReference.ts:263: createLocalReferencePosition
keeps the segment and offset but never adds the reference to the segment's
list, so nothing slides or detaches it; localReferencePositionToPosition
reads its segment's position, plus the offset while the segment is not
removed, -1 once the segment is unlinked) are pinned by 24 more farms
(tests/golden/localref_transient_vectors.json.gz, make_farm_golden.py
--transient), again for the tree pass: anchored by the leaf id of their
segment, which splits never move (a split leaves the id on the head).  Two
wrong rules fail them: anchoring by text unit (the reference follows a split
into its tail) fails 12 of the 734 checkpoints, keeping the offset on a
removed segment 283.
"""
import gzip
import json
import os

import numpy as np
import pytest

from fixtures_util import doc_inits, replay_ref_farm
from fluidframework_amd.abi import (DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, DOC_REFS, MTE_E_CAPACITY, MTE_E_INVALID_ARG,
                                    MTE_E_UNSUPPORTED, REF_SLIDE_ON_REMOVE, REF_STAY_ON_REMOVE, REF_TRANSIENT,
                                    MergeTreeError)
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner

HERE = os.path.dirname(os.path.abspath(__file__))
VECTORS = os.path.join(HERE, "golden", "localref_vectors.json.gz")
STAY_VECTORS = os.path.join(HERE, "golden", "localref_stay_vectors.json.gz")
TRANSIENT_VECTORS = os.path.join(HERE, "golden", "localref_transient_vectors.json.gz")


def ref_sets(path=VECTORS):
    with gzip.open(path, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def tree_factory(k):
    from oracle import OracleEngine
    e = OracleEngine(k, tree="items")
    e.lib.oti_set_limit(e.ctx, 1 << 20)
    return e


def oracle_factory(k):
    from oracle import OracleEngine
    return OracleEngine(k)


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def test_localref_vectors_shape():
    sets = ref_sets()
    assert len(sets) == 40
    n_refs = sum(1 for s in sets for ev in s["events"] for e in ev if e[0] == "F")
    n_rm = sum(1 for s in sets for ev in s["events"] for e in ev if e[0] == "X")
    assert n_refs > 2000 and n_rm > 300
    # the references slid, detached (-1) and were removed (null) at checkpoints
    vals = [p for s in sets for cp in s["checkpoints"] for st in cp["states"] for p in st["refs"]]
    assert vals.count(-1) > 50 and vals.count(None) > 300


def test_oracle_localref_farms():
    sets = ref_sets()
    passed, failures = replay_ref_farm(oracle_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def test_stay_vectors_shape():
    sets = ref_sets(STAY_VECTORS)
    assert len(sets) == 32 and all(s["stay"] > 0 for s in sets)
    made = [e for s in sets for ev in s["events"] for e in ev if e[0] == "F"]
    assert len(made) > 3000 and sum(1 for e in made if e[2] == REF_STAY_ON_REMOVE) > 1400
    vals = [p for s in sets for cp in s["checkpoints"] for st in cp["states"] for p in st["refs"]]
    assert vals.count(-1) > 2000 and vals.count(None) > 3000


def test_tree_oracle_stay_farms():
    """The tree restatement equals the reference at every checkpoint of the
    StayOnRemove farms, and the flat restatement, whose compaction at minSeq is
    not the reference's lazy zamboni, does not (so the farms do reach the
    unlink of a tombstone holding a StayOnRemove reference)."""
    sets = ref_sets(STAY_VECTORS)
    total = sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
    passed, failures = replay_ref_farm(tree_factory, sets)
    assert not failures, failures[:2]
    assert passed == total
    _, flat_failures = replay_ref_farm(oracle_factory, sets)
    assert len(flat_failures) > 50


@pytest.mark.gpu
def test_gpu_stay_farms():
    sets = ref_sets(STAY_VECTORS)
    passed, failures = replay_ref_farm(device_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def test_transient_vectors_shape():
    sets = ref_sets(TRANSIENT_VECTORS)
    assert len(sets) == 24 and all(s["transient"] > 0 for s in sets)
    made = [e for s in sets for ev in s["events"] for e in ev if e[0] == "F"]
    assert len(made) > 2000 and sum(1 for e in made if e[2] & REF_TRANSIENT) > 500
    vals = [p for s in sets for cp in s["checkpoints"] for st in cp["states"] for p in st["refs"]]
    assert vals.count(-1) > 1000 and vals.count(None) > 1000


def test_tree_oracle_transient_farms():
    """The tree restatement equals the reference at every checkpoint of the
    Transient farms; the flat restatement refuses Transient references."""
    sets = ref_sets(TRANSIENT_VECTORS)
    passed, failures = replay_ref_farm(tree_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


@pytest.mark.gpu
def test_gpu_transient_farms():
    sets = ref_sets(TRANSIENT_VECTORS)
    passed, failures = replay_ref_farm(device_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def _transient_scenario(factory):
    """"abcdef" as "abc" + "def" (two segments); a Transient reference on 'e'
    (segment "def", offset 1) and one on 'b'; a remote insert of "XY" at 4
    splits "def" -- the reference stays on the head "d", offset 1, so it reads
    4 ('X', not 'e': nothing moves a Transient reference); a remote remove of
    [0, 3) makes 'b''s read its removed segment's position, offset dropped,
    and 'd''s 0 + 1.  The flat restatement refuses Transient references."""
    inits, text = doc_inits(["abc"], flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS)
    e = factory(4)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, Interner(4))
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": 3, "seg": "def"}})
    e.apply_batch(bb.build())
    bb = BatchBuilder(1, Interner(4))
    bb.add_ref(0, cl, 4, REF_TRANSIENT)
    bb.add_ref(0, cl, 1, REF_TRANSIENT)
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 2, "referenceSequenceNumber": 1,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": 4, "seg": "XY"}})
    e.apply_batch(bb.build())
    mid = list(e.read_refs(0, 2))
    bb = BatchBuilder(1, Interner(4))
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 3, "referenceSequenceNumber": 2,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 0, "pos2": 3}})
    e.apply_batch(bb.build())
    return e, mid, list(e.read_refs(0, 2)), list(e.read_refs(0, 2, transient=True))


def test_tree_oracle_transient_scenario():
    e, mid, end, end_t = _transient_scenario(tree_factory)
    assert (e.statuses() == 0).all()
    assert mid == [4, 1] and end == [1, 0] and end_t == end
    assert list(_transient_scenario(oracle_factory)[0].statuses()) == [MTE_E_UNSUPPORTED]


@pytest.mark.gpu
def test_gpu_transient_scenario():
    e, mid, end, end_t = _transient_scenario(device_factory)
    assert (e.statuses() == 0).all()
    assert mid == [4, 1] and end == [1, 0] and end_t == end


def test_localref_farm_live():
    """The committed vectors are what the erased reference computes now (build
    container only: the reference does not travel)."""
    import subprocess
    import ref_util
    if not ref_util.ref_available():
        pytest.skip("reference sources not in this container")
    keys = ("seed", "clients", "steps", "initialText", "nCheckpoints", "maxText", "rollback", "refs", "rollbackTypes",
            "stay", "transient")
    for s in ref_sets()[:4] + ref_sets(STAY_VECTORS)[:2] + ref_sets(TRANSIENT_VECTORS)[:2]:
        inp = {"sets": [{k: s[k] for k in keys if k in s}]}
        p = subprocess.run(["node", os.path.join(os.path.dirname(HERE), "oracle", "ref_farm.js"), ref_util.build_ref()],
                           input=json.dumps(inp), capture_output=True, text=True, timeout=600, check=True)
        live = json.loads(p.stdout)["sets"][0]
        assert live["log"] == s["log"] and live["events"] == s["events"] and live["checkpoints"] == s["checkpoints"]


def _scenario(factory):
    """Hand-built: "abcdef"; a SlideOnRemove reference on 'c' (2) and a Simple one
    on 'd' (3); a remote remove of [2, 4) slides the first to 'e' (offset 0)
    and detaches the second; a reference on 'f' (5) whose segment a later
    remote remove of [4, 6) takes with nothing after it slides back to 'b'."""
    inits, text = doc_inits(["abcdef"], flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS)
    it = Interner(4)
    e = factory(4)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, it)
    r1 = bb.add_ref(0, cl, 2, REF_SLIDE_ON_REMOVE)
    r2 = bb.add_ref(0, cl, 3, 0)
    r3 = bb.add_ref(0, cl, 5, REF_SLIDE_ON_REMOVE)
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 2, "pos2": 4}})
    e.apply_batch(bb.build())
    mid = list(e.read_refs(0, 3))
    bb = BatchBuilder(1, it)
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 2, "referenceSequenceNumber": 1,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 2, "pos2": 4}})
    e.apply_batch(bb.build())
    end = list(e.read_refs(0, 3))
    return e, (r1, r2, r3), mid, end


def test_oracle_localref_scenario():
    e, slots, mid, end = _scenario(oracle_factory)
    assert (e.statuses() == 0).all() and slots == (0, 1, 2)
    assert mid == [2, -1, 3] and end == [1, -1, 1]


@pytest.mark.gpu
def test_gpu_localref_scenario():
    e, slots, mid, end = _scenario(device_factory)
    assert (e.statuses() == 0).all()
    assert mid == [2, -1, 3] and end == [1, -1, 1]


def _off_scenario(factory):
    """A remote remove of the whole text "abc" leaves no segment to slide to:
    the SlideOnRemove reference on 'b' and the Simple one on 'c' come off the
    removed segment's list but keep pointing at it (mergeTree.ts:935-942) --
    detached for localReferencePositionToPosition, the segment's position (0,
    offset 0 on a removed segment) read as Transient references
    (mte_read_refs_transient, mergeTree.ts:1106-1109).  The Simple reference
    of _scenario, detached beside a segment to slide to (link(undefined),
    localReference.ts:447-449), stays detached either way."""
    inits, text = doc_inits(["abc"], flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS)
    e = factory(4)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, Interner(4))
    bb.add_ref(0, cl, 1, REF_SLIDE_ON_REMOVE)
    bb.add_ref(0, cl, 2, 0)
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 0, "pos2": 3}})
    e.apply_batch(bb.build())
    e2 = _scenario(factory)[0]
    return (e, list(e.read_refs(0, 2)), list(e.read_refs(0, 2, transient=True)),
            list(e2.read_refs(0, 3, transient=True)))


def test_oracle_refs_off_the_string_transient():
    e, plain, transient, simple = _off_scenario(oracle_factory)
    assert (e.statuses() == 0).all()
    assert plain == [-1, -1] and transient == [0, 0] and simple == [1, -1, 1]


@pytest.mark.gpu
def test_gpu_refs_off_the_string_transient():
    e, plain, transient, simple = _off_scenario(device_factory)
    assert (e.statuses() == 0).all()
    assert plain == [-1, -1] and transient == [0, 0] and simple == [1, -1, 1]


@pytest.mark.gpu
def test_gpu_localref_farms():
    sets = ref_sets()
    passed, failures = replay_ref_farm(device_factory, sets)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def test_packer_ref_rules():
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, Interner(4))
    for bad in (REF_STAY_ON_REMOVE | REF_SLIDE_ON_REMOVE, REF_TRANSIENT | REF_SLIDE_ON_REMOVE):
        with pytest.raises(MergeTreeError) as ei:
            bb.add_ref(0, cl, 0, bad)
        assert ei.value.code == MTE_E_INVALID_ARG
    assert bb.add_ref(0, cl, 0) == 0 and bb.add_ref(0, cl, 1) == 1 and bb.add_ref(0, cl, 1, REF_TRANSIENT) == 2
    bb.remove_ref(0, cl, 0)
    assert bb.add_ref(0, cl, 2) == 0  # a removed slot is reused
    with pytest.raises(MergeTreeError) as ei:
        bb.remove_ref(0, cl, 5)
    assert ei.value.code == MTE_E_INVALID_ARG
    with pytest.raises(MergeTreeError):
        bb.add_ref(0, DocClients("A"), 0)  # observer documents have no local view


def test_packer_ref_capacity_refuses_only_that_document():
    # a slot >= the context's ref capacity made mte_submit fail the
    # whole batch; the packer now refuses the reference for its document alone
    cl, other = DocClients("B", local=True), DocClients("B", local=True)
    cl.ref_cap = other.ref_cap = 3
    bb = BatchBuilder(2, Interner(4))
    assert [bb.add_ref(0, cl, i) for i in range(3)] == [0, 1, 2]
    with pytest.raises(MergeTreeError) as ei:
        bb.add_ref(0, cl, 0)
    assert ei.value.code == MTE_E_CAPACITY
    assert bb.add_ref(1, other, 0) == 0  # the other document is unaffected
    bb.remove_ref(0, cl, 1)
    assert bb.add_ref(0, cl, 0) == 1  # a freed slot is below the capacity


def test_oracle_rejects_refs_outside_refs_docs():
    inits, text = doc_inits(["abc"], flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT)
    e = oracle_factory(0)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, Interner(0))
    bb.add_ref(0, cl, 1)
    with pytest.raises(MergeTreeError):
        e.apply_batch(bb.build())


def test_engine_ref_capacity_reaches_the_packer():
    """set_ref_capacity is what the document's client map checks
    (EngineBase.doc_clients), below and above the default of 1,024."""
    e = oracle_factory(0)
    for cap in (5, 4096):
        e.set_ref_capacity(cap)
        cl = e.doc_clients("B", local=True)
        assert cl.ref_cap == cap
        bb = BatchBuilder(1, Interner(0))
        for i in range(cap):
            assert bb.add_ref(0, cl, 0) == i
        with pytest.raises(MergeTreeError) as ei:
            bb.add_ref(0, cl, 0)
        assert ei.value.code == MTE_E_CAPACITY


@pytest.mark.gpu
def test_gpu_engine_ref_capacity_reaches_the_packer():
    from fluidframework_amd.engine import DeviceEngine
    e = DeviceEngine(0)
    e.set_ref_capacity(7)
    assert e.doc_clients("B", local=True).ref_cap == 7


def _slide_events(factory, slide_events, per_op=None):
    """A remote group op whose first member removes 'c' under 300 SlideOnRemove
    references (they slide to 'd') and whose second removes 'e' under 2 (to
    'f'), in an MTE_DOC_REFS | MTE_DOC_EVENTS document with or without
    MTE_DOC_SLIDE_EVENTS (slide records are opt-in, so a host that
    does not read them keeps the old event capacity)."""
    from fluidframework_amd.abi import DOC_EVENTS, DOC_SLIDE_EVENTS
    flags = DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS | DOC_EVENTS | (DOC_SLIDE_EVENTS if slide_events else 0)
    inits, text = doc_inits(["abcdefgh"], flags=flags)
    e = factory(4)
    if per_op is not None:
        e.set_event_capacity(per_op)
    e.load_docs(inits, text)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, Interner(4))
    for _ in range(300):
        bb.add_ref(0, cl, 2, REF_SLIDE_ON_REMOVE)
    bb.add_ref(0, cl, 4, REF_SLIDE_ON_REMOVE)
    bb.add_ref(0, cl, 4, REF_SLIDE_ON_REMOVE)
    bb.add_message(0, cl, {"clientId": "C", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op",
                           "contents": {"type": 3, "ops": [{"type": 1, "pos1": 2, "pos2": 3},
                                                           {"type": 1, "pos1": 3, "pos2": 4}]}})
    e.apply_batch(bb.build())
    return e


def test_tree_oracle_slide_records_are_opt_in():
    """slide records are opt-in (MTE_DOC_SLIDE_EVENTS), so a
    document that does not ask for them keeps the old event volume; one that
    does gets them with every reference's snapshot after each record that slid
    one."""
    from fluidframework_amd.abi import DELTA_REFPOS, DELTA_SLIDE
    e = _slide_events(tree_factory, False)
    assert (e.statuses() == 0).all()
    d = e.read_deltas(0)
    assert len(d) == 2 and set(d["kind"] & 0xff) == {1}  # the two removes' ranges only
    e = _slide_events(tree_factory, True)
    d = e.read_deltas(0)
    k = d["kind"] & 0xff
    assert (k == 1).sum() == 2
    slides, snaps = d[(k & 0xc0) == DELTA_SLIDE], d[k == DELTA_REFPOS]
    assert len(slides) == 302 and len(snaps) == 2 * 302  # one snapshot per record that slid
    # the snapshot after the first member: the 300 references on 'd' at 2
    # ("abdefgh"), the 2 on 'e' at 3; after the second: on 'd' at 2, on 'f' at 3
    first, second = snaps[snaps["op"] == snaps["op"].min()], snaps[snaps["op"] == snaps["op"].max()]
    assert (first["pos"][:300] == 2).all() and (first["pos"][300:] == 3).all()
    assert (second["pos"][:300] == 2).all() and (second["pos"][300:] == 3).all()
    assert list(e.read_refs(0, 302)) == [2] * 300 + [3, 3]
    # order keys: 'd' is held unit 3 ("abcdefgh" with 'c' still held), 'f' unit 5
    assert (first["len"][:300] == 3).all() and (second["len"][300:] == 5).all()


@pytest.mark.gpu
def test_gpu_slide_records_opt_in_and_capacity():
    from fluidframework_amd.abi import DELTA_REFPOS
    e = _slide_events(device_factory, False, per_op=1)
    assert (e.statuses() == 0).all() and len(e.read_deltas(0)) == 2  # fits: slides not recorded
    # with slide events the region grows by 2 x the reference slots in use for
    # each remote remove (908 records > 1 x 304 + 256, < that + 2 x 2 x 302)
    e = _slide_events(device_factory, True, per_op=1)
    t = _slide_events(tree_factory, True)
    np.testing.assert_array_equal(e.read_deltas(0), t.read_deltas(0))  # record for record
    assert (e.read_deltas(0)["kind"] & 0xff == DELTA_REFPOS).sum() == 604
