"""Reconnection of pending interval-collection ops (rebaseLocalInterval,
intervalCollection.ts:1735-1803): MTE_OP_REF records with b = 4 --
Client.rebasePosition (client.ts:755-786) from the view the op was made in
(refSeq = its sequenceNumber, localSeq = its own) to the current one -- and
b = 5 -- the slide of a pending interval end whose segment a remote remove
took (:1782-1799).  Both answer with an MTE_DELTA_REBASE event.

Hand-built documents on the restatement of the HBM tree pass (oracle/titems.c)
and on the device; the interval farms with reconnection pin them against the
reference (tests/test_intervals.py)."""
import pytest

from fixtures_util import doc_inits
from fluidframework_amd.abi import (DELTA_REBASE, DOC_EVENTS, DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, DOC_REFS,
                                    MTE_E_INVALID_ARG, REF_STAY_ON_REMOVE, MergeTreeError)
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner

FLAGS = DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS | DOC_EVENTS


def titems(k):
    from oracle import OracleEngine
    return OracleEngine(k, tree="items")


def device(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def _msg(cid, seq, ref, contents, msn=0):
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


def _scenario(factory, full_remove=False):
    """"abcdef"; B (local) inserts "XY" at 2 (localSeq 1, pending) and puts a
    StayOnRemove reference on 'd' (5 in "abXYcdef"), as a pending interval end;
    C removes "cd" (seq 1, refSeq 0: [2, 4) of "abcdef"), D inserts "ZZ" at 0
    (seq 2).  Then the reconnection queries of an interval op B made at
    (seq 0, localSeq 1)."""
    inits, text = doc_inits(["abcdef"], flags=FLAGS)
    e = factory(4)
    e.load_docs(inits, text)
    it = Interner(4)
    cl = DocClients("B", local=True)
    bb = BatchBuilder(1, it)
    bb.add_local(0, cl, {"type": 0, "pos1": 2, "seg": "XY"})
    ref = bb.add_ref(0, cl, 5, REF_STAY_ON_REMOVE)
    bb.add_message(0, cl, _msg("C", 1, 0, {"type": 1, "pos1": 2, "pos2": 6 if full_remove else 4}))
    if full_remove:
        bb.add_message(0, cl, _msg("C", 2, 1, {"type": 1, "pos1": 0, "pos2": 2}))
    else:
        bb.add_message(0, cl, _msg("D", 2, 1, {"type": 0, "pos1": 0, "seg": "ZZ"}))
    e.apply_batch(bb.build())
    assert (e.statuses() == 0).all(), e.statuses()
    bb = BatchBuilder(1, it)
    bb.add_rebase(0, cl, 4, 0, 1)     # 'c' at (0, 1): removed since -> slides to 'e'
    bb.add_rebase(0, cl, 1, 0, 1)     # 'b': stays
    bb.add_rebase(0, cl, 100, 0, 1)   # past the end: the last leaf, offset 0
    bb.add_rebase(0, cl, 2, 0, 0)     # localSeq 0: 'c' (the pending "XY" not yet there) -> 'e'
    bb.add_ref_rebase(0, cl, ref, 1)  # the end on 'd' -> 'e'
    e.apply_batch(bb.build())
    ev = e.read_deltas(0)
    return e, ref, [(int(x["kind"]), int(x["pos"])) for x in ev], list(e.read_refs(0, ref + 1))


@pytest.mark.parametrize("factory", [titems, pytest.param(device, marks=pytest.mark.gpu)])
def test_rebase_positions_and_slide(factory):
    e, ref, ev, refs = _scenario(factory)
    assert (e.statuses() == 0).all()
    # "ZZ" + "ab" + "XY" + "ef": 'e' at 6, 'b' at 3; the last leaf "ef" at 6;
    # at localSeq 0 "XY" is not counted: 'e' at 4
    assert ev == [(DELTA_REBASE, 6), (DELTA_REBASE, 3), (DELTA_REBASE, 6), (DELTA_REBASE, 4), (DELTA_REBASE, 6)]
    assert refs[ref] == 6


@pytest.mark.parametrize("factory", [titems, pytest.param(device, marks=pytest.mark.gpu)])
def test_rebase_off_the_string(factory):
    """Everything acked is removed: only the pending "XY" is left, which no
    reference may slide to (a pending insert) -- positions detach (-1), the
    last leaf included, and the interval end cannot move (the reference would
    throw; it detaches)."""
    e, ref, ev, refs = _scenario(factory, full_remove=True)
    assert (e.statuses() == 0).all()
    assert ev == [(DELTA_REBASE, -1)] * 5
    assert refs[ref] == -1


def test_packer_rebase_rules():
    bb = BatchBuilder(1, Interner(4))
    cl = DocClients("B", local=True)
    with pytest.raises(MergeTreeError) as ei:
        bb.add_rebase(0, cl, 0, 0, 1)  # no local op yet: localSeq 1 is in the future
    assert ei.value.code == MTE_E_INVALID_ARG
    with pytest.raises(MergeTreeError):
        bb.add_ref_rebase(0, cl, 0, 0)  # no reference in slot 0
