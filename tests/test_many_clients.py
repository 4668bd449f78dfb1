"""More than 31 clients sending inside one collab window (SURVEY.md 8(a) row
a2, getOrAddShortClientId, client.ts:683-698: the reference numbers clients
without a cap).  The engine's short ids are slots a host recycles once the
window's minSeq passed every seq their client used (DocClients), so only the
clients sending inside one window need distinct slots; removedClientIds is a
bitmask over them.  The flat passes hold it in one 32-bit plane
(MTE_MAX_CLIENTS = 32); the documents the HBM tree pass replays --
MTE_DOC_LOCAL_CLIENT and MTE_DOC_TREE ones -- hold the upper half in a plane of
their own (mte_htree.h kRmHiPlane; titems.c item.rmask is 64 bits), so they
take MTE_MAX_CLIENTS_TREE = 64.

Pinned by 20 farms the reference itself ran with 34 to 56 clients
(tests/golden/many_clients_vectors.json.gz, tests/golden/make_farm_golden.py
--many; rollbacks, references and the legacy length calculation among them):
at their busiest 34 to 56 short ids are needed at once (window_senders).  Every
client of every farm as a local-client document (3,536 client checkpoints)
and every observer of the farms without references as a remote-only
MTE_DOC_TREE document equal the reference, on the restatement, the GPU and
through Node.  A mutation that drops the removers of short ids >= 32 from the
visibility rule fails 812 of the 3,536.
"""
import gzip
import json
import os
import subprocess

import pytest

from fixtures_util import doc_inits, replay_ref_farm
from fluidframework_amd.abi import (DOC_NEW_LENGTH_CALC, DOC_TREE, MTE_E_CLIENT_RANGE,
                                    MTE_E_UNSUPPORTED, MTE_MAX_CLIENTS, MTE_MAX_CLIENTS_TREE, MergeTreeError)
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
VECTORS = os.path.join(HERE, "golden", "many_clients_vectors.json.gz")


def many_sets():
    with gzip.open(VECTORS, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def window_senders(log):
    # as tests/golden/make_farm_golden.py: the short ids a document needs at once
    last, msn, most = {}, 0, 0
    for cid, seq, _ref, m, _t, _c in log:
        last[cid] = seq
        most = max(most, sum(1 for v in last.values() if v > msn) + 1)
        msn = max(msn, m)
    return most


def tree_factory(k):
    from oracle import OracleEngine
    e = OracleEngine(k, tree="items")
    e.lib.oti_set_limit(e.ctx, 1 << 20)
    return e


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def _local(factory):
    sets = many_sets()
    passed, failures = replay_ref_farm(factory, sets, exact_regen=True)
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets) == 3536


def _observers(factory):
    sets = [s for s in many_sets() if not s.get("refs")]
    passed, failures = replay_ref_farm(factory, sets, observers_only=True, extra_flags=DOC_TREE)
    assert not failures, failures[:2]
    assert passed == sum(len(s["checkpoints"]) for s in sets) == 64


def test_many_clients_vectors_shape():
    sets = many_sets()
    assert len(sets) == 20
    most = [window_senders(s["log"]) for s in sets]
    assert all(m > MTE_MAX_CLIENTS for m in most) and max(most) == 56 <= MTE_MAX_CLIENTS_TREE
    assert sum(1 for s in sets if s.get("legacy")) == 4 and sum(1 for s in sets if s.get("refs")) == 4


def test_tree_oracle_many_clients_every_client():
    _local(tree_factory)


def test_tree_oracle_many_clients_remote_only_tree_documents():
    _observers(tree_factory)


def test_flat_documents_keep_32_short_ids():
    """A document of remote clients alone not flagged MTE_DOC_TREE replays on
    the flat passes: its packer refuses the 33rd client inside the window."""
    s = next(s for s in many_sets() if not s.get("refs") and not s.get("legacy"))
    with pytest.raises(MergeTreeError) as ei:
        replay_ref_farm(tree_factory, [s], observers_only=True)
    assert ei.value.code == MTE_E_CLIENT_RANGE
    assert DocClients("A").max_clients == MTE_MAX_CLIENTS
    assert DocClients("A", local=True).max_clients == DocClients("A", tree=True).max_clients == MTE_MAX_CLIENTS_TREE


def _wide_remover(factory):
    """40 clients insert one segment each into "abc" with refSeq 0, then the
    40th removes the first one's: its remover has short id 40, which the
    segment read-out (mte_seg.removers, 32 bits) cannot carry."""
    inits, text = doc_inits(["abc"], flags=DOC_NEW_LENGTH_CALC | DOC_TREE)
    e = factory(0)
    e.load_docs(inits, text)
    cl = DocClients("obs", tree=True)
    bb = BatchBuilder(1, Interner(0))
    for i in range(40):
        bb.add_message(0, cl, {"clientId": f"c{i}", "sequenceNumber": i + 1, "referenceSequenceNumber": 0,
                               "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": 0,
                                                                                     "seg": "x"}})
    bb.add_message(0, cl, {"clientId": "c39", "sequenceNumber": 41, "referenceSequenceNumber": 40,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 39, "pos2": 40}})
    e.apply_batch(bb.build())
    return e, cl


def test_tree_oracle_segment_readout_refuses_wide_removers():
    e, cl = _wide_remover(tree_factory)
    assert (e.statuses() == 0).all() and cl.ids["c39"] == 40
    assert e.read_doc(0)["text"] == "x" * 39 + "abc"
    with pytest.raises(MergeTreeError) as ei:
        e.read_segments(0)
    assert ei.value.code == MTE_E_UNSUPPORTED


def test_node_many_clients_on_restatement():
    p = subprocess.run(["node", os.path.join(ROOT, "tests", "node", "farm_gpu.js"), "batched", "all",
                        "many_clients_vectors.json.gz"], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, MTE_NODE_ADDON="oracle"))
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(p.stdout)
    assert j["nFailures"] == 0, j["failures"]
    assert j["passed"] == 3536


@pytest.mark.gpu
def test_gpu_many_clients_every_client():
    _local(device_factory)


@pytest.mark.gpu
def test_gpu_many_clients_remote_only_tree_documents():
    _observers(device_factory)


@pytest.mark.gpu
def test_gpu_segment_readout_refuses_wide_removers():
    e, cl = _wide_remover(device_factory)
    assert (e.statuses() == 0).all()
    assert e.read_doc(0)["text"] == "x" * 39 + "abc"
    with pytest.raises(MergeTreeError) as ei:
        e.read_segments(0)
    assert ei.value.code == MTE_E_UNSUPPORTED


@pytest.mark.gpu
def test_node_many_clients_on_gpu():
    p = subprocess.run(["node", os.path.join(ROOT, "tests", "node", "farm_gpu.js"), "batched", "all",
                        "many_clients_vectors.json.gz"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    j = json.loads(p.stdout)
    assert j["nFailures"] == 0, j["failures"]
    assert j["passed"] == 3536
