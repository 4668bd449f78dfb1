"""SharedString interval collections: IntervalCollection
(packages/dds/sequence/src/intervalCollection.ts) in the Node host
(fluidframework_amd/node/intervals.js) over the engine's local references
(MTE_DOC_REFS): StayOnRemove ends for pending local adds / changes,
SlideOnRemove ends created in a sequenced op's perspective and slid at once
(MTE_OP_REF b = 2), the conversion at the ack (b = 3), pending changes per end,
pending property keys.

Pinned by 29 farms the reference itself ran with its own IntervalCollection
(oracle/ref_interval_farm.js -> tests/golden/interval_vectors.json.gz, made by
tests/golden/make_interval_golden.py): every interval op the host emits must be
the op the reference sent, and at every checkpoint every client's text and
intervals (id, start and end positions, properties) must equal the reference
client's -- on the restatement (the host's batches replayed, test below), on the
GPU through Python and through Node.
"""
import base64
import gzip
import json
import os
import subprocess

import numpy as np
import pytest

from fixtures_util import doc_inits
from fluidframework_amd.abi import (DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, DOC_REFS, OP_DTYPE, PROP_DTYPE,
                                    PROPSET_DTYPE)

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
VECTORS = os.path.join(HERE, "golden", "interval_vectors.json.gz")


def interval_sets():
    with gzip.open(VECTORS, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def node(*args, timeout=600):
    r = subprocess.run(["node", *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def _batch(b):
    dec = lambda k: base64.b64decode(b[k])  # noqa: E731
    return {"op_offsets": np.frombuffer(dec("offsets"), np.uint64).copy(),
            "ops": np.frombuffer(dec("ops"), OP_DTYPE).copy(),
            "text": np.frombuffer(dec("text"), np.uint16).copy(),
            "propsets": np.frombuffer(dec("propsets"), PROPSET_DTYPE).copy(),
            "props": np.frombuffer(dec("props"), PROP_DTYPE).copy()}


def replay_packed(factory, sets, lines):
    """The Node host's batches (tests/node/interval_farm.js pack) on an engine:
    every client's text and intervals at every checkpoint against the reference."""
    layout = [(si, ci) for si, s in enumerate(sets) for ci in range(len(s["names"]))]
    inits, text = doc_inits([sets[si]["initialText"] for si, _ in layout],
                            flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT | DOC_REFS)
    eng = factory(8)
    eng.load_docs(inits, text)
    passed, failures = 0, []
    for j, line in enumerate(lines):
        rec = json.loads(line)
        for b in rec["batches"]:
            eng.apply_batch(_batch(b))
        st = eng.statuses()
        for d, (si, ci) in enumerate(layout):
            have = rec["states"][d]
            if have is None:
                continue
            want = sets[si]["checkpoints"][j]["states"][ci]
            if st[d] != 0:
                failures.append((si, ci, j, "status", int(st[d])))
                continue
            pos = eng.read_refs(d, have["nRefs"]) if have["nRefs"] else []
            got = [[i, int(pos[a]), int(pos[b]), p] for i, a, b, p in have["intervals"]]
            if eng.read_doc(d)["text"] != want["text"] or got != want["intervals"]:
                failures.append((si, ci, j, "state", got[:3], want["intervals"][:3]))
            else:
                passed += 1
    return passed, failures


@pytest.fixture(scope="module")
def packed():
    out = node("tests/node/interval_farm.js", "pack").splitlines()
    tail = json.loads(out[-1])
    return out[:-1], tail


def test_interval_vectors_shape():
    sets = interval_sets()
    assert len(sets) == 29
    ops = [e[5]["opName"] for s in sets for e in s["log"] if e[4] == "iv"]
    assert len(ops) > 4000 and {"add", "change", "delete"} <= set(ops)
    ends = [x for s in sets for cp in s["checkpoints"] for st in cp["states"] for iv in st["intervals"]
            for x in iv[1:3]]
    assert ends.count(-1) > 0  # ends that slid off the string


def test_host_emits_the_reference_interval_ops(packed):
    _, tail = packed
    assert tail["nFailures"] == 0, tail["failures"]
    assert tail["opsChecked"] > 2000


def test_oracle_interval_farms(packed):
    from oracle import OracleEngine
    sets = interval_sets()
    passed, failures = replay_packed(lambda k: OracleEngine(k), sets, packed[0])
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def test_interval_farm_live():
    """The committed vectors are what the erased reference computes now (build
    container only)."""
    import ref_util
    if not ref_util.ref_available():
        pytest.skip("reference sources not in this container")
    keys = ("seed", "clients", "steps", "initialText", "nCheckpoints", "maxText", "intervals")
    for s in interval_sets()[:3]:
        p = subprocess.run(["node", os.path.join(ROOT, "oracle", "ref_interval_farm.js"), ref_util.build_ref()],
                           input=json.dumps({"sets": [{k: s[k] for k in keys}]}), capture_output=True, text=True,
                           timeout=600, check=True)
        live = json.loads(p.stdout)["sets"][0]
        assert live["log"] == s["log"] and live["checkpoints"] == s["checkpoints"]


@pytest.mark.gpu
def test_gpu_interval_farms(packed):
    from fluidframework_amd.engine import DeviceEngine
    sets = interval_sets()
    passed, failures = replay_packed(lambda k: DeviceEngine(k), sets, packed[0])
    assert not failures, failures[:2]
    assert passed == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


@pytest.mark.gpu
def test_node_interval_farms_on_gpu():
    j = json.loads(node("tests/node/interval_farm.js", "gpu").strip().splitlines()[-1])
    assert j["nFailures"] == 0, j["failures"]
    sets = interval_sets()
    assert j["passed"] == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)


def ext_sets():
    with gzip.open(os.path.join(HERE, "golden", "interval_ext_vectors.json.gz"), "rt", encoding="utf-8") as fh:
        return json.load(fh)


def test_interval_ext_vectors_shape():
    v = ext_sets()
    sets = v["sets"]
    assert len(sets) == 11 and [x[0] for x in v["seeds_the_reference_failed"]] == [9508]
    states = [st for s in sets for cp in s["checkpoints"] for st in cp["states"]]
    assert all({"events", "order", "summary", "queries"} <= set(st) for st in states)
    kinds = {(e[0], e[-1]) for st in states for e in st["events"]}
    assert {("add", False), ("delete", False), ("change", False), ("props", False), ("change", True)} <= kinds


@pytest.mark.gpu
def test_node_interval_events_order_queries_summaries_on_gpu():
    """IntervalCollection events (addInterval / deleteInterval / changeInterval /
    propertyChanged, except those a merge-tree op raises), the tree's order,
    serializeInternal() and findOverlappingIntervals / previousInterval /
    nextInterval / the position iterators equal the reference's at every
    checkpoint of the ext farms, and every loadable final summary loads into a
    fresh client with the reference's intervals.  The changeInterval events an
    end sliding inside a merge-tree op raises are compared with the rest of
    the list (mtEvents)."""
    j = json.loads(node("tests/node/interval_farm.js", "ext").strip().splitlines()[-1])
    assert j["nFailures"] == 0, (j["extFail"], j["extFirst"], j["failures"][:2])
    sets = ext_sets()["sets"]
    assert j["passed"] == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
    assert j["loaded"] + j["unloadable"] == len(sets) and j["loaded"] > 0
    # previousInterval / nextInterval read the end tree, restated as the
    # reference's red-black tree (node/rbtree.js): every query as the reference
    assert j["prevNext"]["equal"] == j["prevNext"]["n"], j["prevNext"]
    # the ends that slide inside a merge-tree op raise changeInterval there
    # (MTE_DELTA_SLIDE records): the whole event list, those included
    assert j["mtEvents"]["equal"] == j["mtEvents"]["n"], j["mtEvents"]
    assert j["orderOff"] == 0


def reconnect_sets():
    with gzip.open(os.path.join(HERE, "golden", "interval_reconnect_vectors.json.gz"), "rt", encoding="utf-8") as fh:
        return json.load(fh)


def test_interval_reconnect_vectors_shape():
    """The reference's reconnection farms (make_interval_golden.py --reconnect):
    clients go offline, hold merge-tree and interval ops, and re-send them in
    order -- regeneratePendingOp ("G") and rebaseLocalInterval ("K") -- among
    remote edits; seeds whose reference run threw (a rebased interval end with
    no segment at its slide position, "Non-transient references need segment",
    or its own end-tree crash) are listed, not kept."""
    v = reconnect_sets()
    sets = v["sets"]
    assert len(sets) == 33 and len(v["seeds_the_reference_failed"]) == 31
    # localSeq views: the reference's (block partial lengths) against its own leaf rule
    lv = [s["leafViews"] for s in sets]
    assert sum(x["calls"] for x in lv) > 6000 and 0 < sum(x["differ"] for x in lv) < 0.04 * sum(x["calls"] for x in lv)
    assert sum(x["differ"] == 0 for x in lv) == 8
    ev = [e for s in sets for cl in s["events"] for e in cl]
    assert sum(e[0] == "K" for e in ev) > 1000 and sum(e[0] == "G" for e in ev) > 800
    assert sum(e[0] == "J" for e in ev) == sum(e[0] == "K" for e in ev)
    # rebased ends that moved: the rebase does more than re-send
    moved = 0
    for s in sets:
        for cl in s["events"]:
            q = [e[1] for e in cl if e[0] == "J"]
            k = [s["log"][e[1]][5] for e in cl if e[0] == "K"]
            ends = lambda v: (v.get("start"), v.get("end"))  # noqa: E731
            moved += sum(1 for a, b in zip(q, k) if a["opName"] != "delete" and "value" in b and
                         ends(a["value"]) != ends(b["value"]))
    assert moved > 100


@pytest.mark.gpu
def test_node_interval_reconnect_on_gpu():
    """Interval collections across reconnection (rebaseLocalInterval,
    intervalCollection.ts:1735-1803, through MTE_OP_REF b = 4 / 5 on the HBM
    tree pass, with the reference's block-level localSeq views): on all 33
    reference farms every op a client re-sends equals the reference's --
    rebased adds and changes exactly, regenerated merge-tree ops as
    test_reconnect compares them -- and at every checkpoint the text,
    intervals, events, order, summary and queries equal the reference
    client's."""
    from fixtures_util import canon_regen
    j = json.loads(node("tests/node/interval_farm.js", "reconnect").strip().splitlines()[-1])
    assert j["nFailures"] == 0, (j["extFail"], j["extFirst"], j["failures"][:2])
    sets = reconnect_sets()["sets"]
    assert j["passed"] == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
    bad = [x for x in j["regens"] if canon_regen(x[0], x[2], False) != canon_regen(x[1], x[2], False)]
    assert not bad, bad[:2]
    assert len(j["regens"]) > 800
    # previousInterval / nextInterval (the end tree) and the whole event lists,
    # the changeInterval events slides raise mid-op included: as the reference
    assert j["prevNext"]["equal"] == j["prevNext"]["n"], j["prevNext"]
    assert j["mtEvents"]["equal"] == j["mtEvents"]["n"], j["mtEvents"]
    # the order among intervals whose ends slid off the string
    assert j["orderOff"] == 0, j["orderOff"]


def _farm(mode, addon):
    env = dict(os.environ, MTE_NODE_ADDON=addon)
    r = subprocess.run(["node", "tests/node/interval_farm.js", mode], cwd=ROOT, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode", ["ext", "reconnect"])
def test_node_interval_farms_on_restatement(mode):
    """The Node host over the CPU restatement (oracle/mte_shim.c: the same
    N-API functions served by titems.c, the HBM tree pass's specification):
    every checkpoint of the ext and reconnect farms -- text, intervals, the
    whole event lists (mid-op changeInterval included), order, summaries and
    queries, previousInterval / nextInterval included -- equals the
    reference's, and every rebased op the reference's."""
    from fixtures_util import canon_regen
    j = _farm(mode, "oracle")
    assert j["nFailures"] == 0, (j["extFail"], j["extFirst"], j["failures"][:2])
    sets = (reconnect_sets() if mode == "reconnect" else ext_sets())["sets"]
    assert j["passed"] == sum(len(s["names"]) * len(s["checkpoints"]) for s in sets)
    assert j["prevNext"]["equal"] == j["prevNext"]["n"] > 1000, j["prevNext"]
    assert j["mtEvents"]["equal"] == j["mtEvents"]["n"], j["mtEvents"]
    assert j["orderOff"] == 0
    assert j["endRebuilds"] == 0, j["endRebuilds"]
    if mode == "reconnect":
        bad = [x for x in j["regens"] if canon_regen(x[0], x[2], False) != canon_regen(x[1], x[2], False)]
        assert not bad, bad[:2]


def _batch_run(mode, docs, msgs):
    r = subprocess.run(["node", "tests/node/interval_batch.js", mode, str(docs), str(msgs)], cwd=ROOT,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_interval_documents_batch_on_restatement():
    """Documents whose collections hold intervals queue their merge-tree
    messages like any other: 100 documents x 120 remote messages (removes that
    slide interval ends, group ops among them) replay in ONE run, and every
    document's changeInterval events (positions as each record left the
    document, MTE_DELTA_REFPOS), intervals, end-tree queries and summary equal
    a replay of one message per run (tests/node/interval_batch.js)."""
    j = _batch_run("oracle", 100, 120)
    assert j["runs"] == 1 and j["equal"] == j["docs"] == 100, j
    assert j["events"] > 5000


@pytest.mark.gpu
def test_gpu_interval_documents_batch():
    """As above on the engine: 1,000 interval-holding documents x 120 messages
    in one mte_run, every document equal to the message-by-message replay."""
    j = _batch_run("gpu", 1000, 120)
    assert j["runs"] == 1 and j["equal"] == j["docs"] == 1000, j
    assert j["events"] > 50000
