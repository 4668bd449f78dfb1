"""Delta events: MTE_DOC_EVENTS documents record what
MergeTree.mergeTreeDeltaCallback reports after each insert / remove / annotate
(mergeTree.ts:1409-1416, 1893-1900, 1978-1985), the ranges SharedString's
"sequenceDelta" events carry (sequence.ts:203-211, sequenceDeltaEvent.ts), and
from them the catch-up rewrite of the legacy summary format
(createOpsFromDelta, sequence.ts:116-161, 688-725).

Pinned against the reference itself (tests/golden/delta_vectors.json.gz, made by
tests/golden/make_delta_golden.py through oracle/ref_replay.js): per message,
the position (Client.getPosition) and length of every delta segment.  Segment
boundaries are not the reference's (the flat passes split on op boundaries and
never append-merge), so the comparison is on what does not depend
on them: inserts and removes as createOpsFromDelta merges them (the rewritten
catch-up ops), annotates as the set of own-view units they changed.  A
document flagged MTE_DOC_TREE replays on the HBM tree pass, with the
reference's own segments: its records equal the reference's callbacks range
for range (tree restatement and GPU).
"""
import gzip
import json
import os

import numpy as np
import pytest

from fluidframework_amd import gen
from fluidframework_amd.abi import DOC_EVENTS, DOC_TREE

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "delta_vectors.json.gz")


def golden():
    with gzip.open(GOLD, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def ops_from_delta(events):
    """createOpsFromDelta (sequence.ts:116-161) over each message's ranges:
    consecutive removes at one position merge, annotates that continue the
    last one merge (same props within one op)."""
    out = []
    for op, kind, pos, ln in events:
        last = out[-1] if out and out[-1][0] == op else None
        if kind == 1 and last is not None and last[2] == pos:
            last[3] += ln
        elif kind == 2 and last is not None and last[2] + last[3] == pos:
            last[3] += ln
        else:
            out.append([op, kind, pos, ln])
    return out


def canonical(events):
    """(inserts + removes as createOpsFromDelta rewrites them, annotated runs of
    the own view) — what does not depend on segment boundaries.  An annotate's
    ranges over segments removed in the own view have zero own length, so
    they are left out of its runs."""
    ir = ops_from_delta([e[:4] for e in events if e[1] != 2])
    runs = ops_from_delta([e[:4] for e in events if e[1] == 2 and not e[4]])
    return ir, runs


def compare(got_events, want_events):
    g = canonical(got_events)
    w = canonical(want_events)
    if g[0] != w[0]:
        return "insert/remove ranges differ"
    if g[1] != w[1]:
        return "annotated runs differ"
    return None


def run_set(factory, S):
    st = gen.generate(S["config"], n_docs=S["n_docs"], ops_per_doc=S["ops_per_doc"], **S["params"])
    inits = st["inits"].copy()
    inits["flags"] |= DOC_EVENTS
    e = factory(st["n_keys"])
    e.load_docs(inits, st["init_text"])
    e.apply_batch(st["batch"])
    assert (e.statuses() == 0).all()
    bad = []
    for d, doc in enumerate(S["docs"]):
        ev = e.read_deltas(d)
        got = [[int(x["op"]), int(x["kind"]), int(x["pos"]), int(x["len"]), int(x["removed"])] for x in ev]
        why = compare(got, doc["events"])
        if why:
            bad.append((S["name"], d, why))
    return bad


def oracle_factory(k):
    from oracle import OracleEngine
    return OracleEngine(k)


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


@pytest.mark.parametrize("i", range(3))
def test_oracle_deltas_match_reference(i):
    S = golden()[i]
    bad = run_set(oracle_factory, S)
    assert not bad, bad[:3]


def run_set_exact(factory, S):
    """Every record equal to the reference's callback ranges (MTE_DOC_TREE)."""
    st = gen.generate(S["config"], n_docs=S["n_docs"], ops_per_doc=S["ops_per_doc"], **S["params"])
    inits = st["inits"].copy()
    inits["flags"] |= DOC_EVENTS | DOC_TREE
    e = factory(st["n_keys"])
    e.load_docs(inits, st["init_text"])
    e.apply_batch(st["batch"])
    assert (e.statuses() == 0).all()
    bad = []
    for d, doc in enumerate(S["docs"]):
        got = [[int(x["op"]), int(x["kind"]), int(x["pos"]), int(x["len"]), int(x["removed"])]
               for x in e.read_deltas(d)]
        if got != doc["events"]:
            k = 0
            while k < min(len(got), len(doc["events"])) and got[k] == doc["events"][k]:
                k += 1
            bad.append((S["name"], d, k, got[k:k + 2], doc["events"][k:k + 2]))
    return bad


def tree_factory(k):
    from oracle import OracleEngine
    e = OracleEngine(k, tree="items")
    e.lib.oti_set_limit(e.ctx, 1 << 20)
    return e


@pytest.mark.parametrize("i", range(3))
def test_tree_oracle_deltas_segment_exact(i):
    bad = run_set_exact(tree_factory, golden()[i])
    assert not bad, bad[:3]


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(3))
def test_gpu_tree_deltas_segment_exact(i):
    bad = run_set_exact(device_factory, golden()[i])
    assert not bad, bad[:3]


def test_ops_from_delta_merges():
    ev = [[4, 1, 7, 2], [4, 1, 7, 3], [4, 1, 9, 1], [5, 2, 0, 2], [5, 2, 2, 1], [5, 2, 9, 1]]
    assert ops_from_delta(ev) == [[4, 1, 7, 5], [4, 1, 9, 1], [5, 2, 0, 3], [5, 2, 9, 1]]


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(3))
def test_gpu_deltas_match_reference(i):
    S = golden()[i]
    bad = run_set(device_factory, S)
    assert not bad, bad[:3]


@pytest.mark.gpu
def test_gpu_deltas_equal_oracle_exactly():
    """Same segmentation on both sides: the GPU's events equal the restatement's
    record for record, local-client documents included."""
    from oracle import OracleEngine
    from fluidframework_amd.engine import DeviceEngine
    st = gen.generate(3, n_docs=48, ops_per_doc=700, length_mode=2, max_lag=32)
    inits = st["inits"].copy()
    inits["flags"] |= DOC_EVENTS
    outs = []
    for E in (DeviceEngine, OracleEngine):
        e = E(st["n_keys"])
        e.load_docs(inits, st["init_text"])
        e.apply_batch(st["batch"])
        outs.append([e.read_deltas(d) for d in range(48)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
