"""mergeTreeMaintenanceCallback records (MTE_DOC_MAINT_EVENTS, MTE_DELTA_MAINT;
mergeTree.ts:695-725, 1313-1320, 1687-1694): SPLIT, APPEND, UNLINK and
ACKNOWLEDGED, the structural changes SharedString reports as "maintenance"
events (sequence.ts:212-216, SequenceMaintenanceEvent).

Remote-only documents (MTE_DOC_TREE, or the legacy length calculation) get the
same records from the tree pass: pinned by 260 generated lagging documents the
reference replayed as an observer (oracle/ref_replay.js maint,
tests/golden/maint_observer_vectors.json.gz: SPLIT, APPEND and UNLINK).

Pinned by 38 farms the reference itself ran with every client's callback
recorded (oracle/ref_farm.js maint -> tests/golden/maint_farm_vectors.json.gz,
made by tests/golden/make_farm_golden.py --maint): per event of every client
(its local ops, rollbacks and the messages it applied, its own as acks) the
callbacks in order, each with its segments' positions once the event is
applied and their lengths at the callback.  Plain farms with lagging clients,
rollbacks, local references, the legacy length calculation and long farms
(the lazy zamboni's appends) and reconnect farms (an ack of a regenerated op
acknowledges each re-sent segment as a group of its own, one callback and one
zamboni each: resetPendingDeltaToOps, client.ts:802-857) match exactly, on the
tree restatement (titems.c), on the GPU (the HBM tree pass) and through the
Node host -- except the ACKNOWLEDGED callback of an annotate made while
MTE_ANNOTATE_SLOTS (32) others were pending, which the engine does not track
(check() leaves those out and counts them).
"""
import gzip
import json
import os

import pytest

from fixtures_util import replay_ref_farm

HERE = os.path.dirname(os.path.abspath(__file__))
VECTORS = os.path.join(HERE, "golden", "maint_farm_vectors.json.gz")


def maint_sets():
    with gzip.open(VECTORS, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def tree_factory(k):
    from oracle import OracleEngine
    e = OracleEngine(k, tree="items")
    e.lib.oti_set_limit(e.ctx, 1 << 20)
    return e


def device_factory(k):
    from fluidframework_amd.engine import DeviceEngine
    return DeviceEngine(k)


def check(factory, sets):
    """(clients whose callback lists equal the reference's, clients, the acks
    of untracked annotates skipped, first difference).  An annotate made while
    MTE_ANNOTATE_SLOTS others are pending has no segment group in the engine:
    the reference's ACKNOWLEDGED callback at its ack is left out (the host
    counts those acks, DocClients.untracked_acks)."""
    got = {}
    passed, failures = replay_ref_farm(factory, sets, maint=got)
    assert not failures, failures[:2]
    equal, first, skipped = 0, None, 0
    for si, s in enumerate(sets):
        for ci in range(len(s["names"])):
            g, w = got.get((si, ci), []), s["maint"][ci]
            untracked = set(got.get(("untracked", si, ci), []))
            if untracked:
                skipped += sum(1 for x in w if x[1] == -4 and x[0] in untracked)
                w = [x for x in w if not (x[1] == -4 and x[0] in untracked)]
            if g == w:
                equal += 1
            elif first is None:
                k = 0
                while k < min(len(g), len(w)) and g[k] == w[k]:
                    k += 1
                first = (si, ci, k, g[k:k + 2], w[k:k + 2])
    n = sum(len(s["names"]) for s in sets)
    return equal, n, skipped, first


def test_maint_vectors_shape():
    sets = maint_sets()
    assert len(sets) == 38
    kinds = [e[1] for s in sets for cl in s["maint"] for e in cl]
    assert {-1, -2, -3, -4} <= set(kinds) and kinds.count(-1) > 100


def test_tree_oracle_maintenance_callbacks():
    equal, n, skipped, first = check(tree_factory, maint_sets())
    assert equal == n, first
    assert skipped < 10, skipped


@pytest.mark.gpu
def test_gpu_maintenance_callbacks():
    equal, n, skipped, first = check(device_factory, maint_sets())
    assert equal == n, first
    assert skipped < 10, skipped


def _node_farm(mode):
    import subprocess
    root = os.path.dirname(HERE)
    r = subprocess.run(["node", "tests/node/maint_farm.js", mode], cwd=root, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_node_maintenance_events_on_restatement():
    """SharedString "maintenance" events through the Node host
    (BatchClient.on("maintenance"), tests/node/maint_farm.js) over the CPU
    restatement's addon: every client of the 38 farms gets the reference's
    callback list, event by event."""
    j = _node_farm("oracle")
    assert j["equal"] == j["clients"] == sum(len(s["names"]) for s in maint_sets()), j["first"]
    assert j["callbacks"] > 30000 and j["skipped"] < 10, j


@pytest.mark.gpu
def test_gpu_node_maintenance_events():
    j = _node_farm("gpu")
    assert j["equal"] == j["clients"], j["first"]
    assert j["skipped"] < 10, j


OBSERVER_VECTORS = os.path.join(HERE, "golden", "maint_observer_vectors.json.gz")


def _group(ev):
    from fluidframework_amd.abi import DELTA_MAINT
    out = []
    for x in ev:
        k = int(x["kind"])
        if k & 0xff00 != DELTA_MAINT:
            continue
        t, mi = -(k & 0xff), int(x["op"])
        if int(x["removed"]) == 0 or not out or out[-1][0] != mi or out[-1][1] != t:
            out.append([mi, t, []])
        out[-1][2].append([int(x["pos"]), int(x["len"])])
    return out


def check_observers(factory):
    """Remote-only documents (the reference client as an observer, through
    oracle/ref_replay.js maint; tests/golden/make_delta_golden.py --maint): new
    length-calc ones flagged MTE_DOC_TREE, legacy ones on the tree pass anyway.
    Returns (documents, equal, first difference)."""
    from fluidframework_amd import gen
    from fluidframework_amd.abi import DOC_EVENTS, DOC_MAINT_EVENTS, DOC_TREE
    with gzip.open(OBSERVER_VECTORS, "rt", encoding="utf-8") as fh:
        sets = json.load(fh)["sets"]
    n = equal = 0
    first = None
    for S in sets:
        st = gen.generate(S["config"], n_docs=S["n_docs"], ops_per_doc=S["ops_per_doc"], **S["params"])
        inits = st["inits"].copy()
        inits["flags"] |= DOC_EVENTS | DOC_MAINT_EVENTS | DOC_TREE
        e = factory(st["n_keys"])
        e.set_event_capacity(64)
        e.load_docs(inits, st["init_text"])
        e.apply_batch(st["batch"])
        status = e.statuses()
        for d, doc in enumerate(S["docs"]):
            n += 1
            got, want = _group(e.read_deltas(d)), doc["maint"]
            # a document the reference failed on ("MergeTree insert failed") fails here too
            if got == want and (doc["error"] is None) == (int(status[d]) == 0):
                equal += 1
            elif first is None:
                first = (S["name"], d, doc["error"], int(status[d]), got[:2], want[:2])
    return n, equal, first


def test_tree_oracle_maintenance_of_remote_only_documents():
    n, equal, first = check_observers(tree_factory)
    assert equal == n == 260, first


@pytest.mark.gpu
def test_gpu_maintenance_of_remote_only_documents():
    n, equal, first = check_observers(device_factory)
    assert equal == n == 260, first
