"""matchProperties never matches NaN (NaN !== NaN, properties.ts:66-100), so the
reference's zamboni does not append-merge two segments holding NaN
(mergeTree.ts:712) and its summary writers do not coalesce them
(snapshotV1.ts:215, snapshotlegacy.ts:170) -- ADVICE r04 (medium).  The hosts
intern NaN under a value id with MTE_VALUE_UNEQUAL set (include/mte.h) and the
tree passes' scours, their restatements (titems.c, tree.c) and the summary
writers treat such an id as equal to nothing.

Pinned by 24 streams the reference itself replayed (tests/golden/
make_nan_golden.py -> nan_merge_vectors.json.gz: plain and incr annotates on two
keys, then no-op messages until minSeq reaches the last seq, so every block's
scour has run): the visible segments in order -- the segmentation the
append-merges leave -- with their properties, the text and the per-position
properties, on the tree restatement and on the GPU (observer documents with
MTE_DOC_LOCAL_CLIENT: incr replays on the HBM tree pass)."""
import gzip
import json
import os

import numpy as np
import pytest

from fixtures_util import as_msg, doc_inits, prop_runs
from fluidframework_amd.abi import DOC_LOCAL_CLIENT, DOC_NEW_LENGTH_CALC, MTE_VALUE_UNEQUAL
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner, units_to_str

HERE = os.path.dirname(os.path.abspath(__file__))


def vectors():
    with gzip.open(os.path.join(HERE, "golden", "nan_merge_vectors.json.gz"), "rt", encoding="utf-8") as fh:
        return json.load(fh)["docs"]


def _segs(view, interner, text):
    out, pos = [], 0
    for ln, kind, planes in view["segs"]:
        p = {k: (None if isinstance(v, float) and v != v else v) for k, v in interner.decode_props(planes).items()}
        seg = view["text"][pos:pos + ln] if kind == 0 else {"marker": kind - 1}
        out.append([seg, p or None])
        pos += ln
    return out


def replay(engine_factory, docs):
    n_keys = 4
    inits, text = doc_inits([""] * len(docs), flags=DOC_NEW_LENGTH_CALC | DOC_LOCAL_CLIENT)
    interner = Interner(n_keys)
    eng = engine_factory(n_keys)
    eng.load_docs(inits, text)
    bb = BatchBuilder(len(docs), interner)
    for d, doc in enumerate(docs):
        cl = DocClients("A", local=True)
        for m in doc["msgs"]:
            bb.add_message(d, cl, as_msg(m))
    eng.apply_batch(bb.build())
    st = eng.statuses()
    got = []
    for d in range(len(docs)):
        v = eng.read_doc(d)
        got.append({"status": int(st[d]), "text": v["text"], "props": prop_runs(v, interner),
                    "segs": _segs(v, interner, text)})
    return got, interner


def test_nan_vectors_shape():
    docs = vectors()
    assert len(docs) == 24
    # the case the rule decides: adjacent segments, both NaN under the same
    # keys, everything else equal -- the reference keeps them apart
    pairs = sum(1 for d in docs for a, b in zip(d["segs"], d["segs"][1:])
                if a[1] and a[1] == b[1] and None in a[1].values() and isinstance(a[0], str) and
                isinstance(b[0], str) and not a[0].endswith("\n"))
    assert pairs > 50, pairs


def test_interner_nan_id_matches_nothing():
    it = Interner(4)
    a, b = it.value(float("nan")), it.value(float("nan"))
    assert a == b and a & MTE_VALUE_UNEQUAL and it.json_of(a) == "NaN"
    assert not it.value(1) & MTE_VALUE_UNEQUAL
    assert np.isnan(it.decode_props([a, 0, 0, 0])[it.key_names[0]] if it.key_names else
                    json.loads(it.json_of(a)))


def _check(got, docs):
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, docs))
           if g["status"] != 0 or g["text"] != w["text"] or g["props"] != w["props"] or g["segs"] != w["segs"]]
    assert not bad, bad[0]


def test_tree_restatement_keeps_nan_segments_apart():
    from oracle import OracleEngine

    def fac(k):
        e = OracleEngine(k, tree="items")
        e.lib.oti_set_limit(e.ctx, 1 << 20)
        return e
    docs = vectors()
    got, _ = replay(fac, docs)
    _check(got, docs)


@pytest.mark.gpu
def test_gpu_keeps_nan_segments_apart():
    from fluidframework_amd.engine import DeviceEngine
    docs = vectors()
    got, _ = replay(lambda k: DeviceEngine(k), docs)
    _check(got, docs)


def test_vectors_see_the_rule():
    """With NaN interned as an ordinary value id (equal to itself) the
    restatement merges what the reference keeps apart: the vectors pin the rule."""
    from oracle import OracleEngine
    import fluidframework_amd.packing as P

    def fac(k):
        e = OracleEngine(k, tree="items")
        e.lib.oti_set_limit(e.ctx, 1 << 20)
        return e
    docs = vectors()
    orig = P.Interner.value
    try:
        P.Interner.value = lambda self, v: orig(self, v) & ~MTE_VALUE_UNEQUAL
        got, _ = replay(fac, docs)
    finally:
        P.Interner.value = orig
    assert sum(g["segs"] != w["segs"] for g, w in zip(got, docs)) >= 12
