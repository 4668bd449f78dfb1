"""Reader of tests/golden/ref_vectors.json.gz: per-document digests and errors
of the REFERENCE merge-tree on seeded generated streams (written by
tests/golden/make_ref_golden.py in the build container)."""
import gzip
import json
import os

import numpy as np

from fluidframework_amd import gen
from fluidframework_amd.abi import MTE_E_INSERT_FAILED

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_vectors.json.gz")
ERRORS = {"MergeTree insert failed": MTE_E_INSERT_FAILED}


def load():
    with gzip.open(PATH, "rt", encoding="utf-8") as fh:
        return json.load(fh)["sets"]


def stream_of(rec):
    return gen.generate(rec["config"], n_docs=rec["n_docs"], ops_per_doc=rec["ops_per_doc"], **rec["params"])


def expected(rec):
    """-> (digests uint64[n, 4], statuses int32[n]) the reference produced"""
    dg = np.array([[int(x, 16) for x in d["digest"]] for d in rec["docs"]], dtype=np.uint64)
    st = np.array([0 if d["error"] is None else ERRORS[d["error"].split(":")[0]] for d in rec["docs"]], np.int32)
    return dg, st


def check(engine_factory, rec):
    """Replay one golden set on an engine; returns the docs that differ."""
    s = stream_of(rec)
    e = engine_factory(s["n_keys"])
    gen.load_stream(e, s)
    e.apply_batch(s["batch"])
    dg, st = expected(rec)
    got_st = e.statuses()
    got_dg = e.digest()
    bad = []
    for d in range(rec["n_docs"]):
        if got_st[d] != st[d]:
            bad.append((d, "status", int(got_st[d]), int(st[d])))
        elif st[d] == 0 and not np.array_equal(got_dg[d], dg[d]):
            bad.append((d, "digest"))
    return bad
