"""The erased reference (oracle/_ref/ts, oracle/ts_erase.py) pinned by the
reference's own golden fixtures: packages/dds/merge-tree/src/test/results/*.json
(30 files, 64 rounds each) replayed through its Client as
test/client.replay.spec.ts:16-60 does (oracle/ref_fixture_replay.js): every
sender a client of its own applying its ops locally, every client applying
every message, all clients' texts equal to initialText / resultText at every
round — 3,840 checkpoints.  This is what makes the reference-run vectors
(tests/golden/{ref,farm,reconnect,delta}_vectors) a pin: the tree they come
from reproduces the reference's own fixtures.  Build container only (the
reference does not travel to the GPU box)."""
import json
import os
import subprocess

import pytest

import ref_util
from fixtures_util import load_fixtures

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = os.path.join(os.path.dirname(HERE), "oracle", "ref_fixture_replay.js")

pytestmark = pytest.mark.skipif(not ref_util.ref_available(),
                                reason="the reference sources exist only in the build container")


def test_erased_reference_passes_every_fixture_checkpoint():
    out_dir = ref_util.build_ref()
    fx = load_fixtures()
    p = subprocess.run(["node", "--max-old-space-size=8192", SCRIPT, out_dir], input=json.dumps(fx),
                       capture_output=True, text=True, timeout=1800)
    assert p.returncode == 0, p.stderr[-4000:]
    res = json.loads(p.stdout)
    assert len(res) == len(fx) == 30
    passed = 0
    for f, r in zip(fx, res):
        assert r["error"] is None, (f["name"], r["error"])
        assert r["diverged"] == [], (f["name"], r["diverged"][:5])
        assert len(r["texts"]) == len(f["rounds"])
        for rd, (initial, result) in zip(f["rounds"], r["texts"]):
            assert initial == rd["initialText"], f["name"]
            assert result == rd["resultText"], f["name"]
            passed += 2
    assert passed == 3840


def test_stubs_hold_no_merge_arithmetic():
    # only loggers, error classes and the summary builder stay stubbed: every
    # other imported value is erased from the reference's sources
    src = open(os.path.join(os.path.dirname(HERE), "oracle", "ref_stubs.js")).read()
    exported = src[src.index("module.exports"):]
    assert set(x.strip() for x in exported[exported.index("{") + 1:exported.index("}")].split(",")) == \
        {"ChildLogger", "LoggingError", "UsageError", "SummaryTreeBuilder", "bufferToString"}


def _load_gz(name):
    import gzip
    with gzip.open(os.path.join(HERE, "golden", name), "rt", encoding="utf-8") as fh:
        return json.load(fh)


def test_reconnect_vectors_are_what_the_erased_reference_computes_today():
    # the first reconnect farms, re-run through oracle/ref_farm.js on today's tree
    out_dir = ref_util.build_ref()
    sets = _load_gz("reconnect_vectors.json.gz")["sets"][:4]
    farm = os.path.join(os.path.dirname(HERE), "oracle", "ref_farm.js")
    for s in sets:
        one = {"sets": [{"seed": s["seed"], "clients": s["clients"], "steps": s["steps"],
                         "initialText": s["initialText"], "nCheckpoints": s["nCheckpoints"], "maxText": s["maxText"],
                         "reconnect": s["reconnect"], "allowDiverge": True}]}
        p = subprocess.run(["node", farm, out_dir], input=json.dumps(one), capture_output=True, text=True,
                           timeout=600, check=True)
        live = json.loads(p.stdout)["sets"][0]
        assert live["log"] == s["log"] and live["events"] == s["events"] and live["checkpoints"] == s["checkpoints"]


def test_delta_vectors_are_what_the_erased_reference_computes_today():
    from fluidframework_amd import gen
    rec = _load_gz("delta_vectors.json.gz")["sets"][0]
    st = gen.generate(rec["config"], n_docs=8, ops_per_doc=rec["ops_per_doc"], **rec["params"])
    docs = ref_util.stream_docs(st, 0, 8)
    for d in docs:
        d["deltas"] = True
        d["props"] = False
    res = ref_util.ref_replay(docs)
    for r, want in zip(res, rec["docs"][:8]):
        assert r["error"] == want["error"]
        assert [[mi, kind, p, n, rm] for mi, kind, rng in r["deltas"] for p, n, rm in rng] == want["events"]
