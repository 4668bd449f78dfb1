"""Helpers to replay the reference's golden replay fixtures through an engine.

Fixture data: tests/golden/replay_fixtures.json.gz (derived by
tests/golden/make_golden.py from packages/dds/merge-tree/src/test/results/).
The replay mirrors test/client.replay.spec.ts:16-60 from the point of view of
client "A" (the original client, which never sends): initialText of round 0 is
inserted before collaboration (seq 0, LocalClientId), every message is applied
as a remote op, and the text must equal resultText after each round.
"""
import gzip
import json
import os

import numpy as np

from fluidframework_amd.abi import DOC_INIT_DTYPE, NO_PROPS
from fluidframework_amd.packing import BatchBuilder, DocClients, Interner, utf16_units

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "replay_fixtures.json.gz")
_cache = None


def load_fixtures():
    global _cache
    if _cache is None:
        with gzip.open(GOLDEN, "rt", encoding="utf-8") as fh:
            _cache = json.load(fh)
    return _cache


def as_msg(m):
    cid, seq, ref, msn, typ, contents = m
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": typ, "contents": contents}


def doc_inits(texts, flags=0):
    inits = np.zeros(len(texts), DOC_INIT_DTYPE)
    parts, off = [], 0
    for i, t in enumerate(texts):
        u = utf16_units(t)
        inits[i] = (off, len(u), flags, NO_PROPS, 0, 0)
        parts.append(u)
        off += len(u)
    text = np.concatenate(parts) if parts else np.zeros(0, np.uint16)
    return inits, text


def replay_fixtures(engine_factory, files=None, check=True, rounds=None, fresh_clients=False):
    """Replay fixtures (all docs side by side, one batch per round).

    fresh_clients: every round's senders get new long ids ("B" -> "B#r").  Every
    op of a fixture round has refSeq == msn == the round's start, so a client's
    identity only matters inside its round and the reference's texts are the
    same; 8 x 64 = 512 distinct clients per document exercise the engine's
    client-slot recycling (DocClients).

    Returns (checkpoints_passed, failures)."""
    fx = load_fixtures()
    if files is not None:
        fx = [fx[i] for i in files]
    n = len(fx)
    interner = Interner(8)
    eng = engine_factory(8)
    inits, text = doc_inits([f["rounds"][0]["initialText"] for f in fx])
    eng.load_docs(inits, text)
    clients = [DocClients("A") for _ in range(n)]
    n_rounds = max(len(f["rounds"]) for f in fx)
    if rounds is not None:
        n_rounds = min(n_rounds, rounds)
    passed, failures = 0, []
    for r in range(n_rounds):
        bb = BatchBuilder(n, interner)
        for d, f in enumerate(fx):
            if r < len(f["rounds"]):
                if check:
                    got = eng.read_doc(d)["text"]
                    if got != f["rounds"][r]["initialText"]:
                        failures.append((f["name"], r, "initial", got, f["rounds"][r]["initialText"]))
                    else:
                        passed += 1
                for m in f["rounds"][r]["msgs"]:
                    msg = as_msg(m)
                    if fresh_clients:
                        msg["clientId"] = f"{msg['clientId']}#{r}"
                    bb.add_message(d, clients[d], msg)
        eng.apply_batch(bb.build())
        st = eng.statuses()
        for d, f in enumerate(fx):
            if st[d] != 0:
                failures.append((f["name"], r, "status", int(st[d]), 0))
            elif check and r < len(f["rounds"]):
                got = eng.read_doc(d)["text"]
                if got != f["rounds"][r]["resultText"]:
                    failures.append((f["name"], r, "result", got, f["rounds"][r]["resultText"]))
                else:
                    passed += 1
    return passed, failures, eng
