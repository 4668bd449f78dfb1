"""The CPU restatement against the reference's golden replay fixtures.

30 files x 64 rounds (packages/dds/merge-tree/src/test/results/*.json,
replayed as test/client.replay.spec.ts:16-60 does): initialText before and
resultText after every round = 3,840 checkpoints."""
from fixtures_util import load_fixtures, replay_fixtures

from oracle import OracleEngine


def test_fixture_inventory():
    fx = load_fixtures()
    assert len(fx) == 30
    assert sum(len(r["msgs"]) for f in fx for r in f["rounds"]) == 61200
    assert all(len(f["rounds"]) == 64 for f in fx)


def test_oracle_replays_all_fixtures(oracle_lib):
    passed, failures, eng = replay_fixtures(lambda k: OracleEngine(k))
    assert failures == []
    assert passed == 30 * 64 * 2


def test_oracle_fixture_stats(oracle_lib):
    # the stats are per batch; a single-batch replay of one fixture must
    # account for every op
    passed, failures, eng = replay_fixtures(lambda k: OracleEngine(k), files=[0], rounds=1)
    assert failures == []
    st = eng.stats()
    assert st["ops_applied"] == len(load_fixtures()[0]["rounds"][0]["msgs"])
