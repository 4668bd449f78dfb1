"""Known-answer and edge-case scenarios on the CPU restatement."""
import pytest

from scenarios import PROPS_AT, SCENARIOS, expected_of, props_at, run_scenario

from oracle import OracleEngine


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_oracle(oracle_lib, name):
    st, text, rd, interner = run_scenario(OracleEngine(8), name)
    for pos, want in PROPS_AT.get(name, []):
        assert props_at(rd, interner, pos) == want, pos
    exp = expected_of(name)
    if exp is None:
        assert st == 0
    elif exp.startswith("ERR:"):
        assert st == int(exp[4:])
    else:
        assert st == 0
        assert text == exp
