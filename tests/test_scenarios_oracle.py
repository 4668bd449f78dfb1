"""Known-answer and edge-case scenarios on the CPU restatement."""
import pytest

from scenarios import SCENARIOS, expected_of, run_scenario

from oracle import OracleEngine


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_oracle(oracle_lib, name):
    st, text, rd, _ = run_scenario(OracleEngine(8), name)
    exp = expected_of(name)
    if exp is None:
        assert st == 0
    elif exp.startswith("ERR:"):
        assert st == int(exp[4:])
    else:
        assert st == 0
        assert text == exp
