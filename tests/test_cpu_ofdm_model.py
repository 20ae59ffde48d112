"""The 32K OFDM kernel's phase-serial bound (tools/ofdm_phase_model.py) recomputed from
the committed session counters: the measured time per symbol is at or above the bound (it is a lower
bound) and within 10 % of it."""
import json
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("tag", ["r3u", "r3f1"])
def test_ofdm_phase_serial_bound(tag):
    pmc, bench = ROOT / "profiles" / f"r3_{tag}_pmc_sq.txt", ROOT / "profiles" / f"r3_{tag}_bench.json"
    if not pmc.exists() or not bench.exists():
        pytest.skip("session profiles absent")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "ofdm_phase_model.py"), str(pmc), str(bench)],
                         capture_output=True, text=True, check=True).stdout
    m = json.loads(out)
    assert m["valu"] > 0 and m["lds"] > 0 and m["hbm_share"] > 0
    assert m["phase_serial_bound"] == pytest.approx(m["valu"] + m["lds"] + m["hbm_share"], abs=2)
    assert 1.0 <= m["measured_over_bound"] <= 1.10
