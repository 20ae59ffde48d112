"""The 32K OFDM kernel's per-symbol resource model (tools/ofdm_phase_model.py) recomputed
from the committed session counters and the measured store rate: the measured time per symbol is at
or above every single-resource lower bound (LDS array, VALU issue, the CU's measured store rate) and
the launch at or above the chip's measured store bound; the serial sum is arithmetic, not a bound."""
import json
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("tag", ["r3_r3u", "r3_r3f1"])
def test_ofdm_resource_model(tag):
    pmc, bench = ROOT / "profiles" / f"{tag}_pmc_sq.txt", ROOT / "profiles" / f"{tag}_bench.json"
    rates = ROOT / "profiles" / "r4_store_rate.jsonl"
    if not pmc.exists() or not bench.exists() or not rates.exists():
        pytest.skip("session profiles absent")
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "ofdm_phase_model.py"), str(pmc), str(bench), str(rates)],
                         capture_output=True, text=True, check=True).stdout
    m = json.loads(out)
    assert m["valu"] > 0 and m["lds"] > 0 and m["store_lone_cu"] > 0
    assert m["serial_sum"] == pytest.approx(m["valu"] + m["lds"] + m["store_lone_cu"], abs=2)
    assert m["cycles_per_symbol"] >= m["largest_single_resource_bound"]
    assert m["launch_ms"] >= m["chip_store_bound_ms"]
    # the measured per-CU store rate is well above the r3 model's fair 1/256 share of 8 TB/s
    assert m["store_lone_cu"] < 0.5 * m["store_fair_share_r3"]
    assert m["measured_over_serial_sum"] > 1.0
