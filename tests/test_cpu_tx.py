"""The native transmitter tool (gr-dvbt2ll_amd/dvbt2ll/dvbt2ll_tx, over the C ABI): presets equal
the Python configurations, argument handling, and a clean failure without a GPU."""
import subprocess
from pathlib import Path

import pytest

from dvbt2ll.configs import CONFIGS

TOOL = Path(__file__).resolve().parents[1] / "gr-dvbt2ll_amd" / "dvbt2ll" / "dvbt2ll_tx"
FM_NAMES = ("framesize rate constellation rotation fecblocks tiblocks carriermode fftsize guardinterval "
            "l1constellation pilotpattern t2frames numdatasyms paprmode version preamble inputmode "
            "reservedbiasbits l1scrambled inband").split()


def run(*args):
    return subprocess.run([str(TOOL), *args], capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_tx_presets_match_configs(name):
    cfg = CONFIGS[name]
    r = run("--preset", name, "--print-params")
    assert r.returncode == 0, r.stderr
    got = dict(line.split("=") for line in r.stdout.split())
    want = dict(zip(FM_NAMES, cfg.fm_args()))
    want.update(misogroup=cfg.misogroup, equalization=cfg.equalization, bandwidth=cfg.bandwidth, tsrate=cfg.tsrate)
    assert {k: int(v) for k, v in got.items()} == {k: int(v) for k, v in want.items()}


def test_tx_set_overrides_and_bad_args():
    r = run("--preset", "cfg1", "--set", "inputmode=1", "--set", "tsrate=123", "--print-params")
    got = dict(line.split("=") for line in r.stdout.split())
    assert got["inputmode"] == "1" and got["tsrate"] == "123"
    assert run("--help").returncode == 0
    assert run("--set", "nosuch=1", "--print-params").returncode == 2
    assert run("--format", "s8", "--in", "x", "--out", "y").returncode == 2
    assert run("--in", "x").returncode == 2          # missing --out


def test_tx_fails_cleanly_without_device(tmp_path):
    """no CPU fallback: without a visible gfx950 device the tool reports the C ABI's error"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = run("--in", "/dev/null", "--out", str(tmp_path / "iq.bin"))
    assert r.returncode == 1 and "chain create" in r.stderr


@pytest.mark.parametrize("name", ["mplp3_4k", "mix_4k"])
def test_tx_mplp_presets_match_configs(name):
    """the transmitter's multi-PLP presets resolve to exactly configs.py's frames (dvbt2ll_mplp_params ints)"""
    from dvbt2ll.configs import MPLP_CONFIGS, IF_CONFIGS
    m = {**MPLP_CONFIGS, **IF_CONFIGS}[name]
    r = subprocess.run([str(TOOL), "--mplp", name, "--print-params"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert [int(x) for x in r.stdout.split()] == m.mplp_array()
