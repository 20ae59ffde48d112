"""CPU: the C-ABI library loads and exports every symbol include/dvbt2ll_hip.h declares (no
compute calls without a GPU); the python mirror keeps the reference block names."""
import re
from pathlib import Path

import dvbt2ll

HDR = Path(__file__).resolve().parents[1] / "include" / "dvbt2ll_hip.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HDR.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(dvbt2ll_\w+)\s*\(", text)))


def test_header_symbols_exported():
    lib = dvbt2ll.lib()
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(dvbt2ll.EXPORTS)


def test_library_metadata_without_gpu():
    lib = dvbt2ll.lib()
    assert b"gfx950" in lib.dvbt2ll_version()
    assert lib.dvbt2ll_strerror(-1) == b"invalid parameter combination"
    assert lib.dvbt2ll_device_count() >= 0


def test_reference_block_names():
    for n in ("bbheaderbch_bb", "interleavermod_bc", "framemapperfint_cc", "pilotgenp1insert_cc", "ldpc_bb"):
        assert hasattr(dvbt2ll, n)
        assert hasattr(getattr(dvbt2ll, n), "make")
    assert dvbt2ll.FFTSIZE_16K_T2GI == 11 and dvbt2ll.C2_5 == 7 and dvbt2ll.PREAMBLE_T2_LITE_MISO == 4


def test_no_cpu_fallback_without_gpu():
    """the product fails loudly when no gfx950 device is visible (no silent CPU path)"""
    import pytest
    lib = dvbt2ll.lib()
    if lib.dvbt2ll_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(dvbt2ll.DVBT2Error):
        dvbt2ll.bbheaderbch_bb(0, 4, 0, 0, 8, 4000000)
    with pytest.raises(dvbt2ll.DVBT2Error):
        dvbt2ll.Chain(dvbt2ll.CONFIGS["cfg1"], max_frames=1)


def test_gr_adapter_driver_built_and_fails_cleanly_without_gpu(tmp_path):
    """the header-only GNU Radio adapters compile (build() makes tests/adapter/gr_flowgraph against
    the stand-in GR headers); without a GPU, make() throws and the driver exits 1 with the ABI's error"""
    import subprocess
    import pytest
    drv = Path(__file__).resolve().parent / "adapter" / "gr_flowgraph"
    assert drv.exists()
    if dvbt2ll.lib().dvbt2ll_device_count() > 0:
        pytest.skip("a GPU is visible")
    (tmp_path / "in.ts").write_bytes(b"\x47" * 188)
    r = subprocess.run([str(drv), str(tmp_path / "in.ts"), str(tmp_path / "o"), "1", "1"] + ["0"] * 24,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "bbheaderbch_bb" in r.stderr, r.stderr
