"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/make_golden.py)."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

from dvbt2ll.configs import CONFIGS, ts_for_frames

GOLD = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg4"])
def test_oracle_reproduces_golden(name):
    import sys
    sys.path.insert(0, str(GOLD))
    import make_golden
    g = np.load(GOLD / ("%s.npz" % name))
    nframes = g["bbbits"].shape[0]
    ts, base = ts_for_frames(CONFIGS[name], 0, nframes)
    np.testing.assert_array_equal(ts, g["ts"])
    st = make_golden.stages(CONFIGS[name], nframes)
    for k in ("bbbits", "codeword"):
        np.testing.assert_array_equal(st[k], g[k])
    np.testing.assert_array_equal(st["p1"].view(np.uint32), g["p1"].view(np.uint32))
    for k in ("cells", "mapped", "carriers"):
        if k in g:
            np.testing.assert_array_equal(st[k].view(np.uint32), g[k].view(np.uint32))
        else:
            assert hashlib.sha256(st[k].tobytes()).digest() == g[k + "_sha256"].tobytes()
