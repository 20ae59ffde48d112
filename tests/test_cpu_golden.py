"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/make_golden.py): every stage,
raw where the fixture keeps it and as a SHA-256 digest elsewhere, plus the IQ digest of the oracle's
carriers through the IFFT model."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

from dvbt2ll.configs import CONFIGS

GOLD = Path(__file__).resolve().parent / "golden"
NAMES = ["cfg1", "cfg1q", "cfg4", "cfg2", "cfg3", "cfg5"]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    import sys
    sys.path.insert(0, str(GOLD))
    import make_golden
    g = np.load(GOLD / ("%s.npz" % name))
    st = make_golden.stages(CONFIGS[name], int(g["nframes"]))
    assert int(st["ts_consumed"]) == int(g["ts_consumed"]) and int(st["ts_base"]) == int(g["ts_base"])
    np.testing.assert_array_equal(st["p1"].view(np.uint32), g["p1"].view(np.uint32))
    for k in ("ts", "bbbits", "codeword", "cells", "mapped", "carriers"):
        if k in g:
            np.testing.assert_array_equal(st[k].view(np.uint8), g[k].view(np.uint8), err_msg=k)
        else:
            assert _sha(st[k]) == g[k + "_sha256"].tobytes(), k
    assert _sha(st["iq"]) == g["iq_sha256"].tobytes()
