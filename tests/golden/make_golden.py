"""Generate tests/golden/*.npz: per-stage outputs of the oracle chain for small seeded inputs.

The reference (GNU Radio OOT module) cannot be built or run here, so these fixtures are produced
by the oracle restatement (oracle/dvbt2_oracle.c), whose primitives are pinned by the known-answer
tests in tests/test_cpu_oracle.py.  They freeze the pinned behaviour: the CPU suite checks the
oracle still reproduces them, and the GPU suite checks the HIP blocks against them directly.

    python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parent), str(HERE.parents[1] / "gr-dvbt2ll_amd")]

from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402
import oracle_lib as O  # noqa: E402

CASES = {"cfg1": (2, True), "cfg1q": (2, True), "cfg4": (1, False)}   # name: (frames, keep carriers)


def stages(cfg, nframes):
    ts, base = ts_for_frames(cfg, 0, nframes)
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    off = 0
    out = {k: [] for k in ("bbbits", "codeword", "cells", "mapped", "carriers")}
    for _ in range(nframes):
        bits, cons = bb.work(ts[off:], F)
        off += cons
        cw = ld.work(bits, F)
        cells = im.work(cw, F)
        mapped = fm.work(cells)
        out["bbbits"].append(np.packbits(bits))
        out["codeword"].append(np.packbits(cw))
        out["cells"].append(cells)
        out["mapped"].append(mapped)
        out["carriers"].append(pg.carriers(mapped))
    res = {k: np.stack(v) for k, v in out.items()}
    res["ts"] = ts
    res["ts_base"] = np.int64(base)
    res["ts_consumed"] = np.int64(off)
    res["p1"] = pg.p1()
    res["normalization"] = np.float64(pg.normalization)
    return res


def main():
    import hashlib
    for name, (nframes, keep) in CASES.items():
        st = stages(CONFIGS[name], nframes)
        if not keep:   # large: keep only digests of the bit-exact float stages
            for k in ("cells", "mapped", "carriers"):
                st[k + "_sha256"] = np.frombuffer(hashlib.sha256(st.pop(k).tobytes()).digest(), np.uint8)
        np.savez_compressed(HERE / ("%s.npz" % name), **st)
        print("wrote", name)


if __name__ == "__main__":
    main()
