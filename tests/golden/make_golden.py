"""Generate tests/golden/*.npz: per-stage outputs of the oracle chain for small seeded inputs.

The reference (GNU Radio OOT module) cannot be built or run here, so these fixtures are produced
by the oracle restatement (oracle/dvbt2_oracle.c), whose primitives are pinned by the known-answer
tests in tests/test_cpu_oracle.py.  They freeze the pinned behaviour: the CPU suite checks the
oracle still reproduces them, and the GPU suite checks the HIP blocks against them directly.

    python tests/golden/make_golden.py
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parent), str(HERE.parents[1] / "gr-dvbt2ll_amd")]

from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402
import oracle_lib as O  # noqa: E402

# name: (frames, what is kept): "all" every stage; "bits" the TS and bit stages, digests of the float
# stages; "digest" digests only (the 32K configs: the benched frame shapes)
CASES = {"cfg1": (2, "all"), "cfg1q": (2, "all"), "cfg4": (1, "bits"), "cfg2": (1, "digest"), "cfg3": (1, "digest"),
         "cfg5": (1, "digest")}


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
    # each frame's IQ as the GPU writes it: the oracle's carriers through oracle/ifft_model.c (the OFDM
    # kernels' operation order) after the oracle's P1
    res["iq"] = np.stack([O.model_frame(c, pg.guard, pg.normalization, res["p1"]) for c in res["carriers"]])
    return res


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def main():
    for name, (nframes, keep) in CASES.items():
        st = stages(CONFIGS[name], nframes)
        st["iq_sha256"] = digest(st.pop("iq"))
        st["nframes"] = np.int64(nframes)
        big = ("cells", "mapped", "carriers") + (("ts", "bbbits", "codeword") if keep == "digest" else ())
        if keep != "all":   # large: keep only digests of these stages
            for k in big:
                st[k + "_sha256"] = digest(st.pop(k))
        np.savez_compressed(HERE / ("%s.npz" % name), **st)
        print("wrote", name)


if __name__ == "__main__":
    main()
