"""GPU debug aid for the fused BB + BCH pass: per FEC block of a two-frame chain run, where the stored
interleaver-input codeword differs from the oracle's (BBFRAME bytes / BCH parity / LDPC parity)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT / "gr-dvbt2ll_amd"), str(ROOT / "tests")]
import dvbt2ll  # noqa: E402
from dvbt2ll import enums as E  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402
import oracle_lib as O  # noqa: E402
import plan_probe as PP  # noqa: E402


def run(framesize, rate, mode=E.INPUTMODE_NORMAL, inband=E.INBAND_OFF, const=E.MOD_16QAM, F=3, base="cfg4"):
    cfg = CONFIGS[base].with_(framesize=framesize, rate=rate, inputmode=mode, inband=inband, constellation=const,
                              fecblocks=F)
    nb = 2 * F
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ch.debug_keep_codewords()
    ch.run(0, 2)
    got = ch.debug_codewords(nb)
    ts, _ = ts_for_frames(cfg, 0, 2)
    bits, _ = O.BB(*cfg.bb_args()).work(ts, nb)
    fp = PP.fec_plan(framesize, rate, cfg.constellation)
    nbch, q, kbch = fp["nbch"], fp["q"], fp["kbch"]
    nldpc = 64800 if framesize else 16200
    cw = O.LDPC(framesize, rate).work(bits, nb).reshape(nb, nldpc)
    if fp["parity_il"]:
        t, s = np.divmod(np.arange(nldpc - nbch), 360)
        cw = cw.copy()
        cw[:, nbch:] = cw[:, nbch + q * s + t]
    want = np.packbits(cw, axis=1)
    L, NB = kbch // 8, nbch // 8
    print("code", framesize, rate, "mode", mode, "inband", inband, "L", L, "NB", NB)
    for b in range(nb):
        g, w = got[b, :nldpc // 8], want[b]
        d = np.nonzero(g != w)[0]
        bb, bc, ld = d[d < L], d[(d >= L) & (d < NB)], d[d >= NB]
        print(" block %d: BBFRAME bytes bad %d %s | BCH bad %d | LDPC bad %d" % (b, bb.size, bb[:24].tolist(), bc.size,
                                                                              ld.size))
        if bb.size:
            i = bb[0]
            print("   first bad byte %d: got %s want %s" % (i, g[i:i + 8].tolist(), w[i:i + 8].tolist()))


if __name__ == "__main__":
    run(E.FECFRAME_SHORT, E.C4_5, const=E.MOD_256QAM, base="cfg1", F=8)
    run(E.FECFRAME_NORMAL, E.C1_2)
    run(E.FECFRAME_NORMAL, E.C1_2, mode=E.INPUTMODE_HIEFF)
    run(E.FECFRAME_NORMAL, E.C3_5, inband=E.INBAND_ON)
