"""Parse the generated standard-table header (EN 302 755 data) for the CPU tests, so LDPC
parity checks and BCH generators are recomputed independently of both the oracle and the
product code."""
import re
from pathlib import Path

HDR = Path(__file__).resolve().parents[1] / "gr-dvbt2ll_amd" / "csrc" / "gen" / "dvbt2_std_tables.h"
_text = HDR.read_text()


def _array(name):
    m = re.search(r"%s\[[^\]]*\](?:\[[^\]]*\])?\s*=\s*\{(.*?)\};" % re.escape(name), _text, re.S)
    return [int(v, 0) for v in re.findall(r"0x[0-9A-Fa-f]+|\d+", m.group(1))]


_codes = [tuple(int(v) for v in re.findall(r"-?\d+", row))
          for row in re.findall(r"\{([^{}]*)\}, /\* \w+ \*/", _text.split("T2_LDPC_CODES[] = {")[1].split("};")[0])]
_rowlen = _array("T2_LDPC_ROWLEN")
_addr = _array("T2_LDPC_ADDR")

FEC = {(1, 0): (32400, 90), (1, 1): (38880, 72), (1, 2): (43200, 60), (1, 3): (48600, 45), (1, 4): (51840, 36),
       (1, 5): (54000, 30), (0, 6): (5400, 30), (0, 7): (6480, 27), (0, 0): (7200, 25), (0, 1): (9720, 18),
       (0, 2): (10800, 15), (0, 3): (11880, 12), (0, 4): (12600, 10), (0, 5): (13320, 8)}


def fec(framesize, rate):
    return FEC[(framesize, rate)]


def ldpc_rows(framesize, rate):
    for fs, r, nrows, q, row_off, addr_off, naddr in _codes:
        if fs == framesize and r == rate:
            out, off = [], addr_off
            for g in range(nrows):
                n = _rowlen[row_off + g]
                out.append(_addr[off: off + n])
                off += n
            return out
    raise KeyError((framesize, rate))


def bch_generator(normal, P):
    flat = _array("T2_BCH_MINPOLY_NORMAL" if normal else "T2_BCH_MINPOLY_SHORT")
    w = 17 if normal else 15
    polys = [flat[i * w:(i + 1) * w] for i in range(12)]
    acc = [1]
    for m in polys[: (P // 16 if normal else 12)]:
        r = [0] * (len(acc) + len(m) - 1)
        for i, a in enumerate(acc):
            if a:
                for j, b in enumerate(m):
                    r[i + j] ^= b
        acc = r
    assert len(acc) == P + 1
    return acc[::-1]   # highest power first
