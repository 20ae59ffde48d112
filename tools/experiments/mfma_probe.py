"""Match the MFMA probe's accumulators (tools/experiments/mfma_probe.hip) against candidate lane maps.

C/D map (dtype-independent on gfx950, cdna_hip_programming.md §3): lane l, register r ->
row (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31.  A/B candidates: lane l holds row/column
l & 31 and k = KH * (l >> 5) + perm(j) for element j of its register block.
"""
import sys

import numpy as np


def cd_map():
    rows = np.zeros((64, 16), int)
    cols = np.zeros((64, 16), int)
    for l in range(64):
        for r in range(16):
            rows[l, r] = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)
            cols[l, r] = l & 31
    return rows, cols


def elements(words, bits, per_lane):
    """per lane, the element values (0/1) in register order"""
    w = words.reshape(64, -1)
    out = np.zeros((64, per_lane), np.int64)
    per_word = 32 // bits
    for l in range(64):
        for j in range(per_lane):
            v = (int(w[l, j // per_word]) >> (bits * (j % per_word))) & ((1 << bits) - 1)
            out[l, j] = 1 if v else 0
    return out


def check(name, ea, eb, c, K, cands):
    rows, cols = cd_map()
    for cname, kmap in cands.items():
        A = np.zeros((32, K), np.int64)
        B = np.zeros((K, 32), np.int64)
        for l in range(64):
            for j in range(ea.shape[1]):
                k = kmap(l, j)
                if k is None:
                    continue
                A[l & 31, k] = ea[l, j]
                B[k, l & 31] = eb[l, j]
        ref = A @ B
        got = np.zeros((32, 32), np.int64)
        for l in range(64):
            for r in range(16):
                got[rows[l, r], cols[l, r]] = int(round(float(c[l, r])))
        ok = np.array_equal(ref, got)
        print(f"{name} {cname}: {'MATCH' if ok else 'no'} (max |diff| {np.abs(ref - got).max()})")


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mfma_probe.bin"
    raw = np.fromfile(path, np.uint32)
    o = 0
    a4 = raw[o:o + 512]; o += 512
    b4 = raw[o:o + 512]; o += 512
    c4 = raw[o:o + 1024].view(np.float32).reshape(64, 16); o += 1024
    a8 = raw[o:o + 256]; o += 256
    b8 = raw[o:o + 256]; o += 256
    c8 = raw[o:o + 1024].view(np.int32).reshape(64, 16)
    # fp4: 64 nibbles per lane in 8 dwords; K = 64 -> 32 per lane half
    ea, eb = elements(a4, 4, 64), elements(b4, 4, 64)
    check("fp4", ea, eb, c4, 64, {
        "k=32h+j (j<32, low 4 dwords)": lambda l, j: 32 * (l >> 5) + j if j < 32 else None,
        "k=32h+j (j<32, high 4 dwords)": lambda l, j: 32 * (l >> 5) + (j - 32) if j >= 32 else None,
        "k=16h+j interleaved 16": lambda l, j: (16 * (l >> 5) + 32 * (j >> 4) + (j & 15)) if j < 32 else None,
    })
    ea, eb = elements(a8, 8, 16), elements(b8, 8, 16)
    check("i8", ea, eb, c8, 32, {
        "k=16h+j": lambda l, j: 16 * (l >> 5) + j,
        "k=8h+16(j>>3)+(j&7)": lambda l, j: 8 * (l >> 5) + 16 * (j >> 3) + (j & 7),
    })


if __name__ == "__main__":
    main()
