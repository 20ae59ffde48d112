# wrong-output probe: the piece is the raw window (no CRC, sync substitution, header, tail or PRBS)
EDITS = [("""      if (q + 1 < q1) build(q + 1, wn, a);""", """      if (q + 1 < q1) {
#pragma unroll
        for (int k = 0; k < 4; k++) a[k] = wn.a[k] ^ wn.p[k];
      }""")]
