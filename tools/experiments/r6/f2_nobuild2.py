# wrong-output probe: the piece is the raw window (no CRC, sync substitution, header, tail or PRBS); the cursors
# still advance (the TS is streamed as in the product)
EDITS = [("""      if (q + 1 < q1) build(q + 1, wn, a);""", """      if (q + 1 < q1) {
#pragma unroll
        for (int k = 0; k < 4; k++) a[k] = wn.a[k] ^ wn.p[k];
        if (!HEM) {
          R.rel += 32;
          R.m += 32;
          R.m -= R.m >= 188 ? 188 : 0;
        } else {
          R.sh += 32;
          R.r += 32;
          if (R.r >= 187) {
            R.r -= 187;
            R.sh += 1;
          }
        }
      }""")]
