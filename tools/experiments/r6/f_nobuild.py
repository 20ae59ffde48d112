# wrong-output probe: the fused BB + BCH pass with the A piece = the raw TS window (no CRC, header, PRBS, tail)
EDITS = [("      if (q + 1 < q1) build(q + 1, wn, a);",
          "      if (q + 1 < q1) win_bytes(wn.w, wn.o, a);")]
