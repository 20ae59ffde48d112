# wrong-output probe: every TS window read from the buffer's start (no TS streaming from HBM)
EDITS = [("""      TsWin w = ts_fetch<HEM>(R.tin, io.ts_len, rel);
      prbs(c, w);""", """      TsWin w = ts_fetch<HEM>(R.tin, io.ts_len, (rel & 63) + 64);
      prbs(c, w);""")]
