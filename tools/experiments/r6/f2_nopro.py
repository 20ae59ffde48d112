# wrong-output probe: no CRC prologue per segment
EDITS = [("""      for (int q = qa; q < q0; q++) {
        TsWin w = ts_fetch<false>(R.tin, io.ts_len, R.rel);""", """      R.rel += 32 * BBCH_PRO;
      for (int q = q0; q < q0; q++) {
        TsWin w = ts_fetch<false>(R.tin, io.ts_len, R.rel);""")]
