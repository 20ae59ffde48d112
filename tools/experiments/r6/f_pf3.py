# experiment: TS pieces fetched three chunks ahead
EDITS = [
("""    auto fetch2 = [&]() -> TsWin {
      const int64_t rel = HEM ? R.sh + 32 + (R.r + 32 >= 187 ? 1 : 0) - io.ts_base : R.rel + 32;
      return ts_fetch<HEM>(R.tin, io.ts_len, rel);
    };""",
"""    auto fetch2 = [&]() -> TsWin {   // two chunks after the cursor's
      const int64_t rel = HEM ? R.sh + 64 + (R.r + 64 >= 374 ? 2 : R.r + 64 >= 187 ? 1 : 0) - io.ts_base : R.rel + 64;
      return ts_fetch<HEM>(R.tin, io.ts_len, rel);
    };
    auto fetch1 = [&]() -> TsWin {   // one chunk after the cursor's
      const int64_t rel = HEM ? R.sh + 32 + (R.r + 32 >= 187 ? 1 : 0) - io.ts_base : R.rel + 32;
      return ts_fetch<HEM>(R.tin, io.ts_len, rel);
    };"""),
("""      build(q0, w, a);
      wn1 = fetch(q0 + 1);""",
"""      build(q0, w, a);
      wn1 = fetch(q0 + 1);
      wn2 = fetch1();"""),
("""    TsWin wn1;""", """    TsWin wn1, wn2;"""),
("""      const TsWin wn = wn1;
      wn1 = fetch2();""",
"""      const TsWin wn = wn1;
      wn1 = wn2;
      wn2 = fetch2();"""),
]
