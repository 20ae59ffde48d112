# experiment: TS pieces fetched two chunks ahead (the window for q + 2 issued in iteration q)
EDITS = [
("""    auto fetch = [&](int q) -> TsWin {   // every lane loads (dead rows from a safe address): no branch to merge
      return ts_fetch<HEM>(R.tin, io.ts_len, HEM ? R.sh - io.ts_base : R.rel);
    };""",
"""    auto fetch = [&](int q) -> TsWin {   // every lane loads (dead rows from a safe address): no branch to merge
      return ts_fetch<HEM>(R.tin, io.ts_len, HEM ? R.sh - io.ts_base : R.rel);
    };
    // the piece one chunk after the cursor's (the cursor is at the next chunk to build)
    auto fetch2 = [&]() -> TsWin {
      const int64_t rel = HEM ? R.sh + 32 + (R.r + 32 >= 187 ? 1 : 0) - io.ts_base : R.rel + 32;
      return ts_fetch<HEM>(R.tin, io.ts_len, rel);
    };"""),
("""      const TsWin w = fetch(q0);
      build(q0, w, a);""",
"""      const TsWin w = fetch(q0);
      build(q0, w, a);
      wn1 = fetch(q0 + 1);"""),
("""    uint32_t a[4];
    {
      const bfr_t bs = bload(q0);""",
"""    uint32_t a[4];
    TsWin wn1;
    {
      const bfr_t bs = bload(q0);"""),
("""      const bfr_t bs = bload(qn);
      const TsWin wn = fetch(qn);""",
"""      const bfr_t bs = bload(qn);
      const TsWin wn = wn1;
      wn1 = fetch2();"""),
]
