# wrong-output probe: every chunk multiplies the segment's first chunk's B fragments (no generator-table streaming)
EDITS = [("""      const bfr_t bs = bload(qn);
      wl = fetch2(q + 2);""", """      const bfr_t bs = bload(q0);
      wl = fetch2(q + 2);""")]
