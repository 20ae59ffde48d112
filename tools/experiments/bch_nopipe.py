# BCH matrix-core pass without the register double-buffering of the B fragments
EDITS = [("""    uint4 bc[NT], bx[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) bc[t] = bq[t * 64 + lane];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (u < 3) {
#pragma unroll
        for (int t = 0; t < NT; t++) bx[t] = bq[((u + 1) * NT + t) * 64 + lane];
      }
      const uint32_t w""", """#pragma unroll
    for (int u = 0; u < 4; u++) {
      uint4 bc[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) bc[t] = bq[(u * NT + t) * 64 + lane];
      const uint32_t w"""),
         ("""      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < NT; t++) bc[t] = bx[t];
    }""", """      __builtin_amdgcn_sched_barrier(0);
    }""")]
