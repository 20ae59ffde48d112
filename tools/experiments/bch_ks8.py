# BCH matrix-core pass with 8 K slices (one per XCD) instead of 16
EDITS = [("  const int slice = (int)blockIdx.x % BCH_KS, tile = (int)blockIdx.x / BCH_KS;\n  const int q0 = slice * d.bch_nq / BCH_KS, q1 = (slice + 1) * d.bch_nq / BCH_KS;",
          "  const int slice = (int)blockIdx.x % 8, tile = (int)blockIdx.x / 8;\n  const int q0 = slice * d.bch_nq / 8, q1 = (slice + 1) * d.bch_nq / 8;"),
         ("dim3(tiles * BCH_KS), dim3(FEC_THREADS)", "dim3(tiles * 8), dim3(FEC_THREADS)")]
