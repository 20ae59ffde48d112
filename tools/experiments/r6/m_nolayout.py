# wrong-output probe: ldpc_map_kernel without the LDPC info-group layout (D keeps stale LDS contents)
EDITS = [("  for (int it = tid; it < ngroups * (FEC_DW_PASS / 4); it += FEC_THREADS) {",
          "  for (int it = tid; it < 0; it += FEC_THREADS) {")]
