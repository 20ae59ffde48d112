# wrong-output probe: ldpc_map_kernel without the LDPC parity rows (ldpc_rows); the scans run on stale rows
EDITS = [("  ldpc_rows<DW>(D, cur, ents, rowp, q, tid, FEC_THREADS);\n  __syncthreads();\n  {\n    // q <= 128",
          "  if (DW != FEC_DW_PASS) ldpc_rows<DW>(D, cur, ents, rowp, q, tid, FEC_THREADS);\n  __syncthreads();\n  {\n    // q <= 128")]
