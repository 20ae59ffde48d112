# wrong-output probe: the LDPC parity rows only (no accumulate scan, no column-parity correction)
EDITS = [("  const uint32_t *cur = fec_ldpc<FEC_DW_PASS>(fd, D, ngroups, ents, rowp, Wv, tid);",
          "  uint32_t *cur = D + ngroups * FEC_DW_PASS;\n  ldpc_rows<FEC_DW_PASS>(D, cur, ents, rowp, fd.q, tid, FEC_THREADS);\n  __syncthreads();")]
