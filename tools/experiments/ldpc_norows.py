# wrong-output experiment: the chain's LDPC pass without rows / accumulate / column parities
EDITS = [("    const uint32_t *cur = fec_ldpc(d, D, ngroups, ents, rowp, Wv, tid);",
          "    const uint32_t *cur = D + ngroups * FEC_DW;")]
