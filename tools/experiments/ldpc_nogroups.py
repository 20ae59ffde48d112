# wrong-output experiment: the chain's LDPC pass without the info-group layout
EDITS = [("""    for (int it = tid; it < ngroups * FEC_DW; it += FEC_THREADS) {
      const int g = it / FEC_DW;
      ldpc_group_word(D, frame, g, it - g * FEC_DW);
    }
    __syncthreads();
    const uint32_t *cur = fec_ldpc(d, D, ngroups, ents, rowp, Wv, tid);""",
          """    const uint32_t *cur = fec_ldpc(d, D, ngroups, ents, rowp, Wv, tid);""")]
