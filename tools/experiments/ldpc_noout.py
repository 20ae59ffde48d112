# wrong-output experiment: the chain's LDPC pass without its codeword output
EDITS = [("    for (int i = (L >> 2) + tid; i < (cwb + 3) >> 2; i += FEC_THREADS) {",
          "    for (int i = (L >> 2) + tid; i < (L >> 2); i += FEC_THREADS) {")]
