# wrong-output probe: the interleaver-input words without ldpc_out_word (one LDS word each instead)
EDITS = [("    w[k] = i < nw ? ldpc_out_word(fd, frame, cur, i) : 0u;",
          "    w[k] = i < nw ? cur[i & 511] : 0u;")]
