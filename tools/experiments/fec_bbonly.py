# wrong-output experiment: the chain's FEC kernel stops after the BBFRAME (written to the codeword
# buffer): the cost of a BB-only first pass at the product kernel's occupancy
EDITS = [("    // ---- BCH on wave 0 (raised issue priority",
          "    if (MODE == FEC_TS_TO_TEMPU) {\n"
          "      uint32_t *dw = (uint32_t *)(io.out + (int64_t)bi * io.cw_stride);\n"
          "      for (int i = tid; i < (L + 3) >> 2; i += FEC_THREADS) dw[i] = ((const uint32_t *)frame)[i];\n"
          "      break;\n    }\n    // ---- BCH on wave 0 (raised issue priority")]
