# LDPC pass phase cost by subtraction (wrong output): no interleaver-input word stores
EDITS = [("      dstw[i] = v;", "      if (v == 0x9E3779B9u) dstw[i] = v;")]
