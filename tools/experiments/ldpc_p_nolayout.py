# LDPC pass phase cost by subtraction (wrong output): no info-group layout (D left as it is)
EDITS = [("""    for (int it = tid; it < ngroups * (FEC_DW_PASS / 4); it += FEC_THREADS) {""",
          """    for (int it = tid; it < 0; it += FEC_THREADS) {""")]
