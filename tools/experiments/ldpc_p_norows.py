# LDPC pass phase cost by subtraction (wrong output): no parity-row accumulation (rows left as they are)
EDITS = [("  ldpc_rows<DW>(D, cur, ents, rowp, q, tid, FEC_THREADS);", "  if (DW != FEC_DW_PASS) ldpc_rows<DW>(D, cur, ents, rowp, q, tid, FEC_THREADS);")]
