# wrong-output probe: ldpc_map_kernel without the BBFRAME / BCH-partial loads from HBM (synthetic frame bytes)
EDITS = [("      u[k] = tid + FEC_THREADS * k < nqi ? rowq[tid + FEC_THREADS * k] : make_uint4(0u, 0u, 0u, 0u);",
          "      u[k] = make_uint4((uint32_t)tid * 0x9E3779B9u, (uint32_t)k, (uint32_t)blk, 0x1234567u);"),
         ("    const uint32_t par = tid < (PB + 3) >> 2 ? fio.bch_part[(int64_t)blk * BCH_PART_WORDS + tid] : 0u;",
          "    const uint32_t par = (uint32_t)blk * 0x85EBCA6Bu;")]
