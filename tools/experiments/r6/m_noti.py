# wrong-output probe: ldpc_map_kernel without the TI store (map_store_quads)
EDITS = [("    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);\n  } else {\n    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);",
          "  } else {")]
