# experiment: the TI quad table entries of the first store round loaded before the LDPC
EDITS = [("""  // rows without the column-parity correction: ldpc_out_word applies Wv as it reads them""", """  QuadRound pre;
  map_quads_load<FEC_THREADS>(md, blk, tid, 0, pre);
  // rows without the column-parity correction: ldpc_out_word applies Wv as it reads them"""),
("""    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);""",
 """    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid, &pre);"""),
("""    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);""",
 """    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid, &pre);"""),
]
