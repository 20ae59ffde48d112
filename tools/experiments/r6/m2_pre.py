# experiment: the TI quad table entries of the first store round loaded before the column twist (map_cells)
EDITS = [("""  uint8_t *idx = smem + 4 * ncw;
  __syncthreads();
  map_cells<FEC_THREADS>(md, cww, idx, tid);""", """  uint8_t *idx = smem + 4 * ncw;
  QuadRound pre;
  map_quads_load<FEC_THREADS>(md, blk, tid, 0, pre);
  __syncthreads();
  map_cells<FEC_THREADS>(md, cww, idx, tid);"""),
("""    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);""",
 """    map_store_quads<FEC_THREADS, true>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid, &pre);"""),
("""    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid);""",
 """    map_store_quads<FEC_THREADS, false>(md, mio.out_pairs, mio.frame_stride, idx, blk, tid, &pre);"""),
]
