# experiment: ldpc_map_kernel at 6 workgroups per CU with the TI quad table loads before map_cells
EDITS = [('__global__ __launch_bounds__(FEC_THREADS, FEC_PASS_WG_PER_CU) void ldpc_map_kernel(FecDev fd, FecIO fio, MapDev md,', '__global__ __launch_bounds__(FEC_THREADS, 6) void ldpc_map_kernel(FecDev fd, FecIO fio, MapDev md,'),
("""  uint8_t *idx = smem + 4 * ncw;
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
