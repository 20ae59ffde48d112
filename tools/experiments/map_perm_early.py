# map kernel (compact path): the cell-interleaver permutation quads requested at kernel start (in flight
# during the codeword load and the column twist / demux) instead of after the demux barrier
EDITS = [
 ("""__device__ void map_store_pairs(const MapDev &d, uint16_t *out_pairs, int64_t frame_stride, const uint8_t *idx,
                                uint16_t *stage, int blk, int tid, bool alias) {""",
  """__device__ void map_store_pairs(const MapDev &d, uint16_t *out_pairs, int64_t frame_stride, const uint8_t *idx,
                                uint16_t *stage, int blk, int tid, bool alias, const uint2 *pqe) {"""),
 ("""      pq[k] = ld_off((const uint2 *)d.ci_perm, (uint32_t)q * 8u);
      wv[k] = idxw[q];""",
  """      pq[k] = pqe[k];
      wv[k] = idxw[q];"""),
 ("""  const int cs = d.cs, nl = d.nldpc;
  if (!io.apply_ci)
    for (int i = tid; i < 256; i += MAP_THREADS) lut[i] = d.lut[i];""",
  """  const int cs = d.cs, nl = d.nldpc;
  uint2 pqe[CQ];
  if (compact) {
#pragma unroll
    for (int k = 0; k < CQ; k++)
      pqe[k] = ld_off((const uint2 *)d.ci_perm, (uint32_t)min(tid + k * MAP_THREADS, ((cs + 3) >> 2) - 1) * 8u);
  }
  if (!io.apply_ci)
    for (int i = tid; i < 256; i += MAP_THREADS) lut[i] = d.lut[i];"""),
 ("""  map_store_pairs<MAP_THREADS, CQ>(d, io.out_pairs, io.frame_stride, idx, stage, blk, tid, compact);""",
  """  map_store_pairs<MAP_THREADS, CQ>(d, io.out_pairs, io.frame_stride, idx, stage, blk, tid, compact, pqe);"""),
]
