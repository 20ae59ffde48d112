# map kernel block order: each XCD takes one of 8 contiguous ranges of the block-in-frame index r for
# every frame of the launch (frame-major inside the range), so its L2 holds 1/8 of the partition-delta
# table instead of re-reading the whole table from the Infinity Cache for every frame
EDITS = [("static_assert(MAP_THREADS == L1_NT,",
          """__device__ __forceinline__ int map_rgroup_block(int i, int n, int F) {
  const int L = xcd_major(i, n), nf = n / F;
  int base = 0, rlo = 0, sz = 1;
  for (int g = 0; g < 8; g++) {
    rlo = g * F / 8;
    sz = (g + 1) * F / 8 - rlo;
    if (L < base + sz * nf) break;
    base += sz * nf;
  }
  const int k = L - base;
  return (k / sz) * F + rlo + k % sz;
}
static_assert(MAP_THREADS == L1_NT,"""),
         ("  const int blk = xcd_major((int)blockIdx.x - nl1, (int)gridDim.x - nl1);",
          "  const int blk = map_rgroup_block((int)blockIdx.x - nl1, (int)gridDim.x - nl1, d.F);")]
