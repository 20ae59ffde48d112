# ldpc_map_kernel blocks r-grouped per XCD: in each group of 8 frames, XCD x takes the FEC block indices
# [x F / 8, (x + 1) F / 8) of all 8 frames (r-major), so each XCD's L2 holds an eighth of the TI-store quad
# table (2.5 B per cell, re-read from MALL for every frame with the frame-major order)
EDITS = [(
    """  const int blk = xcd_major((int)blockIdx.x - nl1, (int)gridDim.x - nl1);
  const int L = fd.kbch >> 3, PB = fd.P >> 3;""",
    """  const int nb = (int)gridDim.x - nl1, wg = (int)blockIdx.x - nl1, F = md.F;
  int blk;
  if (nb % (8 * F) == 0) {
    const int x = wg & 7, i = wg >> 3, g = i / F, lg = x * F + (i - g * F);
    blk = (8 * g + (lg & 7)) * F + (lg >> 3);
  } else {
    blk = xcd_major(wg, nb);
  }
  const int L = fd.kbch >> 3, PB = fd.P >> 3;""")]
