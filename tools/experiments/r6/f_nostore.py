# wrong-output probe: the fused BB + BCH pass without the BBFRAME stores
EDITS = [("      *(uint4 *)((R.live ? R.row : io.out + (int64_t)io.nblocks * io.cw_stride) + P0) = make_uint4(a[0], a[1], a[2], a[3]);",
          "      if (a[0] == 0x9E3779B9u && a[1] == (uint32_t)q) *(uint4 *)((R.live ? R.row : io.out + (int64_t)io.nblocks * io.cw_stride) + P0) = make_uint4(a[0], a[1], a[2], a[3]);")]
