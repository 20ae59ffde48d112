# wrong-output probe: ldpc_map_kernel without the L1-post workgroups' work (they still launch and return)
EDITS = [("    if ((int)blockIdx.x < l1io.nframes) l1post_frame(l1d, l1io, blockIdx.x, (uint32_t *)smem);\n", "")]
