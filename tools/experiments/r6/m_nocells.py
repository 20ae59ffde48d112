# wrong-output probe: ldpc_map_kernel without the column twist + demux (map_cells); idx keeps stale LDS bytes
EDITS = [("  __syncthreads();\n  map_cells<FEC_THREADS>(md, cww, idx, tid);\n  __syncthreads();\n  if (md.rotation) {",
          "  __syncthreads();\n  __syncthreads();\n  if (md.rotation) {")]
