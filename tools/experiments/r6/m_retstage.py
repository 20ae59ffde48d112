# wrong-output probe: ldpc_map_kernel ends after staging the BBFRAME, BCH parity and LDPC tables in LDS
EDITS = [("  // four words of a group per item, one 16-byte LDS write\n",
          "  if (md.cs > 0) return;\n")]
