# 8K ofdm_kernel with the next unit's first direct aux quad prefetched too (2 VGPRs spilled at the cap)
EDITS = [("  static constexpr bool AUX_PRE = N == 4096;", "  static constexpr bool AUX_PRE = N == 4096 || N == 8192;")]
