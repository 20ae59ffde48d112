# experiment: no asm pin of the accumulators before the build (the compiler schedules MFMAs and build freely)
EDITS = [("      for (int t = 0; t < NT; t++) asm volatile(\"\" : \"+v\"(acc[t]));\n", "      for (int t = 0; t < NT; t++) {}\n")]
