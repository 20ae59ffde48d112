# wrong-output probe: the fused BB + BCH pass without the CRC-8 streaming (no lookups, no lane exchanges)
EDITS = [("        crc = crc_chunk(tp, tq, raw, e, h, crc, slot);\n#pragma unroll\n        for (int k = 0; k < 4; k++) pd[k] = raw[k];",
          "        slot = raw[0] ^ crc;\n        crc = raw[1];\n#pragma unroll\n        for (int k = 0; k < 4; k++) pd[k] = raw[k];")]
