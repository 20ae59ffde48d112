# wrong-output probe: the NM CRC replaced by two XORs
EDITS = [("""        crc = crc_chunk(tp, tq, pmask, raw, e, h, crc, slot);""",
          """        slot = raw[0] ^ crc;
        crc = raw[1];""")]
