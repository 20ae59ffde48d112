# wrong-output probe: no BBFRAME staging or stores
EDITS = [("""      *(uint4 *)(stg + (wave * 32 + (lane & 31)) * BBCH_STG_STRIDE + (q & 3) * 32 + h * 16) =
          make_uint4(a[0], a[1], a[2], a[3]);
      if ((q & 3) == 3 || q == q1 - 1) {""", """      if (q < 0) {""")]
