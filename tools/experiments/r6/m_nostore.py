# wrong-output probe: the TI store's loads and pair math without its stores
EDITS = [("      if (c < nch && 64 * c + lane < nqd) {\n        if (!((e[u].x | e[u].y) & 0x80008000u)) {",
          "      if (c < nch && 64 * c + lane < nqd && v.x == 0x5A5A5A5Au && v.y == qa[u]) {\n        if (!((e[u].x | e[u].y) & 0x80008000u)) {")]
