# wrong-output probe: the TI store without the quad-entry loads (entries synthesised from the offset; the
# offset-table loads and the store pattern are unchanged)
EDITS = [("      e[u] = ld_off(qs, (uint32_t)(64 * c + lane) * 8u);\n      qa[u] = (uint32_t)kc(qb, c) + (uint32_t)ld_off(qo, (uint32_t)(64 * c + lane) * 2u);",
          "      qa[u] = (uint32_t)kc(qb, c) + (uint32_t)ld_off(qo, (uint32_t)(64 * c + lane) * 2u);\n      e[u] = make_uint2((qa[u] & 0x1FFFu) * 0x10001u, ((qa[u] + 7u) & 0x1FFFu) * 0x10001u);")]
