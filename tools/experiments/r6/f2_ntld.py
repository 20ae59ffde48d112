# experiment: the TS window loads nontemporal
EDITS = [("""  const u32x4 x = ((g4uptr)src)->v;""", """  const u32x4 x = __builtin_nontemporal_load(&((g4uptr)src)->v);""")]
