# IQ stores without the non-temporal hint (write-back through L2 instead of streaming)
EDITS = [("""      typedef float f4v __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(f4v{a.x, a.y, b.x, b.y}, (f4v *)(base + n * 8u));""",
          """      typedef float f4v __attribute__((ext_vector_type(4)));
      *(f4v *)(base + n * 8u) = f4v{a.x, a.y, b.x, b.y};""")]
