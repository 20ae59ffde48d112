# wrong-output experiment: the chain's FEC kernel without the BCH (parity zero) -- bounds what moving
# the BCH out of the fused kernel can save
EDITS = [("      switch (P) {   // compile-time register geometry",
          "      if (d.kbch > 0) { a[0] = a[1] = a[2] = 0; } else\n      switch (P) {   // compile-time register geometry")]
