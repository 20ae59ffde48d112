# persistent 32K kernel, two units per workgroup (straight-line: the prefetch covers the first unit's stores)
import runpy, pathlib
EDITS = runpy.run_path(str(pathlib.Path(__file__).with_name("o32_persistent.py")))["EDITS"]
EDITS += [("""  for (int k = 0; k < nk; k++) {
    // the thread index laundered""", """#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (k >= nk) break;
    // the thread index laundered"""),
("""  return O32_PERSISTENT && nunits >= 2 * g ? g : 0;   // short launches keep one workgroup per unit""",
 """  return O32_PERSISTENT && nunits >= 2 * g ? ((nunits / 2 + 7) / 8) * 8 : 0;""")]
