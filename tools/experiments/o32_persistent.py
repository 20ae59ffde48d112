# persistent 32K kernel (one workgroup per CU walking its XCD's units; the next unit's half-0 inputs
# requested ahead of the current unit's stores), thread index laundered per iteration
import runpy, pathlib
EDITS = [("""constexpr bool O32_PERSISTENT = false;""", """constexpr bool O32_PERSISTENT = true;""")]
EDITS += runpy.run_path(str(pathlib.Path(__file__).with_name("o32_launder.py")))["EDITS"]
