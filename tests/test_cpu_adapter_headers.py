"""the GNU Radio adapters (include/dvbt2ll/*_impl_hip.h) compile against gr-dvbt2ll's
own public headers, unmodified, where they lie (/root/reference/include: the make() declarations of
include/dvbt2ll/{bbheaderbch_bb,interleavermod_bc,framemapperfint_cc,pilotgenp1insert_cc}.h:49 and the
enums of dvbt2ll_config.h:60-202); only GNU Radio's and Boost's headers, absent from the image, are
stand-ins (tests/gr_stub/{gnuradio,boost}).  Each adapter's out-of-class make() definition must match
the real declaration, and every enumerator the C ABI receives as an int must have the value
dvbt2ll/enums.py gives it.  Skipped where the reference is absent (the GPU box)."""
import subprocess
from pathlib import Path

import pytest

from dvbt2ll import enums as E

ROOT = Path(__file__).resolve().parents[1]
REFINC = Path("/root/reference/include")
pytestmark = pytest.mark.skipif(not (REFINC / "dvbt2ll" / "bbheaderbch_bb.h").exists(),
                                reason="reference headers absent")
ADAPTERS = ["bbheaderbch_bb", "ldpc_bb", "interleavermod_bc", "framemapperfint_cc", "pilotgenp1insert_cc"]


def _compile(tmp_path, src):
    f = tmp_path / "tu.cpp"
    f.write_text(src)
    return subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-Wall", "-Wextra", "-Wno-unused-parameter",
                           "-I" + str(ROOT / "tests" / "gr_stub"), "-I" + str(REFINC), "-I" + str(ROOT / "include"),
                           str(f)], capture_output=True, text=True)


@pytest.mark.parametrize("name", ADAPTERS)
def test_adapter_make_matches_reference_header(tmp_path, name):
    r = _compile(tmp_path, "#define DVBT2LL_HIP_DEFINE_MAKE\n#include <dvbt2ll/%s_impl_hip.h>\n" % name)
    assert r.returncode == 0, r.stderr


def test_adapter_rejects_a_wrong_make_signature(tmp_path):
    """the check has teeth: a make() whose signature differs from the reference declaration fails"""
    r = _compile(tmp_path, "#include <dvbt2ll/bbheaderbch_bb.h>\nnamespace gr { namespace dvbt2ll {\n"
                 "bbheaderbch_bb::sptr bbheaderbch_bb::make(dvbt2_framesize_t, dvbt2_code_rate_t, int, "
                 "dvbt2_inband_t, int, int) { return bbheaderbch_bb::sptr(); }\n}}\n")
    assert r.returncode != 0


def test_enum_values_match_reference_header(tmp_path):
    names = [n for n in dir(E) if n.isupper() and isinstance(getattr(E, n), int)]
    assert len(names) > 60
    body = "".join("static_assert((int)gr::dvbt2ll::%s == %d, \"%s\");\n" % (n, getattr(E, n), n) for n in names)
    r = _compile(tmp_path, "#include <dvbt2ll/dvbt2ll_config.h>\n" + body)
    assert r.returncode == 0, r.stderr
