"""CPU checks of the header-compatible helpers Tonk takes beside siamese.h (SURVEY.md s8(b):
TonkineseTools.h:61-62 includes SiameseTools.h and SiameseSerializers.h).

* tests/native/tools_check.cpp, compiled against include/ (tonk_amd's SiameseTools.h /
  SiameseSerializers.h), prints the results of PCGRandom, the little-endian readers/writers, the
  Write/ReadByteStream cursors and WindowedMinMax (min and max orderings, expiring windows,
  resets, a wrapping clock) on seeded inputs.  The same driver compiled against the REFERENCE
  headers (oracle/_ref/tools_check_ref, when the reference tree was present at build time) must
  print the same, and so must the committed fixture tests/golden/tools_check.txt (that build's
  output; tests/golden/make_tools_check.sh regenerates it).
* libtonk_amd.so exports siamese::GetTimeUsec / GetTimeMsec (the reference's
  SiameseTools.cpp:81-117), which the Tonk relink (oracle/tonk.mk: unit_tests_amd) takes from it;
  they read the wall clock (gettimeofday) in microseconds / milliseconds.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import pytest

from conftest import ROOT

OURS = os.path.join(ROOT, "tests", "native", "_build", "tools_check")
REF = os.path.join(ROOT, "oracle", "_ref", "tools_check_ref")
FIXTURE = os.path.join(ROOT, "tests", "golden", "tools_check.txt")


def _run(exe: str) -> str:
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "native"), "_build/tools_check"], check=True,
                       capture_output=True)
    return subprocess.run([exe], check=True, capture_output=True, text=True, timeout=60).stdout


def test_helpers_match_reference_fixture():
    got = _run(OURS)
    want = open(FIXTURE).read()
    assert got == want


def test_helpers_match_reference_headers_build():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/tools_check_ref not built (reference tree absent at build time)")
    ref = subprocess.run([REF], check=True, capture_output=True, text=True, timeout=60).stdout
    assert ref == open(FIXTURE).read(), "fixture is stale: regenerate with tests/golden/make_tools_check.sh"
    assert _run(OURS) == ref


def test_fixture_covers_every_helper():
    text = open(FIXTURE).read()
    for key in ("pcg 0:", "pcg hash", "serial hash", "stream hash", "winminmax 0:", "winminmax 3:",
                "SIAMESE_PACKET_NUM_INC 6 0"):
        assert key in text, key


def test_library_exports_the_clocks():
    lib = ctypes.CDLL(os.path.join(ROOT, "tonk_amd", "libtonk_amd.so"))
    usec = getattr(lib, "_ZN7siamese11GetTimeUsecEv")  # siamese::GetTimeUsec()
    msec = getattr(lib, "_ZN7siamese11GetTimeMsecEv")  # siamese::GetTimeMsec()
    usec.restype = msec.restype = ctypes.c_uint64
    t0 = time.time()
    u, m = usec(), msec()
    assert abs(u / 1e6 - t0) < 2.0  # gettimeofday's wall clock, as the reference
    assert abs(m - u // 1000) <= 5
    assert usec() >= u
