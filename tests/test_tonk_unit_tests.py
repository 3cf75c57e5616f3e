"""Tonk's own unit_tests (tests/TonkUnitTest.cpp of the reference: sender bandwidth control,
lossy full-duplex transfers under the Mau simulator with memcmp checks, compression, time sync)
built from the reference sources with the Siamese codec replaced by libtonk_amd.so
(oracle/tonk.mk -> oracle/_ref/tonk/unit_tests_amd).  Tonk's sources are linked unchanged: this is
the drop-in check of SURVEY.md s8(f)1."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "oracle", "_ref", "tonk", "unit_tests_amd")


@pytest.mark.gpu
@pytest.mark.skipif(not os.environ.get("TONK_AMD_TONK_UNIT_TESTS"),
                    reason="opt-in (TONK_AMD_TONK_UNIT_TESTS=1): ~5 min on one MI355X (SUCCESS, "
                           "profiles/r01_tonk_unit_tests_gpu.txt), longer than a parity test should run")
def test_tonk_unit_tests_with_mi355x_codec():
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/tonk/unit_tests_amd not built (needs /root/reference at build time)")
    # the C ABI watchdog prints call/wait counts to stderr every 5 s (Tonk's own log is buffered)
    env = dict(os.environ, TONK_AMD_CAPI_WATCH="5")
    r = subprocess.run([EXE], stdin=subprocess.DEVNULL, capture_output=True, text=True, timeout=1200, env=env)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    assert "SUCCESS" in log, log[-3000:]
