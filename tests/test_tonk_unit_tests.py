"""Tonk's own unit_tests (tests/TonkUnitTest.cpp of the reference: sender bandwidth control,
lossy full-duplex transfers under the Mau simulator with memcmp checks, compression, time sync)
built from the reference sources with the Siamese codec replaced by libtonk_amd.so
(oracle/tonk.mk -> oracle/_ref/tonk/unit_tests_amd).  Tonk's sources are linked unchanged: this is
the drop-in check of SURVEY.md s8(f)1.

unit_tests_amd_lz additionally replaces PacketCompression.cpp with the GPU MessageCompressor
(integration/tonk/PacketCompressionAmd.cpp): every reliable datagram Tonk sends is
compressed on the GPU, concurrent connections' calls combined into one launch (compress.cpp).
Both binaries run in the default -m gpu pass.  The compressor's parity is tests/test_compress.py."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT

BINARIES = ["unit_tests_amd", "unit_tests_amd_lz"]
if os.environ.get("TONK_AMD_TONK_BINARY"):
    BINARIES = [os.environ["TONK_AMD_TONK_BINARY"]]


@pytest.mark.gpu
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("binary", BINARIES)
def test_tonk_unit_tests_with_mi355x_codec(binary):
    """Every Tonk unit test must pass, on the binary's one and only run.  TestBandwidthControl is
    a wall-clock simulation (100 lossy connections through the Mau proxy, 300 s limit) whose
    outcome depends on how fast the codec calls are from the first second on: the C ABI's calls
    go through the launch-free persistent executor (server.h), so no runtime enqueue under a
    process-wide lock can stall every connection."""
    exe = os.path.join(ROOT, "oracle", "_ref", "tonk", binary)
    if not os.path.exists(exe):
        pytest.skip(f"oracle/_ref/tonk/{binary} not built (needs /root/reference at build time)")
    # the C ABI watchdog prints call/wait counts to stderr every 5 s (Tonk's own log is buffered)
    # The log streams to gpurun_out/ while the test runs (a run that writes nothing for minutes
    # looks hung to the GPU-box harness).
    env = dict(os.environ, TONK_AMD_CAPI_WATCH="5")
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"tonk_{binary}.log")
    with open(path, "w") as f:
        r = subprocess.run([exe], stdin=subprocess.DEVNULL, stdout=f, stderr=subprocess.STDOUT, timeout=700, env=env)
    with open(path) as f:
        log = f.read()
    assert r.returncode == 0, log[-3000:]
    assert "SUCCESS" in log, log[-3000:]
