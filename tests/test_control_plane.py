"""CPU parity of the engine's host control plane (no GPU).

tests/native/cp_harness drives tonk_amd/csrc/{encoder,decoder,engine}.cpp through each golden
scenario; the device programs they emit are executed by the oracle's CPU interpreter of the
program format (oracle_run_program).  The resulting transcript -- every recovery packet digest,
every decode with recovered-payload digests, every acknowledgement, the codec statistics --
must equal the REFERENCE codec's transcript byte for byte.

Modes: ``sync`` runs each program as soon as a result is needed (one program per API call, as
the C-ABI does); ``batch`` defers execution over ``batch`` originals (as the device-resident
session does), which exercises chain snapshots, expansion of in-flight rows and multi-level
programs.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import NATIVE, _make, first_diff, golden_text

SCENARIOS = ["c1_256_p3", "c2_4096_p1_ack64", "c2_4096_p1_noack", "c3_4096_p2_ack64_s0",
             "c3_4096_p2_ack64_s1", "c3_4096_p2_ack64_s63", "c4_4096_p1_ack64_s511", "c5_65536_ge5_b4",
             "var_1_1500_p2_ack32", "tiny_1_20_p5_ack16", "big_9000_p3_ack64", "hiloss_p20_arq",
             "norecloss_p5_arq", "single_p0", "burst8_p5"]
MODES = [("sync", 0), ("batch", 1000), ("batch", 4096), ("sync-dirty", 0), ("batch-dirty", 1000)]


@pytest.fixture(scope="module")
def harness():
    _make(NATIVE, "_build/cp_harness")
    return os.path.join(NATIVE, "_build", "cp_harness")


@pytest.mark.parametrize("mode,batch", MODES)
@pytest.mark.parametrize("name", SCENARIOS)
def test_control_plane_matches_reference(harness, golden_index, tmp_path, name, mode, batch):
    sc = golden_index["scenarios"][name]
    sid = sc["stream"]
    out = tmp_path / "t.txt"
    # "-dirty": flushes visit only the codecs touched since the last one (the C ABI's context)
    base, dirty = mode.split("-")[0], int(mode.endswith("-dirty"))
    args = [harness, str(out), f"mode={base}", f"batch={batch}", f"dirty={dirty}"] + sc["args"] + [
        f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = out.read_text()
    want = golden_text(name)
    assert got == want, first_diff(want, got)
