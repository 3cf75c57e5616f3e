"""CPU parity of the engine's host control plane (no GPU).

tests/native/cp_harness drives tonk_amd/csrc/{encoder,decoder,engine}.cpp through each golden
scenario; the device programs they emit are executed by the oracle's CPU interpreter of the
program format (oracle_run_program).  The resulting transcript -- every recovery packet digest,
every decode with recovered-payload digests, every acknowledgement, the codec statistics --
must equal the REFERENCE codec's transcript byte for byte.

Modes: ``sync`` runs each program as soon as a result is needed (one program per API call, as
the C-ABI does); ``batch`` defers execution over ``batch`` originals (as the device-resident
session does), which exercises chain snapshots, expansion of in-flight rows and multi-level
programs; ``batch-pipe`` adds the session's level pipelining (a program's upper levels run
beside the next program's first levels) and checks those pairs for read/write hazards.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import NATIVE, _make, first_diff, golden_text

SCENARIOS = ["c1_256_p3", "c2_4096_p1_ack64", "c2_4096_p1_noack", "c3_4096_p2_ack64_s0",
             "c3_4096_p2_ack64_s1", "c3_4096_p2_ack64_s63", "c4_4096_p1_ack64_s511", "c5_65536_ge5_b4",
             "var_1_1500_p2_ack32", "tiny_1_20_p5_ack16", "big_9000_p3_ack64", "hiloss_p20_arq",
             "norecloss_p5_arq", "single_p0", "burst8_p5", "rtx_p2_ack64", "rtx_p5_ack32", "rtx_p3_noack",
             "rtx_restart_p1_ack4", "rtx_restart_p2_ack2"]
MODES = [("sync", 0), ("batch", 1000), ("batch", 4096), ("sync-dirty", 0), ("batch-dirty", 1000),
         ("batch-pipe", 1000), ("batch-pipe", 4096), ("batch-pipedrain", 1000), ("batch-pipeexp", 512),
         ("batch-pipesplit", 1000), ("sync-exp", 0), ("batch-pipecontig", 4096), ("batch-pipecontigsplit", 1000)]


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
    # "-dirty": flushes visit only the codecs touched since the last one (the C ABI's context);
    # "-pipe": levels pipelined across programs as the session launches them, every pair of
    # levels that would run together checked for hazards; "-pipedrain": every second program
    # also completes all in-flight ones (the session's record mode), so rows are reused sooner
    base, dirty = mode.split("-")[0], int(mode.endswith("-dirty"))
    # "-pipeexp": also the few-stream session's expansion limit (expansions over 16 terms are
    # read as rows, one level up) and its back substitution over materialized rows (from 2
    # unknowns)
    pipe, drain = int("-pipe" in mode), 2 * int(mode.endswith("-pipedrain"))
    # "-exp" alone: the same limits on per-call programs (the siamese.h C ABI's contexts)
    few = mode.endswith("exp")
    expand = 16 if few else 0xFFFFFFFF
    backsub = 2 if few else 0xFFFFFFFF
    # the batched session splits direct dense ranges over 48 packets (Context::dense_split);
    # "-pipesplit" splits every range over 16, so most Siamese rows take the two-level form
    split = 16 if mode.endswith("split") else 48 if mode in ("batch-pipe", "batch-pipedrain", "batch-pipecontig") else 0
    # "-pipecontig": every original in a row reserved up front, in order, borrowed by the codecs
    # (the batched session's layout): windows are long segments, so Siamese rows read their sum
    # ranges straight from the packets and consecutive ones are grouped (Encoder::defer_dense)
    contig = int("contig" in mode)
    # (every mode also checks that no op of a level writes a row another op of that level uses)
    # "sync-exp" and "batch-dirty" also encode ahead as the C ABI does (Encoder::encode_is_quiet,
    # rewind): up to 15 and 3 recovery packets
    ahead = 15 if mode == "sync-exp" else 3 if mode == "batch-dirty" else 0
    args = [harness, str(out), f"mode={base}", f"batch={batch}", f"dirty={dirty}", f"pipeline={pipe}",
            f"drain={drain}", f"expand={expand}", f"backsub={backsub}", f"split={split}", f"contig={contig}",
            f"ahead={ahead}"] + sc["args"] + [
        f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = out.read_text()
    want = golden_text(name)
    assert got == want, first_diff(want, got)


@pytest.mark.parametrize("contig", [0, 1])
@pytest.mark.parametrize("batch_name,sid", [("cfg2_64x4096_p2_ack64", 0), ("cfg2_64x4096_p2_ack64", 37),
                                             ("cfg3_rank7_64x12288_p1_ack64", 448),
                                             ("cfg3_rank7_64x12288_p1_ack64", 511)])
def test_control_plane_batch_streams(harness, golden_index, tmp_path, batch_name, sid, contig):
    """Streams of the multi-stream fixtures (BASELINE configs[2], the rank-7 shard of configs[3])
    through the control plane in the bench's batch mode, pipelined as the session launches it in
    record mode: transcript digest == reference's, no launch-order hazard."""
    import hashlib
    entry = golden_index["batches"][batch_name]
    out = tmp_path / "t.txt"
    args = [harness, str(out), "mode=batch", "batch=4096", "dirty=0", "pipeline=1", "drain=2", "split=48",
            f"contig={contig}"] + entry["args"] + [
        f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == entry["streams"][str(sid)]["sha256"]
