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
    # ... and "sync-exp" / "batch-pipeexp" take the C ABI's and the few-stream session's lane-sum
    # snapshot levels (Context::short_scans)
    short = int(mode in ("sync-exp", "batch-pipeexp"))
    args = [harness, str(out), f"mode={base}", f"batch={batch}", f"dirty={dirty}", f"pipeline={pipe}",
            f"drain={drain}", f"expand={expand}", f"backsub={backsub}", f"split={split}", f"contig={contig}",
            f"ahead={ahead}", f"short={short}"] + sc["args"] + [
        f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = out.read_text()
    want = golden_text(name)
    assert got == want, first_diff(want, got)


@pytest.mark.parametrize("mode", [["mode=batch", "batch=4096"], ["mode=batch", "batch=1000", "pipeline=1", "split=48", "contig=1"],
                                  ["mode=sync", "dirty=1", "expand=16", "backsub=2"]])
@pytest.mark.parametrize("name", ["c2_4096_p1_ack64", "c3_4096_p2_ack64_s63", "c5_65536_ge5_b4", "hiloss_p20_arq",
                                  "burst8_p5", "big_9000_p3_ack64"])
def test_control_plane_lane_eliminations(harness, golden_index, tmp_path, name, mode):
    """The decoder's Siamese-row eliminations through its running lane sums only (ddirect=0), the
    path rows with long or fragmented sum ranges take (the default reads short ranges of long
    runs straight from the packets, Decoder::eliminate_direct): transcript == reference's."""
    sc = golden_index["scenarios"][name]
    sid = sc["stream"]
    out = tmp_path / "t.txt"
    r = subprocess.run([harness, str(out), "ddirect=0"] + mode + sc["args"] +
                       [f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    want = golden_text(name)
    assert out.read_text() == want, first_diff(want, out.read_text())


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


@pytest.mark.parametrize("family,streams", [("cfg2", range(48, 64)), ("cfg4", range(0, 3)), ("p5_ack32", range(0, 8))])
def test_control_plane_vs_reference_build(harness, tmp_path, family, streams):
    """Whole streams through the control plane against transcripts the reference codec compiled
    from /root/reference (oracle/_ref/golden_gen, built by __graft_entry__.build) writes for the
    same seeds: configs[2] streams 48-63 (stream 56 is the decoder far behind whose thousands of
    failed solves Decoder::decode counts instead of repeating, with the list walks it caches), the
    decoder-stress configs[4] and a 5 %-loss family, in the C ABI's per-call mode with
    encode-ahead and in the batched session's mode."""
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "golden_gen")
    if not os.path.exists(exe):
        pytest.skip("reference build absent (oracle/_ref)")
    args = {
        "cfg2": "n=4096 pmin=1300 pmax=1300 loss=85899345 ge=0 gb=0 bg=0 lossrec=1 fec=2621 ack=64 ackbytes=256 arq=0 flush=4096",
        "cfg4": "n=65536 pmin=1300 pmax=1300 loss=0 ge=1 gb=56512727 bg=1073741824 lossrec=1 fec=6554 ack=256 ackbytes=256 arq=2048 flush=4096",
        "p5_ack32": "n=4096 pmin=1300 pmax=1300 loss=214748364 ge=0 gb=0 bg=0 lossrec=1 fec=5243 ack=32 ackbytes=256 arq=0 flush=4096",
    }[family].split()
    first = min(streams)
    ref = subprocess.run([exe, "transcripts", str(tmp_path / "r"), "threads=4", f"streams={max(streams) + 1 - first}",
                          f"stream={first}"] + args, capture_output=True, text=True, timeout=600)
    assert ref.returncode == 0, ref.stderr[-2000:]
    modes = [["mode=sync", "dirty=1", "expand=16", "backsub=2", "ahead=15", "short=1"],
             ["mode=batch", "batch=4096", "pipeline=1", "drain=2", "split=48", "contig=1"]]
    for s in streams:
        want = (tmp_path / f"r{s}.txt").read_text()
        for m in modes:
            out = tmp_path / "o.txt"
            r = subprocess.run([harness, str(out)] + m + args + [f"stream={s}", f"seed_data={1000 + s}",
                                                                 f"seed_loss={2000 + s}"],
                               capture_output=True, text=True, timeout=600)
            assert r.returncode == 0, r.stderr[-2000:]
            assert out.read_text() == want, f"stream {s} {m}: " + first_diff(want, out.read_text())


@pytest.mark.parametrize("name,mode", [
    ("wrap_p1_ack256_64B", ["mode=sync", "dirty=1", "expand=16", "backsub=2", "ahead=15", "short=1"]),
    ("wrap_p1_ack256_64B", ["mode=batch", "batch=4096", "pipeline=1", "drain=2", "split=48", "contig=1"]),
    ("wrap_p1_full_64B", ["mode=sync", "dirty=1", "expand=16", "backsub=2", "ahead=15", "short=1"]),
    ("full_p3_noack", ["mode=sync", "dirty=1", "expand=16", "backsub=2", "ahead=15", "short=1"]),
    ("full_p1_noack", ["mode=sync", "dirty=0", "expand=4294967295", "backsub=4294967295"]),
    ("full_p1_noack", ["mode=batch", "batch=4096", "pipeline=1", "drain=2", "split=48", "contig=1"]),
    ("full_p1_noack", ["mode=batch", "batch=1000", "dirty=1", "ahead=3"])])
def test_control_plane_long_streams(harness, golden_index, tmp_path, name, mode):
    """The window-full fixtures (full_*: no acks, 50,000 originals, the 16,000-packet window fills
    and a refused add waits for an acknowledgement, siamese.cpp:80-93, SiameseEncoder.cpp:91-96)
    and 4.3 M originals, past the 22-bit packet-number period (SiameseCommon.h:102): windows,
    Siamese sums, Cauchy rows and LDPC pairs straddle column 0x3FFFFF -> 0, in the C ABI's
    per-call mode and the batched session's pipelined contiguous mode.  wrap_p1_ack256: the
    reference decoder disables itself after the wrap and the encoder window fills up (the
    engine must do the same); wrap_p1_full: no acks, the 16,000-packet window fills ~360 times
    and recoveries continue across the wrap.  Transcript digest == the reference codec's.
    (The batched mode of wrap_p1_full takes ~4 minutes on one core: run by hand, not here.)"""
    import hashlib
    e = golden_index["long"].get(name) or golden_index["scenarios"][name]
    sid = e["stream"]
    out = tmp_path / "t.txt"
    r = subprocess.run([harness, str(out)] + mode + ["arena_mb=4096"] + e["args"] +
                       [f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    assert text.splitlines()[-1] == e["summary"]
    assert hashlib.sha256(text.encode()).hexdigest() == e["sha256"]
