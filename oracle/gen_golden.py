#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: generate tests/golden fixtures from the REFERENCE codec.

Runs oracle/_ref/golden_gen (our workload driver linked against the reference Siamese codec
compiled from /root/reference by oracle/Makefile) for every scenario below and writes

  tests/golden/<name>.txt.gz     full transcript (every recovery packet digest, every decode,
                                 every ack, final stats) for small/medium scenarios
  tests/golden/scenarios.json    parameters + sha256 of each transcript (+ summary line)

The reference also memcmp-checks every recovered packet against the true payload while it
runs (golden_gen exits non-zero otherwise), so no fixture can pin a wrong decode.

usage: python oracle/gen_golden.py [--bench-streams 64 --bench-originals 49152]
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from tonk_amd import WorkloadParams  # noqa: E402  (parameter helpers only)

GEN = os.path.join(HERE, "_ref", "golden_gen")
OUT = os.path.join(ROOT, "tests", "golden")


def scenarios():
    """name -> (WorkloadParams, stream id, store full transcript?)"""
    s = {}
    s["c1_256_p3"] = (WorkloadParams(n=256, loss=0.03, ack=0), 0, True)                      # config 1
    s["c2_4096_p1_ack64"] = (WorkloadParams(n=4096, loss=0.01, ack=64), 0, True)             # config 2
    s["c2_4096_p1_noack"] = (WorkloadParams(n=4096, loss=0.01, ack=0), 0, True)              # config 2 stress
    for sid in (0, 1, 63):
        s[f"c3_4096_p2_ack64_s{sid}"] = (WorkloadParams(n=4096, loss=0.02, ack=64), sid, True)  # config 3
    s["c4_4096_p1_ack64_s511"] = (WorkloadParams(n=4096, loss=0.01, ack=64), 511, True)     # config 4
    s["c5_65536_ge5_b4"] = (WorkloadParams(n=65536, loss=0.05, burst=4, fec=0.10, ack=256, arq=2048), 0, True)
    s["var_1_1500_p2_ack32"] = (WorkloadParams(n=2000, payload=1, payload_max=1500, loss=0.02, ack=32), 0, True)
    s["tiny_1_20_p5_ack16"] = (WorkloadParams(n=3000, payload=1, payload_max=20, loss=0.05, ack=16), 0, True)
    s["big_9000_p3_ack64"] = (WorkloadParams(n=1500, payload=9000, loss=0.03, ack=64), 0, True)
    s["hiloss_p20_arq"] = (WorkloadParams(n=3000, loss=0.20, ack=64, arq=500), 0, True)
    s["norecloss_p5_arq"] = (WorkloadParams(n=3000, loss=0.05, ack=0, arq=300, loss_on_recovery=False), 0, True)
    s["single_p0"] = (WorkloadParams(n=200, loss=0.0, ack=1), 0, True)
    s["burst8_p5"] = (WorkloadParams(n=8192, loss=0.05, burst=8, fec=0.10, ack=128, arq=1024), 0, True)
    # siamese_encoder_retransmit under a virtual clock (RTO from acks / the initial RTO without)
    s["rtx_p2_ack64"] = (WorkloadParams(n=3000, loss=0.02, ack=64, rtx=16, rtx_msec=1), 0, True)
    s["rtx_p5_ack32"] = (WorkloadParams(n=3000, loss=0.05, ack=32, rtx=8, rtx_msec=3), 0, True)
    s["rtx_p3_noack"] = (WorkloadParams(n=2000, loss=0.03, ack=0, rtx=16, rtx_msec=2), 0, True)
    # frequent acks that acknowledge everything, so the encoder window restarts (StartNewWindow)
    # and the next RTT scan starts on placeholder elements (their send timestamps persist)
    s["rtx_restart_p1_ack4"] = (WorkloadParams(n=3000, loss=0.01, ack=4, rtx=2, rtx_msec=5), 0, True)
    s["rtx_restart_p2_ack2"] = (WorkloadParams(n=3000, loss=0.02, ack=2, rtx=1, rtx_msec=7), 0, True)
    # the 16,000-packet window (siamese.h:163): no acknowledgements, the sender asks
    # siamese_encoder_is_ready before every add and acks are forced by a refused add (workload.h
    # hold_full; SiameseEncoder.cpp:91-96, siamese.cpp:80-93)
    s["full_p1_noack"] = (WorkloadParams(n=50000, loss=0.01, ack=0, full=1), 0, True)
    s["full_p3_noack"] = (WorkloadParams(n=50000, loss=0.03, ack=0, full=1), 0, True)
    return s


def long_streams():
    """name -> (WorkloadParams, stream id): streams past the 22-bit packet-number period
    (SiameseCommon.h:102 kColumnPeriod = 0x400000): 4.3 M originals, so windows, Siamese sums,
    Cauchy rows and LDPC pairs straddle column 0x3FFFFF -> 0.  With acks every 256 at 1 % loss a
    window held open by an unrecovered loss straddles the wrap and the reference decoder disables
    itself (every later call returns Siamese_Disabled; the encoder's window then fills up): the
    engine must do exactly the same.  With no acks but the window-full behaviour (hold_full) the
    16,000-packet window fills ~360 times, windows straddle the wrap and the decoder recovers
    across it.  Digests only (the transcripts are 5-20 MB); 64-byte payloads for the CPU
    control-plane tests, 1300-byte ones (the bench's) for the GPU."""
    out = {}
    for size in (64, 1300):
        out[f"wrap_p1_ack256_{size}B"] = (WorkloadParams(n=4300000, payload=size, loss=0.01, ack=256), 0)
        out[f"wrap_p1_full_{size}B"] = (WorkloadParams(n=4300000, payload=size, loss=0.01, ack=0, full=1), 0)
    return out


def batches():
    """name -> (WorkloadParams, first stream id, stream count): many independent streams driven
    through ONE batched session on one GPU; the fixture holds each stream's transcript digest."""
    return {
        # BASELINE.json configs[2]: 64 independent streams x 4096 originals, 2% loss, batched on 1 GPU
        "cfg2_64x4096_p2_ack64": (WorkloadParams(n=4096, loss=0.02, ack=64), 0, 64),
        # BASELINE.json configs[3], the shard of rank 7 of 8 (streams 448..511), 3 bench steps
        "cfg3_rank7_64x12288_p1_ack64": (WorkloadParams(n=3 * 4096, loss=0.01, ack=64), 7 * 64, 64),
    }


def run(wp: WorkloadParams, sid: int) -> str:
    args = [GEN, "transcript", "/dev/stdout"] + wp.args() + [f"seed_data={1000 + sid}", f"seed_loss={2000 + sid}"]
    r = subprocess.run(args, capture_output=True, check=True)
    return r.stdout.decode()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench-streams", type=int, default=64)
    ap.add_argument("--bench-originals", type=int, default=12 * 4096)
    a = ap.parse_args()
    if not os.path.exists(GEN):
        print("build the reference first: make -C oracle", file=sys.stderr)
        return 2
    os.makedirs(OUT, exist_ok=True)
    index = {"generator": "oracle/_ref/golden_gen (reference codec from /root/reference)", "scenarios": {}}
    for name, (wp, sid, full) in scenarios().items():
        text = run(wp, sid)
        digest = hashlib.sha256(text.encode()).hexdigest()
        index["scenarios"][name] = {"args": wp.args(), "stream": sid, "sha256": digest,
                                    "lines": text.count("\n"), "summary": text.strip().splitlines()[-1],
                                    "file": f"{name}.txt.gz" if full else None}
        if full:
            # mtime 0: regenerating identical transcripts leaves the fixture files unchanged
            with open(os.path.join(OUT, f"{name}.txt.gz"), "wb") as raw, \
                    gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(text.encode())
        print(f"{name}: {index['scenarios'][name]['lines']} lines {digest[:16]}")

    # Bench configuration (bench.py default): per-stream transcript digests for streams 0..S-1.
    wp = WorkloadParams(n=a.bench_originals, loss=0.01, ack=64)
    bench = {"args": wp.args(), "streams": {}}
    for sid in range(a.bench_streams):
        text = run(wp, sid)
        bench["streams"][str(sid)] = {"sha256": hashlib.sha256(text.encode()).hexdigest(),
                                      "summary": text.strip().splitlines()[-1]}
    index["bench"] = bench
    index["batches"] = {}
    for name, (wp, base, count) in batches().items():
        entry = {"args": wp.args(), "stream_base": base, "streams": {}}
        for sid in range(base, base + count):
            text = run(wp, sid)
            entry["streams"][str(sid)] = {"sha256": hashlib.sha256(text.encode()).hexdigest(),
                                          "summary": text.strip().splitlines()[-1]}
        index["batches"][name] = entry
        print(f"{name}: {count} streams from {base}")
    index["long"] = {}
    for name, (wp, sid) in long_streams().items():
        text = run(wp, sid)
        index["long"][name] = {"args": wp.args(), "stream": sid, "sha256": hashlib.sha256(text.encode()).hexdigest(),
                               "lines": text.count("\n"), "summary": text.strip().splitlines()[-1]}
        print(f"{name}: {index['long'][name]['lines']} lines")
    with open(os.path.join(OUT, "scenarios.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
