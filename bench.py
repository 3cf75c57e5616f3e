#!/usr/bin/env python3
"""Siamese FEC encode+decode throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[3], per-GPU shard; weak scaling): every GPU runs 64
independent connection streams (encoder + decoder + lossy channel each, stream ids
rank*64 .. rank*64+63), 1300-byte payloads, 1% uniform loss on originals and recovery packets,
recovery rate f = max(2p, 1%) = 2%, acknowledgements every 64 originals.  Payloads are
synthetic (PCG, seed 1000 + stream id) and already resident in HBM when timing starts.

A step = 65536 originals per stream, in 16 device programs of 4096: the host control planes (16
worker threads per GPU) turn every add/encode/ack/decode into device ops and each program's byte
work runs as one merged launch sequence on the GPU, pipelined with the host building the next.  `value` is whole-job
payload GiB/s over all ranks; the timed region is bracketed by a barrier and a device sync.

roofline: algorithmic HBM bytes (SURVEY.md s8(d) B_alg, counted exactly per step) divided by
the summed duration of the executor (tamd_exec24; tamd_exec16 under TONK_AMD_SLICE=1024) launches of the timed steps (HIP events on the launch
stream), against the 8.0 TB/s HBM3E peak.  cpu_baseline: the reference codec (compiled from
/root/reference by oracle/Makefile, shipped prebuilt in oracle/_ref) on a sample of the same
workload, on rank 0 after the timed region, with the host cores the job owns (16 per GPU).

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg2|cfg1|cfg4]

--gpus N without torch.distributed.run starts N rank processes itself (one per GPU, gloo
rendezvous on 127.0.0.1); under torch.distributed.run the ranks come from the environment.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _hugepage_heap_relaunch() -> None:
    """Run the bench in a child process whose glibc heap uses transparent huge pages
    (GLIBC_TUNABLES=glibc.malloc.hugetlb=1: madvise(MADV_HUGEPAGE) on malloc's arenas; the
    GPU boxes run THP in "madvise" mode).  The host control plane walks per-stream windows,
    row tables and term lists spread over the heap; with 2 MB pages it costs 9 % less CPU per
    original on one core of the box (profiles/r03e_cp_hugetlb_ab.txt).  A tunable is read only
    at process start, hence the child; it dies with this process (PR_SET_PDEATHSIG), and this
    process touches no GPU and exits with the child's code.  TONK_AMD_HUGEPAGE_HEAP=0 runs
    in-process as before; a process under a profiler (rocprofv3's preload) is never relaunched."""
    if os.environ.get("TONK_AMD_HUGEPAGE_HEAP", "1") == "0" or not sys.platform.startswith("linux"):
        return
    tun = os.environ.get("GLIBC_TUNABLES", "")
    if "glibc.malloc.hugetlb" in tun or "rocprof" in os.environ.get("LD_PRELOAD", "") or \
            any(k.startswith("ROCPROF") for k in os.environ):
        return
    import ctypes
    import signal
    libc = ctypes.CDLL(None, use_errno=True)

    def die_with_parent() -> None:
        libc.prctl(1, int(signal.SIGKILL))  # PR_SET_PDEATHSIG

    env = dict(os.environ, GLIBC_TUNABLES=(tun + ":" if tun else "") + "glibc.malloc.hugetlb=1")
    child = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             preexec_fn=die_with_parent)
    while True:
        try:
            rc = child.wait()
            break
        except KeyboardInterrupt:
            child.send_signal(signal.SIGINT)
    sys.exit(rc if rc >= 0 else 128 - rc)


if __name__ == "__main__":
    _hugepage_heap_relaunch()

import tonk_amd  # noqa: E402

METRIC = "Siamese FEC encode+decode GiB/s (device-resident), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
STREAMS_PER_GPU = 64
ORIGINALS_PER_STEP = int(os.environ.get("TONK_AMD_BENCH_PROGRAM", 8192))  # per stream per device program
                                                                            # (tamd_session_step; env: A/B)
# (8192 since late round 6, 4096 before: the same host work per original, and launches twice as
# long drain relatively less -- frac 0.594 -> 0.635 at the same GiB/s, profiles/r06v_program_size.txt)
SINGLE_PROGRAM = 4096  # cfg1 / cfg4 (profiles/r06_single_step_sweep.txt)
# A bench step: 8 programs, 65536 originals per stream (round 5: 16 of 4096; 4 before): the driver's
# `--steps 20` then times ~110 ms instead of ~28 ms.  The inputs are a pool of INPUT_POOL rows per
# side per stream that original i reads as row i mod INPUT_POOL (tonk_amd.h input_pool).
PROGRAMS_PER_STEP = 65536 // ORIGINALS_PER_STEP
INPUT_POOL = 65536
LOSS = 0.01
ACK = 64
PAYLOAD = 1300


def host_threads(local_world: int) -> int:
    try:
        cpus = len(os.sched_getaffinity(0))
    except Exception:
        cpus = os.cpu_count() or 8
    per = max(1, cpus // max(1, local_world))
    env = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    if os.environ.get("TONK_AMD_HOST_THREADS"):  # A/B override (profiling)
        return max(1, int(os.environ["TONK_AMD_HOST_THREADS"]))
    return max(1, min(16, per, env))


def cpu_baseline(threads: int, n_orig: int, runs: int = 5, pool: int = 16384) -> dict | None:
    """The reference codec (oracle/_ref, compiled from /root/reference sources) on the bench's own
    workload: the same 64 streams, each over the bench's full stream length (`n_orig` originals,
    fresh codecs), on `threads` host threads; `runs` timed passes, median reported with the spread.
    Scenario generation -- payloads and loss draws -- happens before each pass's clock (SURVEY.md
    s8(d)); the payload bytes come from a pool of `pool` packets per stream, reused cyclically
    (the codec's work does not depend on the bytes; recovered packets are still checked)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "golden_gen")
    if not os.path.exists(exe):
        return None
    wp = tonk_amd.WorkloadParams(n=n_orig, payload=PAYLOAD, loss=LOSS, ack=ACK)
    args = [exe, "time", f"threads={threads}", f"streams={STREAMS_PER_GPU}", "reps=1", f"runs={runs}",
            f"pool={pool}"] + wp.args()
    r = subprocess.run(args, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        return None
    passes = [json.loads(l) for l in r.stdout.strip().splitlines() if l.startswith("{")]
    if len(passes) != runs:
        return None
    vals = sorted(j["gib_per_s"] for j in passes)
    secs = sum(j["seconds"] for j in passes)
    return {"value": round(vals[len(vals) // 2], 4), "unit": "GiB/s", "cores": threads, "kind": "reference",
            "spread": [round(vals[0], 4), round(vals[-1], 4)],
            "sample": f"the bench's workload: {STREAMS_PER_GPU} streams x {n_orig} originals (its full stream "
                      f"length) x {PAYLOAD} B, same loss/FEC/ack, steady state, fresh codecs per pass, loss draws "
                      f"and payloads generated before the clock (payload pool of {pool} packets per stream), "
                      f"{threads} host threads, median of {runs} passes, {secs:.2f} s timed in total"}


def host_cpus() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 8


# The executor kernel the library launches (engine.cpp slice_from_env: 1536-byte slices unless
# TONK_AMD_SLICE=1024).
EXEC_KERNEL = "tamd_exec16" if os.environ.get("TONK_AMD_SLICE", "").strip() == "1024" else "tamd_exec24"


def _timed_counter_values(csv_dir: str, counter: str, kernel: str = EXEC_KERNEL) -> list[float]:
    """Per-dispatch values of `counter` for `kernel`'s dispatches inside the timed region (between
    the two tamd_timed_region markers Device::set_timing launches), in dispatch order."""
    import csv
    import glob
    rows = []
    for f in glob.glob(os.path.join(csv_dir, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if r[1].startswith("tamd_timed_region")]
    if len(marks) < 2:
        return []
    return [v for _, k, v in rows[marks[0] + 1:marks[1]] if k.split("(")[0].strip() == kernel]


def pmc_traffic(workload: str, steps: int, warmup: int, timeout_s: int = 240) -> dict | None:
    """HBM traffic per timed executor launch of THIS workload, measured now: two rocprofv3 PMC
    passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass) over a rerun of the same
    workload with the same steps (child processes), restricted to the dispatches between the
    timed-region markers, so the launches counted are the ones the line's roofline averages.  gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half
    the bytes of 16-B-per-lane reads, so it is doubled; tools/pmc_calib.hip measures the same
    factor 2 for tamd_exec24's row pattern (16 B + 8 B per lane over 1344-byte rows:
    profiles/r03_pmc_calib.txt); WRITE_SIZE is exact for both store patterns.  Both counters are KiB and count L2 fabric requests (Infinity-Cache hits
    included).  Returns None when rocprofv3 is unavailable or a pass fails."""
    import shutil
    import signal
    import tempfile
    rp = shutil.which("rocprofv3")
    if not rp:
        return None
    vals, alg = {}, []
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"tamd_pmc_{counter.lower()}_", dir="/tmp")
        cmd = [rp, "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--workload", workload, "--steps", str(steps),
               "--warmup", str(warmup), "--no-cpu-baseline", "--no-end-to-end", "--no-verify", "--no-pmc"]
        env = dict(os.environ, TMPDIR="/tmp")
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, cwd="/tmp",
                             env=env, start_new_session=True)
        try:
            out, _ = p.communicate(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return {"error": f"{counter} pass timed out"}
        if p.returncode != 0:
            return {"error": f"{counter} pass exited {p.returncode}"}
        try:
            line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
            alg.append(float(line["roofline"]["alg_bytes_per_launch"]))
        except (IndexError, KeyError, TypeError, ValueError):
            return {"error": f"{counter} pass printed no bench line"}
        vals[counter] = _timed_counter_values(d, counter)
        shutil.rmtree(d, ignore_errors=True)
        if not vals[counter]:
            return {"error": f"{counter}: no timed {EXEC_KERNEL} dispatches in the counter csv"}
    f, w = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
    per = [(a * 2.0 + b) * 1024.0 for a, b in zip(f, w)]
    mean = sum(per) / len(per)
    alg_pl = sum(alg) / len(alg)
    return {"traffic_per_timed_launch": round(mean, 1), "traffic_over_alg": round(mean / alg_pl, 4),
            "alg_bytes_per_launch": round(alg_pl, 1), "timed_dispatches": len(per),
            "per_launch_mb": [round(x / 1e6, 1) for x in per],
            "read_bytes_per_launch": round(sum(f) / len(f) * 2048.0, 1),
            "write_bytes_per_launch": round(sum(w) / len(w) * 1024.0, 1),
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this workload (--steps {steps} "
                      f"--warmup {warmup}), timed-region dispatches; FETCH x2, WRITE x1 (gfx950)"}


def verify_schedule(threads: int, device: int) -> dict:
    """Byte-check of the timed schedule (untimed pass): the bench configuration's fixture
    (tests/golden/scenarios.json "bench": 64 streams x 49152 originals, 1% loss, ack 64, made by
    the reference codec) through one session with the bench's threads, deferred fill and early
    launch, rows released at their program's completion; every recovery packet and recovered
    original is digested on the launch stream right after the launch that completes its
    program (record mode), and each stream's transcript digest must equal the reference's."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", "scenarios.json")
    try:
        with open(path) as f:
            entry = json.load(f)["bench"]
    except (OSError, ValueError, KeyError):
        return {"digests_match": None, "note": "fixture missing"}
    wp = tonk_amd.WorkloadParams.from_args(entry["args"])
    n_streams = len(entry["streams"])
    t0 = time.perf_counter()
    sess = tonk_amd.Session(wp, n_streams=n_streams, device=device, threads=threads,
                            arena_bytes=2 * wp.n * n_streams * 1344 + (4 << 30), record=True)
    try:
        sess.generate()
        fr = sess.free_running()
        done = 0
        while done < wp.n:
            sess.step(min(ORIGINALS_PER_STEP, wp.n - done))
            done += ORIGINALS_PER_STEP
        sess.finish()
        bad = []
        for i in range(n_streams):
            want = entry["streams"][str(i)]
            got = hashlib.sha256((sess.transcript(i) + want["summary"] + "\n").encode()).hexdigest()
            if got != want["sha256"]:
                bad.append(i)
    finally:
        sess.close()
    return {"digests_match": not bad, "streams_differing": bad, "streams": n_streams, "originals_per_stream": wp.n,
            "seconds": round(time.perf_counter() - t0, 2),
            "schedule": (f"{threads} host threads, free-running streams, parallel program assembly, "
                         "pipelined levels, release at completion" if fr else
                         f"{threads} host threads, one pass per step")}


def end_to_end(threads: int, device: int, loss: float, steps: int = 3, warmup: int = 1) -> dict | None:
    """The PCIe-inclusive rate (north_star): the same workload with packets starting
    and ending in pinned host memory -- copies on their own streams, overlapped with the codec
    work.  Measured three ways: both ends of every connection on this GPU (each original crosses
    PCIe twice: into the encoder and into the decoder), the sender's end only (originals H2D,
    recovery packets D2H: what a sending host's GPU moves) and the receiver's end only (originals
    and received recovery packets H2D, recovered originals D2H).  D2H is timed on its own copies
    (HIP events): `d2h_copy_gb_per_s` is the rate while a copy runs, `d2h_gb_per_s` its bytes over
    the step time.  Reported beside `value`, never as it."""
    n_orig = (warmup + steps) * ORIGINALS_PER_STEP
    wp = tonk_amd.WorkloadParams(n=n_orig, payload=PAYLOAD, loss=loss, ack=ACK)

    def run(mask: int) -> dict:
        try:
            sess = tonk_amd.Session(wp, n_streams=STREAMS_PER_GPU, device=device, threads=threads,
                                    arena_bytes=(2 * n_orig * STREAMS_PER_GPU * 1344) + (4 << 30), stage_host=mask)
        except RuntimeError as e:
            return {"error": str(e)}
        try:
            sess.generate()
            for _ in range(warmup):
                sess.step(ORIGINALS_PER_STEP)
            sess.wait()
            s0 = sess.summary()
            t0 = time.perf_counter()
            for _ in range(steps):
                sess.step(ORIGINALS_PER_STEP)
            sess.wait()
            t1 = time.perf_counter()
            s1 = sess.summary()
        finally:
            sess.close()
        payload = s1["payload_bytes"] - s0["payload_bytes"]
        h2d = s1["h2d_bytes"] - s0["h2d_bytes"]
        d2h = s1["d2h_bytes"] - s0["d2h_bytes"]
        d2h_s = (s1["d2h_copy_us"] - s0["d2h_copy_us"]) / 1e6
        dt = t1 - t0
        return {"value": round(payload / dt / 2**30, 4), "unit": "GiB/s", "ms_per_step": round(dt * 1e3 / steps, 4),
                "h2d_gb_per_s": round(h2d / dt / 1e9, 2), "d2h_gb_per_s": round(d2h / dt / 1e9, 2),
                "d2h_copy_gb_per_s": round(d2h / d2h_s / 1e9, 2) if d2h_s > 0 else None,
                "d2h_copy_ms_per_step": round(d2h_s * 1e3 / steps, 4),
                "h2d_bytes_per_step": h2d // steps, "d2h_bytes_per_step": d2h // steps}

    both = run(3)
    out = dict(both)
    out.update({"steps": steps, "per_side": {"sender": run(1), "receiver": run(2)},
                "note": "pinned hipMemcpyAsync on copy streams: H2D of the originals into the encoder (sender) "
                        "and the decoder (receiver), D2H of recovery packets (sender) and recovered originals "
                        "(receiver, packed by a gather kernel), H2D of the received recovery packets (receiver); "
                        "`value` here has both ends on this GPU"})
    return out


# Workload names follow BASELINE.json's 0-based configs[] index.
SINGLE_STREAM = {
    # BASELINE.json configs[1]: one stream, 4096 originals, 1% loss, bit-exact vs CPU
    "cfg1": dict(n=4096, loss=0.01, ack=64),
    # BASELINE.json configs[4]: decoder stress, 65536 originals, 5% Gilbert-Elliott loss (mean
    # burst 4), f = 10%, acks every 256, ARQ after 2048
    "cfg4": dict(n=65536, loss=0.05, burst=4, fec=0.10, ack=256, arq=2048),
}
# Batched configurations: 64 streams per GPU, `loss` uniform, f = max(2p, 1%), ack every 64.
BATCHED = {
    # BASELINE.json configs[3] (the headline): 512 streams sharded 64/GPU, 1% loss
    "cfg3": dict(loss=0.01),
    # BASELINE.json configs[2]: 64 streams x 4096 originals, 2% loss, batched on one GPU
    # (the headline's schedule: programs of ORIGINALS_PER_STEP originals per stream)
    "cfg2": dict(loss=0.02),
}


def single_stream(name: str, device: int, step: int, reps: int = 3) -> dict:
    """One connection stream run start to finish (generate untimed; steps of 4096 originals,
    end-of-stream flush and device sync timed), the median of `reps` fresh sessions, next to the
    reference codec on one host thread over the same stream."""
    wp = tonk_amd.WorkloadParams(payload=PAYLOAD, **SINGLE_STREAM[name])
    times, payload, ok, runs = [], 0, True, []
    # The timed reps run without per-launch timing events (they add ~20 us of event work to a
    # single stream's few launches); one more rep with them gives the per-program breakdown.
    for rep in range(reps + 1):
        timed = rep < reps
        sess = tonk_amd.Session(wp, n_streams=1, device=device, threads=1, arena_bytes=(3 * wp.n * 1344) + (1 << 30))
        try:
            sess.generate()
            sess.wait()
            sess.set_timing(not timed)
            h0 = sess.host_ms()
            t0 = time.perf_counter()
            done = 0
            while done < wp.n:
                sess.step(min(step, wp.n - done))
                done += step
            sess.finish()
            t1 = time.perf_counter()
            sess.set_timing(False)
            h1 = sess.host_ms()
            fr = sess.free_running()
            kms, launches = sess.kernel_ms()
            summ = sess.summary()
        finally:
            sess.close()
        if timed:
            times.append(t1 - t0)
            payload = summ["payload_bytes"]
            ok = ok and summ["missing_at_end"] == 0 and summ["disabled_codecs"] == 0
            continue
        programs = summ["programs"]
        breakdown = {
            "programs": programs, "launches": launches,
            "wall_us_per_program": round((t1 - t0) * 1e6 / max(1, programs), 2),
            "kernel_us_per_launch": round(kms * 1e3 / max(1, launches), 2),
            "kernel_us_per_program": round(kms * 1e3 / max(1, programs), 2),
            # host phases per program (tamd_session_host_ms): control planes, layout, fill, launch
            "schedule": "free-running" if fr else "passes",
            "host_us_per_program": {k: round((h1[k] - h0[k]) * 1e3 / max(1, programs), 2)
                                    for k in h1 if k not in ("slot_reallocs", "upload_enqueue_max")},
            "note": "one extra run with per-launch timing events (not among the timed runs)"}
    times.sort()
    dt = times[len(times) // 2]
    out = {"metric": METRIC, "value": round(payload / dt / 2**30, 4), "unit": "GiB/s", "n_gpus": 1,
           "ms_per_stream": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u8", "data": "synthetic",
           "config": {"workload": f"BASELINE.json {name}: 1 stream", **SINGLE_STREAM[name], "payload_bytes": PAYLOAD,
                      "originals_per_step": step},
           "checks": {"all_recovered": ok}, "per_program": breakdown, "cpu_baseline": None}
    exe = os.path.join(ROOT, "oracle", "_ref", "golden_gen")
    if os.path.exists(exe):
        def run(r: int) -> dict | None:
            res = subprocess.run([exe, "time", "threads=1", "streams=1", f"reps={r}"] + wp.args(),
                                 capture_output=True, text=True, timeout=600)
            return json.loads(res.stdout.strip().splitlines()[-1]) if res.returncode == 0 else None
        probe = run(1)
        if probe:
            r = int(min(200, max(1, round(3.0 / max(probe["seconds"], 1e-3)))))
            j = run(r)
            if j:
                out["cpu_baseline"] = {"value": round(j["gib_per_s"], 4), "unit": "GiB/s", "cores": 1,
                                       "kind": "reference", "sample": f"the same stream x {r} repetitions, 1 host thread"}
    return out


def capi_bench(threads: int, runs: int = 3) -> dict:
    """`--workload capi`: the drop-in path Tonk actually links -- libtonk_amd.so through the
    siamese.h C ABI (every siamese_encode / siamese_decode is one synchronous program on the GPU
    and a readback; siamese.cpp:158-167 / TonkineseOutgoing.cpp:1284-1328 call it inline) -- on
    BASELINE.json configs[2] (64 streams x 4096 originals, 2% loss, f = 4%, ack every 64), each
    stream's codec pair driven by the same workload loop on `threads` host threads
    (tests/native/_build/capi_gen: oracle/golden_gen.cpp linked against our library), beside the
    reference codec with the same arguments (oracle/_ref/golden_gen).  Reports GiB/s and the per-call
    latency percentiles of siamese_encode and siamese_decode for both."""
    n, loss = 4096, 0.02
    wp = tonk_amd.WorkloadParams(n=n, payload=PAYLOAD, loss=loss, ack=ACK)
    common = ["time", f"threads={threads}", f"streams={STREAMS_PER_GPU}", "reps=1", f"runs={runs}", "lat=1"] + wp.args()

    def leg(exe: str) -> dict | None:
        if not os.path.exists(exe):
            return None
        r = subprocess.run([exe] + common, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            return {"error": f"exit {r.returncode}: {r.stderr[-300:]}"}
        passes = [json.loads(l) for l in r.stdout.strip().splitlines() if l.startswith("{")]
        passes.sort(key=lambda j: j["gib_per_s"])
        med = passes[len(passes) // 2]
        return {"value": round(med["gib_per_s"], 4), "unit": "GiB/s",
                "spread": [round(passes[0]["gib_per_s"], 4), round(passes[-1]["gib_per_s"], 4)],
                "encode_us": med.get("encode_us"), "decode_us": med.get("decode_us"), "bad": med["bad"]}

    ours = leg(os.path.join(ROOT, "tests", "native", "_build", "capi_gen"))
    ref = leg(os.path.join(ROOT, "oracle", "_ref", "golden_gen"))
    line = {"metric": "Siamese FEC encode+decode GiB/s through the siamese.h C ABI (host buffers, per-call programs)",
            "value": ours.get("value") if ours else None, "unit": "GiB/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": "BASELINE.json configs[2] through siamese.h: 64 streams x 4096 originals, 1300 B, "
                                   "2% loss, f=4%, ack every 64; one codec pair per stream, "
                                   f"{threads} host threads, median of {runs} passes",
                       "streams": STREAMS_PER_GPU, "originals_per_stream": n, "host_threads": threads},
            "capi": ours,
            "cpu_baseline": dict(ref, cores=threads, kind="reference",
                                 sample="the same streams through the reference codec's siamese.h, same threads")
            if ref else None}
    return line


def compress_messages(n_streams: int, n_msgs: int, seed: int = 7):
    """Synthetic reliable-message streams for the compression step: per stream, messages of
    64..1300 bytes mixing word runs (compressible), random bytes (not) and repeats of earlier
    stretches within the 24 KB history.  Returns (uint8 [streams, stride], lengths)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    words = [b"siamese ", b"tonk ", b"packet ", b"recovery ", b"window ", b"lane ", b"sum ", b"ack ",
             b"datagram ", b"stream ", b"0x1f ", b"42 "]
    text = np.frombuffer(b"".join(words[i] for i in rng.integers(0, len(words), 400000)), dtype=np.uint8)
    lens = rng.integers(64, 1301, size=(n_streams, n_msgs)).astype(np.uint32)
    kinds = rng.integers(0, 4, size=(n_streams, n_msgs))
    stride = int(lens.sum(axis=1).max()) + 64
    data = np.zeros((n_streams, stride), dtype=np.uint8)
    noise = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    for s in range(n_streams):
        pos = 0
        for k in range(n_msgs):
            n = int(lens[s, k])
            kind = int(kinds[s, k])
            if kind == 3 and pos > 4096:
                src = pos - int(rng.integers(n, min(pos, 20000) + 1))
                data[s, pos:pos + n] = data[s, src:src + n]
            elif kind == 0:
                o = int(rng.integers(0, len(noise) - n))
                data[s, pos:pos + n] = noise[o:o + n]
            else:
                o = int(rng.integers(0, len(text) - n))
                data[s, pos:pos + n] = text[o:o + n]
            pos += n
    return data, lens.reshape(-1).tolist(), stride


def compress_bench(device: int, steps: int, warmup: int, cpu: bool) -> dict:
    """`--workload compress`: SURVEY s8(f)4, Tonk's MessageCompressor (PacketCompression.h:92)
    on 64 streams x 1024 messages per step, device resident; the reference compressor (zstd level
    1 over the same ring, oracle/_ref/libmsgcodec_ref.so) on 16 host threads beside it."""
    import ctypes
    import torch
    from tonk_amd.compress import compress_batch
    n_streams, n_msgs, max_bytes = 64, 1024, 1300
    data, lens, stride = compress_messages(n_streams, n_msgs)
    import numpy as np
    lens_np = np.asarray(lens, dtype=np.uint32)
    torch.cuda.set_device(device)
    dev = torch.from_numpy(data).cuda()
    out = torch.zeros(n_streams * n_msgs * max_bytes, dtype=torch.uint8, device="cuda")
    in_bytes = float(sum(lens))
    per_job = int(os.environ.get("TONK_AMD_LZ_JOB", "0"))  # consecutive messages per wave (0: the library's auto, A/B knob)
    for _ in range(warmup):
        compress_batch(dev.data_ptr(), stride, n_streams, n_msgs, lens_np, max_bytes, out.data_ptr(), per_job)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = 0.0
    written = []
    for _ in range(steps):
        written, ms = compress_batch(dev.data_ptr(), stride, n_streams, n_msgs, lens_np, max_bytes, out.data_ptr(),
                                     per_job)
        kms += ms
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    out_bytes = float(np.where(written > 0, written, lens_np).sum())
    line = {
        "metric": "Tonk MessageCompressor input GiB/s (device-resident, zstd-block compatible)",
        "value": round(in_bytes * steps / (t1 - t0) / 2**30, 4), "unit": "GiB/s", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "ms_per_step": round((t1 - t0) * 1e3 / steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "64 streams x 1024 messages of 64-1300 B (word runs, random, repeats), max 1300",
                   "streams": n_streams, "messages_per_stream": n_msgs, "messages_per_wave": per_job or "auto (one job per wave slot: 32 on 256 CUs)"},
        "ratio": round(in_bytes / out_bytes, 4),
        "compressed_messages": int((written > 0).sum()),
        "kernel": {"name": "tamd_lz_compress", "ms_per_step": round(kms / steps, 4),
                   "input_gib_per_s": round(in_bytes * steps / (kms / 1e3) / 2**30, 4) if kms else None},
        "cpu_baseline": None,
    }
    ref = os.path.join(ROOT, "oracle", "_ref", "libmsgcodec_ref.so")
    if cpu and os.path.exists(ref):
        L = ctypes.CDLL(ref)
        L.ref_comp_bench.restype = ctypes.c_double
        L.ref_comp_bench.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_uint,
                                     ctypes.POINTER(ctypes.c_uint), ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        threads = min(16, host_cpus())
        arr = (ctypes.c_uint * len(lens))(*lens)
        bi, bo = ctypes.c_uint64(0), ctypes.c_uint64(0)
        runs = []
        for _ in range(3):
            sec = L.ref_comp_bench(data.ctypes.data, stride, n_streams, n_msgs, arr, max_bytes, threads, 2,
                                   ctypes.byref(bi), ctypes.byref(bo))
            runs.append(in_bytes * 2 / sec / 2**30)
        runs.sort()
        line["cpu_baseline"] = {"value": round(runs[1], 4), "unit": "GiB/s", "cores": threads, "kind": "reference",
                                "spread": [round(runs[0], 4), round(runs[-1], 4)],
                                "ratio": round(bi.value / bo.value, 4) if bo.value else None,
                                "sample": "the same 64 streams x 1024 messages, fresh compressors, 2 repetitions "
                                          "per run, median of 3 runs"}
    return line


def per_gpu_entries(rows: list[list[float]]) -> list[dict]:
    """The line's per_gpu list from every rank's gathered [rank, GiB/s, roofline frac, device busy
    frac, ms per step, executor us per launch] (None entries: a --dry-run, nothing measured)."""
    def r(x, nd):
        return None if x is None or x != x else round(x, nd)
    return [{"rank": int(v[0]), "stream_base": stream_base(int(v[0])), "value": r(v[1], 4), "unit": "GiB/s",
             "roofline_frac": r(v[2], 4), "device_busy_frac": r(v[3], 4), "ms_per_step": r(v[4], 4),
             "avg_launch_us": r(v[5], 3)} for v in rows]


def stream_base(rank: int) -> int:
    """Weak scaling: rank r owns streams [64 r, 64 r + 64) -- disjoint, no data-path exchange."""
    return rank * STREAMS_PER_GPU


class Dist:
    """Control-plane synchronisation between ranks (gloo; the data path has no collective)."""

    def __init__(self, world: int):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op_name: str) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op_name))
        return float(t.item())

    def allmax(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def allsum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def gather(self, xs: list[float]) -> list[list[float]]:
        """Every rank's `xs`, in rank order (all_gather)."""
        if self.dist is None:
            return [list(xs)]
        import torch
        t = torch.tensor(xs, dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [p.tolist() for p in parts]

    def close(self) -> None:
        if self.dist is not None:
            self.dist.destroy_process_group()


MAX_CORES = 128


class HostEnv:
    """Host-side conditions of the timed region (the headline is host-bound): the
    cgroup CPU-quota throttling of this job (cpu.stat), this process's CPU time, and how busy the
    worker cores were in total (/proc/stat, every process) -- busy well above our own CPU time
    on those cores means another job's threads shared them."""

    def __init__(self, cores: list[int]):
        self.cores = list(cores)
        self.a = self._sample()

    @staticmethod
    def _cpu_stat() -> dict:
        out = {}
        try:
            with open("/sys/fs/cgroup/cpu.stat") as f:
                for line in f:
                    k, v = line.split()
                    out[k] = int(v)
        except (OSError, ValueError):
            pass
        return out

    def _proc_stat(self) -> dict:
        busy = {}
        try:
            with open("/proc/stat") as f:
                for line in f:
                    if line.startswith("cpu") and line[3].isdigit():
                        v = line.split()
                        c = int(v[0][3:])
                        if c in self.cores:
                            t = [int(x) for x in v[1:]]
                            busy[c] = (sum(t) - t[3] - t[4], sum(t))  # (busy, total) jiffies
        except (OSError, ValueError):
            pass
        return busy

    def _sample(self):
        return (time.perf_counter(), os.times(), self._cpu_stat(), self._proc_stat())

    def report(self) -> dict:
        t1, o1, c1, p1 = self._sample()
        t0, o0, c0, p0 = self.a
        wall = t1 - t0
        own = (o1.user + o1.system) - (o0.user + o0.system)
        out = {"wall_s": round(wall, 4), "process_cpu_s": round(own, 4)}
        if c0 and c1:
            out["throttled_ms"] = round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 3)
            out["nr_throttled"] = c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0)
        if p0 and p1:
            b = sum(p1[c][0] - p0[c][0] for c in p1 if c in p0)
            tot = sum(p1[c][1] - p0[c][1] for c in p1 if c in p0)
            out["worker_cores_busy_frac"] = round(b / tot, 4) if tot else None
            hz = os.sysconf("SC_CLK_TCK")
            out["worker_cores_busy_s"] = round(b / hz, 3)
        return out


def pad_cores(cores: list[int]) -> list[float]:
    """A rank's core list as a fixed-size vector for all_gather (-1 = none)."""
    c = list(cores)[:MAX_CORES]
    return [float(x) for x in c] + [-1.0] * (MAX_CORES - len(c))


def unpad_cores(v: list[float]) -> list[int]:
    return [int(x) for x in v if x >= 0]


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script (rank i on GPU i,
    gloo rendezvous on 127.0.0.1) before anything here touches a GPU; rank 0 prints the line.
    Returns the worst exit code."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true", help="skip the PCIe-inclusive side measurement")
    ap.add_argument("--no-verify", action="store_true", help="skip the untimed byte check of the timed schedule")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 HBM-traffic passes (roofline.traffic)")
    ap.add_argument("--workload", choices=sorted(BATCHED) + sorted(SINGLE_STREAM) + ["compress", "capi"], default="cfg3",
                    help="BASELINE.json configs[] index: cfg3 (the headline, 64 streams per GPU), cfg2 (64 "
                         "streams, 2%% loss), cfg1 / cfg4 (one stream, start to finish)")
    ap.add_argument("--step", type=int, default=0,
                    help="cfg1 / cfg4: originals per device program (default SINGLE_PROGRAM, 4096: the best of the 256..4096 sweep in profiles/r06_single_step_sweep.txt for both)")
    ap.add_argument("--dry-run", action="store_true",
                    help="form the ranks and print the shard plan without touching a GPU (tests)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0:
        if a.gpus > 1:
            return spawn_ranks(a.gpus, sys.argv[1:])
        world = 1
    elif a.gpus != world and a.gpus != 1:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # With several ranks, gloo's connection messages go to stdout from C++ (fd 1); the bench line
    # keeps the real stdout to itself and everything else that writes to fd 1 goes to stderr.
    line_out = sys.stdout
    if world > 1:
        sys.stdout.flush()
        line_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)

    if a.workload == "compress":  # SURVEY s8(f)4 side line (not the headline)
        if world > 1:
            print("bench.py: the compress workload runs on one GPU", file=sys.stderr)
            return 2
        print(json.dumps(compress_bench(local_rank, min(a.steps, 10), min(a.warmup, 2), not a.no_cpu_baseline)),
              flush=True)
        return 0

    if a.workload == "capi":  # the siamese.h drop-in path (side line, not the headline)
        if world > 1:
            print("bench.py: the capi workload runs on one GPU", file=sys.stderr)
            return 2
        print(json.dumps(capi_bench(host_threads(1))), flush=True)
        return 0

    if a.workload in SINGLE_STREAM:
        if world > 1:
            print("bench.py: single-stream workloads run on one GPU (replicas only)", file=sys.stderr)
            return 2
        step = a.step or SINGLE_PROGRAM
        print(json.dumps(single_stream(a.workload, local_rank, step)), flush=True)
        return 0

    loss = BATCHED[a.workload]["loss"]
    d = Dist(world)
    if a.dry_run:
        # Host-core plan without a GPU: TONK_AMD_TOPOLOGY lists every device's NUMA local_cpulist
        # (';'-separated, one CPU per core), as /sys/bus/pci/devices/<gpu>/local_cpulist gives
        # them on a GPU node; the session computes the same plan there (tamd_cpu_share).
        topo = os.environ.get("TONK_AMD_TOPOLOGY")
        cores = []
        if topo:
            lists = topo.split(";")
            cores = tonk_amd.cpu_share(lists, local_rank, lists[local_rank], os.environ.get("TONK_AMD_CPU_SLOT"))
        # a share smaller than the pool shrinks the pool to one worker per core (the session does
        # the same, tamd_session_create): fewer workers, never two on one core
        workers = min(host_threads(local_world), len(cores)) if cores else host_threads(local_world)
        bases = d.gather([float(stream_base(rank)), float(rank), float(local_rank), float(workers)] + pad_cores(cores))
        nan = float("nan")
        per_rank = d.gather([float(rank), nan, nan, nan, nan, nan])  # (the same gather as a measured run)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "streams_per_gpu": STREAMS_PER_GPU,
                              "ranks": [{"rank": int(v[1]), "local_rank": int(v[2]), "stream_base": int(v[0]),
                                         "host_threads": int(v[3]), "host_cores": unpad_cores(v[4:])} for v in bases],
                              "per_gpu": per_gpu_entries(per_rank)}), file=line_out, flush=True)
        d.close()
        return 0

    threads = host_threads(local_world)
    total_steps = a.warmup + a.steps
    n_orig = total_steps * ORIGINALS_PER_STEP * PROGRAMS_PER_STEP
    wp = tonk_amd.WorkloadParams(n=n_orig, payload=PAYLOAD, loss=loss, ack=ACK)
    # TONK_AMD_BENCH_DEVICE: every rank on this device -- a rehearsal of the N-rank path on a
    # one-GPU box (the ranks then share one GPU and its host cores: not a scaling measurement)
    device = int(os.environ.get("TONK_AMD_BENCH_DEVICE", local_rank))
    if "TONK_AMD_BENCH_DEVICE" in os.environ and local_world > 1 and "TONK_AMD_CPU_SLOT" not in os.environ:
        os.environ["TONK_AMD_CPU_SLOT"] = f"{local_rank}/{local_world}"  # (disjoint cores all the same)
    pool = min(INPUT_POOL, n_orig)
    sess = tonk_amd.Session(wp, n_streams=STREAMS_PER_GPU, device=device,
                            stream_base=stream_base(rank), threads=threads,
                            arena_bytes=(2 * pool * STREAMS_PER_GPU * 1344) + (4 << 30), input_pool=pool)
    sess.generate()
    sess_cpus = sess.cpus()
    rank_cores = d.gather(pad_cores(sess_cpus))

    for _ in range(a.warmup * PROGRAMS_PER_STEP):
        sess.step(ORIGINALS_PER_STEP)
    sess.wait()
    s0 = sess.summary()
    h0 = sess.host_ms()
    sess.set_timing(True)
    d.barrier()
    env = HostEnv(sess.cpus())
    t0 = time.perf_counter()
    for _ in range(a.steps * PROGRAMS_PER_STEP):
        sess.step(ORIGINALS_PER_STEP)
    sess.wait()
    t1 = time.perf_counter()
    host_env = env.report()
    host_env["heap"] = "glibc hugetlb (THP)" if "glibc.malloc.hugetlb=1" in os.environ.get("GLIBC_TUNABLES", "") \
        else "glibc default"
    d.barrier()
    sess.set_timing(False)
    kernel_ms, launches = sess.kernel_ms()
    arena_base, arena_bytes = sess.arena()
    s1 = sess.summary()
    h1 = sess.host_ms()
    # per device program (a quarter of a bench step)
    host = {k: round((h1[k] - h0[k]) / (a.steps * PROGRAMS_PER_STEP), 4) for k in h1}
    elapsed = d.allmax(t1 - t0)

    payload = s1["payload_bytes"] - s0["payload_bytes"]
    alg = s1["alg_bytes"] - s0["alg_bytes"]
    op_trace = (s1["acc_bytes"] - s0["acc_bytes"]) + (s1["store_bytes"] - s0["store_bytes"])
    total_payload = d.allsum(payload)
    value = total_payload / elapsed / 2**30

    # Correctness of the run itself: finish the streams (lossless flush) and require that every
    # original was received or recovered and no codec was disabled.
    sess.finish()
    fin = sess.summary()
    ok = fin["missing_at_end"] == 0 and fin["disabled_codecs"] == 0
    sess.close()
    all_ok = d.allsum(0.0 if ok else 1.0) == 0.0

    achieved = alg / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else 0.0
    # Every rank's own figures (BASELINE.json configs[3]: per-GPU GiB/s beside the aggregate): its
    # payload over its own timed region, its executor's roofline fraction and busy share.
    own_ms = (t1 - t0) * 1e3 / a.steps
    per_rank = d.gather([float(rank), payload / (t1 - t0) / 2**30, achieved / HBM_PEAK_GBS,
                         (kernel_ms / 1e3) / (t1 - t0), own_ms,
                         kernel_ms * 1e3 / launches if launches else 0.0])
    pmc = pmc_traffic(a.workload, a.steps, a.warmup) if (rank == 0 and world == 1 and not a.no_pmc) else None
    traffic = pmc.get("traffic_per_timed_launch") if pmc else None
    workload = {
        "cfg3": "configs[3] per-GPU shard: 64 independent streams/GPU, 65536 originals per stream per step " f"({PROGRAMS_PER_STEP} programs), "
                "1300 B payloads, 1% uniform loss, f=2%, ack every 64",
        "cfg2": "configs[2]: 64 independent streams/GPU, 65536 originals per stream per step " f"({PROGRAMS_PER_STEP} programs), 1300 B payloads, "
                "2% uniform loss, f=4%, ack every 64",
    }[a.workload]
    out = {
        "metric": METRIC,
        "value": round(value, 4),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": workload,
            "streams_per_gpu": STREAMS_PER_GPU, "originals_per_step": ORIGINALS_PER_STEP * PROGRAMS_PER_STEP,
            "originals_per_program": ORIGINALS_PER_STEP, "payload_bytes": PAYLOAD, "input_pool_per_stream": pool,
            "loss": loss, "ack_every": ACK, "host_threads_per_gpu": len(sess_cpus) or threads,
            "parallelism": f"streams sharded {STREAMS_PER_GPU}/GPU x {world} GPU, no collective",
            # each rank's pinned worker cores (its share of its GPU's NUMA node, tamd_cpu_share)
            "host_cores": [unpad_cores(v) for v in rank_cores],
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": round(traffic, 1) if traffic else None,
            "traffic_over_alg": pmc.get("traffic_over_alg") if pmc else None,
            # the same fraction on the bytes the counters saw move (traffic per timed launch of the
            # PMC passes over this run's average launch): B_alg charges every received original
            # to the decoder, which the executor partly reads from L2 / Infinity Cache instead
            "frac_counters": (round(traffic / (kernel_ms * 1e-3 / launches) / 1e9 / HBM_PEAK_GBS, 4)
                              if traffic and launches and kernel_ms else None),
            "pmc": pmc,
            "kernel": EXEC_KERNEL,
            "launches": launches,
            "avg_launch_us": round(kernel_ms * 1e3 / launches, 3) if launches else None,
            "alg_bytes_per_launch": round(alg / launches, 1) if launches else None,
            # op-trace bytes (every row an instruction reads or writes): the
            # gap to alg_bytes is what L2 / Infinity Cache serve
            "op_trace_bytes_per_launch": round(op_trace / launches, 1) if launches else None,
            "device_busy_frac": round((kernel_ms / 1e3) / (t1 - t0), 4),
            # (placement diagnostics: the executor's launch time differs between processes)
            "arena": {"base": hex(arena_base), "bytes": arena_bytes, "base_mod_1g": arena_base % (1 << 30)},
            # (with several ranks this object is rank 0's executor; per_gpu holds every rank's)
            "scope": "rank 0" if world > 1 else "the one GPU",
        },
        "per_gpu": per_gpu_entries(per_rank),
        "cpu_baseline": None,
        "host_ms_per_program": host,  # (rank 0's, as host_env)
        "host_env": host_env,
        "checks": {"all_recovered": all_ok, "recovered": fin["recovered"], "lost_originals": fin["lost_originals"],
                   "lost_recoveries": fin["lost_recoveries"]},
    }
    # The CPU leg runs after every rank's timed region: the reference codec on the host cores the
    # job owns (16 per GPU, so N x 16 at N GPUs, capped by this process's CPU set).
    if rank == 0 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(min(host_cpus(), threads * local_world), n_orig)
    if rank == 0 and world == 1 and not a.no_end_to_end:
        out["end_to_end"] = end_to_end(threads, device, loss)
    if rank == 0 and a.workload == "cfg3" and not a.no_verify:
        v = verify_schedule(threads, device)
        out["checks"]["digests_match"] = v["digests_match"]
        out["checks"]["verify"] = v
    d.barrier()
    if rank == 0:
        print(json.dumps(out), file=line_out, flush=True)
    d.close()
    return 0 if all_ok and out["checks"].get("digests_match") is not False else 1


if __name__ == "__main__":
    sys.exit(main())
