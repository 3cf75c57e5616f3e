"""TEST/DIAGNOSIS ONLY: drive configs[2] streams through the C ABI driver (capi_gen, linked to
libtonk_amd.so) under a given environment and thread count, and print how many streams' transcripts
differ from the reference codec's digests (tests/golden/scenarios.json).

usage: python tools/capi_digest_check.py THREADS STREAMS [K=V ...]"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
threads, streams = int(sys.argv[1]), int(sys.argv[2])
env = dict(os.environ, **dict(a.split("=", 1) for a in sys.argv[3:]))
entry = json.load(open(os.path.join(ROOT, "tests", "golden", "scenarios.json")))["batches"]["cfg2_64x4096_p2_ack64"]
with tempfile.TemporaryDirectory() as d:
    prefix = os.path.join(d, "s")
    out = subprocess.run([os.path.join(ROOT, "tests", "native", "_build", "capi_gen"), "transcripts", prefix,
                          f"threads={threads}", f"streams={streams}", "stream=0"] + entry["args"],
                         capture_output=True, timeout=600, env=env)
    bad = [s for s in range(streams)
           if not os.path.exists(f"{prefix}{s}.txt") or
           hashlib.sha256(open(f"{prefix}{s}.txt", "rb").read()).hexdigest() != entry["streams"][str(s)]["sha256"]]
    print(f"threads={threads} streams={streams} env={sys.argv[3:]} rc={out.returncode} differing={len(bad)} {bad[:8]}")
    if out.returncode:
        print(out.stderr.decode()[-1500:])
