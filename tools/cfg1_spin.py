"""configs[1] single-stream runs (as bench.py single_stream times them) with and without a short
host busy-spin right before the timed region: is the cold control plane the core's clock?"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonk_amd
import bench
wp = tonk_amd.WorkloadParams(payload=1300, **bench.SINGLE_STREAM['cfg1'])
for rep in range(8):
    spin = rep % 2 == 1
    sess = tonk_amd.Session(wp, n_streams=1, device=0, threads=1, arena_bytes=(3 * wp.n * 1344) + (1 << 30))
    sess.generate(); sess.wait(); sess.set_timing(False)
    if spin:
        t = time.perf_counter()
        x = 0
        while time.perf_counter() - t < 0.005:
            x += 1
    h0 = sess.host_ms()
    t0 = time.perf_counter(); sess.step(4096); sess.finish(); t1 = time.perf_counter()
    h1 = sess.host_ms()
    print(json.dumps({"spin": spin, "wall_us": round((t1 - t0) * 1e6, 1),
                      "control_us": round((h1["control_sum"] - h0["control_sum"]) * 1e3, 1)}))
    sess.close()
