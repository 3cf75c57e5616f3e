import time, json, sys
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonk_amd
import bench
wp = tonk_amd.WorkloadParams(payload=1300, **bench.SINGLE_STREAM['cfg1'])
for rep in range(6):
    timing = rep % 2 == 0
    sess = tonk_amd.Session(wp, n_streams=1, device=0, threads=1, arena_bytes=(3 * wp.n * 1344) + (1 << 30))
    sess.generate(); sess.wait(); sess.set_timing(timing)
    t0 = time.perf_counter(); sess.step(4096); t1 = time.perf_counter(); sess.finish(); t2 = time.perf_counter()
    h = sess.host_ms(); s = sess.summary()
    print(json.dumps({"timing": timing, "step_us": round((t1-t0)*1e6,1), "finish_us": round((t2-t1)*1e6,1), "programs": s["programs"], "host": {k: round(v*1e3,1) for k,v in h.items()}}))
    sess.close()
