"""get_action p50 through RolloutEngine.get_action (device actions) with and without the prepared-argument
fast path (BCMPC_PY_FASTPATH), small-K workloads, alternating processes."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, REPO)
    import time
    import numpy as np
    import bench
    out = {}
    for n in ("ppo_defaults", "ppo_mpc_default", "cfg1"):
        wl = bench.WORKLOADS[n]
        prob = bench.synthetic_problem(wl)
        eng = bench.make_engine(wl, prob, 0, "auto")
        ts = []
        for i in range(400):
            t0 = time.perf_counter()
            eng.get_action(prob["state"], None, seed=7 + i)
            if i >= 50:
                ts.append(time.perf_counter() - t0)
        eng.close()
        out[n] = round(float(np.percentile(ts, 50)) * 1e3, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        for r in range(2):
            for v in ("1", "0"):
                env = dict(os.environ, BCMPC_PY_FASTPATH=v)
                res = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True)
                print(json.dumps({"round": r, "fastpath": v, "p50_ms": res.stdout.strip().splitlines()[-1]}), flush=True)
