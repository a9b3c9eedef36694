"""Team-kernel A/B on the small-K workloads: get_action p50 and HIP-event kernel time per library.
usage: python tools/ab_smallk.py lib1.so[,lib2.so...] [workloads] -- each library in its own process"""
import json, os, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ["REPO"])
import bench
out = {}
for name in os.environ["WLS"].split():
    wl = bench.WORKLOADS[name]
    p = bench.synthetic_problem(wl)
    eng = bench.make_engine(wl, p, 0, "auto")
    ts, ks = [], []
    for i in range(220):
        t0 = time.perf_counter()
        eng.get_action(p["state"], None, seed=0x5EED + i)
        if i >= 20:
            ts.append(time.perf_counter() - t0)
    eng.set_timing(True)
    for i in range(60):
        eng.get_action(p["state"], None, seed=0x5EED + i)
        ks.append(eng.last_kernel_ms()[0])
    out[name] = dict(kernel=eng.info()["kernel"], p50_ms=float(np.median(ts) * 1e3), kernel_ms=float(np.mean(ks)))
    eng.close()
print(json.dumps(out))
'''


def main():
    libs = sys.argv[1].split(",")
    wls = sys.argv[2] if len(sys.argv) > 2 else "ppo_defaults ppo_mpc_default runsh_recipe runsh_noln cfg1"
    for rnd in range(2):
        for lib in libs:
            env = dict(os.environ, REPO=REPO, WLS=wls)
            if lib != "default":
                env["BCMPC_LIB"] = os.path.join(REPO, lib)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
            print(f"round {rnd} {lib}: {line}", flush=True)


if __name__ == "__main__":
    main()
