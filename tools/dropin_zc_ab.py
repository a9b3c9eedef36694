"""Drop-in controller p50 (bench.dropin_small_k: back to back and with 50 us of host work between calls) for the
small-K workloads, alternating library variants given as BCMPC_* environment settings per run.
usage: python tools/dropin_zc_ab.py [--rounds 2] "label:ENV=V,ENV2=V2" ...   (one process per variant and round)"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(names):
    sys.path.insert(0, REPO)
    import bench
    out = {}
    for n in names:
        wl = bench.WORKLOADS[n]
        d = bench.dropin_small_k(n, wl, bench.synthetic_problem(wl), 0, calls=300)
        out[n] = {"b2b": d["p50_ms"], "gap50": d["p50_gap50us_ms"], "kernel": d["kernel"]}
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--names", default="ppo_defaults,ppo_mpc_default,cfg1")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.names.split(","))
    for r in range(a.rounds):
        for v in a.variants:
            label, _, envs = v.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val
            res = subprocess.run([sys.executable, __file__, "--child", "--names", a.names], env=env,
                                 capture_output=True, text=True, timeout=300)
            line = res.stdout.strip().splitlines()[-1] if res.stdout.strip() else res.stderr[-300:]
            print(json.dumps({"round": r, "variant": label, "result": line}), flush=True)


if __name__ == "__main__":
    main()
