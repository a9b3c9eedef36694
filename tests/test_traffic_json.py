"""tools/traffic_json.py (the PMC traffic file bench.py quotes): per-dispatch means with the first dispatch
dropped, the gfx950 FETCH_SIZE x2 correction plus WRITE_SIZE, per (workload, precision) key, the cfg3
calibration note -- on synthetic rocprofv3 counter CSVs."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(path, kernel, values):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, v in enumerate(values):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": kernel, "Counter_Name": "X", "Counter_Value": v})
        w.writerow({"Dispatch_Id": 99, "Kernel_Name": "bcmpc::argmin_final", "Counter_Name": "X", "Counter_Value": 1e9})


def test_traffic_json_per_launch(tmp_path):
    src = tmp_path / "tag"
    k = "void bcmpc::rollout_x3<512, 4, 8, 0, false, 0, false>(bcmpc::RolloutArgs)"
    _csv(src / "traffic_cfg3_split_fetch", k, [999.0, 5000.0, 5200.0])     # KB; the first dispatch is warm-up
    _csv(src / "traffic_cfg3_split_write", k, [10.0, 500.0, 500.0])
    _csv(src / "traffic_cfg3_split_hbm_fetch", k, [0.0, 35000.0, 35000.0])
    out = tmp_path / "t.json"
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "traffic_json.py"), str(src), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    d = json.load(open(out))
    rec = d["cfg3:split:device"]
    assert rec["dispatches"] == 2 and rec["fetch_size_kb"] == 5100.0 and rec["write_size_kb"] == 500.0
    assert rec["hbm_bytes_per_launch"] == 5100.0 * 1024 * 2 + 500.0 * 1024      # FETCH x2 + WRITE
    assert rec["algorithmic_bytes_per_launch"] > 0 and "rollout_x3" in rec["kernel"]
    assert "calibration" in rec["correction"]
    assert list(d) == ["cfg3:split:device"]                                     # (the hbm pass is not a line)
