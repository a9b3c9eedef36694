import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


def golden_names(kind: str = "mpc"):
    """Fixture names; kind "mpc" = MPCcontroller cases, "policy" = MPCcontrollerPolicyNet cases."""
    names = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))
    return [n for n in names if n.startswith("policy_") == (kind == "policy")]


class Golden:
    """One committed fixture + everything needed to rebuild its inputs."""

    def __init__(self, name):
        from oracle import mpc_oracle as orc
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = z
        self.meta = json.loads(str(z["meta"]))
        m = self.meta
        self.K, self.H, self.S, self.A = m["K"], m["H"], m["S"], m["A"]
        self.weights = orc.synthetic_weights(self.S, self.A, m["hidden"], m["L"], m["act"], m["ln"],
                                             seed_base=m["weight_seed_base"])
        assert self.weights.digest() == m["weight_digest"], "synthetic weight generator drifted"
        if "W0" in z.files:   # stored weights must equal the regenerated ones
            for i, k in enumerate(self.weights.kernels):
                assert np.array_equal(z[f"W{i}"], k)
        self.norm = orc.synthetic_normalization(self.S, self.A, seed=m["norm_seed"])
        assert np.array_equal(self.norm[0], z["mean_obs"]) and np.array_equal(self.norm[9], z["std_deltas"])
        self.state = z["state"]
        self.costs = z["costs"]
        self.argmin = int(z["argmin"])
        self.opt_action = z["opt_action"]
        self.near = z["near_threshold"]
        self.top2_gap = float(z["top2_gap"])
        self.low = -np.ones(self.A, dtype=np.float32)
        self.high = np.ones(self.A, dtype=np.float32)
        self.policy = None
        if m.get("policy"):
            L = m["pl"]
            self.policy = orc.PolicyWeights([z[f"PW{i}"] for i in range(L + 1)], [z[f"PB{i}"] for i in range(L + 1)],
                                            z["P_ob_mean"], z["P_ob_std"], z["P_logstd"])
            ref = orc.synthetic_policy(self.S, self.A, m["ph"], L, seed=m["policy_seed"])
            assert all(np.array_equal(a, b) for a, b in zip(ref.kernels, self.policy.kernels))

    def actions(self):
        """The [H, K, A] action tensor the reference consumed (regenerated, then re-injected)."""
        from oracle import mpc_oracle as orc
        m = self.meta
        inject = m.get("inject")
        if inject == "philox":
            return orc.device_rng_actions(m["rng_seed"], m["cand_offset"], self.K, self.H, self.low, self.high)
        rs = np.random.RandomState(m["seed"])
        ap = rs.uniform(low=self.low, high=self.high, size=[self.H, self.K, self.A])
        if inject == "tie":
            lo, best = (int(x) for x in self.z["tie_pair"])
            ap[:, lo, :] = ap[:, best, :]
            ap[:, min(self.K - 1, best + 7), :] = ap[:, best, :]
        elif inject == "nan":
            ap[2, 37, 0] = np.nan
            ap[1, 90, 3] = np.nan
        return ap

    def dyn(self):
        from oracle import mpc_oracle as orc
        return orc.NumpyDynamics(self.weights, self.norm)


@pytest.fixture(params=golden_names("mpc"))
def golden(request):
    return Golden(request.param)


@pytest.fixture(params=golden_names("policy"))
def golden_policy(request):
    return Golden(request.param)
