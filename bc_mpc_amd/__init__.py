"""bc_mpc_amd -- MI355X-native random-shooting MPC rollout engine.

Drop-in for Bonnieccc/bc-mpc's ``controllers.MPCcontroller.get_action`` hot
path (controllers.py:57-88 -> dynamics.py:106-119 -> cost_functions.py:9-63),
and its siblings MPCcontrollerPolicyNet / MPCcontrollerReward /
MPCcontrollerPolicyNetReward / MCTScontrollerPolicyNetReward (controllers.py:90-457).
The compute path is libbcmpc.so (HIP, gfx950); see DESIGN.md.
"""
from . import _lib
from .controllers import (Controller, MCTScontrollerPolicyNetReward, MPCcontroller, MPCcontrollerPolicyNet,
                          MPCcontrollerPolicyNetReward, MPCcontrollerReward, RandomController)
from .cem import CEMcontroller
from .cost_functions import cheetah_cost_fn, trajectory_cost_fn
from .engine import MLPSpec, PolicySpec, RolloutEngine, StepResult

__all__ = ["Controller", "MPCcontroller", "MPCcontrollerPolicyNet", "MPCcontrollerReward",
           "MPCcontrollerPolicyNetReward", "MCTScontrollerPolicyNetReward", "CEMcontroller", "RandomController", "PolicySpec", "cheetah_cost_fn",
           "trajectory_cost_fn", "MLPSpec", "RolloutEngine", "StepResult"]

_lib.load()   # fail loudly at import when the HIP library is missing
