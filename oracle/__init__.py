"""CPU oracle package -- test infrastructure only (see mpc_oracle.py header)."""
from .mpc_oracle import *  # noqa: F401,F403
