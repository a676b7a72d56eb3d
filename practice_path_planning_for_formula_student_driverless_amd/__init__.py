"""MI355X-native batched raceline optimizer (steps 7-8 of the reference FS-driverless pipeline).

The compute path is ``_lib/librl.so`` (hand-written HIP for gfx950, C-ABI in
``include/rl_abi.h``).  ``raceline`` mirrors the reference's functions over it.
"""
from .abi import RL_MODE_MINCURV, RL_MODE_MINTIME, Problem, RlCfg, default_cfg, set_mu  # noqa: F401

__version__ = "0.1.0"
