"""Shim for core/utils/utils.py -> raft_optical_flow_amd.utils.utils."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))))
from raft_optical_flow_amd.utils.utils import (  # noqa: E402,F401
    InputPadder, bilinear_sampler, coords_grid, forward_interpolate, upflow8)
