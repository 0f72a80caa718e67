"""Shim: `sys.path.append('core'); from raft import RAFT` (reference demo.py:1-12) -> raft_optical_flow_amd."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))
from raft_optical_flow_amd.raft import RAFT  # noqa: E402,F401
from raft_optical_flow_amd.raft import autocast  # noqa: E402,F401
