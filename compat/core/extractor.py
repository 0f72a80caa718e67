"""Shim for core/extractor.py -> raft_optical_flow_amd.extractor."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))
from raft_optical_flow_amd.extractor import (  # noqa: E402,F401
    BasicEncoder, BottleneckBlock, ResidualBlock, SmallEncoder)
