"""Top-level `alt_cuda_corr` module (the reference's plugin name, core/corr.py:5-9),
backed by libraft_hip.so.  Put this directory on sys.path."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from raft_optical_flow_amd.alt_cuda_corr import backward, forward  # noqa: E402,F401
