"""Shim for core/corr.py -> raft_optical_flow_amd.corr (CorrBlock, AlternateCorrBlock on HIP)."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))))
from raft_optical_flow_amd.corr import AlternateCorrBlock, CorrBlock  # noqa: E402,F401
