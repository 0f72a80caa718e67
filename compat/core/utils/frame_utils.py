"""Shim for core/utils/frame_utils.py (the .flo / .pfm functions evaluate.py's Sintel
submission uses) -> raft_optical_flow_amd.io.  The image readers (read_gen) and the KITTI
16-bit PNG flow IO need cv2, which is not part of this build."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))))
from raft_optical_flow_amd.io import readFlow, readPFM, writeFlow, write_flo_batch  # noqa: E402,F401
