"""raft_optical_flow_amd — MI355X-native (gfx950) RAFT inference path.

Drop-in for the reference's core/ API: RAFT, CorrBlock, AlternateCorrBlock,
BasicUpdateBlock / SmallUpdateBlock, BasicEncoder / SmallEncoder, InputPadder,
and the alt_cuda_corr plugin module; the compute runs in libraft_hip.so
(hand-written HIP kernels, C-ABI in include/raft_hip.h).
"""
from .corr import AlternateCorrBlock, CorrBlock  # noqa: F401
from .extractor import BasicEncoder, SmallEncoder  # noqa: F401
from .raft import RAFT  # noqa: F401
from .update import BasicUpdateBlock, SmallUpdateBlock  # noqa: F401
from .utils.utils import InputPadder, coords_grid, upflow8  # noqa: F401

__version__ = "0.1.0"
