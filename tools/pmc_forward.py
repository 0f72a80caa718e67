"""Workload for the in-forward PMC passes (tools/pmc_forward.sh): bench.py's config-2 forward
(B=1, 436x1024 padded to 440x1024, iters=32, f16x3, the bench's first frame pair), run
eagerly twice after a calibration copy of known byte count.  The summary
(tools/pmc_forward_summary.py) reads the counters of the LAST forward only.

    python tools/pmc_forward.py [batch] [precision]
"""
import argparse
import os
import sys

import torch

# the lookup counters are for the lookup-only kernel that bench.py's roofline times (the forward
# otherwise runs convf1 inside the lookup launch, raft_corr_lookup_convf1)
os.environ.setdefault("RAFT_FUSE_CONVF1", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raft_optical_flow_amd import RAFT, InputPadder, _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402
from raft_optical_flow_amd.init import seeded_images, seeded_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
prec = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(dev).eval()
m.conv_precision = prec
i1, i2 = seeded_images(B, 436, 1024, seed=1)
i1, i2 = InputPadder(i1.shape).pad(i1.to(dev), i2.to(dev))
# calibration: a 64 MiB contiguous copy through raft_nhwc_to_nchw (C = 1: 4-B accesses)
n = 16 * 1024 * 1024
src = torch.randn(n, device=dev)
dst = torch.empty(n, device=dev)
_lib.call("raft_nhwc_to_nchw", src.data_ptr(), 1, dst.data_ptr(), 1, 1, 1, n, K.stream_handle())
torch.cuda.synchronize()
pl = m.plan(B, 440, 1024, 32, True, device=dev)
pl.set_inputs(i1, i2)
with torch.no_grad():
    for _ in range(2):
        pl.run()
torch.cuda.synchronize()
print("pmc forward done", B, m.resolved_precision())
