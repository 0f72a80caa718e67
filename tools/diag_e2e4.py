"""Dev diagnostic: determinism of raft_corr_lookup_conv (repeated launches on fixed inputs) and of
RAFT forwards (fused / unfused plans, repeated graph replays)."""
import argparse
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raft_optical_flow_amd import RAFT, _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict, smooth_images  # noqa: E402

spec = importlib.util.spec_from_file_location("tlc", os.path.join(ROOT, "tests", "test_gpu_lookup_conv.py"))
tlc = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tlc)
_lib.load()
# 1. the kernel alone: _case builds inputs and runs it once; re-run its launch by re-calling _case with the
#    same seed (fresh buffers) and compare
for (B, h, w) in [(1, 16, 24), (1, 55, 128)]:
    ref = tlc._case(B, h, w, "f16x3", seed=5)
    worst = [0.0, 0.0, 0.0]
    for rep in range(10):
        d = tlc._case(B, h, w, "f16x3", seed=5)
        worst[0] = max(worst[0], float((d["c1"] - ref["c1"]).abs().max()))
        worst[1] = max(worst[1], float((d["f1"] - ref["f1"]).abs().max()))
        worst[2] = max(worst[2], float((d["flow_b"] - ref["flow_b"]).abs().max()))
    print(f"kernel {B}x{h}x{w}: max diff over 10 re-runs c1 {worst[0]:.3e} f1 {worst[1]:.3e} flow {worst[2]:.3e}",
          flush=True)
# 2. RAFT replays
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to("cuda").eval()
i1, i2 = smooth_images(1, 128, 192, seed=3)
i1, i2 = i1.cuda(), i2.cuda()
for fuse in ("1", "0"):
    os.environ["RAFT_FUSE_CONVC1"] = fuse
    outs = []
    with torch.no_grad():
        for rep in range(6):
            outs.append(m(i1, i2, iters=12, test_mode=True)[1])
    torch.cuda.synchronize()
    diffs = [float((o - outs[0]).abs().max()) for o in outs[1:]]
    print(f"RAFT fuse={fuse}: replay diffs vs first {['%.2e' % x for x in diffs]}", flush=True)
os.environ["RAFT_FUSE_CONVC1"] = "1"
os.environ["RAFT_HIP_GRAPH"] = "0"
m.hip_graph = False
with torch.no_grad():
    outs = [m(i1, i2, iters=12, test_mode=True)[1] for _ in range(5)]
print(f"RAFT fuse=1 eager: diffs vs first {['%.2e' % float((o - outs[0]).abs().max()) for o in outs[1:]]}")
