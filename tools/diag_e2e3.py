"""Dev diagnostic: the fused-vs-unfused RAFT sequence after the lookup-conv kernel cases ran in the
same process (the order tests/test_gpu_lookup_conv.py runs them in)."""
import argparse
import importlib.util
import os
import sys
import warnings

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raft_optical_flow_amd import RAFT  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict, smooth_images  # noqa: E402

spec = importlib.util.spec_from_file_location("tlc", os.path.join(ROOT, "tests", "test_gpu_lookup_conv.py"))
tlc = importlib.util.module_from_spec(spec)
spec.loader.exec_module(tlc)
from raft_optical_flow_amd import _lib  # noqa: E402
_lib.load()
pre = os.environ.get("PRE", "all")
if pre == "all":
    for (B, h, w) in [(1, 55, 128), (2, 17, 21), (1, 16, 40)]:
        for prec in ["f16x3", "f16", "bf16"]:
            tlc._case(B, h, w, prec)
    tlc._case(1, 19, 35, "f16x3", coord_sigma=40.0, seed=9)
    tlc._case(1, 16, 24, "f16x3", fscale=200.0, seed=3)
elif pre == "rg":
    tlc._case(1, 16, 24, "f16x3", fscale=200.0, seed=3)
elif pre == "noise":
    x = torch.randn(64 << 20, device="cuda") * 1e6
    del x
torch.cuda.synchronize()
DEV = "cuda"
warnings.simplefilter("always")
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(DEV).eval()
i1, i2 = smooth_images(1, 128, 192, seed=3)
i1, i2 = i1.to(DEV), i2.to(DEV)
with torch.no_grad(), warnings.catch_warnings(record=True) as wl:
    os.environ["RAFT_FUSE_CONVC1"] = "1"
    _, up_a = m(i1, i2, iters=12, test_mode=True)
    pa = m._plans[next(iter(m._plans))]
    torch.cuda.synchronize()
    up_a0 = up_a.clone()
    _, up_a2 = m(i1, i2, iters=12, test_mode=True)   # same plan: capture + replay
    _, up_a3 = m(i1, i2, iters=12, test_mode=True)
    torch.cuda.synchronize()
    os.environ["RAFT_FUSE_CONVC1"] = "0"
    _, up_b = m(i1, i2, iters=12, test_mode=True)
    torch.cuda.synchronize()
    m.check_range_guard()
    print(f"PRE={pre}: plan A flag {int(pa.range_flag.item())}; fused run1 vs run2 {float((up_a0 - up_a2).abs().max()):.3e}, "
          f"run2 vs run3 {float((up_a2 - up_a3).abs().max()):.3e}; fused vs unfused {float((up_a0 - up_b).abs().max()):.3e} "
          f"/ {float((up_a3 - up_b).abs().max()):.3e}; up_a changed later {float((up_a - up_a0).abs().max()):.3e}")
    for w_ in wl:
        if "unclosed" not in str(w_.message):
            print("warning:", str(w_.message)[:150])
