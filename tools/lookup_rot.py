"""Corr-lookup kernel alone, cache-cold (bench.py's rotation: launch k reads pyramid k % NROT),
config-2 geometry (B x 55 x 128, r = 4, 4 levels), coords = grid + N(0, spread^2).
    python tools/lookup_rot.py [spread]     (RAFT_HIP_LIB selects a variant library)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

spread = float(sys.argv[1]) if len(sys.argv) > 1 else 0.7
h, w, L, r = 55, 128, 4, 4
dev = "cuda"
for B, nrot, reps in ((1, 16, 8), (8, 3, 8)):
    g = torch.Generator(device=dev).manual_seed(0)
    nfl = K.pyramid_floats(B, h, w, L)
    pyrs = [torch.randn(nfl, device=dev, generator=g) for _ in range(nrot)]
    ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
    grid = torch.stack([xs, ys], -1).float().reshape(1, h * w, 2).repeat(B, 1, 1).reshape(-1, 2)
    coords = (grid + spread * torch.randn(grid.shape, device=dev, generator=g)).contiguous()
    out = torch.empty(B * h * w, L * 81, device=dev)

    def fn():
        for k in range(nrot):
            _lib.call("raft_corr_lookup", pyrs[k].data_ptr(), B, h, w, L, r, coords.data_ptr(), 0, out.data_ptr(),
                      L * 81, 0, None, 0, None, K.stream_handle())

    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / (reps * nrot))
    t = min(ts)
    alg = B * h * w * (L * 100 * 4 + L * 81 * 4 + 8)
    print(f"{os.environ.get('RAFT_HIP_LIB', 'current')} B={B}: {t:.2f} us  {alg / t / 1e3:.0f} GB/s  frac {alg / t / 1e3 / 8000:.3f}")
    del pyrs
    torch.cuda.empty_cache()
