import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import load_golden
from raft_optical_flow_amd import CorrBlock
g = load_golden("lookup_b2c64_16x20.npz")
t = lambda x: torch.from_numpy(x).cuda()
cb = CorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=4)
out = cb(t(g["coords"])).cpu().numpy()
ref = g["corr_r4"]
d = np.abs(out - ref)
print("max", np.nanmax(d), "nan mismatch", (np.isnan(out) != np.isnan(ref)).sum())
idx = np.argwhere(d > 1e-5)
print(len(idx), idx[:20])
for b, c, y, x in idx[:10]:
    print(b, c, y, x, out[b, c, y, x], ref[b, c, y, x], g["coords"][b, :, y, x])
bad = d > 1e-5
print("bad per level", [int(bad[:, l * 81:(l + 1) * 81].sum()) for l in range(4)])
print("bad per pixel count hist", np.bincount(bad.sum(1).ravel())[:20], "pixels with any", int((bad.sum(1) > 0).sum()), "of", bad.shape[0] * bad.shape[2] * bad.shape[3])
for (b, y, x) in [tuple(v) for v in np.argwhere(bad.sum(1) > 0)[:4]]:
    m = bad[b, :, y, x].reshape(4, 9, 9)
    print("pixel", b, y, x, g["coords"][b, :, y, x])
    for l in range(4):
        if m[l].any():
            print(" level", l); print(m[l].astype(int))
