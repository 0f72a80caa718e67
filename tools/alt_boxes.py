"""Window-box statistics of the alternate lookup's MFMA tile kernel on a real run's coords
(config 3: RAFT-full, alternate_corr, B=8, 440x1024, iters=32, seeded weights and frames as
bench.py): per 8x8 query tile and level, the box of the tile's (2r+2)^2 windows, the bands the
kernel runs over it (csrc/alt_corr.hip alt_corr_mfma_kernel: whole box rows per 96-pixel band)
and the tiles that fall back to the per-pixel path.
    python tools/alt_boxes.py [B] [iters]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import RAFT, InputPadder  # noqa: E402
from raft_optical_flow_amd.init import seeded_images, seeded_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda", 0)
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=True))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(dev).eval()
i1, i2 = seeded_images(B, 436, 1024, seed=1)
i1, i2 = InputPadder(i1.shape).pad(i1.to(dev), i2.to(dev))
with torch.no_grad():
    lo, _ = m(i1, i2, iters=iters, test_mode=True)
h, w = lo.shape[-2:]
ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
coords = torch.stack([xs, ys], 0)[None].float() + lo  # [B,2,h,w]
print(f"flow: |mean| {lo.abs().mean():.2f} px, max {lo.abs().max():.1f} px (1/8 res)")
R, AT, NB = 4, 8, 96
WD = 2 * R + 2
tot_bands = tot_fall = tot_tiles = 0
for lvl in range(4):
    c = coords / 2 ** lvl
    x0 = torch.floor(c[:, 0]) - R
    y0 = torch.floor(c[:, 1]) - R
    th, tw = -(-h // AT), -(-w // AT)
    pad = (0, tw * AT - w, 0, th * AT - h)
    big = 1e9

    def tile_red(t, fn, fill):
        t = torch.nn.functional.pad(t, pad, value=fill)
        t = t.view(B, th, AT, tw, AT).permute(0, 1, 3, 2, 4).reshape(B, th, tw, AT * AT)
        return fn(t)

    mnx = tile_red(x0, lambda t: t.min(-1).values, big)
    mxx = tile_red(x0, lambda t: t.max(-1).values, -big)
    mny = tile_red(y0, lambda t: t.min(-1).values, big)
    mxy = tile_red(y0, lambda t: t.max(-1).values, -big)
    bw = (mxx - mnx + WD)
    bh = (mxy - mny + WD)
    fits = (bw <= NB) & (bh <= NB)
    br = torch.clamp(NB // torch.clamp(bw, min=1), min=1)
    bands = torch.where(fits, torch.ceil(bh / br), torch.zeros_like(bh))
    nt = fits.numel()
    tot_tiles += nt
    tot_bands += float(bands.sum())
    tot_fall += int((~fits).sum())
    q = torch.quantile(bw[fits].float(), torch.tensor([0.5, 0.9, 0.99], device=dev)) if fits.any() else None
    print(f"level {lvl}: tiles {nt}, per-pixel fallback {int((~fits).sum())}, bands mean "
          f"{float(bands[fits].mean()) if fits.any() else 0:.2f} max {float(bands.max()):.0f}, box width p50/p90/p99 "
          f"{q.tolist() if q is not None else None}, box height mean {float(bh[fits].float().mean()):.1f}")
print(f"total: {tot_bands:.0f} bands over {tot_tiles} tile-levels, {tot_fall} per-pixel fallbacks")
