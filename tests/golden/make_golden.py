"""Generate the golden vectors in tests/golden/ by running the REFERENCE.

Runs only in the build container, where the reference snapshot is mounted at
/root/reference (read-only).  It imports the reference's own `core/` modules
(core/raft.py, core/corr.py, core/update.py, core/extractor.py,
core/utils/utils.py) and `liteflownet3_correlation.IterativeCorrBlock` (the
reference's pure-PyTorch mimic of AlternateCorrBlock), feeds them seeded
inputs and the portable seeded weights of `raft_optical_flow_amd.init`, and
stores inputs + outputs as .npz data.  No reference source is copied: the
fixtures are numbers only.  Nothing at test time reads /root/reference.

    python tests/golden/make_golden.py            # all fixtures
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RAFT_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "core"))
sys.path.insert(0, REF)

from raft_optical_flow_amd.init import seeded_images, seeded_state_dict, smooth_images  # noqa: E402

torch.set_num_threads(8)


def ref_modules():
    import corr as rcorr  # noqa: F401  (core/corr.py)
    import raft as rraft  # core/raft.py
    import update as rupdate  # core/update.py
    import utils.utils as rutils  # core/utils/utils.py
    return rraft, rcorr, rupdate, rutils


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.0f} KB)")


def make_args(small: bool, alternate=False):
    return argparse.Namespace(small=small, mixed_precision=False, alternate_corr=alternate, dropout=0)


def ref_model(small: bool, seed: int):
    rraft, *_ = ref_modules()
    m = rraft.RAFT(make_args(small))
    sd = seeded_state_dict(m, seed)
    missing, unexpected = m.load_state_dict(sd, strict=True), None
    m.eval()
    return m


@torch.no_grad()
def gen_lookup():
    _, rcorr, _, _ = ref_modules()
    from liteflownet3_correlation import IterativeCorrBlock
    g = torch.Generator().manual_seed(11)
    B, C, H, W = 2, 64, 16, 20
    f1 = torch.randn(B, C, H, W, generator=g)
    f2 = torch.randn(B, C, H, W, generator=g)
    ys, xs = torch.meshgrid(torch.arange(H).float(), torch.arange(W).float(), indexing="ij")
    base = torch.stack([xs, ys], 0)[None].repeat(B, 1, 1, 1)
    coords = base + 3.0 * torch.randn(B, 2, H, W, generator=g)
    coords[0, :, 0, 0] = torch.tensor([-30.0, 5.0])       # far out of bounds
    coords[0, :, 0, 1] = torch.tensor([W + 7.5, H + 0.25])
    coords[1, :, 3, 3] = torch.tensor([5.0, 7.0])          # exact integers
    out = {}
    for r in (4, 3):
        cb = rcorr.CorrBlock(f1, f2, num_levels=4, radius=r)
        out[f"corr_r{r}"] = cb(coords)
        it = IterativeCorrBlock(f1, f2, radius=r, num_levels=4)
        out[f"iter_r{r}"] = it(coords)
    save("lookup_b2c64_16x20.npz", fmap1=f1, fmap2=f2, coords=coords, **out)

    # pyramid itself, small enough to store whole
    f1 = torch.randn(1, 32, 8, 12, generator=g)
    f2 = torch.randn(1, 32, 8, 12, generator=g)
    cb = rcorr.CorrBlock(f1, f2, num_levels=4, radius=4)
    save("pyramid_b1c32_8x12.npz", fmap1=f1, fmap2=f2,
         **{f"level{i}": p for i, p in enumerate(cb.corr_pyramid)})

    # 1-pixel pyramid level: W-1 == 0 in bilinear_sampler (core/utils/utils.py:61-62)
    f1 = torch.randn(1, 16, 6, 8, generator=g)
    f2 = torch.randn(1, 16, 6, 8, generator=g)
    ys, xs = torch.meshgrid(torch.arange(6).float(), torch.arange(8).float(), indexing="ij")
    coords = torch.stack([xs, ys], 0)[None] + 0.3
    cb = rcorr.CorrBlock(f1, f2, num_levels=3, radius=2)   # levels 6x8, 3x4, 1x2
    save("lookup_degenerate_6x8.npz", fmap1=f1, fmap2=f2, coords=coords, corr=cb(coords))


@torch.no_grad()
def gen_update_and_upsample():
    rraft, _, rupdate, _ = ref_modules()
    g = torch.Generator().manual_seed(12)
    H, W = 16, 24
    for small in (False, True):
        m = ref_model(small, seed=0)
        ub = m.update_block
        hdim = 96 if small else 128
        cdim = 64 if small else 128
        cor_planes = 4 * (2 * (3 if small else 4) + 1) ** 2
        net = torch.tanh(torch.randn(1, hdim, H, W, generator=g))
        inp = torch.relu(torch.randn(1, cdim, H, W, generator=g))
        corr = torch.randn(1, cor_planes, H, W, generator=g) * 2.0
        flow = torch.randn(1, 2, H, W, generator=g) * 3.0
        net2, mask, delta = ub(net, inp, corr, flow)
        tag = "small" if small else "full"
        extra = {} if mask is None else {"mask_out": mask}
        save(f"update_{tag}_16x24.npz", net=net, inp=inp, corr=corr, flow=flow,
             net_out=net2, delta_out=delta, **extra)
        if not small:
            up = m.upsample_flow(flow, mask)
            save("upsample_16x24.npz", flow=flow, mask=mask, flow_up=up)
    _, _, _, rutils = ref_modules()
    flow = torch.randn(2, 2, 5, 7, generator=g) * 2
    save("upflow8_5x7.npz", flow=flow, flow_up=rutils.upflow8(flow))


@torch.no_grad()
def gen_encoders():
    g = torch.Generator().manual_seed(13)
    img = torch.rand(2, 3, 64, 96, generator=g) * 2 - 1
    m = ref_model(False, seed=0)
    ms = ref_model(True, seed=0)
    save("encoders_64x96.npz", image=img, fnet=m.fnet(img), cnet=m.cnet(img[:1]),
         fnet_small=ms.fnet(img), cnet_small=ms.cnet(img[:1]))


@torch.no_grad()
def gen_raft_e2e(full_size: bool):
    cases = [
        # name, small, seed, images, iters
        ("raft_full_smooth_b2_128x192_i12", False, 0, smooth_images(2, 128, 192, seed=3), 12),
        ("raft_full_rand_b1_128x192_i32", False, 0, seeded_images(1, 128, 192, seed=1), 32),
        ("raft_small_smooth_b1_128x192_i12", True, 0, smooth_images(1, 128, 192, seed=4), 12),
    ]
    for name, small, seed, (i1, i2), iters in cases:
        m = ref_model(small, seed)
        low, up = m(i1, i2, iters=iters, test_mode=True)
        save(name + ".npz", image1=i1, image2=i2, iters=iters, seed=seed, flow_low=low, flow_up=up)
    if full_size:
        i1, i2 = seeded_images(1, 440, 1024, seed=1)
        m = ref_model(False, 0)
        low, up = m(i1, i2, iters=32, test_mode=True)
        # images regenerate from the seed; flow_up kept on every 8th row + global checksums
        save("raft_full_rand_b1_440x1024_i32.npz", iters=32, seed=0, img_seed=1, flow_low=low,
             flow_up_rows8=up[:, :, ::8], flow_up_sum=up.double().sum(), flow_up_abs=up.double().abs().sum())


@torch.no_grad()
def gen_lookup_big_radius():
    """CorrBlock / IterativeCorrBlock at radius 5 and 6 (the reference takes any r; RAFT uses 3, 4)
    on the inputs of lookup_b2c64_16x20.npz."""
    _, rcorr, _, _ = ref_modules()
    from liteflownet3_correlation import IterativeCorrBlock
    with np.load(os.path.join(HERE, "lookup_b2c64_16x20.npz")) as z:
        f1, f2, coords = (torch.from_numpy(z[k]) for k in ("fmap1", "fmap2", "coords"))
    out = {}
    for r in (5, 6):
        out[f"corr_r{r}"] = rcorr.CorrBlock(f1, f2, num_levels=4, radius=r)(coords)
    out["iter_r6_err"] = (IterativeCorrBlock(f1, f2, radius=6, num_levels=4)(coords) - out["corr_r6"]).abs().max()
    save("lookup_b2c64_16x20_r56.npz", **out)


@torch.no_grad()
def gen_caller():
    """Caller-side helpers of core/utils/utils.py: InputPadder pads (both modes, many sizes) and a
    padded tensor, forward_interpolate (scipy griddata 'nearest') on smooth / leaving / zero flows,
    bilinear_sampler with its mask."""
    _, _, _, rutils = ref_modules()
    g = torch.Generator().manual_seed(21)
    dims = [(436, 1024), (540, 960), (1080, 1920), (375, 1242), (370, 1226), (100, 100), (8, 8), (13, 21)]
    pads = np.array([[rutils.InputPadder((1, 3, h, w), mode=m)._pad for (h, w) in dims] for m in ("sintel", "kitti")])
    x = torch.rand(2, 3, 13, 21, generator=g) * 255
    out = {"dims": np.array(dims), "pads": pads, "pad_in": x,
           "pad_sintel": rutils.InputPadder(x.shape).pad(x)[0],
           "pad_kitti": rutils.InputPadder(x.shape, mode="kitti").pad(x)[0]}
    ys, xs = torch.meshgrid(torch.arange(55).float(), torch.arange(128).float(), indexing="ij")
    smooth = torch.stack([4 * torch.sin(xs / 17 + ys / 23) + 1.3, 3 * torch.cos(ys / 11 - xs / 29) - 0.7])
    leaving = smooth * 6 + torch.randn(2, 55, 128, generator=g) * 2
    zero = torch.zeros(2, 16, 24)
    for name, f in (("fi_smooth", smooth), ("fi_leaving", leaving), ("fi_zero", zero)):
        out[name + "_in"] = f
        out[name + "_out"] = rutils.forward_interpolate(f)
    img = torch.randn(2, 3, 9, 11, generator=g)
    coords = torch.rand(2, 5, 7, 2, generator=g) * torch.tensor([14.0, 12.0]) - torch.tensor([2.0, 1.5])
    coords[0, 0, 0] = torch.tensor([4.0, 3.0])     # exact integers
    smp, msk = rutils.bilinear_sampler(img, coords, mask=True)
    out.update(bs_img=img, bs_coords=coords, bs_out=smp, bs_mask=msk)
    save("caller_utils.npz", **out)


@torch.no_grad()
def gen_config4():
    """Config 4 shape: 540x960 frames padded (InputPadder 'sintel') to 544x960, B=1, iters=32."""
    i1, i2 = seeded_images(1, 544, 960, seed=2)
    m = ref_model(False, 0)
    low, up = m(i1, i2, iters=32, test_mode=True)
    save("raft_full_rand_b1_544x960_i32.npz", iters=32, seed=0, img_seed=2, flow_low=low,
         flow_up_rows8=up[:, :, ::8], flow_up_sum=up.double().sum(), flow_up_abs=up.double().abs().sum())


@torch.no_grad()
def gen_bf16():
    """Config 5 arithmetic: the reference with mixed_precision=True under CPU bf16 autocast
    (core/raft.py:177,193,225 enter `autocast(enabled=mixed_precision)`; the module attribute
    is pointed at torch.autocast('cpu', bfloat16) for the run)."""
    rraft, *_ = ref_modules()
    saved = rraft.autocast
    rraft.autocast = lambda enabled=True: torch.autocast("cpu", dtype=torch.bfloat16, enabled=enabled)
    try:
        for (h, w, iters, img_seed) in ((128, 192, 32, 1),):
            i1, i2 = seeded_images(1, h, w, seed=img_seed)
            m = rraft.RAFT(argparse.Namespace(small=False, mixed_precision=True, alternate_corr=False, dropout=0))
            m.load_state_dict(seeded_state_dict(m, 0))
            m.eval()
            low, up = m(i1, i2, iters=iters, test_mode=True)
            save(f"raft_full_rand_b1_{h}x{w}_i{iters}_bf16.npz", iters=iters, seed=0, img_seed=img_seed,
                 flow_low=low.float(), flow_up=up.float())
    finally:
        rraft.autocast = saved


@torch.no_grad()
def gen_bf16_config5():
    """Config 5 at its real size: 1080x1920 (a multiple of 8: no padding), iters=32, the reference
    with mixed_precision=True under CPU bf16 autocast (as gen_bf16); flow_low and every 8th row of
    flow_up are stored (plus the whole field's sum and absolute sum)."""
    rraft, *_ = ref_modules()
    saved = rraft.autocast
    rraft.autocast = lambda enabled=True: torch.autocast("cpu", dtype=torch.bfloat16, enabled=enabled)
    try:
        i1, i2 = seeded_images(1, 1080, 1920, seed=5)
        m = rraft.RAFT(argparse.Namespace(small=False, mixed_precision=True, alternate_corr=False, dropout=0))
        m.load_state_dict(seeded_state_dict(m, 0))
        m.eval()
        low, up = m(i1, i2, iters=32, test_mode=True)
        low, up = low.float(), up.float()
        save("raft_full_rand_b1_1080x1920_i32_bf16.npz", iters=32, seed=0, img_seed=5, flow_low=low,
             flow_up_rows8=up[:, :, ::8], flow_up_sum=up.double().sum(), flow_up_abs=up.double().abs().sum())
    finally:
        rraft.autocast = saved


@torch.no_grad()
def gen_raft_small_demo():
    """Config 1: raft-small.pth on demo-frames 0016 -> 0017, iters=12 (reference demo.py path)."""
    from PIL import Image
    rraft, _, _, rutils = ref_modules()
    sd = torch.load(os.path.join(REF, "raft-small.pth"), map_location="cpu", weights_only=True)
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    m = rraft.RAFT(make_args(True))
    m.load_state_dict(sd)
    m.eval()

    def load(p):
        return torch.from_numpy(np.array(Image.open(p)).astype(np.uint8)).permute(2, 0, 1).float()[None]

    i1 = load(os.path.join(REF, "demo-frames", "frame_0016.png"))
    i2 = load(os.path.join(REF, "demo-frames", "frame_0017.png"))
    padder = rutils.InputPadder(i1.shape)
    p1, p2 = padder.pad(i1, i2)
    low, up = m(p1, p2, iters=12, test_mode=True)
    # the two demo PNGs are kept byte-for-byte (data files of the reference); flow_up every 4th row
    png = {f"png{j}": np.frombuffer(open(os.path.join(REF, "demo-frames", f"frame_00{n}.png"), "rb").read(), np.uint8)
           for j, n in ((1, 16), (2, 17))}
    save("raft_small_demo_0016_0017_i12.npz", **png, pad=np.array(padder._pad), flow_low=low,
         flow_up_rows4=up[:, :, ::4], flow_up_sum=up.double().sum(), flow_up_abs=up.double().abs().sum())
    save("raft_small_weights.npz", **{k: v for k, v in sd.items()})


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--full-size", action="store_true", help="also the 440x1024 iters=32 case (slow)")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    jobs = {"lookup": gen_lookup, "update": gen_update_and_upsample, "enc": gen_encoders,
            "e2e": lambda: gen_raft_e2e(a.full_size), "demo": gen_raft_small_demo,
            "config4": gen_config4, "bf16": gen_bf16, "bf16big": gen_bf16_config5, "caller": gen_caller, "bigr": gen_lookup_big_radius}
    for k, f in jobs.items():
        if not a.only or k in a.only.split(","):
            f()
