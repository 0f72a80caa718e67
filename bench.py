"""Benchmark: RAFT inference image-pairs/s on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step = one RAFT-full forward (random-init weights, seeded) over one batch of
synthetic frame pairs already resident in HBM: 436x1024 frames replicate-padded
to 440x1024 (InputPadder), iters=32, all-pairs correlation, test_mode, replayed
as one hipGraph.  Each rank processes its own batch (frame pairs shard across
GPUs with no data-path collective; weights are broadcast once over RCCL), so
scaling is weak.  Rank 0 prints one JSON line.

The line also carries
  roofline      the corr-lookup kernel (the metric's "corr-lookup GB/s vs HBM
                peak"): algorithmic bytes P*2904 per pair-iteration / its
                average launch time measured with HIP events on its stream;
                with --alternate-corr (config 3) the on-the-fly lookup's four
                per-level launches instead, against the fp32 VALU peak
                (2*P*L*(2r+2)^2*C flops per iteration);
  lookup_b8     the same kernel at B=8 (where the >=50% target is
                quoted), on a random B=8 pyramid with the run's coords (omitted
                when the run itself is at B >= 8 or uses the alternate corr);
  update_gemm   the same accounting for the update-block convolutions (MFMA-bound;
                peak per conv arithmetic: f32 MFMA 157.3 TF, f16x3 = f16 MFMA / 3);
  fp32_exact    with the default f16x3 conv arithmetic: the same run with exact
                f32 MFMA convs (value, ms_per_step), rank 0, N = 1;
  cpu_baseline  the numpy oracle (oracle/raft_oracle.py) on the host cores for one
                pair of the same workload (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3  # dense f32 MFMA (= f32 vector) peak
F16_MFMA_PEAK_TF = 2500.0  # dense f16 MFMA peak
# fp32-equivalent peak of the update convolutions per conv arithmetic
CONV_PEAK_TF = {"fp32": FP32_MFMA_PEAK_TF, "f16x3": F16_MFMA_PEAK_TF / 3, "f16": F16_MFMA_PEAK_TF}
DTYPE = {"fp32": "fp32", "f16x3": "fp32 (convs: f16x3 split MFMA, fp32 accumulate)",
         "f16": "f16 convs, fp32 accumulate (mixed precision)"}


def lookup_bytes_per_pixel(levels=4, r=4):
    """per query pixel L*(2r+2)^2*4 read + L*(2r+1)^2*4 written + 8 B coords."""
    return levels * (2 * r + 2) ** 2 * 4 + levels * (2 * r + 1) ** 2 * 4 + 8


def alt_lookup_flops(P, levels=4, r=4, C=256):
    """alternate-corr lookup, 2*P*L*(2r+2)^2*C flops per iteration (the reference's
    integer-tap inner products, correlation_kernel.cu:43-114)."""
    return 2 * P * levels * (2 * r + 2) ** 2 * C


def update_flops_per_pixel(pu, with_mask):
    """2*MACs of the update-block convolutions per 1/8-res pixel (one iteration)."""
    def f(pc):
        return 2 * pc.n * pc.kh * pc.kw * pc.cin_real
    tot = 0
    for pc in [pu.convc1, pu.convc2, pu.convf1, pu.convf2, pu.conv]:
        if pc is not None:
            tot += f(pc)
    for zr, q, _ctx in pu.gru:  # the inp context GEMM runs once per pair, not per iteration
        tot += f(zr) + f(q)
    tot += f(pu.fh1_mask if with_mask else pu.fh1) + f(pu.fh2)
    if with_mask:
        tot += f(pu.mask2)
    return tot


def time_kernel_events(fn, reps):
    """Average GPU duration of fn() (kernel launches on the current stream): the reps
    launches are captured in one hipGraph and timed with HIP events around its replay
    on the launch stream, so host launch overhead is not part of the figure."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record(s)
    g.replay()
    end.record(s)
    end.synchronize()
    return start.elapsed_time(end) / reps * 1e-3  # seconds


def lookup_at_b8(plan, dev, h8, w8, B8=8, reps=50):
    """the lookup's HBM roofline measured at B=8 (163.5 MB algorithmic per launch at
    config 2), where it is not launch/latency-bound: a B=8 pyramid of the same geometry (random
    values: the lookup is data-independent) and the B=1 run's final coords replicated 8x."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib = _lib.load()
    L, r = plan.pk.levels, plan.pk.radius
    pyr = torch.randn(int(lib.raft_corr_pyramid_floats(B8, h8, w8, L)), device=dev)
    coords = plan.ub.coords.repeat(B8, 1).contiguous()
    ntap = L * (2 * r + 1) ** 2
    out = torch.empty(B8 * h8 * w8, ntap, device=dev)

    def fn():
        _lib.call("raft_corr_lookup", pyr.data_ptr(), B8, h8, w8, L, r, coords.data_ptr(), 0, out.data_ptr(), ntap, 0,
                  None, 0, K.stream_handle())

    t = time_kernel_events(fn, reps)
    alg = B8 * h8 * w8 * lookup_bytes_per_pixel(L, r)
    del pyr
    return {"kernel": "raft_corr_lookup", "batch": B8, "bound": "hbm", "achieved": round(alg / t / 1e9, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": alg, "launch_us": round(t * 1e6, 2)}


def cpu_baseline(args):
    """The oracle (numpy restatement of the reference path) on one pair of the same workload."""
    import numpy as np
    from oracle import raft_oracle as O
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    p = {k: v.numpy() for k, v in seeded_state_dict(m, 0).items()}
    i1, i2 = seeded_images(1, args.height, args.width, seed=1)
    # InputPadder 'sintel' mode (core/utils/utils.py:7-24): replicate pad, centred, to multiples of 8
    ph, pw = (-args.height) % 8, (-args.width) % 8
    pads = ((0, 0), (0, 0), (ph // 2, ph - ph // 2), (pw // 2, pw - pw // 2))
    i1 = np.pad(i1.numpy(), pads, mode="edge")
    i2 = np.pad(i2.numpy(), pads, mode="edge")
    t0 = time.perf_counter()
    O.raft_forward(p, i1, i2, iters=args.iters)
    dt = time.perf_counter() - t0
    return {"value": round(1.0 / dt, 4), "unit": "image-pairs/s", "cores": threads, "kind": "port",
            "sample": f"1 pair {args.height}x{args.width} (padded to {i1.shape[2]}x{i1.shape[3]}), iters={args.iters}, "
                      f"numpy oracle, {dt:.1f} s"}


def load_traffic():
    """HBM bytes per lookup launch from the committed PMC pass (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", "lookup_pmc.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1, help="frame pairs per GPU per step")
    ap.add_argument("--height", type=int, default=436)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=32)
    ap.add_argument("--alternate-corr", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-fp32-exact", action="store_true", help="skip the exact-f32 comparison run")
    ap.add_argument("--precision", choices=["fp32", "f16x3", "f16"], default=None,
                    help="conv arithmetic (default: the RAFT default, f16x3)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from raft_optical_flow_amd import RAFT, InputPadder
    from raft_optical_flow_amd.dist import broadcast_state_dict
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict

    model = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=args.alternate_corr))
    if rank == 0:
        model.load_state_dict(seeded_state_dict(model, 0))
    model.to(dev).eval()
    model.conv_precision = args.precision
    prec = model.resolved_precision()
    if world > 1:
        broadcast_state_dict(model, src=0)  # one RCCL broadcast over xGMI

    # synthetic frames resident in HBM: a pool of distinct pairs, cycled per step
    pool = []
    for k in range(4):
        i1, i2 = seeded_images(args.batch, args.height, args.width, seed=1 + 1000 * rank + k)
        i1, i2 = i1.to(dev), i2.to(dev)
        padder = InputPadder(i1.shape)
        pool.append(padder.pad(i1, i2))
    H, W = pool[0][0].shape[-2:]
    plan = model.plan(args.batch, H, W, args.iters, test_mode=True, device=dev)

    def timed(plan, barrier):
        def step(k):
            plan.set_inputs(*pool[k % len(pool)])
            if args.no_graph:
                plan.run()
            else:
                plan.replay()

        if not args.no_graph:
            plan.capture()
        for k in range(args.warmup):
            step(k)
        torch.cuda.synchronize()
        if barrier:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(k)
        torch.cuda.synchronize()
        if barrier:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    elapsed = timed(plan, world > 1)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pairs = world * args.batch * args.steps
    value = pairs / elapsed

    # ---- per-kernel live timing (HIP events on the launch stream) -------------------
    from raft_optical_flow_amd import kernels as K
    lk = [l for l in plan.launches[plan.loop_start:plan.loop_end] if getattr(l, "name", None) in
          ("raft_corr_lookup", "raft_alt_corr_lookup_nhwc")]
    reps = 200
    h8, w8 = H // 8, W // 8
    P = args.batch * h8 * w8
    if not args.alternate_corr:
        t_lookup = time_kernel_events(lambda: [l(K.stream_handle()) for l in lk[:1]], reps)
        bytes_per_launch = P * lookup_bytes_per_pixel()
        achieved = bytes_per_launch / t_lookup / 1e9
        # the committed PMC pass was taken at config 2 (B=1, 440x1024): only that shape carries it
        traffic = load_traffic() if (args.batch, H, W) == (1, 440, 1024) else None
        roof = {"kernel": "raft_corr_lookup", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                "algorithmic_bytes_per_launch": bytes_per_launch, "launch_us": round(t_lookup * 1e6, 2)}
    else:
        # alternate corr: FP32 VALU-bound, 2*P*L*(2r+2)^2*C flops over the L per-level launches
        nl = plan.pk.levels
        t_lookup = time_kernel_events(lambda: [l(K.stream_handle()) for l in lk[:nl]], reps)
        fl = alt_lookup_flops(P, nl, plan.pk.radius, plan.pk.fdim)
        roof = {"kernel": f"raft_alt_corr_lookup_nhwc x{nl}", "bound": "valu", "achieved": round(fl / t_lookup / 1e12, 2),
                "peak": FP32_MFMA_PEAK_TF, "unit": "TFLOP/s", "frac": round(fl / t_lookup / 1e12 / FP32_MFMA_PEAK_TF, 4),
                "traffic": None, "algorithmic_flops_per_iteration": fl, "launch_us": round(t_lookup * 1e6, 2)}

    # at B >= 8 the main roofline line already is the batched measurement
    lookup_b8 = None if (args.alternate_corr or args.batch >= 8) else lookup_at_b8(plan, dev, h8, w8)

    it_launches = plan.launches[plan.loop_start:plan.loop_end]
    upd = [l for l in it_launches if getattr(l, "name", None) == "raft_conv2d"]
    n_iter_convs = len(upd) // args.iters
    # one non-final iteration's conv GEMMs (no mask head)
    one_iter = upd[:n_iter_convs - 0]
    pu = plan.pk.update
    t_upd = time_kernel_events(lambda: [l(K.stream_handle()) for l in one_iter], 50)
    fl = P * update_flops_per_pixel(pu, with_mask=False)
    upd_tf = fl / t_upd / 1e12
    peak = CONV_PEAK_TF[prec]
    update_roof = {"kernel": f"raft_conv2d (update block, one iteration, {prec})", "bound": "mfma",
                   "achieved": round(upd_tf, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                   "frac": round(upd_tf / peak, 4), "iteration_us": round(t_upd * 1e6, 1),
                   "flops_per_iteration": fl}

    exact = None
    if prec != "fp32" and world == 1 and not args.no_fp32_exact:
        model.conv_precision = "fp32"
        plan32 = model.plan(args.batch, H, W, args.iters, test_mode=True, device=dev)
        e32 = timed(plan32, False)
        exact = {"value": round(args.batch * args.steps / e32, 3), "ms_per_step": round(e32 / args.steps * 1e3, 3)}
        model.conv_precision = args.precision

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        out = {
            "metric": "image-pairs/s at Sintel 436x1024, 32 iters; corr-lookup GB/s vs HBM peak",
            "value": round(value, 3), "unit": "image-pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": DTYPE[prec],
            "data": "synthetic (seeded uint8-valued frames, random-init seeded weights)",
            "config": {"workload": f"RAFT-full inference, {args.height}x{args.width} padded to {H}x{W}, "
                                   f"{args.batch} pair(s)/GPU/step, iters={args.iters}, "
                                   f"{'alternate' if args.alternate_corr else 'all-pairs'} corr, "
                                   f"{'eager' if args.no_graph else 'hipGraph'}",
                       "global_batch": world * args.batch, "parallelism": f"frame-pair sharding x{world}"},
            "roofline": roof,
            "lookup_b8": lookup_b8,
            "update_gemm": update_roof,
            "fp32_exact": exact,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
