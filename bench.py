"""Benchmark: RAFT inference image-pairs/s on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: spawns one rank per GPU itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step = one RAFT-full forward (random-init weights, seeded) over one batch of
synthetic frame pairs already resident in HBM: 436x1024 frames replicate-padded
to 440x1024 (InputPadder), iters=32, all-pairs correlation, test_mode, replayed
as one hipGraph.  Each rank processes its own batch (frame pairs shard across
GPUs with no data-path collective; weights are broadcast once over RCCL), so
scaling is weak.  Rank 0 prints one JSON line.

The line also carries
  roofline      the forward's own lookup launch (the metric's "corr-lookup GB/s vs HBM
                peak"): with the all-pairs RAFT-full loop that is raft_corr_lookup_conv
                (the window lookup fused with the motion encoder's convc1 and convf1:
                the 324-channel correlation rows never leave the CU), HBM-bound:
                algorithmic bytes per pair-iteration = P * (L*(2r+2)^2*4 window reads +
                8 coords + 4*(256 + 128) convc1 / convf1 outputs + 8 flow) over its
                per-dispatch duration in the forward (the library's device launch span,
                raft_debug_launch_span, over one eager forward whose kernels run back to
                back; the rocprofv3 per-dispatch mean of the same kernel in the forward is
                committed under profiles/, tools/roofline_rocprof.py); without the fused launch (fp32
                mode) the lookup-only kernel (HIP event pairs in an eager forward)
                with SURVEY 8(d)'s P*2904 B; `traffic` = HBM bytes per launch from a
                committed in-forward PMC summary taken on the current kernel source;
                with --alternate-corr (config 3) the on-the-fly lookup against its peak;
  lookup_b1, lookup_b8  the standalone lookup kernel (raft_corr_lookup, what CorrBlock.__call__
                runs) at B=1 and B=8 (where the >=50% target is quoted),
                cache-cold over rotating pyramids, P*2904 B per launch;
  iteration     one refinement iteration's launches (lookup launch + update convs), replayed;
  update_gemm   the update block's main-stream convolutions of one iteration, timed
                as a replayed graph (MFMA-bound; fp32-equivalent peak per conv arithmetic:
                f32 MFMA 157.3 TF, f16x3 = f16 MFMA / 3, f16 / bf16 2.5 PF);
  dominant_kernel  the step's dominant kernel, conv_halo_kernel<3,3,64> (convc2 and
                the flow-head conv1), with the MFMA-busy PMC of the newest committed
                profiles/rNN_halo_pmc.json taken on the current conv_halo.hip;
  drop_in_forward  the same workload through RAFT.forward() itself (the unchanged caller's call, default
                range guard: one host flag read per forward), beside `value`'s plan.replay() loop;
  fp32_exact    with the default f16x3 conv arithmetic: the same run with exact
                f32 MFMA convs (value, ms_per_step), rank 0, N = 1;
  cpu_baseline  the reference's CPU path restated with the same torch CPU operators
                (oracle/torch_cpu.py) on the host cores, whole pairs of the same
                workload for ~12 s (rank 0, N = 1 only).
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
CONV_PEAK_TF = {"fp32": FP32_MFMA_PEAK_TF, "f16x3": F16_MFMA_PEAK_TF / 3, "f16": F16_MFMA_PEAK_TF,
                "bf16": F16_MFMA_PEAK_TF}
DTYPE = {"fp32": "fp32", "f16x3": "fp32 (convs: f16x3 split MFMA, fp32 accumulate)",
         "f16": "f16 convs, fp32 accumulate (mixed precision)",
         "bf16": "bf16 convs, fp32 accumulate (bf16 mixed precision; corr volume + lookup fp32-accurate)"}


def lookup_bytes_per_pixel(levels=4, r=4):
    """per query pixel L*(2r+2)^2*4 read + L*(2r+1)^2*4 written + 8 B coords."""
    return levels * (2 * r + 2) ** 2 * 4 + levels * (2 * r + 1) ** 2 * 4 + 8


def alt_lookup_flops(P, levels=4, r=4, C=256):
    """alternate-corr lookup, 2*P*L*(2r+2)^2*C flops per iteration (the reference's
    integer-tap inner products, correlation_kernel.cu:43-114)."""
    return 2 * P * levels * (2 * r + 2) ** 2 * C


def fused_lookup_bytes_per_pixel(levels=4, r=4, c1=256, f1=128):
    """raft_corr_lookup_conv per query pixel: L*(2r+2)^2*4 window reads + 8 B coords + the convc1 and
    convf1 output rows (4*(c1 + f1) B) + the 8-B flow row; the correlation rows stay in LDS."""
    return levels * (2 * r + 2) ** 2 * 4 + 8 + 4 * (c1 + f1) + 8


def inforward_launch_us(plan, name):
    """Mean duration of the launches called `name` inside one eagerly enqueued forward of `plan`:
    HIP event pairs on the launch stream around each such launch (the other launches run as in
    the forward, so caches are in the forward's state)."""
    from raft_optical_flow_amd import kernels as K
    main = torch.cuda.current_stream()
    side = plan.side_stream or torch.cuda.Stream(device=plan.device)
    pairs = []
    torch.cuda.synchronize()
    # the GPU spins while the host enqueues the whole forward, so every launch (and each event pair)
    # sits in the queue before the GPU reaches it: the pairs time the kernels back to back, as in the
    # graph replay, not the host's launch latency
    torch.cuda._sleep(100_000_000)
    for l in plan.launches:
        if l is K.FORK:
            side.wait_stream(main)
        elif l is K.JOIN:
            main.wait_stream(side)
        elif not l.side and l.name == name:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            l(main.cuda_stream)
            b.record(main)
            pairs.append((a, b))
        else:
            l(side.cuda_stream if l.side else main.cuda_stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) * 1e3, len(pairs)


def inforward_span_us(plan):
    """Per-dispatch duration of the forward's fused lookup launches (raft_corr_lookup_conv) as they
    run in the forward: the library's launch-span timing (raft_debug_launch_span: the device
    realtime counter at each launch's first work-group start and last work-group end) over one
    eager forward enqueued behind a GPU spin, so its kernels run back to back as in the graph
    replay.  Returns (mean us, launches) or None."""
    import ctypes
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    main = torch.cuda.current_stream()
    side = plan.side_stream or torch.cuda.Stream(device=plan.device)
    torch.cuda.synchronize()
    _lib.call("raft_debug_launch_span", 1)
    try:
        torch.cuda._sleep(100_000_000)
        for l in plan.launches:
            if l is K.FORK:
                side.wait_stream(main)
            elif l is K.JOIN:
                main.wait_stream(side)
            else:
                l(side.cuda_stream if l.side else main.cuda_stream)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 512)()
        _lib.call("raft_debug_launch_span_read", buf, 512)
    finally:
        _lib.call("raft_debug_launch_span", 0)
    spans = [(buf[2 * k + 1] - buf[2 * k]) * 0.01 for k in range(256) if buf[2 * k] != 2 ** 64 - 1 and buf[2 * k + 1]]
    return (sum(spans) / len(spans), len(spans)) if spans else None


def inforward_graph_us(plan, name, reps=5):
    """Per-dispatch duration of the launches called `name` INSIDE the graph-replayed forward: the
    plan's whole launch list captured as one hipGraph with timing events (external event-record
    nodes) around each such launch on the main stream, replayed `reps` times; the mean over the
    last replay's pairs.  The other launches run as in the forward (caches in the forward's state).
    Returns (us, pairs), or None when events cannot be captured."""
    from raft_optical_flow_amd import kernels as K
    try:
        side = plan.side_stream or torch.cuda.Stream(device=plan.device)
        pairs = []
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            for l in plan.launches:
                if l is K.FORK:
                    side.wait_stream(cur)
                elif l is K.JOIN:
                    cur.wait_stream(side)
                elif not l.side and l.name == name:
                    a = torch.cuda.Event(enable_timing=True, external=True)
                    b = torch.cuda.Event(enable_timing=True, external=True)
                    a.record(cur)
                    l(cur.cuda_stream)
                    b.record(cur)
                    pairs.append((a, b))
                else:
                    l(side.cuda_stream if l.side else cur.cuda_stream)
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        us = sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) * 1e3
        del g
        return us, len(pairs)
    except Exception:  # noqa: BLE001 (event capture unsupported: the caller falls back)
        torch.cuda.synchronize()
        return None


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


def halo_bn(ns, batch, h, w):
    """The N tile conv_halo_launch / conv_halo_launch_pair picks (csrc/conv_halo.hip) for a launch
    of the convs with output channels `ns` (one, or a raft_conv2d_pair): 64 unless 32 keeps more
    CUs busy."""
    spatial = batch * -(-h // 8) * -(-w // 16)
    return 64 if sum(spatial * (-(-n // 64)) for n in ns) > 128 else 32


def launch_convs(l):
    """The raft_conv2d_params of a conv launch: one, the two of a raft_conv2d_pair, or every conv
    of a raft_conv2d_chain."""
    if l.name == "raft_conv2d_chain":
        return tuple(l.keep[1])
    return l.keep if isinstance(l.keep, tuple) else (l.keep,)


def rotated_lookup(plan, batch, h8, w8, nrot, reps):
    """Average duration of the corr-lookup kernel at `batch` pairs, cache-cold: one hipGraph of
    reps x nrot launches, launch k on its own pyramid k % nrot (random values: the lookup's cost
    does not depend on them) with the forward's own final coords, timed with HIP events around the
    replay on the launch stream.  nrot is chosen so the windows the nrot launches touch exceed the
    256 MiB Infinity Cache, so no launch is served from a cache its predecessor warmed
    (back-to-back replays of ONE launch would be: its ~28 MB per pair stays resident).
    In a graph replay consecutive kernels run with no gap, so this average is the per-dispatch
    duration rocprofv3 reports for the same launches (tools/forward_avg.py)."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    dev = plan.device
    L, r = plan.pk.levels, plan.pk.radius
    nfl = int(_lib.load().raft_corr_pyramid_floats(batch, h8, w8, L))
    pyrs = [torch.randn(nfl, device=dev) for _ in range(nrot)]
    reps_b = -(-batch // plan.B)
    coords = plan.ub.coords.view(plan.B, -1, 2).repeat(reps_b, 1, 1)[:batch].reshape(-1, 2).contiguous()
    ntap = L * (2 * r + 1) ** 2
    out = torch.empty(batch * h8 * w8, ntap, device=dev)

    def fn():
        for k in range(nrot):
            _lib.call("raft_corr_lookup", pyrs[k].data_ptr(), batch, h8, w8, L, r, coords.data_ptr(), 0,
                      out.data_ptr(), ntap, 0, None, 0, None, K.stream_handle())

    t = time_kernel_events(fn, reps) / nrot
    del pyrs
    torch.cuda.empty_cache()
    alg = batch * h8 * w8 * lookup_bytes_per_pixel(L, r)
    return {"kernel": "corr_lookup_kernel<4,4,false> (raft_corr_lookup)", "batch": batch, "bound": "hbm",
            "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg,
            "launch_us": round(t * 1e6, 2),
            "timing": f"HIP events around a hipGraph of {reps * nrot} launches rotating over {nrot} pyramids "
                      f"({nrot * nfl * 4 / 2**30:.1f} GiB; cache-cold), the forward's final coords"}


def load_pmc(kind, source):
    """The newest committed PMC summary profiles/r<NN>_<kind> taken on the current kernel source: its
    source_sha must equal the sha1 of that .hip file (else the counters are stale and None is
    returned).  Returns (summary, file name) or (None, None)."""
    import glob
    import hashlib
    with open(os.path.join(ROOT, "raft_optical_flow_amd", "csrc", source), "rb") as f:
        sha = hashlib.sha1(f.read()).hexdigest()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{kind}")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("source_sha") == sha:
            return d, os.path.basename(path)
    return None, None


def cpu_baseline(args, budget_s=12.0):
    """The reference's CPU path, restated with the same torch CPU operators (oracle/torch_cpu.py:
    bit-identical flow and the same speed as the reference's own core/ in the build container),
    on the host cores: one warm-up pair at iters=2, then whole pairs of the bench workload until
    `budget_s` seconds have passed (at least one)."""
    from oracle import torch_cpu as T
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    p = seeded_state_dict(m, 0)
    i1, i2 = seeded_images(1, args.height, args.width, seed=1)
    # InputPadder 'sintel' mode (core/utils/utils.py:7-24): replicate pad, centred, to multiples of 8
    ph, pw = (-args.height) % 8, (-args.width) % 8
    pads = (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)
    i1 = torch.nn.functional.pad(i1, pads, mode="replicate")
    i2 = torch.nn.functional.pad(i2, pads, mode="replicate")
    T.raft_forward(p, i1, i2, iters=2)
    n, t0 = 0, time.perf_counter()
    while n == 0 or time.perf_counter() - t0 < budget_s:
        T.raft_forward(p, i1, i2, iters=args.iters)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "image-pairs/s", "cores": threads, "kind": "port",
            "sample": f"{n} pair(s) {args.height}x{args.width} (padded to {i1.shape[2]}x{i1.shape[3]}), "
                      f"iters={args.iters}, oracle/torch_cpu.py (the reference's torch CPU ops; reference "
                      f"core/ measured 0.227 vs 0.226 pairs/s for this restatement at 8 threads in the build "
                      f"container), torch.set_num_threads({threads}), {dt:.1f} s"}


def spawn_ranks(n):
    """`bench.py --gpus N` (N > 1) without a launcher: start N rank processes of this script, rank r on
    cuda:r (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, as torch.distributed.run
    sets them), and exit with the worst of their exit codes.  This process never touches the GPU
    (torch.cuda.device_count() does not initialise it on this image): the ranks are children, not an
    exec.  Rank 0 prints the JSON line on the inherited stdout.  A failed rank stops the others."""
    import socket
    import subprocess
    rehearse = os.environ.get("RAFT_BENCH_REHEARSE_1GPU") == "1"
    visible = torch.cuda.device_count()
    if not rehearse and n > visible:
        raise SystemExit(f"bench.py: --gpus {n} but only {visible} GPU(s) are visible")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # the exact child PIDs this process started
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 1


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
    ap.add_argument("--precision", choices=["fp32", "f16x3", "f16", "bf16"], default=None,
                    help="conv arithmetic (default: the RAFT default, f16x3)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(--nproc-per-node {args.gpus}) or drop --gpus")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box (tests / development only): every rank on
    # cuda:0 over gloo (RCCL, like NCCL, refuses two ranks on one device)
    rehearse = os.environ.get("RAFT_BENCH_REHEARSE_1GPU") == "1"
    if not rehearse and local_rank >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs cuda:{local_rank}, only {torch.cuda.device_count()} visible")
    dev_index = 0 if rehearse else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
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
    if rank != 0:  # the per-kernel figures and the JSON line are rank 0's
        dist.destroy_process_group()
        return

    # ---- per-kernel live timing (HIP events on the launch stream, hipGraph replays) ----------
    from raft_optical_flow_amd import kernels as K
    h8, w8 = H // 8, W // 8
    P = args.batch * h8 * w8
    pu = plan.pk.update
    roof, lookup_b1 = None, None
    if not args.alternate_corr:
        # 16 pyramids: 16 x 28 MB of windows per rotation at B=1 (> the 256 MiB Infinity Cache)
        lookup_b1 = rotated_lookup(plan, args.batch, h8, w8, nrot=max(3, -(-16 // args.batch)), reps=4)
        pmc, _ = load_pmc("lookup_pmc.json", "corr_pyramid.hip")
        # the committed PMC pass is of config 2 (B=1, 440x1024) on the current kernel source
        lookup_b1["traffic"] = (pmc["hbm_bytes_per_launch"] if pmc and [args.batch, H, W] == pmc["shape_bhw"]
                                else None)
        names = [getattr(l, "name", "") for l in plan.launches]
        L_, r_ = plan.pk.levels, plan.pk.radius
        if "raft_corr_lookup_conv" in names:
            us, n = inforward_launch_us(plan, "raft_corr_lookup_conv")
            alg = P * fused_lookup_bytes_per_pixel(L_, r_, pu.convc1.n, pu.convf1.n)
            kname = "lookup_conv_kernel (raft_corr_lookup_conv: window lookup + convc1 + convf1, one launch)"
            src = "lookup_conv.hip"
        else:
            lname = "raft_corr_lookup_convf1" if "raft_corr_lookup_convf1" in names else "raft_corr_lookup"
            us, n = inforward_launch_us(plan, lname)
            alg = P * lookup_bytes_per_pixel(L_, r_)
            kname = f"corr_lookup_kernel ({lname})"
            src = "corr_pyramid.hip"
        roof = {"kernel": kname, "batch": args.batch, "bound": "hbm", "achieved": round(alg / us / 1e3, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / us / 1e3 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": alg, "launch_us": round(us, 2),
                "timing": f"HIP event pairs around each of the {n} launches of an eagerly enqueued forward (queued "
                          f"behind a spin so the GPU runs them back to back)"}
        fpmc, fname = load_pmc("lookup_conv_pmc.json" if src == "lookup_conv.hip" else "lookup_pmc.json", src)
        roof["traffic"] = (fpmc["hbm_bytes_per_launch"] if fpmc and [args.batch, H, W] == fpmc["shape_bhw"]
                           else None)
        if roof["traffic"] is not None:
            roof["traffic_source"] = f"profiles/{fname} (in-forward FETCH_SIZE/WRITE_SIZE)"
    else:
        # alternate corr: FP32 VALU-bound, 2*P*L*(2r+2)^2*C flops over the L per-level launches
        nl = plan.pk.levels
        lk = [l for l in plan.launches[plan.loop_start:plan.loop_end]
              if getattr(l, "name", None) in ("raft_alt_corr_lookup_levels", "raft_alt_corr_lookup_levels_prec")]
        t_it = time_kernel_events(lambda: lk[0](K.stream_handle()), 20)
        fl = alt_lookup_flops(P, nl, plan.pk.radius, plan.pk.fdim)
        # RAFT (r = 4, C = 256) runs the MFMA tile kernel (csrc/alt_corr.hip, f16x3 box GEMM) unless
        # RAFT_ALT_MFMA=0 selects the fp32 VALU tile kernel; the peak is that arithmetic's
        mfma = os.environ.get("RAFT_ALT_MFMA", "1") != "0" and plan.pk.radius == 4 and plan.pk.fdim % 32 == 0 \
            and plan.pk.fdim <= 256
        kname, bound, pk_tf = (("alt_corr_mfma_kernel<4>", "mfma (f16x3 box GEMM)", CONV_PEAK_TF["f16x3"]) if mfma
                               else ("alt_corr_tile_kernel<4>", "valu", FP32_MFMA_PEAK_TF))
        roof = {"kernel": f"{kname} (raft_alt_corr_lookup_levels: {nl} levels, one launch per iteration)",
                "bound": bound,
                "achieved": round(fl / t_it / 1e12, 2), "peak": round(pk_tf, 1), "unit": "TFLOP/s",
                "frac": round(fl / t_it / 1e12 / pk_tf, 4), "traffic": None,
                "algorithmic_flops_per_iteration": fl, "iteration_us": round(t_it * 1e6, 2),
                "timing": "HIP events around a hipGraph replay of the last iteration's lookups (final coords)"}

    # the >= 50 % lookup target is quoted at B = 8: 3 rotating B=8 pyramids (6.6 GB)
    lookup_b8 = None
    if not args.alternate_corr and args.batch < 8:
        lookup_b8 = rotated_lookup(plan, 8, h8, w8, nrot=3, reps=8)

    # the update block's main-stream convolutions of one (non-final) iteration, replayed as a graph
    # (their operands are L2 / MALL-resident in the forward as well: 7 MB activations, <= 2 MB weights)
    lk_idx = [i for i, l in enumerate(plan.launches) if getattr(l, "name", "") in
              ("raft_corr_lookup", "raft_corr_lookup_convf1", "raft_corr_lookup_conv", "raft_alt_corr_lookup_levels",
               "raft_alt_corr_lookup_levels_prec")]
    per_it = len(lk_idx) // args.iters
    # one whole (non-final) iteration: its lookup launch and every update launch up to the next lookup
    it_all = [l for l in plan.launches[lk_idx[per_it]:lk_idx[2 * per_it]] if not isinstance(l, str)]
    t_it = time_kernel_events(lambda: [l(K.stream_handle()) for l in it_all], 20)
    iteration = {"launches": len(it_all), "iteration_us": round(t_it * 1e6, 1),
                 "timing": "HIP events around a hipGraph of 20 replays of one iteration's launches"}
    if roof is not None and roof["kernel"].startswith("lookup_conv"):
        # the fused lookup's own duration in the iteration: the replayed iteration with and without
        # it (graph-replayed kernels run back to back, as rocprofv3 times a dispatch; an event pair
        # around one launch adds its own ~3-4 us)
        rest = [l for l in it_all if getattr(l, "name", "") != "raft_corr_lookup_conv"]
        lk = [l for l in it_all if getattr(l, "name", "") == "raft_corr_lookup_conv"][0]
        t_rest = time_kernel_events(lambda: [l(K.stream_handle()) for l in rest], 20)
        # the forward's own launch 32 times back to back in one graph (warm caches: a lower bound)
        b2b = time_kernel_events(lambda: [lk(K.stream_handle()) for _ in range(32)], 4) / 32 * 1e6
        roof["event_pair_us"] = roof["launch_us"]
        roof["iteration_delta_us"] = round((t_it - t_rest) * 1e6, 2)
        roof["back_to_back_us"] = round(b2b, 2)
        # the figure: the launch's per-dispatch time inside the graph-replayed forward (event-record
        # nodes around its 32 dispatches), as rocprofv3's in-forward mean reports it; without event
        # capture the iteration delta (also in-forward, and the larger figure)
        ig = inforward_graph_us(plan, "raft_corr_lookup_conv")
        sp = inforward_span_us(plan)
        if sp:
            roof["inforward_span_us"] = round(sp[0], 2)
        us, how = ((ig[0], f"HIP event-record nodes around each of the {ig[1]} dispatches inside the captured forward "
                           f"graph, mean of the last replay") if ig else
                   (sp[0], f"device realtime span (first work-group start to last work-group end, stores completed) "
                           f"of each of the forward's {sp[1]} fused lookup launches, one eager forward enqueued behind a "
                           f"GPU spin so its kernels run back to back (raft_debug_launch_span)") if sp else
                   (roof["iteration_delta_us"], "one iteration's graph with minus without the launch"))
        roof["launch_us"] = round(us, 2)
        roof["achieved"] = round(roof["algorithmic_bytes_per_launch"] / us / 1e3, 1)
        roof["frac"] = round(roof["achieved"] / HBM_PEAK_GBS, 4)
        roof["limiter"] = ("per-CU L2 ingest + latency (one 2x16-pixel work-group per CU streams the whole 360 KB split "
                           "convc1 weight; PMC: profiles/*lookup_conv_pmc.json): priced against the HBM roofline its "
                           "algorithmic bytes define")
        roof["timing"] = (how + "; event_pair_us: HIP event pairs around each launch of an eager forward; "
                          "iteration_delta_us: one iteration's graph with minus without the launch; back_to_back_us: "
                          "32 back-to-back replays of the forward's own launch (warm caches)")
    it_convs = [plan.launches[i] for i in range(lk_idx[per_it] + 1, lk_idx[2 * per_it])
                if getattr(plan.launches[i], "name", "") in ("raft_conv2d", "raft_conv2d_pair", "raft_conv2d_chain")
                and not plan.launches[i].side]
    t_upd = time_kernel_events(lambda: [l(K.stream_handle()) for l in it_convs], 20)
    fl = P * sum(2 * c.n * c.kh * c.kw * (c.in0_c + c.in1_c) for l in it_convs for c in launch_convs(l))
    peak = CONV_PEAK_TF[prec]
    update_roof = {"kernel": f"raft_conv2d (update block, one iteration, {prec}; main-stream convs)", "bound": "mfma",
                   "achieved": round(fl / t_upd / 1e12, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                   "frac": round(fl / t_upd / 1e12 / peak, 4), "convs_us": round(t_upd * 1e6, 1),
                   "flops_per_iteration": fl,
                   "timing": "HIP events around a hipGraph of 20 replays of one iteration's conv launches"}

    # the dominant kernel of the step: conv_halo_kernel<3,3,64> (the update block's 3x3 launches with
    # N-tile 64 at B=1: the convc2 | convf2 pair and the flow head's conv1), flops 2*M*N*K per conv
    dom = [l for l in it_convs
           if all(c.kh == 3 and c.kw == 3 and c.n > 4 and c.precision != 0 for c in launch_convs(l))
           and halo_bn([c.n for c in launch_convs(l)], args.batch, h8, w8) == 64]
    chained = [l for l in it_convs if l.name == "raft_conv2d_chain"]
    dominant = None
    if chained:
        # the chained launch (conv_chain_kernel): every update conv from convc2|convf2 to the flow
        # head's conv1 in one persistent launch, flops 2*M*N*K per conv
        cfl = sum(2 * P * c.n * c.kh * c.kw * (c.in0_c + c.in1_c) for l in chained for c in launch_convs(l))
        dt = time_kernel_events(lambda: [l(K.stream_handle()) for l in chained], 50)
        dominant = {"kernel": "conv_chain_kernel<f16x3> (raft_conv2d_chain: convc2|convf2, conv, z|r1, q1, z|r2, q2, "
                              "flow-head conv1 of one iteration, one launch)",
                    "bound": "mfma", "achieved": round(cfl / dt / 1e12, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(cfl / dt / 1e12 / peak, 4), "launches": len(chained),
                    "launch_us": round(dt / len(chained) * 1e6, 2), "flops_per_launch": cfl // len(chained),
                    "timing": "HIP events around a hipGraph of 50 replays of that launch"}
    elif dom:
        dfl = sum(2 * P * c.n * 9 * (c.in0_c + c.in1_c) for l in dom for c in launch_convs(l))
        dt = time_kernel_events(lambda: [l(K.stream_handle()) for l in dom], 50)
        dominant = {"kernel": "conv_halo_kernel<3,3,64> (the convc2 | convf2 pair and the flow-head conv1 of one "
                              "iteration)",
                    "bound": "mfma", "achieved": round(dfl / dt / 1e12, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(dfl / dt / 1e12 / peak, 4), "launches": len(dom),
                    "launch_us": round(dt / len(dom) * 1e6, 2), "flops_per_launch": dfl // len(dom),
                    "timing": "HIP events around a hipGraph of 50 replays of those launches"}
        hpmc, hname = load_pmc("halo_pmc.json", "conv_halo.hip")
        if hpmc:
            # the one-tile f16x3 3x3 N-64 instantiation, whatever its trailing template arguments (tile
            # rows, multi-tile flag, loader waves): the entry with the most dispatches
            keys = [k for k in hpmc if k.startswith("conv_halo_kernel<3, 3, 64, 1, false, 8")
                    or k == "conv_halo_kernel<3, 3, 64, 1, false>"]
            ent = max((hpmc[k] for k in keys), key=lambda e: e.get("dispatches", 0), default={})
            dominant["mfma_busy"] = ent.get("mfma_busy")
            dominant["mfma_busy_source"] = f"profiles/{hname}"

    # the drop-in path itself: RAFT.forward() as demo.py / evaluate.py call it (core/raft.py:145-251;
    # demo.py:58-67), on the same padded pool pairs, with the default range guard (one host-side flag
    # read per forward) and the plan's hipGraph replay
    drop_in = None
    if world == 1:
        def fwd(k):
            with torch.no_grad():
                return model(*pool[k % len(pool)], iters=args.iters, test_mode=True)
        for k in range(max(1, args.warmup)):
            fwd(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            fwd(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        drop_in = {"value": round(args.batch * args.steps / dt, 3), "ms_per_step": round(dt / args.steps * 1e3, 3),
                   "range_guard": model.range_guard,
                   "timing": f"{args.steps} RAFT.forward(image1, image2, iters={args.iters}, test_mode=True) calls "
                             f"back to back (torch.no_grad), wall clock between two synchronizes; each forward "
                             f"replays the plan's graph and reads its range-guard flag on the host"}

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
            "lookup_b1": lookup_b1,
            "lookup_b8": lookup_b8,
            "iteration": iteration,
            "update_gemm": update_roof,
            "dominant_kernel": dominant,
            "drop_in_forward": drop_in,
            "fp32_exact": exact,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
