"""Frame-pair sharding on the GPU.

* Two ranks (gloo collectives, both on cuda:0 of the one-GPU box) each run their shard of a
  batch through the HIP forward; the gathered flows must equal the unsharded batch's.  The
  weights reach rank 1 only through `broadcast_state_dict`, which moves the model's DEVICE
  tensors (rank 1 starts from different random weights).
* One rank over RCCL ("nccl", device_id=cuda:0): the bench's N>1 code path on the device —
  process-group init with device_id, broadcast_state_dict and gather_flows of device tensors,
  barrier and the max-over-ranks timing all_reduce."""
import argparse
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_PAIRS, H, W, ITERS = 4, 128, 192, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from raft_optical_flow_amd import RAFT
        from raft_optical_flow_amd.dist import broadcast_state_dict, gather_flows, shard_indices
        from raft_optical_flow_amd.init import seeded_state_dict, smooth_images
        torch.manual_seed(100 + rank)
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        if rank == 0:
            m.load_state_dict(seeded_state_dict(m, 0))
        m = m.cuda().eval()
        nbytes = broadcast_state_dict(m, src=0)  # the model's device tensors (gloo broadcasts CUDA tensors)
        assert nbytes > 20e6 and next(m.parameters()).is_cuda
        i1, i2 = smooth_images(N_PAIRS, H, W, seed=3)
        mine = shard_indices(N_PAIRS, rank, world)
        with torch.no_grad():
            _, up = m(i1[mine].cuda(), i2[mine].cuda(), iters=ITERS, test_mode=True)
        got = gather_flows(up.cpu(), dst=0)
        if rank == 0:
            with torch.no_grad():
                _, full = m(i1.cuda(), i2.cuda(), iters=ITERS, test_mode=True)
            full = full.cpu()
            err = 0.0
            for r, part in enumerate(got):
                for j, i in enumerate(shard_indices(N_PAIRS, r, world)):
                    err = max(err, float((part[j] - full[i]).abs().max()))
            q.put((rank, err, float(full.abs().max())))
        else:
            q.put((rank, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_batch_equals_unsharded_world2():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, err, peak = res[0]
    print(f"sharded vs unsharded (2 ranks, {N_PAIRS} pairs {H}x{W}): max |diff| {err:.2e}, max |flow| {peak:.2f}")
    assert peak > 0.1 and err < 1e-3, (err, peak)


def _nccl_worker(port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from raft_optical_flow_amd import RAFT
        from raft_optical_flow_amd.dist import broadcast_state_dict, gather_flows
        from raft_optical_flow_amd.init import seeded_state_dict, smooth_images
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        sd = seeded_state_dict(m, 0)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        nbytes = broadcast_state_dict(m, src=0)
        same = all(torch.equal(v.cpu(), sd[k]) for k, v in m.state_dict().items())
        i1, i2 = smooth_images(2, H, W, seed=3)
        with torch.no_grad():
            _, up = m(i1.to(dev), i2.to(dev), iters=ITERS, test_mode=True)
        got = gather_flows(up, dst=0)
        dist.barrier()
        tt = torch.tensor([1.5], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        q.put((nbytes, same, len(got), bool(got[0].is_cuda), float((got[0] - up).abs().max()), float(tt.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world1_broadcast_and_gather_on_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    nbytes, same, n, on_dev, err, tmax = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    print(f"RCCL world 1: broadcast {nbytes / 1e6:.1f} MB, gather on device {on_dev}")
    assert nbytes > 20e6 and same
    assert n == 1 and on_dev and err == 0.0 and tmax == 1.5


@pytest.mark.timeout(300)
def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` as the driver invokes it (no launcher): the script spawns the two ranks
    itself (here in the one-GPU rehearsal mode, RAFT_BENCH_REHEARSE_1GPU=1: both on cuda:0, gloo), and
    rank 0's JSON line reports both GPUs' pairs."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RAFT_BENCH_REHEARSE_1GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--height", "128", "--width", "192", "--iters", "4", "--no-cpu-baseline",
                        "--no-fp32-exact"], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2 and out["value"] > 0


@pytest.mark.timeout(300)
def test_dataparallel_forward_equals_unwrapped():
    """The reference's own multi-GPU API (nn.DataParallel, demo.py:45, train.py:172): DataParallel(RAFT)
    on the box's GPU gives the unwrapped forward's flow, and explicit replicas (what DataParallel makes
    per forward on >1 GPU) reuse the source's packed weights and plans across forwards and match it
    too, run from a worker thread as parallel_apply does."""
    import threading
    from torch.nn.parallel import replicate
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_state_dict, smooth_images
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    m.load_state_dict(seeded_state_dict(m, 0))
    m = m.cuda().eval()
    i1, i2 = smooth_images(2, H, W, seed=5)
    i1, i2 = i1.cuda(), i2.cuda()
    with torch.no_grad():
        ref_low, ref_up = m(i1, i2, iters=ITERS, test_mode=True)
        dp = torch.nn.DataParallel(m, device_ids=[0])
        low, up = dp(i1, i2, iters=ITERS, test_mode=True)
    assert torch.equal(low, ref_low) and torch.equal(up, ref_up)
    packed = m.packed(torch.device("cuda", 0))
    res, errs = [], []

    def run(rep):
        try:
            with torch.no_grad(), torch.cuda.device(0):
                res.append(rep(i1, i2, iters=ITERS, test_mode=True))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    for _ in range(2):  # two forwards, each with a fresh replica (as DataParallel does)
        rep = replicate(m, [0])[0]
        th = threading.Thread(target=run, args=(rep,))
        th.start()
        th.join()
        assert not errs, errs
        assert rep.packed(torch.device("cuda", 0)) is packed  # no re-pack per replica
    for lo, u in res:
        assert torch.equal(lo, ref_low) and torch.equal(u, ref_up)
