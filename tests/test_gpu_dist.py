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
