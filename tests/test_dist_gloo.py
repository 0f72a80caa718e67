"""Multi-process (world_size 2, gloo, CPU) tests of the frame-pair sharding path:
one flat-buffer weight broadcast from rank 0, disjoint pair shards, flow gather."""
import argparse
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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
        from raft_optical_flow_amd.init import seeded_state_dict
        torch.manual_seed(100 + rank)  # ranks start with different random weights
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        if rank == 0:
            m.load_state_dict(seeded_state_dict(m, 0))
        nbytes = broadcast_state_dict(m, src=0)
        ref = seeded_state_dict(m, 0)
        same = all(torch.equal(m.state_dict()[k], ref[k]) for k in ref)
        shard = shard_indices(10, rank, world)
        flow = torch.full((1, 2, 3, 4), float(rank))
        got = gather_flows(flow, dst=0)
        gathered = None if got is None else [float(t[0, 0, 0, 0]) for t in got]
        q.put((rank, same, nbytes, shard, gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_broadcast_shard_gather_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, same0, nb0, sh0, g0), (r1, same1, nb1, sh1, g1) = res
    assert same0 and same1, "weights differ after the broadcast"
    assert nb0 == nb1 and nb0 >= 5_257_536 * 4  # one flat fp32 buffer (+ int64 counters)
    assert sh0 == [0, 2, 4, 6, 8] and sh1 == [1, 3, 5, 7, 9]
    assert g0 == [0.0, 1.0] and g1 is None
