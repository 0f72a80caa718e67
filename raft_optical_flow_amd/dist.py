"""Multi-GPU frame-pair sharding (one process per GPU).

The reference's only parallelism is nn.DataParallel (`demo.py:45`,
`evaluate.py:179`, `train.py:172`): one process that re-broadcasts the weights
to every GPU and scatters/gathers on every forward.  Here each rank is its own
process (torch.distributed, backend "nccl" = RCCL over xGMI on ROCm):

  * the state_dict is flattened into ONE buffer and broadcast from rank 0 once
    (21 MB for RAFT-full) — no per-forward weight traffic;
  * frame pairs are independent, so pair i is processed by rank i mod world;
    there is no collective on the data path;
  * results can be gathered to rank 0 (gather_flows) or written per rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def broadcast_state_dict(model: torch.nn.Module, src: int = 0, group=None) -> int:
    """Broadcast every floating/integer tensor of model.state_dict() from `src`
    with one collective on a flat buffer.  Returns the number of bytes sent."""
    sd = model.state_dict()
    keys = [k for k, v in sd.items() if torch.is_tensor(v)]
    dev = next(model.parameters()).device
    flat_f = torch.cat([sd[k].detach().reshape(-1).to(dev, torch.float32) for k in keys
                        if sd[k].is_floating_point()]) if keys else torch.empty(0, device=dev)
    ints = [k for k in keys if not sd[k].is_floating_point()]
    flat_i = torch.cat([sd[k].detach().reshape(-1).to(dev, torch.int64) for k in ints]) if ints else None
    dist.broadcast(flat_f, src=src, group=group)
    if flat_i is not None:
        dist.broadcast(flat_i, src=src, group=group)
    off = 0
    offi = 0
    with torch.no_grad():
        for k in keys:
            t = sd[k]
            n = t.numel()
            if t.is_floating_point():
                t.copy_(flat_f[off:off + n].view_as(t).to(t.dtype))
                off += n
            else:
                t.copy_(flat_i[offi:offi + n].view_as(t).to(t.dtype))
                offi += n
    return flat_f.numel() * 4 + (flat_i.numel() * 8 if flat_i is not None else 0)


def shard_indices(n_items: int, rank: int, world: int):
    """Frame pairs owned by `rank`: i with i % world == rank."""
    return list(range(rank, n_items, world))


def gather_flows(flow: torch.Tensor, dst: int = 0, group=None):
    """Gather equally shaped per-rank flow batches to `dst` (list on dst, None elsewhere), on the
    flows' device with RCCL; gloo (no gather of device tensors) goes through host copies."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    via_host = flow.is_cuda and dist.get_backend(group) == "gloo"
    src = flow.detach().cpu() if via_host else flow.contiguous()
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == dst else None
    dist.gather(src.contiguous(), bufs, dst=dst, group=group)
    if bufs is not None and via_host:
        bufs = [b.to(flow.device) for b in bufs]
    return bufs
