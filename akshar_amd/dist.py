"""Multi-GPU sharding and reassembly (one process per GPU, torch.distributed over RCCL/xGMI).

Every `encode(line)` of the reference is independent (tokenizer.py:167-193), so a batch shards
by document: each rank encodes a contiguous, byte-balanced range of rows with no data-path
collective. When the caller wants the whole batch's id streams on every rank, `gather_ids`
reassembles them with one all-gather of the per-rank sizes and one all-gather of the padded id
buffers. Works with the "nccl" (RCCL) backend on device tensors and with "gloo"
on CPU tensors (tests).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_rows(offs, world, rank):
    """Row range [r0, r1) of `rank`: contiguous rows, balanced by byte count.

    offs: int64 row offsets (numpy or torch, n+1 entries). Rank k takes the rows whose start
    byte falls in [k*B/world, (k+1)*B/world).
    """
    o = offs.cpu().numpy() if isinstance(offs, torch.Tensor) else np.asarray(offs)
    n = len(o) - 1
    total = int(o[-1])
    if total == 0:
        cuts = [n * k // world for k in range(world + 1)]
    else:
        targets = [total * k // world for k in range(world + 1)]
        cuts = [int(np.searchsorted(o[:-1], t, side="left")) for t in targets]
        cuts[0], cuts[-1] = 0, n
    return cuts[rank], cuts[rank + 1]


def gather_ids(ids, out_offs, group=None):
    """All-gather per-rank (ids, row offsets) into the whole batch's, in rank order.

    ids: int32 [n_ids]; out_offs: int64 [n_rows + 1] with out_offs[0] == 0. Returns
    (all_ids int32, all_offs int64) identical on every rank.
    """
    world = dist.get_world_size(group)
    dev = ids.device
    sizes = torch.tensor([ids.numel(), out_offs.numel() - 1], dtype=torch.int64, device=dev)
    all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_sizes, sizes, group=group)
    all_sizes = all_sizes.view(world, 2).cpu()
    max_ids = int(all_sizes[:, 0].max())
    max_rows = int(all_sizes[:, 1].max())
    pid = torch.zeros(max(max_ids, 1), dtype=ids.dtype, device=dev)
    pid[:ids.numel()] = ids
    poff = torch.zeros(max_rows + 1, dtype=torch.int64, device=dev)
    poff[:out_offs.numel()] = out_offs
    gid = torch.empty(world * pid.numel(), dtype=ids.dtype, device=dev)
    goff = torch.empty(world * poff.numel(), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(gid, pid, group=group)
    dist.all_gather_into_tensor(goff, poff, group=group)
    gid = gid.view(world, -1)
    goff = goff.view(world, -1)
    parts, offs = [], [torch.zeros(1, dtype=torch.int64, device=dev)]
    base = 0
    for r in range(world):
        ni, nr = int(all_sizes[r, 0]), int(all_sizes[r, 1])
        parts.append(gid[r, :ni])
        offs.append(goff[r, 1:nr + 1] + base)
        base += ni
    return torch.cat(parts), torch.cat(offs)
