"""Multi-GPU sharding and reassembly (one process per GPU, torch.distributed over RCCL/xGMI).

Every `encode(line)` of the reference is independent (tokenizer.py:167-193), so a batch shards
by document: each rank encodes a contiguous, byte-balanced range of rows with no data-path
collective. When the caller wants the whole batch's id streams on every rank, `gather_ids`
reassembles them with one all-gather of the per-rank sizes and exact-size broadcasts of each
rank's slice straight into the final buffers. Works with the "nccl" (RCCL)
backend on device tensors and with "gloo" on CPU tensors (tests).
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


def gather_ids(ids, out_offs, group=None, out=None):
    """All-gather per-rank (ids, row offsets) into the whole batch's, in rank order.

    ids: int32 [n_ids]; out_offs: int64 [n_rows + 1] with out_offs[0] == 0. Returns
    (all_ids int32, all_offs int64) identical on every rank.

    One all-gather of the per-rank sizes (16 bytes each), then every rank's exact-size slices
    travel straight into the final buffers: each rank writes its own ids and its offsets rebased by
    the ids before it into its slice of the result (its only device copy), and broadcasts that
    slice to the others, which receive into theirs (one broadcast per source rank, all in flight
    together; no padding, no compaction, no concatenation). `out` = (all_ids, all_offs) preallocated
    by the caller may be passed; if `ids` already is this rank's slice of out[0], it is not copied.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ids.device
    sizes = torch.tensor([ids.numel(), out_offs.numel() - 1], dtype=torch.int64, device=dev)
    all_sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(all_sizes, sizes, group=group)
    sz = all_sizes.view(world, 2).cpu().tolist()
    tot_ids = sum(x[0] for x in sz)
    tot_rows = sum(x[1] for x in sz)
    if out is None:
        all_ids = torch.empty(tot_ids, dtype=ids.dtype, device=dev)
        all_offs = torch.empty(tot_rows + 1, dtype=torch.int64, device=dev)
    else:
        all_ids, all_offs = out
        if all_ids.numel() < tot_ids or all_offs.numel() < tot_rows + 1:
            raise ValueError("gather_ids: out buffers hold %d ids / %d offsets, %d / %d needed"
                             % (all_ids.numel(), all_offs.numel(), tot_ids, tot_rows + 1))
    all_offs[0] = 0
    ib = [0] * (world + 1)
    rb = [0] * (world + 1)
    for r in range(world):
        ib[r + 1] = ib[r] + sz[r][0]
        rb[r + 1] = rb[r] + sz[r][1]
    mine_ids = all_ids[ib[rank]:ib[rank + 1]]
    mine_offs = all_offs[rb[rank] + 1:rb[rank + 1] + 1]
    if sz[rank][0] and mine_ids.data_ptr() != ids.data_ptr():
        mine_ids.copy_(ids)
    if sz[rank][1]:
        torch.add(out_offs[1:], ib[rank], out=mine_offs)
    work = []
    for r in range(world):
        if sz[r][0]:
            work.append(dist.broadcast(all_ids[ib[r]:ib[r + 1]], src=dist.get_global_rank(group, r) if group else r,
                                       group=group, async_op=True))
        if sz[r][1]:
            work.append(dist.broadcast(all_offs[rb[r] + 1:rb[r + 1] + 1],
                                       src=dist.get_global_rank(group, r) if group else r, group=group, async_op=True))
    for w in work:
        w.wait()
    return all_ids[:tot_ids], all_offs[:tot_rows + 1]
