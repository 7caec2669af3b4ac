"""Multi-GPU sharding and reassembly (one process per GPU, torch.distributed over RCCL/xGMI).

Every `encode(line)` of the reference is independent (tokenizer.py:167-193), so a batch shards
by document: each rank encodes a contiguous, byte-balanced range of rows with no data-path
collective. When the caller wants the whole batch's id streams on every rank, `gather_ids`
reassembles them with one all-gather of the per-rank sizes and ONE all-gather of the per-rank
(offsets | ids) records padded to the largest shard. Works with the "nccl" (RCCL)
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


def gather_ids(ids, out_offs, group=None, out=None, id_bound=None):
    """All-gather per-rank (ids, row offsets) into the whole batch's, in rank order.

    ids: int32 [n_ids]; out_offs: int64 [n_rows + 1] with out_offs[0] == 0. Returns
    (all_ids int32, all_offs int64) identical on every rank. id_bound: every id is below it (the
    model's vocabulary size); at most 32,768, the ids cross the links as int16 (half the bytes;
    the values are unchanged).

    Two collectives per call, whatever the world size:
      1. all_gather_into_tensor of the per-rank sizes (16 bytes each);
      2. ONE all_gather_into_tensor of a fixed-size record per rank, padded to the largest shard:
         [its row offsets rebased by the ids of the ranks before it (int64, as int32 pairs) |
          its ids (int32, or int16 pairs)]. Shards are byte-balanced (shard_rows), so the padding
         is small.
    The records are then copied into the final buffers, one slice per rank (`out` = (all_ids,
    all_offs) preallocated by the caller receives them in place; an int16 record widens in that
    copy). With RCCL over xGMI the data all-gather is one ring / direct collective on every link at
    once; per-rank broadcasts would serialise on the communicator's stream.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = ids.device
    narrow = id_bound is not None and 0 < id_bound <= 32768 and ids.dtype == torch.int32
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
    for r in range(world):
        ib[r + 1] = ib[r] + sz[r][0]
    max_ids = max(x[0] for x in sz)
    max_rows = max(x[1] for x in sz)
    # int32 words per rank record: offsets first, and an even length, so every record's offsets
    # are 8-byte aligned and read as int64 in place
    id_words = (max_ids + 1) // 2 if narrow else max_ids
    rec = 2 * max_rows + id_words + (id_words & 1)
    if rec == 0:
        return all_ids[:0], all_offs[:1]
    mine = torch.empty(rec, dtype=torch.int32, device=dev)
    n_ids, n_rows = sz[rank]
    if n_rows:
        torch.add(out_offs[1:], ib[rank], out=mine[:2 * max_rows].view(torch.int64)[:n_rows])
    body = mine[2 * max_rows:].view(torch.int16) if narrow else mine[2 * max_rows:]
    if n_ids:
        body[:n_ids].copy_(ids.view(torch.int32))
    gathered = torch.empty(world * rec, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(gathered, mine, group=group)
    g = gathered.view(world, rec)
    g_offs = g[:, :2 * max_rows].view(torch.int64)
    g_ids = g[:, 2 * max_rows:]
    if narrow:
        g_ids = g_ids.view(torch.int16)  # (the last dimension is contiguous)
    flat_ids = all_ids.view(torch.int32)
    rb = 0
    for r in range(world):
        if sz[r][1]:
            all_offs[1 + rb:1 + rb + sz[r][1]].copy_(g_offs[r, :sz[r][1]])
        if sz[r][0]:
            flat_ids[ib[r]:ib[r + 1]].copy_(g_ids[r, :sz[r][0]])
        rb += sz[r][1]
    return all_ids[:tot_ids], all_offs[:tot_rows + 1]
