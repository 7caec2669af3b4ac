"""Multi-process sharding + reassembly on CPU (gloo, world_size 2): the N > 1 path of bench.py
and akshar_amd.dist, checked against the single-process result (oracle ids)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from akshar_amd import dist as adist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from akshar_amd import synth
        from akshar_amd.models import BPEModel
        from oracle import oracle as O
        from tests.conftest import BPE_PATH
        buf, offs = synth.generate(synth.KIND_HINGLISH, 3000, seed=5)
        r0, r1 = adist.shard_rows(offs.astype(np.int64), world, rank)
        sub_offs = (offs[r0:r1 + 1] - offs[r0]).astype(np.uint64)
        sub = buf[int(offs[r0]):int(offs[r1])]
        ids, oo = O.OracleBPE(BPEModel(BPE_PATH)).encode_batch(sub if len(sub) else np.zeros(1, np.uint8), sub_offs)
        all_ids, all_offs = adist.gather_ids(torch.from_numpy(ids.astype(np.int32)),
                                             torch.from_numpy(oo.astype(np.int64)))
        # the same gather with the ids crossing as int16 (the 24k vocabulary fits): identical result
        n_ids, n_offs = adist.gather_ids(torch.from_numpy(ids.astype(np.int32)),
                                         torch.from_numpy(oo.astype(np.int64)), id_bound=32768)
        assert torch.equal(n_ids, all_ids) and torch.equal(n_offs, all_offs)
        q.put((rank, r0, r1, all_ids.numpy(), all_offs.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_rows_balanced_and_complete():
    offs = np.cumsum([0] + [10, 200, 5, 5, 5, 300, 1, 1, 1, 1]).astype(np.int64)
    for world in (1, 2, 3, 4, 8):
        cuts = [adist.shard_rows(offs, world, r) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(offs) - 1
        assert all(a[1] == b[0] for a, b in zip(cuts, cuts[1:]))


def test_gloo_world2_gather_matches_single_process():
    from akshar_amd import synth
    from akshar_amd.models import BPEModel
    from oracle import oracle as O
    from tests.conftest import BPE_PATH
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, offs = synth.generate(synth.KIND_HINGLISH, 3000, seed=5)
    ref_ids, ref_offs = O.OracleBPE(BPEModel(BPE_PATH)).encode_batch(buf, offs)
    res.sort()
    assert res[0][2] == res[1][1] and 0 < res[0][2] < 3000
    for _, _, _, ids, oo in res:
        assert np.array_equal(ids.astype(np.uint32), ref_ids)
        assert np.array_equal(oo.astype(np.uint64), ref_offs)


def _hip_worker(rank, world, port, kind, q):
    """One rank: its byte-balanced shard of a fixed batch through the HIP engine on cuda:0, then the
    all-gather that reassembles the id streams (gloo on CPU tensors here; RCCL on the GPU node)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from akshar_amd import engine, synth
        from tests.conftest import BPE_PATH, SPM_PATH
        buf, offs = synth.generate(synth.KIND_HINGLISH, 20000, seed=11)
        r0, r1 = adist.shard_rows(offs.astype(np.int64), world, rank)
        sub_offs = (offs[r0:r1 + 1] - offs[r0]).astype(np.int64)
        sub = buf[int(offs[r0]):int(offs[r1])]
        pad = np.zeros(((len(sub) + 15) // 16) * 16 + 16, dtype=np.uint8)
        pad[:len(sub)] = sub
        gb, go = engine.to_device(pad, sub_offs, dev=0)
        model = engine.SPM(SPM_PATH, dev=0) if kind == "spm" else engine.BPE(BPE_PATH, dev=0)
        ids, oo = model.encode_batch(gb, go)
        all_ids, all_offs = adist.gather_ids(ids.cpu(), oo.cpu())
        q.put((rank, r0, r1, all_ids.numpy(), all_offs.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["spm", "bpe"])
def test_gloo_world2_hip_shards_match_oracle(kind):
    """Config 5's data path at world size 2: both ranks run the HIP engine on their shard_rows shard
    (cuda:0), gather_ids reassembles, and every rank holds the oracle's ids for the whole batch."""
    from akshar_amd import synth
    from akshar_amd.models import BPEModel, SPMModel
    from oracle import oracle as O
    from tests.conftest import BPE_PATH, SPM_PATH
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hip_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buf, offs = synth.generate(synth.KIND_HINGLISH, 20000, seed=11)
    oracle = O.OracleSPM(SPMModel(SPM_PATH)) if kind == "spm" else O.OracleBPE(BPEModel(BPE_PATH))
    ref_ids, ref_offs = oracle.encode_batch(buf, offs)
    res.sort()
    assert res[0][2] == res[1][1] and 0 < res[0][2] < 20000
    for _, _, _, ids, oo in res:
        assert np.array_equal(ids.astype(np.uint32), ref_ids)
        assert np.array_equal(oo.astype(np.uint64), ref_offs)


def _nccl_worker(port, q):
    """world size 1 over the nccl (= RCCL) backend on cuda:0: librccl loads, both all-gathers of
    gather_ids run on device tensors, and the reassembled streams equal the rank's own."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from akshar_amd import engine, synth
        from tests.conftest import SPM_PATH
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            assert dist.get_backend() == "nccl"
            buf, offs = synth.generate(synth.KIND_HINGLISH, 50000, seed=13)
            pad = np.zeros(((len(buf) + 15) // 16) * 16 + 16, dtype=np.uint8)
            pad[:len(buf)] = buf
            gb, go = engine.to_device(pad, offs.astype(np.int64), dev=0)
            ids, oo = engine.SPM(SPM_PATH, dev=0).encode_batch(gb, go)
            all_ids, all_offs = adist.gather_ids(ids, oo)
            n_ids, n_offs = adist.gather_ids(ids, oo, id_bound=32768)  # int16 on the wire
            torch.cuda.synchronize()
            ok = all_ids.is_cuda and torch.equal(all_ids, ids) and torch.equal(all_offs, oo)
            ok = ok and torch.equal(n_ids, ids) and torch.equal(n_offs, oo)
            q.put(("ok" if ok else "mismatch", int(all_ids.numel())))
        finally:
            dist.destroy_process_group()
    except Exception as e:  # reported to the parent, which fails the test with it
        q.put(("error", repr(e)))


@pytest.mark.gpu
def test_nccl_world1_gather_ids_on_device():
    """The RCCL code path of bench.py --workload cfg5 / gather_ids, in a child process (the
    process group never touches the pytest process)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "ok", res
    assert p.exitcode == 0 and res[1] > 50000


def _edge_worker(rank, world, port, q):
    """Uneven shards: rank 1 holds no rows at all; rank 2 passes preallocated out buffers."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = {0: [[5, 6, 7], [8]], 1: [], 2: [[9, 10], [], [11, 12, 13, 14]]}[rank]
        ids = torch.tensor([x for r in rows for x in r], dtype=torch.int32)
        offs = torch.tensor(np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64))
        out = None
        if rank == 2:
            out = (torch.full((20,), -1, dtype=torch.int32), torch.full((10,), -1, dtype=torch.int64))
        all_ids, all_offs = adist.gather_ids(ids, offs, out=out)
        n_ids, n_offs = adist.gather_ids(ids, offs, id_bound=32768)  # int16 on the wire (odd counts)
        assert n_ids.tolist() == all_ids.tolist() and n_offs.tolist() == all_offs.tolist()
        q.put((rank, all_ids.tolist(), all_offs.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_gather_uneven_and_empty_shards():
    """gather_ids with an empty rank and a caller-provided output: every rank gets the whole batch's
    ids in rank order and offsets rebased across ranks (one size all-gather + one all-gather of the
    padded per-rank records), with the ids as int32 and as int16 on the wire."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_edge_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, ids, offs in res:
        assert ids == [5, 6, 7, 8, 9, 10, 11, 12, 13, 14]
        assert offs == [0, 3, 4, 6, 6, 10]
