#!/usr/bin/env python3
"""Benchmark: the reference's encode hot path on MI355X (BASELINE.json metric).

Workload: 10 M synthetic Hinglish sentences per GPU, encoded end to end
exactly as `aksharTokenizer(model_path="models/akshar.json", model_type="bpe").encode(line)`
(tokenizer.py:167-193): normalize_text (NFC, roman lowercasing, allowlist, elongation collapse)
-> HF NFKC -> Whitespace pre-tokenizer -> 24k BPE merges -> <s> ... </s>. Rows are packed UTF-8
+ int64 offsets already resident in HBM when timing starts; ids + row offsets are written back
to HBM. One step = one encode of the whole per-GPU batch.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R] [--gather]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N (one rank/GPU;
  each rank encodes its own 10 M-row shard: weak scaling, no data-path collective; --gather adds
  the RCCL all-gather that reassembles the id streams on every rank, timed separately).

Prints ONE JSON line (rank 0) with value = whole-job MB/s of raw UTF-8 input, tokens/s,
the dominant kernel's HBM roofline (HIP events around its launches on the encode stream) and
the CPU baseline (the oracle restatement, 1 thread, timed on a bounded sample on this host).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MB of raw UTF-8 tokenized/sec @1 GPU (+ tokens/s); bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 1234
TRAFFIC_FILE = "r01_v7_tiles_pmc.json"  # PMC HBM bytes of the tile kernel at the default config


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=10_000_000, help="rows per GPU (config 4: 10 M)")
    ap.add_argument("--gather", action="store_true", help="also all-gather the id streams (RCCL)")
    ap.add_argument("--cpu-rows", type=int, default=400_000, help="CPU baseline sample (rows)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-others", action="store_true", help="skip the config 2/3/5 side measurements")
    return ap.parse_args()


def log(rank, msg):
    """progress on stderr (the JSON line is the only stdout output)"""
    if rank == 0:
        print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


def cpu_baseline(args, buf, offs):
    """The oracle (plain C, one thread) on the first --cpu-rows rows of rank 0's shard."""
    from akshar_amd.models import BPEModel
    from oracle import oracle as O
    n = min(args.cpu_rows, len(offs) - 1)
    sub_offs = offs[:n + 1].astype(np.uint64)
    sub = buf[:int(sub_offs[-1])]
    ob = O.OracleBPE(BPEModel(os.path.join(ROOT, "models", "akshar.json")))
    t = time.perf_counter()
    ids, _ = ob.encode_batch(sub, sub_offs)
    dt = time.perf_counter() - t
    return {"value": round(len(sub) / 1e6 / dt, 3), "unit": "MB/s", "cores": 1, "kind": "port",
            "tokens_per_s": round(len(ids) / dt, 1),
            "sample": "first %d rows (%.1f MB) of the same synthetic Hinglish batch, oracle/akshar_oracle.c "
                      "or_bpe_encode single-threaded, %.1f s" % (n, len(sub) / 1e6, dt)}


def other_configs(dev, rows=1_000_000):
    """SURVEY.md §8 configs 2, 3 and 5 on this GPU (1 M synthetic rows each, inputs in HBM): the
    single-GPU rates of the other rows of the scope table, reported beside the headline line."""
    from akshar_amd import engine, synth

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps

    out = {}
    spm = engine.SPM(os.path.join(ROOT, "models", "akshar.model"), dev=dev)
    for kind, name in ((synth.KIND_DEVANAGARI, "devanagari"), (synth.KIND_HINGLISH, "hinglish")):
        buf, offs = synth.generate(kind, rows, seed=SEED + 7)
        pad = np.zeros(((len(buf) + 15) // 16) * 16 + 16, dtype=np.uint8)
        pad[:len(buf)] = buf
        gb, go = engine.to_device(pad, offs.astype(np.int64), dev=dev)
        mb = len(buf) / 1e6
        ops = {"segment": lambda: engine.segment_batch(gb, go, flags=3),
               "segment_raw": lambda: engine.segment_batch(gb, go, flags=engine.AK_RAW),
               "normalize": lambda: engine.normalize_batch(gb, go),
               "switches": lambda: engine.switches_batch(gb, go),
               "spm_encode": lambda: spm.encode_batch(gb, go),
               "analyze_fused": lambda: engine.analyze_batch(gb, go)}
        res = {k: round(mb / timed(f), 1) for k, f in ops.items()}
        res["rows"], res["mb"] = rows, round(mb, 1)
        out[name] = res
    d, h = out["devanagari"], out["hinglish"]
    t3 = sum(1.0 / h[k] for k in ("normalize", "switches", "segment"))
    return {"unit": "MB/s of raw UTF-8 (1 M synthetic rows, inputs in HBM, one-lane-per-row staged kernels)",
            "cfg2_segment_devanagari": d["segment"], "cfg2_segment_devanagari_raw": d["segment_raw"],
            "cfg3_normalize_switches_segment_hinglish": h["analyze_fused"],
            "cfg3_as_three_separate_ops": round(1.0 / t3, 1),
            "cfg5_spm_encode_hinglish_per_gpu": h["spm_encode"], "detail": out}


def main():
    args = parse()
    dist = args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1
    rank, world, local = 0, 1, 0
    if dist:
        import torch.distributed as tdist
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        backend = os.environ.get("AK_BENCH_BACKEND", "nccl")  # gloo: rehearse N ranks on one GPU
        if backend == "nccl":
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(torch.cuda.device_count(), 1)
            tdist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from akshar_amd import engine, synth
    rows = args.rows
    log(rank, "generating %d rows" % rows)
    buf, offs = synth.generate(synth.KIND_HINGLISH, rows, seed=SEED, first=rank * rows)
    log(rank, "generated %.1f MB" % (offs[-1] / 1e6))
    nbytes = int(offs[-1])
    pad = np.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:nbytes] = buf
    gbuf, goffs = engine.to_device(pad, offs.astype(np.int64), dev=local)
    bpe = engine.BPE(os.path.join(ROOT, "models", "akshar.json"), dev=local)
    cap = nbytes // 2 + 2 * rows + 1024
    torch.cuda.synchronize()

    def step():
        return bpe.encode_batch(gbuf, goffs, cap=cap, nbytes=nbytes)

    for i in range(args.warmup):
        ids, oo = step()
        torch.cuda.synchronize()
        log(rank, "warmup %d done" % i)
    n_ids = int(ids.numel())

    engine.profile_enable(True)
    engine.profile_reset()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ids, oo = step()
        log(rank, "step %d enqueued" % i)
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = engine.profile_read()
    passes = engine.profile_tile_passes(local)
    fb_rows = engine.fallback_rows(local)
    engine.profile_enable(False)

    gather_ms = None
    if dist and args.gather:
        from akshar_amd import dist as adist
        torch.cuda.synchronize()
        tg = time.perf_counter()
        adist.gather_ids(ids, oo)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3

    if dist:
        rdev = dev if tdist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([nbytes, n_ids], dtype=torch.float64, device=rdev)
        tdist.all_reduce(tot)
        job_bytes, job_ids = float(tot[0]), float(tot[1])
    else:
        job_bytes, job_ids = float(nbytes), float(n_ids)

    ms_step = elapsed / args.steps * 1e3
    value = job_bytes * args.steps / elapsed / 1e6
    toks = job_ids * args.steps / elapsed

    # dominant kernel: per-launch algorithmic bytes / its average launch duration (HIP events the
    # library records around its own launches on the encode stream)
    kern = max(("count", "emit", "tiles"), key=lambda k: prof[k][0])
    k_ms, k_n = prof[kern]
    avg_s = k_ms / max(k_n, 1) / 1e3
    read_bytes = nbytes + 8 * (rows + 1)  # raw UTF-8 rows + u64 row offsets
    if kern == "count":
        write_bytes = 4 * rows  # u32 count per row
    elif kern == "emit":
        write_bytes = 4 * n_ids + 8 * (rows + 1)  # u32 ids + u64 row offsets
    else:
        write_bytes = 4 * n_ids + 4 * rows  # u32 ids into the row slots + u32 count per row
    algo = read_bytes + write_bytes
    achieved = algo / avg_s / 1e9 if avg_s > 0 else 0.0
    kname = {"count": "k_rows_fast<OP_BPE,3,false> (count pass)", "emit": "k_rows_fast<OP_BPE,3,true> (emit pass)",
             "tiles": "k_bpe_tiles<3> (tile-cooperative encode)"}[kern]
    traffic, traffic_src = None, None
    tfile = os.path.join(ROOT, "profiles", TRAFFIC_FILE)
    if kern == "tiles" and os.path.exists(tfile):
        t = json.load(open(tfile))
        if t.get("rows") == rows and t.get("bytes") == nbytes:  # the same launch shape, measured by PMC
            traffic = int(t["hbm_bytes_per_launch"])
            traffic_src = "profiles/%s (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, same 10 M-row launch)" % TRAFFIC_FILE
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": kname,
                "kernel_avg_ms": round(avg_s * 1e3, 3), "algorithmic_bytes_per_launch": int(algo),
                "read_frac": round(read_bytes / avg_s / 1e9 / HBM_PEAK_GBS, 5) if avg_s > 0 else 0.0,
                "kernel_ms_per_step": {k: round(v[0] / max(args.steps, 1), 3) for k, v in prof.items() if v[1]}}
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    if passes:
        roofline["tile_pass_cycle_frac"] = passes
        roofline["fallback_rows_per_step"] = fb_rows[0]

    others = None
    if rank == 0 and not args.no_others:
        log(rank, "other configs")
        others = other_configs(local)

    cpu = None
    if rank == 0 and not args.no_cpu:
        log(rank, "timed region done (%.1f ms/step); CPU baseline" % (elapsed / args.steps * 1e3))
        cpu = cpu_baseline(args, buf, offs)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (akshar_amd.synth, seed %d)" % SEED,
            "tokens_per_s": round(toks, 1),
            "config": {"workload": "cfg4: %d synthetic Hinglish sentences per GPU, normalize_text + 24k BPE encode "
                                   "(models/akshar.json), inputs resident in HBM" % rows,
                       "rows_per_gpu": rows, "bytes_per_gpu": nbytes, "ids_per_gpu": n_ids,
                       "parallelism": "dp%d (row shards, no data-path collective)" % world},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if others:
            line["other_configs"] = others
        if gather_ms is not None:
            line["gather_ms"] = round(gather_ms, 3)
        print(json.dumps(line), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
