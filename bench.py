#!/usr/bin/env python3
"""Benchmark: the reference's encode hot path on MI355X (BASELINE.json metric).

Workloads (`--workload`):
  cfg4 (default)  10 M synthetic Hinglish sentences PER GPU, encoded end to end exactly as
                  `aksharTokenizer(model_path="models/akshar.json", model_type="bpe").encode(line)`
                  (tokenizer.py:167-193): normalize_text -> HF NFKC -> Whitespace pre-tokenizer ->
                  24k BPE merges -> <s> ... </s>. Weak scaling: every rank encodes its own 10 M
                  rows, no data-path collective. One step = one encode of the per-GPU batch.
  cfg5            ONE fixed batch of --rows (default 100 M) synthetic Hinglish sentences (the same
                  rows for every N: row i is generated from its global index), cut into contiguous
                  byte-balanced shards (rank 0 sizes every row and broadcasts the cuts, the
                  akshar_amd.dist.shard_rows rule), each rank's shard encoded with the 24k unigram
                  SentencePiece model (`model_type="sentencepiece"`) in chunks straight into one
                  per-rank id buffer, then ONE all-gather reassembles the whole batch's id streams
                  on every rank (akshar_amd.dist.gather_ids: RCCL over xGMI). Strong scaling. One
                  step = encode of the shard + the gather (gather_ms reported separately).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg4|cfg5] [--rows R]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N, or plain
         `python bench.py --gpus N`: with no RANK in the environment the script starts that launcher
         itself as a child process (before any GPU call) and exits with its code.
  At N > 1 cfg4 ends every step with gather_ids (the north star's all-gather that reassembles the
  id streams on every rank, ids as int16 on the wire: the 24k vocabulary fits); --no-gather times
  the encode alone.

Rows are packed UTF-8 + int64 offsets already resident in HBM when the timed region starts. Prints
ONE JSON line (rank 0): value = whole-job MB/s of raw UTF-8 input (max-over-ranks time), tokens/s,
the dominant kernel's HBM roofline (SURVEY.md §8(d) read bytes / its average launch time from HIP
events on the encode stream; PMC traffic from profiles/), the CPU baseline (the oracle, 1 thread
and all host cores, on a bounded sample) and end-to-end host->host rates (N = 1 only).
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MB of raw UTF-8 tokenized/sec @1 GPU (+ tokens/s); bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
SEED = 1234
KERNEL_NAMES = {"tiles": "k_bpe_tiles<3> (tile-cooperative BPE encode)",
                "spm_tiles": "k_spm_tiles<3> (tile-cooperative SentencePiece encode)",
                "emit": "k_rows_stage<OP,3> (staged row kernel, one lane per row)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("cfg4", "cfg5"), default="cfg4")
    ap.add_argument("--rows", type=int, default=None, help="cfg4: rows per GPU (10 M); cfg5: rows of the batch (100 M)")
    ap.add_argument("--chunk-rows", type=int, default=25_000_000, help="cfg5: rows per encode call")
    ap.add_argument("--gather", action="store_true", help="cfg4 at N = 1 (a world-1 group): also all-gather")
    ap.add_argument("--no-gather", action="store_true", help="cfg4 at N > 1: time the encode alone")
    ap.add_argument("--dry-run", action="store_true", help="launcher check: set up the process group, print the "
                    "JSON line with the world size, no GPU work")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="CPU baseline: seconds per leg (up to 8 legs per model)")
    ap.add_argument("--cfg5-rows", type=int, default=25_000_000, help="N = 1: rows of the cfg5 SentencePiece launch block")
    ap.add_argument("--no-cfg5", action="store_true", help="N = 1: skip the cfg5 SentencePiece launch block")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-others", action="store_true", help="skip the config 2/3/5 side measurements")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end host->host rates")
    ap.add_argument("--no-single", action="store_true", help="skip the per-call latency block")
    return ap.parse_args()


T_START = time.perf_counter()


def log(rank, msg):
    """progress on stderr (the JSON line is the only stdout output)"""
    if rank == 0:
        print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


# ------------------------------------------------------------------------------------------ CPU
def cpu_info():
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def cgroup_cpu_quota():
    """The cgroup's CPU limit as 'quota period' (cgroup v2 cpu.max) or None; the cores a process
    may really use can be fewer than its affinity set."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            return open(path).read().strip()
        except OSError:
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return "%d %d" % (q, p) if q > 0 else "max %d" % p
    except (OSError, ValueError):
        return None


def usable_cpus(avail):
    """The CPUs this process can really run on at once: its affinity set, capped by the cgroup
    quota (cpu.max quota / period, rounded up). On the GPU box the affinity set is the whole
    machine but the quota is 16 CPUs."""
    q = cgroup_cpu_quota()
    if q:
        parts = q.split()
        try:
            if parts[0] != "max":
                return max(1, min(avail, -(-int(parts[0]) // int(parts[1]))))
        except (ValueError, IndexError, ZeroDivisionError):
            pass
    return avail


def cpu_baseline(args, buf, offs, kind):
    """The oracle (oracle/akshar_oracle.c) on the same batch, time-bounded legs run inside the C
    library on OpenMP threads (oracle.encode_timed: 2,000-row chunks from a shared cursor,
    per-thread reusable buffers, no Python in the loop): a sweep of 1, 8, 32, 64, 128, 256
    threads (capped at this process's affinity set), plus the per-GPU share of the cores (the
    usable CPUs / 8). `cores` is what a leg can really use: min(threads, affinity, cgroup quota);
    `threads` is the OpenMP thread count. The single thread is the single-process reference the
    >= 10x target is quoted against; the all-core value is the best leg of the sweep."""
    from akshar_amd.models import BPEModel, SPMModel
    from oracle import oracle as O
    model = (O.OracleBPE(BPEModel(os.path.join(ROOT, "models", "akshar.json"))) if kind == "bpe"
             else O.OracleSPM(SPMModel(os.path.join(ROOT, "models", "akshar.model"))))
    cpu_model, nproc, avail = cpu_info()
    usable = usable_cpus(avail)
    sec = args.cpu_seconds
    n = len(offs) - 1

    def leg(threads):
        nb, ni, dt = O.encode_timed(model, buf, offs, threads, sec, chunk_rows=min(2000, n))
        return {"value": round(nb / 1e6 / dt, 3), "unit": "MB/s", "cores": min(threads, usable), "threads": threads,
                "kind": "port",
                "tokens_per_s": round(ni / dt, 1),
                "sample": "%.1f MB (%d-row chunks of the timed batch) in %.2f s on %d OpenMP thread(s), "
                          "oracle/akshar_oracle.c %s encode (or_encode_timed)" % (nb / 1e6, min(2000, n), dt, threads, kind)}

    single = leg(1)
    calib = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(calib):
        c = json.load(open(calib)).get(kind)
        if c:
            single["python_reference_equivalent_mb_s"] = round(single["value"] / c["oracle_over_reference"], 3)
            single["calibration"] = "profiles/cpu_calibration.json: oracle / Python reference = %.2f on the same rows " \
                                    "(build container)" % c["oracle_over_reference"]
    sweep = [single]
    for t in (8, 32, 64, 128, 256):
        if t > avail:
            break
        sweep.append(leg(t))
    if avail not in [x["threads"] for x in sweep]:
        sweep.append(leg(avail))
    share = leg(max(1, usable // 8))
    full = dict(max(sweep, key=lambda x: x["value"]))
    full.update({"cpu_model": cpu_model, "nproc": nproc, "affinity_cpus": avail, "cgroup_cpu_max": cgroup_cpu_quota(),
                 "usable_cpus": usable,
                 "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "per_gpu_share": share,
                 "single_thread": single,
                 "sweep": [{"threads": x["threads"], "cores": x["cores"], "mb_s": x["value"]} for x in sweep],
                 "value_is": "the best leg of the thread sweep (all host cores this process may use); cores = "
                             "min(threads, affinity, cgroup quota)"})
    return full


# ------------------------------------------------------------------------------------------ side configs
def other_configs(dev, rows=1_000_000):
    """SURVEY.md §8 configs 2, 3 and 5 on this GPU (1 M synthetic rows each, inputs in HBM): device
    time of each op's kernels (the library's HIP events) and the wall time of the Python call."""
    from akshar_amd import engine, synth

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        engine.profile_enable(True)
        engine.profile_reset()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / reps
        prof = engine.profile_read()
        engine.profile_enable(False)
        return sum(v[0] for v in prof.values()) / reps / 1e3, wall

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
        res = {}
        for k, f in ops.items():
            kt, wt = timed(f)
            res[k] = {"kernels_mb_s": round(mb / kt, 1), "call_mb_s": round(mb / wt, 1)}
        res["rows"], res["mb"] = rows, round(mb, 1)
        out[name] = res
    d, h = out["devanagari"], out["hinglish"]
    return {"unit": "MB/s of raw UTF-8 (1 M synthetic rows, inputs in HBM); kernels_mb_s = bytes / summed device "
                    "time of the op's kernels, call_mb_s = bytes / wall time of the Python call",
            "cfg2_segment_devanagari": d["segment"]["kernels_mb_s"],
            "cfg3_normalize_switches_segment_hinglish": h["analyze_fused"]["kernels_mb_s"],
            "cfg5_spm_encode_hinglish_per_gpu": h["spm_encode"]["kernels_mb_s"], "detail": out}


# ------------------------------------------------------------------------------------------ end to end
def end_to_end(dev, model, host_buf, host_offs, kind):
    """Host -> host rates (PCIe included; never `value`): (a) packed numpy rows -> numpy ids + row
    offsets (H2D, encode, D2H); (b) list[str] -> list[list[int]] through the drop-in class."""
    from akshar_amd import engine, synth
    from akshar_amd.tokenizer import aksharTokenizer
    nbytes = int(host_offs[-1])
    pad = np.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:nbytes] = host_buf
    offs64 = host_offs.astype(np.int64)

    def arrays():
        gb, go = engine.to_device(pad, offs64, dev=dev)
        ids, oo = model.encode_batch(gb, go, nbytes=nbytes)
        return ids.cpu().numpy(), oo.cpu().numpy()

    arrays()
    torch.cuda.synchronize()
    t = time.perf_counter()
    ids, _ = arrays()
    dt_a = time.perf_counter() - t
    n_list = 200_000
    texts = synth.lines(synth.KIND_HINGLISH, n_list, seed=SEED + 3)
    lb = sum(len(x.encode()) for x in texts)
    mp = os.path.join(ROOT, "models", "akshar.json" if kind == "bpe" else "akshar.model")
    tk = aksharTokenizer(model_path=mp, model_type="bpe" if kind == "bpe" else "sentencepiece")
    tk.encode_batch(texts[:1000])
    t = time.perf_counter()
    res = tk.encode_batch(texts)
    dt_l = time.perf_counter() - t
    return {"arrays_mb_s": round(nbytes / 1e6 / dt_a, 1), "arrays_tokens_per_s": round(len(ids) / dt_a, 1),
            "arrays": "numpy bytes + offsets (%d rows, %.0f MB) -> H2D -> encode -> D2H numpy ids + offsets, %.1f ms"
                      % (len(host_offs) - 1, nbytes / 1e6, dt_a * 1e3),
            "list_mb_s": round(lb / 1e6 / dt_l, 2), "list_tokens_per_s": round(sum(len(r) for r in res) / dt_l, 1),
            "list": "aksharTokenizer.encode_batch(list of %d str) -> list[list[int]] (UTF-8 packing, H2D, encode, D2H, "
                    "Python int lists), %.1f ms" % (n_list, dt_l * 1e3)}


# ------------------------------------------------------------------------------------------ per-call latency
def single_call(dev, calls=1000):
    """Per-call latency of the drop-in class on one 143-byte line: encode(str)
    on both models (ak_*_encode_host: pinned staging, one copy each way, one synchronize) and
    tokenize(str), each `calls` calls after a warmup; the batch-of-one path (encode_batch([str]):
    device packing, read-backs) beside it. Wall-clock microseconds per call, mean and median."""
    from akshar_amd import synth
    from akshar_amd.tokenizer import aksharTokenizer
    line = next(t for t in synth.lines(synth.KIND_HINGLISH, 20000, seed=SEED + 5) if len(t.encode()) >= 143)
    raw = line.encode()[:143]
    while True:  # cut on a char boundary
        try:
            line = raw.decode()
            break
        except UnicodeDecodeError:
            raw = raw[:-1]
    out = {"line_bytes": len(line.encode()), "calls": calls}
    for kind, mp, mt in (("bpe", "akshar.json", "bpe"), ("spm", "akshar.model", "sentencepiece")):
        tk = aksharTokenizer(model_path=os.path.join(ROOT, "models", mp), model_type=mt)
        for name, fn in (("encode", lambda: tk.encode(line)), ("tokenize", lambda: tk.tokenize(line)),
                         ("encode_batch_of_one", lambda: tk.encode_batch([line])[0])):
            for _ in range(50):
                fn()
            ts = []
            for _ in range(calls):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            ts = np.asarray(ts) * 1e6
            out["%s_%s_us" % (kind, name)] = {"mean": round(float(ts.mean()), 1), "median": round(float(np.median(ts)), 1)}
    return out


# ------------------------------------------------------------------------------------------ PMC traffic
def pmc_traffic(kernel, rows, nbytes):
    """HBM bytes per launch of `kernel` measured by rocprofv3 PMC on the same launch shape (newest
    profiles/*_pmc.json whose kernel, rows and bytes match), or (None, None)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("kernel_class") == kernel and t.get("rows") == rows and t.get("bytes") == nbytes:
            return int(t["hbm_bytes_per_launch"]), "profiles/%s (rocprofv3 FETCH_SIZE x1024 x2 + WRITE_SIZE x1024, " \
                                                   "same launch shape)" % os.path.basename(path)
    return None, None


# ------------------------------------------------------------------------------------------ roofline
def roofline_of(prof, kern, steps, rows, nbytes, n_ids):
    """SURVEY.md §8(d) for the dominant kernel: read bytes (raw rows + u64 offsets) per launch / its
    average launch time from the library's HIP events on the encode stream; PMC traffic of the same
    launch shape from profiles/."""
    k_ms, k_n = prof[kern]
    k_n = max(k_n, 1)
    avg_s = k_ms / k_n / 1e3
    launches_per_step = k_n / steps
    rows_l = rows / launches_per_step
    bytes_l = nbytes / launches_per_step
    ids_l = n_ids / launches_per_step
    read_bytes = bytes_l + 8 * (rows_l + 1)  # raw UTF-8 rows + u64 row offsets
    write_bytes = 4 * ids_l + 4 * rows_l     # u32 ids into the row slots + u32 count per row
    achieved = read_bytes / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic, traffic_src = pmc_traffic(kern, int(round(rows_l)), int(round(bytes_l)))
    r = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": KERNEL_NAMES[kern],
         "kernel_avg_ms": round(avg_s * 1e3, 3), "launches_per_step": launches_per_step,
         "achieved_is": "SURVEY.md §8(d) read bytes (sum B + 8 (N + 1)) per launch / average launch time",
         "read_bytes_per_launch": int(read_bytes),
         "total_algorithmic_bytes_per_launch": int(read_bytes + write_bytes),
         "total_frac": round((read_bytes + write_bytes) / avg_s / 1e9 / HBM_PEAK_GBS, 5) if avg_s > 0 else 0.0,
         "kernel_ms_per_step": {k: round(v[0] / max(steps, 1), 3) for k, v in prof.items() if v[1]}}
    if traffic_src:
        r["traffic_source"] = traffic_src
        r["traffic_over_algorithmic"] = round(traffic / (read_bytes + write_bytes), 3)
    return r


def pass_split(engine, fn, dev, counters=None):
    """Per-pass wave-cycle split of the tile kernel from ONE extra, untimed launch with the pass
    clocks on (they instrument the kernel, so the timed steps run without them); `counters` (a dict)
    receives the same launch's event counters (BPE pre-token cache probes and hits)."""
    engine.profile_enable(True, passes=True)
    engine.profile_tile_passes(dev)  # reset the accumulators
    engine.profile_tile_counters(dev)
    fn()
    torch.cuda.synchronize()
    passes = engine.profile_tile_passes(dev)
    ctr = engine.profile_tile_counters(dev)
    engine.profile_enable(False)
    if counters is not None and ctr.get("ptc_probes"):
        counters.update({"probes_per_step": ctr["ptc_probes"], "hits_per_step": ctr["ptc_hits"],
                         "hit_rate": round(ctr["ptc_hits"] / ctr["ptc_probes"], 4),
                         "source": "the pass-clock step's counters (ak_profile_tile_counters): multi-symbol "
                                   "pre-tokens probed in the pre-token result cache, and its hits"})
    return passes


def cfg5_block(args, dev):
    """BASELINE config 5 on this GPU: ONE launch shape of the 100 M-row cfg5 batch (its first
    --cfg5-rows rows, 25 M by default, the per-call chunk bench --workload cfg5 encodes), 24k unigram
    SentencePiece, inputs in HBM; --steps timed launches (HIP events), the read roofline of
    k_spm_tiles, PMC traffic of that launch shape from profiles/, and its own CPU baseline."""
    from akshar_amd import engine, synth
    rows = args.cfg5_rows
    buf, offs = synth.generate(synth.KIND_HINGLISH, rows, seed=SEED, first=0)
    nbytes = int(offs[-1])
    pad = np.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:nbytes] = buf
    gb, go = engine.to_device(pad, offs.astype(np.int64), dev=dev)
    del pad
    spm = engine.SPM(os.path.join(ROOT, "models", "akshar.model"), dev=dev)
    cap = nbytes // 4 + 2 * rows + 1024
    out = torch.empty(cap, dtype=torch.int32, device=gb.device)
    oo = torch.empty(rows + 1, dtype=torch.int64, device=gb.device)

    def run():
        return spm.encode_batch(gb, go, nbytes=nbytes, out=out, out_offs=oo)

    ids, _ = run()
    n_ids = int(ids.numel())
    torch.cuda.synchronize()
    engine.profile_enable(True)
    engine.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    prof = engine.profile_read()
    engine.profile_enable(False)
    roof = roofline_of(prof, "spm_tiles", args.steps, rows, nbytes, n_ids)
    roof["tile_pass_cycle_frac"] = pass_split(engine, run, dev)
    del gb, go, out, oo
    torch.cuda.empty_cache()
    res = {"workload": "cfg5 launch: first %d rows of the cfg5 batch (synthetic Hinglish, seed %d), normalize_text + "
                       "24k unigram SentencePiece (models/akshar.model), inputs in HBM" % (rows, SEED),
           "rows": rows, "bytes": nbytes, "ids": n_ids, "ms_per_launch": round(dt * 1e3, 3),
           "value": round(nbytes / 1e6 / dt, 2), "unit": "MB/s", "tokens_per_s": round(n_ids / dt, 1),
           "roofline": roof}
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(args, buf, offs, "spm")
    return res


# ------------------------------------------------------------------------------------------ launcher
def launch_workers(args):
    """`--gpus N` (N > 1) without a launcher: run torch.distributed.run with N ranks on this node as
    a CHILD process (nothing here has touched the GPU; never exec) and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print("[bench] launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


# ------------------------------------------------------------------------------------------ main
def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_workers(args))
    # a process group whenever launched by torch.distributed.run (even at world size 1: the RCCL
    # path then runs with one rank) or asked for N > 1
    dist = args.gpus > 1 or "RANK" in os.environ
    rank, world, local = 0, 1, 0
    if dist:
        import torch.distributed as tdist
        rank = int(os.environ["RANK"])
        world = int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", rank))
        backend = os.environ.get("AK_BENCH_BACKEND", "nccl")  # gloo: rehearse N ranks on one GPU
        if args.dry_run:
            tdist.init_process_group("gloo")
            if rank == 0:
                print(json.dumps({"dry_run": True, "n_gpus": tdist.get_world_size(), "world_size": tdist.get_world_size(),
                                  "requested_gpus": args.gpus, "backend": backend}), flush=True)
            tdist.barrier()
            tdist.destroy_process_group()
            return
        if backend == "nccl":
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(torch.cuda.device_count(), 1)
            tdist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cdev = dev if (not dist or tdist.get_backend() == "nccl") else torch.device("cpu")

    from akshar_amd import engine, synth
    cfg5 = args.workload == "cfg5"
    if not cfg5:
        rows = args.rows or 10_000_000
        r0 = rank * rows
        log(rank, "cfg4: generating %d rows per GPU" % rows)
    else:
        total_rows = args.rows or 100_000_000
        log(rank, "cfg5: sizing %d rows" % total_rows)
        cuts = torch.zeros(world + 1, dtype=torch.int64)
        if rank == 0:  # byte-balanced contiguous shards (dist.shard_rows rule) from the row lengths
            from akshar_amd import dist as adist
            lens = np.empty(total_rows, dtype=np.uint64)
            synth._lib().ak_synth_sizes(SEED, synth.KIND_HINGLISH, 0, total_rows, lens.ctypes.data)
            offs_all = np.zeros(total_rows + 1, dtype=np.int64)
            np.cumsum(lens, out=offs_all[1:])
            del lens
            cuts = torch.tensor([adist.shard_rows(offs_all, world, k)[0] for k in range(world)] + [total_rows],
                                dtype=torch.int64)
            del offs_all
        if dist:
            cc = cuts.to(cdev)
            tdist.broadcast(cc, 0)
            cuts = cc.cpu()
        r0, r1 = int(cuts[rank]), int(cuts[rank + 1])
        rows = r1 - r0
        log(rank, "cfg5: rank shard rows [%d, %d)" % (r0, r1))
    buf, offs = synth.generate(synth.KIND_HINGLISH, rows, seed=SEED, first=r0)
    nbytes = int(offs[-1])
    log(rank, "generated %.1f MB" % (nbytes / 1e6))
    pad = np.zeros(((nbytes + 15) // 16) * 16 + 16, dtype=np.uint8)
    pad[:nbytes] = buf
    gbuf, goffs = engine.to_device(pad, offs.astype(np.int64), dev=local)
    kind = "spm" if cfg5 else "bpe"
    model = (engine.SPM(os.path.join(ROOT, "models", "akshar.model"), dev=local) if cfg5
             else engine.BPE(os.path.join(ROOT, "models", "akshar.json"), dev=local))
    # id capacity: BPE <= bytes + 2 per row (tile path bound), measured ~0.2 ids per byte for both
    # models; the encode raises (never truncates) if a caller buffer is short
    cap = (nbytes // 4 if cfg5 else nbytes // 2) + 2 * rows + 1024
    if cfg5:  # chunks of the shard encoded straight into one per-rank buffer
        ch = max(1, args.chunk_rows)
        chunks = []
        for c0 in range(0, rows, ch):
            c1 = min(rows, c0 + ch)
            b0, b1 = int(offs[c0]), int(offs[c1])
            chunks.append((c0, c1, b0, b1, goffs[c0:c1 + 1] - b0))
        ids_all = torch.empty(cap, dtype=torch.int32, device=dev)
        offs_all = torch.empty(rows + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    gather_s = [0.0]
    # every id is below the vocabulary size: at <= 32,768 the gather moves them as int16
    id_bound = len(model.model.pieces) if cfg5 else model.model.vocab_size
    do_gather = dist and (args.gather or (world > 1 and not args.no_gather))
    gloo = dist and tdist.get_backend() != "nccl"

    def gather(ids, oo):
        from akshar_amd import dist as adist
        torch.cuda.synchronize()
        tg = time.perf_counter()
        if gloo:  # the one-GPU rehearsal: gloo gathers host tensors
            adist.gather_ids(ids.cpu(), oo.cpu(), id_bound=id_bound)
        else:
            adist.gather_ids(ids, oo, id_bound=id_bound)
        torch.cuda.synchronize()
        gather_s[0] += time.perf_counter() - tg

    def step():
        if not cfg5:
            ids, oo = model.encode_batch(gbuf, goffs, cap=cap, nbytes=nbytes)
            if do_gather:
                gather(ids, oo)
            return ids, oo
        pos = 0
        for c0, c1, b0, b1, co in chunks:
            # rows [c0, c1) start at byte b0 (16-aligned or not: the engine reads aligned blocks)
            ids, oo = model.encode_batch(gbuf[b0:], co, nbytes=b1 - b0, out=ids_all[pos:],
                                         out_offs=offs_all[c0:c1 + 1])
            if pos:
                offs_all[c0:c1 + 1] += pos
            pos += ids.numel()
        ids, oo = ids_all[:pos], offs_all
        if dist:
            gather(ids, oo)
        return ids, oo

    for i in range(args.warmup):
        ids, oo = step()
        torch.cuda.synchronize()
        log(rank, "warmup %d done" % i)
    n_ids = int(ids.numel())
    gather_s[0] = 0.0

    engine.profile_enable(True)  # HIP events only: the timed kernels are the product kernels
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
    engine.profile_enable(False)
    fb_rows = engine.fallback_rows(local)
    ptc = {}
    passes = pass_split(engine, step, local, ptc) if world == 1 else {}  # step() of N > 1 holds a collective

    if dist:
        t = torch.tensor([elapsed, gather_s[0]], dtype=torch.float64, device=cdev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed, gmax = float(t[0]), float(t[1])
        tot = torch.tensor([nbytes, n_ids], dtype=torch.float64, device=cdev)
        tdist.all_reduce(tot)
        job_bytes, job_ids = float(tot[0]), float(tot[1])
        imb = torch.tensor([nbytes], dtype=torch.float64, device=cdev)
        mx, mn = imb.clone(), imb.clone()
        tdist.all_reduce(mx, op=tdist.ReduceOp.MAX)
        tdist.all_reduce(mn, op=tdist.ReduceOp.MIN)
        byte_imbalance = float(mx) / max(float(mn), 1.0)
    else:
        job_bytes, job_ids, gmax, byte_imbalance = float(nbytes), float(n_ids), gather_s[0], 1.0

    ms_step = elapsed / args.steps * 1e3
    value = job_bytes * args.steps / elapsed / 1e6
    toks = job_ids * args.steps / elapsed

    # dominant kernel: per-launch algorithmic bytes / its average launch duration (HIP events the
    # library records around its own launches on the encode stream)
    kern = max(("emit", "tiles", "spm_tiles"), key=lambda k: prof.get(k, (0.0, 0))[0])
    roofline = roofline_of(prof, kern, args.steps, rows, nbytes, n_ids)
    if passes:
        roofline["tile_pass_cycle_frac"] = passes
        roofline["tile_pass_source"] = "one extra untimed step with the pass clocks on"
    roofline["fallback_rows_per_step"] = fb_rows[0]
    if ptc:
        roofline["pretoken_cache"] = ptc

    others = e2e = cpu = c5 = single = None
    if rank == 0 and world == 1 and not cfg5 and not args.no_cfg5:
        log(rank, "cfg5 launch block")
        c5 = cfg5_block(args, local)
    if rank == 0 and world == 1 and not args.no_others:
        log(rank, "other configs")
        others = other_configs(local)
    if rank == 0 and world == 1 and not args.no_e2e:
        log(rank, "end to end")
        e2e = end_to_end(local, model, buf, offs, kind)
    if rank == 0 and world == 1 and not args.no_single:
        log(rank, "per-call latency")
        single = single_call(local)
    if rank == 0 and world == 1 and not args.no_cpu:
        log(rank, "timed region done (%.1f ms/step); CPU baseline" % ms_step)
        cpu = cpu_baseline(args, buf, offs, kind)

    if rank == 0:
        if cfg5:
            wl = ("cfg5: one batch of %d synthetic Hinglish sentences, byte-balanced contiguous shards over %d GPU(s), "
                  "normalize_text + 24k unigram SentencePiece encode (models/akshar.model) in chunks of %d rows, "
                  "+ all-gather of the id streams (N > 1), inputs resident in HBM" % (total_rows, world, args.chunk_rows))
        else:
            wl = ("cfg4: %d synthetic Hinglish sentences per GPU, normalize_text + 24k BPE encode (models/akshar.json), "
                  "inputs resident in HBM" % rows)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if cfg5 else "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (akshar_amd.synth, seed %d)" % SEED, "tokens_per_s": round(toks, 1),
            "config": {"workload": wl, "rows_per_gpu": rows, "bytes_per_gpu": nbytes, "ids_per_gpu": n_ids,
                       "parallelism": ("dp%d (byte-balanced row shards + all-gather)" if cfg5 or do_gather else
                                       "dp%d (row shards, no data-path collective)") % world},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if dist:
            line["world_size"] = tdist.get_world_size()  # the ranks the process group (RCCL) saw
            line["backend"] = tdist.get_backend()
        if cfg5 or do_gather:
            line["gather_ms"] = round(gmax / args.steps * 1e3, 3)
            line["gather"] = ("akshar_amd.dist.gather_ids inside every timed step: all-gather of the per-rank sizes, "
                              "then ONE all_gather_into_tensor of the padded (offsets | ids) records, ids as %s" %
                              ("int16" if id_bound <= 32768 else "int32"))
            line["encode_only_mb_s"] = round(job_bytes * args.steps / max(elapsed - gmax, 1e-9) / 1e6, 2)
            line["shard_byte_imbalance"] = round(byte_imbalance, 5)
        if e2e:
            line["end_to_end"] = e2e
        if single:
            line["single_call_us"] = single
        if c5:
            line["cfg5"] = c5
        if others:
            line["other_configs"] = others
        print(json.dumps(line), flush=True)
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
