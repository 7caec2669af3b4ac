"""Summarise a tools/measure.sh trace / pmc output directory into profiles/<tag>_*.

  python tools/pmc_summary.py gpurun_out/v4/prof r01_v4

writes profiles/<tag>_bench_kernel_stats.csv (the rocprofv3 --stats summary of the bench run),
profiles/<tag>_bench.json (the bench line of that run) and profiles/<tag>_tiles_pmc.json (the PMC
passes over one cfg4-size tile-kernel launch, HBM bytes corrected as MI355X_MICROARCH.md says:
FETCH_SIZE is in KiB and counts half of the 16-B/lane streaming reads on gfx950 -> x1024 x2,
WRITE_SIZE in KiB -> x1024).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, match="bpe_tiles"):
    agg, meta = collections.defaultdict(float), {}
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            meta = {"vgpr": int(r.get("Arch_VGPR_Count") or r.get("VGPR_Count") or 0),
                    "lds_block": int(r.get("LDS_Block_Size") or r.get("Lds_Size") or 0),
                    "scratch": int(r.get("Scratch_Size") or 0)}
    return dict(agg), meta


KERNEL_CLASS = {"bpe_tiles": ("tiles", "k_bpe_tiles<3>"), "spm_tiles": ("spm_tiles", "k_spm_tiles<3>"),
                "rows_tiles<2>": ("row_tiles_seg", "k_rows_tiles<2> (segment)"),
                "rows_tiles<7>": ("row_tiles_analyze", "k_rows_tiles<7> (fused analyze)")}


def op_summary(src, tag, match, rows, nbytes):
    """tools/pmc_op.sh output -> profiles/<tag>_<class>_pmc.json (HBM bytes per launch, SQ counters)
    and profiles/<tag>_<class>_kernel_stats.csv (the kernel trace summary of the same op)."""
    out = os.path.join(ROOT, "profiles")
    cls, kname = KERNEL_CLASS[match]
    allc, meta = {}, {}
    for name in ("fetch", "write", "sq1", "sq2", "mem", "tcp"):
        p = os.path.join(src, name, name + "_counter_collection.csv")
        if os.path.exists(p):
            c, m = counters(p, match)
            allc.update(c)
            meta = meta or m
    rd = allc["FETCH_SIZE"] * 1024 * 2
    # vector-memory pipe: TA / TD busy per CU over the kernel's cycles per XCD (GRBM_GUI_ACTIVE sums
    # the 8 XCDs; 256 CUs each with one TA and one TD)
    gui = allc.get("GRBM_GUI_ACTIVE", 0) / 8.0
    pipe = {}
    if gui > 0:
        pipe = {"ta_busy_frac": round(allc.get("TA_TA_BUSY_sum", 0) / 256.0 / gui, 3),
                "td_busy_frac": round(allc.get("TD_TD_BUSY_sum", 0) / 256.0 / gui, 3)}
    if allc.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        pipe["l1_hit_frac"] = round(1.0 - allc.get("TCP_TCC_READ_REQ_sum", 0) / allc["TCP_TOTAL_CACHE_ACCESSES_sum"], 3)
    wr = allc["WRITE_SIZE"] * 1024
    rec = {"kernel": kname, "kernel_class": cls, "rows": rows, "bytes": nbytes,
           "command": "tools/pmc_op.sh (rocprofv3 --pmc, one run per counter group) over tools/prof_op.py, one launch "
                      "of %d synthetic Hinglish rows (%d bytes)" % (rows, nbytes),
           "counters": allc, **meta, "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
           "valu_per_row": round(allc.get("SQ_INSTS_VALU", 0) / rows, 1),
           "salu_per_row": round(allc.get("SQ_INSTS_SALU", 0) / rows, 1),
           "lds_per_row": round(allc.get("SQ_INSTS_LDS", 0) / rows, 1),
           "wait_frac": round(allc.get("SQ_WAIT_ANY", 0) / max(allc.get("SQ_WAVE_CYCLES", 1), 1), 3),
           "vmem_rd_per_row": round(allc.get("SQ_INSTS_VMEM_RD", 0) / rows, 1), **pipe,
           "note": "read = FETCH_SIZE x 1024 x 2 (gfx950 half-count correction for 16-B/lane streaming reads), "
                   "write = WRITE_SIZE x 1024"}
    json.dump(rec, open(os.path.join(out, "%s_%s_pmc.json" % (tag, cls)), "w"), indent=1)
    st = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if st:
        shutil.copy(st[0], os.path.join(out, "%s_%s_kernel_stats.csv" % (tag, cls)))
    print(json.dumps(rec, indent=1))


def main(src, tag):
    out = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "bench", "bench_kernel_stats.csv"), os.path.join(out, tag + "_bench_kernel_stats.csv"))
    line = [ln for ln in open(os.path.join(src, "bench_stdout.log")) if ln.startswith("{")][-1]
    open(os.path.join(out, tag + "_bench.json"), "w").write(line)
    allc, meta = {}, {}
    for name in ("fetch", "write", "sq1", "sq2"):
        p = os.path.join(src, name, name + "_counter_collection.csv")
        if os.path.exists(p):
            c, m = counters(p)
            allc.update(c)
            meta = meta or m
    rd = allc["FETCH_SIZE"] * 1024 * 2
    wr = allc["WRITE_SIZE"] * 1024
    rec = {"kernel": "k_bpe_tiles<3>",
           "command": "rocprofv3 --pmc <counters> -- python3 tools/prof_op.py bpe 10000000 1 1 (one cfg4-size launch, "
                      "10 M synthetic Hinglish rows); separate passes per counter group (tools/measure.sh, tools/pmc_op.sh)",
           "rows": 10000000, "counters": allc, **meta,
           "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
           "note": "read = FETCH_SIZE x 1024 x 2 (gfx950 half-count correction for 16-B/lane streaming reads), "
                   "write = WRITE_SIZE x 1024"}
    json.dump(rec, open(os.path.join(out, tag + "_tiles_pmc.json"), "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3:  # pmc_summary.py SRC TAG MATCH ROWS BYTES
        op_summary(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
    else:
        main(sys.argv[1], sys.argv[2])
