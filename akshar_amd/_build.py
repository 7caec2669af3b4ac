"""In-tree builds of the native pieces (no JIT cache: the .so files travel with the repo).

  _synth.so       host C corpus generator (bench/test utility)
  _pylist*.so     CPython extension: list[str] -> packed UTF-8, packed ids -> list[list[int]]
  _akshar_hip.so  the product: HIP kernels for gfx950 + the C-ABI declared in include/akshar.h
  oracle/_oracle.so  the CPU restatement (test infrastructure; built by oracle/Makefile)
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("AK_OFFLOAD_ARCH", "gfx950")


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=cwd)


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_synth(force=False):
    src = os.path.join(CSRC, "synth.c")
    out = os.path.join(HERE, "_synth.so")
    if force or _stale(out, [src]):
        _run(["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", "-o", out, src])
    return out


def build_pylist(force=False):
    """The drop-in list API's host plumbing (CPython extension: list[str] packing, id lists)."""
    import sysconfig
    src = os.path.join(CSRC, "ak_pylist.c")
    out = os.path.join(HERE, "_pylist" + sysconfig.get_config_var("EXT_SUFFIX"))
    if force or _stale(out, [src]):
        _run(["gcc", "-O2", "-fPIC", "-shared", "-I", sysconfig.get_paths()["include"], "-o", out, src])
    return out


def hip_sources():
    names = sorted(os.listdir(CSRC))
    srcs = [os.path.join(CSRC, n) for n in names if n.endswith((".hip", ".h", ".hpp", ".cpp"))]
    srcs += [os.path.join(CSRC, "gen", n) for n in sorted(os.listdir(os.path.join(CSRC, "gen")))]
    srcs.append(os.path.join(ROOT, "include", "akshar.h"))
    return srcs


def _deps(src, seen=None):
    """src plus every quoted #include it reaches (include dirs: csrc/, include/)."""
    seen = set() if seen is None else seen
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    with open(src, errors="replace") as f:
        for inc in re.findall(r'#include\s+"([^"]+)"', f.read()):
            for d in (os.path.dirname(src), CSRC, os.path.join(ROOT, "include")):
                cand = os.path.join(d, inc)
                if os.path.exists(cand):
                    _deps(cand, seen)
                    break
    return seen


# per-TU code-generation flags. ak_k_bpe_tiles.hip: without machine LICM the tile kernel keeps its
# per-lane constants and addresses in-loop (rematerialised) and fits the 64 VGPRs of 8 waves/SIMD
# with no scratch spills (with it: 20 VGPRs spilled to scratch in every tile's prologue). The SPM
# and row-tile kernels measured faster WITH machine LICM (A/B on MI355X, tools/gpu_iter.sh AB_VARIANTS: cfg3
# fused analyze 66.8 vs 60.9 GB/s), so only the BPE TU takes the flag.
# ak_k_spm_tiles.hip: passes D2 / N's per-char predicates as bitwise expressions (AK_D2_BITWISE,
# ak_tile.h): -1.2 % SentencePiece kernel time, but +2.7 % for the BPE TU (A/B on MI355X,
# profiles/r06l_ab_d2_bitwise.jsonl), so only the SPM TU takes it.
TU_FLAGS = {"ak_k_bpe_tiles.hip": ["-mllvm", "-disable-machine-licm"], "ak_k_spm_tiles.hip": ["-DAK_D2_BITWISE=1"]}


def build_hip(force=False, jobs=None):
    """Compile each stale .hip TU (own source or any header it reaches changed) to an object in
    parallel, then link the shared library."""
    from concurrent.futures import ThreadPoolExecutor
    out = os.path.join(HERE, "_akshar_hip.so")
    srcs = [os.path.join(CSRC, n) for n in sorted(os.listdir(CSRC)) if n.endswith((".hip", ".cpp"))]
    if not (force or _stale(out, hip_sources())):
        return out
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = [hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
              "-I", CSRC, "-Wall", "-Wno-unused-function"]
    if os.environ.get("AK_HIP_REMARKS"):  # per-kernel VGPR / SGPR / LDS / scratch / occupancy report
        common.append("-Rpass-analysis=kernel-resource-usage")
    objs = []
    cmds = []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, sorted(_deps(src))):
            cmds.append(common + TU_FLAGS.get(os.path.basename(src), []) + ["-c", "-o", obj, src])
    jobs = jobs or min(max(len(cmds), 1), max(1, (os.cpu_count() or 4)), 16)
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(_run, c) for c in cmds]:
            f.result()
    _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out] + objs)
    return out


def build_variant(name, defines=(), tu_flags=None, only=None, csrc=None):
    """Development aid: the library built with extra -D defines / per-TU flags into
    akshar_amd/_variants/<name>.so (selected at run time by AK_LIB_VARIANT=<name>). only: the TU
    names compiled with the defines; every other TU links the default build's object. csrc: another
    source directory (an earlier commit's csrc/, for an A/B on one box)."""
    global TU_FLAGS
    CSRC = csrc or globals()["CSRC"]
    if only:
        build_hip()
    objdir = os.path.join(ROOT, "build", "variants", name)
    os.makedirs(objdir, exist_ok=True)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = [hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include"),
              "-I", CSRC, "-Wall", "-Wno-unused-function"] + ["-D" + d for d in defines]
    flags = TU_FLAGS if tu_flags is None else tu_flags
    from concurrent.futures import ThreadPoolExecutor
    srcs = [os.path.join(CSRC, n) for n in sorted(os.listdir(CSRC)) if n.endswith((".hip", ".cpp"))]
    objs = [os.path.join(objdir if not only or os.path.basename(s) in only else os.path.join(ROOT, "build", "hip"),
                         os.path.basename(s) + ".o") for s in srcs]
    cmds = [common + flags.get(os.path.basename(s), []) + ["-c", "-o", o, s] for s, o in zip(srcs, objs)
            if not only or os.path.basename(s) in only]
    with ThreadPoolExecutor(min(16, os.cpu_count() or 4)) as ex:
        for f in [ex.submit(_run, c) for c in cmds]:
            f.result()
    os.makedirs(os.path.join(HERE, "_variants"), exist_ok=True)
    out = os.path.join(HERE, "_variants", name + ".so")
    _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", out] + objs)
    return out


def build_oracle(force=False):
    oracle = os.path.join(ROOT, "oracle")
    args = ["make", "-s", "-C", oracle]
    if force:
        args.append("-B")
    _run(args)
    return os.path.join(oracle, "_oracle.so")


def build_all(force=False):
    build_synth(force)
    build_pylist(force)
    build_oracle(force)
    build_hip(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
