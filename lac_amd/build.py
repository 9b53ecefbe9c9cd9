"""Build liblac.so in-tree for gfx950:  python -m lac_amd.build [--force]

The library is four translation units (csrc/lac_api.hip, lac_encode.hip,
lac_decode.hip, lac_logits.hip) over shared headers (csrc/*.h, include/*.h),
compiled in parallel to objects under csrc/_obj/ and linked into lac_amd/liblac.so.
An object is rebuilt when its source or any header is newer.  Variants for A/B
runs: build(out=..., extra=("-DLAC_...=0",)) compiles into their own object
directory."""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
# every header the kernels can #include: csrc/*.h and include/*.h, so a header edit rebuilds all
HEADERS = [*sorted(glob.glob(os.path.join(CSRC, "*.h"))), *sorted(glob.glob(os.path.join(REPO, "include", "*.h")))]
DEPS = [*SRCS, *HEADERS]
OUT = os.path.join(HERE, "liblac.so")
ARCH = os.environ.get("LAC_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"]


def _incs():
    return ["-I", os.path.join(REPO, "include"), "-I", CSRC]


def compile_command(src, obj, extra=()):
    return ["hipcc", *FLAGS, *_incs(), *extra, "-c", src, "-o", obj]


def link_command(objs, out=OUT):
    return ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, out: str = OUT, extra=(), jobs: int = 0) -> str:
    tag = "" if not extra else "_" + "_".join(e.lstrip("-").replace("=", "").replace("/", "") for e in extra)
    objdir = os.path.join(CSRC, "_obj" + tag)
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s)[:-4] + ".o") for s in SRCS]
    todo = [(s, o) for s, o in zip(SRCS, objs) if force or _stale(o, [s, *HEADERS])]
    if todo:
        cmds = [compile_command(s, o, extra) for s, o in todo]
        if verbose:
            for c in cmds:
                print(" ".join(c), flush=True)
        n = jobs or min(len(cmds), max(1, min(os.cpu_count() or 1, 16)))
        with ThreadPoolExecutor(n) as ex:
            procs = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds))
        bad = [(c, p) for c, p in zip(cmds, procs) if p.returncode]
        for c, p in zip(cmds, procs):
            if p.stderr and (verbose or p.returncode):
                sys.stderr.write(p.stderr)
        if bad:
            raise subprocess.CalledProcessError(bad[0][1].returncode, bad[0][0])
    if force or todo or _stale(out, objs):
        cmd = link_command(objs, out)
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    # python -m lac_amd.build [--force] [--out PATH] [-DNAME=VALUE ...]  (variants: own objects, own .so)
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else OUT
    build(force="--force" in args, out=out, extra=tuple(a for a in args if a.startswith("-D")))
