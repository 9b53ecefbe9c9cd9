"""Build liblac.so in-tree for gfx950:  python -m lac_amd.build"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "lac_kernels.hip")
# every header the kernels can #include: csrc/*.h and include/*.h (lac_tail.h,
# lac_q1_table.h, ...), so a header edit always rebuilds
DEPS = [SRC, *sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))), *sorted(glob.glob(os.path.join(REPO, "include", "*.h")))]
OUT = os.path.join(HERE, "liblac.so")
ARCH = os.environ.get("LAC_OFFLOAD_ARCH", "gfx950")


def command(out=OUT, extra=()):
    return ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-I", os.path.join(REPO, "include"), "-I", os.path.join(HERE, "csrc"),
            *extra, SRC, "-o", out]


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in DEPS):
        return OUT
    cmd = command()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
