"""Build the in-tree native library shadow_amd/libshd_accel.so for gfx950 (hipcc, no JIT)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", f) for f in ("routing.hip", "blocked.hip", "relay.hip", "api.cpp", "gml.cpp", "codel.hip", "tbucket.hip")]
OUT = os.path.join(HERE, "libshd_accel.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # Rust never contracts 1-(1-p)*(1-e) into an FMA: keep every f32 op separately rounded
         "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SRC + [os.path.join(HERE, "csrc", h) for h in os.listdir(os.path.join(HERE, "csrc"))
                  if h.endswith(".h")] + [os.path.join(ROOT, "include", "shd_accel.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if force or needs_build():
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, *SRC, "-o", OUT + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
