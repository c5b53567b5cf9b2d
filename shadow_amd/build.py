"""Build the in-tree native library shadow_amd/libshd_accel.so for gfx950 (hipcc, no JIT).

Every source compiles to its own object in parallel (build/obj/), then one link."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", f) for f in ("routing.hip", "blocked.hip", "relay.hip", "api.cpp", "gml.cpp",
                                                "codel.hip", "tbucket.hip", "comm.cpp", "equeue.hip",
                                                "hosts.cpp", "rounds.hip", "flush.hip")]
OUT = os.path.join(HERE, "libshd_accel.so")
OBJ = os.path.join(HERE, "build", "obj")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # Rust never contracts 1-(1-p)*(1-e) into an FMA: keep every f32 op separately rounded
         "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"),
         "-I", "/opt/rocm/include"]
LIBS = ["-L/opt/rocm/lib", "-lrccl", "-ldl", "-lpthread"]


def _deps():
    return [os.path.join(HERE, "csrc", h) for h in os.listdir(os.path.join(HERE, "csrc"))
            if h.endswith(".h")] + [os.path.join(ROOT, "include", "shd_accel.h")]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in SRC + _deps())


def _obj(src):
    return os.path.join(OBJ, os.path.basename(src) + ".o")


def build(force: bool = False, verbose: bool = True) -> str:
    if not (force or needs_build()):
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    newest_dep = max(os.path.getmtime(d) for d in _deps())

    def compile_one(src):
        o = _obj(src)
        if not force and os.path.exists(o) and os.path.getmtime(o) > max(os.path.getmtime(src), newest_dep):
            return
        cmd = ["/opt/rocm/bin/hipcc", *FLAGS, "-c", src, "-o", o + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(o + ".tmp", o)

    jobs = min(len(SRC), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, SRC))
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *map(_obj, SRC),
           *LIBS, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
