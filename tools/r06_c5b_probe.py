"""C5b leg alone, with progress markers (python -X faulthandler tools/r06_c5b_probe.py)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    import bench
    from shadow_amd.routing import Engine
    eng = Engine(0)
    t0 = time.time()
    print("engine open", flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "cpu":
        r = bench.routing_leg(eng, 1, 0, 2, 1)
        print("routing leg", time.time() - t0, flush=True)
        cb, fa, ti = bench.cpu_baseline_routing(r["el"], budget_s=2.0)
        print("cpu baseline", json.dumps(cb)[:300], flush=True)
        return
    res = bench.c5b_leg(eng, steps=3, warmup=1, cpu=True)
    print(json.dumps(res), flush=True)
    print("done", time.time() - t0, flush=True)


if __name__ == "__main__":
    main()
