"""Runs bench.py's N > 1 legs (relay_check_sharded, equeue_leg_sharded, the C2 check) at world
size 1 over the RCCL communicator, so their Python and ABI plumbing is exercised on a one-GPU
box before the driver's multi-GPU run."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shadow_amd import dist as D  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

eng = Engine(0)
D.comm_init_rccl(eng)
r = bench.routing_leg(eng, 1, 0, 3, 1)
inputs = bench.relay_inputs()
rl = bench.relay_leg(eng, 1, 0, 2, 1, r["lat"], r["loss"], inputs=inputs)
out = {"relay_check": bench.relay_check_sharded(eng, 1, 0, rl, r["lat"], r["loss"]),
       "equeue_sharded": bench.equeue_leg_sharded(eng, 1, 0, rl, r["lat"], r["loss"])}
print(json.dumps(out), flush=True)
eng.close()
