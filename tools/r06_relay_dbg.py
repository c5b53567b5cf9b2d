"""Debug: the golden relay cases under the stamp variants (pipeline, status / event mismatches)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from shadow_amd.relay import Relay
    from shadow_amd.routing import Engine
    for knobs in ({}, {"RELAY_STAMP": 6}, {"RELAY_FORCE_V3": 1}, {"RELAY_FORCE_V3": 1, "RELAY_STAMP": 6}):
        eng = Engine(0)
        for k, v in knobs.items():
            eng.set_knob(k, v)
        for case in json.load(open(os.path.join(ROOT, "tests", "golden", "relay_cases.json"))):
            rng = np.asarray([[int(v) for v in r] for r in case["rng"]], np.uint64).reshape(-1, 4)
            rl = Relay(case["host_node"], rng, np.asarray([int(v) for v in case["next_id"]], np.uint64),
                       np.asarray(case["lat"], np.uint64), np.asarray(case["loss_bits"], np.uint32).view(np.float32),
                       engine=eng)
            r = rl.round(case["src_off"], np.asarray([int(v) for v in case["send_time"]], np.uint64),
                         case["dst_host"], case["payload"], int(case["round_end"]), int(case["sim_end"]),
                         int(case["bootstrap_end"]))
            e = case["expect"]
            st = np.asarray(e["status"], np.uint8)
            bad = np.flatnonzero(r.status != st)
            print(knobs, case["name"], "pipe", rl.last_pipeline(), "n", len(st), "status bad", len(bad),
                  "first", bad[:6].tolist(), "got", r.status[bad[:6]].tolist(), "want", st[bad[:6]].tolist(),
                  "ev_off ok", r.ev_off.tolist() == e["ev_off"], flush=True)
        eng.close()


if __name__ == "__main__":
    main()
