"""Debug: which path entries did the stamp use?  golden relay1 under the default stamp."""
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
    case = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "relay_cases.json"))) if c["name"] == "relay1"][0]
    eng = Engine(0)
    if len(sys.argv) > 1:
        eng.set_knob("RELAY_STAMP", int(sys.argv[1]))
    rng = np.asarray([[int(v) for v in r] for r in case["rng"]], np.uint64).reshape(-1, 4)
    lat = np.asarray(case["lat"], np.uint64)
    nn = int(round(len(lat) ** 0.5)) if lat.ndim == 1 else lat.shape[0]
    lat = lat.reshape(nn, nn)
    hn = np.asarray(case["host_node"], np.uint32)
    rl = Relay(hn, rng, np.asarray([int(v) for v in case["next_id"]], np.uint64), lat,
               np.asarray(case["loss_bits"], np.uint32).view(np.float32).reshape(nn, nn), engine=eng)
    st = np.asarray([int(v) for v in case["send_time"]], np.uint64)
    so = np.asarray(case["src_off"], np.int64)
    r = rl.round(case["src_off"], st, case["dst_host"], case["payload"], int(case["round_end"]), int(case["sim_end"]),
                 int(case["bootstrap_end"]))
    src = np.repeat(np.arange(len(so) - 1), np.diff(so))
    dst = np.asarray(case["dst_host"], np.int64)
    re_ = int(case["round_end"])
    print("nodes", nn, "hosts", len(hn), "host_node", hn.tolist())
    bad = 0
    for ev_i in range(len(r.ev_pkt)):
        p = int(r.ev_pkt[ev_i])
        d = int(r.ev_deliver[ev_i])
        used = d - int(st[p])
        true = int(lat[hn[src[p]], hn[dst[p]]])
        if d != re_ and used != true:
            cand = [(a, b) for a in range(nn) for b in range(nn) if int(lat[a, b]) == used]
            if bad < 25:
                print("pkt", p, "src", int(src[p]), "srcnode", int(hn[src[p]]), "dstnode", int(hn[dst[p]]), "used", used,
                      "true", true, "candidates", cand[:6])
            bad += 1
    print("latency mismatches", bad, "of", len(r.ev_pkt))


if __name__ == "__main__":
    main()
