"""Reduce tools/pmc_traffic.sh output to profiles/pmc_traffic.json (per-launch HBM bytes).

FETCH_SIZE / WRITE_SIZE are in KB.  The read counter is calibrated on tools/bw_probe's kernel kA
(24 B read + 21 B written per packet, 10M packets, batch order): the measured read factor is
applied to every kernel's FETCH_SIZE (MI355X guide: gfx950 tallies wide reads at half), the
write counter is taken as is (kA's writes come out within a few percent of the byte count).
  routing: sssp_lds_group, one launch (the C2 build's dominant kernel)
  relay:   every relay kernel of one round (pipeline 7: K0 draws, bin histogram + scans, K1
           stamp, K4 bin sort; pipeline 3: K0, K1, K2 radix passes, K3 offsets, K4 segment
           sorts), summed and divided by the number of rounds
"""
import csv
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_traffic"
dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"


def load(run, c):
    acc = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, f"{run}_{c}", "run_counter_collection.csv"))):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1e3)   # KB -> bytes
    return acc


pf, pw = load("probe", "FETCH_SIZE"), load("probe", "WRITE_SIZE")
ka = [k for k in pf if k.startswith("kA(")][0]
n_pkt = 10_000_000
read_factor = 24.0 * n_pkt / (sum(pf[ka]) / len(pf[ka]))
write_factor = 21.0 * n_pkt / (sum(pw[ka]) / len(pw[ka]))
def per_launch(run, sel):
    bf, bw = load(run, "FETCH_SIZE"), load(run, "WRITE_SIZE")
    out = {}
    for k in bf:
        if sel(k):
            out[k] = (read_factor * sum(bf[k]) / len(bf[k]), sum(bw[k]) / len(bw[k]), len(bf[k]))
    return out


sssp = per_launch("bench", lambda k: "sssp_lds_group" in k)
r_read = sum(v[0] * v[2] for v in sssp.values()) / sum(v[2] for v in sssp.values())
r_write = sum(v[1] * v[2] for v in sssp.values()) / sum(v[2] for v in sssp.values())
relay_sel = ("relay_draws", "relay_stamp", "rocprim", "bucket_offsets", "segment_sort", "relay_bin_hist",
             "bin_col_scan", "bin_base_scan", "bin_sort_v7", "red_init")
relay = per_launch("relay", lambda k: any(s in k for s in relay_sel))
rounds = sum(v[2] for k, v in relay.items() if "relay_stamp" in k)
rel_read = sum(v[0] * v[2] for v in relay.values()) / rounds
rel_write = sum(v[1] * v[2] for v in relay.values()) / rounds
def one_kernel(run, sel):
    """(read, write, launches) of the kernel matching sel in a run, or None when the run is absent"""
    if not os.path.exists(os.path.join(src, f"{run}_FETCH_SIZE")):
        return None
    d = per_launch(run, sel)
    n = sum(v[2] for v in d.values())
    if not n:
        return None
    return (sum(v[0] * v[2] for v in d.values()) / n, sum(v[1] * v[2] for v in d.values()) / n, n)


c3 = one_kernel("c3", lambda k: "sssp_lds_group" in k)
c4 = one_kernel("c4", lambda k: "sssp_global_group" in k)
doc = {
    "source": "tools/pmc_traffic.sh + tools/pmc_traffic.py (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE in "
              "separate runs: routing from bench.py --no-relay (C2 builds), relay from tools/relay_only.py 10 "
              "(C5 rounds, pipeline 7, no counters))",
    "read_factor": read_factor, "write_factor_measured": write_factor,
    "routing": r_read + r_write,
    "routing_detail": {"kernel": "sssp_lds_group", "read_bytes": r_read, "write_bytes": r_write},
    "relay": rel_read + rel_write,
    "relay_detail": {"per": "round", "rounds": rounds, "read_bytes": rel_read, "write_bytes": rel_write,
                     "kernels": {k.split("(")[0][:80]: {"launches": v[2], "read_bytes": v[0],
                                                        "write_bytes": v[1]}
                                 for k, v in relay.items()}},
}
for name, v, what in (("c3", c3, "sssp_lds_group on the whole C3 build (AUTO = delta buckets)"),
                      ("c4", c4, "sssp_global_group on one full C4 build (global-label delta-stepping)")):
    if v:
        doc[name] = v[0] + v[1]
        doc[name + "_detail"] = {"kernel": what, "read_bytes": v[0], "write_bytes": v[1], "launches": v[2],
                                 "note": "read factor calibrated on streaming reads; these kernels' reads are "
                                         "random 8-byte label accesses (an uncalibrated width, guide HBM section)"}
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump(doc, open(dst, "w"), indent=1)
print(json.dumps({k: doc.get(k) for k in ("read_factor", "write_factor_measured", "routing", "relay", "c3", "c4")}))

# the raw per-kernel means behind the numbers above (KB per launch, uncalibrated)
if len(sys.argv) > 3:
    with open(sys.argv[3], "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["run", "counter", "kernel", "launches", "mean_KB"])
        for run in ("probe", "bench", "relay", "c3", "c4"):
            if not os.path.exists(os.path.join(src, f"{run}_FETCH_SIZE")):
                continue
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                for k, v in sorted(load(run, c).items()):
                    wr.writerow([run, c, k.split("(")[0], len(v), round(sum(v) / len(v) / 1e3, 1)])
