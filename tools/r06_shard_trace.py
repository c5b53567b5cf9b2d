"""Per-phase timeline of the relay rounds in a rocprofv3 trace of tools/sharded_round_probe.py
(`--kernel-trace --memory-copy-trace`): the probe runs R + 2 plain device rounds, R + 2 sharded
rounds at world size 1, then R + 2 rounds of two in-process ranks.  Every round starts with its
K0 (`relay_draws`, one per rank), so the trace splits into the three legs' rounds; for each leg
this prints the median-span round as a timeline -- each kernel or copy with its start offset,
its duration and the idle gap before it (a gap is host time: a read-back's round trip, the
communicator's waits, launch latency).

    python tools/r06_shard_trace.py <rocprof output dir> [R]
"""
import csv
import os
import statistics
import sys


def load(d):
    ev = []
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"]))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        with open(p) as f:
            for r in csv.DictReader(f):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                          "C " + r["Direction"].replace("MEMORY_COPY_", "").lower()))
    ev.sort()
    return ev


def short(name):
    n = name.split("(")[0]
    for pre in ("K void shd::", "K shd::", "K void ", "K "):
        if n.startswith(pre):
            n = "K " + n[len(pre):]
            break
    return n[:60]


def torch_op(name):
    return "at::" in name or "elementwise" in name or "vectorized" in name


def main():
    d = sys.argv[1]
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ev = [e for e in load(d) if not torch_op(e[2])]
    starts = [i for i, e in enumerate(ev) if "relay_draws" in e[2]]
    per_leg = [R + 2, R + 2, 2 * (R + 2)]
    if len(starts) < sum(per_leg):
        print(f"expected {sum(per_leg)} K0 launches, found {len(starts)}")
        return 1
    legs, at = [], 0
    for name, k, step in (("plain device round", per_leg[0], 1), ("sharded, world 1", per_leg[1], 1),
                          ("sharded, two in-process ranks", per_leg[2], 2)):
        rounds = []
        for j in range(at + 2 * step, at + k, step):   # the first two rounds are warm-up
            a = starts[j]
            b = starts[j + step] if j + step < len(starts) else len(ev)
            rounds.append(ev[a:b])
        at += k
        legs.append((name, rounds))
    for name, rounds in legs:
        spans = [max(e[1] for e in r) - r[0][0] for r in rounds]
        med = statistics.median(spans)
        r = rounds[min(range(len(rounds)), key=lambda i: abs(spans[i] - med))]
        t0 = r[0][0]
        busy = sum(e[1] - e[0] for e in r)
        print(f"== {name}: median span {med / 1e3:.1f} us over {len(rounds)} rounds (device busy {busy / 1e3:.1f} us "
              f"in the round shown)")
        prev_end = t0
        for s, e, n in r:
            gap = s - prev_end
            print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  gap {gap / 1e3:6.1f}  {short(n)}")
            prev_end = max(prev_end, e)
    return 0


if __name__ == "__main__":
    sys.exit(main())
