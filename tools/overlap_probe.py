"""Does a side-stream kernel run beside the persistent global-label SSSP kernel?  (One GPU; the
stand-in for RCCL's send/recv kernels during shd_routing_run_sharded's chunked exchange.)

Queues copy kernels on a torch side stream, then builds C4 rows on the engine's stream, with
SHD_SSSP_RESERVE slots of the kernel left unlaunched (argv[1], default 0).  Run under
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl<R> -o run -- python tools/overlap_probe.py <R>
and reduce with  python tools/overlap_probe.py --trace gpurun_out/ovl<R>/run_kernel_trace.csv
"""
import csv
import os
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--trace":
    rows = list(csv.DictReader(open(sys.argv[2])))
    last = max((r for r in rows if "sssp_global_group" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    s0, s1 = int(last["Start_Timestamp"]), int(last["End_Timestamp"])   # the timed build (not the warm-up)
    side = [r for r in rows if ("elementwise" in r["Kernel_Name"] or "copyBuffer" in r["Kernel_Name"])
            and int(r["Start_Timestamp"]) > s0 - 50_000_000]
    inside = [r for r in side if int(r["Start_Timestamp"]) < s1 and int(r["End_Timestamp"]) > s0]
    ends_inside = [r for r in inside if int(r["End_Timestamp"]) <= s1]
    after = [r for r in side if int(r["Start_Timestamp"]) >= s1]
    print(f"sssp {(s1 - s0) / 1e6:.2f} ms; side copies overlapping it: {len(inside)}, finished inside it: "
          f"{len(ends_inside)}, started after it ended: {len(after)} (of {len(side)})")
    sys.exit(0)

os.environ["SHD_SSSP_RESERVE"] = sys.argv[1] if len(sys.argv) > 1 else "0"
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import prepare, run_rows  # noqa: E402
from shadow_amd import synth  # noqa: E402
from shadow_amd.routing import Engine  # noqa: E402

eng = Engine(0)
n = prepare(eng, synth.barabasi_albert(50_000, 4, 3))
rows = 4096
lat = torch.empty((rows, n), dtype=torch.int64, device="cuda")
loss = torch.empty((rows, n), dtype=torch.float32, device="cuda")
a = torch.empty(64 << 20, dtype=torch.float32, device="cuda")
b = torch.empty_like(a)
run_rows(eng, 3, 0, rows, lat, loss)   # warm-up
side = torch.cuda.Stream()
torch.cuda.synchronize()
with torch.cuda.stream(side):
    for _ in range(40):
        b.copy_(a)
run_rows(eng, 3, 0, rows, lat, loss)
torch.cuda.synchronize()
print(f"reserve={os.environ['SHD_SSSP_RESERVE']} ms_main={eng.last_info()['ms_main']:.2f}")
