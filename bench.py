#!/usr/bin/env python3
"""Benchmark: APSP node-pairs/s (routing build) + packets relayed/s per round (relay).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Headline (``value``): one step is one routing build of BASELINE config 2 (1000-node complete GML
graph, 1000 used nodes) from the device-resident arc CSR to the full 1000 x 1000 (latency u64,
loss f32) table resident in HBM.  At N > 1 the source rows are sharded over the ranks (no
collective inside the SSSP) and the table is all-gathered over RCCL so every rank ends with the
full table; the timed region includes that all-gather (strong scaling: the graph is fixed).

Side legs, each its own JSON object in the same line:
  * ``relay`` -- C5: one round of 100k hosts / 10M packets per step (stamp + loss draw + bucket
    by destination + per-destination sort), inputs resident in HBM.  At N > 1 the hosts are
    sharded by id, every rank stamps its own sources, and the engine exchanges the events over
    its RCCL communicator and merges them per destination (strong scaling: the round is fixed).
  * ``c3`` (N = 1) -- the 10k-node sparse graph: label-correcting SSSP vs delta-stepping vs the
    blocked min-plus APSP, all bit-identical; the blocked kernel's VALU roofline.
  * ``c4`` -- the 50k-node graph, source rows sharded over the ranks, global-label SSSP
    (delta-stepping) + the engine's RCCL all-gather of the 30 GB table (on by default).
  * ``routing_e2e`` / ``relay.e2e_host_buffers`` -- SURVEY 8(d)'s end-to-end figures (host
    buffers in and out, PCIe included); ``relay.equeue`` -- relay + device event-queue merge.
Rank 0 prints ONE JSON line.  Timing: barrier + device sync on both sides of exactly K steps,
max over ranks.  The CPU baselines (rank 0, N = 1) time the C restatement of the reference
(oracle/c) on bounded samples of the same workloads.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "APSP node-pairs/s + packets relayed/s per round, 1/2/4/8 MI355X"
# integer VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md chip table)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
HBM_PEAK_GBS = 8000.0
RELAY_BYTES_PER_PACKET = 84   # 24 rec + 12 path + 24 event + 24 sort r/w
RELAY_BYTES_PER_HOST = 80     # RNG state + event id, read + write


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# SHD_BENCH_REHEARSAL=1: every rank on GPU 0, torch.distributed over gloo and the engine's host
# transport (shd_comm_init_host) instead of RCCL -- a rehearsal of the N > 1 code paths (sharding,
# exchanges, checks) on a one-GPU box; its times are not scaling numbers (the ranks share one GPU).
REHEARSAL = os.environ.get("SHD_BENCH_REHEARSAL", "") == "1"
_DIST_DEV = "cuda"   # where the bench's own reductions live (cpu under gloo)


def dist_setup(n_gpus):
    global _DIST_DEV
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    if REHEARSAL:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if REHEARSAL:
            dist.init_process_group("gloo")
            _DIST_DEV = "cpu"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier_sync(world):
    import torch
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_DIST_DEV)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks_ok(ok, world):
    """True iff every rank's check passed (MIN over the ranks)."""
    if world == 1:
        return bool(ok)
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_DIST_DEV)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def table_checksum(lat, loss):
    """Order-sensitive 64-bit checksum of a (lat u64, loss f32) table (host arrays)."""
    w = np.arange(1, lat.size + 1, dtype=np.uint64).reshape(lat.shape)
    return int(((lat * w).sum(dtype=np.uint64) ^ (loss.view(np.uint32).astype(np.uint64) * w).sum(dtype=np.uint64)))


def load_pmc(name):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        return json.load(open(p)).get(name)
    return None


TIME_EVERY = 4   # routing builds per timed one (shd_routing_set_timing)


def prepare(eng, el):
    from shadow_amd import _native as N
    from shadow_amd.routing import NetworkGraph
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    n = g.n_nodes
    used = np.arange(n, dtype=np.uint32)
    cg = g._cgraph()
    err = N.Error()
    N.check(eng.lib.shd_routing_prepare(eng.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST,
                                        C.byref(err)), "prepare", err)
    return n


def run_rows(eng, algo, rb, re, lat, loss):
    from shadow_amd import _native as N
    err = N.Error()
    N.check(eng.lib.shd_routing_run(eng.ctx, algo, rb, re, N.ptr(lat), N.ptr(loss), C.byref(err)),
            "shd_routing_run", err)


def sharded_build(eng, world, rank, n, algo, steps, warmup, keep=False, gather=True):
    """One step = the routing build of all n rows.  N = 1: every row on this GPU.  N > 1: this
    rank's source rows, then (gather=True) the engine's RCCL all-gather of the table
    (shd_routing_run_sharded) so every rank ends with all of it."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd import dist as D
    per = (n + world - 1) // world
    rb, re = D.shard_range(n, world, rank) if world > 1 else (0, n)
    rows = world * per if (world > 1 and gather) else (re - rb)
    lat = torch.empty((max(rows, 1), n), dtype=torch.int64, device="cuda")
    loss = torch.empty((max(rows, 1), n), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    # the call's arguments are made once: the timed loop holds the build calls and nothing else
    lat_p, loss_p, err = N.ptr(lat), N.ptr(loss), N.Error()
    run = eng.lib.shd_routing_run

    def step():
        if world > 1 and gather:
            D.routing_run_sharded(eng, algo, lat, loss)
        elif re > rb:
            st = run(eng.ctx, algo, rb, re, lat_p, loss_p, C.byref(err))
            if st != 0:
                N.check(st, "shd_routing_run", err)

    for _ in range(warmup):
        step()
    barrier_sync(world)
    infos = []
    # the dominant kernel is timed (HIP events on its dispatch) on every 4th step of the timed
    # region (each timed build pays a few microseconds of queue gap for its events); the build
    # info is read after those steps only
    eng.lib.shd_routing_set_timing(eng.ctx, TIME_EVERY)
    t0 = time.perf_counter()
    for i in range(steps):
        step()
        if i % TIME_EVERY == 0 or i == steps - 1:
            infos.append(eng.last_info())
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    eng.lib.shd_routing_set_timing(eng.ctx, 1)
    built = n if (world > 1 and gather and D.routing_replicates(n, world)) else re - rb
    out = dict(dt=dt, ms_per_step=dt / steps * 1e3, rows=built, rb=rb, infos=infos,
               kernel_ms=float(np.mean([i["ms_main"] for i in infos if i["ms_main"] >= 0] or [0.0])))
    if keep:
        k = n if (world == 1 or gather) else 0
        out["lat"] = lat[:k].cpu().numpy().view(np.uint64)
        out["loss"] = loss[:k].cpu().numpy()
    out["lat_dev"], out["loss_dev"] = lat, loss
    return out


def routing_leg(eng, world, rank, steps, warmup):
    from shadow_amd import _native as N
    from shadow_amd import synth
    el = synth.complete_graph(1000, 1)
    n = prepare(eng, el)
    r = sharded_build(eng, world, rank, n, N.ALGO_AUTO, steps, warmup, keep=True)
    del r["lat_dev"], r["loss_dev"]
    info = r["infos"][-1]
    kernel_ms = max_over_ranks(r["kernel_ms"], world)
    ops_per_launch = 2.0 * r["rows"] * info["arcs"]      # one add + one min per arc per source row
    achieved = ops_per_launch / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
    r.update(n=n, arcs=info["arcs"], kernel_ms=kernel_ms, achieved=achieved, algo=info["algo_used"],
             arcs_kept=info["arcs_kept"], el=el)
    return r


def routing_e2e(eng, el, reps=5):
    """SURVEY 8(d)'s end-to-end figure: shd_routing_build from the host graph arrays (validation,
    CSR build, H2D) to the whole table in pinned host memory (D2H)."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd.routing import NetworkGraph
    g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
    n = g.n_nodes
    used = np.arange(n, dtype=np.uint32)
    lat = torch.empty((n, n), dtype=torch.int64).pin_memory()
    loss = torch.empty((n, n), dtype=torch.float32).pin_memory()
    cg = g._cgraph()
    err = N.Error()

    def once():
        N.check(eng.lib.shd_routing_build(eng.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST, N.ALGO_AUTO,
                                          0, n, C.c_void_p(lat.data_ptr()), C.c_void_p(loss.data_ptr()),
                                          C.byref(err)), "shd_routing_build", err)
    once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    ms = (time.perf_counter() - t0) / reps * 1e3
    return {"ms_per_build": ms, "node_pairs_per_s": n * n / (ms * 1e-3),
            "what": "shd_routing_build: host graph arrays -> validation + CSR + H2D -> build -> D2H of the "
                    "12 MB table into pinned host memory"}


def sssp_roofline(n, arcs, V, ms):
    """SURVEY 8(d) sparse-SSSP roofline: n * (E * 8 + V * 12) bytes per build over HBM."""
    b = float(n) * (arcs * 8 + V * 12)
    ach = b / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "work": "n * (E * 8 + V * 12) B: one 8-byte label read per arc relaxation + the 12-byte table write "
                    "(SURVEY 8(d))", "bytes": b}


def cpu_info():
    """The host the CPU baselines ran on (CPU model, nproc, threads used)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff}


TIDY_WHAT = "tidy: the same Dijkstra, used-node bitmap instead of Vec::contains, dense table written directly"
FAITHFUL_WHAT = "faithful: heap Dijkstra + Vec::contains filter + HashMap materialisation (graph/mod.rs:192-230)"


def cpu_rows_baseline(el, rows, n_total, what):
    """The C restatement on a contiguous sample of source rows, all host cores, extrapolated to
    the whole build: the faithful variant (value) and the tidy one beside it."""
    from oracle import corc
    used = np.arange(el.n_nodes, dtype=np.uint32)
    threads = corc.max_threads()
    k = rows[1] - rows[0]
    out = {}
    for name, variant in (("faithful", corc.FAITHFUL), ("tidy", corc.TIDY)):
        t0 = time.perf_counter()
        code, lat, loss, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed,
                                          used, variant=variant, threads=threads, rows=rows)
        dt = time.perf_counter() - t0
        out[name] = (n_total * n_total / (dt * n_total / k), dt, lat, loss)
    v, dt, lat, loss = out["faithful"]
    tv, tdt, tlat, tloss = out["tidy"]
    cb = dict(value=v, unit="node-pairs/s", cores=threads, kind="port", variant="faithful",
              sample=f"{what}: source rows {rows[0]}-{rows[1] - 1} ({k} of {n_total}) in {dt:.2f} s, "
                     f"extrapolated x{n_total / k:.0f} ({FAITHFUL_WHAT})",
              tidy=dict(value=tv, unit="node-pairs/s", cores=threads, kind="port",
                        sample=f"the same rows in {tdt:.2f} s ({TIDY_WHAT})"), **cpu_info())
    return cb, (lat, loss), (tlat, tloss)


def cpu_bit_exact(cb, faithful, tidy, glat, gloss):
    """bit_exact_vs_gpu of both CPU variants against the GPU rows (latency and loss bits)."""
    def same(t):
        return bool(np.array_equal(t[0], glat) and np.array_equal(t[1].view(np.uint32), gloss.view(np.uint32)))
    cb["bit_exact_vs_gpu"] = same(faithful)
    cb["tidy"]["bit_exact_vs_gpu"] = same(tidy)


def c2_engines(eng, el, reps=5):
    """Every engine on the C2 graph (all rows, identical tables): what AUTO chose it against."""
    import torch
    from shadow_amd import _native as N
    n = prepare(eng, el)
    lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
    loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
    res, ref = {}, None
    for name, algo in (("auto", N.ALGO_AUTO), ("sssp", N.ALGO_SSSP), ("pruned", N.ALGO_PRUNED),
                       ("delta", N.ALGO_DELTA), ("blocked", N.ALGO_BLOCKED)):
        tot, main = [], []
        for _ in range(reps):
            run_rows(eng, algo, 0, n, lat, loss)
            i = eng.last_info()
            tot.append(i["ms_total"])
            main.append(i["ms_main"])
        h = (int(lat.sum().item()), int(loss.view(torch.int32).to(torch.int64).sum().item()))
        ref = ref or h
        res[name] = dict(ms_total=float(np.median(tot)), ms_main=float(np.median(main)),
                         algo_used=int(i["algo_used"]), arcs_kept=int(i["arcs_kept"]), identical_to_auto=h == ref)
        if name == "blocked":
            res[name]["ms_minplus"] = i["ms_minplus"]
    del lat, loss
    torch.cuda.empty_cache()
    return res


def c3_leg(eng, reps=2, cpu=True):
    """C3 (10k-node sparse, BA m=3): the three algorithms on the same rows, bit-identical."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd import synth
    el = synth.barabasi_albert(10_000, 3, 2)
    n = prepare(eng, el)
    lat = torch.empty((n, n), dtype=torch.int64, device="cuda")
    loss = torch.empty((n, n), dtype=torch.float32, device="cuda")
    res, ref = {}, None
    arcs = 0
    for name, algo in (("sssp", N.ALGO_SSSP), ("delta", N.ALGO_DELTA), ("blocked", N.ALGO_BLOCKED)):
        infos = []
        for _ in range(reps):
            run_rows(eng, algo, 0, n, lat, loss)
            infos.append(eng.last_info())
        i = infos[-1]
        arcs = int(i["arcs"])
        h = (int(lat.view(torch.int64).sum().item()), int(loss.view(torch.int32).to(torch.int64).sum().item()))
        ref = ref or h
        res[name] = dict(ms_total=i["ms_total"], ms_main=i["ms_main"], identical_to_sssp=h == ref)
        if name == "blocked":
            ops = 2.0 * n ** 3
            ach = ops / (i["ms_minplus"] * 1e-3) / 1e12
            res[name].update(ms_minplus=i["ms_minplus"], arcs_tight=i["arcs_kept"],
                             roofline={"bound": "valu", "achieved": ach, "peak": VALU_PEAK_TOPS,
                                       "unit": "Tops/s", "frac": ach / VALU_PEAK_TOPS,
                                       "work": "2 V^3 int ops (add + min) of the min-plus closure"})
        else:
            res[name]["roofline"] = sssp_roofline(n, arcs, n, i["ms_main"])
            if name == "delta":   # the AUTO engine's kernel: PMC bytes per launch (profiles/pmc_traffic.json)
                res[name]["roofline"]["traffic"] = load_pmc("c3")
    best = min(v["ms_total"] for v in res.values())
    out = dict(workload="C3: 10k-node Barabasi-Albert m=3 + self-loops, all 10k rows",
               nodes=n, arcs=arcs, node_pairs_per_s=n * n / (best * 1e-3), algorithms=res)
    if cpu:
        cb, fa, ti = cpu_rows_baseline(el, (0, 256), n, "C3")
        cpu_bit_exact(cb, fa, ti, lat[:256].cpu().numpy().view(np.uint64), loss[:256].cpu().numpy())
        out["cpu_baseline"] = cb
    del lat, loss
    torch.cuda.empty_cache()
    return out


def c4_leg(eng, world, rank, steps, gather=True, cpu=True):
    """C4: the 50k-node BA m=4 graph, all 50k source rows (global-label delta-stepping).  N > 1:
    rows sharded over the ranks, then the engine's RCCL all-gather of the 30 GB table (BASELINE
    config 4: "+ RCCL all-gather"); every rank ends with the whole table.  Over xGMI that moves
    (N-1)/N x 30 GB into every GPU: ~26 GB at N = 8, tens of ms at the links' rate."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd import synth
    el = synth.barabasi_albert(50_000, 4, 3)
    n = prepare(eng, el)
    gather = gather and world > 1
    r = sharded_build(eng, world, rank, n, N.ALGO_DELTA, steps, 0 if steps > 1 else 1, gather=gather)
    kernel_ms = max_over_ranks(r["kernel_ms"], world)
    how = ("source rows sharded + RCCL all-gather of the table" if gather else
           "source rows sharded, shards resident (no all-gather)" if world > 1 else "1 GPU, whole table")
    arcs = int(r["infos"][-1]["arcs"])
    out = dict(workload="C4: 50k-node Barabasi-Albert m=4 + self-loops, all 50k rows, global-label "
                        "delta-stepping SSSP, " + how,
               nodes=n, arcs=arcs, steps=steps, ms_per_build=r["ms_per_step"],
               sssp_kernel_ms_per_rank=kernel_ms, value=n * n / (r["ms_per_step"] * 1e-3),
               unit="node-pairs/s", scaling="strong", all_gather=bool(gather),
               roofline=sssp_roofline(r["rows"], arcs, n, kernel_ms))
    if world == 1:   # PMC bytes of one full-build launch (profiles/pmc_traffic.json)
        out["roofline"]["traffic"] = load_pmc("c4")
    if world > 1:   # the rank holding the last 64 rows (claimed rows of its slots) checks them
        from oracle import corc
        lo = n - 64
        lat, loss = r["lat_dev"], r["loss_dev"]
        ok = True
        if rank == (0 if gather else world - 1):
            at = lo if gather else lo - r["rb"]
            code, clat, closs, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed,
                                                np.arange(n, dtype=np.uint32), rows=(lo, n), threads=corc.max_threads())
            ok = code == "OK" and np.array_equal(clat, lat[at:at + 64].cpu().numpy().view(np.uint64)) and \
                np.array_equal(closs.view(np.uint32), loss[at:at + 64].cpu().numpy().view(np.uint32))
        out["check"] = all_ranks_ok(ok, world)
    if cpu and rank == 0 and world == 1:
        # the LAST 64 rows: the persistent kernel's slots take every row past the grid (the first
        # 2 x n_cu rows) from the row counter, so these are claimed rows, not a slot's first row
        lo = n - 64
        cb, fa, ti = cpu_rows_baseline(el, (lo, n), n, "C4")
        lat, loss = r["lat_dev"], r["loss_dev"]
        cpu_bit_exact(cb, fa, ti, lat[lo:].cpu().numpy().view(np.uint64), loss[lo:].cpu().numpy())
        cb["rows_checked"] = [lo, n]
        out["cpu_baseline"] = cb
    del r
    torch.cuda.empty_cache()
    return out


def relay_inputs():
    from shadow_amd import synth
    H, P = 100_000, 10_000_000
    start, runahead = synth.SIM_START + 10**9, 10**6
    b = synth.packet_batch(H, P, start, start + runahead, seed=4)
    return H, P, start, runahead, b, synth.c5_host_nodes(H, 1000), synth.host_rng_states(H, 1)


def _dev(a, dt):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()


def relay_leg(eng, world, rank, steps, warmup, lat_table, loss_table, counters=False, inputs=None):
    import torch
    from shadow_amd import _native as N
    from shadow_amd import dist as D
    H, P, start, runahead, b, host_node, rng0 = inputs or relay_inputs()
    nid0 = np.zeros(H, np.uint64)
    rd = (start + runahead, start + 10**12, 0)
    if world == 1:
        N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(host_node), 1000, N.ptr(lat_table),
                                        N.ptr(loss_table), N.ptr(rng0), N.ptr(nid0)), "relay_setup")
    else:
        rel = D.ShardedRelay(eng, host_node, rng0, nid0, lat_table, loss_table)
    # per-path packet counters: the reference only reads them in log_packet_counts, which is
    # never called, and the CPU baseline does not keep them either -> off in both legs; the
    # cost with them on is reported separately (counters_on_ms_per_round)
    N.check(eng.lib.shd_relay_set_counters(eng.ctx, 1 if counters else 0), "set_counters")
    if world == 1:
        d_off, d_time = _dev(b.src_off, np.int32), _dev(b.send_time, np.int64)
        d_dst, d_pay = _dev(b.dst_host, np.int32), _dev(b.payload, np.int32)
        st = torch.empty(P, dtype=torch.uint8, device="cuda")
        ev_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
        ev_deliver = torch.empty(P, dtype=torch.int64, device="cuda")
        ev_src = torch.empty(P, dtype=torch.int32, device="cuda")
        ev_seq = torch.empty(P, dtype=torch.int64, device="cuda")
        ev_pkt = torch.empty(P, dtype=torch.int32, device="cuda")
        batch = N.Batch(P, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_dst).value,
                        N.ptr(d_pay).value, None)
        out = N.RelayOut(N.ptr(st).value, N.ptr(ev_off).value, N.ptr(ev_deliver).value,
                         N.ptr(ev_src).value, N.ptr(ev_seq).value, N.ptr(ev_pkt).value, 0, 0, 0)
        rnd = N.Round(*rd)

        def step():
            N.check(eng.lib.shd_relay_round_device(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)),
                    "relay_round_device")
            return out.n_sent
    else:
        # hosts sharded by id: this rank's sources; the engine exchanges + merges the events
        lo, hi = rel.lo, rel.hi
        a, e = int(b.src_off[lo]), int(b.src_off[hi])
        d_off = _dev((b.src_off[lo:hi + 1] - b.src_off[lo]).astype(np.uint32), np.int32)
        d_time, d_dst = _dev(b.send_time[a:e], np.int64), _dev(b.dst_host[a:e], np.int32)
        d_pay = _dev(b.payload[a:e], np.int32)
        st = torch.empty(max(e - a, 1), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()

        def step():
            return rel.round_device(d_off, d_time, d_dst, d_pay, rd, st).n_sent

    for _ in range(warmup):
        step()
    barrier_sync(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        n_sent = step()
    barrier_sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world)
    pipe = C.c_int32(0)
    N.check(eng.lib.shd_relay_last_pipeline(eng.ctx, C.byref(pipe)), "last_pipeline")
    return dict(H=H, P=P, dt=dt, ms_per_step=dt / steps * 1e3, n_sent=int(n_sent), batch=b,
                pipeline=int(pipe.value), host_node=host_node, rng0=rng0, start=start, rd=rd)


C5B_HOSTS, C5B_PACKETS, C5B_SLICE_HOSTS = 100_000, 10_000_000, 10_000


def c5b_setup(eng, seed=6):
    """C5b ("to stress random gathers"): the C5 round on the C4 table.  The 50k-node
    BA graph's whole 50k x 50k table is built into the engine's resident table (no copy leaves
    the GPU) and the relay runs on it: 100k hosts, host h on node h mod 50,000, 10M sends.  At
    16 bits per host the host -> node map does not fit the stamp's LDS, so the stamp gathers the
    destinations' nodes from global memory and the path entries from the 20 GB packed table
    (relay_stamp_v6<MAP = false>), and the records still go to their destination bins (pipeline 7)."""
    from shadow_amd import _native as N
    from shadow_amd import synth
    el = synth.barabasi_albert(50_000, 4, 3)
    n = prepare(eng, el)
    log("c5b: graph prepared")
    err = N.Error()
    N.check(eng.lib.shd_routing_run(eng.ctx, N.ALGO_DELTA, 0, 0, None, None, C.byref(err)), "routing_run", err)
    log("c5b: resident table built")
    H, P = C5B_HOSTS, C5B_PACKETS
    start, ra = synth.SIM_START + 10**9, 10**6
    b = synth.packet_batch(H, P, start, start + ra, seed=seed)
    host_node = (np.arange(H, dtype=np.uint64) % n).astype(np.uint32)
    rng0 = synth.host_rng_states(H, 2)
    nid0 = np.zeros(H, np.uint64)
    log("c5b: batch made")
    N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(host_node), n, None, None, N.ptr(rng0), N.ptr(nid0)),
            "relay_setup (resident C4 table)")
    log("c5b: relay set up")
    N.check(eng.lib.shd_relay_set_counters(eng.ctx, 0), "set_counters")
    return dict(el=el, n=n, H=H, P=P, b=b, host_node=host_node, rng0=rng0, rd=(start + ra, start + 10**12, 0))


def c5b_slice_check(eng, cs, status, ev_off, ev_deliver, ev_src, ev_seq, ev_pkt, threads=0, time_it=False):
    """The first round from the setup state against the C restatement on its first 10k source hosts
    (~1M sends): the oracle needs the table only at the pairs those sends use, which come from the
    engine's resident table (shd_routing_lookup_batch) into a lazily allocated n x n array (only
    the touched pages are committed).  Statuses of those sends, and every destination's events
    from those sources (the round's events filtered to src < 10k: a sorted list filtered stays
    sorted; packet indices agree, the slice being the batch's first sends)."""
    from oracle import corc
    from shadow_amd import _native as N
    b, n, hn = cs["b"], cs["n"], cs["host_node"]
    k = C5B_SLICE_HOSTS
    e = int(b.src_off[k])
    src_of = np.repeat(np.arange(k, dtype=np.uint32), np.diff(b.src_off[:k + 1]).astype(np.int64))
    dst = np.minimum(b.dst_host[:e], cs["H"] - 1)
    rows, cols = hn[src_of], hn[dst]
    lat_v = np.zeros(e, np.uint64)
    loss_v = np.zeros(e, np.float32)
    N.check(eng.lib.shd_routing_lookup_batch(eng.ctx, e, N.ptr(np.ascontiguousarray(rows)),
                                             N.ptr(np.ascontiguousarray(cols)), N.ptr(lat_v), N.ptr(loss_v)),
            "lookup_batch")
    lat = np.zeros((n, n), np.uint64)      # calloc: pages are committed only where written
    loss = np.zeros((n, n), np.float32)
    lat[rows, cols] = lat_v
    loss[rows, cols] = loss_v
    # every host stays in the batch (the oracle's per-host state and destination queues cover
    # all of them); the hosts past the slice send nothing
    off = np.concatenate([b.src_off[:k + 1], np.full(cs["H"] - k, b.src_off[k], b.src_off.dtype)])
    reps, t0 = 0, time.perf_counter()
    while True:   # (time_it: repeated for the CPU baseline, ~3 s of CPU work)
        o = corc.relay_round(off, b.send_time[:e], b.dst_host[:e], b.payload[:e], hn, lat, loss,
                             cs["rng0"].copy(), np.zeros(cs["H"], np.uint64), *cs["rd"], threads=threads)
        reps += 1
        if not time_it or time.perf_counter() - t0 > 3.0 or reps >= 50:
            break
    dt = (time.perf_counter() - t0) / reps
    oe = o["events"]
    keep = ev_src < k
    ok = bool(np.array_equal(status[:e], o["status"]) and
              np.array_equal(ev_deliver[keep], oe["deliver"]) and np.array_equal(ev_src[keep], oe["src"]) and
              np.array_equal(ev_seq[keep], oe["seq"]) and np.array_equal(ev_pkt[keep], oe["pkt"]))
    # per destination: the filtered counts are the oracle's offsets
    cnt = np.bincount(np.repeat(np.arange(cs["H"]), np.diff(ev_off.astype(np.int64)))[keep], minlength=cs["H"])
    ok = ok and bool(np.array_equal(np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32), oe["off"]))
    del lat, loss
    return (ok, e, dt) if time_it else ok


def c5b_leg(eng, steps=5, warmup=1, cpu=True):
    import torch
    from shadow_amd import _native as N
    cs = c5b_setup(eng)
    H, P, b = cs["H"], cs["P"], cs["b"]
    d_off, d_time = _dev(b.src_off, np.int32), _dev(b.send_time, np.int64)
    d_dst, d_pay = _dev(b.dst_host, np.int32), _dev(b.payload, np.int32)
    st = torch.empty(P, dtype=torch.uint8, device="cuda")
    ev_off = torch.empty(H + 1, dtype=torch.int32, device="cuda")
    ev_deliver = torch.empty(P, dtype=torch.int64, device="cuda")
    ev_src = torch.empty(P, dtype=torch.int32, device="cuda")
    ev_seq = torch.empty(P, dtype=torch.int64, device="cuda")
    ev_pkt = torch.empty(P, dtype=torch.int32, device="cuda")
    batch = N.Batch(P, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_dst).value, N.ptr(d_pay).value, None)
    out = N.RelayOut(N.ptr(st).value, N.ptr(ev_off).value, N.ptr(ev_deliver).value,
                     N.ptr(ev_src).value, N.ptr(ev_seq).value, N.ptr(ev_pkt).value, 0, 0, 0)
    rnd = N.Round(*cs["rd"])

    def step():
        N.check(eng.lib.shd_relay_round_device(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)),
                "relay_round_device (C5b)")
        return out.n_sent
    step()   # the first round from the setup state: checked
    torch.cuda.synchronize()
    u32 = lambda t: t.cpu().numpy().view(np.uint32)   # noqa: E731
    u64 = lambda t: t.cpu().numpy().view(np.uint64)   # noqa: E731
    ns = out.n_sent
    ok, e, cdt = c5b_slice_check(eng, cs, st.cpu().numpy(), u32(ev_off), u64(ev_deliver)[:ns], u32(ev_src)[:ns],
                                 u64(ev_seq)[:ns], u32(ev_pkt)[:ns], threads=cpu_threads(), time_it=True)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms = dt / steps * 1e3
    pipe = C.c_int32(0)
    N.check(eng.lib.shd_relay_last_pipeline(eng.ctx, C.byref(pipe)), "last_pipeline")
    bytes_round = RELAY_BYTES_PER_PACKET * P + RELAY_BYTES_PER_HOST * H
    ach = bytes_round / (ms * 1e-3) / 1e9
    res = {"workload": "C5b: the C5 round on the C4 table -- 100k hosts, host h on node h mod 50,000 of the "
                       "50k-node BA m=4 graph (table built by the engine, resident), 10M sends per round",
           "hosts": H, "packets": P, "nodes": cs["n"], "steps": steps, "ms_per_round": ms,
           "value": P / (ms * 1e-3), "unit": "packets/s", "pipeline": int(pipe.value),
           "n_sent_last_round": int(out.n_sent),
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS,
                        "work": "84 B/packet + 80 B/host algorithmic (SURVEY 8(d)), whole round; the 8-byte path "
                                "entries are random gathers from the 20 GB packed table"},
           "bit_exact_vs_cpu_slice": ok,
           "checked": f"first round, sends of source hosts 0-{C5B_SLICE_HOSTS - 1} ({e}): statuses and every "
                      f"destination's events from them, against the C restatement"}
    if cpu:
        res["cpu_baseline"] = {"value": e / cdt, "unit": "packets/s", "cores": cpu_threads(), "kind": "port",
                               "sample": f"the check's C restatement: {e} sends of the first {C5B_SLICE_HOSTS} "
                                         f"source hosts on the C4 table (per-packet send_packet restatement, "
                                         f"per-destination heap push, OpenMP over source hosts), {cdt * 1e3:.1f} ms "
                                         f"per run, repeated for ~3 s",
                               "bit_exact_vs_gpu": ok, **cpu_info()}
    del d_off, d_time, d_dst, d_pay, st, ev_off, ev_deliver, ev_src, ev_seq, ev_pkt
    torch.cuda.empty_cache()
    return res


def cpu_threads():
    from oracle import corc
    return corc.max_threads()


def relay_check_sharded(eng, world, rank, rl, lat_table, loss_table):
    """N > 1: one sharded round from the setup state, every rank's statuses and destination events
    against the C restatement of the whole round (the RCCL exchange's own test at this size)."""
    import torch
    from oracle import corc
    from shadow_amd import dist as D
    b, H = rl["batch"], rl["H"]
    rel = D.ShardedRelay(eng, rl["host_node"], rl["rng0"], np.zeros(H, np.uint64), lat_table, loss_table)
    lo, hi = rel.lo, rel.hi
    a, e = int(b.src_off[lo]), int(b.src_off[hi])
    status, ev, md, ml, ns = rel.round((b.src_off[lo:hi + 1] - b.src_off[lo]).astype(np.uint32), b.send_time[a:e],
                                       b.dst_host[a:e], b.payload[a:e], rl["rd"])
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, rl["host_node"], lat_table, loss_table,
                         rl["rng0"].copy(), np.zeros(H, np.uint64), *rl["rd"], threads=corc.max_threads())
    oe = o["events"]
    s0, s1 = int(oe["off"][lo]), int(oe["off"][hi])
    bounds = [D.shard_range(H, world, q) for q in range(world)]
    base = np.array([int(b.src_off[x]) for x, _ in bounds], np.int64)
    sender = np.searchsorted(np.array([y for _, y in bounds]), ev["src"], side="right")
    ok = (np.array_equal(status, o["status"][a:e]) and
          np.array_equal(ev["off"].astype(np.int64), oe["off"][lo:hi + 1].astype(np.int64) - s0) and
          all(np.array_equal(ev[k], oe[k][s0:s1]) for k in ("deliver", "src", "seq")) and
          np.array_equal(ev["pkt"].astype(np.int64) + base[sender], oe["pkt"][s0:s1].astype(np.int64)) and
          (md, ml, ns) == (o["min_deliver"], o["min_latency"], o["n_sent"]))
    del rel
    torch.cuda.empty_cache()
    return all_ranks_ok(ok, world)


def relay_check_and_e2e(eng, rl, lat_table, loss_table, reps=3):
    """One round from the setup state through shd_relay_round with pinned host buffers (the
    call INTEGRATION.md's manager makes: staged batch in, events out, PCIe both ways), timed,
    and its statuses and events compared with the C restatement's."""
    import torch
    from oracle import corc
    from shadow_amd import _native as N
    b, H, P = rl["batch"], rl["H"], rl["P"]
    pin = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).pin_memory()  # noqa: E731
    h_off, h_time = pin(b.src_off, np.int32), pin(b.send_time, np.int64)
    h_dst, h_pay = pin(b.dst_host, np.int32), pin(b.payload, np.int32)
    st = torch.empty(P, dtype=torch.uint8).pin_memory()
    ev_off = torch.empty(H + 1, dtype=torch.int32).pin_memory()
    ev_d = torch.empty(P, dtype=torch.int64).pin_memory()
    ev_s = torch.empty(P, dtype=torch.int32).pin_memory()
    ev_q = torch.empty(P, dtype=torch.int64).pin_memory()
    ev_p = torch.empty(P, dtype=torch.int32).pin_memory()
    hp = lambda t: t.data_ptr()  # noqa: E731
    batch = N.Batch(P, hp(h_off), hp(h_time), hp(h_dst), hp(h_pay), None)
    out = N.RelayOut(hp(st), hp(ev_off), hp(ev_d), hp(ev_s), hp(ev_q), hp(ev_p), 0, 0, 0)
    rnd = N.Round(*rl["rd"])

    def setup():
        N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(rl["host_node"]), 1000, N.ptr(lat_table),
                                        N.ptr(loss_table), N.ptr(rl["rng0"]), N.ptr(np.zeros(H, np.uint64))),
                "relay_setup")
    setup()
    N.check(eng.lib.shd_relay_round(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)), "shd_relay_round")
    ns = out.n_sent
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, rl["host_node"], lat_table, loss_table,
                         rl["rng0"].copy(), np.zeros(H, np.uint64), *rl["rd"], threads=corc.max_threads())
    ev = o["events"]
    ok = (np.array_equal(st.numpy(), o["status"]) and np.array_equal(ev_off.numpy().view(np.uint32), ev["off"])
          and np.array_equal(ev_d.numpy()[:ns].view(np.uint64), ev["deliver"])
          and np.array_equal(ev_s.numpy()[:ns].view(np.uint32), ev["src"])
          and np.array_equal(ev_q.numpy()[:ns].view(np.uint64), ev["seq"])
          and np.array_equal(ev_p.numpy()[:ns].view(np.uint32), ev["pkt"])
          and (out.min_deliver, out.min_latency, ns) == (o["min_deliver"], o["min_latency"], o["n_sent"]))
    t0 = time.perf_counter()
    for _ in range(reps):
        N.check(eng.lib.shd_relay_round(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)), "shd_relay_round")
    ms = (time.perf_counter() - t0) / reps * 1e3
    moved = (H + 1) * 4 + P * (8 + 4 + 4) + P + (H + 1) * 4 + ns * 24
    res = {"ms_per_round": ms, "packets_per_s": P / (ms * 1e-3), "pcie_bytes": moved,
           "what": "shd_relay_round with pinned host buffers: staged batch H2D, round, statuses + events D2H"}
    # the same call with the CPU-drawn f64 chance (INTEGRATION.md's drop-in before shd_relay_flush)
    h_ch = pin(np.random.default_rng(5).random(P), np.float64)
    batch_c = N.Batch(P, hp(h_off), hp(h_time), hp(h_dst), hp(h_pay), hp(h_ch))
    t0 = time.perf_counter()
    for _ in range(reps):
        N.check(eng.lib.shd_relay_round(eng.ctx, C.byref(batch_c), C.byref(rnd), C.byref(out)), "shd_relay_round")
    msc = (time.perf_counter() - t0) / reps * 1e3
    res["with_chance"] = {"ms_per_round": msc, "packets_per_s": P / (msc * 1e-3), "pcie_bytes": moved + P * 8}
    fl, ok_fl = flush_e2e(eng, rl, lat_table, loss_table, setup, reps)
    res["flush"] = fl
    return ok and ok_fl, res


def flush_e2e(eng, rl, lat_table, loss_table, setup, reps=3, n_threads=16):
    """The drop-in round barrier (shd_relay_flush): the round's sends as 16 worker threads' pinned
    staging buffers (per thread: runs of its hosts, 12-byte sends with the CPU's top-32-bit draws),
    grouped on the device; 2-bit statuses and 16-byte events back into pinned memory.  The first
    round (from the setup state) is checked against the C restatement in CPU-chance mode (the same
    u64 draws as f64 chances); then `reps` rounds are timed."""
    from oracle import corc
    from shadow_amd import _native as N
    from shadow_amd import synth
    from shadow_amd.relay import PinnedStages
    b, H, P = rl["batch"], rl["H"], rl["P"]
    rd = rl["rd"]
    time_base = int(b.send_time.min())
    st = synth.stage_round(b, n_threads, time_base, seed=11)
    ps = PinnedStages.pinned(eng.lib, st.run_host, st.run_count, st.sends)
    st2 = torch_pinned_u8((P + 3) // 4)
    ev_off = torch_pinned_u8((H + 1) * 4)
    evs = torch_pinned_u8(P * 16)
    sb = torch_pinned_u8(H * 8)
    out = N.FlushOut(st2.data_ptr(), ev_off.data_ptr(), evs.data_ptr(), sb.data_ptr(), 0, 0, 0, 0, 16)
    rnd = N.Round(*rd)

    def flush():
        N.check(eng.lib.shd_relay_flush(eng.ctx, ps.array, len(ps.stages), time_base, C.byref(rnd), C.byref(out)),
                "shd_relay_flush")
    try:
        setup()
        t0 = time.perf_counter()
        flush()
        first_ms = (time.perf_counter() - t0) * 1e3
        ns = out.n_sent
        chance = (st.draw64 >> np.uint64(11)).astype(np.float64) * 2.0**-53
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, rl["host_node"], lat_table, loss_table,
                             rl["rng0"].copy(), np.zeros(H, np.uint64), *rd, chance=chance, threads=corc.max_threads())
        ev = o["events"]
        inv = np.empty(P, np.int64)
        inv[st.stage_of_send] = np.arange(P)
        e = evs.numpy()[: ns * 16].view(np.uint32).reshape(-1, 4)
        seq_base = sb.numpy()[: H * 8].view(np.uint64)
        status = ((st2.numpy()[:, None] >> (np.arange(4, dtype=np.uint8) * 2)) & 3).reshape(-1)[:P]
        ok = (np.array_equal(status, o["status"][st.stage_of_send])
              and np.array_equal(ev_off.numpy()[: (H + 1) * 4].view(np.uint32), ev["off"])
              and np.array_equal(e[:, 0].astype(np.uint64) + np.uint64(rd[0]), ev["deliver"])
              and np.array_equal(e[:, 1], ev["src"])
              and np.array_equal(e[:, 2].astype(np.uint64) + seq_base[e[:, 1]], ev["seq"])
              and np.array_equal(e[:, 3].astype(np.int64), inv[ev["pkt"].astype(np.int64)])
              and (out.min_deliver, out.min_latency, ns) == (o["min_deliver"], o["min_latency"], o["n_sent"]))
        t0 = time.perf_counter()
        for _ in range(reps):
            flush()
        ms = (time.perf_counter() - t0) / reps * 1e3
        moved = P * 12 + sum(len(x) for x in st.run_host) * 8 + (P + 3) // 4 + (H + 1) * 4 + out.n_sent * 16 + H * 8
        # the 12-byte event form (no source host: the caller's packet names it), same rounds: every
        # round repeats the same stages with the CPU's draws, so its events equal the 16-byte ones
        e16 = evs.numpy()[: out.n_sent * 16].view(np.uint32).reshape(-1, 4).copy()
        out.event_bytes = 12
        flush()
        ns12 = out.n_sent
        host_of_send = np.concatenate([np.repeat(np.asarray(h, np.uint32), np.asarray(c, np.int64))
                                       for h, c in zip(st.run_host, st.run_count)])
        e12 = evs.numpy()[: ns12 * 12].view(np.uint32).reshape(-1, 3)
        t0 = time.perf_counter()
        for _ in range(reps):
            flush()
        ms12 = (time.perf_counter() - t0) / reps * 1e3
        out.event_bytes = 16
        same12 = bool(len(e12) == len(e16) and np.array_equal(e12, e16[:, [0, 2, 3]]) and
                      np.array_equal(host_of_send[e12[:, 2]], e16[:, 1]))
        ok = bool(ok) and same12   # a wrong 12-byte event form fails the bench (advisor, round 5)
        return ({"ms_per_round": ms, "packets_per_s": P / (ms * 1e-3), "pcie_bytes": moved, "first_call_ms": first_ms,
                 "stages": n_threads, "bit_exact_vs_cpu_chance": bool(ok),
                 "events12": {"ms_per_round": ms12, "packets_per_s": P / (ms12 * 1e-3),
                              "pcie_bytes": moved - ns12 * 4,
                              "same_as_16_byte_events": same12,
                              "what": "event_bytes = 12: {deliver_off, seq_off, send} (the source host is the "
                                      "send's run's)"},
                 "what": "shd_relay_flush: 16 worker threads' pinned staging buffers (runs + 12-byte sends with the "
                         "CPU's top-32-bit draws) grouped on the device, round, 2-bit statuses + 16-byte events D2H"},
                ok)
    finally:
        ps.free()


def torch_pinned_u8(n):
    import torch
    return torch.empty(max(int(n), 1), dtype=torch.uint8).pin_memory()


def cpu_baseline_routing(el, budget_s=6.0):
    """Full C2 builds by the C restatement, OpenMP over sources, all host cores: the faithful
    variant (value) and the tidy one beside it; each variant's last table returned."""
    from oracle import corc
    used = np.arange(el.n_nodes, dtype=np.uint32)
    threads = corc.max_threads()
    out = {}
    for name, variant in (("faithful", corc.FAITHFUL), ("tidy", corc.TIDY)):
        reps, t0 = 0, time.perf_counter()
        while True:
            code, lat, loss, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss,
                                              el.directed, used, variant=variant, threads=threads)
            reps += 1
            if time.perf_counter() - t0 > budget_s or reps >= 20:
                break
        out[name] = ((time.perf_counter() - t0) / reps, reps, lat, loss)
    dt, reps, lat, loss = out["faithful"]
    tdt, treps, tlat, tloss = out["tidy"]
    cb = dict(value=el.n_nodes ** 2 / dt, unit="node-pairs/s", cores=threads, kind="port", variant="faithful",
              sample=f"{reps} full C2 builds ({FAITHFUL_WHAT}; OpenMP over sources)",
              tidy=dict(value=el.n_nodes ** 2 / tdt, unit="node-pairs/s", cores=threads, kind="port",
                        sample=f"{treps} full C2 builds ({TIDY_WHAT})"), **cpu_info())
    return cb, (lat, loss), (tlat, tloss)


def cpu_baseline_relay(rl, lat_table, loss_table, budget_s=8.0):
    from oracle import corc
    b = rl["batch"]
    threads = corc.max_threads()
    reps, t0 = 0, time.perf_counter()
    while True:
        rng = rl["rng0"].copy()
        nid = np.zeros(rl["H"], np.uint64)
        corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, rl["host_node"], lat_table,
                         loss_table, rng, nid, *rl["rd"], threads=threads, want_events=False)
        reps += 1
        if time.perf_counter() - t0 > budget_s or reps >= 5:
            break
    dt = (time.perf_counter() - t0) / reps
    return dict(value=rl["P"] / dt, unit="packets/s", cores=threads, kind="port",
                sample=f"{reps} full C5 rounds (per-packet send_packet restatement, per-destination "
                       f"mutex + binary-heap push, OpenMP over source hosts)")


EQ_BYTES_POPPED = 52   # a popped event read from its run (deliver 8, src 4, seq 8, packet 4) and written
                       # to the output (deliver, src, seq, tag 8)


def equeue_leg(eng, rl, lat_table, loss_table, rounds=40, timed=24, cpu=False):
    """The north star's whole relay path, round after round on C5 (1 ms windows, 1-300 ms paths:
    events stay pending for many rounds): the relay round, then shd_equeue_advance -- the merge of
    its events into the device-resident destination queues and the pop of the next window.  The
    24 timed rounds (16-39: the pending set at its steady ~41M events) span several compaction
    cycles of the stored runs, so the mean carries their share whatever the run limit.
    Roofline bytes = the relay's SURVEY 8(d) bytes + the merge's (24 B per batch event read, 28 B
    per kept event written, 56 B per popped event read + written).  CPU baseline: the C
    restatement doing the same rounds -- send_packet with push_packet_to_host into persistent
    per-host heaps, then every host's pop loop below the window (oracle/c/equeue.c) -- and the last
    round's popped events compared with the GPU's."""
    import torch
    from shadow_amd import _native as N
    H, P = rl["H"], rl["P"]
    N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(rl["host_node"]), 1000, N.ptr(lat_table), N.ptr(loss_table),
                                    N.ptr(rl["rng0"]), N.ptr(np.zeros(H, np.uint64))), "relay_setup")
    N.check(eng.lib.shd_equeue_setup(eng.ctx, H), "equeue_setup")
    # the relay leg's counters-on run leaves them on: this leg times the default (counters off)
    N.check(eng.lib.shd_relay_set_counters(eng.ctx, 0), "set_counters")
    st = torch.empty(P, dtype=torch.uint8, device="cuda")
    # the relay writes each round into the queue slot shd_equeue_batch_buffers hands out, and the
    # advance adopts it as a stored run: the round's events are written once, never copied
    out = N.RelayOut()
    qo = N.EqueueOut()
    start0 = start = rl["start"]
    t_relay = t_adv = 0.0
    adv_each = []   # per timed round: a round that compacts the stored runs takes longer
    pops = pend = bytes_merge = n_sent_t = 0
    b = rl["batch"]
    d = [_dev(b.src_off, np.int32), _dev(b.send_time, np.int64), _dev(b.dst_host, np.int32),
         _dev(b.payload, np.int32)]
    t_base = d[1].clone()
    end = start + 10**12
    last = None
    for k in range(rounds):
        d[1].copy_(t_base + k * 10**6)   # the same sends, one window later each round
        batch = N.Batch(P, *(N.ptr(t).value for t in d), None)
        rnd = N.Round(start + 10**6, end, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        N.check(eng.lib.shd_equeue_batch_buffers(eng.ctx, P, C.byref(out)), "equeue_batch_buffers")
        out.status = N.ptr(st).value
        N.check(eng.lib.shd_relay_round_device(eng.ctx, C.byref(batch), C.byref(rnd), C.byref(out)), "relay")
        t1 = time.perf_counter()
        N.check(eng.lib.shd_equeue_advance(eng.ctx, C.byref(out), start + 2 * 10**6, C.byref(qo)), "advance")
        t2 = time.perf_counter()
        if k >= rounds - timed:
            t_relay += t1 - t0
            t_adv += t2 - t1
            adv_each.append(round((t2 - t1) * 1e3, 4))
            pops += qo.n_popped
            pend += qo.n_pending
            n_sent_t += out.n_sent
            # the batch is adopted where the relay wrote it (its bytes are the relay's own); every
            # popped event is read from its run and written to the output
            bytes_merge += EQ_BYTES_POPPED * qo.n_popped
        start += 10**6
        if k == rounds - 1:
            n = qo.n_popped
            last = dict(off=np.zeros(H + 1, np.uint32), deliver=np.zeros(n, np.uint64), src=np.zeros(n, np.uint32),
                        seq=np.zeros(n, np.uint64), tag=np.zeros(n, np.uint64), n_pending=qo.n_pending,
                        next_time=qo.next_time)
            N.check(eng.lib.shd_equeue_copy_popped(eng.ctx, *(N.ptr(last[x]) for x in ("off", "deliver", "src", "seq",
                                                                                        "tag"))), "copy_popped")
    ms = (t_relay + t_adv) / timed * 1e3
    relay_bytes = RELAY_BYTES_PER_PACKET * P + RELAY_BYTES_PER_HOST * H
    algo = relay_bytes + bytes_merge / timed
    ach = algo / (ms * 1e-3) / 1e9
    res = {"workload": "C5 rounds: relay + shd_equeue_advance (merge into the pending destination queues, pop "
                       "the next 1 ms window)", "rounds": rounds, "timed_rounds": timed,
           "relay_ms_per_round": t_relay / timed * 1e3, "advance_ms_per_round": t_adv / timed * 1e3, "advance_ms_each": adv_each,
           "ms_per_round": ms, "value": P / (ms * 1e-3), "unit": "packets relayed + merged/s",
           "popped_per_round": pops / timed, "pending_mean": pend / timed,
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS, "bytes_per_round": algo,
                        "work": "relay 84 B/packet + 80 B/host (SURVEY 8(d)) + merge 52 B per popped event (read "
                                "24, written 28); the round's events are adopted where the relay wrote them"}}
    if cpu:
        from oracle import corc
        threads = corc.max_threads()
        oq = corc.EventQueues(H)
        rng, nid = rl["rng0"].copy(), np.zeros(H, np.uint64)
        start = start0
        tb = b.send_time.copy()
        t_cpu = 0.0
        for k in range(rounds):
            times = tb + np.uint64(k * 10**6)
            t0 = time.perf_counter()
            corc.relay_round_eq(b.src_off, times, b.dst_host, b.payload, rl["host_node"], lat_table, loss_table, rng,
                                nid, start + 10**6, end, 0, queues=oq, batch_no=k, threads=threads)
            o = oq.pop(start + 2 * 10**6, threads=threads, want=k == rounds - 1)
            dt = time.perf_counter() - t0
            if k >= rounds - timed:
                t_cpu += dt
            if k == rounds - 1:
                op = o
            start += 10**6
        cms = t_cpu / timed * 1e3
        same = last is not None and all(np.array_equal(last[x], op[x]) for x in ("off", "deliver", "src", "seq", "tag")) \
            and (last["n_pending"], last["next_time"]) == (op["n_pending"], op["next_time"])
        res["cpu_baseline"] = {"value": P / (cms * 1e-3), "unit": "packets relayed + merged/s", "cores": threads,
                               "kind": "port", "ms_per_round": cms,
                               "sample": f"the same {rounds} C5 rounds through oracle/c (send_packet + "
                                         f"push_packet_to_host into per-host binary heaps under per-destination "
                                         f"mutexes, then every host's pop loop), last {timed} timed",
                               "bit_exact_vs_gpu": bool(same)}
    return res


def equeue_leg_sharded(eng, world, rank, rl, lat_table, loss_table, rounds=6, timed=3):
    """N > 1: the whole relay path per round over the engine communicator -- each rank's sharded
    relay round (its source hosts; events exchanged to their destination ranks), the agreed next
    window (shd_round_window, a collective), and the merge + pop into the rank's own destination
    queues (shd_equeue_advance).  Time per round = the max over the ranks."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd import dist as D
    from shadow_amd.equeue import EventQueues
    from shadow_amd.rounds import Runahead, next_window
    H, b = rl["H"], rl["batch"]
    rel = D.ShardedRelay(eng, rl["host_node"], rl["rng0"], np.zeros(H, np.uint64), lat_table, loss_table)
    N.check(eng.lib.shd_relay_set_counters(eng.ctx, 0), "set_counters")
    q = EventQueues(eng, H)
    Runahead(eng, False, int(lat_table.min()), 10**6)   # fixed 1 ms windows, as the 1-GPU leg
    lo, hi = rel.lo, rel.hi
    a, e = int(b.src_off[lo]), int(b.src_off[hi])
    d_off = _dev((b.src_off[lo:hi + 1] - b.src_off[lo]).astype(np.uint32), np.int32)
    d_time, d_dst = _dev(b.send_time[a:e], np.int64), _dev(b.dst_host[a:e], np.int32)
    d_pay = _dev(b.payload[a:e], np.int32)
    t_base = d_time.clone()
    st = torch.empty(max(e - a, 1), dtype=torch.uint8, device="cuda")
    start, end = rl["start"], rl["start"] + 10**12
    t_tot, pops = 0.0, 0
    barrier_sync(world)
    for k in range(rounds):
        d_time.copy_(t_base + k * 10**6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = rel.round_device(d_off, d_time, d_dst, d_pay, (start + 10**6, end, 0), st)
        win = next_window(eng, None, end)
        qo = q.advance_device(out, win[1] if win else 2**63)
        dt = time.perf_counter() - t0
        if k >= rounds - timed:
            t_tot += dt
            pops += qo.n_popped
        start += 10**6
    ms = max_over_ranks(t_tot / timed * 1e3, world)
    return {"workload": f"C5 rounds over {world} ranks: shd_relay_round_sharded + shd_round_window + "
                        f"shd_equeue_advance into each rank's destination queues", "rounds": rounds,
            "timed_rounds": timed, "ms_per_round": ms, "value": rl["P"] / (ms * 1e-3),
            "unit": "packets relayed + merged/s", "popped_per_round_rank0": pops / timed}


def codel_leg(eng, steps=5, cpu=True):
    """the destination side of C5 -- 100k CoDel router queues, each fed the
    ~100 packets a C5 round delivers to it and drained by as many pops (interface reads 2 ms
    apart, so standing delays cross TARGET for longer than INTERVAL and the drop path runs),
    one batch per step."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd.codel import CoDelQueues, POP
    H, per = 100_000, 100
    rng = np.random.default_rng(6)
    t0 = 946684800 * 10**9 + 10**9
    n = H * 2 * per
    # per host: 100 pushes at arrival times, then 100 pops; arrivals bunched so queues build up
    arr = np.sort(rng.integers(0, 5 * 10**6, size=(H, per)), axis=1).astype(np.uint64) + np.uint64(t0)
    pops = arr[:, -1:] + np.arange(1, per + 1, dtype=np.uint64)[None, :] * np.uint64(2_000_000)
    tarr = np.concatenate([arr, pops], axis=1).reshape(-1)
    size = np.concatenate([np.full((H, per), 1500, np.uint32), np.full((H, per), POP, np.uint32)], axis=1).reshape(-1)
    pkt = np.concatenate([np.arange(H * per, dtype=np.uint32).reshape(H, per), np.zeros((H, per), np.uint32)],
                         axis=1).reshape(-1)
    off = (np.arange(H + 1, dtype=np.uint64) * (2 * per)).astype(np.uint32)
    q = CoDelQueues(eng, H, 2 * per)
    dev = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()  # noqa: E731
    d_off, d_time, d_size, d_pkt = dev(off, np.int32), dev(tarr, np.int64), dev(size, np.int32), dev(pkt, np.int32)
    pop_out = torch.empty(n, dtype=torch.int32, device="cuda")
    fate = torch.zeros(H * per, dtype=torch.int64, device="cuda")
    ops = N.CodelOps(n, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_size).value, N.ptr(d_pkt).value)

    def step():
        eng.lib.shd_codel_setup(eng.ctx, H, 2 * per)
        N.check(eng.lib.shd_codel_run_device(eng.ctx, C.byref(ops), N.ptr(pop_out), N.ptr(fate), H * per),
                "codel_run")
    step()
    torch.cuda.synchronize()
    s0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - s0) * 1e3 / steps
    f = fate.cpu().numpy().view(np.uint64)
    dropped = int(np.count_nonzero((f & np.uint64(3)) == 2))
    out = {"workload": "C5 destinations: 100k CoDel queues x (100 pushes + 100 pops) per batch",
           "ops": n, "ms_per_batch": ms, "value": n / (ms * 1e-3), "unit": "queue ops/s",
           "dropped": dropped, "work": "one lane per host replays its ops in order (sequential state machine)"}
    if cpu:   # the C restatement (oracle/c/queues.c) over the whole batch, all host cores
        from oracle import corc
        threads = corc.max_threads()
        corc.codel_run(H, off, tarr, size, pkt, H * per, threads=threads)   # warm (page faults)
        s1 = time.perf_counter()
        pop_ref, fate_ref = corc.codel_run(H, off, tarr, size, pkt, H * per, threads=threads)
        dt = time.perf_counter() - s1
        out["cpu_baseline"] = {"value": n / dt, "unit": "queue ops/s", "cores": threads, "kind": "port",
                               "sample": "the whole batch (20M ops) through oracle/c/queues.c (CoDelQueue "
                                         "restated, hosts over OpenMP threads)",
                               "bit_exact_vs_gpu": bool(np.array_equal(pop_ref, pop_out.cpu().numpy().view(np.uint32))
                                                        and np.array_equal(fate_ref, f))}
    return out


def tbucket_leg(eng, steps=5, cpu=True):
    """the source side of C5 -- 100k upstream relays, each with the token
    bucket of a 10 Mbit/s interface (create_token_bucket: 1,250 B per 1 ms refill, capacity
    2,750 B) and ~100 forwarding attempts of C5 sizes spread over 20 ms, so buckets run dry,
    block and skip.  The buckets are re-created each step (identical work per step)."""
    import torch
    from shadow_amd import _native as N
    from shadow_amd.tbucket import SIM_START, create_token_bucket
    H, per = 100_000, 100
    rng = np.random.default_rng(7)
    t0 = SIM_START + 10**9
    n = H * per
    tarr = (np.sort(rng.integers(0, 20 * 10**6, size=(H, per)), axis=1).astype(np.uint64)
            + np.uint64(t0)).reshape(-1)
    u = rng.random(n)
    size = np.where(u < 0.2, 66, np.where(u < 0.8, 1514, rng.integers(67, 1515, n))).astype(np.uint32)
    flags = np.zeros(n, np.uint8)
    off = (np.arange(H + 1, dtype=np.uint64) * per).astype(np.uint32)
    c, i, v = create_token_bucket(10_000_000 // 8)
    caps, incs, itvs, last = (np.full(H, x, np.uint64) for x in (c, i, v, t0))
    dev = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()  # noqa: E731
    d_off, d_time, d_size, d_flags = dev(off, np.int32), dev(tarr, np.int64), dev(size, np.int32), dev(flags, np.uint8)
    status = torch.empty(n, dtype=torch.uint8, device="cuda")
    value = torch.empty(n, dtype=torch.int64, device="cuda")
    ops = N.TbOps(n, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_size).value, N.ptr(d_flags).value)

    def step():
        N.check(eng.lib.shd_tb_setup(eng.ctx, H, N.ptr(caps), N.ptr(incs), N.ptr(itvs), N.ptr(last)), "tb_setup")
        N.check(eng.lib.shd_tb_run_device(eng.ctx, C.byref(ops), N.ptr(status), N.ptr(value)), "tb_run")
    step()
    torch.cuda.synchronize()
    s0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - s0) * 1e3 / steps
    st = status.cpu().numpy()
    out = {"workload": "C5 sources: 100k token-bucket relays (10 Mbit/s) x 100 forwarding attempts per batch",
           "ops": n, "ms_per_batch": ms, "value": n / (ms * 1e-3), "unit": "relay attempts/s",
           "forwarded": int(np.count_nonzero(st == 0)), "blocked": int(np.count_nonzero(st == 1)),
           "skipped": int(np.count_nonzero(st == 2)),
           "work": "one lane per relay replays its attempts in order (sequential state machine); "
                   "step includes shd_tb_setup (host -> device copy of 100k buckets)"}
    if cpu:   # the C restatement (oracle/c/queues.c) over the whole batch, all host cores
        from oracle import corc
        threads = corc.max_threads()
        corc.tb_run(caps, incs, itvs, last, off, tarr, size, flags, threads=threads)   # warm
        s1 = time.perf_counter()
        ost, oval, _ = corc.tb_run(caps, incs, itvs, last, off, tarr, size, flags, threads=threads)
        dt = time.perf_counter() - s1
        out["cpu_baseline"] = {"value": n / dt, "unit": "relay attempts/s", "cores": threads, "kind": "port",
                               "sample": "the whole batch (10M attempts) through oracle/c/queues.c (TokenBucket + "
                                         "forward_until_blocked restated, relays over OpenMP threads)",
                               "bit_exact_vs_gpu": bool(np.array_equal(ost, st) and np.array_equal(
                                   oval, value.cpu().numpy().view(np.uint64)))}
    return out

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--relay-steps", type=int, default=None)
    ap.add_argument("--c4-steps", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-relay", action="store_true")
    ap.add_argument("--no-c3", action="store_true")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--no-c5b", action="store_true")
    ap.add_argument("--no-codel", action="store_true")
    ap.add_argument("--no-tbucket", action="store_true")
    ap.add_argument("--no-equeue", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--c4-no-gather", action="store_true")
    args = ap.parse_args()
    world, rank, local = dist_setup(args.gpus)
    from shadow_amd.routing import Engine
    eng = Engine(local)
    host_comm = None
    if world > 1:   # the engine's own communicator: RCCL over xGMI, one rank per GPU
        from shadow_amd import dist as D
        if REHEARSAL:
            host_comm = D.HostComm(eng)   # (kept alive: it holds the transport callback)
        else:
            D.comm_init_rccl(eng)
    cpu = rank == 0 and world == 1 and not args.no_cpu_baseline

    r = routing_leg(eng, world, rank, args.steps, args.warmup)
    value = args.steps * r["n"] ** 2 / r["dt"]
    res = {
        "metric": METRIC, "value": value, "unit": "node-pairs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u32 latency (u64 out) + f32 loss", "data": "synthetic",
        "config": {"workload": "C2: APSP routing-table build, 1000-node complete undirected GML "
                               "graph + self-loops, 1000 used nodes",
                   "nodes": r["n"], "arcs": int(r["arcs"]), "arcs_after_prune": int(r["arcs_kept"]),
                   "algo": int(r["algo"]),
                   "parallelism": ("1 GPU" if world == 1 else
                                   f"whole table on each of {world} ranks (12 MB: replicated, no exchange; "
                                   "shd_routing_run_sharded)" if r["rows"] == r["n"] else
                                   f"source-row shards x{world} + engine RCCL all-gather (shd_routing_run_sharded)")},
        "roofline": {"bound": "valu", "achieved": r["achieved"], "peak": VALU_PEAK_TOPS,
                     "unit": "Tops/s", "frac": r["achieved"] / VALU_PEAK_TOPS,
                     "traffic": load_pmc("routing"),
                     "kernel": "sssp_lds_group", "kernel_ms": r["kernel_ms"],
                     "work": "2 int ops (add, min) per arc relaxation per source row = 2*n*A "
                             "(A = arcs before pruning: the reference's Dijkstra work)"},
    }
    if cpu:
        cb, fa, ti = cpu_baseline_routing(r["el"])
        cpu_bit_exact(cb, fa, ti, r["lat"], r["loss"])
        res["cpu_baseline"] = cb
    checks = {}
    if world > 1:   # the multi-GPU run checks itself: every rank's whole table against the C restatement
        from oracle import corc
        el = r["el"]
        code, olat, oloss, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed,
                                            np.arange(el.n_nodes, dtype=np.uint32), threads=corc.max_threads())
        checks["c2_table_bit_exact_all_ranks"] = all_ranks_ok(
            code == "OK" and np.array_equal(r["lat"], olat) and
            np.array_equal(r["loss"].view(np.uint32), oloss.view(np.uint32)), world)
    if world == 1 and not args.no_e2e:
        res["routing_e2e"] = routing_e2e(eng, r["el"])
        res["c2_engines"] = c2_engines(eng, r["el"])
    if not args.no_relay:
        ks = args.relay_steps or max(3, args.steps // 2)
        inputs = relay_inputs()
        rl = relay_leg(eng, world, rank, ks, min(args.warmup, 2), r["lat"], r["loss"], inputs=inputs)
        pv = ks * rl["P"] / rl["dt"]
        ms = rl["ms_per_step"]
        bytes_round = RELAY_BYTES_PER_PACKET * rl["P"] + RELAY_BYTES_PER_HOST * rl["H"]
        ach = bytes_round / (ms * 1e-3) / 1e9
        rel = {"metric": "packets relayed/s per round", "value": pv, "unit": "packets/s",
               "steps": ks, "ms_per_round": ms, "n_sent_last_round": int(rl["n_sent"]),
               "pipeline": rl["pipeline"],
               "scaling": "strong",
               "path_counters": "off (reference reads them only in the never-called "
                                "log_packet_counts; CPU baseline keeps none)",
               "config": {"workload": "C5: 100k hosts on the C2 table, 10M packets per round "
                                      "(src uniform, dst != src, 20% ACK / 60% 1448 B / 20% U[1,1448])",
                          "hosts": rl["H"], "packets": rl["P"],
                          "parallelism": (f"hosts sharded x{world}: the stamp's destination bins sent to their "
                                          f"ranks over RCCL (one sizing all-gather, one grouped send/recv) and "
                                          f"bin-sorted there (shd_relay_round_sharded)")
                          if world > 1 else "1 GPU"},
               "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": ach / HBM_PEAK_GBS, "traffic": load_pmc("relay"),
                            "work": "84 B/packet + 80 B/host algorithmic (SURVEY 8(d)), whole round"}}
        if world == 1:
            rl_c = relay_leg(eng, world, rank, max(2, ks // 3), 1, r["lat"], r["loss"], counters=True,
                             inputs=inputs)
            rel["counters_on_ms_per_round"] = rl_c["ms_per_step"]
            if eng.lib.shd_relay_set_counters(eng.ctx, 0) != 0:   # back to the default for what follows
                raise RuntimeError("shd_relay_set_counters failed")
            ok, e2e = relay_check_and_e2e(eng, rl, r["lat"], r["loss"])
            rel["e2e_host_buffers"] = e2e
            rel["bit_exact_vs_cpu"] = bool(ok)
        if cpu:
            rel["cpu_baseline"] = cpu_baseline_relay(rl, r["lat"], r["loss"])
            rel["cpu_baseline"]["bit_exact_vs_gpu"] = rel["bit_exact_vs_cpu"]
        if world == 1 and not args.no_equeue:
            rel["equeue"] = equeue_leg(eng, rl, r["lat"], r["loss"], cpu=cpu)
        if world > 1:
            checks["relay_round_bit_exact_all_ranks"] = relay_check_sharded(eng, world, rank, rl, r["lat"], r["loss"])
            if not args.no_equeue:
                rel["equeue"] = equeue_leg_sharded(eng, world, rank, rl, r["lat"], r["loss"])
        res["relay"] = rel
    if world == 1 and not args.no_c3:
        res["c3"] = c3_leg(eng, cpu=cpu)
    if not args.no_c4:
        res["c4"] = c4_leg(eng, world, rank, args.c4_steps, gather=not args.c4_no_gather, cpu=cpu)
        if "check" in res["c4"]:
            checks["c4_last_rows_bit_exact"] = res["c4"].pop("check")
    if world == 1 and not args.no_c5b:
        res["c5b"] = c5b_leg(eng, cpu=cpu)
    if checks:
        res["parity_check"] = checks
    if world == 1 and not args.no_codel:
        res["codel"] = codel_leg(eng, cpu=cpu)
    if world == 1 and not args.no_tbucket:
        res["tbucket"] = tbucket_leg(eng, cpu=cpu)
    if rank == 0:
        print(json.dumps(res), flush=True)
    eng.close()
    del host_comm
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
