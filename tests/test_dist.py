"""World-size-2 gloo tests (CPU) of the sharding contract the C ABI implements for N > 1 ranks
(include/shd_accel.h: shd_shard_range, shd_routing_run_sharded, shd_relay_round_sharded,
shd_equeue_setup under a communicator, shd_round_window).

The engine's collectives need a GPU; here every rank computes its share with the C restatement
and moves exactly what the ABI moves, with gloo, one process per rank:
  * routing: rank r builds the source rows shd_shard_range gives it; the table ends whole on
    every rank;
  * relay: rank r stamps its own source hosts (its RNG streams and event ids) into events grouped
    by destination; rank q receives, from every sender, the per-destination offset block of its
    destination shard and the records; it merges the per-sender runs by (deliver, src, seq);
    ev_pkt stays the packet's index in the SENDER rank's batch; min deliver / min latency / sent
    are reduced over the ranks;
  * queues + window: rank r's queues hold its destination shard; the next window's start is the
    minimum over every rank's queue heads (a collective), the runahead the minimum latency used
    by any rank's sends; each rank pops its hosts below the window end.
The union over the ranks must equal one single-process run of the reference semantics, round
after round.  (The same contract runs on the GPU with two engine ranks in one process:
tests/test_comm_gpu.py.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corc

U64_MAX = 2**64 - 1
ROUNDS = 4
END = 10**9 + 300 * 10**6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    from shadow_amd import synth
    H, NN = 600, 25
    el = synth.complete_graph(NN, 7)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    return el, H, lat, loss, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)


def _batch(H, ws, we, rnd):
    from shadow_amd import synth
    return synth.packet_batch(H, 30_000, ws, we, seed=21 + rnd)


def _shard(total, world, rank):
    from shadow_amd.dist import shard_range   # the library's own shd_shard_range (no GPU needed)
    return shard_range(total, world, rank)


def _i64(x):   # a u64 reduction value through an int64 tensor (only u64::MAX exceeds 2^63)
    return min(int(x), 2**63 - 1)


def _u64(x):
    return U64_MAX if int(x) == 2**63 - 1 else int(x)


def _relay_shard(rank, world, H, b, host_node, lat, loss, rng, nid, we):
    """This rank's part of shd_relay_round_sharded: stamp own sources, exchange per destination
    shard (offset block + records), merge.  Returns (merged CSR over own hosts, reductions)."""
    lo, hi = _shard(H, world, rank)
    bounds = [_shard(H, world, r) for r in range(world)]
    a, e = int(b.src_off[lo]), int(b.src_off[hi])
    off = np.zeros(H + 1, np.uint32)   # this rank's sends only (the others' hosts send nothing here)
    off[lo + 1:hi + 1] = b.src_off[lo + 1:hi + 1] - a
    off[hi + 1:] = e - a
    o = corc.relay_round(off, b.send_time[a:e], b.dst_host[a:e], b.payload[a:e], host_node, lat, loss,
                         rng, nid, we, END, 0)
    ev = o["events"]
    recs = np.stack([ev["deliver"].view(np.int64), ev["src"].astype(np.int64), ev["seq"].view(np.int64),
                     ev["pkt"].astype(np.int64)], 1)
    # sizing: events per destination shard
    cut = [int(ev["off"][b0]) for b0, _ in bounds] + [int(ev["off"][H])]
    send_n = torch.tensor([cut[k + 1] - cut[k] for k in range(world)], dtype=torch.int64)
    recv_n = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(recv_n, send_n)
    # part 0: every peer's offset block over its destination shard; part 1: the records
    blocks = [ev["off"][b0:b1 + 1].astype(np.int64) - int(ev["off"][b0]) for b0, b1 in bounds]
    n_own = hi - lo
    r_off = torch.empty(world * (n_own + 1), dtype=torch.int64)
    dist.all_to_all_single(r_off, torch.from_numpy(np.concatenate(blocks)), [n_own + 1] * world,
                           [b1 - b0 + 1 for b0, b1 in bounds])
    got = torch.empty((int(recv_n.sum()), 4), dtype=torch.int64)
    dist.all_to_all_single(got, torch.from_numpy(recs.copy()), recv_n.tolist(), send_n.tolist())
    g, ro = got.numpy(), r_off.numpy().reshape(world, n_own + 1)
    # destination of every received record from its sender's offset block, then the merge
    dst = np.empty(len(g), np.int64)
    at = 0
    for q in range(world):
        k = int(recv_n[q])
        dst[at:at + k] = np.repeat(np.arange(n_own), np.diff(ro[q]))
        at += k
    order = np.lexsort((g[:, 2].view(np.uint64), g[:, 1], g[:, 0].view(np.uint64), dst))
    g, dst = g[order], dst[order]
    m_off = np.searchsorted(dst, np.arange(n_own + 1)).astype(np.uint32)
    red = torch.tensor([_i64(o["min_deliver"]), _i64(o["min_latency"])], dtype=torch.int64)
    dist.all_reduce(red, op=dist.ReduceOp.MIN)
    ns = torch.tensor([o["n_sent"]], dtype=torch.int64)
    dist.all_reduce(ns)
    merged = dict(off=m_off, deliver=g[:, 0].view(np.uint64).copy(), src=g[:, 1].astype(np.uint32),
                  seq=g[:, 2].view(np.uint64).copy(), pkt=g[:, 3].astype(np.uint32))
    return merged, _u64(red[0]), _u64(red[1]), int(ns[0]), o["status"].copy(), a


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.relay import RunaheadState, next_window
        el, H, lat, loss, host_node, rng0 = _case()
        n = el.n_nodes
        # ---- routing: this rank's rows, then the whole table on every rank
        rb, re = _shard(n, world, rank)
        per = (n + world - 1) // world
        code, rl, rp, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed,
                                       np.arange(n, dtype=np.uint32), rows=(rb, re))
        assert code == "OK"
        mine = torch.zeros((per, n, 2), dtype=torch.int64)
        mine[: re - rb, :, 0] = torch.from_numpy(rl.view(np.int64))
        mine[: re - rb, :, 1] = torch.from_numpy(rp.view(np.int32).astype(np.int64))
        full = torch.zeros((world * per, n, 2), dtype=torch.int64)
        dist.all_gather_into_tensor(full, mine)
        table = (full[:n, :, 0].numpy().view(np.uint64).copy(),
                 full[:n, :, 1].numpy().astype(np.int32).view(np.float32).copy())
        # ---- relay -> own queues -> agreed window -> pops, round after round
        lo, hi = _shard(H, world, rank)
        rng, nid = rng0.copy(), np.zeros(H, np.uint64)
        mq = corc.EventQueues(hi - lo)
        ra = RunaheadState(True, int(lat.min()))
        ws, we = 10**9, 10**9 + ra.get()
        out = []
        for rnd in range(ROUNDS):
            b = _batch(H, ws, we, rnd)
            merged, md, ml, ns, status, a = _relay_shard(rank, world, H, b, host_node, lat, loss, rng, nid, we)
            mq.push_batch(merged["off"], merged["deliver"], merged["src"], merged["seq"], merged["pkt"], rnd)
            if ml != U64_MAX:
                ra.update_lowest_used_latency(ml)
            head = torch.tensor([_i64(mq.pop(0, want=False)["next_time"])], dtype=torch.int64)
            dist.all_reduce(head, op=dist.ReduceOp.MIN)
            win = next_window(_u64(head[0]), ra.get(), END)
            popped = mq.pop(win[1])
            out.append(dict(merged=merged, md=md, ml=ml, ns=ns, status=status, base=a, win=win, popped=popped))
            ws, we = win
        q.put((rank, table, out, rng[lo:hi].copy(), nid[lo:hi].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_world2_sharding_contract_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, table, out, rng, nid = q.get(timeout=240)
        res[rank] = (table, out, rng, nid)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.relay import RunaheadState, next_window
    el, H, lat, loss, host_node, rng0 = _case()
    # routing: every rank holds the single-process table
    code, want_lat, want_loss, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                                np.arange(el.n_nodes, dtype=np.uint32))
    for r in range(world):
        assert np.array_equal(res[r][0][0], want_lat)
        assert np.array_equal(res[r][0][1].view(np.uint32), want_loss.view(np.uint32))
    # relay + queues + window: one process, persistent per-host heaps (push_packet_to_host)
    rng, nid = rng0.copy(), np.zeros(H, np.uint64)
    oq = corc.EventQueues(H)
    ra = RunaheadState(True, int(lat.min()))
    ws, we = 10**9, 10**9 + ra.get()
    bounds = [_shard(H, world, r) for r in range(world)]
    for rnd in range(ROUNDS):
        b = _batch(H, ws, we, rnd)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng, nid, we, END, 0)
        ev = o["events"]
        oq.push_batch(ev["off"], ev["deliver"], ev["src"], ev["seq"], ev["pkt"], rnd)
        if o["min_latency"] != U64_MAX:
            ra.update_lowest_used_latency(o["min_latency"])
        win = next_window(oq.pop(0, want=False)["next_time"], ra.get(), END)
        op = oq.pop(win[1])
        for r in range(world):
            lo, hi = bounds[r]
            x = res[r][1][rnd]
            assert x["win"] == win
            assert (x["md"], x["ml"], x["ns"]) == (o["min_deliver"], o["min_latency"], o["n_sent"])
            a, e = int(b.src_off[lo]), int(b.src_off[hi])
            assert np.array_equal(x["status"], o["status"][a:e])
            # the merged batch of the rank's destinations; ev_pkt = index in the sender's batch
            m, s0, s1 = x["merged"], int(ev["off"][lo]), int(ev["off"][hi])
            assert np.array_equal(m["off"].astype(np.int64), ev["off"][lo:hi + 1].astype(np.int64) - s0)
            for k in ("deliver", "src", "seq"):
                assert np.array_equal(m[k], ev[k][s0:s1]), k
            sender_base = np.array([int(b.src_off[b0]) for b0, _ in bounds], np.int64)
            sender = np.searchsorted(np.array([b1 for _, b1 in bounds]), m["src"], side="right")
            assert np.array_equal(m["pkt"].astype(np.int64) + sender_base[sender], ev["pkt"][s0:s1].astype(np.int64))
            # the popped events of the rank's hosts
            p, s0, s1 = x["popped"], int(op["off"][lo]), int(op["off"][hi])
            assert np.array_equal(p["off"].astype(np.int64), op["off"][lo:hi + 1].astype(np.int64) - s0)
            for k in ("deliver", "src", "seq"):
                assert np.array_equal(p[k], op[k][s0:s1]), k
        assert sum(res[r][1][rnd]["popped"]["n_pending"] for r in range(world)) == op["n_pending"]
        ws, we = win
    for r in range(world):   # source-owned RNG streams and event ids advanced exactly
        lo, hi = bounds[r]
        assert np.array_equal(res[r][2], rng[lo:hi]) and np.array_equal(res[r][3], nid[lo:hi])


def test_shard_ranges_partition_rows_and_hosts():
    """shd_shard_range: contiguous blocks of ceil(total / n) covering [0, total) in rank order."""
    for n in (1, 2, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [_shard(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            per = (n + w - 1) // w
            assert all(hi - lo <= per for lo, hi in parts)
