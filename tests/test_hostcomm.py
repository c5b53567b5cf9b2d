"""The engine communicator over the caller's host transport (shd_comm_init_host), world size 2,
one process per rank over gloo on 127.0.0.1.

* CPU: the gloo all-to-all-v that shadow_amd.dist hands the engine as its callback moves every
  rank's blocks (sizes, offsets, repeated offsets, empty blocks) exactly.
* GPU (-m gpu): two PROCESSES on cuda:0, each with its own engine context, run the product's
  sharded paths -- the routing build through the chunked table exchange, and relay rounds through
  shd_relay_round_sharded -- over that transport; every rank's table and events against the C
  restatement.  These are the code paths the RCCL runs take (RCCL itself refuses two ranks on one
  GPU); only the transport differs.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(target, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, out = q.get(timeout=timeout)
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return res


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _a2av_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from shadow_amd.dist import host_all_to_allv
        a2av = host_all_to_allv()
        # block to rank r: bytes r*16 + rank .. of length 3 + 5 r + rank (rank 1's block to rank 0
        # is empty); rank 1 sends the SAME block (offset 0) to every rank
        sizes = [(3 + 5 * r + rank) if not (rank == 1 and r == 0) else 0 for r in range(world)]
        if rank == 1:
            sizes = [0, 9]
            payload = np.arange(100, 109, dtype=np.uint8)
            send = np.concatenate([payload, np.zeros(7, np.uint8)])
            offs = [0, 0]
        else:
            blocks = [(np.arange(sizes[r], dtype=np.uint8) + 16 * r + rank).astype(np.uint8) for r in range(world)]
            send = np.concatenate(blocks + [np.zeros(5, np.uint8)])
            offs = list(np.cumsum([0] + sizes[:-1]))
        recv_sizes = {0: [3, 0], 1: [8, 9]}[rank]
        roffs = [0, 11]
        recv = np.full(32, 0xEE, np.uint8)
        u = C.c_uint64 * world
        a2av(send.ctypes.data, u(*sizes), u(*offs), recv.ctypes.data, u(*recv_sizes), u(*roffs))
        q.put((rank, recv.copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_host_all_to_allv_over_gloo():
    res = _spawn(_a2av_worker, 2)
    r0, r1 = res[0], res[1]
    # rank 0 receives its own block (3 bytes: 0, 1, 2) and nothing from rank 1
    assert list(r0[:3]) == [0, 1, 2] and (r0[3:] == 0xEE).all()
    # rank 1 receives rank 0's block to it (8 bytes from 16) and its own shared block (100..108)
    assert list(r1[:8]) == list(range(16, 24))
    assert list(r1[11:20]) == list(range(100, 109))
    assert (r1[8:11] == 0xEE).all() and (r1[20:] == 0xEE).all()


# ----------------------------------------------------------------------------- GPU, 2 processes
def _gpu_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import torch
        from shadow_amd import _native as N
        from shadow_amd import dist as D
        from shadow_amd import synth
        from shadow_amd.routing import Engine
        from tests.graphs import engine_graph_from_edges
        eng = Engine(0)
        eng.set_knob("SHARD_REPLICATE_MB", 0)   # exchange the row shards (C2-sized tables replicate)
        eng.set_knob("SHARD_CHUNK_ROWS", 7)     # in chunks, the last one short
        hc = D.HostComm(eng)
        # ---- routing: this rank's rows, the table whole on both ranks
        n = 301
        el = synth.complete_graph(n, 12)
        used = np.arange(n, dtype=np.uint32)
        g = engine_graph_from_edges(el)
        cg = g._cgraph()
        err = N.Error()
        N.check(eng.lib.shd_routing_prepare(eng.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST, C.byref(err)),
                "prepare", err)
        per = (n + world - 1) // world
        lt = torch.empty((world * per, n), dtype=torch.int64, device="cuda")
        ls = torch.empty((world * per, n), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        D.routing_run_sharded(eng, N.ALGO_AUTO, lt, ls)
        table = (lt[:n].cpu().numpy().view(np.uint64).copy(), ls[:n].cpu().numpy().view(np.uint32).copy())
        # ---- relay rounds: this rank's source hosts, its destinations' events
        H, NN, P = 5000, 50, 400_000
        el2 = synth.complete_graph(NN, 3)
        code, lat, loss, _ = corc.routing(NN, el2.src, el2.dst, el2.latency_ns, el2.packet_loss, False,
                                          np.arange(NN, dtype=np.uint32))
        assert code == "OK"
        host_node, rng0 = synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)
        rel = D.ShardedRelay(eng, host_node, rng0, np.zeros(H, np.uint64), lat, loss)
        start, ra = 10**9, 10**6
        rounds = []
        for rnd in range(3):
            b = synth.packet_batch(H, P, start, start + ra, seed=90 + rnd)
            a, e = int(b.src_off[rel.lo]), int(b.src_off[rel.hi])
            off = (b.src_off[rel.lo:rel.hi + 1] - b.src_off[rel.lo]).astype(np.uint32)
            rd = (start + ra, start + 10**12, start + ra // 2 if rnd == 0 else 0)
            rounds.append(rel.round(off, b.send_time[a:e], b.dst_host[a:e], b.payload[a:e], rd))
            start += ra
        # a rank whose staging cannot be allocated (injected on rank 1) still takes part: the
        # staging status round fails the next round on both ranks, and neither commits it
        if rank == 1:
            eng.set_knob("TEST_FAIL", 3)
        try:
            rel.round(off, b.send_time[a:e], b.dst_host[a:e], b.payload[a:e], rd)
            fail_code = "OK"
        except N.ShdError as ex:
            fail_code = ex.code
        eng.set_knob("TEST_FAIL", 0)
        st, nid = rel.host_state()
        q.put((rank, dict(table=table, rounds=rounds, lo=rel.lo, hi=rel.hi, rng=st[rel.lo:rel.hi].copy(),
                          nid=nid[rel.lo:rel.hi].copy(), fail_code=fail_code)))
        del hc
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_host_comm_two_processes_routing_and_relay():
    from shadow_amd import synth
    res = _spawn(_gpu_worker, 2, timeout=280)
    n = 301
    el = synth.complete_graph(n, 12)
    code, lat, loss, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                      np.arange(n, dtype=np.uint32))
    assert [res[r]["fail_code"] for r in (0, 1)] == ["NOMEM", "NOMEM"]
    for r in (0, 1):
        assert np.array_equal(res[r]["table"][0], lat)
        assert np.array_equal(res[r]["table"][1], loss.view(np.uint32))
    H, NN, P = 5000, 50, 400_000
    el2 = synth.complete_graph(NN, 3)
    code, lat2, loss2, _ = corc.routing(NN, el2.src, el2.dst, el2.latency_ns, el2.packet_loss, False,
                                        np.arange(NN, dtype=np.uint32))
    host_node, rng0 = synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    start, ra = 10**9, 10**6
    for rnd in range(3):
        b = synth.packet_batch(H, P, start, start + ra, seed=90 + rnd)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat2, loss2, orng, onid,
                             start + ra, start + 10**12, start + ra // 2 if rnd == 0 else 0)
        bases = np.array([int(b.src_off[res[r]["lo"]]) for r in (0, 1)], np.int64)
        for r in (0, 1):
            lo, hi = res[r]["lo"], res[r]["hi"]
            status, ev, md, ml, ns = res[r]["rounds"][rnd]
            a, e = int(b.src_off[lo]), int(b.src_off[hi])
            assert np.array_equal(status, o["status"][a:e])
            oe = o["events"]
            s0, s1 = int(oe["off"][lo]), int(oe["off"][hi])
            assert np.array_equal(ev["off"], (oe["off"][lo:hi + 1] - oe["off"][lo]).astype(np.uint32))
            assert np.array_equal(ev["deliver"], oe["deliver"][s0:s1])
            assert np.array_equal(ev["src"], oe["src"][s0:s1])
            assert np.array_equal(ev["seq"], oe["seq"][s0:s1])
            sender = (ev["src"] >= res[1]["lo"]).astype(np.int64)
            assert np.array_equal(ev["pkt"].astype(np.int64) + bases[sender], oe["pkt"][s0:s1].astype(np.int64))
            assert (md, ml, ns) == (o["min_deliver"], o["min_latency"], o["n_sent"])
        start += ra
    for r in (0, 1):
        lo, hi = res[r]["lo"], res[r]["hi"]
        assert np.array_equal(res[r]["rng"], orng[lo:hi])
        assert np.array_equal(res[r]["nid"], onid[lo:hi])
