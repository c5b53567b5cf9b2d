"""The exact N >= 2 code paths at BASELINE.json's real sizes, in one process on one GPU.

RCCL refuses two ranks on one GPU, so two contexts on cuda:0 under the in-process communicator
(shd_comm_init_local) stand in for two ranks; everything below the transport -- row shards, the
chunked table exchange with its slot reserve, the relay's sizing exchange, the packed record
exchange, the receiver's merge, the per-rank queues and the agreed window -- is the code the
driver's multi-GPU runs execute (the seam they replace: manager.rs:404-464).

  * C4 -- the 50k-node BA m=4 graph sharded over two ranks: each rank's 15 GB share moves in
          ~256 MB row chunks while the next chunk is built, the build leaving 32 slots free
          from the second chunk on (api.cpp shd_routing_run_sharded).  Rows on both sides of
          every chunk boundary of both ranks and the last 64 rows against the row-range oracle
          (graph/mod.rs:185-230); the two ranks' 30 GB tables identical.
  * C5 -- 100k hosts x 10M packets per round, sharded by host over two ranks, three rounds of
          shd_relay_round_sharded -> per-rank shd_equeue_advance under the window shd_round_window
          agrees, against the C restatement's relay into per-host heaps (worker.rs:328-413,
          event_queue.rs:28-48, controller.rs:86-111).
"""
import numpy as np
import pytest

from oracle import corc
from tests.test_comm_gpu import _run_ranks, _slice_batch

pytestmark = pytest.mark.gpu


def _chunk_rows(per: int, row_bytes: int) -> int:
    """api.cpp chunk_rows() at its defaults: ~256 MB of table per chunk, at least 4 chunks."""
    return min(max(1, (256 << 20) // row_bytes), (per + 3) // 4)


def _ranges_to_check(n, world, per, cs):
    rows = set()
    for r in range(world):
        rb, re = r * per, min(n, (r + 1) * per)
        for s in range(rb, re, cs):   # both sides of every chunk start
            rows.update(x for x in (s - 1, s) if 0 <= x < n)
        rows.add(re - 1)
    rows.update(range(n - 64, n))
    rows = sorted(rows)
    out, a = [], rows[0]
    for x, y in zip(rows, rows[1:] + [None]):
        if y != x + 1:
            out.append((a, x + 1))
            a = y
    return out


def test_c4_two_ranks_chunked_exchange_bit_exact():
    import ctypes as C

    import torch

    from shadow_amd import _native as N
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    from tests.graphs import engine_graph_from_edges
    n, world = 50_000, 2
    el = synth.barabasi_albert(n, 4, 3)
    used = np.arange(n, dtype=np.uint32)
    per = (n + world - 1) // world
    cs = _chunk_rows(per, n * 12)
    assert per * n * 12 > (256 << 20) and cs < per   # the chunked path, not one all-gather
    engines = [Engine(0) for _ in range(world)]
    try:
        for e in engines:
            assert e.get_knob("SHARD_RESERVE_SLOTS") is None   # the default 32-slot reserve
            assert e.get_knob("SHARD_CHUNK_ROWS") is None
        D.comm_init_local(engines)
        g = engine_graph_from_edges(el)
        bufs = []
        for e in engines:
            cg = g._cgraph()
            err = N.Error()
            N.check(e.lib.shd_routing_prepare(e.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST, C.byref(err)),
                    "prepare", err)
            bufs.append((torch.empty((world * per, n), dtype=torch.int64, device="cuda"),
                         torch.empty((world * per, n), dtype=torch.float32, device="cuda")))
        torch.cuda.synchronize()
        _run_ranks([lambda e=e, b=b: D.routing_run_sharded(e, N.ALGO_DELTA, b[0], b[1])
                    for e, b in zip(engines, bufs)])
        torch.cuda.synchronize()
        for e in engines:
            info = e.last_info()
            assert info["algo_used"] == N.ALGO_DELTA and info["wide_latency"] == 0
        # both ranks hold the same whole table (their own rows and every received chunk)
        assert torch.equal(bufs[0][0][:n], bufs[1][0][:n])
        assert torch.equal(bufs[0][1][:n].view(torch.int32), bufs[1][1][:n].view(torch.int32))
        ranges = _ranges_to_check(n, world, per, cs)
        assert len(ranges) >= 2 * ((per + cs - 1) // cs)
        for lo, hi in ranges:
            code, lat, loss, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, False, used,
                                              rows=(lo, hi))
            assert code == "OK"
            got_l = bufs[1][0][lo:hi].cpu().numpy().view(np.uint64)
            got_p = bufs[1][1][lo:hi].cpu().numpy().view(np.uint32)
            assert np.array_equal(got_l, lat), (lo, hi)
            assert np.array_equal(got_p, loss.view(np.uint32)), (lo, hi)
        del bufs
        torch.cuda.empty_cache()
    finally:
        for e in engines:
            e.close()


def test_c5_two_ranks_relay_queues_window_bit_exact():
    import torch

    from oracle.relay import RunaheadState, next_window
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.rounds import Runahead, next_window as eng_window
    from shadow_amd.routing import Engine
    H, NN, P, world = 100_000, 1000, 10_000_000, 2
    el = synth.complete_graph(NN, 1)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    engines = [Engine(0) for _ in range(world)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        queues = [EventQueues(e, H) for e in engines]
        min_possible = int(lat.min())
        for e in engines:
            Runahead(e, True, min_possible)
        ora = RunaheadState(True, min_possible)
        oq = corc.EventQueues(H)
        orng, onid = rng0.copy(), np.zeros(H, np.uint64)
        end_time = synth.SIM_START + 10**9 + 10**12
        ws = synth.SIM_START + 10**9
        we = ws + ora.get()
        dev = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()  # noqa: E731
        bases = []
        for rnd in range(3):
            b = synth.packet_batch(H, P, ws, we, seed=4 + rnd)
            rd = (we, end_time, 0)
            o = corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                                    *rd, queues=oq, batch_no=rnd)
            if o["min_latency"] != 2**64 - 1:
                ora.update_lowest_used_latency(o["min_latency"])
            want_win = next_window(min(oq.pop(0, want=False)["next_time"], 2**64 - 1), ora.get(), end_time)
            parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
            bases.append([p[4] for p in parts])   # per round: each sender rank's batch base
            d_parts = [[dev(p[0], np.int32), dev(p[1], np.int64), dev(p[2], np.int32), dev(p[3], np.int32)]
                       for p in parts]
            sts = [torch.empty(max(len(p[1]), 1), dtype=torch.uint8, device="cuda") for p in parts]
            torch.cuda.synchronize()

            def rank_round(i):
                out = rels[i].round_device(*d_parts[i], rd, sts[i])
                win = eng_window(engines[i], None, end_time)
                qo = queues[i].advance_device(out, win[1])
                return win, (out.min_deliver, out.min_latency, out.n_sent), queues[i].popped(qo)
            res = _run_ranks([lambda i=i: rank_round(i) for i in range(world)])
            op = oq.pop(want_win[1])
            for i, ((win, red, p), q) in enumerate(zip(res, queues)):
                assert win == want_win, (rnd, i, win, want_win)
                assert red == (o["min_deliver"], o["min_latency"], o["n_sent"])
                a0, a1 = int(b.src_off[rels[i].lo]), int(b.src_off[rels[i].hi])
                assert np.array_equal(sts[i][: a1 - a0].cpu().numpy(), o["status"][a0:a1])
                a, z = int(op["off"][q.lo]), int(op["off"][q.hi])
                assert np.array_equal(p.off.astype(np.int64), op["off"][q.lo:q.hi + 1].astype(np.int64) - a)
                assert np.array_equal(p.deliver, op["deliver"][a:z])
                assert np.array_equal(p.src, op["src"][a:z])
                assert np.array_equal(p.seq, op["seq"][a:z])
                # tag = batch << 32 | the packet's index in its SENDER rank's batch of that round
                sender = (p.src >= rels[1].lo).astype(np.int64)
                batch = (p.tag >> np.uint64(32)).astype(np.int64)
                glob = (p.tag & np.uint64(0xFFFFFFFF)).astype(np.int64) + np.asarray(bases, np.int64)[batch, sender]
                assert np.array_equal(glob, (op["tag"][a:z] & np.uint64(0xFFFFFFFF)).astype(np.int64))
                assert np.array_equal(p.tag >> np.uint64(32), op["tag"][a:z] >> np.uint64(32))
            assert sum(p.n_pending for _, _, p in res) == op["n_pending"]
            ws, we = want_win
        for r in rels:   # the own hosts' RNG streams and event ids after three rounds
            st, nid = r.host_state()
            assert np.array_equal(st[r.lo:r.hi], orng[r.lo:r.hi])
            assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
    finally:
        for e in engines:
            e.close()
