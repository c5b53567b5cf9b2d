"""GPU tests of the engine's multi-GPU path through the C ABI (shd_comm_*, shd_*_sharded).

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so the two-rank tests use the
in-process communicator (shd_comm_init_local): two contexts on cuda:0, each driven by its own
host thread, exactly as two ranks would run; the sharding, the sizing exchange, the packed
record exchange and the merge are the same code as under RCCL.  The RCCL transport itself runs
at world size 1 here (and at 8 in the driver's scaling bench)."""
import threading

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def _run_ranks(fns):
    res, errs = [None] * len(fns), []

    def wrap(i):
        try:
            res[i] = fns[i]()
        except BaseException as e:   # noqa: BLE001 -- reported below
            errs.append(e)
    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    if errs:
        raise errs[0]
    return res


def _case(H, NN, seed):
    from shadow_amd import synth
    el = synth.complete_graph(NN, seed)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    return el, lat, loss, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)


def _slice_batch(b, lo, hi):
    a, e = int(b.src_off[lo]), int(b.src_off[hi])
    return (b.src_off[lo:hi + 1] - b.src_off[lo]).astype(np.uint32), b.send_time[a:e], b.dst_host[a:e], b.payload[a:e], a


def _check_rank(rank_out, o, lo, hi, a_of, b):
    status, ev, md, ml, ns = rank_out
    a, e = int(b.src_off[lo]), int(b.src_off[hi])
    assert np.array_equal(status, o["status"][a:e])
    oe = o["events"]
    s0, s1 = int(oe["off"][lo]), int(oe["off"][hi])
    assert np.array_equal(ev["off"], (oe["off"][lo:hi + 1] - oe["off"][lo]).astype(np.uint32))
    assert np.array_equal(ev["deliver"], oe["deliver"][s0:s1])
    assert np.array_equal(ev["src"], oe["src"][s0:s1])
    assert np.array_equal(ev["seq"], oe["seq"][s0:s1])
    # ev_pkt is the index in the sender rank's batch: the sender's batch base gives the global one
    glob = ev["pkt"].astype(np.int64) + a_of(ev["src"])
    assert np.array_equal(glob, oe["pkt"][s0:s1].astype(np.int64))
    assert (md, ml, ns) == (o["min_deliver"], o["min_latency"], o["n_sent"])


@pytest.mark.parametrize("path", ["bins", "x24"])
def test_local_two_ranks_relay_rounds(engine, knob, path):
    """Three rounds on two ranks, both exchange forms: the stamp's bins sent to their destination
    ranks and sorted there (default, pipeline 8), and the packed 24-byte events merged per
    destination (RELAY_SHARD_X24, the fallback form)."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    H, NN, P = 5000, 50, 400_000
    _, lat, loss, host_node, rng0 = _case(H, NN, 3)
    engines = [Engine(0), Engine(0)]
    try:
        for e in engines:
            knob("RELAY_SHARD_X24", 1 if path == "x24" else 0, eng=e)
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        assert [(r.lo, r.hi) for r in rels] == [(0, 2500), (2500, 5000)]
        orng, onid = rng0.copy(), np.zeros(H, np.uint64)
        start, ra = 10**9, 10**6
        for rnd in range(3):
            b = synth.packet_batch(H, P, start, start + ra, seed=90 + rnd)
            o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                                 start + ra, start + 10**12, start + ra // 2 if rnd == 0 else 0)
            rd = (start + ra, start + 10**12, start + ra // 2 if rnd == 0 else 0)
            parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
            outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
            assert [r.last_pipeline() for r in rels] == ([8, 8] if path == "bins" else [7, 7])
            bases = np.array([p[4] for p in parts], np.int64)

            def a_of(src):
                return bases[(src >= 2500).astype(np.int64)]
            for r, out in zip(rels, outs):
                _check_rank(out, o, r.lo, r.hi, a_of, b)
            for r in rels:   # each rank's own hosts carry the advanced streams and ids
                st, nid = r.host_state()
                assert np.array_equal(st[r.lo:r.hi], orng[r.lo:r.hi])
                assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
            start += ra
    finally:
        for e in engines:
            e.close()


def test_local_two_ranks_failure_is_global(engine):
    """A bad destination on rank 1 fails the round on both ranks; no rank commits state."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd._native import ShdError
    from shadow_amd.routing import Engine
    H, NN = 1000, 20
    _, lat, loss, host_node, rng0 = _case(H, NN, 5)
    engines = [Engine(0), Engine(0)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        b = synth.packet_batch(H, 50_000, 10**9, 10**9 + 10**6, seed=7)
        parts = [list(_slice_batch(b, r.lo, r.hi)) for r in rels]
        parts[1][2] = parts[1][2].copy()
        parts[1][2][5] = H + 9
        rd = (10**9 + 10**6, 10**12, 0)

        def go(r, p):
            try:
                r.round(*p[:4], rd)
            except ShdError as e:
                return e.code
            return "OK"
        codes = _run_ranks([lambda r=r, p=p: go(r, p) for r, p in zip(rels, parts)])
        assert codes == ["NO_HOST", "NO_HOST"]
        for r in rels:
            st, nid = r.host_state()
            assert np.array_equal(st, rng0) and not nid.any()
    finally:
        for e in engines:
            e.close()


def test_local_two_ranks_failure_after_gather_is_global(engine, knob):
    """A failure on rank 1 after the sizing gather (injected: TEST_FAIL=1) rides the exchange's
    status part: both ranks return it, neither commits host state, and the next round, with the
    failure gone, is bit-exact against the restatement (advisor round 5)."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd._native import ShdError
    from shadow_amd.routing import Engine
    H, NN = 1000, 20
    _, lat, loss, host_node, rng0 = _case(H, NN, 5)
    engines = [Engine(0), Engine(0)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        b = synth.packet_batch(H, 50_000, 10**9, 10**9 + 10**6, seed=7)
        parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
        rd = (10**9 + 10**6, 10**12, 0)

        def go(r, p):
            try:
                r.round(*p[:4], rd)
            except ShdError as e:
                return e.code
            return "OK"
        knob("TEST_FAIL", 1, eng=engines[1])
        codes = _run_ranks([lambda r=r, p=p: go(r, p) for r, p in zip(rels, parts)])
        assert codes == ["HIP", "HIP"]
        for r in rels:
            st, nid = r.host_state()
            assert np.array_equal(st, rng0) and not nid.any()
        knob("TEST_FAIL", 0, eng=engines[1])
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                             np.zeros(H, np.uint64), *rd)
        outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
        assert [r.last_pipeline() for r in rels] == [8, 8]
        bases = np.array([p[4] for p in parts], np.int64)
        for r, out in zip(rels, outs):
            _check_rank(out, o, r.lo, r.hi, lambda src: bases[(src >= 500).astype(np.int64)], b)
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("chunk_rows", [None, 7, 64, "replicate"])
def test_local_two_ranks_routing_sharded(engine, chunk_rows):
    """Row shards + the table exchange: one all-gather, or row chunks exchanged while the next
    chunk is built (SHD_SHARD_CHUNK_ROWS forces the chunked path on a small graph; 7 leaves a
    short last chunk, 64 a rank whose last chunk is shorter than its peer's); "replicate" is the
    small-table default, every rank building the whole table (SHD_SHARD_REPLICATE_MB=0 turns it
    off for the exchange cases)."""
    import torch
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    from tests.graphs import engine_graph_from_edges
    import ctypes as C
    from shadow_amd import _native as N
    n = 301
    el = synth.complete_graph(n, 12)
    used = np.arange(n, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    engines = [Engine(0), Engine(0)]
    try:
        for e in engines:
            if chunk_rows != "replicate":
                e.set_knob("SHARD_REPLICATE_MB", 0)
            if chunk_rows not in (None, "replicate"):
                e.set_knob("SHARD_CHUNK_ROWS", chunk_rows)
        D.comm_init_local(engines)
        g = engine_graph_from_edges(el)
        per = (n + 1) // 2
        bufs = []
        for e in engines:
            cg = g._cgraph()
            err = N.Error()
            N.check(e.lib.shd_routing_prepare(e.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST, C.byref(err)),
                    "prepare", err)
            bufs.append((torch.empty((2 * per, n), dtype=torch.int64, device="cuda"),
                         torch.empty((2 * per, n), dtype=torch.float32, device="cuda")))
        torch.cuda.synchronize()
        _run_ranks([lambda e=e, b=b: D.routing_run_sharded(e, N.ALGO_AUTO, b[0], b[1]) for e, b in zip(engines, bufs)])
        for lt, ls in bufs:
            assert np.array_equal(lt[:n].cpu().numpy().view(np.uint64), lat)
            assert np.array_equal(ls[:n].cpu().numpy().view(np.uint32), loss.view(np.uint32))
    finally:
        for e in engines:
            e.close()


def test_rccl_world_one(engine):
    """The RCCL transport at world size 1: the sharded relay and routing calls go through
    ncclAllToAll / grouped send-recv / ncclAllGather with this rank alone."""
    import ctypes as C

    import torch
    from shadow_amd import _native as N
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    from tests.graphs import engine_graph_from_edges
    H, NN = 2000, 40
    el, lat, loss, host_node, rng0 = _case(H, NN, 8)
    e = Engine(0)
    try:
        D.comm_init_rccl(e)
        r = D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss)
        b = synth.packet_batch(H, 100_000, 10**9, 10**9 + 10**6, seed=8)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                             np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
        out = r.round(b.src_off, b.send_time, b.dst_host, b.payload, (10**9 + 10**6, 10**12, 0))
        _check_rank(out, o, 0, H, lambda src: np.zeros(len(src), np.int64), b)
        g = engine_graph_from_edges(el)
        cg = g._cgraph()
        used = np.arange(NN, dtype=np.uint32)
        err = N.Error()
        N.check(e.lib.shd_routing_prepare(e.ctx, C.byref(cg), N.ptr(used), NN, N.ROUTE_SHORTEST, C.byref(err)),
                "prepare", err)
        lt = torch.empty((NN, NN), dtype=torch.int64, device="cuda")
        ls = torch.empty((NN, NN), dtype=torch.float32, device="cuda")
        D.routing_run_sharded(e, N.ALGO_AUTO, lt, ls)
        assert np.array_equal(lt.cpu().numpy().view(np.uint64), lat)
        assert np.array_equal(ls.cpu().numpy().view(np.uint32), loss.view(np.uint32))
    finally:
        e.close()


@pytest.mark.parametrize("dynamic", [True, False])
def test_local_two_ranks_relay_into_queues_with_window(engine, dynamic):
    """The north star's relay path at N = 2 through the C ABI alone, round after round: each rank's
    sharded relay output (its destination shard) goes into its own device queues
    (shd_equeue_setup under the communicator), the next window comes from shd_round_window (the
    runahead updated by every round's min latency, the minimum over both ranks' queues), and each
    rank pops its hosts' events below that window.  Compared per round with one process:
    the C restatement's relay into persistent per-host heaps, Runahead and the controller's window
    (manager.rs:404-464, runahead.rs:43-115, controller.rs:86-111)."""
    import torch
    from oracle.relay import RunaheadState, next_window
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.equeue import EventQueues
    from shadow_amd.rounds import Runahead, next_window as eng_window
    from shadow_amd.routing import Engine
    H, NN, P = 4000, 40, 200_000
    _, lat, loss, host_node, rng0 = _case(H, NN, 11)
    engines = [Engine(0), Engine(0)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        queues = [EventQueues(e, H) for e in engines]
        assert [(q.lo, q.hi) for q in queues] == [(r.lo, r.hi) for r in rels]
        min_possible = int(lat.min())
        cfg = 2 * 10**6 if not dynamic else None
        for e in engines:
            Runahead(e, dynamic, min_possible, cfg)
        ora = RunaheadState(dynamic, min_possible, cfg)
        oq = corc.EventQueues(H)
        orng, onid = rng0.copy(), np.zeros(H, np.uint64)
        end_time = 10**9 + 400 * 10**6
        ws, we = 10**9, 10**9 + ora.get()
        bases = np.zeros((5, 2), np.int64)   # per round: each sender rank's batch base in the whole batch
        for rnd in range(5):
            b = synth.packet_batch(H, P, ws, we, seed=120 + rnd)
            rd = (we, end_time, 0)
            o = corc.relay_round_eq(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid,
                                    *rd, queues=oq, batch_no=rnd)
            if o["min_latency"] != 2**64 - 1:
                ora.update_lowest_used_latency(o["min_latency"])
            want_win = next_window(min(oq.pop(0, want=False)["next_time"], 2**64 - 1), ora.get(), end_time)
            parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
            bases[rnd] = [parts[0][4], parts[1][4]]

            def rank_round(i):
                r, p, e = rels[i], parts[i], engines[i]
                d = [_dev(p[0], np.int32), _dev(p[1], np.int64), _dev(p[2], np.int32), _dev(p[3], np.int32)]
                st = torch.empty(max(len(p[1]), 1), dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                out = r.round_device(*d, rd, st)
                win = eng_window(e, None, end_time)
                qo = queues[i].advance_device(out, win[1] if win else 2**63)
                return win, queues[i].popped(qo)
            res = _run_ranks([lambda i=i: rank_round(i) for i in range(2)])
            assert res[0][0] == res[1][0] == want_win, (rnd, res[0][0], want_win)
            op = oq.pop(want_win[1])
            for (win, p), q in zip(res, queues):
                a, z = int(op["off"][q.lo]), int(op["off"][q.hi])
                assert np.array_equal(p.off.astype(np.int64), op["off"][q.lo:q.hi + 1].astype(np.int64) - a)
                assert np.array_equal(p.deliver, op["deliver"][a:z])
                assert np.array_equal(p.src, op["src"][a:z])
                assert np.array_equal(p.seq, op["seq"][a:z])
                # tag: batch << 32 | the packet's index in its SENDER rank's batch of that round
                sender = (p.src >= rels[1].lo).astype(np.int64)
                batch = (p.tag >> np.uint64(32)).astype(np.int64)
                glob = (p.tag & np.uint64(0xFFFFFFFF)).astype(np.int64) + bases[batch, sender]
                assert np.array_equal(glob, (op["tag"][a:z] & np.uint64(0xFFFFFFFF)).astype(np.int64))
                assert np.array_equal(p.tag >> np.uint64(32), op["tag"][a:z] >> np.uint64(32))
            assert sum(p.n_pending for _, p in res) == op["n_pending"]
            ws, we = want_win
    finally:
        for e in engines:
            e.close()


def _dev(a, dt):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()


@pytest.mark.parametrize("world,H,path", [(3, 5003, "bins"), (4, 4099, "bins"), (5, 3001, "bins"), (3, 5003, "x24"),
                                          (8, 2000, "bins")])
def test_local_many_ranks_relay_rounds(engine, knob, world, H, path):
    """World sizes past two with host counts that split unevenly (the last rank's shard and last
    bin are short; with 8 ranks on 2000 hosts every shard ends inside a bin of 32): two rounds,
    every rank's statuses, events, reductions, streams and ids against the C restatement, and
    the same round through the bin exchange and the packing form."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    NN, P = 40, 60 * H
    _, lat, loss, host_node, rng0 = _case(H, NN, 7 + world)
    engines = [Engine(0) for _ in range(world)]
    try:
        for e in engines:
            knob("RELAY_SHARD_X24", 1 if path == "x24" else 0, eng=e)
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        bounds = [(r.lo, r.hi) for r in rels]
        assert bounds[0][0] == 0 and bounds[-1][1] == H
        orng, onid = rng0.copy(), np.zeros(H, np.uint64)
        start, ra = 10**9, 10**6
        for rnd in range(2):
            b = synth.packet_batch(H, P, start, start + ra, seed=300 + world + rnd)
            rd = (start + ra, start + 10**12, start + ra // 2 if rnd == 0 else 0)
            o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid, *rd)
            parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
            outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
            assert {r.last_pipeline() for r in rels} == ({8} if path == "bins" else {7})
            bases = np.array([p[4] for p in parts], np.int64)
            his = np.array([hi for _, hi in bounds], np.int64)

            def a_of(src):
                return bases[np.searchsorted(his, src.astype(np.int64), side="right")]
            for r, out in zip(rels, outs):
                _check_rank(out, o, r.lo, r.hi, a_of, b)
            for r in rels:
                st, nid = r.host_state()
                assert np.array_equal(st[r.lo:r.hi], orng[r.lo:r.hi])
                assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
            start += ra
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("world,chunk_rows", [(3, None), (4, 9), (8, 5), (8, None)])
def test_local_many_ranks_routing_sharded(engine, world, chunk_rows):
    """The sharded routing build past two ranks: uneven row shards (301 rows), one all-gather or
    chunked exchanges with short last chunks; every rank's whole table against the C restatement."""
    import ctypes as C

    import torch
    from shadow_amd import _native as N
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    from tests.graphs import engine_graph_from_edges
    n = 301
    el = synth.complete_graph(n, 20 + world)
    used = np.arange(n, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(n, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    engines = [Engine(0) for _ in range(world)]
    try:
        for e in engines:
            e.set_knob("SHARD_REPLICATE_MB", 0)
            if chunk_rows:
                e.set_knob("SHARD_CHUNK_ROWS", chunk_rows)
        D.comm_init_local(engines)
        g = engine_graph_from_edges(el)
        per = (n + world - 1) // world
        bufs = []
        for e in engines:
            cg = g._cgraph()
            err = N.Error()
            N.check(e.lib.shd_routing_prepare(e.ctx, C.byref(cg), N.ptr(used), n, N.ROUTE_SHORTEST, C.byref(err)),
                    "prepare", err)
            bufs.append((torch.empty((world * per, n), dtype=torch.int64, device="cuda"),
                         torch.empty((world * per, n), dtype=torch.float32, device="cuda")))
        torch.cuda.synchronize()
        _run_ranks([lambda e=e, b=b: D.routing_run_sharded(e, N.ALGO_AUTO, b[0], b[1]) for e, b in zip(engines, bufs)])
        for lt, ls in bufs:
            assert np.array_equal(lt[:n].cpu().numpy().view(np.uint64), lat)
            assert np.array_equal(ls[:n].cpu().numpy().view(np.uint32), loss.view(np.uint32))
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("world,H", [(4, 3), (3, 7)])
def test_local_ranks_without_hosts_or_sends(engine, world, H):
    """More ranks than hosts (a rank owning no host) and ranks whose hosts send nothing: every
    rank agrees on the round (the bin exchange needs every rank on pipeline 7, so the packing
    form runs) and the results match the C restatement."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    NN = 3
    _, lat, loss, host_node, rng0 = _case(H, NN, 31)
    engines = [Engine(0) for _ in range(world)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        bounds = [(r.lo, r.hi) for r in rels]
        b = synth.packet_batch(H, 40, 10**9, 10**9 + 10**6, seed=5)
        # the first host sends nothing
        keep = np.ones(b.n, bool)
        keep[: int(b.src_off[1])] = False
        cnt = np.diff(b.src_off.astype(np.int64))
        cnt[0] = 0
        off = np.zeros(H + 1, np.uint32)
        np.cumsum(cnt, out=off[1:])
        b = synth.PacketBatch(off, b.send_time[keep], b.dst_host[keep], b.payload[keep])
        rd = (10**9 + 10**6, 10**12, 0)
        orng, onid = rng0.copy(), np.zeros(H, np.uint64)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid, *rd)
        parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
        outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
        bases = np.array([p[4] for p in parts], np.int64)
        his = np.array([hi for _, hi in bounds], np.int64)

        def a_of(src):
            return bases[np.searchsorted(his, src.astype(np.int64), side="right")]
        for r, out in zip(rels, outs):
            _check_rank(out, o, r.lo, r.hi, a_of, b)
    finally:
        for e in engines:
            e.close()
