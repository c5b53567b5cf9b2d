"""Shape-sweep parity of the relay stamp (worker.rs:361-411 restated by corc.relay_round).

The stamp kernel (relay.hip relay_stamp_v6) walks host groups in source-node order; each group
stages its source nodes' path rows in LDS when they fit (rows x n_nodes <= 2048 entries) and,
when a workgroup walks more than one group, prefetches the next group's rows while the current
one runs.  Round 4 shipped an out-of-bounds LDS index in that prefetch (a next group spanning
three or more source nodes read another node's row).  These tests run every branch -- staged and
unstaged rows, prefetched or not, one or many groups per workgroup, groups spanning 1 to 64
source nodes -- against the C restatement, comparing every status and every event field, on one
context and on two in-process ranks (the sharded round)."""
import numpy as np
import pytest

from oracle import corc
from tests.test_comm_gpu import _check_rank, _run_ranks, _slice_batch

pytestmark = pytest.mark.gpu

N_CU = 256            # MI355X compute units: the stamp's persistent grid (relay.hip relay_device_v7)
ROW_LDS = 2048        # kS5RowLds: staged path-table entries per group
GROUP_SENDS = 4096    # kS6Cap: v7_group_size's default sends per group


def _tables(n_nodes, seed):
    """A random path table: distinct latencies (us granularity) and losses up to 0.3, so a
    wrong row changes deliver times and drop decisions."""
    rng = np.random.default_rng(seed)
    lat = rng.integers(1_000, 300_000, size=(n_nodes, n_nodes)).astype(np.uint64) * np.uint64(1000)
    loss = rng.uniform(0.0, 0.3, size=(n_nodes, n_nodes)).astype(np.float32)
    return lat, loss


def _batch(H, per_host, seed, start, span, same_instant=False):
    from shadow_amd.synth import PacketBatch
    rng = np.random.default_rng(seed)
    n = H * per_host
    src = np.repeat(np.arange(H, dtype=np.uint32), per_host)
    dst = rng.integers(0, H - 1, size=n, dtype=np.uint32)
    dst = dst + (dst >= src).astype(np.uint32)
    u = rng.random(n)
    pay = np.where(u < 0.2, 0, np.where(u < 0.8, 1448, rng.integers(1, 1449, size=n))).astype(np.uint32)
    if same_instant:
        t = np.full(n, start, np.uint64)
    else:
        t = rng.integers(start, start + span, size=n, dtype=np.uint64).reshape(H, per_host)
        t = np.sort(t, axis=1).reshape(-1)
    off = (np.arange(H + 1, dtype=np.uint64) * per_host).astype(np.uint32)
    return PacketBatch(off, t, dst, pay)


def _group_size(n_src, G, n, S=GROUP_SENDS):
    """relay.hip v7_group_size (S = the RELAY_GROUP_SENDS knob)."""
    if not S or not n or not n_src or not G:
        return 64
    want = int(min(64.0, max(8.0, S / (n / n_src))))
    m = -(-n_src // (G * want))
    return int(min(64, max(1, -(-n_src // (G * m)))))


def _stamp_branches(host_node, lo, hi, n_nodes, n_packets, sends, pipeline=7, S=GROUP_SENDS):
    """Which stamp branches a round over hosts [lo, hi) runs: staged groups, unstaged groups,
    prefetched groups and the largest source-node count of a prefetched one.  Pipeline 7 sizes
    its groups by v7_group_size, pipeline 3 takes 64 hosts; both launch min(groups, CUs)."""
    n_src = hi - lo
    order = lo + np.argsort(host_node[lo:hi], kind="stable")
    G = min(-(-n_src // 64), N_CU)
    gs = _group_size(n_src, G, n_packets, S) if pipeline == 7 else 64
    ng = -(-n_src // gs)
    out = dict(groups=ng, G=G, gs=gs, staged=0, unstaged=0, prefetched=0, pf_rows_max=0)
    for g in range(ng):
        hs = order[g * gs:(g + 1) * gs]
        rows = len(np.unique(host_node[hs]))
        staged = rows * n_nodes <= ROW_LDS
        out["staged" if staged else "unstaged"] += 1
        prev = g - G
        if prev >= 0 and staged:
            ph = order[prev * gs:(prev + 1) * gs]
            if sends[ph].sum() > 0:   # the previous group of the workgroup ran a chunk
                out["prefetched"] += 1
                out["pf_rows_max"] = max(out["pf_rows_max"], rows)
    return out


def _check_single(engine, lat, loss, host_node, rng0, nid0, b, rd):
    from shadow_amd.relay import Relay
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                         nid0.copy(), *rd)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, *rd)
    assert rl.last_pipeline() in (7, 3)   # 3: a bin over bin_sort_v7's LDS stage
    bad = np.flatnonzero(r.status != o["status"])
    assert len(bad) == 0, f"{len(bad)} status mismatches, first at sends {bad[:8].tolist()}"
    ev = o["events"]
    assert np.array_equal(r.ev_off, ev["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
    assert (r.min_deliver, r.min_latency, r.n_sent) == (o["min_deliver"], o["min_latency"], o["n_sent"])
    return rl


SWEEP = [(nn, hpn, sph) for nn in (20, 40, 200, 682, 683) for hpn in (1, 3, 10, 25) for sph in (8, 75, 200)]
_seen = []


@pytest.mark.parametrize("n_nodes,hpn,sph", SWEEP)
def test_stamp_shape_sweep(engine, n_nodes, hpn, sph):
    """n_nodes x hosts-per-node x sends-per-host against the C restatement, statuses and every
    event field; host h on node h mod n_nodes (the probe's layout)."""
    H = n_nodes * hpn
    lat, loss = _tables(n_nodes, n_nodes)
    host_node = (np.arange(H) % n_nodes).astype(np.uint32)
    from shadow_amd import synth
    rng0 = synth.host_rng_states(H, 1)
    nid0 = np.zeros(H, np.uint64)
    b = _batch(H, sph, 1000 + n_nodes * 31 + hpn * 7 + sph, 10**9, 10**6)
    rl = _check_single(engine, lat, loss, host_node, rng0, nid0, b, (10**9 + 10**6, 10**12, 0))
    pipe = rl.last_pipeline()
    _seen.append(dict(_stamp_branches(host_node, 0, H, n_nodes, b.n, np.diff(b.src_off.astype(np.int64)), pipe),
                      pipeline=pipe))


@pytest.mark.parametrize("n_nodes,hpn,sph,S,rows", [(40, 1, 8, 256, 20), (30, 2, 4, 128, 15), (32, 4, 6, 192, 8),
                                                   (20, 1, 8, 96, 10), (64, 1, 4, 128, 32)])
def test_stamp_prefetch_wide_groups(engine, knob, n_nodes, hpn, sph, S, rows):
    """Few hosts per node and small groups (the RELAY_GROUP_SENDS knob): a workgroup walks
    several groups, each spanning `rows` source nodes whose staged rows are prefetched while the
    previous group runs -- the overrun's shape at its widest (pipeline 7, no bin overflow)."""
    from shadow_amd import synth
    knob("RELAY_GROUP_SENDS", S)
    H = n_nodes * hpn
    lat, loss = _tables(n_nodes, 5 * n_nodes + hpn)
    host_node = (np.arange(H) % n_nodes).astype(np.uint32)
    rng0 = synth.host_rng_states(H, 1)
    b = _batch(H, sph, 500 + n_nodes + S, 10**9, 10**6)
    br = _stamp_branches(host_node, 0, H, n_nodes, b.n, np.diff(b.src_off.astype(np.int64)), 7, S)
    assert br["prefetched"] and br["pf_rows_max"] == rows, br
    rl = _check_single(engine, lat, loss, host_node, rng0, np.zeros(H, np.uint64), b, (10**9 + 10**6, 10**12, 0))
    assert rl.last_pipeline() == 7
    _seen.append(dict(br, pipeline=7))


def test_stamp_shape_sweep_covered_every_branch():
    """The sweep above ran every branch of the stamp's group walk at least once."""
    if len(_seen) < len(SWEEP) + 5:
        pytest.skip("the sweep did not run in this session")
    assert any(s["groups"] > s["G"] for s in _seen)             # several groups per workgroup
    assert any(s["groups"] <= s["G"] for s in _seen)            # one group per workgroup
    assert any(s["unstaged"] for s in _seen) and any(s["staged"] for s in _seen)
    assert any(s["prefetched"] for s in _seen)
    assert any(s["pf_rows_max"] >= 3 for s in _seen)            # the round-4 overrun's shape
    assert max(s["pf_rows_max"] for s in _seen) >= 20
    assert {s["pipeline"] for s in _seen} == {3, 7}


def _probe_case(same_instant):
    from shadow_amd import synth
    H, NN, P = 2000, 40, 150_000
    el = synth.complete_graph(NN, 8)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                      np.arange(NN, dtype=np.uint32))
    assert code == "OK"
    host_node, rng0 = synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)
    start = 10**9
    b = synth.packet_batch(H, P, start, start + 10**6, seed=7)
    if same_instant:
        b.send_time[:] = start
    return H, lat, loss, host_node, rng0, b, (start + 10**6, start + 10**12, 0)


@pytest.mark.parametrize("same_instant", [False, True])
def test_probe_batch_single_context(engine, same_instant):
    """Round 4's probe batch (2000 hosts on 40 nodes, 150k sends, seed 7) on one context."""
    H, lat, loss, host_node, rng0, b, rd = _probe_case(same_instant)
    _check_single(engine, lat, loss, host_node, rng0, np.zeros(H, np.uint64), b, rd)


@pytest.mark.parametrize("same_instant", [False, True])
def test_probe_batch_two_ranks(engine, same_instant):
    """The probe batch through shd_relay_round_sharded on two in-process ranks: a rank's 1000
    hosts form groups of 32 that span up to 3 source nodes, the shape whose prefetched rows the
    round-4 stamp read out of bounds.  Statuses, every event field, reductions, RNG streams and
    event ids against the C restatement."""
    from shadow_amd import dist as D
    from shadow_amd.routing import Engine
    H, lat, loss, host_node, rng0, b, rd = _probe_case(same_instant)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid, *rd)
    engines = [Engine(0), Engine(0)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
        for r in rels:
            br = _stamp_branches(host_node, r.lo, r.hi, lat.shape[0], int(b.src_off[r.hi] - b.src_off[r.lo]),
                                 np.diff(b.src_off.astype(np.int64)))
            assert br["pf_rows_max"] >= 3, br
        outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
        assert [r.last_pipeline() for r in rels] == [8, 8]   # the bins went to their ranks as stamped
        bases = np.array([p[4] for p in parts], np.int64)
        split = rels[1].lo

        def a_of(src):
            return bases[(src >= split).astype(np.int64)]
        for r, out in zip(rels, outs):
            _check_rank(out, o, r.lo, r.hi, a_of, b)
        for r in rels:
            st, nid = r.host_state()
            assert np.array_equal(st[r.lo:r.hi], orng[r.lo:r.hi])
            assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("n_nodes,hpn,sph", [(40, 25, 75), (20, 10, 200), (200, 3, 8), (683, 1, 75)])
def test_shape_sweep_two_ranks(engine, n_nodes, hpn, sph):
    """A few sweep shapes on two in-process ranks (each rank's own group walk) with equal send
    times, so most destinations also take the merge's tie path."""
    from shadow_amd import dist as D
    from shadow_amd import synth
    from shadow_amd.routing import Engine
    H = n_nodes * hpn
    lat, loss = _tables(n_nodes, 3 * n_nodes)
    host_node = (np.arange(H) % n_nodes).astype(np.uint32)
    rng0 = synth.host_rng_states(H, 1)
    b = _batch(H, sph, 77 + n_nodes + hpn + sph, 10**9, 10**6, same_instant=True)
    rd = (10**9 + 10**6, 10**12, 0)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, orng, onid, *rd)
    engines = [Engine(0), Engine(0)]
    try:
        D.comm_init_local(engines)
        rels = [D.ShardedRelay(e, host_node, rng0, np.zeros(H, np.uint64), lat, loss) for e in engines]
        parts = [_slice_batch(b, r.lo, r.hi) for r in rels]
        outs = _run_ranks([lambda r=r, p=p: r.round(*p[:4], rd) for r, p in zip(rels, parts)])
        bases = np.array([p[4] for p in parts], np.int64)
        split = rels[1].lo

        def a_of(src):
            return bases[(src >= split).astype(np.int64)]
        for r, out in zip(rels, outs):
            _check_rank(out, o, r.lo, r.hi, a_of, b)
        for r in rels:
            st, nid = r.host_state()
            assert np.array_equal(st[r.lo:r.hi], orng[r.lo:r.hi])
            assert np.array_equal(nid[r.lo:r.hi], onid[r.lo:r.hi])
    finally:
        for e in engines:
            e.close()
