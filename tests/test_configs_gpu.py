"""Parity at BASELINE.json's configured sizes, against the C restatement:

  * C3 -- the 10k-node BA graph, the whole 10k x 10k table, every routing engine;
  * C4 -- the 50k-node BA m=4 graph: its table is 30 GB, so source-row slices at the start, the
          middle and the end of the used set, built by the global-label kernel, checked against
          the row-range oracle (orc_shortest_paths_rows);
  * C5 -- 100k hosts x 10M packets per round on the C2 table, two consecutive rounds (RNG
          streams and event ids carried), every status and every event compared;
  * C5b -- the C5 round on the resident C4 table (50k nodes), checked on a 1M-send slice.
"""
import numpy as np
import pytest

from oracle import corc
from tests.graphs import engine_graph_from_edges

pytestmark = pytest.mark.gpu


def _assert_rows(t, lat, loss):
    assert np.array_equal(t.lat, lat)
    assert np.array_equal(t.loss.view(np.uint32), loss.view(np.uint32))


@pytest.fixture(scope="module")
def c4():
    from shadow_amd import synth
    el = synth.barabasi_albert(50_000, 4, 3)
    return el, engine_graph_from_edges(el), np.arange(50_000, dtype=np.uint32)


@pytest.mark.parametrize("rows", [(0, 64), (25_000, 25_064), (49_936, 50_000)])
def test_c4_row_slices_bit_exact(engine, c4, rows):
    el, g, used = c4
    code, lat, loss, _ = corc.routing(50_000, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                      used, rows=rows)
    assert code == "OK"
    for algo in (1, 3):   # label-correcting SSSP, delta-stepping (both on the global-label kernel)
        t = g.compute_shortest_paths(used, engine, algo=algo, rows=rows)
        info = engine.last_info()
        assert info["algo_used"] == algo and info["wide_latency"] == 0
        _assert_rows(t, lat, loss)


def test_c4_claimed_rows_bit_exact(engine, c4):
    """C4 rows [0, 2048) in one launch: the 2 x n_cu slots (512 on MI355X) take their first rows by
    index and every later row from the row counter, so rows 1536-1599 and 1984-2047 are claimed
    rows of the same kernel that runs the benchmarked build -- compared against the row-range
    oracle (graph/mod.rs:185-230)."""
    el, g, used = c4
    t = g.compute_shortest_paths(used, engine, algo=3, rows=(0, 2048))
    info = engine.last_info()
    assert info["algo_used"] == 3 and info["wide_latency"] == 0
    for lo, hi in ((1536, 1600), (1984, 2048)):
        code, lat, loss, _ = corc.routing(50_000, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                          used, rows=(lo, hi))
        assert code == "OK"
        assert np.array_equal(t.lat[lo:hi], lat)
        assert np.array_equal(t.loss[lo:hi].view(np.uint32), loss.view(np.uint32))
    del t


def test_c3_full_table_bit_exact(engine):
    from shadow_amd import synth
    el = synth.barabasi_albert(10_000, 3, 2)
    used = np.arange(10_000, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(10_000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    g = engine_graph_from_edges(el)
    for algo, ran in ((0, 3), (1, 1), (3, 3), (4, 4)):   # AUTO runs delta buckets on a sparse graph
        t = g.compute_shortest_paths(used, engine, algo=algo)
        assert engine.last_info()["algo_used"] == ran
        _assert_rows(t, lat, loss)
        del t


def test_c5_full_two_rounds_bit_exact(engine):
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    H, P = 100_000, 10_000_000
    el = synth.complete_graph(1000, 1)
    used = np.arange(1000, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(1000, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    host_node = synth.c5_host_nodes(H, 1000)
    rng0 = synth.host_rng_states(H, 1)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    rl = Relay(host_node, rng0, onid.copy(), lat, loss, engine=engine)
    start, ra = synth.SIM_START + 10**9, 10**6
    for rnd in range(2):
        b = synth.packet_batch(H, P, start, start + ra, seed=4 + rnd)
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                             orng, onid, start + ra, start + 10**12, 0)
        r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, start + ra, start + 10**12, 0)
        assert rl.last_pipeline() == 7
        assert np.array_equal(r.status, o["status"])
        ev = o["events"]
        assert np.array_equal(r.ev_off, ev["off"])
        for k in ("deliver", "src", "seq", "pkt"):
            assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
        assert (r.min_deliver, r.min_latency, r.n_sent) == (o["min_deliver"], o["min_latency"], o["n_sent"])
        st, nid = rl.host_state()
        assert np.array_equal(st, orng) and np.array_equal(nid, onid)
        start += ra


def test_c5b_relay_on_resident_c4_table(engine):
    """C5b: 100k hosts on the C4 graph's 50k nodes (host h on node h mod 50,000),
    10M sends, the relay reading the engine's resident 30 GB C4 table (pipeline 7 with the
    stamp's global host -> node map: the packed map does not fit its LDS).  The first round from the setup state against the C restatement
    on the sends of source hosts 0-9,999 (~1M): their statuses and every destination's events from
    them (bench.c5b_slice_check)."""
    import bench
    from shadow_amd.relay import Relay
    cs = bench.c5b_setup(engine)   # (turns the per-path counters off: 2 x 20 GB at 50k nodes)
    try:
        b, H = cs["b"], cs["H"]
        # the Relay wrapper over the same resident table (lat = None), host buffers in and out
        rl = Relay(cs["host_node"], cs["rng0"], np.zeros(H, np.uint64), engine=engine)
        r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, *cs["rd"])
        assert rl.last_pipeline() == 7   # the bins, the stamp gathering the destinations' nodes
        assert bench.c5b_slice_check(engine, cs, r.status, r.ev_off, r.ev_deliver, r.ev_src, r.ev_seq, r.ev_pkt)
    finally:   # the session engine's default for the tests that follow
        assert engine.lib.shd_relay_set_counters(engine.ctx, 1) == 0
