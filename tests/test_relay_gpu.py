"""GPU parity tests of the per-round relay: statuses, event order per destination, RNG streams,
event ids and round reductions, bit-exact against the golden fixtures and the C restatement."""
import json
import os

import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _u64(xs):
    return np.asarray([int(v) for v in xs], np.uint64)


def test_golden_relay_cases(engine):
    from shadow_amd.relay import Relay
    for case in json.load(open(os.path.join(GOLD, "relay_cases.json"))):
        rng = np.asarray([[int(v) for v in r] for r in case["rng"]], np.uint64).reshape(-1, 4)
        rl = Relay(case["host_node"], rng, _u64(case["next_id"]), np.asarray(case["lat"], np.uint64),
                   np.asarray(case["loss_bits"], np.uint32).view(np.float32), engine=engine)
        r = rl.round(case["src_off"], _u64(case["send_time"]), case["dst_host"], case["payload"],
                     int(case["round_end"]), int(case["sim_end"]), int(case["bootstrap_end"]))
        e = case["expect"]
        assert r.status.tolist() == e["status"], case["name"]
        assert r.ev_off.tolist() == e["ev_off"], case["name"]
        got = [[str(t), int(s), str(q), int(p)] for t, s, q, p in
               zip(r.ev_deliver.tolist(), r.ev_src.tolist(), r.ev_seq.tolist(), r.ev_pkt.tolist())]
        assert got == e["ev"], case["name"]
        assert str(r.min_deliver) == e["min_deliver"] and str(r.min_latency) == e["min_latency"]
        st, nid = rl.host_state()
        assert [[str(v) for v in row] for row in st.tolist()] == e["rng"]
        assert [str(v) for v in nid.tolist()] == e["next_id"]


def _c5_like(n_hosts, n_nodes, n_packets, seed, start=10**9, runahead=10**6):
    from shadow_amd import synth
    el = synth.complete_graph(n_nodes, seed)
    used = np.arange(n_nodes, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    b = synth.packet_batch(n_hosts, n_packets, start, start + runahead, seed=seed)
    return lat, loss, synth.c5_host_nodes(n_hosts, n_nodes), synth.host_rng_states(n_hosts, 1), b


@pytest.mark.parametrize("pipe", [7, 3, 1])
@pytest.mark.parametrize("chance_mode", [False, True])
def test_multi_round_vs_c_oracle(engine, chance_mode, pipe, knob):
    """Three consecutive rounds on 20k hosts / 1M packets: streams and ids carry across rounds
    (bin-placement pipeline, radix-sort pipeline and the 64-bit fallback pipeline)."""
    from shadow_amd.relay import Relay
    knob("RELAY_FORCE_V1", 1 if pipe == 1 else 0)
    knob("RELAY_FORCE_V3", 1 if pipe == 3 else 0)
    H, NN = 20_000, 200
    lat, loss, host_node, rng0, _ = _c5_like(H, NN, 1000, 11)
    nid0 = np.zeros(H, np.uint64)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    orng, onid = rng0.copy(), nid0.copy()
    start, ra = 10**9, 10**6
    for rnd in range(3):
        from shadow_amd import synth
        b = synth.packet_batch(H, 1_000_000, start, start + ra, seed=50 + rnd)
        chance = np.random.default_rng(rnd).random(b.n) if chance_mode else None
        o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                             orng, onid, start + ra, start + 100 * ra, start + ra // 2 if rnd == 0 else 0,
                             chance=chance)
        r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, start + ra, start + 100 * ra,
                     start + ra // 2 if rnd == 0 else 0, chance=chance)
        assert np.array_equal(r.status, o["status"])
        ev = o["events"]
        assert np.array_equal(r.ev_off, ev["off"])
        assert np.array_equal(r.ev_deliver, ev["deliver"])
        assert np.array_equal(r.ev_src, ev["src"])
        assert np.array_equal(r.ev_seq, ev["seq"])
        assert np.array_equal(r.ev_pkt, ev["pkt"])
        assert (r.min_deliver, r.min_latency, r.n_sent) == (o["min_deliver"], o["min_latency"], o["n_sent"])
        st, nid = rl.host_state()
        assert np.array_equal(st, orng) and np.array_equal(nid, onid)
        assert rl.last_pipeline() == pipe
        start += ra


@pytest.mark.parametrize("rel_ids", [False, True])
def test_bin_pipeline_long_runs(engine, rel_ids):
    """Pipeline 7 with destination runs in every class of its per-destination sort: wave
    bitonic (<= 64, <= 128, <= 256 events) and the rank sort of longer runs, inside bins that
    still fit the LDS stage; event ids absolute (32-bit) or relative to a base above 2^40."""
    from shadow_amd.relay import Relay
    H, NN = 3000, 40
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 150_000, 17)
    dst = b.dst_host.copy()
    dst[::300] = 7        # ~500 extra events: rank-sort run
    dst[1::1000] = 70     # ~150 extra: 256-wide bitonic
    dst[2::2000] = 130    # ~75 extra: 128-wide bitonic
    src = np.repeat(np.arange(H), np.diff(b.src_off)).astype(np.uint32)
    dst[(dst == src)] = (dst[(dst == src)] + 1) % H
    nid0 = (np.arange(H, dtype=np.uint64) + np.uint64(2**41)) if rel_ids else np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, dst, b.payload, host_node, lat, loss, rng0.copy(),
                         nid0.copy(), 10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, dst, b.payload, 10**9 + 10**6, 10**12, 0)
    assert rl.last_pipeline() == 7
    ev = o["events"]
    sizes = np.diff(ev["off"].astype(np.int64))
    assert sizes[7] > 256 and 128 < sizes[70] <= 256 and 64 < sizes[130] <= 128
    assert np.array_equal(r.status, o["status"])
    assert np.array_equal(r.ev_off, ev["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
    assert (r.min_deliver, r.min_latency, r.n_sent) == (o["min_deliver"], o["min_latency"], o["n_sent"])


def test_hot_destination_bucket(engine):
    """One destination receiving far more than one LDS bucket (oversized-segment sort path)."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    H, NN = 500, 20
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 200_000, 5)
    dst = b.dst_host.copy()
    dst[::3] = 7
    src = np.repeat(np.arange(H), np.diff(b.src_off)).astype(np.uint32)
    dst[(dst == src)] = (dst[(dst == src)] + 1) % H
    nid0 = np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, dst, b.payload, host_node, lat, loss, rng0.copy(),
                         nid0.copy(), 10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, dst, b.payload, 10**9 + 10**6, 10**12, 0)
    ev = o["events"]
    assert int(ev["off"][8] - ev["off"][7]) > 1024
    assert rl.last_pipeline() == 3   # the hot bin overflows pipeline 7's LDS stage: radix rerun
    assert np.array_equal(r.ev_off, ev["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
    del synth


def test_packet_counts(engine):
    from shadow_amd.relay import Relay
    H, NN = 1000, 30
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 50_000, 3)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    src = np.repeat(np.arange(H), np.diff(b.src_off))
    sent = r.status == 2
    want = np.zeros((NN, NN), np.uint64)
    np.add.at(want, (host_node[src[sent]], host_node[b.dst_host[sent]]), 1)
    assert np.array_equal(rl.packet_counts(), want)


def test_empty_and_all_skipped_rounds(engine):
    from shadow_amd.relay import Relay
    H = 10
    rl = Relay(np.zeros(H, np.uint32), np.ones((H, 4), np.uint64), np.zeros(H, np.uint64),
               np.full((1, 1), 10**6, np.uint64), np.zeros((1, 1), np.float32), engine=engine)
    r = rl.round(np.zeros(H + 1, np.uint32), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                 np.zeros(0, np.uint32), 10, 100, 0)
    assert r.n_sent == 0 and r.min_deliver == 2**64 - 1
    off = np.arange(H + 1, dtype=np.uint32)
    r = rl.round(off, np.full(H, 500, np.uint64), (np.arange(H) + 1) % H, np.ones(H, np.uint32), 10, 100, 0)
    assert r.n_sent == 0 and (r.status == 0).all()
    st, _ = rl.host_state()
    assert (st == 1).all()   # no draw for completed sends


def test_wide_latency_table_and_failed_round_keeps_state(engine):
    """Paths >= 2^32 ns take the 64-bit pipeline; a round naming an unknown host fails with
    NO_HOST and leaves every RNG stream and event id untouched."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    from shadow_amd._native import ShdError
    H, NN = 300, 12
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 20_000, 8)
    lat = lat * np.uint64(3)
    lat[0, 1] = np.uint64(5 * 2**32)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**13, 0)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    bad = b.dst_host.copy()
    bad[len(bad) // 2] = H + 5
    with pytest.raises(ShdError, match="NO_HOST"):
        rl.round(b.src_off, b.send_time, bad, b.payload, 10**9 + 10**6, 10**13, 0)
    st, nid = rl.host_state()
    assert np.array_equal(st, rng0) and (nid == 0).all()
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**13, 0)
    assert np.array_equal(r.status, o["status"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), o["events"][k]), k
    del synth


@pytest.mark.parametrize("lds_map", [True, False])
@pytest.mark.parametrize("n_hosts", [300, 2000, 5000])
def test_bucket_size_classes(engine, n_hosts, lds_map, knob):
    """Destination runs of every size class of the per-run sort (<= 64, <= 128, <= 256 events
    per destination, and longer runs on the merge path) against the C restatement; both stamp
    kernels (host -> node map resident in LDS, or gathered from global memory)."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    knob("RELAY_NO_LDS_MAP", 0 if lds_map else 1)
    NN = 50
    lat, loss, host_node, rng0, b = _c5_like(n_hosts, NN, 400_000, 13)
    nid0 = np.arange(n_hosts, dtype=np.uint64) * np.uint64(7)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), nid0.copy(), 10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    ev = o["events"]
    sizes = np.diff(ev["off"].astype(np.int64))
    assert sizes.max() > 64
    assert np.array_equal(r.status, o["status"])
    assert np.array_equal(r.ev_off, ev["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
    del synth


def test_many_source_nodes_per_workgroup(engine):
    """One host per node on a 3000-node table: a stamp workgroup's source rows do not fit the
    LDS stage, so the path gathers go to global memory (the other tests use the staged rows)."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    NN = 3000
    el = synth.barabasi_albert(NN, 2, 23)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    assert code == "OK"
    H = NN
    b = synth.packet_batch(H, 300_000, 10**9, 10**9 + 10**6, seed=29)
    host_node = np.random.default_rng(3).permutation(NN).astype(np.uint32)
    rng0 = synth.host_rng_states(H, 1)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    assert np.array_equal(r.status, o["status"])
    ev = o["events"]
    assert np.array_equal(r.ev_off, ev["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k


def test_sim_end_inside_round_and_wide_event_ids(engine):
    """sim_end falls inside the round: every host's sends from sim_end on are skipped (no draw,
    worker.rs:334-341).  Event ids start above 2^40, so records carry relative ids."""
    from shadow_amd.relay import Relay
    from shadow_amd._native import ShdError
    H, NN = 4000, 100
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 400_000, 19)
    nid0 = (np.uint64(1) << np.uint64(40)) + np.arange(H, dtype=np.uint64) * np.uint64(1000)
    sim_end = 10**9 + 6 * 10**5                      # 60% into the send window
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), nid0.copy(), 10**9 + 10**6, sim_end, 0)
    assert 0 < int((o["status"] == 0).sum()) < len(b.send_time)
    rl = Relay(host_node, rng0, nid0, lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, sim_end, 0)
    assert np.array_equal(r.status, o["status"])
    ev = o["events"]
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), ev[k]), k
    st, nid = rl.host_state()
    # a drawing send after a skipped one (send times going backwards) is rejected, state kept
    t = b.send_time.copy()
    h = int(np.argmax(np.diff(b.src_off) > 3))
    a0 = int(b.src_off[h])
    t[a0], t[a0 + 1] = np.uint64(sim_end + 5), np.uint64(sim_end - 5)
    with pytest.raises(ShdError, match="INVALID"):
        rl.round(b.src_off, t, b.dst_host, b.payload, 10**9 + 10**6, sim_end, 0)
    st2, nid2 = rl.host_state()
    assert np.array_equal(st, st2) and np.array_equal(nid, nid2)


def test_bin_pipeline_failed_round_keeps_state(engine):
    """Pipeline 7: a round naming an unknown host fails with NO_HOST (the stamp skips placing
    that packet, the histogram skips counting it) and leaves RNG streams and event ids
    untouched; the next valid round runs on pipeline 7 bit-exact."""
    from shadow_amd.relay import Relay
    from shadow_amd._native import ShdError
    H, NN = 2000, 40
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 100_000, 21)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    bad = b.dst_host.copy()
    bad[::997] = H + 3
    with pytest.raises(ShdError, match="NO_HOST"):
        rl.round(b.src_off, b.send_time, bad, b.payload, 10**9 + 10**6, 10**12, 0)
    st, nid = rl.host_state()
    assert np.array_equal(st, rng0) and (nid == 0).all()
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    assert rl.last_pipeline() == 7
    assert np.array_equal(r.status, o["status"]) and np.array_equal(r.ev_off, o["events"]["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), o["events"][k]), k


def test_bin_pipeline_large_workgroup_segment_stays_on_bins(engine):
    """64 hosts = one stamp workgroup, 5,000 sends into two bins: every bin fits pipeline 7's
    LDS stage, and the workgroup's segment of each (~2,500 records) is far past the 8-bit slot
    counters the stamp had before round 6, which made this round rerun on the radix pipeline.
    The counters are 32-bit now: pipeline 7, bit-exact."""
    from shadow_amd.relay import Relay
    H, NN = 64, 8
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 5_000, 23)
    orng, onid = rng0.copy(), np.zeros(H, np.uint64)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss,
                         orng, onid, 10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, 10**9 + 10**6, 10**12, 0)
    assert rl.last_pipeline() == 7
    assert np.array_equal(r.status, o["status"]) and np.array_equal(r.ev_off, o["events"]["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), o["events"][k]), k
    st, nid = rl.host_state()
    assert np.array_equal(st, orng) and np.array_equal(nid, onid)


def test_device_batch_unaligned_inputs(engine):
    """shd_relay_round_device with the batch arrays one element past a 16-byte boundary: the
    histogram's vector form needs 16-byte aligned destinations, so its flattened-position form
    runs; statuses and events bit-exact against the C oracle, on pipeline 7."""
    import ctypes as C

    import torch

    from shadow_amd import _native as N
    from shadow_amd.relay import Relay
    H, NN = 3000, 40
    lat, loss, host_node, rng0, b = _c5_like(H, NN, 200_000, 29)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    keep = []

    def dev(a, np_dt, t_dt, pad=1):   # the array `pad` elements into a fresh device buffer
        buf = torch.zeros(len(a) + pad, dtype=t_dt, device="cuda")
        buf[pad:] = torch.from_numpy(np.ascontiguousarray(a, np_dt).view(t_dt == torch.int64 and np.int64 or np.int32)).cuda()
        keep.append(buf)
        return buf.data_ptr() + pad * buf.element_size()

    n = b.n
    batch = N.Batch(n, dev(b.src_off, np.uint32, torch.int32, 0), dev(b.send_time, np.uint64, torch.int64),
                    dev(b.dst_host, np.uint32, torch.int32), dev(b.payload, np.uint32, torch.int32), None)
    outs = [torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(H + 1, dtype=torch.int32, device="cuda"),
            torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
            torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda")]
    out = N.RelayOut(*(t.data_ptr() for t in outs), 0, 0, 0)
    rd = N.Round(10**9 + 10**6, 10**12, 0)
    N.check(engine.lib.shd_relay_round_device(engine.ctx, C.byref(batch), C.byref(rd), C.byref(out)), "round")
    assert rl.last_pipeline() == 7
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                         np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    ns = out.n_sent
    assert ns == o["n_sent"]
    assert np.array_equal(outs[0].cpu().numpy(), o["status"])
    assert np.array_equal(outs[1].cpu().numpy().view(np.uint32), o["events"]["off"])
    for t, k, dt in ((outs[2], "deliver", np.uint64), (outs[3], "src", np.uint32), (outs[4], "seq", np.uint64),
                     (outs[5], "pkt", np.uint32)):
        assert np.array_equal(t[:ns].cpu().numpy().view(dt), o["events"][k]), k


@pytest.mark.parametrize("loss01", [0.999, 0.3, 0.001])
@pytest.mark.parametrize("above", [False, True])
def test_draw_top_bits_at_the_drop_threshold(engine, loss01, above):
    """K0 keeps a draw's top 32 bits only.  The drop test chance >= reliability is
    draw >> 11 >= T = ceil(reliability * 2^53), and for reliability = 1f32 - loss with a loss in
    [0, 1] T is a multiple of 2^21, so the top bits decide it exactly (relay.hip draw_drops).
    Host 0's first draw is crafted (Xoshiro256++ output solved for s3) to sit just below or at
    the threshold; the statuses match the oracle's f64 comparison on pipeline 7."""
    from fractions import Fraction
    import math

    from shadow_amd import synth
    from shadow_amd.relay import Relay
    M = 2**64 - 1
    lf = np.float32(loss01)
    q = np.float32(1.0) - lf                         # reliability as Rust computes it (f32)
    T = math.ceil(Fraction(float(q)) * 2**53)       # chance >= reliability  <=>  draw >> 11 >= T
    assert T % 2**21 == 0
    X64 = (T if above else T - 1) << 11
    s0, s1, s2 = 0x0123456789ABCDEF, 0x0FEDCBA987654321, 0x13579BDF2468ACE0
    r = (X64 - s0) & M
    s3 = ((((r >> 23) | (r << 41)) & M) - s0) & M   # rotl(s0 + s3, 23) + s0 == X64
    H = 4
    rng0 = synth.host_rng_states(H, 1)
    rng0[0] = np.array([s0, s1, s2, s3], np.uint64)
    host_node = np.array([0, 1, 0, 1], np.uint32)
    lat = np.array([[1000, 5000], [5000, 1000]], np.uint64)
    loss = np.array([[0, lf], [lf, 0]], np.float32)
    src_off = np.array([0, 3, 3, 3, 3], np.uint32)   # host 0 sends three packets to host 1
    t = np.array([10**9, 10**9 + 10, 10**9 + 20], np.uint64)
    dst = np.array([1, 1, 1], np.uint32)
    pay = np.array([1448, 1448, 1448], np.uint32)
    rd = (10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    res = rl.round(src_off, t, dst, pay, *rd)
    orng = rng0.copy()
    o = corc.relay_round(src_off, t, dst, pay, host_node, lat, loss, orng, np.zeros(H, np.uint64), *rd)
    assert rl.last_pipeline() == 7
    assert res.status.tolist() == o["status"].tolist()
    assert res.status[0] == (1 if above else 2)      # dropped at the threshold, sent just below it
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(res, "ev_" + k), o["events"][k]), k
    st, _ = rl.host_state()
    assert np.array_equal(st, orng)


def test_clamped_deliver_times_tie_everywhere(engine):
    """Path latencies far below the round's span: almost every event's deliver time clamps to
    round_end (worker.rs:398-401), so each destination run is one big tie that the EventQueue
    order breaks by (src host, event id).  The per-destination sorts' 32-bit fast path must see
    the ties and fall back to the packet order; bit-exact against the C oracle."""
    from shadow_amd import synth
    from shadow_amd.relay import Relay
    H, NN, P = 2000, 30, 200_000
    lat = np.full((NN, NN), 1000, np.uint64)          # 1 us everywhere
    loss = np.zeros((NN, NN), np.float32)
    host_node = synth.c5_host_nodes(H, NN)
    rng0 = synth.host_rng_states(H, 1)
    b = synth.packet_batch(H, P, 10**9, 10**9 + 10**6, seed=41)
    rd = (10**9 + 10**6, 10**12, 0)
    rl = Relay(host_node, rng0, np.zeros(H, np.uint64), lat, loss, engine=engine)
    r = rl.round(b.src_off, b.send_time, b.dst_host, b.payload, *rd)
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, lat, loss, rng0.copy(),
                         np.zeros(H, np.uint64), *rd)
    assert rl.last_pipeline() == 7
    assert (r.ev_deliver == 10**9 + 10**6).mean() > 0.99
    assert np.array_equal(r.status, o["status"]) and np.array_equal(r.ev_off, o["events"]["off"])
    for k in ("deliver", "src", "seq", "pkt"):
        assert np.array_equal(getattr(r, "ev_" + k), o["events"][k]), k
