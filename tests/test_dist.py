"""World-size-2 gloo tests of the multi-GPU sharding logic on the CPU.

The device compute is replaced by the C restatement (test infrastructure) behind the same ``ops``
interface, so these tests check the sharding, the all-to-all exchange plan, the global packet
ids, the k-way merge contract and the MIN reductions against a single-process run.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleOps:
    """CPU stand-in for shadow_amd.dist.DeviceOps (same interface)."""

    def __init__(self, el=None, host_node=None, lat=None, loss=None, rng=None, next_id=None):
        self.el, self.host_node, self.lat, self.loss = el, host_node, lat, loss
        self.rng, self.next_id = rng, next_id

    def routing_rows(self, rb, re, lat_out, loss_out):
        el = self.el
        used = np.arange(el.n_nodes, dtype=np.uint32)
        code, lat, loss, _ = corc.routing(el.n_nodes, el.src, el.dst, el.latency_ns, el.packet_loss,
                                          el.directed, used)
        assert code == "OK"
        lat_out[: re - rb].copy_(torch.from_numpy(lat[rb:re].view(np.int64)))
        loss_out[: re - rb].copy_(torch.from_numpy(loss[rb:re]))

    def relay_round(self, src_off, send_time, dst_host, payload, n_hosts, round_):
        r = corc.relay_round(src_off.numpy().view(np.uint32), send_time.numpy().view(np.uint64),
                             dst_host.numpy().view(np.uint32), payload.numpy().view(np.uint32),
                             self.host_node, self.lat, self.loss, self.rng, self.next_id, *round_)
        ev = r["events"]
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt).copy())  # noqa: E731
        return dict(status=t(r["status"], np.uint8), ev_off=t(ev["off"], np.int32),
                    ev_deliver=t(ev["deliver"], np.int64), ev_src=t(ev["src"], np.int32),
                    ev_seq=t(ev["seq"], np.int64), ev_pkt=t(ev["pkt"], np.int32),
                    min_deliver=r["min_deliver"], min_latency=r["min_latency"], n_sent=r["n_sent"])

    def merge(self, n_runs, n_dst, run_base, run_off, deliver, src, seq, pkt):
        off = run_off.numpy().reshape(n_runs, n_dst + 1).astype(np.int64)
        base = run_base.numpy().astype(np.int64)
        d, s, q, p = deliver.numpy(), src.numpy(), seq.numpy(), pkt.numpy()
        ev_off = [0]
        rows = []
        for dd in range(n_dst):
            seg = []
            for r in range(n_runs):
                a, b = base[r] + off[r, dd], base[r] + off[r, dd + 1]
                seg.extend(zip(d[a:b].view(np.uint64), s[a:b], q[a:b].view(np.uint64), p[a:b]))
            seg.sort(key=lambda e: (int(e[0]), int(e[1]), int(e[2])))
            rows.extend(seg)
            ev_off.append(len(rows))
        arr = lambda i, dt: torch.tensor(np.array([e[i] for e in rows], dtype=dt).view(  # noqa: E731
            {np.uint64: np.int64, np.int32: np.int32}.get(dt, dt)))
        return dict(ev_off=torch.tensor(ev_off, dtype=torch.int32), ev_deliver=arr(0, np.uint64),
                    ev_src=arr(1, np.int32), ev_seq=arr(2, np.uint64), ev_pkt=arr(3, np.int32))


def _relay_case():
    from shadow_amd import synth
    H, NN = 300, 25
    el = synth.complete_graph(NN, 7)
    used = np.arange(NN, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False, used)
    b = synth.packet_batch(H, 40_000, 10**9, 10**9 + 10**6, seed=21)
    return H, lat, loss, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1), b


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shadow_amd import dist as D
        from shadow_amd import synth
        # ---- routing: sharded rows + all-gather
        el = synth.complete_graph(37, 3)
        ops = OracleOps(el=el)
        per = (37 + world - 1) // world
        lat_full = torch.zeros((world * per, 37), dtype=torch.int64)
        loss_full = torch.zeros((world * per, 37), dtype=torch.float32)
        lat, loss = D.sharded_routing(ops, 37, lat_full, loss_full)
        # ---- relay: hosts sharded by id; this rank stamps only its source hosts
        H, tl, tloss, host_node, rng0, b = _relay_case()
        lo, hi = D.host_shard(H, world, rank)
        a, e = int(b.src_off[lo]), int(b.src_off[hi])
        off = np.zeros(H + 1, np.uint32)
        off[lo + 1:hi + 1] = b.src_off[lo + 1:hi + 1] - a
        off[hi + 1:] = e - a
        rops = OracleOps(host_node=host_node, lat=tl, loss=tloss, rng=rng0.copy(),
                         next_id=np.zeros(H, np.uint64))
        T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt))  # noqa: E731
        rd = (10**9 + 10**6, 10**12, 0)
        out = D.sharded_relay_round(rops, H, T(off, np.int32), T(b.send_time[a:e], np.int64),
                                    T(b.dst_host[a:e], np.int32), T(b.payload[a:e], np.int32), rd)
        q.put((rank, lat.numpy().copy(), loss.numpy().copy(),
               {k: (v.numpy().copy() if torch.is_tensor(v) else v) for k, v in out.items()},
               rops.rng[lo:hi].copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_world2_sharded_routing_and_relay_match_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, lat, loss, out, rng = q.get(timeout=240)
        res[rank] = (lat, loss, out, rng)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # routing: every rank holds the full table, equal to the single-process build
    from shadow_amd import synth
    el = synth.complete_graph(37, 3)
    code, want_lat, want_loss, _ = corc.routing(37, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                                np.arange(37, dtype=np.uint32))
    for r in range(world):
        assert np.array_equal(res[r][0].view(np.uint64), want_lat)
        assert np.array_equal(res[r][1].view(np.uint32), want_loss.view(np.uint32))
    # relay: the union of per-rank destination events equals one single-process round
    H, tl, tloss, host_node, rng0, b = _relay_case()
    rng_full = rng0.copy()
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, tl, tloss, rng_full,
                         np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    ev = o["events"]
    from shadow_amd.dist import host_shard
    for r in range(world):
        lo, hi = host_shard(H, world, r)
        out = res[r][2]
        a, e = int(ev["off"][lo]), int(ev["off"][hi])
        assert np.array_equal(out["ev_off"].astype(np.int64), ev["off"][lo:hi + 1].astype(np.int64) - a)
        assert np.array_equal(out["ev_deliver"].view(np.uint64), ev["deliver"][a:e])
        assert np.array_equal(out["ev_src"].view(np.uint32), ev["src"][a:e])
        assert np.array_equal(out["ev_seq"].view(np.uint64), ev["seq"][a:e])
        assert np.array_equal(out["ev_pkt"].view(np.uint32), ev["pkt"][a:e])
        assert out["min_deliver"] == o["min_deliver"] and out["min_latency"] == o["min_latency"]
        assert out["n_sent"] == o["n_sent"]
        assert np.array_equal(res[r][3], rng_full[lo:hi])   # source-owned streams advanced exactly


def test_shards_partition_rows_and_hosts():
    from shadow_amd.dist import host_shard, row_shard
    for n in (1, 2, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            parts = [row_shard(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert host_shard(n, w, w - 1)[1] == n
