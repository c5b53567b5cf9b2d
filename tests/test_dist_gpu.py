"""Two ranks on one GPU (gloo for the collectives, HIP engine for the compute): the sharded
routing build and the sharded relay round with the device k-way merge, bit-exact against one
single-process C-restatement run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import corc

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case():
    from shadow_amd import synth
    H, NN = 3000, 200
    el = synth.complete_graph(NN, 5)
    b = synth.packet_batch(H, 300_000, 10**9, 10**9 + 10**6, seed=33)
    return H, NN, el, b, synth.c5_host_nodes(H, NN), synth.host_rng_states(H, 1)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import ctypes as C
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from shadow_amd import _native as N
        from shadow_amd import dist as D
        from shadow_amd.routing import Engine, NetworkGraph
        dev = torch.device("cuda", 0)
        eng = Engine(0)
        H, NN, el, b, host_node, rng0 = _case()
        g = NetworkGraph(el.node_ids, el.src, el.dst, el.latency_ns, el.packet_loss, el.directed)
        used = np.arange(NN, dtype=np.uint32)
        cg = g._cgraph()
        err = N.Error()
        N.check(eng.lib.shd_routing_prepare(eng.ctx, C.byref(cg), N.ptr(used), NN, 0, C.byref(err)), "prep")
        ops = D.DeviceOps(eng, dev)
        per = (NN + world - 1) // world
        lat_full = torch.zeros((world * per, NN), dtype=torch.int64, device=dev)
        loss_full = torch.zeros((world * per, NN), dtype=torch.float32, device=dev)
        lat, loss = D.sharded_routing(ops, NN, lat_full, loss_full)
        lat_np = lat.cpu().numpy().view(np.uint64).copy()
        loss_np = loss.cpu().numpy().copy()
        N.check(eng.lib.shd_relay_setup(eng.ctx, H, N.ptr(host_node), NN, N.ptr(lat_np), N.ptr(loss_np),
                                        N.ptr(rng0), N.ptr(np.zeros(H, np.uint64))), "relay_setup")
        lo, hi = D.host_shard(H, world, rank)
        a, e = int(b.src_off[lo]), int(b.src_off[hi])
        off = np.zeros(H + 1, np.uint32)
        off[lo + 1:hi + 1] = b.src_off[lo + 1:hi + 1] - a
        off[hi + 1:] = e - a
        T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x).view(dt)).to(dev)  # noqa: E731
        out = D.sharded_relay_round(ops, H, T(off, np.int32), T(b.send_time[a:e], np.int64),
                                    T(b.dst_host[a:e], np.int32), T(b.payload[a:e], np.int32),
                                    (10**9 + 10**6, 10**12, 0))
        n = int(out["ev_off"][-1].item())
        q.put((rank, lat_np, loss_np,
               {k: (v[:n].cpu().numpy().copy() if torch.is_tensor(v) and k != "ev_off" and k != "status"
                    else v.cpu().numpy().copy() if torch.is_tensor(v) else v) for k, v in out.items()}))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_one_gpu_bit_exact():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, lat, loss, out = q.get(timeout=240)
        res[rank] = (lat, loss, out)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    H, NN, el, b, host_node, rng0 = _case()
    code, want_lat, want_loss, _ = corc.routing(NN, el.src, el.dst, el.latency_ns, el.packet_loss, False,
                                                np.arange(NN, dtype=np.uint32))
    o = corc.relay_round(b.src_off, b.send_time, b.dst_host, b.payload, host_node, want_lat, want_loss,
                         rng0.copy(), np.zeros(H, np.uint64), 10**9 + 10**6, 10**12, 0)
    ev = o["events"]
    from shadow_amd.dist import host_shard
    for r in range(world):
        lat, loss, out = res[r]
        assert np.array_equal(lat, want_lat) and np.array_equal(loss.view(np.uint32), want_loss.view(np.uint32))
        lo, hi = host_shard(H, world, r)
        a, e = int(ev["off"][lo]), int(ev["off"][hi])
        assert np.array_equal(out["ev_off"].astype(np.int64), ev["off"][lo:hi + 1].astype(np.int64) - a)
        assert np.array_equal(out["ev_deliver"].view(np.uint64), ev["deliver"][a:e])
        assert np.array_equal(out["ev_src"].view(np.uint32), ev["src"][a:e])
        assert np.array_equal(out["ev_seq"].view(np.uint64), ev["seq"][a:e])
        assert np.array_equal(out["ev_pkt"].view(np.uint32), ev["pkt"][a:e])
        assert (out["min_deliver"], out["min_latency"], out["n_sent"]) == (o["min_deliver"], o["min_latency"],
                                                                          o["n_sent"])
