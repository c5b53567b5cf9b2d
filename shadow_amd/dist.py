"""Multi-GPU sharding of the two paths over torch.distributed (RCCL on ROCm, gloo in CPU tests).

One process per GPU:
  * routing build: the used-node source rows are split into contiguous shards; every rank runs
    its rows (no collective inside the SSSP -- rows are independent) and one all-gather leaves
    the full table on every rank;
  * relay: hosts are split by id into contiguous ranges.  A rank stamps the sends of ITS source
    hosts (their RNG streams / event ids live there) into events grouped by destination; the
    events bound for rank r's hosts are one contiguous slice, exchanged with one all-to-all(v)
    per array; the receiver k-way merges the per-sender runs (senders own disjoint source
    ranges, so the merge by (deliver, src, seq) is EventQueue order again).  min deliver time
    and min latency are all-reduced with MIN.  Every event has deliver >= round_end,
    so exchanging at the round barrier is exact.

The local compute goes through an ``ops`` object: :class:`DeviceOps` runs the HIP engine on
torch device tensors; the CPU tests plug in the C restatement instead to check the sharding,
exchange and merge logic with gloo at world size 2.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N

U64_MAX = (1 << 64) - 1
I64_MAX = (1 << 63) - 1


def row_shard(n: int, world: int, rank: int):
    per = (n + world - 1) // world
    return min(rank * per, n), min((rank + 1) * per, n)


def host_shard(n_hosts: int, world: int, rank: int):
    return row_shard(n_hosts, world, rank)


def _u64_as_i64(x: int) -> int:
    """u64 reduction value as an int64 tensor element: values >= 2^63 (only "none", u64::MAX,
    occurs in practice) clamp to I64_MAX, which maps back to u64::MAX."""
    return I64_MAX if x >= I64_MAX else int(x)


def _host_coll(group) -> bool:
    """gloo moves host tensors only: stage device tensors through the CPU (tests on one GPU)."""
    return dist.get_backend(group) == "gloo"


def _a2a(out, inp, out_splits=None, in_splits=None, group=None):
    if _host_coll(group) and inp.is_cuda:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_gather(out, inp, group=None):
    if _host_coll(group) and inp.is_cuda:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_reduce(t, op, group=None):
    if _host_coll(group) and t.is_cuda:
        c = t.cpu()
        dist.all_reduce(c, op=op, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=op, group=group)


class DeviceOps:
    """Local compute on the HIP engine (device tensors)."""

    def __init__(self, engine, device):
        self.eng = engine
        self.device = device

    def empty(self, n, dtype):
        return torch.empty(n, dtype=dtype, device=self.device)

    def routing_rows(self, rb, re, lat_out, loss_out):
        err = N.Error()
        st = self.eng.lib.shd_routing_run(self.eng.ctx, N.ALGO_AUTO, rb, re, N.ptr(lat_out),
                                          N.ptr(loss_out), C.byref(err))
        N.check(st, "shd_routing_run", err)

    def relay_round(self, src_off, send_time, dst_host, payload, n_hosts, round_):
        n = send_time.numel()
        out = dict(status=self.empty(max(n, 1), torch.uint8), ev_off=self.empty(n_hosts + 1, torch.int32),
                   ev_deliver=self.empty(max(n, 1), torch.int64), ev_src=self.empty(max(n, 1), torch.int32),
                   ev_seq=self.empty(max(n, 1), torch.int64), ev_pkt=self.empty(max(n, 1), torch.int32))
        b = N.Batch(n, N.ptr(src_off).value, N.ptr(send_time).value, N.ptr(dst_host).value,
                    N.ptr(payload).value, None)
        o = N.RelayOut(*(N.ptr(out[k]).value for k in ("status", "ev_off", "ev_deliver", "ev_src",
                                                        "ev_seq", "ev_pkt")), 0, 0, 0)
        rd = N.Round(*round_)
        N.check(self.eng.lib.shd_relay_round_device(self.eng.ctx, C.byref(b), C.byref(rd), C.byref(o)),
                "shd_relay_round_device")
        out.update(min_deliver=o.min_deliver, min_latency=o.min_latency, n_sent=o.n_sent)
        return out

    def merge(self, n_runs, n_dst, run_base, run_off, deliver, src, seq, pkt):
        n = int(deliver.numel())
        out = dict(ev_off=self.empty(n_dst + 1, torch.int32), ev_deliver=self.empty(max(n, 1), torch.int64),
                   ev_src=self.empty(max(n, 1), torch.int32), ev_seq=self.empty(max(n, 1), torch.int64),
                   ev_pkt=self.empty(max(n, 1), torch.int32))
        o = N.RelayOut(None, *(N.ptr(out[k]).value for k in ("ev_off", "ev_deliver", "ev_src", "ev_seq",
                                                              "ev_pkt")), 0, 0, 0)
        N.check(self.eng.lib.shd_events_merge_device(
            self.eng.ctx, n_runs, n_dst, N.ptr(run_base), N.ptr(run_off),
            N.ptr(deliver) if n else None, N.ptr(src) if n else None, N.ptr(seq) if n else None,
            N.ptr(pkt) if n else None, n, C.byref(o)), "shd_events_merge_device")
        return out


def sharded_routing(ops, n: int, lat_full, loss_full, group=None):
    """Rows [rb, re) locally, then all-gather -> the full n x n table on every rank.

    ``lat_full`` / ``loss_full`` are (world * per, n) buffers (per = ceil(n / world)); rank r's
    rows live in slice [r * per, (r + 1) * per).  Returns views of the first n rows.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    per = (n + world - 1) // world
    rb, re = row_shard(n, world, rank)
    shard_lat = lat_full[rank * per:(rank + 1) * per]
    shard_loss = loss_full[rank * per:(rank + 1) * per]
    if re > rb:
        ops.routing_rows(rb, re, shard_lat, shard_loss)
    if world > 1:
        _all_gather(lat_full, shard_lat.contiguous(), group)
        _all_gather(loss_full, shard_loss.contiguous(), group)
    return lat_full[:n], loss_full[:n]


def sharded_relay_round(ops, n_hosts, src_off, send_time, dst_host, payload, round_, group=None):
    """One relay round with hosts sharded by id; ``src_off`` covers ALL hosts (hosts owned by
    other ranks have no packets here).  Returns this rank's destinations' events (dst range
    [lo, hi), ev_off indexed by d - lo, packet ids global = sender batch base + local index),
    this rank's packet statuses, and the all-reduced round reductions."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = send_time.device
    out = ops.relay_round(src_off, send_time, dst_host, payload, n_hosts, round_)
    lo, hi = host_shard(n_hosts, world, rank)
    if world == 1:
        out.update(lo=lo, hi=hi)
        return out
    bounds = [host_shard(n_hosts, world, r) for r in range(world)]
    ev_off = out["ev_off"].to(torch.int64)
    n_sent_local = int(out["n_sent"])
    cuts = torch.tensor([b[0] for b in bounds] + [n_hosts], device=dev)
    pos = ev_off[cuts]                                          # event positions of the shard cuts
    send_counts = (pos[1:] - pos[:-1]).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    _a2a(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    # packet ids become global: + this rank's batch base (exclusive prefix of batch sizes)
    nb = torch.tensor([send_time.numel()], dtype=torch.int64, device=dev)
    all_nb = torch.empty(world, dtype=torch.int64, device=dev)
    _all_gather(all_nb, nb, group)
    pkt_base = int(all_nb[:rank].sum().item())

    if sum(rc) >= 2**31 or pkt_base + send_time.numel() >= 2**32:
        raise OverflowError("sharded relay: more than 2^31 events or 2^32 packets per round")

    def a2a(x, dtype):
        x = x[:n_sent_local].to(dtype)
        y = torch.empty(sum(rc), dtype=dtype, device=dev)
        _a2a(y, x.contiguous(), rc, sc, group)
        return y

    r_deliver = a2a(out["ev_deliver"], torch.int64)
    r_src = a2a(out["ev_src"], torch.int32)
    r_seq = a2a(out["ev_seq"], torch.int64)
    # global packet ids (sender batch base + local index) stay 64-bit through the exchange; the
    # check above guarantees they fit the engine's u32 packet field
    r_pkt = a2a(out["ev_pkt"].to(torch.int64) + pkt_base, torch.int64)
    r_pkt = (r_pkt - (r_pkt >= 2**31).to(torch.int64) * 2**32).to(torch.int32)   # u32 bits
    # per-destination local offsets of every sender's slice for this rank's hosts (int64 until
    # the exchange: no silent 32-bit wrap; the engine's merge takes u32 offsets)
    off_parts = [ev_off[b0:b1 + 1] - ev_off[b0] for (b0, b1) in bounds]
    send_off = torch.cat(off_parts).to(torch.int64)
    n_own = hi - lo
    r_off = torch.empty(world * (n_own + 1), dtype=torch.int64, device=dev)
    _a2a(r_off, send_off.contiguous(), [n_own + 1] * world, [b1 - b0 + 1 for (b0, b1) in bounds], group)
    r_off = r_off.to(torch.int32)
    run_base = torch.tensor(np.concatenate([[0], np.cumsum(rc)]).astype(np.int64), device=dev).to(torch.int32)
    merged = ops.merge(world, n_own, run_base, r_off, r_deliver, r_src, r_seq, r_pkt)
    red = torch.tensor([_u64_as_i64(out["min_deliver"]), _u64_as_i64(out["min_latency"])],
                       dtype=torch.int64, device=dev)
    _all_reduce(red, dist.ReduceOp.MIN, group)
    tot = torch.tensor([n_sent_local], dtype=torch.int64, device=dev)
    _all_reduce(tot, dist.ReduceOp.SUM, group)
    md, ml = [int(v) for v in red.tolist()]
    merged.update(status=out["status"], lo=lo, hi=hi, n_recv=sum(rc),
                  min_deliver=U64_MAX if md == I64_MAX else md,
                  min_latency=U64_MAX if ml == I64_MAX else ml, n_sent=int(tot.item()))
    return merged


# ------------------------------------------------------------------------------------------
# The engine's own multi-GPU path (C ABI: shd_comm_* / shd_*_sharded).  torch.distributed only
# carries the RCCL unique id from rank 0 to the others; every collective of the two paths runs
# inside the engine over its own communicator.
# ------------------------------------------------------------------------------------------
def comm_init_rccl(engine, group=None):
    """One process per GPU: an engine communicator over RCCL spanning the torch.distributed group."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    uid = (C.c_uint8 * N.COMM_ID_BYTES)()
    if rank == 0:
        N.check(engine.lib.shd_comm_unique_id(uid), "shd_comm_unique_id")
    if world > 1:
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8)
        if dist.get_backend(group) != "gloo":
            t = t.cuda()
        dist.broadcast(t, 0, group=group)
        uid = (C.c_uint8 * N.COMM_ID_BYTES)(*t.cpu().tolist())
    N.check(engine.lib.shd_comm_init(engine.ctx, world, rank, uid), "shd_comm_init")


def comm_init_local(engines):
    """Every rank in this process (one host thread per rank drives the sharded calls)."""
    arr = (C.c_void_p * len(engines))(*[e.ctx for e in engines])
    N.check(engines[0].lib.shd_comm_init_local(arr, len(engines)), "shd_comm_init_local")


def shard_range(total: int, world: int, rank: int):
    lib = N.load()
    lo, hi = C.c_uint32(0), C.c_uint32(0)
    N.check(lib.shd_shard_range(total, world, rank, C.byref(lo), C.byref(hi)), "shd_shard_range")
    return lo.value, hi.value


def routing_replicates(n: int, world: int) -> bool:
    """True when shd_routing_run_sharded builds the whole n x n table on every rank instead of
    exchanging row shards (api.cpp: tables up to SHD_SHARD_REPLICATE_MB, default 64 MiB)."""
    mb = os.environ.get("SHD_SHARD_REPLICATE_MB", "")
    return world > 1 and n * n * 12 <= (int(mb) if mb else 64) << 20


def routing_run_sharded(engine, algo, lat_full, loss_full):
    """Rows of this rank + all-gather inside the engine; ``lat_full`` / ``loss_full`` are device
    tensors of world * ceil(n / world) rows (rows >= n are padding)."""
    err = N.Error()
    N.check(engine.lib.shd_routing_run_sharded(engine.ctx, algo, N.ptr(lat_full), N.ptr(loss_full),
                                               C.byref(err)), "shd_routing_run_sharded", err)


_hip = None


def d2h(dev_ptr: int, n: int, dtype) -> np.ndarray:
    """Copy n elements from an engine-owned device array to a new host array."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so.7")   # the HIP runtime torch and the engine share
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
    out = np.empty(n, dtype)
    if n:
        rc = _hip.hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(dev_ptr), out.nbytes, 2)
        if rc != 0:
            raise RuntimeError(f"hipMemcpy D2H failed ({rc})")
    return out


class ShardedRelay:
    """The relay of one rank under an engine communicator: its shard [lo, hi) of the hosts."""

    def __init__(self, engine, host_node, rng_state, next_event_id, lat, loss):
        self.eng = engine
        host_node = np.ascontiguousarray(host_node, np.uint32)
        self.n_hosts = len(host_node)
        w, r = C.c_int32(0), C.c_int32(0)
        N.check(engine.lib.shd_comm_info(engine.ctx, C.byref(w), C.byref(r)), "shd_comm_info")
        self.world, self.rank = w.value, r.value
        self.lo, self.hi = shard_range(self.n_hosts, self.world, self.rank)
        lat = np.ascontiguousarray(lat, np.uint64)
        loss = np.ascontiguousarray(loss, np.float32)
        N.check(engine.lib.shd_relay_setup(engine.ctx, self.n_hosts, N.ptr(host_node), lat.shape[0], N.ptr(lat),
                                           N.ptr(loss), N.ptr(np.ascontiguousarray(rng_state, np.uint64)),
                                           N.ptr(np.ascontiguousarray(next_event_id, np.uint64))),
                "shd_relay_setup")

    def round_device(self, d_off, d_time, d_dst, d_pay, round_, d_status) -> N.RelayOut:
        n = int(d_time.numel())
        b = N.Batch(n, N.ptr(d_off).value, N.ptr(d_time).value if n else None, N.ptr(d_dst).value if n else None,
                    N.ptr(d_pay).value if n else None, None)
        out = N.RelayOut(N.ptr(d_status).value if n else None, None, None, None, None, None, 0, 0, 0)
        rd = N.Round(*round_)
        N.check(self.eng.lib.shd_relay_round_sharded(self.eng.ctx, C.byref(b), C.byref(rd), C.byref(out)),
                "shd_relay_round_sharded")
        return out

    def round(self, src_off, send_time, dst_host, payload, round_):
        """Host arrays of this rank's sends (src_off over its hi - lo hosts) -> (status, events of
        its destinations as a dict of host arrays, min_deliver, min_latency, n_sent)."""
        dev = lambda a, np_dt, dt: torch.from_numpy(np.ascontiguousarray(a, np_dt).view(dt)).cuda()  # noqa: E731
        d_off = dev(src_off, np.uint32, np.int32)
        d_time = dev(send_time, np.uint64, np.int64)
        d_dst = dev(dst_host, np.uint32, np.int32)
        d_pay = dev(payload, np.uint32, np.int32)
        d_status = torch.empty(max(len(send_time), 1), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        out = self.round_device(d_off, d_time, d_dst, d_pay, round_, d_status)
        n_own = self.hi - self.lo
        off = d2h(out.ev_off, n_own + 1, np.uint32)
        m = int(off[-1])
        ev = dict(off=off, deliver=d2h(out.ev_deliver, m, np.uint64), src=d2h(out.ev_src, m, np.uint32),
                  seq=d2h(out.ev_seq, m, np.uint64), pkt=d2h(out.ev_pkt, m, np.uint32))
        status = d_status.cpu().numpy()[: len(send_time)].copy()
        return status, ev, out.min_deliver, out.min_latency, out.n_sent

    def host_state(self):
        rng = np.zeros((self.n_hosts, 4), np.uint64)
        nid = np.zeros(self.n_hosts, np.uint64)
        N.check(self.eng.lib.shd_relay_get_host_state(self.eng.ctx, N.ptr(rng), N.ptr(nid)),
                "shd_relay_get_host_state")
        return rng, nid
