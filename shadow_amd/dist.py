"""Multi-GPU driving of the engine (C ABI: shd_comm_* / shd_*_sharded), one process per GPU.

Every collective of the two paths runs inside the engine over its own communicator (RCCL over
xGMI); torch.distributed only carries the RCCL unique id from rank 0 to the
others.  The sharding contract the ABI implements:
  * routing build: the used-node source rows are split into contiguous shards; every rank runs
    its rows (no collective inside the SSSP -- rows are independent) and the table ends whole on
    every rank (shd_routing_run_sharded);
  * relay: hosts are split by id into contiguous ranges (shd_shard_range).  A rank stamps the
    sends of ITS source hosts (their RNG streams and event ids live there) and receives the
    events of ITS destination hosts, merged in EventQueue order; ev_pkt is the packet's index in
    its sender rank's batch (the sender is the rank owning ev_src); min deliver time, min latency
    and the sent count are reduced over all ranks (shd_relay_round_sharded);
  * the destination queues of a rank hold its own hosts (shd_equeue_setup under the
    communicator), and the next window is agreed over all ranks (shd_round_window).
Every event has deliver >= round_end, so exchanging at the round barrier is exact.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N

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


def host_all_to_allv(group=None):
    """The all-to-all-v of shd_comm_init_host over a torch.distributed CPU group (gloo): a Python
    callable with the C callback's arguments (raw host pointers and per-rank sizes / offsets)."""
    def a2av(send, s_bytes, s_off, recv, r_bytes, r_off):
        world = dist.get_world_size(group)
        sb = [int(s_bytes[r]) for r in range(world)]
        rb = [int(r_bytes[q]) for q in range(world)]
        # the blocks to the ranks, back to back (a block's offset may repeat: the same bytes)
        parts = [np.ctypeslib.as_array(C.cast(C.c_void_p(send + int(s_off[r])), C.POINTER(C.c_uint8)), (sb[r],))
                 if sb[r] else np.zeros(0, np.uint8) for r in range(world)]
        inp = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(0, np.uint8))
        out = torch.empty(sum(rb), dtype=torch.uint8)
        dist.all_to_all_single(out, inp, rb, sb, group=group)
        o = out.numpy()
        at = 0
        for q in range(world):
            if rb[q]:
                dst = np.ctypeslib.as_array(C.cast(C.c_void_p(recv + int(r_off[q])), C.POINTER(C.c_uint8)), (rb[q],))
                dst[:] = o[at:at + rb[q]]
            at += rb[q]
    return a2av


class HostComm:
    """An engine communicator over the caller's host transport (shd_comm_init_host): here
    torch.distributed on a CPU group (gloo), for processes that cannot pair up over RCCL (several
    processes on one GPU, hosts without an RCCL peer).  Keep the object alive while the engine
    uses the communicator (it holds the C callback)."""

    def __init__(self, engine, group=None):
        fn = host_all_to_allv(group)

        def cb(user, send, s_bytes, s_off, recv, r_bytes, r_off):
            try:
                fn(send, s_bytes, s_off, recv, r_bytes, r_off)
                return 0
            except Exception:   # noqa: BLE001 -- a failed transport is reported to the engine
                import traceback
                traceback.print_exc()
                return 1
        self._cb = N.ALL_TO_ALLV(cb)
        self._ops = N.HostCommOps(None, self._cb)
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        N.check(engine.lib.shd_comm_init_host(engine.ctx, world, rank, C.byref(self._ops)), "shd_comm_init_host")


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


def d2h(engine, dev_ptr: int, n: int, dtype) -> np.ndarray:
    """Copy n elements from an engine-owned device array to a new host array (shd_copy_to_host,
    on the engine's own HIP runtime and stream)."""
    out = np.empty(n, dtype)
    if n:
        N.check(engine.lib.shd_copy_to_host(engine.ctx, out.ctypes.data_as(C.c_void_p), C.c_void_p(dev_ptr),
                                            out.nbytes), "shd_copy_to_host")
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
        out = N.RelayOut(N.ptr(d_status).value if n else None, None, None, None, None, None, 0, 0, 0, 0, 0)
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
        off = d2h(self.eng, out.ev_off, n_own + 1, np.uint32)
        m = int(off[-1])
        e = self.eng
        ev = dict(off=off, deliver=d2h(e, out.ev_deliver, m, np.uint64), src=d2h(e, out.ev_src, m, np.uint32),
                  seq=d2h(e, out.ev_seq, m, np.uint64), pkt=d2h(e, out.ev_pkt, m, np.uint32))
        status = d_status.cpu().numpy()[: len(send_time)].copy()
        return status, ev, out.min_deliver, out.min_latency, out.n_sent

    def flush(self, run_host, run_count, sends, time_base: int, round_end: int, sim_end: int,
              bootstrap_end: int = 0, pinned=None):
        """``shd_relay_flush`` under the communicator: every rank passes the SAME stages (all worker
        threads' buffers); this rank's result: statuses of its own hosts' sends in stage order (0
        for the other ranks' sends), its destinations' events (ev_off over [lo, hi]), seq_base
        entries [lo, hi), and the all-rank reductions."""
        from .relay import FlushResult, PinnedStages
        if pinned is None:
            pinned = PinnedStages.wrap(run_host, run_count, sends)
        n = pinned.n
        st2 = np.zeros((n + 3) // 4, np.uint8)
        ev_off = np.zeros(self.hi - self.lo + 1, np.uint32)
        events = np.zeros((max(n, 1), 4), np.uint32)
        seq_base = np.zeros(self.n_hosts, np.uint64)
        out = N.FlushOut(N.ptr(st2).value, N.ptr(ev_off).value, N.ptr(events).value, N.ptr(seq_base).value,
                         0, 0, 0, 0)
        rd = N.Round(round_end, sim_end, bootstrap_end)
        N.check(self.eng.lib.shd_relay_flush(self.eng.ctx, pinned.array, len(pinned.stages), int(time_base),
                                             C.byref(rd), C.byref(out)), "shd_relay_flush")
        status = ((st2[:, None] >> (np.arange(4, dtype=np.uint8) * 2)) & 3).reshape(-1)[:n]
        return FlushResult(status, ev_off, events[:out.n_events], seq_base, out.min_deliver, out.min_latency,
                           out.n_sent)

    def last_pipeline(self) -> int:
        """8: the bins went to their destination ranks as stamped (relay_round_sharded_v7); else the
        packing path ran on the local pipeline 7, 3 or 1."""
        p = C.c_int32(0)
        N.check(self.eng.lib.shd_relay_last_pipeline(self.eng.ctx, C.byref(p)), "shd_relay_last_pipeline")
        return p.value

    def host_state(self):
        rng = np.zeros((self.n_hosts, 4), np.uint64)
        nid = np.zeros(self.n_hosts, np.uint64)
        N.check(self.eng.lib.shd_relay_get_host_state(self.eng.ctx, N.ptr(rng), N.ptr(nid)),
                "shd_relay_get_host_state")
        return rng, nid
