"""Host-side mirror of the per-round packet relay (``Worker::send_packet`` batched per round).

Mirrors ``src/main/core/worker.rs:328-413`` (send_packet), ``:497-629`` (WorkerShared tables,
push_packet_to_host) and the destination ``EventQueue`` order (``core/work/event.rs:84-155``).
A round's staged sends are flushed once at the round barrier (``core/manager.rs:455-464``);
the result is, per destination host, its new packet events in the order its EventQueue would
pop them, plus the round reductions (min deliver time, min latency used).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N
from .routing import Engine, default_engine


@dataclass
class RoundResult:
    status: np.ndarray        # u8 per packet: 0 skipped (now >= sim_end), 1 dropped, 2 sent
    ev_off: np.ndarray        # u32 [n_hosts+1]: destination h's events are [ev_off[h], ev_off[h+1])
    ev_deliver: np.ndarray    # u64 [n_sent]
    ev_src: np.ndarray        # u32 [n_sent]
    ev_seq: np.ndarray        # u64 [n_sent] (src_host_event_id)
    ev_pkt: np.ndarray        # u32 [n_sent] index of the packet in the batch
    min_deliver: int          # u64::MAX when nothing was sent
    min_latency: int
    n_sent: int

    def events_for(self, dst: int):
        a, b = int(self.ev_off[dst]), int(self.ev_off[dst + 1])
        return list(zip(self.ev_deliver[a:b].tolist(), self.ev_src[a:b].tolist(),
                        self.ev_seq[a:b].tolist(), self.ev_pkt[a:b].tolist()))


@dataclass
class FlushResult:
    status: np.ndarray        # u8 per send in stage order (decoded from the 2-bit statuses)
    ev_off: np.ndarray        # u32 [n_hosts+1]
    events: np.ndarray        # (n_sent, 4) u32: deliver - round_end, src host, seq - seq_base[src], send index
    seq_base: np.ndarray      # u64 [n_hosts]: each host's first event id of the round
    min_deliver: int
    min_latency: int
    n_sent: int


class PinnedStages:
    """Staging buffers for ``Relay.flush``.  ``wrap`` points the C structs at the caller's arrays;
    ``pinned`` copies them into shd_host_alloc memory, as a drop-in's worker threads would stage
    into pinned buffers from the start."""

    def __init__(self):
        self.stages, self.keep, self.allocs, self.n = [], [], [], 0
        self.array = None

    @classmethod
    def wrap(cls, run_host, run_count, sends):
        p = cls()
        for h, c, sd in zip(run_host, run_count, sends):
            h = np.ascontiguousarray(h, np.uint32)
            c = np.ascontiguousarray(c, np.uint32)
            sd = np.ascontiguousarray(sd, np.uint32).reshape(-1, 3)
            p.keep += [h, c, sd]
            p.stages.append(N.Stage(len(h), N.ptr(h).value, N.ptr(c).value, sd.shape[0], N.ptr(sd).value))
            p.n += sd.shape[0]
        p.array = (N.Stage * max(len(p.stages), 1))(*p.stages)
        return p

    @classmethod
    def pinned(cls, lib, run_host, run_count, sends):
        p = cls()
        p.lib = lib
        for h, c, sd in zip(run_host, run_count, sends):
            sd = np.ascontiguousarray(sd, np.uint32).reshape(-1, 3)
            views = []
            for a in (np.ascontiguousarray(h, np.uint32), np.ascontiguousarray(c, np.uint32), sd):
                ptr = lib.shd_host_alloc(max(a.nbytes, 1))
                if not ptr:
                    p.free()
                    raise MemoryError("shd_host_alloc")
                p.allocs.append(ptr)
                C.memmove(ptr, a.ctypes.data, a.nbytes)
                views.append(ptr)
            p.stages.append(N.Stage(len(h), views[0], views[1], sd.shape[0], views[2]))
            p.n += sd.shape[0]
        p.array = (N.Stage * max(len(p.stages), 1))(*p.stages)
        return p

    def free(self):
        for ptr in self.allocs:
            self.lib.shd_host_free(ptr)
        self.allocs = []


def group_by_source(n_hosts: int, src_host: np.ndarray):
    """Stable grouping of staged sends by source host -> (order, src_off).

    Worker threads stage sends in per-thread buffers; each host runs on one thread per round,
    so a stable sort by source keeps every host's send order.
    """
    src_host = np.asarray(src_host, np.uint32)
    order = np.argsort(src_host, kind="stable")
    counts = np.bincount(src_host, minlength=n_hosts)
    off = np.zeros(n_hosts + 1, np.uint32)
    np.cumsum(counts, out=off[1:])
    return order, off


class Relay:
    """Device-resident relay tables of one GPU (``shd_relay_setup``)."""

    def __init__(self, host_node, rng_state, next_event_id, lat=None, loss=None,
                 engine: Engine | None = None):
        self.eng = engine or default_engine()
        self.host_node = np.ascontiguousarray(host_node, np.uint32)
        self.n_hosts = len(self.host_node)
        rng = np.ascontiguousarray(rng_state, np.uint64).reshape(self.n_hosts, 4)
        nid = np.ascontiguousarray(next_event_id, np.uint64)
        if lat is not None:
            lat = np.ascontiguousarray(lat, np.uint64)
            loss = np.ascontiguousarray(loss, np.float32)
            n_nodes = lat.shape[0]
        else:
            n_nodes = int(self.host_node.max()) + 1
        self.n_nodes = n_nodes
        N.check(self.eng.lib.shd_relay_setup(self.eng.ctx, self.n_hosts, N.ptr(self.host_node),
                                             n_nodes, N.ptr(lat), N.ptr(loss), N.ptr(rng),
                                             N.ptr(nid)), "shd_relay_setup")

    def round(self, src_off, send_time, dst_host, payload, round_end: int, sim_end: int,
              bootstrap_end: int = 0, chance=None) -> RoundResult:
        src_off = np.ascontiguousarray(src_off, np.uint32)
        send_time = np.ascontiguousarray(send_time, np.uint64)
        dst_host = np.ascontiguousarray(dst_host, np.uint32)
        payload = np.ascontiguousarray(payload, np.uint32)
        if chance is not None:
            chance = np.ascontiguousarray(chance, np.float64)
        n = len(send_time)
        b = N.Batch(n, N.ptr(src_off).value, N.ptr(send_time).value, N.ptr(dst_host).value,
                    N.ptr(payload).value, N.ptr(chance).value if chance is not None else None)
        rd = N.Round(round_end, sim_end, bootstrap_end)
        status = np.zeros(n, np.uint8)
        ev_off = np.zeros(self.n_hosts + 1, np.uint32)
        ev_deliver = np.zeros(n, np.uint64)
        ev_src = np.zeros(n, np.uint32)
        ev_seq = np.zeros(n, np.uint64)
        ev_pkt = np.zeros(n, np.uint32)
        out = N.RelayOut(N.ptr(status).value, N.ptr(ev_off).value, N.ptr(ev_deliver).value,
                         N.ptr(ev_src).value, N.ptr(ev_seq).value, N.ptr(ev_pkt).value, 0, 0, 0)
        N.check(self.eng.lib.shd_relay_round(self.eng.ctx, C.byref(b), C.byref(rd), C.byref(out)),
                "shd_relay_round")
        ns = out.n_sent
        return RoundResult(status, ev_off, ev_deliver[:ns], ev_src[:ns], ev_seq[:ns], ev_pkt[:ns],
                           out.min_deliver, out.min_latency, ns)

    def device_buffers(self, n_packets: int):
        """Device output tensors for ``round_device`` (torch, on the engine's GPU)."""
        import torch
        n = max(int(n_packets), 1)
        return dict(status=torch.empty(n, dtype=torch.uint8, device="cuda"),
                    ev_off=torch.empty(self.n_hosts + 1, dtype=torch.int32, device="cuda"),
                    ev_deliver=torch.empty(n, dtype=torch.int64, device="cuda"),
                    ev_src=torch.empty(n, dtype=torch.int32, device="cuda"),
                    ev_seq=torch.empty(n, dtype=torch.int64, device="cuda"),
                    ev_pkt=torch.empty(n, dtype=torch.int32, device="cuda"))

    def round_device(self, d_off, d_time, d_dst, d_pay, round_end: int, sim_end: int, bootstrap_end: int,
                     bufs) -> N.RelayOut:
        """``shd_relay_round_device``: batch and outputs stay on the GPU (torch tensors); the
        returned RelayOut holds the device pointers, n_sent and the reductions -- the form
        ``EventQueues.advance_device`` takes."""
        n = int(d_time.numel())
        b = N.Batch(n, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_dst).value, N.ptr(d_pay).value, None)
        out = N.RelayOut(*(N.ptr(bufs[k]).value for k in ("status", "ev_off", "ev_deliver", "ev_src", "ev_seq",
                                                           "ev_pkt")), 0, 0, 0, 0, 0)
        rd = N.Round(round_end, sim_end, bootstrap_end)
        N.check(self.eng.lib.shd_relay_round_device(self.eng.ctx, C.byref(b), C.byref(rd), C.byref(out)),
                "shd_relay_round_device")
        return out

    def round_device_into(self, d_off, d_time, d_dst, d_pay, round_end: int, sim_end: int, bootstrap_end: int,
                          out: N.RelayOut) -> N.RelayOut:
        """``shd_relay_round_device`` into a prepared output (e.g. ``EventQueues.batch_buffers``
        with ``status`` set): the events land where the queues adopt them."""
        n = int(d_time.numel())
        b = N.Batch(n, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_dst).value, N.ptr(d_pay).value, None)
        rd = N.Round(round_end, sim_end, bootstrap_end)
        N.check(self.eng.lib.shd_relay_round_device(self.eng.ctx, C.byref(b), C.byref(rd), C.byref(out)),
                "shd_relay_round_device")
        return out

    def flush(self, run_host, run_count, sends, time_base: int, round_end: int, sim_end: int,
              bootstrap_end: int = 0, pinned=None, event_bytes: int = 16, pinned_out: bool = False) -> "FlushResult":
        """``shd_relay_flush``: the worker threads' staging buffers as they stand (per stage: the
        runs' hosts and counts and the (n, 3) u32 send records {time_off, dst | SEND_PAYLOAD,
        draw_hi}).  ``pinned``: a PinnedStages holding them in pinned memory (the drop-in's path);
        else the arrays are passed as they are."""
        if pinned is None:
            pinned = PinnedStages.wrap(run_host, run_count, sends)
        n = pinned.n
        st2 = np.zeros((n + 3) // 4, np.uint8)
        ev_off = np.zeros(self.n_hosts + 1, np.uint32)
        events = np.zeros((max(n, 1), event_bytes // 4), np.uint32)   # 12 bytes: no source host column
        seq_base = np.zeros(self.n_hosts, np.uint64)
        bufs, allocs = [st2, ev_off, events, seq_base], []
        if pinned_out:   # the outputs in pinned memory too: the device writes them where they lie
            lib = self.eng.lib
            for i, a in enumerate(bufs):
                ptr = lib.shd_host_alloc(max(a.nbytes, 1))
                if not ptr:
                    for q in allocs:
                        lib.shd_host_free(q)
                    raise MemoryError("shd_host_alloc")
                allocs.append(ptr)
                bufs[i] = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), (max(a.nbytes, 1),))[: a.nbytes] \
                    .view(a.dtype).reshape(a.shape)
        try:
            out = N.FlushOut(*(N.ptr(a).value for a in bufs), 0, 0, 0, 0, event_bytes)
            rd = N.Round(round_end, sim_end, bootstrap_end)
            N.check(self.eng.lib.shd_relay_flush(self.eng.ctx, pinned.array, len(pinned.stages), int(time_base),
                                                 C.byref(rd), C.byref(out)), "shd_relay_flush")
            st2, ev_off, events, seq_base = (a.copy() for a in bufs)
        finally:
            for q in allocs:
                self.eng.lib.shd_host_free(q)
        status = ((st2[:, None] >> (np.arange(4, dtype=np.uint8) * 2)) & 3).reshape(-1)[:n]
        return FlushResult(status, ev_off, events[:out.n_sent], seq_base, out.min_deliver, out.min_latency,
                           out.n_sent)

    def host_state(self):
        rng = np.zeros((self.n_hosts, 4), np.uint64)
        nid = np.zeros(self.n_hosts, np.uint64)
        N.check(self.eng.lib.shd_relay_get_host_state(self.eng.ctx, N.ptr(rng), N.ptr(nid)),
                "shd_relay_get_host_state")
        return rng, nid

    def last_pipeline(self) -> int:
        """Device pipeline of the last round: 7 bin placement, 3 radix sort, 1 64-bit records."""
        v = C.c_int32(0)
        N.check(self.eng.lib.shd_relay_last_pipeline(self.eng.ctx, C.byref(v)), "last_pipeline")
        return v.value

    def packet_counts(self):
        c = np.zeros((self.n_nodes, self.n_nodes), np.uint64)
        N.check(self.eng.lib.shd_path_packet_counts(self.eng.ctx, N.ptr(c)), "packet_counts")
        return c
