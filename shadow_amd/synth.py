"""Synthetic workloads for BASELINE.json's configs; numpy, seeded.

C2: 1k-node complete undirected graph + self-loops, integer-ms latencies U[1,300], 10% of edges
    forced to tie a 2-hop path, loss f32 U[0,0.01), self-loops U[1,50] ms.          (seed 1)
C3: 10k-node Barabasi-Albert m=3 + self-loops, integer-us latencies U[100,50000],
    loss f32 U[0,0.02).                                                               (seed 2)
C4: 50k-node Barabasi-Albert m=4, otherwise as C3.                                   (seed 3)
C5: 100k hosts on the C2 graph (host h on node h mod 1000), 10M packets per round, sources
    uniform, destination != source uniform, payload 20% 0 B / 60% 1448 B / 20% U[1,1448],
    send times U[window) sorted per host, packets grouped by source in send order.    (seed 4)
Host RNG states follow the reference's seed derivation (sim_config.rs:49-53,223-244;
host.rs:218) for host names ``host%06d`` with general.seed = 1.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

MS = 1_000_000
US = 1_000
SIM_START = 946_684_800 * 1_000_000_000   # EmulatedTime::SIMULATION_START (emulated_time.rs)


@dataclass
class EdgeList:
    node_ids: np.ndarray
    src: np.ndarray
    dst: np.ndarray
    latency_ns: np.ndarray
    packet_loss: np.ndarray
    directed: bool = False

    @property
    def n_nodes(self) -> int:
        return len(self.node_ids)


def _with_self_loops(n, src, dst, lat, loss, rng, loop_lo, loop_hi, loop_unit, loss_max):
    ls = np.arange(n, dtype=np.uint32)
    llat = rng.integers(loop_lo, loop_hi + 1, size=n).astype(np.uint64) * np.uint64(loop_unit)
    lloss = rng.uniform(0.0, loss_max, size=n).astype(np.float32)
    return (np.concatenate([ls, src]).astype(np.uint32), np.concatenate([ls, dst]).astype(np.uint32),
            np.concatenate([llat, lat]).astype(np.uint64), np.concatenate([lloss, loss]).astype(np.float32))


def complete_graph(n: int = 1000, seed: int = 1, tie_frac: float = 0.10) -> EdgeList:
    """C2 (and smaller test instances): complete undirected graph + self-loops."""
    rng = np.random.default_rng(seed)
    W = rng.integers(1, 301, size=(n, n)).astype(np.int64)
    W = np.triu(W, 1)
    W = W + W.T
    iu, ju = np.triu_indices(n, 1)
    # force ties: a fraction of edges get the latency of a random 2-hop detour (capped at 300)
    m = len(iu)
    pick = rng.random(m) < tie_frac
    x = rng.integers(0, n, size=m)
    detour = W[iu, x] + W[x, ju]
    sel = pick & (detour <= 300) & (x != iu) & (x != ju)
    lat_ms = W[iu, ju].copy()
    lat_ms[sel] = detour[sel]
    lat = lat_ms.astype(np.uint64) * np.uint64(MS)
    loss = rng.uniform(0.0, 0.01, size=m).astype(np.float32)
    s, d, l, p = _with_self_loops(n, iu.astype(np.uint32), ju.astype(np.uint32), lat, loss, rng,
                                  1, 50, MS, 0.01)
    return EdgeList(np.arange(n, dtype=np.uint32), s, d, l, p, False)


def barabasi_albert(n: int, m: int, seed: int, lat_lo_us: int = 100, lat_hi_us: int = 50_000,
                    loss_max: float = 0.02) -> EdgeList:
    """C3/C4: preferential-attachment graph (m edges per new node) + self-loops."""
    rng = np.random.default_rng(seed)
    src, dst = [], []
    targets = list(range(m))
    repeated = []
    for v in range(m, n):
        src.extend([v] * m)
        dst.extend(targets)
        repeated.extend(targets)
        repeated.extend([v] * m)
        chosen = set()
        while len(chosen) < m:
            chosen.add(repeated[int(rng.integers(0, len(repeated)))])
        targets = sorted(chosen)
    src = np.asarray(src, np.uint32)
    dst = np.asarray(dst, np.uint32)
    lat = rng.integers(lat_lo_us, lat_hi_us + 1, size=len(src)).astype(np.uint64) * np.uint64(US)
    loss = rng.uniform(0.0, loss_max, size=len(src)).astype(np.float32)
    s, d, l, p = _with_self_loops(n, src, dst, lat, loss, rng, lat_lo_us, lat_hi_us, US, loss_max)
    return EdgeList(np.arange(n, dtype=np.uint32), s, d, l, p, False)


CONFIGS = {
    "c2": lambda: complete_graph(1000, 1),
    "c3": lambda: barabasi_albert(10_000, 3, 2),
    "c4": lambda: barabasi_albert(50_000, 4, 3),
}


# ------------------------------------------------------------------------------ host RNG seeds
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _rotl(x, k):
    k = np.uint64(k)
    return (x << k) | (x >> (np.uint64(64) - k))


def siphash13_batch(msgs: np.ndarray) -> np.ndarray:
    """SipHash-1-3 (k0 = k1 = 0) of equal-length byte strings (rows of a uint8 array)."""
    with np.errstate(over="ignore"):
        n, L = msgs.shape
        v0 = np.full(n, 0x736F6D6570736575, np.uint64)
        v1 = np.full(n, 0x646F72616E646F6D, np.uint64)
        v2 = np.full(n, 0x6C7967656E657261, np.uint64)
        v3 = np.full(n, 0x7465646279746573, np.uint64)

        def rnd(v0, v1, v2, v3):
            v0 = v0 + v1; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
            v2 = v2 + v3; v3 = _rotl(v3, 16); v3 ^= v2
            v0 = v0 + v3; v3 = _rotl(v3, 21); v3 ^= v0
            v2 = v2 + v1; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)
            return v0, v1, v2, v3

        full = L // 8
        words = msgs[:, :full * 8].copy().view("<u8").reshape(n, full) if full else None
        for w in range(full):
            m = words[:, w]
            v3 ^= m
            v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
            v0 ^= m
        tail = np.zeros((n, 8), np.uint8)
        tail[:, :L - full * 8] = msgs[:, full * 8:]
        b = tail.view("<u8").reshape(n) | np.uint64((L & 0xFF) << 56)
        v3 ^= b
        v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        v0 ^= b
        v2 ^= np.uint64(0xFF)
        for _ in range(3):
            v0, v1, v2, v3 = rnd(v0, v1, v2, v3)
        return v0 ^ v1 ^ v2 ^ v3


def splitmix_fill(seed: np.ndarray) -> np.ndarray:
    """Xoshiro256PlusPlus::seed_from_u64 for many seeds -> [n, 4] states."""
    with np.errstate(over="ignore"):
        x = seed.astype(np.uint64).copy()
        out = np.empty((len(seed), 4), np.uint64)
        for i in range(4):
            x = x + np.uint64(0x9E3779B97F4A7C15)
            z = x.copy()
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[:, i] = z ^ (z >> np.uint64(31))
        return out


def xoshiro_next_batch(s: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        res = _rotl(s[:, 0] + s[:, 3], 23) + s[:, 0]
        t = s[:, 1] << np.uint64(17)
        s[:, 2] ^= s[:, 0]
        s[:, 3] ^= s[:, 1]
        s[:, 1] ^= s[:, 2]
        s[:, 0] ^= s[:, 3]
        s[:, 2] ^= t
        s[:, 3] = _rotl(s[:, 3], 45)
        return res


def host_names(n_hosts: int):
    return [f"host{h:06d}" for h in range(n_hosts)]


def host_rng_states(n_hosts: int, global_seed: int = 1) -> np.ndarray:
    """Initial Xoshiro256++ state per host (HostId order = sorted names = numeric order)."""
    g = splitmix_fill(np.array([global_seed], np.uint64))
    randomness = xoshiro_next_batch(g)[0]
    names = np.frombuffer("".join(host_names(n_hosts)).encode(), np.uint8).reshape(n_hosts, 10)
    msgs = np.concatenate([names, np.full((n_hosts, 1), 0xFF, np.uint8)], axis=1)
    seeds = siphash13_batch(msgs) ^ randomness
    return splitmix_fill(seeds)


# ------------------------------------------------------------------------------ C5 packets
@dataclass
class PacketBatch:
    src_off: np.ndarray     # u32 [n_hosts+1]
    send_time: np.ndarray   # u64
    dst_host: np.ndarray    # u32
    payload: np.ndarray     # u32

    @property
    def n(self) -> int:
        return len(self.send_time)


def packet_batch(n_hosts: int, n_packets: int, window_start: int, window_end: int,
                 seed: int = 4) -> PacketBatch:
    rng = np.random.default_rng(seed)
    src = np.sort(rng.integers(0, n_hosts, size=n_packets, dtype=np.uint32))
    dst = rng.integers(0, n_hosts - 1, size=n_packets, dtype=np.uint32)
    dst = dst + (dst >= src).astype(np.uint32)          # uniform over hosts != src
    u = rng.random(n_packets)
    payload = np.where(u < 0.2, 0, np.where(u < 0.8, 1448,
                       rng.integers(1, 1449, size=n_packets))).astype(np.uint32)
    t = rng.integers(window_start, window_end, size=n_packets, dtype=np.uint64)
    order = np.lexsort((t, src))                         # group by source, send-time order
    src, t = src[order], t[order]
    counts = np.bincount(src, minlength=n_hosts)
    off = np.zeros(n_hosts + 1, np.uint32)
    np.cumsum(counts, out=off[1:])
    return PacketBatch(off, t.astype(np.uint64), dst, payload)


def c5_host_nodes(n_hosts: int, n_nodes: int) -> np.ndarray:
    return (np.arange(n_hosts, dtype=np.uint32) % np.uint32(n_nodes)).astype(np.uint32)


@dataclass
class StagedRound:
    """A grouped batch laid out as the drop-in's per-worker-thread staging buffers
    (shd_relay_flush): stage k = one thread's buffer, its hosts' runs in the thread's run order.
    ``stage_of_send[i]`` = the grouped index of the send at stage-order position i."""
    run_host: list
    run_count: list
    sends: list            # per stage: (n, 3) u32 records {time_off, dst | payload bit, draw_hi}
    stage_of_send: np.ndarray
    draw64: np.ndarray     # per grouped send: the u64 the host RNG returned (chance = draw >> 11 * 2^-53)


def stage_round(b: PacketBatch, n_threads: int, time_base: int, seed: int = 7) -> StagedRound:
    """Spread the hosts of ``b`` over ``n_threads`` worker threads (each host on one thread, the
    thread_per_core scheduler's invariant), every thread running its hosts in a shuffled order, and
    draw a u64 per send for the CPU-side loss draw (worker.rs:365)."""
    rng = np.random.default_rng(seed)
    H = len(b.src_off) - 1
    thread = rng.integers(0, n_threads, size=H)
    cnt = np.diff(b.src_off.astype(np.int64))
    draw64 = rng.integers(0, 2**64, size=len(b.send_time), dtype=np.uint64)
    pay = (b.payload > 0).astype(np.uint32) << np.uint32(31)
    rec_all = np.stack([(b.send_time - np.uint64(time_base)).astype(np.uint32), b.dst_host | pay,
                        (draw64 >> np.uint64(32)).astype(np.uint32)], axis=1)
    run_host, run_count, sends, order = [], [], [], []
    for k in range(n_threads):
        hs = np.flatnonzero(thread == k).astype(np.uint32)
        rng.shuffle(hs)
        run_host.append(hs)
        run_count.append(cnt[hs].astype(np.uint32))
        c = cnt[hs]
        idx = np.repeat(b.src_off[hs].astype(np.int64) - (np.cumsum(c) - c), c) + np.arange(int(c.sum()))
        order.append(idx.astype(np.int64))
        sends.append(np.ascontiguousarray(rec_all[idx]))
    return StagedRound(run_host, run_count, sends, np.concatenate(order), draw64)
