"""Host-side mirror of the reference's token-bucket relays (``TokenBucket`` and the bucket part
of ``Relay::forward_until_blocked``, src/main/network/relay/{token_bucket.rs:6-157,
mod.rs:200-302}), batched over relays on the MI355X engine.

``TokenBuckets(engine, capacity, refill_increment, refill_interval, last_refill)`` keeps one
bucket per relay on the device (all three parameters 0: no bucket, ``RateLimit::Unlimited``);
``create_token_bucket(bytes_per_second)`` gives the reference's parameters for a rate limit.
``run(relay_off, time, size, flags)`` replays a batch of forwarding attempts grouped by relay and
returns, per attempt, FORWARDED / BLOCKED / SKIPPED and the balance / duration / deadline.  No
CPU fallback: without the native library or a gfx950 GPU every call raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N

FORWARDED, BLOCKED, SKIPPED = 0, 1, 2
EXEMPT = 1
MTU = 1500
MS = 1_000_000
SIM_START = 946684800 * 1_000_000_000   # EmulatedTime::SIMULATION_START


def create_token_bucket(bytes_per_second: int) -> tuple[int, int, int]:
    """relay/mod.rs:291-302 -> (capacity, refill_increment, refill_interval_ns)."""
    refill = max(1, int(bytes_per_second) // 1000)
    return refill + MTU, refill, MS


class TokenBuckets:
    def __init__(self, engine, capacity, refill_increment, refill_interval, last_refill=SIM_START):
        self.eng = engine
        cap = np.ascontiguousarray(capacity, np.uint64)
        self.n_relays = len(cap)
        inc = np.ascontiguousarray(np.broadcast_to(np.asarray(refill_increment, np.uint64), cap.shape))
        itv = np.ascontiguousarray(np.broadcast_to(np.asarray(refill_interval, np.uint64), cap.shape))
        last = np.ascontiguousarray(np.broadcast_to(np.asarray(last_refill, np.uint64), cap.shape))
        N.check(engine.lib.shd_tb_setup(engine.ctx, self.n_relays, N.ptr(cap), N.ptr(inc), N.ptr(itv),
                                        N.ptr(last)), "shd_tb_setup")

    def run(self, relay_off, time, size, flags=None):
        """Returns (status[n_ops] u8, value[n_ops] u64).  Host arrays in, host arrays out."""
        import torch
        relay_off = np.ascontiguousarray(relay_off, np.uint32)
        time = np.ascontiguousarray(time, np.uint64)
        size = np.ascontiguousarray(size, np.uint32)
        flags = np.zeros(len(time), np.uint8) if flags is None else np.ascontiguousarray(flags, np.uint8)
        assert len(relay_off) == self.n_relays + 1 and int(relay_off[-1]) == len(time) == len(size) == len(flags)
        n = len(time)
        dev = lambda a, dt: torch.from_numpy(a.view(dt)).cuda()  # noqa: E731
        d_off, d_time, d_size = dev(relay_off, np.int32), dev(time, np.int64), dev(size, np.int32)
        d_flags = dev(flags, np.uint8)
        status = torch.empty(max(n, 1), dtype=torch.uint8, device="cuda")
        value = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        ops = N.TbOps(n, N.ptr(d_off).value, N.ptr(d_time).value, N.ptr(d_size).value, N.ptr(d_flags).value)
        st = self.eng.lib.shd_tb_run_device(self.eng.ctx, C.byref(ops), N.ptr(status), N.ptr(value))
        torch.cuda.synchronize()
        N.check(st, "shd_tb_run_device")
        return status.cpu().numpy()[:n].copy(), value.cpu().numpy().view(np.uint64)[:n].copy()

    def state(self, relay: int) -> dict:
        s = N.TbState()
        N.check(self.eng.lib.shd_tb_get_state(self.eng.ctx, int(relay), C.byref(s)), "shd_tb_get_state")
        return {k: int(getattr(s, k)) for k, _ in N.TbState._fields_}
