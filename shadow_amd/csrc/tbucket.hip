// Upstream token-bucket relays on the GPU: one bucket per relay (host
// interface), device-resident across calls; a call replays every relay's forwarding attempts of
// a batch in order, lane per relay.
//
// Reference semantics: src/main/network/relay/token_bucket.rs (FlyearthR/shadow)
//   :37-60   new_inner: a bucket only when capacity, increment and interval are all non-zero;
//            it starts full
//   :75-86   conforming_remove: lazy refill, then balance.checked_sub(decrement) or the
//            conforming duration
//   :94-120  compute_conforming_duration: ceil(missing / increment) refills; 0 -> ZERO,
//            1 -> the span to the next refill, n -> span + interval * (n - 1), saturating
//   :127-157 lazy_refill: n = elapsed / interval whole refills, balance + increment * n
//            (u64 saturating) clamped to the capacity, last_refill += interval * n
// and src/main/network/relay/mod.rs
//   :224-229 local packets and bootstrapping bypass the bucket; no bucket = RateLimit::Unlimited
//   :230-252 a removal that does not conform blocks the relay (forward_later(duration)); the
//            relay stays Pending (:112-133, no forwarding) until now + duration
// Times: EmulatedTime ns (u64); SimulationTime saturates at SIMTIME_MAX, EmulatedTime at
// EMUTIME_MAX.  A product or sum beyond SIMTIME_MAX that does not overflow u64 is where the
// reference panics (from_c_simtime(..).unwrap()); it is reported as SHD_ERR_INVALID.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "ctx.h"

namespace shd {

constexpr uint64_t kSimtimeMax = 17500059273709551614ull;   // simulation_time.rs:377
constexpr uint64_t kEmutimeMax = ~0ull - 1ull;               // emulated_time.rs:27
constexpr uint8_t kTbForwarded = 0, kTbBlocked = 1, kTbSkipped = 2;
constexpr uint8_t kTbExempt = 1;

struct TbRelay {   // 48 bytes per relay; capacity 0 = no bucket (unlimited)
    uint64_t capacity, balance, increment, interval, last_refill, pending;
};

// SimulationTime::saturating_mul / saturating_add (simulation_time.rs:135-148)
__device__ __forceinline__ uint64_t simtime_sat_mul(uint64_t t, uint64_t k, bool& bad) {
    const uint64_t hi = __umul64hi(t, k);
    if (hi) return kSimtimeMax;
    const uint64_t p = t * k;
    bad |= p > kSimtimeMax;
    return p;
}
__device__ __forceinline__ uint64_t simtime_sat_add(uint64_t a, uint64_t b, bool& bad) {
    const uint64_t s = a + b;
    if (s < a) return kSimtimeMax;
    bad |= s > kSimtimeMax;
    return s;
}
// EmulatedTime::saturating_add (emulated_time.rs:95-108)
__device__ __forceinline__ uint64_t emutime_sat_add(uint64_t t, uint64_t d) {
    const uint64_t s = t + d;
    return (s < t || s > kEmutimeMax) ? kEmutimeMax : s;
}

constexpr uint32_t kAttBatch = 8;   // attempts per lane loaded ahead of the state machine

__global__ __launch_bounds__(256) void tb_run(uint32_t n_relays, const uint32_t* __restrict__ off,
                                              const uint64_t* __restrict__ time, const uint32_t* __restrict__ size,
                                              const uint8_t* __restrict__ flags, TbRelay* __restrict__ st,
                                              uint8_t* __restrict__ status, uint64_t* __restrict__ value,
                                              uint32_t* __restrict__ err) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n_relays) return;
    TbRelay s = st[r];
    bool bad = false;
    const uint32_t b = off[r], e = off[r + 1];
    // attempts are read kAttBatch at a time into registers (loads clamped into the range, all
    // issued before the state machine runs): one memory latency per batch instead of per attempt
    for (uint32_t k0 = b; k0 < e; k0 += kAttBatch) {
        uint64_t tm[kAttBatch];
        uint32_t sz[kAttBatch];
        uint8_t fl[kAttBatch];
#pragma unroll
        for (uint32_t i = 0; i < kAttBatch; ++i) {
            const uint32_t k = min(k0 + i, e - 1);
            tm[i] = time[k];
            sz[i] = size[k];
            fl[i] = flags[k];
        }
#pragma unroll
        for (uint32_t i = 0; i < kAttBatch; ++i) {
            const uint32_t k = k0 + i;
            if (k >= e) break;
            const uint64_t now = tm[i];
            uint8_t stt = kTbForwarded;
            uint64_t v;
            if (now < s.pending) {             // Pending: no forwarding before the scheduled task
                stt = kTbSkipped;
                v = s.pending;
            } else if (s.capacity == 0) {      // RateLimit::Unlimited
                v = ~0ull;
            } else if (fl[i] & kTbExempt) { // local or bootstrapping: no tokens taken
                v = s.balance;
            } else {
                // lazy_refill (token_bucket.rs:127-157)
                const bool before = now < s.last_refill;   // duration_since(..).unwrap() panics
                bad |= before;
                uint64_t span = before ? 0ull : now - s.last_refill;
                if (span >= s.interval) {
                    const uint64_t n = span / s.interval;
                    const uint64_t tok = __umul64hi(s.increment, n) ? ~0ull : s.increment * n;
                    const uint64_t sum = s.balance + tok < s.balance ? ~0ull : s.balance + tok;
                    s.balance = sum < s.capacity ? sum : s.capacity;
                    s.last_refill = emutime_sat_add(s.last_refill, simtime_sat_mul(s.interval, n, bad));
                    bad |= now < s.last_refill;
                    span = now < s.last_refill ? 0ull : now - s.last_refill;
                }
                const uint64_t next_span = s.interval - span;
                const uint64_t dec = sz[i];
                if (s.balance >= dec) {
                    s.balance -= dec;
                    v = s.balance;
                } else {   // compute_conforming_duration (token_bucket.rs:94-120)
                    const uint64_t req = dec - s.balance;
                    const uint64_t nr = req / s.increment + (req % s.increment ? 1u : 0u);
                    v = nr == 0 ? 0ull
                      : nr == 1 ? next_span
                                : simtime_sat_add(next_span, simtime_sat_mul(s.interval, nr - 1, bad), bad);
                    stt = kTbBlocked;
                    s.pending = emutime_sat_add(now, v);
                }
            }
            status[k] = stt;
            value[k] = v;
        }
    }
    st[r] = s;
    if (bad) atomicOr(err, 1u);
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_tb_setup(shd_ctx* ctx, uint32_t n_relays, const uint64_t* capacity,
                        const uint64_t* refill_increment, const uint64_t* refill_interval_ns,
                        const uint64_t* last_refill) {
    if (!ctx || (n_relays && (!capacity || !refill_increment || !refill_interval_ns || !last_refill)))
        return SHD_ERR_INVALID;
    std::vector<TbRelay> h(n_relays);
    for (uint32_t r = 0; r < n_relays; ++r) {
        const bool any = capacity[r] || refill_increment[r] || refill_interval_ns[r];
        const bool all = capacity[r] && refill_increment[r] && refill_interval_ns[r];
        if (any && !all) return SHD_ERR_INVALID;   // TokenBucket::new -> None (the reference unwraps)
        h[r] = TbRelay{capacity[r], capacity[r], refill_increment[r], refill_interval_ns[r], last_refill[r], 0};
    }
    TbState& T = ctx->tb;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_TRY(T.st.ensure(std::max<size_t>(n_relays, 1) * sizeof(TbRelay)));
    SHD_TRY(T.err.ensure(16));
    if (n_relays)
        SHD_HIP(hipMemcpyAsync(T.st.p, h.data(), (size_t)n_relays * sizeof(TbRelay), hipMemcpyHostToDevice,
                               ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    T.n_relays = n_relays;
    T.ready = true;
    return SHD_OK;
}

shd_status shd_tb_run_device(shd_ctx* ctx, const shd_tb_ops* ops, uint8_t* status, uint64_t* value) {
    if (!ctx || !ops) return SHD_ERR_INVALID;
    TbState& T = ctx->tb;
    if (!T.ready) return SHD_ERR_STATE;
    hipStream_t s = ctx->stream;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_HIP(hipMemsetAsync(T.err.p, 0, 4, s));
    if (T.n_relays)
        tb_run<<<div_up(T.n_relays, 256), 256, 0, s>>>(T.n_relays, ops->relay_off, ops->time, ops->size,
                                                      ops->flags, T.st.as<TbRelay>(), status, value,
                                                      T.err.as<uint32_t>());
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipMemcpyAsync(ctx->h_pin + 28, T.err.p, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    return (uint32_t)ctx->h_pin[28] ? SHD_ERR_INVALID : SHD_OK;
}

shd_status shd_tb_get_state(shd_ctx* ctx, uint32_t relay, shd_tb_state* out) {
    if (!ctx || !out) return SHD_ERR_INVALID;
    TbState& T = ctx->tb;
    if (!T.ready || relay >= T.n_relays) return SHD_ERR_INVALID;
    TbRelay h;
    SHD_HIP(hipMemcpy(&h, T.st.as<TbRelay>() + relay, sizeof(h), hipMemcpyDeviceToHost));
    out->capacity = h.capacity;
    out->balance = h.balance;
    out->refill_increment = h.increment;
    out->refill_interval = h.interval;
    out->last_refill = h.last_refill;
    out->pending_until = h.pending;
    return SHD_OK;
}

}  // extern "C"
