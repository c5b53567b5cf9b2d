// CoDel inbound router queues on the GPU: one queue per destination host,
// device-resident across calls; a call replays every host's push/pop operations of a batch in
// order, lane per host.
//
// Reference semantics: src/main/network/router/codel_queue.rs (FlyearthR/shadow)
//   :19-33   TARGET 10 ms, INTERVAL 100 ms, LIMIT usize::MAX; CONFIG_MTU 1500 (definitions.h:124)
//   :125-147 pop: codel_pop, then store mode / drop_from_store_mode / drop_from_drop_mode
//   :149-198 the two drop paths (control law reset with delta, repeated drops)
//   :201-255 codel_pop (RFC 8289 dodequeue) and process_standing_delay (interval_end)
//   :258-286 should_drop, was_dropping_recently (16 intervals), apply_control_law
//            time + round(INTERVAL / sqrt(count)) in f64 (round half away from zero), saturating
//   :291-306 push (never full: LIMIT is unbounded)
// The host's packets in the queue live in a per-host ring of `capacity` entries; a push beyond it
// is reported (SHD_ERR_INVALID) instead of growing, the one deviation from the unbounded VecDeque.
// The per-host work is a short sequential state machine, so the lane-per-host kernel is
// latency-bound by design; it keeps the queues resident next to the relay output they consume.
#include <algorithm>
#include <cmath>
#include <cstdint>

#include "ctx.h"

namespace shd {

constexpr uint64_t kTarget = 10000000ull;
constexpr uint64_t kInterval = 100000000ull;
constexpr uint64_t kMtu = 1500;
constexpr uint32_t kPop = 0xFFFFFFFFu;
constexpr uint32_t kHasIntervalEnd = 1u, kHasDropNext = 2u, kModeDrop = 4u;
constexpr uint32_t kOpBatch = 16;   // ops per lane loaded ahead of the state machine

struct CodelHost {   // 48 bytes per host
    uint64_t interval_end, drop_next, cur, prev, total;
    uint32_t head, count;
};

__device__ __forceinline__ uint64_t sat_add(uint64_t a, uint64_t b) { return a + b < a ? ~0ull : a + b; }
__device__ __forceinline__ uint64_t sat_sub(uint64_t a, uint64_t b) { return a > b ? a - b : 0ull; }

__device__ __forceinline__ uint64_t control_law(uint64_t t, uint64_t count) {
    // IEEE f64 sqrt and division (correctly rounded on gfx950), as Rust's f64 ops
    const double sq = count == 0 ? 1.0 : sqrt((double)count);
    const double div = (double)kInterval / sq;
    return sat_add(t, (uint64_t)round(div));   // Rust f64::round: half away from zero
}

struct CodelLane {
    CodelHost s;
    uint32_t flags;
    const uint4* ring;   // {pkt, size, ts lo, ts hi}
    uint4* ring_w;
    uint32_t cap;
    uint64_t* fate;
    uint32_t n_ids;
    uint32_t* status;

    __device__ void mark(uint32_t pkt, uint32_t op, uint32_t kind) {
        if (pkt < n_ids) fate[pkt] = ((uint64_t)op << 2) | kind;
        else atomicOr(status, 2u);
    }
    // codel_pop (dodequeue): returns false when the queue is empty
    __device__ bool codel_pop(uint64_t now, uint32_t* pkt, bool* ok_to_drop) {
        if (s.count == 0) {
            flags &= ~kHasIntervalEnd;
            return false;
        }
        const uint4 e = ring[s.head];
        s.head = s.head + 1 == cap ? 0 : s.head + 1;
        --s.count;
        s.total = sat_sub(s.total, e.y);
        const uint64_t ts = ((uint64_t)e.w << 32) | e.z;
        const uint64_t standing = sat_sub(now, ts);
        *pkt = e.x;
        if (standing < kTarget || s.total <= kMtu) {   // process_standing_delay
            flags &= ~kHasIntervalEnd;
            *ok_to_drop = false;
        } else if (flags & kHasIntervalEnd) {
            *ok_to_drop = now >= s.interval_end;
        } else {
            s.interval_end = sat_add(now, kInterval);
            flags |= kHasIntervalEnd;
            *ok_to_drop = false;
        }
        return true;
    }
    __device__ bool should_drop(uint64_t now) const { return (flags & kHasDropNext) && now >= s.drop_next; }
    __device__ bool dropping_recently(uint64_t now) const {
        return (flags & kHasDropNext) && sat_sub(now, s.drop_next) < kInterval * 16;
    }
    // pop (codel_queue.rs:125-198); returns the dequeued packet or kPop
    __device__ uint32_t pop(uint64_t now, uint32_t op) {
        uint32_t pkt = 0;
        bool drop = false;
        if (!codel_pop(now, &pkt, &drop)) {
            flags &= ~kModeDrop;
            return kPop;
        }
        if (!drop) {
            flags &= ~kModeDrop;
            return pkt;
        }
        if (!(flags & kModeDrop)) {   // drop_from_store_mode
            mark(pkt, op, 2);
            uint32_t nxt = 0;
            bool nd = false;
            const bool have = codel_pop(now, &nxt, &nd);
            flags |= kModeDrop;
            const uint64_t delta = sat_sub(s.cur, s.prev);
            s.cur = dropping_recently(now) && delta > 1 ? delta : 1;
            s.drop_next = control_law(now, s.cur);
            flags |= kHasDropNext;
            s.prev = s.cur;
            return have ? nxt : kPop;
        }
        // drop_from_drop_mode
        bool have = true;
        bool item_drop = true;
        while (have && (flags & kModeDrop) && should_drop(now)) {
            mark(pkt, op, 2);
            ++s.cur;
            have = codel_pop(now, &pkt, &item_drop);
            if (have && item_drop) s.drop_next = control_law(s.drop_next, s.cur);
            else flags &= ~kModeDrop;
        }
        return have ? pkt : kPop;
    }
};

__global__ __launch_bounds__(256) void codel_run(uint32_t n_hosts, const uint32_t* __restrict__ off,
                                                 const uint64_t* __restrict__ time,
                                                 const uint32_t* __restrict__ size,
                                                 const uint32_t* __restrict__ pkt, CodelHost* st,
                                                 uint32_t* flags_arr, uint4* ring, uint32_t cap,
                                                 uint32_t* __restrict__ pop_out,
                                                 uint64_t* __restrict__ fate, uint32_t n_ids,
                                                 uint32_t* status) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= n_hosts) return;
    CodelLane L;
    L.s = st[h];
    L.flags = flags_arr[h];
    L.ring = ring + (size_t)h * cap;
    L.ring_w = ring + (size_t)h * cap;
    L.cap = cap;
    L.fate = fate;
    L.n_ids = n_ids;
    L.status = status;
    // The host's ops are read kOpBatch at a time into registers (loads clamped into the range,
    // all issued before the state machine runs), so a lane waits for one memory latency per
    // batch instead of one per op, and its consecutive 8-byte times share cache lines.
    const uint32_t kb = off[h], ke = off[h + 1];
    for (uint32_t k0 = kb; k0 < ke; k0 += kOpBatch) {
        uint64_t tm[kOpBatch];
        uint32_t sz[kOpBatch], pk[kOpBatch];
#pragma unroll
        for (uint32_t i = 0; i < kOpBatch; ++i) {
            const uint32_t k = min(k0 + i, ke - 1);
            tm[i] = time[k];
            sz[i] = size[k];
            pk[i] = pkt[k];
        }
#pragma unroll
        for (uint32_t i = 0; i < kOpBatch; ++i) {
            const uint32_t k = k0 + i;
            if (k >= ke) break;
            const uint64_t now = tm[i];
            if (sz[i] == kPop) {
                const uint32_t got = L.pop(now, k);
                pop_out[k] = got;
                if (got != kPop) L.mark(got, k, 1);
            } else {
                pop_out[k] = kPop;
                if (L.s.count == cap) {   // the reference's queue never fills (LIMIT = usize::MAX)
                    atomicOr(status, 1u);
                    continue;
                }
                uint32_t tail = L.s.head + L.s.count;
                if (tail >= cap) tail -= cap;
                L.ring_w[tail] = make_uint4(pk[i], sz[i], (uint32_t)now, (uint32_t)(now >> 32));
                ++L.s.count;
                L.s.total += sz[i];
            }
        }
    }
    st[h] = L.s;
    flags_arr[h] = L.flags;
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_codel_setup(shd_ctx* ctx, uint32_t n_hosts, uint32_t capacity) {
    if (!ctx || capacity == 0) return SHD_ERR_INVALID;
    CodelState& C = ctx->codel;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_TRY(C.st.ensure(std::max<size_t>(n_hosts, 1) * sizeof(CodelHost)));
    SHD_TRY(C.flags.ensure(std::max<size_t>(n_hosts, 1) * 4));
    SHD_TRY(C.ring.ensure(std::max<size_t>((size_t)n_hosts * capacity, 1) * 16));
    SHD_TRY(C.status.ensure(16));
    SHD_HIP(hipMemsetAsync(C.st.p, 0, (size_t)n_hosts * sizeof(CodelHost), ctx->stream));
    SHD_HIP(hipMemsetAsync(C.flags.p, 0, (size_t)n_hosts * 4, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    C.n_hosts = n_hosts;
    C.cap = capacity;
    C.ready = true;
    return SHD_OK;
}

shd_status shd_codel_run_device(shd_ctx* ctx, const shd_codel_ops* ops, uint32_t* pop_out,
                                uint64_t* fate, uint32_t n_ids) {
    if (!ctx || !ops) return SHD_ERR_INVALID;
    CodelState& C = ctx->codel;
    if (!C.ready) return SHD_ERR_STATE;
    hipStream_t s = ctx->stream;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_HIP(hipMemsetAsync(C.status.p, 0, 4, s));
    if (C.n_hosts)
        codel_run<<<div_up(C.n_hosts, 256), 256, 0, s>>>(
            C.n_hosts, ops->host_off, ops->time, ops->size, ops->pkt, C.st.as<CodelHost>(),
            C.flags.as<uint32_t>(), C.ring.as<uint4>(), C.cap, pop_out, fate, n_ids,
            C.status.as<uint32_t>());
    SHD_HIP(hipGetLastError());
    SHD_HIP(hipMemcpyAsync(ctx->h_pin + 24, C.status.p, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const uint32_t st = (uint32_t)ctx->h_pin[24];
    if (st) {
        // the batch ran with the offending pushes / marks skipped: the queues now hold a state
        // the reference never reaches (and a ring slot freed by a pop may have been reused), so
        // they cannot be rolled back -- shd_codel_setup must run again before the next batch
        C.ready = false;
        return SHD_ERR_INVALID;
    }
    return SHD_OK;
}

shd_status shd_codel_get_state(shd_ctx* ctx, uint32_t host, shd_codel_state* out) {
    if (!ctx || !out) return SHD_ERR_INVALID;
    CodelState& C = ctx->codel;
    if (!C.ready || host >= C.n_hosts) return SHD_ERR_INVALID;
    CodelHost hs;
    uint32_t fl = 0;
    SHD_HIP(hipMemcpy(&hs, C.st.as<CodelHost>() + host, sizeof(hs), hipMemcpyDeviceToHost));
    SHD_HIP(hipMemcpy(&fl, C.flags.as<uint32_t>() + host, 4, hipMemcpyDeviceToHost));
    out->len = hs.count;
    out->mode = (fl & kModeDrop) ? 1 : 0;
    out->has_interval_end = (fl & kHasIntervalEnd) ? 1 : 0;
    out->has_drop_next = (fl & kHasDropNext) ? 1 : 0;
    out->interval_end = hs.interval_end;
    out->drop_next = hs.drop_next;
    out->current_drop_count = hs.cur;
    out->previous_drop_count = hs.prev;
    out->total_bytes_stored = hs.total;
    return SHD_OK;
}

}  // extern "C"
