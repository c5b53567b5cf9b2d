// Device-resident destination event queues.
//
// Reference: every sent packet becomes Event::new_packet(deliver, src_host, src_event_id) pushed
// into the destination host's Mutex<EventQueue> (src/main/core/worker.rs:619-629), a
// BinaryHeap<Reverse<..>> ordered by (time, Packet before Local, src host id, src event id)
// (src/main/core/work/event.rs:84-155, event_queue.rs:28-48).  At the next round the host pops
// every event with time < window_end (src/main/host/host.rs:697-706), in that order; what
// remains waits for a later round (a latency longer than one window keeps an event pending for
// several rounds).  next_event_time() is the head's time (event_queue.rs:43-45).
//
// Here the packet events of all destinations of this GPU stay on the device as one CSR of
// per-host runs sorted by (deliver, src, seq).  One call (shd_equeue_advance) merges a round's
// batch (the relay output: per destination already in that order) into the pending runs and
// splits the merged runs at window_end: the prefix is handed back for Host::execute, the suffix
// stays pending.  Keys are unique ((src, seq) never repeats: event ids are per-host monotone),
// so every event's merged rank is its index in its own run plus the number of smaller events in
// the other run -- a binary search, no atomics, deterministic.
#include <algorithm>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "ctx.h"

namespace shd {

struct EqRuns {   // a CSR of per-host runs
    const uint32_t* off;
    const uint64_t* deliver;
    const uint32_t* src;
    const uint64_t* seq;
    const uint64_t* tag;   // pending runs: the packet tag; batch runs: nullptr (tag from pkt)
    const uint32_t* pkt;   // batch runs only
};

__device__ __forceinline__ bool eq_less(uint64_t ta, uint32_t sa, uint64_t qa, uint64_t tb, uint32_t sb,
                                        uint64_t qb) {
    if (ta != tb) return ta < tb;
    if (sa != sb) return sa < sb;
    return qa < qb;
}

__device__ __forceinline__ uint32_t lower_bound_time(const uint64_t* t, uint32_t b, uint32_t e, uint64_t x) {
    while (b < e) {
        const uint32_t m = (b + e) >> 1;
        if (t[m] < x) b = m + 1; else e = m;
    }
    return b;
}

// per host: events of the merged run that are popped (deliver < window_end) and kept; the
// time of the first kept event (the queue head after the pop) into next[0] by atomic min
__global__ __launch_bounds__(256) void eq_count(uint32_t n_hosts, EqRuns P, EqRuns B, bool has_b,
                                                uint64_t window_end, uint32_t* __restrict__ pop,
                                                uint32_t* __restrict__ keep,
                                                unsigned long long* __restrict__ next) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    uint64_t head = ~0ull;
    if (h < n_hosts) {
        const uint32_t pb = P.off[h], pe = P.off[h + 1];
        const uint32_t lp = lower_bound_time(P.deliver, pb, pe, window_end);
        uint32_t np = lp - pb, nk = pe - lp;
        if (lp < pe) head = P.deliver[lp];
        if (has_b) {
            const uint32_t bb = B.off[h], be = B.off[h + 1];
            const uint32_t lb = lower_bound_time(B.deliver, bb, be, window_end);
            np += lb - bb;
            nk += be - lb;
            if (lb < be) head = B.deliver[lb] < head ? B.deliver[lb] : head;
        }
        pop[h] = np;
        keep[h] = nk;
    } else if (h == n_hosts) {
        pop[h] = 0;
        keep[h] = 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(head, o);
        head = w < head ? w : head;
    }
    if ((threadIdx.x & 63) == 0 && head != ~0ull) atomicMin(next, (unsigned long long)head);
}

struct EqOut {
    uint64_t* deliver;
    uint32_t* src;
    uint64_t* seq;
    uint64_t* tag;
};

// One wave per host: every event of its pending run and of its batch run goes to its merged
// rank, in the popped output (rank < pop count) or the new pending run.  The rank is a binary
// search in the other run; both runs' deliver times are staged in LDS first (when they fit
// kEqCapP / kEqCapB), so the searches step through LDS and touch global memory only on an equal
// deliver time (the (src, seq) tie-break).  Every event is read and written once, coalesced.
constexpr uint32_t kEqCapP = 640, kEqCapB = 192;   // 1024 + 256: 847 us at C5 (LDS-limited occupancy)
__global__ __launch_bounds__(256) void eq_merge(uint32_t n_hosts, EqRuns P, EqRuns B, bool has_b,
                                                uint64_t batch_no, const uint32_t* __restrict__ pop_off,
                                                const uint32_t* __restrict__ keep_off, EqOut popped,
                                                EqOut pending) {
    __shared__ uint64_t s_p[4][kEqCapP];
    __shared__ uint64_t s_b[4][kEqCapB];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t h = blockIdx.x * 4 + w;
    if (h >= n_hosts) return;   // wave-uniform; the kernel has no workgroup barrier
    const uint32_t pb = P.off[h], pe = P.off[h + 1];
    const uint32_t bb = has_b ? B.off[h] : 0u, be = has_b ? B.off[h + 1] : 0u;
    const uint32_t np = pe - pb, nb = be - bb;
    const uint32_t po = pop_off[h], npop = pop_off[h + 1] - po, ko = keep_off[h];
    const bool stage = np <= kEqCapP && nb <= kEqCapB;
    uint64_t* sp = s_p[w];
    uint64_t* sb = s_b[w];
    if (stage) {
        for (uint32_t i = lane; i < np; i += 64) sp[i] = P.deliver[pb + i];
        for (uint32_t j = lane; j < nb; j += 64) sb[j] = B.deliver[bb + j];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    auto put = [&](uint32_t m, uint64_t t, uint32_t s, uint64_t q, uint64_t tg) {
        const EqOut& o = m < npop ? popped : pending;
        const uint32_t at = m < npop ? po + m : ko + (m - npop);
        o.deliver[at] = t;
        o.src[at] = s;
        o.seq[at] = q;
        o.tag[at] = tg;
    };
    for (uint32_t i = lane; i < np; i += 64) {   // pending events: rank among the batch's
        const uint64_t t = stage ? sp[i] : P.deliver[pb + i], q = P.seq[pb + i];
        const uint32_t s = P.src[pb + i];
        const uint64_t tg = P.tag[pb + i];
        uint32_t a = 0, b = nb;
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            const uint64_t tm = stage ? sb[m] : B.deliver[bb + m];
            const bool less = tm != t ? tm < t : eq_less(tm, B.src[bb + m], B.seq[bb + m], t, s, q);
            if (less) a = m + 1; else b = m;
        }
        put(i + a, t, s, q, tg);
    }
    for (uint32_t j = lane; j < nb; j += 64) {   // batch events: rank among the pending ones
        const uint64_t t = stage ? sb[j] : B.deliver[bb + j], q = B.seq[bb + j];
        const uint32_t s = B.src[bb + j];
        const uint64_t tg = (batch_no << 32) | B.pkt[bb + j];
        uint32_t a = 0, b = np;
        while (a < b) {
            const uint32_t m = (a + b) >> 1;
            const uint64_t tm = stage ? sp[m] : P.deliver[pb + m];
            const bool less = tm != t ? tm < t : eq_less(tm, P.src[pb + m], P.seq[pb + m], t, s, q);
            if (less) a = m + 1; else b = m;
        }
        put(j + a, t, s, q, tg);
    }
}

// the advance's totals (events popped, events kept, new head time) into one word triple, so the
// host reads them with one copy
__global__ void eq_totals(uint32_t n_hosts, const uint32_t* __restrict__ pop_off, const uint32_t* __restrict__ keep_off,
                          const unsigned long long* __restrict__ next, uint64_t* __restrict__ out) {
    if (threadIdx.x == 0) {
        out[0] = pop_off[n_hosts];
        out[1] = keep_off[n_hosts];
        out[2] = *next;
    }
}

static shd_status eq_scan(EqState& Q, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s) {
    size_t tmp = 0;
    SHD_HIP(rocprim::exclusive_scan(nullptr, tmp, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
    SHD_TRY(Q.scan_tmp.ensure(tmp));
    SHD_HIP(rocprim::exclusive_scan(Q.scan_tmp.p, tmp, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
    return SHD_OK;
}

static shd_status eq_alloc(EqState& Q, int k, uint64_t n) {
    // half again as much as asked when a buffer must grow: the pending set creeps up over the
    // first rounds, and a reallocation (free + malloc) costs more than the merge
    const size_t m = std::max<uint64_t>(n, 1) * 3 / 2 + 1;
    if ((size_t)std::max<uint64_t>(n, 1) * 8 <= Q.deliver[k].bytes && (size_t)std::max<uint64_t>(n, 1) * 4 <= Q.src[k].bytes)
        return SHD_OK;
    SHD_TRY(Q.deliver[k].ensure(m * 8));
    SHD_TRY(Q.src[k].ensure(m * 4));
    SHD_TRY(Q.seq[k].ensure(m * 8));
    SHD_TRY(Q.tag[k].ensure(m * 8));
    return SHD_OK;
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_equeue_setup(shd_ctx* ctx, uint32_t n_hosts) {
    if (!ctx || n_hosts == 0) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    EqState& Q = ctx->eq;
    for (int k = 0; k < 2; ++k) {
        SHD_TRY(Q.off[k].ensure((size_t)(n_hosts + 1) * 4));
        SHD_TRY(eq_alloc(Q, k, 1));
    }
    SHD_TRY(Q.pop_cnt.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.keep_cnt.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.pop_off.ensure((size_t)(n_hosts + 1) * 4));
    SHD_TRY(Q.next.ensure(32));   // [0] head time accumulator, [1..3] totals
    SHD_HIP(hipMemsetAsync(Q.off[0].p, 0, (size_t)(n_hosts + 1) * 4, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    Q.cur = 0;
    Q.n_hosts = n_hosts;
    Q.n_pending = 0;
    Q.n_popped = 0;
    Q.batches = 0;
    Q.ready = true;
    return SHD_OK;
}

shd_status shd_equeue_advance(shd_ctx* ctx, const shd_relay_out* d_batch, uint64_t window_end,
                              shd_equeue_out* out) {
    if (!ctx || !out) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    const bool has_b = d_batch != nullptr;
    if (has_b && (!d_batch->ev_off || (d_batch->n_sent && (!d_batch->ev_deliver || !d_batch->ev_src ||
                                                          !d_batch->ev_seq || !d_batch->ev_pkt))))
        return SHD_ERR_INVALID;
    if (has_b && Q.batches >= 0xFFFFFFFFull) return SHD_ERR_INVALID;   // tag bits exhausted
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint32_t H = Q.n_hosts;
    const int c = Q.cur, n = 1 - c;
    const uint64_t n_in = Q.n_pending + (has_b ? d_batch->n_sent : 0);
    if (n_in >= 0xFFFFFFFFull) return SHD_ERR_INVALID;   // 32-bit positions
    SHD_TRY(eq_alloc(Q, n, n_in));
    const uint64_t n_cap = std::max<uint64_t>(n_in, 1) * 3 / 2 + 1;   // growth headroom, as eq_alloc
    if (Q.ps.bytes < std::max<uint64_t>(n_in, 1) * 4) {
        SHD_TRY(Q.pd.ensure(n_cap * 8));
        SHD_TRY(Q.ps.ensure(n_cap * 4));
        SHD_TRY(Q.pq.ensure(n_cap * 8));
        SHD_TRY(Q.pt.ensure(n_cap * 8));
    }
    EqRuns P{Q.off[c].as<uint32_t>(), Q.deliver[c].as<uint64_t>(), Q.src[c].as<uint32_t>(),
             Q.seq[c].as<uint64_t>(), Q.tag[c].as<uint64_t>(), nullptr};
    EqRuns B{};
    if (has_b)
        B = EqRuns{d_batch->ev_off, d_batch->ev_deliver, d_batch->ev_src, d_batch->ev_seq, nullptr,
                   d_batch->ev_pkt};
    SHD_HIP(hipMemsetAsync(Q.next.p, 0xFF, 8, s));
    eq_count<<<div_up((uint64_t)H + 1, 256), 256, 0, s>>>(H, P, B, has_b, window_end, Q.pop_cnt.as<uint32_t>(),
                                                          Q.keep_cnt.as<uint32_t>(),
                                                          Q.next.as<unsigned long long>());
    SHD_HIP(hipGetLastError());
    SHD_TRY(eq_scan(Q, Q.pop_cnt.as<uint32_t>(), Q.pop_off.as<uint32_t>(), H + 1, s));
    SHD_TRY(eq_scan(Q, Q.keep_cnt.as<uint32_t>(), Q.off[n].as<uint32_t>(), H + 1, s));
    EqOut popped{Q.pd.as<uint64_t>(), Q.ps.as<uint32_t>(), Q.pq.as<uint64_t>(), Q.pt.as<uint64_t>()};
    EqOut pending{Q.deliver[n].as<uint64_t>(), Q.src[n].as<uint32_t>(), Q.seq[n].as<uint64_t>(),
                  Q.tag[n].as<uint64_t>()};
    if (n_in)
        eq_merge<<<div_up(H, 4), 256, 0, s>>>(H, P, B, has_b, Q.batches, Q.pop_off.as<uint32_t>(),
                                              Q.off[n].as<uint32_t>(), popped, pending);
    SHD_HIP(hipGetLastError());
    // totals and the new head time: one pinned read-back
    eq_totals<<<1, 64, 0, s>>>(H, Q.pop_off.as<uint32_t>(), Q.off[n].as<uint32_t>(),
                               Q.next.as<unsigned long long>(), Q.next.as<uint64_t>() + 1);
    SHD_HIP(hipMemcpyAsync(ctx->h_pin + 32, Q.next.as<uint64_t>() + 1, 24, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const uint32_t n_pop = (uint32_t)ctx->h_pin[32], n_keep = (uint32_t)ctx->h_pin[33];
    if ((uint64_t)n_pop + n_keep != n_in) return SHD_ERR_INVALID;   // batch ev_off / n_sent disagree
    Q.cur = n;
    Q.n_pending = n_keep;
    Q.n_popped = n_pop;
    if (has_b) ++Q.batches;
    out->off = Q.pop_off.as<uint32_t>();
    out->deliver = Q.pd.as<uint64_t>();
    out->src = Q.ps.as<uint32_t>();
    out->seq = Q.pq.as<uint64_t>();
    out->tag = Q.pt.as<uint64_t>();
    out->n_popped = n_pop;
    out->n_pending = n_keep;
    out->next_time = ctx->h_pin[34];
    return SHD_OK;
}

shd_status shd_equeue_copy_popped(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                                  uint64_t* seq, uint64_t* tag) {
    if (!ctx) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t n = Q.n_popped;
    if (off) SHD_HIP(hipMemcpyAsync(off, Q.pop_off.p, (size_t)(Q.n_hosts + 1) * 4, hipMemcpyDeviceToHost, s));
    if (n) {
        if (deliver) SHD_HIP(hipMemcpyAsync(deliver, Q.pd.p, n * 8, hipMemcpyDeviceToHost, s));
        if (src) SHD_HIP(hipMemcpyAsync(src, Q.ps.p, n * 4, hipMemcpyDeviceToHost, s));
        if (seq) SHD_HIP(hipMemcpyAsync(seq, Q.pq.p, n * 8, hipMemcpyDeviceToHost, s));
        if (tag) SHD_HIP(hipMemcpyAsync(tag, Q.pt.p, n * 8, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

shd_status shd_equeue_pending(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                              uint64_t* seq, uint64_t* tag, uint64_t* n_pending) {
    if (!ctx) return SHD_ERR_INVALID;
    EqState& Q = ctx->eq;
    if (!Q.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int c = Q.cur;
    const uint64_t n = Q.n_pending;
    if (n_pending) *n_pending = n;
    if (off) SHD_HIP(hipMemcpyAsync(off, Q.off[c].p, (size_t)(Q.n_hosts + 1) * 4, hipMemcpyDeviceToHost, s));
    if (n) {
        if (deliver) SHD_HIP(hipMemcpyAsync(deliver, Q.deliver[c].p, n * 8, hipMemcpyDeviceToHost, s));
        if (src) SHD_HIP(hipMemcpyAsync(src, Q.src[c].p, n * 4, hipMemcpyDeviceToHost, s));
        if (seq) SHD_HIP(hipMemcpyAsync(seq, Q.seq[c].p, n * 8, hipMemcpyDeviceToHost, s));
        if (tag) SHD_HIP(hipMemcpyAsync(tag, Q.tag[c].p, n * 8, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

}  // extern "C"
