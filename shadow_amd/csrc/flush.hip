// shd_relay_flush: the drop-in form of the relay round -- the worker threads' staging buffers as
// they stand at the round barrier, grouped by source host on the device, with the CPU-drawn loss
// draws, and compact outputs for the trip back over PCIe.
//
// Reference: Worker::send_packet (src/main/core/worker.rs:328-413) runs on every worker thread;
// each host runs on one thread per round (scheduler/thread_per_core.rs:188-206), so a host's sends
// are ONE contiguous run in ONE thread's buffer, in send order.  The round's sends reach the device
// as those buffers (stage = thread), each a list of runs (host, count) and 12-byte send records:
//   time_off = now - time_base, dst | SHD_SEND_PAYLOAD (payload_size > 0 is all the drop rule reads,
//   worker.rs:370), draw_hi = the source host's next_u64() >> 32 at send time.  gen::<f64>() is
//   (next_u64 >> 11) * 2^-53 and consumes exactly one next_u64, so the CPU stream advances as in
//   the reference; the top 32 bits decide `chance >= reliability` exactly for every reliability
//   1f32 - loss (relay.hip draw_drops).
// The device turns the runs into the grouped layout the pipelines take (src_off, one contiguous
// range per host in host order), runs the round with those draws (the device streams are left
// untouched), and writes back per send a 2-bit status in stage order, and per event a 16-byte
// record {deliver - round_end, src host, event id - the host's first id of the round, send index
// in stage order} grouped by destination in EventQueue order (event.rs:84-155).
#include <algorithm>
#include <cstring>

#include "ctx.h"
#include "scan.h"

namespace shd {

// relay.hip: the round (pipelines + checks + commit) on a grouped device batch; the sharded
// round on this rank's grouped sends
shd_status relay_flush_round(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o);
shd_status relay_flush_round_sharded(shd_ctx* ctx, const shd_batch* b, const shd_round* rd, shd_relay_out* o);

struct Send12 {
    uint32_t time_off, dst, draw_hi;
};
static_assert(sizeof(Send12) == sizeof(shd_send12), "12-byte staged send");

// per run: its host's run index (+1); a second run of one host is an error (red[0]), as is a
// host outside the relay (red[1])
__global__ __launch_bounds__(256) void fl_runs(uint32_t n_runs, const uint32_t* __restrict__ run_host,
                                               uint32_t n_hosts, uint32_t* __restrict__ hrun,
                                               unsigned long long* __restrict__ red) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n_runs) return;
    const uint32_t h = run_host[r];
    if (h >= n_hosts) {
        atomicMin(&red[1], (unsigned long long)r);
        return;
    }
    if (atomicExch(&hrun[h], r + 1) != 0) atomicMin(&red[0], (unsigned long long)h);
}

// Zero-copy staging: when every staging buffer is pinned host memory the device reads it where it
// lies (a device view of the pinned pages) instead of one copy per buffer -- at C5 three copies per
// worker thread, each with ~11 us of launch gap, plus the re-read of the uploaded sends.
struct FlStage {
    const uint32_t* rh;    // device views of the stage's run_host / run_count / sends
    const uint32_t* rc;
    const Send12* sd;
    uint64_t send_base;    // the stage's first send in stage order
    uint32_t run_base, n_runs;
};

// fl_runs on the staged runs themselves: each run's host and count (copied to the device arrays
// the scans read) and its stage
__global__ __launch_bounds__(256) void fl_runs_zc(uint32_t n_runs, const FlStage* __restrict__ st, uint32_t n_stages,
                                                  uint32_t n_hosts, uint32_t* __restrict__ runh,
                                                  uint32_t* __restrict__ runc, uint32_t* __restrict__ rstage,
                                                  uint32_t* __restrict__ hrun, unsigned long long* __restrict__ red) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n_runs) return;
    uint32_t lo = 0, hi = n_stages;   // the last stage whose first run is <= r (stages without runs skipped)
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (st[m].run_base <= r) lo = m; else hi = m;
    }
    while (lo + 1 < n_stages && (st[lo].n_runs == 0 || r - st[lo].run_base >= st[lo].n_runs)) ++lo;
    const uint32_t i = r - st[lo].run_base, h = st[lo].rh[i];
    runh[r] = h;
    runc[r] = st[lo].rc[i];
    rstage[r] = lo;
    if (h >= n_hosts) {
        atomicMin(&red[1], (unsigned long long)r);
        return;
    }
    if (atomicExch(&hrun[h], r + 1) != 0) atomicMin(&red[0], (unsigned long long)h);
}

// per host: its send count (0 without a run); entry n_hosts is 0 so one scan gives src_off[0..H]
__global__ __launch_bounds__(256) void fl_host_counts(uint32_t n_hosts, const uint32_t* __restrict__ hrun,
                                                      const uint32_t* __restrict__ run_count,
                                                      uint32_t* __restrict__ hcnt) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h > n_hosts) return;
    const uint32_t r = h < n_hosts ? hrun[h] : 0u;
    hcnt[h] = r ? run_count[r - 1] : 0u;
}

// one wave per host: its run's records into the grouped arrays the pipelines read, the permutation
// both ways (grouped position <-> send index in stage order).  Under a communicator every rank
// groups every host's sends (the permutation covers all of them) but writes the arrays of its own
// hosts [lo, hi) only, from position src_off[lo] on.
__global__ __launch_bounds__(256) void fl_gather(uint32_t n_hosts, const uint32_t* __restrict__ hrun,
                                                 const uint32_t* __restrict__ run_off,
                                                 const uint32_t* __restrict__ src_off, const Send12* __restrict__ in,
                                                 uint64_t time_base, uint64_t* __restrict__ send_time,
                                                 uint32_t* __restrict__ dst_host, uint32_t* __restrict__ payload,
                                                 uint32_t* __restrict__ draws, uint32_t* __restrict__ perm,
                                                 uint32_t* __restrict__ inv, uint32_t lo, uint32_t hi,
                                                 const FlStage* __restrict__ st, const uint32_t* __restrict__ rstage) {
    const uint32_t h = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (h >= n_hosts) return;
    const uint32_t r = hrun[h];
    if (!r) return;
    const uint32_t from = run_off[r - 1], to = src_off[h], cnt = src_off[h + 1] - to;
    const bool own = h >= lo && h < hi;
    const uint32_t base = src_off[lo];
    // the run's sends: in the uploaded copy, or (zero-copy) in its stage's pinned buffer
    const Send12* rs = in + from;
    if (st) {
        const FlStage& S = st[rstage[r - 1]];
        rs = S.sd + (from - S.send_base);
    }
    for (uint32_t k = lane; k < cnt; k += 64) {
        const uint32_t p = to + k;
        perm[p] = from + k;
        inv[from + k] = p;
        if (!own) continue;
        const Send12 x = rs[k];
        const uint32_t q = p - base;
        send_time[q] = time_base + x.time_off;
        dst_host[q] = x.dst & ~SHD_SEND_PAYLOAD;
        payload[q] = x.dst >> 31;
        draws[q] = x.draw_hi;
    }
}

// a sharded flush: this rank's hosts' offsets from 0 (the batch of the sharded round), and its
// grouped range [src_off[lo], src_off[hi]) in red[2], red[3] for the host
__global__ __launch_bounds__(256) void fl_rebase(const uint32_t* __restrict__ goff, uint32_t lo, uint32_t n_own,
                                                 uint32_t* __restrict__ off, unsigned long long* __restrict__ red) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k <= n_own) off[k] = goff[lo + k] - goff[lo];
    if (k == 0) {
        red[2] = goff[lo];
        red[3] = goff[lo + n_own];
    }
}

// an event record: 16 bytes {deliver - round_end, src, seq_off, send}, or (shd_flush_out.event_bytes
// = 12) 12 bytes without the source host, which the caller's packet (send index) already names
__device__ __forceinline__ void fl_put_event(void* out, bool b12, uint64_t e, uint32_t d, uint32_t s, uint32_t q,
                                             uint32_t send) {
    if (b12) {
        uint32_t* o = static_cast<uint32_t*>(out) + 3 * e;
        o[0] = d;
        o[1] = q;
        o[2] = send;
    } else {
        static_cast<uint4*>(out)[e] = make_uint4(d, s, q, send);
    }
}

// 2-bit statuses in stage order: byte j holds sends 4j .. 4j+3 (send 4j + k in bits 2k, 2k+1);
// sharded: the statuses of grouped positions [base, base + n_own) (this rank's hosts), 0 elsewhere
__global__ __launch_bounds__(256) void fl_status2(uint64_t n, const uint32_t* __restrict__ inv,
                                                  const uint8_t* __restrict__ st, uint8_t* __restrict__ out,
                                                  uint32_t base, uint32_t n_own) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j * 4 >= n) return;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (j * 4 + k < n) {
            const uint32_t p = inv[j * 4 + k] - base;
            if (p < n_own) v |= (uint32_t)(st[p] & 3u) << (2 * k);
        }
    out[j] = (uint8_t)v;
}

// 16-byte event records of a sharded flush: the ids are already relative (RelayState::rel_ids);
// ev_pkt indexes its sender rank's grouped sends, which start at goff[first host of that rank]
__global__ __launch_bounds__(256) void fl_events16x(uint64_t n, uint64_t round_end, const uint64_t* __restrict__ deliver,
                                                    const uint32_t* __restrict__ src, const uint64_t* __restrict__ seq,
                                                    const uint32_t* __restrict__ pkt, const uint32_t* __restrict__ goff,
                                                    uint32_t per, const uint32_t* __restrict__ perm,
                                                    void* __restrict__ out, uint32_t b12) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const uint32_t s = src[e], first = (s / per) * per;
    fl_put_event(out, b12 != 0, e, (uint32_t)(deliver[e] - round_end), s, (uint32_t)seq[e], perm[goff[first] + pkt[e]]);
}

// event records (already grouped by destination in EventQueue order)
__global__ __launch_bounds__(256) void fl_events16(uint64_t n, uint64_t round_end, const uint64_t* __restrict__ deliver,
                                                   const uint32_t* __restrict__ src, const uint64_t* __restrict__ seq,
                                                   const uint32_t* __restrict__ pkt, const uint64_t* __restrict__ seq_base,
                                                   const uint32_t* __restrict__ perm, void* __restrict__ out, uint32_t b12) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const uint32_t s = src[e];
    fl_put_event(out, b12 != 0, e, (uint32_t)(deliver[e] - round_end), s, (uint32_t)(seq[e] - seq_base[s]), perm[pkt[e]]);
}

// a device view of host memory p when it is pinned (hipHostMalloc / registered), else nullptr
static const void* dev_view(const void* p) {
    if (!p) return nullptr;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: not an error of the call
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer || !at.hostPointer) return nullptr;
    return static_cast<const char*>(at.devicePointer) + (static_cast<const char*>(p) - static_cast<const char*>(at.hostPointer));
}

}  // namespace shd

using namespace shd;

extern "C" {

void* shd_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void shd_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

shd_status shd_relay_flush(shd_ctx* ctx, const shd_stage* stages, uint32_t n_stages, uint64_t time_base,
                           const shd_round* round, shd_flush_out* out) {
    if (!ctx || !round || !out || (n_stages && !stages)) return SHD_ERR_INVALID;
    if (out->struct_size != sizeof(shd_flush_out)) return SHD_ERR_INVALID;   // another header's layout
    if (out->event_bytes != 0 && out->event_bytes != 12 && out->event_bytes != 16) return SHD_ERR_INVALID;
    const uint32_t eb = out->event_bytes == 12 ? 12u : 16u;
    RelayState& R = ctx->relay;
    if (!R.ready) return SHD_ERR_STATE;
    if (R.sharded && (!R.x_words.p || !R.xs_pin.p)) return SHD_ERR_STATE;   // set up before the communicator
    // host-side shape checks (each stage's runs cover exactly its records)
    uint64_t n = 0, n_runs = 0;
    for (uint32_t k = 0; k < n_stages; ++k) {
        const shd_stage& S = stages[k];
        if (S.n_runs && (!S.run_host || !S.run_count)) return SHD_ERR_INVALID;
        if (S.n_sends && !S.sends) return SHD_ERR_INVALID;
        uint64_t c = 0;
        for (uint32_t r = 0; r < S.n_runs; ++r) c += S.run_count[r];
        if (c != S.n_sends) return SHD_ERR_INVALID;
        n += S.n_sends;
        n_runs += S.n_runs;
    }
    const uint32_t H = R.n_hosts;
    if (n >= (1ull << 32) || n_runs >= (1ull << 32)) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t nn = std::max<uint64_t>(n, 1), nr = std::max<uint64_t>(n_runs, 1);
    SHD_TRY(R.fl_runh.ensure(nr * 4));
    SHD_TRY(R.fl_runc.ensure(nr * 4));
    SHD_TRY(R.fl_runo.ensure(nr * 4));
    SHD_TRY(R.fl_hrun.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.fl_hcnt.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.fl_send.ensure(nn * 12));
    SHD_TRY(R.fl_perm.ensure(nn * 4));
    SHD_TRY(R.fl_inv.ensure(nn * 4));
    SHD_TRY(R.fl_st2.ensure(nn / 4 + 1));
    SHD_TRY(R.fl_ev16.ensure(nn * 16));
    SHD_TRY(R.pk_off.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.pk_time.ensure(nn * 8));
    SHD_TRY(R.pk_dst.ensure(nn * 4));
    SHD_TRY(R.pk_pay.ensure(nn * 4));
    SHD_TRY(R.draws.ensure(nn * 4));
    SHD_TRY(R.st.ensure(nn));
    SHD_TRY(R.ev_off.ensure((size_t)(H + 1) * 4));
    SHD_TRY(R.ev_deliver.ensure(nn * 8));
    SHD_TRY(R.ev_src.ensure(nn * 4));
    SHD_TRY(R.ev_seq.ensure(nn * 8));
    SHD_TRY(R.ev_pkt.ensure(nn * 4));
    SHD_TRY(R.red.ensure(64));
    SHD_TRY(R.fl_goff.ensure((size_t)(H + 1) * 4));
    // under a communicator: this rank's hosts [lo, hi) (the stages hold every rank's hosts)
    uint32_t lo = 0, hi = H;
    if (R.sharded) shard_range(H, ctx->comm->size, ctx->comm->rank, &lo, &hi);
    // 1. the staging buffers: read where they lie when all are pinned (zero-copy), else copied stage
    //    after stage (pinned host memory -- shd_host_alloc -- moves at the link's rate; pageable
    //    memory is staged by the runtime)
    std::vector<FlStage> tab(n_stages);
    bool zc = n_stages > 0 && !ctx->knobs.on(K_FLUSH_COPY);
    {
        uint64_t at = 0;
        uint32_t ar = 0;
        for (uint32_t k = 0; k < n_stages && zc; ++k) {
            const shd_stage& S = stages[k];
            FlStage& T = tab[k];
            T.rh = static_cast<const uint32_t*>(S.n_runs ? dev_view(S.run_host) : nullptr);
            T.rc = static_cast<const uint32_t*>(S.n_runs ? dev_view(S.run_count) : nullptr);
            T.sd = static_cast<const Send12*>(S.n_sends ? dev_view(S.sends) : nullptr);
            if ((S.n_runs && (!T.rh || !T.rc)) || (S.n_sends && !T.sd)) zc = false;
            T.send_base = at;
            T.run_base = ar;
            T.n_runs = S.n_runs;
            at += S.n_sends;
            ar += S.n_runs;
        }
    }
    if (zc) {
        SHD_TRY(R.fl_tab.ensure((size_t)n_stages * sizeof(FlStage)));
        SHD_TRY(R.fl_tab_pin.ensure((size_t)n_stages * sizeof(FlStage)));
        SHD_TRY(R.fl_rstg.ensure(nr * 4));
        std::memcpy(R.fl_tab_pin.p, tab.data(), (size_t)n_stages * sizeof(FlStage));
        SHD_HIP(hipMemcpyAsync(R.fl_tab.p, R.fl_tab_pin.p, (size_t)n_stages * sizeof(FlStage), hipMemcpyHostToDevice, s));
    }
    if (!zc) {
        uint64_t at = 0, ar = 0;
        for (uint32_t k = 0; k < n_stages; ++k) {
            const shd_stage& S = stages[k];
            if (S.n_runs) {
                SHD_HIP(hipMemcpyAsync(R.fl_runh.as<uint32_t>() + ar, S.run_host, (size_t)S.n_runs * 4,
                                       hipMemcpyHostToDevice, s));
                SHD_HIP(hipMemcpyAsync(R.fl_runc.as<uint32_t>() + ar, S.run_count, (size_t)S.n_runs * 4,
                                       hipMemcpyHostToDevice, s));
            }
            if (S.n_sends)
                SHD_HIP(hipMemcpyAsync(R.fl_send.as<char>() + at * 12, S.sends, S.n_sends * 12, hipMemcpyHostToDevice, s));
            at += S.n_sends;
            ar += S.n_runs;
        }
    }
    // 2. runs -> hosts, per-host counts, the grouped offsets, the gather
    unsigned long long* red = R.red.as<unsigned long long>();
    SHD_HIP(hipMemsetAsync(R.fl_hrun.p, 0, (size_t)(H + 1) * 4, s));
    SHD_HIP(hipMemsetAsync(red, 0xFF, 16, s));
    if (n_runs) {
        if (zc)
            fl_runs_zc<<<div_up(n_runs, 256), 256, 0, s>>>((uint32_t)n_runs, R.fl_tab.as<FlStage>(), n_stages, H,
                                                            R.fl_runh.as<uint32_t>(), R.fl_runc.as<uint32_t>(),
                                                            R.fl_rstg.as<uint32_t>(), R.fl_hrun.as<uint32_t>(), red);
        else
            fl_runs<<<div_up(n_runs, 256), 256, 0, s>>>((uint32_t)n_runs, R.fl_runh.as<uint32_t>(), H,
                                                         R.fl_hrun.as<uint32_t>(), red);
        SHD_TRY(scan_excl2(R.scan, R.fl_runc.as<uint32_t>(), R.fl_runo.as<uint32_t>(), nullptr, nullptr, n_runs, s));
    }
    fl_host_counts<<<div_up((uint64_t)H + 1, 256), 256, 0, s>>>(H, R.fl_hrun.as<uint32_t>(), R.fl_runc.as<uint32_t>(),
                                                                R.fl_hcnt.as<uint32_t>());
    uint32_t* goff = R.sharded ? R.fl_goff.as<uint32_t>() : R.pk_off.as<uint32_t>();   // grouped offsets, all hosts
    SHD_TRY(scan_excl2(R.scan, R.fl_hcnt.as<uint32_t>(), goff, nullptr, nullptr, (uint64_t)H + 1, s));
    if (n)
        fl_gather<<<div_up(H, 4), 256, 0, s>>>(H, R.fl_hrun.as<uint32_t>(), R.fl_runo.as<uint32_t>(), goff,
                                                R.fl_send.as<Send12>(), time_base, R.pk_time.as<uint64_t>(),
                                                R.pk_dst.as<uint32_t>(), R.pk_pay.as<uint32_t>(), R.draws.as<uint32_t>(),
                                                R.fl_perm.as<uint32_t>(), R.fl_inv.as<uint32_t>(), lo, hi,
                                                zc ? R.fl_tab.as<FlStage>() : nullptr,
                                                zc ? R.fl_rstg.as<uint32_t>() : nullptr);
    if (R.sharded)
        fl_rebase<<<div_up((uint64_t)(hi - lo) + 1, 256), 256, 0, s>>>(goff, lo, hi - lo, R.pk_off.as<uint32_t>(), red);
    SHD_HIP(hipGetLastError());
    // h_pin words 32-35: the checks (and, sharded, this rank's grouped range).  Under a communicator a
    // failed check is this rank's alone: the flush returns before the round's collectives, as a call
    // with invalid arguments would, on whichever ranks see the bad runs (every rank sees the same
    // stages, so all of them do).
    SHD_TRY(readback(ctx, s, 32, red, R.sharded ? 32 : 16));
    if (ctx->h_pin[33] != ~0ull) return SHD_ERR_NO_HOST;   // a run of a host the relay does not have
    if (ctx->h_pin[32] != ~0ull) return SHD_ERR_INVALID;   // a host with two runs (two threads, or split)
    const uint64_t base = R.sharded ? ctx->h_pin[34] : 0, n_own = R.sharded ? ctx->h_pin[35] - ctx->h_pin[34] : n;
    // 3. the round on the grouped batch with the CPU's draws (the device streams stay as they are)
    shd_batch db{n_own, R.pk_off.as<uint32_t>(), R.pk_time.as<uint64_t>(), R.pk_dst.as<uint32_t>(),
                 R.pk_pay.as<uint32_t>(), nullptr};
    shd_relay_out dout{};
    dout.status = R.st.as<uint8_t>();
    dout.ev_off = R.ev_off.as<uint32_t>();
    dout.ev_deliver = R.ev_deliver.as<uint64_t>();
    dout.ev_src = R.ev_src.as<uint32_t>();
    dout.ev_seq = R.ev_seq.as<uint64_t>();
    dout.ev_pkt = R.ev_pkt.as<uint32_t>();
    // zero-copy outputs: the events and the 2-bit statuses written by the kernels straight into the
    // caller's pinned buffers, so no copy follows the round (the writes cross the link as they go)
    const bool zo = !ctx->knobs.on(K_FLUSH_COPY);
    void* ev_host = zo && out->events ? const_cast<void*>(dev_view(out->events)) : nullptr;
    uint8_t* st2_host = zo && out->status2 ? static_cast<uint8_t*>(const_cast<void*>(dev_view(out->status2))) : nullptr;
    void* ev_dst = ev_host ? ev_host : R.fl_ev16.p;
    uint8_t* st2_dst = st2_host ? st2_host : R.fl_st2.as<uint8_t>();
    R.cpu_draws = true;
    R.rel_ids = true;   // records carry ids relative to the source's first of the round
    R.fl_ev_out = R.sharded ? nullptr : ev_dst;
    R.fl_b12 = eb == 12 ? 1u : 0u;
    R.fl_direct = false;
    const shd_status st = R.sharded ? relay_flush_round_sharded(ctx, &db, round, &dout)
                                    : relay_flush_round(ctx, &db, round, &dout);
    R.cpu_draws = false;
    R.rel_ids = false;
    R.fl_ev_out = nullptr;
    const bool direct = R.fl_direct && R.last_pipe == 7;   // (a rerun on pipeline 3 / 1 wrote the arrays)
    R.fl_direct = false;
    SHD_TRY(st);
    // 4. compact outputs (the round committed: next_id2 holds every own host's first id of the round)
    const uint64_t ns = dout.n_sent, n_ev = R.sharded ? dout.n_events : ns;
    const uint64_t* seq_base = R.next_id2.as<uint64_t>();
    if (n) fl_status2<<<div_up((n + 3) / 4, 256), 256, 0, s>>>(n, R.fl_inv.as<uint32_t>(), R.st.as<uint8_t>(),
                                                              st2_dst, (uint32_t)base, (uint32_t)n_own);
    if (n_ev && R.sharded)
        fl_events16x<<<div_up(n_ev, 256), 256, 0, s>>>(n_ev, round->round_end, dout.ev_deliver, dout.ev_src,
                                                       dout.ev_seq, dout.ev_pkt, goff,
                                                       (uint32_t)div_up((uint64_t)H, (uint64_t)ctx->comm->size),
                                                       R.fl_perm.as<uint32_t>(), ev_dst, eb == 12 ? 1u : 0u);
    else if (n_ev && !direct)
        fl_events16<<<div_up(ns, 256), 256, 0, s>>>(ns, round->round_end, R.ev_deliver.as<uint64_t>(),
                                                    R.ev_src.as<uint32_t>(), R.ev_seq.as<uint64_t>(),
                                                    R.ev_pkt.as<uint32_t>(), seq_base, R.fl_perm.as<uint32_t>(),
                                                    ev_dst, eb == 12 ? 1u : 0u);
    SHD_HIP(hipGetLastError());
    if (out->status2 && n && !st2_host)
        SHD_HIP(hipMemcpyAsync(out->status2, R.fl_st2.p, (n + 3) / 4, hipMemcpyDeviceToHost, s));
    if (out->ev_off)
        SHD_HIP(hipMemcpyAsync(out->ev_off, dout.ev_off, (size_t)(hi - lo + 1) * 4, hipMemcpyDeviceToHost, s));
    if (out->events && n_ev && !ev_host)
        SHD_HIP(hipMemcpyAsync(out->events, R.fl_ev16.p, n_ev * eb, hipMemcpyDeviceToHost, s));
    if (out->seq_base && hi > lo)
        SHD_HIP(hipMemcpyAsync(out->seq_base + lo, seq_base + lo, (size_t)(hi - lo) * 8, hipMemcpyDeviceToHost, s));
    SHD_TRY(wait_stream(ctx, s));
    out->min_deliver = dout.min_deliver;
    out->min_latency = dout.min_latency;
    out->n_sent = ns;
    out->n_events = n_ev;
    return SHD_OK;
}

}  // extern "C"
