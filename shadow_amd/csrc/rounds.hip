// Round bookkeeping around the two paths: the runahead and the next scheduling window, and the
// RoutingInfo lookups a caller makes between rounds.
//
// Reference:
//   Runahead (src/main/core/scheduler/runahead.rs:12-115): get() = max(min_used_latency or
//     min_possible_latency, min_runahead_config); update_lowest_used_latency() lowers
//     min_used_latency when dynamic runahead is on -- Worker::send_packet calls it with the path
//     latency of every packet it sends (worker.rs:380, 292-303).
//   The window (SimController::manager_finished_current_round, controller.rs:86-111):
//     start = the minimum next event time over all hosts and the round's sent packets
//     (manager.rs:430-435, 455-464; EmulatedTime::MAX when there is none), end = min(start +
//     runahead (checked_add, EmulatedTime::MAX on overflow), end_time), continue iff start < end.
//   RoutingInfo::path lookups (graph/mod.rs:446-448) through worker_getLatency
//     (worker.rs:660-670), which TCP autotuning calls per connection (tcp.c:451-452).
#include <algorithm>
#include <cstring>

#include "ctx.h"

namespace shd {

shd_status min_u64_device(shd_ctx* ctx, const uint64_t* d, uint64_t n, uint64_t* out);

constexpr uint64_t kEmuMax = ~0ull - 1;   // EmulatedTime::MAX (EMUTIME_MAX = u64::MAX - 1)

void round_note(shd_ctx* ctx, uint64_t min_deliver, uint64_t min_latency) {
    RoundState& W = ctx->rnd;
    W.batch_min_deliver = std::min(W.batch_min_deliver, min_deliver);
    if (W.ready && W.dynamic && min_latency != ~0ull && min_latency != 0)
        W.min_used = std::min(W.min_used, min_latency);
}

static uint64_t runahead_of(const RoundState& W) {
    const uint64_t r = W.min_used != ~0ull ? W.min_used : W.min_possible;
    return std::max(r, W.cfg);
}

static void window_of(uint64_t min_next, uint64_t ra, uint64_t end_time, uint64_t* s, uint64_t* e, int32_t* run) {
    // manager.rs:459-464: no next event -> EmulatedTime::MAX
    const uint64_t start = min_next > kEmuMax ? kEmuMax : min_next;
    // checked_add: an overflow, or a sum past EMUTIME_MAX (from_c_emutime), is None -> MAX
    uint64_t end = start + ra;
    if (end < start || end > kEmuMax) end = kEmuMax;
    end = std::min(end, end_time);
    *s = start;
    *e = end;
    *run = start < end ? 1 : 0;
}

// The read-back of a call's few result words and its completion marker in ONE launch: a wave
// copies the words into the pinned host words, a system-scope release orders them before the
// marker, which the host polls (shd::readback).  Replaces a D2H copy plus the marker copy -- two
// DMA operations of a few microseconds each -- on every synchronous call (SHD_SYNC_KERNEL=0: the
// copies).
__global__ __launch_bounds__(64) void readback_mark(const unsigned long long* __restrict__ src, uint32_t n,
                                                    unsigned long long* dst, unsigned long long* marker) {
    for (uint32_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // every lane's words reach the host first
    if (threadIdx.x == 0) __hip_atomic_store(marker, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

shd_status readback_launch(hipStream_t s, const void* d_src, uint32_t n_words, unsigned long long* h_dst,
                           unsigned long long* h_marker) {
    readback_mark<<<1, 64, 0, s>>>(static_cast<const unsigned long long*>(d_src), n_words, h_dst, h_marker);
    SHD_HIP(hipGetLastError());
    return SHD_OK;
}

// one gather of n (row, col) pairs of the resident table
__global__ __launch_bounds__(256) void lookup_gather(uint64_t n, const uint32_t* __restrict__ rows,
                                                     const uint32_t* __restrict__ cols, uint32_t n_cols,
                                                     const uint64_t* __restrict__ lat, const float* __restrict__ loss,
                                                     uint64_t* __restrict__ out_lat, float* __restrict__ out_loss) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t at = (size_t)rows[i] * n_cols + cols[i];
    out_lat[i] = lat[at];
    out_loss[i] = loss[at];
}

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_runahead_setup(shd_ctx* ctx, int32_t dynamic, uint64_t min_possible_latency_ns,
                              uint64_t min_runahead_config_ns) {
    if (!ctx) return SHD_ERR_INVALID;
    uint64_t mp = min_possible_latency_ns;
    if (mp == 0) {   // RoutingInfo::get_smallest_latency_ns of the resident table (manager.rs:246-251)
        if (ctx->t_rows == 0) return SHD_ERR_STATE;
        SHD_HIP(hipSetDevice(ctx->device));
        SHD_TRY(min_u64_device(ctx, ctx->t_lat.as<uint64_t>(), (uint64_t)ctx->t_rows * ctx->t_cols, &mp));
    }
    if (mp == 0) return SHD_ERR_INVALID;   // Runahead::new asserts a non-zero minimum latency
    RoundState& W = ctx->rnd;
    W.dynamic = dynamic != 0;
    W.min_possible = mp;
    W.cfg = min_runahead_config_ns;
    W.min_used = ~0ull;
    W.batch_min_deliver = ~0ull;   // a new run: no relay output is pending
    W.ready = true;
    return SHD_OK;
}

shd_status shd_runahead_get(const shd_ctx* ctx, uint64_t* runahead_ns) {
    if (!ctx || !runahead_ns) return SHD_ERR_INVALID;
    if (!ctx->rnd.ready) return SHD_ERR_STATE;
    *runahead_ns = runahead_of(ctx->rnd);
    return SHD_OK;
}

shd_status shd_window_compute(uint64_t min_next_event_time, uint64_t runahead_ns, uint64_t end_time,
                              uint64_t* window_start, uint64_t* window_end, int32_t* running) {
    if (!window_start || !window_end || !running || runahead_ns == 0) return SHD_ERR_INVALID;
    window_of(min_next_event_time, runahead_ns, end_time, window_start, window_end, running);
    return SHD_OK;
}

shd_status shd_round_window(shd_ctx* ctx, uint64_t cpu_next_event_time, uint64_t end_time,
                            uint64_t* window_start, uint64_t* window_end, int32_t* running) {
    if (!ctx || !window_start || !window_end || !running) return SHD_ERR_INVALID;
    RoundState& W = ctx->rnd;
    // a local failure is carried through the reduction (never a return before it: the peers wait)
    shd_status st = W.ready ? SHD_OK : SHD_ERR_STATE;
    uint64_t m = std::min(cpu_next_event_time, W.batch_min_deliver);
    if (ctx->eq.ready) m = std::min(m, ctx->eq.head);
    if (ctx->comm && ctx->comm->size > 1) {
        SHD_HIP(hipSetDevice(ctx->device));
        Comm& C = *ctx->comm;
        hipStream_t s = ctx->stream;
        // rows of (status, minimum) per rank in comm_scratch (sized by shd_comm_init*)
        uint64_t* w = ctx->comm_scratch.as<uint64_t>();
        ctx->h_pin[46] = (uint64_t)st;
        ctx->h_pin[47] = m;
        if (hipMemcpyAsync(w + 2 * (size_t)C.rank, ctx->h_pin + 46, 16, hipMemcpyHostToDevice, s) != hipSuccess &&
            st == SHD_OK)
            st = SHD_ERR_HIP;
        SHD_TRY(C.all_gather(w + 2 * (size_t)C.rank, w, 16, s));
        std::vector<uint64_t> all(2 * (size_t)C.size);
        SHD_HIP(hipMemcpyAsync(all.data(), w, all.size() * 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < C.size; ++q)
            if ((shd_status)all[2 * q] != SHD_OK) return (shd_status)all[2 * q];
        for (int q = 0; q < C.size; ++q) m = std::min(m, all[2 * q + 1]);
    }
    // Without the device queues the caller took the relay output into its own queues, whose
    // heads it reports in cpu_next_event_time from now on: the output's earliest deliver time
    // counts for this one window (manager.rs:455-464 folds a round's minimum into the next window
    // once), then it is consumed.  With the queues it stays until shd_equeue_advance merges it.
    if (!ctx->eq.ready) W.batch_min_deliver = ~0ull;
    SHD_TRY(st);
    window_of(m, runahead_of(W), end_time, window_start, window_end, running);
    return SHD_OK;
}

shd_status shd_copy_to_host(shd_ctx* ctx, void* dst, const void* d_src, size_t bytes) {
    if (!ctx || (bytes && (!dst || !d_src))) return SHD_ERR_INVALID;
    if (!bytes) return SHD_OK;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_HIP(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

shd_status shd_routing_lookup(shd_ctx* ctx, uint32_t src_row, uint32_t dst_col,
                              uint64_t* latency_ns, float* packet_loss) {
    if (!ctx) return SHD_ERR_INVALID;
    if (ctx->t_rows == 0) return SHD_ERR_STATE;
    if (src_row >= ctx->t_rows || dst_col >= ctx->t_cols) return SHD_ERR_INVALID;
    const size_t i = (size_t)src_row * ctx->t_cols + dst_col;
    if (ctx->h_mirror_lat) {   // host mirror: a plain read, no device round trip
        if (latency_ns) *latency_ns = ctx->h_mirror_lat[i];
        if (packet_loss) *packet_loss = ctx->h_mirror_loss[i];
        return SHD_OK;
    }
    SHD_HIP(hipSetDevice(ctx->device));
    if (latency_ns)
        SHD_HIP(hipMemcpyAsync(latency_ns, ctx->t_lat.as<uint64_t>() + i, 8, hipMemcpyDeviceToHost, ctx->stream));
    if (packet_loss)
        SHD_HIP(hipMemcpyAsync(packet_loss, ctx->t_loss.as<float>() + i, 4, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

shd_status shd_routing_lookup_batch(shd_ctx* ctx, uint64_t n, const uint32_t* src_row, const uint32_t* dst_col,
                                    uint64_t* latency_ns, float* packet_loss) {
    if (!ctx || (n && (!src_row || !dst_col))) return SHD_ERR_INVALID;
    if (ctx->t_rows == 0) return SHD_ERR_STATE;
    for (uint64_t k = 0; k < n; ++k)
        if (src_row[k] >= ctx->t_rows || dst_col[k] >= ctx->t_cols) return SHD_ERR_INVALID;
    if (!n) return SHD_OK;
    if (ctx->h_mirror_lat) {
        for (uint64_t k = 0; k < n; ++k) {
            const size_t i = (size_t)src_row[k] * ctx->t_cols + dst_col[k];
            if (latency_ns) latency_ns[k] = ctx->h_mirror_lat[i];
            if (packet_loss) packet_loss[k] = ctx->h_mirror_loss[i];
        }
        return SHD_OK;
    }
    SHD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    // one scratch: rows, cols (in), lat, loss (out)
    SHD_TRY(ctx->lk_scratch.ensure((size_t)n * 20));
    char* base = ctx->lk_scratch.as<char>();
    uint64_t* d_lat = reinterpret_cast<uint64_t*>(base);
    uint32_t* d_rows = reinterpret_cast<uint32_t*>(base + n * 8);
    uint32_t* d_cols = d_rows + n;
    float* d_loss = reinterpret_cast<float*>(d_cols + n);
    SHD_HIP(hipMemcpyAsync(d_rows, src_row, n * 4, hipMemcpyHostToDevice, s));
    SHD_HIP(hipMemcpyAsync(d_cols, dst_col, n * 4, hipMemcpyHostToDevice, s));
    lookup_gather<<<div_up(n, 256), 256, 0, s>>>(n, d_rows, d_cols, ctx->t_cols, ctx->t_lat.as<uint64_t>(),
                                                  ctx->t_loss.as<float>(), d_lat, d_loss);
    SHD_HIP(hipGetLastError());
    if (latency_ns) SHD_HIP(hipMemcpyAsync(latency_ns, d_lat, n * 8, hipMemcpyDeviceToHost, s));
    if (packet_loss) SHD_HIP(hipMemcpyAsync(packet_loss, d_loss, n * 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

shd_status shd_routing_mirror(shd_ctx* ctx, int32_t enable) {
    if (!ctx) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    drop_mirror(ctx);
    if (!enable) return SHD_OK;
    if (ctx->t_rows == 0) return SHD_ERR_STATE;
    const size_t cells = (size_t)ctx->t_rows * ctx->t_cols;
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_mirror_lat), cells * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&ctx->h_mirror_loss), cells * 4, hipHostMallocDefault) != hipSuccess) {
        drop_mirror(ctx);
        return SHD_ERR_NOMEM;
    }
    hipStream_t s = ctx->stream;
    SHD_HIP(hipMemcpyAsync(ctx->h_mirror_lat, ctx->t_lat.p, cells * 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipMemcpyAsync(ctx->h_mirror_loss, ctx->t_loss.p, cells * 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

}  // extern "C"
