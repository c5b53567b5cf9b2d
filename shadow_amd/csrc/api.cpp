// C ABI entry points (include/shd_accel.h): context lifetime, routing build front ends,
// resident-table lookups.  The relay entry points live in relay.hip.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <vector>

#include "ctx.h"

namespace shd {
shd_status routing_prepare_impl(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                                uint32_t n_used, uint32_t mode, shd_error* err);
shd_status routing_run_impl(shd_ctx* ctx, uint32_t algo, uint32_t rb, uint32_t re,
                            uint64_t* d_lat, float* d_loss, shd_error* err);
shd_status min_u64_device(shd_ctx* ctx, const uint64_t* d, uint64_t n, uint64_t* out);
}  // namespace shd

using namespace shd;

// The resident table is about to be rebuilt or replaced: nothing may keep reading it.  A relay
// set up on the resident table (shd_relay_setup with NULL tables) must be set up again.
namespace shd {
void drop_mirror(shd_ctx* ctx) {
    if (ctx->h_mirror_lat) (void)hipHostFree(ctx->h_mirror_lat);
    if (ctx->h_mirror_loss) (void)hipHostFree(ctx->h_mirror_loss);
    ctx->h_mirror_lat = nullptr;
    ctx->h_mirror_loss = nullptr;
}
}  // namespace shd

static void drop_resident_table(shd_ctx* ctx) {
    drop_mirror(ctx);
    ctx->t_rows = 0;
    ctx->t_full = false;
    if (ctx->relay.ready && !ctx->relay.own_table) ctx->relay.ready = false;
}

namespace shd {
// Wait for the stream by polling a pinned host word that a marker kernel (or copy), enqueued
// behind the work, sets to 1: the marker lands when every earlier operation on the stream has completed
// (streams run in order), and the host sees it within a few hundred ns, while
// hipStreamSynchronize's wake-up costs several us on every synchronous call (the C2 build
// is ~0.1 ms).  A wait longer than 20 ms (long kernels, or a fault that stops the queue) falls
// back to hipStreamSynchronize, which also reports a failed kernel.
shd_status readback_launch(hipStream_t s, const void* d_src, uint32_t n_words, unsigned long long* h_dst,
                           unsigned long long* h_marker);
shd_status wait_stream(shd_ctx* ctx, hipStream_t s) {
    if (!ctx->spin_wait) {
        SHD_HIP(hipStreamSynchronize(s));
        return SHD_OK;
    }
    volatile unsigned long long* done = ctx->h_pin + kPinMarker;
    *done = 0;
    // the marker from a one-wave kernel (readback_mark, no words): a D2H copy of it goes through
    // the runtime's blit kernel and left ~30 us of idle device before it (round-6 trace)
    if (ctx->knobs.get(K_SYNC_KERNEL, 1) != 0) {
        SHD_TRY(readback_launch(s, nullptr, 0, nullptr, const_cast<unsigned long long*>(done)));
        return wait_marker(ctx, s);
    }
    SHD_HIP(hipMemcpyAsync(const_cast<unsigned long long*>(done), ctx->g_one.p, 8, hipMemcpyDeviceToHost, s));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; *done != 1; ++i) {
        __builtin_ia32_pause();
        if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    if (*done != 1) SHD_HIP(hipStreamSynchronize(s));
    return SHD_OK;
}

// n_bytes (a multiple of 8) from device memory into the pinned words h_pin[at ...], and wait for
// everything before it on stream s: one kernel writes the words and then the marker the host polls
// (rounds.hip readback_mark), or -- SHD_SYNC_KERNEL=0 -- a D2H copy followed by wait_stream's marker
// copy.  A wait past 20 ms falls back to hipStreamSynchronize, which also reports a failed kernel.
shd_status readback(shd_ctx* ctx, hipStream_t s, int at, const void* d_src, size_t n_bytes) {
    return readback_into(ctx, s, d_src, n_bytes, ctx->h_pin + at);
}

// readback into any coherent pinned host words (PinBuf)
shd_status readback_into(shd_ctx* ctx, hipStream_t s, const void* d_src, size_t n_bytes, unsigned long long* h_dst) {
    if (!ctx->spin_wait || ctx->knobs.get(K_SYNC_KERNEL, 1) == 0) {
        SHD_HIP(hipMemcpyAsync(h_dst, d_src, n_bytes, hipMemcpyDeviceToHost, s));
        return wait_stream(ctx, s);
    }
    volatile unsigned long long* done = ctx->h_pin + kPinMarker;
    *done = 0;
    SHD_TRY(readback_launch(s, d_src, (uint32_t)(n_bytes / 8), h_dst, const_cast<unsigned long long*>(done)));
    return wait_marker(ctx, s);
}

// the polled wait of readback_into, for kernels that write their words and the marker themselves
// (the caller zeroes the marker before launching them)
shd_status wait_marker(shd_ctx* ctx, hipStream_t s) {
    volatile unsigned long long* done = ctx->h_pin + kPinMarker;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; *done != 1; ++i) {
        __builtin_ia32_pause();
        if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    if (*done != 1) SHD_HIP(hipStreamSynchronize(s));
    std::atomic_thread_fence(std::memory_order_acquire);
    return SHD_OK;
}
}  // namespace shd

extern "C" {

const char* shd_version(void) { return "shd_accel 0.1 (gfx950)"; }

const char* shd_status_str(shd_status st) {
    switch (st) {
        case SHD_OK: return "ok";
        case SHD_ERR_NO_EDGE: return "no edge connecting nodes";
        case SHD_ERR_MULTI_EDGE: return "more than one edge connecting nodes";
        case SHD_ERR_UNREACHABLE: return "node pair unreachable";
        case SHD_ERR_LATENCY_OVERFLOW: return "path latency overflows u64 ns";
        case SHD_ERR_INVALID: return "invalid argument";
        case SHD_ERR_HIP: return "HIP runtime error";
        case SHD_ERR_NOMEM: return "out of memory";
        case SHD_ERR_NO_HOST: return "no host ID for dest address";
        case SHD_ERR_STATE: return "invalid call order";
    }
    return "unknown";
}

shd_ctx* shd_open(int device_ordinal, shd_status* st) {
    auto fail = [&](shd_status s) -> shd_ctx* {
        if (st) *st = s;
        return nullptr;
    };
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(SHD_ERR_HIP);
    if (device_ordinal < 0 || device_ordinal >= n) return fail(SHD_ERR_INVALID);
    if (hipSetDevice(device_ordinal) != hipSuccess) return fail(SHD_ERR_HIP);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device_ordinal) != hipSuccess) return fail(SHD_ERR_HIP);
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        std::fprintf(stderr, "shd_accel: device %d is %s, this build targets gfx950 only\n",
                     device_ordinal, prop.gcnArchName);
        return fail(SHD_ERR_HIP);
    }
    shd_ctx* ctx = new (std::nothrow) shd_ctx();
    if (!ctx) return fail(SHD_ERR_NOMEM);
    ctx->device = device_ordinal;
    ctx->n_cu = prop.multiProcessorCount;
    ctx->max_lds = prop.sharedMemPerBlock;
    // every knob is read from the environment here, once (knobs.h); shd_set_knob changes them later
    ctx->knobs.from_env();
    ctx->stats_on = ctx->knobs.on(K_SSSP_STATS);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(SHD_ERR_HIP);
    }
    ctx->own_stream = true;
    // coherent (fine-grained) pinned words: readback_mark's stores reach the host without a cache
    if (hipHostMalloc(reinterpret_cast<void**>(&ctx->h_pin), shd::kPinWords * sizeof(unsigned long long),
                      hipHostMallocCoherent) != hipSuccess) {
        ctx->h_pin = nullptr;
        shd_close(ctx);
        return fail(SHD_ERR_HIP);
    }
    {   // the device word the polled waits copy back (shd::wait_stream)
        const unsigned long long one = 1;
        if (ctx->g_one.ensure(8) != SHD_OK ||
            hipMemcpy(ctx->g_one.p, &one, 8, hipMemcpyHostToDevice) != hipSuccess) {
            shd_close(ctx);
            return fail(SHD_ERR_HIP);
        }
        ctx->spin_wait = ctx->knobs.get(K_SPIN_WAIT, 1) != 0;
    }
    // timing-only events: no system-scope fence (cache writeback + invalidate) when recorded --
    // with it each event cost ~5 us of queue gap beside C2's ~80 us kernel
    for (auto& e : ctx->ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
            shd_close(ctx);
            return fail(SHD_ERR_HIP);
        }
    for (auto& e : ctx->sev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            shd_close(ctx);
            return fail(SHD_ERR_HIP);
        }
    if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) {
        ctx->side = nullptr;
        shd_close(ctx);
        return fail(SHD_ERR_HIP);
    }
    if (st) *st = SHD_OK;
    return ctx;
}

void shd_close(shd_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    for (auto& e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : ctx->sev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    drop_mirror(ctx);
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;  // DevBuf destructors free device memory
}

shd_status shd_set_stream(shd_ctx* ctx, void* hip_stream) {
    if (!ctx) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    if (ctx->own_stream && ctx->stream) {
        SHD_HIP(hipStreamSynchronize(ctx->stream));
        SHD_HIP(hipStreamDestroy(ctx->stream));
    }
    if (hip_stream) {
        ctx->stream = static_cast<hipStream_t>(hip_stream);
        ctx->own_stream = false;
    } else {
        SHD_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
    }
    return SHD_OK;
}

shd_status shd_routing_build_device(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                                    uint32_t n_used, uint32_t mode, uint32_t algo,
                                    uint32_t row_begin, uint32_t row_end, uint64_t* d_lat_out,
                                    float* d_loss_out, shd_error* err) {
    if (!ctx || !d_lat_out || !d_loss_out) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    SHD_TRY(routing_prepare_impl(ctx, g, used, n_used, mode, err));
    return routing_run_impl(ctx, algo, row_begin, row_end, d_lat_out, d_loss_out, err);
}

shd_status shd_routing_prepare(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                               uint32_t n_used, uint32_t mode, shd_error* err) {
    if (!ctx) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    drop_resident_table(ctx);
    return routing_prepare_impl(ctx, g, used, n_used, mode, err);
}

shd_status shd_routing_run(shd_ctx* ctx, uint32_t algo, uint32_t row_begin, uint32_t row_end,
                           uint64_t* d_lat_out, float* d_loss_out, shd_error* err) {
    if (!ctx) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    if (!ctx->prep.ready) return SHD_ERR_STATE;
    const uint32_t n = ctx->prep.n_used;
    const uint32_t re = row_end ? row_end : n;
    if (row_begin >= re || re > n) return SHD_ERR_INVALID;
    if ((d_lat_out == nullptr) != (d_loss_out == nullptr)) return SHD_ERR_INVALID;
    if (!d_lat_out) {  // into the context's resident table
        const size_t cells = (size_t)(re - row_begin) * n;
        drop_resident_table(ctx);
        SHD_TRY(ctx->t_lat.ensure(cells * 8));
        SHD_TRY(ctx->t_loss.ensure(cells * 4));
        SHD_TRY(routing_run_impl(ctx, algo, row_begin, re, ctx->t_lat.as<uint64_t>(),
                                 ctx->t_loss.as<float>(), err));
        ctx->t_rows = re - row_begin;
        ctx->t_cols = n;
        ctx->t_row_begin = row_begin;
        ctx->t_full = (row_begin == 0 && re == n);
        return SHD_OK;
    }
    return routing_run_impl(ctx, algo, row_begin, re, d_lat_out, d_loss_out, err);
}

shd_status shd_routing_run_next_hops(shd_ctx* ctx, uint32_t algo, uint32_t row_begin, uint32_t row_end,
                                     uint64_t* d_lat_out, float* d_loss_out, uint32_t* d_next_hop,
                                     shd_error* err) {
    if (!ctx || !d_lat_out || !d_loss_out || !d_next_hop) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    if (!ctx->prep.ready) return SHD_ERR_STATE;
    const uint32_t n = ctx->prep.n_used;
    const uint32_t re = row_end ? row_end : n;
    if (row_begin >= re || re > n) return SHD_ERR_INVALID;
    ctx->nh_out = d_next_hop;
    const shd_status st = routing_run_impl(ctx, algo, row_begin, re, d_lat_out, d_loss_out, err);
    ctx->nh_out = nullptr;
    return st;
}

shd_status shd_routing_build(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                             uint32_t n_used, uint32_t mode, uint32_t algo, uint32_t row_begin,
                             uint32_t row_end, uint64_t* lat_out, float* loss_out,
                             shd_error* err) {
    if (!ctx || !used || n_used == 0) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    const uint32_t re = row_end ? row_end : n_used;
    if (row_begin >= re || re > n_used) return SHD_ERR_INVALID;
    const size_t cells = (size_t)(re - row_begin) * n_used;
    drop_resident_table(ctx);
    SHD_TRY(ctx->t_lat.ensure(cells * 8));
    SHD_TRY(ctx->t_loss.ensure(cells * 4));
    SHD_TRY(routing_prepare_impl(ctx, g, used, n_used, mode, err));
    SHD_TRY(routing_run_impl(ctx, algo, row_begin, re, ctx->t_lat.as<uint64_t>(),
                             ctx->t_loss.as<float>(), err));
    ctx->t_rows = re - row_begin;
    ctx->t_cols = n_used;
    ctx->t_row_begin = row_begin;
    ctx->t_full = (row_begin == 0 && re == n_used);
    if (lat_out)
        SHD_HIP(hipMemcpyAsync(lat_out, ctx->t_lat.p, cells * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (loss_out)
        SHD_HIP(hipMemcpyAsync(loss_out, ctx->t_loss.p, cells * 4, hipMemcpyDeviceToHost, ctx->stream));
    SHD_HIP(hipStreamSynchronize(ctx->stream));
    return SHD_OK;
}

// Rows of this rank's shard into its slice of the full (padded) table, then one all-gather:
// the source rows are independent, so the only collective is the final gather.
// Every rank learns every rank's outcome first, so all of them return the same error (the
// lowest rank's: its rows come first, as the reference's first failing pair would).
// Rows per exchange chunk of shd_routing_run_sharded: about 256 MB of table per rank and chunk
// (C4 at 8 ranks: 3.75 GB per rank in ~15 chunks), at least 4 chunks once a rank's share passes
// 256 MB; SHD_SHARD_CHUNK_ROWS overrides (tests use it to exercise the chunked path on small
// graphs).
static uint64_t chunk_rows(const shd_ctx* ctx, uint64_t per, uint64_t row_bytes, int ranks) {
    if (ctx->knobs.set(K_SHARD_CHUNK_ROWS)) return std::max<uint64_t>(1, ctx->knobs.get64(K_SHARD_CHUNK_ROWS, 1));
    if (ranks <= 1 || per * row_bytes <= (256ull << 20)) return per;
    const uint64_t by_size = std::max<uint64_t>(1, (256ull << 20) / std::max<uint64_t>(row_bytes, 1));
    return std::min<uint64_t>(by_size, (per + 3) / 4);
}

shd_status shd_routing_run_sharded(shd_ctx* ctx, uint32_t algo, uint64_t* d_lat_full,
                                   float* d_loss_full, shd_error* err) {
    if (!ctx || !d_lat_full || !d_loss_full) return SHD_ERR_INVALID;
    if (!ctx->comm || !ctx->prep.ready) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    Comm& C = *ctx->comm;
    const uint32_t n = ctx->prep.n_used;
    const uint64_t per = ((uint64_t)n + C.size - 1) / C.size;
    uint32_t rb = 0, re = 0;
    shard_range(n, C.size, C.rank, &rb, &re);
    hipStream_t s = ctx->stream;
    // Large tables (C4: 3.75 GB per rank) move in row chunks: chunk k goes to every peer on the
    // side stream (grouped point-to-point) while chunk k+1 is built, so the exchange hides
    // under the build instead of following it.  Every rank runs every chunk's exchange, also
    // after a failure (its peers wait for it); the lowest failing rank's error is agreed at the
    // end.  Small tables keep one all-gather.
    const uint64_t row_bytes = (uint64_t)n * 12;
    // A small table (C2: 12 MB, built in ~0.13 ms) is built whole on every rank: the exchange
    // (~10 MB over xGMI plus the all-gather's latency) costs more than the rows it would save.
    // Every rank prepared the same graph and gets the same table; the status agreement below
    // still runs, so a failure on one rank (allocation) fails every rank.
    const uint64_t rep_bytes = ctx->knobs.get64(K_SHARD_REPLICATE_MB, 64) << 20;
    const bool replicate = C.size > 1 && (uint64_t)n * row_bytes <= rep_bytes;
    if (replicate) { rb = 0; re = n; }
    const uint64_t want = chunk_rows(ctx, per, row_bytes, C.size);
    const uint32_t cs = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(per, want));
    const uint32_t n_chunks = !replicate && C.size > 1 && cs < per ? (uint32_t)((per + cs - 1) / cs) : 1u;
    shd_error e{SHD_OK, 0, 0};
    shd_status st = SHD_OK;
    const uint32_t reserve = ctx->knobs.get(K_SHARD_RESERVE_SLOTS, 32);
    auto rows_of = [&](int q, uint32_t k) -> uint32_t {   // rank q's rows in chunk k
        uint32_t a = 0, z = 0;
        shard_range(n, C.size, q, &a, &z);
        const uint64_t lo = (uint64_t)k * cs, cnt = z - a;
        return lo >= cnt ? 0u : (uint32_t)std::min<uint64_t>(cs, cnt - lo);
    };
    for (uint32_t k = 0; k < n_chunks; ++k) {
        const uint32_t mine = n_chunks == 1 ? re - rb : rows_of(C.rank, k);
        const uint32_t a = rb + (n_chunks == 1 ? 0u : k * cs);
        const size_t at = replicate ? 0 : ((size_t)C.rank * per + (size_t)(a - rb)) * n;
        // from the second chunk on, the previous chunk's exchange runs beside this build: leave
        // some CUs a free slot for RCCL's workgroups (SHD_SHARD_RESERVE_SLOTS, default 32 of
        // the global-label kernel's 2 per CU)
        ctx->slot_reserve = k > 0 ? reserve : 0u;
        if (mine && st == SHD_OK) st = routing_run_impl(ctx, algo, a, a + mine, d_lat_full + at, d_loss_full + at, &e);
        ctx->slot_reserve = 0;
        if (n_chunks == 1) break;
        // the build of this chunk has completed (routing_run_impl ends with a stream sync)
        std::vector<const void*> sp(4 * (size_t)C.size);
        std::vector<void*> rp(4 * (size_t)C.size);
        std::vector<size_t> sb(4 * (size_t)C.size), rbytes(4 * (size_t)C.size);
        for (int q = 0; q < C.size; ++q) {
            const size_t qat = ((size_t)q * per + (size_t)k * cs) * n;
            const uint32_t theirs = rows_of(q, k);
            sp[2 * q] = d_lat_full + at;
            sp[2 * q + 1] = d_loss_full + at;
            sb[2 * q] = q == C.rank ? 0 : (size_t)mine * n * 8;
            sb[2 * q + 1] = q == C.rank ? 0 : (size_t)mine * n * 4;
            rp[2 * q] = d_lat_full + qat;
            rp[2 * q + 1] = d_loss_full + qat;
            rbytes[2 * q] = q == C.rank ? 0 : (size_t)theirs * n * 8;
            rbytes[2 * q + 1] = q == C.rank ? 0 : (size_t)theirs * n * 4;
        }
        // a failed exchange is carried into the status agreement below, never returned between
        // two collectives (the peers would wait in the next chunk's exchange)
        const shd_status xs = C.exchange(2, sp.data(), sb.data(), rp.data(), rbytes.data(), ctx->side);
        if (xs != SHD_OK && st == SHD_OK) st = xs;
    }
    if (n_chunks > 1 && hipStreamSynchronize(ctx->side) != hipSuccess && st == SHD_OK) st = SHD_ERR_HIP;
    // status agreement (comm_scratch was sized by shd_comm_init*)
    uint64_t* w = ctx->comm_scratch.as<uint64_t>();
    ctx->h_pin[40] = ((uint64_t)(uint32_t)st << 32) | (uint32_t)e.code;
    ctx->h_pin[41] = ((uint64_t)e.node_a << 32) | e.node_b;
    if (hipMemcpyAsync(w + 2 * C.size, ctx->h_pin + 40, 16, hipMemcpyHostToDevice, s) != hipSuccess && st == SHD_OK)
        st = SHD_ERR_HIP;
    SHD_TRY(C.all_gather(w + 2 * C.size, w, 16, s));   // LocalComm agrees; an RCCL failure is fatal
    std::vector<uint64_t> all(2 * (size_t)C.size);
    SHD_HIP(hipMemcpyAsync(all.data(), w, all.size() * 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    for (int r = 0; r < C.size; ++r) {
        const shd_status sr = (shd_status)(uint32_t)(all[2 * r] >> 32);
        if (sr == SHD_OK) continue;
        if (err) *err = shd_error{(int32_t)(uint32_t)all[2 * r], (uint32_t)(all[2 * r + 1] >> 32),
                                  (uint32_t)all[2 * r + 1]};
        return sr;
    }
    if (n_chunks == 1 && !replicate) {
        SHD_TRY(C.all_gather(d_lat_full + (size_t)C.rank * per * n, d_lat_full, per * n * 8, s));
        SHD_TRY(C.all_gather(d_loss_full + (size_t)C.rank * per * n, d_loss_full, per * n * 4, s));
        SHD_HIP(hipStreamSynchronize(s));
    }
    return SHD_OK;
}

shd_status shd_set_knob(shd_ctx* ctx, const char* name, int64_t value) {
    if (!ctx) return SHD_ERR_INVALID;
    const int k = Knobs::find(name);
    if (k < 0) return SHD_ERR_INVALID;
    ctx->knobs.v[k] = value < 0 ? -1 : value;
    ctx->stats_on = ctx->knobs.on(K_SSSP_STATS);
    ctx->spin_wait = ctx->knobs.get(K_SPIN_WAIT, 1) != 0;
    return SHD_OK;
}

shd_status shd_get_knob(const shd_ctx* ctx, const char* name, int64_t* value) {
    if (!ctx || !value) return SHD_ERR_INVALID;
    const int k = Knobs::find(name);
    if (k < 0) return SHD_ERR_INVALID;
    *value = ctx->knobs.v[k];
    return SHD_OK;
}

shd_status shd_routing_set_timing(shd_ctx* ctx, uint32_t every) {
    if (!ctx) return SHD_ERR_INVALID;
    ctx->time_every = every;
    ctx->time_calls = 0;
    return SHD_OK;
}

shd_status shd_routing_last_info(const shd_ctx* ctx, shd_routing_info* info) {
    if (!ctx || !info) return SHD_ERR_INVALID;
    *info = ctx->info;
    return SHD_OK;
}

shd_status shd_routing_smallest_latency(shd_ctx* ctx, uint64_t* latency_ns) {
    if (!ctx || !latency_ns) return SHD_ERR_INVALID;
    if (ctx->t_rows == 0) return SHD_ERR_STATE;
    SHD_HIP(hipSetDevice(ctx->device));
    return min_u64_device(ctx, ctx->t_lat.as<uint64_t>(), (uint64_t)ctx->t_rows * ctx->t_cols,
                          latency_ns);
}

}  // extern "C"
