// Multi-GPU transports (comm.h) and the communicator entry points of the C ABI.
//
// The reference has no multi-process or multi-GPU path: its parallelism is worker
// threads over hosts inside one process, with a barrier per round (core/manager.rs:404-464).
// The engine shards along the two seams SURVEY §8(e) names -- routing source rows, relay hosts
// -- and moves the bytes with RCCL over xGMI between one process per GPU, or with device
// copies between ranks that share this process.
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include <rccl/rccl.h>

#include "ctx.h"

namespace shd {

#define SHD_NCCL(call)                                                                    \
    do {                                                                                  \
        ncclResult_t r_ = (call);                                                         \
        if (r_ != ncclSuccess) {                                                          \
            std::fprintf(stderr, "shd_accel: %s failed: %s (%s:%d)\n", #call,             \
                         ncclGetErrorString(r_), __FILE__, __LINE__);                     \
            return SHD_ERR_HIP;                                                           \
        }                                                                                 \
    } while (0)

// ------------------------------------------------------------------------------------ RCCL
struct RcclComm final : Comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    shd_status all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t s) override {
        SHD_NCCL(ncclAllToAll(send, recv, count, ncclUint64, comm, s));
        return SHD_OK;
    }
    shd_status exchange(int n_parts, const void* const* send, const size_t* send_bytes, void* const* recv,
                        const size_t* recv_bytes, hipStream_t s, shd_status local) override {
        // the group is posted whatever happens to the own part: the peers' sends and receives
        // must meet theirs
        shd_status st = local;
        for (int k = 0; k < n_parts; ++k) {   // own part: a device copy
            const size_t i = (size_t)rank * n_parts + k;
            if (send_bytes[i] != recv_bytes[i]) st = SHD_ERR_INVALID;
            else if (send_bytes[i] &&
                     hipMemcpyAsync(recv[i], send[i], send_bytes[i], hipMemcpyDeviceToDevice, s) != hipSuccess)
                st = SHD_ERR_HIP;
        }
        SHD_NCCL(ncclGroupStart());
        for (int r = 0; r < size; ++r) {
            if (r == rank) continue;
            for (int k = 0; k < n_parts; ++k) {
                const size_t i = (size_t)r * n_parts + k;
                if (send_bytes[i]) SHD_NCCL(ncclSend(send[i], send_bytes[i], ncclUint8, r, comm, s));
                if (recv_bytes[i]) SHD_NCCL(ncclRecv(recv[i], recv_bytes[i], ncclUint8, r, comm, s));
            }
        }
        SHD_NCCL(ncclGroupEnd());
        return st;
    }
    shd_status all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        if (bytes) SHD_NCCL(ncclAllGather(send, recv, bytes, ncclUint8, comm, s));
        return SHD_OK;
    }
};

// ------------------------------------------------------------------------------------ local
struct LocalGroup {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<int> device;
    std::vector<const void*> ptr;     // published per rank (exchange: n * n * parts pointers)
    std::vector<size_t> bytes;
    std::vector<int> pre, post;       // per rank: status on entry (with its pointers), on exit
    // per rank, on its device: its inputs are complete (recorded on entry) / its pulls are done
    // (recorded on exit); peers order their streams on them instead of the host syncing streams
    std::vector<hipEvent_t> ev_in, ev_out;
    ~LocalGroup() {
        for (auto* v : {&ev_in, &ev_out})
            for (hipEvent_t e : *v)
                if (e) (void)hipEventDestroy(e);
    }
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

struct LocalComm final : Comm {
    std::shared_ptr<LocalGroup> g;
    int device = 0;
    // every collective: the rank's inputs are marked by an event on its stream and its pointers
    // and entry status are published (barrier); each rank's stream waits for a sender's event,
    // then pulls what it receives -- nothing from a rank that entered failed; the exit statuses
    // are agreed (the lowest failing rank's wins, on every rank), and each rank's stream waits
    // for every peer's pulls to finish before anything after the collective can overwrite what
    // the peers read.  No host sync of a stream (round 6: each collective cost two polled stream
    // syncs, ~30 us of idle device apiece -- four of the six host gaps of a world-1 sharded
    // relay round; one rank alone needs no ordering at all).
    shd_status copy(void* dst, const void* src, int src_dev, size_t n, hipStream_t s) {
        if (!n) return SHD_OK;
        const hipError_t e = src_dev == device ? hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s)
                                               : hipMemcpyPeerAsync(dst, device, src, src_dev, n, s);
        return e == hipSuccess ? SHD_OK : SHD_ERR_HIP;
    }
    shd_status enter(hipStream_t s) {
        shd_status st = SHD_OK;
        if (size > 1 && hipEventRecord(g->ev_in[rank], s) != hipSuccess) st = SHD_ERR_HIP;
        g->pre[rank] = (int)st;
        return st;
    }
    // before the first pull from rank q: q's inputs are complete
    shd_status from(int q, hipStream_t s) {
        return q == rank || hipStreamWaitEvent(s, g->ev_in[q], 0) == hipSuccess ? SHD_OK : SHD_ERR_HIP;
    }
    shd_status leave(shd_status st, hipStream_t s) {
        if (size == 1) return st;
        if (hipEventRecord(g->ev_out[rank], s) != hipSuccess && st == SHD_OK) st = SHD_ERR_HIP;
        g->barrier();   // every rank's pulls are enqueued and marked
        for (int q = 0; q < size; ++q)
            if (q != rank && hipStreamWaitEvent(s, g->ev_out[q], 0) != hipSuccess && st == SHD_OK) st = SHD_ERR_HIP;
        g->post[rank] = (int)st;
        g->barrier();
        shd_status all = SHD_OK;
        for (int q = 0; q < size && all == SHD_OK; ++q) all = (shd_status)g->post[q];
        g->barrier();   // every rank has read the statuses and enqueued its waits before the next collective
        return all;
    }
    shd_status all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t s) override {
        shd_status st = enter(s);
        g->ptr[rank] = send;
        g->barrier();
        for (int q = 0; q < size && st == SHD_OK; ++q) {
            st = g->pre[q] != SHD_OK ? (shd_status)g->pre[q] : from(q, s);
            if (st == SHD_OK)
                st = copy(recv + (size_t)q * count, static_cast<const uint64_t*>(g->ptr[q]) + (size_t)rank * count,
                          g->device[q], count * 8, s);
        }
        return leave(st, s);
    }
    shd_status exchange(int n_parts, const void* const* send, const size_t* send_bytes, void* const* recv,
                        const size_t* recv_bytes, hipStream_t s, shd_status local) override {
        // (a caller's own failure enters as this rank's status: the peers skip its parts)
        shd_status st = n_parts < 1 || n_parts > 4 ? SHD_ERR_INVALID : local;   // the group's pointer slots
        const shd_status e0 = enter(s);
        if (st == SHD_OK) st = e0;
        else g->pre[rank] = (int)st;
        const size_t per_rank = (size_t)size * n_parts;
        if (st == SHD_OK)
            for (size_t i = 0; i < per_rank; ++i) {
                g->ptr[rank * per_rank + i] = send[i];
                g->bytes[rank * per_rank + i] = send_bytes[i];
            }
        g->barrier();
        for (int q = 0; q < size && st == SHD_OK; ++q) {
            if (g->pre[q] != SHD_OK) {
                st = (shd_status)g->pre[q];
                break;
            }
            st = from(q, s);
            for (int k = 0; k < n_parts && st == SHD_OK; ++k) {
                const size_t at = (size_t)q * per_rank + (size_t)rank * n_parts + k;   // q's part k to me
                const size_t to = (size_t)q * n_parts + k;
                if (g->bytes[at] != recv_bytes[to]) st = SHD_ERR_INVALID;
                else st = copy(recv[to], g->ptr[at], g->device[q], recv_bytes[to], s);
            }
        }
        return leave(st, s);
    }
    shd_status all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        shd_status st = enter(s);
        g->ptr[rank] = send;
        g->barrier();
        for (int q = 0; q < size && st == SHD_OK; ++q) {
            char* dst = static_cast<char*>(recv) + (size_t)q * bytes;
            if (g->pre[q] != SHD_OK) st = (shd_status)g->pre[q];
            else if (dst != g->ptr[q] && (st = from(q, s)) == SHD_OK) st = copy(dst, g->ptr[q], g->device[q], bytes, s);
        }
        return leave(st, s);
    }
};

// ------------------------------------------------------------------------------------ host
// The caller's host transport (shd_comm_init_host): ranks are processes the caller already
// connects (MPI, torch.distributed gloo, Shadow's own sockets), one all-to-all-v callback moves
// host bytes between them.  Each collective stages the device bytes through pinned host memory
// (the stream is synchronised before the callback), and every rank's block leads with its entry
// status, so all ranks return the lowest failing rank's status, as under LocalComm.  The same
// sharded code paths run as under RCCL; only the transport differs (and is slower: PCIe both
// ways), which is what a multi-process run on hosts without RCCL peers needs.
struct HostComm final : Comm {
    shd_host_comm_ops ops{};
    unsigned char* hs = nullptr;   // pinned staging: the blocks sent
    unsigned char* hr = nullptr;   // and received
    size_t hs_cap = 0, hr_cap = 0;
    std::vector<uint64_t> st_s, st_r, st_b, st_o;   // the staging status round (sized at init)
    const Knobs* kn = nullptr;                     // its context's knobs (fault injection)
    ~HostComm() override {
        if (hs) (void)hipHostFree(hs);
        if (hr) (void)hipHostFree(hr);
    }
    static shd_status grow(unsigned char*& p, size_t& cap, size_t n) {
        if (n <= cap) return SHD_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), n) != hipSuccess) return SHD_ERR_NOMEM;
        cap = n;
        return SHD_OK;
    }
    // One collective: the block to rank r is 8 status bytes + the parts src[r][k] (device, sizes
    // sb[r][k]), its host image at send offset so[r] (blocks may share an offset: the same bytes
    // to every rank); the block from rank q lands at its receive offset and its parts go to
    // dst[q][k] (sizes rb[q][k]).  The own rank's parts are copied on the device.
    shd_status run(int n_parts, const std::vector<const void*>& src, const std::vector<size_t>& sb,
                   const std::vector<size_t>& so, const std::vector<void*>& dst, const std::vector<size_t>& rb,
                   hipStream_t s, shd_status st) {
        const int n = size;
        std::vector<uint64_t> s_bytes(n), s_off(n), r_bytes(n), r_off(n);
        size_t s_end = 0, r_end = 0;
        for (int r = 0; r < n; ++r) {
            size_t t = 8;
            if (r != rank)
                for (int k = 0; k < n_parts; ++k) t += sb[(size_t)r * n_parts + k];
            s_bytes[r] = t;
            s_off[r] = so[r];
            s_end = std::max(s_end, so[r] + t);
            size_t u = 8;
            if (r != rank)
                for (int k = 0; k < n_parts; ++k) u += rb[(size_t)r * n_parts + k];
            r_bytes[r] = u;
            r_off[r] = r_end;
            r_end += u;
        }
        // Every rank enters the transport, whatever happens locally: its peers are already
        // blocked in the caller's collective.  Pinned staging that cannot grow falls back to
        // pageable memory for this call.  A rank left with no staging at all cannot send blocks
        // of the agreed sizes, so the allocation's outcome is agreed first, in a status round of
        // its own (8 bytes per rank, buffers allocated when the communicator was made): every
        // rank then either moves the blocks or returns the lowest failing rank's status.
        std::vector<unsigned char> hs_tmp, hr_tmp;
        unsigned char* S = hs;
        unsigned char* Rv = hr;
        shd_status st_mem = SHD_OK;
        try {
            if (kn && kn->get(K_TEST_FAIL, 0) == 3) throw std::bad_alloc();   // (fault injection, tests)
            if (grow(hs, hs_cap, s_end) == SHD_OK) S = hs;
            else { hs_tmp.resize(s_end); S = hs_tmp.data(); }
            if (grow(hr, hr_cap, r_end) == SHD_OK) Rv = hr;
            else { hr_tmp.resize(r_end); Rv = hr_tmp.data(); }
        } catch (...) {
            st_mem = SHD_ERR_NOMEM;
        }
        {
            for (int r = 0; r < n; ++r) {
                st_s[r] = (uint64_t)st_mem;
                st_b[r] = 8;
                st_o[r] = (uint64_t)r * 8;
            }
            if (ops.all_to_allv(ops.user, st_s.data(), st_b.data(), st_o.data(), st_r.data(), st_b.data(),
                                st_o.data()) != 0)
                return SHD_ERR_HIP;
            for (int q = 0; q < n; ++q)
                if ((shd_status)st_r[q] != SHD_OK) return (shd_status)st_r[q];
        }
        for (int r = 0; r < n; ++r) {
            size_t at = so[r] + 8;
            for (int k = 0; k < n_parts; ++k) {
                const size_t i = (size_t)r * n_parts + k;
                if (r == rank) {
                    if (sb[i] != rb[i]) st = SHD_ERR_INVALID;
                    else if (sb[i] && dst[i] != src[i] &&
                             hipMemcpyAsync(dst[i], src[i], sb[i], hipMemcpyDeviceToDevice, s) != hipSuccess)
                        st = SHD_ERR_HIP;
                    continue;
                }
                if (sb[i] && hipMemcpyAsync(S + at, src[i], sb[i], hipMemcpyDeviceToHost, s) != hipSuccess)
                    st = SHD_ERR_HIP;
                at += sb[i];
            }
        }
        if (hipStreamSynchronize(s) != hipSuccess && st == SHD_OK) st = SHD_ERR_HIP;
        for (int r = 0; r < n; ++r) {
            const uint64_t w = (uint64_t)st;
            std::memcpy(S + so[r], &w, 8);   // shared offsets get the same word
        }
        if (ops.all_to_allv(ops.user, S, s_bytes.data(), s_off.data(), Rv, r_bytes.data(), r_off.data()) != 0)
            return SHD_ERR_HIP;   // the transport failed: the caller's to handle, as RCCL's would be
        shd_status all = SHD_OK;
        for (int q = 0; q < n && all == SHD_OK; ++q) {
            uint64_t w = 0;
            std::memcpy(&w, Rv + r_off[q], 8);
            all = (shd_status)w;
        }
        if (all != SHD_OK) return all;
        for (int q = 0; q < n; ++q) {
            if (q == rank) continue;
            size_t at = r_off[q] + 8;
            for (int k = 0; k < n_parts; ++k) {
                const size_t i = (size_t)q * n_parts + k;
                if (rb[i] && hipMemcpyAsync(dst[i], Rv + at, rb[i], hipMemcpyHostToDevice, s) != hipSuccess)
                    all = SHD_ERR_HIP;
                at += rb[i];
            }
        }
        if (hipStreamSynchronize(s) != hipSuccess && all == SHD_OK) all = SHD_ERR_HIP;   // staging reused next call
        return all;
    }
    shd_status all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t s) override {
        std::vector<const void*> src(size);
        std::vector<void*> dst(size);
        std::vector<size_t> sb(size, count * 8), rb(size, count * 8), so(size);
        size_t off = 0;
        for (int r = 0; r < size; ++r) {
            src[r] = send + (size_t)r * count;
            dst[r] = recv + (size_t)r * count;
            so[r] = off;
            off += 8 + (r == rank ? 0 : count * 8);
        }
        return run(1, src, sb, so, dst, rb, s, SHD_OK);
    }
    shd_status exchange(int n_parts, const void* const* send, const size_t* send_bytes, void* const* recv,
                        const size_t* recv_bytes, hipStream_t s, shd_status local) override {
        if (n_parts < 1) return SHD_ERR_INVALID;
        const size_t m = (size_t)size * n_parts;
        std::vector<const void*> src(send, send + m);
        std::vector<void*> dst(recv, recv + m);
        std::vector<size_t> sb(send_bytes, send_bytes + m), rb(recv_bytes, recv_bytes + m), so(size);
        size_t off = 0;
        for (int r = 0; r < size; ++r) {
            so[r] = off;
            off += 8;
            if (r != rank)
                for (int k = 0; k < n_parts; ++k) off += sb[(size_t)r * n_parts + k];
        }
        return run(n_parts, src, sb, so, dst, rb, s, local);
    }
    shd_status all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
        // one staged block (status + bytes) sent to every peer: every send offset is 0
        std::vector<const void*> src(size, send);
        std::vector<void*> dst(size);
        std::vector<size_t> sb(size, bytes), rb(size, bytes), so(size, 0);
        for (int r = 0; r < size; ++r) dst[r] = static_cast<char*>(recv) + (size_t)r * bytes;
        // (run() stages the part for every peer at the shared offset 8: the same bytes each time)
        return run(1, src, sb, so, dst, rb, s, SHD_OK);
    }
};

}  // namespace shd

using namespace shd;

extern "C" {

shd_status shd_comm_unique_id(uint8_t* id) {
    if (!id) return SHD_ERR_INVALID;
    ncclUniqueId u;
    SHD_NCCL(ncclGetUniqueId(&u));
    static_assert(sizeof(u) == SHD_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, &u, sizeof(u));
    return SHD_OK;
}

shd_status shd_comm_init(shd_ctx* ctx, int32_t n_ranks, int32_t rank, const uint8_t* id) {
    if (!ctx || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    auto c = std::unique_ptr<RcclComm>(new (std::nothrow) RcclComm());
    if (!c) return SHD_ERR_NOMEM;
    // the sharded calls' status-agreement words: sized here, so no rank can fail to allocate them
    // between two collectives
    SHD_TRY(ctx->comm_scratch.ensure(comm_scratch_bytes(n_ranks)));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    SHD_NCCL(ncclCommInitRank(&c->comm, n_ranks, u, rank));
    c->rank = rank;
    c->size = n_ranks;
    ctx->comm = std::move(c);
    ctx->relay.ready = false;   // the relay's source shard follows the communicator: set up again
    ctx->eq.ready = false;      // so do the queues' destination shard
    return SHD_OK;
}

shd_status shd_comm_init_local(shd_ctx** ctxs, int32_t n_ranks) {
    if (!ctxs || n_ranks < 1) return SHD_ERR_INVALID;
    for (int r = 0; r < n_ranks; ++r)
        if (!ctxs[r]) return SHD_ERR_INVALID;
    for (int r = 0; r < n_ranks; ++r) {
        SHD_HIP(hipSetDevice(ctxs[r]->device));
        SHD_TRY(ctxs[r]->comm_scratch.ensure(comm_scratch_bytes(n_ranks)));
    }
    auto g = std::make_shared<LocalGroup>();
    g->n = n_ranks;
    g->device.resize(n_ranks);
    const size_t slots = (size_t)n_ranks * n_ranks * 4;   // exchange: up to 4 parts per peer
    g->ptr.assign(slots, nullptr);
    g->bytes.assign(slots, 0);
    g->pre.assign(n_ranks, 0);
    g->post.assign(n_ranks, 0);
    g->ev_in.assign(n_ranks, nullptr);
    g->ev_out.assign(n_ranks, nullptr);
    for (int r = 0; r < n_ranks; ++r) {
        g->device[r] = ctxs[r]->device;
        SHD_HIP(hipSetDevice(ctxs[r]->device));
        SHD_HIP(hipEventCreateWithFlags(&g->ev_in[r], hipEventDisableTiming));
        SHD_HIP(hipEventCreateWithFlags(&g->ev_out[r], hipEventDisableTiming));
    }
    for (int r = 0; r < n_ranks; ++r) {
        auto c = std::unique_ptr<LocalComm>(new (std::nothrow) LocalComm());
        if (!c) return SHD_ERR_NOMEM;
        c->g = g;
        c->device = ctxs[r]->device;
        c->rank = r;
        c->size = n_ranks;
        ctxs[r]->comm = std::move(c);
        ctxs[r]->relay.ready = false;
        ctxs[r]->eq.ready = false;
    }
    return SHD_OK;
}

shd_status shd_comm_init_host(shd_ctx* ctx, int32_t n_ranks, int32_t rank, const shd_host_comm_ops* ops) {
    if (!ctx || !ops || !ops->all_to_allv || n_ranks < 1 || rank < 0 || rank >= n_ranks) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    auto c = std::unique_ptr<HostComm>(new (std::nothrow) HostComm());
    if (!c) return SHD_ERR_NOMEM;
    SHD_TRY(ctx->comm_scratch.ensure(comm_scratch_bytes(n_ranks)));
    c->ops = *ops;
    c->rank = rank;
    c->size = n_ranks;
    c->kn = &ctx->knobs;
    try {
        for (auto* v : {&c->st_s, &c->st_r, &c->st_b, &c->st_o}) v->resize((size_t)n_ranks);
    } catch (...) {
        return SHD_ERR_NOMEM;
    }
    ctx->comm = std::move(c);
    ctx->relay.ready = false;
    ctx->eq.ready = false;
    return SHD_OK;
}

shd_status shd_comm_info(const shd_ctx* ctx, int32_t* n_ranks, int32_t* rank) {
    if (!ctx) return SHD_ERR_INVALID;
    if (n_ranks) *n_ranks = ctx->comm ? ctx->comm->size : 1;
    if (rank) *rank = ctx->comm ? ctx->comm->rank : 0;
    return SHD_OK;
}

shd_status shd_comm_destroy(shd_ctx* ctx) {
    if (!ctx) return SHD_ERR_INVALID;
    SHD_HIP(hipSetDevice(ctx->device));
    if (ctx->stream) SHD_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->comm && ctx->relay.sharded) ctx->relay.ready = false;
    if (ctx->comm && ctx->comm->size > 1) ctx->eq.ready = false;
    ctx->comm.reset();
    return SHD_OK;
}

shd_status shd_shard_range(uint32_t total, int32_t n_ranks, int32_t rank, uint32_t* lo, uint32_t* hi) {
    if (!lo || !hi || n_ranks < 1 || rank < 0 || rank >= n_ranks) return SHD_ERR_INVALID;
    shard_range(total, n_ranks, rank, lo, hi);
    return SHD_OK;
}

}  // extern "C"
