// Engine context (one per GPU) and grow-only device scratch.
#pragma once
#include <memory>
#include <vector>

#include "comm.h"
#include "common.h"
#include "knobs.h"

namespace shd {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p; bytes = o.bytes;
            o.p = nullptr; o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    shd_status ensure(size_t need) {
        if (need <= bytes) return SHD_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t want = need + need / 8 + 256;
        if (hipMalloc(&p, want) != hipSuccess) return SHD_ERR_NOMEM;
        bytes = want;
        return SHD_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct PinBuf {   // grow-only coherent pinned host memory (a kernel's stores reach the host: readback_into)
    void* p = nullptr;
    size_t bytes = 0;
    PinBuf() = default;
    PinBuf(const PinBuf&) = delete;
    PinBuf& operator=(const PinBuf&) = delete;
    ~PinBuf() { if (p) (void)hipHostFree(p); }
    shd_status ensure(size_t need) {
        if (need <= bytes) return SHD_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        if (hipHostMalloc(&p, need, hipHostMallocCoherent) != hipSuccess) return SHD_ERR_NOMEM;
        bytes = need;
        return SHD_OK;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct ScanScratch {   // look-back states of the hand-written scans (scan.h)
    DevBuf state;       // [tiles][2] u64
    uint32_t epoch = 0;
};

struct CodelState {   // CoDel router queues (codel.hip)
    DevBuf st, flags, ring, status;
    uint32_t n_hosts = 0, cap = 0;
    bool ready = false;
};

// Stored runs of the event queues before they are compacted (the limit, SHD_EQ_MAX_RUNS knob,
// may be set lower, down to 2).  Each advance merges one source per run, each compaction half
// the runs: on C5 (24 rounds at the steady ~41M pending events) the advance averaged 0.370 ms
// at 8 runs, 0.359 at 12 and 0.355 at 15 (a compaction every ~3 / ~6 / ~7 rounds against more
// sources in every pass); 12 keeps the count kernel's lanes to 13 of its 16.
#ifndef SHD_EQ_MAX_RUNS
#define SHD_EQ_MAX_RUNS 12   // (tuning builds: tools/build_variant.sh -DSHD_EQ_MAX_RUNS=n, n <= 15)
#endif
constexpr int kEqMaxRuns = SHD_EQ_MAX_RUNS;
constexpr int kEqSlots = kEqMaxRuns + 2;   // + the compaction target + a batch slot handed out for adoption

struct EqRunBuf {   // one stored run of the event queues: a CSR of per-host sorted events
    DevBuf off, deliver, src, seq, tag;
    DevBuf pkt;                 // an adopted relay output keeps ev_pkt: tag = batch << 32 | pkt
    bool has_pkt = false;
    bool fresh = false;         // adopted by the running advance: its cursor is its offsets
    uint64_t batch = 0;
    uint64_t n = 0, left = 0;   // events stored / not yet popped
    bool live = false;
};

struct EqState {   // destination event queues (equeue.hip): a list of sorted runs (one per batch)
    EqRunBuf run[kEqSlots];         // slots
    int lend = -1;                  // the slot handed out by shd_equeue_batch_buffers (not live yet)
    bool fold_next = false;         // the next pass folds a compaction in (the run limit was reached)
    uint64_t lend_cap = 0;          // events the lent slot holds
    uint64_t cap_hint = 0;          // the largest run capacity grown so far (every later growth takes it)
    DevBuf curs[2];                 // [kEqSlots][n_hosts] u32 cursors (first unpopped), double-buffered
    DevBuf bcut;                    // [n_hosts] the batch's first kept event per host
    DevBuf pd, ps, pq, pt;          // the last call's popped events
    DevBuf pop_cnt, keep_cnt, pop_off, next, left;
    DevBuf ranges;                  // [n_hosts][kEqMaxRuns + 1] (cursor, cut) pairs of the last count
    int ccur = 0;
    uint32_t n_hosts = 0;           // queues held here: all hosts, or a sharded rank's [host_lo, host_lo + n_hosts)
    uint32_t host_lo = 0, n_total = 0;
    uint64_t n_pending = 0, n_popped = 0, batches = 0;
    uint64_t head = ~0ull;          // earliest pending deliver time after the last advance (local)
    ScanScratch scan;               // the advance's look-back scans (scan.h)
    bool ready = false;
};

// Runahead (src/main/core/scheduler/runahead.rs:12-115) and the round window
// (controller.rs:86-111) for shd_round_window.
struct RoundState {
    bool ready = false;
    bool dynamic = false;
    uint64_t min_possible = 0, cfg = 0;   // Runahead::min_possible_latency, min_runahead_config (0: None)
    uint64_t min_used = ~0ull;            // Runahead::min_used_latency (UINT64_MAX: None)
    uint64_t batch_min_deliver = ~0ull;   // relay output not yet merged into the queues: its earliest deliver
};

struct TbState {   // token-bucket relays (tbucket.hip)
    DevBuf st, err;
    uint32_t n_relays = 0;
    bool ready = false;
};

struct RelayState {
    bool ready = false;
    uint32_t n_hosts = 0;
    // source hosts this context stamps: all hosts, or (set up under a communicator of > 1
    // ranks) the rank's shard [src_lo, src_lo + n_src), which is also its destination shard
    uint32_t src_lo = 0, n_src = 0;
    bool sharded = false;
    uint32_t n_nodes = 0;
    bool own_table = false;   // table copied by shd_relay_setup (else: routing resident table)
    bool table_narrow = false;  // every path latency < 2^32 ns -> 16-byte event records (v2)
    bool force_v1 = false;      // SHD_RELAY_FORCE_V1=1 (testing)
    bool force_v3 = false;      // SHD_RELAY_FORCE_V3=1 (testing): radix pipeline, not v7
    int last_pipe = 0;          // pipeline of the last round: 1, 3 or 7
    bool count_on = true;       // per-path packet counters (RoutingInfo::increment_packet_count)
    bool last_v2 = false;
    uint64_t seq_bound = 0;     // >= every host's next event id
    uint64_t last_recv = 0;     // events this rank received in the last sharded round
    uint32_t hn_bits = 0, hn_words = 0;   // packed host -> node map (0 bits: not used)
    unsigned long long red_host[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // counts: per-path packet counters over all committed rounds; counts_round: the running
    // round's increments, added to counts only when the round commits (a failed or rerun round
    // leaves counts untouched)
    DevBuf host_node, order, hn_packed, lat, loss, path, rng, next_id, rng2, next_id2, counts,
        counts_round;
    // per-round scratch
    DevBuf pk_off, pk_time, pk_dst, pk_pay, pk_chance, st, ev_key, ev_key2, ev_val, ev_val2,
        ev_deliver, ev_seq, ev_src, ev_pkt, ev_off, dst_cnt, red, rec, brec, tmp, draws,
        bin_cnt, bin_base, bin_lb;
    ScanScratch scan;     // pipeline 1's destination offsets (scan.h)
    ScanScratch col_scan; // pipeline 7's bin bases (bin_col_scan's look-back states)
    DevBuf rs_counts;     // pipeline 3's radix sort: per-tile digit counts
    ScanScratch rs_scan;
    // sharded rounds: packed outgoing events, exchange words, per-peer offset blocks, what was
    // received, and the merged events of this rank's destinations (engine-owned outputs)
    DevBuf x_rec, x_words, x_off, x_roff, x_rrec, m_off, m_deliver, m_src, m_seq, m_pkt;
    uint64_t x_cap = 0;   // events x_rrec and m_* hold (grown with a growth agreement, never between collectives)
    // relay_round_sharded_v7: the senders' bin scans, the sizing summary (+ its pinned copy) and
    // the per-sender receive / packet bases
    DevBuf xs_sc, xs_out, xs_b;
    PinBuf xs_pin;
    // the exchange's status part: [0] this rank's status after the sizing gather (0 unless a local
    // failure is carried), [1 + q] the one rank q sent (its own slot stays 0)
    DevBuf xs_st;
    bool xs_st_dirty = false;
    // shd_relay_flush (flush.hip): the round's draws came from the CPU (top 32 bits in `draws`), the
    // staged runs and records as uploaded, the send permutation (grouped <-> stage order) and the
    // packed outputs
    bool cpu_draws = false;
    // a sharded shd_relay_flush round: event ids leave the device relative to their source host's
    // first id of the round (a receiver does not hold the other ranks' hosts' ids)
    bool rel_ids = false;
    DevBuf fl_goff;   // the flush's grouped offsets over every host (sharded: all ranks' hosts)
    // a one-context flush round: pipeline 7's bin sort writes the compact event records here
    // (fl_direct says it did; the other pipelines leave the arrays for fl_events16)
    DevBuf fl_tab, fl_rstg;   // zero-copy staging: the stage table, each run's stage
    PinBuf fl_tab_pin;
    void* fl_ev_out = nullptr;
    uint32_t fl_b12 = 0;
    bool fl_direct = false;
    DevBuf fl_runh, fl_runc, fl_runo, fl_hrun, fl_hcnt, fl_send, fl_perm, fl_inv, fl_st2, fl_ev16;
};

struct PreparedGraph {
    bool ready = false;
    uint32_t mode = 0, V = 0, n_used = 0;
    bool directed = false, narrow_arcs = false;
    bool dense_rows = false;  // the arc CSR is the complete graph's dense matrix (routing.hip csr_is_dense)
    uint64_t arcs = 0, max_arc_lat = 0, pruned_arcs = 0, tight_arcs = 0;
    uint32_t mean_arc_lat = 1, min_arc_lat = 1;
    bool reordered = false;   // g_offr / g_usedr / g_arc8r / g_aqr hold the locality order
    bool spread = false;      // g_offs / g_useds / g_arc16s hold the wave-spread order (LDS kernel)
    bool used_ident = false;  // used[j] == j for every node (the LDS kernels then skip that gather)
    uint32_t lds_labels = 0;  // how many of the first (highest-degree) nodes keep LDS labels
    std::vector<uint32_t> used, node_ids, es, ed;
    std::vector<uint64_t> el;
    std::vector<float> ep;
    shd_graph view() const {
        shd_graph g{};
        g.n_nodes = V;
        g.n_edges = (uint32_t)es.size();
        g.edge_src = es.data();
        g.edge_dst = ed.data();
        g.edge_latency_ns = el.data();
        g.edge_packet_loss = ep.data();
        g.node_ids = node_ids.data();
        g.directed = directed;
        return g;
    }
};

}  // namespace shd

struct shd_ctx;
namespace shd {
// h_pin words: [0, 3) routing flags, [8, 16) relay reductions, [32, 34) flush checks,
// [48, 48 + 4 + runs + 1) event-queue counts; [80] is the polled marker
constexpr int kPinWords = 88;
constexpr int kPinMarker = 80;
// Wait until everything enqueued on stream s has finished (see api.cpp)
shd_status wait_stream(shd_ctx* ctx, hipStream_t s);
// n_bytes of device words into h_pin[at ...] and wait for the stream (api.cpp)
shd_status readback(shd_ctx* ctx, hipStream_t s, int at, const void* d_src, size_t n_bytes);
// the same into coherent pinned words of the caller's (PinBuf; n_bytes a multiple of 8, 8-aligned)
shd_status readback_into(shd_ctx* ctx, hipStream_t s, const void* d_src, size_t n_bytes, unsigned long long* h_dst);
// poll the pinned marker h_pin[kPinMarker] (zeroed by the caller) that a kernel sets after writing
// its words into pinned memory; falls back to hipStreamSynchronize after 20 ms
shd_status wait_marker(shd_ctx* ctx, hipStream_t s);
// a committed relay round's (all-rank) reductions: the runahead update (runahead.rs:60-115) and
// the earliest deliver time of the relay output that the queues have not merged yet (rounds.cpp)
void round_note(shd_ctx* ctx, uint64_t min_deliver, uint64_t min_latency);
// free the host mirror of the resident table (it follows the table)
void drop_mirror(shd_ctx* ctx);
}  // namespace shd

struct shd_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipEvent_t ev[8] = {};
    hipStream_t side = nullptr;        // second stream: work that overlaps the main stream's
    hipEvent_t sev[2] = {};            // fork / join events (no timing)
    unsigned long long* h_pin = nullptr;   // shd::kPinWords pinned host words: flag / reduction read-backs
    shd::DevBuf g_one;                     // a device word holding 1 (shd::wait_stream's marker)
    bool spin_wait = true;                 // SHD_SPIN_WAIT=0: hipStreamSynchronize instead
    shd::Knobs knobs;                      // tuning / testing knobs (knobs.h), from the env at shd_open
    int n_cu = 0;
    size_t max_lds = 0;

    // resident routing table of the last build: rows [row_begin, row_begin+rows) x cols
    shd::DevBuf t_lat, t_loss;
    uint32_t t_rows = 0, t_cols = 0, t_row_begin = 0;
    bool t_full = false;
    uint64_t* h_mirror_lat = nullptr;   // pinned host copy of the resident table (shd_routing_mirror)
    float* h_mirror_loss = nullptr;
    shd::DevBuf lk_scratch;             // shd_routing_lookup_batch
    shd_routing_info info{};
    uint32_t time_every = 1, time_calls = 0;   // shd_routing_set_timing
    bool time_now = true;                      // this build records ev[2] / ev[3]
    bool stats_on = false;   // SHD_SSSP_STATS=1: count expansions / sweeps (tuning only)

    shd::PreparedGraph prep;
    shd::DevBuf d_es, d_ed, d_el, d_ep, d_col;   // direct mode edge arrays
    // routing scratch
    shd::DevBuf g_off, g_dst, g_lat, g_q, g_lat64, g_used, g_diag_lat, g_diag_loss, g_flags,
        g_dense, g_prune_dst, g_prune_cnt, g_labels, g_aux, g_arc16, g_arc8, g_aq, g_fw, g_glab, g_pred,
        g_offr, g_usedr, g_arc8r, g_aqr,   // locality-ordered copies (global-label kernel)
        g_offs, g_useds, g_arc16s;         // wave-spread copies (1024-thread LDS kernel)
    uint32_t* nh_out = nullptr;   // next-hop rows of the running build (shd_routing_run_next_hops)
    // global-label slots left unlaunched while a sharded build's previous chunk is still being
    // exchanged on the side stream: the persistent kernel fills every CU's LDS, so RCCL's
    // send/recv workgroups would otherwise wait for it to finish (shd_routing_run_sharded)
    uint32_t slot_reserve = 0;

    std::unique_ptr<shd::Comm> comm;   // multi-GPU communicator (shd_comm_init*), or none
    shd::DevBuf comm_scratch;

    shd::RelayState relay;
    shd::EqState eq;
    shd::RoundState rnd;
    shd::CodelState codel;
    shd::TbState tb;
};
