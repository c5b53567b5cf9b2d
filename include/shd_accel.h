/*
 * shd_accel.h -- C ABI of the MI355X (gfx950) engine for Shadow's two data-parallel paths:
 *
 *   1. the routing build: lexicographic (latency, then packet loss) shortest paths over the
 *      GML network graph into the dense used-node RoutingInfo table, and the direct-path mode;
 *   2. the per-round inter-host packet relay: path latency/loss lookup, seeded per-host loss
 *      draw, delivery-time stamping, and the sort-merge of packet events into destination
 *      hosts' event queues.
 *
 * Plain C types only (no torch / HIP types); caller-owned host buffers unless a function says
 * "device".  No panic or C++ exception crosses this boundary: every entry point returns a
 * shd_status.  One shd_ctx per GPU; a context is not thread-safe (the reference calls the
 * routing build once from the setup thread and flushes the relay once per round from the
 * manager thread).
 *
 * Reference interfaces replaced (FlyearthR/shadow, Shadow 3.0.0):
 *   shd_routing_build      <- NetworkGraph::compute_shortest_paths / get_direct_paths
 *                             (src/main/network/graph/mod.rs:185-254), called from
 *                             generate_routing_info (src/main/core/sim_config.rs:424-461)
 *   shd_routing_lookup     <- RoutingInfo::path (graph/mod.rs:446-448),
 *                             WorkerShared::{latency,reliability} (src/main/core/worker.rs:529-543)
 *   shd_routing_smallest_latency <- RoutingInfo::get_smallest_latency_ns (graph/mod.rs:476-478)
 *   shd_relay_setup        <- WorkerShared tables built in Manager::run (core/manager.rs:309-332)
 *                             + per-host RNG / event-id counter (src/main/host/host.rs:218,580-584)
 *   shd_relay_round        <- the body of Worker::send_packet (src/main/core/worker.rs:328-413)
 *                             for every send of one scheduling round, flushed at the round
 *                             barrier (core/manager.rs:455-464), plus push_packet_to_host /
 *                             EventQueue::push (worker.rs:619-629, core/work/event_queue.rs:28-48)
 *   shd_path_packet_counts <- RoutingInfo::increment_packet_count / log_packet_counts
 *                             (graph/mod.rs:451-474)
 */
#ifndef SHD_ACCEL_H
#define SHD_ACCEL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHD_ABI_VERSION 3

typedef enum shd_status {
    SHD_OK = 0,
    SHD_ERR_NO_EDGE = 1,          /* "No edge connecting node {a} to {b}"      graph/mod.rs:267-270 */
    SHD_ERR_MULTI_EDGE = 2,       /* "More than one edge connecting node .."   graph/mod.rs:271-276 */
    SHD_ERR_UNREACHABLE = 3,      /* reference panics: assert paths.len()==n^2 graph/mod.rs:221 */
    SHD_ERR_LATENCY_OVERFLOW = 4, /* a path latency does not fit u64 ns (reference: overflow panic) */
    SHD_ERR_INVALID = 5,          /* bad argument (null pointer, index out of range, ...)          */
    SHD_ERR_HIP = 6,              /* HIP runtime failure                                           */
    SHD_ERR_NOMEM = 7,            /* host or device allocation failed                              */
    SHD_ERR_NO_HOST = 8,          /* "No host ID for dest address"              worker.rs:350-355 */
    SHD_ERR_STATE = 9             /* call order violated (e.g. relay before setup)                 */
} shd_status;

typedef struct shd_ctx shd_ctx;

/* Error detail; node ids are GML ids (graph/mod.rs:263-264 reports GML ids). */
typedef struct shd_error {
    int32_t code;      /* shd_status */
    uint32_t node_a;
    uint32_t node_b;
} shd_error;

/*
 * Network graph after GML parsing (NetworkGraph, graph/mod.rs:115-183).  Node indices are the
 * petgraph NodeIndex values (= GML node order); edges are in GML order.  edge_latency_ns is
 * ShadowEdge.latency converted to ns (units.rs:377-388), edge_packet_loss the raw f32.
 */
typedef struct shd_graph {
    uint32_t n_nodes;
    uint32_t n_edges;
    const uint32_t* edge_src;        /* node index, [n_edges] */
    const uint32_t* edge_dst;        /* node index, [n_edges] */
    const uint64_t* edge_latency_ns; /* [n_edges], > 0 */
    const float* edge_packet_loss;   /* [n_edges], in [0,1] */
    const uint32_t* node_ids;        /* GML id per node index [n_nodes]; NULL => id == index */
    int32_t directed;                /* GML 'directed' (default 0) */
} shd_graph;

/* Routing modes (network.use_shortest_path, configuration.rs:276; sim_config.rs:442-458). */
#define SHD_ROUTE_SHORTEST 0u
#define SHD_ROUTE_DIRECT 1u

/* Algorithm selection for SHD_ROUTE_SHORTEST (all produce identical bits). */
#define SHD_ALGO_AUTO 0u     /* dense graphs: 2-hop prune + SSSP; sparse: SSSP           */
#define SHD_ALGO_SSSP 1u     /* batched per-source label-correcting SSSP, labels in LDS   */
#define SHD_ALGO_PRUNED 2u   /* dense k-nearest 2-hop edge prune, then SSSP               */
#define SHD_ALGO_DELTA 3u    /* delta-stepping buckets inside the per-source SSSP         */
#define SHD_ALGO_BLOCKED 4u  /* blocked min-plus (Floyd-Warshall) latency + tight-DAG loss */

typedef struct shd_routing_info {
    uint32_t algo_used;        /* SHD_ALGO_* that ran */
    uint32_t wide_latency;     /* 1 if the u64-latency kernels ran (a path >= 2^32-1 ns) */
    uint64_t arcs;             /* arcs after parallel-edge reduction */
    uint64_t arcs_kept;        /* arcs after pruning (== arcs when no prune ran) */
    double ms_total;           /* device time of the last build (HIP events) */
    double ms_main;            /* device time of the dominant kernel; -1 when this call was not
                                  timed (shd_routing_set_timing) */
    double ms_minplus;         /* SHD_ALGO_BLOCKED: device time of the min-plus closure */
} shd_routing_info;

/* ---------------------------------------------------------------- context */
const char* shd_version(void);
const char* shd_status_str(shd_status st);
shd_ctx* shd_open(int device_ordinal, shd_status* st);
void shd_close(shd_ctx* ctx);
/* Stream for all device work of this context (a hipStream_t passed as void*; NULL => the
 * context's own stream).  Lets a caller order the engine behind its own stream. */
shd_status shd_set_stream(shd_ctx* ctx, void* hip_stream);
/* Tuning and testing knobs of this context (no reference counterpart).  No knob changes a result:
 * they pick grids, kernel variants or an equivalent fallback pipeline.  Every knob starts from the
 * environment variable SHD_<name>, read ONCE by shd_open, so the process environment cannot change
 * a context's grids between two calls; shd_set_knob overrides one for this context (value < 0: back
 * to the built-in default), shd_get_knob reads it (-1: the built-in default applies).  `name` is
 * spelled with or without the SHD_ prefix (e.g. "SSSP_SLOTS"); an unknown name is SHD_ERR_INVALID.
 * Relay pipeline knobs (RELAY_FORCE_*, RELAY_NO_LDS_MAP) apply from the next shd_relay_setup. */
shd_status shd_set_knob(shd_ctx* ctx, const char* name, int64_t value);
shd_status shd_get_knob(const shd_ctx* ctx, const char* name, int64_t* value);

/* ---------------------------------------------------------------- routing build */
/*
 * Build rows [row_begin, row_end) of the n_used x n_used table (row-major in `used` order;
 * row_end == 0 means n_used).  lat_out/loss_out receive (row_end-row_begin) * n_used entries;
 * either may be NULL, in which case the table stays only device-resident in the context.
 * Diagonal = the node's single self-loop edge (graph/mod.rs:212-219).  Errors are reported
 * for the whole used set exactly as the reference: missing/multiple self-loop -> NO_EDGE /
 * MULTI_EDGE on the first such node in `used` order; unreachable pair -> UNREACHABLE.
 */
shd_status shd_routing_build(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                             uint32_t n_used, uint32_t mode, uint32_t algo,
                             uint32_t row_begin, uint32_t row_end,
                             uint64_t* lat_out, float* loss_out, shd_error* err);

/*
 * Two-phase form of the same build (what a caller that rebuilds, shards or benchmarks uses):
 * shd_routing_prepare validates the graph and the used set, applies the self-loop rule and
 * uploads the arc CSR (device-resident in the context); shd_routing_run then computes rows
 * [row_begin, row_end) from the resident graph into device buffers on the context's stream
 * (NULL outputs => the context's resident table).  Errors as for shd_routing_build.
 */
shd_status shd_routing_prepare(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                               uint32_t n_used, uint32_t mode, shd_error* err);
shd_status shd_routing_run(shd_ctx* ctx, uint32_t algo, uint32_t row_begin, uint32_t row_end,
                           uint64_t* d_lat_out, float* d_loss_out, shd_error* err);

/*
 * shd_routing_run plus next hops (the north star's; the reference keeps none: petgraph's
 * dijkstra returns scores only, graph/mod.rs:197-200).  Definition, identical for
 * every engine: pred(s, v) = the LOWEST node index u with an arc u -> v (u != v) whose final
 * label extended by that arc equals v's label bit for bit (latency and left-folded loss);
 * next_hop(s, d) = the node after s on d's pred chain, next_hop(s, s) = s (the self-loop), and
 * in direct mode the destination itself.  d_next_hop (device) receives (row_end - row_begin) x
 * n_used node indices (GML order); UINT32_MAX never appears in a successful build.
 */
shd_status shd_routing_run_next_hops(shd_ctx* ctx, uint32_t algo, uint32_t row_begin, uint32_t row_end,
                                     uint64_t* d_lat_out, float* d_loss_out, uint32_t* d_next_hop,
                                     shd_error* err);

/* As shd_routing_build, writing the rows straight into device buffers (hipMalloc'd or torch
 * tensors) on the context's stream; the call returns when the rows are complete. */
shd_status shd_routing_build_device(shd_ctx* ctx, const shd_graph* g, const uint32_t* used,
                                    uint32_t n_used, uint32_t mode, uint32_t algo,
                                    uint32_t row_begin, uint32_t row_end,
                                    uint64_t* d_lat_out, float* d_loss_out, shd_error* err);

shd_status shd_routing_last_info(const shd_ctx* ctx, shd_routing_info* info);

/* Time the dominant kernel on every `every`-th build (default 1 = every build; 0 = never).
 * The duration comes from HIP events recorded with that kernel's dispatch on the context's
 * stream; they cost a few microseconds of queue gap, which a caller timing many builds can
 * spread by sampling. */
shd_status shd_routing_set_timing(shd_ctx* ctx, uint32_t every);

/* Look up one pair of the resident table (row index relative to row_begin of the last build).
 * After shd_routing_mirror the lookup reads the pinned host mirror (no device round trip: what a
 * worker_getLatency-rate caller -- worker.rs:660-670, tcp.c:451-452 -- needs); otherwise it copies
 * the pair from the device. */
shd_status shd_routing_lookup(shd_ctx* ctx, uint32_t src_row, uint32_t dst_col,
                              uint64_t* latency_ns, float* packet_loss);
/* n lookups in one device gather and one copy (host arrays; any output may be NULL). */
shd_status shd_routing_lookup_batch(shd_ctx* ctx, uint64_t n, const uint32_t* src_row, const uint32_t* dst_col,
                                    uint64_t* latency_ns, float* packet_loss);
/* Keep a pinned host copy of the resident table (rows x cols x 12 B) for host-side lookups; it is
 * dropped with the resident table (the next build or prepare).  enable = 0 drops it. */
shd_status shd_routing_mirror(shd_ctx* ctx, int32_t enable);
shd_status shd_routing_smallest_latency(shd_ctx* ctx, uint64_t* latency_ns);

/*
 * assign_ips (src/main/core/sim_config.rs:399-420) with IpAssignment (graph/mod.rs:354-422),
 * host code: hosts in HostId order; ip_in[h] = the host's configured IPv4 address (host byte
 * order, 11.0.0.1 = 0x0B000001) or 0 for none (ip_in may be NULL: no host has one).  Configured
 * addresses are registered first (a repeat is SHD_ERR_INVALID, *err_host = that host: "IP address
 * has already been assigned"); every other host gets the next free address after the last one
 * handed out, from 11.0.0.1 on, skipping x.x.x.0 and x.x.x.255.  ip_out[n_hosts] receives every
 * host's address; used_gml (capacity n_hosts, may be NULL) the ids of the nodes that own an
 * address, ascending (IpAssignment::get_nodes, the `nodes` of generate_routing_info,
 * sim_config.rs:424-461), *n_used their count; host_col (may be NULL) each host's column in
 * that list -- the relay's host -> node map (shd_relay_setup).
 */
shd_status shd_assign_ips(uint32_t n_hosts, const uint32_t* node_gml_id, const uint32_t* ip_in,
                          uint32_t* ip_out, uint32_t* used_gml, uint32_t* n_used, uint32_t* host_col,
                          uint32_t* err_host);

/* ---------------------------------------------------------------- relay */
/*
 * Host tables for the relay: host -> used-node index (IpAssignment + RoutingInfo keys,
 * worker.rs:529-543), the n_nodes x n_nodes table (NULL => the context's resident table from
 * the last full routing build), each host's Xoshiro256++ state (4 x u64, host.rs:218) and next
 * event id (host.rs:580-584).  A relay set up on the resident table stops at the next
 * shd_routing_prepare / shd_routing_build / resident shd_routing_run (relay calls return
 * SHD_ERR_STATE until it is set up again); caller-passed tables are copied and stay valid.
 */
shd_status shd_relay_setup(shd_ctx* ctx, uint32_t n_hosts, const uint32_t* host_node,
                           uint32_t n_nodes, const uint64_t* lat, const float* loss,
                           const uint64_t* rng_state, const uint64_t* next_event_id);

typedef struct shd_round {
    uint64_t round_end;      /* Worker::round_end_time */
    uint64_t sim_end;        /* WorkerShared::sim_end_time */
    uint64_t bootstrap_end;  /* WorkerShared::bootstrap_end_time */
} shd_round;

/*
 * One round's staged sends, grouped by source host: host h's sends are packets
 * [src_off[h], src_off[h+1]) in send order (src_off has n_hosts+1 entries).  chance may be
 * NULL: the engine then draws from the device-resident per-host streams; otherwise chance[i]
 * is the f64 the CPU drew from the host RNG at send time (worker.rs:365).
 */
typedef struct shd_batch {
    uint64_t n_packets;
    const uint32_t* src_off;
    const uint64_t* send_time;   /* emulated ns */
    const uint32_t* dst_host;    /* HostId after DNS resolution (worker.rs:350-355) */
    const uint32_t* payload;     /* packet_getPayloadSize */
    const double* chance;        /* optional */
} shd_batch;

#define SHD_PKT_SKIPPED 0u  /* now >= sim_end: returned before any effect (worker.rs:339-341) */
#define SHD_PKT_DROPPED 1u  /* PDS_INET_DROPPED (worker.rs:370-378) */
#define SHD_PKT_SENT 2u     /* PDS_INET_SENT + event pushed */

/*
 * Outputs (caller-owned host buffers, any may be NULL): status[n_packets]; the round's packet
 * events grouped by destination host in EventQueue pop order (event.rs:84-155):
 * ev_off[n_hosts+1], ev_deliver / ev_src / ev_seq / ev_pkt[n_sent] (ev_pkt = index of the
 * packet in the batch); min_deliver = min over sent deliver times (u64 max if none,
 * worker.rs:406); min_latency = min latency used (runahead.rs:60-115); n_sent.
 */
typedef struct shd_relay_out {
    uint8_t* status;
    uint32_t* ev_off;
    uint64_t* ev_deliver;
    uint32_t* ev_src;
    uint64_t* ev_seq;
    uint32_t* ev_pkt;
    uint64_t min_deliver;
    uint64_t min_latency;
    uint64_t n_sent;
    uint32_t n_dst;      /* destination hosts ev_off covers (ev_off has n_dst + 1 entries) */
    uint32_t n_events;   /* events in ev_* (= ev_off[n_dst]): n_sent on one GPU; a sharded round's
                            n_sent is the all-rank total, n_events what this rank received.  Both
                            are written by the relay calls; a caller building this struct for
                            shd_equeue_advance sets them (the queues check n_dst against their
                            host count and merge n_events events) */
} shd_relay_out;

shd_status shd_relay_round(shd_ctx* ctx, const shd_batch* batch, const shd_round* round,
                           shd_relay_out* out);

/* Device-buffer form (all pointers in shd_batch / shd_relay_out are device pointers; status,
 * ev_* must hold n_packets entries).  Used by the multi-GPU driver and the benchmark. */
shd_status shd_relay_round_device(shd_ctx* ctx, const shd_batch* d_batch, const shd_round* round,
                                  shd_relay_out* d_out);

/* ---------------------------------------------------------------- drop-in flush of staged sends */
/*
 * The round barrier of the drop-in (manager.rs:455-464) without any CPU reorder: the worker threads'
 * staging buffers go to the device as they are.  Each host runs on one worker thread per round
 * (scheduler/thread_per_core.rs:188-206), so its sends form ONE run (host, count) of consecutive
 * records in ONE stage (= one thread's buffer), in send order; stages and runs may come in any
 * order.  A staged send is 12 bytes (worker.rs:328-413 reads nothing else):
 *   time_off  now - time_base (ns; the round's window start is a natural time_base)
 *   dst       destination HostId (resolve_ip_to_host_id, worker.rs:350-355), | SHD_SEND_PAYLOAD
 *             when packet_getPayloadSize > 0 (the drop rule spares empty packets, :370)
 *   draw_hi   the source host's next_u64() >> 32 taken at send time -- in place of gen::<f64>()
 *             (:365), which consumes the same one next_u64, so the CPU stream advances as in the
 *             reference; the top 32 bits decide chance >= reliability exactly
 * The completed check (:334-341) stays on the CPU: staged sends have now < sim_end.
 * Outputs (host buffers; pinned -- shd_host_alloc -- for the link's full rate; any may be NULL):
 *   status2   2-bit SHD_PKT_* per send in stage order (stage 0's sends, then stage 1's, ...):
 *             send i in bits 2(i%4), 2(i%4)+1 of byte i/4; ceil(n/4) bytes
 *   ev_off    [n_hosts + 1]; events[ev_off[h], ev_off[h+1]) are host h's, in EventQueue order
 *   events    n_sent shd_event16 records
 *   seq_base  [n_hosts]: each host's first packet event id of this round (event id = seq_base[src]
 *             + seq_off)
 * Device RNG streams are not used (the draws are the CPU's); event ids, counters and the runahead
 * update as in shd_relay_round.  SHD_ERR_NO_HOST: a run's host or a destination is not a relay
 * host; SHD_ERR_INVALID: a host with two runs, or runs that do not cover a stage's records.
 *
 * Under a communicator of > 1 ranks (shd_relay_setup after it) every rank is handed the SAME
 * stages -- every worker thread's buffer, holding hosts of every shard -- and keeps its own hosts
 * [lo, hi) = shd_shard_range(n_hosts): the device groups every send (one pass, no CPU split), runs
 * its own hosts' sends through shd_relay_round_sharded and returns
 *   status2   every send in stage order: the own hosts' statuses, 0 for the other ranks' sends (an
 *             OR of the ranks' arrays gives every status)
 *   ev_off    [hi - lo + 1]; events: the own destinations' n_events events, seq_off relative to
 *             the source host's first id of the round and send = the index in stage order, for
 *             sources of any rank
 *   seq_base  entries [lo, hi) only (the ranks may share one array)
 *   min_deliver, min_latency, n_sent over all ranks.
 * A failed check (NO_HOST / INVALID runs) returns before the round's collectives on every rank
 * (they all see the same stages); a failure inside the round fails it on every rank.
 */
#define SHD_SEND_PAYLOAD 0x80000000u
typedef struct shd_send12 {
    uint32_t time_off;
    uint32_t dst;
    uint32_t draw_hi;
} shd_send12;

typedef struct shd_stage {
    uint32_t n_runs;
    const uint32_t* run_host;    /* [n_runs] source HostId of each run */
    const uint32_t* run_count;   /* [n_runs] its sends, consecutive in `sends` */
    uint64_t n_sends;
    const shd_send12* sends;     /* [n_sends] */
} shd_stage;

typedef struct shd_event16 {
    uint32_t deliver_off;   /* deliver time - round_end */
    uint32_t src_host;
    uint32_t seq_off;       /* src_host_event_id - seq_base[src_host] */
    uint32_t send;          /* the send's index in stage order */
} shd_event16;

/* 12-byte form (shd_flush_out.event_bytes = 12): the source host is left out -- the caller's
 * packet at index `send` already names it -- so 4 bytes less per event cross PCIe */
typedef struct shd_event12 {
    uint32_t deliver_off;
    uint32_t seq_off;
    uint32_t send;
} shd_event12;

/* Versioned: struct_size must be sizeof(shd_flush_out) as the caller's header declares it (round
 * 5 added n_events and event_bytes at the end; a caller built against that older layout has a
 * pointer here and is refused with SHD_ERR_INVALID instead of having fields read past its object). */
typedef struct shd_flush_out {
    uint32_t struct_size;   /* in: sizeof(shd_flush_out) */
    uint32_t event_bytes;   /* in: 16 (or 0) = shd_event16 records, 12 = shd_event12 records */
    uint8_t* status2;
    uint32_t* ev_off;
    shd_event16* events;        /* shd_event12 records when event_bytes = 12 */
    uint64_t* seq_base;
    uint64_t min_deliver;   /* as shd_relay_out (under a communicator: over all ranks) */
    uint64_t min_latency;
    uint64_t n_sent;
    uint64_t n_events;      /* events returned (= n_sent on one context; the own destinations' events
                               under a communicator) */
} shd_flush_out;

shd_status shd_relay_flush(shd_ctx* ctx, const shd_stage* stages, uint32_t n_stages, uint64_t time_base,
                           const shd_round* round, shd_flush_out* out);
/* Pinned host memory for staging buffers and outputs (hipHostMalloc); NULL on failure. */
void* shd_host_alloc(size_t bytes);
void shd_host_free(void* p);

/* ---------------------------------------------------------------- multi-GPU */
/*
 * The reference is one process whose manager thread runs every round to a barrier
 * (core/manager.rs:404-464); it has no multi-GPU path.  The engine shards the two paths along
 * their natural seams -- routing source rows, relay hosts by id -- over a communicator:
 *   shd_comm_init        one process per GPU, RCCL over xGMI; rank 0 makes the id with
 *                        shd_comm_unique_id and the caller hands it to every rank (MPI, a file,
 *                        torch.distributed ...); collective over the ranks
 *   shd_comm_init_local  every rank in this process (one host thread per rank must then drive
 *                        each sharded call concurrently): device copies between the contexts,
 *                        ordered by HIP events between their streams (no host stream syncs)
 *   shd_comm_init_host   ranks are processes the caller connects itself (MPI, gloo, sockets):
 *                        one all-to-all-v callback moves host bytes; the device bytes are staged
 *                        through pinned host memory around it (slower than RCCL: PCIe both ways)
 * Shards are contiguous blocks of ceil(total / n_ranks) (shd_shard_range).  Initialising or
 * destroying a communicator requires shd_relay_setup again.
 */
#define SHD_COMM_ID_BYTES 128
shd_status shd_comm_unique_id(uint8_t* id /* SHD_COMM_ID_BYTES */);
shd_status shd_comm_init(shd_ctx* ctx, int32_t n_ranks, int32_t rank, const uint8_t* id);
shd_status shd_comm_init_local(shd_ctx** ctxs, int32_t n_ranks);
/* The host transport of shd_comm_init_host.  all_to_allv: every rank calls it together; the
 * send_bytes[r] bytes at send + send_off[r] go to rank r (offsets may repeat: the same bytes to
 * several ranks), the recv_bytes[q] bytes from rank q land at recv + recv_off[q]; host memory,
 * the sizes already agree between the ranks.  Returns 0 on success (anything else fails the
 * call with SHD_ERR_HIP on this rank; the peers are the transport's to release). */
typedef struct shd_host_comm_ops {
    void* user;
    int (*all_to_allv)(void* user, const void* send, const uint64_t* send_bytes, const uint64_t* send_off,
                       void* recv, const uint64_t* recv_bytes, const uint64_t* recv_off);
} shd_host_comm_ops;
shd_status shd_comm_init_host(shd_ctx* ctx, int32_t n_ranks, int32_t rank, const shd_host_comm_ops* ops);
shd_status shd_comm_info(const shd_ctx* ctx, int32_t* n_ranks, int32_t* rank);
shd_status shd_comm_destroy(shd_ctx* ctx);
shd_status shd_shard_range(uint32_t total, int32_t n_ranks, int32_t rank, uint32_t* lo, uint32_t* hi);

/*
 * Routing build over the communicator (after shd_routing_prepare of the same graph on every
 * rank): each rank builds its source rows into its slice of the full table, then one
 * all-gather leaves the whole table on every rank (tables of at most SHD_SHARD_REPLICATE_MB MiB,
 * default 64, are instead built whole on every rank: no exchange; shares above 256 MB per rank
 * are exchanged in row chunks overlapping the build).  d_lat_full / d_loss_full are device buffers
 * of n_ranks * ceil(n_used / n_ranks) rows of n_used (rows >= n_used are padding).  Every rank
 * returns the same status: the lowest failing rank's error.  Replaces the rayon fan-out of
 * compute_shortest_paths (graph/mod.rs:192-210) across GPUs.
 */
shd_status shd_routing_run_sharded(shd_ctx* ctx, uint32_t algo, uint64_t* d_lat_full,
                                   float* d_loss_full, shd_error* err);

/*
 * One relay round over the communicator.  shd_relay_setup (after the communicator, same
 * arguments on every rank) makes this rank own hosts [lo, hi) = shd_shard_range(n_hosts):
 * their RNG streams, event ids and destination events.  d_batch holds the sends of the own
 * hosts only (src_off has hi - lo + 1 entries; host lo + k's sends are [src_off[k],
 * src_off[k+1])); d_out->status (device, n_packets) receives their statuses.  The round's
 * events for the own destinations come back in engine-owned device arrays, valid until the next
 * round: d_out->ev_off[hi - lo + 1] and ev_deliver / ev_src / ev_seq / ev_pkt (ev_pkt = the
 * packet's index in its sender rank's batch; the sender rank owns ev_src).  min_deliver,
 * min_latency and n_sent are reduced over all ranks.  A round that fails on any rank fails on
 * every rank with that rank's status and commits no host state anywhere.
 */
shd_status shd_relay_round_sharded(shd_ctx* ctx, const shd_batch* d_batch, const shd_round* round,
                                   shd_relay_out* d_out);

/* ---------------------------------------------------------------- destination event queues */
/*
 * Device-resident packet-event queues of this context's destination hosts:
 * WorkerShared::push_packet_to_host / EventQueue::push (worker.rs:619-629,
 * event_queue.rs:28-48) and the pop loop of Host::execute (host.rs:697-706) for packet events.
 * shd_equeue_advance merges a round's events (a relay output on the device, NULL for none) into
 * the pending queues and pops, per host, every event with deliver < window_end in EventQueue
 * order (time, src host, src event id; event.rs:84-155); later events stay pending for later
 * rounds.  The popped events are in engine-owned device arrays valid until the next advance.
 * tag = (number of the batch that carried the event << 32) | its ev_pkt in that batch.
 */
typedef struct shd_equeue_out {
    const uint32_t* off;        /* device [n_hosts + 1]: host h's events are [off[h], off[h+1]) */
    const uint64_t* deliver;    /* device [n_popped] */
    const uint32_t* src;
    const uint64_t* seq;
    const uint64_t* tag;
    uint64_t n_popped;
    uint64_t n_pending;         /* events left in the queues */
    uint64_t next_time;         /* earliest pending deliver time (EventQueue::next_event_time
                                   minimum over the hosts); UINT64_MAX when none is left */
} shd_equeue_out;

/* n_hosts = all hosts.  Under a communicator of > 1 ranks the queues hold this rank's destination
 * shard [lo, hi) = shd_shard_range(n_hosts) -- the hosts whose events shd_relay_round_sharded
 * returns here -- and every per-host array (the batch's ev_off, the popped off[]) covers those
 * hi - lo hosts.  A batch whose n_dst differs from the queues' host count is SHD_ERR_INVALID. */
shd_status shd_equeue_setup(shd_ctx* ctx, uint32_t n_hosts);
shd_status shd_equeue_advance(shd_ctx* ctx, const shd_relay_out* d_batch, uint64_t window_end,
                              shd_equeue_out* out);
/* Engine-owned device arrays (ev_off, ev_deliver, ev_src, ev_seq, ev_pkt; n_dst set) for up to
 * max_events events of the next round's relay output: pass them as the shd_relay_round_device
 * output (with the caller's status array), then to shd_equeue_advance, which adopts the batch as
 * a stored run without copying any of it.  Valid until that advance (or the next call). */
shd_status shd_equeue_batch_buffers(shd_ctx* ctx, uint64_t max_events, shd_relay_out* out);
/* Host copies of the last advance's popped events (any pointer may be NULL). */
shd_status shd_equeue_copy_popped(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                                  uint64_t* seq, uint64_t* tag);
/* Host copy of the pending queues (same layout; any pointer may be NULL). */
shd_status shd_equeue_pending(shd_ctx* ctx, uint32_t* off, uint64_t* deliver, uint32_t* src,
                              uint64_t* seq, uint64_t* tag, uint64_t* n_pending);

/* ---------------------------------------------------------------- round window */
/*
 * Runahead (src/main/core/scheduler/runahead.rs:12-115) kept in the context, and the next
 * scheduling window (SimController::manager_finished_current_round, controller.rs:86-111) from
 * the engine's own state.  shd_runahead_setup = Runahead::new(is_runahead_dynamic,
 * min_possible_latency, min_runahead_config) (manager.rs:246-251): min_possible_latency_ns = 0
 * takes RoutingInfo::get_smallest_latency_ns of the resident table; min_runahead_config_ns = 0
 * is None.  Every committed relay round (single or sharded; its min_latency reduced over all
 * ranks) then updates the lowest used latency when dynamic (update_lowest_used_latency,
 * worker.rs:380).  shd_round_window takes the caller's earliest non-packet event time
 * (UINT64_MAX: none) and the experiment end, and returns the window [start, end) the reference's
 * manager would open next: start = the minimum over that time, the pending queues' heads and the
 * last relay output not yet merged (manager.rs:430-464; UINT64_MAX = none, which is
 * EmulatedTime::MAX), end = min(start + runahead (saturating at EmulatedTime::MAX), end_time);
 * *running = start < end.  Under a communicator the minimum is reduced over all ranks: a
 * collective (every rank calls it, and every rank gets the same window).
 */
shd_status shd_runahead_setup(shd_ctx* ctx, int32_t dynamic, uint64_t min_possible_latency_ns,
                              uint64_t min_runahead_config_ns);
shd_status shd_runahead_get(const shd_ctx* ctx, uint64_t* runahead_ns);
shd_status shd_round_window(shd_ctx* ctx, uint64_t cpu_next_event_time, uint64_t end_time,
                            uint64_t* window_start, uint64_t* window_end, int32_t* running);
/* The window arithmetic alone (no context, no GPU): controller.rs:92-111 for a given minimum
 * next event time and runahead. */
shd_status shd_window_compute(uint64_t min_next_event_time, uint64_t runahead_ns, uint64_t end_time,
                              uint64_t* window_start, uint64_t* window_end, int32_t* running);

/* Copy bytes from an engine-owned device array (e.g. shd_equeue_out, a sharded relay output) to
 * host memory on the context's stream; returns when the copy is complete. */
shd_status shd_copy_to_host(shd_ctx* ctx, void* dst, const void* d_src, size_t bytes);

/* Read back the per-host RNG states / next event ids (e.g. to hand RNG use back to the CPU).
 * A sharded context's own hosts carry their current state, the others their setup state. */
shd_status shd_relay_get_host_state(shd_ctx* ctx, uint64_t* rng_state, uint64_t* next_event_id);

/* Per-path packet counters (RoutingInfo::increment_packet_count, graph/mod.rs:451-458): on by
 * default; the reference only reads them in log_packet_counts (never called), so a caller may
 * turn them off.  Counts accumulate over all rounds (n_nodes x n_nodes u64). */
shd_status shd_relay_set_counters(shd_ctx* ctx, int32_t enabled);
shd_status shd_path_packet_counts(shd_ctx* ctx, uint64_t* counts);

/* Which device pipeline ran the last successful round (diagnostics; no reference counterpart):
 * 7 = destination-bin placement, 3 = radix sort by destination, 1 = 64-bit records; 8 = a
 * sharded round whose pipeline-7 bins went to their destination ranks as stamped and were sorted
 * there (no packing or merge pass; otherwise a sharded round reports the local pipeline). */
shd_status shd_relay_last_pipeline(const shd_ctx* ctx, int32_t* pipeline);

/* ---------------------------------------------------------------------------------------
 * CoDel inbound router queues.  Replaces CoDelQueue::push / pop
 * (src/main/network/router/codel_queue.rs:125-306) for every host at once: one queue per host
 * stays on the device; a call replays a batch of operations, grouped by host, each host's in
 * time order.  A push carries (time, total size, packet id); a pop (size == SHD_CODEL_POP)
 * returns the next conforming packet or none, dropping per RFC 8289 as the reference does.
 * ------------------------------------------------------------------------------------- */
#define SHD_CODEL_POP 0xFFFFFFFFu

typedef struct shd_codel_ops {   /* device pointers */
    uint64_t n_ops;
    const uint32_t* host_off;    /* [n_hosts + 1] */
    const uint64_t* time;        /* [n_ops] emulated ns (the `now` argument) */
    const uint32_t* size;        /* [n_ops] packet total size for a push, SHD_CODEL_POP for a pop */
    const uint32_t* pkt;         /* [n_ops] packet id for a push (ignored for a pop) */
} shd_codel_ops;

typedef struct shd_codel_state {   /* one host's queue, for inspection (the reference's fields) */
    uint32_t len, mode;            /* mode: 0 Store, 1 Drop */
    uint32_t has_interval_end, has_drop_next;
    uint64_t interval_end, drop_next;
    uint64_t current_drop_count, previous_drop_count, total_bytes_stored;
} shd_codel_state;

/* (Re)create n_hosts empty queues holding up to `capacity` packets each. */
shd_status shd_codel_setup(shd_ctx* ctx, uint32_t n_hosts, uint32_t capacity);
/* Run a batch.  pop_out[k] = packet id a pop returned (SHD_CODEL_POP for none or for a push);
 * fate[id] = (op index << 2) | 1 (dequeued) or | 2 (dropped) for every packet this batch
 * dequeued or dropped (other entries untouched).  SHD_ERR_INVALID: a queue exceeded its
 * capacity or a packet id >= n_ids (the batch ran with the affected pushes/marks skipped, so the
 * queues are left undefined: every later call returns SHD_ERR_STATE until shd_codel_setup). */
shd_status shd_codel_run_device(shd_ctx* ctx, const shd_codel_ops* ops, uint32_t* pop_out,
                                uint64_t* fate, uint32_t n_ids);
shd_status shd_codel_get_state(shd_ctx* ctx, uint32_t host, shd_codel_state* out);

/* ---------------------------------------------------------------------------------------
 * Token-bucket relays.  Replaces TokenBucket::conforming_remove
 * (src/main/network/relay/token_bucket.rs:68-157) as Relay::forward_until_blocked calls it
 * (src/main/network/relay/mod.rs:200-287), for every relay at once: one bucket per relay stays
 * on the device; a call replays a batch of forwarding attempts, grouped by relay, each relay's
 * in time order.  An attempt is FORWARDED (value = the balance after it; UINT64_MAX for a relay
 * without a bucket), BLOCKED (value = the duration until it would conform; the relay is then
 * Pending until now + value, as forward_later schedules it) or SKIPPED (made while the relay
 * was Pending; value = the pending deadline).  Flag SHD_TB_EXEMPT: a local packet or one sent
 * while bootstrapping, forwarded without tokens (relay/mod.rs:224-229).
 * ------------------------------------------------------------------------------------- */
#define SHD_TB_FORWARDED 0
#define SHD_TB_BLOCKED 1
#define SHD_TB_SKIPPED 2
#define SHD_TB_EXEMPT 1u

typedef struct shd_tb_ops {     /* device pointers */
    uint64_t n_ops;
    const uint32_t* relay_off;  /* [n_relays + 1] */
    const uint64_t* time;       /* [n_ops] emulated ns (Worker::current_time) */
    const uint32_t* size;       /* [n_ops] packet total size (tokens to remove) */
    const uint8_t* flags;       /* [n_ops] SHD_TB_EXEMPT or 0 */
} shd_tb_ops;

typedef struct shd_tb_state {   /* one relay's bucket, for inspection (the reference's fields) */
    uint64_t capacity, balance, refill_increment, refill_interval, last_refill, pending_until;
} shd_tb_state;

/* (Re)create n_relays buckets (TokenBucket::new_inner, token_bucket.rs:37-60; full at start).
 * All three parameters 0 = no bucket (RateLimit::Unlimited); some but not all 0 is
 * SHD_ERR_INVALID (the reference's new() returns None and its caller unwraps).  Host arrays;
 * create_token_bucket (relay/mod.rs:291-302) is capacity = max(1, Bps/1000) + 1500,
 * increment = max(1, Bps/1000), interval = 1 ms. */
shd_status shd_tb_setup(shd_ctx* ctx, uint32_t n_relays, const uint64_t* capacity,
                        const uint64_t* refill_increment, const uint64_t* refill_interval_ns,
                        const uint64_t* last_refill);
/* Run a batch (device pointers); status[k] / value[k] per attempt.  SHD_ERR_INVALID where the
 * reference panics (a time before the bucket's last refill, a SimulationTime past SIMTIME_MAX);
 * the batch still ran. */
shd_status shd_tb_run_device(shd_ctx* ctx, const shd_tb_ops* ops, uint8_t* status, uint64_t* value);
shd_status shd_tb_get_state(shd_ctx* ctx, uint32_t relay, shd_tb_state* out);

/* ---------------------------------------------------------------------------------------
 * GML loader (host code, no GPU needed).  Replaces the reference's
 * gml_parser::parse (src/lib/gml-parser/src/lib.rs:52-57) + NetworkGraph::parse
 * (src/main/network/graph/mod.rs:136-183): GML text -> the shd_graph arrays the routing build
 * takes.  Node index = order of the node in the text (petgraph add_node order); a repeated GML
 * id maps to its later node, as the reference's HashMap insert does.  On failure `msg` holds the
 * reference's message (e.g. "Edge 'latency' must not be 0", "Edge source 7 doesn't exist").
 * ------------------------------------------------------------------------------------- */
typedef struct shd_gml shd_gml;

/* Parse `len` bytes of GML.  SHD_ERR_INVALID: grammar or validation error;
 * SHD_ERR_LATENCY_OVERFLOW: an edge latency does not fit u64 ns (the reference panics in
 * convert(Nano).unwrap(), graph/mod.rs:338). */
shd_status shd_gml_parse(const char* text, size_t len, shd_gml** out, char* msg, size_t msg_len);
/* load_network_graph (graph/mod.rs:481-511) for a GML file: read `path` (xz != 0: decompress it
 * as xz, read_xz :482-494 -- through the system liblzma), require strict UTF-8
 * (String::from_utf8), then shd_gml_parse.  File, decompression and UTF-8 failures are
 * SHD_ERR_INVALID with the reference's context message. */
shd_status shd_gml_load(const char* path, int32_t xz, shd_gml** out, char* msg, size_t msg_len);
/* View of the parsed graph; the arrays stay owned by `g` until shd_gml_free. */
shd_status shd_gml_graph(const shd_gml* g, shd_graph* view);
/* host_bandwidth_down / _up per node in bits/s (UINT64_MAX = attribute absent; values beyond
 * u64 saturate at UINT64_MAX - 1).  Either pointer may be NULL; arrays are [n_nodes]. */
shd_status shd_gml_node_bandwidth(const shd_gml* g, uint64_t* down_bps, uint64_t* up_bps);
void shd_gml_free(shd_gml* g);

#ifdef __cplusplus
}
#endif
#endif /* SHD_ACCEL_H */
