// Generated from include/shd_accel.h by tools/gen_abi.py -- do not edit by hand.
// tests/test_abi_layout.py holds every struct's C layout and the function list against the header.
#![allow(non_camel_case_types, non_upper_case_globals, dead_code)]
use std::os::raw::{c_char, c_int, c_void};

pub type shd_status = i32;
pub const SHD_ABI_VERSION: u32 = 3;
pub const SHD_ROUTE_SHORTEST: u32 = 0;
pub const SHD_ROUTE_DIRECT: u32 = 1;
pub const SHD_ALGO_AUTO: u32 = 0;
pub const SHD_ALGO_SSSP: u32 = 1;
pub const SHD_ALGO_PRUNED: u32 = 2;
pub const SHD_ALGO_DELTA: u32 = 3;
pub const SHD_ALGO_BLOCKED: u32 = 4;
pub const SHD_PKT_SKIPPED: u32 = 0;
pub const SHD_PKT_DROPPED: u32 = 1;
pub const SHD_PKT_SENT: u32 = 2;
pub const SHD_SEND_PAYLOAD: u32 = 0x80000000;
pub const SHD_COMM_ID_BYTES: u32 = 128;
pub const SHD_CODEL_POP: u32 = 0xffffffff;
pub const SHD_TB_FORWARDED: u32 = 0;
pub const SHD_TB_BLOCKED: u32 = 1;
pub const SHD_TB_SKIPPED: u32 = 2;
pub const SHD_TB_EXEMPT: u32 = 1;
pub const SHD_OK: shd_status = 0;
pub const SHD_ERR_NO_EDGE: shd_status = 1;
pub const SHD_ERR_MULTI_EDGE: shd_status = 2;
pub const SHD_ERR_UNREACHABLE: shd_status = 3;
pub const SHD_ERR_LATENCY_OVERFLOW: shd_status = 4;
pub const SHD_ERR_INVALID: shd_status = 5;
pub const SHD_ERR_HIP: shd_status = 6;
pub const SHD_ERR_NOMEM: shd_status = 7;
pub const SHD_ERR_NO_HOST: shd_status = 8;
pub const SHD_ERR_STATE: shd_status = 9;

#[repr(C)] pub struct shd_ctx { _p: [u8; 0] }
#[repr(C)] pub struct shd_gml { _p: [u8; 0] }

#[repr(C)] #[derive(Clone, Copy)] pub struct shd_error {
    pub code: i32,
    pub node_a: u32,
    pub node_b: u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_graph {
    pub n_nodes: u32,
    pub n_edges: u32,
    pub edge_src: *const u32,
    pub edge_dst: *const u32,
    pub edge_latency_ns: *const u64,
    pub edge_packet_loss: *const f32,
    pub node_ids: *const u32,
    pub directed: i32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_routing_info {
    pub algo_used: u32,
    pub wide_latency: u32,
    pub arcs: u64,
    pub arcs_kept: u64,
    pub ms_total: f64,
    pub ms_main: f64,
    pub ms_minplus: f64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_round {
    pub round_end: u64,
    pub sim_end: u64,
    pub bootstrap_end: u64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_batch {
    pub n_packets: u64,
    pub src_off: *const u32,
    pub send_time: *const u64,
    pub dst_host: *const u32,
    pub payload: *const u32,
    pub chance: *const f64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_relay_out {
    pub status: *mut u8,
    pub ev_off: *mut u32,
    pub ev_deliver: *mut u64,
    pub ev_src: *mut u32,
    pub ev_seq: *mut u64,
    pub ev_pkt: *mut u32,
    pub min_deliver: u64,
    pub min_latency: u64,
    pub n_sent: u64,
    pub n_dst: u32,
    pub n_events: u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_send12 {
    pub time_off: u32,
    pub dst: u32,
    pub draw_hi: u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_stage {
    pub n_runs: u32,
    pub run_host: *const u32,
    pub run_count: *const u32,
    pub n_sends: u64,
    pub sends: *const shd_send12,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_event16 {
    pub deliver_off: u32,
    pub src_host: u32,
    pub seq_off: u32,
    pub send: u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_event12 {
    pub deliver_off: u32,
    pub seq_off: u32,
    pub send: u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_flush_out {
    pub struct_size: u32,
    pub event_bytes: u32,
    pub status2: *mut u8,
    pub ev_off: *mut u32,
    pub events: *mut shd_event16,
    pub seq_base: *mut u64,
    pub min_deliver: u64,
    pub min_latency: u64,
    pub n_sent: u64,
    pub n_events: u64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_host_comm_ops {
    pub user: *mut c_void,
    pub all_to_allv: Option<unsafe extern "C" fn(*mut c_void, *const c_void, *const u64, *const u64, *mut c_void, *const u64, *const u64) -> c_int>,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_equeue_out {
    pub off: *const u32,
    pub deliver: *const u64,
    pub src: *const u32,
    pub seq: *const u64,
    pub tag: *const u64,
    pub n_popped: u64,
    pub n_pending: u64,
    pub next_time: u64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_codel_ops {
    pub n_ops: u64,
    pub host_off: *const u32,
    pub time: *const u64,
    pub size: *const u32,
    pub pkt: *const u32,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_codel_state {
    pub len: u32,
    pub mode: u32,
    pub has_interval_end: u32,
    pub has_drop_next: u32,
    pub interval_end: u64,
    pub drop_next: u64,
    pub current_drop_count: u64,
    pub previous_drop_count: u64,
    pub total_bytes_stored: u64,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_tb_ops {
    pub n_ops: u64,
    pub relay_off: *const u32,
    pub time: *const u64,
    pub size: *const u32,
    pub flags: *const u8,
}
#[repr(C)] #[derive(Clone, Copy)] pub struct shd_tb_state {
    pub capacity: u64,
    pub balance: u64,
    pub refill_increment: u64,
    pub refill_interval: u64,
    pub last_refill: u64,
    pub pending_until: u64,
}

extern "C" {
    pub fn shd_version() -> *mut constchar;
    pub fn shd_status_str(st: shd_status) -> *mut constchar;
    pub fn shd_open(device_ordinal: c_int, st: *mut shd_status) -> *mut shd_ctx;
    pub fn shd_close(ctx: *mut shd_ctx);
    pub fn shd_set_stream(ctx: *mut shd_ctx, hip_stream: *mut c_void) -> shd_status;
    pub fn shd_set_knob(ctx: *mut shd_ctx, name: *const c_char, value: i64) -> shd_status;
    pub fn shd_get_knob(ctx: *const shd_ctx, name: *const c_char, value: *mut i64) -> shd_status;
    pub fn shd_routing_build(ctx: *mut shd_ctx, g: *const shd_graph, used: *const u32, n_used: u32, mode: u32, algo: u32, row_begin: u32, row_end: u32, lat_out: *mut u64, loss_out: *mut f32, err: *mut shd_error) -> shd_status;
    pub fn shd_routing_prepare(ctx: *mut shd_ctx, g: *const shd_graph, used: *const u32, n_used: u32, mode: u32, err: *mut shd_error) -> shd_status;
    pub fn shd_routing_run(ctx: *mut shd_ctx, algo: u32, row_begin: u32, row_end: u32, d_lat_out: *mut u64, d_loss_out: *mut f32, err: *mut shd_error) -> shd_status;
    pub fn shd_routing_run_next_hops(ctx: *mut shd_ctx, algo: u32, row_begin: u32, row_end: u32, d_lat_out: *mut u64, d_loss_out: *mut f32, d_next_hop: *mut u32, err: *mut shd_error) -> shd_status;
    pub fn shd_routing_build_device(ctx: *mut shd_ctx, g: *const shd_graph, used: *const u32, n_used: u32, mode: u32, algo: u32, row_begin: u32, row_end: u32, d_lat_out: *mut u64, d_loss_out: *mut f32, err: *mut shd_error) -> shd_status;
    pub fn shd_routing_last_info(ctx: *const shd_ctx, info: *mut shd_routing_info) -> shd_status;
    pub fn shd_routing_set_timing(ctx: *mut shd_ctx, every: u32) -> shd_status;
    pub fn shd_routing_lookup(ctx: *mut shd_ctx, src_row: u32, dst_col: u32, latency_ns: *mut u64, packet_loss: *mut f32) -> shd_status;
    pub fn shd_routing_lookup_batch(ctx: *mut shd_ctx, n: u64, src_row: *const u32, dst_col: *const u32, latency_ns: *mut u64, packet_loss: *mut f32) -> shd_status;
    pub fn shd_routing_mirror(ctx: *mut shd_ctx, enable: i32) -> shd_status;
    pub fn shd_routing_smallest_latency(ctx: *mut shd_ctx, latency_ns: *mut u64) -> shd_status;
    pub fn shd_assign_ips(n_hosts: u32, node_gml_id: *const u32, ip_in: *const u32, ip_out: *mut u32, used_gml: *mut u32, n_used: *mut u32, host_col: *mut u32, err_host: *mut u32) -> shd_status;
    pub fn shd_relay_setup(ctx: *mut shd_ctx, n_hosts: u32, host_node: *const u32, n_nodes: u32, lat: *const u64, loss: *const f32, rng_state: *const u64, next_event_id: *const u64) -> shd_status;
    pub fn shd_relay_round(ctx: *mut shd_ctx, batch: *const shd_batch, round: *const shd_round, out: *mut shd_relay_out) -> shd_status;
    pub fn shd_relay_round_device(ctx: *mut shd_ctx, d_batch: *const shd_batch, round: *const shd_round, d_out: *mut shd_relay_out) -> shd_status;
    pub fn shd_relay_flush(ctx: *mut shd_ctx, stages: *const shd_stage, n_stages: u32, time_base: u64, round: *const shd_round, out: *mut shd_flush_out) -> shd_status;
    pub fn shd_host_alloc(bytes: usize) -> *mut c_void;
    pub fn shd_host_free(p: *mut c_void);
    pub fn shd_comm_unique_id(id: *mut u8) -> shd_status;
    pub fn shd_comm_init(ctx: *mut shd_ctx, n_ranks: i32, rank: i32, id: *const u8) -> shd_status;
    pub fn shd_comm_init_local(ctxs: *mut *mut shd_ctx, n_ranks: i32) -> shd_status;
    pub fn shd_comm_init_host(ctx: *mut shd_ctx, n_ranks: i32, rank: i32, ops: *const shd_host_comm_ops) -> shd_status;
    pub fn shd_comm_info(ctx: *const shd_ctx, n_ranks: *mut i32, rank: *mut i32) -> shd_status;
    pub fn shd_comm_destroy(ctx: *mut shd_ctx) -> shd_status;
    pub fn shd_shard_range(total: u32, n_ranks: i32, rank: i32, lo: *mut u32, hi: *mut u32) -> shd_status;
    pub fn shd_routing_run_sharded(ctx: *mut shd_ctx, algo: u32, d_lat_full: *mut u64, d_loss_full: *mut f32, err: *mut shd_error) -> shd_status;
    pub fn shd_relay_round_sharded(ctx: *mut shd_ctx, d_batch: *const shd_batch, round: *const shd_round, d_out: *mut shd_relay_out) -> shd_status;
    pub fn shd_equeue_setup(ctx: *mut shd_ctx, n_hosts: u32) -> shd_status;
    pub fn shd_equeue_advance(ctx: *mut shd_ctx, d_batch: *const shd_relay_out, window_end: u64, out: *mut shd_equeue_out) -> shd_status;
    pub fn shd_equeue_batch_buffers(ctx: *mut shd_ctx, max_events: u64, out: *mut shd_relay_out) -> shd_status;
    pub fn shd_equeue_copy_popped(ctx: *mut shd_ctx, off: *mut u32, deliver: *mut u64, src: *mut u32, seq: *mut u64, tag: *mut u64) -> shd_status;
    pub fn shd_equeue_pending(ctx: *mut shd_ctx, off: *mut u32, deliver: *mut u64, src: *mut u32, seq: *mut u64, tag: *mut u64, n_pending: *mut u64) -> shd_status;
    pub fn shd_runahead_setup(ctx: *mut shd_ctx, dynamic: i32, min_possible_latency_ns: u64, min_runahead_config_ns: u64) -> shd_status;
    pub fn shd_runahead_get(ctx: *const shd_ctx, runahead_ns: *mut u64) -> shd_status;
    pub fn shd_round_window(ctx: *mut shd_ctx, cpu_next_event_time: u64, end_time: u64, window_start: *mut u64, window_end: *mut u64, running: *mut i32) -> shd_status;
    pub fn shd_window_compute(min_next_event_time: u64, runahead_ns: u64, end_time: u64, window_start: *mut u64, window_end: *mut u64, running: *mut i32) -> shd_status;
    pub fn shd_copy_to_host(ctx: *mut shd_ctx, dst: *mut c_void, d_src: *const c_void, bytes: usize) -> shd_status;
    pub fn shd_relay_get_host_state(ctx: *mut shd_ctx, rng_state: *mut u64, next_event_id: *mut u64) -> shd_status;
    pub fn shd_relay_set_counters(ctx: *mut shd_ctx, enabled: i32) -> shd_status;
    pub fn shd_path_packet_counts(ctx: *mut shd_ctx, counts: *mut u64) -> shd_status;
    pub fn shd_relay_last_pipeline(ctx: *const shd_ctx, pipeline: *mut i32) -> shd_status;
    pub fn shd_codel_setup(ctx: *mut shd_ctx, n_hosts: u32, capacity: u32) -> shd_status;
    pub fn shd_codel_run_device(ctx: *mut shd_ctx, ops: *const shd_codel_ops, pop_out: *mut u32, fate: *mut u64, n_ids: u32) -> shd_status;
    pub fn shd_codel_get_state(ctx: *mut shd_ctx, host: u32, out: *mut shd_codel_state) -> shd_status;
    pub fn shd_tb_setup(ctx: *mut shd_ctx, n_relays: u32, capacity: *const u64, refill_increment: *const u64, refill_interval_ns: *const u64, last_refill: *const u64) -> shd_status;
    pub fn shd_tb_run_device(ctx: *mut shd_ctx, ops: *const shd_tb_ops, status: *mut u8, value: *mut u64) -> shd_status;
    pub fn shd_tb_get_state(ctx: *mut shd_ctx, relay: u32, out: *mut shd_tb_state) -> shd_status;
    pub fn shd_gml_parse(text: *const c_char, len: usize, out: *mut *mut shd_gml, msg: *mut c_char, msg_len: usize) -> shd_status;
    pub fn shd_gml_load(path: *const c_char, xz: i32, out: *mut *mut shd_gml, msg: *mut c_char, msg_len: usize) -> shd_status;
    pub fn shd_gml_graph(g: *const shd_gml, view: *mut shd_graph) -> shd_status;
    pub fn shd_gml_node_bandwidth(g: *const shd_gml, down_bps: *mut u64, up_bps: *mut u64) -> shd_status;
    pub fn shd_gml_free(g: *mut shd_gml);
}
