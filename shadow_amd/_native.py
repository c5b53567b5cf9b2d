"""ctypes binding of include/shd_accel.h (the in-tree libshd_accel.so).

This is the reference-side binding a Python host would use; the Rust equivalent is shown in
INTEGRATION.md.  There is no fallback: if the library is missing or no gfx950 GPU is present,
every call raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SHD_ACCEL_LIB") or os.path.join(HERE, "libshd_accel.so")  # override: tuning builds

SHD_OK = 0
STATUS_NAMES = {0: "OK", 1: "NO_EDGE", 2: "MULTI_EDGE", 3: "UNREACHABLE", 4: "LATENCY_OVERFLOW",
                5: "INVALID", 6: "HIP", 7: "NOMEM", 8: "NO_HOST", 9: "STATE"}

ROUTE_SHORTEST, ROUTE_DIRECT = 0, 1
ALGO_AUTO, ALGO_SSSP, ALGO_PRUNED, ALGO_DELTA, ALGO_BLOCKED = 0, 1, 2, 3, 4
PKT_SKIPPED, PKT_DROPPED, PKT_SENT = 0, 1, 2

EXPORTED = [
    "shd_version", "shd_status_str", "shd_open", "shd_close", "shd_set_stream",
    "shd_routing_build", "shd_routing_prepare", "shd_routing_run", "shd_routing_build_device",
    "shd_routing_last_info", "shd_routing_set_timing",
    "shd_routing_lookup", "shd_routing_smallest_latency", "shd_relay_setup", "shd_relay_round",
    "shd_relay_round_device", "shd_relay_get_host_state",
    "shd_relay_set_counters", "shd_relay_last_pipeline",
    "shd_path_packet_counts",
    "shd_gml_parse", "shd_gml_graph", "shd_gml_node_bandwidth", "shd_gml_free",
    "shd_codel_setup", "shd_codel_run_device", "shd_codel_get_state",
    "shd_tb_setup", "shd_tb_run_device", "shd_tb_get_state",
    "shd_comm_unique_id", "shd_comm_init", "shd_comm_init_local", "shd_comm_info", "shd_comm_destroy",
    "shd_shard_range", "shd_routing_run_sharded", "shd_relay_round_sharded",
    "shd_equeue_setup", "shd_equeue_advance", "shd_equeue_copy_popped", "shd_equeue_pending",
    "shd_routing_run_next_hops", "shd_assign_ips", "shd_gml_load",
    "shd_runahead_setup", "shd_runahead_get", "shd_round_window", "shd_window_compute", "shd_copy_to_host",
    "shd_routing_lookup_batch", "shd_routing_mirror", "shd_equeue_batch_buffers",
    "shd_set_knob", "shd_get_knob", "shd_relay_flush", "shd_host_alloc", "shd_host_free",
    "shd_comm_init_host",
]
COMM_ID_BYTES = 128

# shd_host_comm_ops (include/shd_accel.h): the all-to-all-v callback of shd_comm_init_host
_U64P = C.POINTER(C.c_uint64)
ALL_TO_ALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, _U64P, _U64P, C.c_void_p, _U64P, _U64P)


class HostCommOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("all_to_allv", ALL_TO_ALLV)]


class ShdError(RuntimeError):
    def __init__(self, status: int, where: str, node_a=None, node_b=None):
        self.status = status
        self.code = STATUS_NAMES.get(status, str(status))
        self.node_a, self.node_b = node_a, node_b
        super().__init__(f"{where}: {self.code}" +
                         (f" (nodes {node_a}, {node_b})" if node_a is not None else ""))


class Graph(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_edges", C.c_uint32),
                ("edge_src", C.c_void_p), ("edge_dst", C.c_void_p),
                ("edge_latency_ns", C.c_void_p), ("edge_packet_loss", C.c_void_p),
                ("node_ids", C.c_void_p), ("directed", C.c_int32)]


class Error(C.Structure):
    _fields_ = [("code", C.c_int32), ("node_a", C.c_uint32), ("node_b", C.c_uint32)]


class RoutingInfo(C.Structure):
    _fields_ = [("algo_used", C.c_uint32), ("wide_latency", C.c_uint32), ("arcs", C.c_uint64),
                ("arcs_kept", C.c_uint64), ("ms_total", C.c_double), ("ms_main", C.c_double),
                ("ms_minplus", C.c_double)]


class Round(C.Structure):
    _fields_ = [("round_end", C.c_uint64), ("sim_end", C.c_uint64), ("bootstrap_end", C.c_uint64)]


class Batch(C.Structure):
    _fields_ = [("n_packets", C.c_uint64), ("src_off", C.c_void_p), ("send_time", C.c_void_p),
                ("dst_host", C.c_void_p), ("payload", C.c_void_p), ("chance", C.c_void_p)]


class RelayOut(C.Structure):
    _fields_ = [("status", C.c_void_p), ("ev_off", C.c_void_p), ("ev_deliver", C.c_void_p),
                ("ev_src", C.c_void_p), ("ev_seq", C.c_void_p), ("ev_pkt", C.c_void_p),
                ("min_deliver", C.c_uint64), ("min_latency", C.c_uint64), ("n_sent", C.c_uint64),
                ("n_dst", C.c_uint32), ("n_events", C.c_uint32)]


class Stage(C.Structure):
    _fields_ = [("n_runs", C.c_uint32), ("run_host", C.c_void_p), ("run_count", C.c_void_p),
                ("n_sends", C.c_uint64), ("sends", C.c_void_p)]


class FlushOut(C.Structure):
    """shd_flush_out; versioned by its leading struct_size, which the constructor fills in.
    FlushOut(status2, ev_off, events, seq_base, min_deliver, min_latency, n_sent, n_events,
    event_bytes): the fields' order before round 6, kept for the callers."""
    _fields_ = [("struct_size", C.c_uint32), ("event_bytes", C.c_uint32),
                ("status2", C.c_void_p), ("ev_off", C.c_void_p), ("events", C.c_void_p), ("seq_base", C.c_void_p),
                ("min_deliver", C.c_uint64), ("min_latency", C.c_uint64), ("n_sent", C.c_uint64),
                ("n_events", C.c_uint64)]

    def __init__(self, status2=0, ev_off=0, events=0, seq_base=0, min_deliver=0, min_latency=0, n_sent=0,
                 n_events=0, event_bytes=16):
        super().__init__(C.sizeof(FlushOut), event_bytes, status2, ev_off, events, seq_base, min_deliver,
                         min_latency, n_sent, n_events)


SEND_PAYLOAD = 0x80000000


class EqueueOut(C.Structure):
    _fields_ = [("off", C.c_void_p), ("deliver", C.c_void_p), ("src", C.c_void_p), ("seq", C.c_void_p),
                ("tag", C.c_void_p), ("n_popped", C.c_uint64), ("n_pending", C.c_uint64),
                ("next_time", C.c_uint64)]


class CodelOps(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("host_off", C.c_void_p), ("time", C.c_void_p),
                ("size", C.c_void_p), ("pkt", C.c_void_p)]


class TbOps(C.Structure):
    _fields_ = [("n_ops", C.c_uint64), ("relay_off", C.c_void_p), ("time", C.c_void_p),
                ("size", C.c_void_p), ("flags", C.c_void_p)]


class TbState(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("balance", C.c_uint64), ("refill_increment", C.c_uint64),
                ("refill_interval", C.c_uint64), ("last_refill", C.c_uint64), ("pending_until", C.c_uint64)]


class CodelState(C.Structure):
    _fields_ = [("len", C.c_uint32), ("mode", C.c_uint32), ("has_interval_end", C.c_uint32),
                ("has_drop_next", C.c_uint32), ("interval_end", C.c_uint64), ("drop_next", C.c_uint64),
                ("current_drop_count", C.c_uint64), ("previous_drop_count", C.c_uint64),
                ("total_bytes_stored", C.c_uint64)]


_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the native library; raises if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"shd_accel native library missing at {path}: run "
                           "`python -m shadow_amd.build` (or __graft_entry__.build())")
    # torch bundles its own libamdhip64 with the same soname: load it first so this library and
    # torch share ONE HIP runtime in the process (device pointers and streams then interoperate)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P, U32, U64, I32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "shd_version": (C.c_char_p, []),
        "shd_status_str": (C.c_char_p, [I32]),
        "shd_open": (P, [C.c_int, P]),
        "shd_close": (None, [P]),
        "shd_set_stream": (I32, [P, P]),
        "shd_routing_build": (I32, [P, P, P, U32, U32, U32, U32, U32, P, P, P]),
        "shd_routing_build_device": (I32, [P, P, P, U32, U32, U32, U32, U32, P, P, P]),
        "shd_routing_prepare": (I32, [P, P, P, U32, U32, P]),
        "shd_routing_run": (I32, [P, U32, U32, U32, P, P, P]),
        "shd_routing_last_info": (I32, [P, P]),
        "shd_routing_set_timing": (I32, [P, U32]),
        "shd_routing_lookup": (I32, [P, U32, U32, P, P]),
        "shd_routing_smallest_latency": (I32, [P, P]),
        "shd_relay_setup": (I32, [P, U32, P, U32, P, P, P, P]),
        "shd_relay_round": (I32, [P, P, P, P]),
        "shd_relay_round_device": (I32, [P, P, P, P]),
        "shd_relay_get_host_state": (I32, [P, P, P]),
        "shd_relay_set_counters": (I32, [P, I32]),
        "shd_relay_last_pipeline": (I32, [P, P]),
        "shd_path_packet_counts": (I32, [P, P]),
        "shd_gml_parse": (I32, [P, C.c_size_t, P, P, C.c_size_t]),
        "shd_gml_graph": (I32, [P, P]),
        "shd_gml_node_bandwidth": (I32, [P, P, P]),
        "shd_gml_free": (None, [P]),
        "shd_codel_setup": (I32, [P, U32, U32]),
        "shd_codel_run_device": (I32, [P, P, P, P, U32]),
        "shd_codel_get_state": (I32, [P, U32, P]),
        "shd_tb_setup": (I32, [P, U32, P, P, P, P]),
        "shd_tb_run_device": (I32, [P, P, P, P]),
        "shd_tb_get_state": (I32, [P, U32, P]),
        "shd_comm_unique_id": (I32, [P]),
        "shd_comm_init": (I32, [P, I32, I32, P]),
        "shd_comm_init_local": (I32, [P, I32]),
        "shd_comm_info": (I32, [P, P, P]),
        "shd_comm_destroy": (I32, [P]),
        "shd_shard_range": (I32, [U32, I32, I32, P, P]),
        "shd_routing_run_sharded": (I32, [P, U32, P, P, P]),
        "shd_relay_round_sharded": (I32, [P, P, P, P]),
        "shd_equeue_setup": (I32, [P, U32]),
        "shd_routing_run_next_hops": (I32, [P, U32, U32, U32, P, P, P, P]),
        "shd_assign_ips": (I32, [U32, P, P, P, P, P, P, P]),
        "shd_gml_load": (I32, [C.c_char_p, I32, P, P, C.c_size_t]),
        "shd_equeue_advance": (I32, [P, P, U64, P]),
        "shd_equeue_copy_popped": (I32, [P, P, P, P, P, P]),
        "shd_equeue_pending": (I32, [P, P, P, P, P, P, P]),
        "shd_runahead_setup": (I32, [P, I32, U64, U64]),
        "shd_runahead_get": (I32, [P, P]),
        "shd_round_window": (I32, [P, U64, U64, P, P, P]),
        "shd_window_compute": (I32, [U64, U64, U64, P, P, P]),
        "shd_copy_to_host": (I32, [P, P, P, C.c_size_t]),
        "shd_routing_lookup_batch": (I32, [P, U64, P, P, P, P]),
        "shd_routing_mirror": (I32, [P, I32]),
        "shd_equeue_batch_buffers": (I32, [P, U64, P]),
        "shd_set_knob": (I32, [P, C.c_char_p, C.c_int64]),
        "shd_relay_flush": (I32, [P, P, U32, U64, P, P]),
        "shd_host_alloc": (P, [C.c_size_t]),
        "shd_host_free": (None, [P]),
        "shd_get_knob": (I32, [P, C.c_char_p, P]),
        "shd_comm_init_host": (I32, [P, I32, I32, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, where: str, err: Error | None = None):
    if status != SHD_OK:
        if err is not None and err.code != 0:
            raise ShdError(status, where, err.node_a, err.node_b)
        raise ShdError(status, where)


def ptr(a):
    """Host numpy array -> void*, or device torch tensor -> void* (data_ptr)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return a.ctypes.data_as(C.c_void_p)
