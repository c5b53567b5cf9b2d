"""CPU tests of the C ABI's layout: every struct of include/shd_accel.h
against three mirrors --

* tests/abi/shd_layout.c, `_Static_assert`s of every size and field offset, compiled by gcc;
* the ctypes mirror the GPU tests call through (shadow_amd/_native.py);
* the Rust `-sys` crate's `#[repr(C)]` structs (rust/shadow-accel-sys/src/lib.rs, no Rust
  toolchain here: laid out by C's rules from the crate's own field types),

plus the function list: header = crate = ctypes EXPORTED.  The crate and the assert file are
generated from the header (tools/gen_abi.py); the tests also check they are current."""
import ctypes as C
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_abi as G  # noqa: E402

# header struct -> ctypes mirror (shadow_amd/_native.py); the 12/16-byte records travel as
# numpy (n, 3) / (n, 4) u32 arrays, checked by size only
CTYPES = {"shd_error": "Error", "shd_graph": "Graph", "shd_routing_info": "RoutingInfo", "shd_round": "Round",
          "shd_batch": "Batch", "shd_relay_out": "RelayOut", "shd_stage": "Stage", "shd_flush_out": "FlushOut",
          "shd_host_comm_ops": "HostCommOps", "shd_equeue_out": "EqueueOut", "shd_codel_ops": "CodelOps",
          "shd_codel_state": "CodelState", "shd_tb_ops": "TbOps", "shd_tb_state": "TbState"}
RECORDS = {"shd_send12": 12, "shd_event16": 16, "shd_event12": 12}


@pytest.fixture(scope="module")
def layout():
    return G.probe_layout()


def test_static_asserts_compile(tmp_path):
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-c", "-I", os.path.join(ROOT, "include"),
                           G.LAYOUT_C, "-o", str(tmp_path / "l.o")])


def test_generated_files_are_current(layout):
    assert open(G.LAYOUT_C).read() == G.gen_layout_c(layout), "rerun tools/gen_abi.py (tests/abi/shd_layout.c)"
    assert open(G.RUST).read() == G.gen_rust(), "rerun tools/gen_abi.py (rust/shadow-accel-sys/src/lib.rs)"


def test_every_struct_is_covered(layout):
    assert set(layout) == set(CTYPES) | set(RECORDS)
    for name, size in RECORDS.items():
        assert layout[name]["size"] == size


def test_ctypes_mirror_matches(layout):
    from shadow_amd import _native as N
    for name, cls in CTYPES.items():
        t = getattr(N, cls)
        v = layout[name]
        assert C.sizeof(t) == v["size"], name
        names = [f[0] for f in t._fields_]
        assert names == list(v["fields"]), f"{name}: field order {names}"
        for f, (off, sz) in v["fields"].items():
            assert getattr(t, f).offset == off, f"{name}.{f}"
            assert getattr(t, f).size == sz, f"{name}.{f}"


def test_rust_crate_matches(layout):
    rl = G.rust_layout()
    for name, v in layout.items():
        assert name in rl, name
        assert rl[name]["size"] == v["size"], name
        assert {f: o for f, (o, _) in rl[name]["fields"].items()} == {f: o for f, (o, _) in v["fields"].items()}, name


def test_function_lists_agree():
    from shadow_amd import _native as N
    hdr = sorted(G.parse_functions())
    assert len(hdr) >= 50
    assert sorted(G.rust_functions()) == hdr
    assert sorted(N.EXPORTED) == hdr


def test_flush_out_is_versioned():
    from shadow_amd import _native as N
    o = N.FlushOut(1, 2, 3, 4, event_bytes=12)
    assert o.struct_size == C.sizeof(N.FlushOut) and o.event_bytes == 12 and o.status2 == 1 and o.seq_base == 4
