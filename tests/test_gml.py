"""Native GML loader (shd_gml_parse, host code) against the oracle's GML restatement and the
reference's own GML/unit test vectors.  CPU tests: the loader needs no GPU.

Parity rules: on success the node ids, edge endpoints, latency (ns) and loss bits are identical;
on a validation error (every message the reference names) the message text is identical; on a
grammar error both reject (nom's VerboseError trace is not reproduced).  Inputs are ASCII apart
from "μs": non-ASCII whitespace inside unit strings and non-ASCII key characters (which the
reference tests as `char as u8`) are outside the tested domain."""
import numpy as np
import pytest

from oracle.gml import GmlError, ONE_GBIT_SWITCH_GRAPH, parse_bits_per_sec, parse_network_graph
from tests.golden.make_golden import LOSSY_GRAPH
from tests.graphs import KAT_SHORTEST_PATH

VALIDATION = ("Node '", "Edge '", "Edge source", "Edge target", "'source' doesn't exist",
              "'target' doesn't exist", "Incorrect '", "Duplicate keys", "The 'directed' key",
              "Bool must be", "Value was not an integer")


def _native(text):
    from shadow_amd.routing import NetGraphError, NetworkGraph, RoutingPanic
    try:
        return NetworkGraph.parse(text), None
    except NetGraphError as e:
        return None, str(e)
    except RoutingPanic:
        return None, "overflow"


def _oracle(text):
    try:
        return parse_network_graph(text), None
    except GmlError as e:
        return None, str(e)
    except OverflowError:
        return None, "overflow"


def _same(text):
    """Native and oracle agree on `text`; returns the native graph (or None)."""
    n, nerr = _native(text)
    o, oerr = _oracle(text)
    assert (n is None) == (o is None), (text, nerr, oerr)
    if n is None:
        if oerr.startswith(VALIDATION) or oerr == "overflow":
            assert nerr == oerr, (text, nerr, oerr)
        else:
            assert nerr.startswith("GML parse error"), (text, nerr, oerr)
        return None
    assert n.directed == o.directed
    assert n.node_ids.tolist() == o.node_ids
    assert n.edge_src.tolist() == [e.source for e in o.edges]
    assert n.edge_dst.tolist() == [e.target for e in o.edges]
    assert n.edge_latency_ns.tolist() == [e.latency_ns for e in o.edges]
    assert n.edge_packet_loss.view(np.uint32).tolist() == \
        np.asarray([e.packet_loss for e in o.edges], np.float32).view(np.uint32).tolist()
    return n


@pytest.mark.parametrize("directed", [0, 1])
def test_reference_kat_graph(directed):
    """The GML of graph/mod.rs:566-613 (test_shortest_path)."""
    g = _same(KAT_SHORTEST_PATH.format(directed=directed))
    assert g.directed == bool(directed) and g.n_nodes == 3
    assert g.edge_latency_ns.tolist() == [3333, 5555, 7777, 3, 5, 7, 11]


def test_reference_data_graphs():
    """The built-in 1_gbit_switch graph (configuration.rs:1314-1327) and the inline graph of
    src/test/tcp/tcp-blocking-lossy.yaml."""
    g = _same(ONE_GBIT_SWITCH_GRAPH)
    assert g.bandwidth_down_bps.tolist() == [10**9] and g.bandwidth_up_bps.tolist() == [10**9]
    g = _same(LOSSY_GRAPH)
    assert g.edge_packet_loss.tolist() == [np.float32(0.25)]


@pytest.mark.parametrize("target,ok", [(2, False), (3, True)])
def test_reference_kat_nonexistent_id(target, ok):
    """graph/mod.rs:533-559 test_nonexistent_id."""
    text = f"""graph [
                node [
                  id 1
                ]
                node [
                  id 3
                ]
                edge [
                  source 1
                  target {target}
                  latency "1 ns"
                ]
            ]"""
    g = _same(text)
    assert (g is not None) == ok
    if not ok:
        assert _native(text)[1] == f"Edge target {target} doesn't exist"


EDGE = """graph [
  node [
    id 0
  ]
  edge [
    source 0
    target 0
    latency "{lat}"
  ]
]"""
NODE_BW = """graph [
  node [
    id 0
    host_bandwidth_down "{bw}"
  ]
]"""


def test_reference_kat_units():
    """units.rs:584-640 (Time) and the BitsPerSec cases of units.rs:680-720, through GML."""
    S, M, MS, US = 10**9, 60 * 10**9, 10**6, 10**3
    for txt, ns in [("10", 10 * S), ("10 s", 10 * S), ("10s", 10 * S), ("10   s", 10 * S),
                    ("10sec", 10 * S), ("10  m", 10 * M), ("10  min", 10 * M), ("10 ms", 10 * MS),
                    ("10 μs", 10 * US), ("10 millisecond", 10 * MS), ("10 milliseconds", 10 * MS)]:
        assert _same(EDGE.format(lat=txt)).edge_latency_ns.tolist() == [ns]
    for bad in ("-10 ms", "abc 10 ms", "10.5 ms", "10 abc"):
        assert _same(EDGE.format(lat=bad)) is None
    for txt, bps in [("10", 10), ("10 bit", 10), ("10bit", 10), ("10   bit", 10), ("10  Kbit", 10_000),
                     ("10 Kibit", 10_240), ("10 Mbit", 10**7), ("10 megabit", 10**7),
                     ("10 megabits", 10**7)]:
        assert parse_bits_per_sec(txt) == bps
        assert _same(NODE_BW.format(bw=txt)).bandwidth_down_bps.tolist() == [bps]
    for bad in ("-10 Kbit", "abc 10 Kbit", "10.5 Kbit", "10 abc", "10 mbit"):
        assert _same(NODE_BW.format(bw=bad)) is None
        assert _native(NODE_BW.format(bw=bad))[1].startswith("Node 'host_bandwidth_down' is not a valid unit: ")


@pytest.mark.parametrize("text,msg", [
    (EDGE.format(lat="0 ms"), "Edge 'latency' must not be 0"),
    (EDGE.format(lat="5 xs"), "Edge 'latency' is not a valid unit: Unit was not one of (ns|nanosecond|"
                              "nanoseconds|us|μs|microsecond|microseconds|ms|millisecond|milliseconds|s|"
                              "sec|secs|second|seconds|m|min|mins|minute|minutes|h|hr|hrs|hour|hours)"),
    (EDGE.format(lat="+ ms"), "Edge 'latency' is not a valid unit: invalid digit found in string"),
    (EDGE.format(lat=" ms"), "Edge 'latency' is not a valid unit: cannot parse integer from empty string"),
    (EDGE.format(lat="99999999999999999999 ns"),
     "Edge 'latency' is not a valid unit: number too large to fit in target type"),
    (EDGE.format(lat="10 ms\n"), "Edge 'latency' is not a valid unit: Unable to identify value and unit"),
    (EDGE.format(lat="99999999999 hours"), "overflow"),
    (EDGE.replace('latency "{lat}"', "packet_loss 0.5"), "Edge 'latency' was not provided"),
    (EDGE.replace('"{lat}"', "5"), "Edge 'latency' is not a string"),
    (EDGE.format(lat="1 ms").replace("  ]\n]", '    jitter 3\n  ]\n]'), "Edge 'jitter' is not a string"),
    (EDGE.format(lat="1 ms").replace("  ]\n]", "    packet_loss 0\n  ]\n]"), "Edge 'packet_loss' is not a float"),
    (EDGE.format(lat="1 ms").replace("  ]\n]", "    packet_loss 1.0000001\n  ]\n]"),
     "Edge 'packet_loss' is not in the range [0,1]"),
    (EDGE.format(lat="1 ms").replace("    id 0\n", ""), "Node 'id' was not provided"),
    (EDGE.format(lat="1 ms").replace("id 0", 'id "a"'), "Incorrect 'id' type"),
    (EDGE.format(lat="1 ms").replace("id 0", "id 2147483648"), "Incorrect 'id' type"),
    (EDGE.format(lat="1 ms").replace("    source 0\n", ""), "'source' doesn't exist"),
    (EDGE.format(lat="1 ms").replace("target 0", "target 0.0"), "Incorrect 'target' type"),
    (EDGE.format(lat="1 ms").replace("    source 0\n", "    source 0\n    source 0\n"),
     "Duplicate keys are not supported"),
    (EDGE.format(lat="1 ms").replace("graph [\n", "graph [\n  directed 1\n  directed 0\n"),
     "The 'directed' key must only be specified once"),
    (EDGE.format(lat="1 ms").replace("graph [\n", "graph [\n  directed 2\n"), "Bool must be 0 or 1"),
    (EDGE.format(lat="1 ms").replace("graph [\n", 'graph [\n  directed "1"\n'), "Value was not an integer"),
    (EDGE.format(lat="1 ms").replace("graph [\n", "graph [\n  label 1\n  label 2\n"),
     "Duplicate keys are not supported"),
    (NODE_BW.format(bw="1 Gbit").replace('"1 Gbit"', "5"), "Node 'host_bandwidth_down' is not a string"),
])
def test_validation_messages(text, msg):
    _same(text)
    assert _native(text)[1] == msg


@pytest.mark.parametrize("text", [
    "", "graph", "graph [", "graph [ ]", "graph [\n  node [ id 0 ]\n]", 'graph [\n  label ""\n]',
    "graph [\n  weight 1e\n]", "graph [\n  weight 1.5x\n]", "graph [\n  node [\n    id 0\n  ]]",
    'graph [\n  label "abc\n]', "graph [\n  1key 2\n]", "graph [\n  node [\n  graphics [\n  ]\n  ]\n]",
])
def test_grammar_errors_rejected(text):
    assert _same(text) is None
    assert _native(text)[1].startswith("GML parse error")


def test_grammar_accepts_reference_quirks():
    """Trailing text after the graph is ignored (parse() is not all_consuming); values may
    touch their key ('label"x"'); floats like '1.', '.5', '+.5', '5E-2' and -0.0 loss."""
    base = "graph [\n  node [\n    id 7\n  ]\n  edge [\n    source 7\n    target 7\n" \
           "    latency \"3 us\"\n    packet_loss {p}\n  ]\n]trailing junk"
    for p in ("1.", ".5", "+.5", "5E-2", "-0.0", "0.0000001", "1e-45", "1.0"):
        g = _same(base.format(p=p))
        assert g is not None and g.edge_latency_ns.tolist() == [3000]
    g = _same('graph [\n  label"x"\n  node [\n    id 0\n  ]\n]')
    assert g is not None and g.n_nodes == 1
    g = _same("graph [\n  node [\n    id 0007\n  ]\n  node [\n    id 5\n  ]\n  node [\n    id 7\n  ]\n]")
    assert g.node_ids.tolist() == [7, 5, 7] and g.node_id_to_index(7) == 2   # later node wins


# ------------------------------------------------------------------ randomized parity
_UNITS = ["ns", "us", "μs", "ms", "s", "sec", "second", "m", "min", "h", "hr", "", "millisecond",
          "microseconds", "nanoseconds", "hours"]
_BW = ["1 Gbit", "100 Mbit", "10 Kibit", "10bits", "10", "5 Ti bit", "7 gibibit", "3 Tbit",
       "12 mebibits", "9 kilobit"]


def _rand_gml(rng):
    ws = lambda: str(rng.choice([" ", "  ", "\t", " \t "]))             # noqa: E731
    nl = lambda: str(rng.choice(["\n", "\r\n", "\n\n", " \n\t", "\n  ", "\t\n"]))  # noqa: E731
    n = int(rng.integers(1, 12))
    ids = [int(x) for x in rng.choice(40, size=n, replace=bool(rng.random() < 0.2))]
    parts = [str(rng.choice(["", "\n", "  \n"])), "graph", str(rng.choice(["", " "])), "[", nl()]
    items = []
    if rng.random() < 0.7:
        items.append(f"directed{ws()}{int(rng.integers(0, 2))}{nl()}")
    if rng.random() < 0.3:
        items.append(f'label{ws()}"g{int(rng.integers(0, 9))}"{nl()}')
    for i in ids:
        kv = [f"id{ws()}{i}{nl()}"]
        if rng.random() < 0.4:
            kv.append(f'host_bandwidth_down{ws()}"{rng.choice(_BW)}"{nl()}')
        if rng.random() < 0.4:
            kv.append(f'host_bandwidth_up{ws()}"{rng.choice(_BW)}"{nl()}')
        if rng.random() < 0.3:
            kv.append(f"x{ws()}{rng.uniform(-5, 5):.4f}{nl()}")
        rng.shuffle(kv)
        items.append(f"node{ws()}[{nl()}{''.join(kv)}]{nl()}")
    for _ in range(int(rng.integers(0, 25))):
        a, b = int(rng.choice(ids)), int(rng.choice(ids))
        if rng.random() < 0.05:
            b = int(rng.integers(40, 60))                 # nonexistent target
        lat = f"{int(rng.integers(0 if rng.random() < 0.03 else 1, 5000))}{rng.choice(['', ' ', '  '])}{rng.choice(_UNITS)}"
        kv = [f"source{ws()}{a}{nl()}", f"target{ws()}{b}{nl()}", f'latency{ws()}"{lat}"{nl()}']
        r = rng.random()
        if r < 0.25:
            kv.append(f"packet_loss{ws()}{rng.uniform(0, 1):.{int(rng.integers(1, 9))}f}{nl()}")
        elif r < 0.4:
            kv.append(f"packet_loss{ws()}{rng.uniform(0, 1):.{int(rng.integers(1, 6))}e}{nl()}")
        elif r < 0.45:
            kv.append(f"packet_loss{ws()}{rng.choice(['0', '1', '1.5', '.25', '0.', '-0.0'])}{nl()}")
        if rng.random() < 0.2:
            kv.append(f'jitter{ws()}"{int(rng.integers(0, 50))} {rng.choice(_UNITS)}"{nl()}')
        rng.shuffle(kv)
        items.append(f"edge{ws()}[{nl()}{''.join(kv)}]{nl()}")
    rng.shuffle(items)
    parts += items + ["]", str(rng.choice(["", "\n", " trailing"]))]
    return "".join(parts)


@pytest.mark.parametrize("seed", range(6))
def test_random_graphs_native_vs_oracle(seed):
    rng = np.random.default_rng(7000 + seed)
    ok = 0
    for _ in range(150):
        ok += _same(_rand_gml(rng)) is not None
    assert ok > 20   # the generator keeps most graphs valid


@pytest.mark.parametrize("seed", range(4))
def test_mutation_fuzz_native_vs_oracle(seed):
    """Single-byte deletions / insertions / substitutions of valid graphs: both parsers agree on
    accept/reject, on validation messages, and on every output bit when they accept."""
    rng = np.random.default_rng(9000 + seed)
    alphabet = list(' \t\n"[]0123456789.e+-_abcdilnorstgpx')
    for _ in range(60):
        text = _rand_gml(rng)
        for _ in range(8):
            k = int(rng.integers(0, len(text) + 1))
            op = rng.random()
            if op < 0.34 and k < len(text):
                mut = text[:k] + text[k + 1:]
            elif op < 0.67:
                mut = text[:k] + str(rng.choice(alphabet)) + text[k:]
            else:
                mut = text[:k] + str(rng.choice(alphabet)) + text[k + 1:]
            _same(mut)


def test_native_parse_speed_vs_oracle():
    """The loader is the startup path in front of the APSP: on a 20k-edge
    graph it must beat the Python restatement by a wide margin (C4-scale numbers: DESIGN.md)."""
    import time
    from shadow_amd import synth
    el = synth.barabasi_albert(5000, 2, 11)
    lines = ["graph [", "  directed 0"]
    for i in el.node_ids:
        lines += ["  node [", f"    id {int(i)}", "  ]"]
    for a, b, lat, p in zip(el.src, el.dst, el.latency_ns, el.packet_loss):
        lines += ["  edge [", f"    source {int(el.node_ids[a])}", f"    target {int(el.node_ids[b])}",
                  f'    latency "{int(lat)} ns"', f"    packet_loss {float(p)!r}", "  ]"]
    text = "\n".join(lines + ["]"])
    t0 = time.perf_counter()
    g = _native(text)[0]
    t1 = time.perf_counter()
    o = parse_network_graph(text)
    t2 = time.perf_counter()
    assert g is not None and len(g.edge_src) == len(o.edges)
    assert (t1 - t0) * 5 < (t2 - t1)


# The reference's compressed-graph integration test (src/test/compressed-graph/): its graph
# file, compressed with `xz --force` as its CMakeLists does, loaded with `compression: xz`.
COMPRESSED_GRAPH = """graph [
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
  ]
]
"""


def _xz_file(tmp_path, name, data: bytes):
    import shutil
    import subprocess
    p = tmp_path / name
    p.write_bytes(data)
    if shutil.which("xz"):
        subprocess.check_call(["xz", "--force", str(p)])
    else:   # same container format (CRC64 check, xz's default)
        import lzma
        (tmp_path / (name + ".xz")).write_bytes(lzma.compress(data, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64))
    return str(p) + ".xz"


def test_native_load_xz_reference_compressed_graph(tmp_path):
    from shadow_amd.routing import NetGraphError, load_network_graph
    path = _xz_file(tmp_path, "graph-compressed.gml", COMPRESSED_GRAPH.encode())
    g = load_network_graph(path, compression="xz")
    assert g.node_ids.tolist() == [0] and g.edge_latency_ns.tolist() == [1_000_000]
    assert g.bandwidth_up_bps.tolist() == [10**9] and g.bandwidth_down_bps.tolist() == [10**9]
    with pytest.raises(NetGraphError, match="Failed to read file"):   # read_to_string: not UTF-8
        load_network_graph(path, compression=None)
    with pytest.raises(NetGraphError, match="Failed to decompress"):
        load_network_graph(_corrupt(tmp_path, path), compression="xz")
    with pytest.raises(NetGraphError, match="Failed to"):
        load_network_graph(str(tmp_path / "missing.gml.xz"), compression="xz")


def _corrupt(tmp_path, path):
    b = bytearray(open(path, "rb").read())
    b[len(b) // 2] ^= 0x5A
    q = tmp_path / "corrupt.gml.xz"
    q.write_bytes(bytes(b))
    return str(q)


@pytest.mark.parametrize("seed", range(3))
def test_native_load_xz_random_graphs(tmp_path, seed):
    """Random GML texts: plain file, xz file and in-memory parse give identical arrays."""
    from shadow_amd.routing import NetworkGraph, load_network_graph
    rng = np.random.default_rng(900 + seed)
    text = _rand_gml(rng)
    try:
        want = NetworkGraph.parse(text)
    except Exception:   # noqa: BLE001 -- invalid texts: the loaders must agree on the error too
        want = None
    plain = tmp_path / "g.gml"
    plain.write_text(text)
    for path, comp in ((str(plain), None), (_xz_file(tmp_path, "h.gml", text.encode()), "xz")):
        if want is None:
            with pytest.raises(Exception):
                load_network_graph(path, compression=comp)
            continue
        g = load_network_graph(path, compression=comp)
        for k in ("node_ids", "edge_src", "edge_dst", "edge_latency_ns"):
            assert np.array_equal(getattr(g, k), getattr(want, k)), k
        assert np.array_equal(g.edge_packet_loss.view(np.uint32), want.edge_packet_loss.view(np.uint32))


def test_native_load_rejects_invalid_utf8(tmp_path):
    from shadow_amd.routing import NetGraphError, load_network_graph
    path = _xz_file(tmp_path, "bad.gml", COMPRESSED_GRAPH.encode().replace(b"Gbit", b"G\xffbit"))
    with pytest.raises(NetGraphError, match="utf-8"):
        load_network_graph(path, compression="xz")
