"""The GML loader's parity evidence on the GPU box (the driver's GPU tier runs only -m gpu):
the native loader (host code) against the oracle restatement on the reference's known answers,
random graphs and mutations, the xz path, then loader -> routing build on the GPU end to end."""
import numpy as np
import pytest

from oracle import corc
from tests import test_gml as T

pytestmark = pytest.mark.gpu


def test_loader_reference_kats_on_box():
    for d in (0, 1):
        T.test_reference_kat_graph(d)
    T.test_reference_data_graphs()
    T.test_reference_kat_nonexistent_id(2, False)
    T.test_reference_kat_nonexistent_id(3, True)
    T.test_reference_kat_units()
    T.test_grammar_accepts_reference_quirks()


@pytest.mark.parametrize("seed", range(6))
def test_loader_random_and_mutations_on_box(seed):
    T.test_random_graphs_native_vs_oracle(seed)
    if seed < 4:
        T.test_mutation_fuzz_native_vs_oracle(seed)


def test_loader_xz_on_box(tmp_path):
    T.test_native_load_xz_reference_compressed_graph(tmp_path)
    T.test_native_load_xz_random_graphs(tmp_path, 0)


def test_gml_to_gpu_routing_end_to_end(engine, tmp_path):
    """A 300-node GML file (xz) -> native loader -> GPU routing build == C oracle on the arrays
    the oracle's own GML restatement parsed."""
    from oracle.gml import parse_network_graph
    from shadow_amd.routing import load_network_graph
    from tests.graphs import gml_text, oracle_graph_arrays, random_graph
    rng = np.random.default_rng(77)
    ids, s, d, l, p, directed = random_graph(rng, 300, 0.02, False, max_ms=30)
    text = gml_text(ids * 3 + 1, s, d, l, p)
    path = T._xz_file(tmp_path, "g.gml", text.encode())
    g = load_network_graph(path, compression="xz")
    oi, os_, od, ol, op, odir = oracle_graph_arrays(parse_network_graph(text))
    assert np.array_equal(g.edge_src, os_) and np.array_equal(g.edge_latency_ns, ol)
    used = np.arange(300, dtype=np.uint32)
    code, lat, loss, _ = corc.routing(300, os_, od, ol, op, odir, used)
    t = g.compute_shortest_paths(used, engine)
    assert np.array_equal(t.lat, lat) and np.array_equal(t.loss.view(np.uint32), loss.view(np.uint32))
