"""GML text -> graph, restating the reference's GML front end (test infrastructure only).

Restates:
  * ``src/lib/gml-parser/src/parser.rs:44-262`` (nom grammar: key/item/gml/node/edge/value/
    int/float/string/newline/int_as_bool) and ``src/lib/gml-parser/src/lib.rs:52-57``;
  * ``src/main/core/support/units.rs:214-280`` (TimePrefix), ``:142-178`` (SiPrefixUpper),
    ``:377-388`` (convert with checked_mul), ``:405-438`` (FromStr: regex
    ``^([+-]?[0-9\\.]*)\\s*(.*)$``, suffix stripping, ``ParseIntError`` texts);
  * ``src/main/network/graph/mod.rs:30-113`` (ShadowNode / ShadowEdge ``try_from``),
    ``:136-183`` (NetworkGraph::parse) and ``:335-342`` (edge -> PathProperties).

Floats are parsed with correct round-to-nearest-even to binary32, as Rust's
``str::parse::<f32>`` does (no double rounding through binary64).
"""
from __future__ import annotations

import re
import struct
from dataclasses import dataclass, field
from fractions import Fraction

import numpy as np

U64_MAX = (1 << 64) - 1


class GmlError(ValueError):
    """Parse / validation failure (the reference returns ``Err(String)``)."""


# ----------------------------------------------------------------------------- floats
def decimal_to_f32(text: str) -> np.float32:
    """Correctly rounded decimal -> binary32 (Rust ``str::parse::<f32>`` semantics)."""
    s = text.strip()
    neg = s.startswith("-")
    f = Fraction(s.lstrip("+-")) if s.lstrip("+-") not in ("", ".") else None
    if f is None:
        raise GmlError(f"invalid float literal {text!r}")
    if f == 0:
        return np.float32(-0.0) if neg else np.float32(0.0)
    # find e with 2^e <= f < 2^(e+1)
    e = f.numerator.bit_length() - f.denominator.bit_length()
    if Fraction(2) ** e > f:
        e -= 1
    if e > 127:
        bits = 0x7F800000
    else:
        shift = 23 - max(e, -126)          # subnormals share the exponent of 2^-126
        scaled = f * (Fraction(2) ** shift)
        m = scaled.numerator // scaled.denominator
        rem = scaled - m
        if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and (m & 1)):
            m += 1
        if e < -126:
            bits = m                          # subnormal (m may carry into the smallest normal)
        else:
            if m >= (1 << 24):
                m >>= 1
                e += 1
            bits = 0x7F800000 if e > 127 else (((e + 127) << 23) | (m & 0x7FFFFF))
    if neg:
        bits |= 0x80000000
    return np.frombuffer(struct.pack("<I", bits), dtype=np.float32)[0]


# ----------------------------------------------------------------------------- lexer pieces
_SPACE = " \t"
_MULTISPACE = " \t\r\n"


class _Cursor:
    def __init__(self, text: str):
        self.s = text
        self.i = 0

    def space0(self):
        while self.i < len(self.s) and self.s[self.i] in _SPACE:
            self.i += 1

    def multispace0(self):
        while self.i < len(self.s) and self.s[self.i] in _MULTISPACE:
            self.i += 1

    def newline(self) -> bool:
        """``recognize(tuple((space0, multispace1, space0)))`` (parser.rs:252-254)."""
        j = self.i
        self.space0()
        if self.i >= len(self.s) or self.s[self.i] not in _MULTISPACE:
            self.i = j
            return False
        self.multispace0()
        # multispace1 is greedy over [ \t\r\n]; trailing space0 is then a no-op
        return True

    def tag(self, t: str) -> bool:
        if self.s.startswith(t, self.i):
            self.i += len(t)
            return True
        return False

    def key(self):
        """``[a-zA-Z_][a-zA-Z0-9_]*`` (parser.rs:45-51)."""
        s, i = self.s, self.i
        if i >= len(s) or not (s[i].isascii() and (s[i].isalpha() or s[i] == "_")):
            return None
        j = i + 1
        while j < len(s) and s[j].isascii() and (s[j].isalnum() or s[j] == "_"):
            j += 1
        self.i = j
        return s[i:j]


_FLOAT_RE = re.compile(r"[+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+)(?:[eE][+-]?[0-9]+)?")
# an exponent marker with no digits after its optional sign (no backtracking over the sign)
_FLOAT_BAD_EXP = re.compile(r"[+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+)[eE](?:[+-](?![0-9])|(?![+\-0-9]))")


def _value(c: _Cursor):
    """``value`` (parser.rs:214-224): space0, then int|float|string, each followed by newline."""
    c.space0()
    start = c.i
    # int: digit1 parsed as i32 (parse failure -> alt falls through to float)
    m = re.compile(r"[0-9]+").match(c.s, c.i)
    if m:
        txt = m.group(0)
        if int(txt) <= 0x7FFFFFFF:
            c.i = m.end()
            if c.newline():
                return ("int", int(txt))
        c.i = start
    if _FLOAT_BAD_EXP.match(c.s, c.i):
        raise GmlError("float exponent without digits")   # nom `cut` -> hard failure
    m = _FLOAT_RE.match(c.s, c.i)
    if m:
        c.i = m.end()
        if c.newline():
            return ("float", decimal_to_f32(m.group(0)))
        c.i = start
    if c.tag('"'):
        # escaped_transform(is_not("\""), '\\', ..): the `normal` parser is_not("\"") already
        # swallows backslashes, so the string is simply everything up to the next '"'.
        j = c.s.find('"', c.i)
        if j < 0:
            raise GmlError("unterminated string")
        if j == c.i:
            raise GmlError("empty string")   # is_not matches >= 1 char; index 0 -> Error
        out = c.s[c.i:j]
        c.i = j + 1
        if c.newline():
            return ("str", out)
    c.i = start
    raise GmlError(f"invalid value at offset {start}")


def _kv_block(c: _Cursor) -> dict:
    """``space0 '[' newline many_till((key, value), ']')`` + duplicate-key check."""
    c.space0()
    if not c.tag("["):
        raise GmlError("expected '['")
    if not c.newline():
        raise GmlError("expected newline after '['")
    kvs = []
    while not c.tag("]"):
        k = c.key()
        if k is None:
            raise GmlError(f"expected key at offset {c.i}")
        kvs.append((k, _value(c)))
    d = dict(kvs)
    if len(d) != len(kvs):
        raise GmlError("Duplicate keys are not supported")
    return d


@dataclass
class GmlGraph:
    directed: bool
    nodes: list            # list of dict (key -> (type, value)); 'id' -> int or None
    edges: list            # list of dict with 'source','target' ints
    other: dict = field(default_factory=dict)


def parse_gml(text: str) -> GmlGraph:
    """``gml`` (parser.rs:68-150)."""
    c = _Cursor(text)
    c.multispace0()
    if not c.tag("graph"):
        raise GmlError("expected 'graph'")
    c.space0()
    if not c.tag("["):
        raise GmlError("expected '['")
    if not c.newline():
        raise GmlError("expected newline")
    nodes, edges, directed, others = [], [], [], []
    while not c.tag("]"):
        k = c.key()
        if k is None:
            raise GmlError(f"expected item at offset {c.i}")
        if k == "node" or k == "edge":
            kv = _kv_block(c)
            if not c.newline():
                raise GmlError("expected newline after ']'")
            if k == "node":
                idv = kv.pop("id", None)
                if idv is not None and idv[0] != "int":
                    raise GmlError("Incorrect 'id' type")
                kv["id"] = None if idv is None else (idv[1] & 0xFFFFFFFF)
                nodes.append(kv)
            else:
                for end in ("source", "target"):
                    v = kv.pop(end, None)
                    if v is None:
                        raise GmlError(f"'{end}' doesn't exist")
                    if v[0] != "int":
                        raise GmlError(f"Incorrect '{end}' type")
                    kv[end] = v[1] & 0xFFFFFFFF
                edges.append(kv)
        elif k == "directed":
            v = _value(c)
            if v[0] != "int":
                raise GmlError("Value was not an integer")
            if v[1] not in (0, 1):
                raise GmlError("Bool must be 0 or 1")
            directed.append(bool(v[1]))
        else:
            others.append((k, _value(c)))
    if len(directed) > 1:
        raise GmlError("The 'directed' key must only be specified once")
    od = dict(others)
    if len(od) != len(others):
        raise GmlError("Duplicate keys are not supported")
    return GmlGraph(directed=directed[0] if directed else False, nodes=nodes, edges=edges,
                    other=od)


# ----------------------------------------------------------------------------- units
_TIME_PREFIX_NS = {}
for _names, _ns in (
    (("ns", "nanosecond", "nanoseconds"), 1),
    (("us", "μs", "microsecond", "microseconds"), 10**3),
    (("ms", "millisecond", "milliseconds"), 10**6),
    (("s", "sec", "secs", "second", "seconds"), 10**9),
    (("m", "min", "mins", "minute", "minutes"), 60 * 10**9),
    (("h", "hr", "hrs", "hour", "hours"), 3600 * 10**9),
):
    for _n in _names:
        _TIME_PREFIX_NS[_n] = _ns

_UNIT_RE = re.compile(r"^([+-]?[0-9.]*)\s*(.*)\Z")   # Rust `$`: end of text only


def parse_time(text: str):
    """``Time::<TimePrefix>::from_str`` (units.rs:405-438).  Returns (value:u64, ns_per_unit)."""
    m = _UNIT_RE.match(text)
    if m is None:
        raise GmlError("Unable to identify value and unit")
    value, unit = m.group(1).strip(), m.group(2).strip()
    if unit == "":
        mag = 10**9                                  # TimePrefix::default() == Sec
    elif unit in _TIME_PREFIX_NS:
        mag = _TIME_PREFIX_NS[unit]
    else:
        raise GmlError("Unit was not one of (ns|nanosecond|nanoseconds|us|μs|microsecond|microseconds"
                       "|ms|millisecond|milliseconds|s|sec|secs|second|seconds|m|min|mins|minute"
                       "|minutes|h|hr|hrs|hour|hours)")
    return _parse_u64(value), mag


def _parse_u64(value: str) -> int:
    """Rust ``u64::from_str`` with its ``ParseIntError`` messages: an optional '+', then
    ASCII digits only."""
    if value == "":
        raise GmlError("cannot parse integer from empty string")
    v = value[1:] if value[0] == "+" and len(value) > 1 else value
    if not (v.isascii() and v.isdigit()):
        raise GmlError("invalid digit found in string")
    iv = int(v)
    if iv > U64_MAX:
        raise GmlError("number too large to fit in target type")
    return iv


_SI_UPPER = {"K": 1000, "kilo": 1000, "Ki": 1024, "kibi": 1024, "M": 10**6, "mega": 10**6,
             "Mi": 2**20, "mebi": 2**20, "G": 10**9, "giga": 10**9, "Gi": 2**30, "gibi": 2**30,
             "T": 10**12, "tera": 10**12, "Ti": 2**40, "tebi": 2**40}


def parse_bits_per_sec(text: str) -> int:
    """``BitsPerSec::<SiPrefixUpper>::from_str`` (units.rs:142-178, 405-438, 578): the unit
    minus a "bit"/"bits" suffix is the SI prefix ("" = base).  Returns bits/s (unbounded)."""
    m = _UNIT_RE.match(text)
    if m is None:
        raise GmlError("Unable to identify value and unit")
    value, unit = m.group(1).strip(), m.group(2).strip()
    prefix = unit
    for suf in ("bit", "bits"):
        if unit.endswith(suf):
            prefix = unit[: len(unit) - len(suf)]
            break
    if prefix == "":
        mag = 1
    elif prefix in _SI_UPPER:
        mag = _SI_UPPER[prefix]
    else:
        raise GmlError("Unit prefix was not one of (K|kilo|Ki|kibi|M|mega|Mi|mebi|G|giga|Gi|gibi"
                       "|T|tera|Ti|tebi)")
    return _parse_u64(value) * mag


def time_to_ns(value: int, mag: int) -> int:
    """``convert(TimePrefix::Nano)`` with ``checked_mul`` (units.rs:377-388)."""
    r = value * mag
    if r > U64_MAX:
        raise OverflowError("The resulting value is outside of the bounds")
    return r


# ----------------------------------------------------------------------------- graph
@dataclass
class Edge:
    source: int          # node index (petgraph NodeIndex == insertion order)
    target: int
    latency_ns: int      # u64
    packet_loss: np.float32


@dataclass
class NetworkGraph:
    """``NetworkGraph`` (graph/mod.rs:115-183): node ids, directed flag, edges by index."""
    directed: bool
    node_ids: list       # index -> GML id
    edges: list          # list[Edge] in GML order
    id_to_index: dict

    @property
    def n_nodes(self) -> int:
        return len(self.node_ids)


def _edge_from_gml(kv: dict):
    """``ShadowEdge::try_from`` (graph/mod.rs:74-113) + ``From<&ShadowEdge>`` (:335-342)."""
    kv = dict(kv)
    lat = kv.pop("latency", None)
    if lat is None:
        raise GmlError("Edge 'latency' was not provided")
    if lat[0] != "str":
        raise GmlError("Edge 'latency' is not a string")
    try:
        lat_v, lat_mag = parse_time(lat[1])
    except GmlError as e:
        raise GmlError(f"Edge 'latency' is not a valid unit: {e}") from None
    jit = kv.pop("jitter", None)
    if jit is not None:
        if jit[0] != "str":
            raise GmlError("Edge 'jitter' is not a string")
        try:
            parse_time(jit[1])                   # parsed and ignored
        except GmlError as e:
            raise GmlError(f"Edge 'jitter' is not a valid unit: {e}") from None
    pl = kv.pop("packet_loss", None)
    if pl is None:
        loss = np.float32(0.0)
    elif pl[0] != "float":
        raise GmlError("Edge 'packet_loss' is not a float")
    else:
        loss = pl[1]
    if loss < np.float32(0.0) or loss > np.float32(1.0):
        raise GmlError("Edge 'packet_loss' is not in the range [0,1]")
    if lat_v == 0:
        raise GmlError("Edge 'latency' must not be 0")
    return time_to_ns(lat_v, lat_mag), np.float32(loss)


def parse_network_graph(text: str) -> NetworkGraph:
    """``NetworkGraph::parse`` (graph/mod.rs:136-183)."""
    g = parse_gml(text)
    node_ids, id_map = [], {}
    for kv in g.nodes:
        if kv["id"] is None:
            raise GmlError("Node 'id' was not provided")
        for bw in ("host_bandwidth_down", "host_bandwidth_up"):   # ShadowNode (:30-62)
            if bw in kv:
                if kv[bw][0] != "str":
                    raise GmlError(f"Node '{bw}' is not a string")
                try:
                    parse_bits_per_sec(kv[bw][1])
                except GmlError as e:
                    raise GmlError(f"Node '{bw}' is not a valid unit: {e}") from None
        id_map[kv["id"]] = len(node_ids)
        node_ids.append(kv["id"])
    edges = []
    for kv in g.edges:
        lat, loss = _edge_from_gml(kv)
        if kv["source"] not in id_map:
            raise GmlError(f"Edge source {kv['source']} doesn't exist")
        if kv["target"] not in id_map:
            raise GmlError(f"Edge target {kv['target']} doesn't exist")
        edges.append(Edge(id_map[kv["source"]], id_map[kv["target"]], lat, loss))
    return NetworkGraph(directed=g.directed, node_ids=node_ids, edges=edges, id_to_index=id_map)


ONE_GBIT_SWITCH_GRAPH = """graph [
  directed 0
  node [
    id 0
    host_bandwidth_up "1 Gbit"
    host_bandwidth_down "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "1 ms"
    packet_loss 0.0
  ]
]"""
"""Data constant restated from ``src/main/core/support/configuration.rs:1314-1327``."""
