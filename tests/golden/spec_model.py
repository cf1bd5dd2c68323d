"""Executable model of the reference's NF specifications (test
infrastructure: fixture generation only, in the container that holds the
reference).

vignat, vigfw and vigbridge each ship a behavioural specification
(`vignat/spec.py`, `vigfw/spec.py`, `vigbridge/spec.py`) that the reference's
validator translates into VeriFast contracts (`validator/translate-spec.py`).
They are Python syntax over a small vocabulary: `pop_header`, header
constructors with `...` for unspecified fields, and the abstract state
objects (`emap`, `vector`). This module gives that vocabulary the meaning the
reference's own models give it, and runs a spec text once per packet:

  emap (libvig/verified/emap.h:10-69): a map key -> index, a vector
  index -> key and a dchain of (index, time) cells;
  expire_all(t) drops every index whose time is < t (is_cell_expired,
  double-chain.h:127-129), refresh_idx re-stamps, add allocates
  `the_index_allocated` (the spec leaves the choice to the implementation:
  the caller supplies the implementation's index, or Emap.AUTO for libVig's
  dchain order), full() is
  dchain_out_of_space_fp (double-chain.h:35-39: size <= live count).

  Header fields (translate-spec.py:6-9) are read from the frame the way the
  NF's C structs read them (little-endian loads of network-order bytes;
  ether.type 0x0800 reads as 8, the value the specs assert). pop_header
  fails (on_mismatch: drop) when the frame is too short for the header or
  the outer header announces another protocol; the specs' asserts (IPv4
  ethertype, TCP/UDP protocol) are enforced the same way. The NF's finer
  parse predicates (IHL, total_length) are not part of the specs, so the
  traces that use this model keep to IHL 5 and consistent lengths.

The spec text is read from the reference at generation time only; what the
model derives is committed as fixtures (tests/golden/spec_*.npz).
"""
from __future__ import annotations

import ast
import collections
import textwrap


class Emap:
    def __init__(self, size: int):
        self.size = size
        self.m = {}    # key -> index
        self.v = {}    # index -> key
        self.ch = {}   # index -> time, in LRU order (the dchain's alist)
        # the implementation's choice of `the_index_allocated` where the spec
        # leaves it open (Emap.AUTO): libVig's dchain hands out freed indices
        # last-freed first, then never-used ones in order
        # (double-chain-impl.c, pinned against oracle/_ref)
        self.freed = []
        self.fresh = 0

    def _free(self, i):
        del self.ch[i]
        self.freed.append(i)

    def expire_all(self, t):
        for i in [i for i, ts in self.ch.items() if ts < t]:  # LRU first
            self._free(i)
            k = self.v.pop(i)
            if self.m.get(k) == i:
                del self.m[k]

    def has(self, k):
        return k in self.m

    def get(self, k):
        return self.m[k]

    def has_idx(self, i):
        return i in self.ch

    def get_key(self, i):
        return self.v[i]

    def refresh_idx(self, i, t):
        del self.ch[i]  # (to the MRU end: dchain_rejuvenate_fp)
        self.ch[i] = t

    AUTO = "lowest free index"  # the_index_allocated where unobservable

    def add(self, k, i, t):
        if i is Emap.AUTO:
            if self.freed:
                i = self.freed.pop()
            else:
                i, self.fresh = self.fresh, self.fresh + 1
        elif i in self.freed:
            self.freed.remove(i)
        assert i not in self.ch, "index %d allocated twice" % i
        self.last = i
        self.m[k] = i
        self.v[i] = k
        self.ch[i] = t

    def erase(self, k):
        i = self.m.pop(k)
        self._free(i)
        self.v.pop(i, None)

    def full(self):
        return self.size <= len(self.ch)

    # emap_exists_with_cht / emap_choose_with_cht (emap.h:73-83): row
    # hash % height of the CHT (cht.h:26-34, height = length / index range),
    # the first of its backends allocated in this emap's dchain
    def _row(self, cht, h):
        height = len(cht) // self.size
        r = h % height
        return cht[r * self.size:(r + 1) * self.size]

    def exists_with_cht(self, cht, h):
        return any(b in self.ch for b in self._row(cht, h))

    def choose_with_cht(self, cht, h):
        return next(b for b in self._row(cht, h) if b in self.ch)


class Vector(dict):
    def set(self, i, val):
        self[i] = val


class AutoVector(Vector):
    """A vector indexed by the emap's AUTO indices: `set(the_index_allocated,
    v)` right after `add` refers to the index add just chose."""

    def __init__(self, emap):
        super().__init__()
        self.emap = emap

    def _ix(self, i):
        return self.emap.last if i is Emap.AUTO else i

    def set(self, i, val):
        self[self._ix(i)] = val


class Hdr:
    """A header value: named fields; Ellipsis = left unspecified."""

    def __init__(self, kind, fields):
        self.kind = kind
        self.f = dict(fields)

    def __getattr__(self, name):
        try:
            return self.__dict__["f"][name]
        except KeyError as e:
            raise AttributeError(name) from e


def _le16(b, o):
    return b[o] | (b[o + 1] << 8)


def _le32(b, o):
    return b[o] | (b[o + 1] << 8) | (b[o + 2] << 16) | (b[o + 3] << 24)


def parse(frame: bytes):
    """{header kind: Hdr} of the headers a frame carries (model above)."""
    out = {}
    if len(frame) < 14:
        return out
    out["ether"] = Hdr("ether", {"daddr": bytes(frame[0:6]),
                                 "saddr": bytes(frame[6:12]),
                                 "type": _le16(frame, 12)})
    if out["ether"].type != 8 or len(frame) < 34:
        return out
    ip = {"vihl": frame[14], "tos": frame[15], "len": _le16(frame, 16),
          "pid": _le16(frame, 18), "foff": _le16(frame, 20), "ttl": frame[22],
          "npid": frame[23], "cksum": _le16(frame, 24),
          "saddr": _le32(frame, 26), "daddr": _le32(frame, 30)}
    out["ipv4"] = Hdr("ipv4", ip)
    if ip["npid"] not in (6, 17) or len(frame) < 38:
        return out
    out["tcpudp"] = Hdr("tcpudp", {"src_port": _le16(frame, 34),
                                   "dst_port": _le16(frame, 36)})
    return out


class _Drop(Exception):
    pass


def _header_ctor(kind):
    def make(base=None, **kw):
        f = dict(base.f) if base is not None else {}
        f.update(kw)
        return Hdr(kind, f)
    return make


def _record(*names):
    """A spec value constructor (FlowIdc, ...): hashable, fields by name."""
    return collections.namedtuple("Rec", names)


class _IntDiv(ast.NodeTransformer):
    """`/` is integer division in the specs (translate-spec.py renders it as
    VeriFast's `/` over integers); their operands are non-negative here."""

    def visit_BinOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div):
            node.op = ast.FloorDiv()
        return node


# The spec files are public, untrusted text: before anything runs, their AST
# must stay inside the vocabulary the reference's specs use (assertions,
# assignments, conditionals, arithmetic, calls of the model's constructors
# and of emap/vector methods). No imports, loops, lambdas, comprehensions,
# f-strings or dunder names; no attribute beginning with "_". They run with
# no builtins, over the model objects the caller passes in.
_SPEC_NODES = {
    "Module", "FunctionDef", "arguments", "Assert", "Assign", "AugAssign", "Expr",
    "If", "Return", "Pass", "BinOp", "BoolOp", "UnaryOp", "Compare", "Call",
    "keyword", "Attribute", "Name", "Load", "Store", "Constant", "List", "Tuple",
    "Subscript", "IfExp",
    "Add", "Sub", "Mult", "Div", "FloorDiv", "Mod", "BitAnd", "BitOr", "BitXor",
    "LShift", "RShift", "And", "Or", "Not", "USub", "UAdd", "Invert",
    "Eq", "NotEq", "Lt", "LtE", "Gt", "GtE", "Is", "IsNot", "In", "NotIn"}


class SpecRejected(ValueError):
    pass


def check_spec_ast(tree: ast.AST) -> None:
    """Raise SpecRejected unless every node is in the spec vocabulary."""
    for node in ast.walk(tree):
        kind = type(node).__name__
        if kind not in _SPEC_NODES:
            raise SpecRejected("spec uses %s (line %s)" % (kind, getattr(node, "lineno", "?")))
        if isinstance(node, ast.Name) and node.id.startswith("__"):
            raise SpecRejected("spec names %r" % node.id)
        if isinstance(node, ast.Attribute) and node.attr.startswith("_"):
            raise SpecRejected("spec reads attribute %r" % node.attr)
        if isinstance(node, ast.FunctionDef) and node.name.startswith("__") \
                and node.name != "__spec__":
            raise SpecRejected("spec defines %r" % node.name)
        if isinstance(node, ast.Call) and not isinstance(node.func, (ast.Name, ast.Attribute)):
            raise SpecRejected("spec calls a computed callee (line %s)" % node.lineno)
        if isinstance(node, ast.Constant) and not (isinstance(node.value, (int, bool))
                                                    or node.value in (None, Ellipsis)):
            raise SpecRejected("spec constant %r" % (node.value,))


def compile_spec(text: str):
    """The spec text as a function of one packet's environment (the
    `from state import ...` line's objects come from the caller's env),
    after check_spec_ast has accepted it."""
    body = "\n".join(l for l in text.splitlines()
                     if not l.startswith("from state import"))
    src = "def __spec__():\n" + textwrap.indent(body, "    ") + "\n"
    tree = ast.parse(src)
    check_spec_ast(tree)
    tree = ast.fix_missing_locations(_IntDiv().visit(tree))
    return compile(tree, "<spec>", "exec")


_CTORS = {"ether": _header_ctor("ether"), "ipv4": _header_ctor("ipv4"),
          "tcpudp": _header_ctor("tcpudp")}
_KIND = {v: k for k, v in _CTORS.items()}


def run_packet(code, env: dict, headers: dict):
    """Evaluate the compiled spec for one packet: (ports, headers).
    `pop_header(ipv4, ...)` names the header by its constructor."""
    def pop_header(ctor, on_mismatch):
        k = _KIND[ctor]
        if k not in headers:
            raise _Drop()
        return headers[k]
    g = dict(env, pop_header=pop_header, **_CTORS)
    g["__builtins__"] = {}  # the spec sees the model's objects only
    ns = {}
    exec(code, g, ns)
    try:
        r = ns["__spec__"]()
    except _Drop:  # on_mismatch=([],[]) in every spec: dropped
        return ([], [])
    # a path without a return (vigpol: a new address with the table full)
    # sends nothing
    return ([], []) if r is None else r


def crc32c_u32(h: int, v: int) -> int:
    """One SSE4.2 crc32 step over a zero-extended u32 (reflected 0x82F63B78,
    no final xor): the generated hashes' step (boilerplate-util.h:9)."""
    h ^= v & 0xFFFFFFFF
    for _ in range(32):
        h = (h >> 1) ^ (0x82F63B78 if h & 1 else 0)
    return h


def struct_hash(*fields) -> int:
    """A generated `<Struct>_hash`: one crc step per field in declaration
    order (codegen/main.ml:328-401)."""
    h = 0
    for f in fields:
        h = crc32c_u32(h, f)
    return h


def base_env():
    return {"FlowIdc": _record("sp", "dp", "sip", "dip", "idev", "prot"),
            "a_packet_received": True,
            "vector_get": lambda vec, i: vec[i],
            "vector_set": lambda vec, i, val: vec.set(i, val)}
