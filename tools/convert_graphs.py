"""Convert the reference's Town01 lane graphs (networkx graphs pickled in
`CarlaBEV/assets/Town01/*.pkl`, read by `MapGraph._load_graph`,
CarlaBEV/src/planning/map_graph.py:13-19) into JSON under
carlabev_env_amd/assets/graphs/, so the host scene generator can plan on them
without any pickle on the GPU box.

The pickles are NOT unpickled: this file walks their opcodes with a small
restricted interpreter of its own. Nothing named by a file is imported or
called: the only globals it accepts are networkx's Graph / DiGraph classes and
numpy's ndarray reconstruction triple (`_reconstruct`, `ndarray`, `dtype`),
which it rebuilds symbolically (a graph becomes the dict of its `__dict__`
state; an array becomes numpy.frombuffer of its raw bytes). Any other global,
or any opcode outside the set below, is an error. Runs in the build container
only (it reads /root/reference); the JSON it writes is committed.

JSON format per graph: {"kind": "Graph" | "DiGraph", "graph": {...},
"nodes": [[node, attrs], ...], "adj": [[u, [[v, attrs], ...]], ...] and, for a
DiGraph, "pred" likewise}, in the pickled (= insertion) order, arrays as
{"__ndarray__": [...], "dtype": "<f8", "shape": [...]}.
"""
from __future__ import annotations

import argparse
import json
import os
import pickletools
import struct

import numpy as np

REF = "/root/reference/CarlaBEV/assets"
OUT = os.path.join(os.path.dirname(__file__), "..", "carlabev_env_amd", "assets", "graphs")

ALLOWED = {
    ("networkx.classes.graph", "Graph"): "Graph",
    ("networkx.classes.digraph", "DiGraph"): "DiGraph",
    ("numpy._core.multiarray", "_reconstruct"): "_reconstruct",
    ("numpy.core.multiarray", "_reconstruct"): "_reconstruct",
    ("numpy", "ndarray"): "ndarray",
    ("numpy", "dtype"): "dtype",
}
# networkx caches its view objects (G.nodes, G.edges, G.adj ...) in the
# graph's __dict__ and some of the pickles carry them; they are views of the
# graph's own dicts, so they are kept as inert symbols and never read
VIEWS = {"NodeView", "NodeDataView", "EdgeView", "OutEdgeView", "InEdgeView", "EdgeDataView",
         "OutEdgeDataView", "DegreeView", "DiDegreeView", "AdjacencyView", "AtlasView", "FilterAtlas"}


class Sym:
    """A symbolic stand-in for an object the pickle would construct."""

    def __init__(self, kind, args=None):
        self.kind, self.args, self.state = kind, args, None


class _Mark:
    pass


MARK = _Mark()


def read_pickle_graph(path: str) -> dict:
    data = open(path, "rb").read()
    stack: list = []
    memo: list = []

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(MARK)
        elif name == "MEMOIZE":
            memo.append(stack[-1])
        elif name in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "SHORT_BINBYTES", "BINBYTES", "BININT", "BININT1",
                      "BININT2", "BINFLOAT", "LONG1"):
            stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(name[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif name == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif name == "STACK_GLOBAL":
            nm = stack.pop()
            mod = stack.pop()
            if mod in ("networkx.classes.reportviews", "networkx.classes.coreviews") and nm in VIEWS:
                stack.append(Sym("class:view:" + nm))
                continue
            if (mod, nm) not in ALLOWED:
                raise ValueError(f"{path}: global {mod}.{nm} is not on the allow-list")
            stack.append(Sym("class:" + ALLOWED[(mod, nm)]))
        elif name == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            if isinstance(cls, Sym) and cls.kind.startswith("class:view:"):
                stack.append(Sym(cls.kind[6:]))
                continue
            if not (isinstance(cls, Sym) and cls.kind in ("class:Graph", "class:DiGraph")) or args != ():
                raise ValueError(f"{path}: NEWOBJ of {getattr(cls, 'kind', cls)}")
            stack.append(Sym(cls.kind[6:]))
        elif name == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, Sym):
                raise ValueError(f"{path}: REDUCE of a non-global")
            if fn.kind == "class:_reconstruct":
                if not (isinstance(args[0], Sym) and args[0].kind == "class:ndarray"):
                    raise ValueError(f"{path}: _reconstruct of {args[0]}")
                stack.append(Sym("ndarray"))
            elif fn.kind == "class:dtype":
                stack.append(Sym("dtype", args))
            else:
                raise ValueError(f"{path}: REDUCE of {fn.kind}")
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Sym):
                raise ValueError(f"{path}: BUILD on {type(obj)}")
            if obj.kind == "ndarray":  # (version, shape, dtype, is_fortran, raw bytes)
                _ver, shape, dt, fortran, raw = state
                if fortran:
                    raise ValueError(f"{path}: Fortran-ordered array")
                # kept inside the Sym: the memo may hold the same object
                obj.state = np.frombuffer(raw, dtype=_dtype_of(dt)).reshape(shape).copy()
            elif obj.kind == "dtype":  # (3, byteorder, ...)
                obj.state = state
            elif obj.kind in ("Graph", "DiGraph") or obj.kind.startswith("view:"):
                obj.state = state
            else:
                raise ValueError(f"{path}: BUILD on {obj.kind}")
        else:
            raise ValueError(f"{path}: opcode {name} is not supported")
    if len(stack) != 1 or not (isinstance(stack[0], Sym) and stack[0].kind in ("Graph", "DiGraph")):
        raise ValueError(f"{path}: the pickle is not a single networkx graph")
    return {"kind": stack[0].kind, **stack[0].state}


def _dtype_of(dt) -> np.dtype:
    if not (isinstance(dt, Sym) and dt.kind == "dtype"):
        raise ValueError(f"array dtype {dt}")
    code = dt.args[0]
    order = dt.state[1] if dt.state else "="
    return np.dtype((order if order in "<>" else "") + code)


def _json_value(v):
    if isinstance(v, Sym) and v.kind == "ndarray" and isinstance(v.state, np.ndarray):
        v = v.state
    if isinstance(v, np.ndarray):
        return {"__ndarray__": v.reshape(-1).tolist(), "dtype": v.dtype.str, "shape": list(v.shape)}
    if isinstance(v, dict):
        return {str(k): _json_value(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_json_value(x) for x in v]
    if isinstance(v, (np.floating, np.integer)):
        return v.item()
    if isinstance(v, float) and v != v:
        return None
    if isinstance(v, Sym):
        raise ValueError(f"unresolved {v.kind} in graph data")
    return v


def to_json(g: dict) -> dict:
    out = {"kind": g["kind"], "graph": _json_value(g.get("graph", {})),
           "nodes": [[n, _json_value(a)] for n, a in g["_node"].items()]}
    adj = g.get("_adj", g.get("_succ"))
    out["adj"] = [[u, [[v, _json_value(a)] for v, a in nb.items()]] for u, nb in adj.items()]
    if g["kind"] == "DiGraph":
        out["pred"] = [[u, [[v, _json_value(a)] for v, a in nb.items()]] for u, nb in g["_pred"].items()]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", default="Town01")
    a = ap.parse_args()
    src = os.path.join(REF, a.map)
    os.makedirs(OUT, exist_ok=True)
    prefix = a.map.lower()
    # the graphs PlannerManager loads (scene_generator.py:17-41)
    for fn in (f"{prefix}.pkl", f"{prefix}-vehicles-100.pkl", f"{prefix}-vehicles-2lanes-100.pkl",
               f"{prefix}-vehicles-right-100.pkl", f"{prefix}-vehicles-left-100.pkl"):
        g = read_pickle_graph(os.path.join(src, fn))
        js = to_json(g)
        dst = os.path.join(OUT, fn[:-4] + ".json")
        with open(dst, "w") as f:
            json.dump(js, f, separators=(",", ":"))
        ne = sum(len(nb) for _u, nb in js["adj"])
        print(f"{fn}: {js['kind']} {len(js['nodes'])} nodes, {ne} adjacency entries -> {dst}")


if __name__ == "__main__":
    main()
