"""Random-graph topology for the encoder stages (host side, no GPU work).

Mirrors the reference's ``model/graph.py`` API:

* ``Node`` namedtuple                       -- reference ``model/graph.py:8``
* ``get_graph_info(graph)``                 -- reference ``model/graph.py:11-38``
* ``build_graph(nodes, k, p, seed)``        -- reference ``model/graph.py:41-44``
* ``save_graph(graph, path)``               -- reference ``model/graph.py:47-49``
* ``load_graph(path)``                      -- reference ``model/graph.py:52-54``

The reference loads ``.gpickle`` files with ``nx.read_gpickle`` (removed in
networkx >= 3.0).  Unpickling files is not acceptable here, so
``load_graph`` reads such files with a *disassembling* reader: it walks the
opcode stream with ``pickletools.genops`` and evaluates only the container
opcodes (dicts, ints, strings, memo), never importing or calling anything.
The only object construction a networkx ``Graph`` pickle contains is
``Graph.__new__`` + ``BUILD`` of its ``__dict__``; we rebuild that as a plain
:class:`AdjacencyGraph` with the same neighbour *order*, which is what the
predecessor lists (and therefore the F3 weight mapping) depend on.

Our own graph files are JSON (``stage_{i}.json``): ``{"adj": [[nbrs of 0], ...]}``.
"""
from __future__ import annotations

import collections
import json
import os
import pickletools
from typing import Dict, List, Optional, Sequence, Tuple

# Definition for a Node type used in NodeBlock and GraphBlock modules
# (reference model/graph.py:8).
Node = collections.namedtuple('Node', ['id', 'node_type', 'inputs'])


class AdjacencyGraph:
    """Minimal undirected graph with ordered adjacency (networkx-compatible
    subset: ``number_of_nodes`` / ``neighbors`` / ``edges``)."""

    def __init__(self, adjacency: Sequence[Sequence[int]]) -> None:
        self.adj: List[List[int]] = [list(map(int, a)) for a in adjacency]

    def number_of_nodes(self) -> int:
        return len(self.adj)

    def neighbors(self, i: int):
        return iter(self.adj[i])

    def edges(self) -> List[Tuple[int, int]]:
        return [(i, j) for i, a in enumerate(self.adj) for j in a if i < j]

    def to_json(self) -> str:
        return json.dumps({'adj': self.adj})

    def __eq__(self, other) -> bool:
        return isinstance(other, AdjacencyGraph) and self.adj == other.adj

    def __repr__(self) -> str:
        return f'AdjacencyGraph({self.adj})'


def _as_adjacency(graph) -> AdjacencyGraph:
    if isinstance(graph, AdjacencyGraph):
        return graph
    n = graph.number_of_nodes()
    return AdjacencyGraph([list(graph.neighbors(i)) for i in range(n)])


def get_graph_info(graph) -> Tuple[List[Node], List[int], List[int]]:
    """Node typing of reference ``model/graph.py:11-38``.

    A node is an *input* if its id is below every neighbour, an *output* if it
    is above every neighbour; its inputs are the lower-id neighbours **in
    adjacency order** (this order feeds the F3 sigmoid-weight mapping).
    """
    inputs, outputs, nodes = [], [], []
    g = _as_adjacency(graph)
    for i in range(g.number_of_nodes()):
        nbrs = list(g.neighbors(i))
        node_type = 'intermediate'
        if i < min(nbrs):
            inputs.append(i)
            node_type = 'input'
        elif i > max(nbrs):
            outputs.append(i)
            node_type = 'output'
        nodes.append(Node(i, node_type, [n for n in nbrs if n < i]))
    return nodes, inputs, outputs


def build_graph(nodes: int, k: int, p: float,
                seed: Optional[int] = None) -> AdjacencyGraph:
    """Connected Watts-Strogatz graph (reference ``model/graph.py:41-44``).

    The RNG is networkx's; networkx is only needed when a graph is generated
    rather than loaded."""
    import networkx as nx  # host-only dependency, import lazily
    return _as_adjacency(nx.connected_watts_strogatz_graph(nodes, k, p,
                                                           seed=seed))


def save_graph(graph, path: str) -> None:
    """Save as JSON (our format; reference writes gpickle, ``graph.py:47``)."""
    if path.endswith('.gpickle'):
        path = path[:-len('.gpickle')] + '.json'
    with open(path, 'w') as f:
        f.write(_as_adjacency(graph).to_json())


# --------------------------------------------------------------------------
# Safe gpickle reader: evaluates container opcodes only.
# --------------------------------------------------------------------------
# Names a networkx Graph pickle references.  They are recorded as inert
# placeholders; nothing is imported or instantiated.
_ALLOWED_GLOBALS = {('networkx.classes.graph', 'Graph'),
                    ('networkx.classes.reportviews', 'DegreeView'),
                    ('networkx.classes.coreviews', 'AdjacencyView')}
_MARK = object()


class _Obj(dict):
    """Placeholder for the single allowed object (a Graph's __dict__)."""


def _read_gpickle_adjacency(path: str) -> AdjacencyGraph:
    with open(path, 'rb') as f:
        data = f.read()
    stack: list = []
    memo: Dict[int, object] = {}

    def pop_mark():
        items = []
        while True:
            x = stack.pop()
            if x is _MARK:
                return items[::-1]
            items.append(x)

    result = None
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ('PROTO', 'FRAME'):
            continue
        elif name in ('SHORT_BINUNICODE', 'BINUNICODE', 'UNICODE',
                      'SHORT_BINSTRING', 'BINSTRING'):
            stack.append(arg)
        elif name in ('BININT', 'BININT1', 'BININT2', 'INT', 'LONG1'):
            stack.append(int(arg))
        elif name in ('BINFLOAT', 'FLOAT'):
            stack.append(float(arg))
        elif name == 'NONE':
            stack.append(None)
        elif name in ('NEWTRUE', 'NEWFALSE'):
            stack.append(name == 'NEWTRUE')
        elif name == 'MEMOIZE':
            memo[len(memo)] = stack[-1]
        elif name in ('BINPUT', 'LONG_BINPUT', 'PUT'):
            memo[int(arg)] = stack[-1]
        elif name in ('BINGET', 'LONG_BINGET', 'GET'):
            stack.append(memo[int(arg)])
        elif name == 'MARK':
            stack.append(_MARK)
        elif name == 'EMPTY_DICT':
            stack.append({})
        elif name == 'EMPTY_LIST':
            stack.append([])
        elif name == 'EMPTY_TUPLE':
            stack.append(())
        elif name == 'SETITEMS':
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name == 'SETITEM':
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif name == 'APPENDS':
            items = pop_mark()
            stack[-1].extend(items)
        elif name == 'APPEND':
            v = stack.pop()
            stack[-1].append(v)
        elif name == 'TUPLE':
            stack.append(tuple(pop_mark()))
        elif name in ('TUPLE1', 'TUPLE2', 'TUPLE3'):
            n = int(name[-1])
            items = stack[-n:]
            del stack[-n:]
            stack.append(tuple(items))
        elif name == 'STACK_GLOBAL':
            cls = stack.pop()
            mod = stack.pop()
            if (mod, cls) not in _ALLOWED_GLOBALS:
                raise ValueError(f'{path}: refusing global {mod}.{cls}')
            stack.append(('__global__', mod, cls))
        elif name == 'NEWOBJ':
            _args = stack.pop()
            cls = stack.pop()
            if not (isinstance(cls, tuple) and cls[:1] == ('__global__',)):
                raise ValueError(f'{path}: unexpected NEWOBJ target')
            stack.append(_Obj())
        elif name == 'BUILD':
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, _Obj) or not isinstance(state, dict):
                raise ValueError(f'{path}: unexpected BUILD')
            obj.update(state)
        elif name == 'STOP':
            result = stack.pop()
            break
        else:
            raise ValueError(f'{path}: unsupported pickle opcode {name}')

    if not isinstance(result, _Obj) or '_adj' not in result:
        raise ValueError(f'{path}: not a networkx Graph pickle')
    adj = result['_adj']
    n = len(adj)
    if sorted(adj.keys()) != list(range(n)):
        raise ValueError(f'{path}: node ids are not 0..{n - 1}')
    return AdjacencyGraph([list(adj[i].keys()) for i in range(n)])


def load_graph(path: str) -> AdjacencyGraph:
    """Load a stage graph (reference ``model/graph.py:52-54``).

    Accepts our JSON files and the reference's ``.gpickle`` files (read by the
    safe opcode reader above).  A ``.gpickle`` path whose file is absent falls
    back to a sibling ``.json`` file, and vice versa.
    """
    candidates = [path]
    root, ext = os.path.splitext(path)
    if ext == '.gpickle':
        candidates.append(root + '.json')
    elif ext == '.json':
        candidates.append(root + '.gpickle')
    for cand in candidates:
        if os.path.isfile(cand):
            if cand.endswith('.json'):
                with open(cand) as f:
                    return AdjacencyGraph(json.load(f)['adj'])
            return _read_gpickle_adjacency(cand)
    raise FileNotFoundError(path)
