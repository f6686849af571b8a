"""Graph topology for the oracle -- TEST ORACLE (self-contained).

Restates reference model/graph.py:11-38 (node typing: input if id < every
neighbour, output if id > every neighbour, inputs = lower-id neighbours in
adjacency order).  Graphs are read from the repo's JSON adjacency files
(``graphs/nodes_*_seed_42/stage_{s}.json``) which tests pin against the
reference's gpickles.
"""
from __future__ import annotations

import collections
import json
from typing import List, Sequence

Node = collections.namedtuple('Node', ['id', 'node_type', 'inputs'])


class Adjacency:
    def __init__(self, adj: Sequence[Sequence[int]]):
        self.adj = [list(a) for a in adj]

    def number_of_nodes(self):
        return len(self.adj)

    def neighbors(self, i):
        return iter(self.adj[i])


def load_json(path: str) -> Adjacency:
    with open(path) as f:
        return Adjacency(json.load(f)['adj'])


def graph_info(g):
    nodes, ins, outs = [], [], []
    for i in range(g.number_of_nodes()):
        nb = list(g.neighbors(i))
        kind = 'intermediate'
        if i < min(nb):
            kind = 'input'
            ins.append(i)
        elif i > max(nb):
            kind = 'output'
            outs.append(i)
        nodes.append(Node(i, kind, [n for n in nb if n < i]))
    return nodes, ins, outs
