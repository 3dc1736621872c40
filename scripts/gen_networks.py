#!/usr/bin/env python
"""Topology / trace generator.

Reference ``scripts/gen_networks.py`` (``set_new_caps`` ``:6-21``: copy a GraphML with random
``NodeCap`` in ``[min, max]``; ``set_ingress`` ``:24-38``: mark one more node as Ingress; author
paths hard-coded).  Here as a CLI, plus what BASELINE configs (4) and (5) need:

* ``synthetic`` — connected random geographic topology with N nodes (k-nearest-neighbour mesh over
  a random spanning tree), Topology-Zoo attribute names (``NodeCap``, ``NodeType``, ``Latitude``,
  ``Longitude``, ``LinkDelay``, ``LinkFwdCap``) so :func:`gsc_amd.coordsim.reader.read_network`
  reads it like any shipped network;
* ``trace`` — a ``time,node,inter_arrival_mean`` trace (reference format,
  ``configs/traces/*.csv``) with per-node random-walk rates for every ingress node;
* ``suite`` — regenerate the shipped ``configs/networks/synthetic`` set (50-node + traces, three more
  50-node variants and four 200-node variants for the scheduler-driven generalisation configs).

    python scripts/gen_networks.py caps IN OUT --min-cap 1 --max-cap 2 [--seed S]
    python scripts/gen_networks.py ingress IN OUT --node 3
    python scripts/gen_networks.py synthetic OUT --nodes 50 --ingress 8 [--degree 3] [--seed S]
    python scripts/gen_networks.py trace NETWORK OUT --duration 20000 --interval 200
    python scripts/gen_networks.py suite
"""
from __future__ import annotations

import argparse
import csv
import math
import os
import random
import sys

import networkx as nx
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def set_new_caps(network_file: str, new_network_file: str, min_cap: int, max_cap: int, rng=random) -> str:
    g = nx.read_graphml(network_file)
    for _, d in g.nodes(data=True):
        d["NodeCap"] = rng.randint(min_cap, max_cap)
    nx.write_graphml(g, new_network_file)
    return new_network_file


def set_ingress(network_file: str, new_network_file: str, ingress_id: str) -> str:
    g = nx.read_graphml(network_file)
    g.nodes[str(ingress_id)]["NodeType"] = "Ingress"
    nx.write_graphml(g, new_network_file)
    return new_network_file


def synthetic_topology(n: int, n_ingress: int, degree: int = 3, min_cap: int = 1, max_cap: int = 3,
                       link_cap: int = 1000, n_egress: int = 0, seed: int = 0, ms_per_unit: float = 8.0) -> nx.Graph:
    """Connected geographic graph: random points in the unit square, a random spanning tree
    (each node links to a random earlier node among its 4 nearest), then each node links to its
    ``degree - 1`` nearest neighbours.  ``LinkDelay`` = ceil(euclidean distance * ms_per_unit)."""
    rs = np.random.RandomState(seed)
    pts = rs.rand(n, 2)
    d = np.sqrt(((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1))
    g = nx.Graph(Network=f"synthetic-n{n}-s{seed}")
    for i in range(n):
        g.add_node(str(i), id=i, label=f"n{i}", Latitude=float(25 + 25 * pts[i, 1]),
                   Longitude=float(-125 + 55 * pts[i, 0]), NodeCap=int(rs.randint(min_cap, max_cap + 1)),
                   NodeType="Normal", Internal=1)
    order = rs.permutation(n)
    for k in range(1, n):
        v = order[k]
        prev = order[:k]
        near = prev[np.argsort(d[v, prev])[:4]]
        u = near[rs.randint(len(near))]
        g.add_edge(str(v), str(u))
    for v in range(n):
        for u in np.argsort(d[v])[1:degree]:
            g.add_edge(str(v), str(int(u)))
    for u, v in g.edges:
        g.edges[u, v]["LinkDelay"] = int(max(1, math.ceil(d[int(u), int(v)] * ms_per_unit)))
        g.edges[u, v]["LinkFwdCap"] = int(link_cap)
    nodes = list(rs.permutation(n))
    for v in nodes[:n_ingress]:
        g.nodes[str(v)]["NodeType"] = "Ingress"
    for v in nodes[n_ingress:n_ingress + n_egress]:
        g.nodes[str(v)]["NodeType"] = "Egress"
    assert nx.is_connected(g)
    return g


def make_trace(network_file: str, out_csv: str, duration_ms: int = 20000, interval_ms: int = 200,
               base: float = 12.0, spread: float = 0.5, seed: int = 0) -> str:
    """Per-ingress random-walk inter-arrival means (log-space), one row per node every interval."""
    g = nx.read_graphml(network_file)
    ing = [v for v, dd in g.nodes(data=True) if dd.get("NodeType") == "Ingress"]
    ids = {v: f"pop{i}" for i, v in enumerate(g.nodes)}
    rs = np.random.RandomState(seed)
    level = {v: 0.0 for v in ing}
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["time", "node", "inter_arrival_mean"])
        for t in range(0, duration_ms, interval_ms):
            for v in ing:
                level[v] = float(np.clip(level[v] + rs.normal(0, spread / 4), -spread * 2, spread * 2))
                w.writerow([t, ids[v], round(base * math.exp(level[v]), 3)])
    return out_csv


def suite() -> None:
    out = os.path.join(ROOT, "configs", "networks", "synthetic")
    os.makedirs(out, exist_ok=True)
    n50 = os.path.join(out, "syn50-in8-cap1-3.graphml")
    nx.write_graphml(synthetic_topology(50, 8, degree=3, seed=50), n50)
    make_trace(n50, os.path.join(ROOT, "configs", "traces", "trace_syn50_in8.csv"), seed=50)
    for s in range(1, 4):  # 50-node variants for the scheduler / held-out generalisation runs (scripts/generalize.py)
        nx.write_graphml(synthetic_topology(50, 8, degree=3, seed=100 + s),
                         os.path.join(out, f"syn50-in8-cap1-3-s{s}.graphml"))
    for s in range(4):
        nx.write_graphml(synthetic_topology(200, 16, degree=3, seed=200 + s, ms_per_unit=6.0),
                         os.path.join(out, f"syn200-in16-cap1-3-s{s}.graphml"))
    print(f"wrote {out}")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("caps")
    c.add_argument("src")
    c.add_argument("dst")
    c.add_argument("--min-cap", type=int, required=True)
    c.add_argument("--max-cap", type=int, required=True)
    c.add_argument("--seed", type=int, default=None)
    i = sub.add_parser("ingress")
    i.add_argument("src")
    i.add_argument("dst")
    i.add_argument("--node", required=True)
    s = sub.add_parser("synthetic")
    s.add_argument("dst")
    s.add_argument("--nodes", type=int, required=True)
    s.add_argument("--ingress", type=int, default=4)
    s.add_argument("--egress", type=int, default=0)
    s.add_argument("--degree", type=int, default=3)
    s.add_argument("--min-cap", type=int, default=1)
    s.add_argument("--max-cap", type=int, default=3)
    s.add_argument("--seed", type=int, default=0)
    t = sub.add_parser("trace")
    t.add_argument("network")
    t.add_argument("dst")
    t.add_argument("--duration", type=int, default=20000)
    t.add_argument("--interval", type=int, default=200)
    t.add_argument("--base", type=float, default=12.0)
    t.add_argument("--seed", type=int, default=0)
    sub.add_parser("suite")
    a = ap.parse_args(argv)
    if a.cmd == "caps":
        set_new_caps(a.src, a.dst, a.min_cap, a.max_cap, random.Random(a.seed))
    elif a.cmd == "ingress":
        set_ingress(a.src, a.dst, a.node)
    elif a.cmd == "synthetic":
        nx.write_graphml(synthetic_topology(a.nodes, a.ingress, a.degree, a.min_cap, a.max_cap, n_egress=a.egress,
                                            seed=a.seed), a.dst)
    elif a.cmd == "trace":
        make_trace(a.network, a.dst, a.duration, a.interval, a.base, seed=a.seed)
    else:
        suite()


if __name__ == "__main__":
    sys.exit(main())
