"""Input readers: GraphML topologies, service/SF YAML, simulator config, traces.

Behaviour mirrors ``coordsim/reader/reader.py`` (reference):

* nodes become ``pop{i}`` with ``cap=NodeCap``, ``type=NodeType`` (default
  Normal), ``available_sf={}``, ``remaining_cap`` (reader.py:163-195);
* link delay = ``LinkDelay`` if present, else the WGS-84 distance converted to
  integer milliseconds at 0.77 c, else 3 (reader.py:199-227);
* link ``cap = LinkFwdCap`` (default 1000), ``weight = 1/(cap + 1/delay)``
  (reader.py:114-126) and all-pairs shortest paths by Johnson's algorithm
  stored as ``graph['shortest_paths'][(s, d)] = (path, delay)`` (reader.py:136-160);
* ``get_sf`` fills processing-delay/startup defaults and loads pluggable
  resource functions from ``<path>/<id>.py`` (falling back to identity).

It additionally exports :class:`Topology`, a dense numpy description of a
network (path tables, capacities, ingress list) consumed by the batched HIP
simulator.
"""
from __future__ import annotations

import csv
import importlib.util
import logging
import math
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import networkx as nx
import numpy as np
import yaml

from .geodesic import distance_m

log = logging.getLogger(__name__)

SPEED_OF_LIGHT = 299792458.0
PROPAGATION_FACTOR = 0.77


def get_trace(trace_file: str) -> List[dict]:
    with open(trace_file) as f:
        return [dict(row) for row in csv.DictReader(f)]


def get_config(config_file: str) -> dict:
    with open(config_file) as f:
        return yaml.safe_load(f)


def get_sfc(sfc_file: str) -> Dict[str, List[str]]:
    with open(sfc_file) as f:
        data = yaml.safe_load(f)
    sfc_list = defaultdict(None)
    for name, sfs in data["sfc_list"].items():
        sfc_list[name] = list(sfs)
    return sfc_list


def _identity(x):
    return x


def load_resource_function(name: str, path: str):
    spec = importlib.util.spec_from_file_location(name, f"{path}/{name}.py")
    if spec is None or spec.loader is None:
        raise FileNotFoundError(f'Cannot load file "{name}.py" from "{path}".')
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    if not hasattr(module, "resource_function"):
        raise AttributeError(f'No "resource_function" defined in "{name}.py".')
    return module.resource_function


def get_sf(sf_file: str, resource_functions_path: str = "") -> Dict[str, dict]:
    with open(sf_file) as f:
        data = yaml.safe_load(f)
    sf_list = defaultdict(None)
    for name, details in data["sf_list"].items():
        d = dict(details or {})
        d.setdefault("processing_delay_mean", 1.0)
        d.setdefault("processing_delay_stdev", 1.0)
        d.setdefault("startup_delay", 0.0)
        if "resource_function_id" in d:
            try:
                d["resource_function"] = load_resource_function(d["resource_function_id"], resource_functions_path)
            except Exception as ex:  # same fallback as the reference (reader.py:99-104)
                log.warning(f"{ex} SF {name} will use the default resource function instead.")
                d["resource_function_id"] = "default"
                d["resource_function"] = _identity
        else:
            d["resource_function_id"] = "default"
            d["resource_function"] = _identity
        sf_list[name] = d
    return sf_list


def weight(edge_cap, edge_delay):
    assert edge_delay is not None
    if edge_cap is None:
        return edge_delay
    if edge_cap == 0:
        return math.inf
    if edge_delay == 0:
        return 0
    return 1 / (edge_cap + 1 / edge_delay)


def shortest_paths(g: nx.Graph) -> None:
    apsp = dict(nx.johnson(g, weight="weight"))
    table = {}
    for src, dsts in apsp.items():
        for dst, path in dsts.items():
            d = 0
            if src != dst:
                for i in range(len(path) - 1):
                    d += g[path[i]][path[i + 1]]["delay"]
            table[(src, dst)] = (path, d)
    g.graph["shortest_paths"] = table


def network_diameter(g: nx.Graph):
    if "shortest_paths" not in g.graph:
        shortest_paths(g)
    return max(p[1] for p in g.graph["shortest_paths"].values())


def read_network(file: str, node_cap=None, link_cap=1000, force_link_cap: Optional[float] = None,
                 force_node_cap: Optional[List[float]] = None) -> Tuple[nx.Graph, list, list]:
    if not file.endswith(".graphml"):
        raise ValueError(f"{file} is not a GraphML file")
    gml = nx.read_graphml(file, node_type=int)
    g = nx.Graph()
    for nid, attrs in gml.nodes(data=True):
        cap = attrs.get("NodeCap", None)
        if cap is None:
            cap = node_cap
            log.warning(f"NodeCap not set for node {nid}; using default {node_cap}")
        if force_node_cap is not None:
            cap = np.random.randint(force_node_cap[0], force_node_cap[1])
        if cap is None:
            raise ValueError(f"No NodeCap for node {nid} in {file}")
        g.add_node(f"pop{nid}", name=attrs.get("label", None), type=attrs.get("NodeType", "Normal"),
                   cap=cap, available_sf={}, remaining_cap=cap)
    nodes = dict(gml.nodes(data=True))
    for u, v, attrs in gml.edges(data=True):
        link_delay = attrs.get("LinkDelay", None)
        fwd_cap = attrs.get("LinkFwdCap", link_cap)
        if force_link_cap is not None:
            fwd_cap = force_link_cap
        delay = 3
        if link_delay is None:
            a, b = nodes[u], nodes[v]
            if None not in (a.get("Latitude"), a.get("Longitude"), b.get("Latitude"), b.get("Longitude")):
                dist = distance_m(a["Latitude"], a["Longitude"], b["Latitude"], b["Longitude"])
                delay = int(np.around((dist / SPEED_OF_LIGHT * 1000) * PROPAGATION_FACTOR))
        else:
            delay = link_delay
        g.add_edge(f"pop{u}", f"pop{v}", delay=delay, cap=fwd_cap, remaining_cap=fwd_cap, run_passed_traffic=0)
    for e in g.edges.values():
        e["weight"] = weight(e["cap"], e["delay"])
    shortest_paths(g)
    ing = [(n, d) for n, d in g.nodes.items() if d["type"] == "Ingress"]
    eg = [n for n, d in g.nodes.items() if d["type"] == "Egress"]
    return g, ing, eg


def network_builder(network_file: str, config: dict):
    """``coordsim/reader/builders.py``: apply force_link_cap / force_node_cap from the sim config."""
    force_node_cap = config.get("force_node_cap", None)
    if force_node_cap is not None and not isinstance(force_node_cap, list):
        raise ValueError("force_node_cap should be a list [low, high]")
    return read_network(network_file, force_link_cap=config.get("force_link_cap", None),
                        force_node_cap=force_node_cap)


def reset_cap(g: nx.Graph) -> None:
    for n in g.nodes:
        g.nodes[n]["remaining_cap"] = g.nodes[n]["cap"]
        g.nodes[n]["available_sf"] = {}
    for _, _, d in g.edges(data=True):
        d["remaining_cap"] = d["cap"]
        d["run_passed_traffic"] = 0


def num_ingress(network_path: str) -> int:
    g = nx.read_graphml(network_path, node_type=int)
    return sum(1 for _, d in g.nodes(data=True) if d.get("NodeType") == "Ingress")


# ----------------------------------------------------------------------------------------------
# Dense topology description for the batched device simulator
# ----------------------------------------------------------------------------------------------
@dataclass
class Topology:
    """Dense arrays describing one network (node order = GraphML order, as in the reference)."""

    name: str
    node_ids: List[str]
    node_cap: np.ndarray            # [n] float64
    node_type: np.ndarray           # [n] int8: 0 normal, 1 ingress, 2 egress
    edges: np.ndarray               # [E, 2] int32 (undirected, GraphML order)
    edge_delay: np.ndarray          # [E] float64
    edge_cap: np.ndarray            # [E] float64
    edge_id: np.ndarray             # [n, n] int32 undirected edge index (-1 = no edge)
    path_delay: np.ndarray          # [n, n] float64  shortest-path delay (sum of edge delays)
    path_len: np.ndarray            # [n, n] int32    number of hops
    path_nodes: np.ndarray          # [n, n, H] int32 hop sequence excluding the source (-1 padded)
    ingress: np.ndarray             # [I] int32
    egress: np.ndarray              # [G] int32
    diameter: float = 0.0
    graph: Optional[nx.Graph] = field(default=None, repr=False)

    @property
    def n(self) -> int:
        return len(self.node_ids)

    @property
    def num_edges(self) -> int:
        return int(self.edges.shape[0])

    @property
    def max_hops(self) -> int:
        return int(self.path_nodes.shape[2])

    def edge_index(self) -> np.ndarray:
        """Bidirectional ``[2, 2E]`` edge index (PyG ``from_networkx`` ordering of an undirected graph)."""
        order = {nid: i for i, nid in enumerate(self.node_ids)}
        src, dst = [], []
        # from_networkx on an undirected graph emits both directions per adjacency entry
        g = self.graph
        for u in g.nodes:
            for v in g.adj[u]:
                src.append(order[u])
                dst.append(order[v])
        return np.asarray([src, dst], dtype=np.int64)


def topology_from_graph(g: nx.Graph, ing_nodes, eg_nodes, name: str = "") -> Topology:
    ids = list(g.nodes)
    idx = {nid: i for i, nid in enumerate(ids)}
    n = len(ids)
    cap = np.asarray([float(g.nodes[v]["cap"]) for v in ids], dtype=np.float64)
    ntype = np.zeros(n, dtype=np.int8)
    for v, _ in ing_nodes:
        ntype[idx[v]] = 1
    for v in eg_nodes:
        ntype[idx[v]] = 2
    edges, edelay, ecap = [], [], []
    eid = np.full((n, n), -1, dtype=np.int32)
    for u, v, d in g.edges(data=True):
        eid[idx[u], idx[v]] = eid[idx[v], idx[u]] = len(edges)
        edges.append((idx[u], idx[v]))
        edelay.append(float(d["delay"]))
        ecap.append(float(d["cap"]))
    sp = g.graph["shortest_paths"]
    hops = max(len(p) - 1 for p, _ in sp.values()) if sp else 0
    H = max(1, hops)
    pdelay = np.zeros((n, n), dtype=np.float64)
    plen = np.zeros((n, n), dtype=np.int32)
    pnodes = np.full((n, n, H), -1, dtype=np.int32)
    for (s, t), (path, d) in sp.items():
        i, j = idx[s], idx[t]
        pdelay[i, j] = d
        plen[i, j] = len(path) - 1
        for k, hop in enumerate(path[1:]):
            pnodes[i, j, k] = idx[hop]
    return Topology(name=name, node_ids=ids, node_cap=cap, node_type=ntype,
                    edges=np.asarray(edges, dtype=np.int32).reshape(-1, 2),
                    edge_delay=np.asarray(edelay, dtype=np.float64), edge_cap=np.asarray(ecap, dtype=np.float64),
                    edge_id=eid,
                    path_delay=pdelay, path_len=plen, path_nodes=pnodes,
                    ingress=np.asarray([idx[v] for v, _ in ing_nodes], dtype=np.int32),
                    egress=np.asarray([idx[v] for v in eg_nodes], dtype=np.int32),
                    diameter=float(pdelay.max()) if n else 0.0, graph=g)


def load_topology(network_file: str, config: Optional[dict] = None) -> Topology:
    g, ing, eg = network_builder(network_file, config or {})
    return topology_from_graph(g, ing, eg, name=network_file)
