"""Scalar coord-sim oracle: SimPy-semantics DES + default plugins + readers."""
from .engine import Environment, NORMAL, URGENT
from .reader import (Topology, get_config, get_sf, get_sfc, get_trace, load_topology, network_builder,
                     network_diameter, read_network, topology_from_graph)
from .simulator import Simulator
from .dummy import DummySimulator

__all__ = ["Environment", "NORMAL", "URGENT", "Topology", "get_config", "get_sf", "get_sfc", "get_trace",
           "load_topology", "network_builder", "network_diameter", "read_network", "topology_from_graph",
           "Simulator", "DummySimulator"]
