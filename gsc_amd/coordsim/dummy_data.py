"""Placements / schedules for running the simulator without an agent.

Reference ``coordsim/network/dummy_data.py`` holds literal dicts (``placement``,
``triangle_placement``, ``schedule``, ``triangle_schedule``) for the 3-node networks used by the
stand-alone CLI.  Here they are generated for any network + SFC list:

* ``chain_placement``: SF k of every chain on node ``k mod n`` (the triangle layout for n = 3:
  pop0 -> a, pop1 -> b, pop2 -> c);
* ``chain_schedule``: every node sends SF k to node ``k mod n`` (deterministic, follows the
  placement above);
* ``uniform_schedule`` / ``full_placement``: every node sends every SF to every node with equal
  weight (all SFs everywhere) — the fixed policy of the golden rows in SURVEY §4;
* ``local_schedule``: every SF is processed where the flow currently is.
"""
from __future__ import annotations

from typing import Dict, List


def _sfs(sfc_list: Dict[str, List[str]]) -> List[str]:
    out: List[str] = []
    for chain in sfc_list.values():
        for sf in chain:
            if sf not in out:
                out.append(sf)
    return out


def chain_placement(nodes: List[str], sfc_list) -> Dict[str, List[str]]:
    pl = {v: [] for v in nodes}
    for chain in sfc_list.values():
        for k, sf in enumerate(chain):
            v = nodes[k % len(nodes)]
            if sf not in pl[v]:
                pl[v].append(sf)
    return pl


def full_placement(nodes: List[str], sfc_list) -> Dict[str, List[str]]:
    return {v: list(_sfs(sfc_list)) for v in nodes}


def _schedule(nodes, sfc_list, weight) -> dict:
    return {src: {c: {sf: {dst: weight(src, k, dst) for dst in nodes} for k, sf in enumerate(chain)}
                  for c, chain in sfc_list.items()} for src in nodes}


def chain_schedule(nodes: List[str], sfc_list) -> dict:
    return _schedule(nodes, sfc_list, lambda src, k, dst: 1.0 if dst == nodes[k % len(nodes)] else 0.0)


def uniform_schedule(nodes: List[str], sfc_list) -> dict:
    return _schedule(nodes, sfc_list, lambda src, k, dst: 1.0 / len(nodes))


def local_schedule(nodes: List[str], sfc_list) -> dict:
    return _schedule(nodes, sfc_list, lambda src, k, dst: 1.0 if dst == src else 0.0)


POLICIES = {
    "chain": (chain_placement, chain_schedule),
    "uniform": (full_placement, uniform_schedule),
    "local": (full_placement, local_schedule),
}
