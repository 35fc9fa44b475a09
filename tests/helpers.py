"""Shared test helpers: golden-fixture objects and one-cluster encodings that
both the product and the oracle read."""
from __future__ import annotations

import json
import os

import numpy as np

from spotplanner import capi
from spotplanner.model import Container, Interner, Node, Pod, encode_cluster

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_tests.json")


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def fixture_pod(d) -> Pod:
    return Pod(name=d["name"], namespace=d.get("namespace", "kube-system"),
               containers=[Container(cpu_milli=d["cpu_milli"])], priority=d.get("priority", 0))


def fixture_node(d) -> Node:
    return Node(name=d["name"], cpu_milli=d["cpu_milli"], memory=d["memory"], pods=d["pods"],
                labels=dict(d.get("labels", {})))


class Scenario:
    """Spot nodes (in NodeInfoArray order) with their pods, plus extra
    "query" pods (unbound), encoded as ONE cluster."""

    def __init__(self, spot_nodes, spot_pods, query_pods, interner=None, volumes=None, stamps=None):
        self.interner = interner or Interner()
        self.nodes = list(spot_nodes)
        self.spot_pods = [list(ps) for ps in spot_pods]
        self.query = list(query_pods)
        pods, pod_node = [], []
        for i, ps in enumerate(self.spot_pods):
            pods.extend(ps)
            pod_node.extend([i] * len(ps))
        self.q0 = len(pods)
        pods.extend(self.query)
        pod_node.extend([-1] * len(self.query))
        self.enc = encode_cluster(self.nodes, pods, self.interner, pod_node=pod_node, volumes=volumes, stamps=stamps)
        self.spot = np.arange(len(self.nodes), dtype=np.int32)
        off = np.zeros(len(self.nodes) + 1, np.int32)
        for i, ps in enumerate(self.spot_pods):
            off[i + 1] = off[i] + len(ps)
        self.node_pod_off = off
        self.node_pod_idx = np.arange(self.q0, dtype=np.int32)

    @property
    def ptr(self):
        return self.enc.ptr

    def qidx(self, i):
        return self.q0 + i

    def oracle_snapshot(self):
        from oracle_lib import OracleSnapshot
        return OracleSnapshot(self.ptr, self.spot, self.node_pod_off, self.node_pod_idx)

    def product_snapshot(self):
        import ctypes
        lib = capi.load_planner()
        h = ctypes.c_void_p()
        st = lib.sr_snapshot_create(self.ptr, capi.ptr(self.spot, capi.P32), len(self.spot),
                                    capi.ptr(self.node_pod_off, capi.P32), capi.ptr(self.node_pod_idx, capi.P32),
                                    ctypes.byref(h))
        assert st == capi.SR_OK
        return h


def header_functions():
    """Every function include/sr_planner.h declares."""
    import re
    with open(capi.HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:sr_status|void|int32_t|const char \*)\s*(sr_\w+)\s*\(", text, re.M)))
