"""spotplanner — MI355X drain planner for k8s-spot-rescheduler's hot path.

Python face of libsrplanner.so (C-ABI: include/sr_planner.h).  Module layout
mirrors the reference: `nodes` (nodes/nodes.go), `rescheduler`
(rescheduler.go planning functions), `planner` (predicate checker + cluster
snapshot handles), `model` (Pod / Node objects + the shim's encoding).
"""
from . import capi, model  # noqa: F401

__all__ = ["capi", "model", "nodes", "planner", "rescheduler", "synth"]
