"""accord_deps — MI355X-native batched dependency resolution for Accord PreAccept/Accept.

The compute path is libaccord_deps.so (hand-written HIP for gfx950 behind the C ABI in
include/accord_deps.h). This package is the host-side harness: ctypes bindings
(``native``), the SoA data model (``model``), synthetic workloads (``synth``) and the
multi-GPU sharding/exchange (``dist``).
"""
from . import _abi, model, synth  # noqa: F401

__all__ = ["_abi", "model", "synth"]
