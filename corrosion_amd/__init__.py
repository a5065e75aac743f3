"""corrosion_amd — MI355X-native batched CRDT merge engine for Corrosion's apply hot path.

Product code: the HIP/C++ library libcorro_hip.so (csrc/, C ABI in include/corro_hip.h) and thin
Python mirrors of the reference interfaces it replaces:
  engine.MergeEngine        cr-sqlite `crsql_changes` merge (util.rs:1222-1262)
  sync.SyncStateV1          compute_available_needs (corro-types/src/sync.rs:127-249)
  bookkeeping.BookedVersions gap bookkeeping (corro-types/src/agent.rs:1108-1235)
"""
from ._lib import CorroError, device_count, lib  # noqa: F401
from .bookkeeping import BookedVersions  # noqa: F401
from .engine import MergeEngine  # noqa: F401
from .sync import Full, Partial, SyncStateV1, batch_compute_available_needs  # noqa: F401
from . import agent  # noqa: F401
