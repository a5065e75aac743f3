"""ctypes binding of libcorro_hip.so (the C ABI declared in include/corro_hip.h).

The product path has exactly one implementation: the HIP library. There is no CPU fallback;
loading fails loudly if the library is missing, and compute calls fail with CORRO_E_NO_DEVICE
when no gfx950 device is visible.
"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# CORRO_HIP_LIB: an alternative build of the same library (diagnostic variants, tools/)
LIB_PATH = os.environ.get("CORRO_HIP_LIB") or os.path.join(HERE, "libcorro_hip.so")

CORRO_OK = 0
ERRORS = {-1: "CORRO_E_INVALID", -2: "CORRO_E_NOMEM", -3: "CORRO_E_DEVICE",
          -4: "CORRO_E_UNKNOWN_TABLE", -5: "CORRO_E_UNKNOWN_COLUMN", -6: "CORRO_E_RANGE",
          -7: "CORRO_E_NO_DEVICE"}
CORRO_MEM_HOST, CORRO_MEM_DEVICE, CORRO_MEM_DEVICE_HEADERS = 0, 1, 2
CORRO_PAYLOAD_SYNC, CORRO_PAYLOAD_UNI = 0, 1

# every symbol include/corro_hip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "corro_last_error", "corro_abi_version", "corro_device_count", "corro_ctx_create",
    "corro_ctx_destroy", "corro_lookup_cid", "corro_site_register", "corro_site_count",
    "corro_apply_batch", "corro_state_count", "corro_state_export", "corro_state_reset",
    "corro_db_versions", "corro_value_bytes", "corro_compute_needs", "corro_booked_new", "corro_booked_free",
    "corro_booked_insert_db", "corro_booked_needed", "corro_booked_last", "corro_booked_contains",
    "corro_booked_contains_all", "corro_ctx_set_profiling", "corro_last_timings",
    "corro_bookie_new", "corro_bookie_free", "corro_process_multiple_changes",
    "corro_bookie_take_ready", "corro_process_fully_buffered", "corro_bookie_last",
    "corro_bookie_needed", "corro_bookie_contains_all", "corro_bookie_partial",
    "corro_generate_sync", "corro_partition_ranks", "corro_scan_offsets",
    "corro_compute_needs_onepass", "corro_needs_bound", "corro_extract_changes",
    "corro_bookie_seq_bookkeeping", "corro_bookie_buffered", "corro_bookie_buffered_versions",
    "corro_decode_frames", "corro_site_ids", "corro_packed_record_bytes", "corro_partition_packed",
    "corro_unpack_records", "corro_partition_slots", "corro_unpack_slots", "corro_apply_mapped", "corro_ctx_stream",
    "corro_apply_slots", "corro_slots_flags_back",
    "corro_table_set_pk_interned", "corro_pk_keys", "corro_pk_keys_device", "corro_pk_bytes",
    "corro_pk_canonical", "corro_bookie_buffered_value", "corro_compute_needs_packed",
    "corro_booked_insert_db_batch", "corro_affinity_of_type", "corro_table_set_affinity", "corro_set_affinity_policy",
    "corro_ctx_metrics", "corro_table_committed", "corro_ctx_track_touched", "corro_state_export_touched",
    "corro_ctx_set_store_limit", "corro_partition_var", "corro_unpack_var",
]

CORRO_CS_FULL, CORRO_CS_EMPTY, CORRO_CS_EMPTY_SET = 0, 1, 2
KNOWN = {0: "skipped", 1: "current", 2: "cleared", 3: "partial"}
CORRO_TCID_UNKNOWN = 0xFFFFFFFF
CORRO_VAL_LONG = 255  # val_len of a TEXT/BLOB value longer than 16 bytes


class CorroError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class TableDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ncols", C.c_uint32), ("col_names", C.POINTER(C.c_char_p))]


class Changes(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.c_void_p) for k in (
        "pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "val0", "val1",
        "val_type", "val_len", "ts", "val_off", "val_size", "val_data")] + [("val_data_len", C.c_uint64)]


class ApplyOut(C.Structure):
    _fields_ = [("impact", C.c_void_p)]


class Rows(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("pk", "table_cid", "col_version", "db_version", "cl",
                                          "seq", "site", "ts", "val0", "val1", "val_type",
                                          "val_len")]


class SyncEntries(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.c_void_p) for k in (
        "their_head", "our_head", "tn_off", "tn_start", "tn_end", "tp_off", "tp_ver", "tps_off",
        "tps_start", "tps_end", "on_off", "on_start", "on_end", "op_off", "op_ver", "ops_off",
        "ops_start", "ops_end")]


class ExtractIn(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.c_void_p) for k in ("site", "start", "end", "seq_start", "seq_end")]


class ExtractOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("grp_count", "row_count", "grp_off", "row_off", "version", "last_seq",
                                          "ts", "grp_row_off", "grp_rows")] + [("rows", Rows)]


class Metrics(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("applies", "changes", "overflow_rounds", "deferred_rounds",
                                          "region_growths", "heap_growths", "state_rows", "state_records",
                                          "max_batch")] + [("apply_seconds", C.c_double), ("arena_bytes", C.c_uint64),
                                                                   ("aff_sensitive", C.c_uint64)]


class GapsIn(C.Structure):
    _fields_ = [("n", C.c_uint64)] + [(k, C.c_void_p) for k in ("max", "gap_off", "gap_start", "gap_end",
                                                                 "ver_off", "ver_start", "ver_end")]


class GapsOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("max", "rm_count", "ins_count", "gap_count", "rm_start", "rm_end",
                                          "ins_start", "ins_end", "new_start", "new_end", "status")]


class NeedsPackedOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("need_off", "need_count", "range", "kind", "s_start", "s_end")]


class NeedsOut(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("need_count", "seq_count", "need_off", "seq_off", "kind",
                                          "start", "end", "sr_off", "sr_n", "s_start", "s_end")]


class Changeset(C.Structure):
    _fields_ = [("actor_id", C.c_void_p), ("site", C.c_uint32), ("kind", C.c_uint32),
                ("version_start", C.c_uint64), ("version_end", C.c_uint64), ("seq_start", C.c_uint64),
                ("seq_end", C.c_uint64), ("last_seq", C.c_uint64), ("ts", C.c_uint64),
                ("change_off", C.c_uint64), ("change_count", C.c_uint64)]


class Decoded(C.Structure):
    _fields_ = [("nframes", C.c_uint64), ("nchanges", C.c_uint64), ("nsets", C.c_uint64), ("cs", C.c_void_p),
                ("actor_ids", C.c_void_p), ("status", C.c_void_p), ("changes", Changes), ("set_start", C.c_void_p),
                ("set_end", C.c_void_p), ("cs_dev", C.c_void_p), ("n_dev", C.c_uint64)]


class ProcessOut(C.Structure):
    _fields_ = [("known", C.c_void_p), ("impactful", C.c_void_p), ("n_ready", C.c_uint64)]


class SyncState(C.Structure):
    _fields_ = [("n_actors", C.c_uint64), ("n_need", C.c_uint64), ("n_partials", C.c_uint64),
                ("n_pseqs", C.c_uint64)] + [(k, C.c_void_p) for k in (
        "actor_ids", "heads", "need_off", "need_start", "need_end", "partial_off", "partial_ver",
        "pseq_off", "pseq_start", "pseq_end")]


_lib = None


def _torch_runtime_first():
    """The PyTorch-ROCm wheel bundles its own HIP/HSA runtime (torch/lib/libamdhip64.so, no
    soname) next to the system one libcorro_hip.so links (libamdhip64.so.7), so a process that
    uses both holds two runtimes. They coexist when PyTorch initialises the device first (device
    pointers are process-wide KFD addresses), but PyTorch cannot find the device once the other
    runtime has initialised it. So when PyTorch is installed it is imported and initialises the
    device first; C callers of the library never load it."""
    import importlib.util
    if "torch" not in sys.modules and importlib.util.find_spec("torch") is None:
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # noqa: BLE001 -- torch is an optional neighbour, never a requirement
        pass


def lib():
    """Load the in-tree libcorro_hip.so. Raises if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -m corrosion_amd.build` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    _torch_runtime_first()
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    sig = {
        "corro_last_error": (C.c_char_p, []),
        "corro_abi_version": (i32, []),
        "corro_value_bytes": (i32, [vp, vp, u64, vp, u64, vp]),
        "corro_device_count": (i32, [vp]),
        "corro_ctx_create": (i32, [vp, u32, u64, i32, vp]),
        "corro_ctx_destroy": (None, [vp]),
        "corro_lookup_cid": (i32, [vp, C.c_char_p, C.c_char_p, vp]),
        "corro_site_register": (i32, [vp, vp, u64, vp]),
        "corro_site_count": (i32, [vp, vp]),
        "corro_apply_batch": (i32, [vp, C.POINTER(Changes), i32, C.POINTER(ApplyOut)]),
        "corro_state_count": (i32, [vp, vp]),
        "corro_state_export": (i32, [vp, C.POINTER(Rows), u64, vp]),
        "corro_state_export_touched": (i32, [vp, C.POINTER(Rows), u64, vp]),
        "corro_ctx_track_touched": (i32, [vp, i32]),
        "corro_ctx_set_store_limit": (i32, [vp, u64]),
        "corro_state_reset": (i32, [vp]),
        "corro_db_versions": (i32, [vp, vp, u32]),
        "corro_compute_needs": (i32, [vp, C.POINTER(SyncEntries), i32, C.POINTER(NeedsOut), i32]),
        "corro_scan_offsets": (i32, [vp, vp, vp, u64]),
        "corro_compute_needs_onepass": (i32, [vp, C.POINTER(SyncEntries), C.POINTER(NeedsOut), u64, u64, vp]),
        "corro_needs_bound": (i32, [vp, C.POINTER(SyncEntries), i32, vp, vp]),
        "corro_affinity_of_type": (i32, [C.c_char_p]),
        "corro_ctx_metrics": (i32, [vp, C.POINTER(Metrics)]),
        "corro_table_committed": (i32, [vp, u32, vp]),
        "corro_table_set_affinity": (i32, [vp, u32, vp, u32]),
        "corro_set_affinity_policy": (i32, [vp, i32]),
        "corro_booked_insert_db_batch": (i32, [vp, C.POINTER(GapsIn), C.POINTER(GapsOut)]),
        "corro_compute_needs_packed": (i32, [vp, C.POINTER(SyncEntries), C.POINTER(NeedsPackedOut), u64, u64]),
        "corro_bookie_seq_bookkeeping": (i32, [vp, vp, u64, vp, vp, u64, vp, vp, vp]),
        "corro_site_ids": (i32, [vp, vp, u32, vp]),
        "corro_decode_frames": (i32, [vp, C.c_char_p, u64, i32, i32, C.POINTER(Decoded), i32]),
        "corro_bookie_buffered_versions": (i32, [vp, vp, u64, u64, vp, u64, vp]),
        "corro_bookie_buffered": (i32, [vp, vp, u64, u64, u64, C.POINTER(Rows), u64, vp]),
        "corro_bookie_buffered_value": (i32, [vp, vp, u64, u64, vp, u64, vp]),
        "corro_extract_changes": (i32, [vp, C.POINTER(ExtractIn), i32, C.POINTER(ExtractOut), i32]),
        "corro_booked_new": (i32, [vp]),
        "corro_booked_free": (None, [vp]),
        "corro_booked_insert_db": (i32, [vp, vp, vp, u64, vp, vp, u64, vp, vp, vp, u64, vp]),
        "corro_booked_needed": (i32, [vp, vp, vp, u64, vp]),
        "corro_booked_last": (i32, [vp, vp]),
        "corro_booked_contains": (i32, [vp, u64, vp]),
        "corro_booked_contains_all": (i32, [vp, u64, u64, vp]),
        "corro_ctx_set_profiling": (i32, [vp, i32]),
        "corro_last_timings": (i32, [vp, vp, u32, vp]),
        "corro_bookie_new": (i32, [vp]),
        "corro_bookie_free": (None, [vp]),
        "corro_process_multiple_changes": (i32, [vp, vp, vp, u64, C.POINTER(Changes), i32, C.POINTER(ProcessOut)]),
        "corro_bookie_take_ready": (i32, [vp, vp, vp, u64, vp]),
        "corro_process_fully_buffered": (i32, [vp, vp, vp, u64, vp]),
        "corro_bookie_last": (i32, [vp, vp, vp]),
        "corro_bookie_needed": (i32, [vp, vp, vp, vp, u64, vp]),
        "corro_bookie_contains_all": (i32, [vp, vp, u64, u64, i32, u64, u64, vp]),
        "corro_bookie_partial": (i32, [vp, vp, u64, vp, vp, u64, vp, vp]),
        "corro_generate_sync": (i32, [vp, vp, C.POINTER(SyncState), i32]),
        "corro_partition_ranks": (i32, [vp, C.POINTER(Changes), u32, C.POINTER(Changes), vp]),
        "corro_packed_record_bytes": (i32, [C.POINTER(Changes), vp]),
        "corro_partition_packed": (i32, [vp, C.POINTER(Changes), u32, vp, vp, vp]),
        "corro_unpack_records": (i32, [vp, vp, u64, u32, C.POINTER(Changes)]),
        "corro_partition_slots": (i32, [vp, C.POINTER(Changes), u32, u64, vp, vp, vp]),
        "corro_apply_slots": (i32, [vp, vp, u32, u64, vp, C.POINTER(ApplyOut), vp]),
        "corro_slots_flags_back": (i32, [vp, vp, u32, u64, vp, vp, vp, u64]),
        "corro_unpack_slots": (i32, [vp, vp, u32, u64, vp, C.POINTER(Changes), vp, vp]),
        "corro_apply_mapped": (i32, [vp, C.POINTER(Changes), vp, C.POINTER(ApplyOut)]),
        "corro_ctx_stream": (vp, [vp]),
        "corro_partition_var": (i32, [vp, C.POINTER(Changes), u32, vp, vp, vp, vp, u64, vp]),
        "corro_unpack_var": (i32, [vp, vp, u64, vp, u64, vp, vp, u32, C.POINTER(Changes)]),
        "corro_table_set_pk_interned": (i32, [vp, u32, i32]),
        "corro_pk_keys": (i32, [vp, u32, vp, vp, u64, vp]),
        "corro_pk_keys_device": (i32, [vp, u32, vp, vp, u64, vp]),
        "corro_pk_bytes": (i32, [vp, u32, vp, u64, vp, u64, vp]),
        "corro_pk_canonical": (i32, [C.c_char_p, u64, vp, u64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != CORRO_OK:
        raise CorroError(rc, lib().corro_last_error().decode(errors="replace"))
    return rc


def device_count():
    c = C.c_int(0)
    check(lib().corro_device_count(C.byref(c)))
    return c.value
