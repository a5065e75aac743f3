"""MergeEngine: the device-resident replacement of cr-sqlite's `crsql_changes` merge.

One MergeEngine corresponds to one corrosion writer connection with the CRR schema applied
(corro-types/src/agent.rs:480-482 single writer; schema.rs:362-363 crsql_as_crr). `apply` is the
batched form of the per-change loop in process_complete_version
(/root/reference/crates/corro-agent/src/agent/util.rs:1222-1262): changes are applied in index
order, exactly as consecutive `INSERT INTO crsql_changes` statements would be.
"""
import ctypes as C

import numpy as np

from . import _lib as L

BATCH_FIELDS = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64,
                "db_version": np.int64, "cl": np.uint32, "seq": np.uint32, "site": np.uint32,
                "val0": np.uint64, "val1": np.uint64, "val_type": np.uint8, "val_len": np.uint8,
                "ts": np.uint64, "val_off": np.uint64, "val_size": np.uint32}
VAL_LONG = L.CORRO_VAL_LONG  # val_len of a TEXT/BLOB value longer than 16 bytes (bytes in "val_data")
LONG_FIELDS = ("val_off", "val_size")
FIXED_FIELDS = {k: v for k, v in BATCH_FIELDS.items() if k not in LONG_FIELDS}
REQUIRED = ("pk", "table_cid", "col_version", "db_version", "cl", "seq", "site", "val0")
ROW_FIELDS = {"pk": np.uint64, "table_cid": np.uint32, "col_version": np.int64,
              "db_version": np.int64, "cl": np.int64, "seq": np.uint32, "site": np.uint32,
              "ts": np.uint64, "val0": np.uint64, "val1": np.uint64, "val_type": np.uint8,
              "val_len": np.uint8}


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _int_dtype_ok(t, dt):
    """A device field's tensor must be an integer type of the field's width (signed or unsigned: the
    C ABI reads the bits); a float, bool or wider/narrower tensor is rejected, not reinterpreted."""
    import torch
    ok = {8: (torch.int64, getattr(torch, "uint64", None)), 4: (torch.int32, getattr(torch, "uint32", None)),
          2: (torch.int16, getattr(torch, "uint16", None)), 1: (torch.uint8, torch.int8)}
    return t.dtype in ok.get(np.dtype(dt).itemsize, ())


class MergeEngine:
    def __init__(self, schema, capacity_hint=1 << 20, device=0, interned=()):
        """schema: {table_name: [column names]} in table order (cid k = column k-1, cid 0 = '-1').
        interned: tables whose primary key is not one INTEGER column (BLOB / TEXT / composite pks):
        their rows are keyed by corro_pk_keys' interned ids of the packed pk bytes."""
        lib = L.lib()
        self.schema = list(schema.items())
        descs = (L.TableDesc * max(1, len(self.schema)))()
        self._keep = []
        for i, (name, cols) in enumerate(self.schema):
            arr = (C.c_char_p * max(1, len(cols)))(*[c.encode() for c in cols])
            self._keep.append(arr)
            descs[i].name = name.encode()
            descs[i].ncols = len(cols)
            descs[i].col_names = C.cast(arr, C.POINTER(C.c_char_p))
        h = C.c_void_p()
        L.check(lib.corro_ctx_create(descs, len(self.schema), capacity_hint, device, C.byref(h)))
        self._h = h
        self.device = device
        self.interned = set()
        for name in interned:
            self.set_pk_interned(name)

    def close(self):
        if getattr(self, "_h", None):
            L.lib().corro_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    # ---- schema / sites -------------------------------------------------------------------
    def lookup(self, table, cid):
        out = C.c_uint32()
        L.check(L.lib().corro_lookup_cid(self._h, table.encode(), cid.encode(), C.byref(out)))
        return out.value

    def register_sites(self, site_ids):
        ids = np.ascontiguousarray(site_ids, dtype=np.uint8).reshape(-1, 16)
        ords = np.zeros(max(1, ids.shape[0]), np.uint32)
        L.check(L.lib().corro_site_register(self._h, ids.ctypes.data, ids.shape[0], ords.ctypes.data))
        return ords[: ids.shape[0]]

    def site_ids(self):
        """Registered 16-byte site ids by ordinal (crsql_site_id)."""
        c = C.c_uint32()
        L.check(L.lib().corro_site_ids(self._h, None, 0, C.byref(c)))
        buf = np.zeros(max(1, 16 * c.value), np.uint8)
        L.check(L.lib().corro_site_ids(self._h, buf.ctypes.data, c.value, C.byref(c)))
        return [bytes(buf[16 * i:16 * i + 16]) for i in range(c.value)]

    def site_count(self):
        c = C.c_uint32()
        L.check(L.lib().corro_site_count(self._h, C.byref(c)))
        return c.value

    # ---- primary keys ---------------------------------------------------------------------
    def table_index(self, table):
        if isinstance(table, int):
            return table
        for i, (name, _cols) in enumerate(self.schema):
            if name == table:
                return i
        raise L.CorroError(-4, f"no such table: {table}")

    def set_pk_interned(self, table, on=True):
        t = self.table_index(table)
        L.check(L.lib().corro_table_set_pk_interned(self._h, t, 1 if on else 0))
        name = self.schema[t][0]
        (self.interned.add if on else self.interned.discard)(name)

    # ---- metrics -----------------------------------------------------------------------------
    def metrics(self):
        """Cumulative counters (corro_ctx_metrics) as a dict."""
        m = L.Metrics()
        L.check(L.lib().corro_ctx_metrics(self._h, C.byref(m)))
        return {k: getattr(m, k) for k, _ in L.Metrics._fields_}

    def committed(self, table):
        """corro.changes.committed for one table (corro_table_committed)."""
        c = C.c_uint64()
        L.check(L.lib().corro_table_committed(self._h, self.table_index(table), C.byref(c)))
        return c.value

    # ---- column affinity -------------------------------------------------------------------
    def set_column_types(self, table, decl_types):
        """Register the table's declared column types (one per non-pk column, in cid order): their
        SQLite affinities (corro_affinity_of_type) make the engine store each winning value as the
        affinity converts it, as SQLite's base table does (corro_table_set_affinity)."""
        t = self.table_index(table)
        aff = np.array([L.lib().corro_affinity_of_type(str(d).encode()) for d in decl_types], np.uint8)
        L.check(L.lib().corro_table_set_affinity(self._h, t, aff.ctypes.data if len(aff) else None, len(aff)))

    AFFINITY_POLICIES = {"portable": 0, "sqlite-3.37.2": 1}

    def set_affinity_policy(self, policy):
        """"sqlite-3.37.2" (default): convert every value exactly as SQLite 3.37.2 does, never refusing a
        change (as SQLite does), and count the conversions whose stored form may differ in another SQLite
        version (metrics()["aff_sensitive"]). "portable" (strict, opt-in): convert only values whose
        stored form is the same in every SQLite version with correctly rounded conversions, refuse a
        batch holding any other (CorroError, CORRO_E_RANGE, before any write)
        (corro_set_affinity_policy)."""
        L.check(L.lib().corro_set_affinity_policy(self._h, self.AFFINITY_POLICIES[policy]))

    def pk_keys(self, table, packed):
        """Row keys of packed pks (a list of bytes, pack_columns encoding) of one table."""
        t = self.table_index(table)
        lens = np.array([len(b) for b in packed], np.uint64)
        off = np.zeros(len(packed) + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        buf = np.frombuffer(b"".join(bytes(b) for b in packed) or b"\0", np.uint8)
        keys = np.zeros(max(1, len(packed)), np.uint64)
        L.check(L.lib().corro_pk_keys(self._h, t, buf.ctypes.data, off.ctypes.data, len(packed), keys.ctypes.data))
        return keys[:len(packed)]

    def pk_keys_device(self, table, data, off):
        """Row keys of n packed pks held in device memory: `data` a uint8 CUDA tensor of the packed
        bytes, `off` an int64 CUDA tensor of n + 1 offsets into it (corro_pk_keys_device: interned in
        the HBM intern table, nothing crosses PCIe). Returns an int64 CUDA tensor of n keys (uint64
        bits)."""
        import torch
        t = self.table_index(table)
        n = int(off.numel()) - 1
        keys = torch.empty(max(n, 1), dtype=torch.int64, device=off.device)
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_pk_keys_device(self._h, t, data.data_ptr(), off.data_ptr(), n, keys.data_ptr()))
        return keys[:n]

    def pk_bytes(self, table, keys):
        """Canonical packed pk bytes of row keys of one table."""
        t = self.table_index(table)
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        n = len(keys)
        off = np.zeros(n + 1, np.uint64)
        cap = 64 * n + 64
        while True:
            buf = np.zeros(cap, np.uint8)
            rc = L.lib().corro_pk_bytes(self._h, t, keys.ctypes.data, n, buf.ctypes.data, cap, off.ctypes.data)
            if rc == 0:
                break
            if rc != -6 or int(off[n]) <= cap:
                L.check(rc)
            cap = int(off[n])
        raw = buf.tobytes()
        return [raw[int(off[i]):int(off[i + 1])] for i in range(n)]

    # ---- merge ------------------------------------------------------------------------------
    def apply(self, batch, impact=False):
        """Merge a batch (dict of numpy arrays on the host, or of torch tensors on the GPU).

        Returns the per-change crsql_rows_impacted() growth when impact=True (a numpy array for a
        host batch, a CUDA uint8 tensor for a device batch), else None."""
        return self.apply_prepared(self.prepare(batch, impact))

    def prepare(self, batch, impact=False):
        """Validate a batch and build its C-ABI descriptor (pointers and sizes only) once, so that
        a caller applying the same resident buffers repeatedly (bench.py) pays no per-call
        marshalling; the arrays must stay alive and unchanged in shape while the result is used."""
        for k in REQUIRED:
            if k not in batch or batch[k] is None:
                raise ValueError(f"batch lacks required field {k!r}")
        s = L.Changes()
        keep = []
        on_dev = _is_torch(batch["pk"])
        n = int(batch["pk"].shape[0])
        s.n = n
        for k, dt in BATCH_FIELDS.items():
            a = batch.get(k)
            if a is None:
                setattr(s, k, None)
                continue
            if on_dev:
                if not a.is_cuda or not a.is_contiguous() or not _int_dtype_ok(a, dt):
                    raise ValueError(f"device field {k} must be a contiguous CUDA integer tensor of {np.dtype(dt)} width "
                                     f"(got {a.dtype})")
                if int(a.shape[0]) != n:
                    raise ValueError(f"field {k} has {a.shape[0]} elements, expected {n}")
                setattr(s, k, a.data_ptr() if n else None)
            else:
                a = np.ascontiguousarray(a, dtype=dt)
                if a.shape[0] != n:
                    raise ValueError(f"field {k} has {a.shape[0]} elements, expected {n}")
                keep.append(a)
                setattr(s, k, a.ctypes.data if n else None)
        data = batch.get("val_data")  # long values' bytes (val_off / val_size index them)
        if data is not None:
            if on_dev:
                if not data.is_cuda or not data.is_contiguous() or data.dtype != __import__("torch").uint8:
                    raise ValueError("device val_data must be a contiguous CUDA uint8 tensor")
                s.val_data, s.val_data_len = (data.data_ptr() if data.numel() else None), int(data.numel())
            else:
                data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
                    np.ascontiguousarray(data, dtype=np.uint8)
                keep.append(data)
                s.val_data, s.val_data_len = (data.ctypes.data if data.size else None), int(data.size)
        out = L.ApplyOut()
        imp = None
        if impact:
            if on_dev:  # device batch -> device impact flags (written in place, no copy)
                import torch
                imp = torch.zeros(max(n, 1), dtype=torch.uint8, device=batch["pk"].device)
                out.impact = imp.data_ptr()
            else:
                imp = np.zeros(max(n, 1), np.uint8)
                out.impact = imp.ctypes.data
        return (s, out, keep, imp, n, on_dev, impact)

    def apply_prepared(self, prep):
        """corro_apply_batch on a descriptor from prepare() (a fresh impact buffer is not made:
        the prepared one is overwritten)."""
        s, out, _keep, imp, n, on_dev, impact = prep
        if on_dev:
            import torch
            torch.cuda.current_stream().synchronize()  # the producer's work on torch's stream
        L.check(L.lib().corro_apply_batch(self._h, C.byref(s), L.CORRO_MEM_DEVICE if on_dev else L.CORRO_MEM_HOST,
                                          C.byref(out)))
        return imp[:n] if impact else None

    def count(self):
        c = C.c_uint64()
        L.check(L.lib().corro_state_count(self._h, C.byref(c)))
        return c.value

    def reset(self):
        L.check(L.lib().corro_state_reset(self._h))

    def export(self):
        """crsql_changes rows (unspecified order) as a dict of numpy arrays."""
        m = self.count()
        out = {k: np.zeros(max(m, 1), dt) for k, dt in ROW_FIELDS.items()}
        r = L.Rows()
        for k, a in out.items():
            setattr(r, k, a.ctypes.data)
        w = C.c_uint64()
        L.check(L.lib().corro_state_export(self._h, C.byref(r), max(m, 1), C.byref(w)))
        rows = {k: a[: w.value] for k, a in out.items()}
        rows["long_values"] = self.long_values(rows)
        return rows

    def track_touched(self, on=True):
        """List the rows every apply addresses, for export_touched (corro_ctx_track_touched)."""
        L.check(L.lib().corro_ctx_track_touched(self._h, 1 if on else 0))

    def export_touched(self):
        """The complete current clock rows of every row addressed since the previous call
        (corro_state_export_touched): a dict of numpy arrays like export(), rows of one (table, pk)
        contiguous. A host persisting the state replaces each exported row's clock rows with these."""
        lib = L.lib()
        w = C.c_uint64()
        empty = L.Rows()
        rc = lib.corro_state_export_touched(self._h, C.byref(empty), 0, C.byref(w))
        if rc not in (0, -6):
            L.check(rc)
        m = int(w.value)
        out = {k: np.zeros(max(m, 1), dt) for k, dt in ROW_FIELDS.items()}
        if m:
            r = L.Rows()
            for k, a in out.items():
                setattr(r, k, a.ctypes.data)
            L.check(lib.corro_state_export_touched(self._h, C.byref(r), m, C.byref(w)))
        rows = {k: a[: w.value] for k, a in out.items()}
        rows["long_values"] = self.long_values(rows)
        return rows

    def set_store_limit(self, max_heap_records):
        L.check(L.lib().corro_ctx_set_store_limit(self._h, int(max_heap_records)))

    def value_bytes(self, handles):
        """Bytes of long values by their handles (the val1 of rows with val_len == VAL_LONG)."""
        h = np.ascontiguousarray(handles, dtype=np.uint64)
        n = len(h)
        off = np.zeros(n + 1, np.uint64)
        total = int((h & np.uint64(0xFFFFFF)).sum()) if n else 0
        buf = np.zeros(max(total, 1), np.uint8)
        L.check(L.lib().corro_value_bytes(self._h, h.ctypes.data if n else None, n, buf.ctypes.data, total,
                                          off.ctypes.data))
        raw = buf.tobytes()
        return [raw[int(off[i]):int(off[i + 1])] for i in range(n)]

    def long_values(self, rows):
        """{row index: bytes} for the rows (host arrays) that hold a long value."""
        vl = np.asarray(rows["val_len"])
        idx = np.nonzero(vl == VAL_LONG)[0]
        if len(idx) == 0:
            return {}
        vals = self.value_bytes(np.asarray(rows["val1"])[idx])
        return {int(i): v for i, v in zip(idx, vals)}

    def db_versions(self):
        n = self.site_count()
        out = np.zeros(max(n, 1), np.int64)
        L.check(L.lib().corro_db_versions(self._h, out.ctypes.data, n))
        return out[:n]

    # ---- timing (HIP events on the engine stream) ---------------------------------------
    def set_profiling(self, on=True):
        L.check(L.lib().corro_ctx_set_profiling(self._h, 1 if on else 0))

    def last_timings(self, apply_only=True):
        """ms per stage of the last apply: hist, colscan, plan, scatter, merge (fast + general
        kernels), overflow; with apply_only=False also the last sync-need / extraction count and fill
        kernels and the last extraction index build."""
        arr = (C.c_float * 9)()
        n = C.c_uint32()
        L.check(L.lib().corro_last_timings(self._h, arr, 9, C.byref(n)))
        names = ["k_hist", "k_colscan", "k_plan", "k_scatter", "k_merge", "k_merge_ovf"]
        if not apply_only:
            names += ["k_needs_count", "k_needs_fill", "extract_index"]
        return {names[i]: arr[i] for i in range(min(n.value, len(names)))}

    # ---- multi-GPU ingest -----------------------------------------------------------------
    def partition(self, batch, nranks):
        """Stable pk-hash partition of a device batch by owner rank (corro_partition_ranks).
        Returns (partitioned dict of device tensors, per-rank counts list)."""
        import torch
        n = int(batch["pk"].shape[0])
        s, o = L.Changes(), L.Changes()
        s.n = o.n = n
        out = {}
        for k in BATCH_FIELDS:
            a = batch.get(k)
            if a is None:
                setattr(s, k, None)
                setattr(o, k, None)
                continue
            if not a.is_cuda or not a.is_contiguous():
                raise ValueError(f"field {k} must be a contiguous CUDA tensor")
            out[k] = torch.empty_like(a)
            setattr(s, k, a.data_ptr() if n else None)
            setattr(o, k, out[k].data_ptr() if n else None)
        counts = np.zeros(max(1, nranks), np.uint64)
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_partition_ranks(self._h, C.byref(s), nranks, C.byref(o), counts.ctypes.data))
        return out, [int(c) for c in counts[:nranks]]

    def _device_changes(self, batch):
        n = int(batch["pk"].shape[0])
        s = L.Changes()
        s.n = n
        for k, dt in BATCH_FIELDS.items():
            a = batch.get(k)
            if a is None:
                setattr(s, k, None)
                continue
            if not a.is_cuda or not a.is_contiguous() or not _int_dtype_ok(a, dt) or int(a.shape[0]) != n:
                raise ValueError(f"field {k} must be a contiguous CUDA integer tensor of {n} x {np.dtype(dt)} width")
            setattr(s, k, a.data_ptr() if n else None)
        return s

    def partition_packed(self, batch, nranks, with_perm=False):
        """Stable pk-hash partition of a device batch into whole packed records grouped by owner
        rank (corro_partition_packed): returns (uint8 CUDA tensor of n * rec_bytes, rec_bytes,
        per-rank counts, perm or None) -- one tensor, so one all-to-all moves every field."""
        import torch
        s = self._device_changes(batch)
        n = int(s.n)
        rb = C.c_uint32()
        L.check(L.lib().corro_packed_record_bytes(C.byref(s), C.byref(rb)))
        recs = torch.empty(max(n, 1) * rb.value, dtype=torch.uint8, device=batch["pk"].device)
        perm = torch.empty(max(n, 1), dtype=torch.int32, device=batch["pk"].device) if with_perm else None
        counts = np.zeros(max(1, nranks), np.uint64)
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_partition_packed(self._h, C.byref(s), nranks, recs.data_ptr(),
                                               perm.data_ptr() if perm is not None else None, counts.ctypes.data))
        return recs[:n * rb.value], rb.value, [int(c) for c in counts[:nranks]], (perm[:n] if perm is not None else None)

    def partition_var(self, batch, nranks, with_perm=False):
        """The exchange for every table (corro_partition_var): 80-B records grouped by owner rank plus
        the variable-length bytes they ship (canonical pks of interned tables, long values), routed
        by canonical pk bytes for interned tables. Returns (records uint8 tensor, var uint8 tensor,
        per-rank record counts, per-rank byte counts, perm or None)."""
        import torch
        s = self._device_changes(batch)
        data = batch.get("val_data")
        if data is not None:
            s.val_data, s.val_data_len = (data.data_ptr() if data.numel() else None), int(data.numel())
        n = int(s.n)
        dev = batch["pk"].device
        recs = torch.empty(max(n, 1) * 80, dtype=torch.uint8, device=dev)
        perm = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if with_perm else None
        counts = np.zeros(max(1, nranks), np.uint64)
        vcounts = np.zeros(max(1, nranks), np.uint64)
        torch.cuda.current_stream().synchronize()
        lib = L.lib()
        pp = perm.data_ptr() if perm is not None else None
        rc = lib.corro_partition_var(self._h, C.byref(s), nranks, recs.data_ptr(), pp, counts.ctypes.data, None, 0,
                                     vcounts.ctypes.data)
        total = int(vcounts[:nranks].sum())
        var = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
        if rc == -6 and total:
            rc = lib.corro_partition_var(self._h, C.byref(s), nranks, recs.data_ptr(), pp, counts.ctypes.data,
                                         var.data_ptr(), total, vcounts.ctypes.data)
        L.check(rc)
        return (recs[:n * 80], var[:total], [int(c) for c in counts[:nranks]], [int(c) for c in vcounts[:nranks]],
                perm[:n] if perm is not None else None)

    def unpack_var(self, recs, var, src_counts, src_var):
        """Received records + var bytes (concatenated by source rank) -> a device batch with every
        field, val_data = var (corro_unpack_var; interned pks re-keyed on this engine)."""
        import torch
        n = int(recs.numel()) // 80
        dev = recs.device
        tdt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}
        out = {k: torch.empty(max(n, 1), dtype=tdt[dt], device=dev)[:n] for k, dt in BATCH_FIELDS.items()}
        s = L.Changes()
        s.n = n
        for k in BATCH_FIELDS:
            setattr(s, k, out[k].data_ptr() if n else None)
        sc = np.ascontiguousarray(src_counts, np.uint64)
        sv = np.ascontiguousarray(src_var, np.uint64)
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_unpack_var(self._h, recs.data_ptr() if n else None, n,
                                         var.data_ptr() if var.numel() else None, int(var.numel()),
                                         sc.ctypes.data, sv.ctypes.data, len(sc), C.byref(s)))
        out["val_data"] = var
        return out

    # ---- stream-ordered slot exchange (corro_partition_slots / corro_unpack_slots) ------------
    def stream(self):
        """The engine's HIP stream as a torch stream: collectives issued under
        `torch.cuda.stream(engine.stream())` are ordered with the engine's kernels without a host wait."""
        import torch
        if getattr(self, "_tstream", None) is None:
            self._tstream = torch.cuda.ExternalStream(L.lib().corro_ctx_stream(self._h), device=self.device)
        return self._tstream

    def partition_slots(self, batch, nranks, cap, out=None, counts=None, perm=None):
        """Stable pk-hash partition of an INTEGER device batch into fixed slots of `cap` 48-B records
        per destination (corro_partition_slots): returns (uint8 tensor of nranks * cap * 48, int64
        tensor of the true per-destination counts) -- both written on the engine's stream, nothing
        read back (a count past cap means that slot lost records: corro_unpack_slots reports it)."""
        import torch
        s = self._device_changes(batch)
        dev = batch["pk"].device
        if out is None:
            out = torch.empty(nranks * cap * 48, dtype=torch.uint8, device=dev)
        if counts is None:
            counts = torch.empty(nranks, dtype=torch.int64, device=dev)
        L.check(L.lib().corro_partition_slots(self._h, C.byref(s), nranks, cap, out.data_ptr(), counts.data_ptr(),
                                              perm.data_ptr() if perm is not None else None))
        return out, counts

    def apply_slots(self, recs, nsrc, cap, src_counts, impact=False, overflow=None):
        """corro_apply_slots: merge received slots (nsrc * cap 48-B records, a uint8 CUDA tensor) where
        they lie -- no unpack pass. Returns (impact flags by slot position, a uint8 CUDA tensor of
        nsrc * cap, or None; overflow int32 CUDA tensor [1]: 1 when a source overflowed its slot and
        nothing was applied)."""
        import torch
        n = nsrc * cap
        dev = recs.device
        if overflow is None:
            overflow = torch.zeros(1, dtype=torch.int32, device=dev)
        o = L.ApplyOut()
        imp = None
        if impact:
            imp = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            o.impact = imp.data_ptr()
        L.check(L.lib().corro_apply_slots(self._h, recs.data_ptr(), nsrc, cap, src_counts.data_ptr(), C.byref(o),
                                          overflow.data_ptr()))
        return (imp[:n] if impact else None), overflow

    def slots_flags_back(self, back, nranks, cap, counts, perm, n):
        """corro_slots_flags_back: the all-to-all of the receivers' slot-position flags -> this sender's
        per-input-change flags (uint8 CUDA tensor of n), queued on the engine's stream."""
        import torch
        flags = torch.zeros(max(n, 1), dtype=torch.uint8, device=back.device)
        L.check(L.lib().corro_slots_flags_back(self._h, back.data_ptr(), nranks, cap, counts.data_ptr(), perm.data_ptr(),
                                               flags.data_ptr(), n))
        return flags[:n]

    def unpack_slots(self, recs, nsrc, cap, src_counts, out=None):
        """Received slots -> (SoA device batch of nsrc * cap changes at the same indices, ap int32
        tensor: i for a received change, -1 for padding, overflow int32 tensor [1]) on the engine's
        stream (corro_unpack_slots); merge with apply_mapped."""
        import torch
        n = nsrc * cap
        dev = recs.device
        if out is None:
            tdt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}
            out = {k: torch.empty(max(n, 1), dtype=tdt[BATCH_FIELDS[k]], device=dev)[:n] for k in REQUIRED}
            out["ap"] = torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]
            out["overflow"] = torch.zeros(1, dtype=torch.int32, device=dev)
        s = L.Changes()
        s.n = n
        for k in BATCH_FIELDS:
            a = out.get(k) if k in REQUIRED else None
            setattr(s, k, a.data_ptr() if (a is not None and n) else None)
        L.check(L.lib().corro_unpack_slots(self._h, recs.data_ptr(), nsrc, cap, src_counts.data_ptr(), C.byref(s),
                                           out["ap"].data_ptr(), out["overflow"].data_ptr()))
        return out

    def apply_mapped(self, batch, impact=False):
        """corro_apply_mapped: merge a device batch whose changes with ap == -1 (batch["ap"]) are
        skipped, the rest in index order (the slot layout of unpack_slots)."""
        fields = {k: v for k, v in batch.items() if k in BATCH_FIELDS}
        s, o, _keep, imp, n, _on_dev, impact = self.prepare(fields, impact)
        L.check(L.lib().corro_apply_mapped(self._h, C.byref(s), batch["ap"].data_ptr(), C.byref(o)))
        return imp[:n] if impact else None

    def unpack_records(self, recs, rec_bytes, out=None):
        """Packed records (a uint8 CUDA tensor) -> SoA device batch (corro_unpack_records)."""
        import torch
        n = int(recs.numel()) // rec_bytes
        dev = recs.device
        if out is None:
            tdt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}
            keys = [k for k in FIXED_FIELDS if k in REQUIRED or rec_bytes == 80]
            out = {k: torch.empty(max(n, 1), dtype=tdt[BATCH_FIELDS[k]], device=dev)[:n] for k in keys}
        s = L.Changes()
        s.n = n
        for k in BATCH_FIELDS:
            a = out.get(k)
            setattr(s, k, a.data_ptr() if (a is not None and n) else None)
        torch.cuda.current_stream().synchronize()
        L.check(L.lib().corro_unpack_records(self._h, recs.data_ptr() if n else None, n, rec_bytes, C.byref(s)))
        return out

    # ---- wire decode ------------------------------------------------------------------------
    def decode_frames(self, buf, payload=0, device=False, device_headers=False):
        """Decode length-delimited speedy frames (corro_decode_frames; payload 0 = SyncMessage,
        1 = UniPayload) on the GPU. Returns {"cs": ctypes array of corro_changeset (one per
        frame), "status": int32[], "changes": SoA dict, "set_start"/"set_end"}: host numpy arrays,
        or with device=True CUDA tensors that stay on the GPU (the batch
        corro_process_multiple_changes / corro_apply_batch take with CORRO_MEM_DEVICE). With
        device_headers=True (and device=True) also "cs_dev": the status-0 frames' headers as a CUDA
        uint8 tensor of corro_changeset records built on the device, and "n_dev" of them (for
        CORRO_MEM_DEVICE_HEADERS)."""
        lib = L.lib()
        buf = bytes(buf)
        d = L.Decoded()
        mem = L.CORRO_MEM_DEVICE if device else L.CORRO_MEM_HOST
        L.check(lib.corro_decode_frames(self._h, buf, len(buf), payload, mem, C.byref(d), 0))
        F, NC, NS = d.nframes, d.nchanges, d.nsets
        cs = (L.Changeset * max(F, 1))()
        actors = (C.c_uint8 * max(16 * F, 16))()
        status = np.zeros(max(F, 1), np.int32)
        if device:
            import torch
            tdt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}
            ch = {k: torch.zeros(max(NC, 1), dtype=tdt[dt], device="cuda") for k, dt in BATCH_FIELDS.items()}
            ss = torch.zeros(max(NS, 1), dtype=torch.int64, device="cuda")
            se = torch.zeros(max(NS, 1), dtype=torch.int64, device="cuda")
            vdata = torch.zeros(max(len(buf), 1), dtype=torch.uint8, device="cuda")
            ptr = lambda a: a.data_ptr()  # noqa: E731
            torch.cuda.current_stream().synchronize()
        else:
            ch = {k: np.zeros(max(NC, 1), dt) for k, dt in BATCH_FIELDS.items()}
            ss, se = np.zeros(max(NS, 1), np.uint64), np.zeros(max(NS, 1), np.uint64)
            vdata = None
            ptr = lambda a: a.ctypes.data  # noqa: E731
        d.cs, d.actor_ids, d.status = C.addressof(cs), C.addressof(actors), status.ctypes.data
        d.changes.n = NC
        for k, a in ch.items():
            setattr(d.changes, k, ptr(a))
        if device:
            d.changes.val_data, d.changes.val_data_len = vdata.data_ptr(), len(buf)
        d.set_start, d.set_end = ptr(ss), ptr(se)
        cs_dev = None
        if device and device_headers:
            import torch
            cs_dev = torch.zeros(max(F, 1) * C.sizeof(L.Changeset), dtype=torch.uint8, device="cuda")
            d.cs_dev = cs_dev.data_ptr()
            torch.cuda.current_stream().synchronize()
        if F:
            L.check(lib.corro_decode_frames(self._h, buf, len(buf), payload, mem, C.byref(d), 1))
        changes = {k: a[:NC] for k, a in ch.items()}
        if d.changes.val_data:  # long values: offsets into the frame bytes
            changes["val_data"] = vdata[:len(buf)] if device else np.frombuffer(buf, np.uint8)
        else:
            for k in LONG_FIELDS:
                changes.pop(k)
        out = {"cs": cs, "nframes": F, "actors": actors, "status": status[:F],
               "changes": changes, "set_start": ss[:NS], "set_end": se[:NS]}
        if cs_dev is not None:
            out["cs_dev"], out["n_dev"] = cs_dev, int(d.n_dev) if F else 0
        return out

    # ---- changeset extraction (server side of a sync need) ---------------------------------
    def extract_changes(self, needs):
        """crsql_changes rows per need (corro_extract_changes): needs = {"site": u32[], "start":
        u64[], "end": u64[], optional "seq_start"/"seq_end": u32[]} as numpy arrays (host) or CUDA
        tensors (device). Returns grp_off/row_off (n+1), per group version/last_seq/ts/grp_row_off/
        grp_rows, and "rows" (crsql_changes fields), groups of a need in DESCENDING version order."""
        lib = L.lib()
        on_dev = _is_torch(needs["site"])
        n = int(needs["site"].shape[0])
        s = L.ExtractIn()
        s.n = n
        keep = []
        for k, dt in (("site", np.uint32), ("start", np.uint64), ("end", np.uint64), ("seq_start", np.uint32),
                      ("seq_end", np.uint32)):
            a = needs.get(k)
            if a is None:
                setattr(s, k, None)
                continue
            if on_dev:
                if not a.is_cuda or not a.is_contiguous() or not _int_dtype_ok(a, dt):
                    raise ValueError(f"device need field {k} must be a contiguous CUDA integer tensor of "
                                     f"{np.dtype(dt)} width (got {a.dtype})")
                setattr(s, k, a.data_ptr() if n else None)
            else:
                a = np.ascontiguousarray(a, dtype=dt)
                keep.append(a)
                setattr(s, k, a.ctypes.data if n else None)
        mem = L.CORRO_MEM_DEVICE if on_dev else L.CORRO_MEM_HOST
        if on_dev:
            import torch
            dev = needs["site"].device

            def alloc(cnt, dt):
                tdt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint32: torch.int32,
                       np.uint8: torch.uint8}[dt]
                return torch.empty(max(cnt, 1), dtype=tdt, device=dev)

            def ptr(a):
                return a.data_ptr()
            torch.cuda.current_stream().synchronize()
        else:
            def alloc(cnt, dt):
                return np.zeros(max(cnt, 1), dt)

            def ptr(a):
                return a.ctypes.data
        o = L.ExtractOut()
        gc, rc = alloc(n, np.uint64), alloc(n, np.uint64)
        o.grp_count, o.row_count = ptr(gc), ptr(rc)
        if n:
            L.check(lib.corro_extract_changes(self._h, C.byref(s), mem, C.byref(o), 0))
        if on_dev:
            import torch
            go = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            ro = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            go[1:] = torch.cumsum(gc[:n], 0)
            ro[1:] = torch.cumsum(rc[:n], 0)
            G, R = int(go[-1].item()), int(ro[-1].item())
        else:
            go = np.zeros(n + 1, np.uint64)
            ro = np.zeros(n + 1, np.uint64)
            go[1:] = np.cumsum(gc[:n])
            ro[1:] = np.cumsum(rc[:n])
            G, R = int(go[-1]), int(ro[-1])
        res = {"grp_off": go, "row_off": ro, "version": alloc(G, np.int64), "last_seq": alloc(G, np.uint64),
               "ts": alloc(G, np.uint64), "grp_row_off": alloc(G, np.uint64), "grp_rows": alloc(G, np.uint64)}
        rows = {k: alloc(R, dt) for k, dt in ROW_FIELDS.items()}
        o.grp_off, o.row_off = ptr(go), ptr(ro)
        for k in ("version", "last_seq", "ts", "grp_row_off", "grp_rows"):
            setattr(o, k, ptr(res[k]))
        for k, a in rows.items():
            setattr(o.rows, k, ptr(a))
        if n:
            if on_dev:
                torch.cuda.current_stream().synchronize()
            L.check(lib.corro_extract_changes(self._h, C.byref(s), mem, C.byref(o), 1))
        for k in ("version", "last_seq", "ts", "grp_row_off", "grp_rows"):
            res[k] = res[k][:G]
        res["rows"] = {k: a[:R] for k, a in rows.items()}
        return res

    # ---- sync need diff -------------------------------------------------------------------
    def compute_needs(self, entries):
        """Batched compute_available_needs over CSR entries (see corrosion_amd.sync)."""
        from .sync import _needs_host
        return _needs_host(self, entries)
