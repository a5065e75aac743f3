"""The ctypes mirror (corrosion_amd/_lib.py) against the C header: every struct's size and every
field's offset as gcc lays out include/corro_hip.h (CPU only; a mismatch would pass garbage across
the boundary without any error)."""
import os
import shutil
import subprocess
import tempfile

import pytest

from corrosion_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PAIRS = {  # ctypes mirror -> C typedef
    "TableDesc": "corro_table_desc", "Changes": "corro_changes", "ApplyOut": "corro_apply_out",
    "Rows": "corro_rows", "SyncEntries": "corro_sync_entries", "ExtractIn": "corro_extract_in",
    "ExtractOut": "corro_extract_out", "Metrics": "corro_metrics", "GapsIn": "corro_gaps_in",
    "GapsOut": "corro_gaps_out", "NeedsPackedOut": "corro_needs_packed_out", "NeedsOut": "corro_needs_out",
    "Changeset": "corro_changeset", "Decoded": "corro_decoded", "ProcessOut": "corro_process_out",
    "SyncState": "corro_sync_state",
}


def _c_layout():
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "corro_hip.h"', "int main(void) {"]
    for py, c in PAIRS.items():
        lines.append(f'  printf("{py} size %zu\\n", sizeof({c}));')
        for name, _t in getattr(L, py)._fields_:
            lines.append(f'  printf("{py} {name} %zu\\n", offsetof({c}, {name}));')
    lines += ["  return 0;", "}"]
    d = tempfile.mkdtemp(prefix="corro_abi_")
    try:
        src, exe = os.path.join(d, "layout.c"), os.path.join(d, "layout")
        with open(src, "w") as f:
            f.write("\n".join(lines) + "\n")
        subprocess.check_call([cc, "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        out = subprocess.check_output([exe]).decode()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    got = {}
    for ln in out.splitlines():
        py, name, v = ln.split()
        got[(py, name)] = int(v)
    return got


def test_ctypes_mirror_matches_header_layout():
    import ctypes as C
    got = _c_layout()
    for py in PAIRS:
        st = getattr(L, py)
        assert C.sizeof(st) == got[(py, "size")], py
        for name, _t in st._fields_:
            assert getattr(st, name).offset == got[(py, name)], f"{py}.{name}"
