"""Debug probe: the adversarial multi-batch fold at several capacity hints (with / without row-store
growth), reporting per batch the impact and row mismatches against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests._util import rows_to_tuples  # noqa: E402


def run(cap, npk, zipf, batches=3, n=60000, seed=84, impact=True):
    import corrosion_amd as ca
    sites = synth.site_ids(8, seed)
    e = ca.MergeEngine(synth.adversarial_schema(2), capacity_hint=cap)
    e.register_sites(sites)
    f = O.Fold(sites)
    for k in range(batches):
        b = synth.adversarial_batch(n, 8, 2, npk, seed + k, zipf=zipf)
        got = e.apply(b, impact=impact)
        ref = f.apply(b)
        bad = np.nonzero(got != ref)[0] if impact else np.array([], np.int64)
        g = rows_to_tuples(e.export(), with_ts=True)
        r = rows_to_tuples(f.export(), with_ts=True)
        gs, rs = set(g), set(r)
        print(f"cap={cap} npk={npk} zipf={zipf} batch {k}: impact mismatches {len(bad)} rows gpu {len(g)} "
              f"oracle {len(r)} only-gpu {len(gs - rs)} only-oracle {len(rs - gs)}", flush=True)
        for i in bad[:5]:
            print("   change", int(i), "pk", int(b["pk"][i]), "tcid", hex(int(b["table_cid"][i])), "cl", int(b["cl"][i]),
                  "cv", int(b["col_version"][i]), "got", int(got[i]), "want", int(ref[i]), flush=True)
        for x in sorted(gs - rs)[:3]:
            print("   only gpu   ", x, flush=True)
        for x in sorted(rs - gs)[:3]:
            print("   only oracle", x, flush=True)
    e.close()


if __name__ == "__main__":
    run(1 << 20, 20000, 0.6)
    run(1 << 12, 20000, 0.6)
    run(1 << 12, 300, 1.1)
    run(64, 20000, 0.6)
