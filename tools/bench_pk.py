"""Timing probe of the device pk intern (corro_pk_keys_device): config 2's 2^26 changes with 16-byte
BLOB pks packed in HBM (synth.blob_pks_torch), a cold intern into an empty table, then warm ones
(every key held). Run under rocprofv3 --kernel-trace for the per-kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import synth
    import corrosion_amd as ca
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    b = synth.uniform_batch_torch(n, 1000, 1 << 22, 4, seed=synth.config_seed(2), device="cuda")
    data, off = synth.blob_pks_torch(b["pk"])
    eng = ca.MergeEngine({"t": ["a", "b", "c", "d"]}, capacity_hint=n, interned=("t",))
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        keys = eng.pk_keys_device("t", data, off)
        torch.cuda.synchronize()
        print(f"rep {rep}: {(time.perf_counter() - t0) * 1e3:.3f} ms, keys {int(keys.max()) + 1}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
