"""Linear-probing displacement at the pk table's load (0.6), keys placed in random (claim) order vs in
home order (pk_place_ordered): the mean probe length is the same, but a wave waits for the longest of
its 64 lanes' probes -- ~10 slots in claim order, ~5 in home order. CPU only (numpy)."""
import numpy as np


def place(home, order, m):
    occ = np.full(m, -1, np.int64)
    pos = np.empty(len(home), np.int64)
    for k in order:
        p = home[k]
        while occ[p] >= 0:
            p = (p + 1) % m
        occ[p] = k
        pos[k] = p
    return pos


def main(m=1 << 20, load=0.6, seed=1):
    rng = np.random.default_rng(seed)
    n = int(m * load)
    home = rng.integers(0, m, n)
    for name, order in (("claim order", rng.permutation(n)), ("home order", np.argsort(home, kind="stable"))):
        pos = place(home, order, m)
        disp = (pos - home) % m
        q = rng.integers(0, n, (20000, 64))
        d = disp[q]
        lines = ((pos[q] // 4) - (home[q] // 4)) % (m // 4)  # 128-B lines of 4 slots crossed
        print(f"{name}: mean displacement {disp.mean():.3f}, max {disp.max()}, longest probe of a wave "
              f"{d.max(1).mean():.2f} slots, {lines.max(1).mean():.2f} extra lines")


if __name__ == "__main__":
    main()
