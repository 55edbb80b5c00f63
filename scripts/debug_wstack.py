"""Debug helper: GPU w-stacking driver vs the oracle on small cases."""
import sys
import numpy as np
sys.path.insert(0, "ska-sdp-func_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import wtower_data as wd
from oracle import wtower_oracle as wo
import ska_sdp_func.grid_data as g

N, S = 256, 64
for name, R, C, wpl in [("w0 C1", 200, 1, 0.0), ("w C1", 200, 1, 3.0),
                        ("w C3", 300, 3, 3.0)]:
    case = wd.wstack_case(num_rows=R, num_chan=C, w_planes=wpl if wpl else 1.0)
    if not wpl:
        case["uvw"][:, 2] = 0.0
    rng = np.random.default_rng(1)
    img = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N))
    img[:16] = 0; img[-16:] = 0; img[:, :16] = 0; img[:, -16:] = 0
    a = (case["f0"], case["df"], case["uvw"], S, case["theta"], case["w_step"],
         0.0, 0.0, 8, 16384, 8, 16384, 0.0, case["H"])
    ref = wo.wstack_degrid_all(img, *a, np.zeros((R, C), complex))
    vis = np.zeros((R, C), np.complex128)
    g.wstack_wtower_degrid_all(img, *a, 2, vis)
    err = np.abs(vis - ref).max() / np.abs(ref).max()
    print(name, "degrid rel err", err, flush=True)
    if err > 1e-6:
        bad = np.argsort(-np.abs(vis - ref).ravel())[:5]
        for b in bad:
            r, c = divmod(b, C)
            print("  row", r, "chan", c, "uvw", case["uvw"][r], "gpu", vis[r, c], "ref", ref[r, c])
    y = rng.normal(size=(R, C)) + 1j * rng.normal(size=(R, C))
    gref = wo.wstack_grid_all(y, *a, np.zeros((N, N), complex))
    gi = np.zeros((N, N), np.complex128)
    g.wstack_wtower_grid_all(y, *a, 0, gi)
    for bd in (8, 16, 32, 64):
        c8 = slice(bd, -bd)
        print(name, "border", bd, "grid rel err", np.abs(gi - gref)[c8, c8].max() / np.abs(gref[c8, c8]).max(),
              "max", np.abs(gref[c8, c8]).max(), flush=True)
