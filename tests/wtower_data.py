"""Synthetic inputs for the w-towers tests.

The reference's w-towers tests (tests/grid_data/test_gridder_wtower_uvw.py)
use a 27-antenna Y-shaped array tracked over 90 degrees of hour angle at
declination 40 degrees. Here a Y-shaped array of the same size and extent
is generated (not copied): 3 arms x 9 antennas on power-law radii.
"""
import numpy as np

C_0 = 299792458.0

# Parameters of the reference test (test_gridder_wtower_uvw.py:1536-1560).
REF_CFG = dict(
    image_size=256,
    subgrid_size=64,
    theta=0.0008,
    w_step=280.0,
    shear_u=0.2,
    shear_v=0.1,
    support=10,
    oversampling=16 * 1024,
    w_support=10,
    w_oversampling=16 * 1024,
)
# The reference test's sub-grid offsets (80, 90, 12) place the sub-grid
# 100 km out, beyond every baseline of its 27-antenna array, so that test
# degrids zeros; these offsets put the synthetic array's rows on the
# sub-grid (~90 % of the visibilities on ~150 w-planes).
REF_OFFSETS = (10, 5, 2)


def y_array(arm_len_m=20000.0, n_per_arm=9, seed=5):
    """Antenna positions (x, y, z) [m] of a Y-shaped array."""
    rng = np.random.default_rng(seed)
    ants = []
    for arm in range(3):
        ang = np.radians(5.0 + 120.0 * arm)
        for k in range(1, n_per_arm + 1):
            r = arm_len_m * (k / n_per_arm) ** 1.7
            ants.append((r * np.cos(ang), r * np.sin(ang),
                         rng.normal(0.0, 15.0)))
    return np.array(ants)


def xyz_to_uvw(xyz, ha, dec):
    x, y, z = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    u = x * np.cos(ha) - y * np.sin(ha)
    v0 = x * np.sin(ha) + y * np.cos(ha)
    w = z * np.sin(dec) - v0 * np.cos(dec)
    v = z * np.cos(dec) + v0 * np.sin(dec)
    return np.stack([u, v, w], axis=1)


def baselines(uvw_ant):
    i, j = np.triu_indices(uvw_ant.shape[0], 1)
    return uvw_ant[j] - uvw_ant[i]


def generate_uvw(num_ha=32, dec_deg=40.0, **kw):
    """Baseline (u, v, w) [m] over num_ha hour angles in [0, 90) degrees."""
    ants = y_array(**kw)
    has = np.arange(num_ha) * np.radians(90.0 / num_ha)
    dec = np.radians(dec_deg)
    return np.concatenate([baselines(xyz_to_uvw(ants, ha, dec))
                           for ha in has])


def ref_image(subgrid_size=64):
    """The two-source sub-grid image of the reference test."""
    image = np.zeros((subgrid_size, subgrid_size))
    image[subgrid_size // 4, subgrid_size // 4] = 1.0
    image[5 * subgrid_size // 6, 2 * subgrid_size // 6] = 0.5
    return image


def wstack_case(num_rows=1000, num_chan=3, image_size=256, theta=0.01,
                fov=0.008, w_tower_height=4.0, w_planes=3.0, seed=0,
                uv_frac=0.4):
    """uvw [m] in a disk covering 2 uv_frac of the grid (80 %) and w over
    +-w_planes w-stack planes; f0 = c (1 m wavelength), df = c / 200."""
    from oracle import wtower_oracle as wo
    rng = np.random.default_rng(seed)
    w_step = wo.determine_w_step(theta, fov, 0.0, 0.0)
    rmax = uv_frac * image_size / theta / (1 + (num_chan - 1) / 200.0)
    r = rmax * np.sqrt(rng.random(num_rows))
    ph = rng.random(num_rows) * 2 * np.pi
    wmax = w_planes * w_tower_height * w_step
    uvw = np.stack([r * np.cos(ph), r * np.sin(ph),
                    rng.uniform(-wmax, wmax, num_rows)], axis=1)
    return dict(uvw=uvw, w_step=w_step, f0=C_0, df=C_0 / 200,
                theta=theta, H=w_tower_height)
