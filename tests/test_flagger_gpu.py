"""GPU parity of the HIP flagger (csrc/visibility/sdp_flagger.hip) with the
CPU oracle (oracle/flagger_oracle.c): flags must be bit-identical.

The oracle restates sdp_flagger.cpp:125-428 of the reference and is pinned by
the reference's own known-answer test (tests/test_flagger_oracle.py)."""
import numpy as np
import pytest

from flag_data import make_flag_case
from oracle import flagger_oracle as fo
from test_flagger_oracle import REF_ARGS, reference_fixture

pytestmark = pytest.mark.gpu


def _gpu_flag(vis, flags, device=None, **kw):
    """Run the product flagger; on device tensors if device is given, else
    on numpy arrays (host staging path). Returns the flags as numpy."""
    from ska_sdp_func.visibility import flagger_dynamic_threshold

    if device is None:
        f = flags.copy()
        flagger_dynamic_threshold(vis, f, **kw)
        return f
    import torch

    v = torch.from_numpy(vis).to(device)
    f = torch.from_numpy(flags.copy()).to(device)
    flagger_dynamic_threshold(v, f, **kw)
    torch.cuda.synchronize()
    return f.cpu().numpy()


@pytest.mark.parametrize("dtype", [np.complex128, np.complex64])
@pytest.mark.parametrize("on_device", [False, True])
def test_reference_known_answer(device, dtype, on_device):
    vis, expected = reference_fixture(dtype)
    flags = np.zeros(vis.shape, np.int32)
    out = _gpu_flag(vis, flags, device if on_device else None, **REF_ARGS)
    assert np.array_equal(out, expected)


CASES = [
    # (T, B, C, P, dtype, step, window, wmh, alpha, thr)
    (30, 5, 100, 4, np.complex64, 1, 0, 20, 0.5, 3.5),
    (30, 5, 100, 4, np.complex128, 1, 2, 20, 0.5, 3.5),
    (40, 7, 1024, 1, np.complex64, 1, 0, 20, 0.5, 3.5),
    (40, 7, 1024, 1, np.complex64, 4, 2, 20, 0.2, 3.0),
    (25, 3, 257, 2, np.complex64, 16, 1, 20, 0.5, 2.5),
    (20, 4, 2048, 1, np.complex64, 1, 2, 20, 0.5, 3.5),
    (70, 3, 96, 1, np.complex64, 1, 0, 100, 0.5, 3.5),     # long history
    (24, 6, 64, 1, np.complex128, 2, 3, 7, 0.7, 2.0),
    (16, 2, 33, 3, np.complex64, 5, 0, 1, 0.5, 3.5),
]


@pytest.mark.parametrize("T,B,C,P,dtype,step,window,wmh,alpha,thr", CASES)
def test_matches_oracle(device, T, B, C, P, dtype, step, window, wmh, alpha,
                        thr):
    vis = make_flag_case(T * 1000 + C, T, B, C, P, dtype)
    kw = dict(alpha=alpha, threshold_magnitudes=thr,
              threshold_variations=thr, threshold_broadband=thr,
              sampling_step=step, window=window, window_median_history=wmh)
    flags = np.zeros(vis.shape, np.int32)
    ref = fo.flagger_dynamic_threshold(vis, flags.copy(), **kw)
    out = _gpu_flag(vis, flags, device, **kw)
    assert ref.sum() > 0
    assert np.array_equal(out, ref), (
        f"{np.sum(out != ref)} of {ref.size} flags differ")


def test_existing_flags_kept(device):
    vis = make_flag_case(5, 10, 3, 64, 1)
    flags = (np.random.default_rng(6).uniform(size=vis.shape) < 0.01
             ).astype(np.int32)
    kw = dict(REF_ARGS)
    ref = fo.flagger_dynamic_threshold(vis, flags.copy(), **kw)
    out = _gpu_flag(vis, flags, device, **kw)
    assert np.array_equal(out, ref)
    assert np.all(out[flags == 1] == 1)


def test_location_mismatch(device):
    import torch
    from ska_sdp_func.utility import CError
    from ska_sdp_func.visibility import flagger_dynamic_threshold

    vis = make_flag_case(7, 4, 2, 16, 1)
    flags = torch.zeros(vis.shape, dtype=torch.int32, device=device)
    with pytest.raises(CError, match="Error 6"):
        flagger_dynamic_threshold(vis, flags, **REF_ARGS)


@pytest.mark.parametrize("dtype", [np.complex64, np.complex128])
def test_threshold_boundaries(device, dtype):
    """Magnitudes on the z-score threshold exactly and one unit in the last
    place either side of it (integer magnitudes around median 12 with MAD 1
    and threshold 0.6795 * 2, so z == thr for |m - 12| == 2), and a step
    whose MAD is 0: the comparison shortcuts must decide these exactly as
    the reference's double expression does."""
    T, B, C = 6, 4, 64
    rng = np.random.default_rng(11)
    base = 12.0 + (np.arange(C) % 5) - 2.0          # 10 .. 14
    vis = np.empty((T, B, C, 1), dtype)
    real = np.float32 if dtype == np.complex64 else np.float64
    for t in range(T):
        for b in range(B):
            m = base.astype(real).copy()
            idx = rng.choice(C, 6, replace=False)
            m[idx[0]] = np.nextafter(real(14.0), real(20.0))
            m[idx[1]] = np.nextafter(real(14.0), real(0.0))
            m[idx[2]] = np.nextafter(real(10.0), real(0.0))
            m[idx[3]] = np.nextafter(real(10.0), real(20.0))
            if t == 3:
                m[:] = real(12.0)                    # MAD 0
                m[idx[4]] = real(12.5)
            vis[t, b, :, 0] = m.astype(dtype)
    kw = dict(alpha=0.5, threshold_magnitudes=0.6795 * 2.0,
              threshold_variations=1e6, threshold_broadband=1e6,
              sampling_step=1, window=0, window_median_history=4)
    flags = np.zeros(vis.shape, np.int32)
    ref = fo.flagger_dynamic_threshold(vis, flags.copy(), **kw)
    out = _gpu_flag(vis, flags, device, **kw)
    assert ref.sum() > 0
    assert np.array_equal(out, ref), (
        f"{np.sum(out != ref)} of {ref.size} flags differ")
