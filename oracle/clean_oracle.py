"""CPU restatement of the reference Hogbom CLEAN (TEST INFRASTRUCTURE: only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this
module, as the checker; the product path never imports it).

Follows src/ska-sdp-func/clean/sdp_hogbom_clean.cpp of ska-sdp-func 1.2.2
(the CPU path, sdp_hogbom_clean_cpu):
  cbeam        :33-80    Gaussian CLEAN beam, centre SIZE // 2, stored in T
  CLEAN loop   :183-240  first maximum in flat order; stop when it is below
                         threshold (in T); component += T(gain * peak);
                         residual window -= gain * peak * psf with the
                         products in double and one rounding to T
  restore      :242-266  components (*) beam by sdp_fft_convolution
                         (sdp_fft_convolution.cpp:127-244), whose padding,
                         shift and crop give the "same" alignment
                         out[i] = sum_k in1[k] beam[i - k + (SIZE - 1) // 2]
                         (scipy.signal.convolve mode="same"), rounded to T,
                         plus the residual in T.

Parity unpinned against reference outputs: the reference's own test (tests/clean/test_hogbom_clean.py)
builds its dirty image with the cupy-only gridder path and compares against
a Python CLEAN at 6 / 4 decimals; it holds no golden vectors. This
restatement is checked by a known answer (a delta PSF: the component map
and residual follow g f (1 - g)^k exactly, the stop cycle is predictable)
and by the "same" alignment checked against scipy.signal.convolve.
"""
import numpy as np


def cbeam(details, dtype):
    """SIZE x SIZE beam table in double, values rounded through dtype."""
    sx, sy, theta_deg, size = (float(v) for v in details)
    nb = int(size)
    th = (np.pi / 180) * theta_deg
    ct, st, s2 = np.cos(th), np.sin(th), np.sin(2 * th)
    a = ct * ct / (2 * sx * sx) + st * st / (2 * sy * sy)
    b = s2 / (4 * sx * sx) - s2 / (4 * sy * sy)
    c = st * st / (2 * sx * sx) + ct * ct / (2 * sy * sy)
    d = (np.arange(nb) - nb // 2).astype(np.float64)
    dx, dy = d[:, None], d[None, :]
    beam = np.exp(-(a * dx * dx + 2 * b * dx * dy + c * dy * dy))
    return beam.astype(dtype).astype(np.float64)


def restore(model, beam, residual):
    """T(components (*) beam, "same" alignment) + residual, in T."""
    n, nb = model.shape[0], beam.shape[0]
    h = (nb - 1) // 2
    acc = np.zeros((n, n))
    xs, ys = np.nonzero(model)
    for x, y in zip(xs, ys):                  # flat index order
        v = float(model[x, y])
        i0, i1 = max(0, x - h), min(n, x - h + nb)
        j0, j1 = max(0, y - h), min(n, y - h + nb)
        acc[i0:i1, j0:j1] += v * beam[i0 - x + h:i1 - x + h,
                                      j0 - y + h:j1 - y + h]
    return acc.astype(model.dtype) + residual


def hogbom_clean(dirty, psf, details, loop_gain, threshold, cycle_limit):
    """Returns (clean_model, residual, skymodel, cycles) in dirty's type."""
    T = dirty.dtype.type
    n = dirty.shape[0]
    res = dirty.copy()
    model = np.zeros_like(dirty)
    g = float(T(loop_gain))
    thr = T(threshold)
    cycles = 0
    while cycles < cycle_limit:
        k = int(np.argmax(res))
        if res.flat[k] < thr:
            break
        peak = float(res.flat[k])
        x, y = divmod(k, n)
        model.flat[k] = model.flat[k] + T(g * peak)
        win = psf[n - x:2 * n - x, n - y:2 * n - y].astype(np.float64)
        res = (res.astype(np.float64) - (g * peak) * win).astype(T)
        cycles += 1
    sky = restore(model, cbeam(details, T), res)
    return model, res, sky, cycles
