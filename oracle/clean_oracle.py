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


# Multi-scale CLEAN (src/ska-sdp-func/clean/sdp_ms_clean_cornwell.cpp,
# CPU path, ska-sdp-func 1.2.2).

def conv_same(a, b):
    """sdp_fft_convolution (sdp_fft_convolution.cpp:127-244): linear
    convolution "same"-aligned to a, out[i] = sum_k a[k] b[i - k +
    (n_b - 1) // 2], by FFT in a's precision."""
    import scipy.signal
    return scipy.signal.fftconvolve(a, b, mode="same").astype(a.dtype)


def scale_kernel(scale, size, dtype):
    """:111-166: a delta at (size/2, size/2) for scale 0, else
    exp(-d^2 / (2 s^2)) / (pi 2 s^2) with s = 3/16 scale, rounded to T."""
    T = np.dtype(dtype).type
    c = size // 2
    k = np.zeros((size, size), dtype)
    if scale == 0:
        k[c, c] = 1
        return k
    sigma = T((3.0 / 16.0) * scale)
    tss = T(2.0 * float(sigma) * float(sigma))
    x = (np.arange(size) - c).astype(np.int64)
    d = (x[:, None] * x[:, None] + x[None, :] * x[None, :]).astype(np.float64)
    return (np.exp(-d / float(tss)) / (np.pi * float(tss))).astype(dtype)


def ms_clean_cornwell(dirty, psf, details, scales, loop_gain, threshold,
                      cycle_limit):
    """Returns (clean_model, residual, skymodel, cycles) in dirty's type."""
    T = dirty.dtype.type
    n, L = dirty.shape[0], psf.shape[0]
    S = len(scales)
    kern = [scale_kernel(int(s), L, dirty.dtype) for s in scales]
    beam = cbeam([details[0], details[1], details[2], L],
                 dirty.dtype).astype(dirty.dtype)          # .cpp:401
    spsf = [[conv_same(conv_same(psf, kern[a]), kern[b]) for b in range(S)]
            for a in range(S)]                               # :414-486
    res = [conv_same(dirty, kern[a]) for a in range(S)]    # :488-515
    coupling = [T(max(0.0, float(spsf[a][a].max()))) for a in range(S)]
    comp = np.zeros_like(dirty)
    g, thr = T(loop_gain), T(threshold)
    cycles = 0
    while cycles < cycle_limit:                              # :557-702
        peak, idx = [], []
        for a in range(S):
            k = int(np.argmax(res[a]))
            ok = res[a].flat[k] > 0
            peak.append(res[a].flat[k] if ok else T(0))
            idx.append(k if ok else 0)
        m, mb = 0, T(0)
        for a in range(S):
            biased = T(peak[a]) / coupling[a]
            if biased > mb:
                m, mb = a, biased
        if res[m].flat[idx[m]] < thr:
            break
        gm = T(g * mb)
        x, y = divmod(idx[m], n)
        x0, y0 = n - x, n - y
        comp = comp + gm * kern[m][x0:x0 + n, y0:y0 + n]
        for a in range(S):
            res[a] = res[a] - gm * spsf[a][m][x0:x0 + n, y0:y0 + n]
        cycles += 1
    sky = conv_same(comp, beam) + res[0]                    # :704-749
    return comp, res[0], sky, cycles
