"""CPU restatement of the reference point-source DFT (TEST INFRASTRUCTURE:
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use
this module, as the checker; the product path never imports it).

Follows src/ska-sdp-func/visibility/sdp_dft.cpp of ska-sdp-func 1.2.2:
  dft_point_v00  :24-98   phase = -2 pi (l u + m v + n w), uvw per channel
  dft_point_v01  :253-336 phase = -2 pi ((f0 + c df) / c0) (l u + m v + n w)
The phasor is rounded to the visibility precision (complex<VIS_TYPE>(cos,
sin)), fluxes are cast to it, and the polarisations accumulate over the
components in order in that precision.

Parity unpinned against reference outputs: the reference test (tests/visibility/test_dft.py) compares
its CPU and GPU paths with each other and holds no golden vectors; this
restatement is checked by its loop form (dft_loops, the reference loop nest
written out scalar by scalar) and by known answers (a source at the phase
centre returns its flux, a source at l = 1 gives exp(-2 pi i u)).
"""
import numpy as np

C_0 = 299792458.0


def _accumulate(phase, fluxes, vis_dtype):
    """phase [..., C, S] (double) and fluxes [C, S, P]; returns [..., C, P]
    in vis_dtype, accumulated sequentially over S in that precision."""
    real = np.float32 if vis_dtype == np.complex64 else np.float64
    pr = np.cos(phase).astype(real)
    pi = np.sin(phase).astype(real)
    fr = fluxes.real.astype(real)
    fi = fluxes.imag.astype(real)
    shape = phase.shape[:-1] + (fluxes.shape[-1],)
    acc_re = np.zeros(shape, real)
    acc_im = np.zeros(shape, real)
    for s in range(phase.shape[-1]):
        a, b = pr[..., s, None], pi[..., s, None]
        c, d = fr[:, s, :], fi[:, s, :]
        acc_re = acc_re + (a * c - b * d)
        acc_im = acc_im + (a * d + b * c)
    out = np.empty(shape, vis_dtype)
    out.real = acc_re
    out.imag = acc_im
    return out


def dft_point_v00(source_directions, source_fluxes, uvw_lambda, vis_dtype):
    """[T, B, C, P] visibilities from uvw_lambda [T, B, C, 3]."""
    d = np.asarray(source_directions, np.float64)
    uu, vv, ww = (uvw_lambda[..., k, None] for k in range(3))
    phase = -2.0 * np.pi * (d[:, 0] * uu + d[:, 1] * vv + d[:, 2] * ww)
    flux = np.transpose(source_fluxes, (1, 0, 2))       # [C, S, P]
    return _accumulate(phase, flux, np.dtype(vis_dtype).type)


def dft_point_v01(source_directions, source_fluxes, uvw, channel_start_hz,
                  channel_step_hz, num_channels, vis_dtype):
    """[T, B, C, P] visibilities from uvw [T, B, 3] in metres."""
    d = np.asarray(source_directions, np.float64)
    inv_wl = (channel_start_hz +
              np.arange(num_channels) * channel_step_hz) / C_0
    uu, vv, ww = (uvw[:, :, None, k, None] for k in range(3))
    dot = d[:, 0] * uu + d[:, 1] * vv + d[:, 2] * ww     # [T, B, 1, S]
    phase = -2.0 * np.pi * inv_wl[:, None] * dot          # [T, B, C, S]
    flux = np.transpose(source_fluxes, (1, 0, 2))
    return _accumulate(phase, flux, np.dtype(vis_dtype).type)


def dft_loops(source_directions, source_fluxes, uvw, channel_start_hz,
              channel_step_hz, vis_shape, vis_dtype, v01):
    """The reference loop nest, scalar by scalar (small cases only)."""
    T, B, C, P = vis_shape
    real = np.float32 if np.dtype(vis_dtype) == np.complex64 else np.float64
    out = np.zeros(vis_shape, vis_dtype)
    for t in range(T):
        for b in range(B):
            for c in range(C):
                acc = [[real(0), real(0)] for _ in range(P)]
                if v01:
                    uu, vv, ww = (float(x) for x in uvw[t, b])
                    inv_wl = (channel_start_hz + c * channel_step_hz) / C_0
                else:
                    uu, vv, ww = (float(x) for x in uvw[t, b, c])
                for s in range(source_directions.shape[0]):
                    l, m, n = (float(x) for x in source_directions[s])
                    if v01:
                        phase = -2.0 * np.pi * inv_wl * (l * uu + m * vv +
                                                         n * ww)
                    else:
                        phase = -2.0 * np.pi * (l * uu + m * vv + n * ww)
                    pr, pi = real(np.cos(phase)), real(np.sin(phase))
                    for p in range(P):
                        f = source_fluxes[s, c, p]
                        fr, fi = real(f.real), real(f.imag)
                        acc[p][0] = real(acc[p][0] + real(pr * fr - pi * fi))
                        acc[p][1] = real(acc[p][1] + real(pr * fi + pi * fr))
                for p in range(P):
                    out[t, b, c, p] = complex(acc[p][0], acc[p][1])
    return out
