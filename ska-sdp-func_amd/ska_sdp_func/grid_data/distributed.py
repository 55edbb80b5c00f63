"""Row-sharded ES gridding across the GPUs of a node (one process per GPU).

Not in the reference (which is single-device); this is the MI355X build's
multi-GPU layer for BASELINE.json config 3. Visibility rows are independent,
so each rank grids its own rows and ONE collective combines the ranks:

  mode="image": every rank runs the full gridding call (scatter, FFT,
      screen, correction) on its rows into a partial image (zeros, except
      the caller's input image on the destination rank), then the partial
      images are summed on the destination with torch.distributed.reduce
      (RCCL over xGMI on GPUs). Exact by linearity of FFT, screen and
      correction: (I + sum_r S_r) * C == I * C + sum_r S_r * C.
  mode="grid": every rank scatters its rows into a private uv grid, the
      grids are summed on the destination (reduce), which then runs the
      FFT + screen + correction once (north-star "reduce before FFT").

Degridding needs no collective (replicate the image, shard the rows).

Any object with grid_uvw_es_fft / grid_scatter / grid_finish / grid_size
(GridderUvwEsFft, or a CPU stand-in in tests) can be the per-rank gridder.
"""


def shard_rows(num_rows, rank, world):
    """Contiguous row range [start, stop) of a rank (balanced to +-1)."""
    base, extra = divmod(num_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def grid_sharded(gridder, uvw, freq, vis, weight, dirty, dist, mode="image",
                 dst=0, group=None, grid_buf=None, async_op=False):
    """Grid this rank's rows and combine all ranks onto rank dst.

    uvw / vis / weight are THIS rank's rows. On return rank dst holds the
    gridded image (accumulated onto its input dirty image); other ranks'
    dirty buffers are scratch. grid_buf: [G, G] complex buffer for
    mode="grid" (allocated by the caller, reused across calls).

    async_op (mode="image" only): the reduce is issued asynchronously and
    its work handle returned instead of dirty; the caller waits on it
    before reading dirty on rank dst or reusing the buffer, and can grid
    the next batch into another buffer meanwhile (the collective then
    overlaps the next batch's kernels).

    dst is a GLOBAL rank, as in torch.distributed.reduce, also when a
    group is given (it must then be a member of the group); the
    comparison below therefore uses this process's global rank.
    """
    rank = dist.get_rank()
    if group is not None:
        members = dist.get_process_group_ranks(group)
        if dst not in members:
            raise ValueError(f"dst {dst} is not a member of the group "
                             f"{members}")
    if mode == "image":
        if rank != dst:
            dirty.zero_()
        gridder.grid_uvw_es_fft(uvw, freq, vis, weight, dirty)
        work = dist.reduce(dirty, dst=dst, group=group, async_op=async_op)
        return work if async_op else dirty
    if async_op:
        raise ValueError("async_op needs mode='image'")
    if mode == "grid":
        if grid_buf is None:
            raise ValueError("mode='grid' needs grid_buf")
        gridder.grid_scatter(uvw, freq, vis, weight, grid_buf)
        dist.reduce(grid_buf, dst=dst, group=group)
        if rank == dst:
            gridder.grid_finish(grid_buf, dirty)
        return dirty
    raise ValueError(f"unknown mode {mode!r}")


# Bus bandwidth assumed for one RCCL reduce over the xGMI links of an
# 8-GPU MI355X node when no measurement of the reduce is available (ring
# reduce: every rank moves (N - 1) / N of the buffer; 7 links of ~153 GB/s
# per GPU, of which a ring reduce sustains roughly two).
RING_BUS_GBS = 300.0


def reduce_ms_model(nbytes, world, bus_gbs=RING_BUS_GBS):
    """Modelled time (ms) of one ring reduce of nbytes over world ranks."""
    if world <= 1:
        return 0.0
    return (world - 1) / world * nbytes / (bus_gbs * 1e9) * 1e3


def predicted_speedup(t_scatter_ms, t_fft_image_ms, world, grid_bytes,
                      image_bytes, reduce_ms=None, bus_gbs=RING_BUS_GBS):
    """Strong-scaling model of one sharded gridding call.

    t_scatter_ms: bucketing + tile kernels of the whole call on one GPU (the
    part that divides over the ranks); t_fft_image_ms: FFT + image-plane
    kernels (once per call in mode "grid", once per rank -- concurrently --
    in mode "image"). reduce_ms: {"grid": ms, "image": ms} measured at this
    world size, else the ring model above. Returns {mode: speed-up over one
    GPU, ...} and the modelled per-call times.
    """
    t1 = t_scatter_ms + t_fft_image_ms
    red = dict(reduce_ms or {})
    out = {}
    for mode, nbytes in (("grid", grid_bytes), ("image", image_bytes)):
        r = red.get(mode)
        if r is None:
            r = reduce_ms_model(nbytes, world, bus_gbs)
        t_n = t_scatter_ms / world + r + t_fft_image_ms
        out[mode] = {"speedup": round(t1 / t_n, 3), "ms": round(t_n, 3),
                     "reduce_ms": round(r, 3),
                     "reduce": "measured" if mode in red else
                               f"model ({bus_gbs:.0f} GB/s ring)"}
    return out
