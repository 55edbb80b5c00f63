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
