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
  mode="grid": every rank scatters its rows into a private uv grid and
      the grids are summed on the destination before its column FFTs
      (north-star "reduce before FFT"). With the fused f32 FFT each rank
      first runs the row pass of the inverse FFT on its own grid (linear),
      and only the block the column passes read travels: the row spectra
      of the Hermitian part, (G/2 + 1) x M complex (178 MB at G 8192, N
      5440, against the 512 MiB grid); the destination runs the column
      passes + screen + correction once. Plans without that split (f64,
      rocFFT grids) reduce the whole grid before one finish.

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
        spec = (gridder.row_spectra() if hasattr(gridder, "row_spectra")
                else None)
        if spec is None:
            dist.reduce(grid_buf, dst=dst, group=group)
            if rank == dst:
                gridder.grid_finish(grid_buf, dirty)
            return dirty
        rows, c0, nc = spec
        gridder.grid_rows(grid_buf)
        block = grid_buf[:rows, c0:c0 + nc]
        packed = block.contiguous() if nc < grid_buf.shape[1] else block
        dist.reduce(packed, dst=dst, group=group)
        if rank == dst:
            if packed is not block:
                block.copy_(packed)
            gridder.grid_finish_rows(grid_buf, dirty)
        return dirty
    raise ValueError(f"unknown mode {mode!r}")


def row_spectra_bytes(grid_size, image_size, herm=True, elem_bytes=8):
    """Bytes of the row-spectra block mode="grid" reduces (fused f32 plans:
    the (G/2 + 1) x M Hermitian row spectra, M = 2 (N // 2))."""
    rows = grid_size // 2 + 1 if herm else grid_size
    return rows * 2 * (image_size // 2) * elem_bytes


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


# HBM rate assumed for the pack / unpack copies of the row-spectra block
# (a strided torch copy: read + write of the block on each side).
PACK_GBS = 4000.0


def predicted_speedup(t_scatter_ms, t_fft_image_ms, world, grid_bytes,
                      image_bytes, reduce_ms=None, bus_gbs=RING_BUS_GBS,
                      grid_packed=False):
    """Strong-scaling model of one sharded gridding call.

    t_scatter_ms: bucketing + tile kernels of the whole call on one GPU (the
    part that divides over the ranks); t_fft_image_ms: FFT + image-plane
    kernels (mode "grid": the row pass on every rank concurrently, the
    column passes once on the destination; mode "image": all of it on
    every rank, concurrently). grid_bytes: what mode "grid" reduces (the
    row-spectra block, row_spectra_bytes, or the whole grid); grid_packed:
    that block is packed into a contiguous buffer and unpacked on the
    destination (two read + write copies at PACK_GBS). reduce_ms: {"grid":
    ms, "image": ms} measured at this world size, else the ring model
    above. Returns {mode: speed-up over one GPU, ...} and the modelled
    per-call times.
    """
    t1 = t_scatter_ms + t_fft_image_ms
    red = dict(reduce_ms or {})
    out = {}
    for mode, nbytes in (("grid", grid_bytes), ("image", image_bytes)):
        r = red.get(mode)
        if r is None:
            r = reduce_ms_model(nbytes, world, bus_gbs)
        pack = (2 * 2 * nbytes / (PACK_GBS * 1e9) * 1e3
                if mode == "grid" and grid_packed and world > 1 else 0.0)
        t_n = t_scatter_ms / world + r + pack + t_fft_image_ms
        out[mode] = {"speedup": round(t1 / t_n, 3), "ms": round(t_n, 3),
                     "reduce_ms": round(r, 3),
                     "reduce_bytes": int(nbytes),
                     "reduce": "measured" if mode in red else
                               f"model ({bus_gbs:.0f} GB/s ring)"}
        if pack:
            out[mode]["pack_ms"] = round(pack, 3)
    return out


# W-stack plane sharding for the w-towers imager (config 4): the planes are
# independent until the image sum (ref sdp_grid_wstack_wtower.cpp:608-713),
# so each rank grids a SET of planes (sdp_grid_wstack_wtower_grid_plane_set)
# and the images are reduced once. The sets balance a cost model instead of
# taking every N-th plane.

C_LIGHT = 299792458.0


def wstack_plane_loads(uvw, freq0_hz, dfreq_hz, num_chan, w_step,
                       w_tower_height):
    """Visibilities per w-stack plane, as (first_plane, counts).

    Plane iw holds channel c of a row when w (f0 + c df) / c lies in
    [iw d - d/2, (iw + 1) d - d/2), d = w_tower_height * w_step (the
    reference's plane cells, sdp_grid_wstack_wtower.cpp:336-343). This is
    a cost model: the driver's exact channel clamps may move a visibility on
    a cell boundary to the neighbouring plane, so the range carries one
    plane of margin on each side. uvw: numpy array or torch tensor (any
    device)."""
    import numpy as np
    d = float(w_tower_height) * float(w_step)
    try:
        import torch
        is_torch = isinstance(uvw, torch.Tensor)
    except ImportError:
        is_torch = False
    if is_torch:
        w = uvw[:, 2].to(torch.float64)
    else:
        w = np.asarray(uvw, dtype=np.float64)[:, 2]
    planes = []
    for c in range(int(num_chan)):
        x = w * ((freq0_hz + c * dfreq_hz) / C_LIGHT)
        iw = (torch.floor(x / d + 0.5) if is_torch
              else np.floor(x / d + 0.5))
        planes.append(iw)
    if not planes or len(w) == 0:
        return 0, np.zeros(0, np.int64)
    if is_torch:
        allp = torch.cat(planes).to(torch.int64)
        lo, hi = int(allp.min()), int(allp.max())
        counts = torch.bincount(allp - lo, minlength=hi - lo + 1).cpu().numpy()
    else:
        allp = np.concatenate(planes).astype(np.int64)
        lo, hi = int(allp.min()), int(allp.max())
        counts = np.bincount(allp - lo, minlength=hi - lo + 1)
    counts = np.concatenate([[0], counts, [0]]).astype(np.int64)
    return lo - 1, counts


def assign_planes(loads, world, fixed_cost=0.0):
    """Plane sets of world ranks balancing sum(load + fixed_cost) over the
    occupied planes (longest-processing-time greedy: heaviest plane first,
    each to the least-loaded rank). Empty planes (no modelled load) are
    dealt round-robin at no cost, so every plane of the range belongs to
    exactly one rank. Returns (masks[world][n] int32, per-rank costs)."""
    import numpy as np
    loads = np.asarray(loads, dtype=np.float64)
    n = len(loads)
    masks = np.zeros((world, n), np.int32)
    cost = np.zeros(world)
    occupied = [i for i in range(n) if loads[i] > 0]
    for i in sorted(occupied, key=lambda k: (-loads[k], k)):
        r = int(np.argmin(cost))
        masks[r, i] = 1
        cost[r] += loads[i] + fixed_cost
    empty = [i for i in range(n) if loads[i] <= 0]
    for j, i in enumerate(empty):
        masks[j % world, i] = 1
    return masks, cost


def plane_balance(cost):
    """max / mean of the per-rank modelled costs (1.0 = perfect)."""
    import numpy as np
    cost = np.asarray(cost, dtype=np.float64)
    return float(cost.max() / cost.mean()) if cost.sum() > 0 else 1.0
