"""Row-sharded gridding (ska_sdp_func/grid_data/distributed.py) with the HIP
library on the GPU: two processes on cuda:0, each gridding its own rows
through GridderUvwEsFft, combined by the same grid_sharded() that
bench.py runs over RCCL. The collective here is gloo with the buffers
staged through host memory (RCCL needs one device per rank; the
decomposition under test is the same). Rank 0's image is checked against
the oracle of the whole row set (parity) and against one un-sharded call
of the library on the same device.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from es_data import make_case, rel_l2

pytestmark = pytest.mark.gpu


class HostStagedDist:
    """torch.distributed with reduce() staged through host tensors (gloo
    reduces CPU tensors only); everything else passes through."""

    def __getattr__(self, name):
        return getattr(dist, name)

    @staticmethod
    def reduce(tensor, dst=0, group=None, async_op=False):
        host = tensor.cpu()
        dist.reduce(host, dst=dst, group=group)
        if dist.get_rank() == dst:
            tensor.copy_(host)
        return None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, n, result_path):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (here, root, os.path.join(root, "ska-sdp-func_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import es_oracle
    from ska_sdp_func.grid_data import GridderUvwEsFft
    from ska_sdp_func.grid_data.distributed import grid_sharded, shard_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    uvw, freq, vis, wt, px = make_case(41, 20011, 4, n)
    dirty_in = np.random.default_rng(7).standard_normal((n, n)).astype(
        np.float32)
    g = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa
    lo, hi = shard_rows(len(uvw), rank, world)
    dirty = g(dirty_in)
    plan = GridderUvwEsFft(g(uvw), g(freq), g(vis), g(wt), dirty, px, px,
                           1e-5, False)
    G = plan.grid_size
    if mode == "grid":
        # n 512: grid 770 (rocFFT, whole-grid reduce); n 680: grid 1024,
        # complex row pass (every row reduced); n 1360: grid 2048,
        # real-output row pass (the G/2 + 1 Hermitian rows reduced).
        spec = plan.row_spectra()
        if G & (G - 1):
            assert spec is None
        else:
            rows, c0, nc = spec
            assert (c0, nc) == (0, 2 * (n // 2))
            assert rows == (G // 2 + 1 if 2048 <= G <= 8192 else G)
    grid_buf = torch.zeros((G, G), dtype=torch.complex64, device=dev)
    grid_sharded(plan, g(uvw[lo:hi]), g(freq), g(vis[lo:hi]), g(wt[lo:hi]),
                 dirty, HostStagedDist(), mode=mode, dst=0,
                 grid_buf=grid_buf)
    torch.cuda.synchronize()
    if rank == 0:
        whole = g(dirty_in)
        plan.grid_uvw_es_fft(g(uvw), g(freq), g(vis), g(wt), whole)
        geo = es_oracle.geometry_for(uvw, freq, vis, dirty_in, px, 1e-5,
                                     False)
        ref = es_oracle.grid_uvw_es_fft(geo, uvw, freq, vis, wt, dirty_in)
        out = dirty.cpu().numpy()
        np.save(result_path, np.array([rel_l2(out, ref),
                                       rel_l2(out, whole.cpu().numpy())]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,n", [("image", 512), ("grid", 512),
                                    ("grid", 680), ("grid", 1360)])
def test_sharded_gridding_on_gpu_matches_oracle(tmp_path, mode, n):
    path = str(tmp_path / "err.npy")
    ctx = mp.spawn(_worker, args=(2, _free_port(), mode, n, path), nprocs=2,
                   join=False)
    deadline = time.time() + 240
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                p.terminate()
            pytest.fail("sharded GPU gridding workers did not finish")
    err_oracle, err_whole = (float(x) for x in np.load(path))
    print(f"{mode}: vs oracle {err_oracle:.2e}, vs un-sharded {err_whole:.2e}")
    assert err_oracle < 1e-5
    assert err_whole < 1e-6
