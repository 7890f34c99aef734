"""RCCL smoke on the one-GPU box: a one-rank "nccl" process group runs the real collectives of
dist.py (all-gather, gather to rank 0, variable blocks, f64 feature rows) on device tensors.
Multi-rank RCCL runs are the driver's 8-GPU job; the 2-rank logic is covered over gloo
(tests/test_dist_gloo.py)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    from expecto_amd import dist as edist
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", world_size=1, rank=0)
    ok = []
    y = torch.arange(2 * 2 * 3 * 5 * 7, dtype=torch.float32, device="cuda").view(2, 2, 3, 5, 7)
    full = edist.gather_rows(y, 3, 5, 1)
    ok.append(full.is_cuda and torch.equal(full, y))
    to0 = edist.gather_rows_to(y, 3, 5, 1, 0)
    ok.append(to0.is_cuda and torch.equal(to0, y))
    blocks = edist.gather_blocks_to(y[:, :, :, :2], 3, [2], 1, 0)
    ok.append(len(blocks) == 1 and blocks[0].is_cuda and torch.equal(blocks[0], y[:, :, :, :2]))
    f = torch.arange(4 * 20020, dtype=torch.float64, device="cuda").view(4, 20020)
    f0 = edist.gather_rows_to(f, 0, 4, 1, 0)
    ok.append(f0.dtype == torch.float64 and torch.equal(f0, f))
    torch.cuda.synchronize()
    q.put((dist.get_backend(), ok))
    dist.destroy_process_group()


def test_rccl_one_rank_collectives_on_device_tensors():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    backend, ok = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl" and all(ok), ok
