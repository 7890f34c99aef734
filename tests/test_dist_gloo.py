"""CPU, world_size 2 over gloo: variant sharding, the all-gather and the gather to rank 0 (dist.py)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from expecto_amd import dist as edist
    r, w, _ = edist.init("gloo")
    lo, hi = edist.shard_range(n_total, r, w)
    # y[strand][allele][shift][variant][feat] with the variant id encoded in the values
    v = torch.arange(lo, hi, dtype=torch.float32)
    y = v.view(1, 1, 1, -1, 1).expand(2, 2, 3, hi - lo, 5).contiguous() + torch.arange(5.0)
    full = edist.gather_rows(y, 3, n_total, w)
    to0 = edist.gather_rows_to(y, 3, n_total, w, r)
    ok_to0 = torch.equal(to0, full) if r == 0 else to0 is None
    q.put((r, lo, hi, full.shape,
           bool(torch.equal(full[0, 1, 2, :, 0], torch.arange(n_total, dtype=torch.float32))) and ok_to0))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("n_total", [7, 2, 1])
def test_gather_rows_world2(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, s0, ok0), (r1, lo1, hi1, s1, ok1) = res
    assert (lo0, hi1) == (0, n_total) and hi0 == lo1
    assert tuple(s0) == (2, 2, 3, n_total, 5) and ok0 and ok1


def test_shard_range_covers_everything():
    from expecto_amd.dist import shard_range
    for n in (0, 1, 5, 1000, 100001):
        for w in (1, 2, 3, 8):
            ranges = [shard_range(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in ranges) - min(h - l for l, h in ranges) <= 1
