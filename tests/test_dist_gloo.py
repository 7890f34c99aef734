"""CPU, world_size 2 and 4 over gloo: variant sharding, the all-gather and the gather to rank 0 (dist.py)."""
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
    # streamed batches: variable block sizes per rank (batch 0 of 2 rows, as the chromatin CLI does)
    counts = [min(2, edist.shard_range(n_total, k, w)[1] - edist.shard_range(n_total, k, w)[0]) for k in range(w)]
    blocks = edist.gather_blocks_to(y[:, :, :, :counts[r]], 3, counts, w, r)
    if r == 0:
        ok_blocks = all(torch.equal(b, full[:, :, :, edist.shard_range(n_total, k, w)[0]:][:, :, :, :counts[k]])
                        for k, b in enumerate(blocks))
    else:
        ok_blocks = blocks is None
    to0 = edist.gather_rows_to(y, 3, n_total, w, r)
    # compute_expecto_features' features: f64 [G_r, 20020]-shaped blocks along dim 0 to rank 0
    f = torch.arange(lo, hi, dtype=torch.float64).view(-1, 1) * 10 + torch.arange(3, dtype=torch.float64)
    f0 = edist.gather_rows_to(f, 0, n_total, w, r)
    ok_f = (torch.equal(f0[:, 0], torch.arange(n_total, dtype=torch.float64) * 10) and f0.dtype == torch.float64
            if r == 0 else f0 is None)
    ok_to0 = (torch.equal(to0, full) if r == 0 else to0 is None) and ok_blocks and ok_f
    q.put((r, lo, hi, full.shape,
           bool(torch.equal(full[0, 1, 2, :, 0], torch.arange(n_total, dtype=torch.float32))) and ok_to0))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 7), (2, 2), (2, 1), (4, 7), (4, 3)])
def test_gather_rows(world, n_total):
    """World 4 with 7 variants: shards of 2, 2, 2, 1 (gather_blocks_to pads unequal blocks); with 3,
    one rank holds none (the 4-rank gather before the 8-rank one)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == 0 and res[-1][2] == n_total
    assert all(res[i][2] == res[i + 1][1] for i in range(world - 1))
    assert all(tuple(r[3]) == (2, 2, 3, n_total, 5) and r[4] for r in res)


def test_shard_range_covers_everything():
    from expecto_amd.dist import shard_range
    for n in (0, 1, 5, 1000, 100001):
        for w in (1, 2, 3, 8):
            ranges = [shard_range(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in ranges) - min(h - l for l, h in ranges) <= 1
