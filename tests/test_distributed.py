"""World-size-2 gloo tests of the multi-GPU plumbing (CPU, no GPU needed):
sharded attempts summed across ranks equal the single-process batch, and the
config-4 best-path all_gather picks the same record on every rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from global_body_planner_amd import sharding, terrain_data as td
        from tests.helpers import attempts_oracle
        O = oracle.OracleTerrain.from_data(td.synth_rough(128))
        oracle.set_scan_mode(1)
        per = 700
        base, n = sharding.weak_shard(rank, per)
        s, a, d, _, _ = attempts_oracle(O, n, seed=99, index_base=base, nthreads=2)
        v, sn, tn, f, c = O.validate_pairs(s, a, d, nthreads=2)
        gv = int(((c & 0xFFFF) + (c >> 16)).sum())
        el, sums = sharding.reduce_run(0.1 * (rank + 1), [n, int(v.sum()), gv], "cpu")
        # config 4: every rank proposes a path, rank 1 has the lower cost and a
        # path longer than PATH_MAX (the records are sized first: no rank raises
        # before the all_gather, the long path travels whole)
        k = 3 if rank == 0 else sharding.PATH_MAX + 44
        states = np.full((k, 8), float(rank))
        acts = np.full((k - 1, 10), float(rank))
        best, brec = sharding.gather_best_path(10.0 - rank, 5.0, 0.1, states, acts)
        u = sharding.unpack_path(brec)
        q.put((rank, el, sums, best, u["states"].numpy().tolist(), u["actions"].shape[0]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharding_and_best_path():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every rank sees the same reduction: max time, summed counters
    assert res[0][1] == pytest.approx(0.2) and res[1][1] == pytest.approx(0.2)
    assert res[0][2] == res[1][2]
    # ... equal to the single-process run of the whole 1400-attempt batch
    import oracle
    from global_body_planner_amd import terrain_data as td
    from tests.helpers import attempts_oracle
    O = oracle.OracleTerrain.from_data(td.synth_rough(128))
    oracle.set_scan_mode(1)
    s, a, d, _, _ = attempts_oracle(O, 1400, seed=99, nthreads=2)
    v, sn, tn, f, c = O.validate_pairs(s, a, d, nthreads=2)
    assert res[0][2] == [1400.0, float(v.sum()), float(((c & 0xFFFF) + (c >> 16)).sum())]
    # best path: rank 1's record (cost 9 < 10, 300 states) on both ranks
    k = 256 + 44
    assert res[0][3] == 1 and res[1][3] == 1
    assert res[0][4] == res[1][4] == [[1.0] * 8] * k
    assert res[0][5] == res[1][5] == k - 1


def test_pack_unpack_roundtrip():
    from global_body_planner_amd import sharding
    st = np.arange(40.0).reshape(5, 8)
    ac = np.arange(40.0).reshape(4, 10)
    r = sharding.pack_path(3.5, 2.0, 0.25, st, ac)
    assert r.numel() == sharding.REC_SIZE and r.numel() * 8 < 40_000
    u = sharding.unpack_path(r)
    assert u["cost"] == 3.5 and np.array_equal(u["states"].numpy(), st)
    assert np.array_equal(u["actions"].numpy(), ac)
    assert sharding.strong_shard(1, 3, 10) == (3, 3)
    # a path past the record's capacity gives an unusable record instead of raising
    t = sharding.pack_path(1.0, 2.0, 0.0, np.zeros((sharding.PATH_MAX + 1, 8)),
                           np.zeros((sharding.PATH_MAX, 10)))
    ut = sharding.unpack_path(t)
    assert np.isnan(ut["cost"]) and ut["states"].shape == (0, 8)
    # a sized record holds it (single process: no collective)
    who, rec = sharding.gather_best_path(1.0, 2.0, 0.0, np.ones((300, 8)), np.ones((299, 10)))
    assert who == 0 and sharding.unpack_path(rec)["states"].shape == (300, 8)
