"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI
for "nccl", gloo on CPU for tests).

The extend/validity workload shards with NO data-path collective (SURVEY
§8(e)): attempts are independent given the read-only terrain, which every
rank holds in its own HBM, and the Philox-keyed inputs of rank r's slice are
identical wherever they are generated.  Only the end-of-run timing (MAX) and
counters (SUM) cross ranks.  The multi-restart configuration (config 4) adds
one fixed-size all_gather of each rank's best-path record.
"""
import torch
import torch.distributed as dist

PATH_MAX = 256          # states per best-path record
REC_HEADER = 4          # cost, length, yaw, n_states
REC_SIZE = REC_HEADER + PATH_MAX * 8 + PATH_MAX * 10   # 4612 doubles = 36.9 KB


def weak_shard(rank, per_rank):
    """Rank r owns attempts [r * per_rank, (r + 1) * per_rank) of the global stream."""
    return rank * per_rank, per_rank


def strong_shard(rank, world, n_total):
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi - lo


def reduce_run(elapsed_s, counters, device):
    """(max elapsed over ranks, per-counter sums) — the only cross-rank traffic."""
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    c = torch.tensor([float(v) for v in counters], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [float(v) for v in c.tolist()]


def stop_together(device):
    """Config 4's early stop: a stop poll for
    planner.plan_rrt_connect(stop_poll=...).  After every group of
    half-iterations each rank posts its own verdict (found, or out of time)
    with one all_reduce(MAX) of one number; every rank stops as soon as any
    rank has (the slower trees stop within one group of the first solution).
    Every rank must poll (the device loop polls once per group until the
    answer is stop), so the collectives pair up."""
    def poll(local_stop, found):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return local_stop
        t = torch.tensor([1.0 if local_stop else 0.0], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return bool(t.item() > 0)
    return poll


def pack_path(cost, length, yaw, states, actions, device="cpu", cap=PATH_MAX):
    """Fixed-size best-path record of `cap` states (states [k, 8], actions
    [k-1, 10]).  Never raises: every rank must reach the collective that
    follows.  A path longer than `cap` gives a record with n_states = -k and
    cost NaN (it cannot win); gather_best_path sizes the records so that this
    does not happen."""
    size = REC_HEADER + cap * 8 + cap * 10
    rec = torch.full((size,), float("nan"), dtype=torch.float64, device=device)
    k = 0 if states is None else int(len(states))
    if k > cap:
        rec[1], rec[2], rec[3] = float(length), float(yaw), float(-k)
        return rec
    rec[0], rec[1], rec[2], rec[3] = float(cost), float(length), float(yaw), float(k)
    if k:
        rec[REC_HEADER:REC_HEADER + 8 * k] = torch.as_tensor(states, dtype=torch.float64).reshape(-1)
        if actions is not None and len(actions):
            a = torch.as_tensor(actions, dtype=torch.float64).reshape(-1)
            off = REC_HEADER + cap * 8
            rec[off:off + a.numel()] = a
    return rec


def unpack_path(rec):
    cap = (rec.numel() - REC_HEADER) // 18
    k = int(rec[3].item()) if rec[3] == rec[3] else 0
    k = max(k, 0)  # a truncated record (-k) carries no states
    states = rec[REC_HEADER:REC_HEADER + 8 * k].reshape(k, 8)
    off = REC_HEADER + cap * 8
    actions = rec[off:off + 10 * max(k - 1, 0)].reshape(max(k - 1, 0), 10)
    return {"cost": float(rec[0]), "length": float(rec[1]), "yaw": float(rec[2]),
            "states": states, "actions": actions}


def allgather_best_path(rec):
    """all_gather every rank's record; every rank picks argmin(cost), ties to the
    lowest rank.  NaN cost = no solution.  Records must
    have the same size on every rank."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 0, rec
    world = dist.get_world_size()
    out = [torch.empty_like(rec) for _ in range(world)]
    dist.all_gather(out, rec)
    best, best_cost = 0, float("inf")
    for r, o in enumerate(out):
        c = float(o[0].item())
        if c == c and c < best_cost:
            best, best_cost = r, c
    return best, out[best]


def gather_best_path(cost, length, yaw, states, actions, device="cpu"):
    """Config 4's exchange (rrt_connect.cpp:401-414 across ranks): one
    all_reduce(MAX) of the path lengths sizes the records (at least PATH_MAX
    states), then one all_gather of every rank's record; argmin of the
    reference's path_cost_ (length, or the cost_add_yaw weighted sum), ties to
    the lowest rank.  No rank can fail between the two collectives.  Returns
    (winning rank, its record)."""
    k = 0 if states is None else int(len(states))
    cap = PATH_MAX
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([float(k)], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cap = max(cap, int(t.item()))
    else:
        cap = max(cap, k)
    rec = pack_path(cost, length, yaw, states, actions, device=device, cap=cap)
    return allgather_best_path(rec)
