"""Config 4 (two restart tree pairs, gloo, one GPU) repeated: does every rank's
path end at the goal?  Prints the details of any run whose path does not."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, q, rep):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import global_body_planner_amd as gbp
        from global_body_planner_amd import planner, sharding
        from global_body_planner_amd import terrain_data as td
        data = td.by_name("synth-rough-1024")
        T = gbp.Terrain.from_data(data, device=0)
        xy = (1.0, 10.23, 6.8, 10.23)
        h = T.height_host([[xy[0], xy[1]], [xy[2], xy[3]]])[0]
        start = planner.start_goal_state(h[0], xy[0], xy[1])
        goal = planner.start_goal_state(h[1], xy[2], xy[3])
        out = planner.plan_rrt_connect_device(data, start, goal, batch=8192, max_time=60.0,
                                              seed=20251019 + rank, post_process=True)
        S = out["states"]
        q.put((rep, rank, bool(out["found"]), S.shape[0], bool(np.array_equal(S[-1], goal)),
               S[-1].tolist(), goal.tolist(), out["meet_a"], out["meet_b"], out["vertices_b"]))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        ps = [ctx.Process(target=worker, args=(r, 2, port, q, rep)) for r in range(2)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=240) for _ in ps)
        for p in ps:
            p.join(timeout=60)
        for r in res:
            print(("OK  " if r[4] else "BAD ") + str(r), flush=True)
