import sys, numpy as np
sys.path.insert(0, "/root/repo")
import global_body_planner_amd as gbp
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td
data = td.by_name("synth-rough-1024")
T = gbp.Terrain.from_data(data, device=0)
xy = (1.0, 10.23, 6.8, 10.23)
h = T.height_host([[xy[0], xy[1]], [xy[2], xy[3]]])[0]
start = planner.start_goal_state(h[0], xy[0], xy[1])
goal = planner.start_goal_state(h[1], xy[2], xy[3])
for seed in (20251019, 20251020):
    for pp in (False, True):
        out = planner.plan_rrt_connect_device(data, start, goal, batch=8192, max_time=60.0, seed=seed, post_process=pp, trees=True)
        S = out["states"]
        print(seed, pp, out["found"], S.shape, "first==start", np.array_equal(S[0], start), "last==goal", np.array_equal(S[-1], goal), S[-1][:3], goal[:3], "meet", out["meet_a"], out["meet_b"], "vb", out["vertices_b"], out["b"]["v"][0][:3])
