"""Vertex-level look at a device RRT* divergence (tools/star_diag.py first)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import oracle
import global_body_planner_amd as gbp
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td

data = td.synth_rough(256)
O = oracle.OracleTerrain.from_data(data)
oracle.set_scan_mode(1)
hs, _ = O.ground_height(1.0, 2.55)
hg, _ = O.ground_height(4.02, 2.55)
start = planner.start_goal_state(hs, 1.0, 2.55)
goal = planner.start_goal_state(hg, 4.02, 2.55)
H = int(sys.argv[1]) if len(sys.argv) > 1 else 6
ref = O.plan(start, goal, batch=1024, seed=3, max_halves=H, star=True, stream_a=401, stream_b=402)
dev = planner.plan_rrt_star_connect(data, start, goal, batch=1024, max_time=600.0, seed=3,
                                    max_halves=H, trees=True, device_loop=True, fragile_eps=1e-5)
dev0 = planner.plan_rrt_star_connect(data, start, goal, batch=1024, max_time=600.0, seed=3,
                                     max_halves=H, trees=True, device_loop=True)
T = gbp.Terrain.from_data(data, device=0)
for t, d in (("a", 0), ("b", 1)):
    v = ref[t]["v"]
    print(t, "v equal:", np.array_equal(v, dev[t]["v"]), "parents:", ref[t]["parent"][:20],
          dev[t]["parent"][:20], dev0[t]["parent"][:20])
    bad = np.flatnonzero(ref[t]["parent"] != dev[t]["parent"])
    if not bad.size:
        continue
    k = int(bad[0])
    s_new = v[k]
    for j in range(k):
        dd = oracle.state_distance(s_new, v[j]) if hasattr(oracle, "state_distance") else None
        if not (dd <= 3.0 and dd > 0):
            continue
        r_o, _, _ = O.attempt_connect(v[j], s_new, d, 0.0)   # t_s = poseDistance / V_NOM
        res, _, _ = planner.attempt_connect(T, v[j:j + 1], s_new[None], d)
        print(f"  vertex {k} cand {j}: g[j]={ref[t]['g'][j]:.6f} cp oracle {r_o} engine {res[0]}")

# the resolved rows against the oracle's own decision for the same (s, a)
from global_body_planner_amd import _lib as L
v = ref["a"]["v"]
for j, k in ((3, 10), (4, 10), (3, 5), (0, 4)):
    r_o, sn_o, a_o = O.attempt_connect(v[j], v[k], 0, 0.0)
    ov = O.validate_pairs(v[j][None], a_o[None], np.zeros(1, np.uint8))
    T.set_option(L.OPT_FRAGILE_EPS, 10 ** 10)   # 1e-5 m in 1e-15 units
    hv = T.validate_pairs_host(v[j][None], a_o[None], np.zeros(1, np.uint8))
    T.set_option(L.OPT_FRAGILE_EPS, 1000)
    print(f"pair ({j},{k}): v[j] {v[j][:2]} oracle connect {r_o} a6 {a_o[6]!r} oracle valid {ov[0]} "
          f"flags {ov[3]} | engine host entry eps 1e-5: valid {hv[0]} flags {hv[3]}")


def connect_action(s0, s1, t_s):  # rrt_connect.cpp:53-63, the engine's expression order
    x_td, y_td, z_td, dx_td, dy_td, dz_td = s0[:6]
    x_to, y_to, z_to, dx_to, dy_to, dz_to = s1[:6]
    p_td, dp_td, p_to, dp_to = s0[6], s0[7], s1[6], s1[7]
    a = np.zeros(10)
    a[0] = -(2.0 * (3.0 * x_td - 3.0 * x_to + 2.0 * dx_td * t_s + dx_to * t_s)) / (t_s * t_s)
    a[1] = -(2.0 * (3.0 * y_td - 3.0 * y_to + 2.0 * dy_td * t_s + dy_to * t_s)) / (t_s * t_s)
    a[2] = -(2.0 * (3.0 * z_td - 3.0 * z_to + 2.0 * dz_td * t_s + dz_to * t_s)) / (t_s * t_s)
    a[3] = (2.0 * (3.0 * x_td - 3.0 * x_to + dx_td * t_s + 2.0 * dx_to * t_s)) / (t_s * t_s)
    a[4] = (2.0 * (3.0 * y_td - 3.0 * y_to + dy_td * t_s + 2.0 * dy_to * t_s)) / (t_s * t_s)
    a[5] = (2.0 * (3.0 * z_td - 3.0 * z_to + dz_td * t_s + 2.0 * dz_to * t_s)) / (t_s * t_s)
    a[6] = t_s
    a[7] = 0
    a[8] = -(2.0 * (3.0 * p_td - 3.0 * p_to + 2.0 * dp_td * t_s + dp_to * t_s)) / (t_s * t_s)
    a[9] = (2.0 * (3.0 * p_td - 3.0 * p_to + dp_td * t_s + 2.0 * dp_to * t_s)) / (t_s * t_s)
    return a


T2 = gbp.Terrain.from_data(data, device=0)
for j, k in ((3, 5), (3, 10)):
    s0, s1 = v[j], v[k]
    d = s1[:3] - s0[:3]
    t_s = np.sqrt(0.0 + d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) / 0.75
    a = connect_action(s0, s1, t_s)
    ov = O.validate_pairs(s0[None], a[None], np.zeros(1, np.uint8))
    r = T2.validate_pairs(torch.from_numpy(s0[None]).cuda(), torch.from_numpy(a[None]).cuda(),
                          torch.zeros(1, dtype=torch.uint8).cuda())
    print(f"depth-0 check ({j},{k}) t_s {t_s!r}: oracle valid {ov[0]} flags {ov[3]}; device raw "
          f"valid {r.valid.cpu().numpy()} flags {r.flags.cpu().numpy()}; host entry "
          f"{T2.validate_pairs_host(s0[None], a[None], np.zeros(1, np.uint8))[3]}")
