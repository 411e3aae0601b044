// Compile/link check of the drop-in: the calls GlobalBodyPlanner makes on the
// planner classes (global_body_planner.cpp:43, :88-119, :178-195, :263-264,
// :131 getInterpPath), written against the reference's global names through
// gbp_planner_compat.h.  Built and linked by tests/test_abi.py; run on the
// GPU box by tests/test_gpu_planner.py (argv: nothing; exit 0 = plan found).
#include <cstdio>
#include <string>
#include <vector>

#include "gbp_planner_compat.h"

// a minimal grid_map-shaped type (getSize, getStartIndex, getPosition, at, exists)
namespace fake_grid_map {
struct Vec2i {
  int v[2];
  Vec2i(int a = 0, int b = 0) : v{a, b} {}
  int operator()(int i) const { return v[i]; }
};
struct Pos {
  double px = 0, py = 0;
  double x() const { return px; }
  double y() const { return py; }
};
struct GridMap {
  int nx, ny;
  double res;
  std::vector<float> z;  // grid_map index (i, j) -> z[i*ny + j]
  Vec2i getSize() const { return Vec2i(nx, ny); }
  Vec2i getStartIndex() const { return Vec2i(0, 0); }
  Pos getPosition() const { return Pos(); }
  void getPosition(const Vec2i &idx, Pos &p) const {
    // grid_map: index (0,0) is the max corner (fast_terrain_map.cpp:44-54 reverses it)
    p.px = (nx - 1 - idx(0)) * res;
    p.py = (ny - 1 - idx(1)) * res;
  }
  float at(const char *layer, const Vec2i &idx) const {
    (void)layer;
    return z[(size_t)idx(0) * ny + idx(1)];
  }
  bool exists(const char *layer) const {
    (void)layer;
    return false;
  }
};
}  // namespace fake_grid_map

int main(int argc, char **argv) {
  const bool star = argc > 1 && std::string(argv[1]) == "star";  // algorithm: rrt-star-connect
  // "seq": buildRRTConnect's sequential per-call search (set_engine_batch(0))
  const bool seq = argc > 1 && (std::string(argv[1]) == "seq" || std::string(argv[1]) == "dirseq");
  // "dir" / "dirseq": the direction-sampling parameters switched on
  // (config/params.yaml:21-27 with flag: true, forwarded as :193-205)
  const bool dir = argc > 1 && (std::string(argv[1]) == "dir" || std::string(argv[1]) == "dirseq");
  fake_grid_map::GridMap map{120, 60, 0.05, {}};
  map.z.assign((size_t)map.nx * map.ny, 0.0f);  // flat ground
  FastTerrainMap terrain_;
  terrain_.loadDataFromGridMap(map);  // global_body_planner.cpp:43

  State robot_start_ = {0.5, 1.5, 0.375, 1, 0, 0, 0, 0};
  State robot_goal_ = {4.5, 1.5, 0.375, 1, 0, 0, 0, 0};
  robot_start_[2] += terrain_.getGroundHeight(robot_start_[0], robot_start_[1]);  // :263
  robot_goal_[2] += terrain_.getGroundHeight(robot_goal_[0], robot_goal_[1]);     // :264

  RRTConnectClass rrt_connect_obj;                                    // :89
  RRTStarConnectClass rrt_star_connect_obj;                           // :90
  for (RRTClass *o : {(RRTClass *)&rrt_connect_obj, (RRTClass *)&rrt_star_connect_obj}) {
    o->set_state_action_pair_check_adaptive_step_size_flag_(false);   // :182 setPlannerParameter
    o->set_cost_add_yaw(false, 1.0, 1.0);                             // :190
    o->set_action_direction_sampling(dir, 0.1);
    o->set_state_direction_sampling(dir, 0.05, false);
  }
  if (dir) {
    // the free samplers (planning_utils.cpp:379-515): t_s fixed, t_f in range,
    // and on flat ground the direction variant's tangential forces follow the
    // velocity change (FORWARD: s_near -> s)
    const std::array<double, 3> up = {0.0, 0.0, 1.0};
    const State slow = {0, 0, 0.4, 0.1, 0.5, 0, 0, 0}, fast = {1, 0, 0.4, 1.0, -0.5, 0, 0, 0};
    for (int k = 0; k < 64; k++) {
      const Action a = getRandomAction(up);
      const Action d = getRandomActionDirection(up, slow, fast);
      const Action c = getRandomAction(up, FORWARD, true, 1.0, fast, slow);
      for (const Action *x : {&a, &d, &c})
        if ((*x)[6] != 0.3 || !((*x)[7] >= 0 && (*x)[7] < 0.5)) return 2;
      if (!(d[0] >= 0 && d[3] >= 0 && d[1] <= 0 && d[4] <= 0)) return 3;  // dx grows, dy shrinks
      if (!(c[0] >= 0 && c[3] >= 0 && c[1] <= 0 && c[4] <= 0)) return 4;
    }
  }
  if (seq) rrt_connect_obj.set_engine_batch(0);

  std::vector<State> state_sequence_;
  std::vector<Action> action_sequence_;
  if (!star)
    rrt_connect_obj.buildRRTConnect(terrain_, robot_start_, robot_goal_, state_sequence_,
                                    action_sequence_, 0.0);           // :115
  else
    rrt_star_connect_obj.buildRRTStarConnect(terrain_, robot_start_, robot_goal_, state_sequence_,
                                             action_sequence_, 1.0);  // :121
  RRTConnectClass &rrt_stats = star ? rrt_star_connect_obj : rrt_connect_obj;
  double plan_time, time_to_first_solve, path_duration;
  int success, vertices_generated;
  std::vector<double> length_vector, yaw_vector, cost_vector, cost_vector_times;
  std::vector<std::vector<double>> allStatePosition;
  rrt_stats.getStatistics(plan_time, success, vertices_generated, time_to_first_solve,
                                length_vector, yaw_vector, cost_vector, cost_vector_times,
                                path_duration, allStatePosition);     // :118
  std::vector<State> body_plan_;
  std::vector<double> t_plan_;
  std::vector<int> interp_phase;
  getInterpPath(state_sequence_, action_sequence_, 0.05, body_plan_, t_plan_, interp_phase);  // :131
  std::printf("states %zu actions %zu vertices %d plan_time %.3f path_duration %.3f interp %zu\n",
              state_sequence_.size(), action_sequence_.size(), vertices_generated, plan_time,
              path_duration, body_plan_.size());
  const bool ok = state_sequence_.size() >= 2 && state_sequence_.front() == robot_start_ &&
                  state_sequence_.back() == robot_goal_ &&
                  action_sequence_.size() + 1 == state_sequence_.size() &&
                  body_plan_.size() == t_plan_.size();
  return ok ? 0 : 1;
}
