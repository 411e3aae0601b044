// Config 1 through the ROS node's own entry point, without ROS:
// GlobalBodyPlanner's map_data_source "csv" path (terrain_map_publisher.cpp
// :330-370 -> fast_terrain_map.cpp:31-91, here FastTerrainMap::loadMapFromCSV),
// setStartAndGoalStates (global_body_planner.cpp:209-265: z = 0.375 + ground,
// v = (1, 0, 0) for yaw 0) and callPlanner's rrt-connect branch
// (global_body_planner.cpp:89-131: buildRRTConnect with replan_time_limit,
// getStatistics, getInterpPath), written against the reference's global names.
//
//   node_config1 <csv dir> <engine batch: 0 = sequential> <seeds...>
// prints one JSON line per planner call (wall seconds, the statistics).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gbp_planner_compat.h"

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <csv dir> <engine batch> <seed>...\n", argv[0]);
    return 2;
  }
  FastTerrainMap terrain_;
  terrain_.loadMapFromCSV(argv[1]);
  const int batch = std::atoi(argv[2]);
  State robot_start_ = {1.0, 0.0, 0.375, 1, 0, 0, 0, 0};  // config 1: (1, 0) -> (8, 0)
  State robot_goal_ = {8.0, 0.0, 0.375, 1, 0, 0, 0, 0};
  robot_start_[2] += terrain_.getGroundHeight(robot_start_[0], robot_start_[1]);  // :263
  robot_goal_[2] += terrain_.getGroundHeight(robot_goal_[0], robot_goal_[1]);     // :264
  const double replan_time_limit_ = 0.0;  // first solution (SURVEY §6 config-1 protocol)
  int failures = 0;
  for (int k = 3; k < argc; k++) {
    RRTConnectClass rrt_connect_obj;  // :89
    rrt_connect_obj.set_state_action_pair_check_adaptive_step_size_flag_(false);
    rrt_connect_obj.set_cost_add_yaw(false, 1.0, 1.0);
    rrt_connect_obj.set_engine_batch(batch);
    rrt_connect_obj.setSeed(std::strtoull(argv[k], nullptr, 10));
    std::vector<State> state_sequence_;
    std::vector<Action> action_sequence_;
    const auto t0 = std::chrono::steady_clock::now();
    rrt_connect_obj.buildRRTConnect(terrain_, robot_start_, robot_goal_, state_sequence_,
                                    action_sequence_, replan_time_limit_);  // :115
    const double wall =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double plan_time, time_to_first_solve, path_duration;
    int success, vertices_generated;
    std::vector<double> length_vector, yaw_vector, cost_vector, cost_vector_times;
    std::vector<std::vector<double>> allStatePosition;
    rrt_connect_obj.getStatistics(plan_time, success, vertices_generated, time_to_first_solve,
                                  length_vector, yaw_vector, cost_vector, cost_vector_times,
                                  path_duration, allStatePosition);  // :118
    std::vector<State> body_plan_;
    std::vector<double> t_plan_;
    std::vector<int> interp_phase;
    getInterpPath(state_sequence_, action_sequence_, 0.05, body_plan_, t_plan_, interp_phase);
    const bool ok = state_sequence_.size() >= 2 && state_sequence_.front() == robot_start_ &&
                    state_sequence_.back() == robot_goal_ &&
                    action_sequence_.size() + 1 == state_sequence_.size();
    failures += ok ? 0 : 1;
    std::printf("{\"seed\": %s, \"engine_batch\": %d, \"wall_s\": %.6f, \"plan_time\": %.6f, "
                "\"time_to_first_solve\": %.6f, \"success\": %d, \"vertices\": %d, "
                "\"states\": %zu, \"path_duration\": %.4f, \"cost\": %.6f, \"ok\": %d}\n",
                argv[k], batch, wall, plan_time, time_to_first_solve, success, vertices_generated,
                state_sequence_.size(), path_duration,
                cost_vector.empty() ? -1.0 : cost_vector.back(), ok ? 1 : 0);
    std::fflush(stdout);
  }
  return failures ? 1 : 0;
}
