// gbp_planner.h — C++ host mirror of the reference planner API over the C ABI.
//
// Same class / function names, argument meanings and return conventions as
// the reference (include/global_body_planner/{fast_terrain_map,planning_utils,
// planner_class,rrt,rrt_connect}.h), with every state-validity evaluation,
// terrain query, nearest-neighbour scan and candidate sampling executed by the
// HIP engine (include/gbp.h).  Namespace gbp_amd; include gbp_planner_compat.h
// for the reference's global names (the drop-in under the ROS node, see
// INTEGRATION.md).  No ROS / grid_map / Eigen dependency.
//
// Extensions beyond the reference surface (all batch-synchronous, B = 1
// reproduces the sequential algorithm on the engine's counter-based RNG):
//   planning_utils::isValidStateActionPairBatch, FastTerrainMap::*Batch,
//   PlannerClass::getNearestNeighborBatch, RRTConnectClass::buildRRTConnectBatched.
#pragma once

#include <array>
#include <chrono>
#include <stdexcept>
#include <type_traits>
#include <cstdint>
#include <string>
#include <vector>

#include "gbp.h"

namespace gbp_amd {

namespace planning_utils {
// include/global_body_planner/planning_utils.h:21-66
const double H_MAX = 0.4;
const double H_MIN = 0.075;
const double V_MAX = 2.0;
const double V_NOM = 0.75;
const double P_MAX = 1.0;
const double DP_MAX = 3.0;
const double ANG_ACC_MAX = 7.0;
const double ROBOT_L = 0.3;
const double ROBOT_W = 0.3;
const double ROBOT_H = 0.05;
const double M_CONST = 13;
const double G_CONST = 9.81;
const double F_MAX = 637;
const double MU = 1.0;
const double T_S_MIN = 0.3;
const double T_S_MAX = 0.3;
const double T_F_MIN = 0.0;
const double T_F_MAX = 0.5;
const double KINEMATICS_RES = 0.05;
const double BACKUP_TIME = 0.2;
const double BACKUP_RATIO = 0.5;
const int NUM_GEN_STATES = 6;
const double GOAL_BOUNDS = 0.5;
const int FLIGHT = 0;
const int STANCE = 1;
const int CONNECT_STANCE = 2;
const int FORWARD = 0;
const int REVERSE = 1;
const int POSEDIM = 3;
const int STATEDIM = 8;
const int ACTIONDIM = 10;
typedef std::array<double, STATEDIM> State;
typedef std::array<double, ACTIONDIM> Action;
typedef std::pair<State, Action> StateActionPair;
const double INFTY = 1.7976931348623157e308;
const double MY_PI = 3.14159;
}  // namespace planning_utils

using planning_utils::Action;
using planning_utils::State;

#define GBP_PLANNER_TRAPPED 0
#define GBP_PLANNER_ADVANCED 1
#define GBP_PLANNER_REACHED 2

// Thrown only by constructors / loaders when the engine reports an error
// (the reference's hot path has no error channel; the C ABI returns codes).
struct EngineError : std::runtime_error {
  int status;
  EngineError(int s, const std::string &what);
};

// ---- terrain ingest without ROS ---------------------------------------------
// TerrainMapPublisher::loadCSV (terrain_map_publisher.cpp:290-327): comma
// separated doubles per line, '#' lines skipped, unparsable fields reported
// on stdout and skipped (stod("nan") parses)
std::vector<std::vector<double>> loadCSV(const std::string &filename);

// The arrays FastTerrainMap holds after the reference's CSV -> grid_map ->
// FastTerrainMap path: TerrainMapPublisher::loadMapFromCSV (:330-370) sets a
// grid_map geometry with a FLOAT resolution (:343-346) and float layers
// (x-major transpose at :363-368); FastTerrainMap::loadDataFromGridMap
// (fast_terrain_map.cpp:31-91) reads the cell-centre positions back in
// reversed index order and casts the layers float -> double.  grid_map_core's
// setGeometry / getPosition arithmetic (GridMap.cpp, GridMapMath.cpp; not in
// this image) is restated: size = round(length / res), length = size * res,
// position(index) = (map_position + (0.5 length - 0.5 res)) + res * (-index).
struct TerrainArrays {
  int x_size = 0, y_size = 0;
  std::vector<double> x, y;           // ascending (x_data_, y_data_)
  std::vector<double> z, dx, dy, dz;  // x-major [x_size][y_size]
};
// dir holds xdata.csv, ydata.csv, zdata.csv, dxdata.csv, dydata.csv, dzdata.csv
// (data/<terrain_type>/ in the reference); throws std::runtime_error on a
// missing file or non-square cells (:347-348)
TerrainArrays terrainArraysFromCSV(const std::string &dir);

// ---- FastTerrainMap (fast_terrain_map.h:14-120) ------------------------------
class FastTerrainMap {
 public:
  explicit FastTerrainMap(int device = 0);
  // wrap an existing engine handle (not owned: the caller destroys it)
  static FastTerrainMap borrow(gbp_terrain *handle);
  FastTerrainMap(FastTerrainMap &&o) noexcept;
  ~FastTerrainMap();
  FastTerrainMap(const FastTerrainMap &) = delete;
  FastTerrainMap &operator=(const FastTerrainMap &) = delete;

  // fast_terrain_map.cpp:10-28 (x-major nested vectors, as the reference)
  void loadData(int x_size, int y_size, std::vector<double> x_data, std::vector<double> y_data,
                std::vector<std::vector<double>> z_data, std::vector<std::vector<double>> dx_data,
                std::vector<std::vector<double>> dy_data, std::vector<std::vector<double>> dz_data);
  // flat x-major variant (no nested-vector copies); dx/dy/dz may be null
  void loadDataFlat(int x_size, int y_size, const double *x, const double *y, const double *z,
                    const double *dx, const double *dy, const double *dz);
  // fast_terrain_map.cpp:31-91 for any map type exposing the grid_map calls
  // used there (getSize, getPosition, at, exists); see INTEGRATION.md
  template <class GridMap>
  void loadDataFromGridMap(const GridMap &map);
  // the node's map_data_source "csv" path without ROS (terrainArraysFromCSV)
  void loadMapFromCSV(const std::string &dir);

  double getGroundHeight(const double x, const double y);               // :94-132
  bool heightIsNan(const double x, const double y);                     // :135-157
  std::array<double, 3> getSurfaceNormal(const double x, const double y);  // :160-213
  const std::vector<double> &getXData() const { return x_data_; }       // :216-218
  const std::vector<double> &getYData() const { return y_data_; }       // :221-223

  // batched queries: xy[n][2]
  void getGroundHeightBatch(int64_t n, const double *xy, double *h, uint8_t *is_nan);
  void getSurfaceNormalBatch(int64_t n, const double *xy, double *normal);

  gbp_terrain *handle() const { return handle_; }
  int device() const { return device_; }

 private:
  int device_;
  gbp_terrain *handle_ = nullptr;
  bool owned_ = true;
  int x_size_ = 0, y_size_ = 0;
  std::vector<double> x_data_, y_data_;
};

namespace planning_utils {
// planning_utils.cpp:97-132, planning_utils.h:133-155
State interp(State q1, State q2, double x);
double poseDistance(const State &q1, const State &q2);
double stateDistance(const State &q1, const State &q2);
double stateYawDistance(const State &q1, const State &q2);
double stateDistance(const State &q1, const State &q2, bool cost_add_yaw_flag,
                     double cost_add_yaw_length_weight, double cost_add_yaw_yaw_weight);
bool isWithinBounds(State s1, State s2);
// planning_utils.cpp:237-370 (host arithmetic, identical expressions)
State applyStance(State s, Action a, double t);
State applyStance(State s, Action a);
State applyFlight(State s, double t_f);
State applyAction(State s, Action a);
State applyStanceReverse(State s, Action a, double t);
State applyStanceReverse(State s, Action a);
std::array<double, 3> rotate_grf(std::array<double, 3> surface_norm, std::array<double, 3> grf);
// planning_utils.cpp:519-556 (host arithmetic)
bool isValidAction(Action a);
// planning_utils.cpp:562-635 — evaluated by the engine
bool isValidState(State s, FastTerrainMap &terrain, int phase);
// planning_utils.cpp:645-881 — evaluated by the engine; s_new / t_new are
// written only where the reference writes them
bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain, State &s_new, double &t_new,
                            bool state_action_pair_check_adaptive_step_size_flag);
bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain, State &s_new, double &t_new);
bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain);
bool isValidStateActionPairAdaptiveStepSize(State s, Action a, FastTerrainMap &terrain,
                                            State &s_new, double &t_new);
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain, State &s_new,
                                   double &t_new, bool state_action_pair_check_adaptive_step_size_flag);
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain, State &s_new,
                                   double &t_new);
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain);
bool isValidStateActionPairReverseAdaptiveStepSize(State s, Action a, FastTerrainMap &terrain,
                                                   State &s_new, double &t_new);
// the hot path, batched: one engine launch for n pairs (direction per pair)
void isValidStateActionPairBatch(const std::vector<State> &s, const std::vector<Action> &a,
                                 const std::vector<uint8_t> &direction, FastTerrainMap &terrain,
                                 bool adaptive, std::vector<uint8_t> &valid,
                                 std::vector<State> &s_new, std::vector<double> &t_new,
                                 std::vector<uint32_t> *flags = nullptr);
// planning_utils.cpp:379-515 on the engine's counter-based stream (the
// reference's rand() / clock-seeded engines are not reproducible): draw k of
// the process's free-function stream (seed setRandomSeed, index k counting up
// per thread), sampled by the engine on device 0 (gbp_sample_actions_dir_host)
Action getRandomAction(std::array<double, 3> surf_norm, int direction,
                       bool action_direction_sampling_flag,
                       double action_direction_sampling_probability_threshold, State s,
                       State s_near);                                       // :379-391
Action getRandomAction(std::array<double, 3> surf_norm);                    // :392-442
Action getRandomActionDirection(std::array<double, 3> surf_norm, State s_from,
                                State s_to);                                // :443-515
void setRandomSeed(uint64_t seed);
// planning_utils.cpp:142-193
void interpStateActionPair(State s, Action a, double t0, double dt,
                           std::vector<State> &interp_path, std::vector<double> &interp_t,
                           std::vector<int> &interp_phase);
void getInterpPath(std::vector<State> state_sequence, std::vector<Action> action_sequence,
                   double dt, std::vector<State> &interp_path, std::vector<double> &interp_t,
                   std::vector<int> &interp_phase);
}  // namespace planning_utils

// ---- GraphClass + PlannerClass (graph_class.h, planner_class.h) --------------
// Vertices live in host vectors AND in a device mirror (flat double[V][8]) that
// the nearest-neighbour kernel scans.
class PlannerClass {
 public:
  explicit PlannerClass(int device = 0);
  ~PlannerClass();
  PlannerClass(const PlannerClass &o);
  PlannerClass &operator=(const PlannerClass &o);

  void init(State s, bool cost_add_yaw_flag = false, double cost_add_yaw_length_weight = 1,
            double cost_add_yaw_yaw_weight = 1);                           // graph_class.cpp:141-152
  void addVertex(int index, State s);                                      // :28-31
  State getVertex(int index) const { return vertices_[index]; }            // :18-20
  int getNumVertices() const { return (int)vertices_.size(); }             // :23-25
  void addEdge(int idx1, int idx2);                                        // :36-42
  void removeEdge(int idx1, int idx2);                                     // :44-58
  int getPredecessor(int idx) const;                                       // :62-68
  std::vector<int> getSuccessors(int idx) const { return successors_[idx]; }
  void addAction(int idx, Action a) { actions_[idx] = a; }                 // :75-77
  Action getAction(int idx) const { return actions_[idx]; }
  double getGValue(int idx) const { return g_[idx]; }
  double getYValue(int idx) const { return y_[idx]; }
  void updateGYValue(int idx, double g_val, double y_val);                 // :131-138

  // planner_class.cpp:38-76 on the engine sampler (stream = this tree's id)
  State randomState(FastTerrainMap &terrain);
  // planner_class.cpp:22-35: randomStateDirection with probability p, else
  // randomState (one draw of this tree's stream either way)
  State randomState(FastTerrainMap &terrain, bool state_direction_sampling_flag,
                    double state_direction_sampling_probability_threshold,
                    bool speed_direction_flag, State s_from, State s_to);
  // planner_class.cpp:82-148
  State randomStateDirection(FastTerrainMap &terrain, State s_from, State s_to,
                             bool speed_direction_flag);
  // n consecutive randomState draws of this tree's stream in one launch
  std::vector<State> randomStateBatch(FastTerrainMap &terrain, int n);
  // ... with the direction-biased variant of cfg (s_from / s_to for all n)
  std::vector<State> randomStateBatch(FastTerrainMap &terrain, int n, const gbp_sampling &cfg,
                                      const State &s_from, const State &s_to);
  // planner_class.cpp:185-200 on the engine (ties -> lowest index)
  int getNearestNeighbor(State q);
  std::vector<int> getNearestNeighborBatch(const std::vector<State> &q);
  std::vector<int> neighborhoodDist(State q, double dist);                 // :173-182
  // neighborhoodDist for many queries in one launch; query k only sees
  // vertices with index < limit[k] (limit empty: all), ascending index
  std::vector<std::vector<int>> neighborhoodDistBatch(const std::vector<State> &q, double dist,
                                                      const std::vector<int> &limit = {});
  // :151-171: the engine's k-nearest wavefront scan (N <= GBP_KNN_MAX, plain
  // stateDistance), else (cost_add_yaw's weighted distance) a host sort
  std::vector<int> neighborhoodN(State q, int N);

  void setStream(uint64_t seed, uint64_t stream_id) {
    seed_ = seed;
    stream_id_ = stream_id;
  }
  const std::vector<State> &vertices() const { return vertices_; }

 private:
  void sync_device();
  void sync_yaw();  // the vertices' glibc yaws on the device (cost_add_yaw neighborhoodN)
  void ensure_scratch(int64_t nq);
  int device_;
  std::vector<State> vertices_;
  std::vector<Action> actions_;
  std::vector<int> parent_;
  std::vector<std::vector<int>> successors_;
  std::vector<double> g_, y_;
  bool cost_add_yaw_flag_ = false;
  double cost_add_yaw_length_weight_ = 1, cost_add_yaw_yaw_weight_ = 1;
  double *d_vertices_ = nullptr;
  int64_t d_capacity_ = 0, d_count_ = 0;
  void *d_scratch_ = nullptr;   // nearest-neighbour queries [q][8] + indices [q]
  int64_t d_scratch_cap_ = 0;
  void *d_nbr_ = nullptr;       // neighbourhood queries + output lists
  size_t d_nbr_bytes_ = 0;
  double *d_yaw_ = nullptr;     // atan2(v[4], v[3]) per vertex (glibc), uploaded on demand
  int64_t d_yaw_cap_ = 0, d_yaw_count_ = 0;
  uint64_t seed_ = 1, stream_id_ = 100;
  int64_t draws_ = 0;
};

// ---- RRTClass / RRTConnectClass (rrt.h, rrt_connect.h) -------------------------
class RRTClass {
 public:
  RRTClass() = default;
  virtual ~RRTClass() = default;
  // rrt.cpp:20-70 (candidates drawn from the engine stream, checked in one launch)
  bool newConfig(State s, State s_near, State &s_new, Action &a_new, FastTerrainMap &terrain,
                 int direction);
  // rrt.cpp:77-102
  virtual int extend(PlannerClass &T, State s, FastTerrainMap &terrain, int direction);
  std::vector<int> pathFromStart(PlannerClass &T, int idx);                // rrt.cpp:107-118
  std::vector<State> getStateSequence(PlannerClass &T, std::vector<int> path);
  std::vector<Action> getActionSequence(PlannerClass &T, std::vector<int> path);
  // rrt.cpp:154-169 (same 10 outputs)
  void getStatistics(double &plan_time, int &success_var, int &vertices_generated,
                     double &time_to_first_solve, std::vector<double> &length_vector,
                     std::vector<double> &yaw_vector, std::vector<double> &cost_vector,
                     std::vector<double> &cost_vector_times, double &path_duration,
                     std::vector<std::vector<double>> &allStatePosition);
  void printPath(PlannerClass &T, std::vector<int> path);                  // rrt.cpp:143-152
  void saveStateSequence(PlannerClass &T);                                 // rrt.cpp:253-265
  // rrt.cpp:268-280 (params.yaml:21-27, off by default): newConfig's
  // candidates and every search's targets (sequential, batched and
  // device-resident) draw the direction-biased variants when a flag is on
  // (gbp_sampling, applied to the terrain handle the search runs on)
  void set_action_direction_sampling(bool flag, double threshold) {
    action_direction_sampling_flag_ = flag;
    action_direction_sampling_probability_threshold_ = threshold;
  }
  void set_state_direction_sampling(bool flag, double threshold, bool speed_direction_flag) {
    state_direction_sampling_flag_ = flag;
    state_direction_sampling_probability_threshold_ = threshold;
    state_direction_sampling_speed_direction_flag_ = speed_direction_flag;
  }
  void print_setting_parameters();
  void set_state_action_pair_check_adaptive_step_size_flag_(bool f) {
    state_action_pair_check_adaptive_step_size_flag_ = f;
  }
  void set_cost_add_yaw(bool flag, double lw, double yw) {
    cost_add_yaw_flag_ = flag;
    cost_add_yaw_length_weight_ = lw;
    cost_add_yaw_yaw_weight_ = yw;
  }
  void setSeed(uint64_t seed) { seed_ = seed; }
  // wall clock from the start of the build call to the first goal (the
  // reference's elapsed_to_first restarts with every tree pair)
  double wallTimeToFirst() const { return wall_to_first_; }
  // the last build's path cost / its history (rrt_connect.h getters' data)
  double pathCost() const { return path_cost_; }
  double pathLength() const { return path_length_; }
  double pathYaw() const { return path_yaw_; }
  // the reference's path cost: length, or the cost_add_yaw weighted sum
  // (rrt_connect.cpp:304-313, :193-215)
  double weightedCost(double length, double yaw) const {
    return cost_add_yaw_flag_ ? length * cost_add_yaw_length_weight_ + yaw * cost_add_yaw_yaw_weight_
                              : length;
  }
  const std::vector<double> &costHistory() const { return cost_vector_; }
  // this planner's direction-sampling parameters as the engine's gbp_sampling
  gbp_sampling samplingConfig() const;

 protected:
  // installs samplingConfig() on the terrain handle (the candidate sampler and
  // the device loop's targets read it there)
  void applySampling(FastTerrainMap &terrain) const;
  bool goal_found = false;
  std::chrono::duration<double> elapsed_total{0};
  std::chrono::duration<double> elapsed_to_first{0};
  double wall_to_first_ = -1;
  int success_ = 0;
  int num_vertices = 0;
  double path_length_ = 0, path_yaw_ = 0, path_cost_ = 0;
  std::vector<double> length_vector_, yaw_vector_, cost_vector_, cost_vector_times_;
  double path_duration_ = 0;
  std::vector<std::vector<double>> allStatePosition_;
  bool action_direction_sampling_flag_ = false;
  double action_direction_sampling_probability_threshold_ = 0.15;
  bool state_direction_sampling_flag_ = false;
  double state_direction_sampling_probability_threshold_ = 0.05;
  bool state_direction_sampling_speed_direction_flag_ = false;
  bool state_action_pair_check_adaptive_step_size_flag_ = false;
  bool cost_add_yaw_flag_ = false;
  double cost_add_yaw_length_weight_ = 1, cost_add_yaw_yaw_weight_ = 1;
  uint64_t seed_ = 20251018;
  int64_t extend_counter_ = 0;
};

// The final trees of a batched / device-resident search (for callers that
// replay it, e.g. against a CPU restatement): Ta = [0], Tb = [1].
struct TreeDump {
  std::vector<State> v[2];
  std::vector<Action> a[2];
  std::vector<int32_t> parent[2];
  std::vector<double> g[2];
};

struct BatchStats {
  int64_t max_halves = 0;     // in: stop after this many half-iterations (0 = no limit)
  TreeDump *dump = nullptr;   // in: receives the final trees when set
  // in (device loop): called after every group of halves with this rank's own
  // verdict (local_stop: found, out of time or halves) and whether it found a
  // path; returns nonzero to stop — config 4's ranks answer it with one
  // all_reduce(MAX) of local_stop, so they stop together
  int (*stop_poll)(void *ctx, int local_stop, int found) = nullptr;
  void *stop_ctx = nullptr;
  int64_t polls = 0;          // stop polls made
  int stopped_by_peer = 0;    // the poll stopped a search this rank would have continued
  int64_t halves = 0;         // half-iterations run
  int32_t meet_a = -1, meet_b = -1;  // the joined vertices (RRT*: the best pair)
  int64_t iterations = 0, targets = 0, extends = 0, attempts_checked = 0, connects = 0;
  int64_t vertices_a = 0, vertices_b = 0;
  int64_t rewires = 0, solutions = 0;
  int64_t depth_capped = 0;   // connects stopped at GBP_CONNECT_MAX_DEPTH (TRAPPED)
  int64_t status_reads = 0;   // device loop: host synchronisations
  int64_t fragile_resolved = 0;  // attempts re-decided on the host (GBP_F_RESOLVED)
  int64_t halts[4] = {0, 0, 0, 0};  // device loop: FRAGILE halts in the targets / extend /
                                    // connect / RRT* insertion stage (GBP_PLAN_HALT_*)
  int64_t star_grows = 0;           // device RRT*: insertion sets grown (GBP_PLAN_HALT_STAR_PAIRS)
  int64_t nn_rechecks = 0, nn_scans = 0;  // device loop with GBP_OPT_NN_STATS: the matrix-core
                                          // search's fp64 half-chunk re-checks / segment scans
  double extent_a[4] = {0, 0, 0, 0}, extent_b[4] = {0, 0, 0, 0};  // x_min x_max y_min y_max
  // in (device loop): a warm start, i.e. a replayable continuation of a search
  // (0 vertices = from the roots).  Tree k starts as warm_n[k] vertices (root
  // first, parents before children; g derived as graph_class.cpp:36-42 does),
  // the first half-iteration is warm_half (its targets are the draws a search
  // from the roots would make there) and the candidate stream starts at extend
  // index warm_extend.  max_halves then counts the continuation's halves.
  int64_t warm_n[2] = {0, 0};
  const double *warm_v[2] = {nullptr, nullptr};
  const double *warm_a[2] = {nullptr, nullptr};
  const int32_t *warm_parent[2] = {nullptr, nullptr};
  int64_t warm_half = 0, warm_extend = 0;
  // diagnostics (device loop): time each half-iteration's stage groups
  // (gbp_plan_stage_timing) into stage_us (half, stages 0-3, 6, 7, 4-5)
  bool stage_timing = false;
  double stage_us[7] = {0, 0, 0, 0, 0, 0, 0};
  int64_t stage_halves = 0;
};

class RRTConnectClass : public RRTClass {
 public:
  // rrt_connect.cpp:20-84 (recursive; the pair checks run on the engine)
  int attemptConnect(State s_existing, State s, double t_s, State &s_new, Action &a_new,
                     FastTerrainMap &terrain, int direction);
  // rrt_connect.cpp:85-91
  int attemptConnect(State s_existing, State s, State &s_new, Action &a_new, FastTerrainMap &terrain,
                     int direction);
  int connect(PlannerClass &T, State s, FastTerrainMap &terrain, int direction);  // :98-120
  std::vector<Action> getActionSequenceReverse(PlannerClass &T, std::vector<int> path);
  void postProcessPath(std::vector<State> &state_sequence, std::vector<Action> &action_sequence,
                       FastTerrainMap &terrain);                                    // :139-227
  void runRRTConnect(PlannerClass &Ta, PlannerClass &Tb, FastTerrainMap &terrain);  // :230-314
  void buildRRTConnect(FastTerrainMap &terrain, State s_start, State s_goal,
                       std::vector<State> &state_sequence, std::vector<Action> &action_sequence,
                       double max_time);                                            // :323-467

  // Batch-synchronous RRT-Connect: each half-iteration draws `batch` targets,
  // extends the tree toward all of them against the current snapshot (one
  // engine launch, 6 candidates each), inserts the non-TRAPPED successors in
  // target order, then connects every new vertex to the other tree with the
  // recursive attemptConnect run as lock-step rounds (one launch per round).
  // batch = 1 is runRRTConnect.  Stops at the first solution or max_time.
  bool buildRRTConnectBatched(FastTerrainMap &terrain, State s_start, State s_goal, int batch,
                              double max_time, std::vector<State> &state_sequence,
                              std::vector<Action> &action_sequence, BatchStats *stats = nullptr);

  // buildRRTConnectBatched with the whole search resident on the device
  // (include/gbp.h "device planner loop"): both trees live in HBM, every
  // half-iteration (targets, nearest neighbours, extends, appends, connects)
  // is one stream-ordered kernel sequence with no host round trip, and the
  // host reads one status record per group of half-iterations.  Same RNG
  // streams, same insertion order, same FRAGILE re-decisions as
  // buildRRTConnectBatched: for a given (seed, batch) both build the same trees
  // and return the same path.
  bool buildRRTConnectDevice(FastTerrainMap &terrain, State s_start, State s_goal, int batch,
                             double max_time, std::vector<State> &state_sequence,
                             std::vector<Action> &action_sequence, BatchStats *stats = nullptr,
                             uint64_t stream_a = 101, uint64_t stream_b = 102);

  // buildRRTConnect's anytime restarts (rrt_connect.cpp:323-467) on the
  // batch-synchronous half-iterations: fresh trees every restart, a restart
  // ends after anytime_horizon seconds (poseDistance(start, goal) /
  // planning_rate_estimate, x horizon_expansion_factor per restart) or at its
  // first REACHED connect; every solution is post-processed and the cheapest
  // (path_cost_) kept.  Stops once a solution exists and max_time_opt has
  // passed, or at max_time without one.  Returns the best path.
  // device_loop: each restart's search runs device-resident (buildRRTConnectDevice).
  bool buildRRTConnectBatchedAnytime(FastTerrainMap &terrain, State s_start, State s_goal,
                                     int batch, double max_time, double max_time_opt,
                                     std::vector<State> &state_sequence,
                                     std::vector<Action> &action_sequence,
                                     BatchStats *stats = nullptr, bool device_loop = false);

  // How buildRRTConnect (the call GlobalBodyPlanner::callPlanner makes,
  // global_body_planner.cpp:115) searches: batch > 0 (default 1024) runs its
  // restart loop on the device-resident batched search with that many random
  // targets per half-iteration; 0 runs the reference's sequential
  // runRRTConnect, one engine call per extend / connect.
  void set_engine_batch(int batch) { engine_batch_ = batch; }
  int engine_batch() const { return engine_batch_; }

  // attemptConnect for many independent pairs (lock-step rounds, one engine
  // launch per recursion depth); s_new / a_new are in/out per pair
  void attemptConnectBatchPublic(const std::vector<State> &s_existing, const std::vector<State> &s,
                                 std::vector<double> t_s, FastTerrainMap &terrain, int direction,
                                 std::vector<int> &result, std::vector<State> &s_new,
                                 std::vector<Action> &a_new) {
    attemptConnectBatch(s_existing, s, std::move(t_s), terrain, direction, result, s_new, a_new,
                        nullptr);
  }

 protected:
  double anytime_horizon = 0;
  const double planning_rate_estimate = 16.0;
  double horizon_expansion_factor = 1.2;
  const int max_time_solve = 4000;
  int engine_batch_ = 1024;

  // lock-step attemptConnect for many (s_existing, s, t_s) triples; with
  // max_depth = 0 only REACHED is decided (callers that test == REACHED)
  void attemptConnectBatch(const std::vector<State> &s_existing, const std::vector<State> &s,
                           std::vector<double> t_s, FastTerrainMap &terrain, int direction,
                           std::vector<int> &result, std::vector<State> &s_new,
                           std::vector<Action> &a_new, BatchStats *stats,
                           int max_depth = GBP_CONNECT_MAX_DEPTH);
  // connect each vertex `added` of T to the other tree O (rrt_connect.cpp:98-120,
  // in order, NN against O's snapshot); returns the (T vertex, O vertex) pairs
  // whose connect REACHED
  std::vector<std::pair<int, int>> connectBatch(PlannerClass &T, PlannerClass &O,
                                                FastTerrainMap &terrain, int dir,
                                                const std::vector<int> &added, BatchStats *stats);
  // draw `batch` targets, keep the STANCE-valid ones, extend T toward all of
  // them against T's snapshot; returns the inserted vertices (in target order),
  // their nearest vertices and actions.  With O, the targets are
  // randomState(terrain, state_direction_sampling_*, s_from, s_to) with the
  // reference's s_from / s_to (rrt_connect.cpp:248-252, :283-287) as the
  // trees stand when the half starts; without, plain randomState (RRT*).
  void extendBatch(PlannerClass &T, FastTerrainMap &terrain, int dir, int batch,
                   std::vector<int> &added, std::vector<int> &nearest, std::vector<Action> &a_new,
                   bool insert, BatchStats *stats, const PlannerClass *O = nullptr);
  int halfIterationBatched(PlannerClass &T, PlannerClass &O, FastTerrainMap &terrain, int dir,
                           int batch, int &meet_t, int &meet_o, BatchStats *stats);
};

// ---- RRTStarConnectClass (rrt_star_connect.h, rrt_star_connect.cpp) ------------
class RRTStarConnectClass : public RRTConnectClass {
 public:
  // rrt_star_connect.cpp:11-67: newConfig, then choose-parent among the
  // vertices within delta and rewire them through s_new (connects on the engine)
  int extend(PlannerClass &T, State s, FastTerrainMap &terrain, int direction) override;
  // rrt_star_connect.cpp:70-89
  void getStateAndActionSequences(PlannerClass &Ta, PlannerClass &Tb, int shared_a_idx,
                                  int shared_b_idx, std::vector<State> &state_sequence,
                                  std::vector<Action> &action_sequence);
  // rrt_star_connect.cpp:91-205
  void buildRRTStarConnect(FastTerrainMap &terrain, State s_start, State s_goal,
                           std::vector<State> &state_sequence,
                           std::vector<Action> &action_sequence, double max_time);
  // Batch-synchronous RRT*-Connect: as buildRRTConnectBatched, with every new
  // vertex inserted by choose-parent + rewire (its neighbourhood = the vertices
  // within delta that precede it, as in the sequential algorithm); all
  // neighbourhood scans of a batch run in one launch and all their connects in
  // one pair-check launch, the tree updates then replay sequentially in order.
  // Runs until max_time after the first solution (anytime), keeping the best.
  bool buildRRTStarConnectBatched(FastTerrainMap &terrain, State s_start, State s_goal, int batch,
                                  double max_time, std::vector<State> &state_sequence,
                                  std::vector<Action> &action_sequence, BatchStats *stats = nullptr);
  // The same search resident on the device: gbp_plan_halves_dev with the RRT*
  // insertion stages (gbp_plan_star_config: neighbourhoods, connect checks and
  // the ordered choose-parent / rewire replay in HBM, no per-vertex host
  // loop); same trees, counters and best connection as buildRRTStarConnectBatched
  // for the same seed and batch.  Runs pairs of half-iterations until max_time
  // (or stats->max_halves), reading the status once per group.
  bool buildRRTStarConnectDevice(FastTerrainMap &terrain, State s_start, State s_goal, int batch,
                                 double max_time, std::vector<State> &state_sequence,
                                 std::vector<Action> &action_sequence, BatchStats *stats = nullptr);
  double bestCost() const { return best_cost_; }
  int64_t rewires() const { return rewires_; }

 protected:
  const double delta = 3.0;  // rrt_star_connect.h:59
  double best_cost_ = INFINITY_COST;
  int64_t rewires_ = 0;
  static constexpr double INFINITY_COST = 1.7976931348623157e308;

 private:
  // choose-parent + rewire for the new vertices `added` of T (in order)
  void insertStar(PlannerClass &T, FastTerrainMap &terrain, int dir, const std::vector<int> &added,
                  const std::vector<int> &nearest, const std::vector<Action> &a_new,
                  BatchStats *stats);
};

// ---- implementation of the grid_map adapter (fast_terrain_map.cpp:31-91) -------
// Written against grid_map::GridMap's public API (getSize, getStartIndex,
// getPosition(Index, Position&), at(layer, Index), exists(layer)); a template
// so this header needs no grid_map build (not in this image; untested here).
template <class GridMap>
void FastTerrainMap::loadDataFromGridMap(const GridMap &map) {
  using Index = typename std::decay<decltype(map.getStartIndex())>::type;
  using Position = typename std::decay<decltype(map.getPosition())>::type;
  const int x_size = map.getSize()(0);
  const int y_size = map.getSize()(1);
  std::vector<double> x(x_size), y(y_size), z((size_t)x_size * y_size);
  const bool slopes = map.exists("dx");
  std::vector<double> dx, dy, dz;
  if (slopes) {
    dx.resize(z.size());
    dy.resize(z.size());
    dz.resize(z.size());
  }
  for (int i = 0; i < x_size; i++) {
    Index index((x_size - 1) - i, 0);
    Position position;
    map.getPosition(index, position);
    x[i] = position.x();
  }
  for (int i = 0; i < y_size; i++) {
    Index index(0, (y_size - 1) - i);
    Position position;
    map.getPosition(index, position);
    y[i] = position.y();
  }
  for (int i = 0; i < x_size; i++)
    for (int j = 0; j < y_size; j++) {
      Index index((x_size - 1) - i, (y_size - 1) - j);
      const size_t k = (size_t)i * y_size + j;
      z[k] = (double)map.at("elevation", index);
      if (slopes) {
        dx[k] = (double)map.at("dx", index);
        dy[k] = (double)map.at("dy", index);
        dz[k] = (double)map.at("dz", index);
      }
    }
  loadDataFlat(x_size, y_size, x.data(), y.data(), z.data(), slopes ? dx.data() : nullptr,
               slopes ? dy.data() : nullptr, slopes ? dz.data() : nullptr);
}

}  // namespace gbp_amd

// ---- flat C entry point of the batched planner (Python / bench) -------------
extern "C" {
typedef struct {
  int device, nx, ny;
  const double *x, *y, *z, *dx, *dy, *dz;  // x-major, dx/dy/dz may be NULL
  double start[8], goal[8];
  int batch;            // targets per half-iteration (1 = sequential runRRTConnect)
  double max_time;      // seconds
  uint64_t seed;
  int post_process;     // run postProcessPath on the found path
  int algorithm;        // 0 rrt-connect (first solution), 1 rrt-star-connect (anytime
                        // until max_time), 2 rrt-connect with the reference's anytime
                        // restarts (best post-processed path after max_time_opt),
                        // 3 rrt-connect with the search resident on the device
                        // (same trees and path as 0), 4 = 2 on the device-resident search,
                        // 5 = 1 with the search resident on the device (same trees)
  double max_time_opt;  // algorithm 2: keep restarting until a solution exists and this
                        // many seconds have passed (buildRRTConnect's max_time_opt)
  gbp_sampling sampling;  // direction-biased sampling (RRTClass::set_*_direction_sampling,
                          // params.yaml:21-27); all zero = off, the reference default
  int64_t fragile_eps_fm; // FRAGILE margin in 1e-15 units (GBP_OPT_FRAGILE_EPS); 0 = default
  int adaptive;           // state_action_pair_check_adaptive_step_size_flag (params.yaml:16)
  int nn_stats;           // GBP_OPT_NN_STATS: count the search's fp64 re-checks (diagnostics)
  int64_t max_halves;     // algorithms 0, 1, 3: stop after this many half-iterations
                          // (0 = no limit): a run that can be replayed exactly
  int64_t tree_capacity;  // rows of the tree_* buffers (0 = the trees are not returned)
  double *tree_v[2];      // algorithms 0, 1, 3: the final trees Ta / Tb — states [cap][8],
  double *tree_a[2];      //   the action reaching each vertex [cap][10] (root: zeros),
  int32_t *tree_parent[2];  // parents (root -1) and g values; rows past the result's
  double *tree_g[2];      //   vertices_a / vertices_b are not written
  int (*stop_poll)(void *ctx, int local_stop, int found);  // algorithm 3: see BatchStats
  void *stop_ctx;         //   (NULL: each run stops on its own)
  // algorithm 3: warm start (BatchStats::warm_*): init_n[k] vertices of tree k
  // (0 = the root given by start / goal), states [n][8], actions [n][10] and
  // parents [n] (root -1, parents before children); the first half-iteration
  // and the first extend index of the continuation
  int64_t init_n[2];
  const double *init_v[2];
  const double *init_a[2];
  const int32_t *init_parent[2];
  int64_t first_half;
  int64_t extend_base;
  int stage_timing;       // algorithms 3 / 5: time every half-iteration's stage groups
                          // (gbp_plan_stage_timing; diagnostics, adds events per half)
} gbp_plan_params;

typedef struct {
  int found;
  double time_to_first;  // wall seconds, build start -> first goal
  double total_time;
  int64_t iterations, targets, extends, attempts_checked, connects, vertices_a, vertices_b;
  int n_states;          // path states written (<= capacity)
  double path_length, path_cost, path_duration;
  int64_t rewires, solutions;  // RRT*: edges rewired, tree connections found
  double extent_a[4], extent_b[4];  // x_min, x_max, y_min, y_max of each tree's vertices
  int64_t fragile_resolved;    // decisions re-decided on the host with glibc (GBP_F_RESOLVED)
  int64_t depth_capped;        // connects stopped at GBP_CONNECT_MAX_DEPTH
  int64_t status_reads;        // algorithm 3: host synchronisations of the device loop
  int64_t halts[4];            // algorithm 3/4/5: FRAGILE halts in the targets / extend /
                               // connect / RRT* insertion stage of the device loop
  int64_t nn_rechecks, nn_scans;  // algorithm 3 with nn_stats: the matrix-core search's
                                  // fp64 half-chunk re-checks and segment scans
  double reported_length, reported_yaw;  // the planner's path_length_ / path_yaw_ (what
                                         // getStatistics reports; after postProcessPath
                                         // with its quirk, rrt_connect.cpp:202-215)
  int32_t meet_a, meet_b;      // algorithms 0 / 3: the vertices of Ta / Tb the first REACHED
                               // connect joined; algorithm 1: the best pair
  int64_t halves;              // half-iterations run
  int64_t polls;               // algorithm 3 with stop_poll: polls made
  int32_t stopped_by_peer;     // ... and 1 if another rank's solution ended this search
  double stage_us[7];          // with stage_timing: summed per-half microseconds
                               // (gbp_plan_stage_times: half, stages 0-3, 6, 7, 4-5,
                               // stage 6 before / in its pair checks)
  int64_t stage_halves;        //   over this many timed halves
} gbp_plan_result;

/* plans from start to goal; path_states[capacity][8] / path_actions[capacity][10]
 * (may be NULL).  Returns GBP_OK or a negative status. */
int gbp_plan_rrt_connect(const gbp_plan_params *p, gbp_plan_result *r, double *path_states,
                         double *path_actions, int capacity);

/* terrainArraysFromCSV (host only, no device): the FastTerrainMap arrays of
 * the reference's CSV -> grid_map -> FastTerrainMap path for the CSVs in dir.
 * Call with z == NULL to get nx / ny; then x[nx], y[ny], z/dx/dy/dz[nx][ny]
 * (x-major; any of dx/dy/dz may be NULL) are filled when capacity >= nx * ny.
 * Returns GBP_OK, GBP_E_SHAPE (capacity too small) or GBP_E_INVALID_ARG
 * (unreadable / non-square map). */
int gbp_terrain_arrays_from_csv(const char *dir, int *nx, int *ny, double *x, double *y,
                                double *z, double *dx, double *dy, double *dz, int64_t capacity);

/* RRTConnectClass::attemptConnect (rrt_connect.cpp:20-91) for n independent
 * (s_existing, s) pairs on an engine terrain handle, lock-step batched.
 * t_s[i] <= 0 (or t_s NULL) => poseDistance(s, s_existing) / V_NOM (:89).
 * s_new[n][8] / a_new[n][10] are in/out like the reference's references:
 * written only where the reference writes them.  result[i] = TRAPPED /
 * ADVANCED / REACHED. */
int gbp_attempt_connect_batch(gbp_terrain *t, int64_t n, const double *s_existing,
                              const double *s, const double *t_s, int direction, int adaptive,
                              int32_t *result, double *s_new, double *a_new);
}
