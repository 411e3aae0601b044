// gbp_planner.cpp — C++ host mirror of the reference planner over the C ABI.
// Compiled without FMA contraction (-ffp-contract=off) so the host arithmetic
// (propagation closed forms, isValidAction, distances, connect actions) is
// the reference's.  Every terrain query / state check / NN scan / candidate
// sampling goes through include/gbp.h (the HIP engine): there is no CPU
// evaluation of the validity path here.
#include "gbp_planner.h"
#include "../gbp_um_order.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <climits>
#include <fstream>
#include <numeric>
#include <sstream>

namespace gbp_amd {

EngineError::EngineError(int s, const std::string &what)
    : std::runtime_error(what + ": " + gbp_status_string(s)), status(s) {}

static void chk(int rc, const char *what) {
  if (rc != GBP_OK) throw EngineError(rc, what);
}

static inline double std_min(double a, double b) { return (b < a) ? b : a; }
static inline double std_max(double a, double b) { return (a < b) ? b : a; }

// ============================================================================
// terrain ingest (terrain_map_publisher.cpp:290-370, fast_terrain_map.cpp:31-91)
// ============================================================================
std::vector<std::vector<double>> loadCSV(const std::string &filename) {
  std::vector<std::vector<double>> data;
  std::ifstream input(filename);
  if (!input) throw std::runtime_error("File not found: " + filename);
  int l = 0;
  std::string line;
  while (std::getline(input, line)) {
    l++;
    if (!line.empty() && line[0] == '#') continue;  // :301 comment lines
    std::istringstream ss(line);
    std::vector<double> record;
    std::string num;
    while (std::getline(ss, num, ',')) {
      try {
        record.push_back(std::stod(num));
      } catch (const std::invalid_argument &) {  // :311-314
        std::printf("NaN found in file %s line %d\n", filename.c_str(), l);
      }
    }
    data.push_back(record);
  }
  return data;
}

TerrainArrays terrainArraysFromCSV(const std::string &dir) {
  const auto x_data = loadCSV(dir + "/xdata.csv");  // :333-338
  const auto y_data = loadCSV(dir + "/ydata.csv");
  const auto z_data = loadCSV(dir + "/zdata.csv");
  const auto dx_data = loadCSV(dir + "/dxdata.csv");
  const auto dy_data = loadCSV(dir + "/dydata.csv");
  const auto dz_data = loadCSV(dir + "/dzdata.csv");
  if (x_data.empty() || x_data[0].size() < 2 || y_data.size() < 2 || z_data.empty() ||
      y_data[0].empty() || y_data[1].empty())
    throw std::runtime_error("terrain CSVs too small in " + dir);
  const int x_size = (int)z_data[0].size();  // :341-342
  const int y_size = (int)z_data.size();
  const float x_res = x_data[0][1] - x_data[0][0];  // :343-344 (float)
  const float y_res = y_data[1][0] - y_data[0][0];
  const double x_length = x_data[0].back() - x_data[0].front() + x_res;  // :345-346
  const double y_length = y_data.back()[0] - y_data.front()[0] + y_res;
  if (x_res != y_res)  // :347-348
    throw std::runtime_error(
        "Map did not have square elements, make sure x and y resolution are equal.");
  // grid_map::GridMap::setGeometry(Length(x_length, y_length), x_res, Position(..)) (:352-356)
  const double res = x_res;
  const double pos[2] = {x_data[0].front() - 0.5 * x_res + 0.5 * x_length,
                         y_data.front()[0] - 0.5 * y_res + 0.5 * y_length};
  const int size[2] = {(int)std::round(x_length / res), (int)std::round(y_length / res)};
  const double length[2] = {size[0] * res, size[1] * res};
  if (size[0] != x_size || size[1] != y_size)
    throw std::runtime_error("grid_map size differs from the CSV size");
  for (const auto *layer : {&z_data, &dx_data, &dy_data, &dz_data}) {
    if ((int)layer->size() < y_size) throw std::runtime_error("short terrain layer in " + dir);
    for (int j = 0; j < y_size; j++)
      if ((int)(*layer)[j].size() < x_size) throw std::runtime_error("short terrain row in " + dir);
  }
  // GridMapMath getPositionFromIndex: map position + vector to the first cell
  // + resolution * (-index) (buffer start index 0)
  auto position = [&](int axis, int index) {
    const double to_first_cell = 0.5 * length[axis] - 0.5 * res;
    return (pos[axis] + to_first_cell) + res * (double)(-index);
  };
  TerrainArrays t;
  t.x_size = x_size;
  t.y_size = y_size;
  t.x.resize(x_size);
  t.y.resize(y_size);
  for (int i = 0; i < x_size; i++) t.x[i] = position(0, (x_size - 1) - i);  // fast_terrain_map.cpp:43-48
  for (int i = 0; i < y_size; i++) t.y[i] = position(1, (y_size - 1) - i);  // :49-54
  const size_t cells = (size_t)x_size * y_size;
  t.z.resize(cells);
  t.dx.resize(cells);
  t.dy.resize(cells);
  t.dz.resize(cells);
  // grid_map index (ix, iy) holds data[(y_size-1) - iy][(x_size-1) - ix] as a
  // float (:363-368); loadDataFromGridMap reads index ((x_size-1)-i, (y_size-1)-j)
  // into z_data[i][j] (:57-68): data[j][i]
  for (int i = 0; i < x_size; i++)
    for (int j = 0; j < y_size; j++) {
      const size_t k = (size_t)i * y_size + j;
      t.z[k] = (double)(float)z_data[j][i];
      t.dx[k] = (double)(float)dx_data[j][i];
      t.dy[k] = (double)(float)dy_data[j][i];
      t.dz[k] = (double)(float)dz_data[j][i];
    }
  return t;
}

// ============================================================================
// FastTerrainMap
// ============================================================================
FastTerrainMap::FastTerrainMap(int device) : device_(device) {}

void FastTerrainMap::loadMapFromCSV(const std::string &dir) {
  const TerrainArrays t = terrainArraysFromCSV(dir);
  loadDataFlat(t.x_size, t.y_size, t.x.data(), t.y.data(), t.z.data(), t.dx.data(), t.dy.data(),
               t.dz.data());
}

FastTerrainMap FastTerrainMap::borrow(gbp_terrain *handle) {
  FastTerrainMap m;
  int nx = 0, ny = 0, storage = 0, dev = 0;
  double b[4];
  chk(gbp_terrain_info(handle, &nx, &ny, &storage, b, &dev), "FastTerrainMap::borrow");
  m.device_ = dev;
  m.handle_ = handle;
  m.owned_ = false;
  m.x_size_ = nx;
  m.y_size_ = ny;
  // coordinate copies are not needed by the engine-backed queries; keep the
  // bounds so getXData().front()/back() hold the map edges
  m.x_data_ = {b[0], b[1]};
  m.y_data_ = {b[2], b[3]};
  return m;
}

FastTerrainMap::FastTerrainMap(FastTerrainMap &&o) noexcept
    : device_(o.device_), handle_(o.handle_), owned_(o.owned_), x_size_(o.x_size_),
      y_size_(o.y_size_), x_data_(std::move(o.x_data_)), y_data_(std::move(o.y_data_)) {
  o.handle_ = nullptr;
}

FastTerrainMap::~FastTerrainMap() {
  if (handle_ && owned_) gbp_terrain_destroy(handle_);
}

void FastTerrainMap::loadData(int x_size, int y_size, std::vector<double> x_data,
                              std::vector<double> y_data, std::vector<std::vector<double>> z_data,
                              std::vector<std::vector<double>> dx_data,
                              std::vector<std::vector<double>> dy_data,
                              std::vector<std::vector<double>> dz_data) {
  const size_t cells = (size_t)x_size * y_size;
  std::vector<double> z(cells), dx, dy, dz;
  const bool slopes = dx_data.size() == (size_t)x_size && dy_data.size() == (size_t)x_size &&
                      dz_data.size() == (size_t)x_size;
  if (slopes) {
    dx.resize(cells);
    dy.resize(cells);
    dz.resize(cells);
  }
  for (int i = 0; i < x_size; i++)
    for (int j = 0; j < y_size; j++) {
      const size_t k = (size_t)i * y_size + j;
      z[k] = z_data[i][j];
      if (slopes) {
        dx[k] = dx_data[i][j];
        dy[k] = dy_data[i][j];
        dz[k] = dz_data[i][j];
      }
    }
  loadDataFlat(x_size, y_size, x_data.data(), y_data.data(), z.data(),
               slopes ? dx.data() : nullptr, slopes ? dy.data() : nullptr,
               slopes ? dz.data() : nullptr);
}

void FastTerrainMap::loadDataFlat(int x_size, int y_size, const double *x, const double *y,
                                  const double *z, const double *dx, const double *dy,
                                  const double *dz) {
  gbp_terrain *h = nullptr;
  chk(gbp_terrain_create(device_, x_size, y_size, x, y, z, dx, dy, dz, GBP_STORAGE_AUTO, &h),
      "gbp_terrain_create");
  if (handle_ && owned_) gbp_terrain_destroy(handle_);
  handle_ = h;
  owned_ = true;
  x_size_ = x_size;
  y_size_ = y_size;
  x_data_.assign(x, x + x_size);
  y_data_.assign(y, y + y_size);
}

double FastTerrainMap::getGroundHeight(const double x, const double y) {
  const double xy[2] = {x, y};
  double h;
  chk(gbp_height_batch_host(handle_, 1, xy, &h, nullptr, nullptr), "getGroundHeight");
  return h;
}

bool FastTerrainMap::heightIsNan(const double x, const double y) {
  const double xy[2] = {x, y};
  uint8_t n;
  chk(gbp_height_batch_host(handle_, 1, xy, nullptr, &n, nullptr), "heightIsNan");
  return n != 0;
}

std::array<double, 3> FastTerrainMap::getSurfaceNormal(const double x, const double y) {
  const double xy[2] = {x, y};
  std::array<double, 3> n;
  chk(gbp_normal_batch_host(handle_, 1, xy, n.data(), nullptr), "getSurfaceNormal");
  return n;
}

void FastTerrainMap::getGroundHeightBatch(int64_t n, const double *xy, double *h,
                                          uint8_t *is_nan) {
  chk(gbp_height_batch_host(handle_, n, xy, h, is_nan, nullptr), "getGroundHeightBatch");
}

void FastTerrainMap::getSurfaceNormalBatch(int64_t n, const double *xy, double *normal) {
  chk(gbp_normal_batch_host(handle_, n, xy, normal, nullptr), "getSurfaceNormalBatch");
}

// ============================================================================
// planning_utils
// ============================================================================
namespace planning_utils {

static uint64_t g_seed = 20251018;
static int64_t g_action_draws = 0;

void setRandomSeed(uint64_t seed) {
  g_seed = seed;
  g_action_draws = 0;
}

State interp(State q1, State q2, double x) {  // planning_utils.cpp:97-103
  State q;
  for (int d = 0; d < 8; d++) q[d] = (q2[d] - q1[d]) * x + q1[d];
  return q;
}

double poseDistance(const State &q1, const State &q2) {  // :106-115
  double sum = 0;
  for (int i = 0; i < POSEDIM; i++) sum = sum + (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return std::sqrt(sum);
}

double stateDistance(const State &q1, const State &q2) {  // :116-127
  double sum = 0;
  for (int i = 0; i < 8; i++) sum = sum + 1.0 * (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return std::sqrt(sum);
}

double stateYawDistance(const State &q1, const State &q2) {  // planning_utils.h:133-145
  const double yaw1 = std::atan2(q1[4], q1[3]);
  const double yaw2 = std::atan2(q2[4], q2[3]);
  const double yaw_min = std_min(yaw1, yaw2), yaw_max = std_max(yaw1, yaw2);
  return std_min(yaw_max - yaw_min, yaw_min + 2 * MY_PI - yaw_max);
}

double stateDistance(const State &q1, const State &q2, bool f, double lw, double yw) {
  if (f) return poseDistance(q1, q2) * lw + stateYawDistance(q1, q2) * yw;
  return stateDistance(q1, q2);
}

bool isWithinBounds(State s1, State s2) { return stateDistance(s1, s2) <= GOAL_BOUNDS; }

State applyStance(State s, Action a, double t) {  // :237-274
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  State o;
  o[0] = s[0] + s[3] * t + 0.5 * a_x_td * t * t + (a_x_to - a_x_td) * (t * t * t) / (6.0 * t_s);
  o[1] = s[1] + s[4] * t + 0.5 * a_y_td * t * t + (a_y_to - a_y_td) * (t * t * t) / (6.0 * t_s);
  o[2] = s[2] + s[5] * t + 0.5 * a_z_td * t * t + (a_z_to - a_z_td) * (t * t * t) / (6.0 * t_s);
  o[3] = s[3] + a_x_td * t + (a_x_to - a_x_td) * t * t / (2.0 * t_s);
  o[4] = s[4] + a_y_td * t + (a_y_to - a_y_td) * t * t / (2.0 * t_s);
  o[5] = s[5] + a_z_td * t + (a_z_to - a_z_td) * t * t / (2.0 * t_s);
  o[6] = s[6] + s[7] * t + 0.5 * a_p_td * t * t + (a_p_to - a_p_td) * (t * t * t) / (6.0 * t_s);
  o[7] = s[7] + a_p_td * t + (a_p_to - a_p_td) * t * t / (2.0 * t_s);
  return o;
}

State applyStance(State s, Action a) { return applyStance(s, a, a[6]); }

State applyFlight(State s, double t_f) {  // :282-306
  const double g = 9.81;
  State o;
  o[0] = s[0] + s[3] * t_f;
  o[1] = s[1] + s[4] * t_f;
  o[2] = s[2] + s[5] * t_f - 0.5 * g * t_f * t_f;
  o[3] = s[3];
  o[4] = s[4];
  o[5] = s[5] - g * t_f;
  o[6] = s[6] + s[7] * t_f;
  o[7] = s[7];
  return o;
}

State applyAction(State s, Action a) { return applyFlight(applyStance(s, a), a[7]); }

State applyStanceReverse(State s, Action a, double t) {  // :324-367
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  const double cx = s[3] - a_x_td * t_s - 0.5 * (a_x_to - a_x_td) * t_s;
  const double cy = s[4] - a_y_td * t_s - 0.5 * (a_y_to - a_y_td) * t_s;
  const double cz = s[5] - a_z_td * t_s - 0.5 * (a_z_to - a_z_td) * t_s;
  const double cp = s[7] - a_p_td * t_s - 0.5 * (a_p_to - a_p_td) * t_s;
  State o;
  o[0] = s[0] - cx * (t_s - t) - 0.5 * a_x_td * (t_s * t_s - t * t) -
         (a_x_to - a_x_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  o[1] = s[1] - cy * (t_s - t) - 0.5 * a_y_td * (t_s * t_s - t * t) -
         (a_y_to - a_y_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  o[2] = s[2] - cz * (t_s - t) - 0.5 * a_z_td * (t_s * t_s - t * t) -
         (a_z_to - a_z_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  o[3] = s[3] - a_x_td * (t_s - t) - (a_x_to - a_x_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  o[4] = s[4] - a_y_td * (t_s - t) - (a_y_to - a_y_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  o[5] = s[5] - a_z_td * (t_s - t) - (a_z_to - a_z_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  o[7] = s[7] - a_p_td * (t_s - t) - (a_p_to - a_p_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  o[6] = s[6] - cp * (t_s - t) - 0.5 * a_p_td * (t_s * t_s - t * t) -
         (a_p_to - a_p_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  return o;
}

State applyStanceReverse(State s, Action a) { return applyStanceReverse(s, a, 0); }

std::array<double, 3> rotate_grf(std::array<double, 3> n, std::array<double, 3> f) {  // :198-231
  const double v0 = n[1] * 1.0 - n[2] * 0.0, v1 = n[2] * 0.0 - n[0] * 1.0,
               v2 = n[0] * 0.0 - n[1] * 0.0;
  const double s = std::sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  const double c = n[0] * 0.0 + n[1] * 0.0 + n[2] * 1.0;
  if (s < 0.000001) return f;
  const double K[3][3] = {{0, -v2, v1}, {v2, 0, -v0}, {-v1, v0, 0}};
  std::array<double, 3> out;
  for (int i = 0; i < 3; i++) {
    double acc = 0;
    for (int j = 0; j < 3; j++) {
      const double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
      const double r = (i == j ? 1.0 : 0.0) + K[i][j] + kk * (1 - c) / (s * s);
      acc = j == 0 ? r * f[0] : acc + r * f[j];
    }
    out[i] = acc;
  }
  return out;
}

bool isValidAction(Action a) {  // :519-556
  if ((a[6] <= 0) || (a[7] < 0)) return false;
  const double m = M_CONST, g = G_CONST, mu = MU;
  const double f_x_td = m * a[0], f_y_td = m * a[1], f_z_td = m * (a[2] + g);
  const double f_x_to = m * a[3], f_y_to = m * a[4], f_z_to = m * (a[5] + g);
  if ((std::sqrt(f_x_td * f_x_td + f_y_td * f_y_td + f_z_td * f_z_td) >= F_MAX) ||
      (std::sqrt(f_x_to * f_x_to + f_y_to * f_y_to + f_z_to * f_z_to) >= F_MAX) || (f_z_td < 0) ||
      (f_z_to < 0) || (a[8] >= F_MAX) || (a[9] >= F_MAX))
    return false;
  if ((std::sqrt(f_x_td * f_x_td + f_y_td * f_y_td) >= mu * f_z_td) ||
      (std::sqrt(f_x_to * f_x_to + f_y_to * f_y_to) >= mu * f_z_to))
    return false;
  return true;
}

bool isValidState(State s, FastTerrainMap &terrain, int phase) {
  uint8_t v;
  chk(gbp_valid_states_host(terrain.handle(), 1, s.data(), nullptr, phase, &v, nullptr, nullptr),
      "isValidState");
  return v != 0;
}

static bool pair1(State &s, Action &a, FastTerrainMap &terrain, State &s_new, double &t_new,
                  int direction, bool adaptive) {
  uint8_t v;
  uint32_t f;
  chk(gbp_validate_pairs_host(terrain.handle(), 1, s.data(), a.data(), nullptr, direction,
                              adaptive ? 1 : 0, &v, s_new.data(), &t_new, &f, nullptr),
      "isValidStateActionPair");
  return v != 0;
}

bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain, State &s_new, double &t_new,
                            bool adaptive) {
  return pair1(s, a, terrain, s_new, t_new, FORWARD, adaptive);
}
bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain, State &s_new,
                            double &t_new) {
  return pair1(s, a, terrain, s_new, t_new, FORWARD, false);
}
bool isValidStateActionPair(State s, Action a, FastTerrainMap &terrain) {
  State d{};
  double t = 0;
  return pair1(s, a, terrain, d, t, FORWARD, false);
}
bool isValidStateActionPairAdaptiveStepSize(State s, Action a, FastTerrainMap &terrain,
                                            State &s_new, double &t_new) {
  return pair1(s, a, terrain, s_new, t_new, FORWARD, true);
}
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain, State &s_new,
                                   double &t_new, bool adaptive) {
  return pair1(s, a, terrain, s_new, t_new, REVERSE, adaptive);
}
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain, State &s_new,
                                   double &t_new) {
  return pair1(s, a, terrain, s_new, t_new, REVERSE, false);
}
bool isValidStateActionPairReverse(State s, Action a, FastTerrainMap &terrain) {
  State d{};
  double t = 0;
  return pair1(s, a, terrain, d, t, REVERSE, false);
}
bool isValidStateActionPairReverseAdaptiveStepSize(State s, Action a, FastTerrainMap &terrain,
                                                   State &s_new, double &t_new) {
  return pair1(s, a, terrain, s_new, t_new, REVERSE, true);
}

void isValidStateActionPairBatch(const std::vector<State> &s, const std::vector<Action> &a,
                                 const std::vector<uint8_t> &direction, FastTerrainMap &terrain,
                                 bool adaptive, std::vector<uint8_t> &valid,
                                 std::vector<State> &s_new, std::vector<double> &t_new,
                                 std::vector<uint32_t> *flags) {
  const int64_t n = (int64_t)s.size();
  valid.resize(n);
  s_new.resize(n);
  t_new.resize(n);
  std::vector<uint32_t> f(n);
  if (n == 0) return;
  chk(gbp_validate_pairs_host(terrain.handle(), n, s[0].data(), a[0].data(),
                              direction.empty() ? nullptr : direction.data(), FORWARD,
                              adaptive ? 1 : 0, valid.data(), s_new[0].data(), t_new.data(),
                              f.data(), nullptr),
      "isValidStateActionPairBatch");
  if (flags) flags->swap(f);
}

// The free samplers draw from their own counter stream on a minimal engine
// handle of device 0 (the sampler reads no terrain; the handle carries the
// stream's workspace).  It lives as long as the thread's process: it is not
// destroyed at exit, where the HIP runtime may already be gone.
static constexpr uint64_t FREE_ACTION_STREAM = 0x46524545ull;  // "FREE"

static Action free_action(const std::array<double, 3> &n, int direction, const gbp_sampling &cfg,
                          const State &s, const State &s_near) {
  static thread_local gbp_terrain *h = nullptr;
  if (!h) {
    const double xy[2] = {0.0, 1.0}, z[4] = {0.0, 0.0, 0.0, 0.0};
    chk(gbp_terrain_create(0, 2, 2, xy, xy, z, nullptr, nullptr, nullptr, GBP_STORAGE_AUTO, &h),
        "getRandomAction handle");
  }
  Action a;
  chk(gbp_sample_actions_dir_host(h, 1, n.data(), s.data(), s_near.data(), nullptr, direction, &cfg,
                                  g_seed, FREE_ACTION_STREAM, g_action_draws++, a.data()),
      "getRandomAction");
  return a;
}

Action getRandomAction(std::array<double, 3> surf_norm, int direction,
                       bool action_direction_sampling_flag,
                       double action_direction_sampling_probability_threshold, State s,
                       State s_near) {  // planning_utils.cpp:379-391
  gbp_sampling cfg{};
  cfg.action_flag = action_direction_sampling_flag ? 1 : 0;
  cfg.action_p = action_direction_sampling_probability_threshold;
  return free_action(surf_norm, direction, cfg, s, s_near);
}

Action getRandomAction(std::array<double, 3> surf_norm) {  // :392-442
  const State z{};
  return free_action(surf_norm, FORWARD, gbp_sampling{}, z, z);
}

Action getRandomActionDirection(std::array<double, 3> surf_norm, State s_from,
                                State s_to) {  // :443-515
  gbp_sampling cfg{};
  cfg.action_flag = 1;
  cfg.action_p = 2.0;  // the coin always lands: the direction variant itself
  // FORWARD draws getRandomActionDirection(surf_norm, s_near, s)
  return free_action(surf_norm, FORWARD, cfg, s_to, s_from);
}

void interpStateActionPair(State s, Action a, double t0, double dt, std::vector<State> &path,
                           std::vector<double> &ts, std::vector<int> &phase) {  // :142-173
  const double t_s = a[6], t_f = a[7];
  for (double t = 0; t < t_s; t += dt) {
    ts.push_back(t + t0);
    path.push_back(applyStance(s, a, t));
    phase.push_back(t_f == 0 ? CONNECT_STANCE : STANCE);
  }
  const State s_takeoff = applyStance(s, a);
  for (double t = 0; t < t_f; t += dt) {
    ts.push_back(t_s + t + t0);
    path.push_back(applyFlight(s_takeoff, t));
    phase.push_back(FLIGHT);
  }
  if (t_f > 0) {
    ts.push_back(t0 + t_s + t_f);
    path.push_back(applyFlight(s_takeoff, t_f));
    phase.push_back(STANCE);
  }
}

void getInterpPath(std::vector<State> states, std::vector<Action> actions, double dt,
                   std::vector<State> &path, std::vector<double> &ts,
                   std::vector<int> &phase) {  // :182-193
  double t0 = 0;
  for (size_t i = 0; i < actions.size(); i++) {
    interpStateActionPair(states[i], actions[i], t0, dt, path, ts, phase);
    t0 += (actions[i][6] + actions[i][7]);
  }
  ts.push_back(t0);
  path.push_back(states.back());
}

}  // namespace planning_utils

using namespace planning_utils;

// ============================================================================
// PlannerClass
// ============================================================================
PlannerClass::PlannerClass(int device) : device_(device) {}

PlannerClass::~PlannerClass() {
  if (d_vertices_) gbp_device_free(d_vertices_);
  if (d_scratch_) gbp_device_free(d_scratch_);
  if (d_nbr_) gbp_device_free(d_nbr_);
  if (d_yaw_) gbp_device_free(d_yaw_);
}

PlannerClass::PlannerClass(const PlannerClass &o)
    : device_(o.device_), vertices_(o.vertices_), actions_(o.actions_), parent_(o.parent_),
      successors_(o.successors_), g_(o.g_), y_(o.y_), cost_add_yaw_flag_(o.cost_add_yaw_flag_),
      cost_add_yaw_length_weight_(o.cost_add_yaw_length_weight_),
      cost_add_yaw_yaw_weight_(o.cost_add_yaw_yaw_weight_), seed_(o.seed_),
      stream_id_(o.stream_id_), draws_(o.draws_) {}

PlannerClass &PlannerClass::operator=(const PlannerClass &o) {
  if (this == &o) return *this;
  if (d_vertices_) gbp_device_free(d_vertices_);
  if (d_scratch_) gbp_device_free(d_scratch_);
  if (d_nbr_) gbp_device_free(d_nbr_);
  if (d_yaw_) gbp_device_free(d_yaw_);
  d_vertices_ = nullptr;
  d_scratch_ = nullptr;
  d_nbr_ = nullptr;
  d_yaw_ = nullptr;
  d_capacity_ = d_count_ = d_scratch_cap_ = 0;
  d_yaw_cap_ = d_yaw_count_ = 0;
  d_nbr_bytes_ = 0;
  device_ = o.device_;
  vertices_ = o.vertices_;
  actions_ = o.actions_;
  parent_ = o.parent_;
  successors_ = o.successors_;
  g_ = o.g_;
  y_ = o.y_;
  cost_add_yaw_flag_ = o.cost_add_yaw_flag_;
  cost_add_yaw_length_weight_ = o.cost_add_yaw_length_weight_;
  cost_add_yaw_yaw_weight_ = o.cost_add_yaw_yaw_weight_;
  seed_ = o.seed_;
  stream_id_ = o.stream_id_;
  draws_ = o.draws_;
  return *this;
}

void PlannerClass::init(State s, bool f, double lw, double yw) {  // graph_class.cpp:141-152
  vertices_.clear();
  actions_.clear();
  parent_.clear();
  successors_.clear();
  g_.clear();
  y_.clear();
  d_count_ = 0;
  d_yaw_count_ = 0;
  addVertex(0, s);
  g_[0] = 0;
  y_[0] = 0;
  cost_add_yaw_flag_ = f;
  cost_add_yaw_length_weight_ = lw;
  cost_add_yaw_yaw_weight_ = yw;
}

void PlannerClass::addVertex(int idx, State s) {
  if (idx >= (int)vertices_.size()) {
    vertices_.resize(idx + 1);
    actions_.resize(idx + 1);
    parent_.resize(idx + 1, -1);
    successors_.resize(idx + 1);
    g_.resize(idx + 1, 0);
    y_.resize(idx + 1, 0);
  }
  vertices_[idx] = s;
  if (idx < d_count_) d_count_ = idx;  // re-upload from here
  if (idx < d_yaw_count_) d_yaw_count_ = idx;
}

void PlannerClass::addEdge(int idx1, int idx2) {  // graph_class.cpp:36-42
  parent_[idx2] = idx1;
  successors_[idx1].push_back(idx2);
  g_[idx2] = g_[idx1] + poseDistance(vertices_[idx1], vertices_[idx2]);
  y_[idx2] = y_[idx1] + stateYawDistance(vertices_[idx1], vertices_[idx2]);
}

void PlannerClass::removeEdge(int idx1, int idx2) {  // graph_class.cpp:44-58
  if (parent_[idx2] == idx1) parent_[idx2] = -1;
  std::vector<int> &succ = successors_[idx1];
  for (auto it = succ.begin(); it != succ.end(); ++it)
    if (*it == idx2) {
      succ.erase(it);
      break;
    }
}

int PlannerClass::getPredecessor(int idx) const { return parent_[idx]; }

void PlannerClass::updateGYValue(int idx, double g_val, double y_val) {  // :131-138
  g_[idx] = g_val;
  y_[idx] = y_val;
  for (int succ : successors_[idx])
    updateGYValue(succ, g_[idx] + poseDistance(vertices_[idx], vertices_[succ]),
                  y_[idx] + stateYawDistance(vertices_[idx], vertices_[succ]));
}

void PlannerClass::sync_device() {
  const int64_t V = (int64_t)vertices_.size();
  if (V > d_capacity_) {
    int64_t cap = std::max<int64_t>(1024, d_capacity_);
    while (cap < V) cap *= 2;
    void *p = nullptr;
    chk(gbp_device_alloc(device_, (size_t)cap * sizeof(State), &p), "tree alloc");
    if (d_vertices_) gbp_device_free(d_vertices_);
    d_vertices_ = (double *)p;
    d_capacity_ = cap;
    d_count_ = 0;
  }
  if (d_count_ < V) {
    chk(gbp_memcpy_h2d(d_vertices_ + 8 * d_count_, vertices_[d_count_].data(),
                       (size_t)(V - d_count_) * sizeof(State), nullptr),
        "tree upload");
    chk(gbp_stream_synchronize(nullptr), "tree upload");  // pageable source
    d_count_ = V;
  }
}

void PlannerClass::sync_yaw() {
  const int64_t V = (int64_t)vertices_.size();
  if (V > d_yaw_cap_) {
    int64_t cap = std::max<int64_t>(1024, d_yaw_cap_);
    while (cap < V) cap *= 2;
    void *p = nullptr;
    chk(gbp_device_alloc(device_, (size_t)cap * sizeof(double), &p), "yaw alloc");
    if (d_yaw_) gbp_device_free(d_yaw_);
    d_yaw_ = (double *)p;
    d_yaw_cap_ = cap;
    d_yaw_count_ = 0;
  }
  if (d_yaw_count_ < V) {
    std::vector<double> y((size_t)(V - d_yaw_count_));
    for (int64_t i = d_yaw_count_; i < V; i++) y[i - d_yaw_count_] = gbp_host_yaw(vertices_[i].data());
    chk(gbp_memcpy_h2d(d_yaw_ + d_yaw_count_, y.data(), y.size() * sizeof(double), nullptr),
        "yaw upload");
    chk(gbp_stream_synchronize(nullptr), "yaw upload");  // pageable source
    d_yaw_count_ = V;
  }
}

State PlannerClass::randomState(FastTerrainMap &terrain) {  // planner_class.cpp:38-76
  State q;
  int32_t tries;
  chk(gbp_sample_states_host(terrain.handle(), 1, seed_, stream_id_, draws_++, -1, 1, q.data(),
                             &tries),
      "randomState");
  return q;
}

State PlannerClass::randomState(FastTerrainMap &terrain, bool flag, double p,
                                bool speed_direction_flag, State s_from,
                                State s_to) {  // planner_class.cpp:22-35
  gbp_sampling cfg{};
  cfg.state_flag = flag ? 1 : 0;
  cfg.state_p = p;
  cfg.state_speed_direction = speed_direction_flag ? 1 : 0;
  return randomStateBatch(terrain, 1, cfg, s_from, s_to)[0];
}

State PlannerClass::randomStateDirection(FastTerrainMap &terrain, State s_from, State s_to,
                                         bool speed_direction_flag) {  // :82-148
  return randomState(terrain, true, 2.0, speed_direction_flag, s_from, s_to);  // the coin always lands
}

std::vector<State> PlannerClass::randomStateBatch(FastTerrainMap &terrain, int n,
                                                  const gbp_sampling &cfg, const State &s_from,
                                                  const State &s_to) {
  std::vector<State> q(n);
  if (n <= 0) return q;
  chk(gbp_sample_states_dir_host(terrain.handle(), n, seed_, stream_id_, draws_, &cfg,
                                 s_from.data(), s_to.data(), q[0].data()),
      "randomState(direction)");
  draws_ += n;
  return q;
}

std::vector<State> PlannerClass::randomStateBatch(FastTerrainMap &terrain, int n) {
  std::vector<State> q(n);
  if (n <= 0) return q;
  std::vector<int32_t> tries(n);
  chk(gbp_sample_states_host(terrain.handle(), n, seed_, stream_id_, draws_, -1, 1, q[0].data(),
                             tries.data()),
      "randomStateBatch");
  draws_ += n;
  return q;
}

void PlannerClass::ensure_scratch(int64_t nq) {
  if (nq <= d_scratch_cap_) return;
  int64_t cap = std::max<int64_t>(256, d_scratch_cap_);
  while (cap < nq) cap *= 2;
  void *p = nullptr;
  chk(gbp_device_alloc(device_, (size_t)cap * (sizeof(State) + sizeof(int32_t)), &p),
      "nn scratch alloc");
  if (d_scratch_) gbp_device_free(d_scratch_);
  d_scratch_ = p;
  d_scratch_cap_ = cap;
}

std::vector<int> PlannerClass::getNearestNeighborBatch(const std::vector<State> &q) {
  std::vector<int> idx(q.size(), 0);
  if (q.empty()) return idx;
  sync_device();
  const int64_t nq = (int64_t)q.size();
  ensure_scratch(nq);
  double *dq = (double *)d_scratch_;
  int32_t *di = (int32_t *)(dq + 8 * d_scratch_cap_);
  std::vector<int32_t> out(nq);
  chk(gbp_memcpy_h2d(dq, q[0].data(), (size_t)nq * sizeof(State), nullptr), "nn upload");
  chk(gbp_nearest_batch_dev(nq, dq, (int64_t)vertices_.size(), d_vertices_, di, nullptr, nullptr),
      "getNearestNeighbor");
  chk(gbp_memcpy_d2h(out.data(), di, (size_t)nq * sizeof(int32_t), nullptr), "nn download");
  chk(gbp_stream_synchronize(nullptr), "nn sync");
  for (int64_t i = 0; i < nq; i++) idx[i] = out[i];
  return idx;
}

int PlannerClass::getNearestNeighbor(State q) { return getNearestNeighborBatch({q})[0]; }

std::vector<int> PlannerClass::neighborhoodDist(State q, double dist) {  // :173-182 on the engine
  return neighborhoodDistBatch({q}, dist)[0];
}

std::vector<std::vector<int>> PlannerClass::neighborhoodDistBatch(const std::vector<State> &q,
                                                                  double dist,
                                                                  const std::vector<int> &limit) {
  std::vector<std::vector<int>> out(q.size());
  if (q.empty() || vertices_.empty()) return out;
  sync_device();
  const int64_t nq = (int64_t)q.size();
  int max_out = 256;
  for (int pass = 0; pass < 2; pass++) {
    const size_t bytes = (size_t)nq * (sizeof(State) + sizeof(int32_t) * (max_out + 1)) + 256;
    if (bytes > d_nbr_bytes_) {
      if (d_nbr_) gbp_device_free(d_nbr_);
      d_nbr_ = nullptr;
      d_nbr_bytes_ = 0;
      chk(gbp_device_alloc(device_, bytes, &d_nbr_), "neighbourhood scratch");
      d_nbr_bytes_ = bytes;
    }
    double *dq = (double *)d_nbr_;
    int32_t *dcnt = (int32_t *)(dq + 8 * nq);
    int32_t *dout = dcnt + nq;
    std::vector<int32_t> cnt(nq), lst((size_t)nq * max_out);
    chk(gbp_memcpy_h2d(dq, q[0].data(), (size_t)nq * sizeof(State), nullptr), "nbr upload");
    chk(gbp_neighbors_batch_dev(nq, dq, (int64_t)vertices_.size(), d_vertices_, dist, max_out, dout,
                                dcnt, nullptr),
        "neighborhoodDist");
    chk(gbp_memcpy_d2h(cnt.data(), dcnt, (size_t)nq * sizeof(int32_t), nullptr), "nbr count");
    chk(gbp_memcpy_d2h(lst.data(), dout, lst.size() * sizeof(int32_t), nullptr), "nbr list");
    chk(gbp_stream_synchronize(nullptr), "nbr sync");
    int need = 0;
    for (int64_t i = 0; i < nq; i++) need = std::max(need, (int)cnt[i]);
    if (need > max_out && pass == 0) {  // a list overflowed: once more with room for all
      max_out = need;
      continue;
    }
    for (int64_t i = 0; i < nq; i++) {
      const int lim = limit.empty() ? INT32_MAX : limit[i];
      for (int k = 0; k < std::min<int>(cnt[i], max_out); k++) {
        const int v = lst[(size_t)i * max_out + k];
        if (v < lim) out[i].push_back(v);
      }
      // the engine lists them in the order the map of all V vertices iterates;
      // RRT*'s vertex `lim` saw the map of keys 0..lim (rrt_star_connect.cpp:22-28)
      if (!limit.empty()) {
        const int64_t n_eff = (int64_t)lim + 1;
        std::stable_sort(out[i].begin(), out[i].end(), [n_eff](int a, int b) {
          return gbp::um_rank(a, n_eff) < gbp::um_rank(b, n_eff);
        });
      }
    }
    break;
  }
  return out;
}

std::vector<int> PlannerClass::neighborhoodN(State q, int N) {  // :151-171
  const int V = (int)vertices_.size();
  if (N >= 1 && N <= GBP_KNN_MAX && V > 0) {
    // the engine's k-nearest wavefront scan (gbp_knn_batch_dev): the heap's
    // pop order, ascending (stateDistance, index); with cost_add_yaw the
    // weighted distance (:157-158) on the vertices' glibc yaws
    sync_device();
    ensure_scratch(256);  // one query row (+ its yaw) + N indices
    double *dq = (double *)d_scratch_;
    int32_t *dout = (int32_t *)(dq + 9);
    std::vector<int32_t> out(N);
    double qrow[9];
    std::copy(q.begin(), q.end(), qrow);
    qrow[8] = gbp_host_yaw(q.data());
    chk(gbp_memcpy_h2d(dq, qrow, sizeof qrow, nullptr), "knn upload");
    if (cost_add_yaw_flag_) {
      sync_yaw();
      chk(gbp_knn_yaw_batch_dev(1, dq, dq + 8, V, d_vertices_, d_yaw_, cost_add_yaw_length_weight_,
                                cost_add_yaw_yaw_weight_, N, dout, nullptr, nullptr),
          "neighborhoodN");
    } else {
      chk(gbp_knn_batch_dev(1, dq, V, d_vertices_, N, dout, nullptr, nullptr), "neighborhoodN");
    }
    chk(gbp_memcpy_d2h(out.data(), dout, (size_t)N * sizeof(int32_t), nullptr), "knn download");
    chk(gbp_stream_synchronize(nullptr), "knn sync");
    return std::vector<int>(out.begin(), out.begin() + std::min(N, V));
  }
  // N > GBP_KNN_MAX (or an empty tree): on the host
  std::vector<std::pair<double, int>> d;
  for (int i = 0; i < (int)vertices_.size(); i++)
    d.push_back({stateDistance(q, vertices_[i], cost_add_yaw_flag_, cost_add_yaw_length_weight_,
                               cost_add_yaw_yaw_weight_),
                 i});
  std::sort(d.begin(), d.end());
  std::vector<int> out;
  for (int i = 0; i < std::min<int>(N, (int)d.size()); i++) out.push_back(d[i].second);
  return out;
}

// ============================================================================
// RRTClass
// ============================================================================
gbp_sampling RRTClass::samplingConfig() const {
  gbp_sampling c{};
  c.state_flag = state_direction_sampling_flag_ ? 1 : 0;
  c.state_speed_direction = state_direction_sampling_speed_direction_flag_ ? 1 : 0;
  c.state_p = state_direction_sampling_probability_threshold_;
  c.action_flag = action_direction_sampling_flag_ ? 1 : 0;
  c.action_p = action_direction_sampling_probability_threshold_;
  return c;
}

void RRTClass::applySampling(FastTerrainMap &terrain) const {
  const gbp_sampling c = samplingConfig();
  chk(gbp_terrain_set_sampling(terrain.handle(), &c), "direction sampling");
}

bool RRTClass::newConfig(State s, State s_near, State &s_new, Action &a_new, FastTerrainMap &terrain,
                         int direction) {  // rrt.cpp:20-70 on the engine (6 candidates, one launch)
  applySampling(terrain);  // getRandomAction(surf_norm, direction, flag, p, s, s_near): rrt.cpp:34, :49
  int32_t result, chosen;
  uint32_t counts;
  State sn = s_new;
  Action an = a_new;
  const uint8_t dir = (uint8_t)direction;
  chk(gbp_extend_batch_host(terrain.handle(), 1, s_near.data(), s.data(), &dir, direction,
                            state_action_pair_check_adaptive_step_size_flag_ ? 1 : 0, seed_,
                            extend_counter_++, &result, &chosen, sn.data(), an.data(), &counts,
                            nullptr),
      "newConfig");
  if (result == GBP_TRAPPED) return false;
  s_new = sn;
  a_new = an;
  return true;
}

int RRTClass::extend(PlannerClass &T, State s, FastTerrainMap &terrain, int direction) {
  const int s_near_index = T.getNearestNeighbor(s);  // rrt.cpp:78-102
  const State s_near = T.getVertex(s_near_index);
  State s_new{};
  Action a_new{};
  if (newConfig(s, s_near, s_new, a_new, terrain, direction)) {
    const int s_new_index = T.getNumVertices();
    T.addVertex(s_new_index, s_new);
    T.addEdge(s_near_index, s_new_index);
    T.addAction(s_new_index, a_new);
    T.updateGYValue(s_new_index, T.getGValue(s_near_index) + poseDistance(s_near, s_new),
                    T.getYValue(s_near_index) + stateYawDistance(s_near, s_new));
    return isWithinBounds(s_new, s) ? GBP_PLANNER_REACHED : GBP_PLANNER_ADVANCED;
  }
  return GBP_PLANNER_TRAPPED;
}

std::vector<int> RRTClass::pathFromStart(PlannerClass &T, int s) {  // rrt.cpp:107-118
  std::vector<int> path{s};
  while (s != 0) {
    s = T.getPredecessor(s);
    path.push_back(s);
  }
  std::reverse(path.begin(), path.end());
  return path;
}

std::vector<State> RRTClass::getStateSequence(PlannerClass &T, std::vector<int> path) {
  std::vector<State> out;
  for (int i : path) out.push_back(T.getVertex(i));
  return out;
}

std::vector<Action> RRTClass::getActionSequence(PlannerClass &T, std::vector<int> path) {
  std::vector<Action> out;
  for (size_t i = 1; i < path.size(); ++i) out.push_back(T.getAction(path[i]));
  return out;
}

void RRTClass::getStatistics(double &plan_time, int &success_var, int &vertices_generated,
                             double &time_to_first_solve, std::vector<double> &length_vector,
                             std::vector<double> &yaw_vector, std::vector<double> &cost_vector,
                             std::vector<double> &cost_vector_times, double &path_duration,
                             std::vector<std::vector<double>> &allStatePosition) {
  plan_time = elapsed_total.count();
  success_var = success_;
  vertices_generated = num_vertices;
  time_to_first_solve = elapsed_to_first.count();
  length_vector = length_vector_;
  yaw_vector = yaw_vector_;
  cost_vector = cost_vector_;
  cost_vector_times = cost_vector_times_;
  path_duration = path_duration_;
  allStatePosition = allStatePosition_;
}

void RRTClass::printPath(PlannerClass &T, std::vector<int> path) {
  std::printf("Printing path:");
  for (int idx : path) {
    const State s = T.getVertex(idx);
    std::printf("\n%d or {", idx);
    for (int d = 0; d < 8; d++) std::printf(d ? ", %g" : "%g", s[d]);
    std::printf("} ->");
  }
  std::printf("\b\b  \n");
}

void RRTClass::saveStateSequence(PlannerClass &T) {
  for (int i = 0; i < T.getNumVertices(); ++i) {
    const State s = T.getVertex(i);
    allStatePosition_.push_back({s[0], s[1], s[2]});
  }
}

void RRTClass::print_setting_parameters() {
  std::printf("state_action_pair_check_adaptive_step_size_flag: %d\n",
              (int)state_action_pair_check_adaptive_step_size_flag_);
  std::printf("cost_add_yaw: %d %g %g\n", (int)cost_add_yaw_flag_, cost_add_yaw_length_weight_,
              cost_add_yaw_yaw_weight_);
  std::printf("action_direction_sampling: %d %g\n", (int)action_direction_sampling_flag_,
              action_direction_sampling_probability_threshold_);
  std::printf("state_direction_sampling: %d %g %d\n", (int)state_direction_sampling_flag_,
              state_direction_sampling_probability_threshold_,
              (int)state_direction_sampling_speed_direction_flag_);
  std::printf("engine seed: %llu\n", (unsigned long long)seed_);
}

// ============================================================================
// RRTConnectClass
// ============================================================================
static void tree_extent(const PlannerClass &T, double e[4]) {
  e[0] = e[2] = INFINITY;
  e[1] = e[3] = -INFINITY;
  for (const State &v : T.vertices()) {
    e[0] = std::min(e[0], v[0]);
    e[1] = std::max(e[1], v[0]);
    e[2] = std::min(e[2], v[1]);
    e[3] = std::max(e[3], v[1]);
  }
}

static Action connect_action(const State &s_start, const State &s_goal, double t_s) {
  // rrt_connect.cpp:53-63 (cubic-Hermite stance action, t_f = 0)
  const double x_td = s_start[0], y_td = s_start[1], z_td = s_start[2];
  const double dx_td = s_start[3], dy_td = s_start[4], dz_td = s_start[5];
  const double x_to = s_goal[0], y_to = s_goal[1], z_to = s_goal[2];
  const double dx_to = s_goal[3], dy_to = s_goal[4], dz_to = s_goal[5];
  const double p_td = s_start[6], dp_td = s_start[7], p_to = s_goal[6], dp_to = s_goal[7];
  Action a;
  a[0] = -(2.0 * (3.0 * x_td - 3.0 * x_to + 2.0 * dx_td * t_s + dx_to * t_s)) / (t_s * t_s);
  a[1] = -(2.0 * (3.0 * y_td - 3.0 * y_to + 2.0 * dy_td * t_s + dy_to * t_s)) / (t_s * t_s);
  a[2] = -(2.0 * (3.0 * z_td - 3.0 * z_to + 2.0 * dz_td * t_s + dz_to * t_s)) / (t_s * t_s);
  a[3] = (2.0 * (3.0 * x_td - 3.0 * x_to + dx_td * t_s + 2.0 * dx_to * t_s)) / (t_s * t_s);
  a[4] = (2.0 * (3.0 * y_td - 3.0 * y_to + dy_td * t_s + 2.0 * dy_to * t_s)) / (t_s * t_s);
  a[5] = (2.0 * (3.0 * z_td - 3.0 * z_to + dz_td * t_s + 2.0 * dz_to * t_s)) / (t_s * t_s);
  a[6] = t_s;
  a[7] = 0;
  a[8] = -(2.0 * (3.0 * p_td - 3.0 * p_to + 2.0 * dp_td * t_s + dp_to * t_s)) / (t_s * t_s);
  a[9] = (2.0 * (3.0 * p_td - 3.0 * p_to + dp_td * t_s + 2.0 * dp_to * t_s)) / (t_s * t_s);
  return a;
}

int RRTConnectClass::attemptConnect(State s_existing, State s, double t_s, State &s_new,
                                    Action &a_new, FastTerrainMap &terrain, int direction) {
  std::vector<int> r;
  std::vector<State> sn{s_new};
  std::vector<Action> an{a_new};
  attemptConnectBatch({s_existing}, {s}, {t_s}, terrain, direction, r, sn, an, nullptr);
  if (r[0] != GBP_PLANNER_TRAPPED || sn[0] != s_new) {
    s_new = sn[0];
    a_new = an[0];
  }
  return r[0];
}

int RRTConnectClass::attemptConnect(State s_existing, State s, State &s_new, Action &a_new,
                                    FastTerrainMap &terrain, int direction) {
  const double t_s = poseDistance(s, s_existing) / V_NOM;  // rrt_connect.cpp:89
  return attemptConnect(s_existing, s, t_s, s_new, a_new, terrain, direction);
}

// The recursive attemptConnect (rrt_connect.cpp:20-84) for many independent
// connections, run as lock-step rounds: round d evaluates recursion depth d of
// every still-open connection in ONE engine launch.  Per connection:
//   REACHED  if its depth-0 pair check is valid,
//   ADVANCED if a deeper level's check is valid,
//   TRAPPED  if t_s <= KINEMATICS_RES, isValidAction fails, or (engine
//            convention) the failed check left t_new / s_new
//            unassigned — the reference would recurse on uninitialised values.
void RRTConnectClass::attemptConnectBatch(const std::vector<State> &s_existing,
                                          const std::vector<State> &s0, std::vector<double> t_s,
                                          FastTerrainMap &terrain, int direction,
                                          std::vector<int> &result, std::vector<State> &s_new,
                                          std::vector<Action> &a_new, BatchStats *stats,
                                          int max_depth) {
  const size_t n = s_existing.size();
  result.assign(n, GBP_PLANNER_TRAPPED);
  s_new.resize(n);
  a_new.resize(n);
  std::vector<State> s = s0;
  std::vector<int> open(n);
  std::iota(open.begin(), open.end(), 0);
  std::vector<uint8_t> resolved(stats ? n : 0, 0);  // a level was re-decided on the host
  for (int depth = 0; !open.empty() && depth <= max_depth; depth++) {
    std::vector<int> chk_idx;
    std::vector<State> cs;
    std::vector<Action> ca;
    for (int k : open) {
      if (t_s[k] <= KINEMATICS_RES) continue;  // TRAPPED (:23-24)
      const State &start = (direction == FORWARD) ? s_existing[k] : s[k];
      const State &goal = (direction == FORWARD) ? s[k] : s_existing[k];
      const Action a = connect_action(start, goal, t_s[k]);
      a_new[k] = a;
      if (!isValidAction(a)) continue;  // TRAPPED (:66, :83)
      chk_idx.push_back(k);
      cs.push_back(direction == FORWARD ? start : goal);
      ca.push_back(a);
    }
    open.clear();
    if (chk_idx.empty()) break;
    std::vector<uint8_t> valid;
    std::vector<State> sn(chk_idx.size());
    std::vector<double> tn(chk_idx.size(), 0.0);
    std::vector<uint32_t> fl(chk_idx.size());
    for (size_t j = 0; j < chk_idx.size(); j++) sn[j] = s_new[chk_idx[j]];
    const int64_t m = (int64_t)chk_idx.size();
    chk(gbp_validate_pairs_host(terrain.handle(), m, cs[0].data(), ca[0].data(), nullptr,
                                direction, state_action_pair_check_adaptive_step_size_flag_ ? 1 : 0,
                                nullptr, sn[0].data(), tn.data(), fl.data(), nullptr),
        "attemptConnect");
    if (stats) stats->attempts_checked += m;
    for (size_t j = 0; j < chk_idx.size(); j++) {
      const int k = chk_idx[j];
      if (stats && (fl[j] & GBP_F_RESOLVED)) resolved[k] = 1;
      if (fl[j] & GBP_F_SNEW_SET) s_new[k] = sn[j];
      if (fl[j] & GBP_F_VALID) {
        result[k] = depth == 0 ? GBP_PLANNER_REACHED : GBP_PLANNER_ADVANCED;
      } else if ((fl[j] & GBP_F_TNEW_SET) && (fl[j] & GBP_F_SNEW_SET)) {
        s[k] = sn[j];  // :77 recurse toward the returned state with t_s = t_new
        t_s[k] = tn[j];
        open.push_back(k);
      }
    }
  }
  // still open after level max_depth: TRAPPED by the engine's cap (gbp.h
  // GBP_CONNECT_MAX_DEPTH; with max_depth 0 only REACHED is asked for)
  if (stats && max_depth > 0) stats->depth_capped += (int64_t)open.size();
  if (stats)
    for (uint8_t r : resolved) stats->fragile_resolved += r;
}

int RRTConnectClass::connect(PlannerClass &T, State s, FastTerrainMap &terrain, int direction) {
  const int s_near_index = T.getNearestNeighbor(s);  // rrt_connect.cpp:98-120
  const State s_near = T.getVertex(s_near_index);
  State s_new{};
  Action a_new{};
  const int result = attemptConnect(s_near, s, s_new, a_new, terrain, direction);
  if (result != GBP_PLANNER_TRAPPED) {
    const int s_new_index = T.getNumVertices();
    T.addVertex(s_new_index, s_new);
    T.addEdge(s_near_index, s_new_index);
    T.addAction(s_new_index, a_new);
    T.updateGYValue(s_new_index, T.getGValue(s_near_index) + poseDistance(s_near, s_new),
                    T.getYValue(s_near_index) + stateYawDistance(s_near, s_new));
  }
  return result;
}

std::vector<Action> RRTConnectClass::getActionSequenceReverse(PlannerClass &T,
                                                              std::vector<int> path) {
  std::vector<Action> out;
  for (size_t i = 0; i + 1 < path.size(); ++i) out.push_back(T.getAction(path[i]));
  return out;
}

void RRTConnectClass::postProcessPath(std::vector<State> &state_sequence,
                                      std::vector<Action> &action_sequence,
                                      FastTerrainMap &terrain) {  // rrt_connect.cpp:139-227
  State s = state_sequence.front();
  const State s_goal = state_sequence.back();
  State dummy{};
  Action a_new{};
  std::vector<State> new_states{s};
  std::vector<Action> new_actions;
  path_length_ = 0;
  path_yaw_ = 0;
  path_cost_ = 0;
  while (s != s_goal) {
    std::vector<State> sc = state_sequence;
    std::vector<Action> ac = action_sequence;
    State s_next = sc.back();
    Action a_next = ac.back();
    State old_state{};
    Action old_action{};
    while ((attemptConnect(s, s_next, dummy, a_new, terrain, FORWARD) != GBP_PLANNER_REACHED) &&
           (s != s_next)) {
      old_state = s_next;
      old_action = a_next;
      sc.pop_back();
      ac.pop_back();
      s_next = sc.back();
      // the reference reads back() of the now-empty action copy when it pops
      // down to s itself (UB, never used afterwards): keep the last value
      if (!ac.empty()) a_next = ac.back();
    }
    if (s != s_next) {
      new_states.push_back(s_next);
      new_actions.push_back(a_new);
      const double dl = poseDistance(s, s_next), dy = stateYawDistance(s, s_next);
      path_length_ += dl;
      path_yaw_ += dy;
      path_cost_ += weightedCost(dl, dy);
      s = s_next;
    } else {
      // the reference adds to path_cost_ but not path_length_ here (:210-215)
      new_states.push_back(old_state);
      new_actions.push_back(old_action);
      const double dl = poseDistance(s, old_state), dy = stateYawDistance(s, old_state);
      path_cost_ += weightedCost(dl, dy);
      s = old_state;
    }
  }
  state_sequence = new_states;
  action_sequence = new_actions;
}

void RRTConnectClass::runRRTConnect(PlannerClass &Ta, PlannerClass &Tb,
                                    FastTerrainMap &terrain) {  // rrt_connect.cpp:230-314
  const auto t_start = std::chrono::high_resolution_clock::now();
  while (true) {
    std::chrono::duration<double> el = std::chrono::high_resolution_clock::now() - t_start;
    if (el.count() >= anytime_horizon) {
      anytime_horizon = anytime_horizon * horizon_expansion_factor;
      return;
    }
    // direction-biased draws between the trees (rrt_connect.cpp:248-252)
    State s_from = Ta.getVertex(Ta.getNumVertices() - 1), s_to = Tb.getVertex(0);
    State s_rand = Ta.randomState(terrain, state_direction_sampling_flag_,
                                  state_direction_sampling_probability_threshold_,
                                  state_direction_sampling_speed_direction_flag_, s_from, s_to);
    if (isValidState(s_rand, terrain, STANCE)) {
      if (extend(Ta, s_rand, terrain, FORWARD) != GBP_PLANNER_TRAPPED) {
        const State s_new = Ta.getVertex(Ta.getNumVertices() - 1);
        if (connect(Tb, s_new, terrain, REVERSE) == GBP_PLANNER_REACHED) {
          goal_found = true;
          elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
          break;
        }
      }
    }
    s_from = Ta.getVertex(0);  // :283-287
    s_to = Tb.getVertex(Tb.getNumVertices() - 1);
    s_rand = Tb.randomState(terrain, state_direction_sampling_flag_,
                            state_direction_sampling_probability_threshold_,
                            state_direction_sampling_speed_direction_flag_, s_from, s_to);
    if (isValidState(s_rand, terrain, STANCE)) {
      if (extend(Tb, s_rand, terrain, REVERSE) != GBP_PLANNER_TRAPPED) {
        const State s_new = Tb.getVertex(Tb.getNumVertices() - 1);
        if (connect(Ta, s_new, terrain, FORWARD) == GBP_PLANNER_REACHED) {
          goal_found = true;
          elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
          break;
        }
      }
    }
  }
  path_length_ = Ta.getGValue(Ta.getNumVertices() - 1) + Tb.getGValue(Tb.getNumVertices() - 1);
  path_yaw_ = Ta.getYValue(Ta.getNumVertices() - 1) + Tb.getYValue(Tb.getNumVertices() - 1);
  path_cost_ = weightedCost(path_length_, path_yaw_);
}

void RRTConnectClass::buildRRTConnect(FastTerrainMap &terrain, State s_start, State s_goal,
                                      std::vector<State> &state_sequence,
                                      std::vector<Action> &action_sequence,
                                      double max_time_opt) {  // rrt_connect.cpp:323-467
  if (engine_batch_ > 0) {
    // the same restart loop (anytime horizons, post-processed solutions, the
    // cheapest kept, stop once one exists and max_time_opt has passed), each
    // restart's runRRTConnect run as the device-resident batched search
    const auto t0 = std::chrono::high_resolution_clock::now();
    success_ = 0;
    BatchStats st;
    const bool found = buildRRTConnectBatchedAnytime(terrain, s_start, s_goal, engine_batch_,
                                                     max_time_solve, max_time_opt, state_sequence,
                                                     action_sequence, &st, true);
    elapsed_total = std::chrono::high_resolution_clock::now() - t0;
    elapsed_to_first = std::chrono::duration<double>(wall_to_first_ >= 0 ? wall_to_first_ : 0.0);
    num_vertices = (int)(st.vertices_a + st.vertices_b);
    if (found && elapsed_total.count() <= 5.0) success_ = 1;  // :462-464
    return;
  }
  const auto t_start = std::chrono::high_resolution_clock::now();
  success_ = 0;
  length_vector_.clear();
  yaw_vector_.clear();
  cost_vector_.clear();
  cost_vector_times_.clear();
  wall_to_first_ = -1;
  goal_found = false;
  PlannerClass Ta(terrain.device()), Tb(terrain.device()), Ta_best(terrain.device()),
      Tb_best(terrain.device());
  anytime_horizon = poseDistance(s_start, s_goal) / planning_rate_estimate;
  num_vertices = 0;
  double length_so_far = INFTY, yaw_so_far = INFTY, cost_so_far = INFTY;
  int restart = 0;
  std::chrono::duration<double> el{0};
  while (true) {
    Ta = PlannerClass(terrain.device());
    Tb = PlannerClass(terrain.device());
    Ta.setStream(seed_, 1000 + 2 * restart);
    Tb.setStream(seed_, 1001 + 2 * restart);
    restart++;
    Ta.init(s_start, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
    Tb.init(s_goal, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
    goal_found = false;
    runRRTConnect(Ta, Tb, terrain);
    num_vertices += Ta.getNumVertices() + Tb.getNumVertices();
    el = std::chrono::high_resolution_clock::now() - t_start;
    if (el.count() >= max_time_solve) {
      elapsed_total = el;
      elapsed_to_first = el;
      success_ = 0;
      num_vertices += Ta.getNumVertices() + Tb.getNumVertices();  // counted twice, as :366
      return;
    }
    if (goal_found) {
      if (wall_to_first_ < 0) wall_to_first_ = el.count();
      std::vector<int> path_a = pathFromStart(Ta, Ta.getNumVertices() - 1);
      std::vector<int> path_b = pathFromStart(Tb, Tb.getNumVertices() - 1);
      std::reverse(path_b.begin(), path_b.end());
      std::vector<Action> action_sequence_b = getActionSequenceReverse(Tb, path_b);
      path_b.erase(path_b.begin());
      state_sequence = getStateSequence(Ta, path_a);
      std::vector<State> sb = getStateSequence(Tb, path_b);
      state_sequence.insert(state_sequence.end(), sb.begin(), sb.end());
      action_sequence = getActionSequence(Ta, path_a);
      action_sequence.insert(action_sequence.end(), action_sequence_b.begin(),
                             action_sequence_b.end());
      postProcessPath(state_sequence, action_sequence, terrain);
      if (path_cost_ < cost_so_far) {
        length_so_far = path_length_;
        yaw_so_far = path_yaw_;
        cost_so_far = path_cost_;
        Ta_best = Ta;
        Tb_best = Tb;
        el = std::chrono::high_resolution_clock::now() - t_start;
        length_vector_.push_back(length_so_far);
        yaw_vector_.push_back(yaw_so_far);
        cost_vector_.push_back(cost_so_far);
        cost_vector_times_.push_back(el.count());
      }
    }
    if (goal_found && el.count() >= max_time_opt) break;
  }
  Ta = Ta_best;
  Tb = Tb_best;
  if (goal_found) {
    std::vector<int> path_a = pathFromStart(Ta, Ta.getNumVertices() - 1);
    std::vector<int> path_b = pathFromStart(Tb, Tb.getNumVertices() - 1);
    std::reverse(path_b.begin(), path_b.end());
    std::vector<Action> action_sequence_b = getActionSequenceReverse(Tb, path_b);
    path_b.erase(path_b.begin());
    state_sequence = getStateSequence(Ta, path_a);
    std::vector<State> sb = getStateSequence(Tb, path_b);
    state_sequence.insert(state_sequence.end(), sb.begin(), sb.end());
    action_sequence = getActionSequence(Ta, path_a);
    action_sequence.insert(action_sequence.end(), action_sequence_b.begin(),
                           action_sequence_b.end());
  }
  postProcessPath(state_sequence, action_sequence, terrain);
  elapsed_total = std::chrono::high_resolution_clock::now() - t_start;
  if (elapsed_total.count() <= 5.0) success_ = 1;
  path_duration_ = 0.0;
  for (const Action &a : action_sequence) path_duration_ += (a[6] + a[7]);
}

// one batch-synchronous half-iteration: extend T toward `batch` targets, then
// connect every new vertex to O (direction of the connect = opposite of dir)
void RRTConnectClass::extendBatch(PlannerClass &T, FastTerrainMap &terrain, int dir, int batch,
                                  std::vector<int> &added, std::vector<int> &nearest,
                                  std::vector<Action> &a_out, bool insert, BatchStats *stats,
                                  const PlannerClass *O) {
  added.clear();
  nearest.clear();
  a_out.clear();
  applySampling(terrain);  // newConfig's candidates (rrt.cpp:34, :49)
  // targets: randomState + isValidState(STANCE) (rrt_connect.cpp:249-254); with
  // O, the direction-biased draw between T's last vertex and O's root
  // (FORWARD: T = Ta, :248) or O's root and T's last vertex (REVERSE, :283)
  std::vector<State> cand;
  if (O) {
    const State last = T.getVertex(T.getNumVertices() - 1), root = O->getVertex(0);
    cand = T.randomStateBatch(terrain, batch, samplingConfig(), dir == FORWARD ? last : root,
                              dir == FORWARD ? root : last);
  } else {
    cand = T.randomStateBatch(terrain, batch);
  }
  std::vector<uint8_t> ok(batch);
  std::vector<uint32_t> tflags(batch);
  chk(gbp_valid_states_host(terrain.handle(), batch, cand[0].data(), nullptr, STANCE, ok.data(),
                            tflags.data(), nullptr),
      "target validity");
  if (stats)
    for (uint32_t f : tflags) stats->fragile_resolved += (f & GBP_F_RESOLVED) ? 1 : 0;
  std::vector<State> targets;
  for (int i = 0; i < batch; i++)
    if (ok[i]) targets.push_back(cand[i]);
  if (stats) stats->targets += (int64_t)targets.size();
  if (targets.empty()) return;
  const int64_t n = (int64_t)targets.size();
  // extend (rrt.cpp:77-102), all targets against the current tree snapshot
  std::vector<int> nn = T.getNearestNeighborBatch(targets);
  std::vector<State> s_near(n), s_new(n);
  std::vector<Action> a_new(n);
  for (int64_t i = 0; i < n; i++) s_near[i] = T.getVertex(nn[i]);
  std::vector<int32_t> res(n), chosen(n);
  std::vector<uint32_t> eflags(n);
  chk(gbp_extend_batch_host(terrain.handle(), n, s_near[0].data(), targets[0].data(), nullptr, dir,
                            state_action_pair_check_adaptive_step_size_flag_ ? 1 : 0, seed_,
                            extend_counter_, res.data(), chosen.data(), s_new[0].data(),
                            a_new[0].data(), nullptr, eflags.data()),
      "extend batch");
  if (stats)
    for (int64_t i = 0; i < n; i++) stats->fragile_resolved += (eflags[i] & GBP_F_RESOLVED) ? 1 : 0;
  extend_counter_ += n;
  if (stats) {
    stats->extends += n;
    // newConfig stops at the first valid candidate (rrt.cpp:36-50)
    for (int64_t i = 0; i < n; i++) stats->attempts_checked += chosen[i] >= 0 ? chosen[i] + 1 : 6;
  }
  for (int64_t i = 0; i < n; i++) {
    if (res[i] == GBP_TRAPPED) continue;
    const int idx = T.getNumVertices();
    T.addVertex(idx, s_new[i]);
    if (insert) {  // rrt.cpp:86-92
      T.addEdge(nn[i], idx);
      T.addAction(idx, a_new[i]);
      T.updateGYValue(idx, T.getGValue(nn[i]) + poseDistance(s_near[i], s_new[i]),
                      T.getYValue(nn[i]) + stateYawDistance(s_near[i], s_new[i]));
    }
    added.push_back(idx);
    nearest.push_back(nn[i]);
    a_out.push_back(a_new[i]);
  }
}

std::vector<std::pair<int, int>> RRTConnectClass::connectBatch(PlannerClass &T, PlannerClass &O,
                                                               FastTerrainMap &terrain, int dir,
                                                               const std::vector<int> &added,
                                                               BatchStats *stats) {
  std::vector<std::pair<int, int>> reached;
  if (added.empty()) return reached;
  // connect every new vertex to the other tree (rrt_connect.cpp:98-120)
  std::vector<State> q;
  for (int idx : added) q.push_back(T.getVertex(idx));
  std::vector<int> nno = O.getNearestNeighborBatch(q);
  std::vector<State> s_ex(q.size());
  std::vector<double> t_s(q.size());
  for (size_t k = 0; k < q.size(); k++) {
    s_ex[k] = O.getVertex(nno[k]);
    t_s[k] = poseDistance(q[k], s_ex[k]) / V_NOM;
  }
  const int cdir = (dir == FORWARD) ? REVERSE : FORWARD;
  std::vector<int> cres;
  std::vector<State> csn(q.size(), State{});
  std::vector<Action> can(q.size(), Action{});
  attemptConnectBatch(s_ex, q, t_s, terrain, cdir, cres, csn, can, stats);
  if (stats) stats->connects += (int64_t)q.size();
  for (size_t k = 0; k < q.size(); k++) {
    if (cres[k] == GBP_PLANNER_TRAPPED) continue;
    const int idx = O.getNumVertices();
    O.addVertex(idx, csn[k]);
    O.addEdge(nno[k], idx);
    O.addAction(idx, can[k]);
    O.updateGYValue(idx, O.getGValue(nno[k]) + poseDistance(s_ex[k], csn[k]),
                    O.getYValue(nno[k]) + stateYawDistance(s_ex[k], csn[k]));
    if (cres[k] == GBP_PLANNER_REACHED) reached.push_back({added[k], idx});
  }
  return reached;
}

int RRTConnectClass::halfIterationBatched(PlannerClass &T, PlannerClass &O, FastTerrainMap &terrain,
                                          int dir, int batch, int &meet_t, int &meet_o,
                                          BatchStats *stats) {
  std::vector<int> added, nearest;
  std::vector<Action> a_new;
  extendBatch(T, terrain, dir, batch, added, nearest, a_new, true, stats, &O);
  const std::vector<std::pair<int, int>> reached = connectBatch(T, O, terrain, dir, added, stats);
  if (reached.empty()) return 0;
  meet_t = reached.front().first;
  meet_o = reached.front().second;
  return 1;
}

static void dump_trees(const PlannerClass &Ta, const PlannerClass &Tb, TreeDump *d) {
  if (!d) return;
  const PlannerClass *t[2] = {&Ta, &Tb};
  for (int k = 0; k < 2; k++) {
    const int n = t[k]->getNumVertices();
    d->v[k] = t[k]->vertices();
    d->a[k].resize(n);
    d->parent[k].resize(n);
    d->g[k].resize(n);
    for (int i = 0; i < n; i++) {
      d->a[k][i] = t[k]->getAction(i);
      d->parent[k][i] = t[k]->getPredecessor(i);
      d->g[k][i] = t[k]->getGValue(i);
    }
  }
}

bool RRTConnectClass::buildRRTConnectBatched(FastTerrainMap &terrain, State s_start, State s_goal,
                                             int batch, double max_time,
                                             std::vector<State> &state_sequence,
                                             std::vector<Action> &action_sequence,
                                             BatchStats *stats) {
  const auto t_start = std::chrono::high_resolution_clock::now();
  goal_found = false;
  wall_to_first_ = -1;
  PlannerClass Ta(terrain.device()), Tb(terrain.device());
  Ta.setStream(seed_, 101);
  Tb.setStream(seed_, 102);
  Ta.init(s_start, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  Tb.init(s_goal, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  BatchStats local;
  BatchStats &st = stats ? *stats : local;
  int ia = -1, ib = -1;
  auto more = [&]() { return st.max_halves <= 0 || st.halves < st.max_halves; };
  while (more()) {
    std::chrono::duration<double> el = std::chrono::high_resolution_clock::now() - t_start;
    if (el.count() >= max_time) break;
    st.iterations++;
    st.halves++;
    if (halfIterationBatched(Ta, Tb, terrain, FORWARD, batch, ia, ib, &st)) {
      goal_found = true;
      break;
    }
    if (!more()) break;
    st.halves++;
    if (halfIterationBatched(Tb, Ta, terrain, REVERSE, batch, ib, ia, &st)) {
      goal_found = true;
      break;
    }
  }
  elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
  tree_extent(Ta, st.extent_a);
  tree_extent(Tb, st.extent_b);
  st.vertices_a = Ta.getNumVertices();
  st.vertices_b = Tb.getNumVertices();
  num_vertices = Ta.getNumVertices() + Tb.getNumVertices();
  dump_trees(Ta, Tb, st.dump);
  st.meet_a = ia;
  st.meet_b = ib;
  if (!goal_found) return false;
  wall_to_first_ = elapsed_to_first.count();
  // rrt_connect.cpp:386-401 with the meeting vertices (ia in Ta, ib in Tb)
  std::vector<int> path_a = pathFromStart(Ta, ia);
  std::vector<int> path_b = pathFromStart(Tb, ib);
  std::reverse(path_b.begin(), path_b.end());
  std::vector<Action> action_sequence_b = getActionSequenceReverse(Tb, path_b);
  path_b.erase(path_b.begin());
  state_sequence = getStateSequence(Ta, path_a);
  std::vector<State> sb = getStateSequence(Tb, path_b);
  state_sequence.insert(state_sequence.end(), sb.begin(), sb.end());
  action_sequence = getActionSequence(Ta, path_a);
  action_sequence.insert(action_sequence.end(), action_sequence_b.begin(), action_sequence_b.end());
  path_length_ = Ta.getGValue(ia) + Tb.getGValue(ib);
  path_yaw_ = Ta.getYValue(ia) + Tb.getYValue(ib);
  path_cost_ = weightedCost(path_length_, path_yaw_);  // rrt_connect.cpp:304-313
  path_duration_ = 0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
  return true;
}


// ---- the search resident on the device (include/gbp.h device planner loop) ----
namespace {

struct DeviceTrees {
  gbp_stream stream = nullptr;
  gbp_plan_ws *ws = nullptr;
  gbp_tree *tree[2] = {nullptr, nullptr};
  ~DeviceTrees() {
    if (stream) gbp_stream_synchronize(stream);
    for (gbp_tree *t : tree)
      if (t) gbp_tree_destroy(t);
    if (ws) gbp_plan_ws_destroy(ws);
    if (stream) gbp_stream_destroy(stream);
  }
};

struct HostTree {  // a device tree read back once the search ends
  std::vector<State> v;
  std::vector<Action> a;
  std::vector<int32_t> parent;
  std::vector<double> g;
};

void read_tree(gbp_tree *t, gbp_stream s, HostTree &h) {
  int64_t n = 0;
  chk(gbp_tree_size(t, &n, s), "tree size");
  h.v.resize(n);
  h.a.resize(n);
  h.parent.resize(n);
  h.g.resize(n);
  chk(gbp_tree_read(t, 0, n, h.v[0].data(), h.a[0].data(), h.parent.data(), h.g.data(), s),
      "tree read");
}

std::vector<int> host_path(const HostTree &t, int idx) {  // rrt.cpp:107-118
  std::vector<int> path{idx};
  while (idx != 0) {
    idx = t.parent[idx];
    path.push_back(idx);
  }
  std::reverse(path.begin(), path.end());
  return path;
}

double path_yaw(const HostTree &t, const std::vector<int> &path) {
  // y of the last vertex: updateGYValue's sums along the parent chain (rrt.cpp:91-92)
  double y = 0;
  for (size_t i = 1; i < path.size(); i++)
    y = y + stateYawDistance(t.v[path[i - 1]], t.v[path[i]]);
  return y;
}

void extent(const HostTree &t, double e[4]) {
  e[0] = e[2] = INFINITY;
  e[1] = e[3] = -INFINITY;
  for (const State &v : t.v) {
    e[0] = std::min(e[0], v[0]);
    e[1] = std::max(e[1], v[0]);
    e[2] = std::min(e[2], v[1]);
    e[3] = std::max(e[3], v[1]);
  }
}

}  // namespace

bool RRTConnectClass::buildRRTConnectDevice(FastTerrainMap &terrain, State s_start, State s_goal,
                                            int batch, double max_time,
                                            std::vector<State> &state_sequence,
                                            std::vector<Action> &action_sequence,
                                            BatchStats *stats, uint64_t stream_a,
                                            uint64_t stream_b) {
  const auto t_start = std::chrono::high_resolution_clock::now();
  auto since = [&]() {
    return std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t_start).count();
  };
  goal_found = false;
  wall_to_first_ = -1;
  BatchStats local;
  BatchStats &st = stats ? *stats : local;
  gbp_terrain *h = terrain.handle();
  const int dev = terrain.device();
  const int adaptive = state_action_pair_check_adaptive_step_size_flag_ ? 1 : 0;
  // the target streams (buildRRTConnectBatched's: Ta 101, Tb 102), B draws per half
  const uint64_t tstream[2] = {stream_a, stream_b};
  applySampling(terrain);  // the device loop's targets and candidates read it from the handle
  DeviceTrees D;
  chk(gbp_stream_create(dev, &D.stream), "stream");
  chk(gbp_plan_ws_create(h, batch, &D.ws), "plan workspace");
  if (st.stage_timing) chk(gbp_plan_stage_timing(D.ws, 1), "stage timing");
  int64_t cap = std::max<int64_t>(1 << 16, 4 * (int64_t)batch);
  int64_t known[2] = {1, 1};
  for (int k = 0; k < 2; k++) {
    const int64_t wn = st.warm_n[k];
    if (wn > 0 && (!st.warm_v[k] || !st.warm_a[k] || !st.warm_parent[k] || st.warm_parent[k][0] != -1))
      throw EngineError(GBP_E_INVALID_ARG, "warm start: tree arrays");
    // an RRT-Connect tree: every vertex's parent was added before it (the
    // oracle's warm start refuses anything else, orc_plan)
    for (int64_t i = 1; i < wn; i++)
      if (st.warm_parent[k][i] < 0 || st.warm_parent[k][i] >= i)
        throw EngineError(GBP_E_INVALID_ARG, "warm start: a parent after its child");
    chk(gbp_tree_create(dev, std::max<int64_t>(cap, 2 * wn), &D.tree[k]), "tree");
    const double *root = wn > 0 ? st.warm_v[k] : (k == 0 ? s_start.data() : s_goal.data());
    chk(gbp_tree_init(D.tree[k], root, D.stream), "tree init");
    if (wn > 1)
      chk(gbp_tree_append_host(D.tree[k], wn - 1, st.warm_v[k] + 8, st.warm_a[k] + 10,
                               st.warm_parent[k] + 1, D.stream),
          "warm start: tree append");
    known[k] = std::max<int64_t>(1, wn);
  }
  if (st.warm_half < 0 || st.warm_extend < 0) throw EngineError(GBP_E_INVALID_ARG, "warm start");
  const int32_t half0 = (int32_t)st.warm_half;
  if (st.warm_n[0] > 0 || st.warm_n[1] > 0 || half0 > 0) extend_counter_ = st.warm_extend;
  chk(gbp_plan_reset(D.ws, extend_counter_, D.stream), "plan reset");
  // half h extends tree h % 2 toward its draws [(h / 2) B, (h / 2 + 1) B)
  // groups grow geometrically: a short search is not charged a long group's
  // tail of gated half-iterations, a long one amortises the status read
  const int g_max = (int)std::max<int64_t>(2, std::min<int64_t>(64, (1 << 21) / batch)) & ~1;
  int group = 2;
  int32_t half = half0;
  gbp_plan_status ps{};
  // with a stop poll (config 4's restart trees, one per rank) the ranks stop
  // together: every group ends in one poll, and only its answer ends the loop
  bool go = max_time > 0;
  double t_first = -1;  // when this rank first saw its connection (before any poll wait)
  while (go) {
    bool local_stop = false;
    try {
      if (st.max_halves > 0) group = (int)std::min<int64_t>(group, st.max_halves - (half - half0));
      for (int k = 0; k < 2; k++) {  // room for `group` halves of appends
        int64_t c = 0;
        chk(gbp_tree_capacity(D.tree[k], &c), "tree capacity");
        if (known[k] + (int64_t)group * batch > c)
          chk(gbp_tree_reserve(D.tree[k], std::max<int64_t>(2 * c, known[k] + (int64_t)group * batch),
                               D.stream),
              "tree reserve");
      }
      // the group's halves, one stream-ordered kernel sequence
      chk(gbp_plan_halves_dev(h, D.ws, D.tree[0], D.tree[1], half, group, batch, seed_, tstream[0],
                              tstream[1], adaptive, 0, D.stream),
          "plan halves");
      chk(gbp_plan_status_read(D.ws, &ps, D.stream), "plan status");
      st.status_reads++;
      while (ps.halt) {  // FRAGILE: re-decide on the host, resume where the sequence stopped
        for (int b = 0; b < 4; b++) st.halts[b] += (ps.halt >> b) & 1u;
        const int32_t h0 = ps.halt_half;
        const int k = h0 & 1;
        int resume = -1;
        int64_t nres = 0;
        chk(gbp_plan_resolve_host(h, D.ws, D.tree[k], D.tree[k ^ 1], k == 0 ? FORWARD : REVERSE,
                                  batch, adaptive, &resume, &nres, D.stream),
            "plan resolve");
        if (resume < 0) throw EngineError(GBP_E_INVALID_ARG, "plan resolve: nothing halted");
        chk(gbp_plan_halves_dev(h, D.ws, D.tree[0], D.tree[1], h0, half + group - h0, batch, seed_,
                                tstream[0], tstream[1], adaptive, resume, D.stream),
            "plan halves");
        chk(gbp_plan_status_read(D.ws, &ps, D.stream), "plan status");
        st.status_reads++;
      }
      if (ps.error & 1u) throw EngineError(GBP_E_HIP, "device planner loop: look-back spin exhausted");
      if (ps.error) throw EngineError(GBP_E_SHAPE, "device planner loop: a tree ran out of capacity");
      for (int k = 0; k < 2; k++) chk(gbp_tree_size(D.tree[k], &known[k], D.stream), "tree size");
      half += group;
      if (ps.done) goal_found = true;
      if (ps.done && t_first < 0) t_first = since();
      local_stop = ps.done || since() >= max_time ||
                   (st.max_halves > 0 && half - half0 >= st.max_halves);
    } catch (...) {
      // the peers are (or will be) blocked in this group's poll: post a stop
      // so that their collective completes, then fail here
      if (st.stop_poll) st.stop_poll(st.stop_ctx, 1, 0);
      throw;
    }
    if (st.stop_poll) {
      st.polls++;
      // nonzero = stop (a failed poll answers stop too: planner.py); a local
      // stop always ends this rank's loop, whatever the poll answered
      const int answer = st.stop_poll(st.stop_ctx, local_stop ? 1 : 0, ps.done ? 1 : 0);
      go = !local_stop && answer == 0;
      if (!go && !local_stop) st.stopped_by_peer = 1;
    } else {
      go = !local_stop;
    }
    group = std::min(group * 2, g_max);
  }
  elapsed_to_first = t_first >= 0 ? std::chrono::duration<double>(t_first)
                                  : std::chrono::duration<double>(since());
  extend_counter_ = ps.ext_counter;
  if (st.stage_timing) {
    double us[7];
    int64_t nh = 0;
    chk(gbp_plan_stage_times(D.ws, us, 7, &nh, 1), "stage times");
    for (int k = 0; k < 7; k++) st.stage_us[k] += us[k];
    st.stage_halves += nh;
  }
  const int32_t halves_run = (goal_found ? ps.meet_half + 1 : half) - half0;
  st.halves += halves_run;
  st.iterations += (halves_run + 1) / 2;
  st.targets += ps.stat_targets;
  st.extends += ps.stat_targets;
  st.attempts_checked += ps.stat_attempts;
  st.connects += ps.stat_added;
  st.fragile_resolved += ps.stat_fragile_resolved;
  st.depth_capped += ps.stat_depth_capped;
  st.nn_rechecks += ps.stat_nn_rechecks;
  st.nn_scans += ps.stat_nn_scans;
  HostTree A, B;
  read_tree(D.tree[0], D.stream, A);
  read_tree(D.tree[1], D.stream, B);
  extent(A, st.extent_a);
  extent(B, st.extent_b);
  st.vertices_a = (int64_t)A.v.size();
  st.vertices_b = (int64_t)B.v.size();
  num_vertices = (int)(A.v.size() + B.v.size());
  if (st.dump) {
    const HostTree *t[2] = {&A, &B};
    for (int k = 0; k < 2; k++) {
      st.dump->v[k] = t[k]->v;
      st.dump->a[k] = t[k]->a;
      st.dump->parent[k] = t[k]->parent;
      st.dump->g[k] = t[k]->g;
    }
  }
  if (!goal_found) return false;
  st.solutions++;
  wall_to_first_ = elapsed_to_first.count();
  // the meeting point: connection k of half meet_half joined T's vertex
  // added_base + k to O's vertex o (halves after it never ran)
  const int32_t kconn = (int32_t)(ps.meet >> 32), o = (int32_t)(ps.meet & 0xFFFFFFFFu);
  const int32_t tvtx = ps.added_base + kconn;
  const bool t_is_a = (ps.meet_half & 1) == 0;
  const int ia = t_is_a ? tvtx : o, ib = t_is_a ? o : tvtx;
  st.meet_a = ia;
  st.meet_b = ib;
  // rrt_connect.cpp:386-401 with the meeting vertices (as buildRRTConnectBatched)
  std::vector<int> path_a = host_path(A, ia);
  std::vector<int> path_b = host_path(B, ib);
  std::reverse(path_b.begin(), path_b.end());
  std::vector<Action> action_sequence_b;
  for (size_t i = 0; i + 1 < path_b.size(); ++i) action_sequence_b.push_back(B.a[path_b[i]]);
  const double yaw_b = path_yaw(B, host_path(B, ib));
  path_b.erase(path_b.begin());
  state_sequence.clear();
  for (int i : path_a) state_sequence.push_back(A.v[i]);
  for (int i : path_b) state_sequence.push_back(B.v[i]);
  action_sequence.clear();
  for (size_t i = 1; i < path_a.size(); ++i) action_sequence.push_back(A.a[path_a[i]]);
  action_sequence.insert(action_sequence.end(), action_sequence_b.begin(), action_sequence_b.end());
  path_length_ = A.g[ia] + B.g[ib];
  path_yaw_ = path_yaw(A, path_a) + yaw_b;
  path_cost_ = weightedCost(path_length_, path_yaw_);
  path_duration_ = 0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
  return true;
}

bool RRTConnectClass::buildRRTConnectBatchedAnytime(FastTerrainMap &terrain, State s_start,
                                                    State s_goal, int batch, double max_time,
                                                    double max_time_opt,
                                                    std::vector<State> &state_sequence,
                                                    std::vector<Action> &action_sequence,
                                                    BatchStats *stats, bool device_loop) {
  const auto t_start = std::chrono::high_resolution_clock::now();
  auto since = [](std::chrono::high_resolution_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
  };
  BatchStats local;
  BatchStats &st = stats ? *stats : local;
  wall_to_first_ = -1;
  goal_found = false;
  cost_vector_.clear();
  cost_vector_times_.clear();
  length_vector_.clear();
  yaw_vector_.clear();
  anytime_horizon = poseDistance(s_start, s_goal) / planning_rate_estimate;  // :345
  num_vertices = 0;
  double cost_so_far = INFTY;
  std::vector<State> best_states;
  std::vector<Action> best_actions;
  double best_length = 0, best_yaw = 0;
  for (int restart = 0;; restart++) {  // :350-420, one pair of fresh trees per restart
    if (device_loop) {  // the restart's runRRTConnect as the device-resident search
      const double budget = std::min(anytime_horizon, std::max(0.0, max_time - since(t_start)));
      std::vector<State> states;
      std::vector<Action> actions;
      const double w0 = wall_to_first_;
      const bool found = buildRRTConnectDevice(terrain, s_start, s_goal, batch, budget, states,
                                               actions, &st, 2000 + 2 * restart, 2001 + 2 * restart);
      wall_to_first_ = w0;
      if (!found) anytime_horizon *= horizon_expansion_factor;  // :238-242
      double el = since(t_start);
      if (found) {  // (buildRRTConnectDevice counted the solution)
        if (wall_to_first_ < 0) wall_to_first_ = el;
        postProcessPath(states, actions, terrain);  // :398
        if (path_cost_ < cost_so_far) {             // :401-414
          cost_so_far = path_cost_;
          best_length = path_length_;
          best_yaw = path_yaw_;
          best_states = states;
          best_actions = actions;
          el = since(t_start);
          length_vector_.push_back(best_length);
          yaw_vector_.push_back(best_yaw);
          cost_vector_.push_back(cost_so_far);
          cost_vector_times_.push_back(el);
        }
        goal_found = true;
      }
      if (goal_found && el >= max_time_opt) break;
      if (el >= max_time) break;
      continue;
    }
    PlannerClass Ta(terrain.device()), Tb(terrain.device());
    Ta.setStream(seed_, 2000 + 2 * restart);
    Tb.setStream(seed_, 2001 + 2 * restart);
    Ta.init(s_start, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
    Tb.init(s_goal, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
    const auto t_run = std::chrono::high_resolution_clock::now();
    bool found = false;
    int ia = -1, ib = -1;
    while (true) {  // runRRTConnect (:228-318) at batch granularity
      if (since(t_run) >= anytime_horizon) {
        anytime_horizon *= horizon_expansion_factor;
        break;
      }
      st.iterations++;
      if (halfIterationBatched(Ta, Tb, terrain, FORWARD, batch, ia, ib, &st) ||
          halfIterationBatched(Tb, Ta, terrain, REVERSE, batch, ib, ia, &st)) {
        found = true;
        break;
      }
      if (since(t_start) >= max_time) break;
    }
    num_vertices += Ta.getNumVertices() + Tb.getNumVertices();
    st.vertices_a = Ta.getNumVertices();
    st.vertices_b = Tb.getNumVertices();
    tree_extent(Ta, st.extent_a);
    tree_extent(Tb, st.extent_b);
    double el = since(t_start);
    if (found) {
      st.solutions++;
      if (wall_to_first_ < 0) wall_to_first_ = el;
      std::vector<int> path_a = pathFromStart(Ta, ia);
      std::vector<int> path_b = pathFromStart(Tb, ib);
      std::reverse(path_b.begin(), path_b.end());
      std::vector<Action> action_b = getActionSequenceReverse(Tb, path_b);
      path_b.erase(path_b.begin());
      std::vector<State> states = getStateSequence(Ta, path_a);
      std::vector<State> sb = getStateSequence(Tb, path_b);
      states.insert(states.end(), sb.begin(), sb.end());
      std::vector<Action> actions = getActionSequence(Ta, path_a);
      actions.insert(actions.end(), action_b.begin(), action_b.end());
      path_length_ = Ta.getGValue(ia) + Tb.getGValue(ib);
      path_yaw_ = Ta.getYValue(ia) + Tb.getYValue(ib);
      postProcessPath(states, actions, terrain);  // :398, sets path_length_/path_cost_
      if (path_cost_ < cost_so_far) {  // :401-414
        cost_so_far = path_cost_;
        best_length = path_length_;
        best_yaw = path_yaw_;
        best_states = states;
        best_actions = actions;
        el = since(t_start);
        length_vector_.push_back(best_length);
        yaw_vector_.push_back(best_yaw);
        cost_vector_.push_back(cost_so_far);
        cost_vector_times_.push_back(el);
      }
      goal_found = true;
    }
    if (goal_found && el >= max_time_opt) break;  // :417
    if (el >= max_time) break;                     // no (further) time: the best so far
  }
  elapsed_total = std::chrono::high_resolution_clock::now() - t_start;
  if (!goal_found) return false;
  state_sequence = best_states;
  action_sequence = best_actions;
  path_length_ = best_length;
  path_yaw_ = best_yaw;
  path_cost_ = cost_so_far;
  path_duration_ = 0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
  return true;
}

// ============================================================================
// RRTStarConnectClass
// ============================================================================
void RRTStarConnectClass::insertStar(PlannerClass &T, FastTerrainMap &terrain, int dir,
                                     const std::vector<int> &added,
                                     const std::vector<int> &nearest,
                                     const std::vector<Action> &a_new, BatchStats *stats) {
  if (added.empty()) return;
  // neighbourhoods (rrt_star_connect.cpp:28): vertex k sees the vertices
  // before it, exactly the tree a sequential insertion would scan
  std::vector<State> q;
  for (int idx : added) q.push_back(T.getVertex(idx));
  const std::vector<std::vector<int>> nb = T.neighborhoodDistBatch(q, delta, added);
  // every connect the insertion may need, in one lock-step batch: choose-parent
  // attemptConnect(s_near, s_new) (:36) and rewire attemptConnect(s_new, s_near) (:59)
  std::vector<State> se, ss;
  std::vector<double> ts;
  std::vector<size_t> first(added.size() + 1, 0);
  for (size_t k = 0; k < added.size(); k++) {
    first[k] = se.size();
    for (int j : nb[k]) {
      const State sn = T.getVertex(j);
      se.push_back(sn);  // choose-parent
      ss.push_back(q[k]);
      ts.push_back(poseDistance(q[k], sn) / V_NOM);
      se.push_back(q[k]);  // rewire
      ss.push_back(sn);
      ts.push_back(poseDistance(sn, q[k]) / V_NOM);
    }
  }
  first[added.size()] = se.size();
  std::vector<int> res;
  std::vector<State> dummy(se.size(), State{});
  std::vector<Action> act(se.size(), Action{});
  if (!se.empty())
    attemptConnectBatch(se, ss, ts, terrain, dir, res, dummy, act, stats, /*max_depth=*/0);
  if (stats) stats->connects += (int64_t)se.size();
  // sequential replay of rrt_star_connect.cpp:18-66 for each new vertex in order
  for (size_t k = 0; k < added.size(); k++) {
    const int s_new_idx = added[k];
    const State s_new = q[k];
    const int s_nearest_index = nearest[k];
    const State s_nearest = T.getVertex(s_nearest_index);
    int s_min_idx = s_nearest_index;
    Action a_sel = a_new[k];
    double g_s_new = T.getGValue(s_nearest_index) + poseDistance(s_new, s_nearest);
    double y_s_new = T.getYValue(s_nearest_index) + stateYawDistance(s_new, s_nearest);
    for (size_t i = 0; i < nb[k].size(); i++) {  // choose parent (:31-44)
      const size_t c = first[k] + 2 * i;
      if (res[c] != GBP_PLANNER_REACHED) continue;
      const int j = nb[k][i];
      const State s_near = T.getVertex(j);
      const double g_s_near = T.getGValue(j) + poseDistance(s_near, s_new);
      const double y_s_near = T.getYValue(j) + stateYawDistance(s_near, s_new);
      if (g_s_near < g_s_new) {
        a_sel = act[c];
        s_min_idx = j;
        g_s_new = g_s_near;
        y_s_new = y_s_near;
      }
    }
    T.addEdge(s_min_idx, s_new_idx);  // :47-49
    T.updateGYValue(s_new_idx, g_s_new, y_s_new);
    T.addAction(s_new_idx, a_sel);
    for (size_t i = 0; i < nb[k].size(); i++) {  // rewire (:51-66)
      const int j = nb[k][i];
      if (j == s_min_idx) continue;
      const size_t c = first[k] + 2 * i + 1;
      const State s_near = T.getVertex(j);
      if (res[c] == GBP_PLANNER_REACHED &&
          T.getGValue(j) > (T.getGValue(s_new_idx) + poseDistance(s_near, s_new))) {
        const int s_parent = T.getPredecessor(j);
        T.removeEdge(s_parent, j);
        T.addEdge(s_new_idx, j);
        T.updateGYValue(j, T.getGValue(s_new_idx) + poseDistance(s_near, s_new),
                        T.getYValue(s_new_idx) + stateYawDistance(s_near, s_new));
        T.addAction(j, act[c]);
        rewires_++;
        if (stats) stats->rewires++;
      }
    }
  }
}

int RRTStarConnectClass::extend(PlannerClass &T, State s, FastTerrainMap &terrain, int direction) {
  const int s_nearest_index = T.getNearestNeighbor(s);  // rrt_star_connect.cpp:12-19
  const State s_nearest = T.getVertex(s_nearest_index);
  State s_new{};
  Action a_new{};
  if (!newConfig(s, s_nearest, s_new, a_new, terrain, direction)) return GBP_PLANNER_TRAPPED;
  const int s_new_idx = T.getNumVertices();
  T.addVertex(s_new_idx, s_new);
  insertStar(T, terrain, direction, {s_new_idx}, {s_nearest_index}, {a_new}, nullptr);
  return isWithinBounds(s_new, s) ? GBP_PLANNER_REACHED : GBP_PLANNER_ADVANCED;
}

void RRTStarConnectClass::getStateAndActionSequences(PlannerClass &Ta, PlannerClass &Tb,
                                                     int shared_a_idx, int shared_b_idx,
                                                     std::vector<State> &state_sequence,
                                                     std::vector<Action> &action_sequence) {
  state_sequence.clear();  // rrt_star_connect.cpp:70-89
  action_sequence.clear();
  std::vector<int> path_a = pathFromStart(Ta, shared_a_idx);
  std::vector<int> path_b = pathFromStart(Tb, shared_b_idx);
  std::reverse(path_b.begin(), path_b.end());
  std::vector<Action> action_sequence_b = getActionSequenceReverse(Tb, path_b);
  path_b.erase(path_b.begin());
  state_sequence = getStateSequence(Ta, path_a);
  std::vector<State> sb = getStateSequence(Tb, path_b);
  state_sequence.insert(state_sequence.end(), sb.begin(), sb.end());
  action_sequence = getActionSequence(Ta, path_a);
  action_sequence.insert(action_sequence.end(), action_sequence_b.begin(), action_sequence_b.end());
}

void RRTStarConnectClass::buildRRTStarConnect(FastTerrainMap &terrain, State s_start, State s_goal,
                                              std::vector<State> &state_sequence,
                                              std::vector<Action> &action_sequence,
                                              double max_time) {  // rrt_star_connect.cpp:91-205
  const auto t_start = std::chrono::high_resolution_clock::now();
  success_ = 0;
  length_vector_.clear();
  yaw_vector_.clear();
  cost_vector_.clear();
  cost_vector_times_.clear();
  PlannerClass Ta(terrain.device()), Tb(terrain.device());
  Ta.setStream(seed_, 301);
  Tb.setStream(seed_, 302);
  Ta.init(s_start, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  Tb.init(s_goal, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  int shared_a_idx = -1, shared_b_idx = -1;
  std::vector<int> shared_a, shared_b;
  goal_found = false;
  wall_to_first_ = -1;
  const double length_so_far = INFTY, yaw_so_far = INFTY;  // never updated by the reference
  double cost_so_far = INFTY;
  while (true) {
    State s_rand = Ta.randomState(terrain);
    if (isValidState(s_rand, terrain, STANCE)) {
      if (extend(Ta, s_rand, terrain, FORWARD) != GBP_PLANNER_TRAPPED) {
        const State s_new = Ta.getVertex(Ta.getNumVertices() - 1);
        if (connect(Tb, s_new, terrain, REVERSE) == GBP_PLANNER_REACHED) {
          if (!goal_found) {
            elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
            wall_to_first_ = elapsed_to_first.count();
          }
          goal_found = true;
          shared_a.push_back(Ta.getNumVertices() - 1);
          shared_b.push_back(Tb.getNumVertices() - 1);
        }
      }
    }
    s_rand = Tb.randomState(terrain);
    if (isValidState(s_rand, terrain, STANCE)) {
      if (extend(Tb, s_rand, terrain, REVERSE) != GBP_PLANNER_TRAPPED) {
        const State s_new = Tb.getVertex(Tb.getNumVertices() - 1);
        if (connect(Ta, s_new, terrain, FORWARD) == GBP_PLANNER_REACHED) {
          if (!goal_found) {
            elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
            wall_to_first_ = elapsed_to_first.count();
          }
          goal_found = true;
          shared_a.push_back(Ta.getNumVertices() - 1);
          shared_b.push_back(Tb.getNumVertices() - 1);
        }
      }
    }
    const std::chrono::duration<double> el = std::chrono::high_resolution_clock::now() - t_start;
    if (goal_found && el.count() >= max_time) break;
    for (size_t i = 0; i < shared_a.size(); ++i) {
      const double cost = Ta.getGValue(shared_a[i]) + Tb.getGValue(shared_b[i]);
      if (cost < cost_so_far) {
        cost_so_far = cost;
        shared_a_idx = shared_a[i];
        shared_b_idx = shared_b[i];
        length_vector_.push_back(length_so_far);
        yaw_vector_.push_back(yaw_so_far);
        cost_vector_.push_back(cost_so_far);
        cost_vector_times_.push_back(
            std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t_start)
                .count());
      }
    }
  }
  // the reference leaves the loop before ranking a connection found in its last
  // iteration (shared_a_idx may then be uninitialised): rank once more
  for (size_t i = 0; i < shared_a.size(); ++i) {
    const double cost = Ta.getGValue(shared_a[i]) + Tb.getGValue(shared_b[i]);
    if (cost < cost_so_far) {
      cost_so_far = cost;
      shared_a_idx = shared_a[i];
      shared_b_idx = shared_b[i];
    }
  }
  num_vertices = Ta.getNumVertices() + Tb.getNumVertices();
  if (goal_found && shared_a_idx >= 0)
    getStateAndActionSequences(Ta, Tb, shared_a_idx, shared_b_idx, state_sequence, action_sequence);
  elapsed_total = std::chrono::high_resolution_clock::now() - t_start;
  length_vector_.push_back(length_so_far);
  yaw_vector_.push_back(yaw_so_far);
  cost_vector_.push_back(cost_so_far);
  cost_vector_times_.push_back(elapsed_total.count());
  best_cost_ = cost_so_far;
  if (!state_sequence.empty()) postProcessPath(state_sequence, action_sequence, terrain);
  if (elapsed_total.count() <= 5.0) success_ = 1;
  path_duration_ = 0.0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
}

bool RRTStarConnectClass::buildRRTStarConnectBatched(FastTerrainMap &terrain, State s_start,
                                                     State s_goal, int batch, double max_time,
                                                     std::vector<State> &state_sequence,
                                                     std::vector<Action> &action_sequence,
                                                     BatchStats *stats) {
  const auto t_start = std::chrono::high_resolution_clock::now();
  goal_found = false;
  wall_to_first_ = -1;
  rewires_ = 0;
  cost_vector_.clear();
  cost_vector_times_.clear();
  PlannerClass Ta(terrain.device()), Tb(terrain.device());
  Ta.setStream(seed_, 401);
  Tb.setStream(seed_, 402);
  Ta.init(s_start, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  Tb.init(s_goal, cost_add_yaw_flag_, cost_add_yaw_length_weight_, cost_add_yaw_yaw_weight_);
  BatchStats local;
  BatchStats &st = stats ? *stats : local;
  std::vector<int> shared_a, shared_b;
  int best_a = -1, best_b = -1;
  double cost_so_far = INFTY;
  while (st.max_halves <= 0 || st.halves + 2 <= st.max_halves) {
    const double el =
        std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t_start).count();
    if (el >= max_time) break;
    st.iterations++;
    st.halves += 2;
    for (int half = 0; half < 2; half++) {
      PlannerClass &T = half == 0 ? Ta : Tb;
      PlannerClass &O = half == 0 ? Tb : Ta;
      const int dir = half == 0 ? FORWARD : REVERSE;
      std::vector<int> added, nearest;
      std::vector<Action> a_new;
      extendBatch(T, terrain, dir, batch, added, nearest, a_new, /*insert=*/false, &st);
      insertStar(T, terrain, dir, added, nearest, a_new, &st);
      for (const auto &pr : connectBatch(T, O, terrain, dir, added, &st)) {
        if (!goal_found) {
          elapsed_to_first = std::chrono::high_resolution_clock::now() - t_start;
          wall_to_first_ = elapsed_to_first.count();
        }
        goal_found = true;
        shared_a.push_back(half == 0 ? pr.first : pr.second);
        shared_b.push_back(half == 0 ? pr.second : pr.first);
        st.solutions++;
      }
    }
    for (size_t i = 0; i < shared_a.size(); ++i) {  // rewiring keeps lowering g
      const double cost = Ta.getGValue(shared_a[i]) + Tb.getGValue(shared_b[i]);
      if (cost < cost_so_far) {
        cost_so_far = cost;
        best_a = shared_a[i];
        best_b = shared_b[i];
        cost_vector_.push_back(cost_so_far);
        cost_vector_times_.push_back(
            std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t_start)
                .count());
      }
    }
  }
  tree_extent(Ta, st.extent_a);
  tree_extent(Tb, st.extent_b);
  st.vertices_a = Ta.getNumVertices();
  st.vertices_b = Tb.getNumVertices();
  num_vertices = Ta.getNumVertices() + Tb.getNumVertices();
  best_cost_ = cost_so_far;
  dump_trees(Ta, Tb, st.dump);
  st.meet_a = best_a;
  st.meet_b = best_b;
  if (!goal_found) return false;
  getStateAndActionSequences(Ta, Tb, best_a, best_b, state_sequence, action_sequence);
  path_length_ = Ta.getGValue(best_a) + Tb.getGValue(best_b);
  path_yaw_ = Ta.getYValue(best_a) + Tb.getYValue(best_b);
  path_cost_ = weightedCost(path_length_, path_yaw_);
  path_duration_ = 0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
  return true;
}

bool RRTStarConnectClass::buildRRTStarConnectDevice(FastTerrainMap &terrain, State s_start,
                                                    State s_goal, int batch, double max_time,
                                                    std::vector<State> &state_sequence,
                                                    std::vector<Action> &action_sequence,
                                                    BatchStats *stats) {
  const auto t_start = std::chrono::high_resolution_clock::now();
  auto since = [&]() {
    return std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t_start).count();
  };
  goal_found = false;
  wall_to_first_ = -1;
  rewires_ = 0;
  cost_vector_.clear();
  cost_vector_times_.clear();
  BatchStats local;
  BatchStats &st = stats ? *stats : local;
  gbp_terrain *h = terrain.handle();
  const int dev = terrain.device();
  const int adaptive = state_action_pair_check_adaptive_step_size_flag_ ? 1 : 0;
  // RRT*'s targets are plain randomState draws (extendBatch without O); the
  // candidates keep the action sampling (rrt.cpp:34, :49)
  gbp_sampling cfg = samplingConfig();
  cfg.state_flag = 0;
  chk(gbp_terrain_set_sampling(h, &cfg), "sampling");
  DeviceTrees D;
  chk(gbp_stream_create(dev, &D.stream), "stream");
  chk(gbp_plan_ws_create(h, batch, &D.ws), "plan workspace");
  // neighbour pairs of one half (2 connect checks each) and REACHED connections of the run
  int64_t star_pairs_cap = std::max<int64_t>(1 << 18, 8 * (int64_t)batch);
  chk(gbp_plan_star_config(D.ws, 1, delta, star_pairs_cap, 1 << 22), "star config");
  if (st.stage_timing) chk(gbp_plan_stage_timing(D.ws, 1), "stage timing");
  int64_t cap = std::max<int64_t>(1 << 16, 4 * (int64_t)batch);
  int64_t known[2] = {1, 1};
  for (int k = 0; k < 2; k++) {
    // warm start (a replayable continuation): the given trees, rewired parents included
    const int64_t wn = st.warm_n[k];
    if (wn > 0 && (!st.warm_v[k] || !st.warm_a[k] || !st.warm_parent[k]))
      throw EngineError(GBP_E_INVALID_ARG, "warm start: tree arrays");
    chk(gbp_tree_create(dev, std::max<int64_t>(cap, 2 * wn), &D.tree[k]), "tree");
    if (wn > 0)
      chk(gbp_tree_load_host(D.tree[k], wn, st.warm_v[k], st.warm_a[k], st.warm_parent[k], D.stream),
          "warm start: tree load");
    else
      chk(gbp_tree_init(D.tree[k], k == 0 ? s_start.data() : s_goal.data(), D.stream), "tree init");
    known[k] = std::max<int64_t>(1, wn);
  }
  if (st.warm_half < 0 || (st.warm_half & 1) || st.warm_extend < 0)
    throw EngineError(GBP_E_INVALID_ARG, "warm start");
  const int32_t half0 = (int32_t)st.warm_half;
  if (st.warm_n[0] > 0 || st.warm_n[1] > 0 || half0 > 0) extend_counter_ = st.warm_extend;
  chk(gbp_plan_reset(D.ws, extend_counter_, D.stream), "plan reset");
  const uint64_t tstream[2] = {401, 402};  // buildRRTStarConnectBatched's streams
  const int g_max = (int)std::max<int64_t>(2, std::min<int64_t>(64, (1 << 21) / batch)) & ~1;
  int group = 2;
  int32_t half = half0;
  gbp_plan_status ps{};
  while (since() < max_time && (st.max_halves <= 0 || half - half0 + 2 <= st.max_halves)) {
    if (st.max_halves > 0)
      group = (int)std::min<int64_t>(group, (st.max_halves - (half - half0)) & ~1LL);
    for (int k = 0; k < 2; k++) {
      int64_t c = 0;
      chk(gbp_tree_capacity(D.tree[k], &c), "tree capacity");
      if (known[k] + (int64_t)group * batch > c)
        chk(gbp_tree_reserve(D.tree[k], std::max<int64_t>(2 * c, known[k] + (int64_t)group * batch),
                             D.stream),
            "tree reserve");
    }
    chk(gbp_plan_halves_dev(h, D.ws, D.tree[0], D.tree[1], half, group, batch, seed_, tstream[0],
                            tstream[1], adaptive, 0, D.stream),
        "plan halves");
    chk(gbp_plan_status_read(D.ws, &ps, D.stream), "plan status");
    st.status_reads++;
    while (ps.halt) {  // FRAGILE: re-decide on the host, resume where the sequence stopped
      for (int b = 0; b < 4; b++) st.halts[b] += (ps.halt >> b) & 1u;
      const int32_t h0 = ps.halt_half;
      const int k = h0 & 1;
      int resume = -1;
      int64_t nres = 0;
      if (ps.halt & GBP_PLAN_HALT_STAR_PAIRS) {
        // a half's neighbour pairs outgrew the insertion sets: grow them (the
        // run's kept connections stay) and redo the half's stage 6
        st.star_grows++;
        star_pairs_cap = std::max<int64_t>(2 * star_pairs_cap, (int64_t)ps.star_pairs + ps.star_pairs / 4);
        chk(gbp_plan_star_config(D.ws, 1, delta, star_pairs_cap, 1 << 22), "star config (grow)");
      }
      chk(gbp_plan_resolve_host(h, D.ws, D.tree[k], D.tree[k ^ 1], k == 0 ? FORWARD : REVERSE,
                                batch, adaptive, &resume, &nres, D.stream),
          "plan resolve");
      if (resume < 0) throw EngineError(GBP_E_INVALID_ARG, "plan resolve: nothing halted");
      chk(gbp_plan_halves_dev(h, D.ws, D.tree[0], D.tree[1], h0, half + group - h0, batch, seed_,
                              tstream[0], tstream[1], adaptive, resume, D.stream),
          "plan halves");
      chk(gbp_plan_status_read(D.ws, &ps, D.stream), "plan status");
      st.status_reads++;
    }
    if (ps.error & 1u) throw EngineError(GBP_E_HIP, "device planner loop: look-back spin exhausted");
    if (ps.error & 4u) throw EngineError(GBP_E_SHAPE, "device RRT*: star workspace exhausted");
    if (ps.error) throw EngineError(GBP_E_SHAPE, "device planner loop: a tree ran out of capacity");
    for (int k = 0; k < 2; k++) chk(gbp_tree_size(D.tree[k], &known[k], D.stream), "tree size");
    half += group;
    if (ps.n_shared > 0 && !goal_found) {
      goal_found = true;
      elapsed_to_first = std::chrono::duration<double>(since());
      wall_to_first_ = elapsed_to_first.count();
    }
    if (ps.best_a >= 0 && (cost_vector_.empty() || ps.best_cost < cost_vector_.back())) {
      cost_vector_.push_back(ps.best_cost);  // the best so far, once per group
      cost_vector_times_.push_back(since());
    }
    group = std::min(group * 2, g_max);
  }
  extend_counter_ = ps.ext_counter;
  rewires_ = ps.stat_rewires;
  if (st.stage_timing) {
    double us[7];
    int64_t nh = 0;
    chk(gbp_plan_stage_times(D.ws, us, 7, &nh, 1), "stage times");
    for (int k = 0; k < 7; k++) st.stage_us[k] += us[k];
    st.stage_halves += nh;
  }
  st.halves += half - half0;
  st.iterations += (half - half0) / 2;
  st.targets += ps.stat_targets;
  st.extends += ps.stat_targets;
  st.attempts_checked += ps.stat_attempts;
  st.connects += ps.stat_added + ps.stat_star_connects;
  st.rewires += ps.stat_rewires;
  st.solutions += ps.n_shared;
  st.fragile_resolved += ps.stat_fragile_resolved;
  st.depth_capped += ps.stat_depth_capped;
  st.nn_rechecks += ps.stat_nn_rechecks;
  st.nn_scans += ps.stat_nn_scans;
  HostTree A, B;
  read_tree(D.tree[0], D.stream, A);
  read_tree(D.tree[1], D.stream, B);
  extent(A, st.extent_a);
  extent(B, st.extent_b);
  st.vertices_a = (int64_t)A.v.size();
  st.vertices_b = (int64_t)B.v.size();
  num_vertices = (int)(A.v.size() + B.v.size());
  if (st.dump) {
    const HostTree *t[2] = {&A, &B};
    for (int k = 0; k < 2; k++) {
      st.dump->v[k] = t[k]->v;
      st.dump->a[k] = t[k]->a;
      st.dump->parent[k] = t[k]->parent;
      st.dump->g[k] = t[k]->g;
    }
  }
  best_cost_ = ps.best_a >= 0 ? ps.best_cost : INFINITY_COST;
  st.meet_a = ps.best_a;
  st.meet_b = ps.best_b;
  if (!goal_found || ps.best_a < 0) return false;
  // rrt_star_connect.cpp:70-89 on the device trees
  std::vector<int> path_a = host_path(A, ps.best_a);
  std::vector<int> path_b = host_path(B, ps.best_b);
  std::reverse(path_b.begin(), path_b.end());
  std::vector<Action> action_sequence_b;
  for (size_t i = 0; i + 1 < path_b.size(); ++i) action_sequence_b.push_back(B.a[path_b[i]]);
  const double yaw_b = path_yaw(B, host_path(B, ps.best_b));
  path_b.erase(path_b.begin());
  state_sequence.clear();
  for (int i : path_a) state_sequence.push_back(A.v[i]);
  for (int i : path_b) state_sequence.push_back(B.v[i]);
  action_sequence.clear();
  for (size_t i = 1; i < path_a.size(); ++i) action_sequence.push_back(A.a[path_a[i]]);
  action_sequence.insert(action_sequence.end(), action_sequence_b.begin(), action_sequence_b.end());
  path_length_ = A.g[ps.best_a] + B.g[ps.best_b];
  path_yaw_ = path_yaw(A, path_a) + yaw_b;
  path_cost_ = weightedCost(path_length_, path_yaw_);
  path_duration_ = 0;
  for (const Action &a : action_sequence) path_duration_ += a[6] + a[7];
  return true;
}

}  // namespace gbp_amd

// ============================================================================
// flat C entry point
// ============================================================================
// the layout planner.py's PlanParams mirrors (tests/test_abi.py)
static_assert(sizeof(gbp_plan_params) == 464, "gbp_plan_params layout");
static_assert(sizeof(gbp_plan_result) == 376, "gbp_plan_result layout");

extern "C" int gbp_plan_rrt_connect(const gbp_plan_params *p, gbp_plan_result *r,
                                    double *path_states, double *path_actions, int capacity) {
  using namespace gbp_amd;
  if (!p || !r || p->batch < 1 || p->algorithm < 0 || p->algorithm > 5) return GBP_E_INVALID_ARG;
  try {
    FastTerrainMap terrain(p->device);
    terrain.loadDataFlat(p->nx, p->ny, p->x, p->y, p->z, p->dx, p->dy, p->dz);
    if (p->fragile_eps_fm)
      chk(gbp_terrain_set_option(terrain.handle(), GBP_OPT_FRAGILE_EPS, p->fragile_eps_fm),
          "fragile eps");
    chk(gbp_terrain_set_option(terrain.handle(), GBP_OPT_NN_STATS, p->nn_stats), "nn stats");
    RRTStarConnectClass planner;  // is-a RRTConnectClass: algorithm 0 uses the plain build
    planner.setSeed(p->seed);
    planner.set_state_direction_sampling(p->sampling.state_flag != 0, p->sampling.state_p,
                                         p->sampling.state_speed_direction != 0);
    planner.set_action_direction_sampling(p->sampling.action_flag != 0, p->sampling.action_p);
    planner.set_state_action_pair_check_adaptive_step_size_flag_(p->adaptive != 0);
    State s0, s1;
    std::copy(p->start, p->start + 8, s0.begin());
    std::copy(p->goal, p->goal + 8, s1.begin());
    std::vector<State> states;
    std::vector<Action> actions;
    BatchStats st;
    TreeDump dump;
    st.max_halves = p->max_halves > 0 ? p->max_halves : 0;
    st.stage_timing = p->stage_timing != 0;
    if (p->algorithm == 3 || p->algorithm == 5) {
      if (p->algorithm == 3) {  // one device search per rank: the ranks' polls pair up
        st.stop_poll = p->stop_poll;
        st.stop_ctx = p->stop_ctx;
      }
      for (int k = 0; k < 2; k++) {  // warm start (a replayable continuation)
        st.warm_n[k] = p->init_n[k];
        st.warm_v[k] = p->init_v[k];
        st.warm_a[k] = p->init_a[k];
        st.warm_parent[k] = p->init_parent[k];
      }
      st.warm_half = p->first_half;
      st.warm_extend = p->extend_base;
    } else if (p->init_n[0] || p->init_n[1] || p->first_half || p->extend_base) {
      return GBP_E_INVALID_ARG;
    }
    if (p->tree_capacity > 0) st.dump = &dump;
    const auto t0 = std::chrono::high_resolution_clock::now();
    const bool found =
        p->algorithm == 1
            ? planner.buildRRTStarConnectBatched(terrain, s0, s1, p->batch, p->max_time, states,
                                                 actions, &st)
        : p->algorithm == 5
            ? planner.buildRRTStarConnectDevice(terrain, s0, s1, p->batch, p->max_time, states,
                                                actions, &st)
        : p->algorithm == 2
            ? planner.buildRRTConnectBatchedAnytime(terrain, s0, s1, p->batch, p->max_time,
                                                    p->max_time_opt, states, actions, &st)
        : p->algorithm == 3
            ? planner.buildRRTConnectDevice(terrain, s0, s1, p->batch, p->max_time, states,
                                            actions, &st)
        : p->algorithm == 4
            ? planner.buildRRTConnectBatchedAnytime(terrain, s0, s1, p->batch, p->max_time,
                                                    p->max_time_opt, states, actions, &st, true)
            : planner.buildRRTConnectBatched(terrain, s0, s1, p->batch, p->max_time, states,
                                             actions, &st);
    double ttf = planner.wallTimeToFirst();
    // algorithm 2 / 4's paths are post-processed inside the restarts (as buildRRTConnect)
    if (found && p->post_process && p->algorithm != 2 && p->algorithm != 4)
      planner.postProcessPath(states, actions, terrain);
    const std::chrono::duration<double> tot = std::chrono::high_resolution_clock::now() - t0;
    memset(r, 0, sizeof(*r));
    r->found = found ? 1 : 0;
    r->time_to_first = found ? ttf : -1.0;
    r->total_time = tot.count();
    r->iterations = st.iterations;
    r->targets = st.targets;
    r->extends = st.extends;
    r->attempts_checked = st.attempts_checked;
    r->connects = st.connects;
    r->vertices_a = st.vertices_a;
    r->vertices_b = st.vertices_b;
    r->n_states = found ? (int)states.size() : 0;
    r->rewires = st.rewires;
    for (int k = 0; k < 7; k++) r->stage_us[k] = st.stage_us[k];
    r->stage_halves = st.stage_halves;
    r->solutions = st.solutions;
    for (int k = 0; k < 4; k++) {
      r->extent_a[k] = st.extent_a[k];
      r->extent_b[k] = st.extent_b[k];
    }
    r->fragile_resolved = st.fragile_resolved;
    r->depth_capped = st.depth_capped;
    r->status_reads = st.status_reads;
    for (int k = 0; k < 4; k++) r->halts[k] = st.halts[k];
    r->nn_rechecks = st.nn_rechecks;
    r->nn_scans = st.nn_scans;
    r->reported_length = found ? planner.pathLength() : 0.0;
    r->reported_yaw = found ? planner.pathYaw() : 0.0;
    r->meet_a = st.meet_a;
    r->meet_b = st.meet_b;
    r->halves = st.halves;
    r->polls = st.polls;
    r->stopped_by_peer = st.stopped_by_peer;
    if (st.dump)
      for (int k = 0; k < 2; k++) {
        const int64_t n = std::min<int64_t>(p->tree_capacity, (int64_t)dump.v[k].size());
        for (int64_t i = 0; i < n; i++) {
          if (p->tree_v[k]) std::copy(dump.v[k][i].begin(), dump.v[k][i].end(), p->tree_v[k] + 8 * i);
          if (p->tree_a[k]) std::copy(dump.a[k][i].begin(), dump.a[k][i].end(), p->tree_a[k] + 10 * i);
          if (p->tree_parent[k]) p->tree_parent[k][i] = dump.parent[k][i];
          if (p->tree_g[k]) p->tree_g[k][i] = dump.g[k][i];
        }
      }
    if (found) {
      double len = 0;
      for (size_t i = 1; i < states.size(); i++) len += planning_utils::poseDistance(states[i - 1], states[i]);
      r->path_length = len;
      r->path_cost = (p->algorithm == 1 || p->algorithm == 5) ? planner.bestCost() : planner.pathCost();
      double dur = 0;
      for (const Action &a : actions) dur += a[6] + a[7];
      r->path_duration = dur;
      for (int i = 0; i < std::min<int>(capacity, (int)states.size()); i++) {
        if (path_states) std::copy(states[i].begin(), states[i].end(), path_states + 8 * i);
        if (path_actions && i < (int)actions.size())
          std::copy(actions[i].begin(), actions[i].end(), path_actions + 10 * i);
      }
    }
    return GBP_OK;
  } catch (const EngineError &e) {
    return e.status;
  } catch (...) {
    return GBP_E_INVALID_ARG;
  }
}

extern "C" int gbp_terrain_arrays_from_csv(const char *dir, int *nx, int *ny, double *x,
                                           double *y, double *z, double *dx, double *dy,
                                           double *dz, int64_t capacity) {
  if (!dir || !nx || !ny) return GBP_E_INVALID_ARG;
  try {
    const gbp_amd::TerrainArrays t = gbp_amd::terrainArraysFromCSV(dir);
    *nx = t.x_size;
    *ny = t.y_size;
    if (!z) return GBP_OK;
    const size_t cells = (size_t)t.x_size * t.y_size;
    if (capacity < (int64_t)cells) return GBP_E_SHAPE;
    if (x) std::copy(t.x.begin(), t.x.end(), x);
    if (y) std::copy(t.y.begin(), t.y.end(), y);
    std::copy(t.z.begin(), t.z.end(), z);
    if (dx) std::copy(t.dx.begin(), t.dx.end(), dx);
    if (dy) std::copy(t.dy.begin(), t.dy.end(), dy);
    if (dz) std::copy(t.dz.begin(), t.dz.end(), dz);
    return GBP_OK;
  } catch (...) {
    return GBP_E_INVALID_ARG;
  }
}

extern "C" int gbp_attempt_connect_batch(gbp_terrain *t, int64_t n, const double *s_existing,
                                         const double *s, const double *t_s, int direction,
                                         int adaptive, int32_t *result, double *s_new,
                                         double *a_new) {
  using namespace gbp_amd;
  if (!t) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!s_existing || !s || !result || !s_new || !a_new)) ||
      (direction != GBP_FORWARD && direction != GBP_REVERSE))
    return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  try {
    FastTerrainMap terrain = FastTerrainMap::borrow(t);
    RRTConnectClass rc;
    rc.set_state_action_pair_check_adaptive_step_size_flag_(adaptive != 0);
    std::vector<State> se(n), sq(n), sn(n);
    std::vector<Action> an(n);
    std::vector<double> ts(n);
    for (int64_t i = 0; i < n; i++) {
      std::copy(s_existing + 8 * i, s_existing + 8 * i + 8, se[i].begin());
      std::copy(s + 8 * i, s + 8 * i + 8, sq[i].begin());
      std::copy(s_new + 8 * i, s_new + 8 * i + 8, sn[i].begin());
      std::copy(a_new + 10 * i, a_new + 10 * i + 10, an[i].begin());
      const double v = t_s ? t_s[i] : 0.0;
      ts[i] = (v > 0) ? v : planning_utils::poseDistance(sq[i], se[i]) / planning_utils::V_NOM;
    }
    std::vector<int> r;
    rc.attemptConnectBatchPublic(se, sq, ts, terrain, direction, r, sn, an);
    for (int64_t i = 0; i < n; i++) {
      result[i] = r[i];
      std::copy(sn[i].begin(), sn[i].end(), s_new + 8 * i);
      std::copy(an[i].begin(), an[i].end(), a_new + 10 * i);
    }
    return GBP_OK;
  } catch (const EngineError &e) {
    return e.status;
  } catch (...) {
    return GBP_E_INVALID_ARG;
  }
}
