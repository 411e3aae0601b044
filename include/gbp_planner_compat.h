// gbp_planner_compat.h — the reference's global names for the engine-backed
// planner classes, so code written against
//   #include "global_body_planner/fast_terrain_map.h"
//   #include "global_body_planner/planning_utils.h"
//   #include "global_body_planner/rrt_connect.h"
// compiles unchanged against include/gbp_planner.h.
//
// Names exported: FastTerrainMap, PlannerClass, RRTClass, RRTConnectClass,
// RRTStarConnectClass,
// namespace planning_utils (State, Action, constants, apply*/isValid*/...),
// and the TRAPPED / ADVANCED / REACHED macros of rrt.h:7-9.
#pragma once

#include "gbp_planner.h"

using gbp_amd::FastTerrainMap;
using gbp_amd::PlannerClass;
using gbp_amd::RRTClass;
using gbp_amd::RRTConnectClass;
using gbp_amd::RRTStarConnectClass;
namespace planning_utils = gbp_amd::planning_utils;
using namespace gbp_amd::planning_utils;  // the reference's headers do the same (planning_utils.h)

#ifndef TRAPPED
#define TRAPPED GBP_PLANNER_TRAPPED
#endif
#ifndef ADVANCED
#define ADVANCED GBP_PLANNER_ADVANCED
#endif
#ifndef REACHED
#define REACHED GBP_PLANNER_REACHED
#endif
