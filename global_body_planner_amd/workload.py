"""Benchmark / parity workloads (SURVEY §8(d) "Attempt inputs", configs 2-3).

An attempt batch is (s_near, action, direction):
  s_near    PlannerClass::randomState (planner_class.cpp:38-76) filtered by
            isValidState(., STANCE) — the tree vertices an extend starts from;
  action    getRandomAction(getSurfaceNormal(target)) (planning_utils.cpp:392-442,
            rrt.cpp:25) for a target drawn from the same randomState distribution;
  direction alternating FORWARD / REVERSE (the Ta / Tb halves of runRRTConnect,
            rrt_connect.cpp:257, :292).
Every draw is Philox-addressed by (seed, stream, index), so a slice
[lo, hi) of a batch is identical whichever rank / device generates it.
"""
import torch

from . import _lib as L

STREAM_S_NEAR = 1
STREAM_TARGET = 2
STREAM_ACTION = 3
MAX_TRIES = 256

# BASELINE.md §3 "Concrete input" seeds
CONFIG_SEEDS = {2: 20251017, 3: 20251018}


def make_attempts(terrain, n, seed, index_base=0):
    """Generate attempts [index_base, index_base + n) on the terrain's GPU."""
    s_near, tries = terrain.sample_states(n, seed, STREAM_S_NEAR, index_base,
                                          require_phase=L.STANCE, max_tries=MAX_TRIES)
    target, _ = terrain.sample_states(n, seed, STREAM_TARGET, index_base)
    nrm, _ = terrain.normal(target[:, :2])
    action = terrain.sample_actions(nrm, seed, STREAM_ACTION, index_base)
    idx = torch.arange(index_base, index_base + n, device=s_near.device)
    direction = (idx % 2).to(torch.uint8)
    return s_near, action, direction, target, tries

