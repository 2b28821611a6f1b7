// grid.hpp — candidate grid of the nearest-primitive cache's full map() (rmr_trace.h map_grid_npc):
// host construction, shared by the context upload (rmr_api.cpp build_grid) and the CPU-testable
// C-ABI hook rmr_candidate_grid.
#pragma once
#include <hip/hip_runtime.h>   // (vector types of rmr_internal.h)

#include <cstdint>
#include <vector>

#include "rmr_internal.h"

namespace rmr {

struct CandidateGrid {
    float lo[3] = {0, 0, 0};
    float inv = 1.0f;            // 1 / cell size (the kernel's cell index: floor((p - lo) * inv))
    int dim[3] = {0, 0, 0};
    int n_large = 0;             // leaf indices [0, n_large) are evaluated everywhere
    float sbox[6] = {0, 0, 0, 0, 0, 0};   // the small primitives' box (lo.xyz, hi.xyz), rounded outward
    double eps = 0.0, margin = 0.0;       // float error bound of a distance in the grid; list margin
    std::vector<uint32_t> cells;  // 2 per cell: list offset | count << 24 (255: no list), bound bits
    std::vector<uint16_t> list;   // leaf indices
};

// Small primitives: leaf indices [n_large, dp.size()). E = max |c|_inf + |r|_inf over the scene.
// target: cell count of the region; pad: region growth (fraction of the small primitives' extent).
// False when no grid applies (no small primitive, > 65535 primitives, too many cells or entries).
bool build_candidate_grid(const std::vector<DPrim>& dp, int n_large, double E, double target, double pad,
                          CandidateGrid& g);

}  // namespace rmr
