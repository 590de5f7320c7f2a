// layout.h — host-side problem builder for the HIP engine.
//
// Replaces, for the eval path, what the reference derives at setup in
//   NlpFormulation::GetVariableSets / GetConstraints (towr/src/nlp_formulation.cc:76-378),
//   NodesVariables*::GetPhaseBasedEEParameterization (nodes_variables_phase_based.cc:201-396),
//   TimeDiscretizationConstraint ctor (time_discretization_constraint.cc:37-50),
//   ifopt's Jacobian assembly (ConstraintSet::GetJacobian / setFromTriplets),
// and emits flat, batch-shared device tables: node->column map, polynomial durations, work items,
// CSR pattern, per-candidate slot table and LDS tiles.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "engine_math.h"

namespace tg {

struct TileDesc {
  int32_t i0, i1;   // items [i0, i1)
  int32_t r0, r1;   // rows  [r0, r1)
  int32_t v0, v1;   // values (CSR positions) [v0, v1)
  int32_t type, reserved;
};

struct VarSetInfo { int kind, ee, col0, n; };
struct ConsInfo { int kind, ee, row0, rows; };

struct Layout {
  int n = 0, m = 0;
  int64_t nnz = 0;
  std::vector<VarSetInfo> varsets;
  std::vector<ConsInfo> cons;
  std::vector<SplineMeta> spl;
  std::vector<int32_t> nodecol;
  std::vector<double> dur;
  std::vector<ItemDesc> items;
  std::vector<int32_t> slots;
  std::vector<int64_t> row_ptr;
  std::vector<int32_t> col;
  std::vector<TileDesc> tiles;
  std::vector<double> x0;
  RobotC rb{};
  towr_terrain_t terrain{};
  int32_t fdisc_motion = 0;
  int max_tile_values = 0, max_tile_rows = 0;
  towr_problem_desc_t desc{};
};

// Limits of one LDS tile (doubles) — the kernel's dynamic LDS is sized from these.
constexpr int kTileValueCap = 3072;
constexpr int kTileRowCap = 512;
constexpr int kTileItemCap = 256;

// Returns TOWR_OK or an error code with a message in `err`.
int build_layout(const towr_problem_desc_t& d, Layout& L, std::string& err);

// x0 for another init/terrain on the layout built from `d` (nlp_formulation.cc:121-346).
int initial_x_for(const towr_problem_desc_t& d, const towr_init_t& init, const towr_terrain_t& ter,
                  std::vector<double>& x0, std::string& err);

// Tile groups: contiguous tile ranges of roughly equal value counts; out has n_groups + 1 entries.
void group_tiles(const Layout& L, int n_groups, std::vector<int32_t>& out);

}  // namespace tg
