/*
 * towr_gpu.h — C-ABI of the MI355X (gfx950) constraint/Jacobian evaluation engine for towr's NLP.
 *
 * This is the drop-in boundary for the reference's eval_g / eval_jac_g hot path
 * (hexb66/towr2025). In the reference, IPOPT calls ifopt's IpoptAdapter::eval_g /
 * eval_jac_g, which call ifopt::Problem::EvalConstraints / EvalNonzerosOfJacobian, which call
 * every ifopt::ConstraintSet's GetValues() and FillJacobianBlock(var_set, jac)
 * (towr/include/towr/constraints/time_discretization_constraint.h:50-73,
 *  towr/src/constraints/time_discretization_constraint.cc:65-96). Those callbacks are what
 * this library replaces; IPOPT keeps running on the host.
 *
 * Plain C: POD structs, plain pointers and sizes, int status codes (0 = ok, < 0 = error),
 * no exceptions cross the boundary, no torch types. One handle per host thread; calls on a
 * handle are serialised on that handle's HIP stream.
 *
 * Numbers: every value is IEEE binary64, as in the reference (Eigen double throughout).
 * Jacobian layout: CSR in ifopt order — rows = constraint sets in the order given, each set's
 * rows contiguous; columns = variable sets in the order given; within a row, columns ascend
 * (Eigen::SparseMatrix<double,RowMajor> after setFromTriplets/makeCompressed, which is the
 * (iRow, jCol) order ifopt's IpoptAdapter::eval_jac_g emits).
 */
#ifndef TOWR_GPU_H_
#define TOWR_GPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TOWR_GPU_ABI_VERSION 4

#define TOWR_MAX_EE          4
#define TOWR_MAX_PHASES      48
#define TOWR_MAX_VARSETS     (2 + 5 * TOWR_MAX_EE)
#define TOWR_MAX_CONSTRAINTS 64
#define TOWR_MAX_COSTS       128

/* ---- status codes ---------------------------------------------------------------------- */
#define TOWR_OK                  0
#define TOWR_ERR_INVALID        -1   /* malformed description / argument                       */
#define TOWR_ERR_UNSUPPORTED    -2   /* valid for the reference, not (yet) for this engine     */
#define TOWR_ERR_HIP            -3   /* HIP runtime failure (message in towr_gpu_last_error)    */
#define TOWR_ERR_NO_DEVICE      -4   /* no gfx950 device / extension not loadable on this host  */

/* ---- terrain: HeightMap::TerrainID (towr/include/towr/terrain/height_map.h:79-86) --------- */
enum towr_terrain_id {
  TOWR_TERRAIN_FLAT       = 0, /* FlatGround   p[0]=height                                  (height_map_examples.h:45-52)  */
  TOWR_TERRAIN_BLOCK      = 1, /* Block        p[0]=block_start p[1]=length p[2]=height p[3]=eps (:57-69)            */
  TOWR_TERRAIN_STAIRS     = 2, /* Stairs       p[0]=first_step_start p[1]=first_step_width
                                  p[2]=height_first_step p[3]=height_second_step p[4]=width_top   (:74-84)           */
  TOWR_TERRAIN_GAP        = 3, /* Gap          p[0]=gap_start p[1]=w p[2]=h                  (:89-112)                */
  TOWR_TERRAIN_SLOPE      = 4, /* Slope        p[0]=slope_start p[1]=up_length p[2]=down_length p[3]=height_center (:117-131) */
  TOWR_TERRAIN_CHIMNEY    = 5, /* Chimney      p[0]=x_start p[1]=length p[2]=y_start p[3]=slope (:136-148)             */
  TOWR_TERRAIN_CHIMNEY_LR = 6, /* ChimneyLR    p[0]=x_start p[1]=length p[2]=y_start p[3]=slope (:153-166)             */
  TOWR_TERRAIN_STEPS      = 7  /* FiveStepStairs of towr/test/hopper_example.cc:53-86:
                                  p[0]=stairs_start p[1]=step_depth p[2]=step_height p[3]=num_steps              */
};

typedef struct {
  int32_t id;              /* towr_terrain_id                                                  */
  int32_t reserved;
  double  friction_coeff;  /* HeightMap::friction_coeff_ = 0.5 (height_map.h:136)             */
  double  p[8];            /* per-type parameters, see enum                                    */
} towr_terrain_t;

/* ---- robot: SingleRigidBodyDynamics + KinematicModel (models/examples/ *.h) ---------------- */
typedef struct {
  double  mass;                       /* DynamicModel::m_                                       */
  double  gravity;                    /* DynamicModel::g_ = 9.80665 (dynamic_model.cc:37)        */
  double  inertia[6];                 /* Ixx Iyy Izz Ixy Ixz Iyz, BuildInertiaTensor convention
                                         (single_rigid_body_dynamics.cc:36-44)                   */
  int32_t n_ee;
  int32_t reserved;
  double  nominal_stance[TOWR_MAX_EE][3];  /* KinematicModel::nominal_stance_                  */
  double  max_dev[TOWR_MAX_EE][3];         /* KinematicModel::max_dev_from_nominal_            */
  double  min_dev[TOWR_MAX_EE][3];         /* KinematicModel::min_dev_from_nominal_            */
} towr_robot_t;

/* ---- variable sets: ids of towr/include/towr/variables/variable_names.h:43-75 ------------- */
enum towr_varset_kind {
  TOWR_VAR_BASE_LIN    = 0,  /* "base-lin"      NodesVariablesAll                              */
  TOWR_VAR_BASE_ANG    = 1,  /* "base-ang"      NodesVariablesAll (Euler ZYX)                  */
  TOWR_VAR_EE_MOTION   = 2,  /* "ee-motion_i"   NodesVariablesEEMotion                         */
  TOWR_VAR_EE_ANG      = 3,  /* "ee-ang_i"      NodesVariablesEEAng                            */
  TOWR_VAR_EE_FORCE    = 4,  /* "ee-force_i"    NodesVariablesEEForce                          */
  TOWR_VAR_EE_TORQUE   = 5,  /* "ee-torque_i"   NodesVariablesEETorque                         */
  TOWR_VAR_EE_SCHEDULE = 6   /* "ee-schedule_i" PhaseDurations (only with optimize_timings)    */
};

typedef struct {
  int32_t kind;  /* towr_varset_kind           */
  int32_t ee;    /* endeffector id (ee sets)   */
} towr_varset_t;

/* ---- constraint sets: Parameters::ConstraintName (parameters.h:141-152) --------------------- */
enum towr_constraint_kind {
  TOWR_C_DYNAMIC          = 0, /* DynamicConstraint            dt; T                  (dynamic_constraint.cc:38-148)             */
  TOWR_C_RANGE_OF_MOTION  = 1, /* RangeOfMotionConstraint      dt; T; ee              (range_of_motion_constraint.cc:37-131)     */
  TOWR_C_FORCE            = 2, /* ForceConstraint (node-based) ee; p[0]=force limit   (force_constraint.cc:37-171)               */
  TOWR_C_FORCE_DISCRETIZED= 3, /* ForceConstraintDiscretized   dt; T; ee; p[0]=limit  (force_constraint_discretized.cc:71-221)   */
  TOWR_C_TERRAIN          = 4, /* TerrainConstraint            ee; p[0]=min p[1]=max  (terrain_constraint.cc:36-111)             */
  TOWR_C_BASE_MOTION      = 5, /* BaseMotionConstraint         dt; T; p[0..5]=ax,ay,lz bounds (base_motion_constraint.cc:38-91)  */
  TOWR_C_SPLINE_ACC       = 6, /* SplineAccConstraint          ee=0 base-lin, ee=1 base-ang (spline_acc_constraint.cc:34-86)     */
  TOWR_C_BASE_HEIGHT      = 7, /* BaseHeightConstraint         p[0]=safety distance   (base_height_constraint.cc:35-110)         */
  TOWR_C_SWING            = 8, /* SwingConstraint              ee; p[0]=t_swing_avg (0.3, swing_constraint.h:68)                  */
  TOWR_C_TOTAL_DURATION   = 9, /* TotalDurationConstraint      ee; T                  (total_duration_constraint.cc:36-72)       */
  TOWR_C_TORQUE_DISCRETIZED = 10, /* TorqueConstraintDiscretized ee; T; dt; p[0..3] = tx_min, tx_max, ty_min, ty_max;
                                     p[4] = k_friction                     (torque_constraint_discretized.cc:69-235) */
  TOWR_C_TORQUE           = 11, /* TorqueConstraint (node-based) ee; p[0..4] as above      (torque_constraint.cc:36-194)  */
  TOWR_C_TERRAIN_HARD     = 12, /* TerrainConstraintHard       ee; T; dt              (terrain_constraint_hard.cc:35-132)       */
  TOWR_C_EE_LINEAR        = 13, /* EELinearConstraint          T; dt; ip[0] = target (0 motion, 1 ang), ip[1] = deriv (0 pos,
                                     1 vel), ip[2] = n_terms (<= 6), ip[3 + i] = ee_i * 3 + dim_i; p[i] = coeff_i;
                                     (ee_linear_constraint.cc:5-48; the bound tolerance is setup data, not used here)  */
  TOWR_C_LINEAR_EQ        = 14  /* LinearEqualityConstraint    g = M x_set (linear_constraint.cc:35-80): ip[0] = variable set
                                     (index in AddVariableSet order), ip[1] = rows of M; M itself is side data
                                     TOWR_DATA_LINEAR_M (towr_gpu_create_ex). Jacobian = M.sparseView(): the nonzeros of M.
                                     The offset v only enters the bounds (-v), which stay with the caller            */
};

/* Role of a constraint set in the description:
 *   TOWR_ROLE_HARD: an ifopt constraint set (AddConstraintSet) — its rows are part of g and J;
 *   TOWR_ROLE_SOFT: only wrapped by a SoftConstraint cost term (AddCostSet(SoftConstraint(c)),
 *                   soft_constraint.cc:34-69) — not part of g / J; the cost term evaluates it.       */
enum towr_constraint_role { TOWR_ROLE_HARD = 0, TOWR_ROLE_SOFT = 1 };

typedef struct {
  int32_t kind;   /* towr_constraint_kind                                                       */
  int32_t ee;     /* endeffector id, or spline id for TOWR_C_SPLINE_ACC                        */
  double  T;      /* total horizon the constraint was constructed with                         */
  double  dt;     /* discretisation step of TimeDiscretizationConstraint subclasses            */
  double  p[6];   /* per-kind parameters (see enum)                                            */
  int32_t ip[9];  /* per-kind integer parameters (EELinear, LinearEquality)                     */
  int32_t role;   /* towr_constraint_role (0 = hard)                                            */
} towr_constraint_t;

/* ---- cost terms: NlpFormulation::GetCosts (nlp_formulation.cc:604-680) ------------------------ */
enum towr_cost_kind {
  TOWR_COST_NODE        = 0, /* NodeCost: ip[0] = variable set kind (towr_varset_kind), ee, ip[1] = deriv
                                (0 pos, 1 vel), ip[2] = dim; weight             (node_cost.cc:36-79)       */
  TOWR_COST_ENERGY      = 1, /* EnergyCost: weight, dt, p[0] = torque weight   (energy_cost.cc:36-152)    */
  TOWR_COST_ANG_MOMENTUM= 2, /* AngularMomentumCost: weight, dt                 (angular_momentum_cost.cc:39-208) */
  TOWR_COST_EE_BASE_POS = 3, /* EEBasePosCost: ee, weight, dt, p[0..2] = p_ref_B  (ee_base_pos_cost.cc:38-162) */
  TOWR_COST_BASE_HEIGHT = 4, /* BaseHeightCost of the fork: weight, dt (the reference's default 0.01 must be given),
                                p[0] = target base height above the mean stance-foot height
                                (base_height_cost.cc:36-142, added by hand in test/biped_example.cc:199-203)     */
  TOWR_COST_SOFT        = 5  /* SoftConstraint: 0.5 (g - b)^T (g - b) over constraint set ip[0] (any role), b = mid-point
                                of its bounds, given as side data TOWR_DATA_SOFT_BOUNDS (soft_constraint.cc:34-69);
                                W = identity as in the reference (no weight: `weight` is ignored)                 */
};
typedef struct {
  int32_t kind;    /* towr_cost_kind                                                             */
  int32_t ee;
  double  weight;
  double  dt;
  double  p[4];
  int32_t ip[4];
} towr_cost_t;

/* ---- initial guess (NlpFormulation::MakeBaseVariables etc., nlp_formulation.cc:121-346) ---- */
enum towr_init_mode {
  TOWR_INIT_FORMULATION = 0,  /* NlpFormulation::GetVariableSets initialisation                  */
  TOWR_INIT_PROCEDURAL  = 1   /* plain SetByLinearInterpolation of towr/test/procedural_example.cc:134-166 */
};

typedef struct {
  int32_t mode;                   /* towr_init_mode                                             */
  int32_t reserved;
  double  base_lin_p0[3], base_lin_v0[3], base_ang_p0[3], base_ang_v0[3];  /* initial_base_     */
  double  base_lin_p1[3], base_lin_v1[3], base_ang_p1[3], base_ang_v1[3];  /* final_base_       */
  double  ee_p0[TOWR_MAX_EE][3];  /* initial_ee_W_                                              */
  double  ee_p1[TOWR_MAX_EE][3];  /* procedural mode only: goal footholds                        */
} towr_init_t;

/* ---- full problem description --------------------------------------------------------------- */
typedef struct {
  int32_t        abi_version;               /* TOWR_GPU_ABI_VERSION                                */
  int32_t        angular_rep;               /* 0 = EulerZYX (Parameters::AngularRepresentation)    */
  towr_robot_t   robot;
  towr_terrain_t terrain;
  /* Parameters (parameters.cc:40-105)                                                            */
  double   total_time;                      /* Parameters::GetTotalTime()                          */
  double   duration_base_polynomial;        /* 0.1                                                  */
  int32_t  ee_polynomials_per_swing_phase;  /* 2                                                    */
  int32_t  force_polynomials_per_stance_phase;   /* 3                                               */
  int32_t  torque_polynomials_per_stance_phase;  /* 3                                               */
  int32_t  optimize_timings;                /* Parameters::IsOptimizeTimings()                     */
  double   bound_phase_duration[2];         /* (0.2, 1.0)                                          */
  int32_t  n_phases[TOWR_MAX_EE];
  int32_t  contact_at_start[TOWR_MAX_EE];   /* ee_in_contact_at_start_                              */
  double   phase_durations[TOWR_MAX_EE][TOWR_MAX_PHASES];  /* ee_phase_durations_                 */
  int32_t  n_varsets;                       /* order = ifopt AddVariableSet order                   */
  int32_t  n_constraints;                   /* order = ifopt AddConstraintSet order                 */
  towr_varset_t     varsets[TOWR_MAX_VARSETS];
  towr_constraint_t constraints[TOWR_MAX_CONSTRAINTS];
  towr_init_t       init;
  int32_t           n_costs;                /* order = ifopt AddCostSet order (cost terms)          */
  int32_t           reserved_costs;
  towr_cost_t       costs[TOWR_MAX_COSTS];
} towr_problem_desc_t;

typedef struct towr_gpu_handle_s* towr_gpu_handle;

/* ---- side data: what the POD description cannot hold (towr_gpu_create_ex) --------------------- */
enum towr_data_kind {
  TOWR_DATA_LINEAR_M    = 0, /* index = constraint (TOWR_C_LINEAR_EQ); count = rows * n_set; data = M row-major
                                (LinearEqualityConstraint::M_, linear_constraint.cc:35-45)                       */
  TOWR_DATA_SOFT_BOUNDS = 1  /* index = cost term (TOWR_COST_SOFT); count = 2 * rows of the wrapped set;
                                data = lower[0..rows-1], upper[0..rows-1] = the wrapped set's GetBounds(), from
                                which the engine forms b = (upper + lower) / 2 as SoftConstraint's ctor does  */
};
typedef struct {
  int32_t       kind;    /* towr_data_kind                                                          */
  int32_t       index;   /* constraint or cost index in the description                             */
  int64_t       count;   /* doubles at `data`                                                       */
  const double* data;    /* host memory, copied at creation                                         */
} towr_data_t;

/* ---- lifecycle ------------------------------------------------------------------------------- */
/* Builds the layout (variable maps, time grids, CSR pattern, per-item slot tables) on the host and
 * uploads it to `device`. device < 0 creates a layout-only handle (sizes, structure, x0; every
 * evaluation entry point then returns TOWR_ERR_NO_DEVICE) — used by host-side structure checks. Replaces NlpFormulation::GetVariableSets/GetConstraints + ifopt
 * Problem::AddVariableSet/AddConstraintSet (nlp_formulation.cc:76-378, hopper_example.cc:154-161). */
int towr_gpu_create(const towr_problem_desc_t* desc, int device, towr_gpu_handle* out);
/* Same, with side data (LinearEqualityConstraint matrices, SoftConstraint bounds); every
 * TOWR_C_LINEAR_EQ set and TOWR_COST_SOFT term needs its entry (else TOWR_ERR_INVALID).            */
int towr_gpu_create_ex(const towr_problem_desc_t* desc, int32_t n_data, const towr_data_t* data, int device,
                       towr_gpu_handle* out);
int towr_gpu_destroy(towr_gpu_handle h);
const char* towr_gpu_last_error(towr_gpu_handle h);   /* h may be NULL: last global error         */
int towr_gpu_abi_version(void);

/* n = ifopt Problem::GetNumberOfOptimizationVariables, m = GetNumberOfConstraints,
 * nnz = nonzeros of GetJacobianOfConstraints (what IpoptAdapter::get_nlp_info reports).          */
int towr_gpu_sizes(towr_gpu_handle h, int32_t* n, int32_t* m, int64_t* nnz);

/* Jacobian structure, 0-based (IpoptAdapter::eval_jac_g with values == NULL; C_STYLE indexing). */
int towr_gpu_jac_structure(towr_gpu_handle h, int32_t* iRow, int32_t* jCol);
/* Same pattern as CSR: row_ptr[m+1], col[nnz].                                                   */
int towr_gpu_jac_csr(towr_gpu_handle h, int64_t* row_ptr, int32_t* col);

/* Starting point x0 = ifopt Problem::GetVariableValues() after NlpFormulation initialisation.    */
int towr_gpu_initial_x(towr_gpu_handle h, double* x0);

/* x0 of another instance that shares this layout (same robot, gait, horizon, constraint list):
 * only the start/goal states and the terrain differ (BASELINE config 5's randomised batch).      */
int towr_gpu_initial_x_for(towr_gpu_handle h, const towr_init_t* init, const towr_terrain_t* terrain, double* x0);
/* Column range of variable set i (AddVariableSet order): kind, ee, first column, size.          */
int towr_gpu_varset_info(towr_gpu_handle h, int32_t i, int32_t* kind, int32_t* ee, int32_t* col0, int32_t* n);

/* ---- single-problem host callbacks (what IpoptAdapter calls) -------------------------------- */
/* g = ifopt Problem::EvalConstraints(x)          (IpoptAdapter::eval_g)                         */
int towr_gpu_eval_g(towr_gpu_handle h, const double* x, double* g);
/* values = ifopt Problem::EvalNonzerosOfJacobian(x)  (IpoptAdapter::eval_jac_g, values != NULL) */
int towr_gpu_eval_jac_values(towr_gpu_handle h, const double* x, double* values);
/* both at once (one fused launch)                                                                */
int towr_gpu_eval_g_jac(towr_gpu_handle h, const double* x, double* g, double* values);
/* IPOPT's callback pair without a second evaluation: eval_g_keep_jac evaluates g and the Jacobian at x
 * into the handle's device staging and returns g; the values stay on the device with a copy of x.
 * eval_jac_values_kept(x) copies them into `values` (a DMA in place when `values` is registered) when x
 * is bit-identical to the kept x, else it evaluates the values as towr_gpu_eval_jac_values does. Any
 * other host-pointer evaluation on the handle drops the kept values. (ifopt IpoptAdapter::eval_g /
 * eval_jac_g, hopper_example.cc:175-180)                                                           */
int towr_gpu_eval_g_keep_jac(towr_gpu_handle h, const double* x, double* g);
int towr_gpu_eval_jac_values_kept(towr_gpu_handle h, const double* x, double* values);
/* Objective (IpoptAdapter::eval_f = Problem::EvaluateCostFunction, the sum of every cost term's
 * GetCost) and its dense gradient (eval_grad_f = Problem::EvaluateCostFunctionGradient). A problem
 * without cost terms has f = 0 and a zero gradient.                                               */
int towr_gpu_eval_f(towr_gpu_handle h, const double* x, double* f);
int towr_gpu_eval_grad_f(towr_gpu_handle h, const double* x, double* grad);
/* Batched objective on the device: F[b], GRAD[b*ldgrad + j]; stream as for eval_batch_device.    */
int towr_gpu_eval_cost_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx,
                                    double* F, double* GRAD, int64_t ldgrad, void* stream);

/* ---- trajectory export: SaveTrajectoryToCSV (towr/src/utils/save_data.cpp:9-130) ------------ */
/* Samples at t = 0, dt, 2dt, ... (accumulated) while t <= T + 1e-9, T = the base-linear spline's total
 * time. Row layout, n_cols = 19 + 25 * n_ee doubles:
 *   t | base-lin pos vel acc | base-ang pos vel acc (the raw angular spline: Euler angles or rotation
 *   vector and its derivatives) | per ee: motion pos vel acc | ee-ang pos vel acc | force | torque |
 *   is_contact (1.0 / 0.0)                                                                        */
int towr_gpu_trajectory_size(towr_gpu_handle h, double dt, int32_t* n_samples, int32_t* n_cols);
/* one problem, host buffers: out = n_samples x n_cols row-major                                   */
int towr_gpu_sample_trajectory(towr_gpu_handle h, const double* x, double dt, double* out);
/* B problems on the device: OUT[b * ldo + k * n_cols + c], ldo >= n_samples * n_cols              */
int towr_gpu_sample_trajectory_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx, double dt,
                                            double* OUT, int64_t ldo, void* stream);

/* ---- batched evaluation over independent problems that share the layout ---------------------- */
/* Per-problem terrain parameters (the only per-instance input to g/J besides x). `terrains` is a
 * host array of B entries of the description terrain's curvature class (Gap or not; see
 * towr_gpu_pattern_outside for what curved terrain does to the pattern).
 * Once set, every BATCH entry point (eval_batch, eval_batch_device[_kernel], eval_cost_batch_device)
 * uses terrain b for problem b and requires exactly B problems (else TOWR_ERR_INVALID); B = 0 clears
 * the set. The single-problem entry points (eval_g, eval_jac_values, eval_g_jac, eval_f,
 * eval_grad_f, sample_trajectory*) always use the description's terrain.                         */
int towr_gpu_set_batch_terrain(towr_gpu_handle h, int32_t B, const towr_terrain_t* terrains);

/* Frozen-pattern check (curved terrain). On Gap terrain ForceConstraintDiscretized and
 * TorqueConstraintDiscretized add a row's motion block only where its scale is non-zero
 * (force_constraint_discretized.cc:58, torque_constraint_discretized.cc:57), so the reference's
 * Jacobian pattern moves with x; IPOPT's structure, and this engine's CSR, are fixed at x0 (the
 * description's). These return how many entries the reference's Jacobian at x holds OUTSIDE that
 * frozen pattern (0 on terrains without curvature): entries the frozen structure cannot deliver. The
 * values on the frozen pattern are always the reference's, or 0.0 where the reference has no entry.
 * Both are HOST passes, not device kernels: the predicate is a floating-point tie (is a scale exactly
 * 0.0?), so it is evaluated with the reference's own host operations (std::pow, no contraction). Both are
 * synchronous. The batch form ("_device": X lives in HBM) copies X to the host on `stream`, waits for
 * it, evaluates the B problems on up to 16 host threads with the batch terrains like eval_batch_device,
 * and writes counts[B] in host memory (bench.py `pattern_watch` times it on a 4096-problem Gap batch).
 * Layout-only handles answer the single form. */
int towr_gpu_pattern_outside(towr_gpu_handle h, const double* x, int64_t* count);
int towr_gpu_pattern_outside_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx,
                                          int32_t* counts, void* stream);

/* Device-resident batch: X[b*ldx + j], G[b*ldg + i], V[b*ldv + k] are DEVICE pointers (HBM);
 * `stream` is the hipStream_t to launch on (NULL = HIP's default stream, as in the HIP API).
 * want_g / want_jac select outputs.
 * Asynchronous with respect to the host. Streams: some layouts evaluate through scratch owned by
 * the handle (the per-instant records of the phase-duration-optimisation kernels, the SoftConstraint
 * child's g / values). A call issued on a different stream than the handle's previous call waits
 * (on the GPU, through an event) for that call's work before it touches the scratch, so calls on one
 * handle never race but serialise across streams; use one handle per stream to overlap them.     */
int towr_gpu_eval_batch_device(towr_gpu_handle h, int32_t B,
                               const double* X, int64_t ldx,
                               double* G, int64_t ldg,
                               double* V, int64_t ldv,
                               int32_t want_g, int32_t want_jac, void* stream);

/* Host batch (H2D of X, D2H of G and V; contiguous lds = n, m, nnz). Outputs move in chunks: the
 * kernels of chunk i overlap the PCIe transfer of chunk i - 1. Arrays inside memory registered with
 * towr_gpu_register_host are transferred in place; others go through the handle's pinned staging.  */
int towr_gpu_eval_batch(towr_gpu_handle h, int32_t B, const double* X, double* G, double* V);

/* Page-locks caller memory [ptr, ptr + bytes) (hipHostRegister) for this handle until
 * towr_gpu_unregister_host or towr_gpu_destroy. Every host-pointer entry point whose x / g / values
 * (or X / G / V) array lies inside a registered range DMAs straight to / from it, without the
 * staging copy: an IPOPT driver registers its x, g and values arrays once (they are reused by every
 * IpoptAdapter callback, hopper_example.cc:175-180). Ranges must not overlap; the memory must stay
 * allocated while registered.                                                                    */
int towr_gpu_register_host(towr_gpu_handle h, void* ptr, int64_t bytes);
int towr_gpu_unregister_host(towr_gpu_handle h, void* ptr);

/* Launch classes and launches, for roofline accounting. Kernel indices 0..4 are the launch
 * classes: Dynamic, RangeOfMotion, ForceConstraintDiscretized, TorqueConstraintDiscretized and the
 * small kinds (node-value constraints, SplineAcc, BaseMotion, TotalDuration, ...), one kernel each.
 * Indices 5..towr_gpu_num_kernels()-1 are the handle's fusion groups: classes that a step launches
 * together in one kernel (default RangeOfMotion + ForceConstraintDiscretized; environment variable
 * TOWR_GPU_FUSE at handle creation). towr_gpu_kernel_info gives a kernel's name, tiles (or units)
 * per problem (0 = not used by this handle) and algorithmic bytes per problem (CSR values and g rows
 * written + distinct x entries read); towr_gpu_eval_batch_device_kernel launches that kernel alone.
 * towr_gpu_step_launches lists the kernels one evaluation launches (returns their count).       */
int towr_gpu_kernel_info(towr_gpu_handle h, int32_t kernel, const char** name, int32_t* n_tiles,
                         int64_t* bytes_per_problem);
int towr_gpu_eval_batch_device_kernel(towr_gpu_handle h, int32_t kernel, int32_t B,
                                      const double* X, int64_t ldx, double* G, int64_t ldg,
                                      double* V, int64_t ldv, void* stream);
int towr_gpu_num_kernels(void);
int towr_gpu_step_launches(towr_gpu_handle h, int32_t* kernels, int32_t cap);
/* The implementation launch class `kernel` (0..4) uses on this handle: 0 = tile kernel, 1 = record +
 * stream kernels (every CSR unit composed and written once; phase-duration optimisation), -1 = the
 * class is not used. Introspection for tests and profiling.                                      */
int towr_gpu_kernel_path(towr_gpu_handle h, int32_t kernel);

/* Sets the launch geometry (tiles per workgroup); 0 = automatic. For benchmarking.              */
int towr_gpu_set_tiles_per_block(towr_gpu_handle h, int32_t tiles_per_block);

/* Per-launch algorithmic byte count used for the roofline: 8*(n + m + nnz) + terrain bytes.     */
int64_t towr_gpu_algorithmic_bytes_per_call(towr_gpu_handle h);

#ifdef __cplusplus
}
#endif

#endif /* TOWR_GPU_H_ */
