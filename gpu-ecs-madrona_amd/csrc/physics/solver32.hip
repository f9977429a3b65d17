// The solver with two worlds per wave (MW_SOLVER_LANES=32: each world's
// per-world phases on its half, ballots and broadcasts over the half, the
// level passes over both worlds' merged schedule on all 64 lanes), as
// namespace lanes32 -- the variant the physics module picks for worlds whose
// dependency levels are narrow (solver.hip, SolverNode in physics.hip).
#define MW_SOLVER_LANES 32
// Two worlds' images per block: LDS bounds this variant to 2 waves per SIMD,
// so registers are free up to 256 -- the velocity solves keep their lever
// arms and angular terms (simple_taskgraph SolverNode 0.369 -> 0.342 ms).
#ifndef MW_SOLVER_VEL_ARMS
#define MW_SOLVER_VEL_ARMS 2
#endif
#ifndef MW_SOLVER_WAVES_PER_EU
#define MW_SOLVER_WAVES_PER_EU 2
#endif
#define MW_SOLVER_NS lanes32
#define MW_SOLVER_C(name) name##_32
#include "solver.hip"
