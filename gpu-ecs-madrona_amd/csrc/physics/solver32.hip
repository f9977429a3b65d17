// The solver with two worlds per wave (MW_SOLVER_LANES=32: each world's
// per-world phases on its half, ballots and broadcasts over the half, the
// level passes over both worlds' merged schedule on all 64 lanes), as
// namespace lanes32 -- the variant the physics module picks for worlds whose
// dependency levels are narrow (solver.hip, SolverNode in physics.hip).
#define MW_SOLVER_LANES 32
#define MW_SOLVER_NS lanes32
#define MW_SOLVER_C(name) name##_32
#include "solver.hip"
