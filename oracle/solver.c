/* oracle/solver.c — TEST INFRASTRUCTURE ONLY: instantiates the generic GN/LM loop
 * (solver_impl.h) for float and double. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "solver.h"

#define REAL float
#define OACC double
#include "solver_impl.h"
#undef REAL
#undef OACC
#define OACC long double
#define REAL double
#include "solver_impl.h"
#undef REAL

int oracle_solve_f32(oracle_problem_float* P, int lm, const oracle_params* sp, double* costs) {
    return oracle_solve_float(P, lm, sp, costs);
}
int oracle_solve_f64(oracle_problem_double* P, int lm, const oracle_params* sp, double* costs) {
    return oracle_solve_double(P, lm, sp, costs);
}
