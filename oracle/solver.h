/* oracle/solver.h — TEST INFRASTRUCTURE ONLY: generic GN/LM loop (solver_impl.h). */
#pragma once
typedef struct {
    long long n;
    const unsigned char* act;
    int use_pre;
    void* ctx;
    double (*cost)(void* ctx);
    void (*jtf)(void* ctx, float* r, float* diag);
    double (*apply)(void* ctx, const float* p, float* Ap);
    double (*model_cost)(void* ctx, const float* delta);
    void (*update)(void* ctx, const float* delta);
    void (*save)(void* ctx);
    void (*revert)(void* ctx);
    /* materialized-Jacobian path (NULL: matrix-free): cusparseOuter after PCGInit1, and
     * the SpMV apply of the PCG loop, which carries no LM CtC term (solverGPUGaussNewton.t
     * :1660-1757); the LM residual reset keeps the matrix-free apply (computeAdelta). */
    void (*materialize)(void* ctx);
    double (*apply_mat)(void* ctx, const float* p, float* Ap);
} oracle_problem_float;
typedef struct {
    long long n;
    const unsigned char* act;
    int use_pre;
    void* ctx;
    double (*cost)(void* ctx);
    void (*jtf)(void* ctx, double* r, double* diag);
    double (*apply)(void* ctx, const double* p, double* Ap);
    double (*model_cost)(void* ctx, const double* delta);
    void (*update)(void* ctx, const double* delta);
    void (*save)(void* ctx);
    void (*revert)(void* ctx);
    /* materialized-Jacobian path (NULL: matrix-free): cusparseOuter after PCGInit1, and
     * the SpMV apply of the PCG loop, which carries no LM CtC term (solverGPUGaussNewton.t
     * :1660-1757); the LM residual reset keeps the matrix-free apply (computeAdelta). */
    void (*materialize)(void* ctx);
    double (*apply_mat)(void* ctx, const double* p, double* Ap);
} oracle_problem_double;
typedef struct {
    int nIterations, lIterations, residual_reset_period;
    float min_relative_decrease, min_trust_region_radius, max_trust_region_radius, q_tolerance,
        function_tolerance, trust_region_radius, radius_decrease_factor, min_lm_diagonal, max_lm_diagonal;
} oracle_params;
/* reference defaults, solverGPUGaussNewton.t:41-55 */
static inline oracle_params oracle_default_params(void) {
    oracle_params p = {10, 10, 10, 1e-3f, 1e-32f, 1e16f, 0.0001f, 0.000001f, 1e4f, 2.0f, 1e-6f, 1e32f};
    return p;
}
int oracle_solve_f32(oracle_problem_float* P, int lm, const oracle_params* sp, double* costs);
int oracle_solve_f64(oracle_problem_double* P, int lm, const oracle_params* sp, double* costs);
