/* A C99 program that uses libopt_amd.so exactly as the reference's examples use Opt:
 * Opt.h only, the call sequence of examples/shared/OptSolver.h:46-106
 * (Opt_NewState with a zeroed Opt_InitializationParameters, Opt_ProblemDefine,
 * Opt_ProblemPlan, Opt_SetSolverParameter, Opt_ProblemSolve, Opt_ProblemCurrentCost,
 * Opt_PlanFree, Opt_ProblemDelete). Host buffers (backend_cpu), so the program itself
 * needs no GPU API. Input: the image_warping problem in a flat binary file written by
 * tests/test_c_caller_gpu.py; output: "final cost=<value>".
 *
 *   caller <energy.t> <problem.bin> <backend> <nIterations> <lIterations>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "Opt.h"

static float* read_floats(FILE* f, size_t n) {
    float* p = (float*)malloc(n * sizeof(float));
    if (!p || fread(p, sizeof(float), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return p;
}

int main(int argc, char** argv) {
    if (argc != 6) { fprintf(stderr, "usage: caller energy.t problem.bin backend nIter lIter\n"); return 2; }
    FILE* f = fopen(argv[2], "rb");
    if (!f) { perror(argv[2]); return 2; }
    int dims[2];
    if (fread(dims, sizeof(int), 2, f) != 2) return 2;
    const size_t N = (size_t)dims[0] * dims[1];
    float* offset = read_floats(f, 2 * N);
    float* angle = read_floats(f, N);
    float* urshape = read_floats(f, 2 * N);
    float* constraints = read_floats(f, 2 * N);
    float* mask = read_floats(f, N);
    float* w = read_floats(f, 2);
    fclose(f);

    Opt_InitializationParameters ip;
    memset(&ip, 0, sizeof(ip));
    ip.verbosityLevel = 0;
    ip.collectPerKernelTimingInfo = 0;
    ip.doublePrecision = 0;
    strcpy(ip.backend, argv[3]);
    ip.numthreads = 1;
    Opt_State* state = Opt_NewState(ip);
    Opt_Problem* problem = state ? Opt_ProblemDefine(state, argv[1], "gaussNewtonGPU") : NULL;
    unsigned int udims[2] = {(unsigned)dims[0], (unsigned)dims[1]};
    Opt_Plan* plan = problem ? Opt_ProblemPlan(state, problem, udims) : NULL;
    if (!plan) { fprintf(stderr, "plan failed\n"); return 1; }
    int nIter = atoi(argv[4]), lIter = atoi(argv[5]);
    Opt_SetSolverParameter(state, plan, "nIterations", &nIter);
    Opt_SetSolverParameter(state, plan, "lIterations", &lIter);
    /* problemparams in declared-index order (energies/image_warping.t) */
    void* params[7] = {offset, angle, urshape, constraints, mask, &w[0], &w[1]};
    Opt_ProblemSolve(state, plan, params);
    printf("final cost=%.10f\n", Opt_ProblemCurrentCost(state, plan));
    Opt_PlanFree(state, plan);
    Opt_ProblemDelete(state, problem);
    free(offset); free(angle); free(urshape); free(constraints); free(mask); free(w);
    return 0;
}
