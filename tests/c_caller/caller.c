/* A C99 program that uses libopt_amd.so exactly as the reference's examples use Opt:
 * Opt.h only, the call sequence of examples/shared/OptSolver.h:46-106
 * (Opt_NewState with a zeroed Opt_InitializationParameters, Opt_ProblemDefine,
 * Opt_ProblemPlan, Opt_SetSolverParameter, Opt_ProblemSolve, Opt_ProblemCurrentCost,
 * Opt_PlanFree, Opt_ProblemDelete).
 *
 * backend_cpu / backend_cpu_mt: problemparams are host arrays.
 * backend_cuda: the arrays are device allocations made and filled by this program with
 * the HIP runtime's C API (hipMalloc / hipMemcpy), as the reference harness does with
 * cudaMalloc / cudaMemcpy (examples/shared/OptImage.h:49-51,95-105); the unknowns are
 * copied back after the solve (OptImage::copyTo).
 *
 * Input: a flat binary problem written by tests/test_c_caller_gpu.py:
 *   int32 kind (0: image_warping, 1: arap_mesh_deformation graph)
 *   kind 0: int32 W, H; float Offset[2N], Angle[N], UrShape[2N], Constraints[2N],
 *           Mask[N]; float w_fitSqrt, w_regSqrt
 *   kind 1: int32 N, E; float Offset[3N], Angle[3N], UrShape[3N], Constraints[3N];
 *           int32 v0[E], v1[E]; float w_fitSqrt, w_regSqrt
 * Output: "final cost=<value>" and a checksum of the unknowns read back.
 *
 *   caller <energy.t> <problem.bin> <backend> <nIterations> <lIterations>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime_api.h>
#include "Opt.h"

static void* read_bytes(FILE* f, size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p || fread(p, 1, n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
    return p;
}

#define HIPCHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); exit(3); } } while (0)

/* A problem array as the caller hands it to Opt: the host copy, and with backend_cuda
 * a device allocation holding the same bytes. */
typedef struct { void* host; void* dev; size_t bytes; } Buf;

static int g_device = 0;

static Buf buf_read(FILE* f, size_t bytes) {
    Buf b;
    b.host = read_bytes(f, bytes);
    b.dev = NULL;
    b.bytes = bytes;
    if (g_device) {
        HIPCHECK(hipMalloc(&b.dev, bytes ? bytes : 4));
        HIPCHECK(hipMemcpy(b.dev, b.host, bytes, hipMemcpyHostToDevice));
    }
    return b;
}
static void* buf_ptr(const Buf* b) { return g_device ? b->dev : b->host; }
static void buf_fetch(Buf* b) {   /* unknowns back to the host copy */
    if (g_device) HIPCHECK(hipMemcpy(b->host, b->dev, b->bytes, hipMemcpyDeviceToHost));
}
static void buf_free(Buf* b) {
    if (b->dev) HIPCHECK(hipFree(b->dev));
    free(b->host);
}
static double checksum(const Buf* b) {
    const float* v = (const float*)b->host;
    double s = 0.0;
    for (size_t i = 0; i < b->bytes / sizeof(float); ++i) s += v[i];
    return s;
}

int main(int argc, char** argv) {
    if (argc != 6) { fprintf(stderr, "usage: caller energy.t problem.bin backend nIter lIter\n"); return 2; }
    g_device = strcmp(argv[3], "backend_cuda") == 0;
    FILE* f = fopen(argv[2], "rb");
    if (!f) { perror(argv[2]); return 2; }
    int hdr[3];
    if (fread(hdr, sizeof(int), 3, f) != 3) return 2;
    const int kind = hdr[0];
    const size_t n0 = (size_t)hdr[1], n1 = (size_t)hdr[2];
    Buf arr[8];
    int narr = 0;
    int edge_count = (int)n1;
    float* w;
    void* params[9];
    if (kind == 0) {   /* image_warping: declared indices 0..6 (energies/image_warping.t) */
        const size_t N = n0 * n1, F = sizeof(float);
        const size_t sz[5] = {2 * N * F, N * F, 2 * N * F, 2 * N * F, N * F};
        for (int k = 0; k < 5; ++k) arr[narr++] = buf_read(f, sz[k]);
        w = (float*)read_bytes(f, 2 * sizeof(float));
        for (int k = 0; k < 5; ++k) params[k] = buf_ptr(&arr[k]);
        params[5] = &w[0];
        params[6] = &w[1];
    } else {           /* ARAP: [w_fit, w_reg, Offset, Angle, UrShape, Constraints, G] */
        const size_t N = n0, E = n1, F = sizeof(float);
        for (int k = 0; k < 4; ++k) arr[narr++] = buf_read(f, 3 * N * F);
        arr[narr++] = buf_read(f, E * sizeof(int));
        arr[narr++] = buf_read(f, E * sizeof(int));
        w = (float*)read_bytes(f, 2 * sizeof(float));
        params[0] = &w[0];
        params[1] = &w[1];
        for (int k = 0; k < 4; ++k) params[2 + k] = buf_ptr(&arr[k]);
        /* a Graph: the edge-count pointer, then one vertex array per slot
           (examples/shared/NamedParameters.h:35-49, OptGraph.h:37-52) */
        params[6] = &edge_count;
        params[7] = buf_ptr(&arr[4]);
        params[8] = buf_ptr(&arr[5]);
    }
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
    unsigned int udims[2] = {(unsigned)n0, (unsigned)n1};
    Opt_Plan* plan = problem ? Opt_ProblemPlan(state, problem, udims) : NULL;
    if (!plan) { fprintf(stderr, "plan failed\n"); return 1; }
    int nIter = atoi(argv[4]), lIter = atoi(argv[5]);
    Opt_SetSolverParameter(state, plan, "nIterations", &nIter);
    Opt_SetSolverParameter(state, plan, "lIterations", &lIter);
    Opt_ProblemSolve(state, plan, params);
    printf("final cost=%.10f\n", Opt_ProblemCurrentCost(state, plan));
    /* the unknowns: Offset, Angle (image: arrays 0, 1; graph: arrays 0, 1) */
    buf_fetch(&arr[0]);
    buf_fetch(&arr[1]);
    printf("unknowns checksum=%.10e %.10e\n", checksum(&arr[0]), checksum(&arr[1]));
    Opt_PlanFree(state, plan);
    Opt_ProblemDelete(state, problem);
    for (int k = 0; k < narr; ++k) buf_free(&arr[k]);
    free(w);
    return 0;
}
