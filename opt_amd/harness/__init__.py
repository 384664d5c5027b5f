"""Host-side mirror of the reference's example harness (examples/shared + each example's
main.cpp / CombinedSolver.h): the data formats the examples read, the problem
construction each example performs, the profiled solve loop, and the results CSV /
final-cost report. The reference builds these as C++ against mLib, OpenMesh and the CUDA
runtime; here they are plain numpy over the same files, driving libopt_amd.so through
the C ABI (opt_amd.api.OptSolver).

    python -m opt_amd.harness image_warping --data /path/to/examples/data --useOpt
"""
from . import formats, problems, results  # noqa: F401
