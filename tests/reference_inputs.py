"""Problem inputs of the reference's own end-to-end cost test (examples/test_final_cost.py),
rebuilt from the data fixtures in tests/golden/ exactly as the example harness builds
them, plus the expected final costs that test holds (CUDA reference values,
test_final_cost.py:55-66; compared within 1e-5 relative, :116-121)."""
import os

import numpy as np

from opt_amd.harness import problems

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# examples/test_final_cost.py:58-66 (CUDA, small size, nIterations = lIterations = 1)
REFERENCE_FINAL_COST = {
    "image_warping": 1774.3405,
    "optical_flow": 0.52119255,     # cost of the first solve (the coarse level, sigma 5)
    "arap_mesh_deformation": 7183.464843,
}
# Not reproducible from the reference's files: poisson_image_editing (its harness reads
# the strided mask at (stride x, stride y) of the already-strided image,
# examples/poisson_image_editing/src/main.cpp:95-101, i.e. out of bounds for the
# test's stride 4), shape_from_shading (no reference value, test_final_cost.py:64).
REFERENCE_RTOL = 1e-5   # test_final_cost.py:121


def image_warping_cat512(alpha=1.0):
    """examples/image_warping (file = 1, stride = 1) from the cat512 fixture, built by the
    harness mirror (opt_amd/harness/problems.py: image_warping)."""
    z = np.load(os.path.join(GOLDEN, "iw_cat512.npz"))
    return problems.image_warping(z["mask"], z["constraints"], alpha)


def optical_flow_dogdance(level=1):
    """examples/optical_flow (stride 16) from the dogdance fixture: the first solve the
    harness runs is level 1 (opt_amd/harness/problems.py: optical_flow)."""
    z = np.load(os.path.join(GOLDEN, "of_dogdance_s16.npz"))
    return problems.optical_flow(z["src"], z["tar"], level)


def arap_armadillo():
    """examples/arap_mesh_deformation on small_armadillo, one sqrt(3) subdivision
    (opt_amd/harness/problems.py: arap)."""
    z = np.load(os.path.join(GOLDEN, "arap_armadillo.npz"))
    return problems.arap(z["verts"].astype(np.float32), z["faces"], z["marker_pos"], z["marker_idx"], 1)
