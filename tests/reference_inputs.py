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
    # the energies with no hand-written family (generated kernels)
    "cotangent_mesh_smoothing": 2091.86303,
    "embedded_mesh_deformation": 0.367129057645,      # LM (its args.config)
    "intrinsic_image_decomposition": 3.3105300000e6,  # stride 12 (53 x 30 px)
    "volumetric_mesh_deformation": 189.74081,
}
# solver kind each example's args.config selects (useOpt / useOptLM)
REFERENCE_KIND = {"embedded_mesh_deformation": "LMGPU"}
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


def cotangent_head():
    """examples/cotangent_mesh_smoothing on head.ply (opt_amd/harness/problems.py)."""
    z = np.load(os.path.join(GOLDEN, "mesh_head.npz"))
    return problems.cotangent_mesh_smoothing(z["verts"], z["faces"])


def volumetric_head():
    """examples/volumetric_mesh_deformation: the lattice over head.ply's bounding box."""
    z = np.load(os.path.join(GOLDEN, "mesh_head.npz"))
    return problems.volumetric_mesh_deformation(z["verts"], 0)


def embedded_raptor():
    """examples/embedded_mesh_deformation on raptor_simplify2k (.off + .mrk)."""
    z = np.load(os.path.join(GOLDEN, "mesh_raptor2k.npz"))
    return problems.embedded_mesh_deformation(z["verts"], z["faces"], z["marker_pos"], z["marker_idx"])


def intrinsic_ye():
    """examples/intrinsic_image_decomposition on ye_high2.png at stride 12."""
    z = np.load(os.path.join(GOLDEN, "iid_ye_s12.npz"))
    return problems.intrinsic_image_decomposition(z["rgb"], 1)


GENERATED_EXAMPLES = {"cotangent_mesh_smoothing": cotangent_head, "embedded_mesh_deformation": embedded_raptor,
                      "intrinsic_image_decomposition": intrinsic_ye, "volumetric_mesh_deformation": volumetric_head}
