"""Problem inputs of the reference's own end-to-end cost test (examples/test_final_cost.py),
rebuilt from the data fixtures in tests/golden/ exactly as the example harness builds
them, plus the expected final costs that test holds (CUDA reference values,
test_final_cost.py:55-66; compared within 1e-5 relative, :116-121)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# examples/test_final_cost.py:58-66 (CUDA, small size, nIterations = lIterations = 1)
REFERENCE_FINAL_COST = {
    "image_warping": 1774.3405,
}
REFERENCE_RTOL = 1e-5   # test_final_cost.py:121


def image_warping_cat512(alpha=1.0):
    """examples/image_warping/src/main.cpp:92-183 (file = 1, stride = 1) and
    CombinedSolver.h:116-219: Offset = UrShape = (x, y), Angle = 1e-5, Mask = red channel
    of cat512_mask.png, Constraints = (-1, -1) except the marker targets (blended by
    alpha) and every border pixel pinned to itself, both only where Mask == 0; later
    markers overwrite earlier ones. Weights w_fit = 100, w_reg = 0.01 (square-rooted)."""
    z = np.load(os.path.join(GOLDEN, "iw_cat512.npz"))
    m = z["mask"].astype(np.float32)
    H, W = m.shape
    cons = [list(map(int, c)) for c in z["constraints"]]
    for y in range(H):
        for x in range(W):
            if y == 0 or x == 0 or y == H - 1 or x == W - 1:
                cons.append([x, y, x, y])
    C = np.full((H, W, 2), -1.0, np.float32)
    a = np.float32(alpha)
    for x, y, nx, ny in cons:
        if m[y, x] == 0:
            C[y, x, 0] = (np.float32(1) - a) * np.float32(x) + a * np.float32(nx)
            C[y, x, 1] = (np.float32(1) - a) * np.float32(y) + a * np.float32(ny)
    ys, xs = np.mgrid[0:H, 0:W]
    U = np.stack([xs, ys], -1).astype(np.float32)
    return {
        "W": W, "H": H,
        "Offset": U.reshape(-1).copy(),
        "Angle": np.full(W * H, 1e-5, np.float32),
        "UrShape": U.reshape(-1).copy(),
        "Constraints": C.reshape(-1),
        "Mask": m.reshape(-1),
        "w_fitSqrt": float(np.sqrt(np.float32(100.0), dtype=np.float32)),
        "w_regSqrt": float(np.sqrt(np.float32(0.01), dtype=np.float32)),
    }
