"""Pack the inputs of the reference's own end-to-end cost test into fixtures.

The reference's examples/test_final_cost.py runs every example at a small size with
nIterations = lIterations = 1 (examples/shared/ArgParser.h defaults, the example's
args.config) and checks the "final cost=" the solver logs (Opt_ProblemCurrentCost,
API/src/solverGPUGaussNewton.t:1903) against CUDA reference costs within 1e-5
relative (test_final_cost.py:55-66, 116-121). This script extracts the INPUT data
those runs read — data files only, nothing executable — exactly as the example
harness loads them:

  image_warping (examples/image_warping/src/main.cpp:92-183, file = 1, stride = 1):
    cat512_mask.png red channel (the Mask), cat512.constraints (marker list).
    The harness builds Offset = UrShape = (x, y), Angle = 1e-5, the border pins and
    the Constraints image from these (CombinedSolver.h:168-219); tests/reference_inputs.py
    restates that construction.

Data licence: public domain (examples/data/copyright.txt).

    python tests/golden/make_reference_fixtures.py /root/reference
"""
import os
import sys

import numpy as np
from PIL import Image


def main(ref):
    data = os.path.join(ref, "examples", "data")
    here = os.path.dirname(os.path.abspath(__file__))
    mask = np.array(Image.open(os.path.join(data, "cat512_mask.png")))[..., 0].astype(np.uint8)   # .x of RGBA
    with open(os.path.join(data, "cat512.constraints")) as f:
        tok = f.read().split()
    n = int(tok[0])
    cons = np.array([int(t) for t in tok[1:1 + 4 * n]], np.int32).reshape(n, 4)
    out = os.path.join(here, "iw_cat512.npz")
    np.savez_compressed(out, mask=mask, constraints=cons)
    print(out, mask.shape, cons.shape)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
