"""Pack the reference's own shape_from_shading example inputs into a fixture.

Reads examples/data/shape_from_shading/default{.SFSSolverParameters,_*.imagedump}
from a reference checkout (plain binary: TerraSolverParameters.h:7-45 and the
SimpleBuffer header, SimpleBuffer.cpp:16-59; -inf depths clamped to -10000 as
SimpleBuffer's clampInfinity does) and writes tests/golden/sfs_default.npz. Pure data:
inputs only (the reference holds no expected outputs for this energy).

    python tests/golden/make_sfs_fixture.py /root/reference
"""
import os
import sys

import numpy as np


def imagedump(path):
    raw = open(path, "rb").read()
    w, h, ch, dt = np.frombuffer(raw[:16], dtype=np.int32)
    a = np.frombuffer(raw[16:], dtype=np.float32 if dt == 0 else np.uint8).copy()
    if dt == 0:
        a[np.isinf(a) & (a > 0)] = np.finfo(np.float32).max
        a[np.isinf(a) & (a < 0)] = -10000.0
    return a.reshape(h * ch, w) if ch == 1 else a.reshape(h, w, ch)


def main(ref):
    d = os.path.join(ref, "examples", "data", "shape_from_shading", "default")
    p = np.fromfile(d + ".SFSSolverParameters", dtype=np.float32)
    # weightFitting, weightRegularizer, weightShading, fx, fy, ux, uy, lightingCoefficients[9]
    params = np.concatenate([p[[0, 1, 3, 7, 8, 9, 10]], p[27:36]]).astype(np.float32)
    X0 = imagedump(d + "_initialUnknown.imagedump")
    D = imagedump(d + "_targetDepth.imagedump")
    Im = imagedump(d + "_targetIntensity.imagedump")
    mask = imagedump(d + "_maskEdgeMap.imagedump")   # rows then columns map, stacked
    H, W = D.shape
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sfs_default.npz")
    np.savez_compressed(out, params=params, X0=X0, D_i=D, Im=Im, edgeMaskR=mask[:H], edgeMaskC=mask[H:])
    print(out, W, H, params)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
