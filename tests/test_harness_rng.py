"""CPU: the C++ standard-library draws the robust_nonrigid_alignment harness makes
(CombinedSolver.h:109-120: std::mt19937(230948), uniform_int_distribution<>,
normal_distribution<>), restated in opt_amd/harness/problems.py, against this image's
g++ / libstdc++ (GCC 11: Lemire's uniform_int; the polar normal method)."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opt_amd.harness import problems  # noqa: E402

SRC = r"""
#include <cstdio>
#include <random>
int main() {
    std::mt19937 rnd(230948);
    std::uniform_int_distribution<> u(0, 10001);
    std::normal_distribution<> n(0.0f, 0.5608228);
    for (int i = 0; i < 40; ++i) {
        int k = u(rnd);
        double a = n(rnd), b = n(rnd), c = n(rnd);
        std::printf("%d %.17g %.17g %.17g\n", k, a, b, c);
    }
    std::mt19937 r2(5489);
    std::printf("%u\n", (unsigned)r2());
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_std_random_restatement_matches_libstdcxx(tmp_path):
    src = tmp_path / "r.cpp"
    src.write_text(SRC)
    exe = tmp_path / "r"
    subprocess.run(["g++", "-O1", "-std=c++17", str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    assert int(out[40]) == problems.StdMt19937(5489)()
    rng = problems.StdMt19937(230948)
    nd = problems.StdNormal(0.0, 0.5608228)
    for line in out[:40]:
        k, a, b, c = line.split()
        assert problems.std_uniform_int(rng, 0, 10001, lemire=True) == int(k)
        np.testing.assert_array_equal([nd(rng), nd(rng), nd(rng)], [float(a), float(b), float(c)])
