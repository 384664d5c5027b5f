"""opt_amd — MI355X-native Gauss-Newton / Levenberg-Marquardt runtime behind Opt's C ABI.

The product is the C-ABI shared library ``opt_amd/libopt_amd.so`` (``include/Opt.h``,
``include/opt_amd.h``). This package is the host-side mirror of the reference's own
driver class (``examples/shared/OptSolver.h:46-106``) over ctypes, used by the tests
and the benchmark. There is no CPU compute path: loading fails loudly if the HIP
library has not been built.
"""
from .api import (  # noqa: F401
    LIB_PATH,
    OptError,
    OptSolver,
    load_library,
)

__all__ = ["LIB_PATH", "OptError", "OptSolver", "load_library"]
