"""MI355X-native Metropolis-Hastings interior-layout sampler (drop-in for the reference's
KernelWrapper DLL surface, KernelFolder/Kernel/Kernel.cu:873).

The product is libmhgpu.so (csrc/: HIP kernels for gfx950 + the C ABI of include/mh_kernel.h).
This Python package is the host-side mirror of that ABI (ctypes) plus the rooms the tests and
bench use. The directory name contains hyphens, so load it with load_package() below (or
importlib) rather than a plain import.
"""
from .abi import (COST_FIELDS, EXPORTS, LIB_PATH, MHError, Room, Session, STRUCT_LAYOUT,  # noqa: F401
                  debug_collectives, debug_math, device_cus, debug_rng, evaluate_costs, kernel_wrapper,
                  last_error, load_library, MH_PROBE_COUNT, probe_width, release_cache,
                  wrapper_step_kernel)
from .rooms import clone_cfg, main_fixture, synthetic_room  # noqa: F401
