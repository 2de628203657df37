"""insite_amd — MI355X-native implementation of the INSITE ODE-discovery hot path.

Host side of the drop-in: the ``SINDY`` plugin (``insite_amd.sindy``) mirrors
``libs_m/ct/src/models/sindy.py:57-760`` of the reference and drives the HIP kernels of
``libinsite_hip.so`` through the C ABI (``include/insite_hip.h``) via ``insite_amd.ops``.
"""
from .library import PolyLibrary, polynomial_library  # noqa: F401

__all__ = ["PolyLibrary", "polynomial_library"]
