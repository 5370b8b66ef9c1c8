"""sdf3d_amd -- MI355X-native SDF sphere-tracing renderer.

Drop-in replacement for the device programs of ezorzin/SDF3D
(Code/shader/voxel_fragment.frag et al.): a hand-written HIP kernel for
gfx950 behind the C-ABI in include/sdf_abi.h.  This package holds the ctypes
binding (abi), the scene/camera presets (scenes), the host-side renderer
(renderer), the multi-device frame driver (multigpu) and the algorithmic
cost model used for roofline accounting (costmodel).
"""
from . import abi, scenes
from .abi import SdfError, load_library
from .renderer import Renderer, owned_rows, tiling
from .scenes import CONFIGS, Frame, config, orbit_view, reference

__all__ = ["abi", "scenes", "SdfError", "load_library", "Renderer", "owned_rows", "tiling",
           "CONFIGS", "Frame", "config", "orbit_view", "reference"]
