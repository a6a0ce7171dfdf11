"""nart_amd: MI355X-native render path for shanesimmsart/nart's tiled path tracer.

The package holds the C-ABI libraries (built in-tree into nart_amd/lib) and their Python
bindings; see DESIGN.md for the architecture and INTEGRATION.md for the drop-in boundary.
"""
from .api import (HIP_SYMBOLS, PIXEL_FLOATS, SCENE_SYMBOLS, HipRenderer, bvh_info, NartError, NativeLibraryMissing,  # noqa: F401
                  RenderParams, RenderStats, Scene, combine_tiles, default_params, filter_table, finalize,
                  hip_lib, load_sessions, parse_args, read_exr, scene_lib, session_geometry, shard_buckets,
                  write_exr)

__all__ = ["HipRenderer", "bvh_info", "NartError", "NativeLibraryMissing", "RenderParams", "RenderStats", "Scene",
           "combine_tiles", "default_params", "filter_table", "finalize", "load_sessions", "parse_args", "read_exr",
           "write_exr", "hip_lib", "scene_lib", "session_geometry", "PIXEL_FLOATS", "HIP_SYMBOLS", "SCENE_SYMBOLS"]
