"""raymarchrenderer_amd — MI355X-native (gfx950) SDF ray-march path tracer.

The hot path of TheBinaryCodeX/RayMarchRenderer (RayMarch.glsl / RayMarch2.glsl / RayMarch3.glsl)
as HIP kernels behind a C ABI (include/rmr.h, librmr.so), with Python front-ends that mirror the
reference's Graphics / Camera / Screen host interfaces.
"""
from . import abi
from ._lib import RMRError, lib
from .renderer import (Camera, Graphics, Renderer, Screen, camera_view, default_camera_view, encode_bmp,
                       parity_schedule, save_name, tile_spiral, time_schedule)

__all__ = ["abi", "lib", "RMRError", "Renderer", "Graphics", "Camera", "Screen", "camera_view",
           "default_camera_view", "encode_bmp", "tile_spiral", "time_schedule", "parity_schedule", "save_name"]
