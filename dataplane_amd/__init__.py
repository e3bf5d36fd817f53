# SPDX-License-Identifier: Apache-2.0
"""MI355X (gfx950) per-burst packet path of githedgehog/dataplane.

Product code: csrc/ (HIP kernel, C ABI runtime, table compiler) built into
lib/libdpgpu.so, plus the NetworkFunction-shaped host mirror (nf.py).
"""
from . import _abi  # noqa: F401
from .nf import GpuPathNf, Packet, PipelineData  # noqa: F401

__all__ = ["GpuPathNf", "Packet", "PipelineData"]
