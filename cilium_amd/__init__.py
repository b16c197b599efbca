"""cilium_amd — MI355X-native batched flow classifier with Cilium's verdict
semantics (reference: carlanton/cilium 1.0.0-rc9).

Layers:
  libgpuflow.so (csrc/)  C ABI + HIP kernels for gfx950 (the product)
  bpf.py                 pkg/bpf mirror (map syscalls -> libgpuflow)
  maps/                  pkg/maps/* typed key/value layouts
  datapath.py            program loading + classify calls on HBM batches
  synth.py               seeded synthetic workloads (BASELINE configs)
"""
from . import _lib  # noqa: F401  (fails loudly if libgpuflow.so is missing)
from . import bpf  # noqa: F401

__all__ = ["bpf"]
