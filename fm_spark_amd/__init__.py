"""fm_spark_amd — MI355X-native FM mini-batch SGD hot path of Rainbowboys/fm_spark.

Layers:
  csrc/      HIP kernels for gfx950 + the C-ABI of include/fm_hip.h (libfm_hip.so)
  _native    ctypes binding (no fallback: the HIP library must load)
  engine     FMContext: one device's tables, step / predict / export
  ml         host mirror of the reference's spark.ml API (FactorizationMachinesSGD, ...)
  sampler    randomSplit replay through the C-ABI
  data       synthetic Criteo-shaped batches, LIBSVM reader
"""

__all__ = ["engine", "ml", "linalg", "sampler", "data"]
