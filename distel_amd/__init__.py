"""distel_amd — MI355X-native EL+ saturation engine (DistEL hot path on HIP/gfx950).

Layout:
  csrc/        HIP kernels + C-ABI implementation (include/el_gpu.h)
  lib/         built libel_gpu.so (in-tree; travels to the GPU box)
  ir.py        normalized-axiom IR (AxiomLoader input boundary), .elax text form
  engine.py    ctypes binding of the C-ABI; no CPU fallback
  classifier.py  ELClassifier / AxiomProcessor mirror (per-rule-type entry points)
  result.py    result-node output format (ResultRearranger, final-saxioms, AxiomCounter)
  generators.py  seeded G1–G5 workloads
"""
__version__ = "0.1.0"
