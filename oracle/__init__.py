"""ORACLE -- test infrastructure only.

CPU restatements of the reference path (pnnl/ERT-Conditional-Diffusion-Model,
ERT_Conditional_Diffusion.py:80-164, :308-320) used as the parity checker and
as the CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product never does.

  ref_torch  -- PyTorch-CPU restatement, bit-identical to the reference
                (pinned by tests/golden/*.npz produced from the reference).
  ref_numpy  -- independent float64 restatement incl. hand-derived backward
                and Adam (pinned against the same fixtures within 1e-6).
  philox     -- numpy port of the device counter RNG (member-keyed noise).
"""
