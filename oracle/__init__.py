"""ORACLE package -- test infrastructure only.

CPU restatements of the reference (AdrienWohrer/diff-icp, torch path) used as the parity
checker.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything here; the product (diff-icp_amd/) never does.
  torch_ref.py   -- float64 torch restatement (dense, row-chunked), autograd-capable
  difficp_ref.c  -- plain-C/OpenMP restatement of the ODE fwd/VJP and E-step (c_ref.py)
Pinned against tests/golden/*.npz generated from the reference itself
(tests/golden/make_golden.py, run in the build container only).
"""
