"""CPU oracle (test infrastructure only; see ref_flow.py header).  PARITY UNPINNED."""
