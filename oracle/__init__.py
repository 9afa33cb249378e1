"""CPU oracle (test infrastructure only; see gp_oracle.py header)."""
