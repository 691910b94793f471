"""CPU oracle (test infrastructure only; see magot_oracle.py)."""
