"""CPU oracle (test infrastructure only) -- see inf_oracle.py header."""
