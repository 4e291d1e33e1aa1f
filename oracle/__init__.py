"""CPU oracle — test infrastructure only (see nngp_oracle.py's header)."""
