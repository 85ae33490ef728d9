"""CPU oracle for the correlation hot path -- test infrastructure only (see oracle.py)."""
