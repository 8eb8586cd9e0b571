"""CPU oracle for the SHPL path -- test infrastructure only (see shpl_oracle.c)."""
