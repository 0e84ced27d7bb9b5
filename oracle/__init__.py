"""TEST INFRASTRUCTURE ONLY: CPU parity oracle (see oracle/nex_oracle.h)."""
